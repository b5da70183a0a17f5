# round 5 (j): coalesced wave-scan canonical prefix and the weak unions fused into the row
# pass -- golden + parity, C3/C4 A/B (DR_CANON_TILES, DR_WU_FUSE), timelines -> gpurun_out/r5j/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_exceptions.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in "DR_CANON_TILES=1 DR_WU_FUSE=1" "DR_CANON_TILES=0 DR_WU_FUSE=1" "DR_CANON_TILES=1 DR_WU_FUSE=0"; do
    for c in c3 c4; do
      tag=$(echo "$v" | tr -d ' =_A-Z' )
      env $v timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/${c}_${tag}_$rep.json 2> $O/${c}_${tag}_$rep.err
      python3 -c "import json; d=json.loads(open('$O/${c}_${tag}_$rep.json').read()); print('$c', '$v', 'rep $rep', round(d['ms_per_step'],4), round(d['detail']['ms']['summary'],4))"
    done
  done
done
for c in c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > $O/prof_$c.json 2> $O/prof_$c.err
  python3 tools/timeline.py $O/prof_$c > $O/timeline_$c.txt 2>&1 || true
done
echo done
