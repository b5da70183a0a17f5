# round 5 (j): coalesced wave-scan canonical prefix (k_canon_prefix) -- golden parity, C3 A/B
# against the run form, C3/C4 kernel traces -> gpurun_out/r5j/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for t in 1 0; do
    DR_CANON_TILES=$t timeout -k 10 300 python3 -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu > $O/c3_t${t}_$rep.json 2> $O/c3_t${t}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/c3_t${t}_$rep.json').read()); print('c3 waves=$t rep $rep', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu > $O/prof_c3.json 2> $O/prof_c3.err
python3 tools/timeline.py $O/prof_c3 > $O/timeline_c3.txt 2>&1 || true
grep canon_prefix $O/timeline_c3.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
python3 tools/timeline.py $O/prof_c4 > $O/timeline_c4.txt 2>&1 || true
echo done
