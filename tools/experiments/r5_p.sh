# round 5 (p): k_canon -- next bad round found 64 rounds a thread, positions' presence-prefix
# defaults written by k_kcand -- parity suites, C3/C4 lines, canon timing -> gpurun_out/r5p/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_exceptions.py tests/test_gpu_dups.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for c in c3 c4; do
    timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/${c}_$rep.json 2> $O/${c}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/${c}_$rep.json').read()); print('$c rep $rep', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 python3 tools/canon_timing.py c4 c3 > $O/canon_timing.jsonl 2> $O/canon_timing.err
cat $O/canon_timing.jsonl
for c in c3 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > $O/prof_$c.json 2> $O/prof_$c.err
  python3 tools/timeline.py $O/prof_$c > $O/timeline_$c.txt 2>&1 || true
done
grep k_canon $O/timeline_c3.txt $O/timeline_c4.txt || true
echo done
