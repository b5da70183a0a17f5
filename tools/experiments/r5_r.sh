# round 5 (r): long-DAG canonical prefixes as an extra workgroup of the pop sweeps --
# parity suites, C3/C4 lines, C3 timeline -> gpurun_out/r5r/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for c in c3 c4; do
    timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/${c}_$rep.json 2> $O/${c}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/${c}_$rep.json').read()); print('$c rep $rep', round(d['ms_per_step'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu > $O/prof_c3.json 2> $O/prof_c3.err
python3 tools/timeline.py $O/prof_c3 > $O/timeline_c3.txt 2>&1 || true
cat $O/timeline_c3.txt
echo done
