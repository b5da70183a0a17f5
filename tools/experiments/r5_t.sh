# round 5 (t): k_gsweep with register/LDS row ORs, U for fully new rounds, no fence per
# round, sweeps bounded at the target round -- irregular suite, gsweep timing -> gpurun_out/r5t/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_irregular.py tests/test_gpu_exceptions.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/gsweep_bench.py 256 > $O/gsweep.jsonl 2> $O/gsweep.err || echo "gsweep bench ended rc=$?"
cat $O/gsweep.jsonl
echo done
