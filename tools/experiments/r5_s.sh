# round 5 (s): appends return without waiting for their copies; incremental exception totals --
# the suites that append between queries, batch, c4-loop -> gpurun_out/r5s/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_exceptions.py tests/test_gpu_irregular.py tests/test_batch.py tests/test_gpu_dups.py tests/test_gpu_setweak.py tests/test_coin.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop_$rep.json 2> $O/loop_$rep.err
  python3 -c "import json; d=json.loads(open('$O/loop_$rep.json').read()); print({k: round(v['p50'],1) for k, v in d['detail']['latency_us'].items()}, d['detail']['verify_vs_replay'])"
done
echo done
timeout -k 10 240 python3 -u tools/gsweep_bench.py 256 > $O/gsweep.jsonl 2> $O/gsweep.err || echo "gsweep bench ended rc=$?"
cat $O/gsweep.jsonl
echo done2
