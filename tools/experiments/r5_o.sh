# round 5 (o): C5 wave form with the commit rule inside the cone pass; commit split auto for
# the per-call waveReady -- batch + split + golden tests, C5 lines, c4-loop -> gpurun_out/r5o/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_batch.py tests/test_gpu_split.py tests/test_gpu_golden.py tests/test_gpu_graph.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu > $O/c5.json 2> $O/c5.err
python3 -c "import json; d=json.loads(open('$O/c5.json').read()); print('c5', round(d['ms_per_step'],4), d['roofline']['kernel'], d['roofline']['bound'], round(d['roofline']['ms_per_launch'],4))"
timeout -k 10 300 python3 -u bench.py --config c5 --dags 512 --steps 5 --warmup 2 --no-cpu > $O/c5_512.json 2> $O/c5_512.err
python3 -c "import json; d=json.loads(open('$O/c5_512.json').read()); print('c5/512', round(d['ms_per_step'],4), d['roofline']['kernel'], round(d['roofline']['ms_per_launch'],4))"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/pmc_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/pmc_write.log 2>&1
timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop.json 2> $O/loop.err
python3 -c "import json; d=json.loads(open('$O/loop.json').read()); print({k: round(v['p50'],1) for k, v in d['detail']['latency_us'].items()}, d['detail']['verify_vs_replay'])"
echo done
