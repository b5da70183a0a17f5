# round 4: hipGraph replay -- its GPU tests, then C4 / C3 bench lines with and without the graph
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_graph.py tests/test_gpu_golden.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print(round(d['ms_per_step'],4), 'ms', d.get('replay_form'), d['roofline'].get('frac'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c4_graph 300 --steps 100 --warmup 10 --no-cpu --verify --graph
line c4_nograph 300 --steps 100 --warmup 10 --no-cpu --verify
line c3_graph 300 --config c3 --steps 100 --warmup 10 --no-cpu --verify --graph
line c3_nograph 300 --config c3 --steps 100 --warmup 10 --no-cpu --verify
