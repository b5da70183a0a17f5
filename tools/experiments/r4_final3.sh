# round 4 closing check (v9): parity subset after the WS<16 batch fix, the C3/C4/deep lines,
# rocprof kernel stats of the C4 and C3 benches -> gpurun_out/r4v9/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4v9
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dups.py tests/test_gpu_graph.py tests/test_gpu_irregular.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo "$name FAILED"; tail -5 $O/bench_$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print(round(d['ms_per_step'],4), 'ms', d['roofline'].get('frac'), d['roofline'].get('bound'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c4 400 --steps 20 --warmup 5
line c3 300 --config c3 --steps 20 --warmup 5 --no-cpu --verify
line c4_deep 300 --config c4-deep --steps 5 --warmup 2 --no-cpu --verify
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 20 --warmup 5 --no-cpu > $O/prof_c3.json 2> $O/prof_c3.err
echo done
