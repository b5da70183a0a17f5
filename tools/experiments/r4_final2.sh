# round 4 closing check (v8): every GPU test, smoke, the bench lines, rocprof kernel stats of the
# C4 bench -> gpurun_out/r4v8/ (copied into profiles/r04/ afterwards)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4v8
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo "$name FAILED"; tail -5 $O/bench_$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print(round(d['ms_per_step'],4), 'ms', d['roofline'].get('frac'), d['roofline'].get('bound'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c4 400 --steps 20 --warmup 5
line c3 300 --config c3 --steps 20 --warmup 5 --no-cpu --verify
line c4_deep 300 --config c4-deep --steps 5 --warmup 2 --no-cpu --verify
line c4_dups 300 --config c4-dups --steps 5 --warmup 2 --no-cpu --verify
line c5 300 --config c5 --steps 10 --warmup 2 --no-cpu
line c5_512 300 --config c5 --dags 512 --steps 20 --warmup 5 --no-cpu
line share8 200 --rank-share 8 --steps 20
line colshard1 300 --colshard --steps 20 --warmup 5 --no-cpu
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
echo done
