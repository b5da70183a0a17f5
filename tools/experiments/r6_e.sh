# round 6 (e): re-check of the restored tree after the session restart: the whole GPU
# suite, smoke, the default bench line, C4/C3 verified, rocprof kernel stats and
# timelines for C4/C3, the PMC traffic passes for C4 -> gpurun_out/r6e/
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
if grep -q -i "illegal memory\|memory access fault\|hipErrorLaunchFailure" $O/gpu_tests.log; then echo "GPU fault in tests: stopping"; exit 3; fi
step 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
line() {  # name, args...
  local name=$1; shift
  step 400 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['roofline']['frac'] if d.get('roofline') else None, d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay', d['detail'].get('verify_vs_unsharded'))))"
}
line bench_default || exit 1
line bench_c4 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line bench_c3 --config c3 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line bench_c4up --config c4-up --no-cpu --steps 5 --warmup 1 || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4.json 2> $O/prof_c4.err || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || exit 1
step 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o fetch -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 1
step 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o write -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || exit 1
echo done
