# round 6 (i): C5 sparse records (live leaders only) tests + line + PMC; the C4/C3 lines with
# this round's traffic file; k_own_emit at 256 threads (C4); the replay graph form
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 600 python3 -u -m pytest tests/test_batch.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
line() {  # name, args...
  local name=$1; shift
  step 400 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); r=d.get('roofline') or {}; print('$name', round(d['ms_per_step'],4), r.get('frac'), r.get('traffic'), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay', d['detail'].get('verify_vs_unsharded'))))"
}
line bench_c5 --config c5 --no-cpu --steps 20 --warmup 3 || exit 1
for cfg in c5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${cfg}_$ctr -o run -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 > $O/${cfg}_$ctr.json 2> $O/${cfg}_$ctr.err || { echo "$cfg $ctr failed"; exit 1; }
  done
done
line bench_c4 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line bench_c3 --config c3 --no-cpu --verify --steps 50 --warmup 5 || exit 1
DR_OWN_NT=256 step 400 python3 -u bench.py --no-cpu --verify --steps 50 --warmup 5 > $O/bench_c4_own256.json 2> $O/bench_c4_own256.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_c4_own256.json').read()); print('own256', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle'))"
line bench_c4_graph --no-cpu --graph --steps 50 --warmup 5 || exit 1
line bench_c3_graph --config c3 --no-cpu --graph --steps 50 --warmup 5 || exit 1
DR_OWN_NT=256 step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_own256 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4_own256.json 2> $O/prof_c4_own256.err || exit 1
echo done
