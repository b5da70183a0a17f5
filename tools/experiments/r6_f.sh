# round 6 (f): A/B of the delivery sweep (round-5 tree vs HEAD timing builds), then the
# fused row pass (weak unions) + the canonical re-emission inside the delivery sweeps:
# GPU tests, C4/C3 verified, rocprof timelines -> gpurun_out/r6f/
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 200 python3 tools/sweep_timing.py c4 > $O/swt_head_c4.json 2> $O/swt_head_c4.err || exit 1
(cd ab_r5 && step 200 python3 tools/sweep_timing.py c4) > $O/swt_r5_c4.json 2> $O/swt_r5_c4.err || exit 1
step 900 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_irregular.py tests/test_gpu_incremental.py tests/test_gpu_wsplit.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
line() {  # name, args...
  local name=$1; shift
  step 400 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['roofline']['frac'] if d.get('roofline') else None, d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay', d['detail'].get('verify_vs_unsharded'))))"
}
line bench_c4 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line bench_c3 --config c3 --no-cpu --verify --steps 50 --warmup 5 || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4.json 2> $O/prof_c4.err || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || exit 1
DR_FUSE=0 step 400 python3 -u bench.py --no-cpu --steps 50 --warmup 5 > $O/bench_c4_fuse0.json 2> $O/bench_c4_fuse0.err || exit 1
DR_FUSE=2 step 400 python3 -u bench.py --no-cpu --steps 50 --warmup 5 > $O/bench_c4_fuse2.json 2> $O/bench_c4_fuse2.err || exit 1
DR_FUSE=1 step 400 python3 -u bench.py --no-cpu --steps 50 --warmup 5 > $O/bench_c4_fuse1.json 2> $O/bench_c4_fuse1.err || exit 1
for f in fuse0 fuse1 fuse2; do python3 -c "import json; d=json.loads(open('$O/bench_c4_$f.json').read()); print('$f', round(d['ms_per_step'],4))"; done
echo done
