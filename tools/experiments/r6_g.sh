# round 6 (g): the fused row pass (weak unions), the canonical re-emission inside the
# delivery sweeps, the speculative prefixes beside the walk and the pop plan beside the sweeps, the live delivery-query count, C5's sparse cone records: GPU tests,
# C4/C3/C5 verified, rocprof timelines, the fusion variants, the sweep's workgroup span
# against its rocprof duration -> gpurun_out/r6g/
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 900 python3 -u -m pytest tests/test_gpu_irregular.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_wsplit.py tests/test_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
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
line bench_c5 --config c5 --no-cpu --verify --steps 20 --warmup 3 || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4.json 2> $O/prof_c4.err || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || exit 1
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --config c5 --no-cpu --steps 5 --warmup 2 > $O/prof_c5.json 2> $O/prof_c5.err || exit 1
step 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_swt -o swt -- python3 tools/sweep_timing.py c4 > $O/swt_c4.json 2> $O/swt_c4.err || exit 1
for f in 0 3 15; do
  DR_FUSE=$f step 400 python3 -u bench.py --no-cpu --steps 50 --warmup 5 > $O/bench_c4_fuse$f.json 2> $O/bench_c4_fuse$f.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_c4_fuse$f.json').read()); print('fuse$f', round(d['ms_per_step'],4))"
done
line wsplit8 --wave-split 8 --steps 20 --warmup 3 || exit 1
line wsplit4 --wave-split 4 --steps 20 --warmup 3 || exit 1
line wsplit2 --wave-split 2 --steps 20 --warmup 3 || exit 1
echo done
