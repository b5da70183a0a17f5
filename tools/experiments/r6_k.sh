# round 6 (k): each query's own rounds emitted by its sweep workgroup (DR_OPT_FUSE bit 32):
# tests, C4/C3 lines per mask, timelines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 900 python3 -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_irregular.py tests/test_gpu_wsplit.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
for m in 23 55; do
  for cfg in c4 c3; do
    DR_FUSE=$m step 400 python3 -u bench.py --config $cfg --no-cpu --verify --steps 50 --warmup 5 > $O/bench_${cfg}_f$m.json 2> $O/bench_${cfg}_f$m.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_f$m.json').read()); print('$cfg f$m', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle'))"
  done
done
DR_FUSE=55 step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_f55 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4.json 2> $O/prof_c4.err || exit 1
DR_FUSE=55 step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_f55 -o c3 -- python3 bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || exit 1
echo done
