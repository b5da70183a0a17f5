# round 4: k_kcand over all lanes -- parity subset, c4-deep / c4 lines, c4-deep kernel times
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dups.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print(round(d['ms_per_step'],4), 'ms', d['roofline'].get('frac'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c4_deep 300 --config c4-deep --steps 10 --warmup 2 --no-cpu --verify
line c4 300 --steps 50 --warmup 5 --no-cpu --verify
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu > $O/prof.json 2> $O/prof.err
python3 tools/prof_db.py $(ls $O/prof/*/run_results.db | head -1) > $O/deep_kernels.txt
head -16 $O/deep_kernels.txt
