set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dups.py tests/test_gpu_incremental.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d2_tests.log 2>&1 || { tail -30 gpurun_out/r4d2_tests.log; exit 1; }
tail -1 gpurun_out/r4d2_tests.log
timeout -k 10 300 python3 -u bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu --verify > gpurun_out/r4d2_deep.json 2> gpurun_out/r4d2_deep.err
python3 -c "import json; d=json.load(open('gpurun_out/r4d2_deep.json')); print('deep', d['ms_per_step'], d['detail']['ms'], d['detail']['verify_vs_oracle'])"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4dp2 -o run -- python3 bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu > gpurun_out/r4dp2.json 2> gpurun_out/r4dp2.err
