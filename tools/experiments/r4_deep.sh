# round 4: deep-window check -- parity tests touching the memo, then the c4-deep and C4 lines
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_dups.py tests/test_gpu_golden.py tests/test_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1 || { tail -30 gpurun_out/r4d_tests.log; exit 1; }
tail -1 gpurun_out/r4d_tests.log
timeout -k 10 300 python3 -u bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu --verify > gpurun_out/r4d_deep.json 2> gpurun_out/r4d_deep.err
python3 -c "import json; d=json.load(open('gpurun_out/r4d_deep.json')); print('deep', d['ms_per_step'], d['detail']['ms'], d['detail']['verify_vs_oracle'])"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4d_c4.json 2> gpurun_out/r4d_c4.err
python3 -c "import json; d=json.load(open('gpurun_out/r4d_c4.json')); print('c4', d['ms_per_step'], d['detail']['ms'])"
timeout -k 10 300 python3 -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/r4d_c5.json 2> gpurun_out/r4d_c5.err
python3 -c "import json; d=json.load(open('gpurun_out/r4d_c5.json')); print('c5', d['ms_per_step'], d['detail']['step_phases_ms'])"
timeout -k 10 300 python3 -u bench.py --config c5 --dags 512 --steps 20 --warmup 5 --no-cpu > gpurun_out/r4d_c5_512.json 2> gpurun_out/r4d_c5_512.err
python3 -c "import json; d=json.load(open('gpurun_out/r4d_c5_512.json')); print('c5_512', d['ms_per_step'], d['detail']['step_phases_ms'])"
