# round 4: kernel trace of the fused sharded replay (G=1, 8) and the headline bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_shard -o run -- python3 tools/shard_replay_bench.py --runs 10 --shards 1,8 --stepped 0 > gpurun_out/r4p_shard.jsonl 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4p_bench -o run -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/r4p_bench.json 2>gpurun_out/r4p_bench.err
find gpurun_out/r4p_shard gpurun_out/r4p_bench -name '*kernel_stats.csv' | head
