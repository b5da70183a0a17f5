# round 4, step a: sharded replay (fused / stepped) and split-commit parity, then timings
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 300 python -u tools/shard_replay_bench.py --runs 20 > gpurun_out/r4a_shard.jsonl 2>&1
cut -c1-300 gpurun_out/r4a_shard.jsonl
timeout -k 10 300 python -u bench.py --rank-share 8 --steps 20 > gpurun_out/r4a_share8.json 2> gpurun_out/r4a_share8.err
cut -c1-600 gpurun_out/r4a_share8.json
