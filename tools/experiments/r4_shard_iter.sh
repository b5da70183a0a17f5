# round 4: sharded replay iteration -- shard GPU tests, plain timings (every G, both forms), kernel trace (G=1, 8 fused)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 > gpurun_out/r4s_shard.jsonl 2>&1
cut -c1-200 gpurun_out/r4s_shard.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4s_prof -o run -- python3 tools/shard_replay_bench.py --runs 10 --shards 1,8 --stepped 0 > gpurun_out/r4s_prof.jsonl 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4s_share -o run -- python3 bench.py --rank-share 8 --steps 10 > gpurun_out/r4s_share.json 2>gpurun_out/r4s_share.err
cut -c1-400 gpurun_out/r4s_share.json
for g in 0 1 2 3; do true;  DR_SHARD_PASS_GEO=$g timeout -k 10 120 python3 -u tools/shard_replay_bench.py --runs 10 --shards 1,8 --stepped 0 > gpurun_out/r4s_geo$g.jsonl 2>&1; done
