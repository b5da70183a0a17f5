# round 4: the whole GPU suite, then the sharded replay timings (fused / stepped) and the N=8 commit share
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { tail -60 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 300 python -u tools/shard_replay_bench.py --runs 20 > gpurun_out/r4a_shard.jsonl 2>&1
cut -c1-300 gpurun_out/r4a_shard.jsonl
timeout -k 10 300 python -u bench.py --rank-share 8 --steps 20 > gpurun_out/r4a_share8.json 2> gpurun_out/r4a_share8.err
cut -c1-700 gpurun_out/r4a_share8.json
