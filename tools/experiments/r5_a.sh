# round 5 (a): k_gsweep barrier fix check, stepped sharded replay kernel trace (G=1, 8),
# the per-wave drop-in loop line -> gpurun_out/r5a/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_irregular.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 10 --shards 1,8 --stepped 1 > $O/shard.jsonl 2>&1
cut -c1-160 $O/shard.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/shard_replay_bench.py --runs 3 --shards 1,8 --stepped 1 > $O/prof.jsonl 2>&1
timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop.json 2> $O/loop.err
cut -c1-600 $O/loop.json
echo done
