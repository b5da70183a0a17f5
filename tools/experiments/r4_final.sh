# round 4 closing check: every GPU test, smoke, the bench lines, rocprof kernel stats of the C4 bench
# and the sharded replay, PMC traffic -> gpurun_out/r4f/ (copied into profiles/r04/ afterwards)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_shard -o run -- python3 tools/shard_replay_bench.py --runs 20 --stepped 0 > $O/prof_shard.jsonl 2>&1
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 30 > $O/shard_replay.jsonl 2>&1
echo done
