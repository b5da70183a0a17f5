# round 5 (y): the stepped sharded replay with wave 0's round words loaded before the ring
# copy and the weak-column scan over the frontier's nonzero words: shard tests, replay
# times at G = 1..8 (both forms), a kernel trace at G = 1 and 8 -> gpurun_out/r5y/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 > $O/shard.jsonl 2>&1
python3 -c "
import json
for l in open('$O/shard.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['G'], d['form'], round(d['ms_wall_median'],3), d['replay_ok'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/shard_replay_bench.py --runs 3 --shards 1,8 --stepped 1 > $O/prof.jsonl 2>&1
python3 tools/shard_timeline.py $O/prof > $O/timeline_g1.txt 2>&1 || true
python3 tools/shard_timeline.py $O/prof -1 > $O/timeline_g8.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || true
rm -rf $O/prof
echo done
