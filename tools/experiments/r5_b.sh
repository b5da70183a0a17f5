# round 5 (b): the stepped sharded replay rewrite (shard_step.hpp) -- shard GPU tests,
# timings at G = 1, 2, 4, 8 (both forms), kernel trace of the stepped form -> gpurun_out/r5b/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 > $O/shard.jsonl 2>&1
python3 -c "
import json
for l in open('$O/shard.jsonl'):
    d=json.loads(l); print(d['G'], d['form'], round(d['ms_wall_median'],4), d['replay_ok'], d['steps'], d.get('host_syncs'), {k: round(v,4) for k,v in d['phases_ms'].items()})
"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/shard_replay_bench.py --runs 3 --shards 1,8 --stepped 1 > $O/prof.jsonl 2>&1
echo done
