# round 5 (f): stepped replay back to the vote before the walk, separate emission; variant STEP_NT=128
# -> gpurun_out/r5f/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ() { python3 -c "
import json,sys
for l in open('$1'):
    d=json.loads(l); print('$2', d['G'], d['form'], round(d['ms_wall_median'],4), d['replay_ok'], d['steps'], d.get('host_syncs'), {k: round(v,4) for k,v in d['phases_ms'].items()})
"; }
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 > $O/shard.jsonl 2>&1
summ $O/shard.jsonl base
DR_SHARD_STEP_NT=128 timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 --stepped 1 > $O/shard_nt128.jsonl 2>&1
summ $O/shard_nt128.jsonl nt128
DR_SHARD_STEP_NT=128 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread -k "stepped or c4_full or memo_replay_generated" > $O/tests_nt128.log 2>&1 || { echo "NT64 TESTS FAILED"; tail -30 $O/tests_nt128.log; exit 1; }
tail -1 $O/tests_nt128.log
DR_SHARD_HOST_TIMING=1 timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 5 --shards 1 --stepped 1 > $O/host_timing.jsonl 2> $O/host_timing.err
tail -3 $O/host_timing.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/shard_replay_bench.py --runs 3 --shards 1,8 --stepped 1 > $O/prof.jsonl 2>&1
echo done
