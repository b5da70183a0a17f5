# round 4: sharded replay variants (wu beside / before the pass, emission fused / apart) and the
# commit split on / off, plain timings + the fused sweep's per-query ticks
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v
mkdir -p $O
for v in "1 0" "0 0" "1 1"; do set -- $v
  DR_SHARD_WU_SIDE=$1 DR_SHARD_EMIT_FUSED=$2 timeout -k 10 120 python3 -u tools/shard_replay_bench.py --runs 20 --shards 1,8 --stepped 0 > $O/shard_wu$1_em$2.jsonl 2>&1
  echo "wu_side=$1 emit_fused=$2: $(python3 -c "import json; print([(d['G'], round(d['ms_wall_median'],3), round(d['device_ms'],3), {k: round(x,3) for k,x in d['phases_ms'].items()}) for d in map(json.loads, open('$O/shard_wu$1_em$2.jsonl'))])")"
done
timeout -k 10 120 python3 -u tools/ms_timing.py c4 1,8 > $O/mst.jsonl 2>&1; cut -c1-600 $O/mst.jsonl
for sp in 1 2 0; do
  DR_BENCH_COMMIT_SPLIT=$sp timeout -k 10 200 python3 -u bench.py --rank-share 8 --steps 20 > $O/share_split$sp.json 2> $O/share_split$sp.err
  echo "split=$sp: $(python3 -c "import json; d=json.load(open('$O/share_split$sp.json')); print(d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'])")"
done
