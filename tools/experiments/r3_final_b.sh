#!/bin/bash
# Round-3 final check, part B: the other configs' lines (C3, C2, C1, C5 at 4096 and at one
# rank's share of 512, with their CPU baselines), the column-sharded replay (one-rank RCCL
# line, local-mode sweep over G) and one rank's share of the wave-range commit split.
# usage: tools/r3_final_b.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 400 python -u -m pytest tests/test_batch.py -x -q --timeout 300 --timeout-method thread > $OUT/batch_tests.log 2>&1 &&
step 300 python -u tools/batch_timing.py 512 4096 > $OUT/batch_timing.jsonl 2> $OUT/batch_timing.err &&
step 300 python bench.py --config c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
step 200 python bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
step 120 python bench.py --config c1 --steps 20 > $OUT/bench_c1.json 2> $OUT/bench_c1.err &&
step 300 python bench.py --config c5 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err &&
step 200 python bench.py --config c5 --dags 512 --no-cpu --steps 10 --warmup 3 > $OUT/bench_c5_512.json 2> $OUT/bench_c5_512.err &&
step 120 python bench.py --colshard --no-cpu --steps 10 --warmup 3 > $OUT/bench_cs1.json 2> $OUT/bench_cs1.err &&
step 150 python tools/shard_replay_bench.py > $OUT/shard_replay.jsonl 2> $OUT/shard_replay.err &&
step 120 python bench.py --rank-share 8 --steps 20 > $OUT/rank_share_8.json 2> $OUT/rank_share_8.err &&
step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c3 -o c3 -- python bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
python tools/timeline.py $OUT/prof_c3 > $OUT/timeline_c3.txt
rc=$?
echo "exit $rc" > $OUT/status_b.txt
exit $rc
