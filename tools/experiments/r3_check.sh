#!/bin/bash
# Round-3 GPU session: parity tests, smoke, default bench (CPU baselines included),
# rocprof kernel trace, PMC traffic passes, and the other configs' lines.  Every GPU
# step has its own time limit; the chain stops at the first failure.
# usage: tools/r3_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3}
mkdir -p $OUT
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
step 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --no-cpu --steps 5 --warmup 2 > $OUT/bench_prof.json 2> $OUT/prof.err &&
step 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o fetch -- python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err &&
step 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o write -- python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/pmc_write.json 2> $OUT/pmc_write.err &&
step 120 python bench.py --colshard --no-cpu --steps 10 --warmup 3 > $OUT/bench_cs1.json 2> $OUT/bench_cs1.err &&
step 150 python tools/shard_replay_bench.py > $OUT/shard_replay.jsonl 2> $OUT/shard_replay.err &&
step 120 python bench.py --rank-share 8 --steps 20 > $OUT/rank_share_8.json 2> $OUT/rank_share_8.err &&
step 300 python bench.py --config c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
step 200 python bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err &&
step 120 python bench.py --config c1 --steps 20 > $OUT/bench_c1.json 2> $OUT/bench_c1.err
rc=$?
echo "exit $rc" > $OUT/status.txt
exit $rc
