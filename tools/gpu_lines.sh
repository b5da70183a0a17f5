#!/bin/bash
# The other bench lines (C3, C5, C4 paper, C4 deep weak edges, the per-wave drop-in
# loop) and the kernel tuning table.  usage: tools/gpu_lines.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lines}
mkdir -p $OUT
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 300 python bench.py --config c4-loop > $OUT/bench_loop.json 2> $OUT/bench_loop.err &&
step 400 python bench.py --config c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
step 400 python bench.py --config c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err &&
step 300 python bench.py --deliver paper --no-cpu > $OUT/bench_paper.json 2> $OUT/bench_paper.err &&
step 400 python bench.py --config c4-deep --steps 3 --warmup 1 --no-cpu > $OUT/bench_deep.json 2> $OUT/bench_deep.err &&
step 200 python -u tools/tune.py > $OUT/tune.txt 2>&1
rc=$?
echo "exit $rc" > $OUT/status.txt
exit $rc
