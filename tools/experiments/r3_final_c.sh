#!/bin/bash
# Round-3 closing check at the final commit: every GPU test, smoke, the default C4 line,
# the C5 lines (4096 with the CPU baseline, 512) after the batch plan reuse, C3, and the
# C3 / C4 timelines (multi-item scans in the planning kernels).
# usage: tools/r3_final_c.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final_c}
mkdir -p $OUT
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
step 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
step 300 python bench.py --config c5 --steps 20 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err &&
step 200 python bench.py --config c5 --dags 512 --no-cpu --steps 20 --warmup 3 > $OUT/bench_c5_512.json 2> $OUT/bench_c5_512.err &&
step 300 python bench.py --config c3 --no-cpu --steps 50 --warmup 5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c3 -o c3 -- python bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $OUT/prof_c3.json 2> $OUT/prof_c3.err &&
python tools/timeline.py $OUT/prof_c3 > $OUT/timeline_c3.txt &&
step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_tl -o tl -- python bench.py --no-cpu --steps 5 --warmup 2 > $OUT/prof_tl.json 2> $OUT/prof_tl.err &&
python tools/timeline.py $OUT/prof_tl > $OUT/timeline_c4.txt
rc=$?
echo "exit $rc" > $OUT/status.txt
exit $rc
