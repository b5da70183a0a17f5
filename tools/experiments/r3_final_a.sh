#!/bin/bash
# Round-3 final check, part A: parity tests, smoke, the default bench line (C4 with the CPU
# baselines, oracle verify), rocprof kernel statistics, PMC traffic passes.  Each GPU step
# has its own time limit; the chain stops at the first failure.  usage: tools/r3_final_a.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
step 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
step 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --no-cpu --steps 5 --warmup 2 > $OUT/bench_prof.json 2> $OUT/prof.err &&
step 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o fetch -- python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err &&
step 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o write -- python bench.py --no-cpu --steps 2 --warmup 1 > $OUT/pmc_write.json 2> $OUT/pmc_write.err &&
step 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_tl -o tl -- python bench.py --no-cpu --steps 5 --warmup 2 > $OUT/prof_tl.json 2> $OUT/prof_tl.err &&
python tools/timeline.py $OUT/prof_tl > $OUT/timeline_c4.txt
rc=$?
echo "exit $rc" > $OUT/status.txt
exit $rc
