#!/bin/bash
# k_own_emit at 256 threads per query: replay parity, C3 / C4 lines and timelines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-own}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --config c3 --no-cpu --steps 50 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 200 python bench.py --no-cpu --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c3 -o c3 -- python bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err &&
python tools/timeline.py $O/prof_c3 > $O/timeline_c3.txt &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_tl -o tl -- python bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_tl.json 2> $O/prof_tl.err &&
python tools/timeline.py $O/prof_tl > $O/timeline_c4.txt
rc=$?
echo "exit $rc" > $O/status.txt
exit $rc
