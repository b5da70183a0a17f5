#!/bin/bash
# K pass on its own wavefront (workgroup form of the C5 batch kernel) + batch host phases
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-kw}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_batch.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/batch_timing.py 512 1024 4096 > $O/timing.jsonl 2> $O/timing.err &&
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 10 --warmup 3 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 200 python bench.py --config c5 --dags 512 --no-cpu --steps 10 --warmup 3 > $O/c5_512.json 2> $O/c5_512.err
rc=$?
echo "exit $rc" > $O/status.txt
exit $rc
