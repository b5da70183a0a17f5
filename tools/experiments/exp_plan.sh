#!/bin/bash
# batch plan reuse: the batch tests, then the C5 lines (4096 and 512 DAGs) with their step phases
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-plan}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_batch.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 20 --warmup 3 > $O/c5.json 2> $O/c5.err &&
timeout -k 10 200 python bench.py --config c5 --dags 512 --no-cpu --steps 20 --warmup 3 > $O/c5_512.json 2> $O/c5_512.err
rc=$?
echo "exit $rc" > $O/status.txt
exit $rc
