#!/bin/bash
# C5 batch kernel forms: parity tests, per-phase timings at several batch sizes, bench lines.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c5}
mkdir -p $OUT
fatal() { [ $1 -eq 124 ] || [ $1 -ge 128 ]; }
run() { local name=$1 t=$2; shift 2; echo "[step] $name" >&2; timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name $rc" >> $OUT/status.txt; if fatal $rc; then echo "fatal $rc in $name" >&2; exit $rc; fi; return 0; }
run batch_tests 500 python -u -m pytest tests/test_batch.py -x -q --timeout 300 --timeout-method thread
run batch_timing 300 python -u tools/batch_timing.py 512 1024 2048 4096
run c5_4096 200 python bench.py --config c5 --no-cpu --steps 10 --warmup 3
run c5_512 200 python bench.py --config c5 --dags 512 --no-cpu --steps 10 --warmup 3
echo done >> $OUT/status.txt
