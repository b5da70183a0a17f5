#!/bin/bash
# Chain restarts expanded in wave 0: parity, C3/C4/C2 lines, C3 timeline.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-v15}
mkdir -p $OUT
fatal() { [ $1 -eq 124 ] || [ $1 -ge 128 ]; }
run() { local name=$1 t=$2; shift 2; echo "[step] $name" >&2; timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name $rc" >> $OUT/status.txt; if fatal $rc; then echo "fatal $rc in $name" >&2; exit $rc; fi; return $rc; }
run tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_coin.py tests/test_gpu_dups.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread || exit 1
run c4 200 python bench.py --no-cpu --steps 100 --warmup 10
run c3 200 python bench.py --config c3 --no-cpu --steps 50 --warmup 5
run c2 200 python bench.py --config c2 --no-cpu --steps 50 --warmup 5
run prof_c3 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c3 -o c3 -- python bench.py --config c3 --no-cpu --steps 5 --warmup 2
python tools/timeline.py $OUT/prof_c3 > $OUT/timeline_c3.txt
echo done >> $OUT/status.txt
