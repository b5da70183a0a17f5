#!/bin/bash
# Full GPU tests, smoke, C4/C3/C5 lines, batch timings and the C4/C3 timelines.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-v14}
mkdir -p $OUT
fatal() { [ $1 -eq 124 ] || [ $1 -ge 128 ]; }
run() { local name=$1 t=$2; shift 2; echo "[step] $name" >&2; timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name $rc" >> $OUT/status.txt; if fatal $rc; then echo "fatal $rc in $name" >&2; exit $rc; fi; return $rc; }
run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run c4 200 python bench.py --no-cpu --steps 100 --warmup 10
run c3 200 python bench.py --config c3 --no-cpu --steps 50 --warmup 5
run c5_4096 200 python bench.py --config c5 --no-cpu --steps 10 --warmup 3
run c5_512 200 python bench.py --config c5 --dags 512 --no-cpu --steps 10 --warmup 3
run batch_timing 300 python -u tools/batch_timing.py 512 4096
run prof_c4 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c4 -o c4 -- python bench.py --no-cpu --steps 5 --warmup 2
python tools/timeline.py $OUT/prof_c4 > $OUT/timeline_c4.txt
run prof_c3 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c3 -o c3 -- python bench.py --config c3 --no-cpu --steps 5 --warmup 2
python tools/timeline.py $OUT/prof_c3 > $OUT/timeline_c3.txt
echo done >> $OUT/status.txt
