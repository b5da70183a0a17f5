# round 5 (ag): k_canon with the first row group of each walked round loaded a round ahead; the prefix
# microbenchmark, every GPU test, C3/C4 lines with timelines -> gpurun_out/r5v/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ag
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c3 c4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 50 --warmup 10 --no-cpu --verify > $O/$c.json 2> $O/$c.err
  python3 -c "import json; d=json.loads(open('$O/$c.json').read()); print('$c', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle'))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu > $O/prof_$c.json 2> $O/prof_$c.err
  python3 tools/timeline.py $O/prof_$c --last > $O/timeline_$c.txt 2>&1 || true
  cp $O/prof_$c/run_kernel_stats.csv $O/kernel_stats_$c.csv 2>/dev/null || true
  rm -rf $O/prof_$c
  grep "k_canon<" $O/kernel_stats_$c.csv | cut -d, -f1,4
done
echo done
