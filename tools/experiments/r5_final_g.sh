# round 5 final (g, the second stream created at the first fork): every GPU test, smoke, the default bench line (CPU legs included),
# its rocprofv3 kernel statistics -> gpurun_out/r5fa/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5fg
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c4.json 2> $O/bench_c4.err
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read()); print('c4', round(d['ms_per_step'],4), d['value'], d['roofline']['frac'], d['detail']['verify_vs_oracle'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
echo done
cp $O/prof_c4/run_kernel_stats.csv $O/kernel_stats_c4.csv 2>/dev/null || true
python3 tools/timeline.py $O/prof_c4 --last > $O/timeline_c4.txt 2>&1 || true
rm -rf $O/prof_c4
timeout -k 10 300 python3 -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err
python3 -c "import json; d=json.loads(open('$O/bench_c3.json').read()); print('c3', round(d['ms_per_step'],4), d['detail']['verify_vs_oracle'])"
timeout -k 10 300 python3 -u bench.py --rank-share 8 --no-cpu > $O/share8.json 2> $O/share8.err
timeout -k 10 300 python3 -u bench.py --colshard --no-cpu > $O/colshard1.json 2> $O/colshard1.err
python3 -c "import json; d=json.loads(open('$O/colshard1.json').read()); print('colshard1', round(d['detail']['colshard']['ms'],4), d['detail']['colshard']['verify_vs_unsharded'])"
timeout -k 10 400 python3 -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
python3 -c "import json; d=json.loads(open('$O/bench_c5.json').read()); print('c5', round(d['ms_per_step'],4), round(d['roofline']['ms_per_launch'],4), d['cpu_baseline']['bitset_all_dags']['matches_gpu'])"
echo done2
