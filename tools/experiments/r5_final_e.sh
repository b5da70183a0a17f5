# round 5 final (e): smoke and the default bench line (CPU legs included) on the final tree
# (the full GPU test suite ran on this source as r5af) -> gpurun_out/r5fe/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5fe
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench_c4.json 2> $O/bench_c4.err
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read()); print('c4', round(d['ms_per_step'],4), d['value'], d['roofline']['frac'], d['detail']['verify_vs_oracle'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $O/prof_c4.json 2> $O/prof_c4.err
cp $O/prof_c4/run_kernel_stats.csv $O/kernel_stats_c4.csv
rm -rf $O/prof_c4
echo done
