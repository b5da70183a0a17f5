# round 6 final (c): provenance of the last tree -- smoke, the C4 and C5 lines, the loop
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ff
mkdir -p $O
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py --no-cpu --verify --steps 100 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 python3 bench.py --config c4-loop --no-cpu > $O/bench_loop.json 2> $O/bench_loop.err || exit 1
for f in bench_c4 bench_c5 bench_loop; do
  python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', round(d['ms_per_step'],4), d.get('provenance',{}).get('build_id'), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay')))"
done
echo done
