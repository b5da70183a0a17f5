# round 5 (n): the per-call loop (c4-loop) with the append's phases; a kernel trace of a
# short loop; the c4-up general-sweep line; C5 with the form label -> gpurun_out/r5n/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop.json 2> $O/loop.err
python3 -c "import json; d=json.loads(open('$O/loop.json').read()); print({k: round(v['p50'],1) for k, v in d['detail']['latency_us'].items()}, d['detail']['verify_vs_replay'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_loop -o run -- python3 bench.py --config c4-loop --loop-waves 40 --steps 1 --warmup 0 --no-cpu > $O/prof_loop.json 2> $O/prof_loop.err
python3 tools/timeline.py $O/prof_loop --last --start k_round_summary > $O/timeline_loop.txt 2>&1 || true
timeout -k 10 300 python3 -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu > $O/c5.json 2> $O/c5.err
python3 -c "import json; d=json.loads(open('$O/c5.json').read()); print('c5', round(d['ms_per_step'],4), d['roofline']['kernel'], d['roofline']['bound'], round(d['roofline']['ms_per_launch'],4))"
timeout -k 10 300 python3 -u bench.py --config c5 --dags 512 --steps 5 --warmup 2 --no-cpu > $O/c5_512.json 2> $O/c5_512.err
python3 -c "import json; d=json.loads(open('$O/c5_512.json').read()); print('c5/512', round(d['ms_per_step'],4), d['roofline']['kernel'], d['roofline']['bound'], round(d['roofline']['ms_per_launch'],4))"
timeout -k 10 600 python3 -u bench.py --config c4-up --steps 1 --warmup 1 --no-cpu > $O/c4up.json 2> $O/c4up.err
python3 -c "import json; d=json.loads(open('$O/c4up.json').read()); print('c4-up', round(d['ms_per_step'],3), d['detail']['exceptions'], d['detail']['ms'])"
echo done
