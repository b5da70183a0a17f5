# round 5 (u): the per-call loop after DevBuf::ensure's geometric growth (no hipFree per
# call); its HIP API trace around one wave; the default C4 line -> gpurun_out/r5u/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop.json 2> $O/loop.err
python3 -c "import json; d=json.loads(open('$O/loop.json').read()); print({k: round(v['p50'],1) for k, v in d['detail']['latency_us'].items()}, d['detail']['verify_vs_replay'])"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/api_loop -o run -- python3 bench.py --config c4-loop --loop-waves 40 --steps 1 --warmup 0 --no-cpu > $O/api_loop.json 2> $O/api_loop.err
python3 tools/apitrace.py $O/api_loop k_round_summary 3 900 > $O/apitrace_loop.txt 2>&1 || true
rm -rf $O/api_loop
timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 10 --no-cpu > $O/c4.json 2> $O/c4.err
python3 -c "import json; d=json.loads(open('$O/c4.json').read()); print('c4', round(d['ms_per_step'],4))"
echo done
