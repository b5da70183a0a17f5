# round 5 (w): k_commit with every row load of a wave in flight at once: the commit tests,
# the N = 8 share line, the per-call loop -> gpurun_out/r5w/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "commit or wave or split or parity or golden" > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --rank-share 8 --no-cpu > $O/share8.json 2> $O/share8.err
python3 -c "import json; d=json.loads(open('$O/share8.json').read()); r=d['roofline']; print('share8', round(d['ms_per_step'],4), round(r['ms_per_launch']*1e3,2), 'us', round(r['frac'],3), d['detail'].get('verify_vs_full_replay', d['detail'].get('verify')))"
timeout -k 10 300 python3 -u bench.py --config c4-loop --steps 1 --warmup 0 --no-cpu > $O/loop.json 2> $O/loop.err
python3 -c "import json; d=json.loads(open('$O/loop.json').read()); print({k: round(v['p50'],1) for k, v in d['detail']['latency_us'].items()}, d['detail']['verify_vs_replay'])"
echo done
