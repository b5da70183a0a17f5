# round 6 (c): the launch-cost probe, the whole GPU suite (static pop queries, wave split,
# shard continuation), the wave-split shares, the C4/C3 lines with timelines, and the
# host-wait change measured both ways -> gpurun_out/r6c/
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
line() {  # name, env spin, args...
  local name=$1 spin=$2; shift 2
  DR_WAIT_SPIN_US=$spin timeout -k 10 300 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay', d['detail'].get('verify_vs_unsharded'))), [round(s['ms'],4) for s in d['detail'].get('shares', [])])"
}
line wsplit8 200 --wave-split 8 --steps 20 --warmup 3 || exit 1
line wsplit4 200 --wave-split 4 --steps 20 --warmup 3 || exit 1
line wsplit2 200 --wave-split 2 --steps 20 --warmup 3 || exit 1
line c4_a 200 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line c3_a 200 --config c3 --no-cpu --verify --steps 50 --warmup 5 || exit 1
line c4up 200 --config c4-up --no-cpu --steps 20 --warmup 2 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c4 -o c4 -- python3 bench.py --no-cpu --steps 5 --warmup 2 > $O/prof_c4.json 2> $O/prof_c4.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu --steps 5 --warmup 2 > $O/prof_c3.json 2> $O/prof_c3.err || exit 1
echo done
