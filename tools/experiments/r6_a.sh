# round 6 (a): the shard continuation / staged-append / error tests, then the host-wait
# change measured both ways (DR_WAIT_SPIN_US: 200 = bounded spin then block, huge = the
# old pure spin) on the C4 line and the per-call loop -> gpurun_out/r6a/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 60 tools/experiments/launch_probe > $O/launch_probe.txt 2>&1
cat $O/launch_probe.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wsplit.py tests/test_gpu_shard.py tests/test_gpu_incremental.py tests/test_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
line() {  # name, env, args...
  local name=$1 spin=$2; shift 2
  DR_WAIT_SPIN_US=$spin timeout -k 10 300 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay')), d.get('provenance'))"
}
for N in 8 4 2; do
  DR_WAIT_SPIN_US=200 timeout -k 10 300 python3 -u bench.py --wave-split $N --steps 20 --warmup 3 > $O/wsplit$N.json 2> $O/wsplit$N.err
  python3 -c "import json; d=json.loads(open('$O/wsplit$N.json').read()); print('wsplit$N', round(d['ms_per_step'],4), d['detail']['verify_vs_unsharded'], [round(s['ms'],4) for s in d['detail']['shares']])"
done
line c4_spin200_a 200 --no-cpu --steps 50 --warmup 5
line c4_spinold_a 1000000000 --no-cpu --steps 50 --warmup 5
line c4_spin200_b 200 --no-cpu --steps 50 --warmup 5
line c4_spinold_b 1000000000 --no-cpu --steps 50 --warmup 5
line loop_spin200 200 --config c4-loop --steps 1 --warmup 0 --no-cpu
line loop_spinold 1000000000 --config c4-loop --steps 1 --warmup 0 --no-cpu
echo done
