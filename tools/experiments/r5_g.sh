# round 5 (g): stepped replay (vote before the walk, separate emission; STEP_NT=128 variant)
# + register-resident leader chains (k_chain_reg, n <= 256): parity, goldens, C3/C4 lines
# -> gpurun_out/r5g/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
summ() { python3 -c "
import json,sys
for l in open('$1'):
    d=json.loads(l); print('$2', d['G'], d['form'], round(d['ms_wall_median'],4), d['replay_ok'], d['steps'], d.get('host_syncs'), {k: round(v,4) for k,v in d['phases_ms'].items()})
"; }
timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 > $O/shard.jsonl 2>&1
summ $O/shard.jsonl base
DR_SHARD_STEP_NT=128 timeout -k 10 300 python3 -u tools/shard_replay_bench.py --runs 20 --stepped 1 > $O/shard_nt128.jsonl 2>&1
summ $O/shard_nt128.jsonl nt128
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { echo "$name FAILED"; tail -5 $O/bench_$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/bench_$name.json')); print(round(d['ms_per_step'],4), 'ms', d['roofline'].get('frac'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c3 300 --config c3 --steps 20 --warmup 5 --no-cpu --verify
DR_CHAIN_REG=0 timeout -k 10 300 python3 -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu > $O/bench_c3_noreg.json 2> $O/bench_c3_noreg.err
python3 -c "import json; d=json.load(open('$O/bench_c3_noreg.json')); print('c3 chain_reg=0:', round(d['ms_per_step'],4))"
line c4 300 --steps 20 --warmup 5 --no-cpu
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu > $O/prof_c3.json 2> $O/prof_c3.err
echo done
