# round 5 (ah, no degree scratch in the wave form: 127 VGPRs, no spill): two prefetch register sets, branch-free prefetch, pinned current words; (ab): the wave-form C5 kernel with its offsets and leaders in registers: batch
# tests, phase timings, C5 lines -> gpurun_out/r5ah/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5ah
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u tools/batch_timing.py 512 4096 > $O/batch_timing.jsonl 2> $O/batch_timing.err
python3 -c "
import json
for l in open('$O/batch_timing.jsonl'):
    d=json.loads(l)
    if d['form']=='wave': print(d['dags'], 'wave', round(d['kernel_ms'],3), d['cone_pass_us']['mean'], d['emission_us']['mean'], d['cone_pass_cycles_mean'])
"
timeout -k 10 300 python3 -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu > $O/c5.json 2> $O/c5.err
python3 -c "import json; d=json.loads(open('$O/c5.json').read()); print('c5', round(d['ms_per_step'],4), round(d['roofline']['ms_per_launch'],4), d['roofline']['kernel'])"
timeout -k 10 300 python3 -u bench.py --config c5 --dags 512 --steps 20 --warmup 3 --no-cpu > $O/c5_512.json 2> $O/c5_512.err
python3 -c "import json; d=json.loads(open('$O/c5_512.json').read()); print('c5/512', round(d['ms_per_step'],4), round(d['roofline']['ms_per_launch'],4), d['roofline']['kernel'])"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c5_fetch -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/pmc_c5_fetch.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5_write -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/pmc_c5_write.log 2>&1
python3 tools/pmc_traffic.py $O/pmc_c5_fetch/run_counter_collection.csv $O/pmc_c5_write/run_counter_collection.csv > $O/traffic_c5.json
grep -A3 replay_small $O/traffic_c5.json
echo done
