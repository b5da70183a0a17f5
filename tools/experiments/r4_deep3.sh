# round 4: c4-deep -- k_canon segment stats, the bench line, kernel medians
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d8
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dups.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 -u tools/canon_timing.py c4-deep c4 c3 > $O/canon.jsonl 2> $O/canon.err && timeout -k 10 200 python3 -u tools/sweep_timing.py c4-deep > $O/sweep.json 2>&1
cat $O/canon.jsonl
timeout -k 10 300 python3 -u bench.py --config c4-deep --steps 10 --warmup 2 --no-cpu --verify > $O/deep.json 2> $O/deep.err
timeout -k 10 300 python3 -u bench.py --steps 50 --warmup 5 --no-cpu --verify > $O/c4.json 2> $O/c4.err
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', d['ms_per_step'], d['detail'].get('verify_vs_oracle'))"
python3 -c "import json; d=json.load(open('$O/deep.json')); print(d['ms_per_step'], d['detail'].get('verify_vs_oracle'))"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu > $O/prof.json 2> $O/prof.err
python3 tools/prof_db.py $(find $O/prof -name run_results.db | head -1) > $O/deep_kernels.txt
head -10 $O/deep_kernels.txt
