# round 5 (h): exceptions to the regular graph (per-edge memo exceptions), full GPU suite,
# c4-far / c4-q8 lines verified against the bitset oracle, C3/C4 lines -> gpurun_out/r5h/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c4-far c4-q8; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 5 --warmup 2 --no-cpu --verify > $O/$c.json 2> $O/$c.err
  python3 -c "import json,sys; d=json.loads(open('$O/$c.json').read()); print('$c', round(d['ms_per_step'],4), d['detail']['verify_vs_oracle'], d['detail']['exceptions'], d['detail']['ms'])"
done
for c in c3 c4; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 3 --no-cpu > $O/$c.json 2> $O/$c.err
  python3 -c "import json,sys; d=json.loads(open('$O/$c.json').read()); print('$c', round(d['ms_per_step'],4), d['detail']['ms'])"
done
echo done
