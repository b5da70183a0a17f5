# round 6 final (a): the whole GPU suite, smoke, the default bench line (CPU legs), C4/C3/C5
# verified, c4-up against the general sweep, the per-call loop, the wave-split shares
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6fa}
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
step 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
step 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
line() {  # name, args...
  local name=$1; shift
  step 500 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); r=d.get('roofline') or {}; det=d['detail']; print('$name', round(d['ms_per_step'],4), r.get('frac'), det.get('verify_vs_oracle', det.get('verify_vs_replay', det.get('verify_vs_unsharded', det.get('verify_vs_general')))))"
}
line bench_default || exit 1
line bench_c4 --no-cpu --verify --steps 100 --warmup 5 || exit 1
line bench_c3 --config c3 --no-cpu --verify --steps 100 --warmup 5 || exit 1
line bench_c5 --config c5 --steps 20 --warmup 3 || exit 1
line bench_c4up --config c4-up --no-cpu --verify-general --steps 20 --warmup 2 || exit 1
line bench_loop --config c4-loop --steps 1 --warmup 0 --no-cpu || exit 1
line wsplit8 --wave-split 8 --steps 20 --warmup 3 || exit 1
line wsplit4 --wave-split 4 --steps 20 --warmup 3 || exit 1
line wsplit2 --wave-split 2 --steps 20 --warmup 3 || exit 1
echo done
