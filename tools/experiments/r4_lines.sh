# round 4: the bench lines (each under its own limit; one failure stops the script) -> gpurun_out/r4l_*.json
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l
mkdir -p $O
line() {  # name, limit, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
  echo "$name: $(python3 -c "import json,sys; d=json.load(open('$O/$name.json')); print(round(d['ms_per_step'],4), 'ms', d['roofline'].get('frac'), d['roofline'].get('bound'), (d.get('detail') or {}).get('verify_vs_oracle'))")"
}
line c4 400 --steps 20 --warmup 5
line c3 300 --config c3 --steps 20 --warmup 5 --no-cpu
line c4_deep 300 --config c4-deep --steps 5 --warmup 2 --no-cpu --verify
line c4_dups 300 --config c4-dups --steps 5 --warmup 2 --no-cpu --verify
line c4_nomemo 300 --no-memo --steps 3 --warmup 1 --no-cpu
line c5 300 --config c5 --steps 10 --warmup 2 --no-cpu
line c5_512 300 --config c5 --dags 512 --steps 20 --warmup 5 --no-cpu
line share8 200 --rank-share 8 --steps 20
line colshard1 300 --colshard --steps 20 --warmup 5 --no-cpu
