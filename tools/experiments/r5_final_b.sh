# round 5 final (b): the other config lines and the PMC passes -> gpurun_out/r5fb/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5fb
mkdir -p $O
line() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay')))"
}
line c3 --config c3
line c2 --config c2
line c1 --config c1
line c5 --config c5
line c5_512 --config c5 --dags 512 --no-cpu
line c4far --config c4-far --no-cpu --verify
line c4q8 --config c4-q8 --no-cpu --verify
line c4deep --config c4-deep --no-cpu --verify
line c4dups --config c4-dups --no-cpu --verify
line loop --config c4-loop --steps 1 --warmup 0 --no-cpu
line share8 --rank-share 8 --no-cpu
line colshard1 --colshard --no-cpu
for c in c4 c3 c5; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu > $O/pmc_${c}_fetch.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu > $O/pmc_${c}_write.log 2>&1
done
echo done
