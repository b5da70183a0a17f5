# round 5 final (h): the C4 variant lines on the last tree, verified against the bitset
# oracle, and the per-call loop -> gpurun_out/r5fh/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5fh
mkdir -p $O
line() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/$name.json 2> $O/$name.err
  python3 -c "import json; d=json.loads(open('$O/$name.json').read()); print('$name', round(d['ms_per_step'],4), d['detail'].get('verify_vs_oracle', d['detail'].get('verify_vs_replay')))"
}
line c4far --config c4-far --no-cpu --verify
line c4q8 --config c4-q8 --no-cpu --verify
line c4deep --config c4-deep --no-cpu --verify
line c4dups --config c4-dups --no-cpu --verify
line c2 --config c2 --no-cpu --verify
line loop --config c4-loop --steps 1 --warmup 0 --no-cpu
echo done
