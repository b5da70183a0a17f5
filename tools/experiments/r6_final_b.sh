# round 6 final (b): rocprof kernel statistics and timelines of the C4, C3 and C5 lines, the PMC
# traffic passes of C4 and C3 (and C4 with the XCD-grouped delivery queries, DR_FUSE=31)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6fb}
mkdir -p $O
step() { local t=$1; shift; echo "[step] $*" >&2; timeout -k 10 $t "$@"; }
for cfg in c4 c3 c5; do
  step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o $cfg -- python3 bench.py --config $cfg --no-cpu --steps 5 --warmup 2 > $O/prof_$cfg.json 2> $O/prof_$cfg.err || exit 1
  echo "prof $cfg ok"
done
for cfg in c4 c3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${cfg}_$ctr -o run -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 > $O/${cfg}_$ctr.json 2> $O/${cfg}_$ctr.err || { echo "$cfg $ctr failed"; exit 1; }
    echo "$cfg $ctr ok"
  done
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  DR_FUSE=31 timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/c4x_$ctr -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $O/c4x_$ctr.json 2> $O/c4x_$ctr.err || { echo "c4x $ctr failed"; exit 1; }
  echo "c4x $ctr ok"
done
echo done
