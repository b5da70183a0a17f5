# round 6: PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes) of the C4, C3 and C5
# bench lines -> gpurun_out/r6_pmc/; tools/pmc_traffic.py merges them into profiles/r06/traffic.json
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6_pmc
mkdir -p $O
for cfg in c4 c3 c5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${cfg}_$ctr -o run -- python3 bench.py --config $cfg --no-cpu --steps 2 --warmup 1 > $O/${cfg}_$ctr.json 2> $O/${cfg}_$ctr.err || { echo "$cfg $ctr failed"; exit 1; }
    echo "$cfg $ctr ok"
  done
done
echo done
