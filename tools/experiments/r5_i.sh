# round 5 (i): C3 A/B of k_canon_prefix's tile form vs the run form, kernel traces -> gpurun_out/r5i/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5i
mkdir -p $O
for rep in 1 2; do
  for t in 1 0; do
    DR_CANON_TILES=$t timeout -k 10 300 python3 -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu > $O/c3_t${t}_$rep.json 2> $O/c3_t${t}_$rep.err
    python3 -c "import json; d=json.loads(open('$O/c3_t${t}_$rep.json').read()); print('c3 tiles=$t rep $rep', round(d['ms_per_step'],4))"
  done
done
for t in 1 0; do
  DR_CANON_TILES=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_t$t -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu > $O/prof_t$t.json 2> $O/prof_t$t.err
done
python3 tools/timeline.py $O/prof_t1 > $O/timeline_t1.txt 2>&1 || true
python3 tools/timeline.py $O/prof_t0 > $O/timeline_t0.txt 2>&1 || true
echo done
