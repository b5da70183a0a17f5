# round 6: the C4 line three times on one box (host-side spread between boxes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6rep
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu --steps 200 --warmup 5 > $O/c4_$i.json 2> $O/c4_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); print('c4 run $i', round(d['ms_per_step'],4), d['provenance']['build_id'])"
done
echo done
