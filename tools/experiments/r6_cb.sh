# round 6: k_copy workgroup size (bytes per workgroup) on the per-call loop's append copy
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6cb
mkdir -p $O
for b in 4096 1024 512 4096 1024 512; do
  DR_COPY_BLK=$b timeout -k 10 300 python3 bench.py --config c4-loop --no-cpu > $O/loop_$b.json 2> $O/loop_$b.err || { tail -20 $O/loop_$b.err; exit 1; }
  cp $O/loop_$b.json $O/loop_${b}_$SECONDS.json
  python3 -c "
import json; d=json.load(open('$O/loop_$b.json')); l=d['detail']['latency_us']
print('blk $b', round(d['ms_per_step'],1), d['detail']['verify_vs_replay'], {k: round(v['p50'],1) for k,v in l.items()})"
done
DR_COPY_BLK=1024 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o loop -- python3 bench.py --config c4-loop --no-cpu --loop-waves 60 > $O/prof.json 2> $O/prof.err || exit 1
echo done
