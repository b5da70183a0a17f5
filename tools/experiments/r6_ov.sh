# round 6: DR_OPT_CALL_OVERLAP (the canonical cone forked in dr_wave_ready): per-call tests,
# then the c4-loop line with the overlap on and off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6ov
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for ov in 1 1; do
  DR_CALL_OVERLAP=$ov timeout -k 10 300 python3 bench.py --config c4-loop --no-cpu > $O/loop_ov$ov.json 2> $O/loop_ov$ov.err && cp $O/loop_ov$ov.json $O/loop_ov${ov}_$SECONDS.json || { tail -20 $O/loop_ov$ov.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/loop_ov$ov.json')); l=d['detail']['latency_us']
print('ov$ov', round(d['ms_per_step'],1), d['detail']['verify_vs_replay'], {k: round(v['p50'],1) for k,v in l.items()})"
done
echo done
