# round 6: the C5 batch's output copy by k_copy into the mapped pinned region vs the DMA engine
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6bc
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_batch.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in kernel dma kernel dma; do
  DR_BATCH_COPY=$m timeout -k 10 300 python3 bench.py --config c5 --no-cpu --steps 20 --warmup 3 > $O/c5_$m.json 2> $O/c5_$m.err || { tail -20 $O/c5_$m.err; exit 1; }
  cp $O/c5_$m.json $O/c5_${m}_$SECONDS.json
  python3 -c "
import json; d=json.load(open('$O/c5_$m.json')); p=d['detail']['step_phases_ms']; print('$m', round(d['ms_per_step'],4), {k: round(v,4) for k,v in p.items()})"
done
echo done
