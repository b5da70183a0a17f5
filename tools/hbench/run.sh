# host-only: dr_append_rounds_packed's build (host_rounds.cpp) on the C4 DAG, 600 per-wave
# appends of 4 rounds, this tree's builder against the previous one (same output checksum)
cd $GRAFT_REPO_ROOT
mkdir -p /tmp/hbdata gpurun_out/hb
timeout -k 10 120 python3 -c "
import numpy as np
from dag_rider_amd.gen import CONFIGS, generate
d = generate(CONFIGS['c4'], nthreads=16)
for k in ('slot_off', 'slot_src', 'strong', 'weak_off', 'weak_tgt'):
    getattr(d, k).tofile('/tmp/hbdata/%s.bin' % k)
" || exit 1
for t in 16 8; do
  for o in 0 1 0 1; do
    echo -n "threads $t prev=$o: "; OMP_NUM_THREADS=$t timeout -k 5 60 tools/hbench/append_build_bench 600 $o || exit 1
  done
done
for o in 0 1; do echo -n "threads 16 prev=$o gap 200 us: "; OMP_NUM_THREADS=16 timeout -k 5 60 tools/hbench/append_build_bench 600 $o 200 || exit 1; done
echo -n "active wait: "; OMP_WAIT_POLICY=active OMP_NUM_THREADS=16 timeout -k 5 60 tools/hbench/append_build_bench 600 0
echo -n "passive wait: "; OMP_WAIT_POLICY=passive OMP_NUM_THREADS=16 timeout -k 5 60 tools/hbench/append_build_bench 600 0
