# round 5 (aa): where the wave-form C5 kernel's time goes (phase stamps and cone-pass cycle
# counters of the profiling build) -> gpurun_out/r5aa/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 400 python3 -u tools/batch_timing.py 512 4096 > $O/batch_timing.jsonl 2> $O/batch_timing.err
cat $O/batch_timing.jsonl
echo done
