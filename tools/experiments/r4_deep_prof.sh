set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4dp -o run -- python3 bench.py --config c4-deep --steps 5 --warmup 2 --no-cpu > gpurun_out/r4dp.json 2> gpurun_out/r4dp.err
echo ok
