cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab1
mkdir -p $O
timeout -k 10 200 python3 tools/sweep_timing.py c4 > $O/r6_c4.json 2> $O/r6_c4.err || exit 1
(cd ab_r5 && timeout -k 10 200 python3 tools/sweep_timing.py c4) > $O/r5_c4.json 2> $O/r5_c4.err || exit 1
echo done
