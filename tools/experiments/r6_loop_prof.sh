# round 6: kernel and HIP API trace of the per-call loop (60 waves) on the final tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6lp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/prof_loop -o loop -- python3 bench.py --config c4-loop --no-cpu --loop-waves 60 > $O/prof_loop.json 2> $O/prof_loop.err || { tail -20 $O/prof_loop.err; exit 1; }
echo done
