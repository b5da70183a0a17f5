# round 5 (x): rocprof kernel statistics of the N = 8 share line (k_commit's device time
# against its HIP-event time) -> gpurun_out/r5x/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --rank-share 8 --no-cpu > $O/share8.json 2> $O/share8.err
cp $O/prof/run_kernel_stats.csv $O/kernel_stats_share8.csv
python3 tools/timeline.py $O/prof --last --start k_commit > $O/timeline_share8.txt 2>&1 || true
rm -rf $O/prof
head -5 $O/kernel_stats_share8.csv | cut -c1-200
echo done
