# per-kernel times of the segmented decode (rocprofv3 kernel trace) for a few layouts
mkdir -p gpurun_out/segprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/segprof -o run -- python3 $GRAFT_REPO_ROOT/tools/seg_bench.py "16 x 1" "mix" "Poisson stream" > $GRAFT_REPO_ROOT/gpurun_out/segprof/bench.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT
echo "rc=$rc"; tail -4 gpurun_out/segprof/bench.log
f=$(find gpurun_out/segprof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -30
exit $rc
