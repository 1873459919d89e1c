# kernel trace of the long-stream workloads (whole frames, block mix)
mkdir -p gpurun_out/segprof2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segprof2 -o run -- python3 tools/workloads.py frames mix > gpurun_out/segprof2/wl.log 2>&1; rc=$?
echo "rc=$rc"; grep case gpurun_out/segprof2/wl.log
grep -E "rpp_" gpurun_out/segprof2/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
exit $rc
