# kernel trace of the segmented decode of one 16 MiB generator stream
mkdir -p gpurun_out/segprof3
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segprof3 -o run -- python3 tools/seg_bench.py generator > gpurun_out/segprof3/b.log 2>&1; rc=$?
echo "rc=$rc"; grep layout gpurun_out/segprof3/b.log | cut -c1-300
exit $rc
