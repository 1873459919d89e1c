# kernel trace of the segmented decode on single long streams and 16 x 1 MiB (bs 128)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/segtrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o gen -- python3 tools/seg_bench.py "16 MiB generator stream" > gpurun_out/segtrace_gen.log 2>&1; echo "gen=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o gen16 -- python3 tools/seg_bench.py "16 x 1 MiB generator" > gpurun_out/segtrace_gen16.log 2>&1; echo "gen16=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o poi -- python3 tools/seg_bench.py "16 MiB Poisson stream" > gpurun_out/segtrace_poi.log 2>&1; echo "poi=$?"
find gpurun_out/segtrace -name "*.csv" | head -20
