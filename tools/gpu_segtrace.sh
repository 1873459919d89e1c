# kernel trace of the segmented decode on single long streams (bs 128 and 512)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/segtrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o s128 -- python3 tools/seg_bench.py "16 MiB generator stream" "16 MiB Poisson stream" > gpurun_out/segtrace.log 2>&1; echo "trace128=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o s512 -- python3 tools/seg_bench.py --bs=512 "16 x 1 MiB Poisson" > gpurun_out/segtrace512.log 2>&1; echo "trace512=$?"
ls gpurun_out/segtrace
