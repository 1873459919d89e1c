# kernel trace of the segmented decode of one 16 MiB stream at bs 512
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/segtrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o p512 -- python3 tools/seg_bench.py --bs=512 "16 MiB Poisson stream" > gpurun_out/segtrace_p512.log 2>&1; echo "p512=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o gen -- python3 tools/seg_bench.py "16 MiB generator stream" > gpurun_out/segtrace_gen.log 2>&1; echo "gen=$?"
