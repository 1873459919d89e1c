# segmented decode on single long streams: parse diagnostics, seg_bench (bs 128, 512), then the GPU suite
mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/seg_parse_diag.py > gpurun_out/diag.log 2>&1; echo "diag=$?"
tail -3 gpurun_out/diag.log
timeout -k 10 300 python3 -u tools/seg_bench.py "16 MiB generator stream" "16 MiB Poisson stream" "16 x 1 MiB generator" > gpurun_out/segb.log 2>&1; echo "segb=$?"
tail -3 gpurun_out/segb.log
timeout -k 10 300 python3 -u tools/seg_bench.py --bs=512 "16 MiB Poisson stream" "16 x 1 MiB Poisson" "8 x 4 MiB" > gpurun_out/segb512.log 2>&1; echo "segb512=$?"
tail -3 gpurun_out/segb512.log
bash tools/gpu_tests.sh
