# bs 512 / 256 / 128 long streams (seg_bench), then the segmented parity tests and the GPU suite
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/seg_bench.py --bs=512 "16 MiB Poisson stream" "16 MiB generator stream" "8 x 4 MiB" > gpurun_out/segb512.log 2>&1; echo "segb512=$?"
cut -c1-250 gpurun_out/segb512.log | grep layout
timeout -k 10 300 python3 -u tools/seg_bench.py --bs=256 "16 MiB Poisson stream" "16 MiB generator stream" > gpurun_out/segb256.log 2>&1; echo "segb256=$?"
cut -c1-250 gpurun_out/segb256.log | grep layout
timeout -k 10 300 python3 -u tools/seg_bench.py "16 MiB Poisson stream" "16 MiB generator stream" "16 x 1 MiB generator" > gpurun_out/segb128.log 2>&1; echo "segb128=$?"
cut -c1-250 gpurun_out/segb128.log | grep layout
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "segmented or bs512 or other_block" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seg.log 2>&1; rc=$?; echo "pytest=$rc"
tail -2 gpurun_out/pytest_seg.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_tests.sh
