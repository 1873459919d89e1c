# segmented decode at bs 512 / other bs: parity, then seg_bench bs 512 and 128
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "segmented or bs512 or other_block" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seg.log 2>&1; rc=$?; echo "pytest=$rc"
grep -E "passed|failed|Error|error" gpurun_out/pytest_seg.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/seg_bench.py --bs=512 "16 MiB Poisson" "generator stream" "16 x 1 MiB" > gpurun_out/seg_bench512.jsonl 2> gpurun_out/seg_bench.err; echo "seg_bench512=$?"; cat gpurun_out/seg_bench512.jsonl
timeout -k 10 200 python tools/seg_bench.py --bs=256 "16 MiB Poisson" > gpurun_out/seg_bench256.jsonl 2>> gpurun_out/seg_bench.err; echo "seg_bench256=$?"; cat gpurun_out/seg_bench256.jsonl
timeout -k 10 300 python tools/seg_bench.py > gpurun_out/seg_bench128.jsonl 2>> gpurun_out/seg_bench.err; echo "seg_bench128=$?"; cat gpurun_out/seg_bench128.jsonl
