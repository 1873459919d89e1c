# GPU check of the segmented decode: its tests first (verbose), then the decode tests around it
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "segmented_decode" > gpurun_out/pytest_seg.log 2>&1; rc=$?; echo "pytest_seg=$rc"
tail -25 gpurun_out/pytest_seg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "decode or large or configs3 or truncated or corrupt" > gpurun_out/pytest_dec.log 2>&1; rc=$?; echo "pytest_dec=$rc"
tail -8 gpurun_out/pytest_dec.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_bench.jsonl 2>&1; rc=$?; echo "seg_bench=$rc"
cat gpurun_out/seg_bench.jsonl
exit $rc
