# Decode check: the fs 8-13 and segmented-decode tests (verbose), the other decode tests, the
# long-stream layouts (seg_bench), the bench line and the generator workload
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "high_rice or segmented_decode" > gpurun_out/pytest_seg.log 2>&1; rc=$?; echo "pytest_seg=$rc"
tail -5 gpurun_out/pytest_seg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "decode or large or configs3 or truncated or corrupt or rice or full_size" > gpurun_out/pytest_dec.log 2>&1; rc=$?; echo "pytest_dec=$rc"
tail -3 gpurun_out/pytest_dec.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/seg_bench.py > gpurun_out/seg_bench.jsonl 2>&1; rc=$?; echo "seg_bench=$rc"
cut -c1-220 gpurun_out/seg_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python tools/workloads.py gen > gpurun_out/gen.jsonl 2>&1; echo "gen=$?"
cat gpurun_out/gen.jsonl
