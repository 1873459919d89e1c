# facade zero-copy (decode of short-stream batches, encode input) vs the copy version (lib/h2d)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -2 gpurun_out/facade_test.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/facade_zc.log
for d in 2 1; do
  timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 --depth=$d >> gpurun_out/facade_zc.log 2>&1 || { echo "zc d$d failed"; exit 1; }
  LD_LIBRARY_PATH=$PWD/dwarfs_amd/lib/h2d timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 --depth=$d | sed 's/facade_bench/facade_bench_h2d/' >> gpurun_out/facade_zc.log 2>&1 || { echo "h2d d$d failed"; exit 1; }
done
timeout -k 10 150 tests/cpp/build/facade_test --bench 256 16 64 --kib=1024 >> gpurun_out/facade_zc.log 2>&1 || { echo "zc 1m failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 64 16 64 --kib=4096 >> gpurun_out/facade_zc.log 2>&1 || { echo "zc 4m failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 16 4 16 --kib=16384 >> gpurun_out/facade_zc.log 2>&1 || { echo "zc 16m failed"; exit 1; }
cat gpurun_out/facade_zc.log
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; echo "bench=$?"; tail -1 gpurun_out/bench.log | cut -c1-400
