# GPU check: parity tests (stop at first failure), C++ facade test and facade throughput
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/cpp/build/facade_test --bench 4096 1 8 64 > gpurun_out/facade_bench.log 2>&1; echo "facade_bench=$?"
cat gpurun_out/facade_bench.log
