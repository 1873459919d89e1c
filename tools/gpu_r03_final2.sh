# final tree check: GPU tests, smoke, facade test
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -1 gpurun_out/facade_test.log
