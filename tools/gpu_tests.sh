# GPU test suite only (stops at the first failure)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -15
exit $rc
