# iteration: decode timing (bench workload, 1 wave/SIMD and 4 waves/SIMD), then the GPU parity tests
mkdir -p gpurun_out
for a in "4096 16" "1024 4"; do timeout -k 10 120 python tools/occ_run.py $a 2>&1 | tail -1 || exit 1; done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -5 gpurun_out/pytest_gpu.log
exit $rc
