# quick iteration: parity tests (stop at first failure) + short bench, no CPU baseline
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; echo "bench=$?"
tail -2 gpurun_out/bench.log
