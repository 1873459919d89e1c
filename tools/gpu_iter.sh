# quick iteration: parity tests + bench (no CPU baseline); stops at the first GPU failure
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout=240 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; echo "bench=$?"
  tail -3 gpurun_out/bench.log
fi
