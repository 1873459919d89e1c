mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=240 -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
fi
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --cpu-seconds 3 > gpurun_out/bench.log 2>&1; echo "bench=$?"
fi
tail -3 gpurun_out/smoke.log; tail -30 gpurun_out/pytest_gpu.log; tail -5 gpurun_out/bench.log
