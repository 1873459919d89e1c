# Two-stage decode: parity tests first (stop at first failure), then the bench and a kernel trace
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1; rc=$?; echo "bench=$rc"
tail -2 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/trace.log 2>&1; echo "trace=$?"
cat gpurun_out/trace/*/run_kernel_stats.csv 2>/dev/null | head -20 || find gpurun_out/trace -name "*stats*"
