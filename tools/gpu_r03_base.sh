# Round-3 baseline: GPU tests, bench (with CPU baseline), kernel trace of the bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/trace.log 2>&1; echo "trace=$?"
grep -E "rpp_" gpurun_out/trace/run_kernel_stats.csv | cut -c1-200
