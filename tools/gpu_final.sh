# Round-end GPU session: all GPU tests, the default bench (CPU baseline included),
# a kernel trace of the bench, and the PMC passes for profiles/pmc_latest.json
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench=$rc"; tail -1 gpurun_out/bench_full.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof/trace.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh
