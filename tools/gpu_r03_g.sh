# GPU tests, facade (driver-thread pipeline): correctness, throughput at depth 1/2/4
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -2 gpurun_out/facade_test.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/facade_bench.log
for d in 2 1 4; do
  timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 --depth=$d >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench64k d$d failed"; exit 1; }
done
timeout -k 10 150 tests/cpp/build/facade_test --bench 256 16 64 --kib=1024 >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench1m failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 64 16 64 --kib=4096 >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench4m failed"; exit 1; }
cat gpurun_out/facade_bench.log
export TMPDIR=/tmp
rm -rf gpurun_out/segtrace
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/segtrace -o gen16 -- python3 tools/seg_bench.py "16 x 1 MiB generator" > gpurun_out/segtrace_gen16.log 2>&1; echo "gen16=$?"
cat gpurun_out/segtrace_gen16.log | tail -2
f=$(find gpurun_out/segtrace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-160 "$f" | head -25
