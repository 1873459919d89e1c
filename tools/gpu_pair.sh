# Paired decode: its parity tests, bench A/B (fused vs paired), facade test + throughput, then the whole GPU suite
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "paired" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pair.log 2>&1; rc=$?; echo "pytest_pair=$rc"
grep -E "passed|failed|Error|error|assert" gpurun_out/pytest_pair.log | tail -15
[ $rc -eq 0 ] || exit $rc
for path in fused paired fused paired; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --decode-path $path > gpurun_out/bench_$path.log 2>&1 || exit 1
  python -c "import json,sys; j=json.loads(open('gpurun_out/bench_$path.log').read().strip().splitlines()[-1]); c=j['config']; print('$path', j['value'], c['encode_kernel_us'], c['decode_kernel_us'])"
done
timeout -k 10 120 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; echo "facade_test=$?"; tail -2 gpurun_out/facade_test.log
timeout -k 10 300 tests/cpp/build/facade_test --bench 4096 1 8 64 > gpurun_out/facade_bench.log 2>&1; echo "facade_bench=$?"
cat gpurun_out/facade_bench.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest_all=$rc"
grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -8
exit $rc
