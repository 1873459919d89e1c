# Facade throughput (1/16/64 threads) after the queue changes; paired vs fused at 8192 x 32 KiB and 16384 x 16 KiB
mkdir -p gpurun_out
timeout -k 10 120 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; echo "facade_test=$?"; tail -2 gpurun_out/facade_test.log
timeout -k 10 300 tests/cpp/build/facade_test --bench 4096 1 16 64 > gpurun_out/facade_bench.log 2>&1; echo "facade_bench=$?"
cat gpurun_out/facade_bench.log
for cfgs in "8192 32768" "16384 16384"; do
  set -- $cfgs
  for path in fused paired; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --blocks $1 --block-bytes $2 --decode-path $path > gpurun_out/bench_${1}_$path.log 2>&1 || exit 1
    python -c "import json,sys; j=json.loads(open('gpurun_out/bench_${1}_$path.log').read().strip().splitlines()[-1]); c=j['config']; print('$1x$2 $path', j['value'], c['encode_kernel_us'], c['decode_kernel_us'])"
  done
done
