# facade throughput: 4096 x 64 KiB at 16/64/256 threads, 256 x 1 MiB at 64 threads
mkdir -p gpurun_out
timeout -k 10 300 tests/cpp/build/facade_test --bench 4096 16 64 256 > gpurun_out/facade_bench.log 2>&1; echo "facade_bench=$?"
timeout -k 10 300 tests/cpp/build/facade_test --bench 256 64 --kib=1024 >> gpurun_out/facade_bench.log 2>&1; echo "facade_bench1m=$?"
cat gpurun_out/facade_bench.log
