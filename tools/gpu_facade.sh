# facade throughput: 4096 x 64 KiB at 16/64/256 threads; 256 x 1 MiB and 64 x 4 MiB (mkdwarfs -S 22) at 16/64 threads
mkdir -p gpurun_out
timeout -k 10 300 tests/cpp/build/facade_test --bench 4096 16 64 256 > gpurun_out/facade_bench.log 2>&1; echo "facade_bench=$?"
timeout -k 10 300 tests/cpp/build/facade_test --bench 256 16 64 --kib=1024 >> gpurun_out/facade_bench.log 2>&1; echo "facade_bench1m=$?"
timeout -k 10 300 tests/cpp/build/facade_test --bench 64 16 64 --kib=4096 >> gpurun_out/facade_bench.log 2>&1; echo "facade_bench4m=$?"
cat gpurun_out/facade_bench.log
