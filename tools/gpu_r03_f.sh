# stream concurrency of small decode/encode launches; facade at pipeline depth 1
mkdir -p gpurun_out
timeout -k 10 120 tools/stream_overlap > gpurun_out/stream_overlap.jsonl 2>&1; echo "overlap=$?"; cat gpurun_out/stream_overlap.jsonl
timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 --depth=1 > gpurun_out/facade_bench_d1.log 2>&1; echo "facade_d1=$?"; cat gpurun_out/facade_bench_d1.log
