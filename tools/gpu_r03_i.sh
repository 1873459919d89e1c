# graph-replayed bench step vs eager; the graph-replay parity test; the facade as built (copies for encode, zero-copy short-stream decode)
mkdir -p gpurun_out
timeout -k 10 160 python -u -m pytest tests/test_gpu_host_pipeline.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k graph > gpurun_out/pytest_graph.log 2>&1; rc=$?; echo "pytest_graph=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_graph.log | head -8
for v in graph eager graph eager; do
  if [ $v = graph ]; then a=""; else a="--no-graph"; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["encode_kernel_us"], c["decode_kernel_us"], c.get("step_launch"))')"
done
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -2 gpurun_out/facade_test.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/facade_final.log
timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 >> gpurun_out/facade_final.log 2>&1 || { echo "64k failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 256 16 64 --kib=1024 >> gpurun_out/facade_final.log 2>&1 || { echo "1m failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 64 16 64 --kib=4096 >> gpurun_out/facade_final.log 2>&1 || { echo "4m failed"; exit 1; }
timeout -k 10 150 tests/cpp/build/facade_test --bench 16 4 16 --kib=16384 >> gpurun_out/facade_final.log 2>&1 || { echo "16m failed"; exit 1; }
cat gpurun_out/facade_final.log
