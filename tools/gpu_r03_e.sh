# decode entry-state A/B (main / spec1 / spec2), then the facade pipeline (correctness + throughput, depth sweep)
mkdir -p gpurun_out
for v in main spec1 spec2 main spec1 spec2; do
  if [ "$v" = main ]; then lib=dwarfs_amd/lib/libricepp_amd.so; else lib=dwarfs_amd/lib/libricepp_amd_$v.so; fi
  RICEPP_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["encode_kernel_us"], c["decode_kernel_us"])')"
done
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -3 gpurun_out/facade_test.log
[ $rc -eq 0 ] || exit $rc
for d in 4 2 8; do
  timeout -k 10 150 tests/cpp/build/facade_test --bench 4096 16 64 --depth=$d >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench64k d$d failed"; exit 1; }
  tail -2 gpurun_out/facade_bench.log
done
timeout -k 10 150 tests/cpp/build/facade_test --bench 256 16 64 --kib=1024 >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench1m failed"; exit 1; }
tail -2 gpurun_out/facade_bench.log
timeout -k 10 150 tests/cpp/build/facade_test --bench 64 16 64 --kib=4096 >> gpurun_out/facade_bench.log 2>&1 || { echo "facade_bench4m failed"; exit 1; }
tail -2 gpurun_out/facade_bench.log
