# Two-stage vs fused decode: parity subset, bench lines and secondary workloads for both paths
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  RICEPP_DECODE=$([ $f = 0 ] && echo two-stage || echo fused) timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_f$f.log 2>&1 || exit 1
  echo "fused=$f $(tail -1 gpurun_out/bench_f$f.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], c["encode_kernel_us"], c["decode_kernel_us"])')"
  RICEPP_DECODE=$([ $f = 0 ] && echo two-stage || echo fused) timeout -k 10 300 python tools/workloads.py gen mix > gpurun_out/wl_f$f.log 2>&1 || exit 1
  cat gpurun_out/wl_f$f.log
done
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/trace.log 2>&1; echo "trace=$?"
grep -E "rpp_" gpurun_out/trace/run_kernel_stats.csv | cut -d, -f1-4
