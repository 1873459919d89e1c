# A/B session: parity tests on the default build, then the bench line and the
# generator workload for each library variant given as arguments
# (dwarfs_amd/lib/libricepp_amd_<name>.so; "main" = the default build)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1; rc=$?; echo "pytest=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  if [ "$v" = main ]; then lib=dwarfs_amd/lib/libricepp_amd.so; else lib=dwarfs_amd/lib/libricepp_amd_$v.so; fi
  RICEPP_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], c["encode_kernel_us"], c["decode_kernel_us"])')"
  RICEPP_AMD_LIB=$PWD/$lib timeout -k 10 200 python tools/workloads.py gen > gpurun_out/gen_$v.jsonl 2>&1 || exit 1
  echo "$v gen: $(grep 4096 gpurun_out/gen_$v.jsonl)"
done
