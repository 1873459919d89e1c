# Round-3: GPU tests after the correctness-contract changes, then the configs[3] mix bench at 8 GiB and 32 GiB
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
grep -E "passed|failed|Error|error" gpurun_out/pytest_gpu.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mix --mix-gib 8 --steps 5 --warmup 1 > gpurun_out/bench_mix8.log 2>&1; echo "mix8=$?"; tail -1 gpurun_out/bench_mix8.log
timeout -k 10 400 python bench.py --workload mix --steps 3 --warmup 1 > gpurun_out/bench_mix32.log 2>&1; echo "mix32=$?"; tail -1 gpurun_out/bench_mix32.log
