# rows decode kernel (bs 16 / 32, lib variant "rows"): all GPU tests on it, then the configs[4] sweep main vs rows, and the bench
mkdir -p gpurun_out
RL=$PWD/dwarfs_amd/lib/libricepp_amd_rows.so
RICEPP_AMD_LIB=$RL timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rows.log 2>&1; rc=$?; echo "pytest_rows=$rc"; tail -15 gpurun_out/pytest_rows.log
[ $rc -eq 0 ] || exit $rc
RICEPP_AMD_LIB=$RL timeout -k 10 170 python -u tools/workloads.py sweep > gpurun_out/sweep_rows.jsonl 2> gpurun_out/sweep_rows.err; echo "sweep_rows=$?"; cat gpurun_out/sweep_rows.jsonl
timeout -k 10 170 python -u tools/workloads.py sweep > gpurun_out/sweep_main.jsonl 2> gpurun_out/sweep_main.err; echo "sweep_main=$?"; cat gpurun_out/sweep_main.jsonl
RICEPP_AMD_LIB=$RL timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_rows.log 2>&1; echo "bench=$?"; tail -1 gpurun_out/bench_rows.log | cut -c1-200
