# rows decode kernel (bs 16 / 32, lib variant "rows"): all GPU tests on it, then the configs[4] sweep main vs rows, and the bench
mkdir -p gpurun_out
RL=$PWD/dwarfs_amd/lib/libricepp_amd_rows.so
RICEPP_AMD_LIB=$RL timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rows.log 2>&1; rc=$?; echo "pytest_rows=$rc"; tail -15 gpurun_out/pytest_rows.log
[ $rc -eq 0 ] || exit $rc
RICEPP_AMD_LIB=$RL timeout -k 10 170 python -u tools/workloads.py sweep > gpurun_out/sweep_rows.jsonl 2> gpurun_out/sweep_rows.err; echo "sweep_rows=$?"; cat gpurun_out/sweep_rows.jsonl
timeout -k 10 170 python -u tools/workloads.py sweep > gpurun_out/sweep_main.jsonl 2> gpurun_out/sweep_main.err; echo "sweep_main=$?"; cat gpurun_out/sweep_main.jsonl
RICEPP_AMD_LIB=$RL timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_rows.log 2>&1; echo "bench=$?"; tail -1 gpurun_out/bench_rows.log | cut -c1-200
# the round-end profile set on these sources (main build): PMC passes, bench kernel trace, profiles, default bench with traffic
mkdir -p gpurun_out/prof gpurun_out/profiles_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest_main=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1; rc=$?; echo "pmc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof/trace.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/save_profiles.py r03 > gpurun_out/save_profiles.log 2>&1 || exit 1
cp profiles/pmc_latest.json profiles/r03_bench_kernel_stats.csv profiles/r03_pmc_summary.txt gpurun_out/profiles_out/
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench_full=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-200
