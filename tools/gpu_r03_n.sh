# decode kernel with amdgpu_waves_per_eu(4, 4): GPU tests, headline bench A/B against the build without it (lib "nowpe",
# alternated), then the round-end profile set on these sources (smoke, facade test, PMC + trace + profiles, bench with traffic)
set -u
mkdir -p gpurun_out/prof gpurun_out/profiles_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_wpe_$i.log 2>&1 || exit 1
  echo "wpe4 $(tail -1 gpurun_out/bench_wpe_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
  RICEPP_AMD_LIB=$PWD/dwarfs_amd/lib/libricepp_amd_nowpe.so timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/bench_nowpe_$i.log 2>&1 || exit 1
  echo "nowpe $(tail -1 gpurun_out/bench_nowpe_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tests/cpp/build/facade_test > gpurun_out/facade_test.log 2>&1; rc=$?; echo "facade_test=$rc"; tail -1 gpurun_out/facade_test.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1; rc=$?; echo "pmc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof/trace.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/save_profiles.py r03 > gpurun_out/save_profiles.log 2>&1 || exit 1
cp profiles/pmc_latest.json profiles/r03_bench_kernel_stats.csv profiles/r03_pmc_summary.txt gpurun_out/profiles_out/
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench_full=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/workloads.py > gpurun_out/workloads.jsonl 2> gpurun_out/workloads.err; echo "workloads=$?"
