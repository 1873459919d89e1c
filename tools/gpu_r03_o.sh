# bench defaults (steps / warmup) compared on one box, then the round-end trace, profiles and default bench with the new defaults
set -u
mkdir -p gpurun_out/prof gpurun_out/profiles_out
export TMPDIR=/tmp
for sw in "20 3" "100 20" "200 50" "20 3" "100 20"; do
  set -- $sw
  timeout -k 10 120 python bench.py --steps $1 --warmup $2 --no-cpu > gpurun_out/bench_sw.log 2>&1 || exit 1
  echo "steps=$1 warmup=$2 $(tail -1 gpurun_out/bench_sw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1; rc=$?; echo "pmc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --no-cpu > gpurun_out/prof/trace.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/save_profiles.py r03 > gpurun_out/save_profiles.log 2>&1 || exit 1
cp profiles/pmc_latest.json profiles/r03_bench_kernel_stats.csv profiles/r03_pmc_summary.txt gpurun_out/profiles_out/
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench_full=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-300
