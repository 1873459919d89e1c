# Parity tests of the decode fast loops, then configs[4]'s sweep and the bench line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sweep.log 2>&1; rc=$?; echo "pytest=$rc"
tail -3 gpurun_out/pytest_sweep.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/workloads.py sweep gen > gpurun_out/sweep.jsonl 2>&1; echo "sweep=$?"
grep case gpurun_out/sweep.jsonl | cut -c1-200
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-700
