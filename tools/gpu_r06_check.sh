# Round-6 GPU session: full GPU tests, the bs 128 cs 2 at-scale check, and the bench line.
set -e
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/gpu_tests.txt 2>&1
tail -3 gpurun_out/r06/gpu_tests.txt
timeout -k 10 300 python -u tools/branch_diag.py default 3 > gpurun_out/r06/branch_default.jsonl
cat gpurun_out/r06/branch_default.jsonl | cut -c1-120
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r06/bench_nocpu.json
cat gpurun_out/r06/bench_nocpu.json
