# all workloads with a steady-clock warm-up before each timing
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/workloads.py > gpurun_out/workloads.jsonl 2> gpurun_out/workloads.err; echo "workloads=$?"
cut -c1-160 gpurun_out/workloads.jsonl
