# Round-6 GPU session: the secondary numbers for DESIGN's round-6 table -- configs[4] sweep, one-block
# latency, the configs[3] mix bench line.  Output: gpurun_out/r06/num_*
set -e
mkdir -p gpurun_out/r06
timeout -k 10 600 python3 tools/workloads.py sweep > gpurun_out/r06/num_sweep.jsonl
timeout -k 10 300 python3 tools/small_batch_latency.py > gpurun_out/r06/num_latency.jsonl
timeout -k 10 300 python3 bench.py --workload mix --mix-gib 32 --no-cpu > gpurun_out/r06/num_mix.json
tail -c 600 gpurun_out/r06/num_mix.json
