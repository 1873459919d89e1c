# Round-6 GPU session: the giant streams (DwarFS -S 28..30 blocks) with the final library: tools/workloads.py
# giant and five timings of the 7.5 Gbit stream.  Output: gpurun_out/r06/giant3_*.jsonl
set -e
mkdir -p gpurun_out/r06
timeout -k 10 600 python3 tools/workloads.py giant > gpurun_out/r06/giant3_streams.jsonl
cut -c1-300 gpurun_out/r06/giant3_streams.jsonl
timeout -k 10 300 python3 tools/giant_prof.py 0 5 > gpurun_out/r06/giant3_prof.jsonl
cat gpurun_out/r06/giant3_prof.jsonl
