set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06/shl64_hazard.jsonl
timeout -k 10 120 tools/shl64_hazard 1024 2000 > $O
timeout -k 10 120 tools/shl64_hazard 16384 1000 >> $O
cat $O
