set -e
mkdir -p gpurun_out/r06
timeout -k 10 120 tools/vgpr_alloc_repro 16384 2000 > gpurun_out/r06/vgpr_alloc_repro.jsonl
timeout -k 10 120 tools/vgpr_alloc_repro 4096 8000 >> gpurun_out/r06/vgpr_alloc_repro.jsonl
cat gpurun_out/r06/vgpr_alloc_repro.jsonl
