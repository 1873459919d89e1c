# Round-6 GPU session: configs[3] mix and the 7.5 Gbit stream before / after the segmented decode's unit
# frames, 64-bit sub-block positions and stage choice by density (variant library "pre" = the previous
# commit, "both" = 64 KiB stage always + guess bound 8192), alternating.  Output: gpurun_out/r06/mixab*.jsonl
set -e
mkdir -p gpurun_out/r06
for rep in 1 2; do
for v in pre base both; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --workload mix --mix-gib 32 --no-cpu --steps 5 --warmup 2 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/mixab.jsonl
  [ $v = pre ] || RICEPP_AMD_LIB=$lib timeout -k 10 200 python3 tools/giant_prof.py 0 3 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/mixab_giant.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/mixab.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d.get('ms_per_step'))
for l in open('gpurun_out/r06/mixab_giant.jsonl'):
    d=json.loads(l); print(d['lib'], d['decode_ms'], d['decode_GiBps'])
"
