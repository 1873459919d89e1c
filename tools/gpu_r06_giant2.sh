# Round-6 GPU session: A/B of the extraction stage rule and the guess kernel's unit bound on the 7.5 Gbit
# stream and the configs[3] mix (variant libraries from tools/variant.sh).  Output: gpurun_out/r06/giant2_*
set -e
mkdir -p gpurun_out/r06
for v in base stage64 guess8k both; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 200 python3 tools/giant_prof.py 0 3 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/giant2.jsonl
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --workload mix --mix-gib 32 --no-cpu --steps 5 --warmup 2 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/giant2_mix.jsonl
done
cut -c1-250 gpurun_out/r06/giant2.jsonl
python3 -c "
import json
for l in open('gpurun_out/r06/giant2_mix.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d.get('ms_per_step'), {k:v for k,v in d.items() if 'decode' in k and not isinstance(v, dict)})
"
