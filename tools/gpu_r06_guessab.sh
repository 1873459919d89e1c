# Round-6 GPU session: the guess kernel's unit bound (variants g16k / g64k against 8192) on the 7.7 Gbit
# generator stream and the configs[3] mix.  Output: gpurun_out/r06/guessab*.jsonl
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/guessab.jsonl gpurun_out/r06/guessab_mix.jsonl
for rep in 1 2; do
for v in base g16k g64k; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 200 python3 tools/giant_prof.py 0 3 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/guessab.jsonl
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --workload mix --mix-gib 32 --no-cpu --steps 5 --warmup 2 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/guessab_mix.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/guessab.jsonl'):
    d=json.loads(l); print(d['lib'], d['decode_ms'], d['decode_GiBps'], d['segmented_stats_per_call'])
for l in open('gpurun_out/r06/guessab_mix.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d['ms_per_step'])
"
