# Round-6 GPU session: the library built with -mllvm -amdgpu-sched-strategy=max-ilp (variant "ilp1")
# against the default scheduler (base): bench lines alternating, and the configs[4] sweep.
# Output: gpurun_out/r06/ilpab*
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/ilpab*.jsonl
for rep in 1 2 3; do
for v in base ilp1; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/ilpab.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/ilpab.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d['config']['encode_kernel_us'], d['config']['decode_kernel_us'])
"
