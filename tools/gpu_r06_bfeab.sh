# Round-6 GPU session: the library built with the emission's high word by v_bfe_u32 (variant "bfe")
# against the shift pair (base): bench lines alternating, then the GPU suite on the variant.
# Output: gpurun_out/r06/bfeab*
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/bfeab*.jsonl
for rep in 1 2 3; do
for v in base bfe; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/bfeab.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/bfeab.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d['config']['encode_kernel_us'], d['config']['decode_kernel_us'])
"
RICEPP_AMD_LIB=dwarfs_amd/lib/libricepp_amd_bfe.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/bfeab_tests.txt 2>&1
tail -2 gpurun_out/r06/bfeab_tests.txt
