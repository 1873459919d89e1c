# Round-6 GPU session: the decode scan steps as update_dpp builtins (variant "dppb", the compiler's hazard
# recognizer places the wait states) against the inline-asm steps (base): bench lines alternating, then the
# GPU suite on the variant.  Output: gpurun_out/r06/dppab*.
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/dppab.jsonl gpurun_out/r06/dppab_sweep.jsonl
for rep in 1 2 3; do
for v in base dppb; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/dppab.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/dppab.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d['config']['encode_kernel_us'], d['config']['decode_kernel_us'])
"
for v in base dppb; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 tools/workloads.py sweep gen | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/dppab_sweep.jsonl
done
RICEPP_AMD_LIB=dwarfs_amd/lib/libricepp_amd_dppb.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/dppab_tests.txt 2>&1
tail -2 gpurun_out/r06/dppab_tests.txt
