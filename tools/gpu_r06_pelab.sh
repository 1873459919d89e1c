# Round-6 GPU session: the fused decode's sub-block end by v_readlane of the end lane's terminator
# (variant "pel", before the list writes) against the list read-back (base): one-block latency, the bench
# decode, then the GPU suite on the variant.  Output: gpurun_out/r06/pelab*
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/pelab*.jsonl
for rep in 1 2; do
for v in base pel; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 tools/small_batch_latency.py | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/pelab_latency.jsonl
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --steps 50 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/pelab_bench.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/r06/pelab_latency.jsonl'):
    d=json.loads(l); print(d['lib'], d['blocks'], d['decode_fused_us'])
for l in open('gpurun_out/r06/pelab_bench.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d['config']['decode_kernel_us'])
"
RICEPP_AMD_LIB=dwarfs_amd/lib/libricepp_amd_pel.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/pelab_tests.txt 2>&1
tail -2 gpurun_out/r06/pelab_tests.txt
