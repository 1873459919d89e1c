# Round-6 GPU session: the segmented decode with unit frames and 64-bit positions (streams compressed past
# 2^29 bytes): segmented / long-stream tests, the full GPU suite, then the configs[3] mix against the
# previous commit's library ("pre") and the 7.5 Gbit stream.  Output: gpurun_out/r06/seg64_*
set -e
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "segment or 2_27 or 2_29 or tiles or frame or mix or long" > gpurun_out/r06/seg64_tests.txt 2>&1
tail -2 gpurun_out/r06/seg64_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/seg64_all.txt 2>&1
tail -2 gpurun_out/r06/seg64_all.txt
rm -f gpurun_out/r06/seg64_mix.jsonl gpurun_out/r06/seg64_giant.jsonl
for rep in 1 2; do
for v in pre base; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 bench.py --workload mix --mix-gib 32 --no-cpu --steps 5 --warmup 2 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/seg64_mix.jsonl
done
done
timeout -k 10 200 python3 tools/giant_prof.py 0 3 >> gpurun_out/r06/seg64_giant.jsonl
python3 -c "
import json
for l in open('gpurun_out/r06/seg64_mix.jsonl'):
    d=json.loads(l); print(d['lib'], d['value'], d.get('ms_per_step'), d['roofline']['achieved'])
for l in open('gpurun_out/r06/seg64_giant.jsonl'):
    d=json.loads(l); print('giant', d['decode_ms'], d['decode_GiBps'], d['segmented_stats_per_call'])
"
