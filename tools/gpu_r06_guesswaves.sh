# Round-6 GPU session: the guess kernel with 4 / 8 waves per unit for batches up to 16384 units (variants
# w4 / w8) against 16 waves up to 2048 units (base): the 7.7 Gbit generator stream, and the 16 MiB /
# 504 MiB cases of seg_parse_diag.  Output: gpurun_out/r06/guesswaves*
set -e
mkdir -p gpurun_out/r06
rm -f gpurun_out/r06/guesswaves.jsonl gpurun_out/r06/guesswaves_diag.txt
for rep in 1 2; do
for v in base w4 w8; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 200 python3 tools/giant_prof.py 0 3 | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r06/guesswaves.jsonl
done
done
for v in base w4 w8; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  echo "== $v" >> gpurun_out/r06/guesswaves_diag.txt
  RICEPP_AMD_LIB=$lib timeout -k 10 300 python3 tools/seg_parse_diag.py 2>/dev/null | cut -c1-60 >> gpurun_out/r06/guesswaves_diag.txt
done
python3 -c "
import json
for l in open('gpurun_out/r06/guesswaves.jsonl'):
    d=json.loads(l); print(d['lib'], d['decode_ms'], d['decode_GiBps'], d['segmented_stats_per_call'])
"
cat gpurun_out/r06/guesswaves_diag.txt
