# Round-6 GPU session: standalone emission-branch probe, every ingredient
# combination, at 8 and 3 waves per SIMD.  Output: gpurun_out/r06/branch_repro2.jsonl
set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06/branch_repro2.jsonl
: > $O
for lds in 256 13312; do
  for v in 0 1 2 4 8 16 31; do
    for mode in 0 4; do
      timeout -k 10 60 tools/vccz_repro 16384 20000 $lds $mode $v >> $O
    done
  done
done
for v in 3 5 6 7 9 17 24 27 28 30; do
  timeout -k 10 60 tools/vccz_repro 16384 20000 13312 4 $v >> $O
done
cat $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flac.py -x -q -k fixtures --timeout 120 --timeout-method thread > gpurun_out/r06/flac_fixtures.txt 2>&1
tail -3 gpurun_out/r06/flac_fixtures.txt
