# Round-6 GPU session: in-place 64-bit shift probe + the shift-copy variants of the faulty encode build
set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06/shift64_probe.jsonl
: > $O
for lds in 4096 40960; do for v in 0 1; do timeout -k 10 60 tools/shift64_repro 16384 20000 $lds $v >> $O; done; done
cat $O
REPS=3 VARIANTS="asm_sh64 asm_sh64s" bash tools/gpu_r06_branch3.sh
