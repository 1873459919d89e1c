set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06/shift64_probe2.jsonl
: > $O
for lds in 4096 40960; do for v in 2 3; do timeout -k 10 60 tools/shift64_repro 16384 20000 $lds $v >> $O; done; done
cat $O
REPS=3 VARIANTS="asm_sh64d asm_sh64sd" bash tools/gpu_r06_branch3.sh
