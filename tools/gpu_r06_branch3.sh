# Round-6 GPU session: the real encode kernel with its emission branches
# edited in the assembly (tools/asm_variant.py).  Output: gpurun_out/r06/branch_asm.jsonl
set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06/branch_asm.jsonl
: > $O
for v in ${VARIANTS:-asm_none asm_vccw asm_nop}; do
  RICEPP_AMD_LIB=dwarfs_amd/lib/libricepp_amd_$v.so timeout -k 10 300 python -u tools/branch_diag.py $v ${REPS:-3} >> $O
done
cat $O
