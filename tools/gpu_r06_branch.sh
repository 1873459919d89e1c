# Round-6 GPU session: the emission-branch investigation (DESIGN.md §4
# "Uniform branches").  Standalone probe first, then the real kernel in three
# builds.  Output: gpurun_out/r06/branch_*.jsonl
set -e
mkdir -p gpurun_out/r06
O=gpurun_out/r06
: > $O/branch_repro.jsonl
for lds in 0 40960; do
  for mode in 0 1 2 3 4; do
    timeout -k 10 60 tools/vccz_repro 16384 20000 $lds $mode >> $O/branch_repro.jsonl
  done
done
: > $O/branch_kernel.jsonl
for v in valu valuchk saluchk; do
  RICEPP_AMD_LIB=dwarfs_amd/lib/libricepp_amd_$v.so timeout -k 10 300 python -u tools/branch_diag.py $v 3 >> $O/branch_kernel.jsonl
done
timeout -k 10 300 python -u tools/branch_diag.py default 2 >> $O/branch_kernel.jsonl
cat $O/branch_repro.jsonl $O/branch_kernel.jsonl
