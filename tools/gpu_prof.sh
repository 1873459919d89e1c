# rocprofv3 kernel trace + PMC passes for the bench workload
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
OUT=gpurun_out/prof
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_kernels.py 5 > $OUT/trace.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SMEM"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$tag -o run -- python3 tools/prof_kernels.py 2 > $OUT/pmc_$tag.log 2>&1; rc=$?; echo "pmc $grp = $rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
