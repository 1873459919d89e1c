# PMC passes for the bench workload (decode/encode kernels); summary -> gpurun_out/prof/pmc_summary.txt
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT/pmc_*
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SALU" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$i -o run -- python3 tools/prof_kernels.py 2 > $OUT/pmc_$i.log 2>&1; rc=$?; echo "pmc $grp = $rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt; cat $OUT/pmc_summary.txt
