# instruction-mix / stall / LDS counters of the bench kernels (one rocprofv3 pass per group)
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/diag/pmc_$i -o run -- python3 tools/prof_kernels.py 2 > gpurun_out/diag/pmc_$i.log 2>&1; rc=$?; echo "pmc $i = $rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/diag/pmc_$i.log; exit $rc; }
done
python3 tools/pmc_summary.py gpurun_out/diag
