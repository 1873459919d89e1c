# PMC passes (one counter group per run) over the bench workload's kernels; summary per rpp_* kernel
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rm -rf gpurun_out/pmc/*
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/prof_kernels.py 2 > gpurun_out/pmc/p$i.log 2>&1; rc=$?; echo "pmc $grp = $rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt; cat gpurun_out/pmc/summary.txt
