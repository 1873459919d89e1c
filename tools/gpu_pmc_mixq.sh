# Two PMC passes of the configs[3] mix (MIX_GIB, default 8) for the decode kernels' issue profile:
# summaries -> gpurun_out/prof/mixq_summary.txt
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"; do
  i=$((i+1))
  rm -rf $OUT/mixq/p$i
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex rpp_ --output-format csv -d $OUT/mixq/p$i -o run -- python3 tools/prof_mix.py ${MIX_GIB:-8} 1 1 auto > $OUT/mixq_$i.log 2>&1; rc=$?
  echo "pmc mixq $i = $rc"; tail -1 $OUT/mixq_$i.log
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT/mixq > $OUT/mixq_summary.txt; cat $OUT/mixq_summary.txt
