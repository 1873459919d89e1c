# LDS conflict attribution: one PMC pass per library variant (the variants
# repeat one class of LDS instruction of the decode fast loop with the same
# addresses, so the counter's increase is that class's conflict cycles).
# usage: bash tools/gpu_attr.sh name1 name2 ...   (name "base" = the default library)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/attr
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = base ]; then lib=dwarfs_amd/lib/libricepp_amd.so; else lib=dwarfs_amd/lib/libricepp_amd_$v.so; fi
  RICEPP_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/$v/p1 -o run -- python3 tools/prof_kernels.py 2 > $OUT/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  echo "== $v" >> $OUT/summary.txt; python3 tools/pmc_summary.py $OUT/$v >> $OUT/summary.txt 2>&1
done
cat $OUT/summary.txt
