# Round-end style GPU session: parity tests, default bench (with CPU baseline),
# rocprofv3 kernel-trace stats of the bench command, PMC traffic passes.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
OUT=gpurun_out/prof
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench=$rc"; tail -1 gpurun_out/bench_default.log
[ $rc -eq 0 ] || exit $rc
rm -rf $OUT/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $OUT/trace_bench.log 2>&1; rc=$?; echo "trace=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf $OUT/pmc_*
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$i -o run -- python3 tools/prof_kernels.py 2 > $OUT/pmc_$i.log 2>&1; rc=$?; echo "pmc $grp = $rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
