# PMC passes (one counter per run) of the configs[3] mix: gpurun_out/prof/mix_<COUNTER>/
set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
  rm -rf $OUT/mix_$c
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex rpp_ --output-format csv -d $OUT/mix_$c -o run -- python3 tools/prof_mix.py ${MIX_GIB:-32} 1 2 ${MIX_PATH:-auto} > $OUT/mix_$c.log 2>&1; rc=$?
  echo "pmc mix $c = $rc"; tail -2 $OUT/mix_$c.log
  [ $rc -eq 0 ] || exit $rc
done
