# decode correctness of flag-variant builds: tools/gpu_bisect.sh <tag>...
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  RICEPP_AMD_LIB=$PWD/dwarfs_amd/lib/libricepp_amd_fv$v.so timeout -k 10 100 python tools/dbg_decode2.py 128 > gpurun_out/bisect_$v.log 2>&1 || exit 1
  cut -c1-70 gpurun_out/bisect_$v.log
done
