# Round-6 GPU session: per-kernel times of the configs[3] mix decode, previous commit ("pre") against the
# unit frames + 64-bit positions build.  Output: gpurun_out/r06/mixprof_*/
set -e
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in pre base; do
  lib=dwarfs_amd/lib/libricepp_amd_$v.so; [ $v = base ] && lib=dwarfs_amd/lib/libricepp_amd.so
  RICEPP_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/mixprof_$v -o run -- python3 tools/prof_mix.py 32 1 3 auto > gpurun_out/r06/mixprof_$v.log 2>&1
done
