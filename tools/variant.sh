# Diagnostic: builds the library with extra compile flags into
# dwarfs_amd/lib/libricepp_amd_<name>.so (load it with RICEPP_AMD_LIB=...)
# usage: bash tools/variant.sh <name> [-DFLAG=V ...]
set -e
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -fPIC -shared "$@" -Iinclude \
  -o dwarfs_amd/lib/libricepp_amd_$name.so dwarfs_amd/csrc/ricepp_kernels.hip dwarfs_amd/csrc/ricepp_decode2.hip \
  dwarfs_amd/csrc/fits_lsb.hip dwarfs_amd/csrc/batch_image.hip dwarfs_amd/csrc/pcm_transform.hip dwarfs_amd/csrc/flac_kernels.hip \
  dwarfs_amd/csrc/ricepp_frame.cpp dwarfs_amd/csrc/ricepp_facade.cpp
