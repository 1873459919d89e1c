# Diagnostic: builds library variants with extra compiler flags: tools/flagvar.sh <tag> <flags...>
set -e
tag=$1; shift
hipcc -O3 -std=c++20 --offload-arch=gfx950 -fPIC -shared "$@" -Iinclude \
  -o dwarfs_amd/lib/libricepp_amd_fv$tag.so dwarfs_amd/csrc/ricepp_kernels.hip dwarfs_amd/csrc/fits_lsb.hip dwarfs_amd/csrc/batch_image.hip dwarfs_amd/csrc/ricepp_frame.cpp dwarfs_amd/csrc/ricepp_facade.cpp
