# Diagnostic: builds encode ablation variants (-DRPP_EABLATE=mask) into dwarfs_amd/lib/
set -e
for m in "$@"; do
  hipcc -O3 -std=c++20 --offload-arch=gfx950 -fPIC -shared -DRPP_EABLATE=$m -Iinclude \
    -o dwarfs_amd/lib/libricepp_amd_eabl$m.so dwarfs_amd/csrc/ricepp_kernels.hip dwarfs_amd/csrc/fits_lsb.hip dwarfs_amd/csrc/batch_image.hip dwarfs_amd/csrc/ricepp_frame.cpp dwarfs_amd/csrc/ricepp_facade.cpp &
done
wait
