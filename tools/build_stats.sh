hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -DRPP_STATS -Iinclude -o dwarfs_amd/lib/libricepp_amd_stats.so dwarfs_amd/csrc/ricepp_kernels.hip dwarfs_amd/csrc/ricepp_frame.cpp
