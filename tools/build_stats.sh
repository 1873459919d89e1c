# Diagnostic build with per-phase s_memtime stamps (-DRPP_STATS) -> dwarfs_amd/lib/libricepp_amd_stats.so
bash "$(dirname "$0")/variant.sh" stats -DRPP_STATS
