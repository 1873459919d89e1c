// ricepp_internal.h -- launchers shared between the kernel translation units
// (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace rpp_internal {

// rpp_decode_kernel: one wave per stream, parse and values fused (any bs).
int launch_decode_fused(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, hipStream_t stream);

// rpp_parse_kernel: sub-block start positions of every stream into sb_pos
// (stream b's entries from sb_base[b]: nsb_b header positions, then the end).
int launch_parse(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets, const uint64_t* d_in_bytes,
                 uint32_t nblocks, const uint64_t* d_n_samples, const uint64_t* d_sb_base, uint32_t* d_sb_pos,
                 int32_t* d_status, hipStream_t stream);

}  // namespace rpp_internal
