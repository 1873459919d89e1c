// batch_image.hip -- laying out a batch of compressed blocks on MI355X
// (rpp_exclusive_scan_u64 and rpp_pack_batch of include/ricepp_amd.h).
//
// The DwarFS writer appends compressed blocks back to back
// (src/writer/filesystem_writer.cpp:255-287): block b starts at the sum of the
// (rounded) encoded sizes of blocks 0..b-1.  The encode kernel writes block b
// at a worst-case-capacity slot; before the batch leaves the GPU it is packed:
//
//   scan  one 1024-thread workgroup: 4096 sizes per pass (4 per lane, 64-bit),
//         wave scans by lane shuffles, the 16 wave totals scanned by wave 0, a
//         carry between passes.  Latency-bound on purpose: a batch holds
//         thousands of blocks, and one small launch replaces a fill + two-kernel
//         scan + copy.
//   pack  one workgroup per block, 16-byte loads and stores (source slots and
//         packed offsets are both 16-aligned, so whole 16-byte granules are in
//         bounds on both sides): an HBM copy of the compressed bytes only, so the
//         device->host transfer that follows moves sum(sizes), not the
//         worst-case capacity.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace {

constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kScanPerLane = 4;
constexpr uint32_t kScanTile = kScanThreads * kScanPerLane;
constexpr uint32_t kPackThreads = 256;

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

// out[i] = sum_{j<i} round_up(in[j], align); *total = the full sum (if non-null).
__global__ __launch_bounds__(kScanThreads) void rpp_exscan_u64_kernel(const uint64_t* in, uint64_t n, uint64_t align,
                                                                      uint64_t* out, uint64_t* total) {
  __shared__ uint64_t wave_tot[kScanThreads / 64];
  __shared__ uint64_t tile_tot;
  const uint32_t t = threadIdx.x, lane = t % 64, wv = t / 64;
  const uint64_t amask = align - 1;
  uint64_t carry = 0;
  for (uint64_t base = 0; base < n; base += kScanTile) {
    const uint64_t i0 = base + (uint64_t)kScanPerLane * t;
    uint64_t v[kScanPerLane], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPerLane; ++k) {
      v[k] = i0 + k < n ? (in[i0 + k] + amask) & ~amask : 0u;
      s += v[k];
    }
    const uint64_t incl = wave_incl_scan_u64(s, lane);
    if (lane == 63) wave_tot[wv] = incl;
    __syncthreads();
    if (wv == 0) {
      const uint64_t w = lane < kScanThreads / 64 ? wave_tot[lane] : 0u;
      const uint64_t wi = wave_incl_scan_u64(w, lane);
      if (lane < kScanThreads / 64) wave_tot[lane] = wi - w;  // exclusive
      if (lane == kScanThreads / 64 - 1) tile_tot = wi;
    }
    __syncthreads();
    uint64_t run = carry + wave_tot[wv] + incl - s;
#pragma unroll
    for (uint32_t k = 0; k < kScanPerLane; ++k) {
      if (i0 + k < n) out[i0 + k] = run;
      run += v[k];
    }
    carry += tile_tot;
    __syncthreads();  // wave_tot / tile_tot are rewritten by the next pass
  }
  if (total && t == 0) *total = carry;
}

__global__ __launch_bounds__(kPackThreads) void rpp_pack_kernel(const uint8_t* src, const uint64_t* src_off,
                                                                const uint64_t* sizes, const uint64_t* dst_off,
                                                                uint8_t* dst) {
  const uint32_t b = blockIdx.x;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* s = reinterpret_cast<const u32x4*>(src + src_off[b]);
  u32x4* d = reinterpret_cast<u32x4*>(dst + dst_off[b]);
  const uint64_t n16 = (sizes[b] + 15) / 16;
  for (uint64_t i = threadIdx.x; i < n16; i += kPackThreads) d[i] = __builtin_nontemporal_load(s + i);
}

int launch_scan(const uint64_t* d_in, uint64_t n, uint64_t align, uint64_t* d_out, uint64_t* d_total,
                hipStream_t stream) {
  hipLaunchKernelGGL(rpp_exscan_u64_kernel, dim3(1), dim3(kScanThreads), 0, stream, d_in, n, align, d_out, d_total);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // namespace

extern "C" int rpp_exclusive_scan_u64(const uint64_t* d_in, uint64_t n, uint64_t* d_out, void* stream) {
  if (n == 0) return RPP_OK;
  if (!d_in || !d_out) return RPP_INVALID_ARGUMENT;
  return launch_scan(d_in, n, 1, d_out, nullptr, (hipStream_t)stream);
}

extern "C" int rpp_pack_batch(const uint8_t* d_src, const uint64_t* d_src_offsets, const uint64_t* d_sizes,
                              uint32_t nblocks, uint8_t* d_dst, uint64_t* d_dst_offsets, uint64_t* d_total,
                              void* stream) {
  if (!d_total) return RPP_INVALID_ARGUMENT;
  if (nblocks == 0) {
    return hipMemsetAsync(d_total, 0, sizeof(uint64_t), (hipStream_t)stream) == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
  }
  if (!d_src || !d_src_offsets || !d_sizes || !d_dst || !d_dst_offsets) return RPP_INVALID_ARGUMENT;
  const int st = launch_scan(d_sizes, nblocks, 16, d_dst_offsets, d_total, (hipStream_t)stream);
  if (st != RPP_OK) return st;
  hipLaunchKernelGGL(rpp_pack_kernel, dim3(nblocks), dim3(kPackThreads), 0, (hipStream_t)stream, d_src, d_src_offsets,
                     d_sizes, d_dst_offsets, d_dst);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}
