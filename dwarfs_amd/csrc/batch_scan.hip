// batch_scan.hip -- image offsets of a batch of compressed blocks on MI355X
// (the C ABI rpp_exclusive_scan_u64 of include/ricepp_amd.h).
//
// The DwarFS writer appends compressed blocks back to back
// (src/writer/filesystem_writer.cpp:255-287): block b starts at the sum of the
// encoded sizes of blocks 0..b-1.  For a batch encoded on the GPU (sizes in
// HBM, all-gathered across ranks) this exclusive prefix sum is one launch of
// one 1024-thread workgroup: 4096 sizes per pass (4 per lane, 64-bit), wave
// scans by lane shuffles, the 16 wave totals scanned by wave 0, a carry
// between passes.  Latency-bound on purpose: a batch holds thousands of
// blocks, not millions, and one small launch replaces the framework's
// fill + two-kernel scan + copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace {

constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kScanPerLane = 4;
constexpr uint32_t kScanTile = kScanThreads * kScanPerLane;

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ __launch_bounds__(kScanThreads) void rpp_exscan_u64_kernel(const uint64_t* in, uint64_t n,
                                                                      uint64_t* out) {
  __shared__ uint64_t wave_tot[kScanThreads / 64];
  __shared__ uint64_t tile_tot;
  const uint32_t t = threadIdx.x, lane = t % 64, wv = t / 64;
  uint64_t carry = 0;
  for (uint64_t base = 0; base < n; base += kScanTile) {
    const uint64_t i0 = base + (uint64_t)kScanPerLane * t;
    uint64_t v[kScanPerLane], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPerLane; ++k) {
      v[k] = i0 + k < n ? in[i0 + k] : 0u;
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
}

}  // namespace

extern "C" int rpp_exclusive_scan_u64(const uint64_t* d_in, uint64_t n, uint64_t* d_out, void* stream) {
  if (n == 0) return RPP_OK;
  if (!d_in || !d_out) return RPP_INVALID_ARGUMENT;
  hipLaunchKernelGGL(rpp_exscan_u64_kernel, dim3(1), dim3(kScanThreads), 0, (hipStream_t)stream, d_in, n, d_out);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}
