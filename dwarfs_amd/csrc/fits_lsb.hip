// fits_lsb.hip -- unused-LSB detection of 16-bit FITS image data on MI355X
// (the C ABI rpp_unused_lsb_batch of include/ricepp_amd.h).
//
// Reference: src/writer/categorizer/fits_categorizer.cpp:118-178.  mkdwarfs'
// FITS categorizer ORs every 16-bit sample of an image (merge_sample_bits,
// :118-162, stored big-endian) and takes the number of trailing zero bits of
// the result (get_unused_lsb_count, :165-178): the `unused_lsb_count` the
// ricepp codec is then configured with (std::countr_zero, so an all-zero
// image gives 16).  The reference short-circuits once bit 0 is set; the
// result (0) is the same.
//
// An HBM-bound OR reduction: 2-D grid (chunk, image); each 256-thread block
// ORs chunks of an image (256 KiB for big batches, 64 KiB when the batch is
// too small to give the 256 CUs a few blocks each) with 16-byte loads, four
// in flight per lane (ragged head/tail samples separately), reduces in
// registers/LDS and merges with one atomicOr per block; a one-wave second
// launch turns the per-image OR into the count.  Blocks stride over the
// chunks, so an image longer than the max_samples the grid was sized for is
// still read whole.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace {

constexpr uint32_t kLsbThreads = 256;
constexpr uint32_t kLsbChunkBig = 131072;   // 256 KiB per block
constexpr uint32_t kLsbChunkSmall = 32768;  // 64 KiB per block (small batches)
constexpr uint64_t kLsbMinBlocks = 1024;    // 4 blocks per CU before the big chunk is used

__global__ __launch_bounds__(kLsbThreads) void rpp_lsb_or_kernel(const uint16_t* in, const uint64_t* offsets,
                                                                 const uint64_t* n_samples, uint32_t chunk,
                                                                 uint32_t* acc) {
  __shared__ uint32_t red[kLsbThreads / 64];
  const uint32_t img = blockIdx.y;
  const uint64_t n = n_samples[img];
  const uint16_t* p = in + offsets[img];
  uint32_t v = 0;
  for (uint64_t c0 = (uint64_t)blockIdx.x * chunk; c0 < n; c0 += (uint64_t)gridDim.x * chunk) {
    const uint64_t c1 = n - c0 < chunk ? n : c0 + chunk;
    // samples [c0, c1): an aligned middle of 8-sample groups plus ragged ends
    const uintptr_t addr = (uintptr_t)(p + c0);
    uint64_t head = ((16u - (addr & 15u)) & 15u) / 2u;  // samples before the first 16-B boundary
    if (addr & 1u) head = c1 - c0;                      // odd address: scalar loads only
    if (head > c1 - c0) head = c1 - c0;
    const uint64_t m0 = c0 + head;
    const uint64_t groups = (c1 - m0) / 8u;
    const uint4* q = reinterpret_cast<const uint4*>(p + m0);
    uint64_t g = threadIdx.x;
    // four independent 16-byte loads in flight per lane
    for (; g + 3u * kLsbThreads < groups; g += 4u * kLsbThreads) {
      const uint4 w0 = q[g], w1 = q[g + kLsbThreads], w2 = q[g + 2u * kLsbThreads], w3 = q[g + 3u * kLsbThreads];
      v |= (w0.x | w0.y | w0.z | w0.w) | (w1.x | w1.y | w1.z | w1.w) | (w2.x | w2.y | w2.z | w2.w) |
           (w3.x | w3.y | w3.z | w3.w);
    }
    for (; g < groups; g += kLsbThreads) {
      const uint4 w = q[g];
      v |= w.x | w.y | w.z | w.w;
    }
    for (uint64_t i = c0 + threadIdx.x; i < m0; i += kLsbThreads) v |= p[i];
    for (uint64_t i = m0 + 8u * groups + threadIdx.x; i < c1; i += kLsbThreads) v |= p[i];
  }
  if (__syncthreads_or(v) == 0) return;  // (uniform: nothing to merge)
  v = (v | (v >> 16)) & 0xFFFFu;  // the two samples of a word
  // wave OR (xor butterfly), then across the block's waves
  for (int d = 32; d >= 1; d >>= 1) v |= (uint32_t)__shfl_xor((int)v, d);
  if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = 0;
    for (uint32_t w = 0; w < kLsbThreads / 64; ++w) r |= red[w];
    if (r) atomicOr(&acc[img], r);
  }
}

__global__ void rpp_lsb_count_kernel(const uint32_t* acc, uint32_t nimages, uint32_t big_endian, uint32_t* counts) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nimages) return;
  uint32_t b16 = acc[i] & 0xFFFFu;
  if (big_endian) b16 = ((b16 >> 8) | (b16 << 8)) & 0xFFFFu;  // convert<std::endian::big>
  counts[i] = b16 ? (uint32_t)__builtin_ctz(b16) : 16u;     // std::countr_zero<uint16_t>
}

}  // namespace

extern "C" int rpp_unused_lsb_batch(const uint16_t* d_in, const uint64_t* d_offsets, const uint64_t* d_n_samples,
                                    uint64_t max_samples, uint32_t nimages, uint32_t big_endian,
                                    uint32_t* d_work, uint32_t* d_counts, void* stream) {
  if (nimages == 0) return RPP_OK;
  if (!d_in || !d_offsets || !d_n_samples || !d_work || !d_counts) return RPP_INVALID_ARGUMENT;
  if (nimages > 65535u) return RPP_INVALID_ARGUMENT;  // grid.y limit; callers split larger batches
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(d_work, 0, sizeof(uint32_t) * nimages, s) != hipSuccess) return RPP_HIP_ERROR;
  // max_samples sizes the grid; longer images are still covered (blocks
  // stride over the chunks), so it is a hint, not a bound
  uint64_t chunk = kLsbChunkBig;
  if ((max_samples + kLsbChunkBig - 1) / kLsbChunkBig * nimages < kLsbMinBlocks) chunk = kLsbChunkSmall;
  uint64_t chunks = (max_samples + chunk - 1) / chunk;
  if (chunks > 0x7FFFFFFFull) chunks = 0x7FFFFFFFull;
  if (chunks == 0) chunks = 1;
  hipLaunchKernelGGL(rpp_lsb_or_kernel, dim3((uint32_t)chunks, nimages), dim3(kLsbThreads), 0, s, d_in, d_offsets,
                     d_n_samples, (uint32_t)chunk, d_work);
  hipLaunchKernelGGL(rpp_lsb_count_kernel, dim3((nimages + 255) / 256), dim3(256), 0, s, d_work, nimages,
                     big_endian, d_counts);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}
