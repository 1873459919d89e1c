// pcm_transform.hip -- PCM sample unpack/pack on MI355X (the C ABI
// rpp_pcm_unpack / rpp_pcm_pack of include/ricepp_amd.h).
//
// Reference: src/pcm_sample_transformer.cpp:44-173 (basic_pcm_sample_transformer)
// behind include/dwarfs/pcm_sample_transformer.h:40-71, used by the FLAC
// compressor (src/compression/flac.cpp:211,322) to turn interleaved PCM bytes
// (1..4 bytes per sample, big/little endian, signed/unsigned, LSB/MSB padded,
// `bits` significant bits) into int32 samples and back.  Per sample:
//   unpack: t = bytes as uint32 in the stored order; Lsb padding: t >>= 8*B-bits;
//           signed: sign-extend from bit bits-1 (bits < 32; no masking above it,
//           as in :147-155); unsigned: (int32)t - (1 << (bits-1))  (:156-157)
//   pack:   unsigned: s += 1 << (bits-1); Lsb padding: s <<= 8*B-bits; the low
//           B bytes of s in the stored order (:160-171, :97-138)
// All arithmetic is done mod 2^32, which is what the reference's int32
// expressions produce on every target DwarFS builds for (bits = 32 included).
//
// HBM-bound elementwise byte work (no MFMA, no LDS): each lane owns quads of 4
// consecutive samples (kPcmUnroll of them in flight), i.e. B dwords of packed bytes and one 16-byte int32
// quad, so every load/store is a whole dword(x2/x3/x4) and a wave touches one
// contiguous 256*B-byte / 1 KiB span.  Byte reordering is a v_perm per
// sample.  Unaligned buffers and the ragged tail use a per-sample byte path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace {

constexpr uint32_t kPcmThreads = 256;
constexpr int kPcmUnroll = 4;                  // quads (4 samples) in flight per lane
constexpr uint32_t kPcmMaxBlocks = 1u << 20;   // grid-stride beyond 2^30 samples

template <int B, bool BE>
__device__ __forceinline__ uint32_t pcm_assemble(const uint8_t* p) {
  uint32_t t = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) t |= (uint32_t)p[k] << (8 * (BE ? (B - 1 - k) : k));
  return t;
}

template <int B, bool BE>
__device__ __forceinline__ void pcm_scatter(uint8_t* p, uint32_t t) {
#pragma unroll
  for (int k = 0; k < B; ++k) p[k] = (uint8_t)(t >> (8 * (BE ? (B - 1 - k) : k)));
}

template <int B, bool SIGNED, bool LSB>
__device__ __forceinline__ int32_t pcm_unpack_native(uint32_t t, uint32_t bits) {
  if (LSB) t >>= (8u * B - bits);
  if (SIGNED) {
    if (bits < 32u && (t & (1u << (bits - 1u)))) t |= ~0u << bits;
    return (int32_t)t;
  }
  return (int32_t)(t - (1u << (bits - 1u)));
}

template <int B, bool SIGNED, bool LSB>
__device__ __forceinline__ uint32_t pcm_pack_native(int32_t v, uint32_t bits) {
  uint32_t s = (uint32_t)v;
  if (!SIGNED) s += 1u << (bits - 1u);
  if (LSB) s <<= (8u * B - bits);
  return s;
}

// Sample j (0..3) of a lane's quad from its B dwords w[] (stored bytes
// j*B .. j*B+B-1 of the quad), assembled in the stored byte order.
template <int B, bool BE>
__device__ __forceinline__ uint32_t pcm_from_words(const uint32_t* w, int j) {
  uint32_t t = 0;
#pragma unroll
  for (int k = 0; k < B; ++k) {
    const int byte = j * B + k;
    const uint32_t v = (w[byte >> 2] >> (8 * (byte & 3))) & 0xFFu;
    t |= v << (8 * (BE ? (B - 1 - k) : k));
  }
  return t;
}

template <int B>
__device__ __forceinline__ void pcm_load_words(const uint8_t* p, uint32_t* w) {
  if constexpr (B == 1) {
    w[0] = *reinterpret_cast<const uint32_t*>(p);
  } else if constexpr (B == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    w[0] = v.x; w[1] = v.y;
  } else if constexpr (B == 3) {
    // 12 bytes, 4-byte aligned: three adjacent dwords (one dwordx3 load)
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
    w[0] = q[0]; w[1] = q[1]; w[2] = q[2];
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  }
}

template <int B>
__device__ __forceinline__ void pcm_store_words(uint8_t* p, const uint32_t* w) {
  if constexpr (B == 1) {
    *reinterpret_cast<uint32_t*>(p) = w[0];
  } else if constexpr (B == 2) {
    *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
  } else if constexpr (B == 3) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    q[0] = w[0]; q[1] = w[1]; q[2] = w[2];
  } else {
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// vec: src 4-byte aligned and dst 16-byte aligned (checked on the host).
// A workgroup sweeps kPcmUnroll * 256 quads per trip: all loads of a trip are
// issued before the first store, so each lane keeps kPcmUnroll loads in flight.
template <int B, bool BE, bool SIGNED, bool LSB>
__global__ __launch_bounds__(kPcmThreads) void rpp_pcm_unpack_kernel(const uint8_t* __restrict__ src,
                                                                     int32_t* __restrict__ dst, uint64_t n,
                                                                     uint32_t bits, uint32_t vec) {
  const uint64_t tid = (uint64_t)blockIdx.x * kPcmThreads + threadIdx.x;
  uint64_t done = 0;
  if (vec) {
    const uint64_t quads = n / 4u;
    const uint64_t trip = (uint64_t)gridDim.x * kPcmThreads * kPcmUnroll;
    for (uint64_t q0 = (uint64_t)blockIdx.x * kPcmThreads * kPcmUnroll + threadIdx.x; q0 < quads; q0 += trip) {
      uint32_t w[kPcmUnroll][B];
#pragma unroll
      for (int u = 0; u < kPcmUnroll; ++u) {
        const uint64_t q = q0 + (uint64_t)u * kPcmThreads;
        if (q < quads) pcm_load_words<B>(src + q * (4u * B), w[u]);
      }
#pragma unroll
      for (int u = 0; u < kPcmUnroll; ++u) {
        const uint64_t q = q0 + (uint64_t)u * kPcmThreads;
        if (q < quads) {
          int4 o;
          o.x = pcm_unpack_native<B, SIGNED, LSB>(pcm_from_words<B, BE>(w[u], 0), bits);
          o.y = pcm_unpack_native<B, SIGNED, LSB>(pcm_from_words<B, BE>(w[u], 1), bits);
          o.z = pcm_unpack_native<B, SIGNED, LSB>(pcm_from_words<B, BE>(w[u], 2), bits);
          o.w = pcm_unpack_native<B, SIGNED, LSB>(pcm_from_words<B, BE>(w[u], 3), bits);
          *reinterpret_cast<int4*>(dst + q * 4u) = o;
        }
      }
    }
    done = quads * 4u;
  }
  const uint64_t stride = (uint64_t)gridDim.x * kPcmThreads;
  for (uint64_t i = done + tid; i < n; i += stride)
    dst[i] = pcm_unpack_native<B, SIGNED, LSB>(pcm_assemble<B, BE>(src + i * B), bits);
}

// vec: src 16-byte aligned and dst 4-byte aligned.
template <int B, bool BE, bool SIGNED, bool LSB>
__global__ __launch_bounds__(kPcmThreads) void rpp_pcm_pack_kernel(const int32_t* __restrict__ src,
                                                                   uint8_t* __restrict__ dst, uint64_t n,
                                                                   uint32_t bits, uint32_t vec) {
  const uint64_t tid = (uint64_t)blockIdx.x * kPcmThreads + threadIdx.x;
  uint64_t done = 0;
  if (vec) {
    const uint64_t quads = n / 4u;
    const uint64_t trip = (uint64_t)gridDim.x * kPcmThreads * kPcmUnroll;
    for (uint64_t q0 = (uint64_t)blockIdx.x * kPcmThreads * kPcmUnroll + threadIdx.x; q0 < quads; q0 += trip) {
      int4 v[kPcmUnroll];
#pragma unroll
      for (int u = 0; u < kPcmUnroll; ++u) {
        const uint64_t q = q0 + (uint64_t)u * kPcmThreads;
        if (q < quads) v[u] = *reinterpret_cast<const int4*>(src + q * 4u);
      }
#pragma unroll
      for (int u = 0; u < kPcmUnroll; ++u) {
        const uint64_t q = q0 + (uint64_t)u * kPcmThreads;
        if (q >= quads) continue;
        const uint32_t s[4] = {
            pcm_pack_native<B, SIGNED, LSB>(v[u].x, bits), pcm_pack_native<B, SIGNED, LSB>(v[u].y, bits),
            pcm_pack_native<B, SIGNED, LSB>(v[u].z, bits), pcm_pack_native<B, SIGNED, LSB>(v[u].w, bits)};
        uint32_t w[B];
#pragma unroll
        for (int i = 0; i < B; ++i) w[i] = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int k = 0; k < B; ++k) {
            const int byte = j * B + k;
            const uint32_t v8 = (s[j] >> (8 * (BE ? (B - 1 - k) : k))) & 0xFFu;
            w[byte >> 2] |= v8 << (8 * (byte & 3));
          }
        }
        pcm_store_words<B>(dst + q * (4u * B), w);
      }
    }
    done = quads * 4u;
  }
  const uint64_t stride = (uint64_t)gridDim.x * kPcmThreads;
  for (uint64_t i = done + tid; i < n; i += stride)
    pcm_scatter<B, BE>(dst + i * B, pcm_pack_native<B, SIGNED, LSB>(src[i], bits));
}

using UnpackFn = void (*)(const uint8_t*, int32_t*, uint64_t, uint32_t, uint32_t);
using PackFn = void (*)(const int32_t*, uint8_t*, uint64_t, uint32_t, uint32_t);

template <int B>
UnpackFn pick_unpack(int be, int sig, int lsb) {
  const int k = (be ? 4 : 0) | (sig ? 2 : 0) | (lsb ? 1 : 0);
  switch (k) {
  case 0: return rpp_pcm_unpack_kernel<B, false, false, false>;
  case 1: return rpp_pcm_unpack_kernel<B, false, false, true>;
  case 2: return rpp_pcm_unpack_kernel<B, false, true, false>;
  case 3: return rpp_pcm_unpack_kernel<B, false, true, true>;
  case 4: return rpp_pcm_unpack_kernel<B, true, false, false>;
  case 5: return rpp_pcm_unpack_kernel<B, true, false, true>;
  case 6: return rpp_pcm_unpack_kernel<B, true, true, false>;
  default: return rpp_pcm_unpack_kernel<B, true, true, true>;
  }
}

template <int B>
PackFn pick_pack(int be, int sig, int lsb) {
  const int k = (be ? 4 : 0) | (sig ? 2 : 0) | (lsb ? 1 : 0);
  switch (k) {
  case 0: return rpp_pcm_pack_kernel<B, false, false, false>;
  case 1: return rpp_pcm_pack_kernel<B, false, false, true>;
  case 2: return rpp_pcm_pack_kernel<B, false, true, false>;
  case 3: return rpp_pcm_pack_kernel<B, false, true, true>;
  case 4: return rpp_pcm_pack_kernel<B, true, false, false>;
  case 5: return rpp_pcm_pack_kernel<B, true, false, true>;
  case 6: return rpp_pcm_pack_kernel<B, true, true, false>;
  default: return rpp_pcm_pack_kernel<B, true, true, true>;
  }
}

uint32_t pcm_grid(uint64_t n) {
  const uint64_t quads = (n + 3u) / 4u;
  const uint64_t per_block = (uint64_t)kPcmThreads * kPcmUnroll;
  uint64_t blocks = (quads + per_block - 1u) / per_block;
  if (blocks > kPcmMaxBlocks) blocks = kPcmMaxBlocks;
  return (uint32_t)(blocks ? blocks : 1u);
}

}  // namespace

extern "C" int rpp_pcm_check_format(const rpp_pcm_format* f) {
  if (!f) return RPP_INVALID_ARGUMENT;
  if (f->bytes < 1u || f->bytes > 4u) return RPP_UNSUPPORTED_CONFIG;
  if (f->bits < 1u || f->bits > 8u * f->bytes) return RPP_INVALID_ARGUMENT;
  return RPP_OK;
}

extern "C" int rpp_pcm_unpack(const rpp_pcm_format* f, const uint8_t* d_src, int32_t* d_dst, uint64_t n_samples,
                              void* stream) {
  const int st = rpp_pcm_check_format(f);
  if (st != RPP_OK) return st;
  if (n_samples == 0) return RPP_OK;
  if (!d_src || !d_dst) return RPP_INVALID_ARGUMENT;
  const uint32_t vec = ((uintptr_t)d_src % 4u == 0 && (uintptr_t)d_dst % 16u == 0) ? 1u : 0u;
  UnpackFn fn = nullptr;
  switch (f->bytes) {
  case 1: fn = pick_unpack<1>(f->big_endian, f->is_signed, f->lsb_padded); break;
  case 2: fn = pick_unpack<2>(f->big_endian, f->is_signed, f->lsb_padded); break;
  case 3: fn = pick_unpack<3>(f->big_endian, f->is_signed, f->lsb_padded); break;
  default: fn = pick_unpack<4>(f->big_endian, f->is_signed, f->lsb_padded); break;
  }
  hipLaunchKernelGGL(fn, dim3(pcm_grid(n_samples)), dim3(kPcmThreads), 0, (hipStream_t)stream, d_src, d_dst,
                     n_samples, f->bits, vec);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

extern "C" int rpp_pcm_pack(const rpp_pcm_format* f, const int32_t* d_src, uint8_t* d_dst, uint64_t n_samples,
                            void* stream) {
  const int st = rpp_pcm_check_format(f);
  if (st != RPP_OK) return st;
  if (n_samples == 0) return RPP_OK;
  if (!d_src || !d_dst) return RPP_INVALID_ARGUMENT;
  const uint32_t vec = ((uintptr_t)d_src % 16u == 0 && (uintptr_t)d_dst % 4u == 0) ? 1u : 0u;
  PackFn fn = nullptr;
  switch (f->bytes) {
  case 1: fn = pick_pack<1>(f->big_endian, f->is_signed, f->lsb_padded); break;
  case 2: fn = pick_pack<2>(f->big_endian, f->is_signed, f->lsb_padded); break;
  case 3: fn = pick_pack<3>(f->big_endian, f->is_signed, f->lsb_padded); break;
  default: fn = pick_pack<4>(f->big_endian, f->is_signed, f->lsb_padded); break;
  }
  hipLaunchKernelGGL(fn, dim3(pcm_grid(n_samples)), dim3(kPcmThreads), 0, (hipStream_t)stream, d_src, d_dst,
                     n_samples, f->bits, vec);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}
