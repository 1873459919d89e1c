// ricepp_kernels.hip -- MI355X (gfx950) ricepp encode/decode kernels and the
// C ABI declared in include/ricepp_amd.h.
//
// Bitstream format: ricepp (mhx/dwarfs ricepp/, restated in SURVEY.md
// Appendix A).  One wavefront owns one independent stream (a DwarFS block);
// streams shard across the grid with no inter-wave communication.
//
// Encode (per wave, loop over groups of sub-blocks):
//   * a sub-block of `bs` samples is owned by an aligned group of G lanes
//     (G = next pow2 of ceil(bs/8)), each lane holding 8 samples;
//   * zig-zag deltas in registers, per-sub-block cost(fs) by group
//     reductions, exact replay of compute_best_split's hill climb
//     (ricepp/include/ricepp/detail/encode.h:43-90);
//   * code lengths -> one wave-wide prefix scan -> absolute bit positions;
//   * codes OR-ed into an LDS window (ds_or_b32), complete 16-byte chunks
//     streamed to HBM with coalesced dwordx4 stores.
// Decode (per wave, loop over sub-blocks):
//   * the 4-bit header is read wave-uniformly;
//   * a Rice sub-block is parsed in 2048-bit passes: lane l owns 32-bit
//     word l and finds its terminator bits ('1' ending each unary run) by a
//     chain that starts from a speculative entry state taken from its
//     left neighbour's word; entry states are then verified against the
//     left lane's exit state and re-run until consistent (self-synchronising
//     Rice codes converge in one or two rounds);
//   * codes -> values by wave prefix scans of code counts and deltas;
//   * values staged in LDS per chunk and flushed with vector stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace {

constexpr int kWave = 64;
constexpr int kWinWords = 512;   // encode LDS output window (2 KiB)
constexpr int kTileSamples = 1024;  // decode LDS chunk tile (cs*bs <= 1024)

// ---------------------------------------------------------------------------
// pixel traits (ricepp/ricepp_cpuspecific_traits.h:63-75)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v >> 8) | (v << 8)) & 0xFFFFu; }
__device__ __forceinline__ uint32_t px_read(uint32_t v, uint32_t be, uint32_t ulsb) {
  v &= 0xFFFFu;
  if (be) v = bswap16(v);
  return v >> ulsb;
}
__device__ __forceinline__ uint32_t px_write(uint32_t v, uint32_t be, uint32_t ulsb) {
  v = (v << ulsb) & 0xFFFFu;
  return be ? bswap16(v) : v;
}
// encode.h:116-123: d = diff & 0x8000 ? ~(diff << 1) : diff << 1 (16 bit)
__device__ __forceinline__ uint32_t zigzag16(uint32_t px, uint32_t prev) {
  uint32_t diff = (px - prev) & 0xFFFFu;
  return ((diff << 1) ^ (0u - (diff >> 15))) & 0xFFFFu;
}

// ---------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t shfl(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src); }
__device__ __forceinline__ uint32_t shfl_up(uint32_t v, int d) { return (uint32_t)__shfl_up((int)v, d); }
__device__ __forceinline__ uint32_t shfl_down(uint32_t v, int d) { return (uint32_t)__shfl_down((int)v, d); }
__device__ __forceinline__ uint32_t shfl_xor(uint32_t v, int m) { return (uint32_t)__shfl_xor((int)v, m); }

// sum over the aligned group of G lanes containing this lane (G pow2 <= 64)
__device__ __forceinline__ uint32_t group_sum(uint32_t v, uint32_t G) {
  for (uint32_t m = 1; m < G; m <<= 1) v += shfl_xor(v, (int)m);
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = shfl_up(v, d);
    if (l >= (uint32_t)d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  const uint32_t l = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = shfl_up(v, d);
    if (l >= (uint32_t)d) v = v > t ? v : t;
  }
  return v;
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// ===========================================================================
// ENCODE
// ===========================================================================
struct EncParams {
  const uint16_t* in;
  const uint64_t* in_off;
  const uint64_t* n_samples;
  uint8_t* out;
  const uint64_t* out_off;
  uint64_t* out_bytes;
  int32_t* status;
  uint32_t nblocks;
  uint32_t bs, cs, be, ulsb;
};

// Loads the `cnt` (<= 8) samples p[0], p[cs], ... ; unused slots are 0.
__device__ __forceinline__ void load8(const uint16_t* p, uint32_t cs, uint32_t comp, uint32_t cnt,
                                      uint32_t raw[8]) {
  if (cnt == 8 && cs == 1 && ((uintptr_t)p & 15) == 0) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    raw[0] = v.x & 0xFFFFu; raw[1] = v.x >> 16;
    raw[2] = v.y & 0xFFFFu; raw[3] = v.y >> 16;
    raw[4] = v.z & 0xFFFFu; raw[5] = v.z >> 16;
    raw[6] = v.w & 0xFFFFu; raw[7] = v.w >> 16;
  } else if (cnt == 8 && cs == 2 && ((uintptr_t)(p - comp) & 15) == 0) {
    const uint4* q = reinterpret_cast<const uint4*>(p - comp);
    uint4 a = q[0], b = q[1];
    uint32_t sh = 16 * comp;
    raw[0] = (a.x >> sh) & 0xFFFFu; raw[1] = (a.y >> sh) & 0xFFFFu;
    raw[2] = (a.z >> sh) & 0xFFFFu; raw[3] = (a.w >> sh) & 0xFFFFu;
    raw[4] = (b.x >> sh) & 0xFFFFu; raw[5] = (b.y >> sh) & 0xFFFFu;
    raw[6] = (b.z >> sh) & 0xFFFFu; raw[7] = (b.w >> sh) & 0xFFFFu;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) raw[i] = (uint32_t)i < cnt ? (uint32_t)p[cs * i] : 0u;
  }
}

__device__ __forceinline__ uint32_t shr_sum8(const uint32_t d[8], uint32_t f) {
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += d[i] >> f;
  return s;
}

// ORs the (<= 16 bit) code `v` into the window at bit `rel`.
__device__ __forceinline__ void emit_bits(uint32_t* win, uint32_t rel, uint32_t v) {
  uint32_t w = rel >> 5, sh = rel & 31u;
  atomicOr(&win[w], v << sh);
  if (sh) {
    uint32_t hi = v >> (32u - sh);
    if (hi) atomicOr(&win[w + 1], hi);
  }
}

__global__ __launch_bounds__(kWave) void rpp_encode_kernel(EncParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t win[kWinWords];
  const uint32_t b = blockIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t bs = p.bs, cs = p.cs, be = p.be, ulsb = p.ulsb;
  const uint64_t n64 = p.n_samples[b];
  const uint64_t ooff = p.out_off[b];
  if (n64 % cs != 0 || n64 >= RPP_MAX_STREAM_SAMPLES || (ooff & 15u)) {
    if (lane == 0) {
      p.status[b] = RPP_INVALID_ARGUMENT;
      p.out_bytes[b] = 0;
    }
    return;
  }
  const uint32_t N = (uint32_t)n64;
  const uint16_t* in = p.in + p.in_off[b];
  uint8_t* out8 = p.out + ooff;
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out8);

  for (uint32_t i = lane; i < (uint32_t)kWinWords; i += kWave) win[i] = 0;
  __syncthreads();

  // codec.h:69-74,81-86: 16-bit initial value read(in[i]) per component.
  if (lane < cs) emit_bits(win, 16 * lane, N ? px_read(in[lane], be, ulsb) : 0u);
  uint32_t win_w0 = 0;      // global word index held in win[0]
  uint32_t base = 16 * cs;  // absolute bit position of the next sub-block

  const uint32_t chunk_len = cs * bs;
  const uint32_t nchunks = (N + chunk_len - 1) / chunk_len;
  const uint32_t nsb = nchunks * cs;
  const uint32_t m8 = (bs + 7) >> 3;
  uint32_t G = 1;
  while (G < m8) G <<= 1;
  const uint32_t spw = kWave / G;
  const uint32_t g = lane / G, j = lane & (G - 1);

  for (uint32_t s0 = 0; s0 < nsb; s0 += spw) {
    // ---- sub-block geometry (codec.h:88-97: chunk of cs*bs, component i
    //      takes samples i, i+cs, ...) ----
    const uint32_t s = s0 + g;
    const bool sb_valid = s < nsb;
    const uint32_t chunk = s / cs, comp = s - chunk * cs;
    const uint32_t cbase = chunk * chunk_len;
    uint32_t n = 0;
    if (sb_valid) {
      uint32_t rem = (N - cbase) / cs;
      n = rem < bs ? rem : bs;
    }
    const uint32_t k0 = 8 * j;
    const uint32_t cnt = k0 < n ? (n - k0 < 8 ? n - k0 : 8) : 0;
    const uint32_t m_first = cbase + comp + cs * k0;

    // ---- zig-zag deltas (encode.h:116-123) ----
    uint32_t raw[8], d[8];
    load8(in + m_first, cs, comp, cnt, raw);
    uint32_t prev = 0;
    if (cnt) prev = px_read(m_first >= cs ? (uint32_t)in[m_first - cs] : raw[0], be, ulsb);
    uint32_t lsum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t px = px_read(raw[i], be, ulsb);
      d[i] = (uint32_t)i < cnt ? zigzag16(px, prev) : 0u;
      prev = (uint32_t)i < cnt ? px : prev;
      lsum += d[i];
    }
    const uint32_t sum = group_sum(lsum, G);

    // ---- compute_best_split replay (encode.h:43-90) ----
    const uint32_t avg = n ? sum / n : 0u;
    const uint32_t bw = avg ? 32u - (uint32_t)__clz(avg) : 0u;
    const uint32_t start = bw >= 2 ? bw - 2 : 0u;
    const uint32_t bits0 = n * (start + 1) + group_sum(shr_sum8(d, start), G);
    const uint32_t bits1 = n * (start + 2) + group_sum(shr_sum8(d, start + 1), G);
    int cand, dir;
    uint32_t bits;
    if (bits1 <= bits0) {
      cand = (int)start + 1; bits = bits1; dir = 1;
    } else {
      cand = (int)start; bits = bits0; dir = -1;
    }
    bool walking = sb_valid && sum != 0 && bits0 != bits1;
    for (;;) {
      const bool act = walking && cand > 0 && cand < 14;
      if (!__any(act)) break;
      const uint32_t f = act ? (uint32_t)(cand + dir) : 0u;
      const uint32_t t = n * (f + 1) + group_sum(shr_sum8(d, f), G);
      if (act) {
        if (t > bits) {
          walking = false;
        } else {
          bits = t;
          cand += dir;
        }
      } else {
        walking = false;
      }
    }
    // encode.h:127-156: 0 = all-zero, 1 = Rice, 2 = raw
    uint32_t mode = 0, fs = 0;
    if (sb_valid && sum != 0) {
      fs = (uint32_t)cand;
      mode = (fs < 14 && bits < 16 * n) ? 1u : 2u;
    }

    // ---- bit positions: one wave-wide scan ----
    uint32_t lbits = (sb_valid && j == 0) ? 4u : 0u;
    if (mode == 1) lbits += shr_sum8(d, fs) + cnt * (fs + 1);
    else if (mode == 2) lbits += 16 * cnt;
    const uint32_t incl = wave_incl_sum(lbits);
    const uint32_t total = readlane(incl, kWave - 1);
    uint32_t pos = base + incl - lbits - 32 * win_w0;  // window-relative

    // ---- emit codes into the LDS window ----
    if (sb_valid && j == 0) {
      emit_bits(win, pos, mode == 0 ? 0u : (mode == 1 ? fs + 1 : 15u));
      pos += 4;
    }
    if (mode == 1) {
      const uint32_t lowmask = (1u << fs) - 1u;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if ((uint32_t)i < cnt) {
          pos += d[i] >> fs;  // unary zeros are implicit (window is zeroed)
          emit_bits(win, pos, 1u | ((d[i] & lowmask) << 1));
          pos += fs + 1;
        }
      }
    } else if (mode == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if ((uint32_t)i < cnt) {
          emit_bits(win, pos, raw[i]);  // raw stored value (encode.h:148-151)
          pos += 16;
        }
      }
    }
    base += total;
    __syncthreads();

    // ---- stream completed 16-byte chunks to HBM ----
    const uint32_t full_end = base >> 5;
    const uint32_t F = full_end & ~3u;
    if (F > win_w0) {
      const uint32_t nch = (F - win_w0) >> 2;
      for (uint32_t c = lane; c < nch; c += kWave) {
        uint4 v = *reinterpret_cast<const uint4*>(&win[4 * c]);
        *reinterpret_cast<uint4*>(&out32[win_w0 + 4 * c]) = v;
      }
      const uint32_t used = full_end - win_w0 + 1;
      const uint32_t tail0 = F - win_w0;
      uint32_t keep = lane < 4 ? win[tail0 + lane] : 0u;
      __syncthreads();
      for (uint32_t i = lane; i < used && i < (uint32_t)kWinWords; i += kWave) win[i] = 0;
      __syncthreads();
      if (lane < 4) win[lane] = keep;
      __syncthreads();
      win_w0 = F;
    }
  }

  // ---- final flush: full words, then the ceil(bits/8) tail bytes
  //      (bitstream_writer.h:110-120,139-145) ----
  const uint32_t total_bytes = (base + 7) >> 3;
  const uint32_t full_end = base >> 5;
  for (uint32_t w = win_w0 + lane; w < full_end; w += kWave) out32[w] = win[w - win_w0];
  const uint32_t tail_bytes = total_bytes - 4 * full_end;
  if (lane < tail_bytes) out8[4 * full_end + lane] = (uint8_t)(win[full_end - win_w0] >> (8 * lane));
  if (lane == 0) {
    p.out_bytes[b] = total_bytes;
    p.status[b] = RPP_OK;
  }
}

// ===========================================================================
// DECODE
// ===========================================================================
struct DecParams {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint64_t* in_bytes;
  uint16_t* out;
  const uint64_t* out_off;
  const uint64_t* n_samples;
  int32_t* status;
  uint32_t nblocks;
  uint32_t bs, cs, be, ulsb;
};

// 32-bit word `w` of the stream, zero past the end (bitstream_reader.h:165-166
// zero-pads the last packet; reading beyond it is checked separately).
__device__ __forceinline__ uint32_t stream_word(const uint8_t* in, uint32_t nbytes, uint32_t w) {
  const uint32_t byte0 = w * 4u;
  if (byte0 >= nbytes) return 0u;
  if (nbytes - byte0 >= 4) return *reinterpret_cast<const uint32_t*>(in + byte0);
  uint32_t v = 0;
  for (uint32_t k = 0; k < nbytes - byte0; ++k) v |= (uint32_t)in[byte0 + k] << (8 * k);
  return v;
}

// `width` (<= 16) bits at absolute bit position `pos`, LSB first.
__device__ __forceinline__ uint32_t stream_bits(const uint8_t* in, uint32_t nbytes, uint32_t pos,
                                                uint32_t width) {
  const uint32_t w = pos >> 5, sh = pos & 31u;
  uint64_t v = (uint64_t)stream_word(in, nbytes, w) | ((uint64_t)stream_word(in, nbytes, w + 1) << 32);
  return (uint32_t)(v >> sh) & ((1u << width) - 1u);
}

// Terminator chain through one 32-bit word: starting the unary search at bit
// `entry`, mark every '1' that ends a unary run and skip its fs remainder
// bits.  Returns the terminator mask; *exit = where the search continues in
// the next word (0 if it runs off the word while searching).
__device__ __forceinline__ uint32_t chain_word(uint32_t word, uint32_t entry, uint32_t fs,
                                               uint32_t* exit) {
  uint32_t T = 0, sigma = entry, ex = 0;
  while (sigma < 32) {
    const uint32_t y = word >> sigma;
    if (y == 0) break;
    const uint32_t t = sigma + (uint32_t)__builtin_ctz(y);
    T |= 1u << t;
    sigma = t + fs + 1;
  }
  if (sigma >= 32) ex = sigma - 32;
  *exit = ex;
  return T;
}

__device__ __forceinline__ void set_status(int32_t* st, uint32_t b, int32_t v) {
  if (lane_id() == 0) st[b] = v;
}

__global__ __launch_bounds__(kWave) void rpp_decode_kernel(DecParams p) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[kTileSamples];
  const uint32_t b = blockIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t bs = p.bs, cs = p.cs, be = p.be, ulsb = p.ulsb;
  const uint64_t n64 = p.n_samples[b];
  const uint64_t ioff = p.in_off[b];
  const uint64_t nbytes64 = p.in_bytes[b];
  if (n64 % cs != 0 || n64 >= RPP_MAX_STREAM_SAMPLES || (ioff & 3u) || nbytes64 >= (UINT64_C(1) << 29)) {
    set_status(p.status, b, RPP_INVALID_ARGUMENT);
    return;
  }
  const uint32_t N = (uint32_t)n64;
  const uint32_t nbytes = (uint32_t)nbytes64;
  const uint8_t* in = p.in + ioff;
  uint16_t* out = p.out + p.out_off[b];
  // last readable bit + 1: the reader pulls whole 8-byte packets
  // (bitstream_reader.h:149-183), so it only throws past this point.
  const uint32_t lim = 64u * ((nbytes + 7u) >> 3);

  if (16 * cs > lim) {
    set_status(p.status, b, RPP_TRUNCATED_INPUT);
    return;
  }
  uint32_t last[2];
  last[0] = stream_bits(in, nbytes, 0, 16);
  last[1] = cs > 1 ? stream_bits(in, nbytes, 16, 16) : 0u;
  uint32_t P = 16 * cs;

  const uint32_t chunk_len = cs * bs;
  const uint32_t nchunks = (N + chunk_len - 1) / chunk_len;
  for (uint32_t chunk = 0; chunk < nchunks; ++chunk) {
    const uint32_t cbase = chunk * chunk_len;
    const uint32_t clen = N - cbase < chunk_len ? N - cbase : chunk_len;
    const uint32_t n = clen / cs;
    for (uint32_t comp = 0; comp < cs; ++comp) {
      // decode.h:60: 4-bit fs+1 header
      if (P + 4 > lim) {
        set_status(p.status, b, RPP_TRUNCATED_INPUT);
        return;
      }
      const uint32_t fsp1 = stream_bits(in, nbytes, P, 4);
      P += 4;
      uint32_t acc = last[comp];
      if (fsp1 == 0) {
        // decode.h:79-80: all samples = write(last)
        const uint32_t v = px_write(acc, be, ulsb);
        for (uint32_t k = lane; k < n; k += kWave) tile[comp + cs * k] = (uint16_t)v;
      } else if (fsp1 == 15) {
        // decode.h:72-77: raw stored values; last = read(last sample)
        if ((uint64_t)P + 16ull * n > lim) {
          set_status(p.status, b, RPP_TRUNCATED_INPUT);
          return;
        }
        for (uint32_t k = lane; k < n; k += kWave)
          tile[comp + cs * k] = (uint16_t)stream_bits(in, nbytes, P + 16 * k, 16);
        acc = px_read(stream_bits(in, nbytes, P + 16 * (n - 1), 16), be, ulsb);
        P += 16 * n;
      } else {
        // decode.h:62-71: Rice codes, fs = fsp1 - 1
        const uint32_t fs = fsp1 - 1;
        const uint32_t lowmask = (1u << fs) - 1u;
        uint32_t K = 0;             // codes decoded in earlier passes
        uint32_t sigma_carry = P;   // search start of the next code
        uint32_t W0 = P >> 5;       // first word of this pass
        uint32_t e0 = P & 31u;      // exact entry state of lane 0
        for (;;) {
          if (32ull * W0 >= lim) {
            set_status(p.status, b, RPP_TRUNCATED_INPUT);
            return;
          }
          const uint32_t own = stream_word(in, nbytes, W0 + lane);
          uint32_t nxt = shfl_down(own, 1);
          if (lane == kWave - 1) nxt = stream_word(in, nbytes, W0 + kWave);
          const uint32_t prv = shfl_up(own, 1);
          // speculative entry state from the left neighbour's word
          uint32_t entry = e0, ex;
          if (lane != 0) chain_word(prv, 0, fs, &entry);
          uint32_t T = chain_word(own, entry, fs, &ex);
          // verify entry == left lane's exit; re-run until consistent
          for (;;) {
            const uint32_t left_exit = shfl_up(ex, 1);
            const bool bad = lane != 0 && left_exit != entry;
            if (!__any(bad)) break;
            if (bad) {
              entry = left_exit;
              T = chain_word(own, entry, fs, &ex);
            }
          }
          const uint32_t c = (uint32_t)__builtin_popcount(T);
          const uint32_t cincl = wave_incl_sum(c);
          const uint32_t cexcl = cincl - c;
          const uint32_t ctot = readlane(cincl, kWave - 1);
          const uint32_t wbit = 32u * (W0 + lane);
          const uint32_t my_last_sigma = c ? wbit + (31u - (uint32_t)__clz(T)) + fs + 1 : 0u;
          const uint32_t smax = wave_incl_max(my_last_sigma);
          uint32_t sprev = shfl_up(smax, 1);
          if (lane == 0) sprev = 0;
          const uint32_t sigma_in = sprev > sigma_carry ? sprev : sigma_carry;
          const uint64_t own64 = (uint64_t)own | ((uint64_t)nxt << 32);

          // pass A: this lane's delta sum over codes with index < n
          uint32_t dsum = 0;
          {
            uint32_t TT = T, sig = sigma_in, k = K + cexcl;
            while (TT) {
              const uint32_t t = (uint32_t)__builtin_ctz(TT);
              TT &= TT - 1;
              const uint32_t tabs = wbit + t;
              const uint32_t q = tabs - sig;
              const uint32_t rem = (uint32_t)(own64 >> (t + 1)) & lowmask;
              const uint32_t diff = (q << fs) | rem;
              const uint32_t delta = (diff >> 1) ^ (0u - (diff & 1u));
              if (k < n) dsum += delta;
              ++k;
              sig = tabs + fs + 1;
            }
          }
          const uint32_t dincl = wave_incl_sum(dsum);
          // pass B: values
          uint32_t endpos = 0;
          {
            uint32_t TT = T, sig = sigma_in, k = K + cexcl;
            uint32_t v = acc + dincl - dsum;
            while (TT) {
              const uint32_t t = (uint32_t)__builtin_ctz(TT);
              TT &= TT - 1;
              const uint32_t tabs = wbit + t;
              const uint32_t q = tabs - sig;
              const uint32_t rem = (uint32_t)(own64 >> (t + 1)) & lowmask;
              const uint32_t diff = (q << fs) | rem;
              v += (diff >> 1) ^ (0u - (diff & 1u));
              if (k < n) tile[comp + cs * k] = (uint16_t)px_write(v, be, ulsb);
              if (k == n - 1) endpos = tabs + fs + 1;
              ++k;
              sig = tabs + fs + 1;
            }
          }
          if (K + ctot >= n) {
            const uint32_t idx = n - 1 - K;
            const uint64_t owner = __ballot(cexcl <= idx && idx < cincl);
            const int L = (int)__builtin_ctzll(owner);
            const uint32_t E = readlane(endpos, L);
            acc += readlane(dincl, kWave - 1);
            if (E > lim) {
              set_status(p.status, b, RPP_TRUNCATED_INPUT);
              return;
            }
            P = E;
            break;
          }
          K += ctot;
          acc += readlane(dincl, kWave - 1);
          const uint32_t sm = readlane(smax, kWave - 1);
          sigma_carry = sm > sigma_carry ? sm : sigma_carry;
          e0 = readlane(ex, kWave - 1);
          W0 += kWave;
        }
      }
      last[comp] = acc & 0xFFFFu;
    }
    __syncthreads();
    // ---- flush the chunk tile ----
    uint16_t* dst = out + cbase;
    if (((uintptr_t)dst & 15) == 0 && (clen & 7) == 0) {
      for (uint32_t i = lane; i < clen / 8; i += kWave)
        reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(tile)[i];
    } else {
      for (uint32_t i = lane; i < clen; i += kWave) dst[i] = tile[i];
    }
    __syncthreads();
  }
  set_status(p.status, b, RPP_OK);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

uint32_t rpp_abi_version(void) { return 1; }

int rpp_check_config(const rpp_config* c) {
  if (!c) return RPP_INVALID_ARGUMENT;
  if (c->block_size == 0 || c->block_size > 512) return RPP_UNSUPPORTED_CONFIG;
  if (c->component_stream_count != 1 && c->component_stream_count != 2) return RPP_UNSUPPORTED_CONFIG;
  if (c->unused_lsb_count >= 16) return RPP_UNSUPPORTED_CONFIG;
  return RPP_OK;
}

uint64_t rpp_worst_case_bytes(const rpp_config* c, uint64_t n) {
  if (rpp_check_config(c) != RPP_OK) return 0;
  const uint64_t cs = c->component_stream_count, bs = c->block_size;
  const uint64_t per = n / cs;
  const uint64_t num = 16 + 4 * ((per + bs - 1) / bs) + 16 * per;
  return (num * cs + 7) / 8;
}

int rpp_encode_batch(const rpp_config* cfg, const uint16_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_n_samples, uint32_t nblocks, uint8_t* d_out,
                     const uint64_t* d_out_offsets, uint64_t* d_out_bytes, int32_t* d_status,
                     void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_n_samples || !d_out || !d_out_offsets || !d_out_bytes || !d_status)
    return RPP_INVALID_ARGUMENT;
  EncParams p{d_in, d_in_offsets, d_n_samples, d_out, d_out_offsets, d_out_bytes, d_status, nblocks,
              cfg->block_size, cfg->component_stream_count, cfg->big_endian ? 1u : 0u,
              cfg->unused_lsb_count};
  hipLaunchKernelGGL(rpp_encode_kernel, dim3(nblocks), dim3(kWave), 0, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

int rpp_decode_batch(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out,
                     const uint64_t* d_out_offsets, const uint64_t* d_n_samples, int32_t* d_status,
                     void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_in_bytes || !d_out || !d_out_offsets || !d_n_samples || !d_status)
    return RPP_INVALID_ARGUMENT;
  if (cfg->component_stream_count * cfg->block_size > (uint32_t)kTileSamples) return RPP_UNSUPPORTED_CONFIG;
  DecParams p{d_in, d_in_offsets, d_in_bytes, d_out, d_out_offsets, d_n_samples, d_status, nblocks,
              cfg->block_size, cfg->component_stream_count, cfg->big_endian ? 1u : 0u,
              cfg->unused_lsb_count};
  hipLaunchKernelGGL(rpp_decode_kernel, dim3(nblocks), dim3(kWave), 0, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // extern "C"
