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

#ifdef RPP_STATS
// Diagnostic build only (-DRPP_STATS): loop trip counters, summed over waves.
__device__ unsigned long long g_rpp_stats[16];
#define RPP_STAT(i, v) (stat_acc[i] += (v))
// phase timer: adds the s_memtime delta since the previous stamp to slot i
#define RPP_TSTAMP(i)                                                   \
  do {                                                                  \
    unsigned long long now_;                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(now_)::"memory"); \
    stat_acc[i] += (uint32_t)(now_ - tprev_);                            \
    tprev_ = now_;                                                      \
  } while (0)
#else
#define RPP_STAT(i, v) ((void)0)
#define RPP_TSTAMP(i) ((void)0)
#endif

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

// DPP controls (gfx9 encoding)
constexpr int kDppQuadXor1 = 0xB1;     // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;     // quad_perm [2,3,0,1]
constexpr int kDppRowShr1 = 0x111;
constexpr int kDppRowShr2 = 0x112;
constexpr int kDppRowShr4 = 0x114;
constexpr int kDppRowShr8 = 0x118;
constexpr int kDppWaveShr1 = 0x138;
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  // lanes whose source is outside the row / not selected read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, 0xF, false);
}

// Sum over the aligned group of G lanes containing this lane (G pow2 <= 64),
// broadcast to every lane of the group.  All lanes must be active.
__device__ __forceinline__ uint32_t group_sum(uint32_t v, uint32_t G) {
  if (G >= 2) v += dpp<kDppQuadXor1>(v);
  if (G >= 4) v += dpp<kDppQuadXor2>(v);
  if (G >= 8) v += dpp<kDppRowHalfMirror>(v);
  if (G >= 16) v += dpp<kDppRowMirror>(v);
  if (G >= 32) {
    auto t = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = t[0] + t[1];
  }
  if (G >= 64) {
    auto t = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = t[0] + t[1];
  }
  return v;
}

// Inclusive prefix sum over the 64 lanes (all active).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  v += dpp<kDppRowShr1>(v);
  v += dpp<kDppRowShr2>(v);
  v += dpp<kDppRowShr4>(v);
  v += dpp<kDppRowShr8>(v);
  v += dpp<kDppRowBcast15, 0xA>(v);
  v += dpp<kDppRowBcast31, 0xC>(v);
  return v;
}

// Inclusive prefix max over the 64 lanes (all active, values >= 0).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, dpp<kDppRowShr1>(v));
  v = max(v, dpp<kDppRowShr2>(v));
  v = max(v, dpp<kDppRowShr4>(v));
  v = max(v, dpp<kDppRowShr8>(v));
  v = max(v, dpp<kDppRowBcast15, 0xA>(v));
  v = max(v, dpp<kDppRowBcast31, 0xC>(v));
  return v;
}

// Value of lane l-1 (0 for lane 0).
__device__ __forceinline__ uint32_t from_left(uint32_t v) { return dpp<kDppWaveShr1>(v); }

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

// Per-lane sub-block geometry of one encode iteration.
struct EncGeom {
  uint32_t n;        // samples in this lane's sub-block (0: no sub-block)
  uint32_t cnt;      // samples owned by this lane (<= 8)
  uint32_t m_first;  // stream index of the lane's first sample
  uint32_t comp;     // component stream
};

__device__ __forceinline__ EncGeom enc_geom(uint32_t s, uint32_t j, uint32_t nsb, uint32_t N, uint32_t bs,
                                            uint32_t cs) {
  EncGeom g;
  // codec.h:88-97: chunks of cs*bs samples; component i takes i, i+cs, ...
  const uint32_t chunk = cs == 1 ? s : s >> 1;
  g.comp = s - chunk * cs;
  const uint32_t cbase = chunk * cs * bs;
  g.n = 0;
  if (s < nsb) {
    const uint32_t rem = (N - cbase) / cs;
    g.n = rem < bs ? rem : bs;
  }
  const uint32_t k0 = 8 * j;
  g.cnt = k0 < g.n ? min(g.n - k0, 8u) : 0u;
  g.m_first = cbase + g.comp + cs * k0;
  return g;
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef short ss2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 as_us2(uint32_t v) { return __builtin_bit_cast(us2, v); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }

// The lane's 8 stored samples as 4 packed pairs (sample 2k in the low half
// of w[k]) plus the previous same-component sample (the delta reference).
struct EncRaw {
  uint4 a, c;     // cs == 1: a holds the 8 samples; cs == 2: a, c hold 16 interleaved
  uint32_t prev;  // samples, this lane's component is picked at use (not at load)
};

__device__ __forceinline__ void enc_words(const EncRaw& r, uint32_t cs, uint32_t comp, uint32_t w[4]) {
  if (cs == 1) {
    w[0] = r.a.x; w[1] = r.a.y; w[2] = r.a.z; w[3] = r.a.w;
  } else {
    const uint32_t sel = comp ? 0x07060302u : 0x05040100u;
    w[0] = __builtin_amdgcn_perm(r.a.y, r.a.x, sel);
    w[1] = __builtin_amdgcn_perm(r.a.w, r.a.z, sel);
    w[2] = __builtin_amdgcn_perm(r.c.y, r.c.x, sel);
    w[3] = __builtin_amdgcn_perm(r.c.w, r.c.z, sel);
  }
}

// Full iterations (every lane owns 0 or 8 samples): branch-free 16-byte
// loads, so a double-buffered prefetch stays in flight.
__device__ __forceinline__ EncRaw enc_load_vec(const uint16_t* in, const EncGeom& g, uint32_t cs) {
  EncRaw r;
  // codec.h:72-73: a component's first sample is its own reference (last = read(in[i]))
  const uint32_t pi = g.cnt ? (g.m_first >= cs ? g.m_first - cs : g.m_first) : 0u;
  r.prev = in[pi];
  const uint4* q = reinterpret_cast<const uint4*>(g.cnt ? in + (g.m_first - g.comp) : in);
  r.a = q[0];
  r.c = cs == 2 ? q[1] : r.a;
  return r;
}

// Ragged tail / unaligned streams: per-sample loads.
__device__ __forceinline__ EncRaw enc_load_scalar(const uint16_t* in, const EncGeom& g, uint32_t cs) {
  EncRaw r;
  const uint32_t pi = g.m_first >= cs ? g.m_first - cs : g.m_first;
  r.prev = g.cnt ? (uint32_t)in[pi] : 0u;
  uint32_t v[8];
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) v[i] = i < g.cnt ? (uint32_t)in[g.m_first + cs * i] : 0u;
  // stored as the cs == 1 layout (this lane's samples only)
  r.a = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
  r.c = r.a;
  return r;
}

// ORs the (<= 16 bit) code `v` into the window at bit `rel` (two ds_or_b32;
// the second is 0 when the code does not straddle a word).
__device__ __forceinline__ void emit_bits(uint32_t* win, uint32_t rel, uint32_t v) {
  const uint32_t w = rel >> 5, sh = rel & 31u;
  atomicOr(&win[w], v << sh);
  atomicOr(&win[w + 1], (v >> 1) >> (31u - sh));
}

constexpr uint32_t kEncWin = 1024;      // LDS output window (words, 4 KiB)
constexpr uint32_t kEncFlushWords = 256;  // stream out once >= 1 KiB of whole 64-byte lines is ready

struct EncState {
  uint32_t* win;
  uint32_t* out32;
  uint32_t win_w0;  // global word index held in win[0] (multiple of 16)
  uint32_t base;    // absolute bit position of the next sub-block
};

// One group of 64/G sub-blocks: zig-zag deltas, compute_best_split replay,
// bit positions by one wave scan, codes OR-ed into the LDS window.
__device__ __forceinline__ void enc_iteration(EncState& st, const EncRaw& r, const EncGeom& geo, uint32_t G,
                                              uint32_t j, uint32_t be, uint32_t ulsb, bool mask_tail,
                                              uint32_t cs_layout) {
  const uint32_t n = geo.n, cnt = geo.cnt;
  uint32_t rw[4];
  enc_words(r, cs_layout, geo.comp, rw);
  const bool sb_valid = n != 0;
  // ---- pixel values (ricepp_cpuspecific_traits.h:63-67) and zig-zag deltas
  //      (encode.h:116-123), two samples per instruction ----
  us2 v[4], d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = be ? __builtin_amdgcn_perm(rw[k], rw[k], 0x02030001u) : rw[k];
    v[k] = as_us2(x) >> (us2)(unsigned short)ulsb;
  }
  const uint32_t pv = px_read(r.prev, be, ulsb);
  uint32_t prevw = pv << 16;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const us2 pp = as_us2(__builtin_amdgcn_alignbit(as_u32(v[k]), prevw, 16));
    prevw = as_u32(v[k]);
    const us2 diff = v[k] - pp;
    d[k] = (diff << (us2)1) ^ as_us2(__builtin_bit_cast(uint32_t, (__builtin_bit_cast(ss2, diff) >> (ss2)15)));
  }
  if (mask_tail) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t keep = (2u * k < cnt ? 0xFFFFu : 0u) | (2u * k + 1 < cnt ? 0xFFFF0000u : 0u);
      d[k] = as_us2(as_u32(d[k]) & keep);
    }
  }
  const us2 one = {1, 1};
  uint32_t lsum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) lsum = __builtin_amdgcn_udot2(d[k], one, lsum, false);
  auto shr_sum = [&](uint32_t f) -> uint32_t {
    const us2 fv = (us2)(unsigned short)f;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_udot2(d[k] >> fv, one, acc, false);
    return acc;
  };
  const uint32_t sum = group_sum(lsum, G);

  // ---- compute_best_split replay (encode.h:43-90) ----
  // start = max(0, bit_width(sum / n) - 2) without a division:
  // bit_width(floor(s/n)) = t + (s >= n << t), t = floor(log2 s) - floor(log2 n)
  uint32_t bwq = 0;
  if (n != 0 && sum >= n) {
    const uint32_t t = (uint32_t)__clz(n) - (uint32_t)__clz(sum);
    bwq = t + ((n << t) <= sum ? 1u : 0u);
  }
  const uint32_t start = bwq >= 2 ? bwq - 2 : 0u;
  const uint32_t bits0 = n * (start + 1) + group_sum(shr_sum(start), G);
  const uint32_t bits1 = n * (start + 2) + group_sum(shr_sum(start + 1), G);
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
    const uint32_t t = n * (f + 1) + group_sum(shr_sum(f), G);
    if (act && t <= bits) {
      bits = t;
      cand += dir;
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
  if (mode == 1) lbits += shr_sum(fs) + cnt * (fs + 1);
  else if (mode == 2) lbits += 16 * cnt;
  const uint32_t incl = wave_incl_sum(lbits);
  const uint32_t total = readlane(incl, kWave - 1);
  uint32_t pos = st.base + incl - lbits - 32 * st.win_w0;  // window-relative

  // ---- emit codes into the LDS window ----
  if (sb_valid && j == 0) {
    emit_bits(st.win, pos, mode == 0 ? 0u : (mode == 1 ? fs + 1 : 15u));
    pos += 4;
  }
  if (mode == 1) {
    const uint32_t lowmask = (1u << fs) - 1u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if ((uint32_t)i < cnt) {
        const uint32_t di = (i & 1) ? (as_u32(d[i >> 1]) >> 16) : (as_u32(d[i >> 1]) & 0xFFFFu);
        pos += di >> fs;  // unary zeros are implicit (the window is zeroed)
        emit_bits(st.win, pos, 1u | ((di & lowmask) << 1));
        pos += fs + 1;
      }
    }
  } else if (mode == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if ((uint32_t)i < cnt) {
        const uint32_t ri = (i & 1) ? (rw[i >> 1] >> 16) : (rw[i >> 1] & 0xFFFFu);
        emit_bits(st.win, pos, ri);  // raw stored value (encode.h:148-151)
        pos += 16;
      }
    }
  }
  st.base += total;
}

// Streams whole 64-byte lines out once >= kEncFlushWords are complete.
__device__ __forceinline__ void enc_flush(EncState& st, bool final_flush) {
  const uint32_t lane = lane_id();
  __syncthreads();
  const uint32_t full_end = st.base >> 5;  // words before it are complete
  const uint32_t F = full_end & ~15u;
  if (F >= st.win_w0 + kEncFlushWords || (final_flush && F > st.win_w0)) {
    const uint32_t nch = (F - st.win_w0) >> 2;
    for (uint32_t c = lane; c < nch; c += kWave) {
      const uint4 v = *reinterpret_cast<const uint4*>(&st.win[4 * c]);
      *reinterpret_cast<uint4*>(&st.out32[st.win_w0 + 4 * c]) = v;
    }
    const uint32_t used = full_end - st.win_w0 + 1;
    const uint32_t tail0 = F - st.win_w0;
    const uint32_t keep = lane < 16 ? st.win[tail0 + lane] : 0u;
    __syncthreads();
    for (uint32_t i = lane; i < used; i += kWave) st.win[i] = 0;
    __syncthreads();
    if (lane < 16) st.win[lane] = keep;
    __syncthreads();
    st.win_w0 = F;
  }
}

__global__ __launch_bounds__(kWave) void rpp_encode_kernel(EncParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t win[kEncWin];
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

  for (uint32_t i = lane; i < kEncWin; i += kWave) win[i] = 0;
  __syncthreads();

  EncState st{win, reinterpret_cast<uint32_t*>(out8), 0u, 16 * cs};
  // codec.h:69-74,81-86: 16-bit initial value read(in[i]) per component.
  if (lane < cs) emit_bits(win, 16 * lane, N ? px_read(in[lane], be, ulsb) : 0u);

  const uint32_t chunk_len = cs * bs;
  const uint32_t nchunks = (N + chunk_len - 1) / chunk_len;
  const uint32_t nsb = nchunks * cs;
  const uint32_t m8 = (bs + 7) >> 3;
  uint32_t G = 1;
  while (G < m8) G <<= 1;
  const uint32_t spw = kWave / G;
  const uint32_t g = lane / G, j = lane & (G - 1);
  // full iterations: every sub-block complete, lanes own 0 or 8 samples
  const bool vec_ok = (bs & 7u) == 0 && ((uintptr_t)in & 15u) == 0;
  const uint32_t nsb_full = vec_ok ? (N / chunk_len) * cs : 0u;
  const uint32_t nfull = nsb_full / spw;
  const bool empty_lanes = G * 8 != bs;

  // ---- full iterations, double buffered (no register copies between the
  //      load and its use, so the next group's loads stay in flight) ----
  uint32_t it = 0;
  if (nfull) {
    EncGeom ga = enc_geom(g, j, nsb, N, bs, cs), gb;
    EncRaw ra = enc_load_vec(in, ga, cs), rb;
    for (; it + 1 < nfull; it += 2) {
      gb = enc_geom((it + 1) * spw + g, j, nsb, N, bs, cs);
      rb = enc_load_vec(in, gb, cs);
      enc_iteration(st, ra, ga, G, j, be, ulsb, empty_lanes, cs);
      enc_flush(st, false);
      if (it + 2 < nfull) {
        ga = enc_geom((it + 2) * spw + g, j, nsb, N, bs, cs);
        ra = enc_load_vec(in, ga, cs);
      }
      enc_iteration(st, rb, gb, G, j, be, ulsb, empty_lanes, cs);
      enc_flush(st, false);
    }
    if (it < nfull) {
      enc_iteration(st, ra, ga, G, j, be, ulsb, empty_lanes, cs);
      enc_flush(st, false);
      ++it;
    }
  }
  // ---- ragged tail / unaligned streams: per-sample loads ----
  for (uint32_t s0 = it * spw; s0 < nsb; s0 += spw) {
    const EncGeom geo = enc_geom(s0 + g, j, nsb, N, bs, cs);
    const EncRaw r = enc_load_scalar(in, geo, cs);
    enc_iteration(st, r, geo, G, j, be, ulsb, true, 1u);
    enc_flush(st, false);
  }
  enc_flush(st, true);

  // ---- final words and the ceil(bits/8) tail bytes
  //      (bitstream_writer.h:110-120,139-145) ----
  const uint32_t total_bytes = (st.base + 7) >> 3;
  const uint32_t full_end = st.base >> 5;
  for (uint32_t w = st.win_w0 + lane; w < full_end; w += kWave) st.out32[w] = win[w - st.win_w0];
  const uint32_t tail_bytes = total_bytes - 4 * full_end;
  if (lane < tail_bytes) out8[4 * full_end + lane] = (uint8_t)(win[full_end - st.win_w0] >> (8 * lane));
  if (lane == 0) {
    p.out_bytes[b] = total_bytes;
    p.status[b] = RPP_OK;
  }
}

// ===========================================================================
// DECODE
// ===========================================================================
// Two streams per wavefront: lanes 0-31 decode stream 2*blockIdx.x, lanes
// 32-63 stream 2*blockIdx.x+1.  A Rice sub-block of ~1000 bits (Poisson
// sensor data, bs 128) then covers one half-wave of 32 lanes x 32-bit words,
// so every instruction of the serial sub-block loop serves two streams.  All
// per-stream state is uniform within a half; cross-lane ops (DPP row shifts,
// row_bcast15) never cross the half boundary.
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

constexpr uint32_t kHalf = 32;                // lanes per stream
constexpr uint32_t kRingWords = 1024;         // per-stream LDS ring of the compressed stream (4 KiB)
constexpr uint32_t kRingMask = kRingWords - 1;
constexpr uint32_t kChunkWords = 4 * kHalf;   // refill unit: 16 B per lane of a half
constexpr uint32_t kAhead = 288;              // words kept resident ahead of the read position
constexpr uint32_t kPosCap = 512;             // terminator positions of one Rice pass

__device__ __forceinline__ uint32_t half_incl_sum(uint32_t v) {
  v += dpp<kDppRowShr1>(v);
  v += dpp<kDppRowShr2>(v);
  v += dpp<kDppRowShr4>(v);
  v += dpp<kDppRowShr8>(v);
  v += dpp<kDppRowBcast15, 0xA>(v);
  return v;
}

__device__ __forceinline__ uint32_t half_last(uint32_t v) {
  const uint32_t a = readlane(v, kHalf - 1), b = readlane(v, kWave - 1);
  return lane_id() >= kHalf ? b : a;
}

__device__ __forceinline__ uint32_t half_ballot(bool pred) {
  const uint64_t m = __ballot(pred);
  return lane_id() >= kHalf ? (uint32_t)(m >> 32) : (uint32_t)m;
}

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

// This lane's 4 words of the 128-word chunk starting at word `w0`.
__device__ __forceinline__ uint4 load_chunk(const uint8_t* in, uint32_t nbytes, uint32_t w0, bool aligned16) {
  const uint32_t w = w0 + 4 * (lane_id() & (kHalf - 1));
  if (aligned16 && 4 * w + 16 <= nbytes) return *reinterpret_cast<const uint4*>(in + 4 * w);
  return make_uint4(stream_word(in, nbytes, w), stream_word(in, nbytes, w + 1), stream_word(in, nbytes, w + 2),
                    stream_word(in, nbytes, w + 3));
}

// Terminator chain through one 32-bit word: starting the unary search at bit
// `entry`, mark every '1' that ends a unary run and skip its fs remainder
// bits.  Returns the terminator mask; *exit = where the search continues in
// the next word (0 if it runs off the word while searching).  Branch-free
// body, wave-uniform trip count: sigma in [32, 45] = left the word after a
// terminator, 63 = ran off while searching ((0:word) >> 63 == 0 keeps it).
// Pass entry >= 32 for a lane that has nothing to do.
__device__ __forceinline__ uint32_t chain_word(uint32_t word, uint32_t entry, uint32_t fs, uint32_t* exit,
                                               uint32_t* iters = nullptr) {
  uint32_t T = 0, sigma = entry;
  const uint64_t w64 = word;
  while (__any(sigma < 32)) {
    if (iters) ++*iters;
    const bool act = sigma < 32;
    const uint32_t y = (uint32_t)(w64 >> sigma);  // 0 once sigma >= 32
    const uint32_t t = sigma + (uint32_t)__builtin_ctz(y | 0x80000000u);
    const bool hit = y != 0;
    T = hit ? (T | (1u << t)) : T;
    sigma = hit ? t + fs + 1 : (act ? 63u : sigma);
  }
  *exit = sigma < 63 ? sigma - 32 : 0u;
  return T;
}

// Exit state only (the lookback chain).
__device__ __forceinline__ uint32_t chain_exit(uint32_t word, uint32_t entry, uint32_t fs) {
  uint32_t sigma = entry;
  const uint64_t w64 = word;
  while (__any(sigma < 32)) {
    const bool act = sigma < 32;
    const uint32_t y = (uint32_t)(w64 >> sigma);
    const uint32_t t = sigma + (uint32_t)__builtin_ctz(y | 0x80000000u);
    sigma = y != 0 ? t + fs + 1 : (act ? 63u : sigma);
  }
  return sigma < 63 ? sigma - 32 : 0u;
}

// Exact terminator mask of this lane's 32-bit word.  A lane does not know
// where the unary search enters its word (that depends on every code to its
// left), so it runs the terminator chain for every possible entry state
// 0..fs side by side (independent chains: instruction-level parallelism,
// no speculation), giving its transfer function entry -> exit.  The first
// lane of a half has one exact entry (e0).  Entries then resolve left to
// right: a lane whose exit is the same for every entry (chains merged inside
// the word, the common case) breaks the dependency, so the resolution takes
// as many rounds as the longest run of entry-dependent lanes.
template <int NCH>
__device__ __forceinline__ uint32_t resolve_word(uint32_t own, uint32_t fs, uint32_t e0, bool first, bool act,
                                                 uint32_t nit, uint32_t* ex_out) {
  // sig[e]: next search start of the chain entered at e; >= 32 = left the
  // word, exit state sig - 32 (a search that runs off the word -> 32, exit 0)
  uint32_t sig[NCH], T[NCH];
  const uint64_t w64 = own;
  const uint32_t fs1 = fs + 1;
#pragma unroll
  for (int e = 0; e < NCH; ++e) {
    const uint32_t se = first ? (e == 0 ? e0 : 32u) : ((uint32_t)e <= fs ? (uint32_t)e : 32u);
    sig[e] = act ? se : 32u;
    T[e] = 0;
  }
  // stage by stage across the NCH independent chains (keeps them interleaved)
  for (uint32_t it = 0; it < nit; ++it) {
    uint32_t y[NCH], tz[NCH];
#pragma unroll
    for (int e = 0; e < NCH; ++e) y[e] = (uint32_t)(w64 >> sig[e]);  // 0 once sig >= 32
#pragma unroll
    for (int e = 0; e < NCH; ++e) tz[e] = (uint32_t)__builtin_ctz(y[e] | 0x80000000u);
#pragma unroll
    for (int e = 0; e < NCH; ++e) {
      const bool hit = y[e] != 0;
      T[e] |= (hit ? 1u : 0u) << (sig[e] + tz[e]);
      sig[e] = hit ? sig[e] + tz[e] + fs1 : max(sig[e], 32u);
    }
  }
  uint64_t F = 0;
  bool cst = true;
#pragma unroll
  for (int e = 0; e < NCH; ++e) {
    const uint32_t x = sig[e] - 32;
    F |= (uint64_t)x << (4 * e);
    cst = cst && (first || (uint32_t)e > fs || x == sig[0] - 32);
  }
  // resolve entry states left to right
  uint32_t entry = 0;
  bool known = first || !act;
  for (;;) {
    const bool out_known = known || cst;
    const uint32_t out_val = (uint32_t)(F >> (4 * entry)) & 15u;
    const bool lk = from_left(out_known ? 1u : 0u) != 0;
    const uint32_t lv = from_left(out_val);
    entry = (!known && lk) ? lv : entry;
    known = known || lk;
    if (!__any(!known)) break;
  }
  uint32_t Tt = T[0];
#pragma unroll
  for (int e = 1; e < NCH; ++e) Tt = entry == (uint32_t)e ? T[e] : Tt;
  *ex_out = (uint32_t)(F >> (4 * entry)) & 15u;
  return Tt;
}

__global__ __launch_bounds__(kWave) void rpp_decode_kernel(DecParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t ring_s[2][kRingWords];
  __shared__ __attribute__((aligned(16))) uint16_t tile_s[2][kTileSamples];
  __shared__ uint32_t pos_s[2][kPosCap + 1];  // + one dummy slot
  const uint32_t lane = lane_id();
  const uint32_t h = lane >> 5, hl = lane & (kHalf - 1);
  uint32_t* ring = ring_s[h];
  uint16_t* tile = tile_s[h];
  uint32_t* posbuf = pos_s[h];
  const uint32_t bs = p.bs, cs = p.cs, be = p.be, ulsb = p.ulsb;
  const uint32_t b = 2 * blockIdx.x + h;
#ifdef RPP_STATS
  uint32_t stat_acc[16] = {0};
  uint32_t* itp2 = &stat_acc[3];
  unsigned long long tprev_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#else
  uint32_t* itp2 = nullptr;
#endif

  // ---- per-stream setup (uniform within the half) ----
  int32_t status = RPP_OK;
  uint32_t N = 0, nbytes = 0;
  const uint8_t* in = p.in;
  uint16_t* out = p.out;
  if (b < p.nblocks) {
    const uint64_t n64 = p.n_samples[b];
    const uint64_t ioff = p.in_off[b];
    const uint64_t nb64 = p.in_bytes[b];
    if (n64 % cs != 0 || n64 >= RPP_MAX_STREAM_SAMPLES || (ioff & 3u) || nb64 >= (UINT64_C(1) << 29)) {
      status = RPP_INVALID_ARGUMENT;
    } else {
      N = (uint32_t)n64;
      nbytes = (uint32_t)nb64;
      in = p.in + ioff;
      out = p.out + p.out_off[b];
    }
  }
  const bool aligned16 = ((uintptr_t)in & 15u) == 0;
  // last readable bit + 1: the reader pulls whole 8-byte packets
  // (bitstream_reader.h:149-183), so it only throws past this point.
  const uint32_t lim = 64u * ((nbytes + 7u) >> 3);
  const uint32_t chunk_len = cs * bs;
  const uint32_t nsb = b < p.nblocks && status == RPP_OK ? ((N + chunk_len - 1) / chunk_len) * cs : 0u;

  // ---- fill the ring; refills are synchronous but only every ~8 sub-blocks
  //      (a register-carried prefetch made the compiler wait on every
  //      iteration for the output stores queued behind it) ----
  uint32_t fill_w = 0;
  auto refill = [&](bool go) {  // appends 2 chunks (256 words) to this half's ring
    if (go) {
      const uint4 v0 = load_chunk(in, nbytes, fill_w, aligned16);
      const uint4 v1 = load_chunk(in, nbytes, fill_w + kChunkWords, aligned16);
      *reinterpret_cast<uint4*>(&ring[(fill_w + 4 * hl) & kRingMask]) = v0;
      *reinterpret_cast<uint4*>(&ring[(fill_w + kChunkWords + 4 * hl) & kRingMask]) = v1;
    }
    fill_w = go ? fill_w + 2 * kChunkWords : fill_w;
  };
  refill(true);
  refill(true);
  __syncthreads();
  // keeps words [w - 1, w + kAhead) of this half's stream resident
  auto ensure = [&](uint32_t w, bool act) {
    while (__any(act && fill_w < w + kAhead)) refill(act && fill_w < w + kAhead);
    __syncthreads();
  };
  auto rbits = [&](uint32_t pos, uint32_t width) -> uint32_t {  // width <= 16
    const uint32_t w = pos >> 5;
    const uint64_t v = (uint64_t)ring[w & kRingMask] | ((uint64_t)ring[(w + 1) & kRingMask] << 32);
    return (uint32_t)(v >> (pos & 31u)) & ((1u << width) - 1u);
  };

  uint32_t last0 = 0, last1 = 0, P = 16 * cs;
  if (nsb != 0 || (b < p.nblocks && status == RPP_OK)) {
    if (16 * cs > lim) status = RPP_TRUNCATED_INPUT;
    last0 = rbits(0, 16);
    last1 = cs > 1 ? rbits(16, 16) : 0u;
  }

  for (uint32_t s = 0;; ++s) {
    bool active = s < nsb && status == RPP_OK;
    if (!__any(active)) break;
    const uint32_t chunk = cs == 1 ? s : s >> 1;
    const uint32_t comp = s - chunk * cs;
    const uint32_t cbase = chunk * chunk_len;
    const uint32_t clen = active ? min(N - cbase, chunk_len) : 0u;
    const uint32_t n = clen / cs;
    RPP_TSTAMP(4);
    ensure(P >> 5, active);
    RPP_TSTAMP(5);
    // decode.h:60: 4-bit fs+1 header
    if (active && P + 4 > lim) {
      status = RPP_TRUNCATED_INPUT;
      active = false;
    }
    const uint32_t fsp1 = active ? rbits(P, 4) : 0u;
    P += 4;
    RPP_STAT(6, 1);
    RPP_TSTAMP(7);
    uint32_t acc = comp ? last1 : last0;
    if (active && fsp1 == 0) {
      // decode.h:79-80: all samples = write(last)
      const uint32_t v = px_write(acc, be, ulsb);
      for (uint32_t k = hl; k < n; k += kHalf) tile[comp + cs * k] = (uint16_t)v;
    }
    if (active && fsp1 == 15) {
      // decode.h:72-77: raw stored values; last = read(last sample)
      if ((uint64_t)P + 16ull * n > lim) {
        status = RPP_TRUNCATED_INPUT;
        active = false;
      } else {
        for (uint32_t k = hl; k < n; k += kHalf) tile[comp + cs * k] = (uint16_t)rbits(P + 16 * k, 16);
        acc = px_read(rbits(P + 16 * (n - 1), 16), be, ulsb);
        P += 16 * n;
      }
    }
    bool rdo = active && fsp1 != 0 && fsp1 != 15;
    RPP_TSTAMP(9);
    if (__any(rdo)) {
      // decode.h:62-71: Rice codes, fs = fsp1 - 1
      const uint32_t fs = rdo ? fsp1 - 1 : 0u;
      const uint32_t lowmask = (1u << fs) - 1u;
      // wave-uniform chain shape: entries = max fs + 1, steps = ceil(32 / (min fs + 1))
      const uint32_t fa = readlane(rdo ? fs : 0u, 0), fb = readlane(rdo ? fs : 0u, kHalf);
      const bool ra = readlane(rdo ? 1u : 0u, 0) != 0, rb = readlane(rdo ? 1u : 0u, kHalf) != 0;
      const uint32_t fmax = max(ra ? fa : 0u, rb ? fb : 0u);
      const uint32_t fmin = min(ra ? fa : 15u, rb ? fb : 15u);
      const uint32_t nch = fmax + 1;
      const uint32_t nit = (32 + fmin) / (fmin + 1);
      uint32_t K = 0;            // codes decoded in earlier passes
      uint32_t sigma_carry = P;  // search start of the next code
      uint32_t W0 = P >> 5;      // first word of this pass
      uint32_t e0 = P & 31u;     // exact entry state of lane 0 of the half
      while (__any(rdo)) {
        RPP_STAT(0, 1);
        if (rdo && 32ull * W0 >= lim) {
          status = RPP_TRUNCATED_INPUT;
          rdo = false;
        }
        ensure(W0, rdo);
        RPP_TSTAMP(9);
        const uint32_t own = ring[(W0 + hl) & kRingMask];
        // chains for every entry state, then left-to-right resolution
        uint32_t ex, T;
        switch (nch) {
#define RPP_RESOLVE_CASE(k) \
  case k: T = resolve_word<k>(own, fs, e0, hl == 0, rdo, nit, &ex); break;
          RPP_RESOLVE_CASE(1) RPP_RESOLVE_CASE(2) RPP_RESOLVE_CASE(3) RPP_RESOLVE_CASE(4)
          RPP_RESOLVE_CASE(5) RPP_RESOLVE_CASE(6) RPP_RESOLVE_CASE(7) RPP_RESOLVE_CASE(8)
          RPP_RESOLVE_CASE(9) RPP_RESOLVE_CASE(10) RPP_RESOLVE_CASE(11) RPP_RESOLVE_CASE(12)
          RPP_RESOLVE_CASE(13)
          default: T = resolve_word<14>(own, fs, e0, hl == 0, rdo, nit, &ex); break;
#undef RPP_RESOLVE_CASE
        }
        RPP_TSTAMP(10);
        RPP_TSTAMP(11);
        const uint32_t c = (uint32_t)__builtin_popcount(T);
        const uint32_t cincl = half_incl_sum(c);
        const uint32_t cexcl = cincl - c;
        const uint32_t ctot = half_last(cincl);
        const uint32_t need = rdo ? min(ctot, n - K) : 0u;
        const uint32_t wbit = 32u * (W0 + hl);
        // materialise the absolute positions of the first `need` terminators
        {
          uint32_t TT = T, idx = cexcl;
          for (uint32_t it = 0; it < nit; ++it) {  // popcount(T) <= nit
            const bool hit = TT != 0 && idx < need;
            const uint32_t t = (uint32_t)__builtin_ctz(TT | 0x80000000u);
            posbuf[hit ? idx : kPosCap] = wbit + t;
            TT &= TT - 1;
            ++idx;
          }
        }
        __syncthreads();
        RPP_TSTAMP(12);
        // code-parallel extraction: code i of this pass on lane i % 32
        for (uint32_t r = 0; __any(r < need); r += kHalf) {
          const uint32_t i = r + hl;
          const bool valid = i < need;
          const uint32_t ii = valid ? i : 0u;
          const uint32_t t = posbuf[ii];
          const uint32_t sig = ii == 0 ? sigma_carry : posbuf[ii - 1] + fs + 1;
          const uint32_t rp = t + 1, rw = rp >> 5;
          const uint64_t v = (uint64_t)ring[rw & kRingMask] | ((uint64_t)ring[(rw + 1) & kRingMask] << 32);
          const uint32_t rem = (uint32_t)(v >> (rp & 31u)) & lowmask;
          const uint32_t diff = ((t - sig) << fs) | rem;
          const uint32_t delta = valid ? (diff >> 1) ^ (0u - (diff & 1u)) : 0u;
          const uint32_t incl = half_incl_sum(delta);
          if (valid) tile[comp + cs * (K + i)] = (uint16_t)px_write(acc + incl, be, ulsb);
          acc += half_last(incl);
        }
        RPP_TSTAMP(13);
        const uint32_t ex_last = half_last(ex);
        const bool fin = rdo && K + ctot >= n;
        const uint32_t E = posbuf[fin ? n - 1 - K : 0u] + fs + 1;
        const uint32_t lastpos = posbuf[ctot ? ctot - 1 : 0u] + fs + 1;
        __syncthreads();
        if (fin) {
          if (E > lim) status = RPP_TRUNCATED_INPUT;
          P = E;
          rdo = false;
        }
        if (rdo) {
          sigma_carry = ctot ? lastpos : sigma_carry;
          K += ctot;
          e0 = ex_last;
          W0 += kHalf;
        }
      }
    }
    RPP_TSTAMP(14);
    if (active && status == RPP_OK) {
      if (comp) last1 = acc & 0xFFFFu;
      else last0 = acc & 0xFFFFu;
    }
    __syncthreads();
    // ---- chunk complete: flush this half's tile ----
    if (active && status == RPP_OK && comp == cs - 1) {
      uint16_t* dst = out + cbase;
      if (((uintptr_t)dst & 15) == 0 && (clen & 7) == 0) {
        for (uint32_t i = hl; i < clen / 8; i += kHalf)
          reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(tile)[i];
      } else {
        for (uint32_t i = hl; i < clen; i += kHalf) dst[i] = tile[i];
      }
    }
    __syncthreads();
  }
  RPP_TSTAMP(15);
  if (b < p.nblocks && hl == 0) p.status[b] = status;
#ifdef RPP_STATS
  if (lane == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rpp_stats[i], (unsigned long long)stat_acc[i]);
#endif
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

uint32_t rpp_abi_version(void) { return 1; }

#ifdef RPP_STATS
// Diagnostic build only: copies (and optionally clears) the loop counters.
int rpp_stats_fetch(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rpp_stats), sizeof(uint64_t) * 16) != hipSuccess) return RPP_HIP_ERROR;
  if (reset) {
    uint64_t z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rpp_stats), z, sizeof z) != hipSuccess) return RPP_HIP_ERROR;
  }
  return RPP_OK;
}
#endif

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
  hipLaunchKernelGGL(rpp_decode_kernel, dim3((nblocks + 1) / 2), dim3(kWave), 0, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // extern "C"
