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

#include <algorithm>
#include <atomic>
#include <mutex>
#include <stdlib.h>

#include "ricepp_amd.h"
#include "ricepp_internal.h"

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
constexpr int kDppWaveRor1 = 0x13C;
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  // lanes whose source is outside the row / not selected read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, Ctrl, RowMask, 0xF, false);
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

// Orders this wave's LDS accesses (one wave's DS operations execute in
// order); unlike __syncthreads() it does not drain vmcnt, so outstanding
// global loads (prefetches) and stores stay in flight.  One-wave workgroups.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

// DPP move; lanes without a source in range keep `old`.  Called with every
// lane active (a DPP source lane that is switched off reads as out of range).
template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_keep(uint32_t old, uint32_t v) {
  // lanes without a source in range keep `old`
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, Ctrl, RowMask, 0xF, false);
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
  // segment mode (long streams, rpp_encode_batch_ws): work unit u = segment
  // u - seg_base[b] of stream b = seg_map[u]; null seg_map: unit = stream
  const uint32_t* seg_map;
  const uint64_t* seg_base;  // [nblocks + 1]: units before stream b; [nblocks] = total
  uint64_t* seg_bits;        // [units] bits a segment wrote (multi-segment streams)
  uint8_t* scratch;          // segments >= 1 of a stream: slot u - b - 1
  uint64_t slot_bytes;
  // units the workspace holds: a batch with more (its samples exceed the
  // caller's total_samples) is encoded one wave per stream, nothing split
  uint64_t max_units;
  uint32_t seg_chunks;  // chunks per unit (enc_seg_chunks)
};
// segment mode and the batch fits the workspace
__device__ __forceinline__ bool enc_split_ok(const EncParams& p) {
  return p.seg_map && p.seg_base[p.nblocks] <= p.max_units;
}

// Segment mode: a stream of more than seg_chunks chunks is encoded by
// several waves, one per run of seg_chunks chunks.  Every sub-block's codes
// depend only on its samples and the sample before it (encode.h:92-157), so a
// segment starts from the real preceding sample, at bit 0 of its own scratch
// slot (segment 0: after the initial values, in the stream's output), and
// rpp_enc_concat_kernel then places each segment at its bit offset.
// seg_chunks is kEncSegChunks when the batch fills the GPU with units of that
// size, smaller (down to kEncSegChunksMin, so that a unit that is not its
// stream's last holds at least 64 bits) for batches of few blocks, whose
// latency is one wave's pass over a whole block otherwise (enc_seg_chunks)
constexpr uint32_t kEncSegChunks = 256;
constexpr uint32_t kEncSegChunksMin = 16;
constexpr uint64_t kEncTargetUnits = 2048;
// wave priority in the pipelined encode: plans (deltas, split walk,
// positions) at priority 1, the LDS emission at 0 (the reverse and no
// priority measured slower: DESIGN.md §4 "Wave priority")

// Compile-time shape of an encode launch: SPL samples per lane (8 or 16), a
// ricepp sub-block owned by an aligned group of G lanes (G = next pow2 of
// ceil(bs / SPL)), CS component streams.  64 / G sub-blocks per iteration.

// Sum over the aligned group of G lanes containing this lane, broadcast to
// every lane of the group (butterfly; all lanes active).
template <uint32_t G>
__device__ __forceinline__ uint32_t gsum(uint32_t v) {
  if constexpr (G >= 2) v += dpp<kDppQuadXor1>(v);
  if constexpr (G >= 4) v += dpp<kDppQuadXor2>(v);
  if constexpr (G >= 8) v += dpp<kDppRowHalfMirror>(v);
  if constexpr (G >= 16) v += dpp<kDppRowMirror>(v);
  if constexpr (G >= 32) {
    auto t = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = t[0] + t[1];
  }
  if constexpr (G >= 64) {
    auto t = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = t[0] + t[1];
  }
  return v;
}

// Per-lane sub-block geometry of one encode iteration.
struct EncGeom {
  uint32_t n;        // samples in this lane's sub-block (0: no sub-block)
  uint32_t cnt;      // samples owned by this lane (<= SPL)
  uint32_t m_first;  // stream index of the lane's first sample
  uint32_t comp;     // component stream
};

template <uint32_t SPL, uint32_t CS>
__device__ __forceinline__ EncGeom enc_geom(uint32_t s, uint32_t j, uint32_t nsb, uint32_t N, uint32_t bs) {
  EncGeom g;
  // codec.h:88-97: chunks of cs*bs samples; component i takes i, i+cs, ...
  const uint32_t chunk = s / CS;
  g.comp = s % CS;
  const uint32_t cbase = chunk * CS * bs;
  g.n = 0;
  if (s < nsb) {
    const uint32_t rem = (N - cbase) / CS;
    g.n = rem < bs ? rem : bs;
  }
  const uint32_t k0 = SPL * j;
  g.cnt = k0 < g.n ? min(g.n - k0, SPL) : 0u;
  g.m_first = cbase + g.comp + CS * k0;
  return g;
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef short ss2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 as_us2(uint32_t v) { return __builtin_bit_cast(us2, v); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }

// The lane's stored samples as SPL / 2 packed pairs (sample 2k in the low
// half of w[k]) plus the previous same-component stored sample.
template <uint32_t SPL>
struct EncRaw {
  uint32_t w[SPL / 2];
  uint32_t prev;
};

// Full iterations (every lane owns 0 or SPL samples): 16-byte loads.
template <uint32_t SPL, uint32_t CS>
__device__ __forceinline__ EncRaw<SPL> enc_load_vec(const uint16_t* in, const EncGeom& g, bool load_prev) {
  EncRaw<SPL> r;
  // codec.h:72-73: a component's first sample is its own reference (last = read(in[i]))
  if (load_prev) {
    const uint32_t pi = g.cnt ? (g.m_first >= CS ? g.m_first - CS : g.m_first) : 0u;
    r.prev = in[pi];
  } else {
    r.prev = 0;
  }
  const uint4* q = reinterpret_cast<const uint4*>(g.cnt ? in + (g.m_first - g.comp) : in);
  if constexpr (CS == 1) {
#pragma unroll
    for (uint32_t i = 0; i < SPL / 8; ++i) {
      const uint4 v = q[i];
      r.w[4 * i] = v.x; r.w[4 * i + 1] = v.y; r.w[4 * i + 2] = v.z; r.w[4 * i + 3] = v.w;
    }
  } else {
    // interleaved (c0, c1) pairs: keep this lane's component
    const uint32_t sel = g.comp ? 0x07060302u : 0x05040100u;
#pragma unroll
    for (uint32_t i = 0; i < SPL / 4; ++i) {
      const uint4 v = q[i];
      r.w[2 * i] = __builtin_amdgcn_perm(v.y, v.x, sel);
      r.w[2 * i + 1] = __builtin_amdgcn_perm(v.w, v.z, sel);
    }
  }
  return r;
}

// Ragged tail / unaligned streams: per-sample loads.
template <uint32_t SPL, uint32_t CS>
__device__ __forceinline__ EncRaw<SPL> enc_load_scalar(const uint16_t* in, const EncGeom& g) {
  EncRaw<SPL> r;
  const uint32_t pi = g.m_first >= CS ? g.m_first - CS : g.m_first;
  r.prev = g.cnt ? (uint32_t)in[pi] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < SPL / 2; ++k) {
    const uint32_t lo = 2 * k < g.cnt ? (uint32_t)in[g.m_first + CS * 2 * k] : 0u;
    const uint32_t hi = 2 * k + 1 < g.cnt ? (uint32_t)in[g.m_first + CS * (2 * k + 1)] : 0u;
    r.w[k] = lo | (hi << 16);
  }
  return r;
}

// ORs the (<= 16 bit) code `v` into the window at bit `rel` (two ds_or_b32;
// the second is 0 when the code does not straddle a word).
__device__ __forceinline__ void emit_bits(uint32_t* win, uint32_t rel, uint32_t v) {
  const uint32_t w = rel >> 5, sh = rel & 31u;
  atomicOr(&win[w], v << sh);
  atomicOr(&win[w + 1], (v >> 1) >> (31u - sh));
}

// The same for codes of <= 32 bits.  32-bit shifts only: a 64-bit shift
// (v_lshlrev_b64) whose amount the register allocator happens to place in the
// last VGPR of the kernel's allocation reads a wrong amount on gfx950 while
// other waves share the SIMD -- the round-5 bs 128 cs 2 fault (DESIGN.md §4
// "64-bit shifts and the last VGPR"; tools/isa_audit.py guards the build).
__device__ __forceinline__ void emit_bits64(uint32_t* win, uint32_t rel, uint32_t v) {
  const uint32_t sh = rel & 31u;
  uint32_t* w = win + (rel >> 5);
  atomicOr(w, v << sh);
  atomicOr(w + 1, (v >> 1) >> (31u - sh));
}

constexpr uint32_t kEncWin = 1024;      // LDS output window (words, 4 KiB)
constexpr uint32_t kEncFlushWords = 256;  // stream out once >= 1 KiB of whole 64-byte lines is ready

struct EncState {
  uint32_t* win;
  uint32_t* out32;
  uint32_t win_w0;  // global word index held in win[0] (multiple of 16)
  uint32_t base;       // absolute bit position after the emitted codes
  uint32_t plan_base;  // absolute bit position after the planned codes
  uint32_t carry;      // pixel value of the sample before this iteration (DPP-prev mode)
};

// sum over the lane's samples of d >> f (the lane's unary bits at fs = f)
template <uint32_t SPL>
__device__ __forceinline__ uint32_t enc_shr_sum(const us2* d, uint32_t f) {
  const us2 fv = (us2)(unsigned short)f, one = {1, 1};
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t k = 0; k < SPL / 2; ++k) acc = __builtin_amdgcn_udot2(d[k] >> fv, one, acc, false);
  return acc;
}

// One group of 64/G sub-blocks is encoded in three steps, so that the full
// iterations can be software-pipelined (the plan of group i+1 is computed
// while group i is emitted):
//   enc_plan_a: zig-zag deltas, sums, compute_best_split start and first pair
//   enc_plan_b: the split walk, mode, bit positions by one wave scan
//   enc_emit:   header and codes OR-ed into the LDS window
// dpp_prev: every lane full and the previous sample of a lane's first sample
// is the previous lane's last one (CS == 1, bs == G * SPL): no prev loads.
template <uint32_t SPL>
struct EncPlan {
  us2 d[SPL / 2];       // zig-zag deltas
  uint32_t w[SPL / 2];  // stored samples (raw sub-blocks)
  uint32_t n, cnt, sum;
  uint32_t bits, lq;    // best cost so far, this lane's unary bits at that fs
  int cand, dir;
  bool walking;
  uint32_t mode, fs;    // 0 = all-zero, 1 = Rice, 2 = raw
  uint32_t pos;         // absolute bit position of this lane's first bit
  uint32_t end;         // absolute bit position after the group
};

template <uint32_t SPL, uint32_t G, uint32_t CS, bool SH>
__device__ __forceinline__ void enc_plan_a(EncPlan<SPL>& P, EncState& st, const EncRaw<SPL>& r, const EncGeom& geo,
                                           uint32_t selbe, uint32_t be, uint32_t ulsb, bool mask_tail,
                                           bool dpp_prev) {
  constexpr uint32_t NW = SPL / 2;
  const uint32_t n = geo.n, cnt = geo.cnt;
  P.n = n;
  P.cnt = cnt;
  const bool sb_valid = n != 0;
  // ---- pixel values (ricepp_cpuspecific_traits.h:63-67) and zig-zag deltas
  //      (encode.h:116-123), two samples per instruction ----
  us2 v[NW];
#pragma unroll
  for (uint32_t k = 0; k < NW; ++k) {
    P.w[k] = r.w[k];
    v[k] = as_us2(__builtin_amdgcn_perm(r.w[k], r.w[k], selbe));
    if constexpr (SH) v[k] = v[k] >> (us2)(unsigned short)ulsb;
  }
  uint32_t pv;
  if (dpp_prev) {
    const uint32_t lastv = as_u32(v[NW - 1]) >> 16;
    pv = dpp_keep<kDppWaveShr1>(st.carry, lastv);  // lane 0: the carried sample
    st.carry = readlane(lastv, kWave - 1);
  } else {
    pv = px_read(r.prev, be, ulsb);
  }
  uint32_t prevw = pv << 16;
#pragma unroll
  for (uint32_t k = 0; k < NW; ++k) {
    const us2 pp = as_us2(__builtin_amdgcn_alignbit(as_u32(v[k]), prevw, 16));
    prevw = as_u32(v[k]);
    const us2 diff = v[k] - pp;
    P.d[k] = (diff << (us2)1) ^ as_us2(__builtin_bit_cast(uint32_t, (__builtin_bit_cast(ss2, diff) >> (ss2)15)));
  }
  if (mask_tail) {
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) {
      const uint32_t keep = (2u * k < cnt ? 0xFFFFu : 0u) | (2u * k + 1 < cnt ? 0xFFFF0000u : 0u);
      P.d[k] = as_us2(as_u32(P.d[k]) & keep);
    }
  }
  const us2 one = {1, 1};
  uint32_t lsum = 0;
#pragma unroll
  for (uint32_t k = 0; k < NW; ++k) lsum = __builtin_amdgcn_udot2(P.d[k], one, lsum, false);
  const uint32_t sum = gsum<G>(lsum);
  P.sum = sum;

  // ---- compute_best_split replay (encode.h:43-90), first pair ----
  // start = max(0, bit_width(sum / n) - 2) without a division:
  // bit_width(floor(s/n)) = t + (s >= n << t), t = floor(log2 s) - floor(log2 n)
  uint32_t bwq = 0;
  if (n != 0 && sum >= n) {
    const uint32_t t = (uint32_t)__clz(n) - (uint32_t)__clz(sum);
    bwq = t + ((n << t) <= sum ? 1u : 0u);
  }
  const uint32_t start = bwq >= 2 ? bwq - 2 : 0u;
  // (the lane's share of the unary bits of the current candidate is kept:
  // the chosen fs needs it again for the bit positions)
  const uint32_t lq0 = enc_shr_sum<SPL>(P.d, start), lq1 = enc_shr_sum<SPL>(P.d, start + 1);
  const uint32_t bits0 = n * (start + 1) + gsum<G>(lq0);
  const uint32_t bits1 = n * (start + 2) + gsum<G>(lq1);
  if (bits1 <= bits0) {
    P.cand = (int)start + 1; P.bits = bits1; P.dir = 1; P.lq = lq1;
  } else {
    P.cand = (int)start; P.bits = bits0; P.dir = -1; P.lq = lq0;
  }
  P.walking = sb_valid && sum != 0 && bits0 != bits1;
}

template <uint32_t SPL, uint32_t G>
__device__ __forceinline__ void enc_plan_b(EncPlan<SPL>& P, EncState& st, uint32_t j) {
  const uint32_t n = P.n, cnt = P.cnt;
  const bool sb_valid = n != 0;
  // ---- compute_best_split replay: the walk.  Almost every sub-block takes
  //      exactly one more candidate (that does not improve), so the first
  //      step runs unconditionally, without a vote and a branch ----
  auto walk_step = [&](bool act) {
    const uint32_t f = act ? (uint32_t)(P.cand + P.dir) : 0u;
    const uint32_t lt = enc_shr_sum<SPL>(P.d, f);
    const uint32_t t = n * (f + 1) + gsum<G>(lt);
    if (act && t <= P.bits) {
      P.bits = t;
      P.lq = lt;
      P.cand += P.dir;
    } else {
      P.walking = false;
    }
  };
  walk_step(P.walking && P.cand > 0 && P.cand < 14);
  for (;;) {
    const bool act = P.walking && P.cand > 0 && P.cand < 14;
    if (!__any(act)) break;
    walk_step(act);
  }
  // encode.h:127-156: 0 = all-zero, 1 = Rice, 2 = raw
  P.mode = 0;
  P.fs = 0;
  if (sb_valid && P.sum != 0) {
    P.fs = (uint32_t)P.cand;
    P.mode = (P.fs < 14 && P.bits < 16 * n) ? 1u : 2u;
  }
  // ---- bit positions: one wave-wide scan ----
  uint32_t lbits = (sb_valid && j == 0) ? 4u : 0u;
  if (P.mode == 1) lbits += P.lq + cnt * (P.fs + 1);
  else if (P.mode == 2) lbits += 16 * cnt;
  const uint32_t incl = wave_incl_sum(lbits);
  P.pos = st.plan_base + incl - lbits;
  st.plan_base += readlane(incl, kWave - 1);
  P.end = st.plan_base;
}

template <uint32_t SPL>
__device__ __forceinline__ void enc_emit(const EncPlan<SPL>& P, EncState& st, uint32_t j, bool mask_tail) {
  const uint32_t cnt = P.cnt, mode = P.mode, fs = P.fs;
  uint32_t pos = P.pos - 32 * st.win_w0;  // window-relative
  if (P.n != 0 && j == 0) {
    emit_bits(st.win, pos, mode == 0 ? 0u : (mode == 1 ? fs + 1 : 15u));
    pos += 4;
  }
  if (mode == 1 && !mask_tail) {
    // every lane owns SPL samples: two codes per packed step.  The '1' of
    // code i sits at e_i = e_(i-1) + k + q_i; the code value (1 | r << 1,
    // <= 15 bits) is OR-ed in by one 64-bit shift and two ds_or_b32.
    const uint32_t k = fs + 1;
    const uint32_t m2 = ((2u << fs) - 1u) * 0x10001u;
    uint32_t e = pos - k;
    us2 qv[SPL / 2];
    us2 qmax = {0, 0};
#pragma unroll
    for (uint32_t h = 0; h < SPL / 2; ++h) {
      qv[h] = P.d[h] >> (us2)(unsigned short)fs;
      qmax = __builtin_elementwise_max(qmax, qv[h]);
    }
    // the pair (2h, 2h+1) spans k + q_(2h+1) + k bits from code 2h's '1':
    // when that fits 32 bits for every pair of the wave (fs <= 13 and unary
    // runs short: Poisson data), one 64-bit shift and two ds_or_b32 per pair
    if (!__any(2u * k + (as_u32(qmax) >> 16) > 32u)) {
#pragma unroll
      for (uint32_t h = 0; h < SPL / 2; ++h) {
        const uint32_t qq = as_u32(qv[h]);
        const uint32_t cc = (as_u32(P.d[h] << (us2)1) & m2) | 0x10001u;
        e += k + (qq & 0xFFFFu);
        const uint32_t d = k + (qq >> 16);
        emit_bits64(st.win, e, (cc & 0xFFFFu) | ((cc >> 16) << d));
        e += d;
      }
    } else {
#pragma unroll
      for (uint32_t h = 0; h < SPL / 2; ++h) {
        const uint32_t qq = as_u32(qv[h]);
        const uint32_t cc = (as_u32(P.d[h] << (us2)1) & m2) | 0x10001u;
        e += k + (qq & 0xFFFFu);
        emit_bits64(st.win, e, cc & 0xFFFFu);
        e += k + (qq >> 16);
        emit_bits64(st.win, e, cc >> 16);
      }
    }
  } else if (mode == 1) {
    const uint32_t lowmask = (1u << fs) - 1u;
#pragma unroll
    for (uint32_t i = 0; i < SPL; ++i) {
      if (i < cnt) {
        const uint32_t di = (i & 1) ? (as_u32(P.d[i >> 1]) >> 16) : (as_u32(P.d[i >> 1]) & 0xFFFFu);
        pos += di >> fs;  // unary zeros are implicit (the window is zeroed)
        emit_bits(st.win, pos, 1u | ((di & lowmask) << 1));
        pos += fs + 1;
      }
    }
  } else if (mode == 2) {
#pragma unroll
    for (uint32_t i = 0; i < SPL; ++i) {
      if (i < cnt) {
        const uint32_t ri = (i & 1) ? (P.w[i >> 1] >> 16) : (P.w[i >> 1] & 0xFFFFu);
        emit_bits(st.win, pos, ri);  // raw stored value (encode.h:148-151)
        pos += 16;
      }
    }
  }
  st.base = P.end;
}

// The three steps back to back (ragged tails, unpipelined groups).
template <uint32_t SPL, uint32_t G, uint32_t CS, bool SH>
__device__ __forceinline__ void enc_iteration(EncState& st, const EncRaw<SPL>& r, const EncGeom& geo, uint32_t j,
                                              uint32_t selbe, uint32_t be, uint32_t ulsb, bool mask_tail,
                                              bool dpp_prev) {
  EncPlan<SPL> P;
  enc_plan_a<SPL, G, CS, SH>(P, st, r, geo, selbe, be, ulsb, mask_tail, dpp_prev);
  enc_plan_b<SPL, G>(P, st, j);
  enc_emit<SPL>(P, st, j, mask_tail);
}

// Streams whole 64-byte lines out once >= kEncFlushWords are complete.
__device__ __forceinline__ void enc_flush(EncState& st, bool final_flush) {
  const uint32_t lane = lane_id();
  wave_lds_fence();
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
    wave_lds_fence();
    for (uint32_t i = lane; i < used; i += kWave) st.win[i] = 0;
    wave_lds_fence();
    if (lane < 16) st.win[lane] = keep;
    wave_lds_fence();
    st.win_w0 = F;
  }
}

// SH: unused_lsb_count != 0 (the pixel read shifts)
template <uint32_t SPL, uint32_t G, uint32_t CS, bool SH>
__global__ __launch_bounds__(kWave) void rpp_encode_kernel(EncParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t win[kEncWin];
  constexpr uint32_t spw = kWave / G;  // sub-blocks per iteration
  uint32_t b = blockIdx.x, seg = 0;
  const bool split = enc_split_ok(p);
  if (split) {
    if (blockIdx.x >= p.seg_base[p.nblocks]) return;
    b = p.seg_map[blockIdx.x];
    seg = blockIdx.x - (uint32_t)p.seg_base[b];
  } else if (b >= p.nblocks) {
    return;
  }
  const uint32_t lane = lane_id();
  const uint32_t bs = p.bs, be = p.be, ulsb = p.ulsb;
  const uint32_t selbe = be ? 0x02030001u : 0x03020100u;
  const uint64_t n64 = p.n_samples[b];
  const uint64_t ooff = p.out_off[b];
  if (n64 % CS != 0 || n64 >= RPP_MAX_STREAM_SAMPLES || (ooff & 15u)) {
    if (lane == 0 && seg == 0) {
      p.status[b] = RPP_INVALID_ARGUMENT;
      p.out_bytes[b] = 0;
    }
    return;
  }
  const uint32_t N = (uint32_t)n64;
  const uint16_t* in = p.in + p.in_off[b];
  const uint32_t chunk_len = CS * bs;
  const uint32_t nchunks = (N + chunk_len - 1) / chunk_len;
  const uint32_t segc = p.seg_chunks;
  const bool multi = split && nchunks > segc;
  // one wave for a whole stream keeps 32-bit bit positions: longer streams
  // must be split (rpp_encode_batch_ws)
  if (!multi && n64 >= rpp_internal::kSegMaxSamples) {
    if (lane == 0 && seg == 0) {
      p.status[b] = RPP_INVALID_ARGUMENT;
      p.out_bytes[b] = 0;
    }
    return;
  }
  // this unit's chunks [c_lo, c_hi)
  const uint32_t c_lo = multi ? seg * segc : 0u;
  const uint32_t c_hi = multi ? min(nchunks, c_lo + segc) : nchunks;
  uint8_t* out8 = seg == 0 ? p.out + ooff : p.scratch + (size_t)(blockIdx.x - b - 1) * p.slot_bytes;
#ifdef RPP_STATS
  uint32_t stat_acc[16] = {0};
  unsigned long long tprev_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif

  for (uint32_t i = lane; i < kEncWin; i += kWave) win[i] = 0;
  __syncthreads();

  const uint32_t bit0 = seg == 0 ? 16 * CS : 0u;
  EncState st{win, reinterpret_cast<uint32_t*>(out8), 0u, bit0, bit0, 0u};
  // codec.h:69-74,81-86: 16-bit initial value read(in[i]) per component.
  if (seg == 0 && lane < CS) emit_bits(win, 16 * lane, N ? px_read(in[lane], be, ulsb) : 0u);
  // DPP-prev mode: the reference of the unit's first sample (the stream's
  // first sample is its own reference)
  st.carry = N ? px_read(in[c_lo ? c_lo * chunk_len - 1 : 0], be, ulsb) : 0u;

  const uint32_t nsb = c_hi * CS;     // sub-blocks [s_lo, nsb) are this unit's
  const uint32_t s_lo = c_lo * CS;
  const uint32_t g = lane / G, j = lane % G;
  // full iterations: every sub-block complete, lanes own 0 or SPL samples
  const bool vec_ok = bs % SPL == 0 && ((uintptr_t)in & 15u) == 0;
  const uint32_t nsb_full = vec_ok ? min(N / chunk_len, c_hi) * CS : 0u;
  const uint32_t nfull = nsb_full > s_lo ? (nsb_full - s_lo) / spw : 0u;
  const bool empty_lanes = G * SPL != bs;
  const bool dpp_prev = CS == 1 && !empty_lanes;

  // ---- full iterations, software-pipelined: group it+1 is planned
  //      (deltas, split, positions) around the emission of group it, so the
  //      two dependency chains overlap.  Two sample buffers: the one just
  //      planned from is reloaded at once with the group after next, about
  //      two steps before its use; unrolled by two so that plans and loaded
  //      samples stay in place (no register copies) ----
  uint32_t it = 0;
  if (nfull) {
    EncGeom g0 = enc_geom<SPL, CS>(s_lo + g, j, nsb, N, bs);
    EncRaw<SPL> r0 = enc_load_vec<SPL, CS>(in, g0, !dpp_prev);
    EncGeom g1 = enc_geom<SPL, CS>(s_lo + spw + g, j, nsb, N, bs);
    EncRaw<SPL> r1 = enc_load_vec<SPL, CS>(in, g1, !dpp_prev);
    EncPlan<SPL> P, Q;
    enc_plan_a<SPL, G, CS, SH>(P, st, r0, g0, selbe, be, ulsb, empty_lanes, dpp_prev);
    // (loads are unconditional: past the last group the geometry is empty
    // and the load reads the stream start; a conditional load would make
    // every later wait cover it)
    g0 = enc_geom<SPL, CS>(s_lo + 2 * spw + g, j, nsb, N, bs);
    r0 = enc_load_vec<SPL, CS>(in, g0, !dpp_prev);
    enc_plan_b<SPL, G>(P, st, j);
    // emits group `it` (plan E) while planning group it+1 (into F, from rn,
    // which then takes group it+3)
    auto step = [&](EncPlan<SPL>& E, EncPlan<SPL>& F, EncRaw<SPL>& rn, EncGeom& gn) {
      RPP_STAT(0, 1);
      RPP_TSTAMP(1);
      __builtin_amdgcn_s_setprio(1);
      enc_plan_a<SPL, G, CS, SH>(F, st, rn, gn, selbe, be, ulsb, empty_lanes, dpp_prev);
      gn = enc_geom<SPL, CS>(s_lo + (it + 3) * spw + g, j, nsb, N, bs);
      rn = enc_load_vec<SPL, CS>(in, gn, !dpp_prev);
      RPP_TSTAMP(2);
      __builtin_amdgcn_s_setprio(0);
      enc_emit<SPL>(E, st, j, empty_lanes);
      __builtin_amdgcn_s_setprio(1);
      RPP_TSTAMP(3);
      enc_plan_b<SPL, G>(F, st, j);
      __builtin_amdgcn_s_setprio(0);
      RPP_TSTAMP(4);
      enc_flush(st, false);
      RPP_TSTAMP(5);
      ++it;
    };
    while (it + 1 < nfull) {
      step(P, Q, r1, g1);  // P = group it, r1 = group it+1 -> Q
      if (it + 1 >= nfull) break;
      step(Q, P, r0, g0);  // Q = group it, r0 = group it+1 -> P
    }
    // the last group: in P after an even number of steps, else in Q
    enc_emit<SPL>((it & 1) ? Q : P, st, j, empty_lanes);
    enc_flush(st, false);
    ++it;
  }
  // ---- ragged tail / unaligned streams: per-sample loads ----
  for (uint32_t s0 = s_lo + it * spw; s0 < nsb; s0 += spw) {
    const EncGeom geo = enc_geom<SPL, CS>(s0 + g, j, nsb, N, bs);
    const EncRaw<SPL> r = enc_load_scalar<SPL, CS>(in, geo);
    enc_iteration<SPL, G, CS, SH>(st, r, geo, j, selbe, be, ulsb, true, false);
    enc_flush(st, false);
  }
  enc_flush(st, true);

  // ---- final words and the ceil(bits/8) tail bytes
  //      (bitstream_writer.h:110-120,139-145) ----
  const uint32_t total_bytes = (st.base + 7) >> 3;
  const uint32_t full_end = st.base >> 5;
  if (multi && seg != 0) {
    // a segment slot: whole words (the last one zero-padded) for the concat
    for (uint32_t w = st.win_w0 + lane; w <= full_end; w += kWave) st.out32[w] = win[w - st.win_w0];
  } else {
    for (uint32_t w = st.win_w0 + lane; w < full_end; w += kWave) st.out32[w] = win[w - st.win_w0];
    const uint32_t tail_bytes = total_bytes - 4 * full_end;
    if (lane < tail_bytes) out8[4 * full_end + lane] = (uint8_t)(win[full_end - st.win_w0] >> (8 * lane));
  }
  if (lane == 0) {
    if (multi) {
      p.seg_bits[blockIdx.x] = st.base;  // (the concat kernel writes size and status)
    } else {
      p.out_bytes[b] = total_bytes;
      p.status[b] = RPP_OK;
    }
  }
#ifdef RPP_STATS
  if (lane == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rpp_stats[i], (unsigned long long)stat_acc[i]);
#endif
}

// Units of each stream (nseg: one per seg_chunks chunks for a stream of
// more than seg_chunks chunks, else 1); entry nblocks is 0 so the exclusive
// scan ends in the total.
__global__ void rpp_enc_units_kernel(const uint64_t* n_samples, uint32_t nblocks, uint32_t chunk_len,
                                     uint32_t seg_chunks, uint64_t* units) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nblocks) return;
  uint64_t u = 0;
  if (i < nblocks) {
    const uint64_t n = n_samples[i];
    const uint64_t nch = (n + chunk_len - 1) / chunk_len;
    u = nch > seg_chunks && n < RPP_MAX_STREAM_SAMPLES ? (nch + seg_chunks - 1) / seg_chunks : 1;
  }
  units[i] = u;
}

__global__ void rpp_enc_unit_map_kernel(const uint64_t* seg_base, uint32_t nblocks, uint64_t max_units,
                                        uint32_t* seg_map) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nblocks || seg_base[nblocks] > max_units) return;  // (over the workspace: nothing is split)
  for (uint64_t u = seg_base[i]; u < seg_base[i + 1]; ++u) seg_map[u] = i;
}

// Places segment k >= 1 of a multi-segment stream at its bit offset o_k in the
// stream's output (seg_off = exclusive scan of seg_bits over all units).  An
// output word belongs to the segment holding its first bit and takes the
// following segment's first bits above that segment's end; the word holding
// o_1 (partly written by segment 0 in place) is merged by segment 1.  The
// last word is written byte by byte up to ceil(bits / 8)
// (bitstream_writer.h:139-145); the last segment writes size and status.
__global__ __launch_bounds__(256) void rpp_enc_concat_kernel(EncParams p, const uint64_t* seg_off) {
  const uint32_t u = blockIdx.x;
  if (!enc_split_ok(p) || u >= p.seg_base[p.nblocks]) return;
  const uint32_t b = p.seg_map[u];
  const uint32_t first = (uint32_t)p.seg_base[b], nseg = (uint32_t)(p.seg_base[b + 1] - first);
  const uint32_t k = u - first;
  if (nseg < 2 || k == 0) return;
  // (bit offsets in the stream are 64-bit: streams go up to 2^30 samples;
  // word indices fit 32 bits)
  const uint64_t base = seg_off[first];
  const uint64_t o_k = seg_off[u] - base;
  const uint32_t L_k = (uint32_t)p.seg_bits[u];
  const uint64_t total_bits = (seg_off[first + nseg - 1] - base) + p.seg_bits[first + nseg - 1];
  const uint64_t total_bytes = (total_bits + 7) >> 3;
  const bool last = k + 1 == nseg;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(p.scratch + (size_t)(u - b - 1) * p.slot_bytes);
  const uint32_t* nxt = last ? nullptr : reinterpret_cast<const uint32_t*>(p.scratch + (size_t)(u - b) * p.slot_bytes);
  const uint64_t o_n = o_k + L_k;  // next segment's offset
  uint8_t* out8 = p.out + p.out_off[b];
  uint32_t* out32 = reinterpret_cast<uint32_t*>(out8);
  auto put = [&](uint32_t w, uint32_t v) {
    if (4ull * w + 4 <= total_bytes) {
      out32[w] = v;
    } else {
      for (uint32_t c = 0; 4ull * w + c < total_bytes; ++c) out8[4ull * w + c] = (uint8_t)(v >> (8 * c));
    }
  };
  // words whose first bit lies in this segment, four per thread (one 16-byte
  // store for a group inside the segment and the stream): word w holds
  // segment bits [32 (w - w_begin) + sh0, + 32), i.e. a funnel shift of
  // slot words w - w_begin and w - w_begin + 1 by the segment's constant sh0
  const uint32_t w_begin = (uint32_t)((o_k + 31) >> 5), w_end = (uint32_t)((o_n + 31) >> 5);
  const uint32_t sh0 = (uint32_t)(32ull * w_begin - o_k);
  const uint32_t nsrc = (L_k + 31) >> 5;  // (the slot's last word is zero-padded past L_k)
  const uint32_t first_next = last ? 0u : nxt[0];  // (the next segment is >= 1024 bits)
  for (uint32_t g = (w_begin >> 2) + threadIdx.x; g < (w_end + 3) >> 2; g += blockDim.x) {
    const int64_t i0 = 4 * (int64_t)g - w_begin;  // slot word of output word 4 g
    uint32_t sw[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) sw[j] = i0 + j >= 0 && i0 + j < (int64_t)nsrc ? src[i0 + j] : 0u;
    uint32_t v[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t w = 4 * g + j;
      v[j] = __builtin_amdgcn_alignbit(sw[j + 1], sw[j], sh0);
      if (!last && 32ull * w + 32 > o_n && 32ull * w < o_n) v[j] |= first_next << (uint32_t)(o_n - 32ull * w);
    }
    if (4 * g >= w_begin && 4 * g + 4 <= w_end && 16ull * g + 16 <= total_bytes) {
      *reinterpret_cast<uint4*>(out32 + 4 * (size_t)g) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j)
        if (4 * g + j >= w_begin && 4 * g + j < w_end) put(4 * g + j, v[j]);
    }
  }
  // the word holding o_1: segment 0's bits below it, segment 1's above
  if (k == 1 && (o_k & 31u) && threadIdx.x == 0) {
    const uint32_t w = (uint32_t)(o_k >> 5), sh = (uint32_t)(o_k & 31u);
    const uint32_t have = 4ull * w < total_bytes ? (uint32_t)min((uint64_t)4, total_bytes - 4ull * w) : 0u;
    uint32_t old = 0;
    for (uint32_t c = 0; c < 4; ++c)
      if (8 * c < sh) old |= (uint32_t)out8[4 * w + c] << (8 * c);
    old &= (1u << sh) - 1u;
    uint32_t v = old | (src[0] << sh);
    if (nseg == 2 && o_n < 32ull * w + 32 && L_k < 32 - sh) v &= (1u << (sh + L_k)) - 1u;
    for (uint32_t c = 0; c < have; ++c) out8[4 * w + c] = (uint8_t)(v >> (8 * c));
  }
  if (last && threadIdx.x == 0) {
    p.out_bytes[b] = total_bytes;
    p.status[b] = RPP_OK;
  }
}

// Host-side kernel choice: SPL 16 for bs > 64 (8 sub-blocks of 128 per
// iteration), else 8; G = next pow2 of ceil(bs / SPL).
typedef void (*EncKernel)(EncParams);
template <uint32_t CS, bool SH>
EncKernel enc_kernel_for(uint32_t bs) {
  if (bs > 64) {
    const uint32_t m = (bs + 15) / 16;
    if (m <= 8) return rpp_encode_kernel<16, 8, CS, SH>;
    if (m <= 16) return rpp_encode_kernel<16, 16, CS, SH>;
    return rpp_encode_kernel<16, 32, CS, SH>;
  }
  const uint32_t m = (bs + 7) / 8;
  if (m <= 1) return rpp_encode_kernel<8, 1, CS, SH>;
  if (m <= 2) return rpp_encode_kernel<8, 2, CS, SH>;
  if (m <= 4) return rpp_encode_kernel<8, 4, CS, SH>;
  return rpp_encode_kernel<8, 8, CS, SH>;
}

// chunks per unit for a batch of total_samples: kEncSegChunks when that gives
// kEncTargetUnits units, else the power of two that comes closest from below
// (a batch of 16 x 64 KiB blocks: 16-chunk units, 16 waves per block)
uint32_t enc_seg_chunks(const rpp_config* cfg, uint64_t total_samples) {
  const uint64_t chunks = total_samples / ((uint64_t)cfg->block_size * cfg->component_stream_count);
  uint32_t c = kEncSegChunks;
  while (c > kEncSegChunksMin && chunks / c < kEncTargetUnits) c >>= 1;
  return c;
}

// streams of more than seg_chunks chunks are split
bool enc_segmented(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples) {
  return max_stream_samples >
         (uint64_t)enc_seg_chunks(cfg, total_samples) * cfg->block_size * cfg->component_stream_count;
}

EncKernel enc_kernel(const rpp_config* cfg) {
  const bool sh = cfg->unused_lsb_count != 0;
  return cfg->component_stream_count == 1
             ? (sh ? enc_kernel_for<1, true>(cfg->block_size) : enc_kernel_for<1, false>(cfg->block_size))
             : (sh ? enc_kernel_for<2, true>(cfg->block_size) : enc_kernel_for<2, false>(cfg->block_size));
}

// rpp_encode_batch_ws workspace: unit counts and bases, the unit -> stream
// map, per-unit bit counts and offsets, and one worst-case scratch slot per
// segment after a stream's first
struct EncWorkspace {
  uint64_t* units;     // [B + 1]
  uint64_t* seg_base;  // [B + 1]
  uint32_t* seg_map;   // [max_units]
  uint64_t* seg_bits;  // [max_units]
  uint64_t* seg_off;   // [max_units]
  uint8_t* scratch;    // [(max_units - B) * slot_bytes]
  uint64_t slot_bytes, max_units, bytes;
  uint32_t seg_chunks;
};

EncWorkspace enc_layout(const rpp_config* cfg, uint64_t total_samples, uint32_t nblocks, uint8_t* base) {
  const uint64_t B = nblocks;
  EncWorkspace w{};
  w.seg_chunks = enc_seg_chunks(cfg, total_samples);
  const uint64_t seg_samples = (uint64_t)w.seg_chunks * cfg->block_size * cfg->component_stream_count;
  w.max_units = B + total_samples / seg_samples;
  w.slot_bytes = (rpp_worst_case_bytes(cfg, seg_samples) + 16 + 15) & ~uint64_t{15};
  uint64_t off = 0;
  auto take = [&](uint64_t bytes) {
    uint8_t* q = base ? base + off : nullptr;
    off = (off + bytes + 255) & ~uint64_t{255};
    return q;
  };
  w.units = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.seg_base = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.seg_map = reinterpret_cast<uint32_t*>(take(w.max_units * 4));
  w.seg_bits = reinterpret_cast<uint64_t*>(take(w.max_units * 8));
  w.seg_off = reinterpret_cast<uint64_t*>(take(w.max_units * 8));
  w.scratch = take((w.max_units - B) * w.slot_bytes);
  w.bytes = off;
  return w;
}

// ===========================================================================
// DECODE
// ===========================================================================
// One stream per wavefront; a workgroup holds up to kDecMaxWaves waves plus
// one shared copy of the transfer tables below.  Per-stream state is
// wave-uniform (scalar registers, uniform branches).
//
// A Rice sub-block (ricepp/include/ricepp/detail/decode.h:62-71) has no
// index: code i+1 starts where code i ends, so the parse is a finite-state
// machine whose state at any bit boundary is "remainder bits still to skip
// before the next unary search" (sigma, 0..fs).  Per 8-bit unit and fs the
// machine's transfer function (sigma -> sigma', and which bits of the byte
// end a code) is a table lookup (g_map_table, 16 B per (fs, byte)).  A
// sub-block is parsed in windows of 64 lane segments of 24 bits starting at
// its 4-bit header:
//   1. each lane composes the maps of its 3 bytes into one segment map;
//   2. a 6-level DPP scan composes the segment maps along the wave (function
//      composition of 8-entry byte maps is two v_perm_b32), so every lane
//      knows its exact entry state -- no speculation, no re-runs;
//   3. the entry state selects each byte's terminator bits -> a 24-bit
//      terminator mask; popcounts -> DPP prefix sums -> code indices and the
//      lane holding the sub-block's last code (its end is the next header);
//   4. each lane turns its terminators into zig-zag deltas (q = gap from the
//      previous code's end, remainder from its registers) into an LDS tile;
//      a chunk's tile is prefix-summed, pixel-encoded and stored.
// fs >= 8 uses 16-entry maps (sigma up to 13), composed by two v_perm_b32
// per dword plus a byte select.
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
  uint32_t waves;          // waves (streams) per workgroup
  uint32_t only_fallback;  // decode only streams whose status is kSegFallback
  const uint64_t* units;   // non-null: skip streams split into more than one unit (segmented decode)
};

// ---- transfer tables (built at compile time) ----
// Entry (fs, byte): dwords {map 0-3, map 4-7, term 0-3, term 4-7}: byte s of
// `map` is the state after the byte when entering it in state s (0..7), byte
// s of `term` the bits of the byte that end a code (the '1' closing a unary
// run) on that path.  Entering in state s >= 8 (fs >= 8 only) skips the byte:
// state s - 8, no terminator.
constexpr uint32_t kMapFs = 14;  // fs 0..13 (fs + 1 = 1..14 is a Rice header)
constexpr uint32_t kMapEntries = kMapFs * 256;

struct MapTable {
  uint32_t w[kMapEntries * 4];
};

constexpr MapTable make_map_table() {
  MapTable t{};
  for (uint32_t fs = 0; fs < kMapFs; ++fs) {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t m[2] = {0, 0}, tm[2] = {0, 0};
      for (uint32_t s = 0; s < 8; ++s) {
        uint32_t c = s, mask = 0, ex = 0;
        for (;;) {
          const uint32_t rest = b >> c;
          if (rest == 0) {  // the unary search runs into the next byte
            ex = 0;
            break;
          }
          const uint32_t tp = c + (uint32_t)__builtin_ctz(rest);
          mask |= 1u << tp;
          c = tp + 1 + fs;  // skip the terminator and fs remainder bits
          if (c >= 8) {
            ex = c - 8;
            break;
          }
        }
        m[s >> 2] |= ex << (8 * (s & 3));
        tm[s >> 2] |= mask << (8 * (s & 3));
      }
      const uint32_t e = (fs * 256 + b) * 4;
      t.w[e] = m[0];
      t.w[e + 1] = m[1];
      t.w[e + 2] = tm[0];
      t.w[e + 3] = tm[1];
    }
  }
  return t;
}

__device__ const MapTable g_map_table = make_map_table();

// The transfer tables into LDS, eight 16-byte loads in flight per lane (a
// one-wave workgroup -- small batches -- copies the 56 KiB in 7 round trips
// instead of 56).  The caller synchronises.
__device__ __forceinline__ void copy_tables(uint4* dsm) {
  const uint4* gt = reinterpret_cast<const uint4*>(g_map_table.w);
  const uint32_t bd = blockDim.x;
  uint32_t i = threadIdx.x;
  for (; i + 7 * bd < kMapEntries; i += 8 * bd) {
    uint4 v[8];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) v[k] = gt[i + k * bd];
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) dsm[i + k * bd] = v[k];
  }
  for (; i < kMapEntries; i += bd) dsm[i] = gt[i];
}

constexpr uint32_t kSegBits = 24;                // bits per lane segment (3 table bytes)
constexpr uint32_t kWinBits = kWave * kSegBits;  // bits per window
constexpr uint32_t kRingWords = 1024;            // per-stream LDS ring of the compressed stream (4 KiB)
constexpr uint32_t kRingMask = kRingWords - 1;
constexpr uint32_t kChunkWords = 4 * kWave;      // refill unit: 16 B per lane
constexpr uint32_t kAhead = 288;                 // words kept resident ahead of the read position
constexpr uint32_t kDecMaxWaves = 16;            // waves per workgroup (one table copy each)
constexpr uint32_t kRingPad = 64;               // ring words 0..63 mirrored after the ring end
constexpr uint32_t kListDump = 512;            // list slot written by masked-off lanes
constexpr uint32_t kListWords = kListDump + 24;  // terminator positions of one sub-block (bs <= 512), dump pairs (MT <= 12)
constexpr uint32_t kListLead = 4;  // words before a decode list: pair -1 = (0, 0), a_(-1) of the fast loop's deltas
constexpr uint32_t kWaveLdsWords = kRingWords + kRingPad + kListLead + kListWords;
constexpr uint32_t kTabBytes = kMapEntries * 16;

__device__ __forceinline__ uint32_t wave_last(uint32_t v) { return readlane(v, kWave - 1); }

// Packed 2 x u16 arithmetic (wraps per half-word).
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as_u32(as_us2(a) + as_us2(b)); }

__device__ __forceinline__ uint32_t wave_incl_sum_pk(uint32_t v) {
  v = pk_add(v, dpp<kDppRowShr1>(v));
  v = pk_add(v, dpp<kDppRowShr2>(v));
  v = pk_add(v, dpp<kDppRowShr4>(v));
  v = pk_add(v, dpp<kDppRowShr8>(v));
  v = pk_add(v, dpp<kDppRowBcast15, 0xA>(v));
  v = pk_add(v, dpp<kDppRowBcast31, 0xC>(v));
  return v;
}

// pixel write (ricepp_cpuspecific_traits.h:69-73) of two packed samples;
// sel = v_perm selector that byte-swaps each half (big endian) or not
__device__ __forceinline__ uint32_t px_write2(uint32_t v, uint32_t sel, uint32_t ulsb) {
  v = as_u32(as_us2(v) << (us2)(unsigned short)ulsb);
  return __builtin_amdgcn_perm(v, v, sel);
}

// ---- state maps ----
// An 8-entry map (states 0..7) is 8 bytes; byte s = image of s.  g after f
// (apply f first): byte s of the result = g[f[s]] = v_perm_b32(g.hi, g.lo, f).
constexpr uint32_t kId0 = 0x03020100u, kId1 = 0x07060504u, kId2 = 0x0B0A0908u, kId3 = 0x0F0E0D0Cu;
constexpr uint32_t kSelByte0 = 0x0C0C0C00u;  // v_perm selector: byte 0 = index, bytes 1-3 = 0

struct Map8 {
  uint32_t lo, hi;
};
__device__ __forceinline__ Map8 comp8(Map8 g, Map8 f) {
  return Map8{__builtin_amdgcn_perm(g.hi, g.lo, f.lo), __builtin_amdgcn_perm(g.hi, g.lo, f.hi)};
}
template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ Map8 scan_step8(Map8 m) {
  const Map8 d{dpp_keep<Ctrl, RowMask>(kId0, m.lo), dpp_keep<Ctrl, RowMask>(kId1, m.hi)};
  return comp8(m, d);
}

// One scan step as two DPP moves into persistent registers: lanes without a
// source (row_shr: the first lanes of each row; row_bcast: the rows the row
// mask leaves out; wave_shr: lane 0) are not written by a DPP move without
// bound_ctrl, so they keep the identity map the register was initialised
// with -- no mask, no vcc.  s_nop 1: a DPP read of a VGPR written by the
// previous VALU instruction needs two wait states.
#define RPP_SCAN8_STEP(NAME, CTRL, RM)                                                           \
  __device__ __forceinline__ Map8 NAME(Map8 m, Map8& keep) {                                              \
    asm("s_nop 1\n\t"                                                                                    \
        "v_mov_b32_dpp %0, %2 " CTRL " row_mask:" RM " bank_mask:0xf\n\t"                                \
        "v_mov_b32_dpp %1, %3 " CTRL " row_mask:" RM " bank_mask:0xf"                                      \
        : "+v"(keep.lo), "+v"(keep.hi)                                                                    \
        : "v"(m.lo), "v"(m.hi));                                                                          \
    return comp8(m, keep);                                                                                \
  }
RPP_SCAN8_STEP(scan8_shr1, "row_shr:1", "0xf")
RPP_SCAN8_STEP(scan8_shr2, "row_shr:2", "0xf")
RPP_SCAN8_STEP(scan8_shr4, "row_shr:4", "0xf")
RPP_SCAN8_STEP(scan8_shr8, "row_shr:8", "0xf")
RPP_SCAN8_STEP(scan8_bc15, "row_bcast:15", "0xa")
RPP_SCAN8_STEP(scan8_bc31, "row_bcast:31", "0xc")
// the persistent destination registers of the six steps and of the final
// shift, initialised to the identity map (opaque to the compiler)
struct ScanRegs {
  Map8 r1, r2, r4, r8, b15, b31, w1;
  // entry-state rounds (w32_count, fs >= 8 loop): lane 0 holds the window's
  // entry state (skip the 4-bit header) in replicated form and is never
  // written
  uint32_t ja, jb;
  __device__ ScanRegs() {
    Map8* all[7] = {&r1, &r2, &r4, &r8, &b15, &b31, &w1};
    for (Map8* x : all) {
      x->lo = kId0;
      x->hi = kId1;
      asm volatile("" : "+v"(x->lo), "+v"(x->hi));
    }
    ja = jb = 0x04040404u;
    asm volatile("" : "+v"(ja), "+v"(jb));
  }
};
// the value of lane l-1 into `keep` (lane 0 keeps its value)
__device__ __forceinline__ uint32_t jshift(uint32_t x, uint32_t& keep) {
  asm("s_nop 1\n\tv_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(keep) : "v"(x));
  return keep;
}
// wave priority over the fast loop's parse chain (profiles/r02_prio_ab.jsonl)
constexpr int kParsePrio = 1;

// fs >= 8: states 0..13 (13 remainder bits still to skip at most).  A state
// is kept replicated in all four bytes of a dword (a v_perm selector that
// yields the looked-up byte in all four bytes).  One byte of the segment:
// states 0..7 go through the byte's 8-entry map (table entry .x/.y); a state
// s >= 8 skips the byte (s - 8).  v_perm gives 0x00 for selectors 8..12 (the
// map bytes are < 0x80) and 0xFF for 13, so s' = max_i16(perm, s - 8) per
// half-word: below 8 the subtraction is negative in both halves.
constexpr int kJacobi16 = 4;  // fixed rounds before the settle check (fs >= 8)
__device__ __forceinline__ uint32_t pk_max_i16(uint32_t a, uint32_t b) {
  return as_u32(__builtin_bit_cast(us2, __builtin_elementwise_max(__builtin_bit_cast(ss2, a), __builtin_bit_cast(ss2, b))));
}
__device__ __forceinline__ uint32_t byte_step(uint32_t S, uint4 e) {
  return pk_max_i16(__builtin_amdgcn_perm(e.y, e.x, S), S - 0x08080808u);
}
// the byte's terminator bits when entered in state S (none when skipped)
__device__ __forceinline__ uint32_t byte_term(uint32_t S, uint4 e) {
  uint32_t skip;  // all ones for s >= 8 (bit 3; s <= 13)
  asm("v_bfe_i32 %0, %1, 3, 1" : "=v"(skip) : "v"(S));
  return __builtin_amdgcn_perm(e.w, e.z, S) & ~skip;
}
#undef RPP_SCAN8_STEP
// exclusive form: the map of lanes 0..l-1 (identity on lane 0)
__device__ __forceinline__ Map8 shift8_wave(Map8 m, Map8& keep) {
  asm("s_nop 1\n\t"
      "v_mov_b32_dpp %0, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_mov_b32_dpp %1, %3 wave_shr:1 row_mask:0xf bank_mask:0xf"
      : "+v"(keep.lo), "+v"(keep.hi)
      : "v"(m.lo), "v"(m.hi));
  return keep;
}

// 16-entry maps (states 0..15) for fs >= 8.
struct Map16 {
  uint32_t w[4];
};
// bytes of g selected by the 4 byte indices (0..15) in idx
__device__ __forceinline__ uint32_t sel16(const Map16& g, uint32_t idx) {
  const uint32_t i7 = idx & 0x07070707u;
  const uint32_t lo = __builtin_amdgcn_perm(g.w[1], g.w[0], i7);
  const uint32_t hi = __builtin_amdgcn_perm(g.w[3], g.w[2], i7);
  const uint32_t m = idx & 0x08080808u;
  const uint32_t mask = (m << 5) - (m >> 3);  // 0xFF in bytes with index >= 8
  return (hi & mask) | (lo & ~mask);
}
__device__ __forceinline__ Map16 comp16(const Map16& g, const Map16& f) {
  return Map16{{sel16(g, f.w[0]), sel16(g, f.w[1]), sel16(g, f.w[2]), sel16(g, f.w[3])}};
}
template <int Ctrl, int RowMask = 0xF>
__device__ __forceinline__ Map16 scan_step16(const Map16& m) {
  const Map16 d{{dpp_keep<Ctrl, RowMask>(kId0, m.w[0]), dpp_keep<Ctrl, RowMask>(kId1, m.w[1]),
                 dpp_keep<Ctrl, RowMask>(kId2, m.w[2]), dpp_keep<Ctrl, RowMask>(kId3, m.w[3])}};
  return comp16(m, d);
}

// Front end of the fs 8..13 parse (32-bit lane segments): states 0..13 and no
// map scan -- the entry states by jacobi rounds of byte steps (states in
// replicated form, byte_step); the per-byte states of the final round give
// the terminator mask tm of the lane's segment; then the counts (inclusive
// prefix incl, the lanes reaching n codes in finm) and the rider's prefix as
// in the fused fast loop.
// (exit_state: each lane's state after its segment, in replicated form, for a
// parse that continues in the next window)
__device__ __forceinline__ void w32_count(uint4 e0, uint4 e1, uint4 e2, uint4 e3, uint32_t n, uint32_t rider,
                                          ScanRegs& sreg, uint32_t& tm, uint32_t& cnt, uint32_t& incl,
                                          uint64_t& finm, uint32_t& rider_incl, uint32_t* exit_state = nullptr) {
  // lanes up to the first one that ends the sub-block (all when none does)
  auto upto_end = [](uint64_t fm) { return (2ull << (uint32_t)__builtin_ctzll(fm | (1ull << 63))) - 1ull; };
  uint32_t S1, S2, S3;
  auto eval = [&](uint32_t S0) {
    S1 = byte_step(S0, e0);
    S2 = byte_step(S1, e1);
    S3 = byte_step(S2, e2);
    return byte_step(S3, e3);
  };
  auto term_mask = [&](uint32_t S0) {
    const uint32_t a0 = byte_term(S0, e0), a1 = byte_term(S1, e1), a2 = byte_term(S2, e2), a3 = byte_term(S3, e3);
    return __builtin_amdgcn_perm(a3, a2, 0x04000C0Cu) | __builtin_amdgcn_perm(a1, a0, 0x0C0C0400u);
  };
  uint32_t ea = jshift(eval(0u), sreg.ja), eb = 0;
#pragma unroll
  for (int r = 0; r < kJacobi16; ++r) {
    if (r & 1) ea = jshift(eval(eb), sreg.ja);
    else eb = jshift(eval(ea), sreg.jb);
  }
  // the last eval ran on the older of ea / eb; where the round changed
  // nothing its byte states are exact
  uint32_t Sold = (kJacobi16 & 1) ? ea : eb;
  uint32_t Snew = (kJacobi16 & 1) ? eb : ea;
  uint64_t unsettled = __ballot(Sold != Snew);
  tm = term_mask(Sold);
  cnt = __builtin_popcount(tm);
  const uint32_t incl2 = wave_incl_sum(cnt | (rider << 16));
  incl = incl2 & 0xFFFFu;
  rider_incl = incl2 >> 16;
  finm = __ballot(incl >= n);
  // more rounds until every lane up to the sub-block's end is settled (lane
  // l is exact after l rounds: at most 64)
  for (uint32_t guard = 0; (unsettled & upto_end(finm)) && guard < 2 * kWave; ++guard) {
    Sold = Snew;
    Snew = jshift(eval(Sold), sreg.ja);
    unsettled = __ballot(Sold != Snew);
    tm = term_mask(Sold);
    cnt = __builtin_popcount(tm);
    incl = wave_incl_sum(cnt);
    finm = __ballot(incl >= n);
  }
  if (exit_state) *exit_state = eval(Sold);
}

// Orders this wave's LDS accesses without waiting on its global stores
// (LDS operations of one wave complete in order; a full __syncthreads()
// would also drain vmcnt, i.e. wait for the previous chunk's output stores).
__device__ __forceinline__ void lds_fence() { asm volatile("" ::: "memory"); }

// Asynchronous global -> LDS copies (global_load_lds): lane l's 16 (4) bytes
// land at LDS byte address m0 + 16 l (4 l).  Issued by asm, so the compiler
// neither waits for them nor counts them: the caller retires them with
// vm_drain() before the words are read.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t m0) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t m0) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0) : "memory");
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Waits for all but the last `after` vector-memory instructions (vmcnt
// decrements in issue order on gfx9), bucketed to a few immediates; a lower
// count only waits longer.
__device__ __forceinline__ void vm_wait_all_but(uint32_t after) {
  if (after >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (after >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (after >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// (a << s) | b in one v_lshl_or_b32 (s uniform)
__device__ __forceinline__ uint32_t lshl_or(uint32_t a, uint32_t sh, uint32_t b) {
  uint32_t r;
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(sh), "v"(b));
  return r;
}
// -(x & 1) in one v_bfe_i32
__device__ __forceinline__ uint32_t neg_lsb(uint32_t x) {
  uint32_t r;
  asm("v_bfe_i32 %0, %1, 0, 1" : "=v"(r) : "v"(x));
  return r;
}

// 16 * byte B of x in one VOP2 operation (SDWA source select)
template <int B>
__device__ __forceinline__ uint32_t sdwa_byte16(uint32_t x) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(x));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(x));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(x));
  else
    asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(x));
  return r;
}
// the table entry at byte offset off16 (16 * entry) from tb
__device__ __forceinline__ uint4 tb_entry(const uint4* tb, uint32_t off16) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(tb) + off16);
}

// v_ffbl_b32: index of the lowest set bit, 0xFFFFFFFF for 0
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
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

// SH: unused_lsb_count != 0 (the pixel write shifts)
template <uint32_t CS, bool SH>
__global__ __launch_bounds__(kWave* kDecMaxWaves) void rpp_decode_kernel(DecParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 dsm[];
  // ---- this wave's stream, and whether the workgroup has anything to do (the
  //      fallback launch skips most streams: leave before the table copy) ----
  const uint32_t b = blockIdx.x * p.waves + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  bool mine = b < p.nblocks;
  if (mine && p.only_fallback) mine = p.status[b] == rpp_internal::kSegFallback;
  if (mine && p.units && p.units[b] > 1) mine = false;
  if (!__syncthreads_or(mine)) return;
  // ---- the transfer tables, one copy per workgroup ----
  copy_tables(dsm);
  __syncthreads();
  const uint4* tab = dsm;
  const uint32_t lane = lane_id();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  // (one opaque scalar word offset, so that ring addresses fold into one
  // scalar base)
  uint32_t ring_w = kTabBytes / 4 + wv * kWaveLdsWords;
  asm("" : "+s"(ring_w));
  uint32_t* ring = reinterpret_cast<uint32_t*>(dsm) + ring_w;
  uint32_t* list = ring + kRingWords + kRingPad + kListLead;  // terminator positions of the current sub-block
  if (lane < kListLead) list[(int)lane - (int)kListLead] = 0u;  // (never written again)
  const uint32_t bs = p.bs, be = p.be, ulsb = p.ulsb;
  const uint32_t selbe = be ? 0x02030001u : 0x03020100u;
  const uint32_t selpack = be ? 0x04050001u : 0x05040100u;  // v_perm(hi, lo): pack two samples (+ swap)
  const uint32_t lane24 = kSegBits * lane;
  if (!mine) return;  // no barrier below this point
#ifdef RPP_STATS
  uint32_t stat_acc[16] = {0};
  unsigned long long tprev_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tprev_)::"memory");
#endif

  // ---- per-stream setup (wave-uniform) ----
  // Bit positions are 32-bit and relative to `in`, which starts at the
  // 4-aligned word holding the stream's first byte; a stream longer than
  // 2^30 bits (blocks of more than ~2^26 samples: mkdwarfs -S 28..30) is
  // rebased as the parse goes (rebase() below), so any stream the C ABI
  // accepts decodes here.
  int32_t status = RPP_OK;
  uint32_t N = 0, nbytes = 0, mis = 0;
  uint64_t nb_all = 0, lim_all = 0;  // the stream's bytes (+ mis) and readable bits from the original base
  const uint8_t* in = p.in;
  uint16_t* out = p.out;
  {
    const uint64_t n64 = p.n_samples[b];
    const uint64_t ioff = p.in_off[b];
    const uint64_t nb64 = p.in_bytes[b];
    if (n64 % CS != 0 || n64 >= RPP_MAX_STREAM_SAMPLES || nb64 >= (UINT64_C(1) << 32) - 8) {
      status = RPP_INVALID_ARGUMENT;
    } else {
      mis = (uint32_t)(ioff & 3u);
      N = (uint32_t)n64;
      nb_all = nb64 + mis;
      // last readable bit + 1: the reader pulls whole 8-byte packets of the
      // stream (bitstream_reader.h:149-183), so it only throws past this point.
      lim_all = 8u * mis + 64u * ((nb64 + 7u) >> 3);
      in = p.in + (ioff - mis);
      out = p.out + p.out_off[b];
    }
  }
  const bool aligned16 = ((uintptr_t)in & 15u) == 0;
  nbytes = (uint32_t)nb_all;
  uint32_t lim = (uint32_t)min(lim_all, (uint64_t)0xFFFFFFFFu);
  uint64_t base_w = 0;  // words `in` has moved by
  const uint32_t chunk_len = CS * bs;
  const uint32_t nchunks = status == RPP_OK ? (N + chunk_len - 1) / chunk_len : 0u;

  // ---- LDS ring of the stream's words: words [fill_w - kRingWords, fill_w)
  //      are resident.  Steady state: at the end of an iteration, a chunk of
  //      256 words lying wholly inside the input is requested by
  //      global_load_lds (no registers, nothing for the compiler to wait on);
  //      it is retired (vmcnt(0), by then long complete) a few iterations
  //      later, and only then counted resident.  ensure() is the synchronous
  //      path (start-up, the zero-padded tail, long sub-blocks). ----
  uint32_t fill_w = 0;
  bool pend = false;  // a requested chunk is in flight
  // vector-memory instructions known to be issued after the pending request
  // (the fast loop's output stores; elsewhere reset to 0 = unknown), so that
  // retiring it need not wait for the stores
  uint32_t vm_after = 0;
  auto retire = [&]() {
    if (pend) {
      vm_wait_all_but(vm_after);
      fill_w += kChunkWords;
      pend = false;
    }
  };
  auto refill_sync = [&]() {  // appends 256 words (zero past the input) synchronously
    const uint32_t w = fill_w + 4 * lane;
    uint4 v;
    if (aligned16 && 4 * w + 16 <= nbytes) {
      v = *reinterpret_cast<const uint4*>(in + 4 * w);
    } else {
      v = make_uint4(stream_word(in, nbytes, w), stream_word(in, nbytes, w + 1), stream_word(in, nbytes, w + 2),
                     stream_word(in, nbytes, w + 3));
    }
    *reinterpret_cast<uint4*>(&ring[w & kRingMask]) = v;
    if ((w & kRingMask) < kRingPad) *reinterpret_cast<uint4*>(&ring[kRingWords + (w & kRingMask)]) = v;
    fill_w += kChunkWords;
  };
  auto request = [&]() {  // asynchronous 256-word chunk (only wholly inside the input)
    if (4u * (fill_w + kChunkWords) > nbytes) return;
    // m0 such that lane l lands at ring slot + 16 l (4 l)
    const uint32_t slot = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&ring[fill_w & kRingMask]);
    const uint8_t* src = in + 4u * fill_w;
    if (aligned16) {
      glds16(src + 16u * lane, slot);
    } else {
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) glds4(src + 256u * q + 4u * lane, slot + 256u * q);
    }
    if ((fill_w & kRingMask) == 0)  // the mirror of words 0..63
      glds4(src + 4u * lane, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&ring[kRingWords]));
    pend = true;
    vm_after = 0;
  };
  refill_sync();
  refill_sync();
  lds_fence();
  // keeps words [w, w + kAhead) of the stream resident
  auto ensure = [&](uint32_t w) {
    if (fill_w < w + kAhead) {
      retire();
      while (fill_w < w + kAhead) refill_sync();
      lds_fence();
    }
  };
  // words w, w + 1, w + 2 are contiguous in LDS thanks to the mirror
  auto wptr = [&](uint32_t w) -> const uint32_t* { return ring + (w & kRingMask); };
  auto peek32 = [&](uint32_t pos) -> uint32_t {
    const uint32_t* q = wptr(pos >> 5);
    return __builtin_amdgcn_alignbit(q[1], q[0], pos & 31u);
  };

  // codec.h:69-74,81-86: the 16-bit initial value of each component
  uint32_t last0 = 0, last1 = 0;
  uint32_t P = 8 * mis + 16 * CS;
  // moves `in` forward by a multiple of the ring's size below P (ring slots
  // and the pending chunk keep their places), once P passes 2^30; between
  // two rebases the parse advances less than 2^31 bits (the fast loop stops
  // at 2^31, see ring_bounds), so positions never wrap
  auto rebase = [&]() {
    if (P < (1u << 30)) return;
    const uint32_t sh = ((P >> 5) - kRingWords) & ~(kRingWords - 1u);
    in += 4ull * sh;
    base_w += sh;
    P -= 32u * sh;
    fill_w -= sh;
    nbytes = (uint32_t)(nb_all - 4ull * base_w);
    lim = (uint32_t)min(lim_all - 32ull * base_w, (uint64_t)0xFFFFFFFFu);
  };
  if (status == RPP_OK) {
    if (P > lim) status = RPP_TRUNCATED_INPUT;
    last0 = __builtin_amdgcn_readfirstlane(peek32(8 * mis) & 0xFFFFu);
    if (CS > 1) last1 = __builtin_amdgcn_readfirstlane(peek32(8 * mis + 16) & 0xFFFFu);
  }
  // this lane's 64 bits from bit sb of the stream (its 24-bit segment of a
  // window and what follows it)
  auto load_x = [&](uint32_t sb, uint32_t& xl, uint32_t& xh) {
    const uint32_t* q = wptr(sb >> 5);
    const uint32_t o = sb & 31u;
    const uint32_t a0 = q[0], a1 = q[1], a2 = q[2];
    xl = __builtin_amdgcn_alignbit(a1, a0, o);
    xh = __builtin_amdgcn_alignbit(a2, a1, o);
  };
  // keep the look-ahead: retire the pending chunk once it is needed soon;
  // request the next once the look-ahead drops below 766 words (it
  // overwrites words [fill_w - 1024, fill_w - 768), all below q >> 5, the
  // next bit to be read)
  auto ring_keep = [&](uint32_t q) {
    if (pend && fill_w < (q >> 5) + kAhead + 128) retire();
    if (!pend && fill_w <= (q >> 5) + 766) request();
  };
  const uint32_t nsb = nchunks * CS;
  // sub-blocks the fast loop may take: those of full 128-sample chunks
  // (CS 1: the 2-sample stores must be dword aligned)
  // bs 128: two codes per lane, 2-sample stores (CS 1: dword aligned);
  // bs 16, 32, 64: one code per lane
  const bool fast_bs = bs == 2 * kWave ? (CS == 2 || (((uintptr_t)out) & 3u) == 0)
                                       : (bs == 16 || bs == 32 || bs == 64);
  const uint32_t nsb_fast = fast_bs ? (N / chunk_len) * CS : 0u;
  // one-code-per-lane stores: this lane's byte offset in a sub-block, far
  // out of range (dropped) for lanes past it
  const uint32_t lane_off1 = lane < bs ? 2u * CS * lane : 0x7FFFFFF0u;
  // the stream's output as a raw buffer (N * 2 < 2^28 bytes; stores past it are dropped)
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(2 * N), 0x00020000);
  ScanRegs sreg;

  for (uint32_t s = 0; s < nsb && status == RPP_OK; ++s) {
    rebase();
    // ---- fast loop (the common case): Rice sub-blocks of 128 codes with fs
    //      5..7 that lie in one window, ring resident.  Straight-line code: at
    //      most 4 terminators per 24-bit segment (codes are >= 6 bits), every
    //      lane owns exactly 2 codes.  Software-pipelined: while sub-block s is
    //      turned into samples, sub-block s+1 is parsed (ring read, table
    //      lookups, scans) in the same basic block, so the LDS latencies and
    //      DPP chains of the two overlap.  Anything else leaves the loop and
    //      takes the general path below for that sub-block. ----
    // MT: terminators a lane segment can hold (codes of >= fs + 1 bits),
    // [LO, HI]: the fs range of this instance (fs 8..13: 32-bit segments)
    // TWO: bs 128, two codes per lane; else bs <= 64, one code per lane
    auto fast = [&]<uint32_t MT, uint32_t LO, uint32_t HI, bool TWO>() {
      // fs >= 8: 32-bit lane segments (2048-bit windows), entry states by
      // jacobi rounds over 14 states; else 24-bit segments and 8-state maps
      constexpr bool W32 = LO >= 8;
      constexpr uint32_t SB = W32 ? 32u : kSegBits;
      const uint32_t n = TWO ? 2 * kWave : bs;
      const uint4* const list4 = reinterpret_cast<const uint4*>(list);
      uint2* const list2 = reinterpret_cast<uint2*>(list);
      // this lane's 32 bits from bit q + SB lane (24-bit segments: the
      // segment and 8 more, where a terminator in it has its <= 7 remainder
      // bits; 32-bit segments: the next 32 bits in xh)
      // (window start word and bit offset are scalar; 24-bit segments: the
      // lane's words lie within 50 words of the window start, inside the
      // ring's mirror; 32-bit segments: the first word index is wrapped per
      // lane, the next two are in the mirror)
      auto seg_bits = [&](uint32_t q, uint32_t& xh) {
        if constexpr (W32) {
          const uint32_t* w = ring + (((q >> 5) + lane) & kRingMask);
          const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
          xh = __builtin_amdgcn_alignbit(w2, w1, q & 31u);
          return __builtin_amdgcn_alignbit(w1, w0, q & 31u);
        } else {
          // (vector addressing from q + lane24 alone: no scalar splitting of
          // q; word wi + 1 <= kRingWords lies in the ring's mirror)
          const uint32_t x = q + lane24;
          const uint32_t* w = ring + ((x >> 5) & kRingMask);
          xh = 0u;
          return __builtin_amdgcn_alignbit(w[1], w[0], x);  // (shift x mod 32)
        }
      };
      // the header's fs (scalar; not clamped: a header outside [LO+1, HI+1]
      // -- which the loop then leaves -- makes lookups read other LDS words or
      // out of range, which reads 0; their results are discarded)
      auto fs_of = [](uint32_t h) { return (h & 15u) - 1u; };
      auto header_ok = [](uint32_t h) { return (uint32_t)((h & 15u) - (LO + 1) <= HI - LO); };
      // Parse of the sub-block at bit q: entry states by the map scan,
      // terminators, (a_i, remainder) of code i into list pair i with a_i =
      // terminator position - (q + 4) - i k (the unary part of code i is then
      // a_i - a_(i-1), a_(-1) = 0).  Returns whether the sub-block ends in the
      // window, and its end (the header of the next) in Pe.
      // The count scan also carries a rider: the previous sub-block's delta
      // sums in the high halves (mod 2^16; counts <= 512 stay in the low
      // halves), so that sub-block's value prefix costs no scan of its own.
      // The next window's bits are read from the ring as soon as Pe is known
      // (into xln / xhn), before this sub-block's list writes, so that the
      // read's LDS latency overlaps them instead of opening the next parse.
      auto parse = [&](uint32_t q, uint32_t xl, uint32_t xh, uint32_t fs, uint4 e0, uint4 e1, uint4 e2, uint4 e3,
                       uint32_t& Pe, uint32_t& xln, uint32_t& xhn, uint32_t rider, uint32_t& rider_incl,
                       auto&& mid) -> uint32_t {
        __builtin_amdgcn_s_setprio(kParsePrio);
        const uint32_t k = fs + 1;
        // (off the chain) the end is q + 4 + n k + a_(n-1)
        const uint32_t pe_base = q + 4u + n * k;
        uint32_t tm, cnt, incl;
        uint32_t tot2;  // lane 63's inclusive sums: the window's code count (low), the rider's total (high)
        if constexpr (!W32) {
          const Map8 M01 = comp8(Map8{e1.x, e1.y}, Map8{e0.x, e0.y});  // (also gives byte 2's entry state)
          const Map8 M = comp8(Map8{e2.x, e2.y}, M01);
          // state 4 at the window start: skip the header.  A selector
          // carries the state in byte 0 (the other bytes are 0xFF or copies
          // of byte 0), so each byte's next state comes out of its v_perm as
          // the next selector, with no masking.
          auto scan_sel = [&]() {
            Map8 S = scan8_shr1(M, sreg.r1);
            S = scan8_shr2(S, sreg.r2);
            S = scan8_shr4(S, sreg.r4);
            S = scan8_shr8(S, sreg.r8);
            S = scan8_bc15(S, sreg.b15);
            S = scan8_bc31(S, sreg.b31);
            const Map8 X = shift8_wave(S, sreg.w1);
            return __builtin_amdgcn_perm(X.hi, X.lo, 0xFFFFFF04u);
          };
          // terminator mask of the segment entered in state sel: byte 0 of
          // a0, a1, a2 -> bytes 0, 1, 2
          auto term_mask = [&](uint32_t sel) {
            const uint32_t a0 = __builtin_amdgcn_perm(e0.w, e0.z, sel);
            const uint32_t a1 = __builtin_amdgcn_perm(e1.w, e1.z, __builtin_amdgcn_perm(e0.y, e0.x, sel));
            const uint32_t a2 = __builtin_amdgcn_perm(e2.w, e2.z, __builtin_amdgcn_perm(M01.hi, M01.lo, sel));
            return __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x0C0C0400u), 0x0C040100u);
          };
          tm = term_mask(scan_sel());
          cnt = __builtin_popcount(tm);
          const uint32_t incl2 = wave_incl_sum(cnt | (rider << 16));
          incl = incl2 & 0xFFFFu;
          // (the rider in the high halves is exact whatever the counts: they
          // sum to at most 512 and never carry into it)
          rider_incl = incl2 >> 16;
          tot2 = readlane(incl2, kWave - 1);
        } else {
          uint64_t finm;
          w32_count(e0, e1, e2, e3, n, rider, sreg, tm, cnt, incl, finm, rider_incl);
          tot2 = readlane(incl, kWave - 1) | (readlane(rider_incl, kWave - 1) << 16);
        }
        const uint32_t excl = incl - cnt;
        RPP_TSTAMP(7);
        // terminator positions t0 < t1 < ... in the segment (garbage past
        // cnt)
        uint32_t t[MT];
#pragma unroll
        for (uint32_t j = 0; j < MT; ++j) {
          t[j] = ffbl(tm);
          tm &= tm - 1;
        }
        RPP_TSTAMP(8);
        // pair excl + j for j = MT-1 .. 0, one instruction each (kept apart:
        // a merged ds_write2 would put two j in one instruction): a slot past
        // this lane's codes belongs to a later lane, which writes it in a
        // later instruction (its j is smaller); lanes without terminators or
        // past the sub-block write the unused pairs from 256
        const uint32_t base = cnt != 0 && excl < n ? excl : 256u;
        uint32_t abase = (uint32_t)((int)(SB * lane - 4u) + __mul24((int)base, -(int)k));
        asm volatile("" : "+v"(abase));  // computed once, not per pair
        const uint32_t xr = xl >> 1;     // the remainder of a terminator at t is bits t+1 .. t+fs
#pragma unroll
        for (int j = MT - 1; j >= 0; --j) {
          // (32-bit segments: the remainder may reach into the next word)
          const uint32_t rem = W32 ? __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(xh, xl, t[j]), 1, fs)
                                   : __builtin_amdgcn_ubfe(xr, t[j], fs);
          list2[base + j] = make_uint2(abase + t[j] - j * k, rem);
          lds_fence();
        }
        // the next sub-block starts after code n-1's remainder: its entry,
        // read back from the list (one broadcast LDS read after the writes,
        // instead of picking the terminator out of the lane that holds it);
        // unused when the sub-block does not end in the window
        // (picking it by readlane out of the lane that holds it measured
        // slower: profiles/r04_decode_ab.jsonl)
        Pe = pe_base + __builtin_amdgcn_readfirstlane(list[2 * (n - 1)]);
        __builtin_amdgcn_s_setprio(0);
        xln = seg_bits(Pe, xhn);
        // (the previous sub-block's stores, off the chain)
        mid(rider_incl, tot2 >> 16);
        RPP_TSTAMP(13);
        return (uint32_t)((tot2 & 0xFFFFu) >= n);
      };
      // codes 2c, 2c+1 of a sub-block on lane c -> zig-zag deltas
      // (decode.h:66-69): d1 and the lane's sum d0 + d1
      // (aprev: a of the code before this lane's first, read from the list;
      // a_(-1) = 0 lies in the list's lead words)
      auto deltas = [&](uint4 tt, uint32_t aprev, uint32_t fs, uint32_t& d1, uint32_t& dsum) {
        if constexpr (TWO) {
          const uint32_t df0 = lshl_or(tt.x - aprev, fs, tt.y), df1 = lshl_or(tt.z - tt.x, fs, tt.w);
          const uint32_t d0 = (df0 >> 1) ^ neg_lsb(df0);
          d1 = (df1 >> 1) ^ neg_lsb(df1);
          dsum = d0 + d1;
        } else {
          // code c on lane c (pair c in tt.x, tt.y); lanes past the
          // sub-block contribute nothing to the prefix
          const uint32_t df = lshl_or(tt.x - aprev, fs, tt.y);
          d1 = (df >> 1) ^ neg_lsb(df);
          dsum = lane < n ? d1 : 0u;
        }
      };
      // inclusive prefix inc of the delta sums -> values -> stored samples of
      // sub-block sx
      // (inc_last: inc of lane 63, the sub-block's delta total)
      auto store = [&](uint32_t d1, uint32_t inc, uint32_t inc_last, uint32_t sx) {
        const uint32_t comp = sx % CS;
        const uint32_t lastc = comp ? last1 : last0;
        const uint32_t v1 = lastc + inc;  // value of sample 2c + 1 (TWO) or c (mod 2^16)
        if constexpr (!TWO) {
          const uint32_t o = SH ? px_write2(v1, selbe, ulsb) : __builtin_amdgcn_perm(v1, v1, selbe);
          __builtin_amdgcn_raw_buffer_store_b16((uint16_t)o, orsrc, lane_off1,
                                                (int)(2 * ((sx / CS) * chunk_len + comp)), 0);
          const uint32_t lnew = lastc + inc_last;
          if (comp) last1 = lnew;
          else last0 = lnew;
          return;
        }
        // samples 2c (low), 2c+1 (high) in stored order: pack and byte-swap
        // in one v_perm when there is no shift
        const uint32_t o = SH ? px_write2(__builtin_amdgcn_perm(v1, v1 - d1, 0x05040100u), selbe, ulsb)
                              : __builtin_amdgcn_perm(v1, v1 - d1, selpack);
        // buffer stores: scalar base + 32-bit lane offset
        if constexpr (CS == 1) {
          __builtin_amdgcn_raw_buffer_store_b32(o, orsrc, 4 * lane, (int)(sx * (2 * n)), 0);
        } else {
          const int sbase = (int)(2 * ((sx / CS) * chunk_len + comp));
          __builtin_amdgcn_raw_buffer_store_b16((uint16_t)o, orsrc, 4 * CS * lane, sbase, 0);
          __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(o >> 16), orsrc, 4 * CS * lane + 2 * CS, sbase, 0);
        }
        // (kept mod 2^32 here, only the low 16 bits count; masked when the
        // loop is left)
        const uint32_t lnew = lastc + inc_last;
        if (comp) last1 = lnew;
        else last0 = lnew;
      };
      // (entry offsets by SDWA byte selects: two VOP2 operations per byte
      // instead of a bit-field extract and a shift-add, both VOP3)
      auto lookups = [&](uint32_t xl, uint32_t fs, uint4& e0, uint4& e1, uint4& e2, uint4& e3) {
        const uint4* tb = tab + 256u * fs;
        e0 = tb_entry(tb, sdwa_byte16<0>(xl));
        e1 = tb_entry(tb, sdwa_byte16<1>(xl));
        e2 = tb_entry(tb, sdwa_byte16<2>(xl));
        if constexpr (W32) e3 = tb_entry(tb, sdwa_byte16<3>(xl));
        if constexpr (!W32) e3 = make_uint4(0u, 0u, 0u, 0u);
      };

      // Ring bounds, recomputed only when the ring changes: the next window
      // start may be at most pn_limit (resident look-ahead, the header
      // inside the input), and ring_keep has something to do once the
      // window start reaches word trig_w (lim >= P + 4 here).
      // (wave-uniform; readfirstlane keeps them in SGPRs for the loop's
      // scalar tests)
      uint32_t pn_limit, trig_bits;
      auto ring_bounds = [&]() {
        pn_limit = __builtin_amdgcn_readfirstlane(min(min(lim - 4u, 32u * (fill_w - kAhead) + 31u), 1u << 31));
        trig_bits =
            __builtin_amdgcn_readfirstlane(32u * (pend ? fill_w - (kAhead + 127u) : (fill_w > 766u ? fill_w - 766u : 0u)));
      };
      // vector-memory stores per loop iteration (the previous sub-block's
      // samples), counted into vm_after only when the ring is kept
      constexpr uint32_t kStoresPerSub = TWO && CS == 2 ? 2u : 1u;
      uint32_t s_keep = s;
      ring_bounds();
      // prologue: parse sub-block s
      uint32_t Pn;
      uint32_t xh;
      uint32_t xl = seg_bits(P, xh);
      const uint32_t h = __builtin_amdgcn_readfirstlane(xl);
      uint32_t fs = fs_of(h);
      uint4 e0, e1, e2, e3;
      lookups(xl, fs, e0, e1, e2, e3);
      uint32_t unused_rider;
      uint32_t xlB, xhB;  // the window of the sub-block at Pn
      uint32_t ok =
          parse(P, xl, xh, fs, e0, e1, e2, e3, Pn, xlB, xhB, 0u, unused_rider, [](uint32_t, uint32_t) {}) & header_ok(h);
      // the look-ahead bound when the window at Pn was read (ring_keep may
      // raise pn_limit afterwards; the window read earlier stays good only
      // below the bound of its time)
      uint32_t pn_read_limit = pn_limit;
      while (ok) {
        // sub-block s at P (ends at Pn) is parsed, its pairs are in the list
        uint4 tt;
        uint32_t aprev;
        if constexpr (TWO) {
          tt = list4[lane];
          aprev = list[4 * lane - 2];
        } else {
          const uint2 t2 = list2[lane];
          tt = make_uint4(t2.x, t2.y, 0u, 0u);
          aprev = list[2 * lane - 2];
        }
        const uint32_t hB = __builtin_amdgcn_readfirstlane(xlB);
        RPP_TSTAMP(1);
        RPP_STAT(0, 1);
        uint32_t d1A, sumA, incA;
        // Does the loop go on to the sub-block at Pn?  (Computed here, tested
        // with the parse's own result after it, so that sub-block s's values
        // still ride on that parse's scan; testing it first, as scalar
        // branches, measured 5 % slower: profiles/r04_decode_ab.jsonl.)
        const uint32_t nxt = (uint32_t)(s + 1 < nsb_fast) & (uint32_t)(Pn <= pn_read_limit) & header_ok(hB);
        pn_read_limit = pn_limit;
        const uint32_t fsB = fs_of(hB);
        lookups(xlB, fsB, e0, e1, e2, e3);
        deltas(tt, aprev, fs, d1A, sumA);
        RPP_TSTAMP(2);
        uint32_t PnB, xlC, xhC;
        ok = parse(Pn, xlB, xhB, fsB, e0, e1, e2, e3, PnB, xlC, xhC, sumA, incA,
                   [&](uint32_t inc, uint32_t inc_last) { store(d1A, inc, inc_last, s); });
        ++s;
        P = Pn;
        if (!(ok & nxt)) {
          if (P > lim) status = RPP_TRUNCATED_INPUT;
          break;
        }
        Pn = PnB;
        fs = fsB;
        xlB = xlC;
        xhB = xhC;
        if (Pn >= trig_bits) {
          vm_after += (s - s_keep) * kStoresPerSub;  // (the stores since the last keep)
          s_keep = s;
          ring_keep(Pn);
          ring_bounds();
        }
        RPP_TSTAMP(15);
      }
    };
    // dispatch on the sub-block's fs class; a loop that stops at a
    // sub-block of the other class hands over to the other loop directly
    while (s < nsb_fast && status == RPP_OK && fill_w >= (P >> 5) + kAhead && P + 4 <= lim) {
      rebase();
      const uint32_t* w = ring + ((P >> 5) & kRingMask);
      const uint32_t h = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbit(w[1], w[0], P & 31u)) & 15u;
      const uint32_t s0 = s;
      // (fs 1: the fs 1-4 instance, 12 terminators per segment; a stream
      // that mixes fs 1 and 2..4 sub-blocks stays in it)
      if (bs == 2 * kWave) {
        if (h - 6u <= 2u) fast.template operator()<4, 5, 7, true>();
        else if (h - 3u <= 2u) fast.template operator()<8, 2, 4, true>();
        else if (h - 9u <= 5u) fast.template operator()<4, 8, 13, true>();
        else if (h == 2u) fast.template operator()<12, 1, 4, true>();
      } else {
        if (h - 6u <= 2u) fast.template operator()<4, 5, 7, false>();
        else if (h - 3u <= 2u) fast.template operator()<8, 2, 4, false>();
        else if (h - 9u <= 5u) fast.template operator()<4, 8, 13, false>();
        else if (h == 2u) fast.template operator()<12, 1, 4, false>();
      }
      last0 &= 0xFFFFu;
      last1 &= 0xFFFFu;
      if (s == s0) break;  // no progress: the general path takes this sub-block
    }
    if (s >= nsb || status != RPP_OK) break;
    // ---- general path: one sub-block of any kind ----
    vm_after = 0;
    const uint32_t comp = s % CS;
    const uint32_t cbase = (s / CS) * chunk_len;
    const uint32_t n = min(N - cbase, chunk_len) / CS;  // samples per component sub-block
    RPP_TSTAMP(4);
    ensure(P >> 5);
    // decode.h:60: 4-bit fs+1 header
    if (P + 4 > lim) {
      status = RPP_TRUNCATED_INPUT;
      break;
    }
    uint32_t xl, xh;
    load_x(P + kSegBits * lane, xl, xh);
    const uint32_t fsp1 = __builtin_amdgcn_readfirstlane(xl) & 15u;
    const uint32_t P4 = P + 4;
    uint16_t* dst = out + cbase + comp;  // sample i of this sub-block at dst[CS * i]
    const bool dw = CS == 1 && (((uintptr_t)dst) & 3u) == 0;
    // stores the packed stored-order samples i0 (low), i0 + 1 (high) of the
    // sub-block (i0 even)
    auto put2 = [&](uint32_t i0, uint32_t o, bool ok0, bool ok1) {
      if (dw && ok1) {
        *reinterpret_cast<uint32_t*>(dst + i0) = o;
      } else {
        if (ok0) dst[CS * i0] = (uint16_t)o;
        if (ok1) dst[CS * (i0 + 1)] = (uint16_t)(o >> 16);
      }
    };
    RPP_STAT(6, 1);
    RPP_TSTAMP(5);
    if (fsp1 == 0) {
      // decode.h:79-80: every sample = write(last)
      const uint32_t v = px_write(comp ? last1 : last0, be, ulsb) * 0x10001u;
      for (uint32_t i0 = 2 * lane; i0 < n; i0 += 2 * kWave) put2(i0, v, true, i0 + 1 < n);
      P = P4;
    } else if (fsp1 == 15) {
      // decode.h:72-77: raw stored values; last = read(last sample)
      if ((uint64_t)P4 + 16ull * n > lim) {
        status = RPP_TRUNCATED_INPUT;
        break;
      }
      for (uint32_t i0 = 2 * lane; i0 < n; i0 += 2 * kWave) {
        put2(i0, peek32(P4 + 16 * i0), true, i0 + 1 < n);
      }
      const uint32_t lv = __builtin_amdgcn_readfirstlane(px_read(peek32(P4 + 16 * (n - 1)) & 0xFFFFu, be, ulsb));
      if (comp) last1 = lv;
      else last0 = lv;
      P = P4 + 16 * n;
    } else {
      // decode.h:62-71: n Rice codes with fs = fsp1 - 1
      const uint32_t fs = fsp1 - 1;
      const uint32_t k = fsp1;
      const uint32_t fmask = (1u << fs) - 1u;
      const uint4* tb = tab + 256u * fs;
      // ---- codes [xdone, m) -> zig-zag deltas (decode.h:66-69) -> values,
      //      2 per lane (m even or m == n) ----
      uint32_t acc = comp ? last1 : last0, start = P4, xdone = 0;  // start: first bit of code xdone's unary run
      auto extract = [&](uint32_t m) {
        for (; xdone < m; xdone += 2 * kWave) {
          const uint32_t i0 = xdone + 2 * lane;
          const bool ok0 = i0 < m, ok1 = i0 + 1 < m;
          const uint2 tt = *reinterpret_cast<const uint2*>(&list[min(i0, kListDump - 2)]);
          const uint32_t t0 = tt.x, t1 = ok1 ? tt.y : t0;
          const uint32_t st0 = dpp_keep<kDppWaveShr1>(start, t1 + k);  // end of code i0 - 1
          const uint32_t r0 = peek32(t0 + 1) & fmask, r1 = peek32(t1 + 1) & fmask;
          const uint32_t df0 = ((t0 - st0) << fs) | r0, df1 = ((t1 - t0 - k) << fs) | r1;
          const uint32_t d0 = ok0 ? (df0 >> 1) ^ (0u - (df0 & 1u)) : 0u;
          const uint32_t d1 = ok1 ? (df1 >> 1) ^ (0u - (df1 & 1u)) : 0u;
          const uint32_t inc = wave_incl_sum(d0 + d1);
          const uint32_t v1 = acc + inc;  // value of sample i0 + 1 (mod 2^16)
          put2(i0, px_write2(((v1 - d1) & 0xFFFFu) | (v1 << 16), selbe, ulsb), ok0, ok1);
          acc += wave_last(inc);
          start = wave_last(t1) + k;
        }
        xdone = m;
        start = __builtin_amdgcn_readfirstlane(list[m - 1]) + k;
      };
      // ---- parse: the terminator position of code i -> list[i] ----
      // q0: first bit of the window; s0: state at q0 (4 = skip the header);
      // done: codes before the window
      uint32_t q0 = P, s0 = 4, done = 0;
      for (;;) {
        RPP_STAT(0, 1);
        const uint32_t sb = q0 + kSegBits * lane;
        // 1. byte transfer functions
        const uint4 e0 = tb[xl & 0xFFu], e1 = tb[__builtin_amdgcn_ubfe(xl, 8, 8)],
                    e2 = tb[__builtin_amdgcn_ubfe(xl, 16, 8)];
        RPP_TSTAMP(10);
        uint32_t tm, xexit;
        if (fs < 8) {
          // 2. segment map, scan along the wave, entry state
          Map8 M = comp8(Map8{e2.x, e2.y}, comp8(Map8{e1.x, e1.y}, Map8{e0.x, e0.y}));
          M = scan_step8<kDppRowShr1>(M);
          M = scan_step8<kDppRowShr2>(M);
          M = scan_step8<kDppRowShr4>(M);
          M = scan_step8<kDppRowShr8>(M);
          M = scan_step8<kDppRowBcast15, 0xA>(M);
          M = scan_step8<kDppRowBcast31, 0xC>(M);
          const Map8 X{dpp_keep<kDppWaveShr1>(kId0, M.lo), dpp_keep<kDppWaveShr1>(kId1, M.hi)};
          // 3. terminators of this lane's segment
          uint32_t sel = __builtin_amdgcn_perm(X.hi, X.lo, s0 | kSelByte0) | kSelByte0;
          const uint32_t t0 = __builtin_amdgcn_perm(e0.w, e0.z, sel);
          sel = __builtin_amdgcn_perm(e0.y, e0.x, sel) | kSelByte0;
          const uint32_t t1 = __builtin_amdgcn_perm(e1.w, e1.z, sel);
          sel = __builtin_amdgcn_perm(e1.y, e1.x, sel) | kSelByte0;
          const uint32_t t2 = __builtin_amdgcn_perm(e2.w, e2.z, sel);
          xexit = __builtin_amdgcn_perm(e2.y, e2.x, sel);
          tm = t0 | (t1 << 8) | (t2 << 16);
        } else {
          const Map16 b0{{e0.x, e0.y, kId0, kId1}}, b1{{e1.x, e1.y, kId0, kId1}}, b2{{e2.x, e2.y, kId0, kId1}};
          Map16 M = comp16(b2, comp16(b1, b0));
          M = scan_step16<kDppRowShr1>(M);
          M = scan_step16<kDppRowShr2>(M);
          M = scan_step16<kDppRowShr4>(M);
          M = scan_step16<kDppRowShr8>(M);
          M = scan_step16<kDppRowBcast15, 0xA>(M);
          M = scan_step16<kDppRowBcast31, 0xC>(M);
          const Map16 X{{dpp_keep<kDppWaveShr1>(kId0, M.w[0]), dpp_keep<kDppWaveShr1>(kId1, M.w[1]),
                         dpp_keep<kDppWaveShr1>(kId2, M.w[2]), dpp_keep<kDppWaveShr1>(kId3, M.w[3])}};
          uint32_t st = sel16(X, s0) & 0xFFu;
          uint32_t t[3];
          const uint4 ee[3] = {e0, e1, e2};
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const uint32_t sel = st | kSelByte0;
            const bool skip = st >= 8;
            t[j] = skip ? 0u : __builtin_amdgcn_perm(ee[j].w, ee[j].z, sel);
            st = skip ? st - 8 : __builtin_amdgcn_perm(ee[j].y, ee[j].x, sel);
          }
          tm = t[0] | (t[1] << 8) | (t[2] << 16);
          xexit = st;
        }
        RPP_TSTAMP(11);
        // 4. code indices: terminators -> list[done + excl + j]
        const uint32_t cnt = __builtin_popcount(tm);
        const uint32_t incl = wave_incl_sum(cnt);
        const uint32_t excl = incl - cnt;
        const uint32_t need = n - done;
        const uint32_t mine = need > excl ? min(cnt, need - excl) : 0u;
        uint32_t* lp = list + done + excl;
        for (uint32_t j = 0; __any(j < mine); ++j) {
          const uint32_t t = ffbl(tm);
          tm &= tm - 1;
          *(j < mine ? lp + j : list + kListDump) = sb + t;
        }
        RPP_TSTAMP(12);
        if (__ballot(incl >= need)) break;
        // continuation window: the sub-block is longer than kWinBits;
        // turn the codes found so far into samples first (the ring only
        // keeps the recent windows resident)
        done += wave_last(incl);
        if ((done & ~1u) > xdone) {
          lds_fence();
          extract(done & ~1u);
        }
        s0 = wave_last(xexit);
        q0 += kWinBits;
        if (q0 >= lim) {  // the open unary search would read past the input
          status = RPP_TRUNCATED_INPUT;
          break;
        }
        ensure(q0 >> 5);
        load_x(q0 + kSegBits * lane, xl, xh);
      }
      if (status != RPP_OK) break;
      lds_fence();
      extract(n);
      if (comp) last1 = acc & 0xFFFFu;
      else last0 = acc & 0xFFFFu;
      // the next sub-block starts after code n-1's remainder
      P = __builtin_amdgcn_readfirstlane(list[n - 1]) + k;
      if (P > lim) {
        status = RPP_TRUNCATED_INPUT;
        break;
      }
    }
    RPP_TSTAMP(14);
    ring_keep(P);
  }
  retire();
  if (lane == 0) p.status[b] = status;
#ifdef RPP_STATS
  if (lane == 0)
    for (int i = 0; i < 16; ++i) atomicAdd(&g_rpp_stats[i], (unsigned long long)stat_acc[i]);
#endif
}


// ===========================================================================
// DECODE, FOUR STREAMS PER WAVE (bs 16 / 32)
// ===========================================================================
// The fast loop of rpp_decode_kernel issues ~100 VALU per sub-block whatever
// its size: its window, scans and list are sized for 64 lanes, so a 16-sample
// sub-block (~130 bits) pays what a 128-sample one (~1000 bits) pays, and
// bs 16 / 32 decode is bound by that issue count.  Here a wave decodes four
// streams, one per 16-lane row: a 384-bit window per row (16 lanes x 24-bit
// segments), the same table-driven exact parse with row-local scans
// (row_shr 1/2/4/8: no row_bcast levels), so one pass over the wave's
// instructions advances four streams by one sub-block each.  Per-row state is
// row-uniform VGPRs; each row has its own LDS ring (refilled for all rows at
// once from per-lane prefetch registers), list and output.  Everything this
// path does not take -- raw or fs >= 8 sub-blocks, a sub-block that does
// not end in its 384-bit window, a read
// past the input, invalid arguments -- marks the stream kSegFallback, and the
// fused kernel's only_fallback launch that follows decodes it from the start
// (with the exact error contract).
constexpr uint32_t kRowsWaves = 4;                   // waves (16 streams) per workgroup
constexpr uint32_t kRowRing = 512;                   // ring words per row (power of two)
constexpr uint32_t kRowPad = 16;                     // ring words 0..15 mirrored after its end
constexpr uint32_t kRowChunk = 64;                   // refill unit: 16 lanes x 16 bytes
constexpr uint32_t kRowDump = 40;                    // first list pair of lanes past the sub-block
constexpr uint32_t kRowMT = 24;                      // terminators per 24-bit segment at most (fs 0: 1-bit codes)
constexpr uint32_t kRowListWords = 4 + 2 * (kRowDump + kRowMT);
constexpr uint32_t kRowWords = kRowRing + kRowPad + kRowListWords;
constexpr uint32_t kRowsLdsBytes = kTabBytes + kRowsWaves * 4 * kRowWords * 4;


// exclusive form of a row-local map scan: the map of row lanes 0..i-1
// (identity on each row's lane 0)
__device__ __forceinline__ Map8 shift8_row(Map8 m, Map8& keep) {
  asm("s_nop 1\n\t"
      "v_mov_b32_dpp %0, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_mov_b32_dpp %1, %3 row_shr:1 row_mask:0xf bank_mask:0xf"
      : "+v"(keep.lo), "+v"(keep.hi)
      : "v"(m.lo), "v"(m.hi));
  return keep;
}
__device__ __forceinline__ uint32_t row_incl_sum(uint32_t v) {
  v += dpp<kDppRowShr1>(v);
  v += dpp<kDppRowShr2>(v);
  v += dpp<kDppRowShr4>(v);
  v += dpp<kDppRowShr8>(v);
  return v;
}

// TWO: bs 32 (two codes per lane), else bs 16 (one code per lane)
template <uint32_t CS, bool SH, bool TWO>
__global__ __launch_bounds__(kWave* kRowsWaves) void rpp_decode_rows_kernel(DecParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 dsm[];
  constexpr uint32_t BS = TWO ? 32 : 16;
  const uint32_t lane = lane_id(), ri = lane & 15u, row = lane >> 4;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t b = (blockIdx.x * kRowsWaves + wv) * 4 + row;  // this row's stream
  copy_tables(dsm);
  __syncthreads();
  const uint4* tab = dsm;
  uint32_t* ring = reinterpret_cast<uint32_t*>(dsm) + kTabBytes / 4 + (wv * 4 + row) * kRowWords;
  uint32_t* list = ring + kRowRing + kRowPad + 4;
  if (ri < 4) list[(int)ri - 4] = 0u;  // pair -1 = (0, 0): a_(-1) of the deltas
  const uint32_t be = p.be, ulsb = p.ulsb;
  const uint32_t selbe = be ? 0x02030001u : 0x03020100u;
  const uint32_t selpack = be ? 0x04050001u : 0x05040100u;
  const uint32_t lane24 = kSegBits * ri;

  // ---- the row's stream (row-uniform values in every lane of the row) ----
  bool active = b < p.nblocks;
  int32_t status = rpp_internal::kSegFallback;
  uint32_t N = 0, nbytes = 0, mis = 0;
  const uint8_t* in = p.in;
  uint16_t* out = p.out;
  if (active) {
    const uint64_t n64 = p.n_samples[b], ioff = p.in_off[b], nb64 = p.in_bytes[b];
    if (n64 % CS != 0 || n64 >= rpp_internal::kSegMaxSamples || nb64 >= (UINT64_C(1) << 29)) {
      active = false;  // (the fused kernel decodes or reports it)
    } else {
      mis = (uint32_t)(ioff & 3u);
      N = (uint32_t)n64;
      nbytes = (uint32_t)nb64 + mis;
      in = p.in + (ioff - mis);
      out = p.out + p.out_off[b];
    }
  }
  const bool aligned16 = ((uintptr_t)in & 15u) == 0;
  const uint32_t lim = 8u * mis + 64u * ((nbytes - mis + 7u) >> 3);
  constexpr uint32_t chunk_len = CS * BS;
  const uint32_t nsb = active ? (N + chunk_len - 1) / chunk_len * CS : 0u;
  // this lane's 16 bytes of the row's chunk at word w (zero past the input)
  auto chunk_part = [&](uint32_t w) -> uint4 {
    const uint32_t x = w + 4 * ri;
    if (aligned16 && 4 * x + 16 <= nbytes) return *reinterpret_cast<const uint4*>(in + 4 * x);
    return make_uint4(stream_word(in, nbytes, x), stream_word(in, nbytes, x + 1), stream_word(in, nbytes, x + 2),
                      stream_word(in, nbytes, x + 3));
  };
  auto put_chunk = [&](uint32_t w, uint4 v) {  // (w: a multiple of kRowChunk)
    const uint32_t slot = (w + 4 * ri) & (kRowRing - 1);
    *reinterpret_cast<uint4*>(&ring[slot]) = v;
    if (slot < kRowPad) *reinterpret_cast<uint4*>(&ring[kRowRing + slot]) = v;
  };
  uint32_t fill_w = 0;
  put_chunk(0, chunk_part(0));
  put_chunk(kRowChunk, chunk_part(kRowChunk));
  fill_w = 2 * kRowChunk;
  uint4 pf = chunk_part(fill_w);  // the next chunk, in flight
  lds_fence();
  auto word_at = [&](uint32_t w) -> const uint32_t* { return ring + (w & (kRowRing - 1)); };

  uint32_t P = 8 * mis + 16 * CS;
  uint32_t last0 = 0, last1 = 0;
  if (active) {
    if (P > lim) active = false;
    const uint32_t* q = word_at((8 * mis) >> 5);
    const uint32_t first = __builtin_amdgcn_alignbit(q[1], q[0], (8 * mis) & 31u);
    last0 = first & 0xFFFFu;
    last1 = first >> 16;
  }
  if (active && nsb == 0) {
    active = false;
    status = RPP_OK;
  }
  // Batches whose streams code at fs >= 5 go to the one-wave kernel whole
  // (every row kSegFallback): its fs 5-7 fast loop decodes such data faster
  // than four rows per wave (configs[4] 16-bit: bs 16 174 vs 156, bs 32 343 vs
  // 292 GiB/s, profiles/r04_paths.jsonl); the rows keep low-fs batches (10-bit:
  // 130 vs 115, 242 vs 228), where the one-wave kernel needs its 12-slot
  // class.  The choice is the batch's, not the stream's: streams left to the
  // rows would run before the one-wave launch, not beside it (a per-stream
  // choice measured 82 GiB/s at bs 16 16-bit).  It is made identically by
  // every wave from the first headers of 8 streams spread over the batch.
  {
    uint32_t votes = 0;
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t sb = (uint32_t)(((uint64_t)p.nblocks * k) / 8);
      const uint64_t n64 = p.n_samples[sb], off = p.in_off[sb], nb = p.in_bytes[sb];
      if (n64 < (uint64_t)CS * BS || nb < 2u * CS + 1u) continue;  // (too short to tell)
      const uint8_t* q = p.in + off + 2u * CS;  // the first header: after the initial values
      if (((uint32_t)q[0] & 15u) - 6u <= 8u) ++votes;
    }
    if (votes >= 5) active = false;
  }
  uint32_t s = 0;  // the row's sub-block
  ScanRegs sreg;
  uint2* const list2 = reinterpret_cast<uint2*>(list);
  const uint4* const list4 = reinterpret_cast<const uint4*>(list);

  // one sub-block of every active row; MT: terminators a segment can hold
  auto step = [&]<uint32_t MT>() {
    const uint32_t q = P;
    const uint32_t* w = word_at(q >> 5);
    const uint32_t h = __builtin_amdgcn_alignbit(w[1], w[0], q & 31u) & 15u;
    const uint32_t o = lane24 + (q & 31u);
    const uint32_t oi = o >> 5;
    const uint32_t xl = __builtin_amdgcn_alignbit(w[oi + 1], w[oi], o);  // (shift o mod 32)
    const bool zero = h == 0;
    const bool rice = h - 1u <= 7u;  // fs 0..7
    const uint32_t fs = rice ? h - 1 : 1u;
    const uint32_t k = fs + 1;
    const uint32_t comp = s % CS, cbase = (s / CS) * chunk_len;
    const uint32_t n = active ? min(N - cbase, chunk_len) / CS : BS;
    // ---- parse: maps, row scan, entry states, terminators, counts ----
    const uint4* tb = tab + 256u * fs;
    const uint4 e0 = tb[xl & 0xFFu], e1 = tb[__builtin_amdgcn_ubfe(xl, 8, 8)], e2 = tb[__builtin_amdgcn_ubfe(xl, 16, 8)];
    const Map8 M01 = comp8(Map8{e1.x, e1.y}, Map8{e0.x, e0.y});
    const Map8 M = comp8(Map8{e2.x, e2.y}, M01);
    Map8 S = scan8_shr1(M, sreg.r1);
    S = scan8_shr2(S, sreg.r2);
    S = scan8_shr4(S, sreg.r4);
    S = scan8_shr8(S, sreg.r8);
    const Map8 X = shift8_row(S, sreg.w1);
    const uint32_t sel = __builtin_amdgcn_perm(X.hi, X.lo, 0xFFFFFF04u);  // state 4: skip the header
    const uint32_t a0 = __builtin_amdgcn_perm(e0.w, e0.z, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(e1.w, e1.z, __builtin_amdgcn_perm(e0.y, e0.x, sel));
    const uint32_t a2 = __builtin_amdgcn_perm(e2.w, e2.z, __builtin_amdgcn_perm(M01.hi, M01.lo, sel));
    uint32_t tm = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x0C0C0400u), 0x0C040100u);
    if (zero) tm = 0;
    const uint32_t cnt = __builtin_popcount(tm);
    const uint32_t incl = row_incl_sum(cnt);
    const uint32_t excl = incl - cnt;
    const uint64_t fin = __ballot(incl >= n);
    const uint32_t mrow = (uint32_t)(fin >> (16 * row)) & 0xFFFFu;
    const uint32_t lz = ffbl(mrow);  // the lane holding code n-1 (0xFFFFFFFF: not in the window)
    uint32_t t[MT];
#pragma unroll
    for (uint32_t j = 0; j < MT; ++j) {
      t[j] = ffbl(tm);
      tm &= tm - 1;
    }
    const uint32_t r = n - 1 - excl;  // (at lane lz: code n-1 is its terminator r)
    uint32_t tsel;
    if constexpr (MT <= 12) {
      uint32_t tp = t[0] | (t[1] << 8) | ((t[2] | (t[3] << 8)) << 16);
      if constexpr (MT > 4) {
        const uint32_t tp1 = t[4] | (t[5] << 8) | ((t[6] | (t[7] << 8)) << 16);
        if constexpr (MT > 8) {
          const uint32_t tp2 = t[8] | (t[9] << 8) | ((t[10] | (t[11] << 8)) << 16);
          tp = r < 4 ? tp : (r < 8 ? tp1 : tp2);
        } else {
          tp = r < 4 ? tp : tp1;
        }
      }
      tsel = __builtin_amdgcn_ubfe(tp, 8 * (r & 3u), 8);
    } else {
      tsel = t[0];
#pragma unroll
      for (uint32_t j = 1; j < MT; ++j) tsel = r == j ? t[j] : tsel;
    }
    const uint32_t tend = (uint32_t)__shfl((int)tsel, (int)((lane & 48u) | (lz & 15u)));
    const uint32_t Pe = zero ? q + 4 : q + kSegBits * lz + tend + k;
    const bool ok = active && (zero || (rice && mrow != 0)) && Pe <= lim;
    // ---- terminators -> (a_i, remainder) list pairs (as the fused loop) ----
    const uint32_t base = ok && !zero && cnt != 0 && excl < n ? excl : kRowDump;
    const uint32_t abase = lane24 - 4u - base * k;
    const uint32_t xr = xl >> 1;
#pragma unroll
    for (int j = (int)MT - 1; j >= 0; --j) {
      list2[base + j] = make_uint2(abase + t[j] - (uint32_t)j * k, __builtin_amdgcn_ubfe(xr, t[j], fs));
      lds_fence();
    }
    // ---- codes -> zig-zag deltas -> values -> stores ----
    uint32_t d0 = 0, d1 = 0, dsum = 0;
    if constexpr (TWO) {
      const uint4 tt = list4[ri];
      const uint32_t aprev = list[4 * ri - 2];
      const uint32_t df0 = lshl_or(tt.x - aprev, fs, tt.y), df1 = lshl_or(tt.z - tt.x, fs, tt.w);
      d0 = (df0 >> 1) ^ neg_lsb(df0);
      d1 = (df1 >> 1) ^ neg_lsb(df1);
      if (zero || 2 * ri >= n) d0 = 0;
      if (zero || 2 * ri + 1 >= n) d1 = 0;
      dsum = d0 + d1;
    } else {
      const uint2 tt = list2[ri];
      const uint32_t aprev = list[2 * ri - 2];
      const uint32_t df = lshl_or(tt.x - aprev, fs, tt.y);
      d1 = (df >> 1) ^ neg_lsb(df);
      if (zero || ri >= n) d1 = 0;
      dsum = d1;
    }
    const uint32_t inc = row_incl_sum(dsum);
    const uint32_t lastc = comp ? last1 : last0;
    const uint32_t v1 = lastc + inc;  // value of the lane's last code (mod 2^16)
    uint16_t* dst = out + cbase + comp;
    if (ok) {
      if constexpr (TWO) {
        const uint32_t v0 = v1 - d1;
        if (CS == 1 && 2 * ri + 1 < n && ((((uintptr_t)dst) & 3u) == 0)) {
          const uint32_t o2 = SH ? px_write2(__builtin_amdgcn_perm(v1, v0, 0x05040100u), selbe, ulsb)
                                 : __builtin_amdgcn_perm(v1, v0, selpack);
          *reinterpret_cast<uint32_t*>(dst + 2 * ri) = o2;
        } else {
          if (2 * ri < n) dst[CS * 2 * ri] = (uint16_t)px_write(v0 & 0xFFFFu, be, ulsb);
          if (2 * ri + 1 < n) dst[CS * (2 * ri + 1)] = (uint16_t)px_write(v1 & 0xFFFFu, be, ulsb);
        }
      } else {
        if (ri < n) dst[CS * ri] = (uint16_t)px_write(v1 & 0xFFFFu, be, ulsb);
      }
    }
    const uint32_t tot = (uint32_t)__shfl((int)inc, (int)(lane | 15u));
    if (ok) {
      const uint32_t lnew = (lastc + tot) & 0xFFFFu;
      if (comp) last1 = lnew;
      else last0 = lnew;
      P = Pe;
      if (++s == nsb) {
        active = false;
        status = RPP_OK;
      }
    } else if (active) {
      active = false;  // kSegFallback: the fused kernel takes the whole stream
    }
    lds_fence();
  };

  while (__any(active)) {
    // list slots per segment: 24 for 1-bit codes (fs 0), 12 for fs 1, 8 for
    // fs 2..4 (codes of >= 3 bits), else 4
    const uint32_t* w = word_at(P >> 5);
    const uint32_t h = __builtin_amdgcn_alignbit(w[1], w[0], P & 31u) & 15u;
    if (__any(active && h == 1u)) step.template operator()<kRowMT>();
    else if (__any(active && h == 2u)) step.template operator()<12>();
    else if (__any(active && h - 3u <= 2u)) step.template operator()<8>();
    else step.template operator()<4>();
    // ---- ring: once a row's look-ahead drops below 40 words, every row with
    //      room takes its prefetched chunk and prefetches the next ----
    if (__any(active && fill_w < (P >> 5) + 40u)) {
      const bool room = fill_w + kRowChunk <= (P >> 5) + kRowRing - 1u;
      if (room) {
        put_chunk(fill_w, pf);
        fill_w += kRowChunk;
        pf = chunk_part(fill_w);
      }
      lds_fence();
    }
  }
  if (ri == 0 && b < p.nblocks) p.status[b] = status;
}

// ===========================================================================
// DECODE, PARSE PASS (rpp_decode_batch stage 1 of 2)
// ===========================================================================
// The serial part of decoding a stream is finding where each sub-block
// starts: sub-block k+1 begins where the n-th code of sub-block k ends
// (codec.h:103-140, decode.h:42-83).  rpp_parse_kernel does only that, with
// the exact table-driven parse of rpp_decode_kernel (window map scan, count
// scan, the lane holding code n-1) and none of its value extraction, and
// records the start bit of every sub-block's header (plus the end of the last
// one) in sb_pos.  The values are then produced by rpp_extract_kernel
// (ricepp_decode2.hip) with all sub-blocks of all streams in parallel.
//
// Bit positions are relative to the 4-byte-aligned word containing the
// stream's first byte (streams may start at any byte offset): the stream's bit
// 0 is at 8 * (in_off & 3).
struct ParseParams {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint64_t* in_bytes;
  const uint64_t* n_samples;
  const uint64_t* sb_base;  // [nblocks] first sb_pos entry of stream b
  uint32_t* sb_pos;         // [sum(nsb_b + 1)] header start bits, then the end
  int32_t* status;
  uint32_t nblocks;
  uint32_t bs;
  uint32_t waves;  // waves (streams or units) per workgroup
  rpp_internal::SegView sv;  // SEG: the units of the segmented decode
  uint32_t wave_words;       // LDS words per wave (kWaveLdsWords, or more for a long-sub-block guess)
};
// Per-wave LDS of the units' parse: bs >= 256 sub-blocks are 2-8 Kib long, so
// a guess that chains kSpecSteps of them needs ~60-90 Kib of the stream
// staged: such launches run 8 waves per workgroup with twice the words each.
constexpr uint32_t kLongSbBs = 256;
__host__ __device__ constexpr uint32_t parse_wave_words(uint32_t bs) {
  return bs >= kLongSbBs ? 2 * kWaveLdsWords : kWaveLdsWords;
}

// segmented-decode parse diagnostics (rpp_parse_diag_read): cycles in the
// guess, cycles in the chain, sub-blocks parsed, units
// (8..11: the guess's lane-serial steps and wave-parallel tail: cycles,
// cycles, tail sub-blocks, tail windows)
__device__ unsigned long long g_parse_diag[16];
__device__ __forceinline__ uint64_t memtime() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// The end (next header) of the sub-block with its header at bit r of the
// staged words st (relative positions), parsed by the whole wave in 2048-bit
// windows of 32-bit lane segments with exact entry states (w32_count, byte
// maps for any fs): the first window enters after the 4-bit header, a later
// one in the state the previous window's last lane left (sub-blocks longer
// than a window: fs 11-13 with outliers, bs 256 / 512).  Returns `lim` when
// the sub-block runs past lim - 64 (the staged words' end).
__device__ __forceinline__ uint32_t seg_sb_end_wave(const uint32_t* st, const uint4* tab, uint32_t r, uint32_t bs,
                                                    uint32_t lane, const ScanRegs& sreg0, uint32_t lim) {
  const uint32_t* w = st + (r >> 5) + lane;
  uint32_t x = __builtin_amdgcn_alignbit(w[1], w[0], r & 31u);
  const uint32_t v = __builtin_amdgcn_readfirstlane(x) & 15u;
  if (v == 0) return r + 4u;
  if (v == 15) return r + 4u + 16u * bs;
  const uint4* tb = tab + 256u * (v - 1u);
  ScanRegs sreg = sreg0;  // (lane 0's entry state: the header's 4 bits, then the carried state)
  uint32_t base = r, need = bs;
  for (;;) {
    const uint4 e0 = tb[x & 0xFFu], e1 = tb[__builtin_amdgcn_ubfe(x, 8, 8)], e2 = tb[__builtin_amdgcn_ubfe(x, 16, 8)],
                e3 = tb[x >> 24];
    uint32_t tm, cnt, incl, unused, ex;
    uint64_t finm;
    w32_count(e0, e1, e2, e3, need, 0u, sreg, tm, cnt, incl, finm, unused, &ex);
    if (finm != 0) {
      const uint32_t lz = (uint32_t)__builtin_ctzll(finm);
      uint32_t t = readlane(tm, (int)lz);
      const uint32_t rr = need - 1u - (readlane(incl, (int)lz) - readlane(cnt, (int)lz));
      for (uint32_t i = 0; i < rr; ++i) t &= t - 1u;  // (scalar: the rr-th terminator of lane lz)
      return base + 32u * lz + (uint32_t)__builtin_ctz(t) + v;
    }
    need -= readlane(incl, kWave - 1);
    base += 32u * kWave;
    if (base + 32u * kWave + 64u > lim) return lim;
    sreg.ja = sreg.jb = readlane(ex, kWave - 1);
    w = st + (base >> 5) + lane;
    x = __builtin_amdgcn_alignbit(w[1], w[0], base & 31u);
  }
}

// Segmented decode, the first header of a unit (ricepp_internal.h): the
// first candidate bit c in [c_first, 4 + 16 bs) of the staged words `st`
// whose chain of kSpecSteps sub-blocks (each parsed exactly as
// decode.h:42-83 would from there) keeps its header values within a range
// (highest - lowest <= `range`: 3, or 5 in a second search when the first
// finds nothing), with zero headers only in an all-zero chain.
// ricepp output does: the Rice parameter follows the local noise level
// (Poisson data stays on one or two values, 6-bit noise with outliers on fs
// 11..13).  Random bits do not, except through the zero high bits of small
// remainders, which read as chains of small headers -- hence the zero rule (a
// CPU replay of the guess on the generator data: 6 of 60 units unstitchable
// without it, 0 with it).  A chain through other bits survives a step with
// probability ~0.35, so some guesses are wrong: the unit's own parse checks
// the same rule over the first kSpecVerify sub-blocks of its chain and asks
// for the next candidate when it fails.  Candidates a few bits before the
// true header often land on the true chain after one sub-block; the stitch
// accepts those.  Candidates are parsed lane by lane out of LDS, up to four
// chains per lane and three codes per read, 256 candidates at a time; after
// every sub-block the survivors are compacted into `list` (512 words of LDS).
// Long sub-blocks (bs 256 / 512: 2-8 Kib each) do not fit kSpecSteps of them
// in the staged words: a chain that reaches their end after kGuessMinSteps
// sub-blocks is finished (a survivor that is checked no further here).
// A wrong guess costs time, never a wrong result.
constexpr uint32_t kSlotsPerGuess = 4;  // candidates per lane of a chunk (one wave: 256-candidate chunks)
constexpr uint32_t kGuessWaveMax = 12;  // survivors below which seg_guess parses wave-parallel
constexpr uint32_t kGuessMinSteps = 4;  // sub-blocks a chain must pass before the staged words may end it
constexpr uint32_t kGuessFin = 1u << 31;  // (list word 2: the chain is finished)
// (chunk0, chunk_step: this wave's share of the chunks when
// several waves search one unit -- rpp_seg_guess_kernel -- with `best`, the
// lowest survivor any of them found so far, in LDS: a wave stops at chunks
// beyond it)
// (kSlots: candidates per lane of a chunk; the multi-wave search takes
// smaller chunks, so that its waves cover the candidates in more, shorter
// lane-serial passes)
template <uint32_t kSlots = kSlotsPerGuess>
__device__ __forceinline__ uint32_t seg_guess(const uint32_t* st, uint32_t* list, uint32_t end_rel, uint32_t bs,
                                              uint32_t lane, uint32_t c_first, uint32_t range, const uint4* tab,
                                              uint32_t chunk0 = 0, uint32_t chunk_step = 1, uint32_t* best = nullptr,
                                              uint32_t steps = rpp_internal::kSpecSteps) {
  using rpp_internal::kSegNone;
  const uint32_t maxsb = 4u + 16u * bs;
  auto peek = [&](uint32_t r) {
    const uint32_t* w = st + (r >> 5);
    return __builtin_amdgcn_alignbit(w[1], w[0], r & 31u);
  };
  uint32_t n_chunks = 0, n_steps = 0, n_slotsteps = 0;
  auto found = [&](uint32_t m) {
    if (best && lane == 0) atomicMin(best, m);
    return m;
  };
  for (uint32_t c0 = c_first + kSlots * kWave * chunk0; c0 < maxsb; c0 += kSlots * kWave * chunk_step) {
    if (best && c0 >= __builtin_amdgcn_readfirstlane(__hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
      break;
    ++n_chunks;
    const uint64_t t_serial = memtime();
    bool tailed = false;
    uint32_t cur[kSlots], org[kSlots], rng[kSlots];  // rng: lowest header | highest << 4
    bool alive[kSlots], fin[kSlots];
    uint32_t nslots = kSlots;
#pragma unroll
    for (uint32_t i = 0; i < kSlots; ++i) {
      org[i] = c0 + lane + kWave * i;
      alive[i] = org[i] < maxsb && org[i] + 4 <= end_rel;
      fin[i] = false;
      cur[i] = alive[i] ? org[i] : 0u;
      rng[i] = 0x0Fu;
    }
    for (uint32_t step = 0; step < steps; ++step) {
      ++n_steps;
      n_slotsteps += nslots;
      const bool may_finish = step >= kGuessMinSteps;
      uint32_t fsv[kSlots];
      bool rice[kSlots];
#pragma unroll
      for (uint32_t i = 0; i < kSlots; ++i) {
        rice[i] = false;
        fsv[i] = 0;
        if (i < nslots && !fin[i]) {
          const uint32_t v = peek(cur[i]) & 15u;
          const uint32_t lo = min(rng[i] & 15u, v), hi = max(rng[i] >> 4, v);
          rng[i] = lo | (hi << 4);
          const uint32_t nc = cur[i] + (v == 15 ? 4u + 16u * bs : 4u);
          // (zero sub-blocks only in an all-zero run: chains of small
          // headers through the zero high bits of small remainders are the
          // common false survivors)
          const bool inside = nc + 4 <= end_rel;
          alive[i] = alive[i] && hi - lo <= range && (lo != 0 || hi == 0) && (inside || may_finish);
          fin[i] = alive[i] && !inside;
          rice[i] = alive[i] && !fin[i] && v - 1u < 14u;
          fsv[i] = v - 1;
          cur[i] = alive[i] && !fin[i] ? nc : 0u;
        }
      }
      // the codes of the Rice sub-blocks, branch-free, up to three per LDS
      // read (a 64-bit window; codes 2 and 3 when the previous one ends in
      // the first 32 bits).  A window without a terminator (a unary run past
      // 32 bits, rare) advances 32 bits and consumes no code.
      uint32_t ncode[kSlots];
#pragma unroll
      for (uint32_t i = 0; i < kSlots; ++i) ncode[i] = 0;
      auto codes = [&](uint32_t i) {
        const uint32_t* w = st + (cur[i] >> 5);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        const uint32_t sh = cur[i] & 31u;
        const uint32_t x = __builtin_amdgcn_alignbit(w1, w0, sh), xn = __builtin_amdgcn_alignbit(w2, w1, sh);
        const uint32_t k1 = fsv[i] + 1, left = bs - ncode[i];
        const uint32_t e1 = ffbl(x) + k1;
        const uint32_t y = __builtin_amdgcn_alignbit(xn, x, e1 & 31u);
        const bool c2 = e1 < 32 && y != 0 && left >= 2;
        const uint32_t e2 = e1 + ffbl(y) + k1;
        const uint32_t z = __builtin_amdgcn_alignbit(xn, x, e2 & 31u);
        const bool c3 = c2 && e2 < 32 && z != 0 && left >= 3;
        const uint32_t e3 = e2 + ffbl(z) + k1;
        const bool zero = x == 0;
        const uint32_t adv = zero ? 32u : c3 ? e3 : c2 ? e2 : e1;
        const uint32_t n = zero ? 0u : 1u + (c2 ? 1u : 0u) + (c3 ? 1u : 0u);
        const bool r = rice[i];
        const uint32_t nxt = cur[i] + adv;
        const bool bad = r && nxt + 4 > end_rel;
        cur[i] = r ? (bad ? 0u : nxt) : cur[i];
        ncode[i] += r ? n : 0u;
        alive[i] = alive[i] && (!bad || may_finish);
        fin[i] = fin[i] || (bad && may_finish);
        rice[i] = r && !bad && ncode[i] < bs;
      };
      static_assert(kSlots == 2 || kSlots == 4, "seg_guess: 2 or 4 candidates per lane");
      for (;;) {
        bool more = rice[0] || rice[1];
        if constexpr (kSlots == 4) more = more || rice[2] || rice[3];
        if (__ballot(more) == 0) break;
        codes(0);
        if (nslots > 1) codes(1);
        if constexpr (kSlots == 4) {
          if (nslots > 2) codes(2);
          if (nslots > 3) codes(3);
        }
      }
      // compact the survivors (in candidate order) into the first slots
      uint32_t cnt = 0;
      bool all_fin = true;
#pragma unroll
      for (uint32_t i = 0; i < kSlots; ++i) {
        if (i < nslots) {
          const uint64_t m = __ballot(alive[i]);
          const uint32_t at = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (alive[i]) {
            list[2 * at] = cur[i];
            list[2 * at + 1] = org[i] | (rng[i] << 16) | (fin[i] ? kGuessFin : 0u);
          }
          cnt += (uint32_t)__builtin_popcountll(m);
          all_fin = all_fin && __ballot(alive[i] && !fin[i]) == 0;
        }
      }
      lds_fence();
      if (cnt == 0 || all_fin) break;
      // few survivors: the remaining steps survivor by survivor (candidate
      // order) with the wave-parallel parse, ~1/20 of a lane-serial step each
      // (any bs: codes past its 2048-bit window are walked one by one)
      if (cnt <= kGuessWaveMax && step + 1 < steps) {
        const uint64_t t_tail = memtime();
        uint32_t n_tail = 0;
        tailed = true;
        if (lane == 0) atomicAdd(&g_parse_diag[8], (unsigned long long)(t_tail - t_serial));
        ScanRegs sreg;
        for (uint32_t idx = 0; idx < cnt; ++idx) {
          uint32_t cur = __builtin_amdgcn_readfirstlane(list[2 * idx]);
          const uint32_t o = __builtin_amdgcn_readfirstlane(list[2 * idx + 1]);
          uint32_t lo = (o >> 16) & 15u, hi = (o >> 20) & 15u;
          bool ok = true;
          for (uint32_t st2 = step + 1; st2 < steps && ok && !(o & kGuessFin); ++st2) {
            const uint32_t* w = st + (cur >> 5);
            const uint32_t v = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbit(w[1], w[0], cur & 31u)) & 15u;
            lo = min(lo, v);
            hi = max(hi, v);
            const uint32_t nc = seg_sb_end_wave(st, tab, cur, bs, lane, sreg, end_rel);
            ++n_tail;
            // (accepting sub-blocks longer than the window as a finished chain,
            // before the walk past it existed, let false chains through random
            // bits survive: 150 reruns per 16 MiB generator stream)
            ok = hi - lo <= range && (lo != 0 || hi == 0) && nc != rpp_internal::kSegNone;
            if (ok && nc + 4 > end_rel) {  // the staged words end: finished (as above) after kGuessMinSteps
              ok = st2 >= kGuessMinSteps;
              break;
            }
            cur = nc;
          }
          if (ok) {
            if (lane == 0) {
              atomicAdd(&g_parse_diag[9], (unsigned long long)(memtime() - t_tail));
              atomicAdd(&g_parse_diag[10], (unsigned long long)n_tail);
              atomicAdd(&g_parse_diag[4], (unsigned long long)n_chunks);
              atomicAdd(&g_parse_diag[5], (unsigned long long)n_steps);
              atomicAdd(&g_parse_diag[6], (unsigned long long)n_slotsteps);
            }
            return found(o & 0xFFFFu);
          }
        }
        if (lane == 0) {
          atomicAdd(&g_parse_diag[9], (unsigned long long)(memtime() - t_tail));
          atomicAdd(&g_parse_diag[10], (unsigned long long)n_tail);
        }
#pragma unroll
        for (uint32_t i = 0; i < kSlots; ++i) alive[i] = false;  // (none survived)
        break;
      }
      nslots = (cnt + kWave - 1) / kWave;
#pragma unroll
      for (uint32_t i = 0; i < kSlots; ++i) {
        const uint32_t idx = kWave * i + lane;
        alive[i] = idx < cnt;
        cur[i] = alive[i] ? list[2 * idx] : 0u;
        const uint32_t o = alive[i] ? list[2 * idx + 1] : 0u;
        org[i] = o & 0xFFFFu;
        rng[i] = (o >> 16) & 0xFFu;
        fin[i] = (o & kGuessFin) != 0;
      }
      lds_fence();
    }
    if (!tailed && lane == 0) atomicAdd(&g_parse_diag[8], (unsigned long long)(memtime() - t_serial));
    uint32_t m = kSegNone;
#pragma unroll
    for (uint32_t i = 0; i < kSlots; ++i)
      if (alive[i]) m = min(m, org[i]);
    m = wave_min_u32(m);
    if (m != kSegNone || c0 + kSlots * kWave >= maxsb) {
      if (lane == 0) {
        atomicAdd(&g_parse_diag[4], (unsigned long long)n_chunks);
        atomicAdd(&g_parse_diag[5], (unsigned long long)n_steps);
        atomicAdd(&g_parse_diag[6], (unsigned long long)n_slotsteps);
      }
      if (m != kSegNone) return found(m);
    }
  }
  return kSegNone;
}

// One wave per unit of rpp_internal::SegView (SEG = true, the only
// instantiation launched: launch_parse_seg): a unit of a split stream
// (ricepp_internal.h) records into its position list / overshoot list; a
// stream of one unit is left to the fused kernel.  (SEG = false, one wave per
// stream writing sb_pos, was the whole-batch two-stage decode, measured
// slower than the fused kernel on every workload and removed.)
template <uint32_t CS, bool SEG>
__global__ __launch_bounds__(kWave* kDecMaxWaves) void rpp_parse_kernel(ParseParams p) {
  using namespace rpp_internal;
  extern __shared__ __attribute__((aligned(16))) uint4 dsm[];
  if constexpr (SEG) {
    // rerun passes (one wave per workgroup): most units have nothing to do;
    // leave before loading the tables
    if (p.sv.pass != 0) {
      const uint32_t w = blockIdx.x * p.waves + threadIdx.x / kWave;
      if (w >= (uint32_t)p.sv.unit_base[p.nblocks] || p.sv.ustate[kUsWords * w + kUsRerun] == kSegNone) return;
    }
  }
  {
    copy_tables(dsm);
  }
  __syncthreads();
  const uint4* tab = dsm;
  const uint32_t lane = lane_id();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint32_t ring_w = kTabBytes / 4 + wv * p.wave_words;
  asm("" : "+s"(ring_w));
  uint32_t* ring = reinterpret_cast<uint32_t*>(dsm) + ring_w;
  const uint32_t bs = p.bs;
  const uint32_t lane24 = kSegBits * lane;
  // guess staging: the wave's words but the 540 of the candidate list
  const uint32_t stage_w = p.wave_words - (kListLead + kListWords);
  // One work item: a stream (SEG = false) or a unit.  Pass 0 of the
  // segmented decode takes units from a queue (one 16-wave workgroup per CU,
  // each wave unit after unit), so that every CU parses whatever the stream
  // mix and the side-stream fused launch leave it; the other launches map one
  // item per wave.
  auto work = [&](const uint32_t wid) {
    // ---- the stream (and, SEG, the unit) of this wave ----
    uint32_t b = wid, u = 0, u0 = 0, ju = 0, nunits = 1;
    if constexpr (SEG) {
      if (wid >= p.sv.units_max) return;
      if (wid >= (uint32_t)p.sv.unit_base[p.nblocks]) return;
      u = wid;
      b = __builtin_amdgcn_readfirstlane(p.sv.unit_map[u]);
      u0 = (uint32_t)p.sv.unit_base[b];
      nunits = (uint32_t)p.sv.unit_base[b + 1] - u0;
      ju = u - u0;
      if (nunits == 1) return;  // (decoded by the fused kernel)
      if (p.sv.pass != 0 && p.sv.ustate[kUsWords * u + kUsRerun] == kSegNone) return;
    } else {
      if (b >= p.nblocks) return;  // no barrier below this point
    }
    const bool multi = SEG && nunits > 1;

    // ---- per-stream setup (wave-uniform) ----
    // SEG: the wave works in its unit's frame (ricepp_internal.h): bit 0 is
    // the unit's first bit S_abs = ju 2^L of the stream, the stream is read
    // from byte S_abs / 8 on (a multiple of 128: alignment kept), and the
    // positions it stores are relative to the unit they belong to
    const uint32_t L = p.sv.seg_log2;
    int32_t status = RPP_OK;
    uint32_t N = 0, nbytes = 0, mis = 0, lim = 0;
    uint64_t Eend64 = 0;
    const uint8_t* in = p.in;
    {
      const uint64_t n64 = p.n_samples[b];
      const uint64_t ioff = p.in_off[b];
      const uint64_t nb64 = p.in_bytes[b];
      if (!rpp_internal::seg_stream_fits(n64, nb64, CS)) {
        status = RPP_INVALID_ARGUMENT;
      } else {
        N = (uint32_t)n64;
        mis = (uint32_t)(ioff & 3u);
        in = p.in + (ioff - mis);
        // last readable bit + 1 (seg_read_limit), bytes from the aligned base
        const uint64_t lim64 = seg_read_limit(mis, nb64), nbytes64 = nb64 + mis;
        const uint64_t sabs = multi ? (uint64_t)ju << L : 0u;
        in += sabs >> 3;
        nbytes = nbytes64 > (sabs >> 3) ? (uint32_t)min<uint64_t>(nbytes64 - (sabs >> 3), kSegWinBytes) : 0u;
        lim = lim64 > sabs ? (uint32_t)min<uint64_t>(lim64 - sabs, kSegWinBits) : 0u;
        if (multi) Eend64 = seg_last_bit(mis, nb64, N, bs, CS) - sabs;
      }
    }
    uint32_t* const pos_out = multi ? nullptr : p.sb_pos + p.sb_base[b];
    const bool aligned16 = ((uintptr_t)in & 15u) == 0;
    const uint32_t chunk_len = CS * bs;
    const uint32_t nchunks = status == RPP_OK ? (N + chunk_len - 1) / chunk_len : 0u;

    // ---- SEG: the unit's region [S, E) of header positions (frame: S = 0) ----
    const bool serial = multi && p.sv.pass == 2;
    uint32_t S = 0, E = 0;
    bool last = false;
    if (multi) {
      last = ju + 1 == nunits;
      E = last ? (uint32_t)(Eend64 + 1) : 1u << L;
      // (a serial pass parses to the stream's end: one that would leave the
      // frame stops at kSegSerialEnd, past its region, and the fused kernel
      // takes the stream)
      if (serial) E = (uint32_t)min<uint64_t>(Eend64 + 1, kSegSerialEnd);
    }

    // ---- SEG: the first header of the unit ----
    // A guess: the first candidate bit in [S + c_first, S + max sub-block) whose
    // chain of kSpecSteps sub-blocks looks like ricepp output (seg_guess).
    uint32_t grange = 3;  // the header range of the guess's chains (seg_guess), which the parse checks
    auto do_guess = [&](uint32_t c_first) -> uint32_t {
      const uint32_t kStW = stage_w;
      const uint32_t w0 = S >> 5;
      for (uint32_t i = lane; i < kStW; i += kWave) ring[i] = stream_word(in, nbytes, w0 + i);
      lds_fence();
      const uint64_t tg = memtime();
      uint32_t g = seg_guess(ring, ring + kStW, min(32u * kStW - 64u, lim - S), bs, lane, c_first, 3, tab);
      grange = 3;
      // none: the true chain's headers may span a wider range for a few
      // sub-blocks; a second search with range 5 (its candidates are checked
      // by the parse with that range)
      if (g == kSegNone && c_first == 0) {
        g = seg_guess(ring, ring + kStW, min(32u * kStW - 64u, lim - S), bs, lane, 0, 5, tab);
        grange = 5;
      }
      if (lane == 0) atomicAdd(&g_parse_diag[0], (unsigned long long)(memtime() - tg));
      lds_fence();  // (the ring is refilled next)
      return g == kSegNone ? kSegNone : S + g;
    };
    uint32_t P = 8u * mis + 16u * CS;  // codec.h:81-86: the initial values
    bool guessed = false;     // (verify the chain from P)
    uint32_t P_first = 0;     // the first guess, taken unverified if no later candidate verifies
    uint32_t* const us = p.sv.ustate + kUsWords * u;
    if (multi) {
      uint32_t flags = 0;
      if (p.sv.pass != 0) {
        P = us[kUsRerun];  // a header of the exact chain (stitch)
        flags = kUfRerunDone;
      } else if (ju != 0) {
        // (searched beforehand by several waves: rpp_seg_guess_kernel)
        const uint32_t pre = __builtin_amdgcn_readfirstlane(us[kUsGuess]);
        // (a guess of rpp_seg_guess_kernel is not checked again here: a wrong
        // one costs a rerun of the unit, in parallel with any others, where a
        // one-wave re-guess would hold up the whole pass)
        P = P_first = pre == kSegNone ? do_guess(0) : pre == kSegNoGuess ? kSegNone : pre;
        guessed = pre == kSegNone;
        if (P == kSegNone) flags = kUfNoGuess;
      }
      if (lane == 0) {
        us[kUsNovr] = 0;
        us[kUsStart] = P;
        us[kUsRerun] = kSegNone;
        us[kUsFlags] = flags;
        us[kUsNpos] = 0;
      }
      if (serial)  // (the serial pass lists the positions of every later unit)
        for (uint32_t k = ju + 1 + lane; k < nunits; k += kWave) p.sv.ustate[kUsWords * (u0 + k) + kUsNpos] = 0;
      if (serial && lane == 0) {  // the stitch bookkeeping of the rest of the stream
        p.sv.uov[u - 1] = kSegOvr - 1;
        p.sv.ulo[u] = 0;  // (list indices: every position this pass lists is exact)
        for (uint32_t k = ju + 1; k < nunits; ++k) {
          p.sv.ulo[u0 + k] = 0;
          p.sv.uov[u0 + k - 1] = 0;
        }
        p.sv.uov[u0 + nunits - 1] = 0;
        p.sv.sst[b] = nunits;
      }
      if (P == kSegNone) return;
    }

    for (uint32_t attempt = 0;; ++attempt) {
      // ---- LDS ring of the stream's words (as rpp_decode_kernel) ----
      uint32_t fill_w = multi ? (P >> 5) & ~(kChunkWords - 1) : 0u;
      bool pend = false;
      auto retire = [&]() {
        if (pend) {
          vm_drain();
          fill_w += kChunkWords;
          pend = false;
        }
      };
      auto refill_sync = [&]() {
        const uint32_t w = fill_w + 4 * lane;
        uint4 v;
        if (aligned16 && 4 * w + 16 <= nbytes) {
          v = *reinterpret_cast<const uint4*>(in + 4 * w);
        } else {
          v = make_uint4(stream_word(in, nbytes, w), stream_word(in, nbytes, w + 1), stream_word(in, nbytes, w + 2),
                         stream_word(in, nbytes, w + 3));
        }
        *reinterpret_cast<uint4*>(&ring[w & kRingMask]) = v;
        if ((w & kRingMask) < kRingPad) *reinterpret_cast<uint4*>(&ring[kRingWords + (w & kRingMask)]) = v;
        fill_w += kChunkWords;
      };
      auto request = [&]() {
        if (4u * (fill_w + kChunkWords) > nbytes) return;
        const uint32_t slot = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&ring[fill_w & kRingMask]);
        const uint8_t* src = in + 4u * fill_w;
        if (aligned16) {
          glds16(src + 16u * lane, slot);
        } else {
    #pragma unroll
          for (uint32_t q = 0; q < 4; ++q) glds4(src + 256u * q + 4u * lane, slot + 256u * q);
        }
        if ((fill_w & kRingMask) == 0)
          glds4(src + 4u * lane, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&ring[kRingWords]));
        pend = true;
      };
      refill_sync();
      refill_sync();
      lds_fence();
      auto ensure = [&](uint32_t w) {
        if (fill_w < w + kAhead) {
          retire();
          while (fill_w < w + kAhead) refill_sync();
          lds_fence();
        }
      };
      auto wptr = [&](uint32_t w) -> const uint32_t* { return ring + (w & kRingMask); };
      auto load_x = [&](uint32_t sb, uint32_t& xl) {
        const uint32_t* q = wptr(sb >> 5);
        xl = __builtin_amdgcn_alignbit(q[1], q[0], sb & 31u);
      };
      auto ring_keep = [&](uint32_t q) {
        if (pend && fill_w < (q >> 5) + kAhead + 128) retire();
        if (!pend && fill_w <= (q >> 5) + 766) request();
      };

      // ---- sub-block start positions, buffered 64 at a time in one VGPR,
      //      then to sb_pos (one-unit streams) or to the list of the unit
      //      whose region holds them (the serial pass crosses units) ----
      uint32_t pbuf = 0, pcnt = 0, pstart = 0;
      uint32_t novr = 0;
      bool stop = false;
      uint32_t lk = ju;  // (SEG) the unit whose list is being written
      uint32_t loff = 0;  // (SEG) its first bit in the wave's frame: list entries are relative to it
      uint64_t lbase = multi ? p.sv.pl_base[u] : 0;
      uint32_t lcap = multi ? (uint32_t)(p.sv.pl_base[u + 1] - lbase) : 0;
      auto flush = [&]() {
        if (multi) {
          if (pstart + pcnt > lcap) {  // below 1 bit per sample: the fused kernel takes the stream
            stop = true;
            if (lane == 0) atomicOr(p.sv.sflags + b, kSfListFull);
          } else if (lane < pcnt) {
            p.sv.plist[lbase + pstart + lane] = pbuf - loff;
          }
        } else {
          if (lane < pcnt) pos_out[pstart + lane] = pbuf;
        }
        pstart += pcnt;
        pcnt = 0;
      };
      auto close_list = [&]() {
        if (lane == 0) p.sv.ustate[kUsWords * (u0 + lk) + kUsNpos] = min(pstart, lcap);
      };
      auto record = [&](uint32_t pos) {
        if (multi && pos >= E) {  // past the region: the overshoot list, or the end
          if (last || serial) {
            stop = true;
            if (lane == 0) atomicOr(p.sv.sflags + b, kSfPastRegion);
          } else {
            // (relative to the next unit's first bit, E)
            if (lane == 0 && novr < kSegOvr) p.sv.ovr[kSegOvr * u + novr] = pos - E;
            if (++novr >= kSegOvr) stop = true;
          }
          return;
        }
        if (serial && (pos >> L) != lk - ju) {  // into the next unit's region
          flush();
          close_list();
          lk = ju + (pos >> L);
          loff = (pos >> L) << L;
          lbase = p.sv.pl_base[u0 + lk];
          lcap = (uint32_t)(p.sv.pl_base[u0 + lk + 1] - lbase);
          pstart = 0;
        }
        pbuf = lane == pcnt ? pos : pbuf;
        if (++pcnt == kWave) flush();
      };

      // SEG, a guessed start: the first kSpecVerify headers of the chain must
      // keep to the guess's rule (seg_guess), else the guess was wrong and the
      // next candidate is tried.  Until then no position has left pbuf
      // (kSpecVerify < 64), so a rejected chain leaves nothing behind.
      uint32_t vcnt = guessed ? 0u : kSpecVerify, vlo = 15, vhi = 0;
      bool vfail = false;
      auto note = [&](uint32_t v) {
        if (vcnt < kSpecVerify) {
          ++vcnt;
          vlo = min(vlo, v);
          vhi = max(vhi, v);
          if (vhi - vlo > grange || (vlo == 0 && vhi != 0)) vfail = stop = true;
        }
      };

      if (!multi && status == RPP_OK && P > lim) status = RPP_TRUNCATED_INPUT;
      // a unit of a split stream parses bs-sample sub-blocks until its region
      // ends (the ragged last chunk is re-parsed by rpp_seg_tail_kernel)
      const uint32_t nsb = multi ? 0xFFFFFFFFu : nchunks * CS;
      const bool fast_bs = bs == 2 * kWave || bs == 16 || bs == 32 || bs == 64;
      // (a unit runs the window loop for any bs <= 128: it only needs the
      // sub-block's end; longer sub-blocks never end in a 1536-bit window)
      const uint32_t nsb_fast = multi ? (bs <= 2 * kWave ? 0xFFFFFFFFu : 0u) : fast_bs ? (N / chunk_len) * CS : 0u;
      ScanRegs sreg;

      uint32_t s = 0;
      const uint64_t t_chain = multi ? memtime() : 0;
      const uint32_t P0 = P;
      while (s < nsb && status == RPP_OK && !stop) {
        // ---- fast loop: Rice sub-blocks of bs codes with fs in [LO, HI] lying
        //      in one window, ring resident; the parse of sub-block s+1 is issued
        //      as soon as the end of s is known ----
        auto fast = [&]<uint32_t MT, uint32_t LO, uint32_t HI>() {
          // fs 8..13: 32-bit lane segments and jacobi entry states (w32_count)
          constexpr bool W32 = LO >= 8;
          constexpr uint32_t SB = W32 ? 32u : kSegBits;
          const uint32_t n = bs;
          auto seg_bits = [&](uint32_t q) {
            if constexpr (W32) {
              const uint32_t* w = ring + (((q >> 5) + lane) & kRingMask);
              return __builtin_amdgcn_alignbit(w[1], w[0], q & 31u);
            } else {
              const uint32_t o = lane24 + (q & 31u);
              uint32_t oi = o >> 5;
              asm("" : "+v"(oi));
              const uint32_t* w = ring + ((q >> 5) & kRingMask) + oi;
              return __builtin_amdgcn_alignbit(w[1], w[0], o);
            }
          };
          auto fs_of = [](uint32_t h) {
            uint32_t r;
            asm("s_and_b32 %0, %1, 15\n\ts_max_u32 %0, %0, %2\n\ts_min_u32 %0, %0, %3\n\ts_sub_u32 %0, %0, 1"
                : "=&s"(r)
                : "s"(h), "n"(LO + 1), "n"(HI + 1)
                : "scc");
            return r;
          };
          auto header_ok = [](uint32_t h) { return (uint32_t)((h & 15u) - (LO + 1) <= HI - LO); };
          // end (next header) of the sub-block at bit q, if it lies in the window
          auto parse = [&](uint32_t q, uint32_t fs, uint4 e0, uint4 e1, uint4 e2, uint4 e3, uint32_t& Pe) -> bool {
            const uint32_t k = fs + 1;
            uint32_t tm, cnt, incl;
            uint64_t finm;
            if constexpr (W32) {
              uint32_t unused_rider;
              w32_count(e0, e1, e2, e3, n, 0u, sreg, tm, cnt, incl, finm, unused_rider);
            } else {
              const Map8 M01 = comp8(Map8{e1.x, e1.y}, Map8{e0.x, e0.y});
              Map8 M = comp8(Map8{e2.x, e2.y}, M01);
              M = scan8_shr1(M, sreg.r1);
              M = scan8_shr2(M, sreg.r2);
              M = scan8_shr4(M, sreg.r4);
              M = scan8_shr8(M, sreg.r8);
              M = scan8_bc15(M, sreg.b15);
              M = scan8_bc31(M, sreg.b31);
              const Map8 X = shift8_wave(M, sreg.w1);
              const uint32_t sel = __builtin_amdgcn_perm(X.hi, X.lo, 0xFFFFFF04u);
              const uint32_t a0 = __builtin_amdgcn_perm(e0.w, e0.z, sel);
              const uint32_t a1 = __builtin_amdgcn_perm(e1.w, e1.z, __builtin_amdgcn_perm(e0.y, e0.x, sel));
              const uint32_t a2 = __builtin_amdgcn_perm(e2.w, e2.z, __builtin_amdgcn_perm(M01.hi, M01.lo, sel));
              tm = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x0C0C0400u), 0x0C040100u);
              cnt = __builtin_popcount(tm);
              incl = wave_incl_sum(cnt);
              finm = __ballot(incl >= n);
            }
            const uint32_t excl = incl - cnt;
            uint32_t t[MT];
    #pragma unroll
            for (uint32_t j = 0; j < MT; ++j) {
              t[j] = ffbl(tm);
              tm &= tm - 1;
            }
            const uint32_t r = n - 1 - excl;
            uint32_t tpk = t[0] | (t[1] << 8) | ((t[2] | (t[3] << 8)) << 16);
            if constexpr (MT > 4) {
              const uint32_t tpk1 = t[4] | (t[5] << 8) | ((t[6] | (t[7] << 8)) << 16);
              tpk = r < 4 ? tpk : tpk1;
            }
            if constexpr (MT > 8) {
              const uint32_t tpk2 = t[8] | (t[9] << 8) | ((t[10] | (t[11] << 8)) << 16);
              tpk = r < 8 ? tpk : tpk2;
            }
            const uint32_t tend = __builtin_amdgcn_ubfe(tpk, 8 * (r & 3u), 8);
            const uint32_t lz = (uint32_t)__builtin_ctzll(finm | (1ull << 63));
            Pe = q + SB * lz + readlane(tend, (int)lz) + k;
            return finm != 0;
          };
          auto lookups = [&](uint32_t xl, uint32_t fs, uint4& e0, uint4& e1, uint4& e2, uint4& e3) {
            const uint4* tb = tab + 256u * fs;
            e0 = tb[xl & 0xFFu];
            e1 = tb[__builtin_amdgcn_ubfe(xl, 8, 8)];
            e2 = tb[__builtin_amdgcn_ubfe(xl, 16, 8)];
            if constexpr (W32) e3 = tb[xl >> 24];
            else e3 = make_uint4(0u, 0u, 0u, 0u);
          };
          uint32_t pn_limit, trig_w;
          auto ring_bounds = [&]() {
            pn_limit = min(lim - 4u, 32u * (fill_w - kAhead) + 31u);
            trig_w = pend ? fill_w - (kAhead + 127u) : (fill_w > 766u ? fill_w - 766u : 0u);
          };
          ring_bounds();
          uint32_t Pn;
          const uint32_t xl = seg_bits(P);
          const uint32_t h = __builtin_amdgcn_readfirstlane(xl);
          uint32_t fs = fs_of(h);
          uint4 e0, e1, e2, e3;
          lookups(xl, fs, e0, e1, e2, e3);
          bool ok = parse(P, fs, e0, e1, e2, e3, Pn) && header_ok(h);
          uint32_t hc = h;  // header of the sub-block at P
          while (ok) {
            // sub-block s at P ends at Pn; parse s+1 at Pn
            const bool nxt = s + 1 < nsb_fast && Pn <= pn_limit && !stop;
            const uint32_t xlB = seg_bits(Pn);
            const uint32_t hB = __builtin_amdgcn_readfirstlane(xlB);
            const uint32_t fsB = fs_of(hB);
            lookups(xlB, fsB, e0, e1, e2, e3);
            uint32_t PnB;
            ok = parse(Pn, fsB, e0, e1, e2, e3, PnB) && header_ok(hB) && nxt;
            record(P);
            if (multi) note(hc & 15u);
            hc = hB;
            ++s;
            P = Pn;
            if (!ok) {
              if (P > lim) status = RPP_TRUNCATED_INPUT;
              break;
            }
            Pn = PnB;
            fs = fsB;
            if ((Pn >> 5) >= trig_w) {
              ring_keep(Pn);
              ring_bounds();
            }
          }
        };
        while (s < nsb_fast && status == RPP_OK && !stop && fill_w >= (P >> 5) + kAhead && P + 4 <= lim) {
          const uint32_t* w = ring + ((P >> 5) & kRingMask);
          const uint32_t h = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_alignbit(w[1], w[0], P & 31u)) & 15u;
          const uint32_t s0 = s;
          if (h - 6u <= 2u) fast.template operator()<4, 5, 7>();
          else if (h - 3u <= 2u) fast.template operator()<8, 2, 4>();
          else if (h - 9u <= 5u) fast.template operator()<4, 8, 13>();
          else if (h == 2u) fast.template operator()<12, 1, 4>();
          if (s == s0) break;  // the general path takes this sub-block
        }
        if (s >= nsb || status != RPP_OK || stop) break;
        // ---- general path: one sub-block of any kind ----
        const uint32_t cbase = (s / CS) * chunk_len;
        const uint32_t n = multi ? bs : min(N - cbase, chunk_len) / CS;
        ensure(P >> 5);
        if (multi) {  // (the end of the stream's last sub-block is a position too)
          record(P);
          if (stop) break;
        }
        if (P + 4 > lim) {  // decode.h:60: the 4-bit header
          status = RPP_TRUNCATED_INPUT;
          break;
        }
        if (!multi) record(P);
        uint32_t xl;
        load_x(P + kSegBits * lane, xl);
        const uint32_t fsp1 = __builtin_amdgcn_readfirstlane(xl) & 15u;
        if (multi) {
          note(fsp1);
          if (vfail) break;
        }
        if (fsp1 == 0) {  // decode.h:79-80
          P += 4;
        } else if (fsp1 == 15) {  // decode.h:72-77: n raw 16-bit values
          if ((uint64_t)P + 4 + 16ull * n > lim) {
            status = RPP_TRUNCATED_INPUT;
            break;
          }
          P += 4 + 16 * n;
        } else {  // decode.h:62-71: n Rice codes; find the end of code n-1
          const uint32_t fs = fsp1 - 1;
          const uint4* tb = tab + 256u * fs;
          uint32_t q0 = P, s0 = 4, done = 0;
          for (;;) {
            const uint4 e0 = tb[xl & 0xFFu], e1 = tb[__builtin_amdgcn_ubfe(xl, 8, 8)],
                        e2 = tb[__builtin_amdgcn_ubfe(xl, 16, 8)];
            uint32_t tm, xexit;
            if (fs < 8) {
              Map8 M = comp8(Map8{e2.x, e2.y}, comp8(Map8{e1.x, e1.y}, Map8{e0.x, e0.y}));
              M = scan_step8<kDppRowShr1>(M);
              M = scan_step8<kDppRowShr2>(M);
              M = scan_step8<kDppRowShr4>(M);
              M = scan_step8<kDppRowShr8>(M);
              M = scan_step8<kDppRowBcast15, 0xA>(M);
              M = scan_step8<kDppRowBcast31, 0xC>(M);
              const Map8 X{dpp_keep<kDppWaveShr1>(kId0, M.lo), dpp_keep<kDppWaveShr1>(kId1, M.hi)};
              uint32_t sel = __builtin_amdgcn_perm(X.hi, X.lo, s0 | kSelByte0) | kSelByte0;
              const uint32_t t0 = __builtin_amdgcn_perm(e0.w, e0.z, sel);
              sel = __builtin_amdgcn_perm(e0.y, e0.x, sel) | kSelByte0;
              const uint32_t t1 = __builtin_amdgcn_perm(e1.w, e1.z, sel);
              sel = __builtin_amdgcn_perm(e1.y, e1.x, sel) | kSelByte0;
              const uint32_t t2 = __builtin_amdgcn_perm(e2.w, e2.z, sel);
              xexit = __builtin_amdgcn_perm(e2.y, e2.x, sel);
              tm = t0 | (t1 << 8) | (t2 << 16);
            } else {
              const Map16 b0{{e0.x, e0.y, kId0, kId1}}, b1{{e1.x, e1.y, kId0, kId1}}, b2{{e2.x, e2.y, kId0, kId1}};
              Map16 M = comp16(b2, comp16(b1, b0));
              M = scan_step16<kDppRowShr1>(M);
              M = scan_step16<kDppRowShr2>(M);
              M = scan_step16<kDppRowShr4>(M);
              M = scan_step16<kDppRowShr8>(M);
              M = scan_step16<kDppRowBcast15, 0xA>(M);
              M = scan_step16<kDppRowBcast31, 0xC>(M);
              const Map16 X{{dpp_keep<kDppWaveShr1>(kId0, M.w[0]), dpp_keep<kDppWaveShr1>(kId1, M.w[1]),
                             dpp_keep<kDppWaveShr1>(kId2, M.w[2]), dpp_keep<kDppWaveShr1>(kId3, M.w[3])}};
              uint32_t st = sel16(X, s0) & 0xFFu;
              uint32_t t[3];
              const uint4 ee[3] = {e0, e1, e2};
    #pragma unroll
              for (int j = 0; j < 3; ++j) {
                const uint32_t sel = st | kSelByte0;
                const bool skip = st >= 8;
                t[j] = skip ? 0u : __builtin_amdgcn_perm(ee[j].w, ee[j].z, sel);
                st = skip ? st - 8 : __builtin_amdgcn_perm(ee[j].y, ee[j].x, sel);
              }
              tm = t[0] | (t[1] << 8) | (t[2] << 16);
              xexit = st;
            }
            const uint32_t cnt = __builtin_popcount(tm);
            const uint32_t incl = wave_incl_sum(cnt);
            const uint32_t need = n - done;
            const uint64_t fin = __ballot(incl >= need);
            if (fin) {
              // terminator need-1-excl of the first lane reaching need
              const uint32_t lz = (uint32_t)__builtin_ctzll(fin);
              uint32_t tmv = readlane(tm, (int)lz);
              const uint32_t r = need - 1 - (readlane(incl, (int)lz) - readlane(cnt, (int)lz));
              for (uint32_t j = 0; j < r; ++j) tmv &= tmv - 1;
              P = q0 + kSegBits * lz + (uint32_t)__builtin_ctz(tmv) + fsp1;
              break;
            }
            done += wave_last(incl);
            s0 = wave_last(xexit);
            q0 += kWinBits;
            if (q0 >= lim) {  // the open unary search would read past the input
              status = RPP_TRUNCATED_INPUT;
              break;
            }
            ensure(q0 >> 5);
            load_x(q0 + kSegBits * lane, xl);
          }
          if (status != RPP_OK) break;
          if (P > lim) {
            status = RPP_TRUNCATED_INPUT;
            break;
          }
        }
        ++s;
        ring_keep(P);
      }
      retire();
      if (vfail) {  // the guess failed its check: the next candidate that chains
        P = attempt < kGuessRetries ? do_guess(P0 - S + 1) : kSegNone;
        if (P == kSegNone) {  // none: the first guess after all (its chain may just vary more)
          P = P_first;
          guessed = false;
        }
        continue;
      }
      if (multi) {
        flush();
        close_list();
        vm_drain();
        if (lane == 0) {
          atomicAdd(&g_parse_diag[1], (unsigned long long)(memtime() - t_chain));
          atomicAdd(&g_parse_diag[2], (unsigned long long)s);
          atomicAdd(&g_parse_diag[3], 1ull);
          if (attempt) atomicAdd(&g_parse_diag[7], (unsigned long long)attempt);
          us[kUsStart] = P0;
          us[kUsNovr] = min(novr, kSegOvr);
          if (status != RPP_OK) us[kUsFlags] |= kUfTrunc;
        }
        return;
      }
      if (status == RPP_OK) record(P);  // the end of the last sub-block
      flush();
      if (lane == 0) p.status[b] = status;
      return;
    }
  };
  const bool queue = SEG && p.sv.pass == 0;
  const uint32_t items = queue ? (uint32_t)p.sv.unit_base[p.nblocks] : 0u;
  for (;;) {
    uint32_t wid = blockIdx.x * p.waves + wv;
    if (queue) {
      uint32_t w = 0;
      if (lane == 0) w = atomicAdd(p.sv.queue, 1u);
      wid = __builtin_amdgcn_readfirstlane(w);
      if (wid >= items) break;
    }
    work(wid);
    if (!queue) break;
  }
}

}  // namespace

// The first guess of every unit j >= 1 of a split stream, searched by
// kGuessWaves waves at once (one workgroup per unit): wave w takes the
// 128-candidate chunks w, w + kGuessWaves, ... of seg_guess's search and
// stops at chunks beyond the lowest survivor any wave has found (LDS); the
// unit's guess is that lowest survivor, the candidate the one-wave search
// returns.  For batches of few units (single long streams), where
// the parse's work queue would run one wave per CU and the lane-serial guess
// is most of a unit's time.
// (16 waves, one workgroup per CU: 8 waves took 1.5-5 % longer on single
// 16 MiB streams, 16 x 1 MiB and 32 MiB frames; 4 waves x 4 slots and
// 16 x 4 slower still -- tools/one_stream_prof.py, profiles/r05_guess_waves_ab.txt)
constexpr uint32_t kGuessWaves = 16;
constexpr uint32_t kGuessSlots = 2;  // candidates per lane of a chunk (128-candidate chunks)
constexpr uint32_t kGuessListWords = 2 * kGuessSlots * kWave;  // a wave's survivors: (position, origin | range)
__host__ __device__ constexpr size_t guess_lds_bytes(uint32_t bs) {
  // (the staged words of parse_wave_words, once per workgroup: 76 KiB at bs <= 128, two workgroups per CU)
  return kTabBytes + 4 * ((size_t)parse_wave_words(bs) - (kListLead + kListWords) + kGuessWaves * kGuessListWords);
}
template <uint32_t CS>
__global__ __launch_bounds__(kWave* kGuessWaves) void rpp_seg_guess_kernel(ParseParams p) {
  using namespace rpp_internal;
  extern __shared__ __attribute__((aligned(16))) uint4 dsm[];
  __shared__ uint32_t best;
  const uint32_t u = blockIdx.x;
  if (u >= p.sv.units_max || u >= (uint32_t)p.sv.unit_base[p.nblocks]) return;  // (uniform: one unit per workgroup)
  const uint32_t b = p.sv.unit_map[u];
  const uint32_t u0 = (uint32_t)p.sv.unit_base[b], nunits = (uint32_t)p.sv.unit_base[b + 1] - u0;
  const uint32_t ju = u - u0;
  if (nunits <= 1 || ju == 0) return;
  const uint64_t n64 = p.n_samples[b], ioff = p.in_off[b], nb64 = p.in_bytes[b];
  if (!rpp_internal::seg_stream_fits(n64, nb64, CS)) return;
  {
    copy_tables(dsm);
  }
  if (threadIdx.x == 0) best = kSegNone;
  __syncthreads();
  const uint4* tab = dsm;
  const uint32_t lane = lane_id();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  // the unit's staged words, shared by the waves, then a survivor list per wave
  const uint32_t stage_w = p.wave_words - (kListLead + kListWords);
  uint32_t* ring = reinterpret_cast<uint32_t*>(dsm) + kTabBytes / 4;
  uint32_t* list = ring + stage_w + wv * kGuessListWords;
  // the unit's frame (as in rpp_parse_kernel): bit 0 at its first bit
  const uint32_t mis = (uint32_t)(ioff & 3u);
  const uint64_t sabs = (uint64_t)ju << p.sv.seg_log2;
  const uint64_t lim64 = seg_read_limit(mis, nb64), nbytes64 = nb64 + mis;
  const uint32_t nbytes =
      nbytes64 > (sabs >> 3) ? (uint32_t)min<uint64_t>(nbytes64 - (sabs >> 3), kSegWinBytes) : 0u;
  const uint8_t* in = p.in + (ioff - mis) + (sabs >> 3);
  const uint32_t lim = lim64 > sabs ? (uint32_t)min<uint64_t>(lim64 - sabs, kSegWinBits) : 0u;
  const uint32_t S = 0;
  const uint32_t w0 = 0;
  for (uint32_t i = threadIdx.x; i < stage_w; i += blockDim.x) ring[i] = stream_word(in, nbytes, w0 + i);
  __syncthreads();
  const uint32_t end_rel = S < lim ? min(32u * stage_w - 64u, lim - S) : 0u;
  const uint64_t tg = memtime();
  // chains of kSpecVerify sub-blocks, the check the one-wave parse makes of a
  // guess: the lowest survivor is the candidate that parse would settle on
  // after rejecting the ones before it (the parse trusts this guess); range 5
  // when none keeps range 3; failing both, the kSpecSteps survivor the parse
  // would take unchecked in the end
  uint32_t g = kSegNone;
  for (uint32_t k = 0; k < 4 && g == kSegNone; ++k) {
    if (k != 0) {
      if (threadIdx.x == 0) best = kSegNone;
      __syncthreads();
    }
    (void)seg_guess<kGuessSlots>(ring, list, end_rel, p.bs, lane, 0, k & 1 ? 5u : 3u, tab, wv, kGuessWaves, &best,
                    k < 2 ? kSpecVerify : kSpecSteps);
    __syncthreads();
    g = best;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    p.sv.ustate[kUsWords * u + kUsGuess] = g == kSegNone ? kSegNoGuess : S + g;
    atomicAdd(&g_parse_diag[0], (unsigned long long)(memtime() - tg));
  }
}

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

uint32_t rpp_abi_version(void) { return 1; }

// diagnostics only (not in the C ABI header): the segmented parse's counters
int rpp_parse_diag_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_parse_diag), sizeof(g_parse_diag)) != hipSuccess) return RPP_HIP_ERROR;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_parse_diag), z, sizeof(z)) != hipSuccess) return RPP_HIP_ERROR;
  }
  return RPP_OK;
}

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
              cfg->unused_lsb_count, nullptr, nullptr, nullptr, nullptr, 0, 0, kEncSegChunks};
  hipLaunchKernelGGL(enc_kernel(cfg), dim3(nblocks), dim3(kWave), 0, (hipStream_t)stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

uint64_t rpp_encode_workspace_bytes(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                    uint32_t nblocks) {
  if (rpp_check_config(cfg) != RPP_OK) return 0;
  if (!enc_segmented(cfg, total_samples, max_stream_samples)) return 0;
  return enc_layout(cfg, total_samples, nblocks, nullptr).bytes;
}

int rpp_encode_batch_ws(const rpp_config* cfg, const uint16_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_n_samples, uint32_t nblocks, uint8_t* d_out, const uint64_t* d_out_offsets,
                        uint64_t* d_out_bytes, int32_t* d_status, uint64_t total_samples,
                        uint64_t max_stream_samples, void* d_workspace, uint64_t workspace_bytes, void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_n_samples || !d_out || !d_out_offsets || !d_out_bytes || !d_status)
    return RPP_INVALID_ARGUMENT;
  if (!enc_segmented(cfg, total_samples, max_stream_samples))  // no stream to split: one wave per stream
    return rpp_encode_batch(cfg, d_in, d_in_offsets, d_n_samples, nblocks, d_out, d_out_offsets, d_out_bytes,
                            d_status, stream);
  const EncWorkspace w = enc_layout(cfg, total_samples, nblocks, static_cast<uint8_t*>(d_workspace));
  if (!d_workspace || workspace_bytes < w.bytes) return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t chunk_len = cfg->block_size * cfg->component_stream_count;
  hipLaunchKernelGGL(rpp_enc_units_kernel, dim3((nblocks + 256) / 256), dim3(256), 0, s, d_n_samples, nblocks,
                     chunk_len, w.seg_chunks, w.units);
  if ((st = rpp_exclusive_scan_u64(w.units, (uint64_t)nblocks + 1, w.seg_base, s)) != RPP_OK) return st;
  hipLaunchKernelGGL(rpp_enc_unit_map_kernel, dim3((nblocks + 255) / 256), dim3(256), 0, s, w.seg_base, nblocks,
                     w.max_units, w.seg_map);
  EncParams p{d_in, d_in_offsets, d_n_samples, d_out, d_out_offsets, d_out_bytes, d_status, nblocks,
              cfg->block_size, cfg->component_stream_count, cfg->big_endian ? 1u : 0u,
              cfg->unused_lsb_count, w.seg_map, w.seg_base, w.seg_bits, w.scratch, w.slot_bytes, w.max_units,
              w.seg_chunks};
  hipLaunchKernelGGL(enc_kernel(cfg), dim3((uint32_t)w.max_units), dim3(kWave), 0, s, p);
  if (w.max_units > nblocks) {  // streams long enough to be split: place the segments
    if ((st = rpp_exclusive_scan_u64(w.seg_bits, w.max_units, w.seg_off, s)) != RPP_OK) return st;
    hipLaunchKernelGGL(rpp_enc_concat_kernel, dim3((uint32_t)w.max_units), dim3(256), 0, s, p,
                       (const uint64_t*)w.seg_off);
  }
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // extern "C"

namespace rpp_internal {

int launch_decode_fused(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, hipStream_t stream, bool only_fallback,
                        const uint64_t* d_units, uint32_t waves, bool rows) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_in_bytes || !d_out || !d_out_offsets || !d_n_samples || !d_status)
    return RPP_INVALID_ARGUMENT;
  // one stream per wave; up to kDecMaxWaves waves share one copy of the
  // transfer tables, fewer when the batch cannot fill the 256 CUs anyway
  uint32_t W = std::min<uint32_t>(kDecMaxWaves, std::max<uint32_t>(1, (nblocks + 255) / 256));
  if (waves) W = std::min<uint32_t>(kDecMaxWaves, waves);
  const size_t lds = kTabBytes + (size_t)W * kWaveLdsWords * 4;
  static void (*const kernels[4])(DecParams) = {rpp_decode_kernel<1, false>, rpp_decode_kernel<1, true>,
                                                 rpp_decode_kernel<2, false>, rpp_decode_kernel<2, true>};
  static std::once_flag attr_once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(attr_once, [] {
    const int mx = (int)(kTabBytes + (size_t)kDecMaxWaves * kWaveLdsWords * 4);
    for (auto k : kernels)
      if (attr_err == hipSuccess)
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
  });
  if (attr_err != hipSuccess) return RPP_HIP_ERROR;
  DecParams p{d_in, d_in_offsets, d_in_bytes, d_out, d_out_offsets, d_n_samples, d_status, nblocks,
              cfg->block_size, cfg->component_stream_count, cfg->big_endian ? 1u : 0u,
              cfg->unused_lsb_count, W, only_fallback ? 1u : 0u, d_units};
  const auto k = kernels[2 * (cfg->component_stream_count - 1) + (cfg->unused_lsb_count ? 1 : 0)];
  if (rows && !only_fallback && !d_units && !waves &&
      (cfg->block_size == 16 || cfg->block_size == 32)) {
    // bs 16 / 32: four streams per wave, then the fused kernel for the
    // streams it left (status kSegFallback)
    static void (*const rk[8])(DecParams) = {
        rpp_decode_rows_kernel<1, false, false>, rpp_decode_rows_kernel<1, true, false>,
        rpp_decode_rows_kernel<2, false, false>, rpp_decode_rows_kernel<2, true, false>,
        rpp_decode_rows_kernel<1, false, true>,  rpp_decode_rows_kernel<1, true, true>,
        rpp_decode_rows_kernel<2, false, true>,  rpp_decode_rows_kernel<2, true, true>};
    static std::once_flag rows_once;
    static hipError_t rows_err = hipSuccess;
    std::call_once(rows_once, [] {
      for (auto f : rk)
        if (rows_err == hipSuccess)
          rows_err = hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)kRowsLdsBytes);
    });
    if (rows_err != hipSuccess) return RPP_HIP_ERROR;
    const auto r = rk[4 * (cfg->block_size == 32 ? 1 : 0) + 2 * (cfg->component_stream_count - 1) +
                      (cfg->unused_lsb_count ? 1 : 0)];
    const uint32_t per_wg = 4 * kRowsWaves;
    hipLaunchKernelGGL(r, dim3((nblocks + per_wg - 1) / per_wg), dim3(kWave * kRowsWaves), kRowsLdsBytes, stream, p);
    p.only_fallback = 1;
  }
  hipLaunchKernelGGL(k, dim3((nblocks + W - 1) / W), dim3(kWave * W), lds, stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

// (below this many units the parse's work queue leaves wave slots idle: each
// unit's guess gets kGuessWaves waves of its own)
// (a bound on the batch's worst-case unit count.  Raised to 16384 / 65536 in
// round 6, the guess kernel made the 7.7 Gbit generator stream slower, 10.1 ->
// 10.7 ms, with 1 rerun instead of 8, and the configs[3] mix 9 % slower:
// profiles/r06_guess_bound_ab.jsonl)
constexpr uint32_t kGuessKernelMaxUnits = 2048;
int launch_seg_guess(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, const uint64_t* d_n_samples, const SegView& sv,
                     hipStream_t stream) {
  if (nblocks == 0 || sv.units_max == 0 || sv.units_max > kGuessKernelMaxUnits) return RPP_OK;
  const uint32_t wave_words = parse_wave_words(cfg->block_size);
  const size_t lds = guess_lds_bytes(cfg->block_size);
  static void (*const kernels[2])(ParseParams) = {rpp_seg_guess_kernel<1>, rpp_seg_guess_kernel<2>};
  static std::once_flag attr_once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(attr_once, [] {
    const int mx = (int)guess_lds_bytes(kLongSbBs);
    for (auto k : kernels)
      if (attr_err == hipSuccess)
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
  });
  if (attr_err != hipSuccess) return RPP_HIP_ERROR;
  ParseParams p{d_in, d_in_offsets, d_in_bytes, d_n_samples, nullptr, nullptr, nullptr, nblocks,
                cfg->block_size, kGuessWaves, sv, wave_words};
  hipLaunchKernelGGL(kernels[cfg->component_stream_count - 1], dim3(sv.units_max), dim3(kWave * kGuessWaves), lds,
                     stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

// CUs of the current device, queried once per device (callers on any thread:
// the facade's driver threads run segmented decodes concurrently)
int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

int launch_parse_seg(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, const uint64_t* d_n_samples,
                     const uint64_t* d_sb_base, uint32_t* d_sb_pos, int32_t* d_status, const SegView& sv,
                     hipStream_t stream) {
  if (nblocks == 0 || sv.units_max == 0) return RPP_OK;
  // pass 0: a work queue, one workgroup per CU; rerun passes have a few units
  // to do: one wave per workgroup, one unit each
  const int cus = device_cu_count();
  // (pass 0: as many waves per workgroup as the unit bound needs to give every
  // CU some, at most 16, so that a batch of few units still spreads over all CUs)
  const uint32_t wave_words = parse_wave_words(cfg->block_size);
  const uint32_t wmax = (uint32_t)((kTabBytes + (size_t)kDecMaxWaves * kWaveLdsWords * 4 - kTabBytes) / (wave_words * 4));
  const uint32_t W = sv.pass == 0 ? std::min<uint32_t>(wmax, std::max<uint32_t>(1, (sv.units_max + cus - 1) / cus))
                                  : 1u;
  const uint32_t grid = sv.pass == 0 ? std::min<uint32_t>((uint32_t)cus, (sv.units_max + W - 1) / W) : sv.units_max;
  const size_t lds = kTabBytes + (size_t)W * wave_words * 4;
  static void (*const kernels[2])(ParseParams) = {rpp_parse_kernel<1, true>, rpp_parse_kernel<2, true>};
  static std::once_flag attr_once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(attr_once, [] {
    const int mx = (int)(kTabBytes + (size_t)kDecMaxWaves * kWaveLdsWords * 4);
    for (auto k : kernels)
      if (attr_err == hipSuccess)
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, mx);
  });
  if (attr_err != hipSuccess) return RPP_HIP_ERROR;
  ParseParams p{d_in, d_in_offsets, d_in_bytes, d_n_samples, d_sb_base, d_sb_pos, d_status, nblocks,
                cfg->block_size, W, sv, wave_words};
  hipLaunchKernelGGL(kernels[cfg->component_stream_count - 1], dim3(grid), dim3(kWave * W), lds, stream, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // namespace rpp_internal
