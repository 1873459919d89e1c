// flac_kernels.hip -- the FLAC block codec on MI355X: RFC 9639 frames of
// interleaved PCM samples, the compute side of DwarFS's flac_block_compressor
// and flac_block_decompressor (src/compression/flac.cpp:215-403, :405-489;
// the reference runs libFLAC++ on the CPU, one block per call).
//
// Parity is unpinned: libFLAC is absent here and the reference holds no FLAC
// fixture.  The decoder accepts every frame kind RFC 9639 defines (constant,
// verbatim, fixed and LPC subframes, wasted bits, both Rice methods, escape
// partitions, the four channel assignments, any block size code), so it reads
// libFLAC's streams; the encoder writes constant, verbatim, fixed and LPC
// subframes (no escape partitions), so its streams differ from libFLAC's but
// are valid FLAC.  Checked against the CPU restatement in oracle/flac_oracle.c
// both ways (tests/test_gpu_flac.py).
//
// Encode (rpp_flac_encode): one wave per 4096-sample frame (libFLAC's level-5
// block size; flac.cpp:311-313 sets level 5 by default, :516).  The frame's
// channels are staged in LDS; per subframe source the wave finds the wasted
// low bits, the constant case, the fixed predictor order with the smallest
// sum of |residual| (orders 0-4, as libFLAC's fixed-order estimate), an LPC
// predictor (levels 3-8: libFLAC's presets' maximum order 6 / 8 / 12;
// tukey(0.5)-windowed autocorrelation, Levinson-Durbin, the order by the
// expected-bits estimate or, exhaustive, every order coded; coefficients
// quantized to libFLAC's automatic precision with error feedback), the Rice
// partition order and per-partition parameters with the fewest bits for each,
// the cheapest subframe, and for two channels the cheapest of the four
// channel assignments;
// then the codes of each row of 64 samples are placed by one wave prefix sum
// and OR-ed into an LDS bit window (MSB-first words, byte-swapped on the way
// out).  Frames go to worst-case slots, are packed back to back
// (rpp_flac_pack_kernel) and get their CRC-16 on the packed bytes
// (rpp_flac_crc_kernel: per-lane CRCs combined by GF(2) shifts).
//
// Decode (rpp_flac_decode): frames are not indexed, so every byte that starts
// a valid frame header (sync, fields, CRC-8) is a candidate
// (rpp_flac_scan_kernel); each candidate is decoded by one wave into a
// scratch slot (rpp_flac_frame_wave_kernel: Rice partitions parsed by all 64
// lanes at once, see there; rpp_flac_frame_kernel, one lane per candidate,
// takes what the wave decoder leaves) and its CRC-16 checked
// (rpp_flac_crc_kernel); the links between valid candidates are checked in
// parallel against their coded numbers (rpp_flac_link_kernel), one lane walks
// the chain of frames from the first only when a link fails
// (rpp_flac_chain_kernel), and the chained frames' samples are placed
// (rpp_flac_place_kernel).  A false candidate (random bytes passing sync,
// CRC-8 and CRC-16) is never placed: the chain only visits the positions
// where the previous frame ends.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "ricepp_amd.h"

namespace {

constexpr uint32_t kFlacBlock = 4096;   // samples per encoded frame
constexpr uint32_t kWave = 64;
constexpr uint32_t kMaxPo = 5;          // partition orders 0..5 (libFLAC level 5: -r 5)
constexpr uint32_t kWinWords = 4352;    // LDS bit window: one subframe (4096 x 33 bits) + slack
constexpr uint32_t kFlacWaveLds = 144 * 1024;  // dynamic LDS cap of the wave decoder

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o);
  return v;
}
__device__ __forceinline__ int32_t wave_min(int32_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int32_t wave_max(int32_t v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
// exclusive wave prefix sum by DPP (row_shr 1/2/4/8, row_bcast 15/31: no
// LDS round trips); total = the wave's sum
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t& total) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
  total = (uint32_t)__builtin_amdgcn_readlane(x, 63);
  return (uint32_t)x - v;
}

// ---- CRCs (RFC 9639 9.1.8 CRC-8 poly 0x07, 9.3 CRC-16 poly 0x8005; init 0) ----
__device__ __forceinline__ uint8_t crc8_byte(uint8_t c, uint8_t b) {
  c ^= b;
#pragma unroll
  for (int k = 0; k < 8; ++k) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
  return c;
}
__device__ __forceinline__ uint16_t crc16_byte(const uint16_t* tab, uint16_t c, uint8_t b) {
  return (uint16_t)((c << 8) ^ tab[(c >> 8) ^ b]);
}
// a * b mod (x^16 + 0x8005) over GF(2)
__device__ __forceinline__ uint32_t gf16_mul(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 15; i >= 0; --i) {
    r <<= 1;
    if (r & 0x10000u) r ^= 0x18005u;
    if ((b >> i) & 1u) r ^= a;
  }
  return r & 0xFFFFu;
}
// x^(8 n) mod P: a CRC advanced over n zero bytes is crc * this
__device__ __forceinline__ uint32_t gf16_xpow8(uint64_t n) {
  uint32_t result = 1, base = 0x100;  // x^8
  while (n) {
    if (n & 1) result = gf16_mul(result, base);
    base = gf16_mul(base, base);
    n >>= 1;
  }
  return result;
}

// ---- frame header fields ----
__device__ __forceinline__ uint32_t bs_code(uint32_t bs, uint32_t& extra_bits) {
  extra_bits = 0;
  if (bs == 192) return 1;
  for (uint32_t c = 2; c <= 5; ++c)
    if (bs == (576u << (c - 2))) return c;
  for (uint32_t c = 8; c <= 15; ++c)
    if (bs == (256u << (c - 8))) return c;
  extra_bits = bs <= 256 ? 8 : 16;
  return bs <= 256 ? 6 : 7;
}
__device__ __forceinline__ uint32_t ss_code(uint32_t bps) {
  switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    case 32: return 7;
    default: return 0;
  }
}
// header bytes of frame fn (channel assignment `assign`) into h[]; returns the length before the CRC-8
__device__ uint32_t build_header(uint8_t* h, uint64_t fn, uint32_t bs, uint32_t assign, uint32_t bps) {
  uint32_t extra;
  const uint32_t bc = bs_code(bs, extra);
  uint32_t n = 0;
  h[n++] = 0xFF;
  h[n++] = 0xF8;  // fixed blocking strategy
  h[n++] = (uint8_t)((bc << 4) | 10u);  // 48 kHz (flac.cpp:311)
  h[n++] = (uint8_t)((assign << 4) | (ss_code(bps) << 1));
  if (fn < 0x80) {
    h[n++] = (uint8_t)fn;
  } else {
    const int m = fn < 0x800 ? 2 : fn < 0x10000 ? 3 : fn < 0x200000 ? 4 : fn < 0x4000000 ? 5 : fn < 0x80000000ull ? 6 : 7;
    h[n++] = m == 7 ? 0xFE : (uint8_t)(((0xFF00u >> m) & 0xFFu) | (uint32_t)(fn >> (6 * (m - 1))));
    for (int i = m - 2; i >= 0; --i) h[n++] = (uint8_t)(0x80u | ((fn >> (6 * i)) & 0x3Fu));
  }
  if (extra == 8) h[n++] = (uint8_t)(bs - 1);
  if (extra == 16) {
    h[n++] = (uint8_t)((bs - 1) >> 8);
    h[n++] = (uint8_t)(bs - 1);
  }
  return n;
}

// ---- encode ----
struct FlacEncParams {
  const int32_t* x;     // interleaved samples [nsamples * channels]
  uint64_t nsamples;    // per channel
  uint32_t channels, bps;
  uint8_t* slots;       // frame slots (slot_bytes each)
  uint64_t slot_bytes;
  uint64_t* sizes;      // [frames] frame bytes (CRC-16 included)
  uint32_t frames;
  uint32_t max_lpc;     // LPC orders 1..max_lpc (0: fixed predictors only)
  uint32_t exhaustive;  // code every LPC order (else the expected-bits estimate picks one)
  uint32_t max_po;      // Rice partition orders 0..max_po (<= kMaxPo)
  // batch launches (rpp_flac_encode_batch): slot g codes frame fdesc[g] =
  // (block, frame number) of block b's samples x + in_off[b] (nsamples[b],
  // chan[b], bpsb[b]); null: one block of the fields above
  const uint2* fdesc;
  const uint64_t* in_off;
  const uint64_t* bnsamples;
  const uint32_t* chan;
  const uint32_t* bpsb;
};

constexpr uint32_t kMaxLpc = 12;  // libFLAC's presets: -l 6 (level 3), 8 (4-6), 12 (7-8)

struct SubPlan {
  uint32_t type;     // 0 constant, 1 verbatim, 2 fixed, 3 LPC
  uint32_t order, wasted, bps;  // bps: of the coded samples (after wasted bits)
  uint32_t po, method;
  uint32_t prec, shift;  // LPC: coefficient precision and shift (coefficients in EncShared::lpcq[src])
  uint64_t bits;
};

struct EncShared {
  int32_t smp[2][kFlacBlock];
  uint32_t win[kWinWords];
  uint32_t kpar[4][1u << kMaxPo];  // Rice parameters per source and partition
  unsigned long long psum[1u << kMaxPo];
  unsigned long long pbits[kMaxPo + 1][1u << kMaxPo];
  uint32_t kt[2u << kMaxPo];  // Rice parameter of partition p of order po at [2^po - 1 + p]
  uint32_t ures[kFlacBlock];  // the planned source's folded residuals (LPC analysis: the windowed samples)
  int32_t lpcq[4][kMaxLpc];   // quantized LPC coefficients of the chosen plan per source
  int32_t lpct[kMaxLpc];      // ... of the LPC order being tried
  double ac[kMaxLpc + 1];     // autocorrelation of the windowed source
  double lerr[kMaxLpc + 1];   // Levinson residual energy per order
  uint32_t bad;               // a residual of the plan being tried does not fit 32 bits
};

// source sample i: 0 / 1 = staged channel, 2 = side (L - R), 3 = mid ((L + R) >> 1)
__device__ __forceinline__ int64_t src_sample(const EncShared& sh, uint32_t src, uint32_t i) {
  const int64_t l = sh.smp[0][i];
  if (src == 0) return l;
  const int64_t r = sh.smp[1][i];
  if (src == 1) return r;
  if (src == 2) return l - r;
  return (l + r) >> 1;
}
__device__ __forceinline__ uint64_t fold(int64_t r) {
  return r >= 0 ? (uint64_t)r << 1 : ((uint64_t)(-(r + 1)) << 1) | 1u;
}
__device__ __forceinline__ int64_t fixed_res(const EncShared& sh, uint32_t src, uint32_t i, uint32_t order,
                                             uint32_t wasted) {
  auto s = [&](uint32_t j) { return src_sample(sh, src, j) >> wasted; };
  switch (order) {
    case 0: return s(i);
    case 1: return s(i) - s(i - 1);
    case 2: return s(i) - 2 * s(i - 1) + s(i - 2);
    case 3: return s(i) - 3 * s(i - 1) + 3 * s(i - 2) - s(i - 3);
    default: return s(i) - 4 * s(i - 1) + 6 * s(i - 2) - 4 * s(i - 3) + s(i - 4);
  }
}

__device__ __forceinline__ int64_t lpc_res(const EncShared& sh, const int32_t* q, uint32_t src, uint32_t i,
                                           uint32_t order, uint32_t shift, uint32_t wasted) {
  int64_t pred = 0;
  for (uint32_t j = 0; j < order; ++j) pred += (int64_t)q[j] * (src_sample(sh, src, i - 1 - j) >> wasted);
  return (src_sample(sh, src, i) >> wasted) - (pred >> shift);
}

// Rice partition plan of the residuals res(i), i in [order, bs): partition
// orders 0..po_cap that divide bs with a first partition longer than the
// predictor order, per partition k = floor(log2(mean u)); the cheapest order
// and method in bpo / bmethod, its parameters in sh.kt[2^bpo - 1 + p].
// Returns the residual's bits (its 6-bit header included), or ~0 when a
// residual does not fit 32 bits.
template <class Res>
__device__ uint64_t rice_plan(EncShared& sh, uint32_t bs, uint32_t order, uint32_t po_cap, Res&& res,
                              uint32_t& bpo, uint32_t& bmethod) {
  const uint32_t lane = lane_id();
  for (uint32_t p = lane; p < (1u << kMaxPo); p += kWave) sh.psum[p] = 0;
  for (uint32_t p = lane; p < (kMaxPo + 1) * (1u << kMaxPo); p += kWave) (&sh.pbits[0][0])[p] = 0;
  if (lane == 0) sh.bad = 0;
  __syncthreads();
  uint32_t pomax = 0;
  while (pomax < po_cap && bs % (2u << pomax) == 0 && (bs >> (pomax + 1)) > order) ++pomax;
  const uint32_t psz = bs >> pomax;  // samples per finest partition
  // (a lane's samples run through the partitions in order: its sums go to LDS
  // once per partition, not once per sample)
  {
    uint32_t cur = ~0u, q = 0, qend = psz, bad = 0;
    uint64_t acc = 0;
    for (uint32_t i = lane; i < bs; i += kWave) {
      if (i < order) continue;
      while (i >= qend) ++q, qend += psz;
      if (q != cur) {
        if (acc) atomicAdd(&sh.psum[cur], (unsigned long long)acc);
        cur = q;
        acc = 0;
      }
      const uint64_t u = fold(res(i));
      bad |= u >> 32 ? 1u : 0u;
      sh.ures[i] = (uint32_t)u;
      acc += u;
    }
    if (acc) atomicAdd(&sh.psum[cur], (unsigned long long)acc);
    if (wave_or(bad) && lane == 0) sh.bad = 1;
  }
  __syncthreads();
  if (sh.bad) return ~0ull;
  // k of every partition of every order (kt[2^po - 1 + p])
  for (uint32_t t = lane; t < (2u << pomax) - 1; t += kWave) {
    const uint32_t po = 31u - (uint32_t)__builtin_clz(t + 1), p = t + 1 - (1u << po);
    const uint32_t per = bs >> po, f = 1u << (pomax - po);
    uint64_t sum = 0;
    for (uint32_t q = p * f; q < (p + 1) * f; ++q) sum += sh.psum[q];
    const uint32_t cnt = per - (p == 0 ? order : 0u);
    const uint64_t mean = cnt ? sum / cnt : 0;
    sh.kt[t] = mean ? min(63u - (uint32_t)__builtin_clzll(mean), 30u) : 0u;
  }
  __syncthreads();
  for (uint32_t po = 0; po <= pomax; ++po) {
    const uint32_t per = bs >> po;
    const uint32_t* kt = sh.kt + (1u << po) - 1;
    uint32_t cur = ~0u, k = 0, p = 0, pend = per;
    uint64_t acc = 0;
    for (uint32_t i = lane; i < bs; i += kWave) {
      if (i < order) continue;
      while (i >= pend) ++p, pend += per;
      if (p != cur) {
        if (acc) atomicAdd(&sh.pbits[po][cur], (unsigned long long)acc);
        cur = p;
        acc = 0;
        k = kt[p];
      }
      acc += (sh.ures[i] >> k) + 1 + k;
    }
    if (acc) atomicAdd(&sh.pbits[po][cur], (unsigned long long)acc);
  }
  __syncthreads();
  uint64_t rbest = ~0ull;
  bpo = 0;
  bmethod = 0;
  for (uint32_t po = 0; po <= pomax; ++po) {
    const uint32_t np = 1u << po;
    uint64_t tot = 6;
    uint32_t kmaxp = 0;
    for (uint32_t p = 0; p < np; ++p) {
      kmaxp = max(kmaxp, sh.kt[np - 1 + p]);
      tot += sh.pbits[po][p];
    }
    const uint32_t method = kmaxp > 14 ? 1u : 0u;
    tot += (uint64_t)np * (method ? 5 : 4);
    if (tot < rbest) {
      rbest = tot;
      bpo = po;
      bmethod = method;
    }
  }
  return rbest;
}

// libFLAC's automatic quantized-coefficient precision (qlp_coeff_precision 0)
__device__ __forceinline__ uint32_t lpc_precision(uint32_t bps, uint32_t bs) {
  if (bps < 16) return max(5u, 2u + bps / 2);
  if (bps == 16) return bs <= 192 ? 7u : bs <= 384 ? 8u : bs <= 576 ? 9u : bs <= 1152 ? 10u : bs <= 2304 ? 11u
                                                                                        : bs <= 4608 ? 12u : 13u;
  return bs <= 384 ? 13u : bs <= 1152 ? 14u : 15u;
}

// Levinson-Durbin recursion over the autocorrelation ac[0..order] (in
// double, every lane alike; lane 0 writes): the residual energy of each order
// to err[1..order] (if err), and the predictor of `order` (x[i] ~ sum lp[j]
// x[i-1-j]) quantized to `prec`-bit coefficients with error feedback to q
// (if q).  Returns the quantization shift (0..15), or -1 when the
// coefficients are all zero or need a negative shift.  Out of line: its
// double arrays would otherwise stay live across the planner's LDS loops.
__device__ __noinline__ int lpc_coefs(const double* ac, uint32_t order, uint32_t prec, int32_t* q, double* err) {
  const bool w = lane_id() == 0;
  double a[kMaxLpc];
  double e = ac[0];
  for (uint32_t i = 0; i < order; ++i) {
    double r = -ac[i + 1];
    for (uint32_t j = 0; j < i; ++j) r -= a[j] * ac[i - j];
    r = e != 0.0 ? r / e : 0.0;
    a[i] = r;
    for (uint32_t j = 0; j < i / 2; ++j) {
      const double t = a[j];
      a[j] += r * a[i - 1 - j];
      a[i - 1 - j] += r * t;
    }
    if (i & 1) a[i / 2] += a[i / 2] * r;
    e *= 1.0 - r * r;
    if (err && w) err[i + 1] = e;
  }
  if (!q) return 0;
  double cmax = 0.0;
  for (uint32_t j = 0; j < order; ++j) cmax = fmax(cmax, fabs(a[j]));
  if (!(cmax > 0.0)) return -1;
  int e2;
  (void)frexp(cmax, &e2);
  int shift = (int)prec - 1 - (e2 - 1) - 1;
  if (shift > 15) shift = 15;
  if (shift < 0) return -1;
  const int32_t qmax = (1 << (prec - 1)) - 1, qmin = -(1 << (prec - 1));
  double carry = 0.0;
  for (uint32_t j = 0; j < order; ++j) {
    carry += -a[j] * (double)(1 << shift);  // (the predictor is the negated error filter)
    int32_t v = (int32_t)lround(carry);
    v = min(max(v, qmin), qmax);
    carry -= v;
    if (w) q[j] = v;
  }
  return shift;
}

// The cheapest subframe of source `src` (samples [0, bs), sbps bits each);
// its Rice parameters go to sh.kpar[src] (LPC coefficients: sh.lpcq[src])
__device__ SubPlan plan_subframe(EncShared& sh, const FlacEncParams& prm, uint32_t src, uint32_t bs,
                                 uint32_t sbps) {
  const uint32_t lane = lane_id();
  SubPlan P{};
  // wasted bits and the constant case
  uint32_t orv = 0;
  int32_t mn = INT32_MAX, mx = INT32_MIN;
  for (uint32_t i = lane; i < bs; i += kWave) {
    const int64_t v = src_sample(sh, src, i);
    orv |= (uint32_t)v;
    mn = min(mn, (int32_t)v);
    mx = max(mx, (int32_t)v);
  }
  orv = wave_or(orv);
  mn = wave_min(mn);
  mx = wave_max(mx);
  uint32_t wasted = 0;
  if (orv) {
    wasted = (uint32_t)__builtin_ctz(orv);
    if (wasted > sbps - 1) wasted = sbps - 1;
  }
  // (a side channel of 32 bits would not fit the int32 staging: never formed, bps < 32 for stereo)
  P.wasted = wasted;
  P.bps = sbps - wasted;
  const uint64_t hdr = 8 + (wasted ? wasted : 0);  // type byte (+ unary wasted count)
  if (mn == mx) {
    P.type = 0;
    P.bits = hdr + P.bps;
    return P;
  }
  P.type = 1;
  P.bits = hdr + (uint64_t)P.bps * bs;
  auto take_kpar = [&](uint32_t bpo) {
    for (uint32_t p = lane; p < (1u << bpo); p += kWave) sh.kpar[src][p] = sh.kt[(1u << bpo) - 1 + p];
    __syncthreads();
  };
  // fixed predictor order: the smallest sum of |residual| (residuals must fit 32 bits)
  uint64_t sabs[5] = {0, 0, 0, 0, 0};
  uint32_t bad = 0;
  for (uint32_t i = lane; i < bs; i += kWave) {
    // the five orders' residuals from x(i-4..i), read once: order o's is the
    // o-th backward difference
    int64_t r[5];
#pragma unroll
    for (uint32_t j = 0; j <= 4; ++j) r[j] = i >= j ? src_sample(sh, src, i - j) >> wasted : 0;
#pragma unroll
    for (uint32_t o = 1; o <= 4; ++o)
#pragma unroll
      for (uint32_t j = 4; j >= o; --j) r[j] = r[j - 1] - r[j];
    // (r[o] now holds the o-th difference at i)
#pragma unroll
    for (uint32_t o = 0; o <= 4; ++o) {
      if (i < o) continue;
      if (r[o] < INT32_MIN || r[o] > INT32_MAX) bad |= 1u << o;
      sabs[o] += (uint64_t)(r[o] < 0 ? -r[o] : r[o]);
    }
  }
  bad = wave_or(bad);
  uint32_t order = 0xFFFFFFFFu;
  uint64_t best = ~0ull;
#pragma unroll
  for (uint32_t o = 0; o <= 4; ++o) {
    const uint64_t s = wave_sum(sabs[o]);
    if (!((bad >> o) & 1u) && o < bs && s < best) {
      best = s;
      order = o;
    }
  }
  if (order != 0xFFFFFFFFu) {
    uint32_t bpo, bmethod;
    const uint64_t rb = rice_plan(sh, bs, order, prm.max_po, [&](uint32_t i) { return fixed_res(sh, src, i, order, wasted); },
                                  bpo, bmethod);
    const uint64_t fbits = rb == ~0ull ? ~0ull : hdr + (uint64_t)order * P.bps + rb;
    if (fbits < P.bits) {
      take_kpar(bpo);
      P.type = 2;
      P.order = order;
      P.po = bpo;
      P.method = bmethod;
      P.bits = fbits;
    }
  }
  // LPC (RFC 9639 9.2.6): orders 1..max_lpc below the block size
  const uint32_t maxo = min(prm.max_lpc, bs > 1 ? bs - 1 : 0u);
  if (maxo == 0) return P;
  // tukey(0.5)-windowed samples (libFLAC's default apodization) in the
  // residual scratch, their autocorrelation in double
  float* xw = reinterpret_cast<float*>(sh.ures);
  const uint32_t np = bs / 4 > 1 ? bs / 4 - 1 : 0u;  // taper length - 1 (p / 2 * bs - 1)
  for (uint32_t i = lane; i < bs; i += kWave) {
    float w = 1.f;
    if (np) {
      if (i <= np) w = 0.5f - 0.5f * cosf(3.14159265358979f * (float)i / (float)np);
      else if (i >= bs - np - 1) w = 0.5f - 0.5f * cosf(3.14159265358979f * (float)(bs - i - 1) / (float)np);
    }
    xw[i] = (float)(src_sample(sh, src, i) >> wasted) * w;
  }
  __syncthreads();
  for (uint32_t lag = 0; lag <= maxo; ++lag) {
    double a = 0.0;
    for (uint32_t i = lane + lag; i < bs; i += kWave) a += (double)xw[i] * (double)xw[i - lag];
    a = wave_sum(a);
    if (lane == 0) sh.ac[lag] = a;
  }
  __syncthreads();
  if (!(sh.ac[0] > 0.0)) return P;
  const uint32_t prec = min(lpc_precision(P.bps, bs), 15u);
  // orders to code: every one (exhaustive) or the one with the fewest
  // expected bits (libFLAC's estimate: 0.5 log2(error / 2n) bits per residual
  // plus the warm-up samples and coefficients)
  uint32_t olo = 1, ohi = maxo;
  if (!prm.exhaustive) {
    (void)lpc_coefs(sh.ac, maxo, prec, nullptr, sh.lerr);
    __syncthreads();
    double bestb = 1e300;
    uint32_t bo = 1;
    for (uint32_t o = 1; o <= maxo; ++o) {
      const double n = (double)(bs - o);
      const double e = sh.lerr[o];
      double bpr = e > 0.0 ? 0.5 * log2(0.5 * e / n) : 0.0;
      if (bpr < 0.0) bpr = 0.0;
      const double b = bpr * n + (double)o * (P.bps + prec);
      if (b < bestb) {
        bestb = b;
        bo = o;
      }
    }
    olo = ohi = bo;
  }
  for (uint32_t o = olo; o <= ohi; ++o) {
    const int shift = __builtin_amdgcn_readfirstlane(lpc_coefs(sh.ac, o, prec, sh.lpct, nullptr));
    __syncthreads();
    if (shift < 0) continue;
    uint32_t bpo, bmethod;
    const uint64_t rb = rice_plan(sh, bs, o, prm.max_po,
                                  [&](uint32_t i) { return lpc_res(sh, sh.lpct, src, i, o, (uint32_t)shift, wasted); },
                                  bpo, bmethod);
    const uint64_t lbits = rb == ~0ull ? ~0ull : hdr + (uint64_t)o * P.bps + 4 + 5 + (uint64_t)o * prec + rb;
    if (lbits < P.bits) {
      take_kpar(bpo);
      if (lane < o) sh.lpcq[src][lane] = sh.lpct[lane];
      __syncthreads();
      P.type = 3;
      P.order = o;
      P.po = bpo;
      P.method = bmethod;
      P.prec = prec;
      P.shift = (uint32_t)shift;
      P.bits = lbits;
    }
  }
  return P;
}

// ORs the low `len` (<= 33) bits of v into the MSB-first window at bit pos
__device__ __forceinline__ void put_bits(uint32_t* win, uint32_t pos, uint64_t v, uint32_t len) {
  if (!len) return;
  const uint32_t w = pos >> 5, sh = pos & 31u;
  v &= len >= 64 ? ~0ull : ((1ull << len) - 1);
  // bits [sh, sh + len) of the 64-bit pair (w, w + 1), MSB first
  const uint64_t x = v << (64u - len - sh);
  atomicOr(&win[w], (uint32_t)(x >> 32));
  if (sh + len > 32) atomicOr(&win[w + 1], (uint32_t)x);
}

// Emits subframe plan P of source src at window bit `pos`; returns the end
// (pos is absolute in the frame; the window holds its bits from wbase on)
__device__ uint32_t emit_subframe(EncShared& sh, const SubPlan& P, uint32_t src, uint32_t bs, uint32_t pos,
                                  uint32_t wbase) {
  const uint32_t lane = lane_id();
  uint32_t* const win = sh.win;
  auto put = [&](uint32_t at_abs, uint64_t v, uint32_t len) { put_bits(win, at_abs - wbase, v, len); };
  // lane 0: header, wasted count, warm-up samples, residual header
  uint32_t head = 8 + P.wasted;
  if (P.type == 0) head += P.bps;
  if (P.type == 2) head += P.order * P.bps + 6;
  if (P.type == 3) head += P.order * P.bps + 4 + 5 + P.order * P.prec + 6;
  const uint32_t per = P.type >= 2 ? bs >> P.po : bs;
  const uint32_t pbits = P.method ? 5u : 4u;
  if (lane == 0) {
    const uint32_t type6 = P.type == 0 ? 0u : P.type == 1 ? 1u : P.type == 2 ? 8u + P.order : 31u + P.order;
    put(pos, (type6 << 1) | (P.wasted ? 1u : 0u), 8);
    uint32_t q = pos + 8;
    if (P.wasted) {
      put(q + P.wasted - 1, 1, 1);  // unary wasted - 1
      q += P.wasted;
    }
    if (P.type == 0) {
      put(q, (uint64_t)(src_sample(sh, src, 0) >> P.wasted), P.bps);
    } else if (P.type >= 2) {
      for (uint32_t i = 0; i < P.order; ++i, q += P.bps)
        put(q, (uint64_t)(src_sample(sh, src, i) >> P.wasted), P.bps);
      if (P.type == 3) {  // precision - 1, shift, coefficients (two's complement)
        put(q, P.prec - 1, 4);
        put(q + 4, P.shift, 5);
        q += 9;
        for (uint32_t j = 0; j < P.order; ++j, q += P.prec) put(q, (uint64_t)(uint32_t)sh.lpcq[src][j], P.prec);
      }
      put(q, (P.method << 4) | P.po, 6);
    }
  }
  // samples in rows of 64 (lane l: sample 64 j + l, LDS reads without bank
  // conflicts); a row's codes are placed by one DPP prefix sum
  uint32_t at = pos + head;
  if (P.type == 1) {
    for (uint32_t j0 = 0; j0 < bs; j0 += kWave) {
      const uint32_t i = j0 + lane;
      if (i < bs) put(at + lane * P.bps, (uint64_t)(src_sample(sh, src, i) >> P.wasted), P.bps);
      at += min(kWave, bs - j0) * P.bps;
    }
  } else if (P.type >= 2) {
    uint32_t p = 0, pend = per;
    for (uint32_t j0 = 0; j0 < bs; j0 += kWave) {
      const uint32_t i = j0 + lane;
      uint32_t len = 0, k = 0, hb = 0;
      uint64_t u = 0;
      if (i < bs && i >= P.order) {
        while (i >= pend) ++p, pend += per;
        k = sh.kpar[src][p];
        hb = i == (p == 0 ? P.order : p * per) ? pbits : 0u;
        u = fold(P.type == 2 ? fixed_res(sh, src, i, P.order, P.wasted)
                             : lpc_res(sh, sh.lpcq[src], src, i, P.order, P.shift, P.wasted));
        len = hb + (uint32_t)(u >> k) + 1 + k;
      }
      uint32_t tot;
      uint32_t a = at + wave_excl_sum(len, tot);
      if (len) {
        if (hb) put(a, k, pbits);
        a += hb + (uint32_t)(u >> k);  // the unary zeros
        put(a, (1ull << k) | (u & ((1ull << k) - 1)), k + 1);
      }
      at += tot;
    }
  }
  __syncthreads();
  return at;
}

// Moves the window's complete words to the slot (byte order of the stream),
// keeping the partial word; win_w0 = slot word of win[0]
__device__ void flush(EncShared& sh, uint8_t* slot, uint32_t& win_w0, uint32_t pos, bool all) {
  const uint32_t lane = lane_id();
  const uint32_t end = all ? (pos + 31) >> 5 : pos >> 5;  // words to write (slot-relative)
  uint32_t* out = reinterpret_cast<uint32_t*>(slot);
  for (uint32_t w = win_w0 + lane; w < end; w += kWave) out[w] = __builtin_bswap32(sh.win[w - win_w0]);
  __syncthreads();
  if (!all) {
    const uint32_t keep = sh.win[end - win_w0];
    __syncthreads();
    for (uint32_t w = lane; w < kWinWords; w += kWave) sh.win[w] = 0;
    __syncthreads();
    if (lane == 0) sh.win[0] = keep;
    __syncthreads();
    win_w0 = end;
  }
}

__global__ __launch_bounds__(64) void rpp_flac_encode_kernel(FlacEncParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  EncShared& sh = *reinterpret_cast<EncShared*>(smem);
  const uint32_t g = blockIdx.x, lane = lane_id();
  if (g >= p.frames) return;
  // this slot's block and frame number
  uint32_t fn = g, C = p.channels, BPS = p.bps;
  uint64_t NS = p.nsamples;
  const int32_t* X = p.x;
  if (p.fdesc) {
    const uint2 d = p.fdesc[g];
    fn = d.y;
    C = p.chan[d.x];
    BPS = p.bpsb[d.x];
    NS = p.bnsamples[d.x];
    X = p.x + p.in_off[d.x];
  }
  const uint64_t f0 = (uint64_t)fn * kFlacBlock;
  const uint32_t bs = (uint32_t)min((uint64_t)kFlacBlock, NS - f0);
  uint8_t* slot = p.slots + (uint64_t)g * p.slot_bytes;
  for (uint32_t w = lane; w < kWinWords; w += kWave) sh.win[w] = 0;
  uint32_t win_w0 = 0;
  auto stage = [&](uint32_t slotc, uint32_t c) {
    for (uint32_t i = lane; i < bs; i += kWave) sh.smp[slotc][i] = X[(f0 + i) * C + c];
  };
  const bool stereo = C == 2 && BPS < 32;
  SubPlan plans[4];
  uint32_t assign = C - 1;
  if (stereo) {
    stage(0, 0);
    stage(1, 1);
    __syncthreads();
    // the four sources' plans, Rice parameters kept per source (kpar[src])
#pragma unroll
    for (uint32_t s = 0; s < 4; ++s) plans[s] = plan_subframe(sh, p, s, bs, s == 2 ? BPS + 1 : BPS);
    const uint64_t ind = plans[0].bits + plans[1].bits, ls = plans[0].bits + plans[2].bits,
                   rs = plans[2].bits + plans[1].bits, ms = plans[3].bits + plans[2].bits;
    uint64_t best = ind;
    assign = 1;
    if (ls < best) best = ls, assign = 8;
    if (rs < best) best = rs, assign = 9;
    if (ms < best) best = ms, assign = 10;
  }
  // header (byte-aligned at the slot start) and its CRC-8
  uint8_t hdr[20];
  const uint32_t hlen = build_header(hdr, fn, bs, assign, BPS);
  uint8_t c8 = 0;
  for (uint32_t i = 0; i < hlen; ++i) c8 = crc8_byte(c8, hdr[i]);
  hdr[hlen] = c8;
  if (lane == 0)
    for (uint32_t i = 0; i <= hlen; ++i) put_bits(sh.win, 8 * i, hdr[i], 8);
  __syncthreads();
  uint32_t pos = 8 * (hlen + 1);
  if (stereo) {
    const uint32_t s0 = assign == 9 ? 2u : assign == 10 ? 3u : 0u;
    const uint32_t s1 = assign == 1 ? 1u : assign == 9 ? 1u : 2u;
    // (plans[] indexed by constants only: a variable index would put it in scratch)
    auto pick = [&](uint32_t i) { return i == 0 ? plans[0] : i == 1 ? plans[1] : i == 2 ? plans[2] : plans[3]; };
    pos = emit_subframe(sh, pick(s0), s0, bs, pos, 32 * win_w0);
    flush(sh, slot, win_w0, pos, false);
    pos = emit_subframe(sh, pick(s1), s1, bs, pos, 32 * win_w0);
    flush(sh, slot, win_w0, pos, false);
  } else {
    for (uint32_t c = 0; c < C; ++c) {
      stage(0, c);
      __syncthreads();
      const SubPlan P = plan_subframe(sh, p, 0, bs, BPS);
      pos = emit_subframe(sh, P, 0, bs, pos, 32 * win_w0);
      flush(sh, slot, win_w0, pos, false);
    }
  }
  pos = (pos + 7) & ~7u;  // zero padding to a byte
  flush(sh, slot, win_w0, pos, true);
  if (lane == 0) p.sizes[g] = pos / 8 + 2;  // + CRC-16 (rpp_flac_crc_kernel)
}

// ---- pack: frames back to back ----
__global__ __launch_bounds__(256) void rpp_flac_pack_kernel(const uint8_t* slots, uint64_t slot_bytes,
                                                          const uint64_t* sizes, const uint64_t* offs,
                                                          uint8_t* out, uint32_t frames) {
  const uint32_t f = blockIdx.x;
  if (f >= frames) return;
  const uint8_t* s = slots + (uint64_t)f * slot_bytes;
  uint8_t* d = out + offs[f];
  const uint64_t n = sizes[f] - 2;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

// lens = sizes - 2 (the CRC covers the frame before it), total = offs[last] + sizes[last]
__global__ void rpp_flac_lens_kernel(const uint64_t* sizes, const uint64_t* offs, uint64_t* lens, uint64_t frames,
                                     uint64_t* total) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < frames) lens[i] = sizes[i] - 2;
  if (i == frames - 1) *total = offs[i] + sizes[i];
}

// block b's frames start at the exclusive scan's entry of its first frame
// (blocks without frames after the last frame, and entry nblocks: the total)
__global__ void rpp_flac_block_off_kernel(const uint64_t* sizes, const uint64_t* offs, uint64_t frames,
                                          const uint32_t* fstart, uint32_t nblocks, uint64_t* out_off) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = frames ? offs[frames - 1] + sizes[frames - 1] : 0;
  if (b <= nblocks) out_off[b] = fstart[b] < frames ? offs[fstart[b]] : total;
}

// ---- CRC-16 of frames: per-lane chunks combined by GF(2) shifts ----
// mode 0: write the CRC after [start, start + len); mode 1: compare with the
// two bytes there and set ok[f]
__device__ __forceinline__ void crc16_table(uint16_t* tab) {
  for (uint32_t i = lane_id(); i < 256; i += kWave) {
    uint16_t d = (uint16_t)(i << 8);
    for (int k = 0; k < 8; ++k) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : d << 1);
    tab[i] = d;
  }
  __syncthreads();
}
__device__ void crc_frames(const uint16_t* tab, const uint8_t* buf, const uint64_t* starts, const uint64_t* lens,
                           uint32_t nf, uint8_t* wbuf, uint32_t* ok) {
  const uint32_t lane = lane_id();
  for (uint32_t f = blockIdx.x; f < nf; f += gridDim.x) {
    const uint64_t len = lens[f];
    if (len == ~0ull) continue;  // (decode: a candidate that did not parse)
    const uint8_t* s = buf + starts[f];
    const uint64_t chunk = (len + kWave - 1) / kWave;
    const uint64_t lo = min(len, chunk * lane), hi = min(len, lo + chunk);
    uint16_t c = 0;
    for (uint64_t i = lo; i < hi; ++i) c = crc16_byte(tab, c, s[i]);
    // advance over the bytes after this lane's chunk
    uint32_t v = gf16_mul(c, gf16_xpow8(len - hi));
#pragma unroll
    for (int o = 32; o; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o);
    if (lane == 0) {
      if (wbuf) {
        wbuf[starts[f] + len] = (uint8_t)(v >> 8);
        wbuf[starts[f] + len + 1] = (uint8_t)v;
      } else {
        ok[f] = (s[len] == (uint8_t)(v >> 8) && s[len + 1] == (uint8_t)v) ? 1u : 0u;
      }
    }
  }
}
__global__ __launch_bounds__(64) void rpp_flac_crc_kernel(const uint8_t* buf, const uint64_t* starts,
                                                        const uint64_t* lens, uint32_t frames, uint8_t* wbuf,
                                                        uint32_t* ok, const uint32_t* count) {
  __shared__ uint16_t tab[256];
  crc16_table(tab);
  crc_frames(tab, buf, starts, lens, count ? min(*count, frames) : frames, wbuf, ok);
}

// ---- decode ----
struct FlacDecParams {
  const uint8_t* in;   // the frames (after the metadata blocks)
  uint64_t nbytes;
  uint32_t channels, bps, max_bs;
  uint64_t nsamples;   // per channel (STREAMINFO)
  uint32_t* cand_at;   // [nbytes] candidate index + 1 starting at that byte (0: none)
  uint64_t* cand_pos;  // [max_cand]
  uint32_t* cand_info; // [max_cand] block size
  uint64_t* cand_len;  // [max_cand] bytes before the CRC-16 (~0: did not parse)
  uint32_t* cand_ok;   // [max_cand] CRC-16 matches
  uint32_t* cand_redo; // [max_cand] left to the lane decoder by the wave decoder
  uint32_t redo_only;  // lane decoder: only the candidates marked in cand_redo (the wave decoder ran)
  uint32_t use_wave;   // the wave decoder takes this stream's frames (they fit its LDS)
  uint32_t wide;       // 32-bit samples: int64 scratch, the lane decoder's int64 instance
  uint32_t* ncand;     // candidates found
  uint32_t max_cand;
  void* scratch;       // [max_cand][channels][max_bs] int32 (int64 for 32-bit samples)
  uint64_t* place;     // [max_cand] first sample of the candidate's frame (kNoPlace: not on the chain)
  uint64_t* link_acc;  // [2] block sizes of the linked candidates, link failures
  int32_t* out;        // interleaved samples [nsamples * channels]
  int32_t* status;
};

// MSB-first bit reader over global memory
// (a 64-bit window of the stream, MSB-aligned: w holds the wbits bits from
// bit position pos on; refilled a byte at a time up to 57+ bits, so one
// code costs a clz and shifts instead of a loop over bytes; bytes past the
// end read as zero and consuming them sets err)
struct BitReader {
  const uint8_t* p;
  uint64_t len;  // bytes readable
  uint64_t pos;  // bit position of w's top bit
  bool err;
  uint64_t w = 0;
  uint32_t wbits = 0;
  uint64_t next = 0;  // next byte to load (pos + wbits == 8 next)
  __device__ BitReader(const uint8_t* p_, uint64_t len_, uint64_t bitpos)
      : p{p_}, len{len_}, pos{bitpos & ~7ull}, err{false}, next{bitpos >> 3} {
    fill();
    skip((uint32_t)(bitpos & 7));
  }
  // at least 33 bits in w afterwards; whole aligned dwords where it can
  // (one load per 4 bytes: a lane's loads are a dependent chain)
  __device__ void fill() {
    while (wbits <= 32) {
      uint32_t v, nb;
      if ((((uintptr_t)(p + next)) & 3u) == 0 && next + 4 <= len) {
        v = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(p + next));
        nb = 4;
      } else {
        v = (next < len ? (uint32_t)p[next] : 0u) << 24;
        nb = 1;
      }
      w |= (uint64_t)v << (32 - wbits);
      wbits += 8 * nb;
      next += nb;
    }
  }
  __device__ void skip(uint32_t n) {  // n <= wbits
    w = n >= 64 ? 0 : w << n;
    wbits -= n;
    pos += n;
    if (pos > 8 * len) err = true;
  }
  __device__ uint64_t get(uint32_t n) {  // n <= 33
    if (n == 0) return 0;
    fill();
    const uint64_t v = w >> (64 - n);
    skip(n);
    return err ? 0 : v;
  }
  __device__ int64_t get_signed(uint32_t n) {
    if (n == 0) return 0;
    uint64_t v = get(n);
    if (n < 64 && ((v >> (n - 1)) & 1u)) v |= ~0ull << n;
    return (int64_t)v;
  }
  __device__ uint64_t unary() {
    uint64_t q = 0;
    for (;;) {
      fill();
      if (w != 0) {
        const uint32_t z = (uint32_t)__builtin_clzll(w);  // < wbits: w's bits past wbits are zero
        skip(z + 1);
        return q + z;
      }
      q += wbits;
      skip(wbits);
      if (err) return q;
    }
  }
};

// Parses a frame header at byte p (no CRC-16); returns its length (0: not a
// valid header for this stream) and the block size, channel assignment and
// coded number (frame number, or first sample with variable blocking)
__device__ uint32_t parse_header(const uint8_t* in, uint64_t nbytes, uint64_t p, uint32_t channels, uint32_t bps,
                                 uint32_t& bs, uint32_t& assign, uint64_t& coded) {
  if (p + 6 > nbytes) return 0;
  const uint8_t* h = in + p;
  if (h[0] != 0xFF || (h[1] & 0xFE) != 0xF8) return 0;
  const uint32_t bc = h[2] >> 4, rc = h[2] & 15u;
  assign = h[3] >> 4;
  const uint32_t sc = (h[3] >> 1) & 7u;
  if (h[3] & 1u) return 0;
  if (bc == 0 || rc == 15 || assign > 10 || sc == 3) return 0;
  const uint32_t sizes[8] = {0, 8, 12, 0, 16, 20, 24, 32};
  if (sc && sizes[sc] != bps) return 0;
  if ((assign < 8 ? assign + 1 : 2u) != channels) return 0;
  uint64_t q = p + 4;
  // coded number
  const uint32_t b0 = in[q++];
  uint32_t more;
  if (!(b0 & 0x80)) more = 0;
  else if ((b0 & 0xE0) == 0xC0) more = 1;
  else if ((b0 & 0xF0) == 0xE0) more = 2;
  else if ((b0 & 0xF8) == 0xF0) more = 3;
  else if ((b0 & 0xFC) == 0xF8) more = 4;
  else if ((b0 & 0xFE) == 0xFC) more = 5;
  else if (b0 == 0xFE) more = 6;
  else return 0;
  if (q + more + 4 > nbytes) return 0;
  uint64_t num = more ? (b0 & (0x7Fu >> (more + 1))) : b0;
  for (uint32_t i = 0; i < more; ++i) {
    if ((in[q] & 0xC0) != 0x80) return 0;
    num = (num << 6) | (in[q++] & 0x3Fu);
  }
  coded = num;
  if (bc == 1) bs = 192;
  else if (bc <= 5) bs = 576u << (bc - 2);
  else if (bc == 6) bs = (uint32_t)in[q++] + 1;
  else if (bc == 7) {
    bs = (((uint32_t)in[q] << 8) | in[q + 1]) + 1;
    q += 2;
  } else bs = 256u << (bc - 8);
  if (rc == 12) q += 1;
  else if (rc == 13 || rc == 14) q += 2;
  if (q + 1 > nbytes) return 0;
  uint8_t c8 = 0;
  for (uint64_t i = p; i < q; ++i) c8 = crc8_byte(c8, in[i]);
  if (c8 != in[q]) return 0;
  return (uint32_t)(q + 1 - p);
}

// (every decode kernel takes the batch's table of streams, one FlacDecParams
// per stream in device memory, and works on stream blockIdx.y)
__global__ __launch_bounds__(256) void rpp_flac_scan_kernel(const FlacDecParams* tab) {
  const FlacDecParams& d = tab[blockIdx.y];
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.nbytes) return;
  uint32_t at = 0;
  if (d.in[p] == 0xFF && p + 1 < d.nbytes && (d.in[p + 1] & 0xFE) == 0xF8) {
    uint32_t bs, assign;
    uint64_t coded;
    const uint32_t hl = parse_header(d.in, d.nbytes, p, d.channels, d.bps, bs, assign, coded);
    if (hl && bs <= d.max_bs) {
      const uint32_t c = atomicAdd(d.ncand, 1u);
      if (c < d.max_cand) {
        d.cand_pos[c] = p;
        d.cand_info[c] = bs;
        at = c + 1;
      }
    }
  }
  d.cand_at[p] = at;
}

// The residual section of a subframe, each residual handed to emit(i, r)
// in sample order (i in [order, bs))
template <class Emit>
__device__ __forceinline__ bool decode_residual(BitReader& r, uint32_t bs, uint32_t order, Emit&& emit) {
  const uint32_t method = (uint32_t)r.get(2);
  if (method > 1) return false;
  const uint32_t pb = method ? 5u : 4u, esc = (1u << pb) - 1;
  const uint32_t po = (uint32_t)r.get(4);
  if (bs % (1u << po) || (bs >> po) < order) return false;
  const uint32_t per = bs >> po;
  for (uint32_t p = 0; p < (1u << po); ++p) {
    const uint32_t lo = p == 0 ? order : p * per, hi = (p + 1) * per;
    const uint32_t k = (uint32_t)r.get(pb);
    if (k == esc) {
      const uint32_t n = (uint32_t)r.get(5);
      for (uint32_t i = lo; i < hi; ++i) emit(i, r.get_signed(n));
    } else {
      for (uint32_t i = lo; i < hi; ++i) {
        const uint64_t q = r.unary();
        const uint64_t u = (q << k) | r.get(k);
        emit(i, (u & 1u) ? -(int64_t)(u >> 1) - 1 : (int64_t)(u >> 1));
        if (r.err) return false;
      }
    }
    if (r.err) return false;
  }
  return true;
}

// A lane's staged samples stg[j * 64], j < n, to dst[j]: 16-byte stores when
// the chunk is whole and aligned
template <class T>
__device__ __forceinline__ void flush_stage(T* dst, const T* stg, uint32_t n) {
  if (n == 64 && (((uintptr_t)dst) & 15u) == 0) {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (uint32_t j = 0; j < 64; j += 4)
        *reinterpret_cast<int4*>(dst + j) = make_int4(stg[j * 64], stg[(j + 1) * 64], stg[(j + 2) * 64], stg[(j + 3) * 64]);
    } else {
#pragma unroll
      for (uint32_t j = 0; j < 64; j += 2)
        *reinterpret_cast<longlong2*>(dst + j) = make_longlong2(stg[j * 64], stg[(j + 1) * 64]);
    }
  } else {
    for (uint32_t j = 0; j < n; ++j) dst[j] = stg[j * 64];
  }
}

// One subframe into dst[i], i < bs.  The prediction runs on values held in
// registers (fixed) or in this lane's LDS ring (LPC), and samples go to a
// 64-sample LDS stage flushed with vector stores: on gfx950 one counter
// orders a lane's global loads and stores, so a store per sample would make
// every bit-reader refill wait for the previous sample's write to land.
// (ring / coef / stg: this lane's column of [n][64] LDS arrays, element j at
// [j * 64]: lanes on distinct banks)
template <class T>
__device__ __forceinline__ bool decode_subframe(BitReader& r, T* dst, uint32_t bs, uint32_t sbps, int64_t* ring,
                                                int32_t* coef, T* stg) {
  if (r.get(1)) return false;
  const uint32_t type = (uint32_t)r.get(6);
  uint32_t wasted = 0;
  if (r.get(1)) wasted = (uint32_t)r.unary() + 1;
  if (r.err || wasted >= sbps) return false;
  const uint32_t b = sbps - wasted;
  auto put = [&](uint32_t i, int64_t v) {
    stg[(i & 63u) * 64] = (T)((uint64_t)v << wasted);
    if ((i & 63u) == 63u || i + 1 == bs) flush_stage(dst + (i & ~63u), stg, (i & 63u) + 1);
  };
  if (type == 0) {
    const int64_t v = r.get_signed(b);
    for (uint32_t i = 0; i < bs; ++i) put(i, v);
  } else if (type == 1) {
    for (uint32_t i = 0; i < bs; ++i) put(i, r.get_signed(b));
  } else if (type >= 8 && type <= 12) {
    const uint32_t order = type - 8;
    if (order > bs) return false;
    int64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;  // the last four samples, newest first
    for (uint32_t i = 0; i < order; ++i) {
      const int64_t v = r.get_signed(b);
      put(i, v);
      h3 = h2, h2 = h1, h1 = h0, h0 = v;
    }
    const bool ok = decode_residual(r, bs, order, [&](uint32_t i, int64_t res) {
      int64_t v;
      switch (order) {
        case 0: v = res; break;
        case 1: v = res + h0; break;
        case 2: v = res + 2 * h0 - h1; break;
        case 3: v = res + 3 * h0 - 3 * h1 + h2; break;
        default: v = res + 4 * h0 - 6 * h1 + 4 * h2 - h3; break;
      }
      put(i, v);
      h3 = h2, h2 = h1, h1 = h0, h0 = v;
    });
    if (!ok) return false;
  } else if (type >= 32) {
    const uint32_t order = type - 31;
    if (order > bs) return false;
    for (uint32_t i = 0; i < order; ++i) {
      const int64_t v = r.get_signed(b);
      put(i, v);
      ring[(i & 31u) * 64] = v;
    }
    const uint32_t prec = (uint32_t)r.get(4) + 1;
    if (prec == 16) return false;
    const int32_t shift = (int32_t)r.get_signed(5);
    if (shift < 0) return false;
    for (uint32_t j = 0; j < order; ++j) coef[j * 64] = (int32_t)r.get_signed(prec);
    if (r.err) return false;
    const bool ok = decode_residual(r, bs, order, [&](uint32_t i, int64_t res) {
      int64_t acc = 0;
      for (uint32_t j = 0; j < order; ++j) acc += (int64_t)coef[j * 64] * ring[((i - 1 - j) & 31u) * 64];
      const int64_t v = res + (acc >> shift);
      put(i, v);
      ring[(i & 31u) * 64] = v;
    });
    if (!ok) return false;
  } else {
    return false;
  }
  return !r.err;
}

// The lane decoder (rpp_flac_frame_kernel): one lane per candidate, each subframe into the candidate's scratch slot,
// planar [channel][max_bs] (T: int32, or int64 for 32-bit samples, whose side
// channel has 33 bits); cand_len = bytes before the CRC-16.  Inter-channel
// decorrelation and interleaving are left to rpp_flac_place_kernel.
template <class T>
__global__ __launch_bounds__(64) void rpp_flac_frame_kernel(const FlacDecParams* tab) {
  __shared__ int64_t rings[32][64];  // each lane's last 32 samples (LPC), lane-minor
  __shared__ int32_t coefs[32][64];  // each lane's LPC coefficients
  __shared__ T stage[64][64];        // each lane's next 64 output samples
  const FlacDecParams& d = tab[blockIdx.y];
  if ((d.wide != 0) != (sizeof(T) == 8)) return;  // (the other instance's streams)
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nc = min(*d.ncand, d.max_cand);
  if (c >= nc || (d.redo_only && !d.cand_redo[c])) return;
  d.cand_len[c] = ~0ull;
  const uint64_t p = d.cand_pos[c];
  uint32_t bs, assign;
  uint64_t coded;
  const uint32_t hl = parse_header(d.in, d.nbytes, p, d.channels, d.bps, bs, assign, coded);
  if (!hl) return;
  const uint32_t C = d.channels;
  T* s = static_cast<T*>(d.scratch) + (uint64_t)c * d.max_bs * C;
  BitReader r(d.in + p, d.nbytes - p, 8ull * hl);
  for (uint32_t ch = 0; ch < C; ++ch) {
    uint32_t sb = d.bps;
    if ((assign == 8 && ch == 1) || (assign == 9 && ch == 0) || (assign == 10 && ch == 1)) sb = d.bps + 1;
    if (!decode_subframe(r, s + (uint64_t)ch * d.max_bs, bs, sb, &rings[0][threadIdx.x], &coefs[0][threadIdx.x],
                         &stage[0][threadIdx.x]))
      return;
  }
  const uint64_t end = ((r.pos + 7) >> 3);
  if (end + 2 > d.nbytes - p) return;
  d.cand_len[c] = end;
}

// ---- the wave decoder: one wave per candidate frame ----
// The frame's bits pass through an LDS window of kFWin big-endian words.  A
// Rice partition (n codes, parameter k) is decoded by all 64 lanes at once:
// lane l takes the 32-bit segment l words after the partition's current
// position and parses it speculatively from its first bit; a lane's true
// entry is the previous lane's exit, so the lanes re-parse until every entry
// agrees (a parse that already visited the true entry needs no re-parse:
// parses that meet continue identically), which Rice codes reach within a
// few codes.  A wave prefix sum over the lanes' code counts then gives each
// code its sample index.  Residuals, warm-up and verbatim samples go to LDS
// ([channel][max_bs] int32); then fixed predictors run as wave prefix sums,
// lane ch runs channel ch's LPC predictor over its column, and the wave
// writes the planar slot.
// Anything this path does not take (32-bit samples, a block too large for
// LDS, a code longer than the window's look-ahead, a residual or sample
// beyond 32 bits) is marked in cand_redo and left to the lane decoder.
constexpr uint32_t kFWin = 512;   // LDS window words
constexpr uint32_t kFLook = 64;   // words a round keeps past its 64 lane segments
constexpr uint64_t kInf = ~0ull;

struct FWin {
  const uint8_t* base;  // the stream, aligned down to a word
  uint64_t lim;         // bytes readable from base
  uint32_t* w;          // LDS: kFWin + 2 words
  uint64_t W;           // word index of w[0] (kInf: none yet)
};

__device__ __forceinline__ uint32_t load_be_word(const FWin& f, uint64_t wi) {
  const uint64_t b = 4 * wi;
  if (b + 4 <= f.lim) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(f.base + b));
  uint32_t v = 0;
  for (uint32_t j = 0; j < 4; ++j) v = (v << 8) | (b + j < f.lim ? (uint32_t)f.base[b + j] : 0u);
  return v;
}
// (uniform) the window holds words [bitpos / 32, + words)
__device__ __forceinline__ void win_cover(FWin& f, uint64_t bitpos, uint32_t words) {
  const uint64_t wi = bitpos >> 5;
  if (f.W != kInf && wi >= f.W && wi + words <= f.W + kFWin) return;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < kFWin + 2; j += kWave) f.w[j] = load_be_word(f, wi + j);
  f.W = wi;
  __syncthreads();
}
// n (1..32) bits at absolute bit x, which the window holds
__device__ __forceinline__ uint32_t wbits(const FWin& f, uint64_t x, uint32_t n) {
  const uint32_t i = (uint32_t)((x >> 5) - f.W);
  const uint64_t v = (((uint64_t)f.w[i] << 32) | f.w[i + 1]) << (x & 31u);
  return (uint32_t)(v >> (64 - n));
}
// the first 1 bit at or after x inside the window (kInf: none)
__device__ __forceinline__ uint64_t next_one(const FWin& f, uint64_t x) {
  uint32_t i = (uint32_t)((x >> 5) - f.W);
  const uint32_t w = f.w[i] << (x & 31u);
  if (w) return x + (uint32_t)__builtin_clz(w);
  for (++i; i < kFWin; ++i)
    if (f.w[i]) return 32 * (f.W + i) + (uint32_t)__builtin_clz(f.w[i]);
  return kInf;
}
__device__ __forceinline__ int32_t sext(uint32_t v, uint32_t n) {  // n in 1..32
  return n >= 32 ? (int32_t)v : (int32_t)(v << (32 - n)) >> (32 - n);
}
// (uniform) n <= 32 bits at pos, advancing it
__device__ __forceinline__ uint32_t ubits(FWin& f, uint64_t& pos, uint32_t n) {
  if (!n) return 0;
  win_cover(f, pos, 2);
  const uint32_t v = wbits(f, pos, n);
  pos += n;
  return v;
}
// lane l gets lane l-1's v (DPP wave_shr:1; lane 0 keeps its own)
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v) {
  const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
  const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp(lo, lo, 0x138, 0xF, 0xF, false);
  const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp(hi, hi, 0x138, 0xF, 0xF, false);
  return ((uint64_t)h << 32) | l;
}
// lane src's v (src uniform)
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)src),
                 hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}

enum : int { kSfOk = 0, kSfBad = 1, kSfRedo = 2 };

// n values of w (0..32) bits each from pos into s[0, n), all lanes
__device__ void wave_raw(FWin& f, uint64_t& pos, int32_t* s, uint32_t n, uint32_t w) {
  for (uint32_t j0 = 0; j0 < n; j0 += kWave) {
    const uint64_t at = pos + (uint64_t)j0 * w;
    win_cover(f, at, (kWave * w + 31) / 32 + 2);
    const uint32_t i = j0 + threadIdx.x;
    if (i < n) s[i] = w ? sext(wbits(f, at + (uint64_t)threadIdx.x * w, w), w) : 0;
  }
  pos += (uint64_t)n * w;
}

// this lane's parse from entry e of its segment [ss, ss + 32): M = code
// starts (bit j: ss + j), X = the first start at or past the segment end
__device__ __forceinline__ void rice_parse(const FWin& f, uint64_t e, uint64_t ss, uint32_t k, uint32_t& M, uint64_t& X,
                                           bool& ovf) {
  M = 0;
  ovf = false;
  uint64_t x = e;
  while (x < ss + 32) {
    M |= 1u << (uint32_t)(x - ss);
    const uint64_t t = next_one(f, x);
    if (t == kInf) {
      ovf = true;
      X = kInf;
      return;
    }
    x = t + 1 + k;
  }
  X = x;
}

// n Rice codes of parameter k from pos, zigzag residuals into s[0, n)
__device__ int wave_rice(FWin& f, uint64_t& pos, int32_t* s, uint32_t n, uint32_t k) {
  const uint32_t lane = threadIdx.x;
  uint32_t done = 0;
  while (done < n) {
    win_cover(f, pos, kWave + kFLook);
    const uint64_t ss = ((pos >> 5) + lane) << 5;
    const uint32_t need = n - done;
    uint64_t e = lane == 0 ? pos : ss;
    uint32_t M;
    uint64_t X;
    bool ovf;
    rice_parse(f, e, ss, k, M, X, ovf);
    for (;;) {
      const uint64_t px = shfl_up_u64(X);
      const uint64_t ne = lane == 0 ? pos : px;
      bool moved = false;
      if (ne != e) {
        moved = true;
        e = ne;
        if (ne >= ss + 32) {  // the previous lane's last code covers this segment
          M = 0;
          X = ne;
          ovf = false;
        } else if ((M >> (uint32_t)(ne - ss)) & 1u) {  // joins the parse already made
          M &= ~0u << (uint32_t)(ne - ss);
        } else {
          rice_parse(f, ne, ss, k, M, X, ovf);
        }
      }
      const uint64_t mv = __ballot(moved);
      if (!mv) break;
      // the lanes below the first that moved are final: enough codes there?
      uint32_t tot;
      const uint32_t ex = wave_excl_sum((uint32_t)__builtin_popcount(M), tot);
      if ((uint32_t)__builtin_amdgcn_readlane((int)ex, (int)__builtin_ctzll(mv)) >= need) break;
    }
    const uint32_t cnt = (uint32_t)__builtin_popcount(M);
    uint32_t tot;
    const uint32_t idx = wave_excl_sum(cnt, tot);
    // a needed code that runs past the window
    if (__ballot(ovf && idx + cnt - 1 < need)) return kSfRedo;
    // (the bound as two tests: a single min(cnt, need - idx) behind an idx < need
    // select was observed to take codes past need on gfx950)
    bool wide = false;
    uint32_t m = M;
    for (uint32_t j = 0; j < cnt && idx + j < need; ++j) {
      const uint64_t x = ss + (uint32_t)__builtin_ctz(m);
      m &= m - 1;
      const uint64_t t = next_one(f, x);
      const uint64_t u = ((t - x) << k) | (k ? wbits(f, t + 1, k) : 0u);
      const int64_t r = (int64_t)(u >> 1) ^ -(int64_t)(u & 1u);
      wide |= r != (int64_t)(int32_t)r;
      s[done + idx + j] = (int32_t)r;
    }
    if (__ballot(wide)) return kSfRedo;
    if (tot >= need) {
      // the partition ends where code `need` would start
      const bool own = idx < need && need - 1 < idx + cnt;
      uint64_t endp = 0;
      if (own) {
        const uint32_t r = need - idx;
        if (r == cnt) {
          endp = X;
        } else {
          uint32_t mm = M;
          for (uint32_t j = 0; j < r; ++j) mm &= mm - 1;
          endp = ss + (uint32_t)__builtin_ctz(mm);
        }
      }
      pos = shfl_u64(endp, (uint32_t)__builtin_ctzll(__ballot(own)));
      done = n;
    } else {
      pos = shfl_u64(X, kWave - 1);
      done += tot;
    }
    if (pos == kInf) return kSfRedo;
  }
  return kSfOk;
}

struct SubInfo {
  uint32_t kind;  // 0: samples final (constant, verbatim), 1: fixed, 2: LPC
  uint32_t order, wasted;
  int32_t shift;
  int32_t coef[32];
};

// One subframe's samples (constant, verbatim) or warm-up samples and
// residuals (fixed, LPC) into s[0, bs); inf: what the predictor needs
__device__ int wave_subframe(FWin& f, uint64_t& pos, int32_t* s, uint32_t bs, uint32_t sbps, SubInfo& inf) {
  if (ubits(f, pos, 1)) return kSfBad;
  const uint32_t type = ubits(f, pos, 6);
  uint32_t wasted = 0;
  if (ubits(f, pos, 1)) {
    uint32_t z = 0;
    for (;;) {
      win_cover(f, pos, 2);
      const uint32_t w = wbits(f, pos, 32);
      if (w) {
        z += (uint32_t)__builtin_clz(w);
        pos += (uint32_t)__builtin_clz(w) + 1;
        break;
      }
      z += 32;
      pos += 32;
      if (z >= sbps) return kSfBad;
    }
    wasted = z + 1;
  }
  if (wasted >= sbps) return kSfBad;
  const uint32_t b = sbps - wasted;
  uint32_t kind = 0, order = 0;
  int32_t shift = 0;
  if (type == 0) {
    const int32_t v = sext(ubits(f, pos, b), b);
    for (uint32_t i = threadIdx.x; i < bs; i += kWave) s[i] = v;
  } else if (type == 1) {
    wave_raw(f, pos, s, bs, b);
  } else {
    if (type >= 8 && type <= 12) kind = 1, order = type - 8;
    else if (type >= 32) kind = 2, order = type - 31;
    else return kSfBad;
    if (order > bs) return kSfBad;
    for (uint32_t i = 0; i < order; ++i) {
      const int32_t v = sext(ubits(f, pos, b), b);
      if (threadIdx.x == 0) s[i] = v;
    }
    if (kind == 2) {
      const uint32_t prec = ubits(f, pos, 4) + 1;
      if (prec == 16) return kSfBad;
      shift = sext(ubits(f, pos, 5), 5);
      if (shift < 0) return kSfBad;
      for (uint32_t j = 0; j < order; ++j) {
        const int32_t cf = sext(ubits(f, pos, prec), prec);
        if (threadIdx.x == 0) inf.coef[j] = cf;
      }
    }
    const uint32_t method = ubits(f, pos, 2);
    if (method > 1) return kSfBad;
    const uint32_t pb = method ? 5u : 4u, esc = (1u << pb) - 1;
    const uint32_t po = ubits(f, pos, 4);
    if (bs % (1u << po) || (bs >> po) < order) return kSfBad;
    const uint32_t per = bs >> po;
    uint32_t i0 = order;
    for (uint32_t p = 0; p < (1u << po); ++p) {
      const uint32_t k = ubits(f, pos, pb), n = per - (p == 0 ? order : 0u);
      if (k == esc) {
        wave_raw(f, pos, s + i0, n, ubits(f, pos, 5));
      } else if (n) {
        const int st = wave_rice(f, pos, s + i0, n, k);
        if (st != kSfOk) return st;
      }
      i0 += n;
      if (pos > 8 * f.lim) return kSfBad;
    }
  }
  if (threadIdx.x == 0) {
    inf.kind = kind;
    inf.order = order;
    inf.wasted = wasted;
    inf.shift = shift;
  }
  return pos > 8 * f.lim ? kSfBad : kSfOk;
}

// A fixed predictor of order o over one LDS column, all lanes: the residual
// is the o-th backward difference of the samples, so the samples are o
// prefix sums of it, level j (o-1 .. 0) starting from D^j x at j taken from
// the warm-up samples.  Modulo 2^32, as the output is (the lane decoder's
// int64 values truncated to int32 give the same bits).
__device__ void fixed_column_scans(int32_t* s, uint32_t bs, uint32_t o) {
  const uint32_t lane = threadIdx.x;
  uint32_t x[4] = {0, 0, 0, 0}, c[4];
  for (uint32_t t = 0; t < o; ++t) x[t] = (uint32_t)s[t];
  c[0] = x[0];
  c[1] = x[1] - x[0];
  c[2] = x[2] - 2 * x[1] + x[0];
  c[3] = x[3] - 3 * x[2] + 3 * x[1] - x[0];
  __syncthreads();
  for (int j = (int)o - 1; j >= 0; --j) {
    uint32_t carry = 0;
    for (uint32_t r0 = (uint32_t)j; r0 < bs; r0 += kWave) {
      const uint32_t i = r0 + lane;
      int v = i == (uint32_t)j ? (int)c[j] : i < bs ? s[i] : 0;
      v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
      if (i < bs) s[i] = (int32_t)(carry + (uint32_t)v);
      carry += (uint32_t)__builtin_amdgcn_readlane(v, kWave - 1);
    }
    __syncthreads();
  }
}

// LPC prediction over one LDS column, one lane, with N >= order taps held in
// registers (coefficients zero past the order, history newest first) so that
// only the newest sample's product is on the per-sample dependency chain;
// false: a sample beyond 32 bits
// (64-bit products: a 32-bit accumulation where libFLAC's bound allows it,
// and an exact double-precision FMA chain, measured no faster)
template <uint32_t N>
__device__ bool lpc_column(int32_t* s, uint32_t bs, const SubInfo& inf) {
  const uint32_t o = inf.order;
  const int32_t sh = inf.shift;
  int32_t c[N], h[N];
#pragma unroll
  for (uint32_t j = 0; j < N; ++j) {
    c[j] = j < o ? inf.coef[j] : 0;
    h[j] = j < o ? s[o - 1 - j] : 0;
  }
  bool ok = true;
  int32_t r = o < bs ? s[o] : 0;
  for (uint32_t i = o; i < bs; ++i) {
    const int32_t rn = i + 1 < bs ? s[i + 1] : 0;
    int64_t acc = 0;
#pragma unroll
    for (uint32_t j = N - 1; j > 0; --j) acc += (int64_t)c[j] * h[j];
    acc += (int64_t)c[0] * h[0];
    const int64_t v = (int64_t)r + (acc >> sh);
    ok &= v == (int64_t)(int32_t)v;
    s[i] = (int32_t)v;
#pragma unroll
    for (uint32_t j = N - 1; j > 0; --j) h[j] = h[j - 1];
    h[0] = (int32_t)v;
    r = rn;
  }
  return ok;
}
__device__ bool predict_column(int32_t* s, uint32_t bs, const SubInfo& inf) {
  if (inf.kind != 2) return true;
  if (inf.order <= 8) return lpc_column<8>(s, bs, inf);
  if (inf.order <= 12) return lpc_column<12>(s, bs, inf);
  return lpc_column<32>(s, bs, inf);
}

__global__ __launch_bounds__(64) void rpp_flac_frame_wave_kernel(const FlacDecParams* tab) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  __shared__ SubInfo info[8];
  __shared__ uint32_t wide;
  const FlacDecParams& d = tab[blockIdx.y];
  if (!d.use_wave) return;
  const uint32_t c = blockIdx.x, lane = threadIdx.x;
  const uint32_t nc = min(*d.ncand, d.max_cand);
  if (c >= nc) return;
  if (lane == 0) {
    d.cand_len[c] = ~0ull;
    d.cand_redo[c] = 0;
    wide = 0;
  }
  const uint64_t p = d.cand_pos[c];
  uint32_t bs, assign;
  uint64_t coded;
  const uint32_t hl = parse_header(d.in, d.nbytes, p, d.channels, d.bps, bs, assign, coded);
  if (!hl) return;
  const uint32_t C = d.channels, mb = d.max_bs;
  const uint32_t mis = (uint32_t)((uintptr_t)d.in & 3u);
  FWin f{d.in - mis, d.nbytes + mis, lds, kInf};
  int32_t* smp = reinterpret_cast<int32_t*>(lds + kFWin + 2);  // [C][max_bs]
  uint64_t pos = 8 * (mis + p + hl);
  for (uint32_t ch = 0; ch < C; ++ch) {
    uint32_t sb = d.bps;
    if ((assign == 8 && ch == 1) || (assign == 9 && ch == 0) || (assign == 10 && ch == 1)) sb = d.bps + 1;
    const int st = wave_subframe(f, pos, smp + (uint64_t)ch * mb, bs, sb, info[ch]);
    if (st == kSfRedo && lane == 0) d.cand_redo[c] = 1;
    if (st != kSfOk) return;
  }
  __syncthreads();
  for (uint32_t ch = 0; ch < C; ++ch)
    if (info[ch].kind == 1 && info[ch].order) fixed_column_scans(smp + (uint64_t)ch * mb, bs, info[ch].order);
  if (lane < C && !predict_column(smp + (uint64_t)lane * mb, bs, info[lane])) wide = 1;
  __syncthreads();
  if (wide) {
    if (lane == 0) d.cand_redo[c] = 1;
    return;
  }
  int32_t* o = static_cast<int32_t*>(d.scratch) + (uint64_t)c * mb * C;
  for (uint32_t ch = 0; ch < C; ++ch) {
    const uint32_t ws = info[ch].wasted;
    for (uint32_t i = lane; i < bs; i += kWave) o[(uint64_t)ch * mb + i] = (int32_t)((uint32_t)smp[(uint64_t)ch * mb + i] << ws);
  }
  const uint64_t end = ((pos + 7) >> 3) - mis - p;
  if (lane == 0 && end + 2 <= d.nbytes - p) d.cand_len[c] = end;
}

constexpr uint64_t kNoPlace = ~0ull;

// CRC-16 check of every candidate that parsed, stream blockIdx.y of the table
__global__ __launch_bounds__(64) void rpp_flac_dec_crc_kernel(const FlacDecParams* tab) {
  __shared__ uint16_t t16[256];
  crc16_table(t16);
  const FlacDecParams& d = tab[blockIdx.y];
  crc_frames(t16, d.in, d.cand_pos, d.cand_len, min(*d.ncand, d.max_cand), nullptr, d.cand_ok);
}

__device__ __forceinline__ bool cand_valid(const FlacDecParams& d, uint32_t c) {
  return d.cand_len[c] != ~0ull && d.cand_ok[c];
}
// the first sample of candidate c's frame by its coded number (fixed
// blocking: frame number x the block size of the frame at byte 0)
__device__ __forceinline__ bool cand_first_sample(const FlacDecParams& d, uint32_t c, uint64_t nominal, uint32_t& bs,
                                                  uint64_t& first) {
  const uint64_t p = d.cand_pos[c];
  uint32_t assign;
  uint64_t coded;
  if (!parse_header(d.in, d.nbytes, p, d.channels, d.bps, bs, assign, coded)) return false;
  if (d.in[p + 1] & 1u) first = coded;  // variable blocking: the sample number
  else if (coded > (d.nsamples / (nominal ? nominal : 1))) return false;
  else first = coded * nominal;
  return true;
}

// Every valid candidate checks its link to the frame after it: that one is a
// valid candidate too and its coded number puts it right after this one (or
// this one ends the stream at the last sample).  When every link holds, the
// valid candidates' block sizes add up to the stream and a valid frame at
// byte 0 starts at sample 0, the valid candidates are exactly the chain the
// serial walk visits (one contiguous run of samples from 0 covers them all)
// and place[] is final; otherwise rpp_flac_chain_kernel walks.
__global__ __launch_bounds__(256) void rpp_flac_link_kernel(const FlacDecParams* tab) {
  const FlacDecParams& d = tab[blockIdx.y];
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nc = min(*d.ncand, d.max_cand);
  if (c >= nc) return;
  d.place[c] = kNoPlace;
  if (!cand_valid(d, c)) return;
  const uint32_t head = d.nbytes ? d.cand_at[0] : 0u;
  bool ok = head != 0;
  uint32_t bs = 0, bs_next;
  uint64_t first = 0, first_next;
  if (ok) ok = cand_first_sample(d, c, d.cand_info[head - 1], bs, first);
  if (ok) ok = first + bs <= d.nsamples;
  if (ok) {
    const uint64_t e = d.cand_pos[c] + d.cand_len[c] + 2;
    if (e == d.nbytes) {
      ok = first + bs == d.nsamples;
    } else if (e > d.nbytes) {
      ok = false;
    } else {
      const uint32_t at = d.cand_at[e];
      ok = at && cand_valid(d, at - 1) && cand_first_sample(d, at - 1, d.cand_info[head - 1], bs_next, first_next) &&
           first_next == first + bs;
    }
  }
  if (!ok) {
    atomicOr(reinterpret_cast<unsigned long long*>(&d.link_acc[1]), 1ull);
    return;
  }
  d.place[c] = first;
  atomicAdd(reinterpret_cast<unsigned long long*>(&d.link_acc[0]), (unsigned long long)bs);
}

// One lane: accepts the links, or walks the chain of frames from byte 0
// (each frame starts where the previous one's CRC-16 ends) and places the
// frames it visits
__global__ void rpp_flac_chain_kernel(const FlacDecParams* tab) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const FlacDecParams& d = tab[blockIdx.y];
  const uint32_t nc = min(*d.ncand, d.max_cand);
  const uint32_t head = d.nbytes ? d.cand_at[0] : 0u;
  if (d.nsamples && !d.link_acc[1] && d.link_acc[0] == d.nsamples && head && d.place[head - 1] == 0) {
    *d.status = RPP_OK;
    return;
  }
  for (uint32_t c = 0; c < nc; ++c) d.place[c] = kNoPlace;
  uint64_t pos = 0, done = 0;
  int32_t st = RPP_OK;
  while (done < d.nsamples) {
    if (pos >= d.nbytes) {
      st = RPP_TRUNCATED_INPUT;
      break;
    }
    const uint32_t at = d.cand_at[pos];
    if (!at) {
      st = RPP_INVALID_ARGUMENT;
      break;
    }
    const uint32_t c = at - 1;
    if (!cand_valid(d, c)) {
      st = RPP_INVALID_ARGUMENT;
      break;
    }
    const uint32_t bs = d.cand_info[c];
    if (done + bs > d.nsamples) {
      st = RPP_INVALID_ARGUMENT;
      break;
    }
    d.place[c] = done;
    done += bs;
    pos += d.cand_len[c] + 2;
  }
  *d.status = st;
}

// One block per candidate on the chain: planar subframes to interleaved
// samples, undoing the stereo decorrelation (left/side, side/right, mid/side)
template <class T>
__global__ __launch_bounds__(256) void rpp_flac_place_kernel(const FlacDecParams* tab) {
  const FlacDecParams& d = tab[blockIdx.y];
  if ((d.wide != 0) != (sizeof(T) == 8)) return;
  const uint32_t c = blockIdx.x;
  if (c >= min(*d.ncand, d.max_cand) || *d.status != RPP_OK) return;
  const uint64_t first = d.place[c];
  if (first == kNoPlace) return;
  uint32_t bs, assign;
  uint64_t coded;
  if (!parse_header(d.in, d.nbytes, d.cand_pos[c], d.channels, d.bps, bs, assign, coded)) return;
  const uint32_t C = d.channels, mb = d.max_bs;
  const T* s = static_cast<const T*>(d.scratch) + (uint64_t)c * mb * C;
  int32_t* o = d.out + first * C;
  if (assign >= 8) {
    for (uint32_t i = threadIdx.x; i < bs; i += blockDim.x) {
      const int64_t x0 = s[i], x1 = s[mb + i];
      int64_t L, R;
      if (assign == 8) L = x0, R = x0 - x1;
      else if (assign == 9) R = x1, L = x0 + x1;
      else {
        const int64_t m = (x0 * 2) | (x1 & 1);
        L = (m + x1) >> 1;
        R = (m - x1) >> 1;
      }
      *reinterpret_cast<int2*>(o + 2 * i) = make_int2((int32_t)L, (int32_t)R);
    }
  } else {
    const uint64_t n = (uint64_t)bs * C;
    for (uint64_t e = threadIdx.x; e < n; e += blockDim.x) {
      const uint32_t i = (uint32_t)(e / C), ch = (uint32_t)(e - (uint64_t)i * C);
      o[e] = (int32_t)s[(uint64_t)ch * mb + i];
    }
  }
}

// libFLAC's level presets (-l max LPC order, -r max partition order; the
// block size stays 4096 and all four stereo assignments are tried)
uint32_t level_max_lpc(uint32_t level) { return level <= 2 ? 0u : level == 3 ? 6u : level <= 6 ? 8u : kMaxLpc; }
uint32_t level_max_po(uint32_t level) { return min(level <= 2 ? 3u : level <= 4 ? 4u : 6u, kMaxPo); }

// the batch's frame table and per-block arrays, laid out in its workspace
struct BatchLayout {
  uint64_t frames = 0, slot = 0, slots_bytes = 0, head_bytes = 0;
};
BatchLayout batch_layout(uint32_t nblocks, const uint64_t* nsamples, const uint32_t* channels, const uint32_t* bps) {
  BatchLayout L;
  uint64_t bound = 0;
  for (uint32_t b = 0; b < nblocks; ++b) {
    L.frames += (nsamples[b] + kFlacBlock - 1) / kFlacBlock;
    bound = std::max<uint64_t>(bound, rpp_flac_frame_bound(channels[b], bps[b]));
  }
  L.slot = (bound + 15) & ~15ull;
  L.slots_bytes = L.frames * L.slot;
  // frame table (8 B per frame) + in_off, nsamples (8 B per block), channels,
  // bps, first frames (4 B per block, + 1)
  L.head_bytes = ((8 * L.frames + 16 * nblocks + 12 * (uint64_t)nblocks + 4 + 15) & ~15ull);
  return L;
}

}  // namespace

extern "C" {

uint64_t rpp_flac_frame_bound(uint32_t channels, uint32_t bps) {
  // header <= 16 bytes; a subframe at most its verbatim size (+1 bit for a
  // side channel) plus 2 bytes of type / wasted fields; padding; CRC-16
  return 16 + (uint64_t)channels * (2 + ((uint64_t)(bps + 1) * kFlacBlock + 7) / 8) + 2 + 16;
}

uint64_t rpp_flac_encode_workspace_bytes(uint64_t nsamples, uint32_t channels, uint32_t bps) {
  const uint64_t frames = (nsamples + kFlacBlock - 1) / kFlacBlock;
  const uint64_t slot = (rpp_flac_frame_bound(channels, bps) + 15) & ~15ull;
  return frames * slot + 3 * 8 * (frames + 1) + 256;
}

int rpp_flac_encode(const int32_t* d_samples, uint64_t nsamples, uint32_t channels, uint32_t bps, uint8_t* d_out,
                    uint64_t* d_total, void* d_workspace, uint64_t workspace_bytes, void* stream) {
  return rpp_flac_encode_ex(d_samples, nsamples, channels, bps, 5, 0, d_out, d_total, d_workspace, workspace_bytes,
                            stream);
}

int rpp_flac_encode_ex(const int32_t* d_samples, uint64_t nsamples, uint32_t channels, uint32_t bps, uint32_t level,
                       uint32_t exhaustive, uint8_t* d_out, uint64_t* d_total, void* d_workspace,
                       uint64_t workspace_bytes, void* stream) {
  if (channels < 1 || channels > 8 || bps < 4 || bps > 32) return RPP_UNSUPPORTED_CONFIG;
  if (level > 8) return RPP_INVALID_ARGUMENT;
  if (!d_total) return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  if (nsamples == 0) return hipMemsetAsync(d_total, 0, 8, s) == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
  if (!d_samples || !d_out || !d_workspace) return RPP_INVALID_ARGUMENT;
  if (workspace_bytes < rpp_flac_encode_workspace_bytes(nsamples, channels, bps)) return RPP_INVALID_ARGUMENT;
  const uint64_t frames = (nsamples + kFlacBlock - 1) / kFlacBlock;
  if (frames > 0x7FFFFFFFu) return RPP_INVALID_ARGUMENT;
  const uint64_t slot = (rpp_flac_frame_bound(channels, bps) + 15) & ~15ull;
  uint8_t* ws = static_cast<uint8_t*>(d_workspace);
  uint8_t* slots = ws;
  uint64_t* sizes = reinterpret_cast<uint64_t*>(ws + frames * slot);
  uint64_t* offs = sizes + frames + 1;
  uint64_t* lens = offs + frames + 1;
  FlacEncParams p{d_samples, nsamples, channels, bps, slots, slot, sizes, (uint32_t)frames,
                  level_max_lpc(level), exhaustive ? 1u : 0u, level_max_po(level),
                  nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t lds = sizeof(EncShared);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(rpp_flac_encode_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return RPP_HIP_ERROR;
  hipLaunchKernelGGL(rpp_flac_encode_kernel, dim3((uint32_t)frames), dim3(64), lds, s, p);
  int st = rpp_exclusive_scan_u64(sizes, frames, offs, s);
  if (st != RPP_OK) return st;
  hipLaunchKernelGGL(rpp_flac_pack_kernel, dim3((uint32_t)frames), dim3(256), 0, s, slots, slot, sizes, offs, d_out,
                     (uint32_t)frames);
  hipLaunchKernelGGL(rpp_flac_lens_kernel, dim3((uint32_t)((frames + 255) / 256)), dim3(256), 0, s, sizes, offs, lens, frames,
                     d_total);
  hipLaunchKernelGGL(rpp_flac_crc_kernel, dim3((uint32_t)(frames < 4096 ? frames : 4096)), dim3(64), 0, s, d_out, offs,
                     lens, (uint32_t)frames, d_out, nullptr, nullptr);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

uint64_t rpp_flac_encode_batch_workspace_bytes(uint32_t nblocks, const uint64_t* h_nsamples, const uint32_t* h_channels,
                                               const uint32_t* h_bps) {
  if (!nblocks || !h_nsamples || !h_channels || !h_bps) return 256;
  const BatchLayout L = batch_layout(nblocks, h_nsamples, h_channels, h_bps);
  return L.slots_bytes + 3 * 8 * (L.frames + 1) + L.head_bytes + 256;
}

int rpp_flac_encode_batch(const int32_t* d_samples, uint32_t nblocks, const uint64_t* h_in_off,
                          const uint64_t* h_nsamples, const uint32_t* h_channels, const uint32_t* h_bps,
                          uint32_t level, uint32_t exhaustive, uint8_t* d_out, uint64_t* d_out_off, void* d_workspace,
                          uint64_t workspace_bytes, void* stream) {
  if (level > 8) return RPP_INVALID_ARGUMENT;
  if (nblocks == 0) return RPP_OK;
  if (!h_in_off || !h_nsamples || !h_channels || !h_bps || !d_out_off || !d_workspace) return RPP_INVALID_ARGUMENT;
  for (uint32_t b = 0; b < nblocks; ++b)
    if (h_channels[b] < 1 || h_channels[b] > 8 || h_bps[b] < 4 || h_bps[b] > 32) return RPP_UNSUPPORTED_CONFIG;
  if (workspace_bytes < rpp_flac_encode_batch_workspace_bytes(nblocks, h_nsamples, h_channels, h_bps))
    return RPP_INVALID_ARGUMENT;
  const BatchLayout L = batch_layout(nblocks, h_nsamples, h_channels, h_bps);
  if (L.frames > 0x7FFFFFFFu) return RPP_INVALID_ARGUMENT;
  if (L.frames && (!d_samples || !d_out)) return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  uint8_t* ws = static_cast<uint8_t*>(d_workspace);
  uint8_t* slots = ws;
  uint64_t* sizes = reinterpret_cast<uint64_t*>(ws + L.slots_bytes);
  uint64_t* offs = sizes + L.frames + 1;
  uint64_t* lens = offs + L.frames + 1;
  uint8_t* head = reinterpret_cast<uint8_t*>(lens + L.frames + 1);
  // the frame table and per-block arrays, staged on the host and copied once
  std::vector<uint8_t> h(L.head_bytes, 0);
  auto* fdesc = reinterpret_cast<uint2*>(h.data());
  auto* in_off = reinterpret_cast<uint64_t*>(h.data() + 8 * L.frames);
  auto* ns = in_off + nblocks;
  auto* ch = reinterpret_cast<uint32_t*>(ns + nblocks);
  auto* bp = ch + nblocks;
  auto* fstart = bp + nblocks;  // [nblocks + 1]
  uint64_t g = 0;
  for (uint32_t b = 0; b < nblocks; ++b) {
    in_off[b] = h_in_off[b];
    ns[b] = h_nsamples[b];
    ch[b] = h_channels[b];
    bp[b] = h_bps[b];
    fstart[b] = (uint32_t)g;
    const uint64_t nf = (h_nsamples[b] + kFlacBlock - 1) / kFlacBlock;
    for (uint64_t f = 0; f < nf; ++f, ++g) fdesc[g] = make_uint2(b, (uint32_t)f);
  }
  fstart[nblocks] = (uint32_t)g;
  if (hipMemcpyAsync(head, h.data(), h.size(), hipMemcpyHostToDevice, s) != hipSuccess) return RPP_HIP_ERROR;
  const uint8_t* dh = head;
  FlacEncParams p{d_samples, 0, 1, 16, slots, L.slot, sizes, (uint32_t)L.frames,
                  level_max_lpc(level), exhaustive ? 1u : 0u, level_max_po(level),
                  reinterpret_cast<const uint2*>(dh), reinterpret_cast<const uint64_t*>(dh + 8 * L.frames),
                  reinterpret_cast<const uint64_t*>(dh + 8 * L.frames) + nblocks,
                  reinterpret_cast<const uint32_t*>(dh + 8 * L.frames + 16 * (uint64_t)nblocks),
                  reinterpret_cast<const uint32_t*>(dh + 8 * L.frames + 16 * (uint64_t)nblocks) + nblocks};
  const uint32_t* d_fstart = reinterpret_cast<const uint32_t*>(dh + 8 * L.frames + 16 * (uint64_t)nblocks) + 2 * nblocks;
  if (L.frames) {
    const size_t lds = sizeof(EncShared);
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(rpp_flac_encode_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return RPP_HIP_ERROR;
    hipLaunchKernelGGL(rpp_flac_encode_kernel, dim3((uint32_t)L.frames), dim3(64), lds, s, p);
  }
  int st = rpp_exclusive_scan_u64(sizes, L.frames, offs, s);
  if (st != RPP_OK) return st;
  if (L.frames) {
    hipLaunchKernelGGL(rpp_flac_pack_kernel, dim3((uint32_t)L.frames), dim3(256), 0, s, slots, L.slot, sizes, offs,
                       d_out, (uint32_t)L.frames);
    hipLaunchKernelGGL(rpp_flac_lens_kernel, dim3((uint32_t)((L.frames + 255) / 256)), dim3(256), 0, s, sizes, offs,
                       lens, L.frames, d_out_off + nblocks);  // (the total; rpp_flac_block_off_kernel writes it too)
    hipLaunchKernelGGL(rpp_flac_crc_kernel, dim3((uint32_t)(L.frames < 4096 ? L.frames : 4096)), dim3(64), 0, s, d_out,
                       offs, lens, (uint32_t)L.frames, d_out, nullptr, nullptr);
  }
  hipLaunchKernelGGL(rpp_flac_block_off_kernel, dim3((nblocks + 256) / 256), dim3(256), 0, s, sizes, offs, L.frames,
                     d_fstart, nblocks, d_out_off);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

uint64_t rpp_flac_decode_workspace_bytes(uint64_t nbytes, uint32_t channels, uint32_t bps, uint32_t max_blocksize,
                                         uint32_t max_candidates) {
  const uint64_t mc = max_candidates;
  const uint64_t per = (uint64_t)max_blocksize * channels;
  // (the take() layout of flac_decode_many, 16-byte aligned pieces: the
  // stream's table entry, then per-candidate scratch of int32 samples, int64
  // for 32-bit streams)
  return 4 * (nbytes + 1) + mc * (8 + 4 + 8 + 4 + 4 + 8) + 7 * 16 + 16 + mc * per * (bps == 32 ? 8 : 4) + 256;
}

uint64_t rpp_flac_decode_batch_workspace_bytes(uint32_t nblocks, const uint64_t* h_nbytes, const uint32_t* h_channels,
                                               const uint32_t* h_bps, const uint32_t* h_max_blocksize,
                                               const uint32_t* h_max_candidates) {
  if (!nblocks || !h_nbytes || !h_channels || !h_bps || !h_max_blocksize || !h_max_candidates) return 256;
  uint64_t total = 256;
  for (uint32_t b = 0; b < nblocks; ++b)
    total += rpp_flac_decode_workspace_bytes(h_nbytes[b], h_channels[b], h_bps[b], h_max_blocksize[b],
                                             h_max_candidates[b]);
  return total;
}

}  // extern "C"

namespace {

// The decode of nblocks streams in one sequence of launches (each kernel's
// grid: .x over a stream's bytes or candidates, .y over the streams; the
// table of per-stream parameters is copied to the head of the workspace).
// Stream b is byte-for-byte what a decode of it alone gives.
int flac_decode_many(const uint8_t* d_frames, uint32_t nblocks, const uint64_t* in_off, const uint64_t* nbytes,
                     const uint32_t* channels, const uint32_t* bps, const uint32_t* max_bs, const uint64_t* nsamples,
                     int32_t* d_out, const uint64_t* out_off, int32_t* d_status, const uint32_t* max_cand,
                     void* d_workspace, uint64_t workspace_bytes, uint32_t* d_ncand, hipStream_t s) {
  if (nblocks > 65535) return RPP_INVALID_ARGUMENT;  // (grid .y)
  for (uint32_t b = 0; b < nblocks; ++b) {
    if (channels[b] < 1 || channels[b] > 8 || bps[b] < 4 || bps[b] > 32 || max_bs[b] < 1 || max_bs[b] > 65536)
      return RPP_UNSUPPORTED_CONFIG;
    if ((nbytes[b] && !d_frames) || (nsamples[b] && !d_out) || max_cand[b] == 0) return RPP_INVALID_ARGUMENT;
  }
  if (!d_status || !d_ncand || !d_workspace) return RPP_INVALID_ARGUMENT;
  uint8_t* ws = static_cast<uint8_t*>(d_workspace);
  auto take = [&](uint64_t bytes) {
    uint8_t* q = ws;
    ws += (bytes + 15) & ~15ull;
    return q;
  };
  const auto* d_tab = reinterpret_cast<const FlacDecParams*>(take(sizeof(FlacDecParams) * (uint64_t)nblocks));
  uint64_t* d_link = reinterpret_cast<uint64_t*>(take(16 * (uint64_t)nblocks));
  std::vector<FlacDecParams> tab(nblocks);
  uint64_t max_bytes = 0, max_mc = 0, wave_lds = 0;
  bool any_wave = false, any_lane32 = false, any_wide = false;
  for (uint32_t b = 0; b < nblocks; ++b) {
    FlacDecParams& d = tab[b];
    const uint64_t mc = max_cand[b], per = (uint64_t)max_bs[b] * channels[b];
    d = FlacDecParams{};
    d.in = d_frames ? d_frames + in_off[b] : nullptr;
    d.nbytes = nbytes[b];
    d.channels = channels[b];
    d.bps = bps[b];
    d.max_bs = max_bs[b];
    d.nsamples = nsamples[b];
    d.cand_at = reinterpret_cast<uint32_t*>(take(4 * (nbytes[b] + 1)));
    d.cand_pos = reinterpret_cast<uint64_t*>(take(8 * mc));
    d.cand_info = reinterpret_cast<uint32_t*>(take(4 * mc));
    d.cand_len = reinterpret_cast<uint64_t*>(take(8 * mc));
    d.cand_ok = reinterpret_cast<uint32_t*>(take(4 * mc));
    d.cand_redo = reinterpret_cast<uint32_t*>(take(4 * mc));
    d.place = reinterpret_cast<uint64_t*>(take(8 * mc));
    d.link_acc = d_link + 2 * (uint64_t)b;
    d.wide = bps[b] == 32;
    d.scratch = take((d.wide ? 8 : 4) * mc * per);
    d.ncand = d_ncand + b;
    d.max_cand = max_cand[b];
    d.out = d_out ? d_out + out_off[b] : nullptr;
    d.status = d_status + b;
    // the wave decoder where the frame's samples fit LDS, the lane decoder for the rest
    const uint64_t lds = 4ull * (kFWin + 2) + 4ull * per;
    d.use_wave = !d.wide && lds <= kFlacWaveLds;
    d.redo_only = d.use_wave;
    if (d.use_wave) wave_lds = std::max(wave_lds, lds);
    any_wave |= d.use_wave != 0;
    any_lane32 |= !d.wide;
    any_wide |= d.wide != 0;
    max_bytes = std::max(max_bytes, nbytes[b]);
    max_mc = std::max(max_mc, mc);
  }
  // (the callers' workspace formulas bound this layout; checked all the same)
  if ((uint64_t)(ws - static_cast<uint8_t*>(d_workspace)) > workspace_bytes) return RPP_INVALID_ARGUMENT;
  if (nblocks == 0) return RPP_OK;
  if (hipMemcpyAsync(const_cast<FlacDecParams*>(d_tab), tab.data(), sizeof(FlacDecParams) * (size_t)nblocks,
                     hipMemcpyHostToDevice, s) != hipSuccess)
    return RPP_HIP_ERROR;
  if (hipMemsetAsync(d_ncand, 0, 4 * (size_t)nblocks, s) != hipSuccess) return RPP_HIP_ERROR;
  const uint32_t B = nblocks, mcx = (uint32_t)max_mc;
  if (max_bytes) hipLaunchKernelGGL(rpp_flac_scan_kernel, dim3((uint32_t)((max_bytes + 255) / 256), B), dim3(256), 0, s, d_tab);
  if (any_wave) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(rpp_flac_frame_wave_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFlacWaveLds);
    if (attr != hipSuccess) return RPP_HIP_ERROR;
    hipLaunchKernelGGL(rpp_flac_frame_wave_kernel, dim3(mcx, B), dim3(64), (size_t)wave_lds, s, d_tab);
  }
  if (any_wide) hipLaunchKernelGGL(rpp_flac_frame_kernel<int64_t>, dim3((mcx + 63) / 64, B), dim3(64), 0, s, d_tab);
  if (any_lane32) hipLaunchKernelGGL(rpp_flac_frame_kernel<int32_t>, dim3((mcx + 63) / 64, B), dim3(64), 0, s, d_tab);
  hipLaunchKernelGGL(rpp_flac_dec_crc_kernel, dim3(mcx < 4096 ? mcx : 4096, B), dim3(64), 0, s, d_tab);
  if (hipMemsetAsync(d_link, 0, 16 * (size_t)nblocks, s) != hipSuccess) return RPP_HIP_ERROR;
  hipLaunchKernelGGL(rpp_flac_link_kernel, dim3((mcx + 255) / 256, B), dim3(256), 0, s, d_tab);
  hipLaunchKernelGGL(rpp_flac_chain_kernel, dim3(1, B), dim3(1), 0, s, d_tab);
  if (any_wide) hipLaunchKernelGGL(rpp_flac_place_kernel<int64_t>, dim3(mcx, B), dim3(256), 0, s, d_tab);
  if (any_lane32) hipLaunchKernelGGL(rpp_flac_place_kernel<int32_t>, dim3(mcx, B), dim3(256), 0, s, d_tab);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

}  // namespace

extern "C" {

int rpp_flac_decode(const uint8_t* d_frames, uint64_t nbytes, uint32_t channels, uint32_t bps,
                    uint32_t max_blocksize, uint64_t nsamples, int32_t* d_out, int32_t* d_status,
                    uint32_t max_candidates, void* d_workspace, uint64_t workspace_bytes, uint32_t* d_ncand,
                    void* stream) {
  if (channels < 1 || channels > 8 || bps < 4 || bps > 32 || max_blocksize < 1 || max_blocksize > 65536)
    return RPP_UNSUPPORTED_CONFIG;
  if (!d_status || !d_ncand) return RPP_INVALID_ARGUMENT;
  if (workspace_bytes < rpp_flac_decode_workspace_bytes(nbytes, channels, bps, max_blocksize, max_candidates))
    return RPP_INVALID_ARGUMENT;
  if ((nbytes && !d_frames) || (nsamples && !d_out) || !d_workspace || max_candidates == 0)
    return RPP_INVALID_ARGUMENT;
  const uint64_t zero = 0;
  return flac_decode_many(d_frames, 1, &zero, &nbytes, &channels, &bps, &max_blocksize, &nsamples, d_out, &zero,
                          d_status, &max_candidates, d_workspace, workspace_bytes, d_ncand, (hipStream_t)stream);
}

int rpp_flac_decode_batch(const uint8_t* d_frames, uint32_t nblocks, const uint64_t* h_in_off,
                          const uint64_t* h_nbytes, const uint32_t* h_channels, const uint32_t* h_bps,
                          const uint32_t* h_max_blocksize, const uint64_t* h_nsamples, int32_t* d_out,
                          const uint64_t* h_out_off, int32_t* d_status, const uint32_t* h_max_candidates,
                          void* d_workspace, uint64_t workspace_bytes, uint32_t* d_ncand, void* stream) {
  if (nblocks == 0) return RPP_OK;
  if (!h_in_off || !h_nbytes || !h_channels || !h_bps || !h_max_blocksize || !h_nsamples || !h_out_off ||
      !h_max_candidates)
    return RPP_INVALID_ARGUMENT;
  for (uint32_t b = 0; b < nblocks; ++b)
    if (h_channels[b] < 1 || h_channels[b] > 8 || h_bps[b] < 4 || h_bps[b] > 32 || h_max_blocksize[b] < 1 ||
        h_max_blocksize[b] > 65536)
      return RPP_UNSUPPORTED_CONFIG;
  if (workspace_bytes <
      rpp_flac_decode_batch_workspace_bytes(nblocks, h_nbytes, h_channels, h_bps, h_max_blocksize, h_max_candidates))
    return RPP_INVALID_ARGUMENT;
  return flac_decode_many(d_frames, nblocks, h_in_off, h_nbytes, h_channels, h_bps, h_max_blocksize, h_nsamples,
                          d_out, h_out_off, d_status, h_max_candidates, d_workspace, workspace_bytes, d_ncand,
                          (hipStream_t)stream);
}

}  // extern "C"
