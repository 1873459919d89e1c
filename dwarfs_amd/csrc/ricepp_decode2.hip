// ricepp_decode2.hip -- two-stage ricepp decode (rpp_decode_batch and
// rpp_decode_batch_ws of include/ricepp_amd.h).
//
// The reference decodes a stream serially: codec::decode walks the
// sub-blocks (ricepp/include/ricepp/codec.h:103-140), each sub-block reads a
// 4-bit header and bs Rice codes (detail/decode.h:42-83), and every value is
// the previous one plus a zig-zag delta.  Two things are serial there, and
// they are split apart here:
//
//   1. where each sub-block starts: sub-block k+1 begins where the n-th code
//      of sub-block k ends.  rpp_parse_kernel (ricepp_kernels.hip) finds the
//      starts, one wave per stream, with the exact table-driven parse and no
//      value work, and writes them to sb_pos.
//   2. the running value `last`: a sub-block's samples are its entry value
//      plus the prefix sums of its own deltas.  rpp_extract_kernel decodes
//      all sub-blocks of all streams at once -- one LANE per sub-block,
//      reading its codes serially out of an LDS tile of the stream (a code
//      is ~12 VALU: two-word read, funnel shift, find-first-set, bit-field
//      extract, zig-zag, add) into registers -- and then joins the sub-blocks'
//      delta sums by a scan: within the 256-sub-block tile through LDS,
//      across the tiles of a long stream by decoupled look-back (tiles are
//      taken in order from an atomic counter, so a tile only ever waits for
//      tiles that are already running).  A raw sub-block (header 15) resets
//      the running value, a zero sub-block (header 0) adds nothing: the scan
//      element is (reset?, value) with the obvious composition.
//
// Lanes whose sub-block is unusual (raw or zero header, the ragged last
// chunk, a code longer than the 32-bit window) take an exact general path
// (decode.h restated with a runtime loop) in the same kernel: once for the
// delta sum, once more for the stores after the scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "ricepp_amd.h"
#include "ricepp_internal.h"

namespace {

constexpr uint32_t kTile = 256;          // sub-blocks (lanes) per tile
constexpr uint32_t kStageWords = 9216;   // 36 KiB of the stream per tile in LDS
// slack after the staged words: a lane whose codes run past their window
// (then decoded again by the general path) reads at most 128 * 45 bits on
constexpr uint32_t kStagePad = 192;
constexpr uint32_t kMaxExtractGrid = 2048;

// ---- workspace layout (rpp_decode_workspace_bytes) ----
struct Workspace {
  uint64_t* sb_cnt;     // [B + 1]
  uint64_t* sb_base;    // [B + 1]
  uint64_t* tile_cnt;   // [B + 1]
  uint64_t* tile_base;  // [B + 1]
  uint64_t* tile_state; // [max_tiles]
  uint32_t* tile_map;   // [max_tiles]
  uint32_t* sb_pos;     // [max_sb + B]
  uint32_t* counter;    // [1]
  uint64_t bytes;
  uint64_t max_tiles;
};

uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// diagnostics (RICEPP_DEC2_DBG & 4): per-phase cycle sums of the extraction
// tiles (wave 0 of each workgroup), read by rpp_diag_read
__device__ unsigned long long g_dec2_diag[8];
__device__ __forceinline__ uint64_t clk() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

Workspace layout(const rpp_config* cfg, uint64_t total_samples, uint32_t nblocks, uint8_t* base) {
  const uint64_t B = nblocks;
  const uint64_t max_sb = total_samples / cfg->block_size + B * cfg->component_stream_count;
  const uint64_t max_tiles = max_sb / kTile + B;
  Workspace w{};
  uint64_t off = 0;
  auto take = [&](uint64_t bytes) {
    uint8_t* p = base ? base + off : nullptr;
    off = align_up(off + bytes, 256);
    return p;
  };
  w.sb_cnt = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.sb_base = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.tile_cnt = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.tile_base = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
  w.tile_state = reinterpret_cast<uint64_t*>(take(max_tiles * 8));
  w.tile_map = reinterpret_cast<uint32_t*>(take(max_tiles * 4));
  w.sb_pos = reinterpret_cast<uint32_t*>(take((max_sb + B) * 4));
  w.counter = reinterpret_cast<uint32_t*>(take(256));
  w.bytes = off;
  w.max_tiles = max_tiles;
  return w;
}

// sub-blocks + 1 (the end entry) and tiles of each stream; entry B is 0 so
// that the exclusive scans end in the totals
__global__ void rpp_dec_count_kernel(const uint64_t* n_samples, uint32_t nblocks, uint32_t chunk_len, uint32_t cs,
                                     uint64_t* sb_cnt, uint64_t* tile_cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nblocks) return;
  uint64_t nsb = 0;
  if (i < nblocks) {
    const uint64_t n = n_samples[i];
    if (n % cs == 0 && n < RPP_MAX_STREAM_SAMPLES) nsb = (n + chunk_len - 1) / chunk_len * cs;
  }
  sb_cnt[i] = i < nblocks ? nsb + 1 : 0;
  tile_cnt[i] = (nsb + kTile - 1) / kTile;
}

__global__ void rpp_dec_tile_map_kernel(const uint64_t* tile_base, uint32_t nblocks, uint32_t* tile_map) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nblocks) return;
  for (uint64_t t = tile_base[i]; t < tile_base[i + 1]; ++t) tile_map[t] = i;
}

struct ExtractParams {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint64_t* in_bytes;
  const uint64_t* n_samples;
  uint16_t* out;
  const uint64_t* out_off;
  const int32_t* status;  // of the parse pass: streams that failed are skipped
  const uint32_t* sb_pos;
  const uint64_t* sb_base;
  const uint64_t* tile_base;
  const uint32_t* tile_map;
  uint64_t* tile_state;
  uint32_t* counter;
  uint32_t nblocks;
  uint32_t bs, be, ulsb;
  uint32_t dbg;  // diagnostics (RICEPP_DEC2_DBG): 1 no fast lanes, 2 fast lanes store sample by sample
};

// pixel traits (ricepp/ricepp_cpuspecific_traits.h:63-75)
__device__ __forceinline__ uint32_t px_read(uint32_t v, uint32_t be, uint32_t ulsb) {
  v &= 0xFFFFu;
  if (be) v = ((v >> 8) | (v << 8)) & 0xFFFFu;
  return v >> ulsb;
}
__device__ __forceinline__ uint32_t px_write(uint32_t v, uint32_t be, uint32_t ulsb) {
  v = (v << ulsb) & 0xFFFFu;
  return be ? (((v >> 8) | (v << 8)) & 0xFFFFu) : v;
}

// stream word w (from the 4-aligned base), zero past the stream's last byte
// (bitstream_reader.h:165-166 zero-pads the last packet)
__device__ __forceinline__ uint32_t stream_word(const uint8_t* in, uint32_t nbytes, uint32_t w) {
  const uint32_t byte0 = w * 4u;
  if (byte0 >= nbytes) return 0u;
  if (nbytes - byte0 >= 4) return *reinterpret_cast<const uint32_t*>(in + byte0);
  uint32_t v = 0;
  for (uint32_t k = 0; k < nbytes - byte0; ++k) v |= (uint32_t)in[byte0 + k] << (8 * k);
  return v;
}

// scan element (reset?, value): bit 16 = a raw sub-block reset the value
constexpr uint32_t kSet = 1u << 16;
__device__ __forceinline__ uint32_t combine(uint32_t a, uint32_t b) {
  return (b & kSet) ? b : ((a & kSet) | ((a + b) & 0xFFFFu));
}

// tile state word: bits 62-63 flag (1 aggregate, 2 inclusive prefix),
// component 0 in bits 0-16, component 1 in bits 17-33
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62;
__device__ __forceinline__ uint64_t pack_state(uint32_t c0, uint32_t c1, uint64_t flag) {
  return flag | (uint64_t)(c0 & 0x1FFFFu) | ((uint64_t)(c1 & 0x1FFFFu) << 17);
}

__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// Bits of the stream for the general path: LDS tile when staged, else global.
struct Reader {
  const uint32_t* st;  // staged words [w0, w0 + nst)
  uint32_t w0, nst;
  const uint8_t* in;
  uint32_t nbytes;
  __device__ __forceinline__ uint32_t word(uint32_t w) const {
    const uint32_t r = w - w0;
    return r < nst ? st[r] : stream_word(in, nbytes, w);
  }
  __device__ __forceinline__ uint32_t peek32(uint32_t pos) const {
    return __builtin_amdgcn_alignbit(word((pos >> 5) + 1), word(pos >> 5), pos & 31u);
  }
};

// decode.h:42-83 restated for one sub-block with a runtime loop: the delta
// sum / reset element, and (STORE) the stored samples written with stride CS.
template <bool STORE>
__device__ uint32_t decode_general(const Reader& rd, uint32_t pos, uint32_t n, uint32_t carry, uint16_t* dst,
                                   uint32_t stride, uint32_t be, uint32_t ulsb) {
  const uint32_t fsp1 = rd.peek32(pos) & 15u;
  pos += 4;
  if (fsp1 == 0) {  // decode.h:79-80
    if (STORE) {
      const uint16_t v = (uint16_t)px_write(carry, be, ulsb);
      for (uint32_t i = 0; i < n; ++i) dst[i * stride] = v;
    }
    return 0u;
  }
  if (fsp1 == 15) {  // decode.h:72-77: raw stored values, last = read(last)
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; ++i, pos += 16) {
      v = rd.peek32(pos) & 0xFFFFu;
      if (STORE) dst[i * stride] = (uint16_t)v;
    }
    return kSet | px_read(v, be, ulsb);
  }
  const uint32_t fs = fsp1 - 1;
  const uint32_t fmask = (1u << fs) - 1u;
  uint32_t acc = STORE ? carry : 0u;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t q = 0;
    for (;;) {  // bitstream_reader::find_first_set
      const uint32_t x = rd.peek32(pos);
      if (x) {
        const uint32_t t = ffbl(x);
        q += t;
        pos += t + 1;
        break;
      }
      q += 32;
      pos += 32;
    }
    const uint32_t d = (q << fs) | (rd.peek32(pos) & fmask);
    pos += fs;
    acc += (d >> 1) ^ (0u - (d & 1u));
    if (STORE) dst[i * stride] = (uint16_t)px_write(acc, be, ulsb);
  }
  return acc & 0xFFFFu;
}

// Pixel write of two packed values (low, high), optional unused-LSB shift.
template <bool SH>
__device__ __forceinline__ uint32_t px_write2(uint32_t v, uint32_t sel, uint32_t ulsb) {
  if (SH) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    us2 x = __builtin_bit_cast(us2, v);
    x = x << (us2)(unsigned short)ulsb;
    v = __builtin_bit_cast(uint32_t, x);
  }
  return __builtin_amdgcn_perm(v, v, sel);
}

template <uint32_t CS, uint32_t BS, bool SH>
__global__ __launch_bounds__(kTile) void rpp_extract_kernel(ExtractParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t stage[kStageWords + kStagePad];
  __shared__ uint32_t scan_buf[kTile];
  __shared__ uint32_t sh_tile, sh_carry[2], sh_min;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = __lane_id();
  const uint32_t be = p.be, ulsb = p.ulsb;
  const uint32_t selbe = be ? 0x02030001u : 0x03020100u;  // byte-swap each half
  const uint32_t chunk_len = CS * BS;
  const uint64_t total_tiles = p.tile_base[p.nblocks];

  const bool timing = (p.dbg & 4) && tid < 64;
  uint64_t tp = timing ? clk() : 0;
  auto stamp = [&](int i) {
    if (timing) {
      const uint64_t now = clk();
      if (tid == 0) atomicAdd(&g_dec2_diag[i], (unsigned long long)(now - tp));
      tp = now;
    }
  };
  for (;;) {
    if (tid == 0) sh_tile = atomicAdd(p.counter, 1u);
    __syncthreads();
    const uint32_t t = sh_tile;
    if (t >= total_tiles) return;  // (uniform)
    const uint32_t b = p.tile_map[t];
    const uint32_t lt = (uint32_t)(t - p.tile_base[b]);
    if (p.status[b] != RPP_OK) {  // the parse failed: nothing to decode
      if (tid == 0) __hip_atomic_store(&p.tile_state[t], kFlagIncl, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      continue;
    }
    // ---- the stream ----
    const uint64_t ioff = p.in_off[b];
    const uint32_t mis = (uint32_t)(ioff & 3u);
    const uint8_t* base = p.in + (ioff - mis);
    const uint32_t nbytes = (uint32_t)p.in_bytes[b] + mis;
    const uint32_t N = (uint32_t)p.n_samples[b];
    const uint32_t nsb = (N + chunk_len - 1) / chunk_len * CS;
    const uint32_t k0 = lt * kTile;
    const uint32_t kcount = min(kTile, nsb - k0);
    const uint32_t* pos_tab = p.sb_pos + p.sb_base[b];
    const uint32_t k = k0 + tid;
    const bool active = tid < kcount;
    const uint32_t start = active ? pos_tab[k] : 0u;
    const uint32_t end = active ? pos_tab[k + 1] : 0u;
    const uint32_t comp = k % CS;
    const uint32_t cbase = (k / CS) * chunk_len;
    const uint32_t n = active ? min(N - cbase, chunk_len) / CS : 0u;
    uint16_t* const out = p.out + p.out_off[b];

    stamp(0);
    // ---- stage the tile's words: 16-byte loads, several in flight per
    //      lane; the group holding the stream's end word by word (zero past
    //      the last byte) ----
    const uint32_t w0 = pos_tab[k0] >> 5;
    const uint32_t wend = (pos_tab[k0 + kcount] >> 5) + 2;
    const uint32_t nst = min(wend - w0, kStageWords);
    {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      const uint32_t nq = (nst + 3) / 4;  // 16-byte groups
      constexpr uint32_t kInFlight = 4;
      for (uint32_t q0 = 0; q0 < nq; q0 += kInFlight * kTile) {
        u4 v[kInFlight];
#pragma unroll
        for (uint32_t j = 0; j < kInFlight; ++j) {
          const uint32_t q = q0 + j * kTile + tid;
          const uint32_t wq = w0 + 4 * q;
          if (q < nq && 4 * wq + 16 <= nbytes) {
            v[j] = *reinterpret_cast<const u4*>(base + 4 * wq);  // (4-byte aligned)
          } else {
            v[j] = u4{stream_word(base, nbytes, wq), stream_word(base, nbytes, wq + 1), stream_word(base, nbytes, wq + 2),
                      stream_word(base, nbytes, wq + 3)};
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < kInFlight; ++j) {
          const uint32_t q = q0 + j * kTile + tid;
          if (q < nq) *reinterpret_cast<u4*>(&stage[4 * q]) = v[j];
        }
      }
    }
    __syncthreads();
    stamp(1);
    const Reader rd{stage, w0, nst, base, nbytes};

    // ---- fast lanes: Rice, a full sub-block, staged, every code <= 32 bits ----
    uint32_t hdr = 0;
    if (active) hdr = rd.peek32(start) & 15u;
    bool fast = active && hdr != 0 && hdr != 15 && n == BS && (end >> 5) + 1 < w0 + nst && !(p.dbg & 1);
    // pairs share one store path (the shuffle outside any condition: a
    // short-circuit && would run it on the fast lanes only)
    if (CS == 2) {
      const int pf = __shfl_xor((int)fast, 1);
      fast = fast && pf;
    }
    uint32_t r[BS / 2];
    uint32_t agg = 0;
    if (fast) {
      const uint32_t fs = hdr - 1;
      uint32_t pos = start + 4 - 32 * w0;
      uint32_t acc = 0, maxq = 0;
#pragma unroll
      for (uint32_t i = 0; i < BS; i += 2) {
        uint32_t v[2];
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) {
          const uint32_t* w = stage + (pos >> 5);
          const uint32_t x = __builtin_amdgcn_alignbit(w[1], w[0], pos & 31u);
          const uint32_t q = ffbl(x);  // 0xFFFFFFFF when the run is longer than the window
          maxq = max(maxq, q);
          const uint32_t q1 = q + 1;
          const uint32_t d = (q << fs) | __builtin_amdgcn_ubfe(x, q1, fs);
          acc += (d >> 1) ^ (0u - (d & 1u));
          pos += q1 + fs;
          v[j] = acc;
        }
        r[i / 2] = __builtin_amdgcn_perm(v[1], v[0], 0x05040100u);
      }
      // exact only if no code ran past its 32-bit window; the end must be
      // where the parse put it
      if (maxq > 31 - fs || pos != end - 32 * w0) fast = false;
      agg = acc & 0xFFFFu;
    }
    if (CS == 2) {
      const int pf = __shfl_xor((int)fast, 1);
      fast = fast && pf;
    }
    // ---- general lanes: the element by the exact runtime loop ----
    if (active && !fast) agg = decode_general<false>(rd, start, n, 0, nullptr, CS, be, ulsb);

    stamp(2);
    // ---- scan of the elements within the tile (per component: stride CS) ----
    scan_buf[tid] = agg;
    __syncthreads();
    for (uint32_t d = CS; d < kTile; d <<= 1) {
      const uint32_t v = tid >= d ? combine(scan_buf[tid - d], scan_buf[tid]) : scan_buf[tid];
      __syncthreads();
      scan_buf[tid] = v;
      __syncthreads();
    }
    // ---- tile carry: decoupled look-back over the stream's earlier tiles ----
    if (tid == 0) {
      uint32_t a0 = scan_buf[kcount - CS], a1 = CS == 2 ? scan_buf[kcount - 1] : 0u;  // tile aggregates
      uint32_t e0, e1;  // exclusive prefix of this tile
      if (lt == 0) {
        // codec.h:81-86: the 16-bit initial value of each component
        const uint32_t lo = stream_word(base, nbytes, 0), hi = stream_word(base, nbytes, 1);
        const uint64_t x = ((uint64_t)hi << 32 | lo) >> (8 * mis);
        e0 = kSet | (uint32_t)(x & 0xFFFFu);
        e1 = kSet | (uint32_t)((x >> 16) & 0xFFFFu);
      } else {
        __hip_atomic_store(&p.tile_state[t], pack_state(a0, a1, kFlagAgg), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
        uint32_t x0 = 0, x1 = 0;  // identity
        for (uint32_t j = t - 1;; --j) {
          uint64_t s;
          do {
            s = __hip_atomic_load(&p.tile_state[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (!(s >> 62)) __builtin_amdgcn_s_sleep(1);
          } while (!(s >> 62));
          const uint32_t s0 = (uint32_t)(s & 0x1FFFFu), s1 = (uint32_t)((s >> 17) & 0x1FFFFu);
          x0 = combine(s0, x0);
          x1 = combine(s1, x1);
          if ((s >> 62) == 2) break;
        }
        e0 = x0;
        e1 = x1;
      }
      __hip_atomic_store(&p.tile_state[t], pack_state(combine(e0, a0), combine(e1, a1), kFlagIncl),
                         __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      sh_carry[0] = e0;
      sh_carry[1] = e1;
    }
    __syncthreads();
    // value before this lane's sub-block
    const uint32_t excl = tid >= CS ? scan_buf[tid - CS] : 0u;
    const uint32_t carry = combine(sh_carry[comp], excl) & 0xFFFFu;

    stamp(3);
    // ---- stores ----
    if (fast) {
      const uint32_t c2 = carry * 0x10001u;
#pragma unroll
      for (uint32_t i = 0; i < BS / 2; ++i) {
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        r[i] = px_write2<SH>(__builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, r[i]) + __builtin_bit_cast(us2, c2)),
                             selbe, ulsb);
      }
      if (p.dbg & 2) {
#pragma unroll
        for (uint32_t i = 0; i < BS / 2; ++i) {
          out[cbase + comp + CS * 2 * i] = (uint16_t)r[i];
          out[cbase + comp + CS * (2 * i + 1)] = (uint16_t)(r[i] >> 16);
        }
      } else if constexpr (CS == 1) {
        uint4* o = reinterpret_cast<uint4*>(out + (size_t)k * BS);
#pragma unroll
        for (uint32_t i = 0; i < BS / 8; ++i) o[i] = make_uint4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
      } else {
        // lane 2c holds component 0 of chunk c, lane 2c+1 component 1; the
        // chunk interleaves them.  The even lane writes chunk dwords
        // [0, BS/2), the odd lane [BS/2, BS); dword j = (c0[j], c1[j]).
        const bool odd = tid & 1u;
        uint32_t o32[BS / 2];
#pragma unroll
        for (uint32_t i = 0; i < BS / 4; ++i) {
          const uint32_t own = odd ? r[BS / 4 + i] : r[i];
          const uint32_t send = odd ? r[i] : r[BS / 4 + i];
          const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);  // swap pairs
          const uint32_t c0 = odd ? recv : own, c1 = odd ? own : recv;
          o32[2 * i] = __builtin_amdgcn_perm(c1, c0, 0x05040100u);      // (c0.lo, c1.lo)
          o32[2 * i + 1] = __builtin_amdgcn_perm(c1, c0, 0x07060302u);  // (c0.hi, c1.hi)
        }
        uint4* o = reinterpret_cast<uint4*>(out + (size_t)(k / 2) * chunk_len + (odd ? BS : 0));
#pragma unroll
        for (uint32_t i = 0; i < BS / 8; ++i)
          o[i] = make_uint4(o32[4 * i], o32[4 * i + 1], o32[4 * i + 2], o32[4 * i + 3]);
      }
    } else if (active) {
      decode_general<true>(rd, start, n, carry, out + cbase + comp, CS, be, ulsb);
    }
    __syncthreads();  // (stage and scan_buf are reused by the next tile)
    stamp(4);
    if (timing && tid == 0) atomicAdd(&g_dec2_diag[7], 1ull);
  }
}

using ExtractKernel = void (*)(ExtractParams);

template <uint32_t CS, bool SH>
ExtractKernel extract_kernel_for(uint32_t bs) {
  switch (bs) {
    case 16: return rpp_extract_kernel<CS, 16, SH>;
    case 32: return rpp_extract_kernel<CS, 32, SH>;
    case 64: return rpp_extract_kernel<CS, 64, SH>;
    case 128: return rpp_extract_kernel<CS, 128, SH>;
    default: return nullptr;
  }
}

// The two-stage decode is selected by RICEPP_DECODE=two-stage; the default is
// the fused one-wave-per-stream kernel (rpp_decode_kernel).  Measured on MI355X
// (DESIGN.md section 4): the parse pass alone costs 86 VALU per 128-sample
// sub-block and is VALU-bound at 74 % (196 us for 4096 x 64 KiB), about what
// the fused kernel needs for parse AND values (258 us), whose value work
// hides in the parse chain's latency; so splitting the passes does not pay
// on this hardware.  The path stays for unaligned-offset and long-stream
// experiments.
bool two_stage(const rpp_config* cfg) {
  const char* e = getenv("RICEPP_DECODE");
  if (!e || std::string(e) != "two-stage") return false;
  return cfg->block_size == 16 || cfg->block_size == 32 || cfg->block_size == 64 || cfg->block_size == 128;
}

}  // namespace

extern "C" {

// diagnostics only (not in the C ABI header): the extraction phase timers
int rpp_diag_read(unsigned long long* out8, int reset) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dec2_diag), sizeof(g_dec2_diag)) != hipSuccess) return RPP_HIP_ERROR;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dec2_diag), z, sizeof(z)) != hipSuccess) return RPP_HIP_ERROR;
  }
  return RPP_OK;
}

uint64_t rpp_decode_workspace_bytes(const rpp_config* cfg, uint64_t total_samples, uint32_t nblocks) {
  if (rpp_check_config(cfg) != RPP_OK) return 0;
  return layout(cfg, total_samples, nblocks, nullptr).bytes;
}

int rpp_decode_batch_ws(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, uint64_t total_samples, void* d_workspace,
                        uint64_t workspace_bytes, void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_in_bytes || !d_out || !d_out_offsets || !d_n_samples || !d_status)
    return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  if (!two_stage(cfg))
    return rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                             d_n_samples, d_status, s);
  const Workspace w = layout(cfg, total_samples, nblocks, static_cast<uint8_t*>(d_workspace));
  if (!d_workspace || workspace_bytes < w.bytes) return RPP_INVALID_ARGUMENT;
  const uint32_t chunk_len = cfg->block_size * cfg->component_stream_count;
  hipLaunchKernelGGL(rpp_dec_count_kernel, dim3((nblocks + 256) / 256), dim3(256), 0, s, d_n_samples, nblocks,
                     chunk_len, cfg->component_stream_count, w.sb_cnt, w.tile_cnt);
  if ((st = rpp_exclusive_scan_u64(w.sb_cnt, (uint64_t)nblocks + 1, w.sb_base, s)) != RPP_OK) return st;
  if ((st = rpp_exclusive_scan_u64(w.tile_cnt, (uint64_t)nblocks + 1, w.tile_base, s)) != RPP_OK) return st;
  hipLaunchKernelGGL(rpp_dec_tile_map_kernel, dim3((nblocks + 255) / 256), dim3(256), 0, s, w.tile_base, nblocks,
                     w.tile_map);
  if (hipMemsetAsync(w.tile_state, 0, w.max_tiles * 8, s) != hipSuccess) return RPP_HIP_ERROR;
  if (hipMemsetAsync(w.counter, 0, 4, s) != hipSuccess) return RPP_HIP_ERROR;
  st = rpp_internal::launch_parse(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_n_samples, w.sb_base, w.sb_pos,
                                  d_status, s);
  if (st != RPP_OK) return st;
  const bool sh = cfg->unused_lsb_count != 0;
  const ExtractKernel k = cfg->component_stream_count == 1
                              ? (sh ? extract_kernel_for<1, true>(cfg->block_size)
                                    : extract_kernel_for<1, false>(cfg->block_size))
                              : (sh ? extract_kernel_for<2, true>(cfg->block_size)
                                    : extract_kernel_for<2, false>(cfg->block_size));
  ExtractParams p{d_in, d_in_offsets, d_in_bytes, d_n_samples, d_out, d_out_offsets, d_status, w.sb_pos, w.sb_base,
                  w.tile_base, w.tile_map, w.tile_state, w.counter, nblocks, cfg->block_size,
                  cfg->big_endian ? 1u : 0u, cfg->unused_lsb_count, 0u};
  if (const char* e = getenv("RICEPP_DEC2_DBG")) p.dbg = (uint32_t)atoi(e);
  const uint32_t grid = (uint32_t)std::min<uint64_t>(w.max_tiles, kMaxExtractGrid);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kTile), 0, s, p);
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

int rpp_decode_batch(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                     const uint64_t* d_n_samples, int32_t* d_status, void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_in_bytes || !d_out || !d_out_offsets || !d_n_samples || !d_status)
    return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  if (!two_stage(cfg))
    return rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                             d_n_samples, d_status, s);
  // the workspace size needs the batch's sample count: read the counts
  // (this call synchronises the stream; rpp_decode_batch_ws does not)
  uint64_t* h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h), (size_t)nblocks * 8, hipHostMallocDefault) != hipSuccess)
    return RPP_HIP_ERROR;
  uint64_t total = 0;
  bool ok = hipMemcpyAsync(h, d_n_samples, (size_t)nblocks * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess;
  if (ok)
    for (uint32_t i = 0; i < nblocks; ++i) total += h[i] < RPP_MAX_STREAM_SAMPLES ? h[i] : 0;
  (void)hipHostFree(h);
  if (!ok) return RPP_HIP_ERROR;
  const uint64_t bytes = rpp_decode_workspace_bytes(cfg, total, nblocks);
  void* ws = nullptr;
  if (hipMallocAsync(&ws, bytes, s) != hipSuccess) return RPP_HIP_ERROR;
  st = rpp_decode_batch_ws(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets, d_n_samples, d_status,
                           total, ws, bytes, s);
  (void)hipFreeAsync(ws, s);
  return st;
}

}  // extern "C"
