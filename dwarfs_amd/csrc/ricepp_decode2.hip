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
#include <map>
#include <mutex>
#include <string>

#include "ricepp_amd.h"
#include "ricepp_internal.h"

namespace {

constexpr uint32_t kTile = 256;          // sub-blocks (lanes) per tile
// The stream's words of a tile in LDS.  64 KiB: a tile's 256 sub-blocks at
// bs 128 take up to 16 bits per sample (with 36 KiB, generator data -- 14
// bits per sample -- left 40 % of each tile's lanes unstaged, on global
// reads), two workgroups per CU.  48 KiB: three workgroups per CU (<= 168
// VGPRs), tiles up to ~12 bits per sample staged whole -- for batches of many
// tiles, where throughput, not one tile's latency, is the time: configs[3]
// mix decode 50.8 -> 47.3 ms, a lone 16 MiB generator stream 0.95 -> 1.03 ms
// (profiles/r05_extract_stage_ab.jsonl)
constexpr uint32_t kStageWords = 16384;
constexpr uint32_t kStageWordsMany = 12288;
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
  uint32_t* tile_map;   // [max_tiles] stream of the t-th tile handed out
  uint32_t* tile_lt;    // [max_tiles] its index within the stream
  uint64_t* lvl_cnt;    // [levels + 1] streams with more than l tiles
  uint64_t* lvl_base;   // [levels + 1]
  uint32_t* sb_pos;     // [max_sb + B] bit positions from the stream's 4-aligned base, low 32 bits
  uint32_t* tile_hi;    // [max_tiles] high 32 bits of the position of each tile's first sub-block
  uint32_t* counter;    // [1]
  // segmented decode (L != 0)
  uint64_t* ucnt;       // [B + 1] units per stream
  uint64_t* unit_base;  // [B + 1]
  uint32_t* unit_map;   // [U_max]
  uint64_t* pl_cnt;     // [U_max + 1] list capacity per unit
  uint64_t* pl_base;    // [U_max + 1]
  uint32_t* plist;      // [list entries]
  uint32_t* ovr;        // [U_max * kSegOvr]
  uint32_t* ustate;     // [U_max * 4]
  uint32_t* ulo;        // [U_max]
  uint32_t* uov;        // [U_max]
  uint32_t* uhit;       // [2 U_max]: overshoot index, list index
  uint32_t* sst;        // [B]
  uint32_t* sflags;     // [B]
  uint32_t* queue;      // [1]
  uint64_t* cnt2;       // [U_max + 1] exact positions per unit
  uint64_t* off2;       // [U_max + 1]
  uint32_t* guard;      // [2] 1: the batch exceeds the promised sizes (rpp_seg_plan_kernel); the stage choice
  uint64_t bytes;
  uint64_t max_tiles;
  uint64_t units_max;
  uint32_t levels;      // most tiles a stream can have
};

__host__ __device__ inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// diagnostics (RICEPP_DEC2_DBG & 4): per-phase cycle sums of the extraction
// tiles (wave 0 of each workgroup), read by rpp_diag_read
__device__ unsigned long long g_dec2_diag[8];
// segmented decode counters (rpp_seg_diag_read): units that met the exact
// chain at once, reruns requested, serial passes, streams left to the fused kernel
__device__ unsigned long long g_seg_diag[8];
__device__ __forceinline__ uint64_t clk() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

Workspace layout(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples, uint32_t nblocks,
                 uint32_t L, uint8_t* base) {
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
  w.tile_lt = reinterpret_cast<uint32_t*>(take(max_tiles * 4));
  w.levels = (uint32_t)((max_stream_samples / cfg->block_size + 2) / kTile + 1);
  w.lvl_cnt = reinterpret_cast<uint64_t*>(take(((uint64_t)w.levels + 1) * 8));
  w.lvl_base = reinterpret_cast<uint64_t*>(take(((uint64_t)w.levels + 1) * 8));
  w.sb_pos = reinterpret_cast<uint32_t*>(take((max_sb + B) * 4));
  w.tile_hi = reinterpret_cast<uint32_t*>(take(max_tiles * 4));
  w.counter = reinterpret_cast<uint32_t*>(take(256));
  w.guard = reinterpret_cast<uint32_t*>(take(256));
  w.max_tiles = max_tiles;
  if (L) {
    // header bits of all streams: at most their worst-case sizes (seg_last_bit)
    const uint64_t bits = 8 * rpp_worst_case_bytes(cfg, total_samples) + 128 * B;
    const uint64_t U = B + (bits >> L) + 1;
    const uint64_t entries = bits / std::max<uint32_t>(cfg->block_size, 32) + 68 * U;
    w.units_max = U;
    w.ucnt = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
    w.unit_base = reinterpret_cast<uint64_t*>(take((B + 1) * 8));
    w.unit_map = reinterpret_cast<uint32_t*>(take(U * 4));
    w.pl_cnt = reinterpret_cast<uint64_t*>(take((U + 1) * 8));
    w.pl_base = reinterpret_cast<uint64_t*>(take((U + 1) * 8));
    w.plist = reinterpret_cast<uint32_t*>(take(entries * 4));
    w.ovr = reinterpret_cast<uint32_t*>(take(U * rpp_internal::kSegOvr * 4));
    w.ustate = reinterpret_cast<uint32_t*>(take(U * rpp_internal::kUsWords * 4));
    w.ulo = reinterpret_cast<uint32_t*>(take(U * 4));
    w.uov = reinterpret_cast<uint32_t*>(take(U * 4));
    w.uhit = reinterpret_cast<uint32_t*>(take(U * 8));
    w.sst = reinterpret_cast<uint32_t*>(take(B * 4));
    w.sflags = reinterpret_cast<uint32_t*>(take(B * 4));
    w.queue = reinterpret_cast<uint32_t*>(take(256));
    w.cnt2 = reinterpret_cast<uint64_t*>(take((U + 1) * 8));
    w.off2 = reinterpret_cast<uint64_t*>(take((U + 1) * 8));
  }
  w.bytes = off;
  return w;
}

// Tiles are handed out level by level: tile l of every stream before tile
// l + 1 of any (a stream's tiles stay in order, as the look-back needs, and a
// long stream has few tiles in flight at once, so its inclusive prefixes keep
// up).  One workgroup per level: streams with more than l tiles, counted, then
// ranked by a block scan.
constexpr uint32_t kLvlThreads = 256;
__device__ __forceinline__ uint32_t block_excl_scan_flag(bool f, uint32_t* sh, uint32_t& total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint64_t m = __ballot(f);
  const uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (lane == 0) sh[wv] = (uint32_t)__builtin_popcountll(m);
  __syncthreads();
  uint32_t off = 0;
  total = 0;
  for (uint32_t i = 0; i < kLvlThreads / 64; ++i) {
    off += i < wv ? sh[i] : 0u;
    total += sh[i];
  }
  __syncthreads();
  return off + before;
}

__global__ __launch_bounds__(kLvlThreads) void rpp_dec_level_map_kernel(const uint64_t* tile_cnt, uint32_t nblocks,
                                                                        uint32_t levels, const uint64_t* lvl_base,
                                                                        uint32_t* tile_map, uint32_t* tile_lt) {
  __shared__ uint32_t sh[kLvlThreads / 64];
  const uint32_t l = blockIdx.x;
  if (l >= levels) return;
  uint64_t r = lvl_base[l];
  for (uint32_t b0 = 0; b0 < nblocks; b0 += kLvlThreads) {
    const uint32_t b = b0 + threadIdx.x;
    const bool f = b < nblocks && tile_cnt[b] > l;
    uint32_t total;
    const uint32_t at = block_excl_scan_flag(f, sh, total);
    if (f) {
      tile_map[r + at] = b;
      tile_lt[r + at] = l;
    }
    r += total;
  }
}

struct ExtractParams {
  const uint8_t* in;
  const uint64_t* in_off;
  const uint64_t* in_bytes;
  const uint64_t* n_samples;
  uint16_t* out;
  const uint64_t* out_off;
  int32_t* status;        // of the parse pass: streams that failed are skipped; RPP_INTERNAL_ERROR on a stalled look-back
  const uint32_t* sb_pos;
  const uint32_t* tile_hi;
  const uint64_t* sb_base;
  const uint64_t* tile_base;
  const uint32_t* tile_map;
  const uint32_t* tile_lt;
  const uint64_t* n_tiles;  // tiles handed out (the level map's total)
  uint64_t* tile_state;
  uint32_t* counter;
  uint32_t nblocks;
  uint32_t bs, be, ulsb;
  uint32_t dbg;  // rpp_decode_options::test_flags (RPP_TEST_*)
  // (batches of many tiles: both stage sizes are launched, and the one
  // rpp_seg_plan_kernel did not choose returns at once; nullptr: run)
  const uint32_t* stage_sel;
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

// Asynchronous global -> LDS copy (global_load_lds_dword): lane l's 4 bytes
// land at LDS byte address m0 + 4 l; retired by s_waitcnt vmcnt(0).
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t m0) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(m0) : "memory");
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
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
      if (pos > 8u * rd.nbytes + 64u) break;  // (never for a parsed start: a bug may not hang the GPU)
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

// BS: the block size of the fast lanes' unrolled decode (16..128); BS = 0 is
// any other block size (the run-time p.bs), decoded by general lanes only.
template <uint32_t CS, uint32_t BS, bool SH, uint32_t STAGE>
__global__ __launch_bounds__(kTile, STAGE == kStageWords ? 2 : 3) void rpp_extract_kernel(ExtractParams p) {
  __shared__ __attribute__((aligned(16))) uint32_t stage[STAGE + kStagePad];
  __shared__ uint32_t scan_buf[kTile];
  __shared__ uint32_t sh_tile, sh_carry[2], sh_min;
  __shared__ uint32_t wtot[kTile / 64][2];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = __lane_id();
  const uint32_t be = p.be, ulsb = p.ulsb;
  const uint32_t selbe = be ? 0x02030001u : 0x03020100u;  // byte-swap each half
  const uint32_t chunk_len = CS * (BS ? BS : p.bs);
  const uint64_t total_tiles = *p.n_tiles;
  if (p.stage_sel && *p.stage_sel != (STAGE == kStageWords ? 1u : 0u)) return;  // (uniform)

  const bool timing = (p.dbg & RPP_TEST_PHASE_TIMERS) && tid < 64;
  // fault injection: tile 1 of every stream never publishes, its successors
  // give up after 2^10 polls instead of 2^22
  const bool stall = p.dbg & RPP_TEST_LOOKBACK_STALL;
  const uint32_t spin_max = stall ? (1u << 10) : (1u << 22);
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
    const uint32_t tg = sh_tile;
    if (tg >= total_tiles) return;  // (uniform)
    const uint32_t b = p.tile_map[tg];
    const uint32_t lt = p.tile_lt[tg];
    const uint32_t t = (uint32_t)p.tile_base[b] + lt;  // the tile's state slot (stream-major)
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
    // the tile's frame: its words from the one holding its first sub-block's
    // header (sb_pos holds the positions' low 32 bits, tile_hi the high bits
    // of the tile's first one; a tile spans a few Mbit at most, so the
    // positions relative to it are the low bits' differences)
    const uint64_t wt = ((uint64_t)p.tile_hi[t] << 27) | (pos_tab[k0] >> 5);
    const uint32_t fbit = 32u * (uint32_t)wt;  // (the frame's first bit, mod 2^32)
    const uint8_t* tbase = base + 4 * wt;
    const uint32_t tbytes =
        nbytes > 4 * wt ? (uint32_t)min<uint64_t>(nbytes - 4 * wt, rpp_internal::kSegWinBytes) : 0u;
    const uint32_t k = k0 + tid;
    const bool active = tid < kcount;
    const uint32_t start = active ? pos_tab[k] - fbit : 0u;
    const uint32_t end = active ? pos_tab[k + 1] - fbit : 0u;
    const uint32_t comp = k % CS;
    const uint32_t cbase = (k / CS) * chunk_len;
    const uint32_t n = active ? min(N - cbase, chunk_len) / CS : 0u;
    uint16_t* const out = p.out + p.out_off[b];

    stamp(0);
    // ---- stage the tile's words: asynchronous global -> LDS copies (no
    //      registers held: every wave issues its 256-byte chunks back to
    //      back), the chunk holding the stream's end word by word (zero past
    //      the last byte) ----
    const uint32_t w0 = 0;
    const uint32_t wend = ((pos_tab[k0 + kcount] - fbit) >> 5) + 2;
    const uint32_t nst = min(wend - w0, STAGE);
    {
      const uint32_t l = tid & 63u, wv = tid >> 6;
      for (uint32_t c = wv; 64 * c < nst; c += kTile / 64) {
        const uint32_t wq = w0 + 64 * c;
        if (4 * (wq + 64) <= tbytes) {
          glds4(tbase + 4 * (wq + l), __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)&stage[64 * c]));
        } else {
          stage[64 * c + l] = stream_word(tbase, tbytes, wq + l);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    stamp(1);
    const Reader rd{stage, w0, nst, tbase, tbytes};

    // ---- fast lanes: Rice, a full sub-block, staged, every code <= 32 bits ----
    uint32_t hdr = 0;
    if (active) hdr = rd.peek32(start) & 15u;
    bool fast = BS != 0 && active && hdr != 0 && hdr != 15 && n == BS && (end >> 5) + 1 < w0 + nst &&
                !(p.dbg & RPP_TEST_NO_FAST_LANES);
    // pairs share one store path (the shuffle outside any condition: a
    // short-circuit && would run it on the fast lanes only)
    if (CS == 2) {
      const int pf = __shfl_xor((int)fast, 1);
      fast = fast && pf;
    }
    uint32_t r[BS ? BS / 2 : 1];
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
    // ---- scan of the elements within the tile (per component: stride CS):
    //      a shuffle scan per wave, then the wave totals through LDS ----
    {
      const uint32_t l = tid & 63u, wv = tid >> 6;
      uint32_t v = agg;
#pragma unroll
      for (uint32_t d = CS; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)v, d);
        if (l >= d) v = combine(y, v);
      }
      if (l >= 64 - CS) wtot[wv][l - (64 - CS)] = v;
      __syncthreads();
      uint32_t pre = 0;
      for (uint32_t w = 0; w < wv; ++w) pre = combine(pre, wtot[w][comp]);
      scan_buf[tid] = combine(pre, v);
      __syncthreads();
    }
    // ---- tile carry: decoupled look-back over the stream's earlier tiles,
    //      64 predecessors at a time (one per lane of wave 0): a long stream
    //      has thousands of tiles in flight at once ----
    if (tid < 64) {
      const uint32_t a0 = scan_buf[kcount - CS], a1 = CS == 2 ? scan_buf[kcount - 1] : 0u;  // tile aggregates
      uint32_t e0, e1;  // exclusive prefix of this tile
      if (lt == 0) {
        // codec.h:81-86: the 16-bit initial value of each component
        const uint32_t lo = stream_word(base, nbytes, 0), hi = stream_word(base, nbytes, 1);
        const uint64_t x = ((uint64_t)hi << 32 | lo) >> (8 * mis);
        e0 = kSet | (uint32_t)(x & 0xFFFFu);
        e1 = kSet | (uint32_t)((x >> 16) & 0xFFFFu);
      } else {
        if (tid == 0 && !(stall && lt == 1))
          __hip_atomic_store(&p.tile_state[t], pack_state(a0, a1, kFlagAgg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        uint32_t x0 = 0, x1 = 0;  // identity: the tiles after the current window
        const uint32_t tfirst = t - lt;  // the stream's first tile (publishes its inclusive prefix)
        for (uint32_t jt = t - 1;; jt -= 64) {
          const bool valid = tid <= jt - tfirst;
          uint64_t s = 0;
          if (valid) {
            // (relaxed: the state word carries its payload, no other data is
            // published with it; the load is coherent at agent scope (sc1).
            // Bounded: a predecessor that never publishes is a bug or a
            // stalled GPU.  The stream is then marked RPP_INTERNAL_ERROR --
            // before anything is built on the missing prefix -- and the tile
            // goes on with an identity prefix only so that the grid drains.)
            for (uint32_t spin = 0;; ++spin) {
              s = __hip_atomic_load(&p.tile_state[jt - tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (s >> 62) break;
              if (spin == spin_max) {
                __hip_atomic_store(&p.status[b], (int32_t)RPP_INTERNAL_ERROR, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd(&g_dec2_diag[6], 1ull);
                s = kFlagIncl;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
            }
          }
          const uint64_t incl = __ballot(valid && (s >> 62) == 2);
          const uint64_t vm = __ballot(valid);
          const int k = incl ? __builtin_ctzll(incl) : 63 - __builtin_clzll(vm);
          uint32_t y0 = 0, y1 = 0;  // the window, oldest tile (lane k) first
          const uint32_t slo = (uint32_t)s, shi = (uint32_t)(s >> 32);
          for (int l = k; l >= 0; --l) {
            const uint64_t sl = ((uint64_t)readlane(shi, l) << 32) | readlane(slo, l);
            y0 = combine(y0, (uint32_t)(sl & 0x1FFFFu));
            y1 = combine(y1, (uint32_t)((sl >> 17) & 0x1FFFFu));
          }
          x0 = combine(y0, x0);
          x1 = combine(y1, x1);
          if (incl) break;
        }
        e0 = x0;
        e1 = x1;
      }
      if (tid == 0 && !(stall && lt == 1)) {
        __hip_atomic_store(&p.tile_state[t], pack_state(combine(e0, a0), combine(e1, a1), kFlagIncl),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (tid == 0) {
        sh_carry[0] = e0;
        sh_carry[1] = e1;
      }
    }
    __syncthreads();
    // value before this lane's sub-block
    const uint32_t excl = tid >= CS ? scan_buf[tid - CS] : 0u;
    const uint32_t carry = combine(sh_carry[comp], excl) & 0xFFFFu;

    stamp(3);
    // ---- stores ----
    // general lanes first: they read the staged words once more
    if (active && !fast) decode_general<true>(rd, start, n, carry, out + cbase + comp, CS, be, ulsb);
    // fast lanes: their BS samples, in output order (lane k's BS samples are
    // output samples [k BS, (k+1) BS) of the tile for either CS)
    uint32_t o32[CS == 1 || !BS ? 1 : BS / 2];  // (cs 1: the words are r itself)
    if (fast) {
      const uint32_t c2 = carry * 0x10001u;
#pragma unroll
      for (uint32_t i = 0; i < BS / 2; ++i) {
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        r[i] = px_write2<SH>(__builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, r[i]) + __builtin_bit_cast(us2, c2)),
                             selbe, ulsb);
      }
      if constexpr (CS == 2) {
        // lane 2c holds component 0 of chunk c, lane 2c+1 component 1; the
        // chunk interleaves them.  The even lane takes chunk dwords [0, BS/2),
        // the odd lane [BS/2, BS); dword j = (c0[j], c1[j]).
        const bool odd = tid & 1u;
#pragma unroll
        for (uint32_t i = 0; i < BS / 4; ++i) {
          const uint32_t own = odd ? r[BS / 4 + i] : r[i];
          const uint32_t send = odd ? r[i] : r[BS / 4 + i];
          const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);  // swap pairs
          const uint32_t c0 = odd ? recv : own, c1 = odd ? own : recv;
          o32[2 * i] = __builtin_amdgcn_perm(c1, c0, 0x05040100u);      // (c0.lo, c1.lo)
          o32[2 * i + 1] = __builtin_amdgcn_perm(c1, c0, 0x07060302u);  // (c0.hi, c1.hi)
        }
      }
    }
    auto word = [&](uint32_t i) -> uint32_t {
      if constexpr (CS == 1) return r[i];
      else return o32[i];
    };
    if constexpr (BS >= 64) {
      // Through LDS, so that every store instruction writes whole 128-byte
      // lines: each wave puts 128 bytes of each lane in a row of its own
      // quarter of the stage (rows padded to 144 bytes), then eight lanes
      // store one row.
      constexpr uint32_t kRow = 36;
      __syncthreads();  // (the staged words are read no more)
      const uint32_t l = tid & 63u, wv = tid >> 6;
      uint32_t* tr = stage + wv * 64 * kRow;
      const uint64_t fm = __ballot(fast);
      uint16_t* const wout = out + (size_t)(k0 + 64 * wv) * BS;
#pragma unroll
      for (uint32_t h = 0; h < BS / 64; ++h) {
        if (fast) {
#pragma unroll
          for (uint32_t j = 0; j < 8; ++j)
            *reinterpret_cast<uint4*>(tr + l * kRow + 4 * j) =
                make_uint4(word(32 * h + 4 * j), word(32 * h + 4 * j + 1), word(32 * h + 4 * j + 2), word(32 * h + 4 * j + 3));
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
          const uint32_t row = 8 * i + (l >> 3), c = l & 7u;
          if ((fm >> row) & 1u)
            *reinterpret_cast<uint4*>(wout + (size_t)row * BS + 64 * h + 8 * c) =
                *reinterpret_cast<const uint4*>(tr + row * kRow + 4 * c);
        }
        asm volatile("" ::: "memory");
      }
    } else if (fast) {
      uint4* o = reinterpret_cast<uint4*>(out + (size_t)k * BS);
#pragma unroll
      for (uint32_t i = 0; i < BS / 8; ++i) o[i] = make_uint4(word(4 * i), word(4 * i + 1), word(4 * i + 2), word(4 * i + 3));
    }
    __syncthreads();  // (stage and scan_buf are reused by the next tile)
    stamp(4);
    if (timing && tid == 0) atomicAdd(&g_dec2_diag[7], 1ull);
  }
}

// ===========================================================================
// Segmented decode of long streams: units, stitch, positions, ragged tail
// (the scheme: ricepp_internal.h; the parse of the units: rpp_parse_kernel
// with SEG = true in ricepp_kernels.hip).
// ===========================================================================
using rpp_internal::kSegNone;
using rpp_internal::kSegOvr;

struct SegArgs {
  rpp_internal::SegView sv;
  const uint8_t* in;
  const uint64_t* in_off;
  const uint64_t* in_bytes;
  const uint64_t* n_samples;
  const uint64_t* sb_base;
  uint32_t* sb_pos;
  uint32_t* tile_hi;     // (the sb_pos entries of tile starts also write their high bits here)
  const uint64_t* tile_base;
  int32_t* status;
  uint64_t* cnt;  // [U_max + 1] exact positions per unit
  uint64_t* off;  // [U_max + 1] their exclusive scan
  uint32_t* uhit; // [U_max] first overshoot header of the unit before that is a header of the unit
  const uint32_t* guard;  // rpp_seg_plan_kernel's verdict: 1 = no stream is split
  uint32_t nblocks, bs, cs;
};

__device__ __forceinline__ bool seg_stream_ok(uint64_t n, uint64_t nb, uint32_t cs) {
  return rpp_internal::seg_stream_fits(n, nb, cs);
}

// unit -> stream, and the list capacity of each unit of a split stream: one
// header per max(bs, 32) bits of its region [j 2^L, min((j+1) 2^L, last bit
// + 1)), i.e. the sub-blocks of data that codes to >= 1 bit per sample (>= 2
// for bs 16; below that the stream goes to the fused kernel), a multiple of 4
// entries.  One thread per unit (its stream by binary search of unit_base,
// where every stream has at least one unit); a thread per stream looping over
// its units took 80 us for one 16 MiB stream.
__global__ void rpp_seg_map_kernel(SegArgs a, uint32_t* unit_map, uint64_t* pl_cnt) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= a.sv.units_max || u >= a.sv.unit_base[a.nblocks]) return;
  uint32_t lo = 0, hi = a.nblocks - 1;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo + 1) / 2;
    if (a.sv.unit_base[mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  const uint32_t i = lo;
  const uint64_t u0 = a.sv.unit_base[i], nu = a.sv.unit_base[i + 1] - u0, k = u - u0;
  unit_map[u] = i;
  uint64_t cap = 0;
  if (nu > 1) {
    const uint32_t L = a.sv.seg_log2;
    const uint64_t Eend =
        rpp_internal::seg_last_bit((uint32_t)(a.in_off[i] & 3u), a.in_bytes[i], a.n_samples[i], a.bs, a.cs);
    const uint64_t S = k << L, E = k + 1 == nu ? Eend + 1 : S + (1ull << L);
    cap = align_up((E - S) / max(a.bs, 32u) + 64, 4);
  }
  pl_cnt[u] = cap;
}

struct UnitGeo {
  uint32_t b, u0, nu;
  uint64_t S, E;  // the unit's region [S, E) of the stream (bits from its 4-aligned base)
};
__device__ __forceinline__ UnitGeo unit_geo(const SegArgs& a, uint32_t u) {
  UnitGeo g;
  g.b = a.sv.unit_map[u];
  g.u0 = (uint32_t)a.sv.unit_base[g.b];
  g.nu = (uint32_t)a.sv.unit_base[g.b + 1] - g.u0;
  const uint32_t j = u - g.u0, L = a.sv.seg_log2;
  g.S = (uint64_t)j << L;
  g.E = g.S + (1ull << L);
  if (g.nu > 1 && j + 1 == g.nu)
    g.E = rpp_internal::seg_last_bit((uint32_t)(a.in_off[g.b] & 3u), a.in_bytes[g.b], a.n_samples[g.b], a.bs, a.cs) + 1;
  return g;
}

__device__ __forceinline__ uint32_t us_word(const SegArgs& a, uint32_t u, uint32_t w) {
  return a.sv.ustate[rpp_internal::kUsWords * u + w];
}

// index of `pos` in unit u's position list (ascending), or kSegNone
__device__ __forceinline__ uint32_t list_find(const SegArgs& a, uint32_t u, uint32_t pos) {
  const uint32_t* l = a.sv.plist + a.sv.pl_base[u];
  uint32_t lo = 0, hi = us_word(a, u, rpp_internal::kUsNpos);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (l[mid] < pos) lo = mid + 1;
    else hi = mid;
  }
  return lo < us_word(a, u, rpp_internal::kUsNpos) && l[lo] == pos ? lo : kSegNone;
}

// One thread per unit of a split stream (not yet resolved): the first of the
// previous unit's overshoot headers that is also a header of this unit's
// chain (i, and its index in the unit's list).
__global__ void rpp_seg_hit_kernel(SegArgs a) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= a.sv.units_max || u >= (uint32_t)a.sv.unit_base[a.nblocks]) return;
  const uint32_t b = a.sv.unit_map[u];
  const uint32_t u0 = (uint32_t)a.sv.unit_base[b], nu = (uint32_t)a.sv.unit_base[b + 1] - u0;
  const uint32_t j = u - u0;
  if (nu <= 1 || j == 0 || j < a.sv.sst[b]) return;
  const uint32_t prev = u - 1;
  const uint32_t np = us_word(a, prev, rpp_internal::kUsNovr);
  uint32_t hit = kSegNone, at = kSegNone;
  for (uint32_t i = 0; i < np && hit == kSegNone; ++i) {
    at = list_find(a, u, a.sv.ovr[kSegOvr * prev + i]);
    if (at != kSegNone) hit = i;
  }
  a.uhit[u] = hit;
  a.uhit[a.sv.units_max + u] = at;
}

// One wave per split stream, 64 units at a time from the first unresolved
// one: where does the exact chain (the previous unit's, by induction) meet
// the unit's own chain?  At the previous unit's overshoot header uhit: from
// there on the unit's positions are exact.  The first unit without a meeting
// decides the rest: if the previous chain stopped early the stream ended
// there; else the unit is parsed again from the last overshoot header (a
// rerun pass) and the stitch resumes there next time.  ulo = the list index
// where the unit's exact positions start.
// Before a rerun pass every later unit without a meeting whose predecessor
// met its own is rerun as well, from that predecessor's last overshoot
// header: exact once the units before are, so one rerun pass settles all of
// a stream's isolated failed guesses.  (Rerunning also the units after a
// failed one measured a cascade: a wrong chain that never meets the true one
// hands its successor a wrong start, breaking a good guess in every pass.)  A rerun is taken as exact only when its
// start is the (by then exact) previous unit's last overshoot header; else
// its chain is stitched like a guessed one.
__global__ __launch_bounds__(64) void rpp_seg_stitch_kernel(SegArgs a) {
  using namespace rpp_internal;
  const uint32_t b = blockIdx.x, lane = threadIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t u0 = (uint32_t)a.sv.unit_base[b], nu = (uint32_t)a.sv.unit_base[b + 1] - u0;
  uint32_t j0 = a.sv.sst[b];
  if (nu <= 1 || j0 >= nu) return;
  if (a.sv.sflags[b] & kSfListFull) {  // the fused kernel decodes this stream
    for (uint32_t k = lane; k < nu; k += 64) {
      a.sv.ulo[u0 + k] = kSegNone;
      a.sv.uov[u0 + k] = 0;
    }
    if (lane == 0) a.sv.sst[b] = nu;
    return;
  }
  if (j0 == 0) {
    if (lane == 0) a.sv.ulo[u0] = 0;
    j0 = 1;
  }
  enum { kOk, kEnd, kFail };
  // unit u's class against the previous unit's chain, taken as exact
  auto classify = [&](uint32_t u, uint32_t& lo, uint32_t& uovp) -> uint32_t {
    const uint32_t prev = u - 1;
    const uint32_t np = us_word(a, prev, kUsNovr);
    const uint32_t h = a.uhit[u];
    if ((us_word(a, u, kUsFlags) & kUfRerunDone) && np == kSegOvr &&
        us_word(a, u, kUsStart) == a.sv.ovr[kSegOvr * prev + kSegOvr - 1]) {
      lo = 0;  // parsed from the previous unit's last overshoot header
      uovp = kSegOvr - 1;
      return kOk;
    }
    if (h != kSegNone) {
      lo = a.uhit[a.sv.units_max + u];
      uovp = h;
      return kOk;
    }
    lo = 0;
    uovp = np;
    return np < kSegOvr ? kEnd : kFail;
  };
  auto request = [&](uint32_t u) {
    a.sv.ustate[kUsWords * u + kUsRerun] = a.sv.ovr[kSegOvr * (u - 1) + kSegOvr - 1];
    atomicAdd(&g_seg_diag[a.sv.pass == 2 ? 2 : 1], 1ull);
    if (us_word(a, u, kUsFlags) & kUfNoGuess) atomicAdd(&g_seg_diag[4], 1ull);
  };
  for (; j0 < nu; j0 += 64) {
    const uint32_t j = j0 + lane;
    const bool in = j < nu;
    const uint32_t u = u0 + j, prev = u - 1;
    uint32_t cls = kOk, lo = 0, uovp = 0;
    if (in) cls = classify(u, lo, uovp);
    const uint64_t ev = __ballot(in && cls != kOk);
    const uint32_t e = ev ? (uint32_t)__builtin_ctzll(ev) : 64u;
    if (in && lane < e) {
      a.sv.ulo[u] = lo;
      a.sv.uov[prev] = uovp;
    }
    if (lane < e && in) atomicAdd(&g_seg_diag[0], 1ull);
    if (e == 64) continue;
    const uint32_t ce = __shfl((int)cls, (int)e);
    if (ce == kFail) {
      if (lane == e) {
        request(u);
        a.sv.sst[b] = j;
      }
      // (a rerun pass next: the later units without a meeting whose
      // predecessor met its own, speculatively -- a unit after another
      // failed one keeps its chain, which may well be the true one)
      if (a.sv.pass != 2) {
        uint32_t pc = (uint32_t)__shfl_up((int)cls, 1);
        if (in && lane > e && cls == kFail && pc == kOk) request(u);
        uint32_t carry = (uint32_t)__shfl((int)cls, 63);
        for (uint32_t k0 = j0 + 64; k0 < nu; k0 += 64) {
          const uint32_t k = k0 + lane;
          uint32_t c2 = kEnd, lo2, uovp2;
          if (k < nu) c2 = classify(u0 + k, lo2, uovp2);
          pc = (uint32_t)__shfl_up((int)c2, 1);
          if (lane == 0) pc = carry;
          if (k < nu && c2 == kFail && pc == kOk) request(u0 + k);
          carry = (uint32_t)__shfl((int)c2, 63);
        }
      }
      return;
    }
    // the chain ended before unit j0 + e: no later unit has exact positions
    if (lane == e) a.sv.uov[prev] = uovp;
    for (uint32_t k = j0 + e + lane; k < nu; k += 64) {
      a.sv.ulo[u0 + k] = kSegNone;
      if (k > j0 + e) a.sv.uov[u0 + k - 1] = 0;
    }
    break;
  }
  if (lane == 0) {
    a.sv.uov[u0 + nu - 1] = 0;
    a.sv.sst[b] = nu;
  }
}

constexpr uint32_t kSegThreads = 256;

// exact positions per unit of a split stream (0 for other units)
__global__ void rpp_seg_count_kernel(SegArgs a) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= a.sv.units_max || u >= (uint32_t)a.sv.unit_base[a.nblocks]) return;
  const UnitGeo g = unit_geo(a, u);
  const uint32_t lo = a.sv.ulo[u];
  uint64_t c = 0;
  if (g.nu > 1 && lo != kSegNone) {
    const uint32_t n = us_word(a, u, rpp_internal::kUsNpos);
    c = (n > lo ? n - lo : 0u) + a.sv.uov[u];
  }
  a.cnt[u] = c;
}

// each unit's exact positions into the stream's sb_pos: its list from ulo,
// then its own overshoot entries; entries past the stream's nsb + 1 dropped.
// (list entries are relative to the unit's first bit S, overshoot entries to
// the next unit's, E: ricepp_internal.h)
__global__ __launch_bounds__(kSegThreads) void rpp_seg_write_kernel(SegArgs a) {
  const uint32_t u = blockIdx.x, tid = threadIdx.x;
  if (u >= (uint32_t)a.sv.unit_base[a.nblocks]) return;
  const UnitGeo g = unit_geo(a, u);
  if (g.nu <= 1) return;
  const uint32_t lo = a.sv.ulo[u];
  if (lo == kSegNone) return;
  const uint64_t N = a.n_samples[g.b];
  const uint32_t chunk_len = a.bs * a.cs;
  const uint64_t cap = (N + chunk_len - 1) / chunk_len * a.cs + 1;
  uint32_t* dst = a.sb_pos + a.sb_base[g.b];
  uint32_t* hi = a.tile_hi + a.tile_base[g.b];
  const uint64_t idx0 = a.off[u] - a.off[g.u0];
  const uint32_t n = us_word(a, u, rpp_internal::kUsNpos);
  const uint32_t nl = n > lo ? n - lo : 0u;
  const uint32_t* l = a.sv.plist + a.sv.pl_base[u] + lo;
  auto put = [&](uint64_t e, uint64_t pos) {
    dst[e] = (uint32_t)pos;
    if (e % kTile == 0 && e + 1 < cap) hi[e / kTile] = (uint32_t)(pos >> 32);  // (a tile's first sub-block)
  };
  for (uint32_t i = tid; i < nl; i += kSegThreads)
    if (idx0 + i < cap) put(idx0 + i, g.S + l[i]);
  const uint32_t nov = a.sv.uov[u];
  for (uint32_t i = tid; i < nov; i += kSegThreads)
    if (idx0 + nl + i < cap) put(idx0 + nl + i, g.E + a.sv.ovr[kSegOvr * u + i]);
}

// One sub-block of n samples from bit `pos` (decode.h:42-83, positions only);
// false when it reads past the stream (the fused kernel's TRUNCATED cases).
__device__ bool seg_parse_one(const uint8_t* in, uint32_t nbytes, uint32_t lim, uint32_t& pos, uint32_t n) {
  auto peek = [&](uint32_t q) {
    return __builtin_amdgcn_alignbit(stream_word(in, nbytes, (q >> 5) + 1), stream_word(in, nbytes, q >> 5), q & 31u);
  };
  if (pos + 4 > lim) return false;
  const uint32_t h = peek(pos) & 15u;
  pos += 4;
  if (h == 0) return true;
  if (h == 15) {
    if ((uint64_t)pos + 16ull * n > lim) return false;
    pos += 16 * n;
    return true;
  }
  for (uint32_t i = 0; i < n; ++i) {
    for (;;) {
      if (pos >= lim) return false;
      const uint32_t x = peek(pos);
      if (x) {
        pos += ffbl(x) + 1;
        break;
      }
      pos += 32;
    }
    pos += h - 1;
  }
  return pos <= lim;
}

// One thread per split stream: enough exact positions?  The ragged last
// chunk (parsed by the units with bs samples) again with its own size; the
// stream's status.
__global__ void rpp_seg_tail_kernel(SegArgs a) {
  using namespace rpp_internal;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t u0 = (uint32_t)a.sv.unit_base[b], nu = (uint32_t)a.sv.unit_base[b + 1] - u0;
  if (nu <= 1) return;
  const uint64_t T = a.off[u0 + nu] - a.off[u0];
  const uint32_t N = (uint32_t)a.n_samples[b], cs = a.cs, chunk_len = a.bs * cs;
  const uint32_t nsb = (N + chunk_len - 1) / chunk_len * cs;
  const uint32_t rag = N % chunk_len;
  const uint64_t need = rag ? nsb - cs + 1 : nsb + 1;
  int32_t st = RPP_OK;
  if (a.sv.sflags[b] & kSfListFull) {
    st = kSegFallback;
  } else if (T < need) {
    st = (a.sv.sflags[b] & kSfPastRegion) ? kSegFallback : RPP_TRUNCATED_INPUT;
    if (st == kSegFallback) atomicAdd(&g_seg_diag[3], 1ull);
  } else if (rag) {
    // (in the frame of the word holding the chunk's first header)
    const uint64_t ioff = a.in_off[b];
    const uint32_t mis = (uint32_t)(ioff & 3u);
    uint32_t* dst = a.sb_pos + a.sb_base[b];
    uint32_t* hi = a.tile_hi + a.tile_base[b];
    // the 64-bit position of the last chunk's first header: its low bits
    // against its tile's first entry
    const uint32_t e0 = nsb - cs, f0 = e0 / kTile * kTile;
    const uint64_t ref = ((uint64_t)hi[e0 / kTile] << 32) | dst[f0];
    const uint64_t wt = (ref + (uint32_t)(dst[e0] - (uint32_t)ref)) >> 5;
    const uint64_t nbytes64 = a.in_bytes[b] + mis, lim64 = rpp_internal::seg_read_limit(mis, a.in_bytes[b]);
    const uint32_t nbytes = nbytes64 > 4 * wt ? (uint32_t)min<uint64_t>(nbytes64 - 4 * wt, rpp_internal::kSegWinBytes) : 0u;
    const uint32_t lim = lim64 > 32 * wt ? (uint32_t)min<uint64_t>(lim64 - 32 * wt, rpp_internal::kSegWinBits) : 0u;
    uint32_t pos = (uint32_t)(dst[nsb - cs] & 31u);
    for (uint32_t c = 0; c < cs && st == RPP_OK; ++c) {
      if (!seg_parse_one(a.in + (ioff - mis) + 4 * wt, nbytes, lim, pos, rag / cs)) st = RPP_TRUNCATED_INPUT;
      else {
        const uint32_t e = nsb - cs + 1 + c;
        dst[e] = (uint32_t)(32 * wt + pos);
        if (e % kTile == 0 && e < nsb) hi[e / kTile] = (uint32_t)((32 * wt + pos) >> 32);
      }
    }
  }
  a.status[b] = st;
}

using ExtractKernel = void (*)(ExtractParams);

template <uint32_t CS, bool SH, uint32_t STAGE>
ExtractKernel extract_kernel_for(uint32_t bs) {
  switch (bs) {
    case 16: return rpp_extract_kernel<CS, 16, SH, STAGE>;
    case 32: return rpp_extract_kernel<CS, 32, SH, STAGE>;
    case 64: return rpp_extract_kernel<CS, 64, SH, STAGE>;
    case 128: return rpp_extract_kernel<CS, 128, SH, STAGE>;
    default: return rpp_extract_kernel<CS, 0, SH, STAGE>;  // (general lanes: bs 256 / 512 / not a power of two)
  }
}
template <uint32_t STAGE>
ExtractKernel extract_kernel(const rpp_config* cfg) {
  const bool sh = cfg->unused_lsb_count != 0;
  return cfg->component_stream_count == 1
             ? (sh ? extract_kernel_for<1, true, STAGE>(cfg->block_size)
                   : extract_kernel_for<1, false, STAGE>(cfg->block_size))
             : (sh ? extract_kernel_for<2, true, STAGE>(cfg->block_size)
                   : extract_kernel_for<2, false, STAGE>(cfg->block_size));
}

// The segmented decode forks the fused launch of a batch's one-unit streams
// onto a side stream, so that it overlaps the units' parse; events order it
// after the unit counts and before the batch's end on the caller's stream.
// Every caller stream has its own side stream and event pair (created once,
// never destroyed), so concurrent callers never wait on each other's work and
// a capture of the caller's stream captures the fork and join; the entry's
// mutex is held from the fork to the join, so two threads sharing one caller
// stream do not interleave their use of the events.
constexpr uint32_t kDecSideWaves = 16;  // (full workgroups: the fused launch holds as few CUs as it can)
struct SideStream {
  hipStream_t s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  std::mutex mu;
};
SideStream* side_stream_for(hipStream_t caller) {
  static std::mutex mu;
  static auto* table = new std::map<std::pair<int, hipStream_t>, SideStream*>;  // (leaked at exit: no HIP calls then)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = table->find({dev, caller});
  if (it != table->end()) return it->second;
  auto* e = new SideStream;
  if (hipStreamCreateWithFlags(&e->s2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->join, hipEventDisableTiming) != hipSuccess)
    return nullptr;  // (a half-built entry is not kept)
  table->emplace(std::make_pair(dev, caller), e);
  return e;
}

// Joins the side stream into the caller's stream on every exit path once
// forked: after an error the caller's stream still waits for the side work,
// which writes d_out / d_status.
class SideFork {
 public:
  explicit SideFork(SideStream* e) : e_{e}, lk_{e->mu} {}
  SideFork(const SideFork&) = delete;
  SideFork& operator=(const SideFork&) = delete;
  bool fork(hipStream_t s) {
    s_ = s;
    forked_ = hipEventRecord(e_->fork, s) == hipSuccess && hipStreamWaitEvent(e_->s2, e_->fork, 0) == hipSuccess;
    return forked_;
  }
  hipStream_t side() const { return e_->s2; }
  bool join() {
    if (!forked_) return true;
    forked_ = false;
    return hipEventRecord(e_->join, e_->s2) == hipSuccess && hipStreamWaitEvent(s_, e_->join, 0) == hipSuccess;
  }
  ~SideFork() { (void)join(); }

 private:
  SideStream* e_;
  std::lock_guard<std::mutex> lk_;
  hipStream_t s_ = nullptr;
  bool forked_ = false;
};

// Block sizes the segmented decode takes: every bs >= 16 (16/32/64/128 with
// unrolled fast lanes in the extraction, the others -- 256, 512, odd sizes --
// with its exact general lanes).  Below 16 samples a sub-block codes to too
// few bits for the units' position lists (one entry per 32 bits): such
// streams are decoded one wave per stream.
bool extract_bs(uint32_t bs) { return bs >= 16; }

uint32_t path_of(const rpp_decode_options* opt) { return opt ? opt->path : RPP_DECODE_AUTO; }

// Segmented decode (units of 2^L bits; 0 = one wave per stream): by default
// when the batch's longest stream would take longer to parse serially than
// the whole batch takes at full occupancy (its samples > 1/1024 of the
// batch's, and >= 2^18).  Measured on MI355X: for
// batches of many short streams the fused kernel wins -- its value work
// hides in the parse chain's latency -- so it is not split.
uint32_t seg_log2_for(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                      const rpp_decode_options* opt) {
  if (!extract_bs(cfg->block_size)) return 0;
  const uint32_t path = path_of(opt);
  if (path == RPP_DECODE_FUSED) return 0;
  if (path != RPP_DECODE_SEGMENTED) {
    if (max_stream_samples < (1u << 18)) return 0;
    // the one-wave kernel when the batch is long enough for its longest
    // stream to finish inside the batch's time: that stream takes ~10.7 ns
    // per sample on one wave, the batch ~1.6 ps per sample over the whole
    // chip, and the segmented decode ~3 ps per sample (configs[3]'s 32 GiB
    // mix of 1/4/16 MiB blocks: one-wave 86 ms, segmented 51 ms,
    // profiles/r04_bench_mix*.json)
    if (max_stream_samples * 3072 < total_samples) return 0;
    // bs 256 / 512: a unit's guess parses lane by lane only (2-8 Kib
    // sub-blocks), so units cost several times more; 1 MiB streams decode
    // faster one wave each (16 x 1 MiB at bs 512: 3.8 ms fused, 21 ms split)
    if (cfg->block_size > 128 && max_stream_samples < (1u << 21)) return 0;
  }
  // about 4096 units for the batch (8 bits per sample: Poisson-like data
  // compresses to 7-8), 2^18..2^23 bits (a unit's guess costs about as much
  // as parsing 2^20 bits, so small batches take small units for parallelism
  // and big ones large units); streams that fit one unit stay on the fused
  // kernel
  uint32_t L = 18;
  while (L < 23 && ((total_samples * 8) >> L) > 4096) ++L;
  if (opt && opt->seg_log2) L = std::min<uint32_t>(26, std::max<uint32_t>(10, opt->seg_log2));  // (range-checked by the caller)
  return L;
}



// ---- the segmented decode's set-up in one workgroup (rpp_seg_plan_kernel) ----
// It replaces eight small launches and nine fills (~100 us of launch gaps for
// a single long stream): the workspace promise check (guard), units per
// stream and their prefix, sub-blocks and tiles per stream and their
// prefixes, the tiles per hand-out level and their prefix (a histogram of the
// streams' tile counts), and the zeroed / 0xFF-filled state of the passes.
constexpr uint32_t kPlanThreads = 1024;

// out[i] = sum_{j<i} in[j] over n entries, by the whole workgroup (4096 per
// pass: wave scans by shuffles, the wave totals by wave 0, a carried total)
__device__ void plan_exscan(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t* sh) {
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  constexpr uint32_t kPer = 4, kTileN = kPlanThreads * kPer, kW = kPlanThreads / 64;
  uint64_t carry = 0;
  for (uint64_t base = 0; base < n; base += kTileN) {
    const uint64_t i0 = base + (uint64_t)kPer * t;
    uint64_t v[kPer], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      v[k] = i0 + k < n ? in[i0 + k] : 0u;
      sum += v[k];
    }
    uint64_t incl = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint64_t u = __shfl_up(incl, d, 64);
      if (lane >= d) incl += u;
    }
    if (lane == 63) sh[wv] = incl;
    __syncthreads();
    if (wv == 0) {
      const uint64_t x = lane < kW ? sh[lane] : 0u;
      uint64_t xi = x;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(xi, d, 64);
        if (lane >= d) xi += u;
      }
      if (lane < kW) sh[lane] = xi - x;
      if (lane == kW - 1) sh[kW] = xi;
    }
    __syncthreads();
    uint64_t run = carry + sh[wv] + incl - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
      if (i0 + k < n) out[i0 + k] = run;
      run += v[k];
    }
    carry += sh[kW];
    __syncthreads();
  }
}

struct PlanArgs {
  SegArgs a;
  uint64_t total_samples, max_stream_samples;
  uint32_t* guard;
  uint64_t *ucnt, *sb_cnt, *tile_cnt, *tile_base, *lvl_cnt, *lvl_base;
  uint32_t levels, chunk_len;
  uint64_t* tile_state;
  uint64_t max_tiles;
  uint32_t* counter;
  uint64_t *pl_cnt, *cnt2;
};

__global__ __launch_bounds__(kPlanThreads) void rpp_seg_plan_kernel(PlanArgs q) {
  using namespace rpp_internal;
  __shared__ uint64_t sh[kPlanThreads / 64 + 1];
  __shared__ uint32_t bad;
  __shared__ unsigned long long sum, sbits, stiles;
  const SegArgs& a = q.a;
  const uint32_t t = threadIdx.x, B = a.nblocks;
  const uint64_t U = a.sv.units_max;
  // the pass state: tile look-back states and counters zeroed, unit states
  // 0xFF (a unit's guess word kSegNone = not searched)
  for (uint64_t i = t; i < q.max_tiles; i += kPlanThreads) q.tile_state[i] = 0;
  for (uint64_t i = t; i <= U; i += kPlanThreads) {
    q.pl_cnt[i] = 0;
    q.cnt2[i] = 0;
  }
  for (uint64_t i = t; i < U * kUsWords; i += kPlanThreads) a.sv.ustate[i] = 0xFFFFFFFFu;
  for (uint32_t i = t; i < B; i += kPlanThreads) {
    a.sv.sst[i] = 0;
    a.sv.sflags[i] = 0;
  }
  if (t == 0) {
    *q.counter = 0;
    *a.sv.queue = 0;
    bad = 0;
    sum = 0;
    sbits = 0;
    stiles = 0;
  }
  __syncthreads();
  // the batch against the workspace's promise (rpp_decode_workspace_bytes):
  // broken, every stream is decoded one wave each (one unit, no sub-blocks)
  unsigned long long part = 0;
  for (uint32_t i = t; i < B; i += kPlanThreads) {
    const uint64_t n = a.n_samples[i];
    if (n % a.cs != 0 || n >= RPP_MAX_STREAM_SAMPLES) continue;  // (not decodable: reported by the kernels)
    part += n;
    if (n > q.max_stream_samples) bad = 1;
  }
  atomicAdd(&sum, part);
  __syncthreads();
  const bool guard = bad || sum > q.total_samples;
  if (t == 0) *q.guard = guard ? 1u : 0u;
  // units (one per 2^L bits of a stream's header range, 1 for short or
  // undecodable streams), sub-blocks + 1 and tiles of the split streams
  unsigned long long pbits = 0, ptiles = 0;
  for (uint32_t i = t; i <= B; i += kPlanThreads) {
    uint64_t c = 0, nsb = 0;
    if (i < B) {
      const uint64_t n = a.n_samples[i], nb = a.in_bytes[i];
      c = 1;
      if (!guard && seg_stream_ok(n, nb, a.cs))
        c = (seg_last_bit((uint32_t)(a.in_off[i] & 3u), nb, n, a.bs, a.cs) >> a.sv.seg_log2) + 1;
      if (!guard && c > 1) {
        nsb = (n + q.chunk_len - 1) / q.chunk_len * a.cs;
        pbits += 8 * nb;
        ptiles += (nsb + kTile - 1) / kTile;
      }
    }
    q.ucnt[i] = c;
    q.sb_cnt[i] = i < B ? nsb + 1 : 0;
    q.tile_cnt[i] = (nsb + kTile - 1) / kTile;
  }
  atomicAdd(&sbits, pbits);
  atomicAdd(&stiles, ptiles);
  // histogram of the tile counts (into lvl_base) for the levels
  for (uint32_t l = t; l <= q.levels; l += kPlanThreads) q.lvl_base[l] = 0;
  __syncthreads();
  for (uint32_t i = t; i < B; i += kPlanThreads)
    atomicAdd(reinterpret_cast<unsigned long long*>(&q.lvl_base[(size_t)std::min<uint64_t>(q.tile_cnt[i], q.levels)]),
              1ull);
  __syncthreads();
  // the extraction's stage: the 48 KiB one (three workgroups per CU) unless
  // the split streams' tiles average more than 90 % of its bits (then many
  // lanes would read past it: generator data at 14 bits per sample, one
  // 2^29-sample stream, 11.8 -> 10.1 ms with 64 KiB; the configs[3] mix at
  // ~8 bits per sample 5 % slower with it -- profiles/r06_giant_stage_ab.jsonl)
  if (t == 0) q.guard[1] = sbits * 10 > stiles * 9 * 32 * kStageWordsMany ? 1u : 0u;
  plan_exscan(q.ucnt, (uint64_t)B + 1, const_cast<uint64_t*>(a.sv.unit_base), sh);
  plan_exscan(q.sb_cnt, (uint64_t)B + 1, const_cast<uint64_t*>(a.sb_base), sh);
  plan_exscan(q.tile_cnt, (uint64_t)B + 1, q.tile_base, sh);
  plan_exscan(q.lvl_base, (uint64_t)q.levels + 1, q.lvl_cnt, sh);  // streams with <= l - 1 tiles
  // streams with more than l tiles = B - (streams with <= l tiles)
  for (uint32_t l = t; l <= q.levels; l += kPlanThreads)
    q.lvl_cnt[l] = l < q.levels ? (uint64_t)B - (q.lvl_cnt[l] + q.lvl_base[l]) : 0u;
  __syncthreads();
  plan_exscan(q.lvl_cnt, (uint64_t)q.levels + 1, q.lvl_base, sh);
}

}  // namespace

extern "C" {

// diagnostics only (not in the C ABI header): the extraction phase timers
int rpp_seg_diag_read(unsigned long long* out8, int reset) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_seg_diag), sizeof(g_seg_diag)) != hipSuccess) return RPP_HIP_ERROR;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_seg_diag), z, sizeof(z)) != hipSuccess) return RPP_HIP_ERROR;
  }
  return RPP_OK;
}

int rpp_diag_read(unsigned long long* out8, int reset) {
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_dec2_diag), sizeof(g_dec2_diag)) != hipSuccess) return RPP_HIP_ERROR;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dec2_diag), z, sizeof(z)) != hipSuccess) return RPP_HIP_ERROR;
  }
  return RPP_OK;
}

uint64_t rpp_decode_workspace_bytes_ex(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                       uint32_t nblocks, const rpp_decode_options* opt) {
  if (rpp_check_config(cfg) != RPP_OK) return 0;
  const uint32_t L = seg_log2_for(cfg, total_samples, max_stream_samples, opt);
  if (!L) return 0;  // the fused kernel needs none
  return layout(cfg, total_samples, max_stream_samples, nblocks, L, nullptr).bytes;
}

uint64_t rpp_decode_workspace_bytes(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                    uint32_t nblocks) {
  return rpp_decode_workspace_bytes_ex(cfg, total_samples, max_stream_samples, nblocks, nullptr);
}

int rpp_decode_batch_ex(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, uint64_t total_samples,
                        uint64_t max_stream_samples, void* d_workspace, uint64_t workspace_bytes,
                        const rpp_decode_options* opt, void* stream) {
  int st = rpp_check_config(cfg);
  if (st != RPP_OK) return st;
  if (opt && (opt->path > RPP_DECODE_SEGMENTED || opt->fused_waves > kDecSideWaves ||
              (opt->seg_log2 && (opt->seg_log2 < 10 || opt->seg_log2 > 26))))
    return RPP_INVALID_ARGUMENT;
  if (nblocks == 0) return RPP_OK;
  if (!d_in || !d_in_offsets || !d_in_bytes || !d_out || !d_out_offsets || !d_n_samples || !d_status)
    return RPP_INVALID_ARGUMENT;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t fused_waves = opt ? opt->fused_waves : 0u;
  const uint32_t L = seg_log2_for(cfg, total_samples, max_stream_samples, opt);
  if (!L)  // (the rows kernel for bs 16 / 32 unless the one-wave path is asked for)
    return rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                             d_n_samples, d_status, s, false, nullptr, fused_waves,
                                             path_of(opt) != RPP_DECODE_FUSED);
  const Workspace w = layout(cfg, total_samples, max_stream_samples, nblocks, L, static_cast<uint8_t*>(d_workspace));
  if (!d_workspace || workspace_bytes < w.bytes) return RPP_INVALID_ARGUMENT;
  // the side stream is created on the current device: the caller's stream
  // must belong to it (include/ricepp_amd.h, rpp_decode_batch_ws)
  {
    int cur = 0, sdev = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(s, &sdev) != hipSuccess) return RPP_HIP_ERROR;
    if (cur != sdev) return RPP_INVALID_ARGUMENT;
  }
  SideStream* side = side_stream_for(s);
  if (!side) return RPP_HIP_ERROR;
  const uint32_t chunk_len = cfg->block_size * cfg->component_stream_count;
  const uint32_t g256 = (nblocks + 256) / 256;
  const uint32_t test = opt ? opt->test_flags : 0u;
  SegArgs a{};
  a.sv = rpp_internal::SegView{w.unit_map, w.unit_base, w.pl_base, w.plist, w.ovr, w.ustate, w.ulo, w.uov,
                               w.sst, w.sflags, w.queue, L, 0, (uint32_t)w.units_max};
  a.in = d_in;
  a.in_off = d_in_offsets;
  a.in_bytes = d_in_bytes;
  a.n_samples = d_n_samples;
  a.sb_base = w.sb_base;
  a.sb_pos = w.sb_pos;
  a.tile_hi = w.tile_hi;
  a.tile_base = w.tile_base;
  a.status = d_status;
  a.cnt = w.cnt2;
  a.off = w.off2;
  a.uhit = w.uhit;
  a.guard = w.guard;
  a.nblocks = nblocks;
  a.bs = cfg->block_size;
  a.cs = cfg->component_stream_count;
  PlanArgs q{a, total_samples, max_stream_samples, w.guard, w.ucnt, w.sb_cnt, w.tile_cnt, w.tile_base, w.lvl_cnt,
             w.lvl_base, w.levels, chunk_len, w.tile_state, w.max_tiles, w.counter, w.pl_cnt, w.cnt2};
  hipLaunchKernelGGL(rpp_seg_plan_kernel, dim3(1), dim3(kPlanThreads), 0, s, q);
  hipLaunchKernelGGL(rpp_dec_level_map_kernel, dim3(w.levels), dim3(kLvlThreads), 0, s, w.tile_cnt, nblocks,
                     w.levels, w.lvl_base, w.tile_map, w.tile_lt);
  // the streams that fit one unit (all of them when the guard tripped): one
  // wave each, parse and values fused, on the side stream while the units are
  // parsed
  SideFork fork{side};
  if (!fork.fork(s)) return RPP_HIP_ERROR;
  st = rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                         d_n_samples, d_status, fork.side(), false, w.ucnt,
                                         fused_waves ? fused_waves : kDecSideWaves);
  if (st != RPP_OK) return st;
  const uint64_t U = w.units_max;
  const uint32_t gu = (uint32_t)((U + 255) / 256);
  hipLaunchKernelGGL(rpp_seg_map_kernel, dim3(gu), dim3(256), 0, s, a, w.unit_map, w.pl_cnt);
  if ((st = rpp_exclusive_scan_u64(w.pl_cnt, U + 1, w.pl_base, s)) != RPP_OK) return st;
  // few units: their first guesses by several waves each, before pass 0
  if ((st = rpp_internal::launch_seg_guess(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_n_samples, a.sv, s)) !=
      RPP_OK)
    return st;
  // pass 0: every unit; three rerun passes; a serial pass for what is left
  for (uint32_t pass : {0u, 1u, 1u, 1u, 2u}) {
    a.sv.pass = pass;  // (the stitch counts the reruns it asks this pass for)
    if (pass != 0) {
      hipLaunchKernelGGL(rpp_seg_hit_kernel, dim3(gu), dim3(256), 0, s, a);
      hipLaunchKernelGGL(rpp_seg_stitch_kernel, dim3(nblocks), dim3(64), 0, s, a);
    }
    st = rpp_internal::launch_parse_seg(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_n_samples, w.sb_base,
                                        w.sb_pos, d_status, a.sv, s);
    if (st != RPP_OK) return st;
  }
  hipLaunchKernelGGL(rpp_seg_count_kernel, dim3(gu), dim3(256), 0, s, a);
  if ((st = rpp_exclusive_scan_u64(w.cnt2, U + 1, w.off2, s)) != RPP_OK) return st;
  hipLaunchKernelGGL(rpp_seg_write_kernel, dim3((uint32_t)U), dim3(kSegThreads), 0, s, a);
  hipLaunchKernelGGL(rpp_seg_tail_kernel, dim3(g256), dim3(256), 0, s, a);
  // (a batch of more tiles than the grid holds: the smaller stage, three
  // workgroups per CU)
  // (a batch that can have more tiles than the grid holds: both stages, the
  // plan kernel's choice by density runs; fewer: the 64 KiB stage)
  const bool many = w.max_tiles >= kMaxExtractGrid;
  ExtractParams p{d_in, d_in_offsets, d_in_bytes, d_n_samples, d_out, d_out_offsets, d_status, w.sb_pos, w.tile_hi,
                  w.sb_base,
                  w.tile_base, w.tile_map, w.tile_lt, w.lvl_base + w.levels, w.tile_state, w.counter, nblocks,
                  cfg->block_size, cfg->big_endian ? 1u : 0u, cfg->unused_lsb_count, test,
                  many ? w.guard + 1 : nullptr};
  const uint32_t grid = (uint32_t)std::min<uint64_t>(w.max_tiles, kMaxExtractGrid);
  hipLaunchKernelGGL(extract_kernel<kStageWords>(cfg), dim3(grid), dim3(kTile), 0, s, p);
  if (many) hipLaunchKernelGGL(extract_kernel<kStageWordsMany>(cfg), dim3(grid), dim3(kTile), 0, s, p);
  if (hipGetLastError() != hipSuccess) return RPP_HIP_ERROR;
  // join the side stream, then the streams whose exact chain left the region
  // the units cover or whose lists overflowed (the fused kernel)
  if (!fork.join()) return RPP_HIP_ERROR;
  st = rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                         d_n_samples, d_status, s, true, nullptr, fused_waves);
  if (st != RPP_OK) return st;
  return hipGetLastError() == hipSuccess ? RPP_OK : RPP_HIP_ERROR;
}

int rpp_decode_batch_ws(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, uint64_t total_samples,
                        uint64_t max_stream_samples, void* d_workspace, uint64_t workspace_bytes, void* stream) {
  return rpp_decode_batch_ex(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets, d_n_samples,
                             d_status, total_samples, max_stream_samples, d_workspace, workspace_bytes, nullptr,
                             stream);
}

// Without a workspace: always one wave per stream (no host synchronisation).
int rpp_decode_batch(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                     const uint64_t* d_n_samples, int32_t* d_status, void* stream) {
  return rpp_internal::launch_decode_fused(cfg, d_in, d_in_offsets, d_in_bytes, nblocks, d_out, d_out_offsets,
                                           d_n_samples, d_status, (hipStream_t)stream, false, nullptr, 0, true);
}

}  // extern "C"
