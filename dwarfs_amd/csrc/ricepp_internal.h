// ricepp_internal.h -- launchers and data shared between the kernel
// translation units (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ricepp_amd.h"

namespace rpp_internal {

// ---------------------------------------------------------------------------
// Segmented decode of long streams (ricepp_decode2.hip, DESIGN.md "Segmented
// decode").  A stream longer than 2^L bits is cut into units of 2^L bits;
// every unit is parsed by its own wave from a guessed first header (unit 0
// from the true start), recording the header positions it visits inside its
// region in a list (in chain order, so ascending) and the first kSegOvr
// headers past the region in an overshoot list.  A guessed chain that meets
// the previous unit's exact chain is exact from the meeting point on (the
// parse is deterministic), so the stitch pass keeps each unit's positions from
// there; a unit whose chain never meets is parsed again from a known header
// (rerun passes, then one serial pass): the result is the serial parse's,
// whatever the guesses were.
// ---------------------------------------------------------------------------
// The one-wave encode of a whole stream and the four-streams-per-wave decode
// keep 32-bit bit positions for any data: streams below 2^27 samples (longer
// ones are encoded in segments, decoded by the other kernels).
constexpr uint64_t kSegMaxSamples = UINT64_C(1) << 27;
// The segmented decode's positions (round 6): a unit's parse works in a
// frame that starts at its unit's first bit S = j 2^L (its wave reads the
// stream from byte S / 8 on), and every position a unit leaves behind is
// stored relative to the S of the unit it belongs to -- list entries and the
// start / rerun / guess words to the unit's own, overshoot entries to the
// next unit's (so that the stitch compares them with that unit's list as
// they are) -- which keeps them far below 2^32 and the sentinels below.  The
// sub-block start list the extraction reads (sb_pos) holds the low 32 bits of
// the positions from the stream's 4-aligned base, and a per-tile word the
// high bits of the tile's first position (a tile spans a few Mbit at most).  Before round 6 all of them were 32-bit
// positions from the stream's base, which limited the segmented decode to
// streams compressed below 2^29 bytes; now any stream below
// RPP_MAX_STREAM_SAMPLES whose byte count fits 32 bits takes it.  A wave's
// frame is at most kSegWinBits long: a serial pass (which parses from one
// unit to the stream's end) that would leave it hands the stream to the
// fused kernel, which rebases its positions as it goes.
constexpr uint64_t kSegMaxBytes = (UINT64_C(1) << 32) - (UINT64_C(1) << 16);
constexpr uint32_t kSegWinBytes = UINT32_C(1) << 28;
constexpr uint32_t kSegWinBits = 8u * kSegWinBytes;         // 2^31
constexpr uint32_t kSegSerialEnd = kSegWinBits - (1u << 24);  // a serial pass's region ends here at the latest
__host__ __device__ inline bool seg_stream_fits(uint64_t n, uint64_t nb, uint32_t cs) {
  return n % cs == 0 && n < RPP_MAX_STREAM_SAMPLES && nb < kSegMaxBytes;
}
constexpr uint32_t kSegOvr = 16;             // headers recorded past a unit's region
constexpr uint32_t kSegNone = 0xFFFFFFFFu;   // no position
constexpr uint32_t kSpecSteps = 12;          // sub-blocks a candidate first header must chain through
constexpr uint32_t kSpecVerify = 24;         // ... and the unit's own parse then checks (< 64)
constexpr uint32_t kGuessRetries = 8;        // next candidates tried after a rejected guess
constexpr int32_t kSegFallback = 0x7F5E0001;  // internal status: decode this stream with the fused kernel

// per-unit state words (SegView::ustate[kUsWords u + i]): overshoot entries,
// the chain's first header, a pending rerun's start, flags, positions listed
constexpr uint32_t kUsWords = 8;
// kUsGuess: the unit's first guess when rpp_seg_guess_kernel searched it
// (kSegNone: not searched; kSegNoGuess: searched, no candidate survived)
enum : uint32_t { kUsNovr = 0, kUsStart = 1, kUsRerun = 2, kUsFlags = 3, kUsNpos = 4, kUsGuess = 5 };
constexpr uint32_t kSegNoGuess = 0xFFFFFFFEu;
enum : uint32_t { kUfRerunDone = 1, kUfNoGuess = 2, kUfTrunc = 4 };
// per-stream flags (SegView::sflags)
enum : uint32_t { kSfPastRegion = 1, kSfListFull = 2 };

struct SegView {
  const uint32_t* unit_map;   // [U] stream of unit u
  const uint64_t* unit_base;  // [B + 1] first unit of stream b (entry B: the number of units)
  const uint64_t* pl_base;    // [U_max + 1] first list entry of unit u (capacity: the next minus this)
  uint32_t* plist;            // header positions of each unit's region, in chain order
  uint32_t* ovr;              // [U_max * kSegOvr] first headers past the region
  uint32_t* ustate;           // [U_max * kUsWords]
  uint32_t* ulo;              // [U_max] the unit's exact positions start at this list index (stitch)
  uint32_t* uov;              // [U_max] overshoot entries of the unit that are its own (stitch)
  uint32_t* sst;              // [B] first unresolved unit of stream b
  uint32_t* sflags;           // [B] kSfPastRegion, kSfListFull
  uint32_t* queue;            // [1] pass 0: the next unit to take
  uint32_t seg_log2;          // L
  uint32_t pass;              // 0 all units; 1 pending reruns; 2 pending reruns, serial to the end
  uint32_t units_max;         // grid bound (U_max)
};

// Last bit position a header (or the end) of a well-formed stream can take,
// relative to the 4-aligned base (bit 0 at 8 * mis): the stream's bytes,
// clamped to rpp_worst_case_bytes of its sample count (codec.h:45-55 bound).
__host__ __device__ inline uint64_t seg_last_bit(uint32_t mis, uint64_t in_bytes, uint64_t n, uint32_t bs,
                                                  uint32_t cs) {
  const uint64_t per = n / cs;
  const uint64_t num = 16 + 4 * ((per + bs - 1) / bs) + 16 * per;
  const uint64_t wc = (num * cs + 7) / 8;
  const uint64_t nb = in_bytes < wc ? in_bytes : wc;
  return 8ull * mis + 8ull * nb;
}

// a stream's last readable bit + 1 from its 4-aligned base: the reader pulls
// whole 8-byte packets (bitstream_reader.h:149-183), zero past its last byte
__host__ __device__ inline uint64_t seg_read_limit(uint32_t mis, uint64_t in_bytes) {
  return 8ull * mis + 64ull * ((in_bytes + 7) >> 3);
}

// rpp_decode_kernel: one wave per stream, parse and values fused (any bs).
// only_fallback: decode only the streams whose status is kSegFallback;
// d_units (the segmented decode's units per stream): skip split streams.
// waves: streams per workgroup (0: by batch size).  rows (bs 16 / 32, a
// whole-batch launch): rpp_decode_rows_kernel first, four streams per wave,
// then the fused kernel for the streams it leaves.
int launch_decode_fused(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out, const uint64_t* d_out_offsets,
                        const uint64_t* d_n_samples, int32_t* d_status, hipStream_t stream, bool only_fallback = false,
                        const uint64_t* d_units = nullptr, uint32_t waves = 0, bool rows = false);

// rpp_parse_kernel over units (SegView): the units of split streams, into
// their position and overshoot lists (single-unit streams are left to the
// fused kernel).
// rpp_seg_guess_kernel: the first guesses of the units of split streams,
// several waves per unit (for batches of few units, whose parse would leave
// most wave slots idle); pass 0 of the parse then starts from them.  Returns
// RPP_OK without launching anything when the batch has too many units.
int launch_seg_guess(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, const uint64_t* d_n_samples, const SegView& sv,
                     hipStream_t stream);

int launch_parse_seg(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, const uint64_t* d_n_samples,
                     const uint64_t* d_sb_base, uint32_t* d_sb_pos, int32_t* d_status, const SegView& sv,
                     hipStream_t stream);

}  // namespace rpp_internal
