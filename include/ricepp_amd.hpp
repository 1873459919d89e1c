// ricepp_amd.hpp -- C++ host facade over the C ABI of ricepp_amd.h.
//
// Source-compatible with the two interfaces the reference exposes for this
// path, so that DwarFS's plugin (src/compression/ricepp.cpp) compiles against
// it with only its #include lines and the namespace changed
// (`namespace ricepp = ricepp_amd;`):
//
//  * the ricepp library API
//      codec_config {block_size, component_stream_count, std::endian byteorder,
//                    unused_lsb_count}      (ricepp/include/ricepp/codec_config.h:36-41)
//      template <std::unsigned_integral PixelT>
//      std::unique_ptr<encoder_interface<PixelT>> create_encoder(codec_config const&)
//                                            (ricepp/include/ricepp/create_encoder.h:39-41)
//      ... create_decoder                     (ricepp/include/ricepp/create_decoder.h:39-41)
//      encoder_interface<PixelT>::encode / worst_case_encoded_bytes
//                                            (ricepp/include/ricepp/encoder_interface.h:38-60)
//      decoder_interface<PixelT>::decode      (ricepp/include/ricepp/decoder_interface.h:37-50)
//    Only PixelT = uint16_t is instantiated, as in the reference
//    (ricepp/ricepp.cpp:36-48).  Errors: std::runtime_error("Unsupported
//    configuration") for a bad config (ricepp/ricepp_cpuspecific.cpp:161,173),
//    std::out_of_range when decoding runs past the input.
//
//  * the DwarFS block codec behind block_compressor / block_decompressor
//      block_compressor / block_decompressor (src/compression/ricepp.cpp:57-255)
//    with the same framing, metadata JSON, constraints and error messages.
//
// Threading and batching.  Every method is const and may be called from many
// threads at once, as the reference's immutable objects can; DwarFS's
// worker_group threads call compress on one shared block_compressor::impl
// (src/writer/filesystem_writer.cpp:255-287) and decompress blocks
// concurrently (src/reader/internal/block_cache.cpp:628-706).  Concurrent
// encode / decode calls with the same configuration on the same device are
// coalesced into one rpp_encode_batch_ws / rpp_decode_batch_ws launch (a
// pipelined batch queue: callers copy their own data into and out of pinned
// staging in parallel, a driver thread per queue launches the batches and
// publishes their results; up to two batches per queue on the device).
// Device contexts (stream, event, device and pinned staging) come from a
// per-device pool and are reused, so no call creates a stream or allocates
// once the pool is warm.  An object runs on the device that was current when
// it was created.
#pragma once

#include <bit>
#include <concepts>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <optional>
#include <span>
#include <stdexcept>
#include <string>
#include <vector>

#include "ricepp_amd.h"

namespace ricepp_amd {

// ricepp::codec_config (ricepp/include/ricepp/codec_config.h:36-41)
struct codec_config {
  size_t block_size;
  size_t component_stream_count;
  std::endian byteorder;
  unsigned unused_lsb_count;
};

// ricepp::encoder_interface (ricepp/include/ricepp/encoder_interface.h:38-60)
template <typename PixelT>
class encoder_interface {
  static_assert(std::unsigned_integral<PixelT>, "PixelT must be an unsigned integral type");

 public:
  using pixel_type = PixelT;

  virtual ~encoder_interface() = default;

  [[nodiscard]] virtual std::vector<uint8_t> encode(std::span<pixel_type const> input) const = 0;
  virtual size_t worst_case_encoded_bytes(size_t pixel_count) const = 0;
  virtual size_t worst_case_encoded_bytes(std::span<pixel_type const> input) const = 0;
  virtual std::span<uint8_t> encode(std::span<uint8_t> output, std::span<pixel_type const> input) const = 0;
};

// ricepp::decoder_interface (ricepp/include/ricepp/decoder_interface.h:37-50)
template <typename PixelT>
class decoder_interface {
  static_assert(std::unsigned_integral<PixelT>, "PixelT must be an unsigned integral type");

 public:
  using pixel_type = PixelT;

  virtual ~decoder_interface() = default;

  virtual void decode(std::span<pixel_type> output, std::span<uint8_t const> input) const = 0;
};

// ricepp::create_encoder / create_decoder: declared for every unsigned PixelT
// like the reference, defined (in ricepp_facade.cpp) for uint16_t.
template <std::unsigned_integral PixelT>
std::unique_ptr<encoder_interface<PixelT>> create_encoder(codec_config const& config);
template <std::unsigned_integral PixelT>
std::unique_ptr<decoder_interface<PixelT>> create_decoder(codec_config const& config);

template <>
std::unique_ptr<encoder_interface<uint16_t>> create_encoder<uint16_t>(codec_config const& config);
template <>
std::unique_ptr<decoder_interface<uint16_t>> create_decoder<uint16_t>(codec_config const& config);

// ---- DwarFS block codec (src/compression/ricepp.cpp) ----

// compression_type::RICEPP (include/dwarfs/compression.h, RICEPP = 7)
inline constexpr int compression_type_ricepp = 7;

class block_compressor {
 public:
  // "ricepp:block_size=N": the factory reads the option without a range check
  // (src/compression/ricepp.cpp:277-281); an unsupported size throws
  // "Unsupported configuration" from create_encoder at compress time (:97-102).
  explicit block_compressor(size_t block_size = 128);
  static std::unique_ptr<block_compressor> create(std::string const& spec);

  std::unique_ptr<block_compressor> clone() const;
  std::vector<uint8_t> compress(std::span<uint8_t const> data, std::string const* metadata) const;
  int type() const { return compression_type_ricepp; }
  std::string describe() const;
  std::string metadata_requirements() const;
  size_t compression_granularity(std::string const& metadata) const;  // get_compression_constraints
  size_t estimate_memory_usage(size_t data_size) const { return data_size; }

 private:
  size_t block_size_;
};

class block_decompressor {
 public:
  explicit block_decompressor(std::span<uint8_t const> data);

  int type() const { return compression_type_ricepp; }
  std::optional<std::string> metadata() const;
  size_t uncompressed_size() const { return frame_.uncompressed_bytes; }
  void start_decompression(std::vector<uint8_t>* target);
  bool decompress_frame(size_t frame_size = 0);  // decodes everything on the first call
  // convenience: block_decompressor::decompress (src/block_decompressor.cpp:41-49)
  static std::vector<uint8_t> decompress(std::span<uint8_t const> data);

 private:
  rpp_frame frame_{};
  std::span<uint8_t const> data_;
  std::unique_ptr<decoder_interface<uint16_t>> decoder_;
  std::vector<uint8_t>* target_ = nullptr;
};

// ---- DwarFS FLAC block codec (src/compression/flac.cpp) ----
//
// flac_block_compressor / flac_block_decompressor: the plugin's framing
// (varint + thrift-compact flac_block_header + a FLAC stream), metadata JSON,
// describe(), constraints and error messages (flac.cpp:215-489), with the PCM
// bytes unpacked, encoded, decoded and packed on the GPU (rpp_pcm_unpack,
// rpp_flac_encode, rpp_flac_decode, rpp_pcm_pack) through a pooled device
// context.  Parity unpinned: the reference codes the stream with libFLAC
// (absent here); this encoder writes valid FLAC (RFC 9639) with fixed and LPC
// predictors, 4096-sample frames and stereo decorrelation, so its bytes differ
// from libFLAC's.  `level` (0..8) and `exhaustive` are validated, reported by
// describe() as the reference does, and select libFLAC's preset limits (LPC
// order 0 / 6 / 8 / 12) and the exhaustive model search (rpp_flac_encode_ex).
// The decoder reads every RFC 9639 frame kind.

// compression_type::FLAC (include/dwarfs/compression.h, FLAC = 6)
inline constexpr int compression_type_flac = 6;

class flac_block_compressor {
 public:
  explicit flac_block_compressor(uint32_t level = 5, bool exhaustive = false);
  // "flac", "flac:level=N", "flac:exhaustive", "flac:level=N:exhaustive"
  // (flac_compressor_factory, flac.cpp:509-525: options level=[0..8],
  // exhaustive)
  static std::unique_ptr<flac_block_compressor> create(std::string const& spec);

  std::unique_ptr<flac_block_compressor> clone() const;
  std::vector<uint8_t> compress(std::span<uint8_t const> data, std::string const* metadata) const;
  int type() const { return compression_type_flac; }
  std::string describe() const;                                       // flac.cpp:363-366
  std::string metadata_requirements() const;                          // :368-379
  size_t compression_granularity(std::string const& metadata) const;  // :381-393
  size_t estimate_memory_usage(size_t data_size) const { return data_size; }  // :395-398

 private:
  uint32_t level_;
  bool exhaustive_;
};

class flac_block_decompressor {
 public:
  // throws "[FLAC] could not initialize decoder: ..." for a stream whose
  // metadata does not parse (flac.cpp:410-418)
  explicit flac_block_decompressor(std::span<uint8_t const> data);

  int type() const { return compression_type_flac; }
  std::optional<std::string> metadata() const;  // :429-440
  size_t uncompressed_size() const { return frame_.uncompressed_bytes; }
  void start_decompression(std::vector<uint8_t>* target);
  bool decompress_frame(size_t frame_size = 0);  // decodes everything on the first call
  static std::vector<uint8_t> decompress(std::span<uint8_t const> data);

 private:
  rpp_flac_frame frame_{};
  rpp_flac_stream_info info_{};
  std::span<uint8_t const> frames_;  // the stream's frames (after its metadata blocks)
  std::vector<uint8_t>* target_ = nullptr;
  bool done_ = false;
};

// ---- PCM sample transformer (include/dwarfs/pcm_sample_transformer.h:36-71) ----
//
// pcm_sample_transformer<int32_t>: (end, sig, pad, bytes, bits) -> unpack / pack
// of interleaved PCM bytes, on the GPU (rpp_pcm_unpack / rpp_pcm_pack) through
// a pooled device context.  Throws std::runtime_error
// ("unsupported number of bytes per sample: N") like
// src/pcm_sample_transformer.cpp:310-311, std::invalid_argument for bits
// outside 1..8*bytes (an assert in the reference, :354) and for spans whose
// sizes disagree (asserts at :185,194).

enum class pcm_sample_endianness { Big, Little };
enum class pcm_sample_signedness { Signed, Unsigned };
enum class pcm_sample_padding { Lsb, Msb };

class pcm_sample_transformer {
 public:
  pcm_sample_transformer(pcm_sample_endianness end, pcm_sample_signedness sig, pcm_sample_padding pad, int bytes,
                         int bits);
  ~pcm_sample_transformer();
  pcm_sample_transformer(pcm_sample_transformer&&) noexcept;
  pcm_sample_transformer& operator=(pcm_sample_transformer&&) noexcept;

  void unpack(std::span<int32_t> dst, std::span<uint8_t const> src) const;
  void pack(std::span<uint8_t> dst, std::span<int32_t const> src) const;

 private:
  rpp_pcm_format fmt_{};
  int device_ = 0;
};

// ---- facade statistics (tests and benchmarks) ----
struct facade_stats {
  uint64_t encode_launches, encode_blocks, decode_launches, decode_blocks;
  uint64_t contexts_created;
  // summed over batches (ns): callers copying their inputs into the pinned
  // staging, the device part as the host sees it (launch to completion
  // published), and callers copying their results out
  uint64_t stage_ns, device_ns, finish_ns;
  // summed over batches (ns): the device part by the device's clock (events
  // recorded before the batch's first copy and after its last operation)
  uint64_t device_event_ns;
  // context buffers (re)allocated, and the time spent doing it (ns): a
  // pinned or device buffer that grows is freed first, which synchronises
  // the whole device
  uint64_t buffer_grows, buffer_grow_ns;
};
facade_stats get_facade_stats();

// ---- facade batch trace (diagnostics: how batches formed and overlapped) ----
// One record per batch once its last caller has left it; times are
// steady_clock nanoseconds.  Off unless enabled; take_facade_trace() returns
// the records so far and clears them.
struct facade_batch_record {
  bool encode;
  uint32_t requests;
  uint64_t in_bytes, out_bytes;
  int inflight_at_close;  // batches of the queue on the device when this one closed
  uint64_t t_open, t_close, t_ready, t_launch, t_done, t_release;
};
void set_facade_trace(bool on);
std::vector<facade_batch_record> take_facade_trace();

// Stops the facade's queues: batches on the device complete, batches not yet
// launched fail (std::runtime_error), calls made afterwards fail, and the
// queue threads are joined.  Registered with std::atexit when the first queue
// is created, so that no thread of the facade makes a HIP call while the HIP
// runtime is torn down at process exit; a program may call it earlier.
void shutdown_facade();

// Test only: the next `n` pooled-context creations fail (as a failed
// hipStreamCreate would), to exercise the error paths of the batch queue.
void inject_context_failures(uint32_t n);

// Test only: the next `n` batch launches fail after their first operation is
// on the device's stream (as a failed kernel launch after the input copy
// would), to exercise the drain of a failed batch before its buffers are reused.
void inject_launch_failures(uint32_t n);

// Benchmarks only: batches of one queue on the device at once (default 2: two
// launches on different streams overlap on the device, more do not; clamped
// to 1..16).
void set_facade_pipeline_depth(int batches);
// Benchmarks: encode batches whose worst-case output exceeds `bytes` go to
// the host by one DMA copy of their slots instead of being packed into mapped
// host memory by a kernel (default: always packed).
void set_facade_pack_limit(size_t bytes);
// Benchmarks: a batch of large requests (blocks of 4 MiB and up) that fills
// while another batch is on the device goes out once it holds this many
// requests (default 4; 1 = as soon as its first caller has copied in).
void set_facade_large_min_fill(int requests);

}  // namespace ricepp_amd
