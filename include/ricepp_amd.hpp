// ricepp_amd.hpp -- C++ host facade over the C ABI of ricepp_amd.h.
//
// Mirrors the two interfaces the reference exposes for this path:
//
//  * the ricepp library API used by DwarFS's plugin
//      ricepp::create_encoder<uint16_t> / create_decoder<uint16_t>
//        (ricepp/include/ricepp/create_encoder.h:39-41, create_decoder.h:39-41)
//      encoder_interface<uint16_t>::encode / worst_case_encoded_bytes
//        (ricepp/include/ricepp/encoder_interface.h:38-60)
//      decoder_interface<uint16_t>::decode (decoder_interface.h:37-50)
//    Errors: std::runtime_error("Unsupported configuration") for a bad
//    config, std::out_of_range when decoding runs past the input.
//
//  * the DwarFS block codec behind block_compressor / block_decompressor
//      ricepp_block_compressor / ricepp_block_decompressor
//        (src/compression/ricepp.cpp:57-182, 184-255)
//    with the same framing, metadata JSON, constraints and error messages.
//
// Host spans in, host spans out: the facade stages through device buffers on
// its own HIP stream (one per object).  Every method is const and may be
// called from several threads at once, as the reference's immutable objects
// can: an encoder / decoder / pcm_sample_transformer serialises its calls on a
// per-object lock; block_compressor::compress creates its encoder per call
// (src/compression/ricepp.cpp:97-102), so DwarFS's worker_group threads
// compressing through one impl (src/writer/filesystem_writer.cpp:259-268) run
// concurrently, one stream each.  The device-resident batch API (rpp_encode_batch /
// rpp_decode_batch) is the fast path; this facade is the drop-in.
#pragma once

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

enum class byteorder { little, big };

// ricepp::codec_config (ricepp/include/ricepp/codec_config.h:36-41)
struct codec_config {
  size_t block_size;
  size_t component_stream_count;
  byteorder order;
  unsigned unused_lsb_count;
};

class encoder {
 public:
  virtual ~encoder() = default;
  virtual std::vector<uint8_t> encode(std::span<uint16_t const> input) const = 0;
  virtual size_t worst_case_encoded_bytes(size_t pixel_count) const = 0;
  virtual size_t worst_case_encoded_bytes(std::span<uint16_t const> input) const = 0;
  virtual std::span<uint8_t> encode(std::span<uint8_t> output, std::span<uint16_t const> input) const = 0;
};

class decoder {
 public:
  virtual ~decoder() = default;
  virtual void decode(std::span<uint16_t> output, std::span<uint8_t const> input) const = 0;
};

// throw std::runtime_error("Unsupported configuration") like
// ricepp/ricepp_cpuspecific.cpp:161,173
std::unique_ptr<encoder> create_encoder(codec_config const& config);
std::unique_ptr<decoder> create_decoder(codec_config const& config);

// ---- DwarFS block codec (src/compression/ricepp.cpp) ----

// compression_type::RICEPP (include/dwarfs/compression.h, RICEPP = 7)
inline constexpr int compression_type_ricepp = 7;

class block_compressor {
 public:
  explicit block_compressor(size_t block_size = 128);  // "ricepp:block_size=N", N in [16, 512]
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
  std::unique_ptr<decoder> decoder_;
  std::vector<uint8_t>* target_ = nullptr;
};

// ---- PCM sample transformer (include/dwarfs/pcm_sample_transformer.h:36-71) ----
//
// pcm_sample_transformer<int32_t>: (end, sig, pad, bytes, bits) -> unpack / pack
// of interleaved PCM bytes, on the GPU (rpp_pcm_unpack / rpp_pcm_pack) through
// a private stream and device staging buffer.  Throws std::runtime_error
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
  struct impl;
  rpp_pcm_format fmt_{};
  std::unique_ptr<impl> impl_;
};

}  // namespace ricepp_amd
