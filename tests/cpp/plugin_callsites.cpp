// Compile-only check (tests/test_native_abi.py) that DwarFS's ricepp and FLAC plugins
// compiles against the facade with only its #include lines and the namespace
// changed.  The function bodies restate the plugin's call expressions
// (src/compression/ricepp.cpp:95-102 create_encoder with designated
// initialisers, :130-139 worst_case_encoded_bytes / encode into a subspan,
// :190-195 create_decoder, :224-228 decode, :254 the decoder member type);
// DwarFS's own types (shared_byte_buffer, thrift headers, DWARFS_THROW) are
// replaced by std:: equivalents.
#include <bit>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <span>
#include <string>
#include <vector>

// was: #include <ricepp/create_decoder.h>
//      #include <ricepp/create_encoder.h>
#include "ricepp_amd.hpp"
namespace ricepp = ricepp_amd;

namespace plugin_shape {

std::vector<uint8_t> compress(std::span<uint8_t const> data, size_t block_size_, int component_count,
                              int unused_lsb_count, int bytes_per_sample, std::string const& endianness) {
  using pixel_type = uint16_t;
  auto byteorder = endianness == "big" ? std::endian::big : std::endian::little;

  auto encoder = ricepp::create_encoder<pixel_type>({
      .block_size = block_size_,
      .component_stream_count = static_cast<size_t>(component_count),
      .byteorder = byteorder,
      .unused_lsb_count = static_cast<unsigned>(unused_lsb_count),
  });

  std::vector<uint8_t> compressed(16);
  std::span<pixel_type const> input{reinterpret_cast<pixel_type const*>(data.data()),
                                    data.size() / bytes_per_sample};
  size_t header_size = compressed.size();
  compressed.resize(header_size + encoder->worst_case_encoded_bytes(input));
  auto output = encoder->encode(std::span<uint8_t>{compressed}.subspan(header_size), input);
  compressed.resize(header_size + output.size());
  compressed.shrink_to_fit();
  return compressed;
}

struct header_values {
  size_t block_size, component_count;
  bool big_endian;
  unsigned unused_lsb_count;
};

class decompressor {
 public:
  explicit decompressor(header_values const& header_, std::span<uint8_t const> data)
      : data_{data},
        decoder_{ricepp::create_decoder<uint16_t>({.block_size = header_.block_size,
                                                   .component_stream_count = header_.component_count,
                                                   .byteorder = header_.big_endian ? std::endian::big
                                                                                   : std::endian::little,
                                                   .unused_lsb_count = header_.unused_lsb_count})} {}

  bool decompress_frame(std::vector<uint8_t>& decompressed_, size_t uncompressed_size_) {
    if (!decoder_) {
      return false;
    }
    decompressed_.resize(uncompressed_size_);
    std::span<uint16_t> output{reinterpret_cast<uint16_t*>(decompressed_.data()), decompressed_.size() / 2};
    decoder_->decode(output, data_);
    decoder_.reset();
    return true;
  }

 private:
  std::span<uint8_t const> data_;
  std::unique_ptr<ricepp::decoder_interface<uint16_t>> decoder_;
};

// the interfaces' pixel_type and const-ness match the reference's
static_assert(std::is_same_v<ricepp::encoder_interface<uint16_t>::pixel_type, uint16_t>);
static_assert(std::is_same_v<decltype(std::declval<ricepp::codec_config>().byteorder), std::endian>);

}  // namespace plugin_shape

// The FLAC plugin's classes forwarding to the facade (INTEGRATION.md §4 "The
// FLAC codec"): src/compression/flac.cpp:215-393 (compressor: compress,
// describe, metadata_requirements, get_compression_constraints) and
// :405-489 (decompressor: metadata, decompress_frame, uncompressed_size).
namespace flac_plugin_shape {

class flac_block_compressor {
 public:
  flac_block_compressor(uint32_t level, bool exhaustive) : gpu_{level, exhaustive} {}
  std::vector<uint8_t> compress(std::vector<uint8_t> const& data, std::string const* metadata) const {
    return gpu_.compress(std::span<uint8_t const>{data}, metadata);
  }
  std::string describe() const { return gpu_.describe(); }
  std::string metadata_requirements() const { return gpu_.metadata_requirements(); }
  size_t granularity(std::string const& metadata) const { return gpu_.compression_granularity(metadata); }
  size_t estimate_memory_usage(size_t data_size) const { return gpu_.estimate_memory_usage(data_size); }
  std::unique_ptr<ricepp::flac_block_compressor> clone() const { return gpu_.clone(); }

 private:
  ricepp::flac_block_compressor gpu_;
};

class flac_block_decompressor {
 public:
  explicit flac_block_decompressor(std::span<uint8_t const> data) : gpu_{data} {}
  std::optional<std::string> metadata() const { return gpu_.metadata(); }
  size_t uncompressed_size() const { return gpu_.uncompressed_size(); }
  void start_decompression(std::vector<uint8_t>* target) { gpu_.start_decompression(target); }
  bool decompress_frame(size_t frame_size) { return gpu_.decompress_frame(frame_size); }

 private:
  ricepp::flac_block_decompressor gpu_;
};

inline std::unique_ptr<ricepp::flac_block_compressor> factory(std::string const& spec) {
  return ricepp::flac_block_compressor::create(spec);  // "flac:level=8:exhaustive"
}

}  // namespace flac_plugin_shape
