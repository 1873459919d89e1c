// ricepp_facade.cpp -- C++ host facade (include/ricepp_amd.hpp) over the C ABI.
//
// Host spans are staged through device buffers on a per-object HIP stream and
// handed to rpp_encode_batch / rpp_decode_batch as a batch of one block.  The
// DwarFS plugin semantics follow src/compression/ricepp.cpp (file:line cited
// at each method).
#include "ricepp_amd.hpp"

#include <hip/hip_runtime.h>

#include <cctype>
#include <charconv>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

namespace ricepp_amd {

namespace {

void hip_check(hipError_t e, char const* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ricepp_amd: ") + what + ": " + hipGetErrorString(e));
}

rpp_config to_rpp(codec_config const& c) {
  rpp_config r{};
  r.block_size = c.block_size > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.block_size);
  r.component_stream_count =
      c.component_stream_count > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.component_stream_count);
  r.big_endian = c.order == byteorder::big ? 1u : 0u;
  r.unused_lsb_count = c.unused_lsb_count;
  return r;
}

[[noreturn]] void throw_status(int st) {
  switch (st) {
    case RPP_UNSUPPORTED_CONFIG: throw std::runtime_error("Unsupported configuration");
    case RPP_TRUNCATED_INPUT: throw std::out_of_range("bitstream_reader::read_packet");
    case RPP_INVALID_ARGUMENT: throw std::invalid_argument("ricepp_amd: invalid argument");
    case RPP_OUTPUT_TOO_SMALL: throw std::length_error("ricepp_amd: output buffer too small");
    default: throw std::runtime_error("ricepp_amd: HIP error");
  }
}

// Growable device scratch + a private stream.
class device_ctx {
 public:
  device_ctx() { hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate"); }
  ~device_ctx() {
    if (buf_) (void)hipFree(buf_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  device_ctx(device_ctx const&) = delete;
  device_ctx& operator=(device_ctx const&) = delete;

  // [params 64 B][in (16-aligned)][out (16-aligned)]
  uint8_t* reserve(size_t bytes) {
    if (bytes > cap_) {
      if (buf_) hip_check(hipFree(buf_), "hipFree");
      buf_ = nullptr;
      hip_check(hipMalloc(reinterpret_cast<void**>(&buf_), bytes), "hipMalloc");
      cap_ = bytes;
    }
    return buf_;
  }
  hipStream_t stream() const { return stream_; }

 private:
  hipStream_t stream_ = nullptr;
  uint8_t* buf_ = nullptr;
  size_t cap_ = 0;
};

size_t align16(size_t v) { return (v + 15) & ~size_t{15}; }

struct params {  // device-side per-block arrays of a batch of one
  uint64_t in_off, n, out_off, in_bytes, out_bytes;
  int32_t status, pad;
};

class encoder_impl final : public encoder {
 public:
  explicit encoder_impl(rpp_config c) : cfg_{c} {}

  size_t worst_case_encoded_bytes(size_t n) const override { return rpp_worst_case_bytes(&cfg_, n); }
  size_t worst_case_encoded_bytes(std::span<uint16_t const> in) const override {
    return worst_case_encoded_bytes(in.size());
  }

  std::vector<uint8_t> encode(std::span<uint16_t const> input) const override {
    std::vector<uint8_t> out(worst_case_encoded_bytes(input.size()));
    auto used = encode(std::span<uint8_t>{out}, input);
    out.resize(used.size());
    return out;
  }

  // ricepp_cpuspecific.cpp:101-108: output must hold the worst case
  std::span<uint8_t> encode(std::span<uint8_t> output, std::span<uint16_t const> input) const override {
    size_t const wc = worst_case_encoded_bytes(input.size());
    if (output.size() < wc) throw std::length_error("ricepp_amd: output smaller than worst_case_encoded_bytes");
    size_t const in_bytes = input.size() * 2;
    size_t const off_in = 64, off_out = off_in + align16(in_bytes);
    std::lock_guard<std::mutex> lock(mu_);  // const and re-entrant like the reference's object
    uint8_t* d = ctx_.reserve(off_out + align16(wc) + 16);
    params hp{0, input.size(), 0, 0, 0, 0, 0};
    auto* dp = reinterpret_cast<params*>(d);
    hipStream_t s = ctx_.stream();
    hip_check(hipMemcpyAsync(dp, &hp, sizeof hp, hipMemcpyHostToDevice, s), "H2D params");
    if (in_bytes) hip_check(hipMemcpyAsync(d + off_in, input.data(), in_bytes, hipMemcpyHostToDevice, s), "H2D input");
    int st = rpp_encode_batch(&cfg_, reinterpret_cast<uint16_t const*>(d + off_in), &dp->in_off, &dp->n, 1,
                              d + off_out, &dp->out_off, &dp->out_bytes, &dp->status, s);
    if (st != RPP_OK) throw_status(st);
    hip_check(hipMemcpyAsync(&hp, dp, sizeof hp, hipMemcpyDeviceToHost, s), "D2H params");
    hip_check(hipStreamSynchronize(s), "sync");
    if (hp.status != RPP_OK) throw_status(hp.status);
    hip_check(hipMemcpyAsync(output.data(), d + off_out, hp.out_bytes, hipMemcpyDeviceToHost, s), "D2H output");
    hip_check(hipStreamSynchronize(s), "sync");
    return output.subspan(0, hp.out_bytes);
  }

 private:
  rpp_config cfg_;
  mutable std::mutex mu_;
  mutable device_ctx ctx_;
};

class decoder_impl final : public decoder {
 public:
  explicit decoder_impl(rpp_config c) : cfg_{c} {}

  // ricepp_cpuspecific.cpp:127-144: decodes exactly output.size() samples
  void decode(std::span<uint16_t> output, std::span<uint8_t const> input) const override {
    size_t const off_in = 64, off_out = off_in + align16(input.size()) + 16;
    std::lock_guard<std::mutex> lock(mu_);  // const and re-entrant like the reference's object
    uint8_t* d = ctx_.reserve(off_out + align16(output.size() * 2) + 16);
    params hp{0, output.size(), 0, input.size(), 0, 0, 0};
    auto* dp = reinterpret_cast<params*>(d);
    hipStream_t s = ctx_.stream();
    hip_check(hipMemcpyAsync(dp, &hp, sizeof hp, hipMemcpyHostToDevice, s), "H2D params");
    if (!input.empty())
      hip_check(hipMemcpyAsync(d + off_in, input.data(), input.size(), hipMemcpyHostToDevice, s), "H2D input");
    int st = rpp_decode_batch(&cfg_, d + off_in, &dp->in_off, &dp->in_bytes, 1,
                              reinterpret_cast<uint16_t*>(d + off_out), &dp->out_off, &dp->n, &dp->status, s);
    if (st != RPP_OK) throw_status(st);
    hip_check(hipMemcpyAsync(&hp, dp, sizeof hp, hipMemcpyDeviceToHost, s), "D2H params");
    hip_check(hipStreamSynchronize(s), "sync");
    if (hp.status != RPP_OK) throw_status(hp.status);
    if (!output.empty())
      hip_check(hipMemcpyAsync(output.data(), d + off_out, output.size() * 2, hipMemcpyDeviceToHost, s), "D2H out");
    hip_check(hipStreamSynchronize(s), "sync");
  }

 private:
  rpp_config cfg_;
  mutable std::mutex mu_;
  mutable device_ctx ctx_;
};

// ---- minimal JSON for the flat metadata objects of the plugin ----
// (the reference uses nlohmann::json; only string and integer members occur)
std::map<std::string, std::string> parse_flat_json(std::string const& s) {
  std::map<std::string, std::string> m;
  size_t i = 0;
  auto skip = [&] {
    while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
  };
  auto str = [&]() -> std::string {
    std::string r;
    if (i >= s.size() || s[i] != '"') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    for (++i; i < s.size() && s[i] != '"'; ++i) {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      r += s[i];
    }
    ++i;
    return r;
  };
  skip();
  if (i >= s.size() || s[i] != '{') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
  ++i;
  for (;;) {
    skip();
    if (i < s.size() && s[i] == '}') break;
    std::string k = str();
    skip();
    if (i >= s.size() || s[i] != ':') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    ++i;
    skip();
    std::string v;
    if (i < s.size() && s[i] == '"') {
      v = "\"" + str();
    } else {
      while (i < s.size() && s[i] != ',' && s[i] != '}' && !std::isspace(static_cast<unsigned char>(s[i]))) v += s[i++];
    }
    m[k] = v;
    skip();
    if (i < s.size() && s[i] == ',') ++i;
  }
  return m;
}

int json_int(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] == '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks integer '") + key + "'");
  int v = 0;
  auto r = std::from_chars(it->second.data(), it->second.data() + it->second.size(), v);
  if (r.ec != std::errc{}) throw std::runtime_error(std::string("ricepp_amd: bad integer '") + key + "'");
  return v;
}

std::string json_str(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] != '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks string '") + key + "'");
  return it->second.substr(1);
}

constexpr uint32_t kRiceppVersion = 1;  // src/compression/ricepp.cpp:55

}  // namespace

std::unique_ptr<encoder> create_encoder(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<encoder_impl>(c);
}

std::unique_ptr<decoder> create_decoder(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<decoder_impl>(c);
}

// ---- block_compressor (src/compression/ricepp.cpp:57-182, 272-296) ----

block_compressor::block_compressor(size_t block_size) : block_size_{block_size} {
  if (block_size < 16 || block_size > 512)
    throw std::runtime_error("ricepp: block_size must be in [16..512]");  // options_, :284-286
}

std::unique_ptr<block_compressor> block_compressor::create(std::string const& spec) {
  // "ricepp" or "ricepp:block_size=N" (option_map, default 128, :280)
  size_t bs = 128;
  std::string name = spec.substr(0, spec.find(':'));
  if (name != "ricepp") throw std::runtime_error("unknown compression: " + name);
  if (auto c = spec.find(':'); c != std::string::npos) {
    std::string opts = spec.substr(c + 1);
    size_t p = 0;
    while (p < opts.size()) {
      size_t e = opts.find(',', p);
      std::string kv = opts.substr(p, e == std::string::npos ? std::string::npos : e - p);
      auto eq = kv.find('=');
      if (kv.substr(0, eq) != "block_size" || eq == std::string::npos)
        throw std::runtime_error("invalid option(s) for ricepp: " + kv);
      bs = std::stoul(kv.substr(eq + 1));
      if (e == std::string::npos) break;
      p = e + 1;
    }
  }
  return std::make_unique<block_compressor>(bs);
}

std::unique_ptr<block_compressor> block_compressor::clone() const {
  return std::make_unique<block_compressor>(*this);
}

std::string block_compressor::describe() const { return "ricepp [block_size=" + std::to_string(block_size_) + "]"; }

std::string block_compressor::metadata_requirements() const {
  // ricepp.cpp:150-159 (nlohmann::json dump: keys sorted)
  return R"({"bytes_per_sample":["set",[2]],"component_count":["range",1,2],)"
         R"("endianness":["set",["big","little"]],"unused_lsb_count":["range",0,8]})";
}

size_t block_compressor::compression_granularity(std::string const& metadata) const {
  auto m = parse_flat_json(metadata);  // ricepp.cpp:161-173
  return static_cast<size_t>(json_int(m, "component_count") * json_int(m, "bytes_per_sample"));
}

std::vector<uint8_t> block_compressor::compress(std::span<uint8_t const> data, std::string const* metadata) const {
  if (!metadata) throw std::runtime_error("internal error: ricepp compression requires metadata");  // :70-73
  auto meta = parse_flat_json(*metadata);
  auto endianness = json_str(meta, "endianness");
  int component_count = json_int(meta, "component_count");
  int unused_lsb_count = json_int(meta, "unused_lsb_count");
  int bytes_per_sample = json_int(meta, "bytes_per_sample");
  if (bytes_per_sample != 2 || unused_lsb_count < 0 || unused_lsb_count > 8 || component_count < 1 ||
      component_count > 2)
    throw std::runtime_error("ricepp_amd: metadata out of range");  // asserts at :82-84
  if (data.size() % static_cast<size_t>(component_count * bytes_per_sample))  // :86-91
    throw std::runtime_error("unexpected data configuration: " + std::to_string(data.size()) +
                             " bytes to compress, " + std::to_string(component_count) + " components, " +
                             std::to_string(bytes_per_sample) + " bytes per sample");
  codec_config cfg{block_size_, static_cast<size_t>(component_count),
                   endianness == "big" ? byteorder::big : byteorder::little,
                   static_cast<unsigned>(unused_lsb_count)};
  auto enc = create_encoder(cfg);
  rpp_frame f{data.size(), static_cast<uint32_t>(block_size_), static_cast<uint32_t>(component_count),
              static_cast<uint32_t>(bytes_per_sample), static_cast<uint32_t>(unused_lsb_count),
              endianness == "big" ? 1u : 0u, kRiceppVersion};
  std::vector<uint8_t> out(64);
  size_t hdr = rpp_frame_header(&f, out.data());
  size_t n = data.size() / 2;
  std::vector<uint16_t> samples(n);
  if (n) std::memcpy(samples.data(), data.data(), n * 2);
  out.resize(hdr + enc->worst_case_encoded_bytes(n));
  auto used = enc->encode(std::span<uint8_t>{out}.subspan(hdr), samples);
  out.resize(hdr + used.size());
  out.shrink_to_fit();
  return out;
}

// ---- block_decompressor (src/compression/ricepp.cpp:184-255) ----

block_decompressor::block_decompressor(std::span<uint8_t const> data) {
  long h = rpp_parse_frame(data.data(), data.size(), &frame_);
  if (h < 0) throw std::runtime_error("ricepp_amd: malformed ricepp block header");
  data_ = data.subspan(static_cast<size_t>(h));
  if (frame_.ricepp_version > kRiceppVersion)  // :243-247
    throw std::runtime_error("[RICEPP] unsupported version: " + std::to_string(frame_.ricepp_version));
  decoder_ = create_decoder({frame_.block_size, frame_.component_count,
                             frame_.big_endian ? byteorder::big : byteorder::little, frame_.unused_lsb_count});
  if (frame_.bytes_per_sample != 2)  // :196-200
    throw std::runtime_error("[RICEPP] unsupported bytes per sample: " + std::to_string(frame_.bytes_per_sample));
}

std::optional<std::string> block_decompressor::metadata() const {
  // :203-212 (nlohmann::json dump: keys sorted)
  return std::string(R"({"bytes_per_sample":)") + std::to_string(frame_.bytes_per_sample) +
         R"(,"component_count":)" + std::to_string(frame_.component_count) + R"(,"endianness":")" +
         (frame_.big_endian ? "big" : "little") + R"(","unused_lsb_count":)" +
         std::to_string(frame_.unused_lsb_count) + "}";
}

void block_decompressor::start_decompression(std::vector<uint8_t>* target) {
  target_ = target;
  target_->reserve(frame_.uncompressed_bytes);  // src/compression/base.cpp:37-51
}

bool block_decompressor::decompress_frame(size_t) {
  if (!target_) throw std::runtime_error("decompression not started");  // :216
  if (!decoder_) return false;
  target_->resize(frame_.uncompressed_bytes);
  std::span<uint16_t> out{reinterpret_cast<uint16_t*>(target_->data()), target_->size() / 2};
  decoder_->decode(out, data_);
  decoder_.reset();
  return true;
}

std::vector<uint8_t> block_decompressor::decompress(std::span<uint8_t const> data) {
  block_decompressor d{data};
  std::vector<uint8_t> out;
  d.start_decompression(&out);
  d.decompress_frame(d.uncompressed_size());
  return out;
}

// ---- pcm_sample_transformer (src/pcm_sample_transformer.cpp:372-377) ----

struct pcm_sample_transformer::impl {
  std::mutex mu;
  device_ctx ctx;
};

pcm_sample_transformer::pcm_sample_transformer(pcm_sample_endianness end, pcm_sample_signedness sig,
                                               pcm_sample_padding pad, int bytes, int bits) {
  fmt_.big_endian = end == pcm_sample_endianness::Big ? 1u : 0u;
  fmt_.is_signed = sig == pcm_sample_signedness::Signed ? 1u : 0u;
  fmt_.lsb_padded = pad == pcm_sample_padding::Lsb ? 1u : 0u;
  fmt_.bytes = bytes < 0 ? 0u : static_cast<uint32_t>(bytes);
  fmt_.bits = bits < 0 ? 0u : static_cast<uint32_t>(bits);
  const int st = rpp_pcm_check_format(&fmt_);
  if (st == RPP_UNSUPPORTED_CONFIG || bytes < 1 || bytes > 4)
    throw std::runtime_error("unsupported number of bytes per sample: " + std::to_string(bytes));
  if (st != RPP_OK) throw std::invalid_argument("pcm_sample_transformer: bits outside 1..8*bytes");
  impl_ = std::make_unique<impl>();
}

pcm_sample_transformer::~pcm_sample_transformer() = default;
pcm_sample_transformer::pcm_sample_transformer(pcm_sample_transformer&&) noexcept = default;
pcm_sample_transformer& pcm_sample_transformer::operator=(pcm_sample_transformer&&) noexcept = default;

void pcm_sample_transformer::unpack(std::span<int32_t> dst, std::span<uint8_t const> src) const {
  if (src.size() != fmt_.bytes * dst.size()) throw std::invalid_argument("pcm unpack: src.size() != bytes * dst.size()");
  if (dst.empty()) return;
  const size_t off_out = align16(src.size());
  std::lock_guard<std::mutex> lock(impl_->mu);
  uint8_t* d = impl_->ctx.reserve(off_out + dst.size_bytes());
  hipStream_t s = impl_->ctx.stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_unpack(&fmt_, d, reinterpret_cast<int32_t*>(d + off_out), dst.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size_bytes(), hipMemcpyDeviceToHost, s), "D2H pcm");
  hip_check(hipStreamSynchronize(s), "sync");
}

void pcm_sample_transformer::pack(std::span<uint8_t> dst, std::span<int32_t const> src) const {
  if (dst.size() != fmt_.bytes * src.size()) throw std::invalid_argument("pcm pack: dst.size() != bytes * src.size()");
  if (src.empty()) return;
  const size_t off_out = align16(src.size_bytes());
  std::lock_guard<std::mutex> lock(impl_->mu);
  uint8_t* d = impl_->ctx.reserve(off_out + dst.size());
  hipStream_t s = impl_->ctx.stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size_bytes(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_pack(&fmt_, reinterpret_cast<int32_t const*>(d), d + off_out, src.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size(), hipMemcpyDeviceToHost, s), "D2H pcm");
  hip_check(hipStreamSynchronize(s), "sync");
}

}  // namespace ricepp_amd
