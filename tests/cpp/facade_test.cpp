// C++ facade test (runs on a GPU box).  Mirrors the reference tests of the
// path: ricepp/test/codec_test.cpp (round trips, worst-case KATs, error
// contract) and test/ricepp_compressor_test.cpp (block_compressor spec
// round trip), checking every stream against the CPU oracle byte for byte.
#include <atomic>
#include <bit>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
#include <span>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ricepp_amd.hpp"

extern "C" {  // CPU oracle (oracle/ricepp_oracle.c), the checker
struct rpo_config {
  uint32_t block_size, component_stream_count, big_endian, unused_lsb_count;
};
size_t rpo_worst_case_bytes(const rpo_config*, size_t);
int rpo_encode(const rpo_config*, const uint16_t*, size_t, uint8_t*, size_t, size_t*);
size_t rpo_frame_header(uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint32_t, int, uint32_t);
// FLAC restatement (oracle/flac_oracle.c), an independent encoder / decoder
typedef struct {
  int subframe_type, fixed_order, lpc_order, lpc_precision, stereo, max_partition_order, rice2, escape,
      padding_block, wasted, variable_blocking, max_lpc_order;
} fo_opts;
size_t fo_encode(const int32_t* x, uint64_t nsamples, uint32_t channels, uint32_t bps, uint32_t blocksize,
                 const fo_opts* opts, uint8_t* out, size_t cap);
int fo_decode(const uint8_t* in, size_t len, int32_t* out, uint64_t cap, uint32_t* channels_out, uint32_t* bps_out,
              uint64_t* nsamples_out);
}

static int failures = 0;
#define CHECK(cond)                                                         \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                           \
    }                                                                       \
  } while (0)

template <class E, class F>
static bool throws(F&& f, char const* msg = nullptr) {
  try {
    f();
  } catch (E const& e) {
    return !msg || std::string(e.what()) == msg;
  } catch (...) {
    return false;
  }
  return false;
}

static uint16_t bswap(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

// codec_test.cpp:43-61 shape: noise U[20000,21000], full-range outliers
static std::vector<uint16_t> make_data(size_t n, unsigned ulsb, bool be, unsigned full_chance, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::uniform_int_distribution<unsigned> dist(0, full_chance);
  std::uniform_int_distribution<unsigned> noise(20000, 21000), full(0, 65535);
  std::vector<uint16_t> v(n);
  uint16_t mask = (uint16_t)(0xFFFFu << ulsb);
  for (auto& x : v) {
    uint16_t s = (uint16_t)((dist(rng) == 0 ? full(rng) : noise(rng)) & mask);
    x = be ? bswap(s) : s;
  }
  return v;
}

static ricepp_amd::codec_config cfg(size_t bs, size_t cs, bool big, unsigned ulsb) {
  return {.block_size = bs,
          .component_stream_count = cs,
          .byteorder = big ? std::endian::big : std::endian::little,
          .unused_lsb_count = ulsb};
}

static std::vector<uint8_t> oracle_encode(ricepp_amd::codec_config const& c, std::vector<uint16_t> const& x) {
  rpo_config oc{(uint32_t)c.block_size, (uint32_t)c.component_stream_count,
                c.byteorder == std::endian::big ? 1u : 0u, c.unused_lsb_count};
  std::vector<uint8_t> out(rpo_worst_case_bytes(&oc, x.size()) + 1);
  size_t n = 0;
  if (rpo_encode(&oc, x.data(), x.size(), out.data(), out.size(), &n) != 0) std::abort();
  out.resize(n);
  return out;
}

static void roundtrip(ricepp_amd::codec_config const& c, size_t n, unsigned full_chance, uint64_t seed) {
  auto x = make_data(n, c.unused_lsb_count, c.byteorder == std::endian::big, full_chance, seed);
  auto enc = ricepp_amd::create_encoder<uint16_t>(c);
  auto bytes = enc->encode(x);
  CHECK(bytes == oracle_encode(c, x));
  auto dec = ricepp_amd::create_decoder<uint16_t>(c);
  std::vector<uint16_t> y(x.size());
  dec->decode(y, bytes);
  CHECK(y == x);
}

int bench(int argc, char** argv);
int exit_in_flight();
void flac_tests();

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "--bench") return bench(argc, argv);
  if (argc > 1 && std::string(argv[1]) == "--exit-in-flight") return exit_in_flight();
  // the batch queue's error paths (round-2 review): the first pooled context
  // fails to come up; the callers of that batch get an exception, none hangs,
  // and the queue and pool work afterwards
  {
    ricepp_amd::inject_context_failures(1);
    auto c = cfg(128, 1, true, 0);
    auto x = make_data(65536, 0, true, 50, 21);
    std::atomic<int> errs{0}, oks{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&] {
        try {
          auto bytes = ricepp_amd::create_encoder<uint16_t>(c)->encode(x);
          ++oks;
        } catch (std::runtime_error const&) {
          ++errs;
        }
      });
    for (auto& t : th) t.join();
    CHECK(errs.load() >= 1);
    CHECK(errs.load() + oks.load() == 8);
    roundtrip(c, 65536, 50, 22);
  }
  // a launch that fails after its input copy is on the stream:
  // the batch's callers get an exception, the context is drained before its
  // buffers go back to the pool, and later batches on it are exact
  for (int dir = 0; dir < 2; ++dir) {
    auto c = cfg(128, 1, true, 0);
    auto x = make_data(65536, 0, true, 50, 23 + dir);
    auto want = oracle_encode(c, x);
    ricepp_amd::inject_launch_failures(1);
    std::atomic<int> errs{0}, oks{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t)
      th.emplace_back([&] {
        try {
          if (dir == 0) {
            CHECK(ricepp_amd::create_encoder<uint16_t>(c)->encode(x) == want);
          } else {
            std::vector<uint16_t> y(x.size());
            ricepp_amd::create_decoder<uint16_t>(c)->decode(y, want);
            CHECK(y == x);
          }
          ++oks;
        } catch (std::runtime_error const&) {
          ++errs;
        }
      });
    for (auto& t : th) t.join();
    CHECK(errs.load() >= 1);
    CHECK(errs.load() + oks.load() == 8);
    for (int k = 0; k < 4; ++k) roundtrip(c, 65536, 50, 30 + k);
  }
  // codec_test.cpp:65-152
  roundtrip(cfg(16, 1, true, 0), 12345, 50, 1);
  roundtrip(cfg(13, 1, true, 4), 4321, 50, 2);
  roundtrip(cfg(32, 1, true, 0), 1500, 0, 3);
  roundtrip(cfg(29, 2, true, 2), 23456, 50, 4);
  roundtrip(cfg(128, 1, false, 0), 65536, 50, 5);
  roundtrip(cfg(512, 2, false, 3), 10000, 50, 6);
  roundtrip(cfg(8, 1, true, 0), 3001, 50, 11);  // the factory accepts any size <= 512
  // DwarFS block sizes (mkdwarfs -S 22 / -S 24): one call = one long stream, encoded and
  // decoded by several waves (the segmented paths behind the facade's _ws launches)
  roundtrip(cfg(128, 1, true, 0), (size_t)8 << 20, 50, 12);
  roundtrip(cfg(128, 2, false, 2), (size_t)2 << 20, 50, 13);

  // codec_test.cpp:154-196: worst-case KATs; incompressible == worst case
  {
    auto c = cfg(29, 1, true, 0);
    auto enc = ricepp_amd::create_encoder<uint16_t>(c);
    auto x = make_data(14443, 0, true, 0, 7);
    CHECK(enc->worst_case_encoded_bytes(x) == 29138);
    std::vector<uint8_t> buf(29138);
    auto used = enc->encode(buf, x);
    CHECK(used.size() == 29138);
    auto enc2 = ricepp_amd::create_encoder<uint16_t>(cfg(29, 2, true, 0));
    CHECK(enc2->worst_case_encoded_bytes(28886) == 58275);
  }
  // codec_test.cpp:198-222
  CHECK(throws<std::runtime_error>([] { ricepp_amd::create_encoder<uint16_t>(cfg(513, 2, true, 0)); },
                                   "Unsupported configuration"));
  CHECK(throws<std::runtime_error>([] { ricepp_amd::create_decoder<uint16_t>(cfg(128, 3, true, 0)); },
                                   "Unsupported configuration"));
  // bitstream_reader.h:150-152: running out of input is std::out_of_range
  {
    auto c = cfg(128, 1, true, 0);
    auto x = make_data(4096, 0, true, 50, 8);
    auto bytes = ricepp_amd::create_encoder<uint16_t>(c)->encode(x);
    bytes.resize((bytes.size() - 1) / 8 * 8);
    std::vector<uint16_t> y(x.size());
    auto dec = ricepp_amd::create_decoder<uint16_t>(c);
    CHECK(throws<std::out_of_range>([&] { dec->decode(y, bytes); }));
  }

  // test/ricepp_compressor_test.cpp:124-161 through the block codec
  struct P {
    int cs, pixels, ulsb, block;
  };
  for (P p : {P{1, 1000, 0, 16}, P{2, 1000, 2, 32}, P{1, 1000, 4, 64}, P{2, 3333, 6, 99}, P{1, 777, 0, 8}}) {
    auto x = make_data((size_t)p.cs * p.pixels, (unsigned)p.ulsb, true, 50, 9);
    std::vector<uint8_t> data(x.size() * 2);
    std::memcpy(data.data(), x.data(), data.size());
    std::string meta = "{\"endianness\":\"big\",\"bytes_per_sample\":2,\"unused_lsb_count\":" +
                       std::to_string(p.ulsb) + ",\"component_count\":" + std::to_string(p.cs) + "}";
    auto comp = ricepp_amd::block_compressor::create("ricepp:block_size=" + std::to_string(p.block));
    CHECK(comp->describe() == "ricepp [block_size=" + std::to_string(p.block) + "]");
    CHECK(comp->compression_granularity(meta) == (size_t)(2 * p.cs));
    auto compressed = comp->compress(data, &meta);
    // framing + bitstream identical to the reference layout
    std::vector<uint8_t> want(64);
    size_t h = rpo_frame_header(want.data(), data.size(), (uint32_t)p.block, (uint32_t)p.cs, 2, (uint32_t)p.ulsb, 1, 1);
    want.resize(h);
    auto body = oracle_encode(cfg((size_t)p.block, (size_t)p.cs, true, (unsigned)p.ulsb), x);
    want.insert(want.end(), body.begin(), body.end());
    CHECK(compressed == want);
    // (ratio < 0.7 needs the compressor test generator; covered by tests/test_gpu_block_codec.py)
    auto back = ricepp_amd::block_decompressor::decompress(compressed);
    CHECK(back == data);
    ricepp_amd::block_decompressor d{compressed};
    CHECK(d.uncompressed_size() == data.size());
    CHECK(*d.metadata() == "{\"bytes_per_sample\":2,\"component_count\":" + std::to_string(p.cs) +
                               ",\"endianness\":\"big\",\"unused_lsb_count\":" + std::to_string(p.ulsb) + "}");
  }
  // plugin error contract (src/compression/ricepp.cpp:70-73, 86-91, 196-200, 243-247)
  {
    ricepp_amd::block_compressor comp{128};
    std::vector<uint8_t> odd(7);
    std::string meta = R"({"endianness":"big","bytes_per_sample":2,"unused_lsb_count":0,"component_count":1})";
    CHECK(throws<std::runtime_error>([&] { comp.compress(odd, nullptr); },
                                     "internal error: ricepp compression requires metadata"));
    CHECK(throws<std::runtime_error>([&] { comp.compress(odd, &meta); },
                                     "unexpected data configuration: 7 bytes to compress, 1 components, 2 bytes per sample"));
    std::vector<uint8_t> v2(64);
    v2.resize(rpo_frame_header(v2.data(), 16, 128, 1, 2, 0, 1, 2));
    CHECK(throws<std::runtime_error>([&] { ricepp_amd::block_decompressor d{v2}; }, "[RICEPP] unsupported version: 2"));
    std::vector<uint8_t> b3(64);
    b3.resize(rpo_frame_header(b3.data(), 16, 128, 1, 3, 0, 1, 1));
    CHECK(throws<std::runtime_error>([&] { ricepp_amd::block_decompressor d{b3}; },
                                     "[RICEPP] unsupported bytes per sample: 3"));
    // the factory does not range-check block_size (src/compression/ricepp.cpp:277-281); an
    // unsupported size fails in create_encoder at compress time (:97-102)
    auto big = ricepp_amd::block_compressor::create("ricepp:block_size=513");
    CHECK(big->describe() == "ricepp [block_size=513]");
    std::vector<uint8_t> two(4);
    CHECK(throws<std::runtime_error>([&] { big->compress(two, &meta); }, "Unsupported configuration"));
    CHECK(comp.metadata_requirements() ==
          R"({"bytes_per_sample":["set",[2]],"component_count":["range",1,2],"endianness":["set",["big","little"]],"unused_lsb_count":["range",0,8]})");
  }
  // concurrency: DwarFS's worker_group calls compress on one block_compressor
  // impl from many threads (src/writer/filesystem_writer.cpp:259-268); the
  // reference's encoder/decoder objects are const and re-entrant.  8 threads
  // share one compressor, one encoder and one decoder; every stream is checked
  // against the oracle.
  {
    auto c = cfg(128, 1, true, 0);
    auto shared_enc = ricepp_amd::create_encoder<uint16_t>(c);
    auto shared_dec = ricepp_amd::create_decoder<uint16_t>(c);
    ricepp_amd::block_compressor comp{128};
    std::string const meta =
        R"({"bytes_per_sample":2,"component_count":1,"endianness":"big","unused_lsb_count":0})";
    std::vector<int> bad(8, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < 8; ++t) {
      pool.emplace_back([&, t] {
        for (int i = 0; i < 6; ++i) {
          auto x = make_data(20000 + 997 * t + 31 * i, 0, true, 50, 1000 + 10 * t + i);
          auto bytes = shared_enc->encode(x);
          if (bytes != oracle_encode(c, x)) ++bad[t];
          std::vector<uint16_t> y(x.size());
          shared_dec->decode(y, bytes);
          if (y != x) ++bad[t];
          std::vector<uint8_t> raw(x.size() * 2);
          std::memcpy(raw.data(), x.data(), raw.size());
          auto framed = comp.compress(raw, &meta);
          if (ricepp_amd::block_decompressor::decompress(framed) != raw) ++bad[t];
        }
      });
    }
    for (auto& th : pool) th.join();
    for (int t = 0; t < 8; ++t) CHECK(bad[t] == 0);
  }
  // test/pcm_sample_transformer_test.cpp:33-52 (uint8_8bit) and :258-293 (int24_20bit_be_lsb)
  {
    using namespace ricepp_amd;
    pcm_sample_transformer x8(pcm_sample_endianness::Big, pcm_sample_signedness::Unsigned, pcm_sample_padding::Msb, 1,
                              8);
    std::vector<uint8_t> packed{0, 1, 42, 254, 255}, repacked(5);
    std::vector<int32_t> unpacked(5);
    x8.unpack(unpacked, packed);
    x8.pack(repacked, unpacked);
    CHECK((unpacked == std::vector<int32_t>{-128, -127, -86, 126, 127}));
    CHECK(repacked == packed);
    pcm_sample_transformer x24(pcm_sample_endianness::Big, pcm_sample_signedness::Signed, pcm_sample_padding::Lsb, 3,
                               20);
    std::vector<int32_t> ref{-524288, -524287, -1, 0, 1, 524286, 524287}, u(7);
    std::vector<uint8_t> p(21), rp(21);
    for (size_t i = 0; i < ref.size(); ++i) {
      const uint32_t v = static_cast<uint32_t>(ref[i]) << 4;
      p[3 * i] = uint8_t(v >> 16), p[3 * i + 1] = uint8_t(v >> 8), p[3 * i + 2] = uint8_t(v);
    }
    x24.unpack(u, p);
    x24.pack(rp, u);
    CHECK(u == ref);
    CHECK(rp == p);
    CHECK(throws<std::runtime_error>(
        [] { pcm_sample_transformer t(pcm_sample_endianness::Big, pcm_sample_signedness::Signed,
                                      pcm_sample_padding::Lsb, 5, 16); },
        "unsupported number of bytes per sample: 5"));
  }
  // batching: 64 threads encoding and decoding at once through one
  // configuration are coalesced into fewer launches than calls, and every
  // result is still the oracle's
  {
    auto c = cfg(64, 2, false, 1);
    auto const before = ricepp_amd::get_facade_stats();
    std::vector<int> bad(64, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < 64; ++t) {
      pool.emplace_back([&, t] {
        auto enc = ricepp_amd::create_encoder<uint16_t>(c);
        auto dec = ricepp_amd::create_decoder<uint16_t>(c);
        for (int i = 0; i < 8; ++i) {
          auto x = make_data(2 * (3000 + 101 * t + 7 * i), 1, false, 50, 5000 + 100 * t + i);
          auto bytes = enc->encode(x);
          if (bytes != oracle_encode(c, x)) ++bad[t];
          std::vector<uint16_t> y(x.size());
          dec->decode(y, bytes);
          if (y != x) ++bad[t];
        }
      });
    }
    for (auto& th : pool) th.join();
    for (int t = 0; t < 64; ++t) CHECK(bad[t] == 0);
    auto const after = ricepp_amd::get_facade_stats();
    CHECK(after.encode_blocks - before.encode_blocks == 64 * 8);
    CHECK(after.decode_blocks - before.decode_blocks == 64 * 8);
    CHECK(after.encode_launches - before.encode_launches < 64 * 8);
    std::printf("batching: %llu encode calls in %llu launches, %llu decode calls in %llu launches, %llu contexts\n",
                (unsigned long long)(after.encode_blocks - before.encode_blocks),
                (unsigned long long)(after.encode_launches - before.encode_launches),
                (unsigned long long)(after.decode_blocks - before.decode_blocks),
                (unsigned long long)(after.decode_launches - before.decode_launches),
                (unsigned long long)after.contexts_created);
  }
  // long blocks from many threads: 16 threads x 3 blocks of 8 MiB, joined into
  // multi-block segmented launches with two batches in flight on separate
  // contexts (the case whose device buffers a stream-ordered allocator mixed
  // up); every stream against the oracle, every decode against its input
  {
    auto c = cfg(128, 1, true, 0);
    std::vector<int> bad(16, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < 16; ++t) {
      pool.emplace_back([&, t] {
        auto enc = ricepp_amd::create_encoder<uint16_t>(c);
        auto dec = ricepp_amd::create_decoder<uint16_t>(c);
        for (int i = 0; i < 3; ++i) {
          auto x = make_data(size_t{4} << 20, 0, true, 50, 7000 + 10 * t + i);
          auto bytes = enc->encode(x);
          if (bytes != oracle_encode(c, x)) ++bad[t];
          std::vector<uint16_t> y(x.size());
          dec->decode(y, bytes);
          if (y != x) ++bad[t];
        }
      });
    }
    for (auto& th : pool) th.join();
    for (int t = 0; t < 16; ++t) CHECK(bad[t] == 0);
  }
  // the batch shape of round 4's all-blocks RPP_INVALID_ARGUMENT record
  // (gpurun_out/r04/f16p.err): 7 concurrent 8 Mi-sample encodes joined into one
  // segmented launch (whose device-side parameter arrays the stream-ordered
  // allocator had overwritten), then decoded back
  {
    auto c = cfg(128, 1, true, 0);
    std::vector<std::vector<uint16_t>> xs(7);
    std::vector<std::vector<uint8_t>> bytes(7);
    for (int t = 0; t < 7; ++t) xs[t] = make_data(size_t{8} << 20, 0, true, 50, 9100 + t);
    std::vector<int> bad(7, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < 7; ++t)
      pool.emplace_back([&, t] { bytes[t] = ricepp_amd::create_encoder<uint16_t>(c)->encode(xs[t]); });
    for (auto& th : pool) th.join();
    pool.clear();
    for (int t = 0; t < 7; ++t)
      pool.emplace_back([&, t] {
        if (bytes[t] != oracle_encode(c, xs[t])) ++bad[t];
        std::vector<uint16_t> y(xs[t].size());
        ricepp_amd::create_decoder<uint16_t>(c)->decode(y, bytes[t]);
        if (y != xs[t]) ++bad[t];
      });
    for (auto& th : pool) th.join();
    for (int t = 0; t < 7; ++t) CHECK(bad[t] == 0);
  }
  // device time by the device's clock is recorded per batch
  CHECK(ricepp_amd::get_facade_stats().device_event_ns > 0);
  flac_tests();
  std::printf("facade_test: %s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}

// Summary of a run's batch trace (facade_test --bench ... --trace): per
// direction the batches, their sizes, how many were on the device at once,
// and the mean time per batch in each phase (open -> close: gathering
// callers; close -> ready: the last caller's copy in; ready -> launch: the
// driver; launch -> done: device; done -> release: copies out).
std::string trace_summary(std::vector<ricepp_amd::facade_batch_record> recs, std::chrono::steady_clock::time_point w0,
                          std::chrono::steady_clock::time_point w1, std::chrono::steady_clock::time_point w2) {
  auto ns = [](std::chrono::steady_clock::time_point t) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
  };
  std::string out;
  for (int enc = 1; enc >= 0; --enc) {
    std::vector<ricepp_amd::facade_batch_record> v;
    for (auto& r : recs)
      if (r.encode == (enc == 1)) v.push_back(r);
    std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.t_launch < b.t_launch; });
    const uint64_t a = ns(enc ? w0 : w1), z = ns(enc ? w1 : w2);
    double ph[5] = {0, 0, 0, 0, 0};
    uint32_t rmin = ~0u, rmax = 0, rsum = 0;
    int closed_busy = 0;
    std::string sizes;  // (at most 40 listed)
    for (auto& r : v) {
      ph[0] += r.t_close - r.t_open;
      ph[1] += r.t_ready - r.t_close;
      ph[2] += r.t_launch - r.t_ready;
      ph[3] += r.t_done - r.t_launch;
      ph[4] += r.t_release - r.t_done;
      rmin = std::min(rmin, r.requests);
      rmax = std::max(rmax, r.requests);
      rsum += r.requests;
      closed_busy += r.inflight_at_close > 0;
      if (&r - v.data() < 40) sizes += (sizes.empty() ? "" : ",") + std::to_string(r.requests);
    }
    // time with >= 2 batches between launch and done, over the run's wall time
    std::vector<std::pair<uint64_t, int>> ev;
    for (auto& r : v) {
      ev.emplace_back(r.t_launch, +1);
      ev.emplace_back(r.t_done, -1);
    }
    std::sort(ev.begin(), ev.end());
    uint64_t two = 0, idle = 0, prev = a;
    int cur = 0;
    for (auto& [t, d] : ev) {
      const uint64_t tt = std::clamp(t, a, z);
      if (cur >= 2) two += tt - prev;
      if (cur == 0) idle += tt - prev;
      prev = tt;
      cur += d;
    }
    if (prev < z && cur == 0) idle += z - prev;
    const double nb = v.empty() ? 1.0 : double(v.size()), wall = double(z - a);
    char buf[1024];
    std::snprintf(buf, sizeof buf,
                  ", \"%s_trace\": {\"batches\": %zu, \"requests\": [%s], \"closed_while_busy\": %d, "
                  "\"two_in_flight_frac\": %.3f, \"device_idle_frac\": %.3f, \"us_per_batch\": {\"gather\": %.0f, "
                  "\"stage\": %.0f, \"driver\": %.0f, \"device\": %.0f, \"finish\": %.0f}}",
                  enc ? "encode" : "decode", v.size(), sizes.c_str(), closed_busy, two / wall, idle / wall,
                  ph[0] / nb / 1e3, ph[1] / nb / 1e3, ph[2] / nb / 1e3, ph[3] / nb / 1e3, ph[4] / nb / 1e3);
    out += buf;
    (void)rmin; (void)rmax; (void)rsum;
  }
  return out;
}

// ---- facade throughput (facade_test --bench [blocks] [threads...]) ----
// DwarFS's worker_group shape: T threads, each compressing / decompressing
// its share of B independent 64 KiB blocks through the facade (host spans in
// and out, so PCIe and host copies are included).  One JSON line per T.
// (--kib=K: blocks of K KiB instead of 64; DwarFS's own block size is
// 16 MiB at mkdwarfs' default -S 24)
int bench(int argc, char** argv) {
  size_t const blocks = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 4096;
  std::vector<int> threads;
  size_t kib = 64;
  int depth = 0;  // 0: the library's default
  int repeat = 1;
  bool trace = false;
  for (int i = 3; i < argc; ++i) {
    if (std::string(argv[i]).rfind("--kib=", 0) == 0) kib = std::strtoul(argv[i] + 6, nullptr, 10);
    else if (std::string(argv[i]).rfind("--repeat=", 0) == 0) repeat = std::atoi(argv[i] + 9);
    else if (std::string(argv[i]) == "--trace") trace = true;
    else if (std::string(argv[i]).rfind("--min-fill=", 0) == 0)
      ricepp_amd::set_facade_large_min_fill(std::atoi(argv[i] + 11));
    else if (std::string(argv[i]).rfind("--depth=", 0) == 0) depth = std::atoi(argv[i] + 8);
    else if (std::string(argv[i]).rfind("--pack-max-mib=", 0) == 0)
      ricepp_amd::set_facade_pack_limit(std::strtoull(argv[i] + 15, nullptr, 10) << 20);
    else threads.push_back(std::atoi(argv[i]));
  }
  if (threads.empty()) threads = {1, 8, 64};
  if (depth) ricepp_amd::set_facade_pipeline_depth(depth);
  size_t const n = kib * 512;  // samples per block
  auto c = cfg(128, 1, true, 0);
  std::vector<std::vector<uint16_t>> in(blocks);
  std::mt19937_64 rng(42);
  std::poisson_distribution<int> pois(1000.0);
  for (auto& v : in) {
    v.resize(n);
    for (auto& x : v) x = bswap((uint16_t)pois(rng));
  }
  // (encoded into preallocated worst-case buffers through the span form, as
  // the plugin does: src/compression/ricepp.cpp:134-137)
  size_t const wc = ricepp_amd::create_encoder<uint16_t>(c)->worst_case_encoded_bytes(n);
  std::vector<std::vector<uint8_t>> encbuf(blocks, std::vector<uint8_t>(wc));
  std::vector<std::span<uint8_t>> enc(blocks);
  std::vector<std::vector<uint16_t>> out(blocks, std::vector<uint16_t>(n));
  std::atomic<bool> failed{false};
  for (int T : threads) {
    auto run = [&](bool encode) {
      std::vector<std::thread> pool;
      auto t0 = std::chrono::steady_clock::now();
      for (int t = 0; t < T; ++t) {
        pool.emplace_back([&, t] {
          auto e = ricepp_amd::create_encoder<uint16_t>(c);
          auto d = ricepp_amd::create_decoder<uint16_t>(c);
          for (size_t b = t; b < blocks && !failed.load(); b += T) {
            try {
              if (encode) enc[b] = e->encode(std::span<uint8_t>{encbuf[b]}, in[b]);
              else d->decode(out[b], enc[b]);
            } catch (std::exception const& x) {
              // (reported and returned from main: never exit() from a worker
              // while the others are still inside the facade)
              std::fprintf(stderr, "facade bench: %s of block %zu (%zu encoded bytes): %s\n",
                           encode ? "encode" : "decode", b, enc[b].size(), x.what());
              failed.store(true);
            }
          }
        });
      }
      for (auto& th : pool) th.join();
      return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    // warm the contexts (both directions: decode grows their buffers
    // differently); three times, since batches form differently from pass to
    // pass and a context first created by a later pass grows its pinned
    // buffers then, ~50-70 ms (each run reports contexts_created and
    // buffer_grows)
    for (int w = 0; w < 3; ++w) {
      run(true);
      run(false);
    }
    for (int rep = 0; rep < repeat; ++rep) {
    if (trace) {
      ricepp_amd::set_facade_trace(true);
      (void)ricepp_amd::take_facade_trace();
    }
    auto s0 = ricepp_amd::get_facade_stats();
    const auto w0 = std::chrono::steady_clock::now();
    double te = run(true);
    const auto w1 = std::chrono::steady_clock::now();
    auto s1 = ricepp_amd::get_facade_stats();
    double td = run(false);
    const auto w2 = std::chrono::steady_clock::now();
    auto s2 = ricepp_amd::get_facade_stats();
    std::string trace_json;
    if (trace) trace_json = trace_summary(ricepp_amd::take_facade_trace(), w0, w1, w2);
    if (failed.load()) return 3;
    bool ok = true;
    int reported = 0;
    for (size_t b = 0; b < blocks; ++b) {
      if (out[b] == in[b]) continue;
      ok = false;
      if (reported++ >= 8) continue;
      // which side is wrong: the stream against the oracle's, the samples
      // against the input (and against the other blocks' inputs)
      auto want = oracle_encode(c, in[b]);
      std::vector<uint8_t> got(enc[b].begin(), enc[b].end());
      size_t ed = 0;
      while (ed < std::min(got.size(), want.size()) && got[ed] == want[ed]) ++ed;
      size_t sd = 0;
      while (sd < n && out[b][sd] == in[b][sd]) ++sd;
      long other = -1;
      for (size_t o = 0; o < blocks && other < 0; ++o)
        if (o != b && out[b] == in[o]) other = (long)o;
      std::fprintf(stderr,
                   "facade bench: block %zu mismatch: stream %zu B (oracle %zu B, first diff %zu); first sample diff "
                   "%zu of %zu; equals input of block %ld\n",
                   b, got.size(), want.size(), ed, sd, n, other);
    }
    double gib = double(blocks) * n * 2 / double(1ull << 30);
    const double ne = double(s1.encode_launches - s0.encode_launches), nd = double(s2.decode_launches - s1.decode_launches);
    std::printf("{\"facade_bench\": true, \"threads\": %d, \"depth\": %d, \"blocks\": %zu, \"block_bytes\": %zu, "
                "\"encode_GiBps\": %.3f, \"decode_GiBps\": %.3f, \"encode_launches\": %.0f, "
                "\"decode_launches\": %.0f, \"encode_us_per_batch\": {\"stage\": %.1f, \"device\": %.1f, "
                "\"device_events\": %.1f, \"finish\": %.1f}, \"decode_us_per_batch\": {\"stage\": %.1f, \"device\": %.1f, "
                "\"device_events\": %.1f, \"finish\": %.1f}, \"contexts_created\": %llu, \"buffer_grows\": %llu, "
                "\"buffer_grow_ms\": %.2f, \"roundtrip_ok\": %s%s}\n",
                T, depth, blocks, n * 2, gib / te, gib / td, ne, nd, (s1.stage_ns - s0.stage_ns) / 1e3 / ne,
                (s1.device_ns - s0.device_ns) / 1e3 / ne, (s1.device_event_ns - s0.device_event_ns) / 1e3 / ne,
                (s1.finish_ns - s0.finish_ns) / 1e3 / ne, (s2.stage_ns - s1.stage_ns) / 1e3 / nd,
                (s2.device_ns - s1.device_ns) / 1e3 / nd, (s2.device_event_ns - s1.device_event_ns) / 1e3 / nd,
                (s2.finish_ns - s1.finish_ns) / 1e3 / nd, (unsigned long long)(s2.contexts_created - s0.contexts_created),
                (unsigned long long)(s2.buffer_grows - s0.buffer_grows), (s2.buffer_grow_ns - s0.buffer_grow_ns) / 1e6,
                ok ? "true" : "false", trace_json.c_str());
    std::fflush(stdout);
    if (!ok) return 1;
    }
  }
  return 0;
}

// ---- process exit while batches are in flight (facade_test --exit-in-flight) ----
// 8 worker threads encode and decode 64 KiB and 4 MiB blocks in a loop; one of
// them calls std::exit(0) while the others' batches are queued or on the
// device.  The facade's atexit hook stops its queues before the HIP runtime
// is torn down: the exit status must be 0 (no abort, no core dump).  Workers
// that get "facade shut down" afterwards stop quietly.
int exit_in_flight() {
  auto c = cfg(128, 1, true, 0);
  std::vector<std::thread> pool;
  std::atomic<int> rounds{0};
  for (int t = 0; t < 8; ++t) {
    pool.emplace_back([&, t] {
      auto x = make_data(t % 2 ? size_t{2} << 20 : 32768, 0, true, 50, 300 + t);
      try {
        auto e = ricepp_amd::create_encoder<uint16_t>(c);
        auto d = ricepp_amd::create_decoder<uint16_t>(c);
        for (int i = 0;; ++i) {
          auto bytes = e->encode(x);
          std::vector<uint16_t> y(x.size());
          d->decode(y, bytes);
          if (y != x) {
            std::fprintf(stderr, "exit-in-flight: round trip mismatch\n");
            std::_Exit(4);
          }
          ++rounds;
          if (t == 0 && rounds.load() >= 200) {
            std::printf("exit-in-flight: exiting after %d round trips\n", rounds.load());
            std::fflush(stdout);
            std::exit(0);
          }
        }
      } catch (std::exception const&) {  // (the facade was shut down under this thread)
      }
    });
  }
  for (auto& th : pool) th.join();
  std::printf("exit-in-flight: workers ended before the exit\n");
  return 5;
}

// ---- FLAC block codec (src/compression/flac.cpp; test/flac_compressor_test.cpp:97-205) ----
// Parity unpinned (libFLAC is absent): the C++ compressor's stream is decoded
// by the independent restatement, and the restatement's streams (LPC order 8,
// as libFLAC level 5 writes) by the C++ decompressor.
static std::vector<int32_t> flac_signal(size_t frames, uint32_t channels, uint32_t bits, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<int32_t> x(frames * channels);
  const double amp = double((int64_t(1) << (bits - 1)) - 1) * 0.6;
  for (size_t i = 0; i < frames; ++i)
    for (uint32_t c = 0; c < channels; ++c)
      x[i * channels + c] = int32_t(amp * std::sin(0.001 * double(i) * (1.0 + c)) + double(int(rng() % 17) - 8));
  return x;
}

void flac_tests() {
  using ricepp_amd::flac_block_compressor;
  using ricepp_amd::flac_block_decompressor;
  const std::string meta16 = R"({"bits_per_sample":16,"bytes_per_sample":2,"endianness":"little",)"
                             R"("number_of_channels":2,"padding":"msb","signedness":"signed"})";
  // factory, describe, requirements, constraints (flac.cpp:363-393, 509-525)
  CHECK(flac_block_compressor::create("flac")->describe() == "flac [level=5]");
  CHECK(flac_block_compressor::create("flac:level=8:exhaustive")->describe() == "flac [level=8, exhaustive]");
  CHECK(flac_block_compressor::create("flac:level=0")->describe() == "flac [level=0]");
  CHECK(throws<std::runtime_error>([] { flac_block_compressor::create("flac:level=9"); }));
  CHECK(throws<std::runtime_error>([] { flac_block_compressor::create("flac:speed=3"); }));
  flac_block_compressor comp;
  CHECK(comp.type() == 6);
  CHECK(comp.metadata_requirements() ==
        R"({"bits_per_sample":["range",8,32],"bytes_per_sample":["range",1,4],"endianness":["set",["big","little"]],)"
        R"("number_of_channels":["range",1,8],"padding":["set",["msb","lsb"]],"signedness":["set",["signed","unsigned"]]})");
  CHECK(comp.compression_granularity(meta16) == 4);
  // error contract (:229-232, :247-253)
  {
    std::vector<uint8_t> odd(7);
    CHECK(throws<std::runtime_error>([&] { comp.compress(odd, nullptr); },
                                     "internal error: flac compression requires metadata"));
    CHECK(throws<std::runtime_error>(
        [&] { comp.compress(odd, &meta16); },
        "unexpected PCM waveform configuration: 7 bytes to compress, 2 channels, 2 bytes per sample"));
  }
  // round trip, 16-bit stereo little endian signed; stream checked by the restatement
  {
    const size_t frames = 3 * 4096 + 1234;
    auto x = flac_signal(frames, 2, 16, 1);
    std::vector<uint8_t> pcm(x.size() * 2);
    for (size_t i = 0; i < x.size(); ++i) {
      pcm[2 * i] = uint8_t(x[i]);
      pcm[2 * i + 1] = uint8_t(uint32_t(x[i]) >> 8);
    }
    auto block = comp.compress(pcm, &meta16);
    CHECK(block.size() < pcm.size() / 2);  // flac_compressor_test.cpp: the output is below half the input
    // framing: varint + flac_block_header + "fLaC" + STREAMINFO
    rpp_flac_frame f{};
    long h = rpp_flac_parse_frame(block.data(), block.size(), &f);
    CHECK(h > 0 && f.uncompressed_bytes == pcm.size() && f.num_channels == 2 && f.bits_per_sample == 16 &&
          f.flags == 0x41);
    std::vector<int32_t> y(x.size());
    uint32_t ch = 0, bps = 0;
    uint64_t ns = 0;
    CHECK(fo_decode(block.data() + h, block.size() - (size_t)h, y.data(), y.size(), &ch, &bps, &ns) == 0);
    CHECK(ch == 2 && bps == 16 && ns == frames && y == x);
    flac_block_decompressor d{block};
    CHECK(d.uncompressed_size() == pcm.size());
    CHECK(*d.metadata() == meta16);
    std::vector<uint8_t> out;
    d.start_decompression(&out);
    CHECK(d.decompress_frame(pcm.size()));
    CHECK(!d.decompress_frame(pcm.size()));
    CHECK(out == pcm);
  }
  // the restatement's LPC streams (orders up to 8, as libFLAC level 5),
  // 24-bit in 3 bytes, big endian, 3 channels -> the C++ decompressor
  {
    const size_t frames = 2 * 4096 + 77;
    auto x = flac_signal(frames, 3, 24, 2);
    fo_opts o{};
    o.stereo = -1;
    o.max_partition_order = 6;
    o.max_lpc_order = 8;
    std::vector<uint8_t> stream(frames * 3 * 4 + 65536);
    size_t len = fo_encode(x.data(), frames, 3, 24, 4096, &o, stream.data(), stream.size());
    CHECK(len > 0);
    stream.resize(len);
    rpp_flac_frame f{frames * 3 * 3, 3, 24, 0x80 | 0x40 | 2};
    std::vector<uint8_t> block(64);
    block.resize(rpp_flac_frame_header(&f, block.data()));
    block.insert(block.end(), stream.begin(), stream.end());
    std::vector<uint8_t> want(frames * 3 * 3);
    for (size_t i = 0; i < x.size(); ++i) {
      const uint32_t v = uint32_t(x[i]);
      want[3 * i] = uint8_t(v >> 16), want[3 * i + 1] = uint8_t(v >> 8), want[3 * i + 2] = uint8_t(v);
    }
    CHECK(flac_block_decompressor::decompress(block) == want);
    // a stream whose metadata does not parse
    std::vector<uint8_t> bad(block.begin(), block.begin() + 12);
    bad.resize(40, 0);
    CHECK(throws<std::runtime_error>([&] { flac_block_decompressor d{bad}; }));
  }
}
