// Host-code sanitizer run (built with -fsanitize=address,undefined by
// tests/cpp/build_sanitize.sh; no GPU): hostile inputs to the parts of the
// library that parse untrusted bytes on the host, and to the CPU oracle.
//
//  * rpp_parse_frame (dwarfs_amd/csrc/ricepp_frame.cpp), the DwarFS block
//    header a reader gets from disk (src/compression/ricepp.cpp:186-201,
//    237-249): random bytes, truncations of valid headers, byte mutations,
//    huge varints, nested/unknown thrift fields; every valid header must
//    round-trip through rpp_frame_header.
//  * the oracle's decoder on random and truncated streams (it must report
//    an error or decode, never read out of bounds), and encode/decode round
//    trips at odd sizes.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ricepp_amd.h"

extern "C" {
struct rpo_config {
  uint32_t block_size, component_stream_count, big_endian, unused_lsb_count;
};
size_t rpo_worst_case_bytes(const rpo_config*, size_t);
int rpo_encode(const rpo_config*, const uint16_t*, size_t, uint8_t*, size_t, size_t*);
int rpo_decode(const rpo_config*, const uint8_t*, size_t, uint16_t*, size_t);
}

static int failures = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      if (failures < 20) std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                             \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  auto rnd = [&](uint64_t n) { return n ? rng() % n : 0; };

  // ---- valid frames round-trip; every prefix and mutation parses safely ----
  long parsed_ok = 0;
  for (int it = 0; it < iters; ++it) {
    rpp_frame f{};
    f.uncompressed_bytes = (it & 7) == 0 ? rng() : rnd(1ull << (rnd(48)));
    f.block_size = (uint32_t)(rnd(2) ? rnd(1024) : rng());
    f.component_count = (uint32_t)rnd(5);
    f.bytes_per_sample = (uint32_t)rnd(5);
    f.unused_lsb_count = (uint32_t)rnd(20);
    f.big_endian = (uint32_t)rnd(2);
    f.ricepp_version = (uint32_t)rnd(4);
    std::vector<uint8_t> buf(64);
    const size_t n = rpp_frame_header(&f, buf.data());
    CHECK(n > 0 && n <= 64);
    buf.resize(n);
    rpp_frame g{};
    const long h = rpp_parse_frame(buf.data(), buf.size(), &g);
    if (h == (long)n && g.uncompressed_bytes == f.uncompressed_bytes && g.big_endian == f.big_endian) ++parsed_ok;
    // truncations (exact-size heap copies, so ASan sees any over-read)
    const size_t cut = rnd(n + 1);
    std::vector<uint8_t> t(buf.begin(), buf.begin() + (long)cut);
    rpp_frame q{};
    (void)rpp_parse_frame(t.empty() ? nullptr : t.data(), t.size(), &q);
    // mutations
    std::vector<uint8_t> m = buf;
    for (int k = 0, nm = 1 + (int)rnd(4); k < nm; ++k) m[rnd(m.size())] ^= (uint8_t)(1u << rnd(8));
    if (rnd(3) == 0) m.push_back((uint8_t)rng());
    (void)rpp_parse_frame(m.data(), m.size(), &q);
  }
  CHECK(parsed_ok == iters);

  // ---- random byte strings (biased to thrift-looking bytes) ----
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> b(rnd(48));
    for (auto& x : b) x = (uint8_t)(rnd(3) ? rng() : (0x10u * rnd(16) + rnd(13)));  // field headers
    rpp_frame q{};
    const long h = rpp_parse_frame(b.empty() ? nullptr : b.data(), b.size(), &q);
    CHECK(h <= (long)b.size());
  }
  // ---- long varints and deep skips ----
  {
    std::vector<uint8_t> v(40, 0xFF);
    rpp_frame q{};
    CHECK(rpp_parse_frame(v.data(), v.size(), &q) < 0);
  }

  // ---- the oracle on hostile streams ----
  for (int it = 0; it < iters / 50; ++it) {
    rpo_config c{(uint32_t)(1 + rnd(512)), (uint32_t)(1 + rnd(2)), (uint32_t)rnd(2), (uint32_t)rnd(16)};
    const size_t n = rnd(3000) / c.component_stream_count * c.component_stream_count;
    std::vector<uint8_t> s(rnd(2000));
    for (auto& x : s) x = (uint8_t)(rnd(4) ? rng() : 0);
    std::vector<uint16_t> out(n);
    (void)rpo_decode(&c, s.empty() ? nullptr : s.data(), s.size(), out.empty() ? nullptr : out.data(), n);
    // round trip at odd sizes, then every truncation of the stream
    // (samples with unused_lsb_count zero low bits, stored in the configured
    // byte order: the round trip is lossless only for those)
    std::vector<uint16_t> x(n);
    for (auto& v : x) {
      uint16_t s = (uint16_t)((rnd(4) ? 20000 + rnd(1000) : rng()) & (0xFFFFu << c.unused_lsb_count));
      v = c.big_endian ? (uint16_t)((s >> 8) | (s << 8)) : s;
    }
    std::vector<uint8_t> e(rpo_worst_case_bytes(&c, n) + 1);
    size_t used = 0;
    CHECK(rpo_encode(&c, x.data(), n, e.data(), e.size(), &used) == 0);
    std::vector<uint8_t> ex(e.begin(), e.begin() + (long)used);
    std::vector<uint16_t> y(n);
    CHECK(rpo_decode(&c, ex.empty() ? nullptr : ex.data(), ex.size(), y.empty() ? nullptr : y.data(), n) == 0);
    CHECK(y == x);
    std::vector<uint8_t> tr(ex.begin(), ex.begin() + (long)rnd(used + 1));
    (void)rpo_decode(&c, tr.empty() ? nullptr : tr.data(), tr.size(), y.empty() ? nullptr : y.data(), n);
  }
  std::printf("fuzz_host: %s (%d failures, %d iterations)\n", failures ? "FAILED" : "OK", failures, iters);
  return failures ? 1 : 0;
}
