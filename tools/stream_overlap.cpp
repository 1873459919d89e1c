// Diagnostic: do decode launches on different streams of one process run
// concurrently on the device?  One launch of B blocks vs S streams with B / S
// blocks each (wall time from the first launch to hipDeviceSynchronize), for
// the 64 KiB blocks of the facade benchmark.  Build:
//   hipcc -O2 -std=c++20 -Iinclude tools/stream_overlap.cpp -Ldwarfs_amd/lib -lricepp_amd \
//     -Wl,-rpath,'$ORIGIN/../dwarfs_amd/lib' -o tools/stream_overlap
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ricepp_amd.h"

#define CK(x)                                                              \
  do {                                                                     \
    if ((x) != hipSuccess) {                                               \
      std::fprintf(stderr, "HIP error %s at %d\n", #x, __LINE__);          \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main() {
  const uint32_t B = 64, n = 32768;
  rpp_config cfg{128, 1, 1, 0};
  std::vector<uint16_t> h(B * (size_t)n);
  uint64_t x = 42;
  for (auto& v : h) {  // noise around 1000 (about 8 bits per sample)
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    v = (uint16_t)(1000 + ((x >> 33) % 200));
  }
  const uint64_t wc = (rpp_worst_case_bytes(&cfg, n) + 15) & ~15ull;
  std::vector<uint64_t> in_off(B), n_s(B, n), out_off(B);
  for (uint32_t i = 0; i < B; ++i) in_off[i] = (uint64_t)i * n, out_off[i] = i * wc;
  uint16_t *d_in, *d_dec;
  uint8_t* d_enc;
  uint64_t *d_in_off, *d_n, *d_out_off, *d_bytes, *d_dec_off;
  int32_t* d_st;
  CK(hipMalloc(&d_in, h.size() * 2));
  CK(hipMalloc(&d_dec, h.size() * 2));
  CK(hipMalloc(&d_enc, B * wc));
  CK(hipMalloc(&d_in_off, B * 8));
  CK(hipMalloc(&d_n, B * 8));
  CK(hipMalloc(&d_out_off, B * 8));
  CK(hipMalloc(&d_bytes, B * 8));
  CK(hipMalloc(&d_dec_off, B * 8));
  CK(hipMalloc(&d_st, B * 4));
  CK(hipMemcpy(d_in, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_in_off, in_off.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_n, n_s.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_out_off, out_off.data(), B * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_dec_off, in_off.data(), B * 8, hipMemcpyHostToDevice));
  if (rpp_encode_batch(&cfg, d_in, d_in_off, d_n, B, d_enc, d_out_off, d_bytes, d_st, nullptr)) return 1;
  CK(hipDeviceSynchronize());
  std::vector<hipStream_t> st(16);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto run = [&](uint32_t S, uint32_t per, bool enc) {
    double best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipDeviceSynchronize());
      auto t0 = std::chrono::steady_clock::now();
      for (uint32_t k = 0; k < S; ++k) {
        const uint32_t b0 = k * per;
        int r = enc ? rpp_encode_batch(&cfg, d_in, d_in_off + b0, d_n + b0, per, d_enc, d_out_off + b0, d_bytes + b0,
                                       d_st + b0, st[k])
                    : rpp_decode_batch(&cfg, d_enc, d_out_off + b0, d_bytes + b0, per, d_dec, d_dec_off + b0, d_n + b0,
                                       d_st + b0, st[k]);
        if (r) std::exit(2);
      }
      CK(hipDeviceSynchronize());
      best = std::min(best, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::printf("{\"op\": \"%s\", \"streams\": %u, \"blocks_per_stream\": %u, \"wall_us\": %.1f}\n", enc ? "encode" : "decode",
                S, per, best);
  };
  for (bool enc : {false, true}) {
    run(1, 1, enc);
    run(1, 8, enc);
    run(1, 64, enc);
    run(2, 8, enc);
    run(4, 8, enc);
    run(8, 8, enc);
    run(2, 32, enc);
    run(4, 16, enc);
    run(8, 1, enc);
  }
  return 0;
}
