// Standalone probe (DESIGN.md §4 "Uniform branches"): does an in-place 64-bit
// shift on gfx950 -- v_lshlrev_b64 v[a:a+1], s, v[a:a+1], the source pair
// being the destination pair -- always give the shifted value?  Each round a
// lane shifts a random 64-bit value in place and, beside it, a copy of it
// from a separate register pair, and counts the rounds where the two differ.
// Template bit 1 puts LDS traffic (two ds_or_b32 of the result, as the encode
// emission does) after each shift, bit 2 makes the shift amount register
// the destination's low half (v_lshlrev_b64 v[a:a+1], va, v[x:y]).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/shift64_repro tools/shift64_repro.hip
// Run:   tools/shift64_repro <waves> <iters> <lds_bytes> <variant 0..3>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ unsigned long long g_cnt[4];

template <int V>
__global__ __launch_bounds__(64) void probe(uint32_t iters, uint32_t seed) {
  extern __shared__ uint32_t win[];
  const uint32_t lane = __lane_id();
  uint32_t s = seed ^ (blockIdx.x * 2654435761u) ^ (lane * 40503u + 1u);
  for (uint32_t i = lane; i < 1024; i += 64) win[i] = 0;
  unsigned long long bad = 0, n = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    const uint32_t lo = s * 2246822519u, hi = (s >> 7) & 0xFFFFu, sh = s & 31u;
    uint32_t a0, a1, b0, b1;
    if constexpr (V & 2) {
      // the encode emission's pair of steps, fixed registers: a shift whose amount register is the destination's
      // low half, then the next code's value written into that pair and shifted in place
      uint32_t r0, r1;
      asm volatile(
          "v_and_b32 v200, 31, %[sh]\n\t"
          "v_mov_b32 v202, %[lo]\n\t"
          "v_mov_b32 v203, 0\n\t"
          "v_lshlrev_b64 v[200:201], v200, v[202:203]\n\t"
          "v_mov_b32 %[r0], v200\n\t"
          "v_mov_b32 %[r1], v201\n\t"
          "v_and_b32 v200, 0xffff, %[hi]\n\t"
          "v_mov_b32 v201, 0\n\t"
          "v_and_b32 v204, 31, %[sh]\n\t"
          "v_lshlrev_b64 v[200:201], v204, v[200:201]\n\t"
          "v_mov_b32 %[a0], v200\n\t"
          "v_mov_b32 %[a1], v201"
          : [r0] "=&v"(r0), [r1] "=&v"(r1), [a0] "=&v"(a0), [a1] "=&v"(a1)
          : [sh] "v"(sh), [lo] "v"(lo), [hi] "v"(hi)
          : "v200", "v201", "v202", "v203", "v204");
      const uint32_t e0 = lo << sh, e1 = sh ? lo >> (32u - sh) : 0u;
      bad += (r0 != e0 || r1 != e1) ? 1u : 0u;
    } else {
      // in place: the value pair is the destination pair
      uint64_t v = ((uint64_t)hi << 32) | lo;
      asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(v) : "v"(sh));
      a0 = (uint32_t)v; a1 = (uint32_t)(v >> 32);
    }
    if constexpr (V & 1) {
      atomicOr(&win[(s >> 5) & 1023u], a0);
      atomicOr(&win[((s >> 5) + 1) & 1023u], a1);
    }
    // the expected value by 32-bit operations only (no 64-bit shift)
    const uint32_t vlo = (V & 2) ? (hi & 0xFFFFu) : lo, vhi = (V & 2) ? 0u : hi;
    b0 = vlo << sh;
    b1 = sh ? __builtin_amdgcn_alignbit(vhi, vlo, 32u - sh) : vhi;
    bad += (a0 != b0 || a1 != b1) ? 1u : 0u;
    ++n;
  }
  atomicAdd(&g_cnt[0], n);
  atomicAdd(&g_cnt[1], bad);
  atomicAdd(&g_cnt[2], (unsigned long long)(win[lane] & 1u));
}

int main(int argc, char** argv) {
  const uint32_t waves = argc > 1 ? atoi(argv[1]) : 16384;
  const uint32_t iters = argc > 2 ? atoi(argv[2]) : 20000;
  const uint32_t lds = argc > 3 ? atoi(argv[3]) : 4096;
  const uint32_t var = argc > 4 ? atoi(argv[4]) & 3 : 0;
  unsigned long long z[4] = {0}, c[4];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z, sizeof z) != hipSuccess) return 1;
  void (*k[4])(uint32_t, uint32_t) = {probe<0>, probe<1>, probe<2>, probe<3>};
  hipLaunchKernelGGL(k[var], dim3(waves), dim3(64), lds, 0, iters, 777u);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 2; }
  if (hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cnt), sizeof c) != hipSuccess) return 1;
  printf("{\"probe\": \"inplace_shl64\", \"variant\": %u, \"waves\": %u, \"iters\": %u, \"lds\": %u, \"lane_ops\": %llu, "
         "\"wrong\": %llu}\n", var, waves, iters, lds, c[0], c[1]);
  return 0;
}
