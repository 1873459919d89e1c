// Standalone reproducer of the round-5 "bs 128 cs 2 encode" fault (DESIGN.md
// §4 "Uniform branches"; no library code): a gfx950 64-bit shift
// (v_lshlrev_b64) that reads a register pair whose halves were written by
// 32-bit VALU instructions just before it.  Each lane builds a random 64-bit
// value in a pair, shifts it by a random amount in 0..31, and compares the
// result with the same shift done by 32-bit instructions (v_lshlrev_b32,
// v_alignbit_b32).  Variants (the instructions between the last write of an
// operand and the shift):
//   0  halves and amount by v_mov_b32 (hi, amount last), shift at once -- the encoder's sequence
//   1  the same with s_nop 0 before the shift       2  s_nop 1      3  s_nop 2     4  s_nop 4
//   5  the pair written by one v_mov_b64, amount earlier (no 32-bit write just before)
//   6  halves by v_mov_b32, then 4 independent VALU ops, then the shift
//   7  as 0, but the result goes to another pair (not in place)
//   8  as 0 with v_lshrrev_b64 (right shift) instead
//   9  as 0 in the encoder's registers v[132:133] / v135, kernel declaring 136 VGPRs
//  10  the same registers, kernel declaring 144 VGPRs (v143 clobbered)
//  11-14  declaring 136 VGPRs, pair / amount at v[134:135]/v131, v[130:131]/v129, v[128:129]/v127,
//         v[126:127]/v125 (distance from the top of the allocation)
//  15  source pair at the top (v[132:133]), result to v[40:41]
//  16  source pair v[40:41], result to the top pair v[132:133]
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/shl64_hazard tools/shl64_hazard.hip
// Run:   tools/shl64_hazard <waves> <iters>     (one JSON line per variant)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ unsigned long long g_bad[32];

#define PAIR_OPS(PRE, MID, SHIFT, OUT0, OUT1)                                                          \
  asm volatile(PRE MID SHIFT "\n\tv_mov_b32 %[r0], " OUT0 "\n\tv_mov_b32 %[r1], " OUT1                 \
               : [r0] "=&v"(r0), [r1] "=&v"(r1), [f] "+v"(f)                                            \
               : [lo] "v"(lo), [hi] "v"(hi), [sh] "v"(sh)                                               \
               : "v40", "v41", "v42", "v43", "v44")
#define PAIR_AT(P0, P1, PAIR, S, DST, D0, D1, ...)                                                        \
  asm volatile("v_mov_b32 " P0 ", %[lo]\n\tv_mov_b32 " P1 ", %[hi]\n\tv_mov_b32 " S ", %[sh]\n\t"              \
               "v_lshlrev_b64 " DST ", " S ", " PAIR "\n\tv_mov_b32 %[r0], " D0 "\n\tv_mov_b32 %[r1], " D1      \
               : [r0] "=&v"(r0), [r1] "=&v"(r1), [f] "+v"(f)                                            \
               : [lo] "v"(lo), [hi] "v"(hi), [sh] "v"(sh)                                               \
               : "v40", "v41", "v125", "v126", "v127", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135" __VA_ARGS__)
#define PAIR_OPS_HI(...)                                                                               \
  asm volatile("v_mov_b32 v132, %[lo]\n\tv_mov_b32 v133, %[hi]\n\tv_mov_b32 v135, %[sh]\n\t"            \
               "v_lshlrev_b64 v[132:133], v135, v[132:133]\n\tv_mov_b32 %[r0], v132\n\tv_mov_b32 %[r1], v133" \
               : [r0] "=&v"(r0), [r1] "=&v"(r1), [f] "+v"(f)                                            \
               : [lo] "v"(lo), [hi] "v"(hi), [sh] "v"(sh)                                               \
               : "v132", "v133", "v134", "v135" __VA_ARGS__)

template <int V>
__global__ __launch_bounds__(64) void probe(uint32_t iters) {
  unsigned long long bad = 0;
  uint32_t s = (blockIdx.x * 2654435761u) ^ (threadIdx.x * 40503u + 1u), f = s;
  for (uint32_t it = 0; it < iters; ++it) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    const uint32_t lo = s * 2246822519u, hi = s ^ 0x5bd1e995u, sh = (s >> 27) & 31u;
    uint32_t r0, r1;
#define SETUP "v_mov_b32 v40, %[lo]\n\tv_mov_b32 v41, %[hi]\n\tv_mov_b32 v44, %[sh]\n\t"
    if constexpr (V == 0) PAIR_OPS(SETUP, "", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 1) PAIR_OPS(SETUP, "s_nop 0\n\t", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 2) PAIR_OPS(SETUP, "s_nop 1\n\t", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 3) PAIR_OPS(SETUP, "s_nop 2\n\t", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 4) PAIR_OPS(SETUP, "s_nop 4\n\t", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 5)
      PAIR_OPS("v_mov_b32 v44, %[sh]\n\tv_mov_b32 v42, %[lo]\n\tv_mov_b32 v43, %[hi]\n\t"
               "v_add_u32 %[f], 1, %[f]\n\tv_add_u32 %[f], 1, %[f]\n\tv_add_u32 %[f], 1, %[f]\n\t"
               "v_mov_b64 v[40:41], v[42:43]\n\t", "", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 6)
      PAIR_OPS(SETUP, "v_add_u32 %[f], 1, %[f]\n\tv_add_u32 %[f], 1, %[f]\n\tv_add_u32 %[f], 1, %[f]\n\t"
               "v_add_u32 %[f], 1, %[f]\n\t", "v_lshlrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 7) PAIR_OPS(SETUP, "", "v_lshlrev_b64 v[42:43], v44, v[40:41]", "v42", "v43");
    if constexpr (V == 8) PAIR_OPS(SETUP, "", "v_lshrrev_b64 v[40:41], v44, v[40:41]", "v40", "v41");
    if constexpr (V == 9) PAIR_OPS_HI();
    if constexpr (V == 10) PAIR_OPS_HI(, "v143");  // (declares 144 VGPRs)
    if constexpr (V == 11) PAIR_AT("v134", "v135", "v[134:135]", "v131", "v[134:135]", "v134", "v135");
    if constexpr (V == 12) PAIR_AT("v130", "v131", "v[130:131]", "v129", "v[130:131]", "v130", "v131");
    if constexpr (V == 13) PAIR_AT("v128", "v129", "v[128:129]", "v127", "v[128:129]", "v128", "v129");
    if constexpr (V == 14) PAIR_AT("v126", "v127", "v[126:127]", "v125", "v[126:127]", "v126", "v127");
    if constexpr (V == 15) PAIR_AT("v132", "v133", "v[132:133]", "v135", "v[40:41]", "v40", "v41");
    if constexpr (V == 16) PAIR_AT("v40", "v41", "v[40:41]", "v135", "v[132:133]", "v132", "v133");
#undef SETUP
    uint32_t e0, e1;
    if constexpr (V == 8) {
      e0 = sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
      e1 = hi >> sh;
    } else {
      e0 = lo << sh;
      e1 = sh ? __builtin_amdgcn_alignbit(hi, lo, 32u - sh) : hi;
    }
    bad += (r0 != e0 || r1 != e1) ? 1u : 0u;
  }
  atomicAdd(&g_bad[V], bad);
  atomicAdd(&g_bad[31], (unsigned long long)(f & 1u));
}

template <int V>
static void run(uint32_t waves, uint32_t iters) {
  unsigned long long z[32] = {0}, c[32];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z);
  hipLaunchKernelGGL(probe<V>, dim3(waves), dim3(64), 0, 0, iters);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); exit(2); }
  (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_bad), sizeof c);
  printf("{\"probe\": \"shl64_hazard\", \"variant\": %d, \"waves\": %u, \"iters\": %u, \"lane_shifts\": %llu, "
         "\"wrong\": %llu}\n", V, waves, iters, (unsigned long long)waves * 64ull * iters, c[V]);
}

int main(int argc, char** argv) {
  const uint32_t waves = argc > 1 ? atoi(argv[1]) : 4096;
  const uint32_t iters = argc > 2 ? atoi(argv[2]) : 2000;
  run<0>(waves, iters); run<1>(waves, iters); run<2>(waves, iters); run<3>(waves, iters); run<4>(waves, iters);
  run<5>(waves, iters); run<6>(waves, iters); run<7>(waves, iters); run<8>(waves, iters);
  run<9>(waves, iters); run<10>(waves, iters); run<11>(waves, iters); run<12>(waves, iters);
  run<13>(waves, iters); run<14>(waves, iters); run<15>(waves, iters); run<16>(waves, iters);
  return 0;
}
