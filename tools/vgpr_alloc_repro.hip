// Standalone reproducer for the round-5 bs 128 cs 2 encode fault (DESIGN.md
// §4 "Uniform branches"; no library code).  The failing encode build declared
// exactly 136 VGPRs, and the very same machine code with the descriptor's
// count raised to 137 or 144 encoded everything right (tools/asm_variant.py
// vg137 / vg144).  Here each wave keeps a per-wave signature in its top eight
// registers v[NV-8 .. NV-1] (the kernel's declared count is NV: nothing above
// is touched), burns VALU time on low registers, and checks the signature is
// still there; many waves share each SIMD.  Counts the rounds in which one of
// the eight registers no longer holds its value.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/vgpr_alloc_repro tools/vgpr_alloc_repro.hip
// Run:   tools/vgpr_alloc_repro <waves> <iters>   (every NV in the table below)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ unsigned long long g_bad[8];

#define STR2(x) #x
#define STR(x) STR2(x)
// writes sig + k into v[NV-8+k], spins on v0-v3, reads the eight back; result: mismatches
#define PROBE_ASM(R0, R1, R2, R3, R4, R5, R6, R7)                                                      \
  asm volatile(                                                                                      \
      "v_add_u32 " R0 ", 0, %[s]\n\tv_add_u32 " R1 ", 1, %[s]\n\tv_add_u32 " R2 ", 2, %[s]\n\t"         \
      "v_add_u32 " R3 ", 3, %[s]\n\tv_add_u32 " R4 ", 4, %[s]\n\tv_add_u32 " R5 ", 5, %[s]\n\t"         \
      "v_add_u32 " R6 ", 6, %[s]\n\tv_add_u32 " R7 ", 7, %[s]\n\t"                                     \
      ".rept 64\n\tv_mul_lo_u32 %[w], %[w], %[w]\n\tv_add_u32 %[w], 1, %[w]\n\t.endr\n\t"              \
      "v_mov_b32 %[b], 0\n\t"                                                                        \
      "v_sub_u32 %[t], " R0 ", %[s]\n\tv_cmp_ne_u32 vcc, 0, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R1 ", %[s]\n\tv_cmp_ne_u32 vcc, 1, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R2 ", %[s]\n\tv_cmp_ne_u32 vcc, 2, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R3 ", %[s]\n\tv_cmp_ne_u32 vcc, 3, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R4 ", %[s]\n\tv_cmp_ne_u32 vcc, 4, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R5 ", %[s]\n\tv_cmp_ne_u32 vcc, 5, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R6 ", %[s]\n\tv_cmp_ne_u32 vcc, 6, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc\n\t" \
      "v_sub_u32 %[t], " R7 ", %[s]\n\tv_cmp_ne_u32 vcc, 7, %[t]\n\tv_addc_co_u32 %[b], vcc, 0, %[b], vcc"   \
      : [b] "=&v"(bad), [t] "=&v"(tmp), [w] "+v"(w)                                                  \
      : [s] "v"(sig)                                                                                 \
      : "vcc", R0, R1, R2, R3, R4, R5, R6, R7)

template <int NV>
__global__ __launch_bounds__(64) void probe(uint32_t iters) {
  uint32_t w = threadIdx.x + 1, tmp, bad;
  unsigned long long total = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t sig = (blockIdx.x << 16) ^ (threadIdx.x << 8) ^ (it * 2654435761u);
    if constexpr (NV == 104) PROBE_ASM("v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103");
    if constexpr (NV == 112) PROBE_ASM("v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111");
    if constexpr (NV == 120) PROBE_ASM("v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119");
    if constexpr (NV == 128) PROBE_ASM("v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127");
    if constexpr (NV == 136) PROBE_ASM("v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135");
    if constexpr (NV == 144) PROBE_ASM("v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143");
    total += bad;
  }
  atomicAdd(&g_bad[0], total);
  atomicAdd(&g_bad[1], (unsigned long long)(w & 1u));  // keep the spin live
}

// The same with the encode emission's operation: a 64-bit shift of a pair in
// the top registers (v_lshlrev_b64 v[a:a+1], vS, v[a:a+1] in place, and with
// the shift amount in the pair's low register), checked against 32-bit math.
#define SHIFT_ASM(P0, P1, PAIR, S)                                                                     \
  asm volatile("v_mov_b32 " P0 ", %[lo]\n\tv_mov_b32 " P1 ", %[hi]\n\tv_mov_b32 " S ", %[sh]\n\t"        \
               "v_lshlrev_b64 " PAIR ", " S ", " PAIR "\n\t"                                          \
               "v_mov_b32 %[r0], " P0 "\n\tv_mov_b32 %[r1], " P1 "\n\t"                                 \
               "v_mov_b32 " P0 ", %[sh]\n\tv_mov_b32 " S ", %[lo]\n\tv_mov_b32 " P1 ", 0\n\t"            \
               "v_lshlrev_b64 " PAIR ", " P0 ", v[%[vx]:%[vy]]\n\t"                                     \
               "v_mov_b32 %[r2], " P0 "\n\tv_mov_b32 %[r3], " P1                                          \
               : [r0] "=&v"(r0), [r1] "=&v"(r1), [r2] "=&v"(r2), [r3] "=&v"(r3)                         \
               : [lo] "v"(lo), [hi] "v"(hi), [sh] "v"(sh), [vx] "i"(0), [vy] "i"(1)                     \
               : P0, P1, S)

template <int NV>
__global__ __launch_bounds__(64) void probe64(uint32_t iters) {
  unsigned long long total = 0;
  uint32_t s = (blockIdx.x * 2654435761u) ^ (threadIdx.x * 40503u + 1u);
  for (uint32_t it = 0; it < iters; ++it) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    const uint32_t lo = s * 2246822519u, hi = s >> 3, sh = s & 31u;
    uint32_t r0, r1, r2, r3;
    if constexpr (NV == 136) SHIFT_ASM("v132", "v133", "v[132:133]", "v135");
    if constexpr (NV == 144) SHIFT_ASM("v140", "v141", "v[140:141]", "v143");
    if constexpr (NV == 128) SHIFT_ASM("v124", "v125", "v[124:125]", "v127");
    if constexpr (NV == 120) SHIFT_ASM("v116", "v117", "v[116:117]", "v119");
    const uint32_t e0 = lo << sh, e1 = sh ? __builtin_amdgcn_alignbit(hi, lo, 32u - sh) : hi;
    total += (r0 != e0 || r1 != e1) ? 1u : 0u;
    (void)r2; (void)r3;
  }
  atomicAdd(&g_bad[2], total);
}

template <int NV>
static void run64(uint32_t waves, uint32_t iters) {
  unsigned long long z[8] = {0}, c[8];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z);
  hipLaunchKernelGGL(probe64<NV>, dim3(waves), dim3(64), 0, 0, iters);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); exit(2); }
  (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_bad), sizeof c);
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(probe64<NV>));
  printf("{\"probe\": \"top_pair_shl64\", \"declared_vgprs\": %d, \"num_regs\": %d, \"waves\": %u, \"iters\": %u, "
         "\"lane_shifts\": %llu, \"wrong\": %llu}\n",
         NV, fa.numRegs, waves, iters, (unsigned long long)waves * 64ull * iters, c[2]);
}

template <int NV>
static void run(uint32_t waves, uint32_t iters) {
  unsigned long long z[8] = {0}, c[8];
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bad), z, sizeof z);
  hipLaunchKernelGGL(probe<NV>, dim3(waves), dim3(64), 0, 0, iters);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); exit(2); }
  (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(g_bad), sizeof c);
  hipFuncAttributes fa;
  (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(probe<NV>));
  printf("{\"probe\": \"top_vgprs\", \"declared_vgprs\": %d, \"num_regs\": %d, \"waves\": %u, \"iters\": %u, "
         "\"lane_register_checks\": %llu, \"corrupted\": %llu}\n",
         NV, fa.numRegs, waves, iters, (unsigned long long)waves * 64ull * iters * 8ull, c[0]);
}

int main(int argc, char** argv) {
  const uint32_t waves = argc > 1 ? atoi(argv[1]) : 16384;
  const uint32_t iters = argc > 2 ? atoi(argv[2]) : 2000;
  run<104>(waves, iters);
  run<112>(waves, iters);
  run<120>(waves, iters);
  run<128>(waves, iters);
  run<136>(waves, iters);
  run<144>(waves, iters);
  run64<120>(waves, 10 * iters);
  run64<128>(waves, 10 * iters);
  run64<136>(waves, 10 * iters);
  run64<144>(waves, 10 * iters);
  return 0;
}
