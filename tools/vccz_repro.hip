// Standalone probe of the encode emission's uniform branch (DESIGN.md §4
// "Uniform branches"); no library code.  Each wave runs `iters` rounds of
//   v_cmp_lt_u32 vcc, 32, x   (x per lane; some lanes inactive)
//   <36 VALU ops on other registers: the round-5 gap>
//   s_cbranch_vccz
// -- the shape the round-5 encode compiled `if (!__any(2k + q > 32))` to --
// and checks each branch against the condition re-evaluated through the
// scalar unit.  Template bits add what surrounded the real branch:
//   1 global loads in flight, 2 LDS ds_or in flight, 4 s_setprio 0 over the
//   region (1 elsewhere), 8 DPP ops just before the compare, 16 a wave-wide
//   DPP scan + LDS atomics + a global store per round (the encoder's other work).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/vccz_repro tools/vccz_repro.hip
// Run:   tools/vccz_repro <waves> <iters> <lds_bytes_per_wave> <exec_mode> <variant>
//   exec_mode 0 all lanes, 1 random half, 2 high half off, 3 low half off,
//   4 random quarter off per round (a divergent if, as the encoder's mode == 1)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__device__ unsigned long long g_cnt[4];

template <int V>
__global__ __launch_bounds__(64) void probe(uint32_t iters, uint32_t mode, uint32_t seed, uint4* buf) {
  extern __shared__ uint32_t win[];
  const uint32_t lane = __lane_id();
  uint32_t s = seed ^ (blockIdx.x * 2654435761u) ^ (lane * 40503u + 1u);
  win[lane] = 0;
  uint32_t f0 = s, f1 = s * 3u, f2 = s * 5u, f3 = s * 7u, acc = 0;
  uint4 ld[4];
  unsigned long long n = 0, wt = 0, wn = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    const uint32_t r = s;
    const uint32_t x = (r & 63u) == 0 ? 33u + (r >> 28) : 20u + ((r >> 8) & 7u);  // > 32 in 1 lane of 64
    bool active = true;
    if (mode == 1) active = (r >> 16) & 1u;
    else if (mode == 2) active = lane < 32;
    else if (mode == 3) active = lane >= 32;
    else if (mode == 4) active = ((r >> 20) & 3u) != 0;
    if constexpr (V & 16) {  // the encoder's other work: scan, LDS atomics, a store
      uint32_t v = r & 255u;
      v += __builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
      atomicOr(&win[(v >> 3) & 63u], v);
      buf[(blockIdx.x * 64 + lane) & 0xFFFFu] = make_uint4(v, r, acc, it);
    }
    if constexpr (V & 1)
      for (int k = 0; k < 4; ++k) ld[k] = buf[(blockIdx.x * 251 + lane * 4 + k + it * 64) & 0xFFFFu];
    if (active) {
      if constexpr (V & 2) { atomicOr(&win[r & 63u], r); atomicOr(&win[(r >> 6) & 63u], r >> 1); }
      if constexpr (V & 4) __builtin_amdgcn_s_setprio(0);
      if constexpr (V & 8) {
        f0 += __builtin_amdgcn_update_dpp(0, (int)f1, 0xB1, 0xF, 0xF, true);
        f2 = __builtin_amdgcn_update_dpp((int)f2, (int)f0, 0x141, 0xF, 0xF, false);
      }
      uint32_t taken;
      asm volatile(
          "v_cmp_lt_u32_e32 vcc, 32, %[x]\n\t"
          ".rept 8\n\t"
          "v_pk_lshlrev_b16 %[f0], 1, %[f0] op_sel_hi:[0,1]\n\t"
          "v_and_or_b32 %[f1], %[f2], %[f1], %[sg]\n\t"
          "v_add_u32_sdwa %[f2], %[f3], %[f2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
          "v_lshrrev_b32 %[f3], 16, %[f3]\n\t"
          ".endr\n\t"
          "v_and_b32 %[f0], 0xffff, %[f0]\n\t"
          "v_and_b32 %[f1], %[f2], %[f1]\n\t"
          "v_lshrrev_b32 %[f2], 3, %[f2]\n\t"
          "v_and_b32 %[f3], 0x1ffffffc, %[f3]\n\t"
          "s_cbranch_vccz 1f\n\t"
          "s_mov_b32 %[t], 0\n\t"
          "s_branch 2f\n"
          "1:\n\t"
          "s_mov_b32 %[t], 1\n"
          "2:"
          : [t] "=s"(taken), [f0] "+v"(f0), [f1] "+v"(f1), [f2] "+v"(f2), [f3] "+v"(f3)
          : [x] "v"(x), [sg] "s"(0x10001u)
          : "vcc");
      if constexpr (V & 4) __builtin_amdgcn_s_setprio(1);
      const uint64_t want_slow = __builtin_amdgcn_ballot_w64(x > 32u);
      ++n;
      if (taken && want_slow) ++wt;
      if (!taken && !want_slow) ++wn;
    }
    if constexpr (V & 1) acc += ld[0].x ^ ld[1].y ^ ld[2].z ^ ld[3].w;
  }
  atomicAdd(&g_cnt[0], n);   // (per lane: every branch is counted by each of its active lanes)
  atomicAdd(&g_cnt[1], wt);
  atomicAdd(&g_cnt[2], wn);
  atomicAdd(&g_cnt[3], (unsigned long long)((f0 ^ f1 ^ f2 ^ f3 ^ acc ^ win[lane]) & 1u));  // keep the work live
}

typedef void (*kfn)(uint32_t, uint32_t, uint32_t, uint4*);
static const kfn kernels[32] = {probe<0>,  probe<1>,  probe<2>,  probe<3>,  probe<4>,  probe<5>,  probe<6>,  probe<7>,
                                probe<8>,  probe<9>,  probe<10>, probe<11>, probe<12>, probe<13>, probe<14>, probe<15>,
                                probe<16>, probe<17>, probe<18>, probe<19>, probe<20>, probe<21>, probe<22>, probe<23>,
                                probe<24>, probe<25>, probe<26>, probe<27>, probe<28>, probe<29>, probe<30>, probe<31>};

int main(int argc, char** argv) {
  const uint32_t waves = argc > 1 ? atoi(argv[1]) : 16384;
  const uint32_t iters = argc > 2 ? atoi(argv[2]) : 20000;
  const uint32_t lds = argc > 3 ? atoi(argv[3]) : 256;
  const uint32_t mode = argc > 4 ? atoi(argv[4]) : 4;
  const uint32_t var = argc > 5 ? atoi(argv[5]) & 31 : 0;
  unsigned long long z[4] = {0}, c[4];
  uint4* buf = nullptr;
  if (hipMalloc(&buf, 65536 * sizeof(uint4)) != hipSuccess || hipMemset(buf, 0, 65536 * sizeof(uint4)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(g_cnt), z, sizeof z) != hipSuccess)
    return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(kernels[var], dim3(waves), dim3(64), lds < 256 ? 256 : lds, 0, iters, mode, 12345u, buf);
  (void)hipEventRecord(b, 0);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 2; }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  if (hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cnt), sizeof c) != hipSuccess) return 1;
  printf("{\"variant\": %u, \"waves\": %u, \"iters\": %u, \"lds\": %u, \"exec_mode\": %u, \"ms\": %.2f, "
         "\"lane_branches\": %llu, \"wrong_taken\": %llu, \"wrong_not_taken\": %llu}\n",
         var, waves, iters, lds, mode, ms, c[0], c[1], c[2]);
  return 0;
}
