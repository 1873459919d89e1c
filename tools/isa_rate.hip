// Instruction-rate microbenchmark (diagnostic only, not product code):
// SIMD cycles per wave64 instruction for the instruction kinds the decode
// fast loop issues, at 1 / 2 / 4 / 8 waves per SIMD.  Each wave runs a loop
// of 32 independent instructions (8 register chains) of one kind; the time
// is the average per-wave s_memtime span, so "cyc/instr/SIMD" =
// span / (instructions per wave * waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 512

#define R8(X) X X X X X X X X
#define BODY_VADD "v_add_u32 %0, %0, %12\n v_add_u32 %1, %1, %12\n v_add_u32 %2, %2, %12\n v_add_u32 %3, %3, %12\n v_add_u32 %4, %4, %12\n v_add_u32 %5, %5, %12\n v_add_u32 %6, %6, %12\n v_add_u32 %7, %7, %12\n"
#define BODY_PERM "v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %1, %1, %12, %13\n v_perm_b32 %2, %2, %12, %13\n v_perm_b32 %3, %3, %12, %13\n v_perm_b32 %4, %4, %12, %13\n v_perm_b32 %5, %5, %12, %13\n v_perm_b32 %6, %6, %12, %13\n v_perm_b32 %7, %7, %12, %13\n"
#define BODY_BFE "v_bfe_u32 %0, %0, %12, 5\n v_bfe_u32 %1, %1, %12, 5\n v_bfe_u32 %2, %2, %12, 5\n v_bfe_u32 %3, %3, %12, 5\n v_bfe_u32 %4, %4, %12, 5\n v_bfe_u32 %5, %5, %12, 5\n v_bfe_u32 %6, %6, %12, 5\n v_bfe_u32 %7, %7, %12, 5\n"
#define BODY_LSHLOR "v_lshl_or_b32 %0, %0, 3, %12\n v_lshl_or_b32 %1, %1, 3, %12\n v_lshl_or_b32 %2, %2, 3, %12\n v_lshl_or_b32 %3, %3, 3, %12\n v_lshl_or_b32 %4, %4, 3, %12\n v_lshl_or_b32 %5, %5, 3, %12\n v_lshl_or_b32 %6, %6, 3, %12\n v_lshl_or_b32 %7, %7, 3, %12\n"
// DPP moves read a register written 8 instructions earlier: no hazard
#define BODY_DPPSHR "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %5, %6 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %6, %7 row_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %7, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define BODY_DPPBC "v_mov_b32_dpp %0, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %1, %2 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %2, %3 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %3, %4 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %4, %5 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %5, %6 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %6, %7 row_bcast:15 row_mask:0xa bank_mask:0xf\n v_mov_b32_dpp %7, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
#define BODY_DPPWS "v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %4, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %5, %6 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %6, %7 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %7, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n"
#define BODY_ADDDPP "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %1, %2, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %2, %3, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %3, %4, %3 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %4, %5, %4 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %5, %6, %5 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %6, %7, %6 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_add_u32_dpp %7, %0, %7 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define BODY_BCNT "v_bcnt_u32_b32 %0, %0, %12\n v_bcnt_u32_b32 %1, %1, %12\n v_bcnt_u32_b32 %2, %2, %12\n v_bcnt_u32_b32 %3, %3, %12\n v_bcnt_u32_b32 %4, %4, %12\n v_bcnt_u32_b32 %5, %5, %12\n v_bcnt_u32_b32 %6, %6, %12\n v_bcnt_u32_b32 %7, %7, %12\n"
#define BODY_FFBL "v_ffbl_b32 %0, %1\n v_ffbl_b32 %1, %2\n v_ffbl_b32 %2, %3\n v_ffbl_b32 %3, %4\n v_ffbl_b32 %4, %5\n v_ffbl_b32 %5, %6\n v_ffbl_b32 %6, %7\n v_ffbl_b32 %7, %0\n"
#define BODY_ALIGN "v_alignbit_b32 %0, %1, %0, %12\n v_alignbit_b32 %1, %2, %1, %12\n v_alignbit_b32 %2, %3, %2, %12\n v_alignbit_b32 %3, %4, %3, %12\n v_alignbit_b32 %4, %5, %4, %12\n v_alignbit_b32 %5, %6, %5, %12\n v_alignbit_b32 %6, %7, %6, %12\n v_alignbit_b32 %7, %0, %7, %12\n"
#define BODY_SNOP0 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
#define BODY_SNOP1 "s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n"
#define BODY_VADD_SNOP "v_add_u32 %0, %0, %12\n s_nop 0\n v_add_u32 %1, %1, %12\n s_nop 0\n v_add_u32 %2, %2, %12\n s_nop 0\n v_add_u32 %3, %3, %12\n s_nop 0\n v_add_u32 %4, %4, %12\n s_nop 0\n v_add_u32 %5, %5, %12\n s_nop 0\n v_add_u32 %6, %6, %12\n s_nop 0\n v_add_u32 %7, %7, %12\n s_nop 0\n"
#define BODY_PERM_DEP "v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n v_perm_b32 %0, %0, %12, %13\n"
#define BODY_ADD_DEP "v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n v_add_u32 %0, %0, %12\n"
// the scan step pattern: dpp -> perm -> dpp, dependent (the decode scan)
#define BODY_SCANDEP "s_nop 1\n v_mov_b32_dpp %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n v_perm_b32 %0, %0, %12, %1\n s_nop 1\n v_mov_b32_dpp %1, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n v_perm_b32 %0, %0, %12, %1\n s_nop 1\n v_mov_b32_dpp %1, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n v_perm_b32 %0, %0, %12, %1\n s_nop 1\n v_mov_b32_dpp %1, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n v_perm_b32 %0, %0, %12, %1\n"
#define BODY_ADDSCAN "s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
#define BODY_SALU "s_add_u32 %8, %8, 1\n s_add_u32 %9, %9, 1\n s_add_u32 %10, %10, 1\n s_add_u32 %11, %11, 1\n s_add_u32 %8, %8, 1\n s_add_u32 %9, %9, 1\n s_add_u32 %10, %10, 1\n s_add_u32 %11, %11, 1\n"
#define BODY_MIX "v_add_u32 %0, %0, %12\n s_add_u32 %8, %8, 1\n v_add_u32 %1, %1, %12\n s_add_u32 %9, %9, 1\n v_add_u32 %2, %2, %12\n s_add_u32 %10, %10, 1\n v_add_u32 %3, %3, %12\n s_add_u32 %11, %11, 1\n"
#define BODY_SMUL "s_mul_i32 %8, %8, %9\n s_mul_i32 %10, %10, %11\n s_mul_i32 %9, %9, %8\n s_mul_i32 %11, %11, %10\n s_mul_i32 %8, %8, %9\n s_mul_i32 %10, %10, %11\n s_mul_i32 %9, %9, %8\n s_mul_i32 %11, %11, %10\n"
#define BODY_READLANE "v_readlane_b32 %8, %0, 5\n v_readlane_b32 %9, %1, 6\n v_readlane_b32 %10, %2, 7\n v_readlane_b32 %11, %3, 9\n v_readlane_b32 %8, %4, 5\n v_readlane_b32 %9, %5, 6\n v_readlane_b32 %10, %6, 7\n v_readlane_b32 %11, %7, 9\n"

#define KERN(NAME, BODY)                                                                                    \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* cyc, uint32_t seed) {       \
    uint32_t a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,  \
             a6 = a0 * 17, a7 = a0 * 19;                                                                    \
    uint32_t k = 0x01020304u + seed, sel = 0x07050301u;                                                    \
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;                                        \
    unsigned long long t0, t1;                                                                             \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");                              \
    for (int it = 0; it < ITERS; ++it) {                                                                    \
      asm volatile(BODY BODY BODY BODY                                                                      \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
                     "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)                                                 \
                   : "v"(k), "v"(sel)                                                                        \
                   : "scc", "vcc");                                 \
    }                                                                                                       \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3;     \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                           \
  }

KERN(k_vadd, BODY_VADD)
KERN(k_perm, BODY_PERM)
KERN(k_bfe, BODY_BFE)
KERN(k_lshlor, BODY_LSHLOR)
KERN(k_dppshr, BODY_DPPSHR)
KERN(k_dppbc, BODY_DPPBC)
KERN(k_dppws, BODY_DPPWS)
KERN(k_adddpp, BODY_ADDDPP)
KERN(k_bcnt, BODY_BCNT)
KERN(k_ffbl, BODY_FFBL)
KERN(k_align, BODY_ALIGN)
KERN(k_snop0, BODY_SNOP0)
KERN(k_snop1, BODY_SNOP1)
KERN(k_vadd_snop, BODY_VADD_SNOP)
KERN(k_perm_dep, BODY_PERM_DEP)
KERN(k_add_dep, BODY_ADD_DEP)
KERN(k_scandep, BODY_SCANDEP)
KERN(k_addscan, BODY_ADDSCAN)
KERN(k_salu, BODY_SALU)
KERN(k_mix, BODY_MIX)
KERN(k_readlane, BODY_READLANE)
KERN(k_smul, BODY_SMUL)

// LDS: 16-byte table lookups, random (table of 256 entries) vs conflict-free
template <int MODE>
__global__ __launch_bounds__(256) void k_lds(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  __shared__ uint4 tab[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) tab[i] = make_uint4(i * 7, i * 13, i, i ^ 5);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = (threadIdx.x * 2654435761u) ^ seed, acc = 0;
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x = x * 1664525u + 1013904223u;
      uint32_t idx;
      if (MODE == 0) idx = (x >> 24);                      // random of 256 entries
      else if (MODE == 1) idx = ((x >> 24) << 4) | (lane & 15);  // 16 copies: slot fixed per lane
      else idx = lane;                                     // trivially conflict-free
      const uint4 v = tab[idx + (MODE == 1 ? 0 : 256 * (j & 3))];
      acc += v.x ^ v.w;
    }
  }
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t);

static void run(const char* name, kfn f, int per_wave_instrs) {
  printf("%-12s", name);
  fflush(stdout);
  for (int wps : {1, 2, 4, 8}) {
    const int nb = 256 * wps;  // 4 waves per workgroup -> one per SIMD
    uint32_t* out;
    unsigned long long* cyc;
    hipMalloc(&out, (size_t)nb * 256 * 4);
    hipMalloc(&cyc, (size_t)nb * 4 * 8);
    hipLaunchKernelGGL(f, dim3(nb), dim3(256), 0, 0, out, cyc, 1u);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(f, dim3(nb), dim3(256), 0, 0, out, cyc, 2u);
    hipDeviceSynchronize();
    unsigned long long* h = (unsigned long long*)malloc((size_t)nb * 4 * 8);
    hipMemcpy(h, cyc, (size_t)nb * 4 * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nb * 4; ++i) avg += (double)h[i];
    avg /= nb * 4;
    const double per = avg / ((double)per_wave_instrs * ITERS);
    printf("  w%d: %6.2f/wave %6.2f/SIMD %5.2f/CU", wps, per, per / wps, per / wps / 4);
    hipFree(out);
    hipFree(cyc);
    free(h);
  }
  printf("\n");
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  printf("cycles per instruction (s_memtime ticks), 1/2/4/8 waves per SIMD\n");
  run("v_add", k_vadd, 32);
  run("v_perm", k_perm, 32);
  run("v_bfe", k_bfe, 32);
  run("v_lshl_or", k_lshlor, 32);
  run("dpp_shr", k_dppshr, 32);
  run("dpp_bcast", k_dppbc, 32);
  run("dpp_wshr", k_dppws, 32);
  run("add_dpp", k_adddpp, 32);
  run("v_bcnt", k_bcnt, 32);
  run("v_ffbl", k_ffbl, 32);
  run("v_alignbit", k_align, 32);
  run("s_nop0", k_snop0, 32);
  run("s_nop1", k_snop1, 32);
  run("vadd+snop", k_vadd_snop, 64);
  run("perm_dep", k_perm_dep, 32);
  run("add_dep", k_add_dep, 32);
  run("scan_dep", k_scandep, 48);  // per 12 instrs: 4 (nop, dpp, perm)
  run("addscan", k_addscan, 32);
  run("s_add", k_salu, 32);
  run("vadd+sadd", k_mix, 32);
  run("readlane", k_readlane, 32);
  run("s_mul", k_smul, 32);
  run("lds_rand", k_lds<0>, 8);
  run("lds_16copy", k_lds<1>, 8);
  run("lds_lane", k_lds<2>, 8);
  return 0;
}
