// Instruction-throughput microbenchmark (diagnostic only): cycles per
// wave-instruction for the ops the decode chains use, 8 independent chains.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 2000
template <int OP>
__global__ void kern(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
  uint32_t a[8];
  uint64_t w = ((uint64_t)seed << 32) | (threadIdx.x * 2654435761u);
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i * 7 + seed;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (OP == 0) a[i] = a[i] + 0x9e3779b9u;                                  // v_add
      if constexpr (OP == 1) a[i] = (uint32_t)(w >> (a[i] & 63)) + a[i];                  // v_lshrrev_b64 + add
      if constexpr (OP == 2) a[i] = (uint32_t)__builtin_ctz(a[i] | 0x80000000u) + a[i] * 3u;  // ffbl
      if constexpr (OP == 3) a[i] = ((uint64_t)a[i] * 3u != w) ? a[i] + 1 : a[i] + 2;      // 64-bit cmp
      if constexpr (OP == 4) a[i] = (a[i] >> (a[i] & 31)) + a[i];                          // v_lshrrev_b32 + add
      if constexpr (OP == 5) a[i] = a[i] < 32u ? a[i] + 5 : max(a[i], 7u);                 // cmp+cndmask+max
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int blocks_per_cu) {
  int nb = 256 * blocks_per_cu;
  uint32_t* out; unsigned long long* cyc;
  hipMalloc(&out, nb * 64 * 4); hipMalloc(&cyc, nb * 8);
  hipLaunchKernelGGL(kern<OP>, dim3(nb), dim3(64), 0, 0, out, cyc, 1u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<OP>, dim3(nb), dim3(64), 0, 0, out, cyc, 2u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = (unsigned long long*)malloc(nb * 8);
  hipMemcpy(h, cyc, nb * 8, hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < nb; ++i) avg += h[i]; avg /= nb;
  double ops = (double)ITERS * 8;
  printf("%-34s waves/SIMD=%d  memtime/op-step=%.2f  wall ns per wave-op-step=%.3f\n", name, blocks_per_cu / 4,
         avg / ops, ms * 1e6 / (ops * nb / 1024.0));
  hipFree(out); hipFree(cyc); free(h);
}

int main() {
  for (int bpc : {4, 8, 16}) {
    run<0>("add", bpc);
    run<1>("lshr_b64+add", bpc);
    run<2>("or+ffbl+mul+add", bpc);
    run<3>("mul64+cmp_u64+cndmask+add", bpc);
    run<4>("lshr_b32+and+add", bpc);
    run<5>("cmp+cndmask+max+add", bpc);
  }
  return 0;
}
