// Diagnostic microbenchmark: cycles per terminator-chain step (the decode's
// serial inner loop) for several loop shapes, at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t ffbl(uint32_t x) { return x ? (uint32_t)__builtin_ctz(x) : ~0u; }
#ifndef WIN64
__device__ __forceinline__ uint32_t win(uint32_t lo, uint32_t hi, uint32_t c) {
  const bool l = c < 32;
  return __builtin_amdgcn_alignbit(l ? hi : 0u, l ? lo : hi, c);
}
#else
__device__ __forceinline__ uint32_t win(uint32_t lo, uint32_t hi, uint32_t c) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (c & 63u));
}
#endif

// VARIANT 0: __any exit every step (seg_chain shape)
// VARIANT 1: fixed 8 steps, no exit test
// VARIANT 2: __any exit every 2 steps
// VARIANT 3: fixed 8 steps, 2 independent chains interleaved
template <int V>
__global__ void kern(uint32_t* out, unsigned long long* cyc, uint32_t seed, int reps) {
  uint32_t lo = (threadIdx.x * 2654435761u) ^ seed, hi = lo * 0x9E3779B9u + 7;
  uint32_t acc = 0, steps = 0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    const uint32_t fsp1 = 7;
    uint32_t c = r & 3, c2 = (r + 1) & 3, cnt = 0;
    if constexpr (V == 0) {
      while (__any(c < 40u)) {
        const bool act = c < 40u;
        const uint32_t t = ffbl(win(lo, hi & 0xFF, c));
        const bool fnd = t != ~0u;
        cnt += (act && fnd) ? 1u : 0u;
        c = act ? (fnd ? c + t + fsp1 : 40u) : c;
        ++steps;
      }
    } else if constexpr (V == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool act = c < 40u;
        const uint32_t t = ffbl(win(lo, hi & 0xFF, c));
        const bool fnd = t != ~0u;
        cnt += (act && fnd) ? 1u : 0u;
        c = act ? (fnd ? c + t + fsp1 : 40u) : c;
      }
      steps += 8;
    } else if constexpr (V == 2) {
      while (__any(c < 40u)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bool act = c < 40u;
          const uint32_t t = ffbl(win(lo, hi & 0xFF, c));
          const bool fnd = t != ~0u;
          cnt += (act && fnd) ? 1u : 0u;
          c = act ? (fnd ? c + t + fsp1 : 40u) : c;
        }
        steps += 2;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool act = c < 40u, act2 = c2 < 40u;
        const uint32_t t = ffbl(win(lo, hi & 0xFF, c)), t2 = ffbl(win(hi, lo, c2));
        const bool fnd = t != ~0u, fnd2 = t2 != ~0u;
        cnt += (act && fnd) ? 1u : 0u;
        cnt += (act2 && fnd2) ? 1u : 0u;
        c = act ? (fnd ? c + t + fsp1 : 40u) : c;
        c2 = act2 ? (fnd2 ? c2 + t2 + fsp1 : 40u) : c2;
      }
      steps += 8;
    }
    acc += cnt + c + c2;
    lo = lo * 1664525u + 1013904223u;
    hi = hi ^ (lo >> 3);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) * 1000 / (steps ? steps : 1);
}

template <int V>
void run(const char* name, int waves_per_simd) {
  int nb = 1024 * waves_per_simd;
  uint32_t* out; unsigned long long* cyc;
  hipMalloc(&out, nb * 64 * 4); hipMalloc(&cyc, nb * 8);
  hipLaunchKernelGGL(kern<V>, dim3(nb), dim3(64), 0, 0, out, cyc, 1u, 2000);
  hipDeviceSynchronize();
  unsigned long long* h = (unsigned long long*)malloc(nb * 8);
  hipMemcpy(h, cyc, nb * 8, hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < nb; ++i) avg += h[i]; avg /= nb * 1000.0;
  printf("%-40s waves/SIMD=%d  cycles/step=%.1f\n", name, waves_per_simd, avg);
  hipFree(out); hipFree(cyc); free(h);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<0>("any-exit every step", w);
    run<1>("fixed 8 steps", w);
    run<2>("any-exit every 2 steps", w);
    run<3>("fixed 8 steps x2 chains (per step pair)", w);
  }
  return 0;
}
