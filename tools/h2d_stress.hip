// Diagnostic: concurrent large host->device copies from mapped pinned memory,
// the facade's pattern (one stream per thread, hipHostMalloc'd staging,
// stream-ordered device buffers), each checked by a kernel on the same stream.
// usage: h2d_stress [threads] [MiB] [iterations] [pool: 0 default, 1 own, 2 hipMalloc]
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__global__ void check_kernel(const uint32_t* d, size_t n, uint32_t seed, unsigned long long* bad,
                             unsigned long long* first) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (d[i] != (uint32_t)(i * 2654435761u) + seed) {
      atomicAdd(bad, 1ull);
      atomicMin(first, (unsigned long long)i);
    }
  }
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? std::atoi(argv[1]) : 4;
  const size_t mib = argc > 2 ? std::strtoul(argv[2], nullptr, 10) : 128;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 50;
  const int pool_kind = argc > 4 ? std::atoi(argv[4]) : 0;
  const size_t n = (mib << 20) / 4;
  std::atomic<long> total_bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      CK(hipSetDevice(0));
      hipStream_t s;
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      hipMemPool_t pool = nullptr;
      if (pool_kind == 1) {
        hipMemPoolProps p{};
        p.allocType = hipMemAllocationTypePinned;
        p.handleTypes = hipMemHandleTypeNone;
        p.location.type = hipMemLocationTypeDevice;
        p.location.id = 0;
        CK(hipMemPoolCreate(&pool, &p));
      }
      uint32_t* h = nullptr;
      CK(hipHostMalloc((void**)&h, n * 4 + 64, hipHostMallocMapped));
      unsigned long long* hr = nullptr;
      CK(hipHostMalloc((void**)&hr, 64, hipHostMallocMapped));
      for (int it = 0; it < iters; ++it) {
        const uint32_t seed = 0x1000u * t + it;
        for (size_t i = 0; i < n; ++i) h[i] = (uint32_t)(i * 2654435761u) + seed;
        void* d = nullptr;
        // a fresh device buffer every iteration, freed after it (as the
        // facade's trim does), so buffers move between streams
        if (pool_kind == 2) CK(hipMalloc(&d, n * 4 + 64));
        else if (pool) CK(hipMallocFromPoolAsync(&d, n * 4 + 64, pool, s));
        else CK(hipMallocAsync(&d, n * 4 + 64, s));
        auto* res = reinterpret_cast<unsigned long long*>((char*)d + n * 4);
        CK(hipMemcpyAsync(d, h, n * 4, hipMemcpyHostToDevice, s));
        CK(hipMemsetAsync(res, 0, 8, s));
        CK(hipMemsetAsync(res + 1, 0xFF, 8, s));
        hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, s, (const uint32_t*)d, n, seed, res, res + 1);
        CK(hipMemcpyAsync(hr, res, 16, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (hr[0]) {
          std::printf("thread %d iter %d: %llu bad words, first at %llu of %zu\n", t, it, hr[0], hr[1], n);
          std::fflush(stdout);
          total_bad += (long)hr[0];
        }
        if (pool_kind == 2) CK(hipFree(d));
        else CK(hipFreeAsync(d, s));
      }
      CK(hipStreamSynchronize(s));
    });
  }
  for (auto& x : th) x.join();
  std::printf("h2d_stress threads=%d MiB=%zu iters=%d pool=%d: %s\n", T, mib, iters, pool_kind,
              total_bad ? "MISMATCH" : "OK");
  return total_bad ? 1 : 0;
}
