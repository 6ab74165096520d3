// ubench_latency.hip — measures the latency terms that bound one CG iteration
// at small sizes (launch boundary, dependent global-load round trip, a
// predecessor's dirty lines).  Build: hipcc --offload-arch=gfx950 -O3 ...
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void k_empty() {}

// one wave chases a pointer chain of length L
__global__ void k_chase(const long* next, long start, int L, long* out) {
  long p = start;
  for (int i = 0; i < L; ++i) p = next[p];
  if (threadIdx.x == 0) out[0] = p;
}

// many blocks: each lane does L dependent loads within its own region
__global__ void k_chase_wide(const long* next, int L, long n, long* out) {
  long p = ((long)blockIdx.x * blockDim.x + threadIdx.x) % n;
  for (int i = 0; i < L; ++i) p = next[p];
  out[(long)blockIdx.x * blockDim.x + threadIdx.x] = p;
}

// writes B bytes (dirty lines left for the successor)
__global__ void k_write(double* a, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    a[i] = (double)i;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto&& f, int reps) -> float {
    f();
    hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / reps;
  };
  // 1. empty kernels back to back (1 block, 133 blocks, 512 blocks)
  for (int g : {1, 133, 512, 2048}) {
    float us = timeit([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, s); }, 2000);
    std::printf("empty kernel grid %4d: %.2f us/launch\n", g, us);
  }
  // graph of 64 empty launches
  {
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < 64; ++i) hipLaunchKernelGGL(k_empty, dim3(133), dim3(256), 0, s);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    float us = timeit([&] { hipGraphLaunch(ge, s); }, 100);
    std::printf("graph of 64 empty (133 blk): %.2f us/kernel\n", us / 64);
  }
  // 2. dependent load latency: chain over a buffer of `bytes`, stride 4 KB + random
  for (long bytes : {1L << 20, 32L << 20, 512L << 20}) {
    long n = bytes / 8;
    std::vector<long> h(n);
    // random cyclic permutation over cache-line-spaced slots
    long m = n / 16;
    std::vector<long> perm(m);
    for (long i = 0; i < m; ++i) perm[i] = i;
    unsigned long long x = 88172645463325252ull;
    for (long i = m - 1; i > 0; --i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      long j = x % (i + 1);
      std::swap(perm[i], perm[j]);
    }
    for (long i = 0; i < m; ++i) h[perm[i] * 16] = perm[(i + 1) % m] * 16;
    long *d, *o;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, 1 << 24));
    CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
    for (int L : {1, 16, 64}) {
      float us = timeit([&] { hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, s, d, perm[0] * 16, L, o); }, 200);
      std::printf("chase %5ld KB L=%2d: %.2f us/launch (%.3f us/hop over empty)\n", bytes >> 10, L, us, 0.0);
    }
    // chase right after a kernel that dirties 8 MB elsewhere
    double* w;
    CK(hipMalloc(&w, 64 << 20));
    for (long wb : {1L << 20, 8L << 20, 64L << 20}) {
      float us = timeit([&] {
        hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, s, w, wb / 8);
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, s, d, perm[0] * 16, 16, o);
      }, 200);
      float us_w = timeit([&] { hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, s, w, wb / 8); }, 200);
      std::printf("  write %5ld KB then chase L=16: %.2f us (write alone %.2f)\n", wb >> 10, us, us_w);
    }
    // wide chase (133 blocks × 256 lanes, each L dependent loads)
    for (int L : {1, 4}) {
      float us = timeit([&] { hipLaunchKernelGGL(k_chase_wide, dim3(133), dim3(256), 0, s, d, L, n, o); }, 200);
      std::printf("wide chase 133x256 L=%d over %ld KB: %.2f us\n", L, bytes >> 10, us);
    }
    hipFree(w);
    hipFree(d);
    hipFree(o);
  }
  return 0;
}
