// ubench_barrier.hip — what one phase of a persistent multi-workgroup kernel
// costs on MI355X against the same phase as its own launch (amg_deep.hip's
// design question).  A phase = every thread gathers one f32 pair of the
// previous phase's vector at a scattered index and writes its own pair.
//   launches: one kernel per phase, plain loads / stores, graph-replayed
//   persist : one launch, G workgroups × 1024, phases separated by a grid
//             barrier; vectors through agent-scope (sc1) loads / stores
// Barrier variants: 8 sharded counters polled by 8 lanes (s_sleep 1 between
// polls, or none), one counter.
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_barrier tools/ubench_barrier.hip
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

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned gu32_t;

__device__ __forceinline__ unsigned long long ld_sc1(const float* p, long i) {
  return __hip_atomic_load((gu64_t*)(p + 2 * i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, long i, unsigned long long v) {
  __hip_atomic_store((gu64_t*)(p + 2 * i), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>  // 0: 8 shards + sleep, 1: 8 shards no sleep, 2: one counter + sleep
__device__ __forceinline__ void gbar(unsigned* bar, unsigned target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int sh = MODE == 2 ? 0 : (blockIdx.x & 7);
    if (lane == 0) __hip_atomic_fetch_add((gu32_t*)(bar + 32 * sh), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spin = 0; spin < (1u << 20); ++spin) {
      unsigned v = (MODE == 2 ? lane == 0 : lane < 8)
                       ? __hip_atomic_load((gu32_t*)(bar + 32 * lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0u;
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if ((unsigned)__builtin_amdgcn_readfirstlane(v) >= target) break;
      if (MODE != 1) __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}

// WORK: 0 barrier only, 1 the gather phase
template <int MODE, int WORK>
__global__ __launch_bounds__(1024) void k_persist(unsigned* bar, int nph, float* v0, float* v1, const int* idx, long n) {
  const long T = (long)gridDim.x * 1024;
  for (int p = 0; p < nph; ++p) {
    if (WORK) {
      const float* src = (p & 1) ? v1 : v0;
      float* dst = (p & 1) ? v0 : v1;
      for (long i = (long)blockIdx.x * 1024 + threadIdx.x; i < n; i += T) {
        const unsigned long long a = ld_sc1(src, idx[i]);
        st_sc1(dst, i, a + 1);
      }
    }
    gbar<MODE>(bar, (unsigned)(p + 1) * gridDim.x);
  }
}

__global__ __launch_bounds__(256) void k_phase(const float* src, float* dst, const int* idx, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long* s = (const unsigned long long*)src;
  ((unsigned long long*)dst)[i] = s[idx[i]] + 1;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  unsigned* bar;
  CK(hipMalloc(&bar, 4096));
  const long nmax = 1 << 20;
  float *v0, *v1;
  int* idx;
  CK(hipMalloc(&v0, nmax * 8));
  CK(hipMalloc(&v1, nmax * 8));
  CK(hipMalloc(&idx, nmax * 4));
  CK(hipMemset(v0, 0, nmax * 8));
  CK(hipMemset(v1, 0, nmax * 8));
  const int nph = 64;
  auto timed = [&](auto&& f, int reps) -> float {
    f();
    CK(hipStreamSynchronize(s));
    hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / reps;
  };
  for (long n : {1024L, 16384L, 131072L}) {
    // scattered but local indices (a neighbour within ±512)
    std::vector<int> h(n);
    unsigned long long x = 88172645463325252ull;
    for (long i = 0; i < n; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      long j = i + (long)(x % 1024) - 512;
      h[i] = (int)(j < 0 ? 0 : (j >= n ? n - 1 : j));
    }
    CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
    // launches, graph-replayed
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int p = 0; p < nph; ++p)
      hipLaunchKernelGGL(k_phase, dim3((n + 255) / 256), dim3(256), 0, s, (p & 1) ? v1 : v0, (p & 1) ? v0 : v1, idx, n);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    const float lu = timed([&] { hipGraphLaunch(ge, s); }, 20);
    std::printf("n %7ld  launches: %.2f us/phase\n", n, lu / nph);
    for (int g : {8, 32, 64, 128, 256}) {
      float t[4];
      int k = 0;
      auto run = [&](auto kern) {
        return timed([&] {
          hipMemsetAsync(bar, 0, 4096, s);
          hipLaunchKernelGGL(kern, dim3(g), dim3(1024), 0, s, bar, nph, v0, v1, (const int*)idx, n);
        }, 20);
      };
      t[k++] = run(k_persist<0, 0>);
      t[k++] = run(k_persist<0, 1>);
      t[k++] = run(k_persist<1, 1>);
      t[k++] = run(k_persist<2, 1>);
      std::printf("n %7ld  G %3d  barrier-only %.2f  phase: shards+sleep %.2f  shards %.2f  one-counter %.2f us/phase\n",
                  n, g, t[0] / nph, t[1] / nph, t[2] / nph, t[3] / nph);
    }
    hipGraphExecDestroy(ge);
    hipGraphDestroy(gr);
  }
  return 0;
}
