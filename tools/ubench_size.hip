// ubench_size.hip — the achievable HBM read rate of ONE launch as a function
// of the bytes it moves: a coalesced 16-B/lane streaming read (the best case
// of any kernel here), launched back to back 200 times per size and timed
// with HIP events, so each launch pays what a graph-replayed kernel of the
// iteration pays (launch, ramp, drain) — the ceiling to read the SpMV's and
// the V-cycle kernels' roofline fractions against.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_size.hip -o ubench_size && ./ubench_size
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(256) void k_read16(const double2* __restrict__ a, double* out, long n) {
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1234.5) out[0] = s;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const long max_bytes = 1L << 30;
  double2* a = nullptr;
  double* out = nullptr;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&out, sizeof(double)));
  CK(hipMemset(a, 0, max_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long sizes_mb[] = {2, 4, 8, 16, 24, 32, 43, 64, 128, 256, 512, 666, 1024};
  const int reps = 200;
  for (int warm = 0; warm < 2; ++warm)
  for (long mb : sizes_mb) {
    const long bytes = mb << 20;
    const long n = bytes / 16;
    // one row per thread up to 256 Ki threads per XCD-balanced grid, then grid-stride
    long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    // rotate over the 1 GiB buffer so consecutive launches of small sizes do
    // not all hit one region (sizes ≤ 256 MB still fit the Infinity Cache)
    k_read16<<<dim3((unsigned)blocks), dim3(256)>>>(a, out, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) {
      // warm 0: consecutive launches read different regions of the 1 GiB
      // buffer (HBM); warm 1: the same region every time (≤ 256 MB stays in
      // the Infinity Cache, as a C3 iteration's 225 MB working set can)
      const long off = warm ? 0 : ((long)r * bytes) % (max_bytes - bytes + 16) / 16;
      k_read16<<<dim3((unsigned)blocks), dim3(256)>>>(a + off, out, n);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    std::printf("{\"same_region\": %d, \"bytes_MB\": %ld, \"us_per_launch\": %.3f, \"GBps\": %.1f, "
                "\"frac_of_8TBps\": %.3f}\n", warm, mb, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
  }
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
