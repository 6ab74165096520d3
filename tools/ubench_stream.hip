// ubench_stream.hip — known-byte kernels to calibrate rocprofv3 FETCH_SIZE /
// WRITE_SIZE for the access widths the GAMG kernels use (MI355X_MICROARCH.md
// §HBM: FETCH_SIZE reads ½ of a 16-B/lane stream; other widths uncalibrated).
// Each kernel reads (and writes) exactly `bytes` once, from a buffer larger
// than the 256 MiB Infinity Cache:
//   k_read16   16 B per lane, coalesced (the guide's calibrated case)
//   k_read8    8 B per lane  (the CG's f64 vectors r, u, w)
//   k_read4    4 B per lane  (SELL column indices)
//   k_read24   3 × 8 B per lane (A_0's symmetric f64 blocks)
//   k_read12   3 × 4 B per lane (A_0's symmetric f32 blocks)
//   k_gather8  8 B per lane at a permuted index inside each 128-B group (the
//              f32 u pairs the SpMV gathers, with perfect line reuse)
//   k_write24  3 × 8 B per lane written
// Run each under its own `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
// pass; tools/fetch_calib.py divides the counters by the known bytes.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_read16(const double2* __restrict__ a, double* out, long n) {
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1234.5) out[0] = s;
}
__global__ void k_read8(const double* __restrict__ a, double* out, long n) {
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 1234.5) out[0] = s;
}
__global__ void k_read4(const int* __restrict__ a, double* out, long n) {
  long s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 1234) out[0] = (double)s;
}
__global__ void k_read24(const double* __restrict__ a, double* out, long rows) {  // 3 × 8 B per lane
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (long)gridDim.x * blockDim.x)
    s += a[3 * i] + a[3 * i + 1] + a[3 * i + 2];
  if (s == 1234.5) out[0] = s;
}
__global__ void k_read12(const float* __restrict__ a, double* out, long rows) {  // 3 × 4 B per lane
  float s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (long)gridDim.x * blockDim.x)
    s += a[3 * i] + a[3 * i + 1] + a[3 * i + 2];
  if (s == 1234.5f) out[0] = s;
}
// lane i reads pair (i & ~15) | perm(i & 15): every 128-B group of 16 pairs is
// read once, in a scrambled order (the gather's access width and line reuse)
__global__ void k_gather8(const float2* __restrict__ a, double* out, long n) {
  float s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long j = (i & ~15L) | ((i * 7 + 3) & 15);
    const float2 v = a[j];
    s += v.x + v.y;
  }
  if (s == 1234.5f) out[0] = s;
}
__global__ void k_write24(double* __restrict__ a, long rows) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (long)gridDim.x * blockDim.x) {
    a[3 * i] = 1.0;
    a[3 * i + 1] = 2.0;
    a[3 * i + 2] = 3.0;
  }
}

int main() {
  const long bytes = 768L << 20;  // > 256 MiB Infinity Cache
  double *a, *o;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
  const dim3 g(2048), b(256);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_read16, g, b, 0, 0, (const double2*)a, o, bytes / 16);
    hipLaunchKernelGGL(k_read8, g, b, 0, 0, a, o, bytes / 8);
    hipLaunchKernelGGL(k_read4, g, b, 0, 0, (const int*)a, o, bytes / 4);
    hipLaunchKernelGGL(k_read24, g, b, 0, 0, a, o, bytes / 24);
    hipLaunchKernelGGL(k_read12, g, b, 0, 0, (const float*)a, o, bytes / 12);
    hipLaunchKernelGGL(k_gather8, g, b, 0, 0, (const float2*)a, o, bytes / 8);
    hipLaunchKernelGGL(k_write24, g, b, 0, 0, a, bytes / 24);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("bytes per kernel: %ld\n", bytes);
  return 0;
}
