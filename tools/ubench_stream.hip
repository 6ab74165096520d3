// ubench_stream.hip — known-byte kernels to calibrate rocprofv3 FETCH_SIZE /
// WRITE_SIZE for the access widths the CG kernel uses (MI355X_MICROARCH.md
// §HBM: FETCH_SIZE reads ½ of a 16-B/lane stream; other widths uncalibrated).
// Each kernel reads (and writes) exactly `bytes` once.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_read8(const double* __restrict__ a, double* out, long n) {
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 1234.5) out[0] = s;
}
__global__ void k_read24(const double* __restrict__ a, double* out, long rows) {  // 3 × 8 B per lane
  double s = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += (long)gridDim.x * blockDim.x)
    s += a[3 * i] + a[3 * i + 1] + a[3 * i + 2];
  if (s == 1234.5) out[0] = s;
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
  hipMemset(a, 0, bytes);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_read8, dim3(2048), dim3(256), 0, 0, a, o, bytes / 8);
    hipLaunchKernelGGL(k_read24, dim3(2048), dim3(256), 0, 0, a, o, bytes / 24);
    hipLaunchKernelGGL(k_write24, dim3(2048), dim3(256), 0, 0, a, bytes / 24);
  }
  hipDeviceSynchronize();
  std::printf("bytes per kernel: %ld\n", bytes);
  return 0;
}
