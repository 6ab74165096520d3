// device_util.hpp — device helpers shared by the mfea kernels (wave64 reductions,
// fence-free last-block finalize, symmetric 3×3 block algebra).
#pragma once
#include "kernels.hpp"

namespace mfea {

// ---------------------------------------------------------------------------
// deterministic block reduction + last-block finalize (agent-scope ticket).
// Every block writes its partial sums, the block that draws the last ticket
// sums all partials in a fixed order and writes `out`.  Result is bitwise
// reproducible for a fixed grid size.  Protocol: cdna_hip_programming.md §6
// Guideline 16 (release → drained wait → relaxed agent atomic; acquire in the
// last block → wait → barrier → plain loads).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Hand-off without fences (MI355X_MICROARCH.md "Valid forms", table row 1):
// the partials are stored write-through (sc1, via agent-scope atomic stores),
// the storing lane drains them (s_waitcnt vmcnt(0)) before its agent-scope
// ticket add, and the last arriver reads every partial with sc1 loads, so no
// release/acquire fence (≈1.7 µs each) is paid on the per-iteration path.
template <int NV, int BS = kBlock>
__device__ __forceinline__ bool block_publish(double (&v)[NV], double* partials,
                                              unsigned* ticket, double* out) {
  constexpr int NW = BS / 64;
  __shared__ double lds[NW * NV];
  __shared__ int is_last;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned G = gridDim.x;
#pragma unroll
  for (int c = 0; c < NV; ++c) v[c] = wave_sum(v[c]);
  if (NW > 1) {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < NV; ++c) lds[wid * NV + c] = v[c];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      double s = NW > 1 ? lds[c] : v[c];
      for (int w = 1; w < NW; ++w) s += lds[w * NV + c];
      __hip_atomic_store(&partials[(size_t)c * G + blockIdx.x], s, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == G - 1);
  }
  __syncthreads();
  if (!is_last) return false;
  // U partials per lane in flight per pass: one memory round trip covers
  // BS·U blocks (the loads are independent; hipcc waits once per pass).
  constexpr int U = BS >= 256 ? 8 : 16;
  double s[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) s[c] = 0.0;
  for (unsigned i0 = threadIdx.x; i0 < G; i0 += BS * U) {
    double t[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned i = i0 + u * BS;
#pragma unroll
      for (int c = 0; c < NV; ++c)
        t[u][c] = i < G ? __hip_atomic_load(&partials[(size_t)c * G + i], __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT)
                        : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NV; ++c) s[c] += t[u][c];
  }
#pragma unroll
  for (int c = 0; c < NV; ++c) s[c] = wave_sum(s[c]);
  if (NW > 1) {
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < NV; ++c) lds[wid * NV + c] = s[c];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      double t = NW > 1 ? lds[c] : s[c];
      for (int w = 1; w < NW; ++w) t += lds[w * NV + c];
      out[c] = t;
    }
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

__device__ __forceinline__ void sym_apply(const double B[6], const double v[3], double o[3]) {
  o[0] = fma(B[0], v[0], fma(B[1], v[1], B[2] * v[2]));
  o[1] = fma(B[1], v[0], fma(B[3], v[1], B[4] * v[2]));
  o[2] = fma(B[2], v[0], fma(B[4], v[1], B[5] * v[2]));
}

__device__ __forceinline__ void sym_inverse(const double A[6], double B[6]) {
  // adjugate / determinant of a symmetric 3×3 (SPD here)
  const double c00 = A[3] * A[5] - A[4] * A[4];
  const double c01 = A[2] * A[4] - A[1] * A[5];
  const double c02 = A[1] * A[4] - A[2] * A[3];
  const double c11 = A[0] * A[5] - A[2] * A[2];
  const double c12 = A[1] * A[2] - A[0] * A[4];
  const double c22 = A[0] * A[3] - A[1] * A[1];
  const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
  const double id = 1.0 / det;
  B[0] = c00 * id; B[1] = c01 * id; B[2] = c02 * id;
  B[3] = c11 * id; B[4] = c12 * id; B[5] = c22 * id;
}

}  // namespace mfea
