// device_util.hpp — device helpers shared by the mfea kernels (wave64 reductions,
// fence-free sharded last-block finalize, symmetric 3×3 block algebra).
#pragma once
#include "kernels.hpp"

namespace mfea {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Ticket layout: one ticket set = kTicketStride unsigned; shard s counter at
// s·16 (64 B apart, separate lines), the top counter at kShards·16.
constexpr int kShards = 8;
static_assert((kShards + 1) * 16 <= kTicketStride, "ticket set too small");

// Sum over the block of NV values, result on thread 0 (others: garbage).
template <int NV, int BS>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* lds) {
  constexpr int NW = BS / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NV; ++c) v[c] = wave_sum(v[c]);
  if (NW > 1) {
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < NV; ++c) lds[wid * NV + c] = v[c];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        double s = lds[c];
        for (int w = 1; w < NW; ++w) s += lds[w * NV + c];
        v[c] = s;
      }
    }
  }
}

__device__ __forceinline__ void store_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Deterministic grid reduction finished inside the launch (no second kernel):
// every block publishes its partial sums; the last arriver of each of
// kShards shards (blocks ≡ s mod kShards) sums its shard's partials in block
// order and publishes a shard sum; the last shard finisher sums the shard sums
// in shard order and writes `out`.  Bitwise reproducible for a fixed grid.
//
// Two levels because same-address agent atomics serialize at ≈12 ns each
// (MI355X_MICROARCH.md, row "fanin"): one counter for 1,300 blocks costs
// ≈16 µs; eight shards of ≤165 plus a top counter of 8 cost ≈2 µs.
//
// Hand-off without fences (MI355X_MICROARCH.md "Valid forms", table row 1):
// payload stored write-through (sc1, agent-scope atomic stores), the storing
// lane drains it (s_waitcnt vmcnt(0)) before its agent-scope ticket add, the
// last arriver reads every payload word with sc1 loads.  No ≈1.7 µs
// release/acquire fence on the per-iteration path.
// partials must hold NV·(gridDim + kShards) doubles.
// ---------------------------------------------------------------------------
template <int NV, int BS = kBlock>
__device__ __forceinline__ bool block_publish(double (&v)[NV], double* partials,
                                              unsigned* ticket, double* out) {
  constexpr int NW = BS / 64;
  __shared__ double lds[NW * NV];
  __shared__ int flag;
  const unsigned G = gridDim.x, b = blockIdx.x;
  const unsigned S = G < (unsigned)kShards ? G : (unsigned)kShards;
  const unsigned shard = b % S;
  const unsigned nshard = (G - shard + S - 1) / S;
  double* spart = partials + (size_t)NV * G;  // shard sums, [c][S]

  block_sum<NV, BS>(v, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < NV; ++c) store_sc1(&partials[(size_t)c * G + b], v[c]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t =
        __hip_atomic_fetch_add(&ticket[shard * 16], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = (t == nshard - 1);
  }
  __syncthreads();
  if (!flag) return false;

  // ---- last block of this shard: sum its blocks' partials in block order
  constexpr int U = BS >= 256 ? 4 : 8;
  double s[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) s[c] = 0.0;
  for (unsigned k0 = threadIdx.x; k0 < nshard; k0 += BS * U) {
    double t[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned k = k0 + u * BS;
      const unsigned blk = shard + k * S;
#pragma unroll
      for (int c = 0; c < NV; ++c) t[u][c] = k < nshard ? load_sc1(&partials[(size_t)c * G + blk]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NV; ++c) s[c] += t[u][c];
  }
  block_sum<NV, BS>(s, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < NV; ++c) store_sc1(&spart[c * S + shard], s[c]);
    __hip_atomic_store(&ticket[shard * 16], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(&ticket[kShards * 16], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    flag = (t == S - 1);
  }
  __syncthreads();
  if (!flag) return false;

  // ---- last shard finisher: shard sums in shard order
  if (threadIdx.x == 0) {
    double r[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) r[c] = 0.0;
    for (unsigned q = 0; q < S; ++q)
#pragma unroll
      for (int c = 0; c < NV; ++c) r[c] += load_sc1(&spart[c * S + q]);
#pragma unroll
    for (int c = 0; c < NV; ++c) out[c] = r[c];
    __hip_atomic_store(&ticket[kShards * 16], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
