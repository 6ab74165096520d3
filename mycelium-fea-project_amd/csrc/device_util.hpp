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

// DPP move of a double (two 32-bit halves), all lanes active
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
// Wave total in every lane, in a fixed order (identical in every wave):
// quad sums by quad_perm, 8- and 16-lane sums by row_half_mirror / row_mirror
// (each step pairs two equal-order partial sums, so all lanes of a row agree
// bitwise), then the four row sums read out as scalars.  VALU only: no LDS
// round trips (a __shfl_xor butterfly is 12 ds_bpermute_b32 per double).
__device__ __forceinline__ double wave_allsum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
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

// ---------------------------------------------------------------------------
// Shared pieces of the CG iteration kernels (cg.hip: SELL operator, ell.hip:
// wave-local lanes).
// ---------------------------------------------------------------------------
constexpr int kCgBS = 256;               // threads per block of the CG kernels
constexpr int kCgMaxG = kCgMaxPartials;  // max blocks (= partials re-read by each wave)

// y += V u with V the symmetric block (v0..v5)
__device__ __forceinline__ void block_mac(const double V[6], const double u[3], double y[3]) {
  y[0] = fma(V[0], u[0], fma(V[1], u[1], fma(V[2], u[2], y[0])));
  y[1] = fma(V[1], u[0], fma(V[3], u[1], fma(V[4], u[2], y[1])));
  y[2] = fma(V[2], u[0], fma(V[4], u[1], fma(V[5], u[2], y[2])));
}

template <bool BLOCK>
__device__ __forceinline__ void apply_m(const double* M, const double r[3], double u[3]) {
  if (BLOCK) {
    sym_apply(M, r, u);
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) u[a] = M[a] * r[a];
  }
}

// ---------------------------------------------------------------------------
// Partial-sum protocol.  part = two parity buffers of [4][kCgMaxG] doubles.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double* part_buf(double* part, int par) {
  return part + (size_t)par * 4 * kCgMaxG;
}

// Every lane ends with the grid total of the partials (block order, then a
// fixed butterfly): identical in every wave of every block.  PU = partial
// groups of 64 loaded per lane (G ≤ 64·PU).  The buffer is zeroed at the start
// of every solve and only blocks < G write it, so the slots ≥ G add exact
// zeros: every load is unconditional (a guarded or selected load makes hipcc
// branch and wait vmcnt(0) on all outstanding loads).
template <int PU>
__device__ __forceinline__ void wave_partials(const double* __restrict__ p, double s[4]) {
  const int lane = threadIdx.x & 63;
  double t[PU][4];
#pragma unroll
  for (int k = 0; k < PU; ++k) {
#pragma unroll
    for (int c = 0; c < 4; ++c) t[k][c] = p[c * kCgMaxG + lane + 64 * k];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < PU; ++k) a += t[k][c];
    s[c] = wave_allsum(a);
  }
}

// block partial (thread 0 stores it; the next launch's waves re-reduce).
// The cross-wave step uses a raw s_barrier behind an LDS-only wait: a
// __syncthreads() would also wait for every outstanding vector store (vmcnt(0)).
template <int BS = kCgBS>
__device__ __forceinline__ void store_block_partial(double (&acc)[4], double* __restrict__ p) {
  constexpr int NW = BS / 64;
  __shared__ double lds[NW * 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = wave_allsum(acc[c]);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) lds[wid * 4 + c] = acc[c];
  }
  if (NW > 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double s = lds[c];
      for (int w = 1; w < NW; ++w) s += lds[w * 4 + c];
      p[c * kCgMaxG + blockIdx.x] = s;
    }
  }
}

// α_j, β_j and the status of iteration j from the reduced partials S and the
// previous slot (identical in every wave of every block).
struct CgScalars {
  double alpha, beta, res;
  int status;
};
__device__ __forceinline__ CgScalars cg_scalars(const double S[4], int f0, double g0, double a0,
                                                double tol2, int it, int max_it, int norm) {
  CgScalars c;
  c.res = norm == 1 ? S[3] : S[2];
  const bool first = f0 == kInit;
  c.beta = first ? 0.0 : S[0] / g0;
  const double den = first ? S[1] : S[1] - c.beta * S[0] / a0;
  c.alpha = S[0] / den;
  if (f0 != kRun && f0 != kInit) c.status = kStop;
  else if (!(c.res > tol2)) c.status = isfinite(c.res) ? kConverged : kBreakdown;
  else if (it >= max_it) c.status = kMaxit;
  else c.status = ((den > 0.0) && isfinite(c.alpha) && isfinite(c.beta)) ? kRun : kBreakdown;
  return c;
}

// block 0 records iteration j's scalars in slots[j + 1]
__device__ __forceinline__ void cg_record(Slot* slots, int j, const double S[4],
                                          const CgScalars& c) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Slot sl;
    sl.v[0] = S[0]; sl.v[1] = S[1]; sl.v[2] = S[2]; sl.v[3] = S[3];
    sl.alpha = c.alpha;
    sl.beta = c.beta;
    sl.res = c.res;
    sl.flag = c.status;
    sl.pad = 0;
    slots[j + 1] = sl;
  }
}

// TRACE: lane 0 of every wave records s_memrealtime (100 MHz) at entry, once
// the partials are reduced, once the last row's SpMV is done, and after its
// stores have drained: trace[(block·4 + wave)·4 + point] (diagnostics only).
template <bool TRACE, int BS = kCgBS>
__device__ __forceinline__ void trace_point(unsigned long long* trace, int point, double dep) {
  if (TRACE) {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
    if ((threadIdx.x & 63) == 0)
      trace[((size_t)blockIdx.x * (BS / 64) + (threadIdx.x >> 6)) * 4 + point] = t;
  }
}

}  // namespace mfea
