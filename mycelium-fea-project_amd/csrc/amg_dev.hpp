// amg_dev.hpp — device helpers shared by the SA-AMG kernels (amg.hip) and the
// persistent deep-level V-cycle (amg_deep.hip): node-block loads / stores,
// the SELL-64 row products, block-Jacobi application, index-list sums.
#pragma once
#include "amg_kernels.hpp"
#include "device_util.hpp"

namespace mfea {

// ---- block / vector helpers (T = storage type, C = compute type) -----------
// Blocks are stored block-major ([position][NB2]): a SELL slot's 64 lanes read
// 64 consecutive blocks (one contiguous run, 16/32-B vector loads per lane),
// and the setup's index-list gathers fetch one contiguous block per item
// instead of NB2 separate cache lines (the component-major layout made the
// Galerkin products ≈ 0.7 TB/s effective).
template <int ND, class T, class C>
__device__ __forceinline__ void bload(const T* __restrict__ v, int64_t /*npos*/, int64_t q, C* m) {
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) m[c] = (C)v[q * (ND * ND) + c];
}
template <int ND, class T, class C>
__device__ __forceinline__ void bstore(T* __restrict__ v, int64_t /*npos*/, int64_t q, const C* m) {
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) v[q * (ND * ND) + c] = (T)m[c];
}
// symmetric blocks stored as their upper triangle (A_0: AmgMatD::sym, sym32),
// block-major.  (Component-major, [NS][npos], was measured slower for the
// SpMV: C3 10.5 vs 9.7 µs — three separate streams instead of one.)
template <int ND>
constexpr int nsym() { return ND * (ND + 1) / 2; }
template <int ND, class T, class C>
__device__ __forceinline__ void bload_sym(const T* __restrict__ v, int64_t /*npos*/, int64_t q, C* m) {
  constexpr int NS = nsym<ND>();
  C t[NS];
#pragma unroll
  for (int c = 0; c < NS; ++c) t[c] = (C)v[q * NS + c];
  if constexpr (ND == 2) {
    m[0] = t[0]; m[1] = t[1];
    m[2] = t[1]; m[3] = t[2];
  } else {
    m[0] = t[0]; m[1] = t[1]; m[2] = t[2];
    m[3] = t[1]; m[4] = t[3]; m[5] = t[4];
    m[6] = t[2]; m[7] = t[4]; m[8] = t[5];
  }
}
template <int ND, class T, class C>
__device__ __forceinline__ void bstore_sym(T* __restrict__ v, int64_t /*npos*/, int64_t q, const C* m) {
  if constexpr (ND == 2) {
    v[q * 3 + 0] = (T)m[0]; v[q * 3 + 1] = (T)m[1]; v[q * 3 + 2] = (T)m[3];
  } else {
    v[q * 6 + 0] = (T)m[0]; v[q * 6 + 1] = (T)m[1]; v[q * 6 + 2] = (T)m[2];
    v[q * 6 + 3] = (T)m[4]; v[q * 6 + 4] = (T)m[5]; v[q * 6 + 5] = (T)m[8];
  }
}
template <int ND, class T, class C>
__device__ __forceinline__ void vload(const T* __restrict__ v, int64_t i, C* o) {
#pragma unroll
  for (int a = 0; a < ND; ++a) o[a] = (C)v[ND * i + a];
}
// v if keep, else +0 — by masking v's bits, not by a select: a select of a
// loaded value let codegen branch around the load and wait for it inside the
// branch (one dependent round trip per slot); the same result bit for bit
__device__ __forceinline__ float keep_or_zero(float v, bool keep) {
  return __uint_as_float(__float_as_uint(v) & (keep ? 0xffffffffu : 0u));
}
__device__ __forceinline__ double keep_or_zero(double v, bool keep) {
  return __longlong_as_double(__double_as_longlong(v) & (keep ? -1ll : 0ll));
}
template <int ND, class T, class C>
__device__ __forceinline__ void vstore(T* __restrict__ v, int64_t i, const C* o) {
#pragma unroll
  for (int a = 0; a < ND; ++a) v[ND * i + a] = (T)o[a];
}
// C += A B
template <int ND>
__device__ __forceinline__ void mm_acc(const double* A, const double* Bm, double* C) {
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      double s = C[a * ND + b];
#pragma unroll
      for (int k = 0; k < ND; ++k) s = fma(A[a * ND + k], Bm[k * ND + b], s);
      C[a * ND + b] = s;
    }
}
// C += Aᵀ B
template <int ND>
__device__ __forceinline__ void mtm_acc(const double* A, const double* Bm, double* C) {
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      double s = C[a * ND + b];
#pragma unroll
      for (int k = 0; k < ND; ++k) s = fma(A[k * ND + a], Bm[k * ND + b], s);
      C[a * ND + b] = s;
    }
}
// exact inverse (adjugate / determinant); a singular block (a free row with
// no active element and reg = 0) gets 0, as PCJACOBI's guard does
template <int ND>
__device__ __forceinline__ void binv(const double* m, double* o) {
  if constexpr (ND == 2) {
    const double det = m[0] * m[3] - m[1] * m[2];
    const double id = det != 0.0 ? 1.0 / det : 0.0;
    o[0] = m[3] * id;
    o[1] = -m[1] * id;
    o[2] = -m[2] * id;
    o[3] = m[0] * id;
  } else {
    const double c00 = m[4] * m[8] - m[5] * m[7];
    const double c01 = m[5] * m[6] - m[3] * m[8];
    const double c02 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
    const double id = det != 0.0 ? 1.0 / det : 0.0;
    o[0] = c00 * id;
    o[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    o[3] = c01 * id;
    o[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    o[6] = c02 * id;
    o[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
  }
}
// symmetric block of the assembled operator (xx xy xz yy yz zz) → ND×ND
template <int ND>
__device__ __forceinline__ void sym_to(const double* s6, double* m) {
  if constexpr (ND == 2) {
    m[0] = s6[0];
    m[1] = s6[1];
    m[2] = s6[1];
    m[3] = s6[3];
  } else {
    m[0] = s6[0]; m[1] = s6[1]; m[2] = s6[2];
    m[3] = s6[1]; m[4] = s6[3]; m[5] = s6[4];
    m[6] = s6[2]; m[7] = s6[4]; m[8] = s6[5];
  }
}

__device__ __forceinline__ bool gated(const int32_t* gate) { return gate && *gate != kRun; }
// The V-cycle kernels load the gate with their first operands and test it only
// before their stores: a test at entry puts one more dependent memory round
// trip (≈ 1 µs: the flag was written on another XCD) in front of every launch,
// and a gated launch (only after convergence) may read whatever it likes.  The
// flag is read by a VECTOR load (agent scope): a scalar load of it — what a
// plain read of a uniform address compiles to — was waited for at the kernel's
// first instruction, the round trip this is meant to hide.
__device__ __forceinline__ int flag_load(const int32_t* p) {
  // an opaque per-lane zero: the value stays a per-lane one, so the compiler
  // waits for the load where the flag is used (the stores), not where a uniform
  // copy of it would have to be settled (the first branch of the kernel)
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return __hip_atomic_load((__attribute__((address_space(1))) int*)p + z, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// gate == NULL: no flag at all (the solve's chunks pass none, capi.hip
// enqueue_amg_chunk: every gated kernel is a pure function of the CG state
// the update kernel freezes once the solve stops, so running it past the stop
// rewrites the same values; the flag load only put its ≈ 1 µs miss — the
// flag is written on another XCD — in front of each launch's first wait)
__device__ __forceinline__ bool gate_open(const int32_t* gate) {
  return gate == nullptr || flag_load(gate) == kRun;
}

// XCD-aware block order for the gathering kernels.  Blocks are dealt
// round-robin over the 8 XCDs (b and b + 8 share one; MI355X_MICROARCH.md),
// each with its own L2: numbering the blocks so that every XCD's share is one
// contiguous row range keeps the neighbour rows a wave gathers in ITS L2
// instead of fetching the same lines into several.  A bijection on
// [0, gridDim.x); used for speed only, nothing depends on the placement.
__device__ __forceinline__ int64_t xcd_block_n(int64_t g) {  // over blocks [0, g) of the grid
  const int64_t b = blockIdx.x;
  const int64_t q = g >> 3, r = g & 7, x = b & 7, i = b >> 3;
  return x * q + (x < r ? x : r) + i;
}
__device__ __forceinline__ int64_t xcd_block() { return xcd_block_n(gridDim.x); }

// position q of a RowRange's span belongs to one of its rows (only the
// first and last slice can hold other ranks' rows)
__device__ __forceinline__ bool pos_mine(const RowRange& g, int64_t q) {
  if (q >= g.pf && q < g.pl) return true;
  const int64_t row = 64 * (q < g.pf ? g.s0 : g.s1) + (q & 63);
  return row >= g.lo && row < g.hi;
}

// One wave per slot row t ∈ [t0, t1) of M's SELL layout (the setup's value
// kernels: every thread owns one position, none idles — a (row, slot) grid
// sized by the widest slice left most threads of the wide-tailed P̃ / R̂
// layouts idle): position q = 64 t + lane, row 64 s + lane of slice
// s = srow[t], slot k = t − sptr[s].  False past the end (wave-uniform).
// blk: the block's index within its part of a fused grid (xcd_block() alone)
__device__ __forceinline__ bool slot_wave(const AmgMatD& M, int64_t t0, int64_t t1, int64_t& q, int64_t& row,
                                          int& k, int64_t blk) {
  const int64_t t = t0 + blk * (kBlock / 64) + (threadIdx.x >> 6);
  if (t >= t1) return false;
  const int s = __builtin_amdgcn_readfirstlane(M.srow[t]);
  k = (int)(t - M.sptr[s]);
  row = 64 * (int64_t)s + (threadIdx.x & 63);
  q = t * 64 + (threadIdx.x & 63);
  return true;
}
__device__ __forceinline__ bool slot_wave(const AmgMatD& M, int64_t t0, int64_t t1, int64_t& q, int64_t& row,
                                          int& k) {
  return slot_wave(M, t0, t1, q, row, k, xcd_block());
}

// a wave-uniform load of read-only plan data through the constant address
// space: a scalar load (s_load, counted by lgkmcnt).  Through a global
// pointer the compiler issues a vector load with a uniform address, and
// vector loads complete in order: the slice bounds then waited behind every
// load issued before them.
__device__ __forceinline__ int32_t uniform_load(const int32_t* p, int64_t i) {
  return ((const __attribute__((address_space(4))) int32_t*)p)[i];
}
// slot range of the wave's slice (scalar loads, wave-uniform)
__device__ __forceinline__ void slice_of(const AmgMatD& M, int64_t row, int64_t& base, int& width) {
  const int s = __builtin_amdgcn_readfirstlane((int)(row >> 6));
  const int a = uniform_load(M.sptr, s), b = uniform_load(M.sptr, s + 1);
  base = (int64_t)a * 64 + (row & 63);
  width = b - a;
}

// y ±= Σ_k M_k x_{col_k} over every SELL slot of one row (the diagonal
// included), in slot order.  Slot k of lane `sub` (S lanes per row, adjacent)
// is the row's slot k·S + sub; a step issues the column loads of U slots, then
// all their value and gather loads, then the FMAs: a row costs one dependent
// round trip (column, then gathers) per step.  Slots past the lane's count ws
// or padded (col < 0) contribute exact zeros.
template <int ND>
constexpr int mac_unroll() { return ND == 2 ? 4 : 2; }

template <int ND, int U, int S, bool SUB, bool SYM, class TV, class XP, class C>
__device__ __forceinline__ void sell_step(const int32_t* __restrict__ col, const TV* __restrict__ val,
                                          int64_t base, int k, int ws, int sub, XP x, C* y) {
  int32_t c[U];
  int64_t q[U];
  C m[U][ND * ND], xc[U][ND];
  // the slots' values need only the position: issued with the columns, so
  // the gathers' wait (vmcnt counts in order) leaves them in flight and the
  // dependent round trip carries the gathers alone
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = k + u < ws ? base + (int64_t)((k + u) * S + sub) * 64 : base;
    c[u] = k + u < ws ? col[q[u]] : -1;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (SYM) bload_sym<ND>(val, 0, q[u], m[u]);
    else bload<ND>(val, 0, q[u], m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) vload<ND>(x, c[u] >= 0 ? c[u] : 0, xc[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      // the SpMV (SYM): masked bits (C3 9.15 → 9.0 µs); the V-cycle's sweeps
      // measured slower that way (C5 iteration 651 → 690 µs): a select there
      if constexpr (SYM) xc[u][b] = keep_or_zero(xc[u][b], c[u] >= 0);
      else xc[u][b] = c[u] >= 0 ? xc[u][b] : (C)0;
    }
#pragma unroll
    for (int a = 0; a < ND; ++a)
#pragma unroll
      for (int b = 0; b < ND; ++b)
        y[a] = fma(SUB ? -m[u][a * ND + b] : m[u][a * ND + b], xc[u][b], y[a]);
  }
}
// one step of the smallest of 1, 2, 4, … UMAX slots covering rem (> 0)
template <int ND, int UMAX, int S, bool SUB, bool SYM, class TV, class XP, class C>
__device__ __forceinline__ int sell_step_by(const int32_t* __restrict__ col, const TV* __restrict__ val,
                                            int64_t base, int k, int rem, int ws, int sub, XP x, C* y) {
  if (UMAX >= 16 && rem > 8) {
    sell_step<ND, (UMAX >= 16 ? 16 : 1), S, SUB, SYM>(col, val, base, k, ws, sub, x, y);
    return 16;
  }
  if (UMAX >= 8 && rem > 4) {
    sell_step<ND, (UMAX >= 8 ? 8 : 1), S, SUB, SYM>(col, val, base, k, ws, sub, x, y);
    return 8;
  }
  if (UMAX >= 4 && rem > 2) {
    sell_step<ND, (UMAX >= 4 ? 4 : 1), S, SUB, SYM>(col, val, base, k, ws, sub, x, y);
    return 4;
  }
  if (rem > 1) {
    sell_step<ND, 2, S, SUB, SYM>(col, val, base, k, ws, sub, x, y);
    return 2;
  }
  sell_step<ND, 1, S, SUB, SYM>(col, val, base, k, ws, sub, x, y);
  return 1;
}
// The steps over a wave's slice: wu steps per lane (uniform over the wave —
// the slice's width), each step the smallest of 1, 2, 4, … UMAX slots that
// covers what is left, so a row of up to UMAX slots per lane is one round
// trip and no step issues more than twice the loads it needs.  (Steps of a
// fixed U = 8 issued 8 loads per lane for the ≈ 1–2 slots each of the 8
// lanes of a C3 R̂ row holds: the down sweep's vector-memory instructions
// were three quarters padding.)  The branches are wave-uniform.
template <int ND, int UMAX, int S, bool SUB, bool SYM, class TV, class XP, class C>
__device__ __forceinline__ void sell_steps(const int32_t* __restrict__ col, const TV* __restrict__ val,
                                           int64_t base, int wu, int ws, int sub, XP x, C* y) {
  for (int k = 0; k < wu;) k += sell_step_by<ND, UMAX, S, SUB, SYM>(col, val, base, k, wu - k, ws, sub, x, y);
}
// One lane per row.  K bounds the widest step (the kernel's VGPR count is its
// widest path's): U·2^(K−1) slots with U = mac_unroll — the f64 SpMV, whose
// level-0 slices are ≤ 4 wide for 98 % of the waves, stays at K = 1 (a 2U path
// put it at 139 VGPRs, one 768-thread block per CU); the streaming level-0
// kernels use K = 2; the restrictions and the latency-bound coarse levels K = 3.
template <int ND, bool SUB, int K = 2, bool SYM = false, class TV, class XP, class C>
__device__ __forceinline__ void sell_mac(const int32_t* __restrict__ col, const TV* __restrict__ val,
                                         int64_t /*npos*/, int64_t base, int w,
                                         XP x, C* y) {
  constexpr int UMAX = mac_unroll<ND>() << (K - 1);
  sell_steps<ND, UMAX, 1, SUB, SYM>(col, val, base, w, w, 0, x, y);
}

// o = s · D⁻¹ v  (D⁻¹ [n][NB2], storage TD, compute C).  dinv_load / dinv_mul
// split it so a kernel can issue the block's load before its gather.
template <int ND, class TD, class C>
__device__ __forceinline__ void dinv_load(const TD* __restrict__ dinv, int64_t i, C* Di) {
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) Di[c] = (C)dinv[i * (ND * ND) + c];
}
template <int ND, class C>
__device__ __forceinline__ void dinv_mul(const C* Di, C s, const C* v, C* o) {
#pragma unroll
  for (int a = 0; a < ND; ++a) {
    C acc = 0;
#pragma unroll
    for (int b = 0; b < ND; ++b) acc = fma(Di[a * ND + b], v[b], acc);
    o[a] = s * acc;
  }
}
template <int ND, class TD, class C>
__device__ __forceinline__ void dinv_apply(const TD* __restrict__ dinv, int64_t /*n*/, int64_t i, C s,
                                           const C* v, C* o) {
  C Di[ND * ND];
  dinv_load<ND>(dinv, i, Di);
  dinv_mul<ND>(Di, s, v, o);
}

// C += Σ_t X[a_t]·Y[b_t] (TX: X[a_t]ᵀ·Y[b_t]) over one index list, in list
// order, U pairs' loads in flight per step (every pair is two dependent hops:
// index, then blocks); pair_sum takes steps of 4.
template <int ND, bool TX, int U, class TX_, class TY_>
__device__ __forceinline__ void pair_sum_u(int t0, int t1, const int32_t* __restrict__ la,
                                           const int32_t* __restrict__ lb, const TX_* __restrict__ X,
                                           const TY_* __restrict__ Y, double* C) {
  for (int t = t0; t < t1; t += U) {
    int32_t ia[U], ib[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u < t1 ? t + u : t0;
      ia[u] = la[tt];
      ib[u] = lb[tt];
    }
    double x[U][ND * ND], y[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bload<ND>(X, 0, ia[u], x[u]);
      bload<ND>(Y, 0, ib[u], y[u]);
    }
    // the pairs past the list (they re-read pair t0) add exact zeros: a
    // guarded sum let codegen sink each pair's loads into its branch — one
    // pair's index and block round trips after another instead of U at once
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) x[u][c] = keep_or_zero(x[u][c], t + u < t1);
      if (TX) mtm_acc<ND>(x[u], y[u], C);
      else mm_acc<ND>(x[u], y[u], C);
    }
  }
}
template <int ND, bool TX, class TX_, class TY_>
__device__ __forceinline__ void pair_sum(int t0, int t1, const int32_t* __restrict__ la,
                                         const int32_t* __restrict__ lb, const TX_* __restrict__ X,
                                         int64_t /*nx*/, const TY_* __restrict__ Y, int64_t /*ny*/, double* C) {
  // four pairs a step whatever the length: the eight-pair path for lists
  // over four (its VGPRs set the kernel's occupancy: A·P 92 → 74) measured
  // slower now that every step's loads are in flight together (C3 setup
  // −13 µs, C5 −160 µs, profiles/r6/ab_pair_sum_u4.log)
  pair_sum_u<ND, TX, 4>(t0, t1, la, lb, X, Y, C);
}
// S += Σ_t X[a_t] over one index list, in list order
template <int ND, int U, class TX_>
__device__ __forceinline__ void list_sum_u(int t0, int t1, const int32_t* __restrict__ la,
                                           const TX_* __restrict__ X, double* S) {
  for (int t = t0; t < t1; t += U) {
    int32_t ia[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ia[u] = la[t + u < t1 ? t + u : t0];
    double x[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) bload<ND>(X, 0, ia[u], x[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)  // (past the list: exact zeros, as pair_sum_u)
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) S[c] += keep_or_zero(x[u][c], t + u < t1);
  }
}
template <int ND, class TX_>
__device__ __forceinline__ void list_sum(int t0, int t1, const int32_t* __restrict__ la,
                                         const TX_* __restrict__ X, int64_t /*nx*/, double* S) {
  list_sum_u<ND, 4>(t0, t1, la, X, S);  // (steps of 4, as pair_sum: profiles/r6/ab_list_sum_u4.log)
}

constexpr double kRhoFloor = 2.0;   // the exact level-0 bound (see the header)
constexpr double kRhoSafety = 1.45; // ω·g ≤ (4/3)·1.45 < 2

// the smoother weight ω_l from the level's Gershgorin bound g = omega[1]
__device__ __forceinline__ double amg_omega(const double* __restrict__ om) {
  return (4.0 / 3.0) / (om[0] > 0.0 ? om[0] : fmax(kRhoFloor, om[1] / kRhoSafety));
}
// ... through scalar loads (omega is written by the setup, read-only in the
// solve's launches): no vector-load ordering, hoistable across stores
__device__ __forceinline__ double amg_omega_s(const double* om) {
  const auto* c = (const __attribute__((address_space(4))) double*)om;
  const double o0 = c[0], o1 = c[1];
  return (4.0 / 3.0) / (o0 > 0.0 ? o0 : fmax(kRhoFloor, o1 / kRhoSafety));
}

// S lanes per row (S = 2, 4) for the SELL operators with wide rows: R's rows
// hold 7–8 blocks on average and up to 29 (A below level 0: 4–5, up to 16),
// so one lane per row issues dozens of scattered loads in sequence; here lane
// `sub` of a row takes slots sub, sub + S, … and the S partial sums meet by a
// fixed butterfly (deterministic).  The S lanes of a row are adjacent, so a
// wave covers 64/S rows of one slice and each slot step reads S runs of 64/S
// consecutive positions.  Every lane ends with the row's full sum.
template <int ND, int S, bool SUB, class TV, class XP, class C>
__device__ __forceinline__ void sell_mac_sub(const int32_t* __restrict__ col, const TV* __restrict__ val,
                                             int64_t base, int w, int sub, XP x, C* y) {
  constexpr int U = 2 * mac_unroll<ND>();  // (U = 4: C2 62.4 vs 60.8 µs per iteration)
  const int wu = (w + S - 1) / S;  // steps: the slice's, uniform
  const int ws = w > sub ? (w - sub + S - 1) / S : 0;
  sell_steps<ND, U, S, SUB, false>(col, val, base, wu, ws, sub, x, y);
#pragma unroll
  for (int o = 1; o < S; o <<= 1)
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] += __shfl_xor(y[a], o, 64);
}

}  // namespace mfea
