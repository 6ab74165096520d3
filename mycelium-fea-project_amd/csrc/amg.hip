// amg.hip — SA-AMG preconditioned CG on device (amg.hpp, amg_kernels.hpp).
//
// Numeric setup per solve (after assembly), level by level, in f64:
//   A_0      gather of the assembled SELL slots (multi-edges summed in slot order)
//   D_l⁻¹    exact inverse of every diagonal block; Gershgorin bound g_l of
//            ρ(D_l⁻¹ A_l); smoother weight ω_l = 4 / (3 ρ̂_l), ρ̂_l = max(2, g_l / 1.45)
//   P_l      (I − ω_l D_l⁻¹ A_l) P_tent, P_tent = aggregate indicator ⊗ I
//   A_{l+1}  P_lᵀ (A_l P_l), both products as fixed-order gathers
// Every producer also writes an f32 copy (A_l, D_l⁻¹, P_l, R_l = P_lᵀ) for
// the V-cycle.
//
// Why ρ̂ = max(2, g/1.45): on level 0, A = Σ_e A_e + reg·I with every element
// matrix A_e = [[S,−S],[−S,S]] ≤ 2·blockdiag(A_e), so ρ(D⁻¹A) ≤ 2 exactly; on
// the coarse levels the measured ρ stays ≈ 2 while the
// Gershgorin bound is ≈ 2.7.  ω_l·λ ≤ (4/3)·g/ρ̂ ≤ (4/3)·1.45 < 2 for every
// eigenvalue λ ≤ g, so the damped block-Jacobi smoother converges in the A
// norm on every level and the V-cycle is symmetric positive definite — the
// requirement for CG — while ω takes the sharp value 2/3 whenever g < 2.9.
//
// Below level 0 the engine by default replaces ρ̂ by 1.75 (omega[0], capi.hip
// opt_amg_coarse_rho_ppm): the measured λ of the Galerkin levels is ≤ 2.0, so
// the over-relaxed ω = 0.76 keeps ω·λ ≈ 1.5 — measured, not proven; a solve
// that fails with it falls back to the rule above.
//
// V-cycle (one per PCG iteration, pre- and post-smoothing by one damped
// block-Jacobi sweep each, exact block-diagonal solve on the coarsest level),
// in f32 (values and vectors; the CG around it stays f64 — a preconditioner
// only has to be a fixed SPD operator: measured, the f32 cycle gives the same
// iteration counts to 1e-8 and to 1e-13 as the f64 one):
//   x_l = ω D⁻¹ b_l                      (fused into the kernel producing b_l)
//   t_l = b_l − A_l x_l                  k_amg_resid
//   b_{l+1} = P_lᵀ t_l, x_{l+1} = ω D⁻¹ b_{l+1}   k_amg_restrict
//   ... recursion ...
//   x_l += P_l e_{l+1}                   k_amg_prolong
//   e_l = x_l + ω D⁻¹ (b_l − A_l x_l)    k_amg_post
// Level 0 reads the CG's f64 residual r as b_0 and writes the CG's f64 u as e_0.
// CG: the single-reduction (Chronopoulos–Gear) recurrences of cg.hip with
// u = M r the V-cycle output: per iteration one update kernel (reads the
// previous partials, forms α, β, the stopping test), the V-cycle, and one
// w = A_0 u kernel (f64 A_0) that writes the next partials (γ, δ, ‖r‖², ‖u‖²).
#include "amg_dev.hpp"

namespace mfea {

// The numeric setup's block index.  x1 (levels of a few thousand rows,
// AmgLevD::x1): the launch has 8× the blocks and only those dealt to XCD 0 work
// (blocks are dealt round-robin over the 8 XCDs) — a small level's chain of
// launches then reads what the previous launch wrote from the same L2 instead
// of another XCD's.  Speed only; −1: this block has no work.
__device__ __forceinline__ int64_t setup_block(int x1, int64_t nmain = -1) {
  if (!x1) return nmain < 0 ? xcd_block() : xcd_block_n(nmain);  // (nmain: the launch's own blocks come first)
  return (blockIdx.x & 7) ? -1 : (int64_t)(blockIdx.x >> 3);
}


// ---------------------------------------------------------------------------
// numeric setup (f64, with f32 copies for the V-cycle)
// ---------------------------------------------------------------------------
// Block-Jacobi inverse and Gershgorin bound per block of a coarse level
// (level 0's are formed with its blocks, k_amg_a0dinv).
template <int ND>
__device__ __forceinline__ double dinv_row(const AmgLevD& L, int64_t i) {
  const AmgMatD& A = L.A;
  double g = 0.0;
  if (i - (threadIdx.x & 63) < A.rg.hi) {
    int64_t base;
    int w;
    slice_of(A, i, base, w);
    if (i >= A.rg.lo && i < A.rg.hi) {
      double D[ND * ND], Di[ND * ND];
      bload<ND>(A.val32, A.npos, base, D);
      binv<ND>(D, Di);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) L.dinv32[i * (ND * ND) + c] = (float)Di[c];
      double rs[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a) rs[a] = 0.0;
      for (int k = 0; k < w; ++k) {
        const int64_t q = base + (int64_t)k * 64;
        if (A.col[q] < 0) continue;
        double m[ND * ND], pm[ND * ND];
        if (k == 0) {
#pragma unroll
          for (int c = 0; c < ND * ND; ++c) m[c] = D[c];
        } else {
          bload<ND>(A.val32, A.npos, q, m);
        }
#pragma unroll
        for (int c = 0; c < ND * ND; ++c) pm[c] = 0.0;
        mm_acc<ND>(Di, m, pm);
#pragma unroll
        for (int a = 0; a < ND; ++a)
#pragma unroll
          for (int b = 0; b < ND; ++b) rs[a] += fabs(pm[a * ND + b]);
      }
#pragma unroll
      for (int a = 0; a < ND; ++a) g = fmax(g, rs[a]);
    }
  }
  return g;
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_dinv(AmgLevD L) {
  __shared__ double red[kBlock / 64];
  const int64_t xb = setup_block(L.x1);
  if (xb < 0) return;
  double g = dinv_row<ND>(L, L.A.rg.lo64() + xb * kBlock + threadIdx.x);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) g = fmax(g, __shfl_xor(g, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = g;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = red[0];
    for (int k = 1; k < kBlock / 64; ++k) m = fmax(m, red[k]);
    // the level's bound g = max over blocks: a max is order-free, so one
    // atomic per block gives the same bits as any reduction (m ≥ 0, so its
    // IEEE bits order as unsigned integers); zeroed by the kernel producing
    // this level's A (k_amg_ac / k_amg_fuse_ac)
    atomicMax(reinterpret_cast<unsigned long long*>(&L.omega[1]),
              static_cast<unsigned long long>(__double_as_longlong(m)));
  }
}

// Level 0's off-diagonal blocks of a row, slots k0 … k0+U−1 (A_ij = Σ of the
// listed SELL slots' K_ij, list order), each handed to blk(q, m): the lists'
// bounds, their first entries and those entries' values are each issued for
// the U slots together — three dependent round trips per batch, where a slot
// by slot walk took two per slot.  A list's further entries (two nodes joined
// by more than one element) are walked after.  Padding and slots past the row
// (empty lists) load what slot k0 / list entry 0 hold and are skipped.
template <int ND, int U, class Blk>
__device__ __forceinline__ void a0_slots(const SellOp& sop, const int32_t* __restrict__ ptr,
                                         const int32_t* __restrict__ lst, int64_t base, int k0, int w,
                                         Blk&& blk) {
  int32_t t0[U], t1[U], g[U];
  int64_t q[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = base + (int64_t)(k0 + u < w ? k0 + u : k0) * 64;
    t0[u] = ptr[q[u]];
    t1[u] = ptr[q[u] + 1];
  }
  bool ok[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    ok[u] = k0 + u < w && t0[u] < t1[u];
    g[u] = lst[ok[u] ? t0[u] : 0];
  }
  double v6[U][6];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int c = 0; c < 6; ++c) v6[u][c] = sop.val[(int64_t)c * sop.G + g[u]];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    double m[ND * ND], e[ND * ND];
    sym_to<ND>(v6[u], e);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) m[c] = 0.0 + e[c];
    for (int t = t0[u] + 1; t < t1[u]; ++t) {
      double w6[6];
      const int64_t gs = lst[t];
#pragma unroll
      for (int c = 0; c < 6; ++c) w6[c] = sop.val[(int64_t)c * sop.G + gs];
      sym_to<ND>(w6, e);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) m[c] += e[c];
    }
    blk(q[u], m);
  }
}

// Level 0 in one row-wise pass (one launch where a0 and a level-0 D⁻¹ were two):
// per row i, the diagonal K_ii + reg·I from the assembled diagonal, its exact
// inverse, every off-diagonal block (Σ of the listed SELL slots' K_ij = −S_e,
// slot order) stored as A_0's f64 symmetric / f32 blocks, and the Gershgorin
// row sums of |D⁻¹ A_ij| accumulated from the blocks in registers — A_0 is
// written once and never read back here.  omega0[1] must be zero before the
// launch (launch_amg_a0 clears it); the blocks' maxima meet by atomic max.
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_a0dinv(AmgLevD L, SellOp sop, const int32_t* __restrict__ row0,
                                                       const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ lst, double reg) {
  __shared__ double red[kBlock / 64];
  const AmgMatD& A = L.A;
  const int64_t i = A.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  double g = 0.0;
  if (i - (threadIdx.x & 63) < A.rg.hi) {
    int64_t base;
    int w;
    slice_of(A, i, base, w);
    if (i >= A.rg.lo && i < A.rg.hi) {
      double s6[6], D[ND * ND], Di[ND * ND];
#pragma unroll
      for (int c = 0; c < 6; ++c) s6[c] = sop.diag[(int64_t)c * sop.N + row0[i]];
      s6[0] += reg;
      s6[3] += reg;
      s6[5] += reg;
      sym_to<ND>(s6, D);
      bstore<ND>(A.val32, A.npos, base, D);
      bstore_sym<ND>(A.sym, A.npos, base, D);
      if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, base, D);  // the four-step cycle's level-0 blocks
      binv<ND>(D, Di);
      if (L.dinv) {  // f64 copy: a one-level hierarchy's exact block solve (k_amg_cg_init)
#pragma unroll
        for (int c = 0; c < ND * ND; ++c) L.dinv[i * (ND * ND) + c] = Di[c];
      }
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) L.dinv32[i * (ND * ND) + c] = (float)Di[c];
      double rs[ND];
      {
        double pm[ND * ND];
#pragma unroll
        for (int c = 0; c < ND * ND; ++c) pm[c] = 0.0;
        mm_acc<ND>(Di, D, pm);
#pragma unroll
        for (int a = 0; a < ND; ++a) {
          rs[a] = 0.0;
#pragma unroll
          for (int b = 0; b < ND; ++b) rs[a] += fabs(pm[a * ND + b]);
        }
      }
      for (int k0 = 1; k0 < w; k0 += 4)
        a0_slots<ND, 4>(sop, ptr, lst, base, k0, w, [&](int64_t q, const double* m) {
          bstore<ND>(A.val32, A.npos, q, m);
          bstore_sym<ND>(A.sym, A.npos, q, m);
          if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, q, m);
          double pm[ND * ND];
#pragma unroll
          for (int c = 0; c < ND * ND; ++c) pm[c] = 0.0;
          mm_acc<ND>(Di, m, pm);
#pragma unroll
          for (int a = 0; a < ND; ++a)
#pragma unroll
            for (int b = 0; b < ND; ++b) rs[a] += fabs(pm[a * ND + b]);
        });
#pragma unroll
      for (int a = 0; a < ND; ++a) g = fmax(g, rs[a]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) g = fmax(g, __shfl_xor(g, off, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = g;
  __syncthreads();
  if (threadIdx.x == 0 && !L.fixed_omega) {
    double mx = red[0];
    for (int k = 1; k < kBlock / 64; ++k) mx = fmax(mx, red[k]);
    atomicMax(reinterpret_cast<unsigned long long*>(&L.omega[1]),
              static_cast<unsigned long long>(__double_as_longlong(mx)));
  }
}

// Level 0 at a fixed ω without the P / Ã part (k_amg_a0full): no Gershgorin
// bound to gather per row, so one thread per SELL position (slot_wave) — a
// row's blocks are formed side by side, three dependent round trips (list
// bounds, list entry, values) for every block where k_amg_a0dinv's row
// thread walked its slots four at a time.  Slot 0 (the diagonal, wave-
// uniform) also writes the row's D⁻¹.  The blocks and D⁻¹ are k_amg_a0dinv's
// bit for bit.
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_a0slot(AmgLevD L, SellOp sop, const int32_t* __restrict__ row0,
                                                       const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ lst, double reg) {
  const AmgMatD& A = L.A;
  int64_t q, i;
  int k;
  if (!slot_wave(A, A.rg.p0 / 64, A.rg.p1 / 64, q, i, k, xcd_block()) || i >= A.n) return;
  if (i < A.rg.lo || i >= A.rg.hi) return;
  if (k == 0) {
    double s6[6], D[ND * ND], Di[ND * ND];
    const int64_t r = row0[i];
#pragma unroll
    for (int c = 0; c < 6; ++c) s6[c] = sop.diag[(int64_t)c * sop.N + r];
    s6[0] += reg;
    s6[3] += reg;
    s6[5] += reg;
    sym_to<ND>(s6, D);
    bstore<ND>(A.val32, A.npos, q, D);
    bstore_sym<ND>(A.sym, A.npos, q, D);
    if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, q, D);
    binv<ND>(D, Di);
    if (L.dinv) {
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) L.dinv[i * (ND * ND) + c] = Di[c];
    }
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) L.dinv32[i * (ND * ND) + c] = (float)Di[c];
    return;
  }
  const int t0 = ptr[q], t1 = ptr[q + 1];
  if (t0 == t1) return;  // padding
  double m[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) m[c] = 0.0;
  for (int t = t0; t < t1; ++t) {
    double v6[6], e[ND * ND];
    const int64_t gs = lst[t];
#pragma unroll
    for (int c = 0; c < 6; ++c) v6[c] = sop.val[(int64_t)c * sop.G + gs];
    sym_to<ND>(v6, e);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) m[c] += e[c];
  }
  bstore<ND>(A.val32, A.npos, q, m);
  bstore_sym<ND>(A.sym, A.npos, q, m);
  if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, q, m);
}

// Level 0 at a fixed ω (AmgLevD::fixed_omega: ρ̂_0 = 2, the exact level-0
// bound): k_amg_a0dinv's row pass without the Gershgorin bound, plus — from
// the same row's blocks — the compact cycle's Ã_0 = ω D⁻¹ A_0 and the row's
// P_0 values, the work k_amg_fuse_p does for level 0 (the fused setup then
// skips that launch).  Ã and P from the stored f32 blocks and D⁻¹, as
// atv_body / pvals_body form them: the same bits.  P reads back A_0 blocks
// this thread stored (its own row: program order).
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_a0full(AmgLevD L, SellOp sop, const int32_t* __restrict__ row0,
                                                       const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ lst, double reg) {
  const AmgMatD& A = L.A;
  const int64_t i = A.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  if (i - (threadIdx.x & 63) >= A.rg.hi) return;
  int64_t base;
  int w;
  slice_of(A, i, base, w);
  if (i < A.rg.lo || i >= A.rg.hi) return;
  const double om = amg_omega(L.omega);
  double s6[6], D[ND * ND], Di[ND * ND], Dq[ND * ND];
#pragma unroll
  for (int c = 0; c < 6; ++c) s6[c] = sop.diag[(int64_t)c * sop.N + row0[i]];
  s6[0] += reg;
  s6[3] += reg;
  s6[5] += reg;
  sym_to<ND>(s6, D);
  bstore<ND>(A.val32, A.npos, base, D);
  bstore_sym<ND>(A.sym, A.npos, base, D);
  if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, base, D);
  binv<ND>(D, Di);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) {
    L.dinv32[i * (ND * ND) + c] = (float)Di[c];
    Dq[c] = (double)(float)Di[c];  // the f32 D⁻¹ the separate kernels read
  }
  auto at_store = [&](int64_t q, const double* m) {  // Ã = ω D⁻¹ A from the f32 block
    double mf[ND * ND], o[ND * ND];
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) {
      mf[c] = (double)(float)m[c];
      o[c] = 0.0;
    }
    mm_acc<ND>(Dq, mf, o);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) o[c] *= om;
    bstore<ND>(A.at32, 0, q, o);
  };
  if (A.at32) at_store(base, D);
  for (int k0 = 1; k0 < w; k0 += 4)
    a0_slots<ND, 4>(sop, ptr, lst, base, k0, w, [&](int64_t q, const double* m) {
      bstore<ND>(A.val32, A.npos, q, m);
      bstore_sym<ND>(A.sym, A.npos, q, m);
      if (!L.compact) bstore_sym<ND>(A.sym32, A.npos, q, m);
      if (A.at32) at_store(q, m);
    });
  const AmgMatD& P = L.P;
  if (L.coarsest || P.wmax <= 0 || i < P.rg.lo || i >= P.rg.hi) return;
  int64_t pb;
  int pw;
  slice_of(P, i, pb, pw);
  const int32_t ai = L.agg[i];
  const bool floating = L.fmask && L.fmask[i];
  for (int k = 0; k < pw; ++k) {
    const int64_t q = pb + (int64_t)k * 64;
    const int32_t J = P.col[q];
    if (J < 0) continue;
    double S[ND * ND], pm[ND * ND];
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) S[c] = pm[c] = 0.0;
    list_sum<ND>(L.pv_ptr[q], L.pv_ptr[q + 1], L.pv_a, A.val32, A.npos, S);
    mm_acc<ND>(Dq, S, pm);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) pm[c] = -om * pm[c];
    if (J == ai) {
#pragma unroll
      for (int a = 0; a < ND; ++a) pm[a * ND + a] += 1.0;
    }
    if (floating) {
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) pm[c] = 0.0;
    }
    bstore<ND>(P.val32, P.npos, q, pm);
  }
}

// P values, one thread per position (slot_wave): every slot of a row in
// flight at once instead of one after another.
template <int ND>
__device__ __forceinline__ void pvals_body(const AmgLevD& L, int64_t blk) {
  const AmgMatD& P = L.P;
  int64_t q, i;
  int k;
  if (!slot_wave(P, P.rg.p0 / 64, P.rg.p1 / 64, q, i, k, blk)) return;
  if (i < P.rg.lo || i >= P.rg.hi) return;
  // the list bounds, D⁻¹ and the row's aggregate / floating flag need no
  // column: issued with it (one round trip fewer ahead of the list's gathers,
  // none after them)
  const int32_t J = P.col[q];
  const int t0 = L.pv_ptr[q], t1 = L.pv_ptr[q + 1];
  const int32_t ai = L.agg[i];
  const bool floating = L.fmask && L.fmask[i];
  double S[ND * ND], pm[ND * ND], Di[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) {
    S[c] = 0.0;
    pm[c] = 0.0;
    Di[c] = L.dinv32[i * (ND * ND) + c];
  }
  if (J < 0) return;
  list_sum<ND>(t0, t1, L.pv_a, L.A.val32, L.A.npos, S);
  mm_acc<ND>(Di, S, pm);
  const double om = amg_omega(L.omega);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) pm[c] = -om * pm[c];
  if (J == ai) {
#pragma unroll
    for (int a = 0; a < ND; ++a) pm[a * ND + a] += 1.0;
  }
  if (floating) {  // a floating row: no coarse correction reaches it
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) pm[c] = 0.0;
  }
  bstore<ND>(P.val32, P.npos, q, pm);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_pvals(AmgLevD L) {
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) pvals_body<ND>(L, xb);
}

// One output block per thread (every SELL position of the product; pads
// have empty lists): AP(i, J) = Σ A[a]·P[b].  The same grid writes R = Pᵀ.
// PTV: also the compact cycle's P̃(i, J) = P(i, J) − ω D_i⁻¹ AP(i, J) — P̃ has
// A·P's layout position for position (amg_symbolic.cpp), so it is formed from
// the block in registers; its operands are loaded before the pair sum.
template <int ND, bool PTV>
__device__ __forceinline__ void ap_body(const AmgLevD& L, int64_t blk) {
  const int64_t k = blk * kBlock + threadIdx.x;
  const int64_t qr = L.R.rg.p0 + k;
  // R = Pᵀ (f32) in R's own SELL layout: the four-step cycle's restriction
  // (the compact cycle restricts with R̂)
  if (!L.compact && qr < L.R.rg.p1 && L.R.col[qr] >= 0 && pos_mine(L.R.rg, qr)) {
    double p[ND * ND], t[ND * ND];
    bload<ND>(L.P.val32, L.P.npos, L.rp[qr], p);
#pragma unroll
    for (int a = 0; a < ND; ++a)
#pragma unroll
      for (int b = 0; b < ND; ++b) t[a * ND + b] = p[b * ND + a];
    bstore<ND>(L.R.val32, L.R.npos, qr, t);
  }
  const int64_t q = L.AP.rg.p0 + k;
  if (q >= L.AP.rg.p1) return;
  // the column (padding test), the list bounds and P̃'s operand indices in
  // one round trip
  const int32_t jc = L.AP.col[q];
  const int t0 = L.ap_ptr[q], t1 = L.ap_ptr[q + 1];
  int32_t qp = -1;
  int64_t r = 0;
  if constexpr (PTV) {
    qp = L.pt_p[q];
    r = 64 * (int64_t)L.PT.srow[q >> 6] + (q & 63);  // the A·P / P̃ row
  }
  if (jc < 0 || !pos_mine(L.AP.rg, q)) return;
  double C[ND * ND], Di[ND * ND], pm[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) C[c] = pm[c] = 0.0;
  if constexpr (PTV) {
    dinv_load<ND>(L.dinv32, L.pt_row[r], Di);
    // (unconditional load, masked: a guarded one made codegen branch and wait)
    bload<ND>(L.P.val32, 0, qp >= 0 ? qp : 0, pm);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) pm[c] = keep_or_zero(pm[c], qp >= 0);
  }
  pair_sum<ND, false>(t0, t1, L.ap_a, L.ap_b, L.A.val32, L.A.npos, L.P.val32, L.P.npos, C);
  bstore<ND>(L.apval, L.AP.npos, q, C);
  if constexpr (PTV) {
    // from the stored (f32) A·P block, as k_amg_ptv forms it: the same bits
    double m[ND * ND], Cs[ND * ND];
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) {
      m[c] = 0.0;
      Cs[c] = (double)(float)C[c];
    }
    mm_acc<ND>(Di, Cs, m);
    const double om = amg_omega(L.omega);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) pm[c] = fma(-om, m[c], pm[c]);
    bstore<ND>(L.PT.val32, 0, q, pm);
  }
}
template <int ND, bool PTV = false>
__global__ __launch_bounds__(kBlock) void k_amg_ap(AmgLevD L) {
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) ap_body<ND, PTV>(L, xb);
}

// The compact cycle's transfers (amg.hpp AmgLevel::PT), after A·P:
// P̃(i, J) = P(i, J) − ω D_i⁻¹ (A·P)(i, J) on A·P's pattern (f64, stored f32),
// one thread per (row, slot) as k_amg_pvals
template <int ND>
__device__ __forceinline__ void ptv_body(const AmgLevD& L, int64_t blk) {
  const AmgMatD& T = L.PT;
  int64_t q, i;
  int k;
  if (!slot_wave(T, T.rg.p0 / 64, T.rg.p1 / 64, q, i, k, blk) || i >= T.n) return;
  const int32_t jc = T.col[q];  // (with the operands' indices: one round trip)
  const int32_t qp = L.pt_p[q], qa = L.pt_ap[q], ir = L.pt_row[i];
  if (jc < 0 || !pos_mine(T.rg, q)) return;
  double Di[ND * ND], ap[ND * ND], pm[ND * ND], m[ND * ND];
  dinv_load<ND>(L.dinv32, ir, Di);
  bload<ND>(L.apval, 0, qa, ap);
  bload<ND>(L.P.val32, 0, qp >= 0 ? qp : 0, pm);  // (unconditional, masked)
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) pm[c] = keep_or_zero(pm[c], qp >= 0);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) m[c] = 0.0;
  mm_acc<ND>(Di, ap, m);
  const double om = amg_omega(L.omega);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) pm[c] = fma(-om, m[c], pm[c]);
  bstore<ND>(T.val32, 0, q, pm);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_ptv(AmgLevD L) {
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) ptv_body<ND>(L, xb);
}
// R̂ = s' D'_J⁻¹ P̃ᵀ D_i / ω in RT's own SELL layout, one thread per (row J,
// slot) as k_amg_pvals: the scalings of x = ω D⁻¹ b on both sides folded in,
// so the down sweep maps x_l to x_{l+1} directly (D_i: A's diagonal block,
// slot 0 of row i)
template <int ND>
__device__ __forceinline__ void rtv_body(const AmgLevD& L, const AmgLevD& N, int64_t blk) {
  const AmgMatD& T = L.RT;
  int64_t q, J;
  int k;
  if (!slot_wave(T, T.rg.p0 / 64, T.rg.p1 / 64, q, J, k, blk) || J >= T.n || !pos_mine(T.rg, q)) return;
  const int32_t i = T.col[q];
  const int32_t qt = L.rt_pt[q], jr = L.rt_row[J];  // (with the column: one round trip)
  if (i < 0) return;
  double p[ND * ND], Dn[ND * ND], D[ND * ND], t[ND * ND], u[ND * ND], o[ND * ND];
  bload<ND>(L.PT.val32, 0, qt, p);
  dinv_load<ND>(N.dinv32, jr, Dn);
  bload<ND>(L.A.val32, 0, (int64_t)L.A.sptr[i >> 6] * 64 + (i & 63), D);
  const double sc = (N.coarsest ? 1.0 : amg_omega(N.omega)) / amg_omega(L.omega);
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int c = 0; c < ND; ++c) t[a * ND + c] = p[c * ND + a];  // P̃ᵀ block
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) u[c] = o[c] = 0.0;
  mm_acc<ND>(Dn, t, u);
  mm_acc<ND>(u, D, o);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) o[c] *= sc;
  bstore<ND>(T.val32, 0, q, o);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_rtv(AmgLevD L, AmgLevD N) {
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) rtv_body<ND>(L, N, xb);
}
// Ã = ω D_i⁻¹ A_ij (compact cycle), one thread per (row, slot)
template <int ND>
__device__ __forceinline__ void atv_body(const AmgLevD& L, int64_t blk) {
  const AmgMatD& A = L.A;
  int64_t q, i;
  int k;
  if (!slot_wave(A, A.rg.p0 / 64, A.rg.p1 / 64, q, i, k, blk) || i >= A.n) return;
  double Di[ND * ND], m[ND * ND], o[ND * ND];
  const int32_t jc = A.col[q];  // (the operands need no column: one round trip)
  dinv_load<ND>(L.dinv32, i, Di);
  bload<ND>(A.val32, 0, q, m);
  if (jc < 0 || !pos_mine(A.rg, q)) return;
  const double om = amg_omega(L.omega);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) o[c] = 0.0;
  mm_acc<ND>(Di, m, o);
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) o[c] *= om;
  bstore<ND>(A.at32, 0, q, o);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_atv(AmgLevD L) {
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) atv_body<ND>(L, xb);
}

// the collapsed cycle (amg_collapse.cpp): T = V_{l+1} R̂ (a < 0: the
// identity, V_coarsest) and V = 2I·[diag] − Ã + Σ P̃·T, one output block per
// thread, f32 blocks summed in list order (fixed: bitwise reproducible)
template <int ND>
__device__ __forceinline__ void fmm_acc(const float* A, const float* B, float* C) {
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      float s = C[a * ND + b];
#pragma unroll
      for (int k = 0; k < ND; ++k) s = fmaf(A[a * ND + k], B[k * ND + b], s);
      C[a * ND + b] = s;
    }
}
template <int ND>
__device__ __forceinline__ void tv_body(const AmgLevD& L, const float* __restrict__ vnext, int64_t blk) {
  const int64_t q = blk * kBlock + threadIdx.x;
  if (q >= L.CT.npos) return;
  const int32_t jc = L.CT.col[q];
  const int t0 = L.ct_ptr[q], t1 = L.ct_ptr[q + 1];  // (with the column: one round trip)
  if (jc < 0) return;
  float C[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) C[c] = 0.0f;
  constexpr int U = 4;  // items in flight (list order kept: the same sums)
  for (int t = t0; t < t1; t += U) {
    int32_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u < t1 ? t + u : t;
      a[u] = L.ct_a[tt];
      b[u] = L.ct_b[tt];
    }
    float r[U][ND * ND], v[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bload<ND>(L.RT.val32, 0, b[u], r[u]);
      bload<ND>(vnext ? vnext : L.RT.val32, 0, a[u] >= 0 ? a[u] : 0, v[u]);  // (no V below: a < 0, a dummy read)
    }
    // unconditional sums (guarded ones let codegen sink each item's loads into
    // its branch: one item's round trips after another): past the list r = 0,
    // and a < 0 (R̂'s block alone) multiplies by the identity — exact, the
    // same sums
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) {
        r[u][c] = keep_or_zero(r[u][c], t + u < t1);
        v[u][c] = keep_or_zero(v[u][c], a[u] >= 0) + (a[u] < 0 && c % (ND + 1) == 0 ? 1.0f : 0.0f);
      }
      fmm_acc<ND>(v[u], r[u], C);
    }
  }
  bstore<ND>(L.CT.val32, 0, q, C);
}
template <int ND>
__device__ __forceinline__ void vv_body(const AmgLevD& L, int64_t blk) {
  const int64_t q = blk * kBlock + threadIdx.x;
  if (q >= L.CV.npos) return;
  // the column, the list bounds and the extra term's index in one round trip
  const int32_t jc = L.CV.col[q];
  const int t0 = L.cv_ptr[q], t1 = L.cv_ptr[q + 1];
  const int32_t ea = L.cv_ext[q];
  const int32_t dg = L.cv_diag[q];
  if (jc < 0) return;
  float C[ND * ND];
  bload<ND>(L.A.at32, 0, ea >= 0 ? ea : 0, C);  // (unconditional, masked)
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) C[c] = keep_or_zero(-C[c], ea >= 0);
  if (dg) {
#pragma unroll
    for (int a = 0; a < ND; ++a) C[a * ND + a] += 2.0f;
  }
  constexpr int U = 4;  // items in flight (list order kept: the same sums)
  for (int t = t0; t < t1; t += U) {
    int32_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u < t1 ? t + u : t;
      a[u] = L.cv_a[tt];
      b[u] = L.cv_b[tt];
    }
    float p[U][ND * ND], tb[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bload<ND>(L.PT.val32, 0, a[u], p[u]);
      bload<ND>(L.CT.val32, 0, b[u], tb[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (past the list: exact zeros, as tv_body)
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) p[u][c] = keep_or_zero(p[u][c], t + u < t1);
      fmm_acc<ND>(p[u], tb[u], C);
    }
  }
  bstore<ND>(L.CV.val32, 0, q, C);
}

// the merged levels' operators (AmgMergeD), one output block per thread, f32
// in list order (bitwise reproducible): DQ's c_1 rows 2 R̂_0 − Σ Ã_1·R̂_0, its
// x_2 rows Σ R̂_1·R̂_0; U = P̃_0 (ext) + Σ P̃_0·P̃_1
// (xb: the block of the products' own numbering — DQ's blocks, then U's)
template <int ND>
__device__ __forceinline__ void mprod_body(const AmgMergeD& m, const float* __restrict__ at1,
                                           const float* __restrict__ r0, const float* __restrict__ r1,
                                           const float* __restrict__ p0, const float* __restrict__ p1,
                                           int64_t gdq, int64_t xb) {
  const bool dq = xb < gdq;
  const AmgMatD& M = dq ? m.DQ : m.U;
  const int64_t q = (dq ? xb : xb - gdq) * kBlock + threadIdx.x;
  if (q >= M.npos) return;
  const bool c1 = dq && q < m.dq_split;
  const int32_t* ext = dq ? m.dq_ext : m.u_ext;
  const int32_t* lp = dq ? m.dq_ptr : m.u_ptr;
  const int32_t* la = dq ? m.dq_a : m.u_a;
  const int32_t* lb = dq ? m.dq_b : m.u_b;
  const int32_t jc = M.col[q];
  const int t0 = lp[q], t1 = lp[q + 1];  // (with the column: one round trip)
  const int32_t e = ext[q];
  if (jc < 0) return;
  const float* X = dq ? (c1 ? at1 : r1) : p0;
  const float* Y = dq ? r0 : p1;
  float S[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) S[c] = 0.0f;
  constexpr int U = 4;
  for (int t = t0; t < t1; t += U) {
    int32_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = t + u < t1 ? t + u : t;
      a[u] = la[tt];
      b[u] = lb[tt];
    }
    float x[U][ND * ND], y[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bload<ND>(X, 0, a[u], x[u]);
      bload<ND>(Y, 0, b[u], y[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (past the list: exact zeros, as tv_body)
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) x[u][c] = keep_or_zero(x[u][c], t + u < t1);
      fmm_acc<ND>(x[u], y[u], S);
    }
  }
  float C[ND * ND];
  bload<ND>(dq ? r0 : p0, 0, e >= 0 ? e : 0, C);  // (unconditional, masked)
  {
    const float f = dq ? 2.0f : 1.0f;
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) C[c] = keep_or_zero(C[c] * f, e >= 0);
  }
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) C[c] = c1 ? C[c] - S[c] : C[c] + S[c];
  bstore<ND>(M.val32, 0, q, C);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_mprod(AmgMergeD m, const float* __restrict__ at1,
                                                      const float* __restrict__ r0, const float* __restrict__ r1,
                                                      const float* __restrict__ p0, const float* __restrict__ p1,
                                                      int64_t gdq) {
  mprod_body<ND>(m, at1, r0, r1, p0, p1, gdq, xcd_block());
}
// Those products riding in a collapse launch (blocks from `nmain` on): their
// inputs are complete before the collapse starts, so they need no launch of
// their own.  All in the last one (V_kc's, the widest): C2 setup 0.211 →
// 0.205 ms; spread over the six collapse launches each took the products'
// own ≈ 11 µs chain — 0.226 ms
struct MprodSlice {
  AmgMergeD m;
  const float *at1 = nullptr, *r0 = nullptr, *r1 = nullptr, *p0 = nullptr, *p1 = nullptr;
  int64_t gdq = 0, b0 = 0, b1 = 0;
};
template <int ND>
__device__ __forceinline__ bool mprod_side(const MprodSlice& ms, int64_t nmain) {
  if ((int64_t)blockIdx.x < nmain) return false;
  const int64_t xb = ms.b0 + (int64_t)blockIdx.x - nmain;
  if (xb < ms.b1) mprod_body<ND>(ms.m, ms.at1, ms.r0, ms.r1, ms.p0, ms.p1, ms.gdq, xb);
  return true;
}
// the collapse's launches (blocks [0, nmain): the level's own work)
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_tv(AmgLevD L, const float* __restrict__ vnext, MprodSlice ms,
                                                   int64_t nmain) {
  if (mprod_side<ND>(ms, nmain)) return;
  const int64_t xb = setup_block(L.x1, nmain);
  if (xb >= 0) tv_body<ND>(L, vnext, xb);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_vv(AmgLevD L, MprodSlice ms, int64_t nmain) {
  if (mprod_side<ND>(ms, nmain)) return;
  const int64_t xb = setup_block(L.x1, nmain);
  if (xb >= 0) vv_body<ND>(L, xb);
}

// A_{l+1}(I, J) = Σ P[a]ᵀ·AP[b], S lanes per output block (AmgLevD::ac_lanes):
// the lists hold 5–40 pairs (C3 level 0 ≈ 30), and one lane walking them in
// steps of 8 chained four dependent index → block round trips; lane `sub`
// takes items sub, sub + S, … (a fixed order) and the S partial sums meet by
// a fixed butterfly — bitwise reproducible.  dinv_next (level l+1 at a fixed
// ω, AmgLevD::fixed_omega): the group of a diagonal block (slot 0 of its row)
// also stores its inverse — from the stored f32 block, the bits k_amg_dinv
// would form — so level l+1 needs no D⁻¹ launch.
template <int ND, int S>
__device__ __forceinline__ void ac_body(const AmgLevD& L, const AmgMatD& Ac, int64_t blk, float* dinv_next) {
  const int64_t t = blk * kBlock + threadIdx.x;
  const int64_t q = L.ac_rg.p0 + t / S;
  const int sub = (int)(t % S);
  // (the S lanes of a block share q: they leave together)
  if (q >= L.ac_rg.p1) return;
  const int32_t jc = Ac.col[q];
  const int t0 = L.ac_ptr[q], t1 = L.ac_ptr[q + 1];  // (with the column: one round trip)
  if (jc < 0 || !pos_mine(L.ac_rg, q)) return;
  double C[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) C[c] = 0.0;
  constexpr int U = 4;
  for (int k = t0 + sub; k < t1; k += U * S) {  // U of this lane's pairs in flight
    int32_t ia[U], ib[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = k + u * S < t1 ? k + u * S : k;
      ia[u] = L.ac_a[tt];
      ib[u] = L.ac_b[tt];
    }
    double x[U][ND * ND], y[U][ND * ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bload<ND>(L.P.val32, 0, ia[u], x[u]);
      bload<ND>(L.apval, 0, ib[u], y[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (past the list: exact zeros, as pair_sum_u)
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) x[u][c] = keep_or_zero(x[u][c], k + u * S < t1);
      mtm_acc<ND>(x[u], y[u], C);
    }
  }
  if constexpr (S > 1) {
#pragma unroll
    for (int o = 1; o < S; o <<= 1)
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) C[c] += __shfl_xor(C[c], o, 64);
  }
  if (sub != 0) return;
  bstore<ND>(Ac.val32, Ac.npos, q, C);
  if (dinv_next) {
    const int64_t ts = q >> 6;
    const int sl = Ac.srow[ts];
    if (ts == (int64_t)Ac.sptr[sl]) {  // slot 0: the diagonal block of row 64·sl + lane
      double D[ND * ND], Di[ND * ND];
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) D[c] = (double)(float)C[c];
      binv<ND>(D, Di);
      const int64_t row = 64 * (int64_t)sl + (q & 63);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) dinv_next[row * (ND * ND) + c] = (float)Di[c];
    }
  }
}
template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_ac(AmgLevD L, AmgMatD Ac, double* omega_next, float* dinv_next) {
  if (blockIdx.x == 0 && threadIdx.x == 0) omega_next[1] = 0.0;  // level l+1's bound, max'ed by its k_amg_dinv
  const int64_t xb = setup_block(L.x1);
  if (xb >= 0) ac_body<ND, S>(L, Ac, xb, dinv_next);
}
// launch helper: the grid of S lanes per output block
static int64_t ac_blocks(const AmgLevD& L) {
  const int64_t n = L.ac_rg.npos() * L.ac_lanes;
  return (n + kBlock - 1) / kBlock > 0 ? (n + kBlock - 1) / kBlock : 1;
}

// The compact cycle's operators fused into the Galerkin chain's launches (no
// launch of their own, no extra dependency): blocks [0, g0) run the chain
// kernel, the rest the compact parts whose inputs are complete by then —
// after level l's D⁻¹: P_l values, Ã_l and R̂_{l−1} (it needs D_l⁻¹, ω_l and
// P̃_{l−1}); after A_l·P_l: A_{l+1} and P̃_l.  Every part keeps its own
// XCD-contiguous share (sub-ranges of one xcd_block() numbering).
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_fuse_p(AmgLevD L, AmgLevD Lp, int64_t g0, int64_t g1) {
  const int64_t xb = setup_block(L.x1);
  if (xb < 0) return;
  if (xb < g0) pvals_body<ND>(L, xb);
  else if (xb < g1) atv_body<ND>(L, xb - g0);
  else rtv_body<ND>(Lp, L, xb - g1);
}
template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_fuse_ac(AmgLevD L, AmgMatD Ac, double* omega_next, int64_t g0,
                                                        float* dinv_next) {
  if (blockIdx.x == 0 && threadIdx.x == 0) omega_next[1] = 0.0;
  const int64_t xb = setup_block(L.x1);
  if (xb < 0) return;
  if (xb < g0) ac_body<ND, S>(L, Ac, xb, dinv_next);
  else ptv_body<ND>(L, xb - g0);
}
// the Galerkin product's launch (fuse: + P̃ from block g0 on) at its lanes
template <int ND>
static void launch_ac(hipStream_t s, const AmgLevD& L, const AmgMatD& Ac, double* omega_next, float* dnext,
                      int64_t blocks, int64_t g0, bool fuse) {
  const dim3 g(L.x1 ? 8 * (unsigned)blocks : (unsigned)blocks), b(kBlock);
#define MFEA_AC(S)                                                                                          \
  if (fuse) hipLaunchKernelGGL((k_amg_fuse_ac<ND, S>), g, b, 0, s, L, Ac, omega_next, g0, dnext); \
  else hipLaunchKernelGGL((k_amg_ac<ND, S>), g, b, 0, s, L, Ac, omega_next, dnext)
  switch (L.ac_lanes) {
    case 8: MFEA_AC(8); break;
    case 4: MFEA_AC(4); break;
    case 2: MFEA_AC(2); break;
    default: MFEA_AC(1); break;
  }
#undef MFEA_AC
}

// ---------------------------------------------------------------------------
// V-cycle (f32; level 0 reads r and writes u in f64)
// ---------------------------------------------------------------------------
// L0: level 0 — A_0's symmetric f32 blocks, 2U unroll for its narrow streaming
// rows; otherwise the full f32 blocks with the 4U tier (sell_mac's K)
template <int ND, class TB, bool L0>
__global__ __launch_bounds__(kBlock) void k_amg_resid(AmgLevD L, const TB* __restrict__ b,
                                                      const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t i = L.A.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  const int64_t n = L.A.rg.hi;
  const bool mine = i >= L.A.rg.lo && i < n;
  if (i - (threadIdx.x & 63) >= n) return;
  const int64_t ii = i < n ? i : n - 1;
  int64_t base;
  int w;
  slice_of(L.A, ii, base, w);
  float y[ND];
  vload<ND>(b, ii, y);
  if constexpr (L0)
    sell_mac<ND, true, 2, true>(L.A.col, L.A.sym32, L.A.npos, base, w, L.x, y);
  else
    sell_mac<ND, true, 3>(L.A.col, L.A.val32, L.A.npos, base, w, L.x, y);
  if (mine && run) vstore<ND>(L.t, i, y);
}

template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_restrict(AmgLevD L, AmgLevD N, const int32_t* gate) {
  const bool run = gate_open(gate);
  const AmgMatD& R = L.R;
  const int64_t I = R.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  const int64_t n = R.rg.hi;
  if (I - (threadIdx.x & 63) >= n) return;
  int64_t base;
  int w;
  slice_of(R, I, base, w);
  const float sc = N.coarsest ? 1.0f : (float)amg_omega(N.omega);
  float Di[ND * ND];
  dinv_load<ND>(N.dinv32, I < n ? I : n - 1, Di);
  float bc[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) bc[a] = 0.0f;
  sell_mac<ND, false, 3>(R.col, R.val32, R.npos, base, w, L.t, bc);  // R = Pᵀ blocks
  if (I < R.rg.lo || I >= n || !run) return;
  vstore<ND>(N.b, I, bc);
  float xn[ND];
  dinv_mul<ND>(Di, sc, bc, xn);
  vstore<ND>(N.x, I, xn);
}


template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_restrict_s(AmgLevD L, AmgLevD N, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t t = xcd_block() * kBlock + threadIdx.x;
  const AmgMatD& R = L.R;
  const int64_t I = R.rg.lo64() + t / S;
  const int sub = (int)(t % S);
  const int64_t n = R.rg.hi;
  if (I - (threadIdx.x & 63) / S >= n) return;  // whole wave past the end
  const int64_t Ic = I < n ? I : n - 1;
  int64_t base;
  int w;
  slice_of(R, Ic, base, w);
  const float sc = N.coarsest ? 1.0f : (float)amg_omega(N.omega);
  float Di[ND * ND], bc[ND];
  dinv_load<ND>(N.dinv32, Ic, Di);
#pragma unroll
  for (int a = 0; a < ND; ++a) bc[a] = 0.0f;
  sell_mac_sub<ND, S, false>(R.col, R.val32, base, w, sub, L.t, bc);
  if (I < R.rg.lo || I >= n || sub != 0 || !run) return;
  vstore<ND>(N.b, I, bc);
  float xn[ND];
  dinv_mul<ND>(Di, sc, bc, xn);
  vstore<ND>(N.x, I, xn);
}

// t = b − A x (f32 level ≥ 1) and e = x + ω D⁻¹ (b − A x) with S lanes per row
template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_resid_s(AmgLevD L, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t t = xcd_block() * kBlock + threadIdx.x;
  const int64_t n = L.A.rg.hi;
  const int64_t i = L.A.rg.lo64() + t / S;
  const int sub = (int)(t % S);
  if (i - (threadIdx.x & 63) / S >= n) return;
  const int64_t ii = i < n ? i : n - 1;
  int64_t base;
  int w;
  slice_of(L.A, ii, base, w);
  float y[ND];
  vload<ND>(L.b, ii, y);
  if (sub != 0) {
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0f;
  }
  sell_mac_sub<ND, S, true>(L.A.col, L.A.val32, base, w, sub, L.x, y);
  if (i >= L.A.rg.lo && i < n && sub == 0 && run) vstore<ND>(L.t, i, y);
}
template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_post_s(AmgLevD L, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t t = xcd_block() * kBlock + threadIdx.x;
  const int64_t n = L.A.rg.hi;
  const int64_t i = L.A.rg.lo64() + t / S;
  const int sub = (int)(t % S);
  if (i - (threadIdx.x & 63) / S >= n) return;
  const int64_t ii = i < n ? i : n - 1;
  int64_t base;
  int w;
  slice_of(L.A, ii, base, w);
  const float om = (float)amg_omega(L.omega);
  float y[ND], x[ND], d[ND], Di[ND * ND];
  vload<ND>(L.b, ii, y);
  vload<ND>(L.x, ii, x);
  dinv_load<ND>(L.dinv32, ii, Di);
  if (sub != 0) {
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0f;
  }
  sell_mac_sub<ND, S, true>(L.A.col, L.A.val32, base, w, sub, L.x, y);
  dinv_mul<ND>(Di, om, y, d);
#pragma unroll
  for (int a = 0; a < ND; ++a) x[a] += d[a];
  if (i >= L.A.rg.lo && i < n && sub == 0 && run) vstore<ND>(L.e, i, x);
}

template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_prolong(AmgLevD L, AmgLevD N, const int32_t* gate) {
  const bool run = gate_open(gate);
  const AmgMatD& P = L.P;
  const int64_t i = P.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  const int64_t n = P.rg.hi;
  if (i - (threadIdx.x & 63) >= n) return;
  int64_t base;
  int w;
  slice_of(P, i, base, w);
  const int64_t ii = i < n ? i : n - 1;
  float x[ND];
  vload<ND>(L.x, ii, x);
  sell_mac<ND, false>(P.col, P.val32, P.npos, base, w, N.coarsest ? N.x : N.e, x);
  if (i >= P.rg.lo && i < n && run) vstore<ND>(L.x, i, x);
}

template <int ND, class TB, class TE, bool L0>
__global__ __launch_bounds__(kBlock) void k_amg_post(AmgLevD L, const TB* __restrict__ b, TE* __restrict__ e,
                                                     const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t i = L.A.rg.lo64() + xcd_block() * kBlock + threadIdx.x;
  const int64_t n = L.A.rg.hi;
  const bool mine = i >= L.A.rg.lo && i < n;
  if (i - (threadIdx.x & 63) >= n) return;
  const int64_t ii = i < n ? i : n - 1;
  int64_t base;
  int w;
  slice_of(L.A, ii, base, w);
  const float om = (float)amg_omega(L.omega);
  float y[ND], x[ND], d[ND], Di[ND * ND];
  vload<ND>(b, ii, y);
  vload<ND>(L.x, ii, x);
  dinv_load<ND>(L.dinv32, ii, Di);
  if constexpr (L0)
    sell_mac<ND, true, 2, true>(L.A.col, L.A.sym32, L.A.npos, base, w, L.x, y);
  else
    sell_mac<ND, true, 3>(L.A.col, L.A.val32, L.A.npos, base, w, L.x, y);
  dinv_mul<ND>(Di, om, y, d);
#pragma unroll
  for (int a = 0; a < ND; ++a) x[a] += d[a];
  if (mine && run) vstore<ND>(e, i, x);
}

// ---------------------------------------------------------------------------
// The compact cycle (amg.hpp AmgLevel::PT): two sweeps per level, on the
// level's smoothed iterate x_l = s D⁻¹ b_l alone (b is never formed).
// Down: blocks [0, gc) form the next level's x_{l+1} = R̂ x_l (S lanes per
// coarse row), blocks from gc on the smoothed part c_l = 2 x_l − Ã x_l
// (= x + ω D⁻¹ (b − A x)), kept in t_l.  Both read only x_l.
template <int ND, int S, int KF = 2>
__global__ __launch_bounds__(kBlock) void k_amg_down(AmgLevD L, AmgLevD N, int64_t gc, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t xb = xcd_block();
  // (rows [rg.lo, rg.hi) of each row set: a distributed level's own rows,
  // swept from the slice boundary below lo; one partition: all of them)
  if (xb < gc) {
    const AmgMatD& R = L.RT;
    const int64_t t = xb * kBlock + threadIdx.x;
    const int64_t n = R.rg.hi;
    const int64_t I = R.rg.lo64() + t / S;
    const int sub = (int)(t % S);
    if (I - (threadIdx.x & 63) / S >= n) return;
    const int64_t Ic = I < n ? I : n - 1;
    int64_t base;
    int w;
    slice_of(R, Ic, base, w);
    float xc[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) xc[a] = 0.0f;
    if constexpr (S == 1) sell_mac<ND, false, 3>(R.col, R.val32, R.npos, base, w, L.x, xc);
    else sell_mac_sub<ND, S, false>(R.col, R.val32, base, w, sub, L.x, xc);
    if (I < n && I >= R.rg.lo && sub == 0 && run) vstore<ND>(N.x, L.rt_row[I], xc);
  } else {
    const int64_t i = L.A.rg.lo64() + (xb - gc) * kBlock + threadIdx.x;
    const int64_t n = L.A.rg.hi;
    if (i - (threadIdx.x & 63) >= n) return;
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    slice_of(L.A, ii, base, w);
    float x[ND], y[ND];
    vload<ND>(L.x, ii, x);
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = x[a] + x[a];
    sell_mac<ND, true, KF>(L.A.col, L.A.at32, L.A.npos, base, w, L.x, y);
    if (i < n && i >= L.A.rg.lo && run) vstore<ND>(L.t, i, y);
  }
}

// Up: e_l = c_l + P̃ e_{l+1} (the coarsest level's output is its x), S lanes
// per row; level 0 writes the CG's u.  P̃'s rows run in A·P's order: row a is
// the level's row pt_row[a] (c gathered, e scattered — within 4096-row windows)
template <int ND, int S, class TE>
__global__ __launch_bounds__(kBlock) void k_amg_up(AmgLevD L, AmgLevD N, TE* __restrict__ e, const int32_t* gate) {
  const bool run = gate_open(gate);
  const AmgMatD& T = L.PT;
  const int64_t t = xcd_block() * kBlock + threadIdx.x;
  const int64_t n = T.rg.hi;  // rows [rg.lo, rg.hi): a distributed level's own P̃ rows
  const int64_t a = T.rg.lo64() + t / S;
  const int sub = (int)(t % S);
  if (a - (threadIdx.x & 63) / S >= n) return;
  const int64_t aa = a < n ? a : n - 1;
  int64_t base;
  int w;
  slice_of(T, aa, base, w);
  const int64_t i = L.pt_row[aa];
  float y[ND];
  vload<ND>(L.t, i, y);
  if (sub != 0) {
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0f;
  }
  const float* src = N.coarsest ? N.x : N.e;
  if constexpr (S == 1) sell_mac<ND, false, 3>(T.col, T.val32, T.npos, base, w, src, y);
  else sell_mac_sub<ND, S, false>(T.col, T.val32, base, w, sub, src, y);
  if (a < n && a >= T.rg.lo && sub == 0 && run) vstore<ND>(e, i, y);
}

// The collapsed cycle below level kc: e_kc = V x_kc in one sweep (V's rows
// by length, vrow → the level's row), S lanes per row
template <int ND, int S>
__global__ __launch_bounds__(kBlock) void k_amg_vapply(AmgLevD L, const int32_t* gate) {
  const bool run = gate_open(gate);
  const AmgMatD& V = L.CV;
  const int64_t t = xcd_block() * kBlock + threadIdx.x;
  const int64_t n = V.n;
  const int64_t a = t / S;
  const int sub = (int)(t % S);
  if (a - (threadIdx.x & 63) / S >= n) return;
  const int64_t aa = a < n ? a : n - 1;
  int64_t base;
  int w;
  slice_of(V, aa, base, w);
  float y[ND];
#pragma unroll
  for (int c = 0; c < ND; ++c) y[c] = 0.0f;
  if constexpr (S == 1) sell_mac<ND, false, 3>(V.col, V.val32, V.npos, base, w, L.x, y);
  else sell_mac_sub<ND, S, false>(V.col, V.val32, base, w, sub, L.x, y);
  if (a < n && sub == 0 && run) vstore<ND>(L.e, L.cv_row[aa], y);
}

// ---------------------------------------------------------------------------
// The V-cycle below level l0 in ONE workgroup: resid / restrict down to the
// coarsest level, prolong / post back up to l0, the phases separated by
// workgroup barriers instead of kernel boundaries.  The deep levels hold a
// few thousand rows at most, so a full-grid launch per phase is ≈ 4.5 µs of
// latency for ≈ 0.1 µs of work; here a phase costs its rows' dependent loads
// (≈ rows/1024 × 3 hops) plus one barrier.  lev: device copy of the level
// views; levels ≥ l0 use f32 b and e.
// ---------------------------------------------------------------------------
constexpr int kTailBS = 1024;

// Phase bodies with the vectors passed explicitly (global memory for
// k_amg_tail, LDS for k_amg_tail_lds — the compiler then addresses each kind
// directly instead of through flat pointers); the operators come from L / N.
template <int ND>
__device__ __forceinline__ void tail_resid(const AmgLevD& L, const float* b, const float* x, float* t) {
  const int64_t n = L.A.n;
  for (int64_t r0 = 0; r0 < n; r0 += kTailBS) {
    const int64_t i = r0 + threadIdx.x;
    if (r0 + (threadIdx.x & ~63) >= n) break;  // whole wave past the end
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    slice_of(L.A, ii, base, w);
    float y[ND];
    vload<ND>(b, ii, y);
    sell_mac<ND, true>(L.A.col, L.A.val32, L.A.npos, base, w, x, y);
    if (i < n) vstore<ND>(t, i, y);
  }
}
template <int ND>
__device__ __forceinline__ void tail_restrict(const AmgLevD& L, const AmgLevD& N, const float* t, float* nb,
                                              float* nx) {
  const int64_t n = L.R.n;
  const float sc = N.coarsest ? 1.0f : (float)amg_omega(N.omega);
  for (int64_t r0 = 0; r0 < n; r0 += kTailBS) {
    const int64_t I = r0 + threadIdx.x;
    if (r0 + (threadIdx.x & ~63) >= n) break;
    int64_t base;
    int w;
    slice_of(L.R, I, base, w);
    float bc[ND], Di[ND * ND];
    dinv_load<ND>(N.dinv32, I < n ? I : n - 1, Di);
#pragma unroll
    for (int a = 0; a < ND; ++a) bc[a] = 0.0f;
    sell_mac<ND, false>(L.R.col, L.R.val32, L.R.npos, base, w, t, bc);
    if (I < n) {
      vstore<ND>(nb, I, bc);
      float xn[ND];
      dinv_mul<ND>(Di, sc, bc, xn);
      vstore<ND>(nx, I, xn);
    }
  }
}
template <int ND>
__device__ __forceinline__ void tail_prolong(const AmgLevD& L, const float* e, float* x) {
  const int64_t n = L.P.n;
  for (int64_t r0 = 0; r0 < n; r0 += kTailBS) {
    const int64_t i = r0 + threadIdx.x;
    if (r0 + (threadIdx.x & ~63) >= n) break;
    int64_t base;
    int w;
    slice_of(L.P, i, base, w);
    const int64_t ii = i < n ? i : n - 1;
    float xv[ND];
    vload<ND>(x, ii, xv);
    sell_mac<ND, false>(L.P.col, L.P.val32, L.P.npos, base, w, e, xv);
    if (i < n) vstore<ND>(x, i, xv);
  }
}
template <int ND>
__device__ __forceinline__ void tail_post(const AmgLevD& L, const float* b, const float* x, float* e_out) {
  const int64_t n = L.A.n;
  const float om = (float)amg_omega(L.omega);
  for (int64_t r0 = 0; r0 < n; r0 += kTailBS) {
    const int64_t i = r0 + threadIdx.x;
    if (r0 + (threadIdx.x & ~63) >= n) break;
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    slice_of(L.A, ii, base, w);
    float y[ND], xv[ND], d[ND], Di[ND * ND];
    vload<ND>(b, ii, y);
    vload<ND>(x, ii, xv);
    dinv_load<ND>(L.dinv32, ii, Di);
    sell_mac<ND, true>(L.A.col, L.A.val32, L.A.npos, base, w, x, y);
    dinv_mul<ND>(Di, om, y, d);
#pragma unroll
    for (int a = 0; a < ND; ++a) xv[a] += d[a];
    if (i < n) vstore<ND>(e_out, i, xv);
  }
}

// The tail's levels travel BY VALUE in the kernel arguments: pointers read
// from there are known to be global, while pointers read from a device array
// of level views made every access of the tail a flat one (no global/LDS
// distinction: each waits on both counters).
constexpr int kTailMaxLev = 4;
struct TailLevels {
  AmgLevD lev[kTailMaxLev];  // levels l0 … l0 + count − 1
};
template <int ND>
__global__ __launch_bounds__(kTailBS) void k_amg_tail(const TailLevels tl, int l0, int nlev,
                                                      const int32_t* gate) {
  if (gated(gate)) return;
  const AmgLevD* lev = tl.lev - l0;
  for (int l = l0; l + 1 < nlev; ++l) {
    const AmgLevD L = lev[l], N = lev[l + 1];
    tail_resid<ND>(L, L.b, L.x, L.t);
    __syncthreads();
    tail_restrict<ND>(L, N, L.t, N.b, N.x);
    __syncthreads();
  }
  for (int l = nlev - 2; l >= l0; --l) {
    const AmgLevD L = lev[l], N = lev[l + 1];
    tail_prolong<ND>(L, N.coarsest ? N.x : N.e, L.x);
    __syncthreads();
    tail_post<ND>(L, L.b, L.x, L.e);
    __syncthreads();
  }
}

// The same tail with the V-cycle vectors of its levels in LDS (b, x, t per
// level; a coarse level's output e lives in its t): every gather of a phase
// reads LDS instead of L2, and a barrier waits for LDS stores only.  Level
// l0's b, x are copied in from global memory first and its e is written
// there; the operators stay in global memory.  kTailLdsMax bytes at most
// (the launcher falls back to k_amg_tail beyond).
constexpr int64_t kTailLdsMax = 64 * 1024;
template <int ND>
__device__ __forceinline__ int64_t tail_lds_off(const AmgLevD* __restrict__ lev, int l, int l0) {
  int64_t off = 0;
  for (int m = l0; m < l; ++m) off += 3 * ND * lev[m].A.n;
  return off;
}
template <int ND>
__global__ __launch_bounds__(kTailBS) void k_amg_tail_lds(const TailLevels tl, int l0, int nlev,
                                                          const int32_t* gate) {
  extern __shared__ float sm[];
  if (gated(gate)) return;
  const AmgLevD* lev = tl.lev - l0;
  {
    const AmgLevD G = lev[l0];
    const int64_t n = G.A.n;
    for (int64_t k = threadIdx.x; k < ND * n; k += kTailBS) {
      sm[k] = G.b[k];
      sm[ND * n + k] = G.x[k];
    }
  }
  __syncthreads();
  for (int l = l0; l + 1 < nlev; ++l) {
    const AmgLevD L = lev[l], N = lev[l + 1];
    float* v = sm + tail_lds_off<ND>(lev, l, l0);  // b x t of level l
    float* w = v + 3 * ND * L.A.n;                 // of level l + 1
    tail_resid<ND>(L, v, v + ND * L.A.n, v + 2 * ND * L.A.n);
    __syncthreads();
    tail_restrict<ND>(L, N, v + 2 * ND * L.A.n, w, w + ND * N.A.n);
    __syncthreads();
  }
  for (int l = nlev - 2; l >= l0; --l) {
    const AmgLevD L = lev[l], N = lev[l + 1];
    float* v = sm + tail_lds_off<ND>(lev, l, l0);
    float* w = v + 3 * ND * L.A.n;
    // level l+1's output: its x if coarsest, else its e (held in its t)
    tail_prolong<ND>(L, N.coarsest ? w + ND * N.A.n : w + 2 * ND * N.A.n, v + ND * L.A.n);
    __syncthreads();
    if (l > l0) {
      tail_post<ND>(L, v, v + ND * L.A.n, v + 2 * ND * L.A.n);
      __syncthreads();
    } else {
      tail_post<ND>(L, v, v + ND * L.A.n, L.e);
    }
  }
}

// ---------------------------------------------------------------------------
// CG (f64)
// ---------------------------------------------------------------------------
// the V-cycle's first smoothing step x_0 = ω D⁻¹ r (f32), or — a single-level
// hierarchy (no free-free coupling) is its own coarsest level — the block
// solve u = D⁻¹ r (f64, rounded to the f32 u) straight into the CG's u
template <int ND>
__device__ __forceinline__ void vcycle_entry(const AmgLevD& L0, const AmgCg& cg, int64_t i, const double* r) {
  if (cg.sweep) return;  // the sweep kernel forms u from r
  if (L0.coarsest) {
    double u[ND];
    dinv_apply<ND>(L0.dinv, L0.A.n, i, 1.0, r, u);
    vstore<ND>(cg.u, i, u);
  } else {
    float rf[ND], x0[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) rf[a] = (float)r[a];
    dinv_apply<ND>(L0.dinv32, L0.A.n, i, (float)amg_omega(L0.omega), rf, x0);
    vstore<ND>(L0.x, i, x0);
  }
}

template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_cg_init(AmgLevD L0, AmgCg cg, const double* __restrict__ b_row) {
  const int64_t i = cg.lo + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= cg.hi) return;
  double r[ND], z[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) {
    r[a] = b_row[3 * (int64_t)cg.row0[i] + a];
    z[a] = 0.0;
  }
  vstore<ND>(cg.r, i, r);
  vstore<ND>(cg.x, i, z);
  vstore<ND>(cg.p, i, z);
  vstore<ND>(cg.s, i, z);
  vcycle_entry<ND>(L0, cg, i, r);
}

template <int ND, bool FIRST, int BS, bool DIST, int KW = 1>
__global__ __launch_bounds__(BS) void k_amg_cg_w(int j, AmgLevD L0, AmgCg cg, Slot* slots, double* part,
                                                 AmgDist d) {
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * BS;
  const int lane = threadIdx.x & 63;
  for (int64_t i = cg.lo64() + xcd_block() * BS + threadIdx.x; i - lane < cg.hi; i += stride) {
    const int64_t ii = i < cg.hi ? i : cg.hi - 1;
    int64_t base;
    int w;
    slice_of(L0.A, ii, base, w);
    double y[ND], u[ND], r[ND];
    vload<ND>(cg.u, ii, u);  // own-row operands in flight with the gather
    vload<ND>(cg.r, ii, r);
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0;
    sell_mac<ND, false, KW, true>(L0.A.col, L0.A.sym, L0.A.npos, base, w, cg.u, y);
    if (i < cg.lo || i >= cg.hi) continue;
    if constexpr (DIST) {  // couplings to free rows of other partitions: K_ig u_g
      for (int t = d.gptr[i]; t < d.gptr[i + 1]; ++t) {
        const int64_t q = d.gslot[t];
        double s6[6], m[ND * ND], ug[ND];
#pragma unroll
        for (int c = 0; c < 6; ++c) s6[c] = d.sval[(int64_t)c * d.G + q];
        sym_to<ND>(s6, m);
        vload<ND>(d.urecv, d.grecv[t], ug);
#pragma unroll
        for (int a = 0; a < ND; ++a)
#pragma unroll
          for (int b = 0; b < ND; ++b) y[a] = fma(m[a * ND + b], ug[b], y[a]);
      }
    }
    vstore<ND>(cg.w, i, y);
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      acc[0] = fma(r[a], u[a], acc[0]);
      acc[1] = fma(y[a], u[a], acc[1]);
      acc[2] = fma(r[a], r[a], acc[2]);
      acc[3] = fma(u[a], u[a], acc[3]);
    }
  }
  store_block_partial<BS>(acc, part_buf(part, FIRST ? 0 : ((j & 1) ^ 1)));
  if (FIRST && blockIdx.x == 0 && threadIdx.x == 0) {
    Slot s0;
    s0.v[0] = s0.v[1] = s0.v[2] = s0.v[3] = 0.0;
    s0.alpha = s0.beta = s0.res = 0.0;
    s0.flag = kInit;
    s0.pad = 0;
    slots[0] = s0;
  }
}

// Partitioned: this rank's sums (its w kernel's block partials in block
// order, as wave_partials does) → its row of gall[q] and gsend.  Every rank
// then adds the gathered rows in rank order (k_amg_cg_update<DIST>): the same
// bits everywhere, so α, β and the stopping test agree across ranks.
// zero_w > 0 (the rows travel as ONE all-reduce sum, capi.hip xchg_sums):
// the other ranks' rows [0, zero_w) of gall are zeroed, so the sum of the
// ranks' buffers is every rank's row exactly (x + 0 + … + 0 = x)
template <int PU>
__global__ __launch_bounds__(64) void k_amg_gsum(const double* __restrict__ p, double* all, int rank, int zero_w,
                                                 double* gsend) {
  double S[4];
  wave_partials<PU>(p, S);
  const int lane = threadIdx.x;
  if (lane < zero_w && lane != rank) {
#pragma unroll
    for (int c = 0; c < 4; ++c) all[4 * lane + c] = 0.0;
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      all[4 * rank + c] = S[c];
      gsend[c] = S[c];
    }
  }
}

template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_pack_u(AmgCg cg, AmgDist d) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= d.n_send) return;
  const int64_t i = d.send_rows[k];  // -1: a fixed node (zeros)
#pragma unroll
  for (int a = 0; a < ND; ++a) d.usend[ND * k + a] = i >= 0 ? cg.u[ND * i + a] : 0.0;
}

template <int ND, int PU, int BS, bool DIST>
__global__ __launch_bounds__(BS) void k_amg_cg_update(int j, AmgLevD L0, AmgCg cg, Slot* slots,
                                                      SolveState* st, double* part, AmgDist d) {
  const int f0 = __builtin_nontemporal_load(&slots[j].flag);
  const double g0 = slots[j].v[0], a0 = slots[j].alpha;
  double tol2 = st->tol2;
  const int base_it = st->base, max_it = st->max_it, norm = st->norm;
  double S[4];
  if constexpr (DIST) {  // the gathered rank sums, rank order (rows ≥ world are 0)
    const int lane = threadIdx.x & 63;
    const double* g = d.gall[j & 1];
#pragma unroll
    for (int c = 0; c < 4; ++c) S[c] = wave_allsum(g[lane * 4 + c]);
  } else {
    wave_partials<PU>(part_buf(part, j & 1), S);
  }
  // the first pass's row operands are issued behind the partials (loads
  // return in order: the scalars need only the partials) and are in flight
  // while α, β are formed — D⁻¹ for level 0's x = ω D⁻¹ r with them, and ω
  // through scalar loads: issued per row behind the stores (vcycle_entry),
  // they put one more round trip at the end of every row (the compiler cannot
  // move a load of ω across the row's stores)
  const int64_t stride = (int64_t)gridDim.x * BS;
  const int64_t i0 = cg.lo + (int64_t)blockIdx.x * BS + threadIdx.x;
  const bool x0_here = !cg.sweep && !L0.coarsest;  // (else vcycle_entry)
  const float om0 = x0_here ? (float)amg_omega_s(L0.omega) : 0.0f;
  double u[ND], w[ND], p[ND], s[ND], x[ND], r[ND];
  float Di[ND * ND];
  if (cg.hi > cg.lo) {
    const int64_t k = i0 < cg.hi ? i0 : cg.hi - 1;
    vload<ND>(cg.u, k, u);
    vload<ND>(cg.w, k, w);
    vload<ND>(cg.p, k, p);
    vload<ND>(cg.s, k, s);
    vload<ND>(cg.x, k, x);
    vload<ND>(cg.r, k, r);
    if (x0_here) dinv_load<ND>(L0.dinv32, k, Di);
  }
  if (norm == 1 && f0 == kInit) {
    // PETSc's preconditioned norm (KSP_NORM_PRECONDITIONED, src/fea_petsc.cpp:336-341):
    // ‖M⁻¹r‖ ≤ rtol‖M⁻¹b‖ with x₀ = 0 — the reference is this first ‖u₀‖²,
    // known only now (every block forms the same value; block 0 keeps it)
    tol2 = fmax(st->rtol2 * S[3], st->atol2);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->tol2 = tol2;
      st->res0 = S[3];
    }
  }
  const CgScalars cs = cg_scalars(S, f0, g0, a0, tol2, base_it + j, max_it, norm);
  cg_record(slots, j, S, cs);
  if (cs.status != kRun) return;
  const double alpha = cs.alpha, beta = cs.beta;
  for (int64_t i = i0; i < cg.hi; i += stride) {
    if (i != i0) {
      vload<ND>(cg.u, i, u);
      vload<ND>(cg.w, i, w);
      vload<ND>(cg.p, i, p);
      vload<ND>(cg.s, i, s);
      vload<ND>(cg.x, i, x);
      vload<ND>(cg.r, i, r);
      if (x0_here) dinv_load<ND>(L0.dinv32, i, Di);
    }
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      p[a] = fma(beta, p[a], u[a]);
      s[a] = fma(beta, s[a], w[a]);
      x[a] = fma(alpha, p[a], x[a]);
      r[a] = fma(-alpha, s[a], r[a]);
    }
    vstore<ND>(cg.p, i, p);
    vstore<ND>(cg.s, i, s);
    vstore<ND>(cg.x, i, x);
    vstore<ND>(cg.r, i, r);
    if (x0_here) {  // level 0's x = ω D⁻¹ r (vcycle_entry's arithmetic)
      float rf[ND], x0[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a) rf[a] = (float)r[a];
      dinv_mul<ND>(Di, om0, rf, x0);
      vstore<ND>(L0.x, i, x0);
    } else {
      vcycle_entry<ND>(L0, cg, i, r);
    }
  }
}

template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_finish(AmgCg cg, double* __restrict__ x_row) {
  const int64_t i = cg.lo + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= cg.hi) return;
#pragma unroll
  for (int a = 0; a < ND; ++a) x_row[3 * (int64_t)cg.row0[i] + a] = cg.x[ND * i + a];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static dim3 slot_grid(int64_t npos) {  // one wave per slot row (slot_wave)
  const int64_t w = kBlock / 64, t = npos / 64;
  return dim3((unsigned)((t + w - 1) / w > 0 ? (t + w - 1) / w : 1));
}
static dim3 rows_grid(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock > 0 ? (n + kBlock - 1) / kBlock : 1)); }

// The w kernel writes one partial per block and every wave of the next
// update kernel re-reads them all (≤ kCgMaxG = 512 blocks).  Measured at C3
// (336k rows): w 16.3 µs at 256 threads × 512 blocks (2.6 grid-stride
// passes, 8 waves per CU), 14.9 at 1024 × 329 (but 329 blocks leave 73 CUs
// with twice the work — the streaming update kernel went 10.7 → 15.3 µs);
// so the update keeps 256-thread blocks.  w: 768-thread blocks above 512·512
// rows (C3: 438 blocks, one pass; same-box A/B of the whole iteration 166.6
// vs 170.0 µs at 512 and 169.5 at 1024; C5 1786 vs 1831 vs 1784), 512 / 256
// below.  Both read the w kernel's partial count, amg_w_grid.  cg.w_block > 0
// overrides the choice (mfea_set_option "amg_w_block").
// Round 4: between 512·512 and 768·512 rows the smallest of 576 / 640 / 704 /
// 768 whose grid fits kCgMaxG blocks in one pass — at C3 704 × 478 blocks
// instead of 768 × 438: two blocks on every CU carry 1,408 rows instead of
// 1,536 where 74 CUs got one (the SpMV is one pass of latency-bound rows).
int amg_w_block(const AmgCg& cg) {
  if (cg.w_block > 0) return cg.w_block;
  const int64_t n = cg.hi > cg.lo ? cg.hi - cg.lo64() : 0;
  if (n <= (int64_t)kCgMaxG * kCgBS) return kCgBS;
  if (n <= (int64_t)kCgMaxG * 512) return 512;
  for (int bs : {576, 640, 704})
    if (n <= (int64_t)kCgMaxG * bs) return bs;
  return 768;
}
int64_t amg_w_grid(const AmgCg& cg) {
  const int64_t n = cg.hi > cg.lo ? cg.hi - cg.lo64() : 0;
  const int bs = amg_w_block(cg);
  const int64_t g = (n + bs - 1) / bs;
  return g < 1 ? 1 : (g > kCgMaxG ? kCgMaxG : g);
}
static int pu_of_grid(int64_t g) { return g <= 64 ? 1 : g <= 128 ? 2 : g <= 256 ? 4 : 8; }

template <int ND>
static void a0_nd(hipStream_t s, const AmgLevD& L0, const SellOp& sop, const int32_t* row0, const int32_t* p,
                  const int32_t* a, double reg, bool full) {
  if (L0.A.n <= 0) return;
  if (full) {  // fixed ω: Ã_0 and P_0 too, no bound (the fused setup skips level 0's P/Ã launch)
    hipLaunchKernelGGL(k_amg_a0full<ND>, rows_grid(L0.A.rg.span()), dim3(kBlock), 0, s, L0, sop, row0, p, a, reg);
    return;
  }
  if (L0.fixed_omega && L0.a0slot) {  // no bound to form: one thread per position
    const int64_t blocks = (L0.A.rg.npos() / 64 + kBlock / 64 - 1) / (kBlock / 64);
    hipLaunchKernelGGL(k_amg_a0slot<ND>, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(kBlock), 0, s, L0, sop,
                       row0, p, a, reg);
    return;
  }
  // level 0's bound, max'ed by the blocks (not at a fixed ω: nothing reads it)
  if (!L0.fixed_omega) (void)hipMemsetAsync(L0.omega + 1, 0, sizeof(double), s);
  hipLaunchKernelGGL(k_amg_a0dinv<ND>, rows_grid(L0.A.rg.span()), dim3(kBlock), 0, s, L0, sop, row0, p, a, reg);
}
void launch_amg_a0(hipStream_t s, int nd, const AmgLevD& L0, const SellOp& sop, const int32_t* row0,
                   const int32_t* a0_ptr, const int32_t* a0_a, double reg, bool full) {
  if (nd == 2) a0_nd<2>(s, L0, sop, row0, a0_ptr, a0_a, reg, full);
  else a0_nd<3>(s, L0, sop, row0, a0_ptr, a0_a, reg, full);
}

// the grid of a setup launch over level L (x1: 8× the blocks, setup_block)
static dim3 xg(const AmgLevD& L, dim3 g) { return dim3(L.x1 ? 8 * g.x : g.x); }
static dim3 xg(const AmgLevD& L, int64_t blocks) { return xg(L, dim3((unsigned)blocks)); }

template <int ND>
static void setup_nd(hipStream_t s, const AmgLevD& L, const AmgLevD* N, bool level0, int stage) {
  if (L.A.n <= 0) return;
  // level 0's D⁻¹ came with its blocks (k_amg_a0dinv, launch_amg_a0)
  if (stage & kSetupDinv && !level0)
    hipLaunchKernelGGL(k_amg_dinv<ND>, xg(L, rows_grid(L.A.rg.span())), dim3(kBlock), 0, s, L);
  if (L.coarsest || !N) return;
  if (stage & kSetupP && L.P.wmax > 0)
    hipLaunchKernelGGL(k_amg_pvals<ND>, xg(L, slot_grid(L.P.rg.npos())), dim3(kBlock), 0, s, L);
  if (stage & kSetupAP) {
    hipLaunchKernelGGL(k_amg_ap<ND>, xg(L, rows_grid(std::max(L.AP.rg.npos(), L.R.rg.npos()))), dim3(kBlock), 0, s, L);
  }
  if (stage & kSetupAC) launch_ac<ND>(s, L, N->A, N->omega, nullptr, ac_blocks(L), 0, false);
}
void launch_amg_level_setup(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD* next, bool level0, int stage) {
  if (nd == 2) setup_nd<2>(s, L, next, level0, stage);
  else setup_nd<3>(s, L, next, level0, stage);
}

template <int ND>
static void compact_level_nd(hipStream_t s, const AmgLevD* lev, int l, int parts = kCompactAll) {
  const AmgLevD& L = lev[l];
  if (!L.compact || L.PT.wmax <= 0) return;
  if (parts & kCompactPT)
    hipLaunchKernelGGL(k_amg_ptv<ND>, xg(L, slot_grid(L.PT.rg.npos())), dim3(kBlock), 0, s, L);
  if (parts & kCompactRT)
    hipLaunchKernelGGL(k_amg_rtv<ND>, xg(L, slot_grid(L.RT.rg.npos())), dim3(kBlock), 0, s, L, lev[l + 1]);
  if (parts & kCompactAT)
    hipLaunchKernelGGL(k_amg_atv<ND>, xg(L, slot_grid(L.A.rg.npos())), dim3(kBlock), 0, s, L);
}
void launch_amg_compact_level(hipStream_t s, int nd, const AmgLevD* lev, int l, int parts) {
  if (nd == 2) compact_level_nd<2>(s, lev, l, parts);
  else compact_level_nd<3>(s, lev, l, parts);
}
// mg (merged levels 0–1, AmgMergeD): their products ride in the last of
// these launches (MprodSlice) — the caller then skips launch_amg_merge_setup.
// Returns whether they did.
template <int ND>
static bool collapse_setup_nd(hipStream_t s, const AmgLevD* lev, int nlev, int coll, int below = 1 << 30,
                              const AmgMergeD* mg = nullptr) {
  if (coll <= 0) return false;
  const int top = std::min(nlev - 2, below - 1);
  int nl = 0;  // launches of the collapse
  for (int l = top; l >= coll && lev[l].collapsed; --l) nl += 2;
  MprodSlice ms;
  int64_t gm = 0;
  if (mg && mg->on && nl > 0) {
    ms.m = *mg;
    ms.at1 = lev[1].A.at32;
    ms.r0 = lev[0].RT.val32;
    ms.r1 = lev[1].RT.val32;
    ms.p0 = lev[0].PT.val32;
    ms.p1 = lev[1].PT.val32;
    ms.gdq = rows_grid(mg->DQ.npos).x;
    gm = ms.gdq + rows_grid(mg->U.npos).x;
  }
  int k = 0;
  auto share = [&](dim3 g) {  // the next launch's slice (all in the last, V_kc's); its grid grows by it
    ms.b0 = 0;
    ms.b1 = k + 1 == nl ? gm : 0;
    ++k;
    return dim3(g.x + (unsigned)(ms.b1 - ms.b0));
  };
  for (int l = top; l >= coll; --l) {  // deepest first: T_l needs V_{l+1}
    const AmgLevD& L = lev[l];
    if (!L.collapsed) break;
    const float* vnext = l + 2 < nlev && lev[l + 1].collapsed ? lev[l + 1].CV.val32 : nullptr;
    const dim3 gt = xg(L, rows_grid(L.CT.npos)), gv = xg(L, rows_grid(L.CV.npos));
    dim3 g = share(gt);
    hipLaunchKernelGGL(k_amg_tv<ND>, g, dim3(kBlock), 0, s, L, vnext, ms, (int64_t)gt.x);
    g = share(gv);
    hipLaunchKernelGGL(k_amg_vv<ND>, g, dim3(kBlock), 0, s, L, ms, (int64_t)gv.x);
  }
  return gm > 0;
}
// the whole numeric setup of a compact-cycle hierarchy, its compact parts
// fused into the chain's launches (k_amg_fuse_p / k_amg_fuse_ac): three
// launches per level (D⁻¹, P values, A·P, A_{l+1}: level 0's D⁻¹ is
// k_amg_a0's partner) instead of seven
static int64_t slot_blocks(int64_t npos) { return (npos / 64 + kBlock / 64 - 1) / (kBlock / 64); }
template <int ND>
static bool setup_fused_nd(hipStream_t s, const AmgLevD* lev, int nlev, int coll, const AmgMergeD* mg) {
  auto compact = [&](int l) { return l + 1 < nlev && lev[l].compact && lev[l].PT.wmax > 0 && !lev[l].coarsest; };
  for (int l = 0; l < nlev; ++l) {
    const AmgLevD& L = lev[l];
    if (L.A.n <= 0) return false;
    const bool last = L.coarsest || l + 1 >= nlev;
    if (l > 0 && !L.fixed_omega)  // (fixed ω: D⁻¹ came with A_l, k_amg_ac)
      hipLaunchKernelGGL(k_amg_dinv<ND>, xg(L, rows_grid(L.A.rg.span())), dim3(kBlock), 0, s, L);
    // (level 0 at a fixed ω: P_0 and Ã_0 came with A_0, k_amg_a0full)
    const bool a0full = l == 0 && L.a0full;
    const int64_t g0 = !last && L.P.wmax > 0 && !a0full ? slot_blocks(L.P.rg.npos()) : 0;
    const int64_t g1 = g0 + (compact(l) && !a0full ? slot_blocks(L.A.npos) : 0);
    const int64_t g2 = g1 + (l > 0 && compact(l - 1) ? slot_blocks(lev[l - 1].RT.npos) : 0);
    if (g2 > 0)
      hipLaunchKernelGGL(k_amg_fuse_p<ND>, xg(L, g2), dim3(kBlock), 0, s, L, l > 0 ? lev[l - 1] : L, g0, g1);
    if (last) break;
    const dim3 gap = rows_grid(std::max(L.AP.rg.npos(), L.compact ? 0 : L.R.rg.npos()));
    float* const dnext = lev[l + 1].fixed_omega ? lev[l + 1].dinv32 : nullptr;
    if (compact(l) && L.PT.npos == L.AP.npos) {  // P̃ formed by the A·P kernel
      hipLaunchKernelGGL((k_amg_ap<ND, true>), xg(L, gap), dim3(kBlock), 0, s, L);
      launch_ac<ND>(s, L, lev[l + 1].A, lev[l + 1].omega, dnext, ac_blocks(L), 0, false);
    } else {
      hipLaunchKernelGGL(k_amg_ap<ND>, xg(L, gap), dim3(kBlock), 0, s, L);
      const int64_t a0 = ac_blocks(L);
      const int64_t a1 = a0 + (compact(l) ? slot_blocks(L.PT.npos) : 0);
      launch_ac<ND>(s, L, lev[l + 1].A, lev[l + 1].omega, dnext, a1, a0, true);
    }
  }
  return collapse_setup_nd<ND>(s, lev, nlev, coll, 1 << 30, mg);
}
bool launch_amg_setup_fused(hipStream_t s, int nd, const AmgLevD* lev, int nlev, int coll, const AmgMergeD* mg) {
  if (nd == 2) return setup_fused_nd<2>(s, lev, nlev, coll, mg);
  return setup_fused_nd<3>(s, lev, nlev, coll, mg);
}
template <int ND>
static void compact_setup_nd(hipStream_t s, const AmgLevD* lev, int nlev, int coll, int l0) {
  for (int l = l0; l + 1 < nlev; ++l) compact_level_nd<ND>(s, lev, l);
  collapse_setup_nd<ND>(s, lev, nlev, coll);
}
void launch_amg_compact_setup(hipStream_t s, int nd, const AmgLevD* lev, int nlev, int coll, int l0) {
  if (nd == 2) compact_setup_nd<2>(s, lev, nlev, coll, l0);
  else compact_setup_nd<3>(s, lev, nlev, coll, l0);
}

// lanes per row: the restriction by R's mean slice width, the f32 operators
// below level 0 by A's (mfea_set_option "amg_restrict_lanes" / "amg_op_lanes"
// > 0 override: 1, 2 or 4)
static int lanes_for(const AmgMatD& M, int forced, double two, double four) {
  if (forced > 0) return forced;
  const double mean_w = M.n > 0 ? (double)M.npos / (double)(((M.n + 63) / 64) * 64) : 0.0;
  return mean_w > four ? 4 : mean_w > two ? 2 : 1;
}
int amg_restrict_lanes(const AmgLevD& L) { return lanes_for(L.R, L.rlanes, 2.5, 5.0); }
int amg_op_lanes(const AmgLevD& L) { return lanes_for(L.A, L.alanes, 3.5, 8.0); }
template <int ND>
static void launch_restrict(hipStream_t s, const AmgLevD& L, const AmgLevD& N, const int32_t* gate) {
  const int64_t n = L.R.rg.span();
  const int S = amg_restrict_lanes(L);
  const dim3 b(kBlock);
  if (S == 8) hipLaunchKernelGGL((k_amg_restrict_s<ND, 8>), rows_grid(8 * n), b, 0, s, L, N, gate);
  else if (S == 4) hipLaunchKernelGGL((k_amg_restrict_s<ND, 4>), rows_grid(4 * n), b, 0, s, L, N, gate);
  else if (S == 2) hipLaunchKernelGGL((k_amg_restrict_s<ND, 2>), rows_grid(2 * n), b, 0, s, L, N, gate);
  else hipLaunchKernelGGL(k_amg_restrict<ND>, rows_grid(n), b, 0, s, L, N, gate);
}
template <int ND>
static void launch_op(hipStream_t s, const AmgLevD& L, bool post, const int32_t* gate) {
  const int64_t n = L.A.rg.span();
  const int S = amg_op_lanes(L);
  const dim3 b(kBlock);
  if (S == 4) {
    if (post) hipLaunchKernelGGL((k_amg_post_s<ND, 4>), rows_grid(4 * n), b, 0, s, L, gate);
    else hipLaunchKernelGGL((k_amg_resid_s<ND, 4>), rows_grid(4 * n), b, 0, s, L, gate);
  } else if (S == 2) {
    if (post) hipLaunchKernelGGL((k_amg_post_s<ND, 2>), rows_grid(2 * n), b, 0, s, L, gate);
    else hipLaunchKernelGGL((k_amg_resid_s<ND, 2>), rows_grid(2 * n), b, 0, s, L, gate);
  } else {
    if (post)
      hipLaunchKernelGGL((k_amg_post<ND, float, float, false>), rows_grid(n), b, 0, s, L, (const float*)L.b, L.e, gate);
    else
      hipLaunchKernelGGL((k_amg_resid<ND, float, false>), rows_grid(n), b, 0, s, L, (const float*)L.b, gate);
  }
}

// the V-cycle's steps on level l (level 0 reads the CG's f64 r and writes
// its u; the others their f32 b, e)
template <int ND>
static void resid_nd(hipStream_t s, const AmgLevD* lev, int l, const AmgCg& cg, const int32_t* gate) {
  if (l == 0)
    hipLaunchKernelGGL((k_amg_resid<ND, double, true>), rows_grid(lev[0].A.rg.span()), dim3(kBlock), 0, s, lev[0],
                       (const double*)cg.r, gate);
  else
    launch_op<ND>(s, lev[l], false, gate);
}
template <int ND>
static void post_nd(hipStream_t s, const AmgLevD* lev, int l, const AmgCg& cg, const int32_t* gate) {
  if (l == 0)
    hipLaunchKernelGGL((k_amg_post<ND, double, float, true>), rows_grid(lev[0].A.rg.span()), dim3(kBlock), 0, s,
                       lev[0], (const double*)cg.r, cg.u, gate);
  else
    launch_op<ND>(s, lev[l], true, gate);
}
template <int ND>
static void prolong_nd(hipStream_t s, const AmgLevD* lev, int l, const int32_t* gate) {
  hipLaunchKernelGGL(k_amg_prolong<ND>, rows_grid(lev[l].P.rg.span()), dim3(kBlock), 0, s, lev[l], lev[l + 1], gate);
}

// the compact cycle's sweeps (lanes per row by the matrices' mean widths)
// R̃ rows hold 8–12 blocks on C3's levels (R's 5–7): 8 lanes from a mean of 6
// (C3 iteration 84.3 vs 86.3 µs at 4 lanes, C2 41.6 vs 44.3)
int amg_down_lanes(const AmgLevD& L) {
  if (L.rlanes > 0) return L.rlanes;
  const int64_t rows = ((L.RT.n + 63) / 64) * 64;
  const double mean_w = rows > 0 ? (double)L.RT.npos / (double)rows : 0.0;
  // (16 lanes past a mean width of 20 measured slower on C5's level 0:
  // iteration 854 vs 751 µs; a small level's launch, one chain long, may gain)
  const int wide = L.small_lanes > 0 && 8 * L.RT.n < L.small_lanes && mean_w > 12.0 ? 16 : 8;
  return mean_w > 6.0 ? wide : lanes_for(L.RT, 0, 2.5, 5.0);
}
// one lane per P̃ row up to a mean width of 8 (measured: C5 iteration 736 µs
// at 1 lane against 759 at 2 and 845 at 4, C3 71.9 / 75.2 / 83.6)
int amg_up_lanes(const AmgLevD& L) { return lanes_for(L.PT, L.ulanes, 8.0, 16.0); }
// the down sweep's Ã rows in steps of 2U (K = 2; K = 3 measured slower even
// on C5's 11-block-wide level 1: iteration 790 vs 760 µs)
template <int ND>
static void down_nd(hipStream_t s, const AmgLevD& L, const AmgLevD& N, const int32_t* gate) {
  const int S = amg_down_lanes(L);
  const int64_t gr = rows_grid(S * L.RT.rg.span()).x, ga = rows_grid(L.A.rg.span()).x;
  auto go = [&](int64_t gc, int64_t blocks) {
    const dim3 g((unsigned)blocks);
    if (S == 16) hipLaunchKernelGGL((k_amg_down<ND, 16>), g, dim3(kBlock), 0, s, L, N, gc, gate);
    else if (S == 8) hipLaunchKernelGGL((k_amg_down<ND, 8>), g, dim3(kBlock), 0, s, L, N, gc, gate);
    else if (S == 4) hipLaunchKernelGGL((k_amg_down<ND, 4>), g, dim3(kBlock), 0, s, L, N, gc, gate);
    else if (S == 2) hipLaunchKernelGGL((k_amg_down<ND, 2>), g, dim3(kBlock), 0, s, L, N, gc, gate);
    else hipLaunchKernelGGL((k_amg_down<ND, 1>), g, dim3(kBlock), 0, s, L, N, gc, gate);
  };
  if (L.dsplit) {  // R̂ rows, then Ã rows (experiment: each row set's own time)
    go(gr, gr);
    go(0, ga);
  } else {
    go(gr, gr + ga);
  }
}
template <int ND, class TE>
static void up_te(hipStream_t s, const AmgLevD& L, const AmgLevD& N, TE* e, const int32_t* gate) {
  const int S = amg_up_lanes(L);
  const dim3 g(rows_grid(S * L.PT.rg.span()));
  if (S == 4) hipLaunchKernelGGL((k_amg_up<ND, 4, TE>), g, dim3(kBlock), 0, s, L, N, e, gate);
  else if (S == 2) hipLaunchKernelGGL((k_amg_up<ND, 2, TE>), g, dim3(kBlock), 0, s, L, N, e, gate);
  else hipLaunchKernelGGL((k_amg_up<ND, 1, TE>), g, dim3(kBlock), 0, s, L, N, e, gate);
}
template <int ND>
static void vapply_nd(hipStream_t s, const AmgLevD& L, const int32_t* gate) {
  const int64_t rows = ((L.CV.n + 63) / 64) * 64;
  const double mean_w = rows > 0 ? (double)L.CV.npos / (double)rows : 0.0;
  // a V of a few thousand rows cannot fill the GPU at 8 lanes per row: its
  // launch is one dependent chain long, so 16 lanes shorten the chain
  // (C2: 2.4 k rows × 50 blocks, iteration 29.1 → 27.7 µs; C5 703 → 695;
  // C3's 24 k rows stay at 8: 67.1 vs 68.8 at 16)
  const int wide = L.small_lanes > 0 && 8 * L.CV.n < L.small_lanes ? 16 : 8;
  const int S = L.vlanes > 0 ? L.vlanes : mean_w > 12.0 ? wide : mean_w > 5.0 ? 4 : mean_w > 2.5 ? 2 : 1;
  const dim3 g(rows_grid(S * L.CV.n));
  if (S == 16) hipLaunchKernelGGL((k_amg_vapply<ND, 16>), g, dim3(kBlock), 0, s, L, gate);
  else if (S == 8) hipLaunchKernelGGL((k_amg_vapply<ND, 8>), g, dim3(kBlock), 0, s, L, gate);
  else if (S == 4) hipLaunchKernelGGL((k_amg_vapply<ND, 4>), g, dim3(kBlock), 0, s, L, gate);
  else if (S == 2) hipLaunchKernelGGL((k_amg_vapply<ND, 2>), g, dim3(kBlock), 0, s, L, gate);
  else hipLaunchKernelGGL((k_amg_vapply<ND, 1>), g, dim3(kBlock), 0, s, L, gate);
}
// levels 0 and 1 merged (AmgMergeD): one down launch over DQ's rows and Ã_0's,
// V_2, one up launch over U's rows into the CG's u
template <int ND>
static void merged_nd(hipStream_t s, const AmgLevD* lev, const AmgCg& cg, const AmgMergeD& m, const int32_t* gate) {
  AmgLevD Ld = lev[0], Nd{}, Lu = lev[0], Nu{};
  Ld.RT = m.DQ;
  Ld.rt_row = m.dq_dst;
  Nd.x = m.B;
  Lu.PT = m.U;
  Nu.e = m.B;
  // DQ's wide rows at 16 lanes whatever their count, U's at one lane (C2
  // iteration 28.1 → 26.7 µs, tools/amg_ab.py: amg_small_lanes 65536 vs 1 Mi
  // with C3 unmerged and slower under that setting; amg_up_lanes 1 vs 2:
  // 27.75 vs 28.2); a caller's amg_small_lanes 0 / amg_up_lanes keep theirs
  if (Ld.small_lanes > 0) Ld.small_lanes = INT32_MAX;
  if (Lu.ulanes <= 0) Lu.ulanes = 1;
  down_nd<ND>(s, Ld, Nd, gate);
  vapply_nd<ND>(s, lev[2], gate);
  up_te<ND, float>(s, Lu, Nu, cg.u, gate);
}
template <int ND>
static void compact_nd(hipStream_t s, const AmgLevD* lev, int nlev, const AmgCg& cg, const int32_t* gate, int l0) {
  if (cg.coll > l0 && cg.coll < nlev - 1 && lev[cg.coll].collapsed && lev[cg.coll].CV.n > 0) {
    const int kc = cg.coll;
    for (int l = l0; l < kc; ++l) down_nd<ND>(s, lev[l], lev[l + 1], gate);
    vapply_nd<ND>(s, lev[kc], gate);
    for (int l = kc - 1; l >= l0; --l) up_te<ND, float>(s, lev[l], lev[l + 1], l == 0 ? cg.u : lev[l].e, gate);
    return;
  }
  const int top = nlev - 1;  // the coarsest level's output is its x
  for (int l = l0; l < top; ++l) down_nd<ND>(s, lev[l], lev[l + 1], gate);
  for (int l = top - 1; l >= l0; --l) {
    if (l == 0) up_te<ND, float>(s, lev[0], lev[1], cg.u, gate);
    else up_te<ND, float>(s, lev[l], lev[l + 1], lev[l].e, gate);
  }
}
bool amg_compact_ok(const AmgLevD* lev, int nlev, int l0) {
  for (int l = l0; l + 1 < nlev; ++l)
    if (!lev[l].compact || lev[l].PT.n != lev[l].A.n || lev[l].A.rg.lo != 0 || lev[l].A.rg.hi != lev[l].A.n)
      return false;
  return nlev - l0 >= 2;
}

// The V-cycle of levels [l0, nlev) on level l0's b, x (the producer of b set
// x = ω D⁻¹ b), leaving level l0's output in its e (level 0: the CG's u).
template <int ND>
static void vcycle_nd(hipStream_t s, const AmgLevD* lev, int nlev, const AmgCg& cg,
                      int tail, const int32_t* gate, int l0, const AmgMergeD* mg) {
  if (mg && mg->on && l0 == 0 && cg.cycle == 1 && cg.coll == 2 && nlev >= 4) {
    merged_nd<ND>(s, lev, cg, *mg, gate);
    return;
  }
  if (cg.cycle == 1 && amg_compact_ok(lev, nlev, l0)) {
    compact_nd<ND>(s, lev, nlev, cg, gate, l0);
    return;
  }
  if (tail > 0 && tail < l0) tail = l0;
  const int top = tail > 0 ? tail : nlev - 1;  // levels [top, nlev) run inside k_amg_tail
  for (int l = l0; l < top; ++l) {
    resid_nd<ND>(s, lev, l, cg, gate);
    launch_restrict<ND>(s, lev[l], lev[l + 1], gate);
  }
  if (tail > 0) {
    TailLevels tl;
    int64_t lds = 0;
    for (int l = tail; l < nlev; ++l) {
      tl.lev[l - tail] = lev[l];
      lds += 3 * ND * lev[l].A.n * (int64_t)sizeof(float);
    }
    if (lds <= kTailLdsMax && lev[tail].tail_lds)
      hipLaunchKernelGGL(k_amg_tail_lds<ND>, dim3(1), dim3(kTailBS), (size_t)lds, s, tl, tail, nlev, gate);
    else
      hipLaunchKernelGGL(k_amg_tail<ND>, dim3(1), dim3(kTailBS), 0, s, tl, tail, nlev, gate);
  }
  for (int l = top - 1; l >= l0; --l) {
    prolong_nd<ND>(s, lev, l, gate);
    post_nd<ND>(s, lev, l, cg, gate);
  }
}
static int clamp_tail(int tail, int nlev) {
  if (tail >= nlev - 1) return 0;  // nothing below the coarsest to fuse
  if (tail > 0 && nlev - tail > kTailMaxLev) return nlev - kTailMaxLev;  // the kernel argument holds 4 levels
  return tail;
}
void launch_amg_down(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD& N) {
  if (nd == 2) down_nd<2>(s, L, N, nullptr);
  else down_nd<3>(s, L, N, nullptr);
}
void launch_amg_up(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD& N, float* e) {
  if (nd == 2) up_te<2, float>(s, L, N, e, nullptr);
  else up_te<3, float>(s, L, N, e, nullptr);
}
void launch_amg_vcycle(hipStream_t s, int nd, const AmgLevD* lev, int nlev, const AmgCg& cg,
                       int tail, const int32_t* gate, int l0, const AmgMergeD* mg) {
  // one level: the coarsest solve u = D⁻¹ r is done by the producer of r
  if (nlev <= 1 || lev[0].A.n <= 0 || l0 >= nlev - 1) return;
  tail = clamp_tail(tail, nlev);
  if (nd == 2) vcycle_nd<2>(s, lev, nlev, cg, tail, gate, l0, mg);
  else vcycle_nd<3>(s, lev, nlev, cg, tail, gate, l0, mg);
}
void launch_amg_merge_setup(hipStream_t s, int nd, const AmgLevD* lev, const AmgMergeD& m) {
  if (!m.on) return;
  const int64_t gdq = rows_grid(m.DQ.npos).x, gu = rows_grid(m.U.npos).x;
  const dim3 g((unsigned)(gdq + gu));
  if (nd == 2)
    hipLaunchKernelGGL(k_amg_mprod<2>, g, dim3(kBlock), 0, s, m, lev[1].A.at32, lev[0].RT.val32, lev[1].RT.val32,
                       lev[0].PT.val32, lev[1].PT.val32, gdq);
  else
    hipLaunchKernelGGL(k_amg_mprod<3>, g, dim3(kBlock), 0, s, m, lev[1].A.at32, lev[0].RT.val32, lev[1].RT.val32,
                       lev[0].PT.val32, lev[1].PT.val32, gdq);
}
void launch_amg_vstep(hipStream_t s, int nd, const AmgLevD* lev, int l, const AmgCg& cg, int step,
                      const int32_t* gate) {
  if (nd == 2) {
    if (step == kStepResid) resid_nd<2>(s, lev, l, cg, gate);
    else if (step == kStepRestrict) launch_restrict<2>(s, lev[l], lev[l + 1], gate);
    else if (step == kStepProlong) prolong_nd<2>(s, lev, l, gate);
    else post_nd<2>(s, lev, l, cg, gate);
  } else {
    if (step == kStepResid) resid_nd<3>(s, lev, l, cg, gate);
    else if (step == kStepRestrict) launch_restrict<3>(s, lev[l], lev[l + 1], gate);
    else if (step == kStepProlong) prolong_nd<3>(s, lev, l, gate);
    else post_nd<3>(s, lev, l, cg, gate);
  }
}

int amg_tail_level(const int64_t* rows, int nlev, int64_t max_rows) {
  for (int l = 1; l + 1 < nlev; ++l)
    if (rows[l] <= max_rows) return l;
  return 0;
}

void launch_amg_cg_init(hipStream_t s, int nd, const AmgLevD& L0, const AmgCg& cg, const double* b_row) {
  if (cg.hi <= cg.lo) return;
  if (nd == 2) hipLaunchKernelGGL(k_amg_cg_init<2>, rows_grid(cg.hi - cg.lo), dim3(kBlock), 0, s, L0, cg, b_row);
  else hipLaunchKernelGGL(k_amg_cg_init<3>, rows_grid(cg.hi - cg.lo), dim3(kBlock), 0, s, L0, cg, b_row);
}

template <int ND, int BS>
static void w_bs(hipStream_t s, int j, bool first, const AmgLevD& L0, const AmgCg& cg, Slot* slots,
                 double* part, const AmgDist* d) {
  const dim3 g((unsigned)amg_w_grid(cg));
  const AmgDist dd = d ? *d : AmgDist{};
  if (d) {
    if (first) hipLaunchKernelGGL((k_amg_cg_w<ND, true, BS, true>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
    else hipLaunchKernelGGL((k_amg_cg_w<ND, false, BS, true>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
  } else if (cg.w_k == 2) {  // slices up to 2U wide in one round trip (wide level-0 rows)
    if (first) hipLaunchKernelGGL((k_amg_cg_w<ND, true, BS, false, 2>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
    else hipLaunchKernelGGL((k_amg_cg_w<ND, false, BS, false, 2>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
  } else {
    if (first) hipLaunchKernelGGL((k_amg_cg_w<ND, true, BS, false>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
    else hipLaunchKernelGGL((k_amg_cg_w<ND, false, BS, false>), g, dim3(BS), 0, s, j, L0, cg, slots, part, dd);
  }
}
template <int ND>
static void w_nd(hipStream_t s, int j, bool first, const AmgLevD& L0, const AmgCg& cg, Slot* slots,
                 double* part, const AmgDist* d) {
  switch (amg_w_block(cg)) {
    case 512: w_bs<ND, 512>(s, j, first, L0, cg, slots, part, d); break;
    case 576: w_bs<ND, 576>(s, j, first, L0, cg, slots, part, d); break;
    case 640: w_bs<ND, 640>(s, j, first, L0, cg, slots, part, d); break;
    case 704: w_bs<ND, 704>(s, j, first, L0, cg, slots, part, d); break;
    case 768: w_bs<ND, 768>(s, j, first, L0, cg, slots, part, d); break;
    case 1024: w_bs<ND, 1024>(s, j, first, L0, cg, slots, part, d); break;
    default: w_bs<ND, kCgBS>(s, j, first, L0, cg, slots, part, d); break;
  }
}
void launch_amg_cg_w(hipStream_t s, int nd, int j, bool first, const AmgLevD& L0, const AmgCg& cg,
                     Slot* slots, double* part, const AmgDist* d) {
  if (nd == 2) w_nd<2>(s, j, first, L0, cg, slots, part, d);
  else w_nd<3>(s, j, first, L0, cg, slots, part, d);
}

void launch_amg_gsum(hipStream_t s, const AmgCg& cg, const double* part_q, const AmgDist& d, int q) {
  double* all = d.gall[q];
  const int r = d.rank, zw = d.zero_w;
  switch (pu_of_grid(amg_w_grid(cg))) {  // the w kernel's grid = its partial count
    case 1: hipLaunchKernelGGL(k_amg_gsum<1>, dim3(1), dim3(64), 0, s, part_q, all, r, zw, d.gsend); break;
    case 2: hipLaunchKernelGGL(k_amg_gsum<2>, dim3(1), dim3(64), 0, s, part_q, all, r, zw, d.gsend); break;
    case 4: hipLaunchKernelGGL(k_amg_gsum<4>, dim3(1), dim3(64), 0, s, part_q, all, r, zw, d.gsend); break;
    default: hipLaunchKernelGGL(k_amg_gsum<8>, dim3(1), dim3(64), 0, s, part_q, all, r, zw, d.gsend); break;
  }
}

void launch_amg_pack_u(hipStream_t s, int nd, const AmgCg& cg, const AmgDist& d) {
  if (d.n_send <= 0) return;
  if (nd == 2) hipLaunchKernelGGL(k_amg_pack_u<2>, rows_grid(d.n_send), dim3(kBlock), 0, s, cg, d);
  else hipLaunchKernelGGL(k_amg_pack_u<3>, rows_grid(d.n_send), dim3(kBlock), 0, s, cg, d);
}

template <int ND, int BS, bool DIST>
static void upd_bs(hipStream_t s, int j, const AmgLevD& L0, const AmgCg& cg, Slot* slots,
                   SolveState* st, double* part, const AmgDist& d) {
  const int64_t gw = amg_w_grid(cg);  // partials to reduce = the w kernel's blocks
  int64_t gu = (cg.hi - cg.lo + BS - 1) / BS;
  gu = gu < 1 ? 1 : (gu > kCgMaxG ? kCgMaxG : gu);
  const dim3 g((unsigned)gu);
  switch (DIST ? 1 : pu_of_grid(gw)) {
    case 1: hipLaunchKernelGGL((k_amg_cg_update<ND, 1, BS, DIST>), g, dim3(BS), 0, s, j, L0, cg, slots, st, part, d); break;
    case 2: hipLaunchKernelGGL((k_amg_cg_update<ND, 2, BS, DIST>), g, dim3(BS), 0, s, j, L0, cg, slots, st, part, d); break;
    case 4: hipLaunchKernelGGL((k_amg_cg_update<ND, 4, BS, DIST>), g, dim3(BS), 0, s, j, L0, cg, slots, st, part, d); break;
    default: hipLaunchKernelGGL((k_amg_cg_update<ND, 8, BS, DIST>), g, dim3(BS), 0, s, j, L0, cg, slots, st, part, d); break;
  }
}
template <int ND>
static void upd_nd(hipStream_t s, int j, const AmgLevD& L0, const AmgCg& cg, Slot* slots,
                   SolveState* st, double* part, const AmgDist* d) {
  if (d) upd_bs<ND, kCgBS, true>(s, j, L0, cg, slots, st, part, *d);
  else upd_bs<ND, kCgBS, false>(s, j, L0, cg, slots, st, part, AmgDist{});
}
void launch_amg_cg_update(hipStream_t s, int nd, int j, const AmgLevD& L0, const AmgCg& cg, Slot* slots,
                          SolveState* st, double* part, const AmgDist* d) {
  if (nd == 2) upd_nd<2>(s, j, L0, cg, slots, st, part, d);
  else upd_nd<3>(s, j, L0, cg, slots, st, part, d);
}

void launch_amg_finish(hipStream_t s, int nd, const AmgCg& cg, double* x_row) {
  if (cg.hi <= cg.lo) return;
  if (nd == 2) hipLaunchKernelGGL(k_amg_finish<2>, rows_grid(cg.hi - cg.lo), dim3(kBlock), 0, s, cg, x_row);
  else hipLaunchKernelGGL(k_amg_finish<3>, rows_grid(cg.hi - cg.lo), dim3(kBlock), 0, s, cg, x_row);
}

// ---------------------------------------------------------------------------
// exchanges (distributed V-cycle / setup): pack / unpack of listed items
// ---------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(kBlock) void k_xpack(const T* __restrict__ src, const int32_t* __restrict__ idx,
                                                  int64_t n, int width, T* __restrict__ buf) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n * width) return;
  const int64_t it = k / width, c = k - it * width;
  buf[k] = src[(int64_t)idx[it] * width + c];
}
template <class T>
__global__ __launch_bounds__(kBlock) void k_xunpack(const T* __restrict__ buf, const int32_t* __restrict__ idx,
                                                    int64_t n, int width, T* __restrict__ dst) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n * width) return;
  const int64_t it = k / width, c = k - it * width;
  dst[(int64_t)idx[it] * width + c] = buf[k];
}
// partitions on one device: every (sender, receiver) transfer of an
// exchange in ONE launch, item to item (no staging buffers): pair p moves
// src_p[sidx_p[k]] → dst_p[ridx_p[k]], k < cnt_p, width scalars each
template <class T>
__global__ __launch_bounds__(kBlock) void k_xcopy(XPairs pr, int width) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int p = 0;
  while (p + 1 < pr.n && k >= pr.off[p + 1] * width) ++p;  // (≤ 64 pairs, uniform prefix)
  if (p >= pr.n || k >= pr.off[p + 1] * width) return;
  const int64_t kk = k - pr.off[p] * width, it = kk / width, c = kk - it * width;
  const T* __restrict__ src = (const T*)pr.src[p];
  T* __restrict__ dst = (T*)pr.dst[p];
  dst[(int64_t)pr.ridx[p][it] * width + c] = src[(int64_t)pr.sidx[p][it] * width + c];
}
void launch_xcopy(hipStream_t s, const XPairs& pr, int width, int bytes) {
  if (pr.n <= 0 || pr.off[pr.n] <= 0) return;
  const dim3 g = rows_grid(pr.off[pr.n] * width);
  if (bytes == 8) hipLaunchKernelGGL(k_xcopy<double>, g, dim3(kBlock), 0, s, pr, width);
  else hipLaunchKernelGGL(k_xcopy<float>, g, dim3(kBlock), 0, s, pr, width);
}
// partitions on one device: every partition's 4 CG sums (gsend) into row
// `rank` of every other partition's gathered sums, one launch
__global__ __launch_bounds__(kBlock) void k_gall_copy(GallCopy g) {
  const int t = threadIdx.x, n = g.n;
  for (int idx = t; idx < n * n * 4; idx += kBlock) {
    const int a = idx / (4 * n), b = (idx / 4) % n, c = idx & 3;
    if (a != b) g.gall[b][4 * g.rank[a] + c] = g.gsend[a][c];
  }
}
void launch_gall_copy(hipStream_t s, const GallCopy& g) {
  if (g.n > 1) hipLaunchKernelGGL(k_gall_copy, dim3(1), dim3(kBlock), 0, s, g);
}
void launch_xpack(hipStream_t s, const void* src, const int32_t* idx, int64_t n, int width, int bytes, void* buf) {
  if (n <= 0) return;
  if (bytes == 8)
    hipLaunchKernelGGL(k_xpack<double>, rows_grid(n * width), dim3(kBlock), 0, s, (const double*)src, idx, n, width,
                       (double*)buf);
  else
    hipLaunchKernelGGL(k_xpack<float>, rows_grid(n * width), dim3(kBlock), 0, s, (const float*)src, idx, n, width,
                       (float*)buf);
}
void launch_xunpack(hipStream_t s, const void* buf, const int32_t* idx, int64_t n, int width, int bytes, void* dst) {
  if (n <= 0) return;
  if (bytes == 8)
    hipLaunchKernelGGL(k_xunpack<double>, rows_grid(n * width), dim3(kBlock), 0, s, (const double*)buf, idx, n,
                       width, (double*)dst);
  else
    hipLaunchKernelGGL(k_xunpack<float>, rows_grid(n * width), dim3(kBlock), 0, s, (const float*)buf, idx, n, width,
                       (float*)dst);
}
template <int ND>
__global__ __launch_bounds__(kBlock) void k_amg_xinit_rows(AmgLevD N, const int32_t* __restrict__ rows, int64_t n,
                                                           const int32_t* gate) {
  const bool run = gate_open(gate);
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const int64_t i = rows[k];
  const float sc = N.coarsest ? 1.0f : (float)amg_omega(N.omega);
  float bc[ND], Di[ND * ND], xn[ND];
  vload<ND>(N.b, i, bc);
  dinv_load<ND>(N.dinv32, i, Di);
  dinv_mul<ND>(Di, sc, bc, xn);
  if (run) vstore<ND>(N.x, i, xn);
}
void launch_amg_xinit_rows(hipStream_t s, int nd, const AmgLevD& N, const int32_t* rows, int64_t n,
                           const int32_t* gate) {
  if (n <= 0) return;
  if (nd == 2) hipLaunchKernelGGL(k_amg_xinit_rows<2>, rows_grid(n), dim3(kBlock), 0, s, N, rows, n, gate);
  else hipLaunchKernelGGL(k_amg_xinit_rows<3>, rows_grid(n), dim3(kBlock), 0, s, N, rows, n, gate);
}

struct OmegaPtrs {
  double* p[kMaxRanks];
};
__global__ void k_amg_bound_max(OmegaPtrs o, int n) {
  if (threadIdx.x != 0) return;
  double m = 0.0;
  for (int k = 0; k < n; ++k) m = fmax(m, o.p[k][1]);
  for (int k = 0; k < n; ++k) o.p[k][1] = m;
}
void launch_amg_bound_max(hipStream_t s, double* const* omegas, int n) {
  OmegaPtrs o{};
  for (int k = 0; k < n && k < kMaxRanks; ++k) o.p[k] = omegas[k];
  hipLaunchKernelGGL(k_amg_bound_max, dim3(1), dim3(64), 0, s, o, n < kMaxRanks ? n : kMaxRanks);
}

}  // namespace mfea
