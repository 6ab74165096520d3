// sweep.hip — whole-matrix SSOR / IC(0) preconditioners for the PCG solve
// (MFEA_PC_SOR, MFEA_PC_ICC): the MI355X-native counterparts of the
// reference's `-pc_type sor` and its source default PCICC (src/fea_petsc.cpp:331;
// the sweep src/fea_petsc_solverAndPC.cpp:331 runs KSPCG × {jacobi, sor, ilu,
// icc, gamg}).
//
// The factorisation is of the WHOLE free system A_0 = K_ff + reg·I (node
// blocks, ND×ND) in the chain-piece multicolour order of amg.hpp SweepPlan:
// colour → piece → step.  With L the block lower part in that order and D̃ a
// block diagonal,
//   M = (D̃ + L) D̃⁻¹ (D̃ + Lᵀ)
//   forward   y_i = D̃_i⁻¹ (r_i − Σ_{j<i} A_ij y_j)     colours 0 … C−1
//   backward  z_i = y_i − D̃_i⁻¹ Σ_{j>i} A_ij z_j       colours C−1 … 0
// SOR (SSOR, ω = 1, PETSc's default): D̃ = D.  ICC: DIC(0), the pivots
// D̃_i = D_i − Σ_{j<i} A_ij D̃_j⁻¹ A_ijᵀ formed in f64 — IC(0) itself wherever
// no three rows couple pairwise (tools/icc_lab.py: identical iteration counts
// on the reference and the tiled networks); a pivot that is not positive
// definite falls back to D_i (PETSc shifts such pivots), so M stays SPD.
//
// One lane per row: a piece's rows sit on consecutive lanes of one wave, so
// its chain recurrence — forward y_l = g_l + G_l y_{l−1} with
// g_l = D̃_l⁻¹(r_l − Σ_lo A y), G_l = −D̃_l⁻¹ A_{l,l−1}; backward
// z_l = h_l + H_l z_{l+1} with H_l = −D̃_l⁻¹ A_{l+1,l}ᵀ — is an inclusive scan
// of affine maps across the lanes (⌈log₂ piece⌉ shuffle steps; G = 0 at a
// piece's first row, H = 0 at its last, so pieces do not mix).  The pieces of
// a colour are independent: one launch per colour and direction, the last
// colour's backward scan in its forward launch (2C − 1 launches per
// application), every load coalesced except the r / u gathers and the few
// cross couplings (piece ends, branch and fusion points).
//
// Arithmetic in f64 throughout (the iterate y / z is stored f64); the
// operator values are f32 (pv, lov, upv, D̃⁻¹), the SAME stored values in
// both sweeps and the scan's G / H formed from them in f64 registers, so
// M⁻¹ is applied as a fixed symmetric operator up to f64 rounding — what
// keeps a CG of thousands of iterations at the 1e-10 bar.
#include "amg_dev.hpp"

namespace mfea {

// ND×ND / upper-triangle helpers on the f32 stored values
template <int ND>
__device__ __forceinline__ void load_blk(const float* __restrict__ v, int64_t q, double* m) {
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) m[c] = (double)v[q * (ND * ND) + c];
}
template <int ND>
__device__ __forceinline__ void load_dt(const float* __restrict__ v, int64_t q, double* m) {
  bload_sym<ND>(v, 0, q, m);
}
// o = M v (TR: Mᵀ v), accumulated into o with sign
template <int ND, bool TR, bool SUB>
__device__ __forceinline__ void bmv(const double* m, const double* v, double* o) {
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      const double mv = TR ? m[b * ND + a] : m[a * ND + b];
      o[a] = fma(SUB ? -mv : mv, v[b], o[a]);
    }
}

// 2×2 / 3×3 SPD test for the DIC pivot: leading minors positive
template <int ND>
__device__ __forceinline__ bool spd(const double* m) {
  if constexpr (ND == 2) {
    return m[0] > 0.0 && m[0] * m[3] - m[1] * m[2] > 0.0;
  } else {
    const double d2 = m[0] * m[4] - m[1] * m[3];
    const double d3 = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                      m[2] * (m[3] * m[7] - m[4] * m[6]);
    return m[0] > 0.0 && d2 > 0.0 && d3 > 0.0;
  }
}

// the wave this thread's lane belongs to among colours [c0, c1) (−1: none)
__device__ __forceinline__ int32_t sweep_wave(const SweepD& sw, int c0, int c1) {
  const int32_t w = sw.cw[c0] + (int32_t)(blockIdx.x * (kSweepBS / 64) + (threadIdx.x >> 6));
  return w < sw.cw[c1] ? w : -1;
}

// T −= X D Xᵀ (X full, D symmetric)
template <int ND>
__device__ __forceinline__ void sub_xdxt(const double* X, const double* D, double* T) {
  double XD[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) XD[c] = 0.0;
  mm_acc<ND>(X, D, XD);
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < ND; ++k) s = fma(XD[a * ND + k], X[b * ND + k], s);
      T[a * ND + b] -= s;
    }
}

// G = −D X (D symmetric ND×ND, X full); TR: G = −D Xᵀ
template <int ND, bool TR>
__device__ __forceinline__ void neg_dx(const double* D, const double* X, double* G) {
#pragma unroll
  for (int a = 0; a < ND; ++a)
#pragma unroll
    for (int b = 0; b < ND; ++b) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < ND; ++k) s = fma(D[a * ND + k], TR ? X[b * ND + k] : X[k * ND + b], s);
      G[a * ND + b] = -s;
    }
}

// Per solve, after A_0's values: the sweeps' operator values from A_0's f64
// blocks — pv (predecessor), lov / upv (cross), D̃⁻¹.  SOR: every row in
// parallel, every colour in one launch.  ICC: one launch per colour (a pivot
// reads the pivots of earlier colours' cross neighbours), the lane of a
// piece's first row walking the piece's chain of pivots
// D̃_l = D_l − A_{l,l−1} D̃_{l−1}⁻¹ A_{l,l−1}ᵀ − Σ_lo X D̃_j⁻¹ Xᵀ (f64).
template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_setup(SweepD sw, AmgMatD A, int c0, int c1) {
  const int32_t w = sweep_wave(sw, c0, c1);
  if (w < 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t e = 64 * (int64_t)w + lane;
  if (sw.row[e] < 0) return;
  if (sw.ppos[e] >= 0) {
    double P[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.ppos[e], P);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) sw.pv[e * (ND * ND) + c] = (float)P[c];
  }
  for (int t = sw.lo_ptr[e]; t < sw.lo_ptr[e + 1]; ++t) {
    double X[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.lo_pos[t], X);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) sw.lov[(int64_t)t * (ND * ND) + c] = (float)X[c];
  }
  for (int t = sw.up_ptr[e]; t < sw.up_ptr[e + 1]; ++t) {
    double X[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.up_pos[t], X);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) sw.upv[(int64_t)t * (ND * ND) + c] = (float)X[c];
  }
  if (!sw.dic) {
    double D[ND * ND], Di[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.dpos[e], D);
    binv<ND>(D, Di);
    bstore_sym<ND>(sw.dt, 0, e, Di);
    return;
  }
  if (sw.ppos[e] >= 0) return;  // not a piece's first row: its first row's lane walks it
  double Dprev[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) Dprev[c] = 0.0;
  const int64_t wend = 64 * (int64_t)w + 64;
  for (int64_t k = e; k < wend; ++k) {
    if (k > e && sw.ppos[k] < 0) break;  // the next piece (or padding)
    double D[ND * ND], T[ND * ND], Di[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.dpos[k], D);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) T[c] = D[c];
    if (k > e) {
      double P[ND * ND];
      bload_sym<ND>(A.sym, 0, sw.ppos[k], P);
      sub_xdxt<ND>(P, Dprev, T);
    }
    for (int t = sw.lo_ptr[k]; t < sw.lo_ptr[k + 1]; ++t) {
      double X[ND * ND], Dj[ND * ND];
      bload_sym<ND>(A.sym, 0, sw.lo_pos[t], X);
      load_dt<ND>(sw.dt, sw.lo_ent[t], Dj);
      sub_xdxt<ND>(X, Dj, T);
    }
    binv<ND>(spd<ND>(T) ? T : D, Di);
    bstore_sym<ND>(sw.dt, 0, k, Di);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) Dprev[c] = Di[c];
  }
}

// acc ∓= Σ_t X_t y[ent_t] over one entry's cross list [t0, t1): the items'
// loads issued together, four at a time (a branch row has 2–4 crosses; one
// at a time they were four dependent round trips each)
template <int ND, bool SUB>
__device__ __forceinline__ void cross_sum(int t0, int t1, const int32_t* __restrict__ ent,
                                          const float* __restrict__ xv, const double* __restrict__ y, double* acc) {
  constexpr int U = 4;
  for (int t = t0; t < t1; t += U) {
    int32_t j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = ent[t + u < t1 ? t + u : t0];
    double X[U][ND * ND], yj[U][ND];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      load_blk<ND>(xv, t + u < t1 ? t + u : t0, X[u]);
      vload<ND>(y, j[u], yj[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (t + u < t1) bmv<ND, false, SUB>(X[u], yj[u], acc);
  }
}

// the affine-map scan across the wave's lanes: x_l = a_l + M_l x_{l∓1}
// composed over `steps` doubling steps (UP: predecessors are lower lanes)
template <int ND, bool UP>
__device__ __forceinline__ void lane_scan(double* a, double* M, int steps) {
  const int lane = threadIdx.x & 63;
  for (int k = 0; k < steps; ++k) {
    const int d = 1 << k;
    double as[ND], Ms[ND * ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) as[i] = UP ? __shfl_up(a[i], d, 64) : __shfl_down(a[i], d, 64);
#pragma unroll
    for (int i = 0; i < ND * ND; ++i) Ms[i] = UP ? __shfl_up(M[i], d, 64) : __shfl_down(M[i], d, 64);
    if (UP ? lane >= d : lane + d < 64) {
      bmv<ND, false, false>(M, as, a);
      double N[ND * ND];
#pragma unroll
      for (int i = 0; i < ND * ND; ++i) N[i] = 0.0;
      mm_acc<ND>(M, Ms, N);
#pragma unroll
      for (int i = 0; i < ND * ND; ++i) M[i] = N[i];
    }
  }
}

// backward sweep of the lane's row: z = y − D̃⁻¹(A_{l,l+1} z_{l+1} + Σ_up X z_j)
// as a suffix scan; P: the lane's own predecessor block (0 on a first row),
// y: its forward iterate.  Stores z (sw.y) and u = z (gated).
template <int ND>
__device__ __forceinline__ void lane_backward(const SweepD& sw, const AmgCg& cg, int64_t e, int32_t v,
                                              const double* Dt, const double* P, bool hasP, double* y,
                                              int steps, bool run, bool cross) {
  double acc[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) acc[a] = 0.0;
  if (cross && v >= 0) cross_sum<ND, false>(sw.up_ptr[e], sw.up_ptr[e + 1], sw.up_ent, sw.upv, sw.y, acc);
  bmv<ND, false, true>(Dt, acc, y);  // h = y − D̃⁻¹ acc
  // H = −D̃⁻¹ (A_{l+1,l})ᵀ where the next lane continues this piece
  double Pn[ND * ND], H[ND * ND];
#pragma unroll
  for (int i = 0; i < ND * ND; ++i) Pn[i] = __shfl_down(P[i], 1, 64);
  const bool next = __shfl_down(hasP ? 1 : 0, 1, 64) && (threadIdx.x & 63) < 63;
  if (next) neg_dx<ND, true>(Dt, Pn, H);
  else {
#pragma unroll
    for (int i = 0; i < ND * ND; ++i) H[i] = 0.0;
  }
  lane_scan<ND, false>(y, H, steps);
  if (v >= 0) {
    vstore<ND>(sw.y, e, y);
    if (run) vstore<ND>(cg.u, v, y);
  }
}

// forward sweep of wave w (one lane per entry); LAST (the last colour, no
// upper couplings): its backward scan follows in registers
template <int ND, bool LAST>
__device__ __forceinline__ void fwd_wave(const SweepD& sw, const AmgCg& cg, int32_t w, bool run) {
  const int64_t e = 64 * (int64_t)w + (threadIdx.x & 63);
  const int32_t v = sw.row[e];
  const int steps = sw.wsteps[w];
  double g[ND], G[ND * ND], Dt[ND * ND], P[ND * ND];
  bool hasP = false;
#pragma unroll
  for (int i = 0; i < ND; ++i) g[i] = 0.0;
#pragma unroll
  for (int i = 0; i < ND * ND; ++i) {
    G[i] = 0.0;
    P[i] = 0.0;
    Dt[i] = 0.0;
  }
  if (v >= 0) {
    double t[ND];
    vload<ND>(cg.r, v, t);
    load_dt<ND>(sw.dt, e, Dt);
    hasP = sw.ppos[e] >= 0;
    if (hasP) load_blk<ND>(sw.pv, e, P);
    cross_sum<ND, true>(sw.lo_ptr[e], sw.lo_ptr[e + 1], sw.lo_ent, sw.lov, sw.y, t);
    bmv<ND, false, false>(Dt, t, g);
    if (hasP) neg_dx<ND, false>(Dt, P, G);
  }
  lane_scan<ND, true>(g, G, steps);
  if constexpr (LAST) {
    lane_backward<ND>(sw, cg, e, v, Dt, P, hasP, g, steps, run, false);
  } else if (v >= 0) {
    vstore<ND>(sw.y, e, g);
  }
}

template <int ND>
__device__ __forceinline__ void bwd_wave(const SweepD& sw, const AmgCg& cg, int32_t w, bool run) {
  const int64_t e = 64 * (int64_t)w + (threadIdx.x & 63);
  const int32_t v = sw.row[e];
  double y[ND], Dt[ND * ND], P[ND * ND];
  bool hasP = false;
#pragma unroll
  for (int i = 0; i < ND; ++i) y[i] = 0.0;
#pragma unroll
  for (int i = 0; i < ND * ND; ++i) {
    P[i] = 0.0;
    Dt[i] = 0.0;
  }
  if (v >= 0) {
    vload<ND>(sw.y, e, y);
    load_dt<ND>(sw.dt, e, Dt);
    hasP = sw.ppos[e] >= 0;
    if (hasP) load_blk<ND>(sw.pv, e, P);
  }
  lane_backward<ND>(sw, cg, e, v, Dt, P, hasP, y, sw.wsteps[w], run, true);
}

template <int ND, bool LAST>
__global__ __launch_bounds__(kSweepBS) void k_sweep_fwd(SweepD sw, AmgCg cg, int c, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int32_t w = sweep_wave(sw, c, c + 1);
  if (w >= 0) fwd_wave<ND, LAST>(sw, cg, w, run);
}

template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_bwd(SweepD sw, AmgCg cg, int c, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int32_t w = sweep_wave(sw, c, c + 1);
  if (w >= 0) bwd_wave<ND>(sw, cg, w, run);
}

static dim3 sweep_grid(const SweepD& sw, int c0, int c1) {
  const int64_t waves = sw.cw[c1] - sw.cw[c0];
  return dim3((unsigned)std::max<int64_t>(1, (waves + kSweepBS / 64 - 1) / (kSweepBS / 64)));
}
template <int ND>
static void setup_nd(hipStream_t s, const SweepD& sw, const AmgLevD& L0) {
  if (sw.dic) {
    for (int c = 0; c < sw.colors; ++c)
      hipLaunchKernelGGL(k_sweep_setup<ND>, sweep_grid(sw, c, c + 1), dim3(kSweepBS), 0, s, sw, L0.A, c, c + 1);
  } else {
    hipLaunchKernelGGL(k_sweep_setup<ND>, sweep_grid(sw, 0, sw.colors), dim3(kSweepBS), 0, s, sw, L0.A, 0,
                       sw.colors);
  }
}
void launch_sweep_setup(hipStream_t s, int nd, const SweepD& sw, const AmgLevD& L0) {
  if (sw.n <= 0 || sw.colors <= 0) return;
  if (nd == 2) setup_nd<2>(s, sw, L0);
  else setup_nd<3>(s, sw, L0);
}

template <int ND>
static void apply_nd(hipStream_t s, const SweepD& sw, const AmgCg& cg, const int32_t* gate) {
  const int C = sw.colors;
  for (int c = 0; c + 1 < C; ++c)
    hipLaunchKernelGGL((k_sweep_fwd<ND, false>), sweep_grid(sw, c, c + 1), dim3(kSweepBS), 0, s, sw, cg, c, gate);
  hipLaunchKernelGGL((k_sweep_fwd<ND, true>), sweep_grid(sw, C - 1, C), dim3(kSweepBS), 0, s, sw, cg, C - 1, gate);
  for (int c = C - 2; c >= 0; --c)
    hipLaunchKernelGGL(k_sweep_bwd<ND>, sweep_grid(sw, c, c + 1), dim3(kSweepBS), 0, s, sw, cg, c, gate);
}
void launch_sweep(hipStream_t s, int nd, const SweepD& sw, const AmgCg& cg, const int32_t* gate) {
  if (sw.n <= 0 || sw.colors <= 0) return;
  if (nd == 2) apply_nd<2>(s, sw, cg, gate);
  else apply_nd<3>(s, sw, cg, gate);
}

}  // namespace mfea
