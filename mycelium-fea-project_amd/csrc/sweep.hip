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
// One lane walks one piece: its rows are coupled in a chain (each to its
// predecessor), so the step-to-step dependence is one block product held in
// registers; the pieces of a colour are independent, one launch per colour
// and sweep direction (the last colour's backward sweep rides in its forward
// launch: 2C − 1 launches per application).  A step's entry arrays are
// step-major over the wave's 64 pieces (coalesced); the few cross couplings
// (piece ends, branch and fusion points) are short per-entry lists.
//
// Arithmetic in f64 throughout (the iterate y / z is stored f64); the
// operator values are f32 (pv, lov, upv, D̃⁻¹), the SAME stored values in
// both sweeps, so M⁻¹ is applied as a fixed symmetric operator up to f64
// rounding — what keeps a CG of thousands of iterations at the 1e-10 bar.
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

// Per solve, after A_0's values: the sweeps' operator values from A_0's f64
// blocks — pv (predecessor), lov / upv (cross), D̃⁻¹.  ICC: one launch per
// colour (a pivot reads the pivots of earlier colours' cross neighbours);
// SOR: every colour in one launch.
template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_setup(SweepD sw, AmgMatD A, int c0, int c1) {
  const int32_t w = sweep_wave(sw, c0, c1);
  if (w < 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t e0 = sw.wbase[w] + lane;
  const int len = sw.wlen[w];
  double Dprev[ND * ND];
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) Dprev[c] = 0.0;
  for (int s = 0; s < len; ++s) {
    const int64_t e = e0 + 64 * (int64_t)s;
    if (sw.row[e] < 0) break;  // past this piece's end
    double D[ND * ND], T[ND * ND], Di[ND * ND];
    bload_sym<ND>(A.sym, 0, sw.dpos[e], D);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) T[c] = D[c];
    if (s > 0) {
      double P[ND * ND];
      bload_sym<ND>(A.sym, 0, sw.ppos[e], P);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) sw.pv[e * (ND * ND) + c] = (float)P[c];
      if (sw.dic) sub_xdxt<ND>(P, Dprev, T);
    }
    for (int t = sw.lo_ptr[e]; t < sw.lo_ptr[e + 1]; ++t) {
      double X[ND * ND];
      bload_sym<ND>(A.sym, 0, sw.lo_pos[t], X);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) sw.lov[(int64_t)t * (ND * ND) + c] = (float)X[c];
      if (sw.dic) {
        double Dj[ND * ND];
        load_dt<ND>(sw.dt, sw.lo_ent[t], Dj);
        sub_xdxt<ND>(X, Dj, T);
      }
    }
    for (int t = sw.up_ptr[e]; t < sw.up_ptr[e + 1]; ++t) {
      double X[ND * ND];
      bload_sym<ND>(A.sym, 0, sw.up_pos[t], X);
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) sw.upv[(int64_t)t * (ND * ND) + c] = (float)X[c];
    }
    binv<ND>(sw.dic && spd<ND>(T) ? T : D, Di);
    bstore_sym<ND>(sw.dt, 0, e, Di);
#pragma unroll
    for (int c = 0; c < ND * ND; ++c) Dprev[c] = Di[c];
  }
}

// backward sweep of one lane's piece, steps len−1 … 0 (the lane's y holds
// the forward iterate; z overwrites it); u = z for the CG (gated store)
template <int ND>
__device__ __forceinline__ void piece_backward(const SweepD& sw, const AmgCg& cg, int64_t e0, int len, bool run) {
  double zn[ND], Pn[ND * ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) zn[a] = 0.0;
#pragma unroll
  for (int c = 0; c < ND * ND; ++c) Pn[c] = 0.0;
  for (int s = len - 1; s >= 0; --s) {
    const int64_t e = e0 + 64 * (int64_t)s;
    const int32_t v = sw.row[e];
    if (v < 0) continue;  // padding past the piece's end: z = 0, no coupling
    double y[ND], Dt[ND * ND], acc[ND], P[ND * ND];
    vload<ND>(sw.y, e, y);
    load_dt<ND>(sw.dt, e, Dt);
    if (s > 0) load_blk<ND>(sw.pv, e, P);
#pragma unroll
    for (int a = 0; a < ND; ++a) acc[a] = 0.0;
    bmv<ND, true, false>(Pn, zn, acc);  // A_{i,next} z_next = (A_{next,i})ᵀ z_next
    for (int t = sw.up_ptr[e]; t < sw.up_ptr[e + 1]; ++t) {
      double X[ND * ND], zj[ND];
      load_blk<ND>(sw.upv, t, X);
      vload<ND>(sw.y, sw.up_ent[t], zj);
      bmv<ND, false, false>(X, zj, acc);
    }
    double z[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) z[a] = y[a];
    bmv<ND, false, true>(Dt, acc, z);
    vstore<ND>(sw.y, e, z);
    if (run) vstore<ND>(cg.u, v, z);
#pragma unroll
    for (int a = 0; a < ND; ++a) zn[a] = z[a];
    if (s > 0) {
#pragma unroll
      for (int c = 0; c < ND * ND; ++c) Pn[c] = P[c];
    }
  }
}

// forward sweep of colour c: y over its pieces; LAST (the last colour): the
// backward sweep of the same pieces follows in the same lane
template <int ND, bool LAST>
__global__ __launch_bounds__(kSweepBS) void k_sweep_fwd(SweepD sw, AmgCg cg, int c, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int32_t w = sweep_wave(sw, c, c + 1);
  if (w < 0) return;
  const int lane = threadIdx.x & 63;
  const int64_t e0 = sw.wbase[w] + lane;
  const int len = sw.wlen[w];
  double yp[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) yp[a] = 0.0;
  int n = 0;  // the lane's piece length
  // one step of look-ahead: the next step's operands are loaded before this
  // step's products (only yp chains the steps)
  int32_t v = sw.row[e0];
  double rn[ND], Pn[ND * ND], Dn[ND * ND];
  if (v >= 0) {
    vload<ND>(cg.r, v, rn);
    load_dt<ND>(sw.dt, e0, Dn);
  }
  for (int s = 0; s < len && v >= 0; ++s) {
    const int64_t e = e0 + 64 * (int64_t)s;
    double t[ND], Dt[ND * ND], P[ND * ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) t[a] = rn[a];
#pragma unroll
    for (int k = 0; k < ND * ND; ++k) Dt[k] = Dn[k];
    if (s > 0) {
#pragma unroll
      for (int k = 0; k < ND * ND; ++k) P[k] = Pn[k];
    }
    const int32_t vn = s + 1 < len ? sw.row[e + 64] : -1;
    if (vn >= 0) {
      vload<ND>(cg.r, vn, rn);
      load_dt<ND>(sw.dt, e + 64, Dn);
      load_blk<ND>(sw.pv, e + 64, Pn);
    }
    if (s > 0) bmv<ND, false, true>(P, yp, t);
    for (int k = sw.lo_ptr[e]; k < sw.lo_ptr[e + 1]; ++k) {
      double X[ND * ND], yj[ND];
      load_blk<ND>(sw.lov, k, X);
      vload<ND>(sw.y, sw.lo_ent[k], yj);
      bmv<ND, false, true>(X, yj, t);
    }
    double y[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0;
    bmv<ND, false, false>(Dt, t, y);
    vstore<ND>(sw.y, e, y);
#pragma unroll
    for (int a = 0; a < ND; ++a) yp[a] = y[a];
    ++n;
    v = vn;
  }
  if constexpr (LAST) piece_backward<ND>(sw, cg, e0, n, run);
}

template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_bwd(SweepD sw, AmgCg cg, int c, const int32_t* gate) {
  const bool run = gate_open(gate);
  const int32_t w = sweep_wave(sw, c, c + 1);
  if (w < 0) return;
  piece_backward<ND>(sw, cg, sw.wbase[w] + (threadIdx.x & 63), sw.wlen[w], run);
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
