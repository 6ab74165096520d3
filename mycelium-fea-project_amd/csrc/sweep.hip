// sweep.hip — block-Jacobi multicolour SSOR / DIC(0) preconditioners for the
// PCG solve (MFEA_PC_SOR, MFEA_PC_ICC): the MI355X-native counterparts of the
// reference's `-pc_type sor` and its source default PCICC
// (src/fea_petsc.cpp:331; the sweep src/fea_petsc_solverAndPC.cpp:331 runs
// KSPCG × {jacobi, sor, ilu, icc, gamg}).
//
// Layout (amg.hpp SweepPlan): the AMG plan's level-0 rows (node blocks of
// A_0 = K_ff + reg·I, depth-first order: hyphal chains contiguous) in blocks
// of 256 consecutive rows, one workgroup each.  Couplings between blocks are
// dropped — PETSc's SOR and ICC are processor-local in parallel, so this is
// its semantics with a 256-row "rank" per workgroup — and inside a block the
// rows are coloured (greedy, in row order), so the rows of one colour are
// independent and each triangular sweep is C workgroup-barrier phases, all in
// ONE launch per application.  With L / U the in-block couplings to earlier /
// later colours and D̃ a block diagonal:
//   M = (D̃ + L) D̃⁻¹ (D̃ + U)
//   forward   y_i = D̃_i⁻¹ (r_i − Σ_{j∈L(i)} A_ij y_j)     colours 0 … C−1
//   backward  z_i = y_i − D̃_i⁻¹ Σ_{j∈U(i)} A_ij z_j       colours C−1 … 0
// SOR (SSOR, ω = 1, PETSc's default): D̃ = D.  ICC: DIC(0), the incomplete
// Cholesky factor with the off-diagonal blocks of A and the diagonal
// D̃_i = D_i − Σ_{j∈L(i)} A_ij D̃_j⁻¹ A_ijᵀ (exact IC(0) wherever the coloured
// graph has no triangles; PETSc's ICC(0) on the natural order otherwise
// differs only in the triangle corrections).  A D̃_i that is not positive
// definite falls back to D_i (PETSc shifts such pivots), so M stays SPD.  The
// sweep runs in f32 (the CG around it in f64, as the GAMG cycle).
#include "amg_dev.hpp"

namespace mfea {

constexpr int kSweepBS = kSweepRows;  // = SweepPlan::rows_per_block

// 2×2 / 3×3 block SPD test for the DIC pivot: leading minors positive
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

// DIC(0) diagonal per block, colour by colour (after A_0's values and D⁻¹):
// D̃_i⁻¹ → sw.dt32
template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_dic(SweepD sw, AmgLevD L0) {
  __shared__ double dti[kSweepBS * ND * ND];  // D̃_j⁻¹ of the block's rows
  const int64_t i = (int64_t)blockIdx.x * kSweepBS + threadIdx.x;
  const bool valid = i < sw.n;
  const int c_i = valid ? sw.color[i] : -1;
  double D[ND * ND], Di[ND * ND];
  if (valid) bload<ND>(L0.A.val32, 0, (int64_t)L0.A.sptr[i >> 6] * 64 + (i & 63), D);
  for (int c = 0; c < sw.colors; ++c) {
    if (c == c_i) {
      double T[ND * ND];
#pragma unroll
      for (int e = 0; e < ND * ND; ++e) T[e] = D[e];
      for (int t = sw.lo_ptr[i]; t < sw.lo_ptr[i + 1]; ++t) {
        double a[ND * ND], ad[ND * ND], dj[ND * ND];
        bload<ND>(L0.A.val32, 0, sw.lo_pos[t], a);
        bload<ND>(dti, 0, sw.lo_loc[t], dj);
#pragma unroll
        for (int e = 0; e < ND * ND; ++e) ad[e] = 0.0;
        mm_acc<ND>(a, dj, ad);  // A_ij D̃_j⁻¹
#pragma unroll
        for (int x = 0; x < ND; ++x)
#pragma unroll
          for (int y = 0; y < ND; ++y) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < ND; ++k) s = fma(ad[x * ND + k], a[y * ND + k], s);  // (A D̃⁻¹ Aᵀ)_xy
            T[x * ND + y] -= s;
          }
      }
      binv<ND>(spd<ND>(T) ? T : D, Di);
#pragma unroll
      for (int e = 0; e < ND * ND; ++e) dti[threadIdx.x * ND * ND + e] = Di[e];
    }
    __syncthreads();
  }
  if (valid) bstore<ND>(sw.dt32, 0, i, &dti[threadIdx.x * ND * ND]);
}

// u = M⁻¹ r for every row (the CG's f64 r in, its f32 u out); gate: the
// iteration's flag, tested before the store only (as the V-cycle's kernels)
template <int ND>
__global__ __launch_bounds__(kSweepBS) void k_sweep_apply(SweepD sw, AmgLevD L0, AmgCg cg, const int32_t* gate) {
  __shared__ float ys[kSweepBS * ND];
  const bool run = gate_open(gate);
  const int64_t i = (int64_t)blockIdx.x * kSweepBS + threadIdx.x;
  const bool valid = i < sw.n;
  const int c_i = valid ? sw.color[i] : -1;
  float rf[ND], Dt[ND * ND];
  if (valid) {
#pragma unroll
    for (int a = 0; a < ND; ++a) rf[a] = (float)cg.r[ND * i + a];
    dinv_load<ND>(sw.dt32, i, Dt);
  }
  for (int c = 0; c < sw.colors; ++c) {  // forward: (D̃ + L) y = r
    if (c == c_i) {
      float t[ND], y[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a) t[a] = rf[a];
      for (int k = sw.lo_ptr[i]; k < sw.lo_ptr[i + 1]; ++k) {
        float m[ND * ND], yj[ND];
        bload<ND>(L0.A.val32, 0, sw.lo_pos[k], m);
        vload<ND>(ys, sw.lo_loc[k], yj);
#pragma unroll
        for (int a = 0; a < ND; ++a)
#pragma unroll
          for (int b = 0; b < ND; ++b) t[a] = fmaf(-m[a * ND + b], yj[b], t[a]);
      }
      dinv_mul<ND>(Dt, 1.0f, t, y);
      vstore<ND>(ys, threadIdx.x, y);
    }
    __syncthreads();
  }
  for (int c = sw.colors - 1; c >= 0; --c) {  // backward: z = y − D̃⁻¹ U z
    if (c == c_i) {
      float s[ND], y[ND], d[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a) s[a] = 0.0f;
      for (int k = sw.up_ptr[i]; k < sw.up_ptr[i + 1]; ++k) {
        float m[ND * ND], zj[ND];
        bload<ND>(L0.A.val32, 0, sw.up_pos[k], m);
        vload<ND>(ys, sw.up_loc[k], zj);
#pragma unroll
        for (int a = 0; a < ND; ++a)
#pragma unroll
          for (int b = 0; b < ND; ++b) s[a] = fmaf(m[a * ND + b], zj[b], s[a]);
      }
      dinv_mul<ND>(Dt, 1.0f, s, d);
      vload<ND>(ys, threadIdx.x, y);
#pragma unroll
      for (int a = 0; a < ND; ++a) y[a] -= d[a];
      vstore<ND>(ys, threadIdx.x, y);
    }
    __syncthreads();
  }
  if (valid && run) {
    float z[ND];
    vload<ND>(ys, threadIdx.x, z);
    vstore<ND>(cg.u, i, z);
  }
}

static dim3 sweep_grid(int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n + kSweepBS - 1) / kSweepBS)); }

void launch_sweep_setup(hipStream_t s, int nd, const SweepD& sw, const AmgLevD& L0) {
  if (!sw.dic || sw.n <= 0) return;
  if (nd == 2) hipLaunchKernelGGL(k_sweep_dic<2>, sweep_grid(sw.n), dim3(kSweepBS), 0, s, sw, L0);
  else hipLaunchKernelGGL(k_sweep_dic<3>, sweep_grid(sw.n), dim3(kSweepBS), 0, s, sw, L0);
}

void launch_sweep(hipStream_t s, int nd, const SweepD& sw, const AmgLevD& L0, const AmgCg& cg, const int32_t* gate) {
  if (sw.n <= 0) return;
  if (nd == 2) hipLaunchKernelGGL(k_sweep_apply<2>, sweep_grid(sw.n), dim3(kSweepBS), 0, s, sw, L0, cg, gate);
  else hipLaunchKernelGGL(k_sweep_apply<3>, sweep_grid(sw.n), dim3(kSweepBS), 0, s, sw, L0, cg, gate);
}

}  // namespace mfea
