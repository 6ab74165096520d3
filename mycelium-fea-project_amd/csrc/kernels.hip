// kernels.hip — hand-written CDNA4 kernels of the mfea engine.  See kernels.hpp for
// the HBM layout and DESIGN.md for the roofline of each kernel.
//
// Compiled with -ffp-contract=off: the assembly and stress kernels restate the
// reference's rounding sequence (src/fea_solver.py:30-68, 260-272) and must not
// have products fused into adds behind our back.  The PCG kernels use explicit
// fma() where fusion is wanted.
#include "kernels.hpp"
#include "device_util.hpp"

#include <math.h>

namespace mfea {

// ---------------------------------------------------------------------------
// launch geometry
// ---------------------------------------------------------------------------
int64_t grid_rows(int64_t rows) { return rows <= 0 ? 0 : (rows + kBlock - 1) / kBlock; }
int64_t grid_elementwise(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  return g < 1 ? 1 : (g > 2048 ? 2048 : g);  // ≥ 8 blocks per CU, grid-stride beyond
}


// ---------------------------------------------------------------------------
// Element stiffness S_e (the 3×3 block of Ke = [[S,−S],[−S,S]]),
// src/fea_solver.py:30-68 / src/fea_petsc.cpp:88-140, same rounding sequence as
// the NumPy reference: L = √((vx²+vy²)+vz²), L_safe = max(L,1e-12), n = v/L_safe,
// k_ax = EA/L_safe, k_b = EI12/L_safe³, S_ab = (n_a n_b)·k_ax + (δ_ab − n_a n_b)·k_b.
// L_safe³ is formed in double-double (≈0.5 ulp; NumPy's pow is ≤1 ulp).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double cube(double a) {
  const double s = a * a;
  const double es = fma(a, a, -s);
  const double c = s * a;
  const double ec = fma(s, a, -c);
  return c + (ec + es * a);
}

__device__ __forceinline__ void bar_block(double vx, double vy, double vz, const Material& m,
                                          double S[6], double* Lout) {
  const double L = sqrt(vx * vx + vy * vy + vz * vz);
  const double Ls = L < 1e-12 ? 1e-12 : L;
  const double n0 = vx / Ls, n1 = vy / Ls, n2 = vz / Ls;
  const double kax = m.EA / Ls;
  const double kb = m.EI12 / cube(Ls);
  const double t00 = n0 * n0, t01 = n0 * n1, t02 = n0 * n2, t11 = n1 * n1, t12 = n1 * n2,
               t22 = n2 * n2;
  S[0] = t00 * kax + (1.0 - t00) * kb;
  S[1] = t01 * kax + (0.0 - t01) * kb;
  S[2] = t02 * kax + (0.0 - t02) * kb;
  S[3] = t11 * kax + (1.0 - t11) * kb;
  S[4] = t12 * kax + (0.0 - t12) * kb;
  S[5] = t22 * kax + (1.0 - t22) * kb;
  if (Lout) *Lout = L;
}

// ---------------------------------------------------------------------------
// Assembly: owner-computes gather into the SELL-64 pattern.  One thread per
// node row; each slot (incident element) recomputes S_e from the two endpoint
// coordinates, writes −S_e (or 0 for an inactive element) with a fully
// coalesced SoA store, and accumulates the diagonal block in element order
// (= scipy's duplicate-summation order, src/fea_solver.py:105).  No atomics,
// no colouring, one launch, bitwise deterministic.
// ---------------------------------------------------------------------------
// One node row of the assembly; q (a free row of the GAMG solves): also
// K_fk x_k into k3 — k_amg_rhs's sum of the stored −S_e terms in slot order,
// the same bits.
__device__ __forceinline__ void assemble_row(int64_t N, int64_t row, const double* __restrict__ xyz,
                                             const int32_t* __restrict__ slice_ptr,
                                             const int32_t* __restrict__ row_len,
                                             const int32_t* __restrict__ s_col,
                                             const int32_t* __restrict__ s_elem,
                                             const uint8_t* __restrict__ active, const Material& m,
                                             int64_t G, double* __restrict__ val, double* __restrict__ diag,
                                             const AsmRhs* q, double* k3) {
  const bool rhs = q != nullptr && row < q->nf;
  const int64_t base = (int64_t)slice_ptr[row >> 6] * 64 + (row & 63);
  const int len = row_len[row];
  const double xi = xyz[3 * row], yi = xyz[3 * row + 1], zi = xyz[3 * row + 2];
  double d[6] = {0, 0, 0, 0, 0, 0};
  // slots in batches of U, each batch's loads issued together (slot → element
  // and column, then activity and coordinates): two dependent round trips per
  // batch instead of two per slot; the sums stay in slot order
  constexpr int U = 4;
  for (int k0 = 0; k0 < len; k0 += U) {
    // every load unconditional (a slot past the row's end re-reads its
    // batch's first slot, k0 < len), the masks applied after: a guarded or
    // selected load made hipcc branch per slot and wait vmcnt(0) in each
    // branch — the batch's gathers had run one slot at a time
    int64_t idx[U];
    int32_t e[U], j[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ok[u] = k0 + u < len;
      idx[u] = base + (int64_t)(ok[u] ? k0 + u : k0) * 64;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      e[u] = s_elem[idx[u]];
      j[u] = s_col[idx[u]];
    }
    uint8_t act[U], cd[U];
    double pj[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t av = active[e[u]];
      act[u] = ok[u] ? av : 0;
      // the neighbour's class from its row position (no load: a select on a
      // loaded code made codegen branch around the load and wait in it)
      cd[u] = rhs && ok[u] && j[u] >= q->nf ? (j[u] < q->top_end ? 1 : j[u] < q->bot_end ? 2 : 3) : 3;
#pragma unroll
      for (int a = 0; a < 3; ++a) pj[u][a] = xyz[3 * (int64_t)j[u] + a];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + u >= len) break;
      double S[6] = {0, 0, 0, 0, 0, 0};
      if (act[u]) {
        // v = p2 − p1 with the row as either endpoint: the sign of v does not
        // change any product n_a n_b, so S is bitwise endpoint-symmetric.
        bar_block(pj[u][0] - xi, pj[u][1] - yi, pj[u][2] - zi, m, S, nullptr);
#pragma unroll
        for (int c = 0; c < 6; ++c) d[c] += S[c];
      }
      double v[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) v[c] = -S[c];
#pragma unroll
      for (int c = 0; c < 6; ++c) val[(int64_t)c * G + idx[u]] = v[c];
      if (cd[u] != 3) {  // a known neighbour (3: free or ghost free row, x₀ = 0)
        const double dy = cd[u] == 2 ? q->dy_bot : q->dy_top;
        k3[0] = fma(v[1], dy, k3[0]);
        k3[1] = fma(v[3], dy, k3[1]);
        k3[2] = fma(v[4], dy, k3[2]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) diag[(int64_t)c * N + row] = d[c];
}

// ---------------------------------------------------------------------------
// Assembly, element-centric (option "asm_kernel" 1; north_star's "one
// wavefront per element batch … colour-partitioned writes"): one lane per
// element of a 64-element batch of ONE colour (symbolic.hpp ElemColour).
// S_e — the bar's BᵀDB, which for this element is k_ax nnᵀ + k_b (I − nnᵀ):
// six values — is formed ONCE per element in registers (the row gather forms
// it twice, once per endpoint row), −S_e goes to the element's slot in each
// endpoint row, and +S_e is added to both rows' diagonal blocks: no two
// elements of a colour share a node, so the colour's launch adds without
// atomics, and the colours run in order — deterministic.  Same S bits as the
// row gather (bar_block is endpoint-symmetric); the diagonal sums run in
// colour order instead of slot order (within a few ulps).  diag is zeroed
// before the first colour.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_assemble_colour(int64_t e0, int64_t e1, const int32_t* __restrict__ entry,
                                                            const int32_t* __restrict__ e2n,
                                                            const int32_t* __restrict__ epos,
                                                            const double* __restrict__ xyz,
                                                            const uint8_t* __restrict__ active, Material m,
                                                            int64_t G, int64_t N, double* __restrict__ val,
                                                            double* __restrict__ diag) {
  const int64_t k = e0 + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= e1) return;
  const int32_t e = entry[k];
  if (e < 0) return;
  const int32_t a = e2n[2 * e], b = e2n[2 * e + 1];
  const int32_t pa = epos[2 * e], pb = epos[2 * e + 1];
  double S[6] = {0, 0, 0, 0, 0, 0};
  if (active[e])
    bar_block(xyz[3 * (int64_t)b] - xyz[3 * (int64_t)a], xyz[3 * (int64_t)b + 1] - xyz[3 * (int64_t)a + 1],
              xyz[3 * (int64_t)b + 2] - xyz[3 * (int64_t)a + 2], m, S, nullptr);
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    val[(int64_t)c * G + pa] = -S[c];
    val[(int64_t)c * G + pb] = -S[c];
  }
  double da[6], db[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    da[c] = diag[(int64_t)c * N + a];
    db[c] = diag[(int64_t)c * N + b];
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    diag[(int64_t)c * N + a] = da[c] + S[c];
    diag[(int64_t)c * N + b] = db[c] + S[c];
  }
}

// Assembly, element pass + row pass (option "asm_kernel" 2): one lane per
// element forms S_e once and writes −S_e to its two slots (no two elements
// share a slot: no conflicts, no colours, one launch); then one lane per row
// sums −val over its slots in slot order into the diagonal block — the row
// gather's own order, so K is bit for bit the row gather's.
__global__ __launch_bounds__(kBlock) void k_assemble_elems(int64_t E, const int32_t* __restrict__ e2n,
                                                           const int32_t* __restrict__ epos,
                                                           const double* __restrict__ xyz,
                                                           const uint8_t* __restrict__ active, Material m,
                                                           int64_t G, double* __restrict__ val) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= E) return;
  const int32_t pa = epos[2 * e], pb = epos[2 * e + 1];
  if (pa < 0) return;
  const int32_t a = e2n[2 * e], b = e2n[2 * e + 1];
  double S[6] = {0, 0, 0, 0, 0, 0};
  if (active[e])
    bar_block(xyz[3 * (int64_t)b] - xyz[3 * (int64_t)a], xyz[3 * (int64_t)b + 1] - xyz[3 * (int64_t)a + 1],
              xyz[3 * (int64_t)b + 2] - xyz[3 * (int64_t)a + 2], m, S, nullptr);
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    val[(int64_t)c * G + pa] = -S[c];
    val[(int64_t)c * G + pb] = -S[c];
  }
}

__global__ __launch_bounds__(kBlock) void k_diag_rows(int64_t N, const int32_t* __restrict__ slice_ptr,
                                                      const int32_t* __restrict__ row_len, int64_t G,
                                                      const double* __restrict__ val, double* __restrict__ diag) {
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (row >= N) return;
  const int64_t base = (int64_t)slice_ptr[row >> 6] * 64 + (row & 63);
  const int len = row_len[row];
  double d[6] = {0, 0, 0, 0, 0, 0};
  for (int k = 0; k < len; ++k) {
#pragma unroll
    for (int c = 0; c < 6; ++c) d[c] += -val[(int64_t)c * G + base + (int64_t)k * 64];
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) diag[(int64_t)c * N + row] = d[c];
}

// RHS: the GAMG solves' RHS too (AsmRhs: k_amg_rhs's outputs from the −S_e
// blocks in registers) — one launch fewer per step
template <bool RHS>
__global__ __launch_bounds__(kBlock) void k_assemble(int64_t N, const double* __restrict__ xyz,
                                                     const int32_t* __restrict__ slice_ptr,
                                                     const int32_t* __restrict__ row_len,
                                                     const int32_t* __restrict__ s_col,
                                                     const int32_t* __restrict__ s_elem,
                                                     const uint8_t* __restrict__ active,
                                                     Material m, int64_t G, double* __restrict__ val,
                                                     double* __restrict__ diag, AsmRhs q) {
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if constexpr (RHS) {
    if (q.dyp) {
      q.dy_top = q.dyp[0];
      q.dy_bot = q.dyp[1];
    }
    double acc[2] = {0.0, 0.0};
    if (row < N) {
      double k3[3] = {0.0, 0.0, 0.0};
      assemble_row(N, row, xyz, slice_ptr, row_len, s_col, s_elem, active, m, G, val, diag, &q, k3);
      if (row < q.nf) {
        const double b[3] = {0.0 - k3[0], 0.0 - k3[1], 0.0 - k3[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a) q.r[3 * row + a] = b[a];
#pragma unroll
        for (int a = 0; a < 3; ++a) acc[0] = fma(b[a], b[a], acc[0]);
      } else {
        const uint8_t c = q.code[row];
        const double xk[3] = {0.0, c == 3 ? 0.0 : (c == 2 ? q.dy_bot : q.dy_top), 0.0};
#pragma unroll
        for (int a = 0; a < 3; ++a) q.x[3 * row + a] = xk[a];
      }
    }
    block_publish<2>(acc, q.partials, q.ticket, q.red_out);
  } else {
    if (row < N) assemble_row(N, row, xyz, slice_ptr, row_len, s_col, s_elem, active, m, G, val, diag, nullptr, nullptr);
  }
}

// ---------------------------------------------------------------------------
// Dirichlet elimination + PCG start (src/fea_solver.py:115-125;
// src/fea_petsc.cpp:286-320).  Free rows: b_i = −Σ_{known j} K_ij x_j,
// x=0, r=b, z=M⁻¹b, p=z.  Known rows: x = prescribed (0, dy, 0), p = 0 so the
// free-row SpMV sees K_fk·p = 0.  Reduces (r·z, b·b, z·z).
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void k_rhs_init(
    int64_t N, int64_t nf, const int32_t* __restrict__ slice_ptr, const int32_t* __restrict__ row_len,
    const int32_t* __restrict__ s_col, const double* __restrict__ val, const double* __restrict__ diag,
    int64_t G, const uint8_t* __restrict__ code, double dy_top, double dy_bot, double reg,
    int precond, double* __restrict__ x, double* __restrict__ r, double* __restrict__ p,
    double* __restrict__ dinv, double* partials, unsigned* ticket, double* red_out) {
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double acc[3] = {0.0, 0.0, 0.0};  // r·z, b·b, z·z
  if (row < nf) {
    const int64_t base = (int64_t)slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = row_len[row];
    double kx = 0.0, ky = 0.0, kz = 0.0;  // (K_fk · x_k) for this row
    for (int k = 0; k < len; ++k) {
      const int64_t idx = base + (int64_t)k * 64;
      const int32_t j = s_col[idx];
      if (j >= nf) {
        const double dy = code[j] == 2 ? dy_bot : dy_top;  // only the y DOF is nonzero
        kx = fma(val[1 * G + idx], dy, kx);
        ky = fma(val[3 * G + idx], dy, ky);
        kz = fma(val[4 * G + idx], dy, kz);
      }
    }
    const double b[3] = {0.0 - kx, 0.0 - ky, 0.0 - kz};  // F_f = 0 − K_fk x_k (py:122)
    double A[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) A[c] = diag[(int64_t)c * N + row];
    A[0] += reg; A[3] += reg; A[5] += reg;                // K_ff + reg·I (py:125)
    double z[3];
    if (precond == 1) {
      double B[6];
      sym_inverse(A, B);
#pragma unroll
      for (int c = 0; c < 6; ++c) dinv[6 * row + c] = B[c];
      sym_apply(B, b, z);
    } else {
      const double d0 = 1.0 / A[0], d1 = 1.0 / A[3], d2 = 1.0 / A[5];
      dinv[3 * row] = d0; dinv[3 * row + 1] = d1; dinv[3 * row + 2] = d2;
      z[0] = d0 * b[0]; z[1] = d1 * b[1]; z[2] = d2 * b[2];
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      x[3 * row + a] = 0.0;
      r[3 * row + a] = b[a];
      p[3 * row + a] = z[a];
      acc[0] = fma(b[a], z[a], acc[0]);
      acc[1] = fma(b[a], b[a], acc[1]);
      acc[2] = fma(z[a], z[a], acc[2]);
    }
  } else if (row < N) {
    x[3 * row] = 0.0;
    x[3 * row + 1] = code[row] == 2 ? dy_bot : dy_top;
    x[3 * row + 2] = 0.0;
    p[3 * row] = 0.0; p[3 * row + 1] = 0.0; p[3 * row + 2] = 0.0;
  }
  block_publish<3>(acc, partials, ticket, red_out);
}

__global__ void k_init_finalize(const double* red, double rtol, double atol, int norm, int max_it,
                                double reg, Slot* slots, SolveState* st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double rz = red[0], bb = red[1], zz = red[2];
  const double ref = norm == 1 ? zz : bb;
  const double t = rtol * rtol * ref, a2 = atol * atol;
  st->tol2 = t > a2 ? t : a2;
  st->reg = reg;
  st->bb0 = bb;
  st->res_final = ref;
  st->res0 = ref;
  st->base = 0;
  st->max_it = max_it;
  st->norm = norm;
  st->done = 0;
  st->iters = 0;
  st->status = 0;
  Slot s0;
  s0.v[0] = 0.0; s0.v[1] = rz; s0.v[2] = bb; s0.v[3] = zz;
  s0.flag = kRun;
  slots[0] = s0;
}

// run(j): iteration base+j executes.  Pure function of globally reduced values,
// so every block (and, multi-GPU, every rank) agrees.
__device__ __forceinline__ bool run_iter(const Slot* slots, const SolveState* st, int j) {
  const Slot& s = slots[j];
  const double res = st->norm == 1 ? s.v[3] : s.v[2];
  return s.flag == kRun && res > st->tol2 && (st->base + j) < st->max_it;
}

// ---------------------------------------------------------------------------
// SpMV  q = (K_ff + reg·I) p  over the free rows, fused with the partial p·q.
// SELL-64: lane l of the wave owning slice s handles row 64 s + l; slot k of
// that row sits at (slice_ptr[s] + k)·64 + l, so every column/value load of a
// wave is one contiguous 256/512-byte transaction.  p is gathered per
// neighbour (24 B, L2/MALL-resident for meshes up to ~10 M DOF).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_spmv_sell(
    int j, int64_t nf, int64_t N, const int32_t* __restrict__ slice_ptr,
    const int32_t* __restrict__ row_len, const int32_t* __restrict__ s_col,
    const double* __restrict__ val, const double* __restrict__ diag, int64_t G,
    const double* __restrict__ p, double* __restrict__ q, Slot* slots, const SolveState* st,
    double* partials, unsigned* ticket) {
  if (!run_iter(slots, st, j)) return;
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double pq[1] = {0.0};
  if (row < nf) {
    const double reg = st->reg;
    const int64_t base = (int64_t)slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = row_len[row];
    const double p0 = p[3 * row], p1 = p[3 * row + 1], p2 = p[3 * row + 2];
    const double d0 = diag[row], d1 = diag[N + row], d2 = diag[2 * N + row],
                 d3 = diag[3 * N + row], d4 = diag[4 * N + row], d5 = diag[5 * N + row];
    double y0 = fma(d0 + reg, p0, fma(d1, p1, d2 * p2));
    double y1 = fma(d1, p0, fma(d3 + reg, p1, d4 * p2));
    double y2 = fma(d2, p0, fma(d4, p1, (d5 + reg) * p2));
    for (int k = 0; k < len; ++k) {
      const int64_t idx = base + (int64_t)k * 64;
      const int64_t c = s_col[idx];
      const double v0 = val[idx], v1 = val[G + idx], v2 = val[2 * G + idx],
                   v3 = val[3 * G + idx], v4 = val[4 * G + idx], v5 = val[5 * G + idx];
      const double q0 = p[3 * c], q1 = p[3 * c + 1], q2 = p[3 * c + 2];
      y0 = fma(v0, q0, fma(v1, q1, fma(v2, q2, y0)));
      y1 = fma(v1, q0, fma(v3, q1, fma(v4, q2, y1)));
      y2 = fma(v2, q0, fma(v4, q1, fma(v5, q2, y2)));
    }
    q[3 * row] = y0; q[3 * row + 1] = y1; q[3 * row + 2] = y2;
    pq[0] = fma(p0, y0, fma(p1, y1, p2 * y2));
  }
  block_publish<1>(pq, partials, ticket, &slots[j].v[0]);
}

// ---------------------------------------------------------------------------
// x += α p ; r −= α q ; z = M⁻¹ r ; reduce (r·z, r·r, z·z) into slot j+1.
// ---------------------------------------------------------------------------
template <bool BLOCK>
__global__ __launch_bounds__(kBlock) void k_update(int j, int64_t n, double* __restrict__ x,
                                                   double* __restrict__ r,
                                                   const double* __restrict__ p,
                                                   const double* __restrict__ q,
                                                   const double* __restrict__ dinv, Slot* slots,
                                                   const SolveState* st, double* partials,
                                                   unsigned* ticket) {
  if (!run_iter(slots, st, j)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) slots[j + 1].flag = kStop;
    return;
  }
  const double pq = slots[j].v[0];
  const double alpha = slots[j].v[1] / pq;
  if (!(pq > 0.0) || !isfinite(alpha)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      slots[j + 1].v[1] = 0.0; slots[j + 1].v[2] = 0.0; slots[j + 1].v[3] = 0.0;
      slots[j + 1].flag = kBreakdown;
    }
    return;
  }
  double acc[3] = {0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  if (!BLOCK) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
      x[i] = fma(alpha, p[i], x[i]);
      const double ri = fma(-alpha, q[i], r[i]);
      r[i] = ri;
      const double zi = dinv[i] * ri;
      acc[0] = fma(ri, zi, acc[0]);
      acc[1] = fma(ri, ri, acc[1]);
      acc[2] = fma(zi, zi, acc[2]);
    }
  } else {
    for (int64_t nd = (int64_t)blockIdx.x * kBlock + threadIdx.x; nd < n / 3; nd += stride) {
      double rv[3], zv[3], B[6];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int64_t i = 3 * nd + a;
        x[i] = fma(alpha, p[i], x[i]);
        rv[a] = fma(-alpha, q[i], r[i]);
        r[i] = rv[a];
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) B[c] = dinv[6 * nd + c];
      sym_apply(B, rv, zv);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        acc[0] = fma(rv[a], zv[a], acc[0]);
        acc[1] = fma(rv[a], rv[a], acc[1]);
        acc[2] = fma(zv[a], zv[a], acc[2]);
      }
    }
  }
  if (block_publish<3>(acc, partials, ticket, &slots[j + 1].v[1]) && threadIdx.x == 0)
    slots[j + 1].flag = kRun;
}

// p = M⁻¹ r + β p, β = (r·z)_{j+1} / (r·z)_j — only if iteration j+1 will run.
template <bool BLOCK>
__global__ __launch_bounds__(kBlock) void k_direction(int j, int64_t n, const double* __restrict__ r,
                                                      double* __restrict__ p,
                                                      const double* __restrict__ dinv,
                                                      const Slot* slots, const SolveState* st) {
  if (!run_iter(slots, st, j + 1)) return;
  const double beta = slots[j + 1].v[1] / slots[j].v[1];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  if (!BLOCK) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
      p[i] = fma(beta, p[i], dinv[i] * r[i]);
  } else {
    for (int64_t nd = (int64_t)blockIdx.x * kBlock + threadIdx.x; nd < n / 3; nd += stride) {
      double rv[3], zv[3], B[6];
#pragma unroll
      for (int a = 0; a < 3; ++a) rv[a] = r[3 * nd + a];
#pragma unroll
      for (int c = 0; c < 6; ++c) B[c] = dinv[6 * nd + c];
      sym_apply(B, rv, zv);
#pragma unroll
      for (int a = 0; a < 3; ++a) p[3 * nd + a] = fma(beta, p[3 * nd + a], zv[a]);
    }
  }
}

// End of a chunk of `chunk` iterations: record the stop point or roll slot
// `chunk` into slot 0.  Once done, slot 0 is poisoned STOP so any chunk the
// host has already queued is a no-op.
__global__ void k_advance(int chunk, Slot* slots, SolveState* st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (st->done) return;
  for (int j = 0; j <= chunk; ++j) {
    if (!run_iter(slots, st, j)) {
      const Slot& s = slots[j];
      const double res = st->norm == 1 ? s.v[3] : s.v[2];
      st->iters = st->base + j;
      st->res_final = res;
      if (s.flag == kBreakdown) st->status = -5;
      else if (s.flag == kRun && res <= st->tol2) st->status = 0;
      else if (s.flag == kRun) st->status = -4;
      else st->status = -5;  // kStop without a recorded reason cannot happen
      st->done = 1;
      slots[0].flag = kStop;
      return;
    }
  }
  slots[0] = slots[chunk];
  st->base += chunk;
}

// ---------------------------------------------------------------------------
// Reaction: Σ over top grip rows of (K·U)_y with the unregularised K
// (src/fea_solver.py:252-254, src/fea_petsc.cpp:360-372).  Top rows are a
// contiguous range of the permutation.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_reaction(int64_t row0, int64_t nrows, int64_t N,
                                                     const int32_t* __restrict__ slice_ptr,
                                                     const int32_t* __restrict__ row_len,
                                                     const int32_t* __restrict__ s_col,
                                                     const double* __restrict__ val,
                                                     const double* __restrict__ diag, int64_t G,
                                                     const double* __restrict__ u, double* partials,
                                                     unsigned* ticket, double* red_out) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double f[1] = {0.0};
  if (t < nrows) {
    const int64_t row = row0 + t;
    const int64_t base = (int64_t)slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = row_len[row];
    double fy = diag[N + row] * u[3 * row] + diag[3 * N + row] * u[3 * row + 1] +
                diag[4 * N + row] * u[3 * row + 2];
    // slots in batches of four, each batch's columns and values issued before
    // its gathers (one latency chain per batch, not per slot); the padding
    // lanes of a batch re-read slot k0 and add nothing.  Terms in slot order.
    constexpr int U = 4;
    for (int k0 = 0; k0 < len; k0 += U) {
      int64_t idx[U], c[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        idx[q] = base + (int64_t)(k0 + q < len ? k0 + q : k0) * 64;
        c[q] = s_col[idx[q]];
      }
      double t[U];
#pragma unroll
      for (int q = 0; q < U; ++q)
        t[q] = val[G + idx[q]] * u[3 * c[q]] + val[3 * G + idx[q]] * u[3 * c[q] + 1] +
               val[4 * G + idx[q]] * u[3 * c[q] + 2];
#pragma unroll
      for (int q = 0; q < U; ++q)
        if (k0 + q < len) fy += t[q];
    }
    f[0] = fy;
  }
  block_publish<1>(f, partials, ticket, red_out);
}

// ---------------------------------------------------------------------------
// Stress / failure, src/fea_solver.py:259-274: for elements active at step
// start, ε = (n·(u2−u1))/L with n = v/L (no L clamp in Python), the dot product
// as BLAS ddot forms it (fma chain x0y0 → +x1y1 → +x2y2), σ = E·ε, deactivate
// if |ε| > max_strain.  Inactive elements record σ = 0.  Reduces #active.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_stress(int64_t E, const int32_t* __restrict__ e2n,
                                                   const double* __restrict__ xyz,
                                                   const double* __restrict__ u, Material m,
                                                   double max_strain, uint8_t* __restrict__ active,
                                                   double* __restrict__ stress, double* partials,
                                                   unsigned* ticket, double* red_out,
                                                   const uint8_t* __restrict__ owned,
                                                   int32_t* __restrict__ fail_list, unsigned* fail_cnt) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double cnt[1] = {0.0};
  if (e < E) {
    const int32_t a = e2n[2 * e], b = e2n[2 * e + 1];
    const uint8_t act0 = active[e];
    uint8_t act = act0;
    double sg = 0.0;
    if (act && a >= 0) {
      const double vx = xyz[3 * b] - xyz[3 * a], vy = xyz[3 * b + 1] - xyz[3 * a + 1],
                   vz = xyz[3 * b + 2] - xyz[3 * a + 2];
      // np.linalg.norm of one 3-vector = sqrt(v·v) through BLAS ddot (py:266)
      const double L = sqrt(fma(vz, vz, fma(vy, vy, vx * vx)));
      const double n0 = vx / L, n1 = vy / L, n2 = vz / L;
      const double du0 = u[3 * b] - u[3 * a], du1 = u[3 * b + 1] - u[3 * a + 1],
                   du2 = u[3 * b + 2] - u[3 * a + 2];
      const double dot = fma(n2, du2, fma(n1, du1, n0 * du0));
      const double strain = dot / L;
      sg = m.E * strain;
      if (fabs(strain) > max_strain) act = 0;
      active[e] = act;
    }
    stress[e] = sg;
    cnt[0] = (act && (!owned || owned[e])) ? 1.0 : 0.0;
    // an (owned) element failing now joins the list (any order): the host's
    // activity then moves by these ids instead of an E-byte copy or reduction
    // (capi.hip post_impl / apply_failures)
    if (fail_list && act0 && !act && (!owned || owned[e])) fail_list[atomicAdd(fail_cnt, 1u)] = (int32_t)e;
  }
  block_publish<1>(cnt, partials, ticket, red_out);
}

// Undo a post's failures (capi.hip spec_undo): the elements k_stress listed
// are active again and the list's counter is zero — a post enqueued behind a
// CG batch that turned out not to be the last one leaves no trace
__global__ __launch_bounds__(kBlock) void k_unfail(const int32_t* __restrict__ fail_list, unsigned* cnt,
                                                   uint8_t* __restrict__ active) {
  const unsigned c = *cnt;
  for (unsigned k = threadIdx.x; k < c; k += kBlock) active[fail_list[k]] = 1;
  __syncthreads();
  if (threadIdx.x == 0) *cnt = 0u;
}

// ---------------------------------------------------------------------------
// Floating free rows on the device: connected components of the active
// element graph, then per component whether a grip row is in it.  A free
// row of a component without a grip is floating: zero load, so the direct
// solve leaves it at exactly zero (src/fea_solver.py:128) and the kept GAMG
// hierarchy masks its P_0 row (capi.hip enqueue_fmask).  Replaces a host
// union-find over every element per new active set.
//
// The rows are in depth-first order of the free-node graph (symbolic.hpp):
// hyphal chains are runs of consecutive rows, so nearly every coupling joins
// two rows of the same 4096-row tile.  Pass 1 (one workgroup per tile) runs
// union-find over the tile's own couplings in LDS and links every row to its
// tile-local root; pass 2 hooks the few couplings between tiles into those
// roots with CAS in HBM; pass 3 flattens.  Roots only ever link under smaller
// rows, so every component ends at its smallest row whatever order the
// hooks ran in: the result is deterministic.
// ---------------------------------------------------------------------------
constexpr int kSlice = 64;  // SELL-64 rows per slice (symbolic.hpp)

__device__ __forceinline__ int32_t cc_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the root of v, halving the path behind it (a parent only ever moves to a
// smaller row of the same component, so a racing shortcut stays valid)
__device__ __forceinline__ int32_t cc_root(int32_t* parent, int32_t v) {
  int32_t cur = cc_load(parent + v);
  if (cur != v) {
    int32_t prev = v, next;
    while (cur > (next = cc_load(parent + cur))) {
      __hip_atomic_store(parent + prev, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prev = cur;
      cur = next;
    }
  }
  return cur;
}

__device__ __forceinline__ int32_t lds_root(volatile int32_t* lp, int32_t v) {
  int32_t cur = lp[v], next;
  if (cur != v) {
    int32_t prev = v;
    while (cur > (next = lp[cur])) {
      lp[prev] = next;
      prev = cur;
      cur = next;
    }
  }
  return cur;
}

// pass 1: union-find over the couplings inside one tile of rows, in LDS;
// parent[row] = its tile-local root (a global row), anchored[row] = 0
template <int kCcTile>
__global__ __launch_bounds__(kBlock) void k_cc_local(int64_t n, const int32_t* __restrict__ slice_ptr,
                                                     const int32_t* __restrict__ row_len,
                                                     const int32_t* __restrict__ s_col,
                                                     const int32_t* __restrict__ s_elem,
                                                     const uint8_t* __restrict__ active, int32_t* __restrict__ parent,
                                                     uint8_t* __restrict__ anchored) {
  __shared__ int32_t lp[kCcTile];
  const int64_t base = (int64_t)blockIdx.x * kCcTile;
  const int rows = (int)min<int64_t>(kCcTile, n - base);
  for (int i = threadIdx.x; i < rows; i += kBlock) lp[i] = i;
  __syncthreads();
  for (int i = threadIdx.x; i < rows; i += kBlock) {
    const int64_t r = base + i;
    const int len = row_len[r];
    const int64_t p0 = (int64_t)slice_ptr[r >> 6] * kSlice + (r & 63);
    for (int k = 0; k < len; ++k) {
      const int64_t pos = p0 + (int64_t)k * kSlice;
      const int32_t c = s_col[pos];
      const int64_t j = (int64_t)c - base;
      if (c < 0 || j <= i || j >= rows || !active[s_elem[pos]]) continue;
      int32_t a = lds_root(lp, i), b = lds_root(lp, (int32_t)j);
      while (a != b) {  // hook the larger root under the smaller
        if (a > b) {
          const int32_t t = a;
          a = b;
          b = t;
        }
        const int32_t old = atomicCAS(&lp[b], b, a);
        if (old == b) break;
        b = lds_root(lp, old);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < rows; i += kBlock) {
    int32_t c = lp[i], next;
    while (c > (next = lp[c])) c = next;
    parent[base + i] = (int32_t)(base + c);
    anchored[base + i] = 0;
  }
}

// pass 2: the couplings between tiles hook tile roots together (CAS in HBM)
__global__ __launch_bounds__(kBlock) void k_cc_cross(int64_t n, const int32_t* __restrict__ slice_ptr,
                                                     const int32_t* __restrict__ row_len,
                                                     const int32_t* __restrict__ s_col,
                                                     const int32_t* __restrict__ s_elem,
                                                     const uint8_t* __restrict__ active, int32_t* parent,
                                                     int tile_rows) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  const int len = row_len[r];
  const int64_t p0 = (int64_t)slice_ptr[r >> 6] * kSlice + (r & 63);
  const int64_t tile = r / tile_rows;
  for (int k = 0; k < len; ++k) {
    const int64_t pos = p0 + (int64_t)k * kSlice;
    const int32_t c = s_col[pos];
    if (c <= r || c / tile_rows == tile || !active[s_elem[pos]]) continue;
    int32_t a = cc_root(parent, (int32_t)r), b = cc_root(parent, c);
    while (a != b) {
      if (a > b) {
        const int32_t t = a;
        a = b;
        b = t;
      }
      const int32_t old = atomicCAS(parent + b, b, a);
      if (old == b) break;
      b = cc_root(parent, old);
    }
  }
}

// pass 3: every row's parent to its root (the walk writes nothing but the
// row's own link, so a concurrent walk reads either link — both lead to the
// root); grip rows [g0, g1) mark their root anchored
__global__ __launch_bounds__(kBlock) void k_cc_flatten(int64_t n, int32_t* parent, int64_t g0, int64_t g1,
                                                       uint8_t* __restrict__ anchored) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int32_t old = cc_load(parent + i);
  int32_t r = old, next;
  while (r > (next = cc_load(parent + r))) r = next;
  if (r != old) __hip_atomic_store(parent + i, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (i >= g0 && i < g1) anchored[r] = 1;
}

// mask[label[i]] = 1 iff free row i's component holds no grip row
__global__ __launch_bounds__(kBlock) void k_cc_mask(int64_t nf, const int32_t* __restrict__ parent,
                                                    const uint8_t* __restrict__ anchored,
                                                    const int32_t* __restrict__ label, uint8_t* __restrict__ mask) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= nf) return;
  mask[label ? label[i] : i] = anchored[parent[i]] ? 0 : 1;
}

__global__ __launch_bounds__(kBlock) void k_element_stiffness(int64_t n, const double* __restrict__ p1,
                                                              const double* __restrict__ p2,
                                                              Material m, double* __restrict__ Ke,
                                                              double* __restrict__ L) {
  const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  double S[6], l;
  bar_block(p2[3 * e] - p1[3 * e], p2[3 * e + 1] - p1[3 * e + 1], p2[3 * e + 2] - p1[3 * e + 2], m,
            S, &l);
  L[e] = l;
  const int sidx[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) {
      const double v = S[sidx[a % 3][b % 3]];
      Ke[36 * e + 6 * a + b] = ((a < 3) == (b < 3)) ? v : -v;
    }
}

// ---------------------------------------------------------------------------
// Generic scalar CSR operator for solve_system(K, known_dofs, known_vals)
// with a caller-supplied K (src/fea_solver.py:112-135).  Known DOFs keep
// dinv = 0, r = 0, p = 0, so the shared update/direction kernels run over all
// n DOFs unmasked and never move a prescribed value.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_csr_rhs_init(
    int64_t n, const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const double* __restrict__ data, const uint8_t* __restrict__ known, const double* __restrict__ kval,
    double reg, double* __restrict__ x, double* __restrict__ r, double* __restrict__ p,
    double* __restrict__ dinv, double* partials, unsigned* ticket, double* red_out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double acc[3] = {0.0, 0.0, 0.0};
  if (i < n) {
    if (known[i]) {
      x[i] = kval[i]; r[i] = 0.0; p[i] = 0.0; dinv[i] = 0.0;
    } else {
      double kx = 0.0, dii = 0.0;
      for (int64_t t = indptr[i]; t < indptr[i + 1]; ++t) {
        const int32_t c = indices[t];
        if (known[c]) kx = fma(data[t], kval[c], kx);
        if (c == i) dii += data[t];
      }
      const double b = 0.0 - kx;
      const double d = 1.0 / (dii + reg);
      const double z = d * b;
      x[i] = 0.0; r[i] = b; p[i] = z; dinv[i] = d;
      acc[0] = b * z; acc[1] = b * b; acc[2] = z * z;
    }
  }
  block_publish<3>(acc, partials, ticket, red_out);
}

__global__ __launch_bounds__(kBlock) void k_spmv_csr(int j, int64_t n, const int64_t* __restrict__ indptr,
                                                     const int32_t* __restrict__ indices,
                                                     const double* __restrict__ data,
                                                     const uint8_t* __restrict__ known, double reg,
                                                     const double* __restrict__ p,
                                                     double* __restrict__ q, Slot* slots,
                                                     const SolveState* st, double* partials,
                                                     unsigned* ticket) {
  if (!run_iter(slots, st, j)) return;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double pq[1] = {0.0};
  if (i < n) {
    double y = 0.0;
    if (!known[i]) {
      y = reg * p[i];
      for (int64_t t = indptr[i]; t < indptr[i + 1]; ++t) y = fma(data[t], p[indices[t]], y);
    }
    q[i] = y;
    pq[0] = p[i] * y;
  }
  block_publish<1>(pq, partials, ticket, &slots[j].v[0]);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
#define MFEA_GRID(n) dim3((unsigned)(n)), dim3(kBlock), 0, s

void launch_assemble(hipStream_t s, int64_t N, const double* xyz, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const int32_t* s_elem,
                     const uint8_t* active, Material m, int64_t G, double* val, double* diag,
                     const AsmRhs* rhs) {
  if (rhs) {  // (the reduction's blocks publish even when N = 0)
    hipLaunchKernelGGL(k_assemble<true>, MFEA_GRID(grid_rows(N > 0 ? N : 1)), N, xyz, slice_ptr, row_len, s_col,
                       s_elem, active, m, G, val, diag, *rhs);
    return;
  }
  if (N <= 0) return;
  hipLaunchKernelGGL(k_assemble<false>, MFEA_GRID(grid_rows(N)), N, xyz, slice_ptr, row_len, s_col, s_elem,
                     active, m, G, val, diag, AsmRhs{});
}

void launch_assemble_colour(hipStream_t s, int colors, const int32_t* cstart, const int32_t* entry,
                            const int32_t* e2n, const int32_t* epos, const double* xyz, const uint8_t* active,
                            Material m, int64_t G, int64_t N, double* val, double* diag) {
  if (N > 0) (void)hipMemsetAsync(diag, 0, (size_t)6 * N * sizeof(double), s);
  for (int c = 0; c < colors; ++c) {
    const int64_t e0 = cstart[c], e1 = cstart[c + 1];
    if (e1 > e0)
      hipLaunchKernelGGL(k_assemble_colour, MFEA_GRID(grid_rows(e1 - e0)), e0, e1, entry, e2n, epos, xyz, active, m,
                         G, N, val, diag);
  }
}

void launch_assemble_elems(hipStream_t s, int64_t E, int64_t N, const int32_t* e2n, const int32_t* epos,
                           const double* xyz, const uint8_t* active, Material m, const int32_t* slice_ptr,
                           const int32_t* row_len, int64_t G, double* val, double* diag) {
  if (E > 0) hipLaunchKernelGGL(k_assemble_elems, MFEA_GRID(grid_rows(E)), E, e2n, epos, xyz, active, m, G, val);
  if (N > 0) hipLaunchKernelGGL(k_diag_rows, MFEA_GRID(grid_rows(N)), N, slice_ptr, row_len, G, val, diag);
}

void launch_rhs_init(hipStream_t s, int64_t N, int64_t nf, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const double* val,
                     const double* diag, int64_t G, const uint8_t* code, double dy_top,
                     double dy_bot, double reg, int precond, double* x, double* r, double* p,
                     double* dinv, double* partials, unsigned* ticket, double* red_out) {
  hipLaunchKernelGGL(k_rhs_init, MFEA_GRID(grid_rows(N > 0 ? N : 1)), N, nf, slice_ptr, row_len, s_col,
                     val, diag, G, code, dy_top, dy_bot, reg, precond, x, r, p, dinv, partials,
                     ticket, red_out);
}

void launch_init_finalize(hipStream_t s, const double* red, double rtol, double atol, int norm,
                          int max_it, double reg, Slot* slots, SolveState* st) {
  hipLaunchKernelGGL(k_init_finalize, dim3(1), dim3(64), 0, s, red, rtol, atol, norm, max_it, reg,
                     slots, st);
}

void launch_spmv_sell(hipStream_t s, int j, int64_t nf, int64_t N, const int32_t* slice_ptr,
                      const int32_t* row_len, const int32_t* s_col, const double* val,
                      const double* diag, int64_t G, const double* p, double* q, Slot* slots,
                      const SolveState* st, double* partials, unsigned* ticket) {
  hipLaunchKernelGGL(k_spmv_sell, MFEA_GRID(grid_rows(nf > 0 ? nf : 1)), j, nf, N, slice_ptr,
                     row_len, s_col, val, diag, G, p, q, slots, st, partials, ticket);
}

void launch_update(hipStream_t s, int j, int64_t n, int precond, double* x, double* r,
                   const double* p, const double* q, const double* dinv, Slot* slots,
                   const SolveState* st, double* partials, unsigned* ticket) {
  if (precond == 1)
    hipLaunchKernelGGL(k_update<true>, MFEA_GRID(grid_elementwise(n / 3)), j, n, x, r, p, q, dinv,
                       slots, st, partials, ticket);
  else
    hipLaunchKernelGGL(k_update<false>, MFEA_GRID(grid_elementwise(n)), j, n, x, r, p, q, dinv,
                       slots, st, partials, ticket);
}

void launch_direction(hipStream_t s, int j, int64_t n, int precond, const double* r, double* p,
                      const double* dinv, const Slot* slots, const SolveState* st) {
  if (precond == 1)
    hipLaunchKernelGGL(k_direction<true>, MFEA_GRID(grid_elementwise(n / 3)), j, n, r, p, dinv,
                       slots, st);
  else
    hipLaunchKernelGGL(k_direction<false>, MFEA_GRID(grid_elementwise(n)), j, n, r, p, dinv, slots,
                       st);
}

void launch_advance(hipStream_t s, int chunk, Slot* slots, SolveState* st) {
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(64), 0, s, chunk, slots, st);
}

void launch_reaction(hipStream_t s, int64_t row0, int64_t nrows, int64_t N,
                     const int32_t* slice_ptr, const int32_t* row_len, const int32_t* s_col,
                     const double* val, const double* diag, int64_t G, const double* u,
                     double* partials, unsigned* ticket, double* red_out) {
  hipLaunchKernelGGL(k_reaction, MFEA_GRID(grid_rows(nrows > 0 ? nrows : 1)), row0, nrows, N,
                     slice_ptr, row_len, s_col, val, diag, G, u, partials, ticket, red_out);
}

void launch_stress(hipStream_t s, int64_t E, const int32_t* e2n, const double* xyz,
                   const double* u, Material m, double max_strain, uint8_t* active,
                   double* stress, double* partials, unsigned* ticket, double* red_out,
                   const uint8_t* owned, int32_t* fail_list, unsigned* fail_cnt) {
  hipLaunchKernelGGL(k_stress, MFEA_GRID(grid_rows(E > 0 ? E : 1)), E, e2n, xyz, u, m, max_strain,
                     active, stress, partials, ticket, red_out, owned, fail_list, fail_cnt);
}

void launch_unfail(hipStream_t s, const int32_t* fail_list, unsigned* cnt, uint8_t* active) {
  hipLaunchKernelGGL(k_unfail, dim3(1), dim3(kBlock), 0, s, fail_list, cnt, active);
}

void launch_floating(hipStream_t s, int64_t n_rows, int64_t n_free, int64_t grip_end, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const int32_t* s_elem, const uint8_t* active,
                     int32_t* parent, uint8_t* anchored, const int32_t* label, uint8_t* mask, int tile_rows) {
  if (n_free <= 0) return;
  tile_rows = tile_rows == 512 || tile_rows == 1024 || tile_rows == 4096 ? tile_rows : 2048;
  const int64_t tiles = (n_rows + tile_rows - 1) / tile_rows;
  auto local = tile_rows == 512 ? k_cc_local<512> : tile_rows == 1024 ? k_cc_local<1024>
               : tile_rows == 4096 ? k_cc_local<4096> : k_cc_local<2048>;
  hipLaunchKernelGGL(local, MFEA_GRID(tiles), n_rows, slice_ptr, row_len, s_col, s_elem, active, parent, anchored);
  hipLaunchKernelGGL(k_cc_cross, MFEA_GRID(grid_rows(n_rows)), n_rows, slice_ptr, row_len, s_col, s_elem, active,
                     parent, tile_rows);
  hipLaunchKernelGGL(k_cc_flatten, MFEA_GRID(grid_rows(n_rows)), n_rows, parent, n_free, grip_end, anchored);
  hipLaunchKernelGGL(k_cc_mask, MFEA_GRID(grid_rows(n_free)), n_free, parent, anchored, label, mask);
}

void launch_element_stiffness(hipStream_t s, int64_t n, const double* p1, const double* p2,
                              Material m, double* Ke, double* L) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_element_stiffness, MFEA_GRID(grid_rows(n)), n, p1, p2, m, Ke, L);
}

void launch_csr_rhs_init(hipStream_t s, int64_t n, const int64_t* indptr, const int32_t* indices,
                         const double* data, const uint8_t* known, const double* kval, double reg,
                         double* x, double* r, double* p, double* dinv, double* partials,
                         unsigned* ticket, double* red_out) {
  hipLaunchKernelGGL(k_csr_rhs_init, MFEA_GRID(grid_rows(n > 0 ? n : 1)), n, indptr, indices, data,
                     known, kval, reg, x, r, p, dinv, partials, ticket, red_out);
}

void launch_spmv_csr(hipStream_t s, int j, int64_t n, const int64_t* indptr,
                     const int32_t* indices, const double* data, const uint8_t* known,
                     double reg, const double* p, double* q, Slot* slots, const SolveState* st,
                     double* partials, unsigned* ticket) {
  hipLaunchKernelGGL(k_spmv_csr, MFEA_GRID(grid_rows(n > 0 ? n : 1)), j, n, indptr, indices, data,
                     known, reg, p, q, slots, st, partials, ticket);
}

}  // namespace mfea
