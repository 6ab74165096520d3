// cg.hip — single-reduction preconditioned CG (Chronopoulos–Gear) on the SELL-64
// node-block operator: ONE kernel per iteration.
//
// Recurrences (x₀ = 0, u = M⁻¹r, w = A u, s = A p):
//   p_i = u_i + β_i p_{i−1}      s_i = w_i + β_i s_{i−1}
//   x_{i+1} = x_i + α_i p_i      r_{i+1} = r_i − α_i s_i
//   u_{i+1} = M⁻¹ r_{i+1}        w_{i+1} = A u_{i+1}
//   γ = (r,u), δ = (w,u);  β_{i+1} = γ_{i+1}/γ_i,  α_{i+1} = γ_{i+1} / (δ_{i+1} − β_{i+1} γ_{i+1} / α_i)
// In exact arithmetic these are the iterates of textbook PCG (the reference's
// KSPCG, src/fea_petsc.cpp:328); one fused reduction (γ, δ, ‖r‖², ‖u‖²) per
// iteration instead of two.  The SpMV w = A u needs u_j of neighbour rows whose
// owners update r, s, w in the same launch, so r, s, w are double-buffered by
// iteration parity and each row recomputes its neighbours' u_j from the
// previous-iteration values: u_j = M_j⁻¹ (r_j − α (w_j + β s_j)).
//
// Scalar hand-off: the block that completes an iteration's reduction (last
// ticket) also forms α, β and the stopping norm for the next iteration and
// writes them into the next slot, so an iteration kernel starts with plain
// scalar loads and no divisions on its critical path.
#include "device_util.hpp"
#include "kernels.hpp"

namespace mfea {

int cg_block_size(int64_t rows) { return rows <= 64 * 1024 ? 64 : 256; }
int64_t cg_grid(int64_t rows) {
  const int bs = cg_block_size(rows);
  int64_t g = (rows + bs - 1) / bs;
  return g < 1 ? 1 : (g > 2048 ? 2048 : g);
}

template <bool BLOCK>
__device__ __forceinline__ void apply_minv(const double* __restrict__ dinv, int64_t row,
                                           const double r[3], double u[3]) {
  if (BLOCK) {
    double B[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) B[c] = dinv[6 * row + c];
    sym_apply(B, r, u);
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) u[a] = dinv[3 * row + a] * r[a];
  }
}

__device__ __forceinline__ void load3(const double* __restrict__ v, int64_t row, double o[3]) {
  o[0] = v[3 * row];
  o[1] = v[3 * row + 1];
  o[2] = v[3 * row + 2];
}
__device__ __forceinline__ void store3(double* __restrict__ v, int64_t row, const double o[3]) {
  v[3 * row] = o[0];
  v[3 * row + 1] = o[1];
  v[3 * row + 2] = o[2];
}

// y += V u with V the symmetric block (v0..v5)
__device__ __forceinline__ void block_mac(const double V[6], const double u[3], double y[3]) {
  y[0] = fma(V[0], u[0], fma(V[1], u[1], fma(V[2], u[2], y[0])));
  y[1] = fma(V[1], u[0], fma(V[3], u[1], fma(V[4], u[2], y[1])));
  y[2] = fma(V[2], u[0], fma(V[4], u[1], fma(V[5], u[2], y[2])));
}

// Finalize the scalars of slot `s` from its freshly reduced sums (thread 0 of
// the reducing block).  prev = the slot whose α, γ the iteration consumed
// (nullptr for the first reduction: β = 0, α = γ/δ).
__device__ __forceinline__ void finalize_slot(Slot* s, const Slot* prev, int norm) {
  const double g = s->v[0], d = s->v[1];
  double beta = 0.0, den = d;
  if (prev) {
    beta = g / prev->v[0];
    den = d - beta * g / prev->alpha;
  }
  const double alpha = g / den;
  s->alpha = alpha;
  s->beta = beta;
  s->res = norm == 1 ? s->v[3] : s->v[2];
  const bool ok = (den > 0.0) && isfinite(alpha) && isfinite(beta);
  // γ = 0 ⇔ r = 0: converged, not a breakdown (the stopping test catches it)
  s->flag = (ok || g == 0.0) ? kRun : kBreakdown;
}

// ---------------------------------------------------------------------------
// Dirichlet elimination / RHS (src/fea_solver.py:115-125; src/fea_petsc.cpp:286-320)
// Free rows: b = 0 − K_fk x_k (only the y DOF of a grip node is nonzero),
// M⁻¹ from K_ii + reg·I, x = 0, r₀ = b, p = s = 0.  Known rows: x = (0, dy, 0),
// every Krylov vector and M⁻¹ = 0, so gathers across the boundary read zeros.
// ---------------------------------------------------------------------------
template <bool BLOCK>
__global__ __launch_bounds__(kBlock) void k_cg_rhs(SellOp op, const uint8_t* __restrict__ code,
                                                   double dy_top, double dy_bot, double reg,
                                                   CgVecs v, double* partials, unsigned* ticket,
                                                   double* red_out) {
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double acc[2] = {0.0, 0.0};  // b·b, u₀·u₀
  const double zero[3] = {0.0, 0.0, 0.0};
  if (row < op.nf) {
    const int64_t base = (int64_t)op.slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = op.row_len[row];
    const int64_t G = op.G;
    double kx = 0.0, ky = 0.0, kz = 0.0;
    for (int k = 0; k < len; ++k) {
      const int64_t idx = base + (int64_t)k * 64;
      const int32_t j = op.s_col[idx];
      if (j >= op.nf) {
        const double dy = code[j] == 2 ? dy_bot : dy_top;
        kx = fma(op.val[1 * G + idx], dy, kx);
        ky = fma(op.val[3 * G + idx], dy, ky);
        kz = fma(op.val[4 * G + idx], dy, kz);
      }
    }
    const double b[3] = {0.0 - kx, 0.0 - ky, 0.0 - kz};
    double A[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) A[c] = op.diag[(int64_t)c * op.N + row];
    A[0] += reg;
    A[3] += reg;
    A[5] += reg;
    double u[3];
    if (BLOCK) {
      double B[6];
      sym_inverse(A, B);
#pragma unroll
      for (int c = 0; c < 6; ++c) v.dinv[6 * row + c] = B[c];
      sym_apply(B, b, u);
    } else {
      const double d[3] = {1.0 / A[0], 1.0 / A[3], 1.0 / A[5]};
      store3(v.dinv, row, d);
#pragma unroll
      for (int a = 0; a < 3; ++a) u[a] = d[a] * b[a];
    }
    store3(v.x, row, zero);
    store3(v.p, row, zero);
    store3(v.r[0], row, b);
    store3(v.s[0], row, zero);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      acc[0] = fma(b[a], b[a], acc[0]);
      acc[1] = fma(u[a], u[a], acc[1]);
    }
  } else if (row < op.N) {
    const double xk[3] = {0.0, code[row] == 2 ? dy_bot : dy_top, 0.0};
    store3(v.x, row, xk);
    store3(v.p, row, zero);
    for (int b = 0; b < 2; ++b) {
      store3(v.r[b], row, zero);
      store3(v.s[b], row, zero);
      store3(v.w[b], row, zero);
    }
    if (BLOCK) {
#pragma unroll
      for (int c = 0; c < 6; ++c) v.dinv[6 * row + c] = 0.0;
    } else {
      store3(v.dinv, row, zero);
    }
  }
  block_publish<2>(acc, partials, ticket, red_out);
}

// k_cg_init_finalize: stopping threshold from the reduced (‖b‖², ‖M⁻¹b‖²).
__global__ void k_cg_init_finalize(const double* red, double rtol, double atol, int norm,
                                   int max_it, double reg, SolveState* st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double bb = red[0], zz = red[1];
  const double ref = norm == 1 ? zz : bb;
  const double t = rtol * rtol * ref, a2 = atol * atol;
  st->tol2 = t > a2 ? t : a2;
  st->reg = reg;
  st->bb0 = bb;
  st->res0 = ref;
  st->res_final = ref;
  st->base = 0;
  st->max_it = max_it;
  st->norm = norm;
  st->done = 0;
  st->iters = 0;
  st->status = 0;
}

// w₀ = A u₀ and the first fused reduction → slots[1] (α₀ = γ₀/δ₀, β₀ = 0).
template <bool BLOCK, int BS>
__global__ __launch_bounds__(BS) void k_cg_first(SellOp op, double reg, CgVecs v, Slot* slots,
                                                 const SolveState* st, double* partials,
                                                 unsigned* ticket) {
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * BS;
  const int64_t G = op.G;
  for (int64_t row = (int64_t)blockIdx.x * BS + threadIdx.x; row < op.nf; row += stride) {
    double r[3], u[3];
    load3(v.r[0], row, r);
    apply_minv<BLOCK>(v.dinv, row, r, u);
    double D[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) D[c] = op.diag[(int64_t)c * op.N + row];
    D[0] += reg;
    D[3] += reg;
    D[5] += reg;
    double y[3] = {0.0, 0.0, 0.0};
    block_mac(D, u, y);
    const int64_t base = (int64_t)op.slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = op.row_len[row];
    for (int k = 0; k < len; ++k) {
      const int64_t idx = base + (int64_t)k * 64;
      const int64_t c = op.s_col[idx];
      double V[6], rc[3], uc[3];
#pragma unroll
      for (int q = 0; q < 6; ++q) V[q] = op.val[q * G + idx];
      load3(v.r[0], c, rc);
      apply_minv<BLOCK>(v.dinv, c, rc, uc);
      block_mac(V, uc, y);
    }
    store3(v.w[0], row, y);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      acc[0] = fma(r[a], u[a], acc[0]);
      acc[1] = fma(y[a], u[a], acc[1]);
      acc[2] = fma(r[a], r[a], acc[2]);
      acc[3] = fma(u[a], u[a], acc[3]);
    }
  }
  if (block_publish<4, BS>(acc, partials, ticket, slots[1].v) && threadIdx.x == 0)
    finalize_slot(&slots[1], nullptr, st->norm);
}

__device__ __forceinline__ bool cg_running(const Slot& cur, const SolveState* st, int j) {
  return cur.flag == kRun && cur.res > st->tol2 && (st->base + j) < st->max_it;
}

// neighbour contribution y += V · M_c⁻¹ (r_c − α (w_c + β s_c))
template <bool BLOCK>
__device__ __forceinline__ void neighbour_mac(const double V[6], int64_t c, double alpha, double beta,
                                              const double* __restrict__ r_old,
                                              const double* __restrict__ s_old,
                                              const double* __restrict__ w_old,
                                              const double* __restrict__ dinv, double y[3]) {
  double rc[3], sc[3], wc[3], uc[3];
  load3(r_old, c, rc);
  load3(s_old, c, sc);
  load3(w_old, c, wc);
#pragma unroll
  for (int a = 0; a < 3; ++a) rc[a] = fma(-alpha, fma(beta, sc[a], wc[a]), rc[a]);
  apply_minv<BLOCK>(dinv, c, rc, uc);
  block_mac(V, uc, y);
}

// ---------------------------------------------------------------------------
// One CG-CG iteration.  Per free row (one lane per row, SELL-64 slot layout):
// own-row vector updates, then w_new = (K_ii + reg) u_new + Σ_slots V u_j with
// neighbour u_j recomputed from previous-iteration r, s, w.  HBM per row:
// 11 × 24 B of vectors + 48 B diag + 52 B per slot.
// ---------------------------------------------------------------------------
template <bool BLOCK, int BS>
__global__ __launch_bounds__(BS) void k_cg_iter(int j, SellOp op, CgVecs v, Slot* slots,
                                                const SolveState* st, double* partials,
                                                unsigned* ticket) {
  const double alpha = slots[j + 1].alpha, beta = slots[j + 1].beta, res = slots[j + 1].res;
  const int flag = slots[j + 1].flag;
  const bool go = (flag == kRun) & (res > st->tol2) & ((st->base + j) < st->max_it);
  const double reg = st->reg;
  // chunks have even length and base is a multiple of the chunk, so the
  // buffer parity is a launch constant: vector addresses need no scalar load
  const int par = j & 1;
  const double* __restrict__ r_old = v.r[par];
  const double* __restrict__ s_old = v.s[par];
  const double* __restrict__ w_old = v.w[par];
  double* __restrict__ r_new = v.r[par ^ 1];
  double* __restrict__ s_new = v.s[par ^ 1];
  double* __restrict__ w_new = v.w[par ^ 1];
  double* __restrict__ xv = v.x;
  double* __restrict__ pv = v.p;
  const double* __restrict__ dinv = v.dinv;
  const double* __restrict__ diag = op.diag;
  const double* __restrict__ val = op.val;
  const int32_t* __restrict__ s_col = op.s_col;
  const int32_t* __restrict__ row_len = op.row_len;
  const int32_t* __restrict__ slice_ptr = op.slice_ptr;
  const int64_t G = op.G, N = op.N, nf = op.nf;
  // No early exit on `go`: the scalar loads (SMEM) and the row's vector loads
  // (VMEM) are in flight together and only the stores/publish are predicated.
  // An iteration queued after convergence costs one wasted pass (≤ 2 chunks).
  const int64_t stride = (int64_t)gridDim.x * BS;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t row = (int64_t)blockIdx.x * BS + threadIdx.x; row - threadIdx.x % 64 < nf;
       row += stride) {
    // every lane of a wave shares the slice → scalar load of its slot offset
    const int slice = __builtin_amdgcn_readfirstlane((int)(row >> 6));
    const int64_t base = (int64_t)slice_ptr[slice] * 64 + (row & 63);
    if (row >= nf) continue;
    const int len = row_len[row];
    double ro[3], so[3], wo[3], pp[3], xx[3], uo[3], rn[3], un[3], sn[3], D[6];
    load3(r_old, row, ro);
    load3(s_old, row, so);
    load3(w_old, row, wo);
    load3(pv, row, pp);
    load3(xv, row, xx);
#pragma unroll
    for (int c = 0; c < 6; ++c) D[c] = diag[(int64_t)c * N + row];
    apply_minv<BLOCK>(dinv, row, ro, uo);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      pp[a] = fma(beta, pp[a], uo[a]);
      sn[a] = fma(beta, so[a], wo[a]);
      xx[a] = fma(alpha, pp[a], xx[a]);
      rn[a] = fma(-alpha, sn[a], ro[a]);
    }
    apply_minv<BLOCK>(dinv, row, rn, un);
    D[0] += reg;
    D[3] += reg;
    D[5] += reg;
    double y[3] = {0.0, 0.0, 0.0};
    block_mac(D, un, y);
    // slots two at a time: both columns, then both gathers, in flight together
    int k = 0;
    for (; k + 1 < len; k += 2) {
      const int64_t i0 = base + (int64_t)k * 64, i1 = i0 + 64;
      const int64_t c0 = s_col[i0], c1 = s_col[i1];
      double V0[6], V1[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        V0[q] = val[q * G + i0];
        V1[q] = val[q * G + i1];
      }
      neighbour_mac<BLOCK>(V0, c0, alpha, beta, r_old, s_old, w_old, dinv, y);
      neighbour_mac<BLOCK>(V1, c1, alpha, beta, r_old, s_old, w_old, dinv, y);
    }
    if (k < len) {
      const int64_t i0 = base + (int64_t)k * 64;
      const int64_t c0 = s_col[i0];
      double V0[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) V0[q] = val[q * G + i0];
      neighbour_mac<BLOCK>(V0, c0, alpha, beta, r_old, s_old, w_old, dinv, y);
    }
    if (go) {
      store3(pv, row, pp);
      store3(xv, row, xx);
      store3(s_new, row, sn);
      store3(r_new, row, rn);
      store3(w_new, row, y);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      acc[0] = fma(rn[a], un[a], acc[0]);
      acc[1] = fma(y[a], un[a], acc[1]);
      acc[2] = fma(rn[a], rn[a], acc[2]);
      acc[3] = fma(un[a], un[a], acc[3]);
    }
  }
  if (!go) {
    // converged / stopped / max_it: propagate STOP (a breakdown was flagged by
    // the reducing block of the previous iteration and stays in that slot)
    if (blockIdx.x == 0 && threadIdx.x == 0) slots[j + 2].flag = kStop;
    return;
  }
  if (block_publish<4, BS>(acc, partials, ticket, slots[j + 2].v) && threadIdx.x == 0)
    finalize_slot(&slots[j + 2], &slots[j + 1], st->norm);
}

// End of a chunk: record where the iteration stopped, or roll the newest slot
// to the front.  Once done, slots[1] is poisoned STOP so chunks the host
// already queued are no-ops.
// One wave: lane j checks slot j+1 in parallel, a ballot finds the first
// iteration that did not run.  The final state is mirrored into mapped pinned
// host memory (`host`), so the host polls without a copy kernel.
__global__ void k_cg_advance(int chunk, Slot* slots, SolveState* st, SolveState* host) {
  if (blockIdx.x != 0) return;
  const int lane = threadIdx.x;
  if (st->done) return;
  int first = -1;
  for (int j0 = 0; j0 <= chunk && first < 0; j0 += 64) {
    const int j = j0 + lane;
    const bool stop = j <= chunk && !cg_running(slots[j + 1], st, j);
    const unsigned long long m = __ballot(stop);
    if (m) first = j0 + __ffsll((long long)m) - 1;
  }
  if (lane != 0) return;
  if (first >= 0) {
    const Slot& cur = slots[first + 1];
    const double res = cur.res;
    st->iters = st->base + first;
    st->res_final = res;
    if (cur.flag == kBreakdown || (cur.flag == kRun && !isfinite(res))) st->status = -5;
    else if (cur.flag == kRun && res <= st->tol2) st->status = 0;
    else if (cur.flag == kRun) st->status = -4;
    else st->status = -5;
    st->done = 1;
    slots[1].flag = kStop;
    *host = *st;
    return;
  }
  slots[1] = slots[chunk + 1];
  st->base += chunk;
}

// ---------------------------------------------------------------------------
void launch_cg_rhs(hipStream_t s, const SellOp& op, const uint8_t* code, double dy_top,
                   double dy_bot, double reg, int precond, const CgVecs& v, double* partials,
                   unsigned* ticket, double* red_out) {
  const dim3 grid((unsigned)grid_rows(op.N > 0 ? op.N : 1));
  if (precond == 1)
    hipLaunchKernelGGL(k_cg_rhs<true>, grid, dim3(kBlock), 0, s, op, code, dy_top, dy_bot, reg, v,
                       partials, ticket, red_out);
  else
    hipLaunchKernelGGL(k_cg_rhs<false>, grid, dim3(kBlock), 0, s, op, code, dy_top, dy_bot, reg, v,
                       partials, ticket, red_out);
}

void launch_cg_init_finalize(hipStream_t s, const double* red, double rtol, double atol, int norm,
                             int max_it, double reg, SolveState* st) {
  hipLaunchKernelGGL(k_cg_init_finalize, dim3(1), dim3(64), 0, s, red, rtol, atol, norm, max_it,
                     reg, st);
}

template <int BS>
static void first_bs(hipStream_t s, const SellOp& op, double reg, int precond, const CgVecs& v,
                     Slot* slots, const SolveState* st, double* partials, unsigned* ticket) {
  const dim3 grid((unsigned)cg_grid(op.nf));
  if (precond == 1)
    hipLaunchKernelGGL((k_cg_first<true, BS>), grid, dim3(BS), 0, s, op, reg, v, slots, st,
                       partials, ticket);
  else
    hipLaunchKernelGGL((k_cg_first<false, BS>), grid, dim3(BS), 0, s, op, reg, v, slots, st,
                       partials, ticket);
}

void launch_cg_first(hipStream_t s, const SellOp& op, double reg, int precond, const CgVecs& v,
                     Slot* slots, const SolveState* st, double* partials, unsigned* ticket) {
  if (cg_block_size(op.nf) == 64)
    first_bs<64>(s, op, reg, precond, v, slots, st, partials, ticket);
  else
    first_bs<256>(s, op, reg, precond, v, slots, st, partials, ticket);
}

template <int BS>
static void iter_bs(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                    Slot* slots, const SolveState* st, double* partials, unsigned* ticket) {
  const dim3 grid((unsigned)cg_grid(op.nf));
  if (precond == 1)
    hipLaunchKernelGGL((k_cg_iter<true, BS>), grid, dim3(BS), 0, s, j, op, v, slots, st, partials,
                       ticket);
  else
    hipLaunchKernelGGL((k_cg_iter<false, BS>), grid, dim3(BS), 0, s, j, op, v, slots, st, partials,
                       ticket);
}

void launch_cg_iter(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                    Slot* slots, const SolveState* st, double* partials, unsigned* ticket) {
  if (cg_block_size(op.nf) == 64)
    iter_bs<64>(s, j, op, precond, v, slots, st, partials, ticket);
  else
    iter_bs<256>(s, j, op, precond, v, slots, st, partials, ticket);
}

void launch_cg_advance(hipStream_t s, int chunk, Slot* slots, SolveState* st, SolveState* host) {
  hipLaunchKernelGGL(k_cg_advance, dim3(1), dim3(64), 0, s, chunk, slots, st, host);
}

}  // namespace mfea
