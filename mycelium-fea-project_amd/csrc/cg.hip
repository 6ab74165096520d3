// cg.hip — single-reduction preconditioned CG (Chronopoulos–Gear) on the SELL-64
// node-block operator: ONE kernel per iteration, no atomics.
//
// Recurrences (x₀ = 0, u = M⁻¹r, w = A u, s = A p):
//   p_i = u_i + β_i p_{i−1}      s_i = w_i + β_i s_{i−1}
//   x_{i+1} = x_i + α_i p_i      r_{i+1} = r_i − α_i s_i
//   u_{i+1} = M⁻¹ r_{i+1}        w_{i+1} = A u_{i+1}
//   γ = (r,u), δ = (w,u);  β_i = γ_i/γ_{i−1},  α_i = γ_i / (δ_i − β_i γ_i / α_{i−1})
// In exact arithmetic these are the iterates of textbook PCG (the reference's
// KSPCG, src/fea_petsc.cpp:328); one fused reduction (γ, δ, ‖r‖², ‖u‖²) per
// iteration instead of two.  The SpMV w = A u needs u_j of neighbour rows whose
// owners update r, s, w in the same launch, so r, s, w are double-buffered by
// iteration parity and each row recomputes its neighbours' u_j from the
// previous-iteration values: u_j = M_j⁻¹ (r_j − α (w_j + β s_j)).
//
// Cross-block reduction by the consumer: iteration j stores one partial
// (γ, δ, ‖r‖², ‖u‖²) per block with plain stores; every wave of iteration j+1
// loads all G ≤ 512 partials (one round trip, in flight together with its row
// loads), sums them in block order and derives α, β and the stopping test
// itself.  The kernel boundary is the only synchronisation: no atomics, no
// last-block tail, no fences.  Every wave sums the same values in the same
// order, so all waves (and, multi-GPU, all ranks after an all-reduce of the
// partial array) agree bitwise.
#include "device_util.hpp"
#include "kernels.hpp"

namespace mfea {

static_assert(kCgMaxG == 512, "launch_cg_iter dispatches PU up to 8");

int cg_block_size(int64_t) { return kCgBS; }
int64_t cg_grid(int64_t rows) {
  int64_t g = (rows + kCgBS - 1) / kCgBS;
  return g < 1 ? 1 : (g > kCgMaxG ? kCgMaxG : g);
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
      if (j >= op.nf && code[j] != 3) {  // a known neighbour (3 = ghost free row: x₀ = 0)
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
    // ghost free rows (3) hold 0 until the solve's displacement halo fills them
    const double xk[3] = {0.0, code[row] == 3 ? 0.0 : (code[row] == 2 ? dy_bot : dy_top), 0.0};
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

// The GAMG solves' RHS (precond 2 of launch_cg_rhs): only what they read —
// b = 0 − K_fk x_k of the free rows (the CG's r₀ source, k_amg_cg_init) and
// the prescribed x of the known and ghost rows (reactions, stress); no
// Jacobi M⁻¹ and no Krylov vectors (the AMG CG keeps its own), ‖M⁻¹b‖² = 0
// (GAMG stops on the unpreconditioned residual).  A row's slots in batches of
// four: columns, then their codes, then the known couplings.  b's terms in
// slot order, as k_cg_rhs.
__global__ __launch_bounds__(kBlock) void k_amg_rhs(SellOp op, const uint8_t* __restrict__ code,
                                                    double dy_top, double dy_bot, CgVecs v,
                                                    double* partials, unsigned* ticket, double* red_out) {
  const int64_t row = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double acc[2] = {0.0, 0.0};
  if (row < op.nf) {
    const int64_t base = (int64_t)op.slice_ptr[row >> 6] * 64 + (row & 63);
    const int len = op.row_len[row];
    const int64_t G = op.G;
    double kx = 0.0, ky = 0.0, kz = 0.0;
    constexpr int U = 4;
    for (int k0 = 0; k0 < len; k0 += U) {
      int64_t idx[U];
      int32_t j[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        idx[u] = base + (int64_t)(k0 + u < len ? k0 + u : k0) * 64;
        j[u] = k0 + u < len ? op.s_col[idx[u]] : 0;
      }
      uint8_t c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) c[u] = k0 + u < len && j[u] >= op.nf ? code[j[u]] : 3;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c[u] != 3) {  // a known neighbour (3: free or ghost free row, x₀ = 0)
          const double dy = c[u] == 2 ? dy_bot : dy_top;
          kx = fma(op.val[1 * G + idx[u]], dy, kx);
          ky = fma(op.val[3 * G + idx[u]], dy, ky);
          kz = fma(op.val[4 * G + idx[u]], dy, kz);
        }
      }
    }
    const double b[3] = {0.0 - kx, 0.0 - ky, 0.0 - kz};
    store3(v.r[0], row, b);
#pragma unroll
    for (int a = 0; a < 3; ++a) acc[0] = fma(b[a], b[a], acc[0]);
  } else if (row < op.N) {
    const double xk[3] = {0.0, code[row] == 3 ? 0.0 : (code[row] == 2 ? dy_bot : dy_top), 0.0};
    store3(v.x, row, xk);
  }
  block_publish<2>(acc, partials, ticket, red_out);
}

// k_cg_init_finalize: stopping threshold from the reduced (‖b‖², ‖M⁻¹b‖²).
// zero[0, nzero): the solve's partial-sum buffers, cleared here instead of by
// a fill launch of their own (one launch boundary less per solve)
__global__ void k_cg_init_finalize(const double* red, double rtol, double atol, int norm,
                                   int max_it, double reg, SolveState* st, double* zero, int64_t nzero) {
  for (int64_t k = threadIdx.x; k < nzero; k += blockDim.x) zero[k] = 0.0;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double bb = red[0], zz = red[1];
  const double ref = norm == 1 ? zz : bb;
  const double t = rtol * rtol * ref, a2 = atol * atol;
  st->tol2 = t > a2 ? t : a2;
  st->rtol2 = rtol * rtol;
  st->atol2 = a2;
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

// w₀ = A u₀ and the first partials (γ₀, δ₀, ‖r₀‖², ‖u₀‖²) → parity 0;
// slots[0] = INIT (no previous α, γ: iteration 0 uses β₀ = 0, α₀ = γ₀/δ₀).
template <bool BLOCK>
__global__ __launch_bounds__(kCgBS) void k_cg_first(SellOp op, double reg, CgVecs v, Slot* slots,
                                                    double* part) {
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t stride = (int64_t)gridDim.x * kCgBS;
  const int64_t G = op.G;
  for (int64_t row = (int64_t)blockIdx.x * kCgBS + threadIdx.x; row < op.nf; row += stride) {
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
  store_block_partial(acc, part_buf(part, 0));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Slot s0;
    s0.v[0] = s0.v[1] = s0.v[2] = s0.v[3] = 0.0;
    s0.alpha = s0.beta = s0.res = 0.0;
    s0.flag = kInit;
    s0.pad = 0;
    slots[0] = s0;
  }
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
// One CG-CG iteration (iteration j of a chunk; chunks are even so the buffer
// parity is j & 1).  Each wave first reduces the previous iteration's block
// partials into (γ_j, δ_j, ‖r_j‖², ‖u_j‖²), forms α_j, β_j and the status of
// iteration j; block 0 records them in slots[j+1].  Then per free row (one
// lane per row, SELL-64 slot layout): own-row vector updates and
// w_new = (K_ii + reg) u_new + Σ_slots V u_j with neighbour u_j recomputed from
// previous-iteration r, s, w.  Stores are predicated on the status (an
// iteration queued after convergence costs one wasted pass, ≤ 2 chunks).
// HBM per free row: 11 × 24 B of vectors + 48 B diag + 52 B per slot.
// ---------------------------------------------------------------------------
// Own-row operands of one free row, loaded ahead of use (software prefetch).
template <bool BLOCK>
struct RowIn {
  double ro[3], so[3], wo[3], pp[3], xx[3], D[6], M[BLOCK ? 6 : 3];
  int len;
  int64_t base;
};

template <bool BLOCK>
__device__ __forceinline__ void load_row(int64_t row, const double* __restrict__ r_old,
                                         const double* __restrict__ s_old,
                                         const double* __restrict__ w_old,
                                         const double* __restrict__ pv, const double* __restrict__ xv,
                                         const double* __restrict__ diag,
                                         const double* __restrict__ dinv,
                                         const int32_t* __restrict__ row_len, int64_t N,
                                         RowIn<BLOCK>& in) {
  load3(r_old, row, in.ro);
  load3(s_old, row, in.so);
  load3(w_old, row, in.wo);
  load3(pv, row, in.pp);
  load3(xv, row, in.xx);
#pragma unroll
  for (int c = 0; c < 6; ++c) in.D[c] = diag[(int64_t)c * N + row];
#pragma unroll
  for (int c = 0; c < (BLOCK ? 6 : 3); ++c) in.M[c] = dinv[(BLOCK ? 6 : 3) * row + c];
  in.len = row_len[row];
}



template <bool BLOCK, int PU, bool TRACE = false>
__global__ __launch_bounds__(kCgBS) void k_cg_iter(int j, SellOp op, CgVecs v, Slot* slots,
                                                   const SolveState* st, double* part,
                                                   unsigned long long* trace) {
  trace_point<TRACE>(trace, 0, 0.0);
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
  const int64_t stride = (int64_t)gridDim.x * kCgBS;
  const int64_t lane = threadIdx.x & 63;

  // 1. the first row's operands, the scalars and the previous partials are
  //    all independent loads: issue them together (one memory round trip)
  int64_t row = (int64_t)blockIdx.x * kCgBS + threadIdx.x;
  RowIn<BLOCK> in;
  if (row < nf) load_row<BLOCK>(row, r_old, s_old, w_old, pv, xv, diag, dinv, row_len, N, in);
  const int f0 = __builtin_nontemporal_load(&slots[j].flag);
  const double g0 = slots[j].v[0], a0 = slots[j].alpha;
  const double tol2 = st->tol2, reg = st->reg;
  const int base_it = st->base, max_it = st->max_it, norm = st->norm;
  double S[4];
  wave_partials<PU>(part_buf(part, par), S);
  trace_point<TRACE>(trace, 1, S[0]);

  // 2. α_j, β_j and the status of iteration j (identical in every wave)
  const CgScalars cs = cg_scalars(S, f0, g0, a0, tol2, base_it + j, max_it, norm);
  const double alpha = cs.alpha, beta = cs.beta;
  const bool go = cs.status == kRun;
  cg_record(slots, j, S, cs);

  // 3. rows (grid-stride; the next row's operands are prefetched)
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  double ylast = 0.0;
  for (; row - lane < nf; row += stride) {
    // every lane of a wave shares the slice → scalar load of its slot offset
    const int slice = __builtin_amdgcn_readfirstlane((int)(row >> 6));
    const int64_t base = (int64_t)slice_ptr[slice] * 64 + (row & 63);
    const bool mine = row < nf;
    RowIn<BLOCK> cur = in;
    const int64_t nrow = row + stride;
    if (nrow < nf) load_row<BLOCK>(nrow, r_old, s_old, w_old, pv, xv, diag, dinv, row_len, N, in);
    if (!mine) continue;
    double uo[3], rn[3], un[3], sn[3], pp[3], xx[3];
    apply_m<BLOCK>(cur.M, cur.ro, uo);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      pp[a] = fma(beta, cur.pp[a], uo[a]);
      sn[a] = fma(beta, cur.so[a], cur.wo[a]);
      xx[a] = fma(alpha, pp[a], cur.xx[a]);
      rn[a] = fma(-alpha, sn[a], cur.ro[a]);
    }
    apply_m<BLOCK>(cur.M, rn, un);
    // own-row results leave now: their write-back overlaps the gathers below
    if (go) {
      store3(pv, row, pp);
      store3(xv, row, xx);
      store3(s_new, row, sn);
      store3(r_new, row, rn);
    }
    double D[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) D[c] = cur.D[c];
    D[0] += reg;
    D[3] += reg;
    D[5] += reg;
    double y[3] = {0.0, 0.0, 0.0};
    block_mac(D, un, y);
    const int len = cur.len;
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
    if (TRACE) ylast = y[0];
    if (go) store3(w_new, row, y);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      acc[0] = fma(rn[a], un[a], acc[0]);
      acc[1] = fma(y[a], un[a], acc[1]);
      acc[2] = fma(rn[a], rn[a], acc[2]);
      acc[3] = fma(un[a], un[a], acc[3]);
    }
  }
  trace_point<TRACE>(trace, 2, ylast);
  if (go) store_block_partial(acc, part_buf(part, par ^ 1));
  if (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    trace_point<TRACE>(trace, 3, acc[0]);
  }
}

// End of a chunk: find the first iteration that did not run (one wave, one
// slot per lane, ballot), record it, or roll slot `chunk` to the front.  The
// final state is mirrored into mapped pinned host memory (`host`), so the host
// polls without a copy kernel; slot 0 is then poisoned so already-queued
// chunks do nothing.
// shift 0: the chunk's updates wrote slots[1..chunk]; slots[0] = slots[chunk]
// rolls over.  shift 1 (chunks that END with an update, amg.hip): slots[1]
// holds the state entering the chunk and its updates wrote slots[2..chunk+1];
// slots[1] = slots[chunk+1] rolls over.  Either way the first stopped state
// slots[1 + j] was written by iteration base + j.
__global__ void k_cg_advance(int chunk, int shift, Slot* slots, SolveState* st, SolveState* host) {
  if (blockIdx.x != 0) return;
  const int lane = threadIdx.x;
  if (st->done) return;
  const int n = chunk + shift;
  int first = -1;
  for (int j0 = 0; j0 < n && first < 0; j0 += 64) {
    const int j = j0 + lane;
    const bool stop = j < n && slots[j + 1].flag != kRun;
    const unsigned long long m = __ballot(stop);
    if (m) first = j0 + __ffsll((long long)m) - 1;
  }
  if (lane != 0) return;
  if (first >= 0) {
    const Slot& cur = slots[first + 1];
    st->iters = st->base + first;
    st->res_final = cur.res;
    st->status = cur.flag == kConverged ? 0 : (cur.flag == kMaxit ? -4 : -5);
    st->done = 1;
    // poison the slot the NEXT queued chunk gates on first: slots[0] for
    // shift 0, slots[1] for shift 1 (the chunk's first update tests
    // slots[1]; left as kRun it would apply stale α, β and move x.  The
    // V-cycle / sweep and w launches take no gate: with x, r, p, s frozen
    // they rewrite what they wrote before, capi.hip enqueue_amg_chunk)
    slots[0].flag = kStop;
    slots[shift].flag = kStop;
    *host = *st;
    return;
  }
  slots[shift] = slots[chunk + shift];
  st->base += chunk;
}

// ---------------------------------------------------------------------------
void launch_cg_rhs(hipStream_t s, const SellOp& op, const uint8_t* code, double dy_top,
                   double dy_bot, double reg, int precond, const CgVecs& v, double* partials,
                   unsigned* ticket, double* red_out) {
  const dim3 grid((unsigned)grid_rows(op.N > 0 ? op.N : 1));
  if (precond == 2)
    hipLaunchKernelGGL(k_amg_rhs, grid, dim3(kBlock), 0, s, op, code, dy_top, dy_bot, v, partials, ticket,
                       red_out);
  else if (precond == 1)
    hipLaunchKernelGGL(k_cg_rhs<true>, grid, dim3(kBlock), 0, s, op, code, dy_top, dy_bot, reg, v,
                       partials, ticket, red_out);
  else
    hipLaunchKernelGGL(k_cg_rhs<false>, grid, dim3(kBlock), 0, s, op, code, dy_top, dy_bot, reg, v,
                       partials, ticket, red_out);
}

void launch_cg_init_finalize(hipStream_t s, const double* red, double rtol, double atol, int norm,
                             int max_it, double reg, SolveState* st, double* zero, int64_t nzero) {
  hipLaunchKernelGGL(k_cg_init_finalize, dim3(1), dim3(zero ? 256 : 64), 0, s, red, rtol, atol, norm, max_it,
                     reg, st, zero, zero ? nzero : (int64_t)0);
}

void launch_cg_first(hipStream_t s, const SellOp& op, double reg, int precond, const CgVecs& v,
                     Slot* slots, double* part) {
  const dim3 grid((unsigned)cg_grid(op.nf));
  if (precond == 1)
    hipLaunchKernelGGL(k_cg_first<true>, grid, dim3(kCgBS), 0, s, op, reg, v, slots, part);
  else
    hipLaunchKernelGGL(k_cg_first<false>, grid, dim3(kCgBS), 0, s, op, reg, v, slots, part);
}

template <int PU, bool TRACE>
static void iter_pu(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                    Slot* slots, const SolveState* st, double* part, unsigned long long* trace) {
  const dim3 grid((unsigned)cg_grid(op.nf));
  if (precond == 1)
    hipLaunchKernelGGL((k_cg_iter<true, PU, TRACE>), grid, dim3(kCgBS), 0, s, j, op, v, slots, st,
                       part, trace);
  else
    hipLaunchKernelGGL((k_cg_iter<false, PU, TRACE>), grid, dim3(kCgBS), 0, s, j, op, v, slots, st,
                       part, trace);
}

template <bool TRACE>
static void iter_dispatch(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                          Slot* slots, const SolveState* st, double* part,
                          unsigned long long* trace) {
  const int64_t g = cg_grid(op.nf);
  if (g <= 64) iter_pu<1, TRACE>(s, j, op, precond, v, slots, st, part, trace);
  else if (g <= 128) iter_pu<2, TRACE>(s, j, op, precond, v, slots, st, part, trace);
  else if (g <= 256) iter_pu<4, TRACE>(s, j, op, precond, v, slots, st, part, trace);
  else iter_pu<8, TRACE>(s, j, op, precond, v, slots, st, part, trace);
}

void launch_cg_iter(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                    Slot* slots, const SolveState* st, double* part, unsigned long long* trace) {
  if (trace) iter_dispatch<true>(s, j, op, precond, v, slots, st, part, trace);
  else iter_dispatch<false>(s, j, op, precond, v, slots, st, part, nullptr);
}

void launch_cg_advance(hipStream_t s, int chunk, Slot* slots, SolveState* st, SolveState* host, int shift) {
  hipLaunchKernelGGL(k_cg_advance, dim3(1), dim3(64), 0, s, chunk, shift, slots, st, host);
}

}  // namespace mfea
