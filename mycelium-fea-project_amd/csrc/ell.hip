// ell.hip — single-reduction PCG (Chronopoulos–Gear, as in cg.hip) on the
// wave-local lane operator of symbolic.hpp ("Ell"): ONE memory round trip per
// iteration.
//
// The SELL kernel (cg.hip) pays a chain of dependent loads per iteration:
// slot offset → neighbour column → neighbour r, s, w (≈ 2.7 µs measured with
// tools/trace_iter.py on C2, after the 2.4 µs hop that brings the row's own
// operands and the partials).  Here every operand a lane needs sits at an
// address computable from its lane index alone:
//   - own vectors, M, the diagonal block and three slot blocks (k-major);
//   - a neighbour owned by a lane of the SAME wave: its fresh u_j is read from
//     the wave's LDS exchange row after that lane wrote it;
//   - an out-of-wave neighbour (slot 0 only): its previous-iteration r, s, w
//     (and its M) were pushed into this lane's halo record by the partner lane
//     in the previous launch; u_j = M_j (r_j − α (w_j + β s_j)) is recomputed
//     with exactly the owner's operations, so every lane sees bitwise the u_j
//     its owner uses.
// Helper lanes (rows with more than three slots or several halo slots) add
// their partial A u into the owner lane in a fixed order; they carry no vector
// state (all zero) and never store.
//
// ND = 2: planar meshes (all z = 0).  The z DOFs decouple exactly (xz, yz
// couplings are exactly 0 and b_z = 0), so every z
// component of every Krylov vector stays exactly 0 and contributes exact
// zeros to every sum: dropping them gives bitwise the 3-DOF iterates with
// 40 % fewer bytes per lane.  Symmetric blocks then hold (xx, xy, yy).
#include <cstdlib>

#include "device_util.hpp"
#include "kernels.hpp"

namespace mfea {

template <int ND>
struct Dof {
  static constexpr int NB = ND == 3 ? 6 : 3;  // components of a symmetric block
  static constexpr int LDSW = ND == 3 ? 4 : 2;  // doubles per lane in an LDS row
};
template <int ND, bool BLOCK>
constexpr int n_minv() { return BLOCK ? Dof<ND>::NB : ND; }
// SELL / row-order component of lane-block component c (2-D: xx, xy, yy)
template <int ND>
__device__ __forceinline__ int blk_src(int c) { return ND == 3 ? c : (c == 2 ? 3 : c); }

template <int ND>
__device__ __forceinline__ void lload(const double* __restrict__ v, int64_t NL, int64_t l,
                                      double* o) {
#pragma unroll
  for (int c = 0; c < ND; ++c) o[c] = v[c * NL + l];
}
template <int ND>
__device__ __forceinline__ void lstore(double* __restrict__ v, int64_t NL, int64_t l,
                                       const double* o) {
#pragma unroll
  for (int c = 0; c < ND; ++c) v[c * NL + l] = o[c];
}

// y += V u (symmetric block)
template <int ND>
__device__ __forceinline__ void bmac(const double* V, const double* u, double* y) {
  if (ND == 3) {
    block_mac(V, u, y);
  } else {  // = block_mac with V_xz = V_yz = 0, u_z = 0
    y[0] = fma(V[0], u[0], fma(V[1], u[1], y[0]));
    y[1] = fma(V[1], u[0], fma(V[2], u[1], y[1]));
  }
}
// u = M r
template <int ND, bool BLOCK>
__device__ __forceinline__ void mapply(const double* M, const double* r, double* u) {
  if (!BLOCK) {
#pragma unroll
    for (int a = 0; a < ND; ++a) u[a] = M[a] * r[a];
  } else if (ND == 3) {
    sym_apply(M, r, u);
  } else {  // = sym_apply with B_xz = B_yz = 0, r_z = 0
    u[0] = fma(M[0], r[0], M[1] * r[1]);
    u[1] = fma(M[1], r[0], M[2] * r[1]);
  }
}

__device__ __forceinline__ int group_info(uint32_t code) { return (int)(int8_t)(code >> 24); }

__device__ __forceinline__ int wave_max_i(int m) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off, 64));
  return m;
}

// LDS stores of this wave visible to its own later LDS loads (DS ops of one
// wave execute in order; the wait keeps the compiler from reordering too)
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Multi-partition: every lane of every wave ends with the total of the gathered
// per-rank partial sums, summed in one fixed order (DPP tree over the rank
// rows) — identical on every rank, since the gathered rows are bitwise copies.
__device__ __forceinline__ void wave_gall(const double* __restrict__ g, double s[4]) {
  const int lane = threadIdx.x & 63;
  double t[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) t[c] = g[lane * 4 + c];
#pragma unroll
  for (int c = 0; c < 4; ++c) s[c] = wave_allsum(t[c]);
}

__device__ __forceinline__ int64_t pair_of(int32_t partner) { return -2 - (int64_t)partner; }

// ---------------------------------------------------------------------------
// Lane operator values and initial vectors (once per solve).
// ---------------------------------------------------------------------------
template <int ND, bool BLOCK>
__global__ __launch_bounds__(kCgBS) void k_ell_init(EllOp op, SellOp sop, CgVecs rv, EllVecs v) {
  constexpr int NB = Dof<ND>::NB, NM = n_minv<ND, BLOCK>();
  const int64_t NL = op.NL;
  const double zero[3] = {0.0, 0.0, 0.0};
  for (int64_t l = (int64_t)blockIdx.x * kCgBS + threadIdx.x; l < NL;
       l += (int64_t)gridDim.x * kCgBS) {
    const int32_t row = op.lane_row[l];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int32_t sp = op.src_pos[k * NL + l];
#pragma unroll
      for (int c = 0; c < NB; ++c)
        op.V[(c * 3 + k) * NL + l] = sp >= 0 ? sop.val[(int64_t)blk_src<ND>(c) * sop.G + sp] : 0.0;
    }
#pragma unroll
    for (int c = 0; c < NB; ++c)
      op.D[c * NL + l] = row >= 0 ? sop.diag[(int64_t)blk_src<ND>(c) * sop.N + row] : 0.0;
#pragma unroll
    for (int c = 0; c < NM; ++c)
      v.M[c * NL + l] = row >= 0 ? rv.dinv[(int64_t)(BLOCK ? 6 : 3) * row + (BLOCK ? blk_src<ND>(c) : c)]
                                 : 0.0;
    double b[3] = {0.0, 0.0, 0.0};
    if (row >= 0) {
#pragma unroll
      for (int c = 0; c < ND; ++c) b[c] = rv.r[0][3 * (int64_t)row + c];
    }
    lstore<ND>(v.r[0], NL, l, b);
    lstore<ND>(v.r[1], NL, l, zero);
    lstore<ND>(v.x, NL, l, zero);
    lstore<ND>(v.p, NL, l, zero);
    for (int q = 0; q < 2; ++q) {
      lstore<ND>(v.s[q], NL, l, zero);
      lstore<ND>(v.w[q], NL, l, zero);
    }
  }
}

// ---------------------------------------------------------------------------
// Multi-partition, before w₀ = A u₀: each remote-halo lane sends its owner's
// [r₀ | M] (helpers take them from the owner lane) into its pair's slot of
// the parity-1 send records.
// ---------------------------------------------------------------------------
template <int ND, bool BLOCK>
__global__ __launch_bounds__(kCgBS) void k_ell_pack0(EllOp op, EllVecs v, DistVecs dv) {
  constexpr int NM = n_minv<ND, BLOCK>(), RW = 3 * ND;
  const int64_t NL = op.NL;
  const int lane = threadIdx.x & 63;
  for (int64_t l = (int64_t)blockIdx.x * kCgBS + threadIdx.x; l - lane < NL;
       l += (int64_t)gridDim.x * kCgBS) {
    double r[ND], M[NM];
    lload<ND>(v.r[0], NL, l, r);
#pragma unroll
    for (int c = 0; c < NM; ++c) M[c] = v.M[c * NL + l];
    const int info = group_info(op.code[l]);
    const int ow = info < 0 ? lane + info : lane;
    double ro[ND], Mo[NM];
#pragma unroll
    for (int a = 0; a < ND; ++a) ro[a] = __shfl(r[a], ow, 64);
#pragma unroll
    for (int c = 0; c < NM; ++c) Mo[c] = __shfl(M[c], ow, 64);
    const int32_t pt = op.partner[l];
    if (pt <= -2) {
      double* rec = dv.xs[1] + pair_of(pt) * RW;
#pragma unroll
      for (int a = 0; a < ND; ++a) rec[a] = ro[a];
#pragma unroll
      for (int c = 0; c < NM; ++c) rec[ND + c] = Mo[c];
    }
  }
}

// ---------------------------------------------------------------------------
// w₀ = A u₀ with the neighbours pulled through nbr_lane (the only gather of
// the solve), halo records of parity 0 (r₀, s₀ = 0, w₀ and M), partials
// (γ₀, δ₀, ‖r₀‖², ‖u₀‖²) → parity 0, slots[0] = INIT.
// DIST: a remote slot-0 neighbour's [r₀ | M] comes from the received parity-1
// records (its M is kept in dv.mr for the iterations), and the lane's own
// parity-0 record goes to its pair's send slot.
// ---------------------------------------------------------------------------
template <int ND, bool BLOCK, bool DIST, int BS>
__global__ __launch_bounds__(BS) void k_ell_first(EllOp op, double reg, EllVecs v, Slot* slots,
                                                  double* part, DistVecs dv) {
  constexpr int NB = Dof<ND>::NB, NM = n_minv<ND, BLOCK>(), RW = 3 * ND;
  const int64_t NL = op.NL;
  const int lane = threadIdx.x & 63;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t l = (int64_t)blockIdx.x * BS + threadIdx.x; l - lane < NL;
       l += (int64_t)gridDim.x * BS) {
    const int32_t pt = op.partner[l];
    double r[ND], M[NM], u[ND], D[NB];
    lload<ND>(v.r[0], NL, l, r);
#pragma unroll
    for (int c = 0; c < NM; ++c) M[c] = v.M[c * NL + l];
    mapply<ND, BLOCK>(M, r, u);
#pragma unroll
    for (int c = 0; c < NB; ++c) D[c] = op.D[c * NL + l];
    D[0] += reg;
    D[ND == 3 ? 3 : 2] += reg;
    if constexpr (ND == 3) D[5] += reg;
    double y[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0;
    bmac<ND>(D, u, y);
    for (int k = 0; k < 3; ++k) {
      const int32_t nl = op.nbr_lane[k * NL + l];
      double rc[ND], Mc[NM], uc[ND], V[NB];
      if (nl >= 0) {
        lload<ND>(v.r[0], NL, nl, rc);
#pragma unroll
        for (int c = 0; c < NM; ++c) Mc[c] = v.M[c * NL + nl];
      } else if (DIST && k == 0 && pt <= -2) {
        const double* rec = dv.xr[1] + pair_of(pt) * RW;
#pragma unroll
        for (int a = 0; a < ND; ++a) rc[a] = rec[a];
#pragma unroll
        for (int c = 0; c < NM; ++c) {
          Mc[c] = rec[ND + c];
          dv.mr[pair_of(pt) * NM + c] = Mc[c];
        }
      } else {
        continue;
      }
      mapply<ND, BLOCK>(Mc, rc, uc);
#pragma unroll
      for (int c = 0; c < NB; ++c) V[c] = op.V[(c * 3 + k) * NL + l];
      bmac<ND>(V, uc, y);
    }
    const int info = group_info(op.code[l]);
    const int maxh = wave_max_i(info > 0 ? info : 0);
    for (int t = 1; t <= maxh; ++t) {
      double yt[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a) yt[a] = __shfl(y[a], (lane + t) & 63, 64);
      if (t <= info) {
#pragma unroll
        for (int a = 0; a < ND; ++a) y[a] += yt[a];
      }
    }
    if (info >= 0) lstore<ND>(v.w[0], NL, l, y);
    // halo push: the owner's r₀, s₀ = 0, w₀ and M
    const int ow = info < 0 ? lane + info : lane;
    double ro[ND], yo[ND], Mo[NM];
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      ro[a] = __shfl(r[a], ow, 64);
      yo[a] = __shfl(y[a], ow, 64);
    }
#pragma unroll
    for (int c = 0; c < NM; ++c) Mo[c] = __shfl(M[c], ow, 64);
    if (pt >= 0) {  // pt = the compact record this lane fills
      double* h = v.h[0];
      const int64_t NR = op.NR;
#pragma unroll
      for (int c = 0; c < ND; ++c) {
        h[c * NR + pt] = ro[c];
        h[(3 + c) * NR + pt] = 0.0;
        h[(6 + c) * NR + pt] = yo[c];
      }
#pragma unroll
      for (int c = 0; c < NM; ++c) v.hM[c * NR + pt] = Mo[c];
    } else if (DIST && pt <= -2) {
      double* rec = dv.xs[0] + pair_of(pt) * RW;
#pragma unroll
      for (int c = 0; c < ND; ++c) {
        rec[c] = ro[c];
        rec[ND + c] = 0.0;
        rec[2 * ND + c] = yo[c];
      }
    }
#pragma unroll
    for (int a = 0; a < ND; ++a) {  // helper lanes: r = u = 0
      acc[0] = fma(r[a], u[a], acc[0]);
      acc[1] = fma(y[a], u[a], acc[1]);
      acc[2] = fma(r[a], r[a], acc[2]);
      acc[3] = fma(u[a], u[a], acc[3]);
    }
  }
  store_block_partial<BS>(acc, part_buf(part, 0));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    Slot s0;
    s0.v[0] = s0.v[1] = s0.v[2] = s0.v[3] = 0.0;
    s0.alpha = s0.beta = s0.res = 0.0;
    s0.flag = kInit;
    s0.pad = 0;
    slots[0] = s0;
  }
}

// ---------------------------------------------------------------------------
// One CG-CG iteration (iteration j of a chunk, buffer parity j & 1).
// Per lane, all loads independent of each other and of α, β:
//   own r, s, w, p, x (5·ND), diagonal block (NB), M, three slot blocks
//   (3·NB), code + partner, halo record r, s, w (3·ND) + M, and the G block
//   partials.  Then α, β; own update (p, x, s, r, u); u → LDS; A u from the
//   LDS row and the halo record; helper partials → owner through LDS; stores;
//   halo push.
// HBM per lane, Jacobi: ND = 3: 440 B read, 120 B written; ND = 2: 264 B
// read, 80 B written (+24·ND B per halo push).
// ---------------------------------------------------------------------------
template <int ND, bool BLOCK>
struct LaneIn {
  double ro[ND], so[ND], wo[ND], pp[ND], xx[ND], D[Dof<ND>::NB], M[n_minv<ND, BLOCK>()];
  double V[3][Dof<ND>::NB];
  double h[3 * ND], hM[n_minv<ND, BLOCK>()];
  uint32_t code;
  int32_t partner;
};

template <int ND, bool BLOCK, bool HC>
__device__ __forceinline__ void load_lane(int64_t l, int par, const EllOp& op, const EllVecs& v,
                                          LaneIn<ND, BLOCK>& in) {
  constexpr int NB = Dof<ND>::NB, NM = n_minv<ND, BLOCK>();
  const int64_t NL = op.NL;
  lload<ND>(v.r[par], NL, l, in.ro);
  lload<ND>(v.s[par], NL, l, in.so);
  lload<ND>(v.w[par], NL, l, in.wo);
  lload<ND>(v.p, NL, l, in.pp);
  lload<ND>(v.x, NL, l, in.xx);
#pragma unroll
  for (int c = 0; c < NB; ++c) in.D[c] = op.D[c * NL + l];
  if (BLOCK) {
#pragma unroll
    for (int c = 0; c < NM; ++c) in.M[c] = v.M[c * NL + l];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int c = 0; c < NB; ++c) in.V[k][c] = op.V[(c * 3 + k) * NL + l];
  in.code = op.code[l];
  in.partner = op.partner[l];
  // Halo records.  Compact (op.hc, large systems): only lanes with an
  // in-partition halo slot own one (12.7 % of the lanes on the tiled meshes).
  // The wave's (mask, base) is one scalar load; lane i reads record base +
  // #(mask lanes below i) — a lane without a halo reads its next neighbour's
  // record (unused), so a wave touches exactly its own contiguous records and
  // every load stays unconditional.  The scalar hop overlaps the lane's other
  // loads (C2 unchanged) and the bytes saved shorten a bandwidth-bound launch
  // (C3 −8 %).  Per lane records (op.hc = 0, indexed by the lane) remain for
  // comparison runs.
  int64_t hi = l;
  if constexpr (HC) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)((l - lane) >> 6));
    const uint64_t m = op.hmask[w];
    hi = (int64_t)op.hbase[w] + __popcll(m & ((1ull << lane) - 1ull));
  }
  const int64_t NR = op.NR;
  const double* __restrict__ h = v.h[par];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int c = 0; c < ND; ++c) in.h[q * ND + c] = h[(q * 3 + c) * NR + hi];
#pragma unroll
  for (int c = 0; c < NM; ++c) in.hM[c] = v.hM[c * NR + hi];
}

// DIST (multi-partition): α, β come from the gathered rank partial sums; a
// remote slot-0 neighbour's record is read from the received records of its
// pair (an index-dependent load: only waves holding such lanes pay a second
// round trip), and the lane's record for the peer goes to the send slot.
template <int ND, bool BLOCK, int PU, bool TRACE, bool DIST, int BS, bool HC>
__global__ __launch_bounds__(BS) void k_ell_iter(int j, EllOp op, EllVecs v, Slot* slots,
                                                 const SolveState* st, double* part,
                                                 unsigned long long* trace, DistVecs dv) {
  constexpr int NB = Dof<ND>::NB, LW = Dof<ND>::LDSW;
  constexpr int NM = n_minv<ND, BLOCK>(), RW = 3 * ND;
  constexpr int NW = BS / 64;
  __shared__ double lds_u[NW][64][LW];       // fresh u of every lane
  __shared__ double lds_y[NW][64][LW];       // helper partials of A u
  __shared__ double lds_b[NW][64][3 * ND];   // owner r, s, w for helper pushes
  trace_point<TRACE, BS>(trace, 0, 0.0);
  const int par = j & 1;
  const int64_t NL = op.NL;
  const int64_t stride = (int64_t)gridDim.x * BS;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* __restrict__ r_new = v.r[par ^ 1];
  double* __restrict__ s_new = v.s[par ^ 1];
  double* __restrict__ w_new = v.w[par ^ 1];
  double* __restrict__ h_new = v.h[par ^ 1];

  int64_t l = (int64_t)blockIdx.x * BS + threadIdx.x;
  LaneIn<ND, BLOCK> in;
  if (l - lane < NL) load_lane<ND, BLOCK, HC>(l, par, op, v, in);
  const int f0 = __builtin_nontemporal_load(&slots[j].flag);
  const double g0 = slots[j].v[0], a0 = slots[j].alpha;
  const double tol2 = st->tol2, reg = st->reg;
  const int base_it = st->base, max_it = st->max_it, norm = st->norm;
  double S[4];
  if constexpr (DIST) {
    wave_gall(dv.gall[par], S);
  } else {
    wave_partials<PU>(part_buf(part, par), S);
  }
  trace_point<TRACE, BS>(trace, 1, S[0]);

  const CgScalars cs = cg_scalars(S, f0, g0, a0, tol2, base_it + j, max_it, norm);
  const double alpha = cs.alpha, beta = cs.beta;
  const bool go = cs.status == kRun;
  cg_record(slots, j, S, cs);

  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  double ylast = 0.0;
  for (bool first = true; l - lane < NL; l += stride, first = false) {  // wave-uniform
    if (!first) load_lane<ND, BLOCK, HC>(l, par, op, v, in);
    if (DIST && in.partner <= -2) {
      const int64_t k = pair_of(in.partner);
      const double* __restrict__ rec = dv.xr[par] + k * RW;
#pragma unroll
      for (int q = 0; q < RW; ++q) in.h[q] = rec[q];
#pragma unroll
      for (int c = 0; c < NM; ++c) in.hM[c] = dv.mr[k * NM + c];
    }
    const int info = group_info(in.code);
    const bool owner = info >= 0;
    if (!BLOCK) {
      // PCJACOBI: M = 1 / (K_ii + reg), bitwise k_cg_rhs's dinv (no M load).
      // A zero diagonal (helper / inert lanes, rows without active elements)
      // has r = 0 throughout, so M = 0 gives the same u = 0 (and no inf·0).
#pragma unroll
      for (int a = 0; a < ND; ++a) {
        const double d = in.D[ND == 3 ? (a == 0 ? 0 : (a == 1 ? 3 : 5)) : 2 * a];
        in.M[a] = d != 0.0 ? 1.0 / (d + reg) : 0.0;
      }
    }
    double uo[ND], rn[ND], un[ND], sn[ND], pp[ND], xx[ND];
    mapply<ND, BLOCK>(in.M, in.ro, uo);
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      pp[a] = fma(beta, in.pp[a], uo[a]);
      sn[a] = fma(beta, in.so[a], in.wo[a]);
      xx[a] = fma(alpha, pp[a], in.xx[a]);
      rn[a] = fma(-alpha, sn[a], in.ro[a]);
    }
    mapply<ND, BLOCK>(in.M, rn, un);
#pragma unroll
    for (int a = 0; a < ND; ++a) lds_u[wv][lane][a] = un[a];
    if (go && owner) {
      lstore<ND>(v.p, NL, l, pp);
      lstore<ND>(v.x, NL, l, xx);
      lstore<ND>(s_new, NL, l, sn);
      lstore<ND>(r_new, NL, l, rn);
    }
    double D[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) D[c] = in.D[c];
    D[0] += reg;
    D[ND == 3 ? 3 : 2] += reg;
    if constexpr (ND == 3) D[5] += reg;
    double y[ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) y[a] = 0.0;
    bmac<ND>(D, un, y);
    // halo neighbour of slot 0: the owner's operations on the pushed record
    double uh[ND];
    {
      double t[ND];
#pragma unroll
      for (int a = 0; a < ND; ++a)
        t[a] = fma(-alpha, fma(beta, in.h[ND + a], in.h[2 * ND + a]), in.h[a]);
      mapply<ND, BLOCK>(in.hM, t, uh);
    }
    lds_fence();
    double uk[3][ND];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int src = (int)((in.code >> (8 * k)) & 63);
#pragma unroll
      for (int a = 0; a < ND; ++a) uk[k][a] = lds_u[wv][src][a];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t src = (in.code >> (8 * k)) & 0xFF;
      if (k == 0 && src == kSrcHalo) {
#pragma unroll
        for (int a = 0; a < ND; ++a) uk[0][a] = uh[a];
      }
      if (src != kSrcNone) bmac<ND>(in.V[k], uk[k], y);
    }
    // helper lanes → owner (t order)
    if (__ballot(info > 0)) {
#pragma unroll
      for (int a = 0; a < ND; ++a) lds_y[wv][lane][a] = y[a];
      lds_fence();
      for (int t0 = 1; __ballot(info >= t0); t0 += 4) {
        double yt[4][ND];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int src = min(lane + t0 + q, 63);
#pragma unroll
          for (int a = 0; a < ND; ++a) yt[q][a] = lds_y[wv][src][a];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (t0 + q <= info) {
#pragma unroll
            for (int a = 0; a < ND; ++a) y[a] += yt[q][a];
          }
      }
    }
    if (TRACE) ylast = y[0];
    if (go && owner) lstore<ND>(w_new, NL, l, y);
    // halo push of the owner's r, s, w; a helper takes them from its owner's
    // LDS row (only waves where a helper pushes pay for it)
    double rsy[3 * ND];
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      rsy[a] = rn[a];
      rsy[ND + a] = sn[a];
      rsy[2 * ND + a] = y[a];
    }
    if (__ballot(in.partner != -1 && !owner)) {
#pragma unroll
      for (int c = 0; c < 3 * ND; ++c) lds_b[wv][lane][c] = rsy[c];
      lds_fence();
      const int ow = owner ? lane : lane + info;
#pragma unroll
      for (int c = 0; c < 3 * ND; ++c) rsy[c] = lds_b[wv][ow][c];
    }
    if (go && in.partner >= 0) {
      const int64_t pt = in.partner, NR = op.NR;
#pragma unroll
      for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int c = 0; c < ND; ++c) h_new[(q * 3 + c) * NR + pt] = rsy[q * ND + c];
    }
    if (DIST && go && in.partner <= -2) {
      double* __restrict__ rec = dv.xs[par ^ 1] + pair_of(in.partner) * RW;
#pragma unroll
      for (int q = 0; q < RW; ++q) rec[q] = rsy[q];
    }
#pragma unroll
    for (int a = 0; a < ND; ++a) {  // helper lanes contribute exact zeros
      acc[0] = fma(rn[a], un[a], acc[0]);
      acc[1] = fma(y[a], un[a], acc[1]);
      acc[2] = fma(rn[a], rn[a], acc[2]);
      acc[3] = fma(un[a], un[a], acc[3]);
    }
    // the LDS rows are rewritten next pass: all reads of this pass are done
    lds_fence();
  }
  trace_point<TRACE, BS>(trace, 2, ylast);
  if (go) store_block_partial<BS>(acc, part_buf(part, par ^ 1));
  if (TRACE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    trace_point<TRACE, BS>(trace, 3, acc[0]);
  }
}

template <int ND>
__global__ __launch_bounds__(kCgBS) void k_ell_finish(EllOp op, EllVecs v, double* x_row) {
  const int64_t NL = op.NL;
  for (int64_t l = (int64_t)blockIdx.x * kCgBS + threadIdx.x; l < NL;
       l += (int64_t)gridDim.x * kCgBS) {
    const int32_t row = op.lane_row[l];
    if (row < 0) continue;
    double xx[3] = {0.0, 0.0, 0.0};  // 2-D: z stays exactly 0
    lload<ND>(v.x, NL, l, xx);
#pragma unroll
    for (int c = 0; c < 3; ++c) x_row[3 * (int64_t)row + c] = xx[c];
  }
}

// ---------------------------------------------------------------------------
// Multi-partition helpers (one wave / tiny grids; off the per-lane path).
// ---------------------------------------------------------------------------
template <int PU>
__global__ __launch_bounds__(64) void k_psum(const double* __restrict__ p, double* row,
                                             double* gsend) {
  double S[4];
  wave_partials<PU>(p, S);  // block order, the order wave_partials uses single-GPU
  if (threadIdx.x == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      row[c] = S[c];
      gsend[c] = S[c];
    }
  }
}

__global__ void k_rank_sum(const double* __restrict__ g, int world, double* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int c = 0; c < 4; ++c) {
    double s = 0.0;
    for (int r = 0; r < world; ++r) s += g[4 * r + c];
    out[c] = s;
  }
}

__global__ __launch_bounds__(kBlock) void k_rows_pack(const int32_t* __restrict__ rows, int64_t n,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
#pragma unroll
  for (int c = 0; c < 3; ++c) out[3 * i + c] = x[3 * r + c];
}

__global__ __launch_bounds__(kBlock) void k_rows_unpack(const int32_t* __restrict__ rows, int64_t n,
                                                        const double* __restrict__ in,
                                                        double* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
#pragma unroll
  for (int c = 0; c < 3; ++c) x[3 * r + c] = in[3 * i + c];
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Launch geometry of the lane kernels: 256-thread blocks, at most 512 of them
// (each wave of the next launch re-reads every block partial).  Measured on
// one box (C2, per iteration of the real solve): 6.09 µs at 256 threads vs
// 6.36 at 128 (grid over all 256 CUs) and 6.54 at 64.  An in-launch grid
// reduction by the last block (no cap, one pass per wave) was slower at C3
// (22.5 vs 20.2 µs: its tail costs more than the passes save) and was
// dropped.  The handle's options (mfea_set_option "ell_block" 64|128|256|512,
// "ell_maxg" — fixed for a handle's life once graphs are captured) reach the
// launchers through EllOp.bs / EllOp.maxg.
// ---------------------------------------------------------------------------
int ell_block_size(const EllOp& op) {
  const int b = op.bs;
  return (b == 64 || b == 128 || b == 512) ? b : 256;
}
// op.maxg caps the grid below kCgMaxG (tests: several passes per wave on
// small systems)
int64_t ell_grid_size(const EllOp& op) {
  const int64_t c = op.maxg;
  const int64_t cap = (c >= 1 && c < kCgMaxG) ? c : (int64_t)kCgMaxG;
  const int b = ell_block_size(op);
  const int64_t g = (op.NL + b - 1) / b;
  return g < 1 ? 1 : (g > cap ? cap : g);
}
// partial groups of 64 each wave loads: ≥ grid / 64
static int pu_of(int64_t g) { return g <= 64 ? 1 : g <= 128 ? 2 : g <= 256 ? 4 : g <= 320 ? 5 : 8; }

static dim3 ell_grid_ew(const EllOp& op) { return dim3((unsigned)grid_rows(op.NL > 0 ? op.NL : 1)); }
static dim3 ell_grid_cg(const EllOp& op) { return dim3((unsigned)cg_grid(op.NL)); }

template <int ND>
static void init_nd(hipStream_t s, const EllOp& op, const SellOp& sop, int precond,
                    const CgVecs& rv, const EllVecs& v) {
  if (precond == 1)
    hipLaunchKernelGGL((k_ell_init<ND, true>), ell_grid_ew(op), dim3(kCgBS), 0, s, op, sop, rv, v);
  else
    hipLaunchKernelGGL((k_ell_init<ND, false>), ell_grid_ew(op), dim3(kCgBS), 0, s, op, sop, rv, v);
}
void launch_ell_init(hipStream_t s, const EllOp& op, const SellOp& sop, int precond,
                     const CgVecs& rv, const EllVecs& v) {
  if (op.nd == 2) init_nd<2>(s, op, sop, precond, rv, v);
  else init_nd<3>(s, op, sop, precond, rv, v);
}

template <int ND, bool DIST, int BS>
static void first_bs(hipStream_t s, const EllOp& op, double reg, int precond, const EllVecs& v,
                     Slot* slots, double* part, const DistVecs& dv) {
  const dim3 grid((unsigned)ell_grid_size(op));
  if (precond == 1)
    hipLaunchKernelGGL((k_ell_first<ND, true, DIST, BS>), grid, dim3(BS), 0, s, op, reg, v, slots,
                       part, dv);
  else
    hipLaunchKernelGGL((k_ell_first<ND, false, DIST, BS>), grid, dim3(BS), 0, s, op, reg, v, slots,
                       part, dv);
}
template <int ND, bool DIST>
static void first_nd(hipStream_t s, const EllOp& op, double reg, int precond, const EllVecs& v,
                     Slot* slots, double* part, const DistVecs& dv) {
  switch (ell_block_size(op)) {
    case 64: first_bs<ND, DIST, 64>(s, op, reg, precond, v, slots, part, dv); break;
    case 128: first_bs<ND, DIST, 128>(s, op, reg, precond, v, slots, part, dv); break;
    case 512: first_bs<ND, DIST, 512>(s, op, reg, precond, v, slots, part, dv); break;
    default: first_bs<ND, DIST, 256>(s, op, reg, precond, v, slots, part, dv); break;
  }
}
void launch_ell_first(hipStream_t s, const EllOp& op, double reg, int precond, const EllVecs& v,
                      Slot* slots, double* part, const DistVecs* dv) {
  const DistVecs d = dv ? *dv : DistVecs{};
  if (op.nd == 2) {
    if (dv) first_nd<2, true>(s, op, reg, precond, v, slots, part, d);
    else first_nd<2, false>(s, op, reg, precond, v, slots, part, d);
  } else {
    if (dv) first_nd<3, true>(s, op, reg, precond, v, slots, part, d);
    else first_nd<3, false>(s, op, reg, precond, v, slots, part, d);
  }
}

template <int ND>
static void pack0_nd(hipStream_t s, const EllOp& op, int precond, const EllVecs& v,
                     const DistVecs& dv) {
  if (precond == 1)
    hipLaunchKernelGGL((k_ell_pack0<ND, true>), ell_grid_cg(op), dim3(kCgBS), 0, s, op, v, dv);
  else
    hipLaunchKernelGGL((k_ell_pack0<ND, false>), ell_grid_cg(op), dim3(kCgBS), 0, s, op, v, dv);
}
void launch_ell_pack0(hipStream_t s, const EllOp& op, int precond, const EllVecs& v,
                      const DistVecs& dv) {
  if (op.nd == 2) pack0_nd<2>(s, op, precond, v, dv);
  else pack0_nd<3>(s, op, precond, v, dv);
}

template <int ND, int PU, bool TRACE, bool DIST, int BS, bool HC>
static void iter_launch_hc(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                           Slot* slots, const SolveState* st, double* part,
                           unsigned long long* trace, const DistVecs& dv) {
  const dim3 grid((unsigned)ell_grid_size(op));
  if (precond == 1)
    hipLaunchKernelGGL((k_ell_iter<ND, true, PU, TRACE, DIST, BS, HC>), grid, dim3(BS), 0, s, j, op,
                       v, slots, st, part, trace, dv);
  else
    hipLaunchKernelGGL((k_ell_iter<ND, false, PU, TRACE, DIST, BS, HC>), grid, dim3(BS), 0, s, j, op,
                       v, slots, st, part, trace, dv);
}
template <int ND, int PU, bool TRACE, bool DIST, int BS>
static void iter_launch(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                        Slot* slots, const SolveState* st, double* part,
                        unsigned long long* trace, const DistVecs& dv) {
  if (op.hc)
    iter_launch_hc<ND, PU, TRACE, DIST, BS, true>(s, j, op, precond, v, slots, st, part, trace, dv);
  else
    iter_launch_hc<ND, PU, TRACE, DIST, BS, false>(s, j, op, precond, v, slots, st, part, trace, dv);
}

template <int ND, bool TRACE, int BS>
static void iter_pu(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                    Slot* slots, const SolveState* st, double* part, unsigned long long* trace,
                    const DistVecs& dv) {
  switch (pu_of(ell_grid_size(op))) {
    case 1: iter_launch<ND, 1, TRACE, false, BS>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    case 2: iter_launch<ND, 2, TRACE, false, BS>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    case 4: iter_launch<ND, 4, TRACE, false, BS>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    case 5: iter_launch<ND, 5, TRACE, false, BS>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    default: iter_launch<ND, 8, TRACE, false, BS>(s, j, op, precond, v, slots, st, part, trace, dv); break;
  }
}

template <int ND, bool TRACE>
static void iter_bs(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                    Slot* slots, const SolveState* st, double* part, unsigned long long* trace,
                    const DistVecs& dv) {
  switch (ell_block_size(op)) {
    case 64: iter_pu<ND, TRACE, 64>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    case 128: iter_pu<ND, TRACE, 128>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    case 512: iter_pu<ND, TRACE, 512>(s, j, op, precond, v, slots, st, part, trace, dv); break;
    default: iter_pu<ND, TRACE, 256>(s, j, op, precond, v, slots, st, part, trace, dv); break;
  }
}

template <int ND>
static void iter_dist(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                      Slot* slots, const SolveState* st, double* part, const DistVecs& dv) {
  // the rank partial sums replace the block partials: PU unused
  switch (ell_block_size(op)) {
    case 64: iter_launch<ND, 1, false, true, 64>(s, j, op, precond, v, slots, st, part, nullptr, dv); break;
    case 128: iter_launch<ND, 1, false, true, 128>(s, j, op, precond, v, slots, st, part, nullptr, dv); break;
    case 512: iter_launch<ND, 1, false, true, 512>(s, j, op, precond, v, slots, st, part, nullptr, dv); break;
    default: iter_launch<ND, 1, false, true, 256>(s, j, op, precond, v, slots, st, part, nullptr, dv); break;
  }
}

void launch_ell_iter(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                     Slot* slots, const SolveState* st, double* part, unsigned long long* trace,
                     const DistVecs* dv) {
  if (dv) {
    if (op.nd == 2) iter_dist<2>(s, j, op, precond, v, slots, st, part, *dv);
    else iter_dist<3>(s, j, op, precond, v, slots, st, part, *dv);
    return;
  }
  const DistVecs d{};
  if (op.nd == 2) {
    if (trace) iter_bs<2, true>(s, j, op, precond, v, slots, st, part, trace, d);
    else iter_bs<2, false>(s, j, op, precond, v, slots, st, part, nullptr, d);
  } else {
    if (trace) iter_bs<3, true>(s, j, op, precond, v, slots, st, part, trace, d);
    else iter_bs<3, false>(s, j, op, precond, v, slots, st, part, nullptr, d);
  }
}

void launch_psum(hipStream_t s, const EllOp& op, const double* p, double* row, double* gsend) {
  switch (pu_of(ell_grid_size(op))) {  // the partitioned iteration's grid
    case 1: hipLaunchKernelGGL(k_psum<1>, dim3(1), dim3(64), 0, s, p, row, gsend); break;
    case 2: hipLaunchKernelGGL(k_psum<2>, dim3(1), dim3(64), 0, s, p, row, gsend); break;
    case 4: hipLaunchKernelGGL(k_psum<4>, dim3(1), dim3(64), 0, s, p, row, gsend); break;
    case 5: hipLaunchKernelGGL(k_psum<5>, dim3(1), dim3(64), 0, s, p, row, gsend); break;
    default: hipLaunchKernelGGL(k_psum<8>, dim3(1), dim3(64), 0, s, p, row, gsend); break;
  }
}

void launch_rank_sum(hipStream_t s, const double* g, int world, double* out) {
  hipLaunchKernelGGL(k_rank_sum, dim3(1), dim3(64), 0, s, g, world, out);
}

void launch_rows_pack(hipStream_t s, const int32_t* rows, int64_t n, const double* x, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_rows_pack, dim3((unsigned)grid_rows(n)), dim3(kBlock), 0, s, rows, n, x, out);
}

void launch_rows_unpack(hipStream_t s, const int32_t* rows, int64_t n, const double* in, double* x) {
  if (n > 0) hipLaunchKernelGGL(k_rows_unpack, dim3((unsigned)grid_rows(n)), dim3(kBlock), 0, s, rows, n, in, x);
}

void launch_ell_finish(hipStream_t s, const EllOp& op, const EllVecs& v, double* x_row) {
  if (op.nd == 2)
    hipLaunchKernelGGL(k_ell_finish<2>, ell_grid_ew(op), dim3(kCgBS), 0, s, op, v, x_row);
  else
    hipLaunchKernelGGL(k_ell_finish<3>, ell_grid_ew(op), dim3(kCgBS), 0, s, op, v, x_row);
}

}  // namespace mfea
