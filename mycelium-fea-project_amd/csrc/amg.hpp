// amg.hpp — smoothed-aggregation algebraic multigrid preconditioner for the
// PCG solve (MFEA_PC_GAMG): the MI355X-native counterpart of the reference's
// `-pc_type gamg` configuration (src/fea_petsc_solverAndPC.cpp:330-391 sweeps
// KSPCG × {jacobi, sor, ilu, icc, gamg}; PETSc GAMG is smoothed aggregation).
//
// Why: Jacobi-PCG needs ≈ 6,800 iterations on the tiled benchmark networks
// (SURVEY §7 hard part 1) and each iteration is a launch-latency-bound grid
// sweep.  One SA V-cycle per iteration cuts that to ≈ 15–25 iterations
// (DESIGN.md §4), so the solve becomes a few dozen bandwidth-bound sweeps.
//
// Split of the work:
//   host, once per (mesh, BC set, active set) — this file / amg_symbolic.cpp:
//     aggregation of every level (standard SA greedy aggregation on the
//     level's block graph, all couplings strong), the SELL-64 patterns of
//     A_l, P_l, R_l = P_lᵀ, A_l·P_l and A_{l+1} = P_lᵀ A_l P_l, and the index
//     lists that turn the numeric setup into pure gathers;
//   device, every solve — amg.hip: A_0 from the assembled operator, block
//     Jacobi inverses and smoother weights, P_l values (block-Jacobi smoothed
//     tentative prolongator), the two Galerkin products, then the V-cycle
//     inside each PCG iteration.  Fixed-order gathers only: no atomics, so the
//     hierarchy and every solve are bitwise reproducible.
//
// The hierarchy is keyed to the active element set: aggregates never span two
// connected components of the CURRENT free-node graph, so a component that
// carries no load (b = 0 there) keeps exactly zero iterates, as in the direct
// solve (src/fea_solver.py:128).  When elements fail the host rebuilds it.
//
// Blocks are node blocks of ND×ND doubles (ND = 2 on planar meshes, whose z
// DOFs decouple exactly — SURVEY Appendix B; ND = 3 otherwise), row-major.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "symbolic.hpp"

namespace mfea {

constexpr int kAmgMaxLevels = 32;

// A node-block matrix pattern in SELL-64 layout: slice s covers rows
// [64 s, 64 s + 64), its entries occupy slot rows sptr[s] .. sptr[s+1]-1;
// entry (slot t, lane l) is at position t·64 + l.  col = -1 marks padding.
struct SellPat {
  int64_t n = 0;                 // rows
  std::vector<int32_t> sptr;     // n_slices + 1 (slot rows)
  std::vector<int32_t> col;      // positions
  std::vector<int32_t> rlen;     // entries per row
  int64_t n_pos() const { return sptr.empty() ? 0 : (int64_t)sptr.back() * 64; }
  int64_t pos(int64_t row, int k) const { return ((int64_t)sptr[row >> 6] + k) * 64 + (row & 63); }
};

// index list per output position (CSR over positions, pads have none)
struct PosList {
  std::vector<int32_t> ptr;  // n_pos + 1
  std::vector<int32_t> a;    // first operand positions
  std::vector<int32_t> b;    // second operand positions (pair lists only)
};

struct AmgLevel {
  SellPat A;                 // slot 0 of every row = its diagonal block
  bool coarsest = false;
  // ---- below: only for non-coarsest levels
  int64_t nc = 0;            // coarse rows (aggregates)
  std::vector<int32_t> agg;  // row → aggregate
  SellPat P;                 // n × nc
  PosList pv;                // P value: A positions of row i whose column lies in the aggregate
  SellPat R;                 // nc × n (R = Pᵀ): col = fine row
  std::vector<int32_t> rp;   // R position → P position (value = P[rp]ᵀ)
  SellPat AP;                // n × nc
  PosList ap;                // AP(i, J) = Σ A[a] · P[b]
  PosList ac;                // A_{l+1}(I, J) = Σ P[a]ᵀ · AP[b]   (positions of level l+1's A)
};

struct AmgPlan {
  int nd = 2;
  std::vector<AmgLevel> lev;  // lev[0] = the free-node system
  // level-0 row i ↔ free row row0[i] of the Pattern (rows are relabelled per
  // level so SELL slices hold rows of similar length; amg_symbolic.cpp)
  std::vector<int32_t> row0;
  // level-0 values: A_0(i, j≠i) = Σ over the SELL slots of the assembled
  // operator (symbolic.hpp) joining i and j; the diagonal = diag[i] + reg·I
  PosList a0;                 // per A_0 position: SELL slot positions (diag: none)
  int64_t pair_items = 0;     // Σ list lengths (memory / setup-traffic report)
  bool capped = false;        // max levels reached with couplings left
};

// Builds the hierarchy for the free rows [0, P.n_free) of P with the element
// activity `active` (P's element order).  Returns "" on success.
// max_levels caps the hierarchy (the coarsest level's block Jacobi is then
// an inexact solve; plan.capped says so).  Measured: a cap costs far more in
// iterations than it saves per cycle (C3: 16 → 35 iterations at 5 levels).
std::string build_amg(const Pattern& P, const std::vector<uint8_t>& active, int nd, AmgPlan& plan,
                      int max_levels = kAmgMaxLevels);

// Partitioned solve (partition.hpp): the V-cycle is block Jacobi over the
// partitions (each partition's hierarchy couples its own free rows only —
// the strips are grip-to-grip, so the cut couplings are weak: 19 iterations
// for 1, 2 and 4 strips of a 4×5-tile network) while the CG
// operator w = A u is global: every owned row adds its couplings to the free
// ghost rows, whose u arrives through the displacement-halo plan (xsend /
// xrecv nodes, the same order on both sides).
struct AmgHalo {
  std::vector<int32_t> send_rows;  // level-0 rows of the xsend nodes, plan order
  std::vector<int32_t> gptr;       // per level-0 row: its ghost couplings [gptr[i], gptr[i+1])
  std::vector<int32_t> gslot;      // SELL slot position of the assembled operator (K_ig = −S_e)
  std::vector<int32_t> grecv;      // index of the ghost's u in the received halo (xrecv order)
};
// xsend_rows / xrecv_rows: Pattern rows of the plan's xsend / xrecv nodes
std::string build_amg_halo(const Pattern& P, const std::vector<uint8_t>& active, const AmgPlan& plan,
                           const std::vector<int32_t>& xsend_rows, const std::vector<int32_t>& xrecv_rows,
                           AmgHalo& halo);

}  // namespace mfea
