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
#include <algorithm>
#include <vector>

#include "symbolic.hpp"

namespace mfea {

// Stable sort of one row's few entries (the symbolic products sort every row:
// insertion sort, no temporary buffer per call as std::stable_sort takes)
template <class It, class Less>
inline void row_stable_sort(It b, It e, Less less) {
  if (e - b > 48) {
    std::stable_sort(b, e, less);
    return;
  }
  for (It i = b + (b != e); i < e; ++i) {
    auto v = std::move(*i);
    It j = i;
    for (; j > b && less(v, *(j - 1)); --j) *j = std::move(*(j - 1));
    *j = std::move(v);
  }
}


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
  // distributed plans (AmgPlan::n_dist > level): rank of every row (new
  // labels), row boundaries per rank in the owner-major labelling of A / P
  // rows (world + 1) and of the A·P rows (their own labelling)
  std::vector<int32_t> owner;
  std::vector<int64_t> own, ap_own;
  std::vector<int32_t> aprow;  // distributed: row label → its A·P row label
  std::vector<int32_t> nat;    // row label → natural (aggregation-order) index
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
  // the compact cycle (amg.hip, option amg_cycle 1): the smoothed transfer
  // P̃ = (I − ω D⁻¹ A) P on A·P's pattern with the level's own row labels,
  // and R̃ = P̃ᵀ.  With them one V(1,1) cycle level is two sweeps instead of four:
  //   down  b_{l+1} = R̃ b_l,  c_l = x_l + ω D⁻¹ (b_l − A x_l)   (x_l = ω D⁻¹ b_l)
  //   up    e_l = c_l + P̃ e_{l+1}
  // (e = x + P e' + ω D⁻¹(b − A(x + P e')) = c + (I − ω D⁻¹ A) P e', and
  // R(b − A x) = R (I − ω A D⁻¹) b = P̃ᵀ b: the same preconditioner).
  SellPat PT;                  // n × nc, rows labelled as A·P's
  std::vector<int32_t> pt_row; // PT row → the level's row
  std::vector<int32_t> pt_ap;  // PT position → its A·P position
  std::vector<int32_t> pt_p;   // PT position → the P position of the same block, or -1
  SellPat RT;                  // nc × n, rows by RT length inside windows (rt_row)
  std::vector<int32_t> rt_row; // RT row → the level-(l+1) row
  std::vector<int32_t> rt_pt;  // RT position → PT position (value = PT[rt_pt]ᵀ)
  std::vector<int64_t> rt_own; // distributed (level l+1 ≤ n_dist): RT rows owner-major, per-rank bounds
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
  // distributed V-cycle (AmgDistSpec): levels [0, n_dist) are split over
  // `world` ranks by row ranges; level n_dist and below are replicated (every
  // rank holds and computes all of their rows).  n_dist = 0: one partition.
  int world = 1;
  int n_dist = 0;
  bool spatial = false;  // rows labelled in Z-order (AmgLayout)
};

// The distributed hierarchy (multi-GPU GAMG): ONE global
// hierarchy, identical on every rank and equal to the one-partition
// hierarchy (same aggregates), whose rows of levels [0, n_dist] are labelled
// owner-major so each rank's rows are one contiguous range (an aggregate
// belongs to the rank holding most of its rows).  A level is split while it
// has more than rep_rows rows (level 0 always is).
struct AmgDistSpec {
  int world = 1;
  std::vector<int32_t> owner;  // per Pattern free row [0, n_free): its rank
  int64_t rep_rows = 32768;
};

// Strength of connection for the level-0 aggregation (PyAMG's symmetric
// strength, PETSc GAMG's -pc_gamg_threshold): a coupling i–j is strong when
// ‖A_ij‖ ≥ θ·√(‖A_ii‖‖A_jj‖), the block norms estimated from the element
// stiffnesses on the host (‖S_e‖ = EA/L · √(1 + (kb_kax/L²)²), kb_kax =
// 12EI / EA: the bending-to-axial ratio's constant; ‖A_ii‖ ≈ Σ_e ‖S_e‖).
// Aggregation follows strong couplings only; P's smoothing and the Galerkin
// products keep every coupling.  θ = 0: every coupling strong.
struct AmgStrength {
  double theta = 0.0;
  double kb_kax = 0.0;
};

// Row labels of the device layout (stage 2 of the symbolic phase).  The
// aggregation always runs in the natural order (depth-first: hyphal chains
// contiguous — the order the iteration counts depend on); the labels only
// decide where rows sit in the SELL slices and vectors.  spatial = 1: every
// level's rows by the Morton (Z-order) key of their coordinates (level 0 the
// nodes', coarse levels their aggregates' centroids), then the usual
// 4096-row length windows — on chord-dense networks the depth-first order
// puts a fifth of the couplings more than 49k rows apart (C5: 22 % of A_0's
// entries; 0.1 % in Z-order), so the gathers of x / u miss every L2.
// spatial = -1: Z-order when more than far_frac of A_0's off-diagonal entries
// lie more than 4096 rows apart in the natural order.  Unsplit plans only.
struct AmgLayout {
  int spatial = 0;
  double far_frac = 0.10;
  // rows of a coarse level sorted by their A length alone (the compact
  // cycle's sweeps read A and R̂, which has labels of its own); false: by
  // A + R length (the four-step cycle's resid and restriction)
  bool by_a = false;
};

// Builds the hierarchy for the free rows [0, P.n_free) of P with the element
// activity `active` (P's element order).  Returns "" on success.
// max_levels caps the hierarchy (the coarsest level's block Jacobi is then
// an inexact solve; plan.capped says so).  Measured: a cap costs far more in
// iterations than it saves per cycle (C3: 16 → 35 iterations at 5 levels).
// dist: the distributed form (NULL: one partition, the plan of before).
std::string build_amg(const Pattern& P, const std::vector<uint8_t>& active, int nd, AmgPlan& plan,
                      int max_levels = kAmgMaxLevels, const AmgDistSpec* dist = nullptr,
                      const AmgStrength& strength = AmgStrength(), const AmgLayout& layout = AmgLayout());

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
// ---- distributed V-cycle: one rank's share of a distributed plan ----------
// One exchange of items (rows of a vector or SELL positions of a matrix):
// per peer (ascending), the items this rank sends and receives, both sides
// enumerating them in ascending item order (no negotiation).
struct XPlan {
  std::vector<int32_t> peers;
  std::vector<int64_t> soff, scnt, roff, rcnt;  // per peer, in items
  std::vector<int32_t> sidx, ridx;              // items, concatenated per peer
  int64_t n_send() const { return (int64_t)sidx.size(); }
  int64_t n_recv() const { return (int64_t)ridx.size(); }
  bool empty() const { return sidx.empty() && ridx.empty(); }
};
struct AmgRank {
  int rank = 0, world = 1, n_dist = 0;
  // per level: rows this rank computes — A / P rows [lo, hi), A·P rows
  // [aplo, aphi) — and of the level below, the coarse rows its restriction
  // produces [rlo, rhi)
  std::vector<int64_t> lo, hi, aplo, aphi, rlo, rhi;
  // V-cycle, per split level l < n_dist: rows of level l read by this rank's
  // A_l rows (x; level 0: also the CG's u), by its R_l rows (t), and rows of
  // level l+1 read by its P_l rows (the coarse output; only while l+1 is split)
  std::vector<XPlan> xa, xr, xp;
  XPlan xg;  // level n_dist (replicated): every rank's restricted rows to all (b, x)
  // numeric setup, per split level l: P positions of the rows its A·P and R
  // rows read, A·P positions of the rows its A_{l+1} rows read
  std::vector<XPlan> sp, sap;
  XPlan sg;  // A positions of level n_dist: all-gather
  // the compact cycle on a plan split at level 0 only (n_dist = 1, levels ≥ 1
  // replicated): this rank's R̂_0 rows [rtlo, rthi); level-0
  // rows its Ã_0 and R̂_0 rows read (the down sweep's x_0 halo); for the
  // setup of R̂_0 = s' D_1⁻¹ P̃_0ᵀ D_0 / ω, the P̃_0 positions and the
  // level-0 diagonal-block positions (A_0 slot 0) its R̂_0 rows read
  bool compact = false;
  int64_t rtlo = 0, rthi = 0;
  XPlan xc, spt, sd;
};
// rank r's share of a distributed plan (plan.n_dist ≥ 1)
std::string build_amg_rank(const AmgPlan& plan, int rank, AmgRank& out);
// Level 0 of rank rk over ITS partition's pattern P (partition.hpp: local
// node / element → global maps node_g, elem_g): row0 (level-0 row → P's row,
// own rows only) and the A_0 slot lists (P's slots of every own row, by the
// global level-0 row of their neighbour).  G: the whole mesh's pattern the
// plan was built on; gkey: the global element activity.
std::string build_amg_level0(const AmgPlan& plan, const Pattern& G, const AmgRank& rk, const Pattern& P,
                             const std::vector<int64_t>& node_g, const std::vector<int64_t>& elem_g,
                             const std::vector<uint8_t>& gkey, PosList& a0, std::vector<int32_t>& row0);

// The compact cycle below level kc as one explicit operator (amg_collapse.cpp):
// V_k = (2I − Ã_k) + P̃_k V_{k+1} R̂_k for k = nlev−2 … kc (V_coarsest = I),
// through T_k = V_{k+1} R̂_k.  Per level k ≥ kc (lev[k − kc]): the patterns in
// the plan's device labels and the index lists of the two products.
struct AmgCollapse {
  int kc = 0;  // 0: none
  struct Lev {
    int k = 0;
    SellPat T;                   // n_{k+1} × n_k, rows in level k+1 labels
    PosList tl;                  // per T position: (V_{k+1} position or −1 = identity, R̂ position)
    SellPat V;                   // n_k × n_k, rows by length (vrow: V row → level row)
    std::vector<int32_t> vrow;
    PosList vl;                  // per V position: (P̃ position, T position)
    std::vector<int32_t> va;     // per V position: the Ã position of the block, or −1
    std::vector<int32_t> vdiag;  // per V position: 1 on the diagonal (+2I)
  };
  std::vector<Lev> lev;
};
// kc = the highest level ≥ max(1, min_level) whose V (and every V below it)
// takes at most max_bytes (f32 blocks + columns) and whose products at most
// max_pairs list items; none (kc = 0) when not even the deepest fits.
std::string build_amg_collapse(const AmgPlan& plan, int64_t max_bytes, int64_t max_pairs, int min_level,
                               AmgCollapse& out);

// Levels 0 and 1 merged around a cycle collapsed at level 2 (amg_collapse.cpp
// build_amg_merge; C2-sized networks, whose launches are latency-bound).
// With x_0 the level-0 iterate the compact cycle computes
//   c_0 = (2I − Ã_0) x_0,  c_1 = (2I − Ã_1) R̂_0 x_0,  x_2 = R̂_1 R̂_0 x_0,
//   e_2 = V_2 x_2,  u = c_0 + P̃_0 (c_1 + P̃_1 e_2),
// so with  DQ = [2R̂_0 − Ã_1 R̂_0 ; R̂_1 R̂_0]  (rows: level 1, then level 2)
// and  U = [P̃_0 | P̃_0 P̃_1]  the cycle is one down launch (DQ rows + Ã_0
// rows), V_2, and one up launch: 3 launches where the two-level form takes 5.
// The vectors live in one buffer B = [c_1 (n1) | x_2 (n2) | e_2 (n2) | scratch].
struct AmgMerge {
  bool on = false;
  int64_t n0 = 0, n1 = 0, n2 = 0;
  SellPat DQ;                   // rows: c_1's (padded to 64) then x_2's; cols: level-0 rows
  std::vector<int32_t> dq_dst;  // DQ row → its index in B
  int64_t dq_split = 0;         // positions below: c_1 rows (Ã_1 × R̂_0 pairs + 2 R̂_0); above: R̂_1 × R̂_0
  std::vector<int32_t> dq_ext;  // per DQ position: the R̂_0 position of the block (× 2), or −1
  PosList dq_l;                 // per DQ position: (Ã_1 or R̂_1 position, R̂_0 position) pairs
  SellPat U;                    // rows: P̃_0's SELL rows (pt_row of level 0); cols: indices in B
  std::vector<int32_t> u_ext;   // per U position: the P̃_0 position of the block, or −1
  PosList u_l;                  // per U position: (P̃_0 position, P̃_1 position) pairs
};
// on = false (nothing built) unless the plan's cycle collapses at level 2
// (coll.kc == 2) on one partition.
std::string build_amg_merge(const AmgPlan& plan, const AmgCollapse& coll, AmgMerge& out);

// Block-Jacobi multicolour sweeps over A_0 (MFEA_PC_SOR, MFEA_PC_ICC; sweep.hip):
// level-0 rows in blocks of `rows_per_block` consecutive rows (one workgroup
// each — the couplings between blocks are dropped, as PETSc's processor-local
// SOR / ICC drops those between ranks), inside a block a greedy colouring of
// the rows' in-block couplings (row order), so one colour's rows are
// independent and the triangular sweeps run colour by colour.  Per row its
// in-block neighbours of earlier colours (lower) and of later colours (upper):
// their index in the block and the A_0 position of the coupling block.
// Whole-matrix SSOR / IC(0) in a chain-piece multicolour order (sweep.hip,
// MFEA_PC_SOR / MFEA_PC_ICC).  The level-0 rows are cut into
// PIECES: runs of at most `piece_len` (≤ 64) rows along a depth-first path of
// A_0's graph, each row coupled to its predecessor and to no other row of
// its piece.  The pieces are coloured (greedy: no two coupled pieces share a
// colour) and the matrix is factorised in the order colour → piece → row, so
// the pieces of one colour are independent and a hyphal chain keeps its
// natural-order factorisation.  Every coupling of A_0 is kept: in-piece
// couplings are the predecessor links, the others ("cross" couplings) join
// pieces of different colours and are lower / upper by colour.
//
// Entries: a colour's pieces, in depth-first order, packed into the 64 lanes
// of consecutive waves (entry = 64·wave + lane; a piece's rows on
// consecutive lanes, never across two waves; the rest of a wave that cannot
// take the next piece is padding, row −1).  A sweep solves a piece's
// recurrence by a scan across its lanes: wsteps[w] = ⌈log₂(longest piece)⌉.
struct SweepPlan {
  int piece_len = 64;
  int colors = 0;
  int64_t n = 0;                         // level-0 rows
  int64_t n_pieces = 0;
  std::vector<int32_t> cwave;            // per colour: first wave (+ end)
  std::vector<int32_t> wsteps;           // per wave: scan steps
  std::vector<int32_t> row;              // per entry: level-0 row (−1: padding)
  std::vector<int32_t> ppos;             // per entry: A_0 position of (row, predecessor) (−1: a piece's first row)
  std::vector<int32_t> dpos;             // per entry: A_0 position of the diagonal block (−1: padding)
  // cross couplings per entry: to earlier colours (lo) / later colours (up):
  // the neighbour's entry and the A_0 position of (row, neighbour)
  std::vector<int32_t> lo_ptr, lo_ent, lo_pos;
  std::vector<int32_t> up_ptr, up_ent, up_pos;
  int64_t n_entries() const { return (int64_t)row.size(); }
};
std::string build_sweep(const AmgPlan& plan, int piece_len, SweepPlan& out);

// xsend_rows / xrecv_rows: Pattern rows of the plan's xsend / xrecv nodes
std::string build_amg_halo(const Pattern& P, const std::vector<uint8_t>& active, const AmgPlan& plan,
                           const std::vector<int32_t>& xsend_rows, const std::vector<int32_t>& xrecv_rows,
                           AmgHalo& halo);

// The GAMG form of a partitioned solve chosen automatically (option
// "amg_dist" −1; capi.hip solve_amg_part): t[0] = the block-Jacobi form's
// step time, t[1] = the global hierarchy's, seconds, −1 while untimed.  The
// form to time next (the global one first), −1 once both are timed; then the
// choice, the faster (ties: the global hierarchy).  Over RCCL every rank
// passes the MAX over ranks of each time, so every rank returns the same
// mode: the two forms issue different exchanges, and ranks on different
// forms would hang (tests/test_amg_cpu.py::test_auto_form_choice_is_collective).
inline int amg_auto_pending(const double t[2]) { return t[1] < 0 ? 1 : t[0] < 0 ? 0 : -1; }
inline int amg_auto_choice(const double t[2]) { return t[1] <= t[0] ? 1 : 0; }

}  // namespace mfea
