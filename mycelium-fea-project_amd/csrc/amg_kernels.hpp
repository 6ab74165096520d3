// amg_kernels.hpp — device views and launchers of the SA-AMG preconditioned CG
// (amg.hip).  Layout of one level l in HBM (n rows = nodes or aggregates,
// ND = 2 or 3 DOFs per row, NB2 = ND² doubles per block, row-major):
//   A.val[npos][NB2]   SELL-64 blocks of A_l, slot 0 of a row = its diagonal
//                      (f64 for the setup and the CG; val32: f32 V-cycle copy)
//   dinv[n][NB2]       block-Jacobi inverse of the diagonal blocks (+ f32 copy)
//   b, x, t, e [n][ND] f32 V-cycle right-hand side, iterate, residual, output
//   P.val[npos_P][NB2] smoothed prolongator (rows = level l, cols = level l+1)
//   R.val32[npos_R][NB2] P transposed: coarse row → fine rows (rp: the P position)
//   apval[npos_AP][NB2] A_l·P_l (setup only)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace mfea {

// The rows of a matrix this rank computes (distributed V-cycle, amg.hpp
// AmgRank; one partition: all of them) and their SELL positions.  A 64-row
// slice ignores ownership, so the range's first and last slices may hold
// other ranks' rows: positions below pf / from pl on are checked (pos_mine).
struct RowRange {
  int64_t lo = 0, hi = 0;  // rows [lo, hi)
  int64_t p0 = 0, p1 = 0;  // SELL positions [p0, p1) of the slices holding them
  int64_t pf = 0, pl = 0;  // end of the first slice's positions, start of the last's
  int64_t s0 = 0, s1 = 0;  // first / last slice
  int64_t rows() const { return hi > lo ? hi - lo : 0; }
  // row kernels sweep from the slice boundary below lo (a wave's 64 rows
  // must share one slice: slice_of reads the wave's first lane) and mask
  // the rows below lo
  __host__ __device__ int64_t lo64() const { return lo & ~(int64_t)63; }
  int64_t span() const { return hi > lo ? hi - lo64() : 0; }
  int64_t npos() const { return p1 > p0 ? p1 - p0 : 0; }
};

struct AmgMatD {
  int64_t n = 0;     // rows
  int64_t npos = 0;  // SELL positions (slot rows · 64)
  int32_t wmax = 0;  // widest slice (host side: launch geometry)
  RowRange rg;       // rows this rank computes
  const int32_t* sptr = nullptr;
  const int32_t* srow = nullptr;  // slot row → its slice (the setup's one-wave-per-slot-row grids)
  const int32_t* col = nullptr;
  double* val = nullptr;   // [npos][NB2] f64 (setup)
  float* val32 = nullptr;  // [npos][NB2] f32 copy for the V-cycle (levels ≥ 1)
  // A_0 only (every block symmetric: K_ij = −Σ S_e, K_ii = Σ S_e + reg·I):
  // the upper triangles, [npos][ND(ND+1)/2], for the CG's w = A u (f64) and
  // the level-0 V-cycle kernels (f32) — 3/4 (ND = 2) of the full blocks' bytes
  double* sym = nullptr;
  float* sym32 = nullptr;
  // the compact cycle: Ã = ω D⁻¹ A (f32 full blocks) of the smoothed part c = 2x − Ã x
  float* at32 = nullptr;
};

struct AmgLevD {
  AmgMatD A;
  double* dinv = nullptr;
  float* dinv32 = nullptr;
  double* omega = nullptr;  // [2]: [1] = Gershgorin bound g_l; [0] > 0: ρ̂_l in place of max(2, g_l / 1.45) (ω_l = amg_omega(omega))
  // V-cycle vectors [n][ND], f32 (level 0: b = the CG's r, e = the CG's u, f64)
  float* b = nullptr;
  float* x = nullptr;
  float* t = nullptr;
  float* e = nullptr;
  int coarsest = 0;
  int rlanes = 0;  // restriction lanes per coarse row (0: by R's mean width)
  int dsplit = 0;  // compact down sweep: its two row sets as two launches
  int vlanes = 0;  // collapsed cycle: lanes per V row (0: by V's mean width)
  int small_lanes = 65536;  // wide rows of a level under this many threads at 8 lanes take 16 (0: never)
  int alanes = 0;  // lanes per row of the f32 operator below level 0 (0: by A's)
  int tail_lds = 1;  // the tail starting at this level keeps its vectors in LDS (if they fit)
  int ulanes = 0;    // compact up sweep: lanes per P̃ row (0: by P̃'s mean width)
  int x1 = 0;        // the numeric setup's launches over this level run on one XCD (amg.hip setup_block)
  int fixed_omega = 0;  // ω from omega[0] (no Gershgorin bound): the fused setup forms D⁻¹ with A (k_amg_ac)
  int a0slot = 0;       // level 0 (fixed ω, not a0full): one thread per position (k_amg_a0slot)
  int a0full = 0;       // level 0 (fixed ω): A_0, D⁻¹, Ã_0 and P_0 in one row pass (k_amg_a0full)
  // transfer to level l+1 (not on the coarsest level)
  AmgMatD P;
  // level 0 of a hierarchy kept over element failures: rows of floating
  // pieces (kernels.hpp launch_floating), whose P rows are formed as zero
  const uint8_t* fmask = nullptr;
  const int32_t* agg = nullptr;
  const int32_t* pv_ptr = nullptr;
  const int32_t* pv_a = nullptr;
  AmgMatD R;  // val32 = Pᵀ blocks in R's layout (setup)
  const int32_t* rp = nullptr;
  float* apval = nullptr;  // A_l·P_l blocks (f32 storage; the setup computes in f64)
  AmgMatD AP;  // pattern only (sptr, col) + npos; values in apval
  const int32_t* ap_ptr = nullptr;
  const int32_t* ap_a = nullptr;
  const int32_t* ap_b = nullptr;
  const int32_t* ac_ptr = nullptr;  // into level l+1's A.val
  const int32_t* ac_a = nullptr;
  const int32_t* ac_b = nullptr;
  RowRange ac_rg;  // level l+1's A rows this rank's Galerkin product forms (= R's rows)
  int ac_lanes = 1;  // lanes per output block of the Galerkin product (by its lists' mean length)
  // the compact cycle (amg.hpp AmgLevel::PT): P̃ (f32, PT.val32) and the scaled
  // restriction R̂ = s' D'⁻¹ P̃ᵀ D / ω (RT.val32; s' = ω' or 1 on the coarsest
  // level), formed by launch_amg_compact_setup once every level is set up
  int compact = 0;
  AmgMatD PT, RT;
  const int32_t* pt_row = nullptr;  // PT row → level row (P̃ has A·P's row order)
  const int32_t* pt_ap = nullptr;
  const int32_t* pt_p = nullptr;
  const int32_t* rt_pt = nullptr;
  const int32_t* rt_row = nullptr;  // RT row → level l+1 row (R̂ rows by length)
  // the compact cycle collapsed below this level (amg.hpp AmgCollapse, levels
  // ≥ kc): T = V_{l+1} R̂ (rows: level l+1) and V (rows by length, vrow → level
  // row), both f32 (val32), with their product lists; V.n > 0 on level kc
  // makes the cycle apply V there instead of recursing
  AmgMatD CT, CV;
  const int32_t* ct_ptr = nullptr;
  const int32_t* ct_a = nullptr;
  const int32_t* ct_b = nullptr;
  const int32_t* cv_row = nullptr;
  const int32_t* cv_ptr = nullptr;
  const int32_t* cv_a = nullptr;
  const int32_t* cv_b = nullptr;
  const int32_t* cv_ext = nullptr;   // Ã position of the block or −1
  const int32_t* cv_diag = nullptr;  // 1: + 2I
  int collapsed = 0;  // 1 on levels ≥ kc that hold CT / CV
};

// Levels 0 and 1 merged around a cycle collapsed at level 2 (amg.hpp AmgMerge):
// DQ (rows: c_1's, then x_2's; dq_dst: their index in B) and U = [P̃_0 | P̃_0 P̃_1]
// (P̃_0's row order), f32 values formed every setup from the lists; B the
// cycle's vectors [c_1 | x_2 | e_2 | scratch] (level 2's x and e point into it).
struct AmgMergeD {
  int on = 0;
  int64_t n1 = 0, n2 = 0;
  AmgMatD DQ, U;
  const int32_t* dq_dst = nullptr;
  int64_t dq_split = 0;
  const int32_t* dq_ext = nullptr;
  const int32_t* dq_ptr = nullptr;
  const int32_t* dq_a = nullptr;
  const int32_t* dq_b = nullptr;
  const int32_t* u_ext = nullptr;
  const int32_t* u_ptr = nullptr;
  const int32_t* u_a = nullptr;
  const int32_t* u_b = nullptr;
  float* B = nullptr;
};
// the merged operators' values (after the levels' setup and the collapse)
void launch_amg_merge_setup(hipStream_t s, int nd, const AmgLevD* lev, const AmgMergeD& m);

// CG vectors of the AMG path (f64): free rows in level-0 order, ND per row
struct AmgCg {
  int64_t n = 0;
  int64_t lo = 0, hi = 0;  // level-0 rows this rank iterates (one partition: [0, n))
  __host__ __device__ int64_t lo64() const { return lo & ~(int64_t)63; }
  int w_block = 0;  // w = A u kernel threads per block (0: by size)
  int w_k = 1;      // w = A u: 2 — slices up to 2U blocks wide in one round trip (sell_mac's K)
  const int32_t* row0 = nullptr;  // level-0 row → Pattern (row-order) free row
  double* x = nullptr;
  double* p = nullptr;
  double* s = nullptr;
  double* r = nullptr;  // level 0's V-cycle input
  double* w = nullptr;
  float* u = nullptr;   // level 0's V-cycle output: the f32 cycle's values, stored
                        // exactly (half the bytes of f64 for every gather of u)
  // 1: the compact cycle (two sweeps per level, AmgLevD::PT) where every
  // level of the cycle has it (compact set: unsplit levels); 0: four steps
  int cycle = 0;
  int coll = 0;  // the compact cycle's collapsed level kc (0: none)
  int sweep = 0;  // 1: the preconditioner is a multicolour sweep (sweep.hip): u is its output only
};

// Whole-matrix SSOR / IC(0) in the chain-piece multicolour order (sweep.hip,
// amg.hpp SweepPlan): the plan's entry arrays and the per-solve values the
// setup launch(es) form from A_0 — the predecessor blocks pv, the cross
// blocks lov / upv (f32, [item][ND²]), D̃⁻¹ (f32 upper triangles: SOR D⁻¹,
// ICC the DIC(0) pivots formed in f64) — and the sweeps' f64 iterate y.
constexpr int kSweepPieceLen = 64;   // rows per piece at most (one wave)
constexpr int kSweepMaxColors = 32;
constexpr int kSweepBS = 256;        // threads per workgroup
struct SweepD {
  int64_t n = 0;   // level-0 rows
  int64_t ne = 0;  // entries (64 per wave)
  int colors = 0;
  int dic = 0;
  int32_t cw[kSweepMaxColors + 1] = {};  // colour → first wave
  const int32_t* wsteps = nullptr;
  const int32_t* row = nullptr;
  const int32_t* ppos = nullptr;
  const int32_t* dpos = nullptr;
  const int32_t* lo_ptr = nullptr;
  const int32_t* lo_ent = nullptr;
  const int32_t* lo_pos = nullptr;
  const int32_t* up_ptr = nullptr;
  const int32_t* up_ent = nullptr;
  const int32_t* up_pos = nullptr;
  float* pv = nullptr;
  float* dt = nullptr;
  float* lov = nullptr;
  float* upv = nullptr;
  double* y = nullptr;
};
void launch_sweep_setup(hipStream_t s, int nd, const SweepD& sw, const AmgLevD& L0);
void launch_sweep(hipStream_t s, int nd, const SweepD& sw, const AmgCg& cg, const int32_t* gate);

// Partitioned solve (amg.hpp AmgHalo): this partition's rank, the gathered
// per-rank partial sums, its ghost couplings and the u halo buffers.
struct AmgDist {
  int rank = 0;
  int zero_w = 0;  // > 0: the sums travel as one all-reduce over [zero_w][4] (the other rows zeroed)
  double* gall[2] = {nullptr, nullptr};  // [64][4] per-rank partial sums by parity
  double* gsend = nullptr;               // [4] this rank's, sent to every rank
  const int32_t* gptr = nullptr;         // per level-0 row: ghost couplings
  const int32_t* gslot = nullptr;        //   SELL slot of K_ig in the assembled operator
  const int32_t* grecv = nullptr;        //   the ghost's index in urecv
  const double* sval = nullptr;          // assembled SELL values val[6][G]
  int64_t G = 0;
  const int32_t* send_rows = nullptr;    // level-0 rows whose u the peers hold as ghosts
  int64_t n_send = 0;
  double* usend = nullptr;               // [n_send][ND]
  const double* urecv = nullptr;         // [n_recv][ND]
};

// ---- numeric setup (every solve) ------------------------------------------
// A_0 from the assembled SELL operator: off-diagonal = Σ of the listed slots'
// K_ij (= −S_e), diagonal = K_ii + reg·I; then level 0's D⁻¹ and bound.
void launch_amg_a0(hipStream_t s, int nd, const AmgLevD& L0, const SellOp& sop, const int32_t* row0,
                   const int32_t* a0_ptr, const int32_t* a0_a, double reg, bool full = false);
// dinv, Gershgorin bound and ω of one level; then P, A·P and A_{l+1}
// (level0: its D⁻¹ was formed by launch_amg_a0).  stage: which of the four
// steps (the distributed setup exchanges values between them)
constexpr int kSetupDinv = 1, kSetupP = 2, kSetupAP = 4, kSetupAC = 8, kSetupAll = 15;  // (kSetupAP: + P̃, R̃)
void launch_amg_level_setup(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD* next, bool level0,
                            int stage = kSetupAll);
// the compact cycle's operators of every level from l0 (after every level's
// setup: R̂ needs the next level's D⁻¹ and ω): P̃, R̂, Ã; then, deepest first,
// the collapsed operators T, V of levels ≥ kc (coll > 0)
void launch_amg_compact_setup(hipStream_t s, int nd, const AmgLevD* lev, int nlev, int coll = 0, int l0 = 0);
// ... of one level, on its row ranges (the distributed setup exchanges P̃ and
// diagonal blocks between forming P̃ and R̂)
constexpr int kCompactPT = 1, kCompactRT = 2, kCompactAT = 4, kCompactAll = 7;
void launch_amg_compact_level(hipStream_t s, int nd, const AmgLevD* lev, int l, int parts);
// one compact sweep of level L on its row ranges: down (x_{l+1} = R̂ x_l into
// N.x, c_l = 2x_l − Ã x_l into L.t) and up (e = c_l + P̃ e_{l+1})
void launch_amg_down(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD& N);
void launch_amg_up(hipStream_t s, int nd, const AmgLevD& L, const AmgLevD& N, float* e);
// the levels' setup (after launch_amg_a0) and the compact operators in one
// sequence, the compact parts fused into the Galerkin chain's launches
// (mg: the merged levels' products ride in the collapse launches; returns
// whether they did — else launch_amg_merge_setup forms them)
bool launch_amg_setup_fused(hipStream_t s, int nd, const AmgLevD* lev, int nlev, int coll,
                            const AmgMergeD* mg = nullptr);
// ---- one V-cycle u = M r (the CG's r → the CG's u); gate = NULL: always,
// else only while *gate == kRun.  tail > 0: levels [tail, nlev) run in one
// single-workgroup launch (k_amg_tail_lds / k_amg_tail, the views passed by value).
// l0 > 0: only levels [l0, nlev), on level l0's b and x (its output: e).
void launch_amg_vcycle(hipStream_t s, int nd, const AmgLevD* lev, int nlev, const AmgCg& cg,
                       int tail, const int32_t* gate, int l0 = 0, const AmgMergeD* mg = nullptr);
// one step of the V-cycle on level l (the distributed schedule interleaves
// exchanges): t = b − A x, restriction into level l+1, x += P e_{l+1}, post-smoothing
constexpr int kStepResid = 0, kStepRestrict = 1, kStepProlong = 2, kStepPost = 3;
void launch_amg_vstep(hipStream_t s, int nd, const AmgLevD* lev, int l, const AmgCg& cg, int step,
                      const int32_t* gate);
// ---- exchanges of the distributed V-cycle and setup (amg.hpp XPlan): items
// of `width` scalars, gathered into / scattered from a contiguous buffer
void launch_xpack(hipStream_t s, const void* src, const int32_t* idx, int64_t n, int width, int bytes, void* buf);
// partitions on one device: an exchange's transfers between partitions in one
// launch, straight from the sender's array to the receiver's (off: prefix of
// the pairs' item counts)
constexpr int kMaxXPairs = 48;
struct XPairs {
  int n = 0;
  int64_t off[kMaxXPairs + 1] = {};
  const void* src[kMaxXPairs] = {};
  void* dst[kMaxXPairs] = {};
  const int32_t* sidx[kMaxXPairs] = {};
  const int32_t* ridx[kMaxXPairs] = {};
};
void launch_xcopy(hipStream_t s, const XPairs& pr, int width, int bytes);
struct GallCopy {
  int n = 0;
  const double* gsend[64] = {};
  double* gall[64] = {};
  int rank[64] = {};
};
void launch_gall_copy(hipStream_t s, const GallCopy& g);
void launch_xunpack(hipStream_t s, const void* buf, const int32_t* idx, int64_t n, int width, int bytes, void* dst);
// the first smoothing step x = s·D⁻¹ b (s = ω, 1 on the coarsest level) of
// the listed rows of level N (the rows the replicated level's all-gather brought)
void launch_amg_xinit_rows(hipStream_t s, int nd, const AmgLevD& N, const int32_t* rows, int64_t n,
                           const int32_t* gate);
// partitions on one device: every partition's Gershgorin bound g (omega[1])
// set to the maximum over them (what an RCCL all-reduce max does across GPUs)
void launch_amg_bound_max(hipStream_t s, double* const* omegas, int n);
// lanes per row of level L's restriction (1, 2, 4, 8) and of its f32
// operator below level 0 (1, 2, 4): by the mean slice width, or the option
int amg_restrict_lanes(const AmgLevD& L);
int amg_op_lanes(const AmgLevD& L);
// the compact cycle: lanes per row of its down (R̃) and up (P̃) sweeps; whether
// levels [l0, nlev) all have it
int amg_down_lanes(const AmgLevD& L);
int amg_up_lanes(const AmgLevD& L);
bool amg_compact_ok(const AmgLevD* lev, int nlev, int l0);
// first level l ≥ 1 (above the coarsest) with at most max_rows rows, or 0
int amg_tail_level(const int64_t* rows, int nlev, int64_t max_rows);
// ---- CG (single-reduction, as cg.hip) ---------------------------------------
// r = b (row-order 3-comp RHS of k_cg_rhs), x = p = s = 0, level-0 x = ω D⁻¹ r
void launch_amg_cg_init(hipStream_t s, int nd, const AmgLevD& L0, const AmgCg& cg, const double* b_row);
// w = A_0 u (+ the ghost couplings when d), partials (γ, δ, ‖r‖², ‖u‖²) →
// parity; first: slots[0] = INIT, parity 0
void launch_amg_cg_w(hipStream_t s, int nd, int j, bool first, const AmgLevD& L0, const AmgCg& cg,
                     Slot* slots, double* part, const AmgDist* d = nullptr);
// partitioned: this rank's block partials of parity q → gall[q] row rank, gsend
void launch_amg_gsum(hipStream_t s, const AmgCg& cg, const double* part_q, const AmgDist& d, int q);
// partitioned: u of the send rows → usend
void launch_amg_pack_u(hipStream_t s, int nd, const AmgCg& cg, const AmgDist& d);
// iteration j: α, β from the partials (d: from the gathered rank sums), p s x
// r update, level-0 x = ω D⁻¹ r
void launch_amg_cg_update(hipStream_t s, int nd, int j, const AmgLevD& L0, const AmgCg& cg,
                          Slot* slots, SolveState* st, double* part,
                          const AmgDist* d = nullptr);
// x (level-0 order, ND per row) → row-order x[3·row + c]
void launch_amg_finish(hipStream_t s, int nd, const AmgCg& cg, double* x_row);
// grid of the w kernel (its partials are re-read by the update kernel)
int64_t amg_w_grid(const AmgCg& cg);

}  // namespace mfea
