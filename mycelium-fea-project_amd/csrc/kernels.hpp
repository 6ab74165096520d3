// kernels.hpp — device kernels of the mfea engine (gfx950 / CDNA4, wave64).
//
// Data layout in HBM (all f64 unless noted), rows = nodes in the permuted
// order of symbolic.cpp (free rows [0,nf), top grip rows, bottom rows):
//   xyz[3N]            node coordinates, interleaved x,y,z
//   slice_ptr[ns+1]    SELL-64 slot offsets; row_len[N] incident elements
//   s_col/s_elem[G]    per slot (slot t, lane l at t·64+l): neighbour row, element
//   val[6][G]          per slot K_ij = −S_e, six symmetric components (SoA)
//   diag[6][N]         per row K_ii = Σ S_e (unregularised)
//   x,r,p,q[3N]        PCG vectors, interleaved DOFs (x holds the full U)
//   dinv[3N] / binv[6N] Jacobi / 3×3 block-Jacobi inverse
// Components of a symmetric 3×3 block: 0 xx, 1 xy, 2 xz, 3 yy, 4 yz, 5 zz.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfea {

constexpr int kBlock = 256;  // 4 wavefronts
constexpr int kTicketStride = 256;  // unsigned per reduction ticket set (device_util.hpp)

// PCG per-iteration scalar slot (see DESIGN.md "PCG scalar slots").
// v[0] = p·q, v[1] = r·z, v[2] = r·r, v[3] = z·z (v[1..3] reduced together),
// flag: 0 RUN, 1 STOP (propagated / after done), 2 BREAKDOWN.
// Single-reduction CG (Chronopoulos–Gear) uses v[0] = γ = r·u, v[1] = δ = w·u,
// v[2] = r·r, v[3] = u·u (reduced together), and the scalars the next
// iteration consumes, computed once by the reducing block: alpha, beta, res
// (the stopping norm², r·r or u·u).  The HS kernels of the CSR path use
// v[0] = p·q, v[1] = r·z, v[2] = r·r, v[3] = z·z.
struct Slot {
  double v[4];
  double alpha;
  double beta;
  double res;
  int32_t flag;
  int32_t pad;
};
enum SlotFlag : int32_t { kRun = 0, kStop = 1, kBreakdown = 2, kInit = 3, kConverged = 4, kMaxit = 5 };

// Device pointers of the node-block (SELL-64) operator and the CG-CG state.
struct SellOp {
  int64_t N, nf, G;
  const int32_t* slice_ptr;
  const int32_t* row_len;
  const int32_t* s_col;
  const double* val;   // 6 × G
  const double* diag;  // 6 × N
};
struct CgVecs {
  double* x;     // 3N (known rows hold the prescribed values)
  double* p;     // 3N
  double* r[2];  // double-buffered by iteration parity
  double* s[2];
  double* w[2];
  double* dinv;  // 3N (Jacobi) or 6N (3×3 block Jacobi); 0 on known rows
};

struct SolveState {
  double tol2;     // stopping threshold on the chosen norm²
  double reg;      // diagonal regularisation
  double bb0;      // ‖b‖²
  double res_final;
  int32_t base;    // absolute iteration index of slot 0
  int32_t max_it;
  int32_t norm;    // 0 unpreconditioned (‖r‖), 1 preconditioned (‖z‖)
  int32_t done;
  int32_t iters;
  int32_t status;  // 0 converged, -4 maxit, -5 breakdown
  int32_t pad[2];
  double res0;     // initial value of the chosen norm² (‖b‖² or ‖M⁻¹b‖²)
  double rtol2;    // rtol², atol²: the AMG / sweep CG forms tol2 for the preconditioned
  double atol2;    // norm from its first ‖u₀‖² = ‖M⁻¹b‖² (k_amg_cg_update)
};

struct Material {
  double EA;    // E·A            (src/fea_solver.py:45 numerator)
  double EI12;  // (12·E)·I       (src/fea_solver.py:58 numerator)
  double E;     // for stress = E·ε (src/fea_solver.py:271)
};

// ---- launchers (defined in kernels.hip) -------------------------------------
// The GAMG solves' RHS formed in the assembly's row pass (k_amg_rhs's work:
// b = 0 − K_fk x_k of the free rows into r, the prescribed x of the others,
// ‖b‖² published to red) — rhs == nullptr: assembly alone
struct AsmRhs {
  const uint8_t* code;
  double dy_top, dy_bot;
  const double* dyp;  // non-null: (dy_top, dy_bot) from device memory (a captured step graph)
  // row classes by position (symbolic.hpp Pattern): top grip rows
  // [nf, top_end), bottom rows [top_end, bot_end), ghost rows after
  int64_t top_end, bot_end;
  int64_t nf;
  double* r;
  double* x;
  double* partials;
  unsigned* ticket;
  double* red_out;
};
void launch_assemble(hipStream_t s, int64_t N, const double* xyz, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const int32_t* s_elem,
                     const uint8_t* active, Material m, int64_t G, double* val, double* diag,
                     const AsmRhs* rhs = nullptr);

// element-centric assembly over an element colouring (symbolic.hpp
// ElemColour; cstart on the host): diag zeroed, then one launch per colour
void launch_assemble_colour(hipStream_t s, int colors, const int32_t* cstart, const int32_t* entry,
                            const int32_t* e2n, const int32_t* epos, const double* xyz, const uint8_t* active,
                            Material m, int64_t G, int64_t N, double* val, double* diag);

// element pass (−S_e to both slots, one launch) + row pass (diagonal blocks
// in slot order: K bit for bit the row gather's)
void launch_assemble_elems(hipStream_t s, int64_t E, int64_t N, const int32_t* e2n, const int32_t* epos,
                           const double* xyz, const uint8_t* active, Material m, const int32_t* slice_ptr,
                           const int32_t* row_len, int64_t G, double* val, double* diag);

void launch_rhs_init(hipStream_t s, int64_t N, int64_t nf, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const double* val,
                     const double* diag, int64_t G, const uint8_t* code, double dy_top,
                     double dy_bot, double reg, int precond, double* x, double* r, double* p,
                     double* dinv, double* partials, unsigned* ticket, double* red_out);

void launch_init_finalize(hipStream_t s, const double* red, double rtol, double atol, int norm,
                          int max_it, double reg, Slot* slots, SolveState* st);

void launch_spmv_sell(hipStream_t s, int j, int64_t nf, int64_t N, const int32_t* slice_ptr,
                      const int32_t* row_len, const int32_t* s_col, const double* val,
                      const double* diag, int64_t G, const double* p, double* q, Slot* slots,
                      const SolveState* st, double* partials, unsigned* ticket);

void launch_update(hipStream_t s, int j, int64_t n, int precond, double* x, double* r,
                   const double* p, const double* q, const double* dinv, Slot* slots,
                   const SolveState* st, double* partials, unsigned* ticket);

void launch_direction(hipStream_t s, int j, int64_t n, int precond, const double* r, double* p,
                      const double* dinv, const Slot* slots, const SolveState* st);

void launch_advance(hipStream_t s, int chunk, Slot* slots, SolveState* st);

void launch_reaction(hipStream_t s, int64_t row0, int64_t nrows, int64_t N,
                     const int32_t* slice_ptr, const int32_t* row_len, const int32_t* s_col,
                     const double* val, const double* diag, int64_t G, const double* u,
                     double* partials, unsigned* ticket, double* red_out);

// owned (multi-partition): count only elements this partition reports; NULL = all.
// fail_list / fail_cnt: the (owned) elements that fail in this launch are
// appended (any order; NULL = no list)
// k_stress's failures undone: listed elements active again, counter zero
void launch_unfail(hipStream_t s, const int32_t* fail_list, unsigned* cnt, uint8_t* active);
void launch_stress(hipStream_t s, int64_t E, const int32_t* e2n, const double* xyz,
                   const double* u, Material m, double max_strain, uint8_t* active,
                   double* stress, double* partials, unsigned* ticket, double* red_out,
                   const uint8_t* owned = nullptr, int32_t* fail_list = nullptr, unsigned* fail_cnt = nullptr);

void launch_element_stiffness(hipStream_t s, int64_t n, const double* p1, const double* p2,
                              Material m, double* Ke, double* L);

// floating free rows of the active element graph given as the SELL-64
// operator pattern (rows [0, n_free) free, [n_free, grip_end) grips; slot
// (row, k): neighbour s_col, element s_elem): mask[label[i]] = 1 for a free
// row i whose component holds no grip row (label NULL: i).  parent /
// anchored: n_rows scratch each.  Four launches, no host wait.
void launch_floating(hipStream_t s, int64_t n_rows, int64_t n_free, int64_t grip_end, const int32_t* slice_ptr,
                     const int32_t* row_len, const int32_t* s_col, const int32_t* s_elem, const uint8_t* active,
                     int32_t* parent, uint8_t* anchored, const int32_t* label, uint8_t* mask,
                     int tile_rows = 2048);

// generic scalar-CSR operator (mfea_solve_csr)
void launch_csr_rhs_init(hipStream_t s, int64_t n, const int64_t* indptr, const int32_t* indices,
                         const double* data, const uint8_t* known, const double* kval, double reg,
                         double* x, double* r, double* p, double* dinv, double* partials,
                         unsigned* ticket, double* red_out);
void launch_spmv_csr(hipStream_t s, int j, int64_t n, const int64_t* indptr,
                     const int32_t* indices, const double* data, const uint8_t* known,
                     double reg, const double* p, double* q, Slot* slots, const SolveState* st,
                     double* partials, unsigned* ticket);

// ---- single-reduction CG on the SELL operator (one kernel per iteration) ----
// k_cg_rhs: b, M⁻¹, x, r₀ = b, p = s = w = 0; reduces (b·b, u₀·u₀) into red[0..1].
// precond 0 Jacobi, 1 block Jacobi, 2 the GAMG solves (k_amg_rhs: b and the
// known rows' x only, u₀·u₀ = 0).
void launch_cg_rhs(hipStream_t s, const SellOp& op, const uint8_t* code, double dy_top,
                   double dy_bot, double reg, int precond, const CgVecs& v, double* partials,
                   unsigned* ticket, double* red_out);
// part: 2 parity buffers × [4][kCgMaxPartials] block partials (cg.hip)
constexpr int kCgMaxPartials = 512;
// k_cg_first: w₀ = A u₀; block partials (γ₀, δ₀, r·r, u·u) → part parity 0;
// slots[0].flag = kInit.
void launch_cg_first(hipStream_t s, const SellOp& op, double reg, int precond, const CgVecs& v,
                     Slot* slots, double* part);
// iteration j of a chunk: reduces part parity j&1, records slots[j+1], writes
// its partials to parity (j&1)^1.
void launch_cg_iter(hipStream_t s, int j, const SellOp& op, int precond, const CgVecs& v,
                    Slot* slots, const SolveState* st, double* part,
                    unsigned long long* trace = nullptr);
// host: mapped pinned mirror of the final SolveState (written once, when done)
void launch_cg_advance(hipStream_t s, int chunk, Slot* slots, SolveState* st, SolveState* host, int shift = 0);
void launch_cg_init_finalize(hipStream_t s, const double* red, double rtol, double atol, int norm,
                             int max_it, double reg, SolveState* st,
                             double* zero = nullptr, int64_t nzero = 0);
int cg_block_size(int64_t rows);
int64_t cg_grid(int64_t rows);

// ---- single-reduction CG on the wave-local lane operator (ell.hip) --------
constexpr uint32_t kSrcNone = 0xFF, kSrcHalo = 0xFE;  // slot source codes (symbolic.hpp)
// Lane arrays are component-major: a[c·NL + lane].  See symbolic.hpp "Ell".
struct EllOp {
  int64_t NL;                // lanes, multiple of 64
  int nd;                    // DOFs per node in the lanes: 2 (planar mesh) or 3
  const uint32_t* code;      // bytes 0..2: slot sources; byte 3: int8 group info
  const int32_t* partner;    // slot-0 halo push: compact record index, -1 none,
                             // -2 - pair for a cross-partition record
  const int32_t* lane_row;   // owner lane → free row, -1
  const int32_t* src_pos;    // [3][NL] SELL position of each slot, -1
  const int32_t* nbr_lane;   // [3][NL] neighbour owner lane (first iteration only)
  double* V;                 // [NB][3][NL] slot blocks (component c, slot k: (c·3+k)·NL)
  double* D;                 // [NB][NL] diagonal block (unregularised), 0 off owners
                             // NB = 6 (xx xy xz yy yz zz) or, nd = 2, 3 (xx xy yy)
  int hc;                    // 1: compact halo records, 0: one record per lane
  int64_t NR;                // stride of h / hM: records (+1 spare) or NL
  const uint64_t* hmask;     // [NL/64] lanes of each wave owning a halo record
  const int32_t* hbase;      // [NL/64] the wave's first record
  int bs = 256;              // launch geometry (handle options): threads per block
  int64_t maxg = 0;          // grid cap below kCgMaxG (0: none)
};
struct EllVecs {  // component c of a lane vector at [c·NL + lane], c < nd
  double* x;      // [3][NL]
  double* p;      // [3][NL]
  double* r[2];   // [3][NL] by iteration parity
  double* s[2];
  double* w[2];
  double* M;      // [3|6][NL] Jacobi / block-Jacobi inverse, 0 off owners
  double* h[2];   // [9][NR] halo records by parity: r, s, w of the slot-0 neighbour at (q·3+c)·NR
  double* hM;     // [3|6][NR] halo record of the slot-0 neighbour's M
};
// ---- multi-partition CG (partition.hpp; one partition per GPU) -------------
// Cross-partition halo records, pair k (partition.hpp) at rec[k·RW + q·nd + c]
// with RW = 3·nd (q = 0 r, 1 s, 2 w).  The exchange before w₀ = A u₀ carries
// [r₀ | M] in the parity-1 slots.  Rank partial sums: gall[par] = [64][4]
// (row = rank, rows >= world stay 0), summed by every wave in a fixed order,
// so every rank derives bitwise the same α, β and stopping decision.
struct DistVecs {
  double* xs[2];    // [NX][RW] records this partition sends, by parity
  double* xr[2];    // [NX][RW] records received from the peers
  double* mr;       // [NX][NM] the peers' M (kept from the first exchange)
  double* gall[2];  // [64][4] partial sums of every rank, by parity
  double* gsend;    // [4] this partition's partial sums
};
constexpr int kMaxRanks = 64;

// values and lane vectors from the SELL operator and k_cg_rhs's row-order b, M⁻¹
void launch_ell_init(hipStream_t s, const EllOp& op, const SellOp& sop, int precond,
                     const CgVecs& rv, const EllVecs& v);
// multi-partition: [r₀ | M] of each remote-halo lane's owner → xs[1]
void launch_ell_pack0(hipStream_t s, const EllOp& op, int precond, const EllVecs& v,
                      const DistVecs& dv);
// w₀ = A u₀ (neighbours pulled once), halo records of parity 0, partials, slots[0] = INIT
void launch_ell_first(hipStream_t s, const EllOp& op, double reg, int precond, const EllVecs& v,
                      Slot* slots, double* part, const DistVecs* dv = nullptr);
void launch_ell_iter(hipStream_t s, int j, const EllOp& op, int precond, const EllVecs& v,
                     Slot* slots, const SolveState* st, double* part,
                     unsigned long long* trace = nullptr, const DistVecs* dv = nullptr);
// launch geometry of the lane CG kernels: threads per block; blocks (≤ 512,
// their partials re-reduced by every wave of the next launch)
int ell_block_size(const EllOp& op);
int64_t ell_grid_size(const EllOp& op);
// x of the owner lanes → row-order x (free rows)
void launch_ell_finish(hipStream_t s, const EllOp& op, const EllVecs& v, double* x_row);
// this partition's block partials of the iteration (parity buffer `p`, the
// iteration kernel's grid for NL lanes) → row[0..3] and gsend[0..3]
void launch_psum(hipStream_t s, const EllOp& op, const double* p, double* row, double* gsend);
// out[c] = Σ_{r < world} g[4r + c] in rank order
void launch_rank_sum(hipStream_t s, const double* g, int world, double* out);
// out[3i + c] = x[3 rows[i] + c] / x[3 rows[i] + c] = in[3i + c]
void launch_rows_pack(hipStream_t s, const int32_t* rows, int64_t n, const double* x, double* out);
void launch_rows_unpack(hipStream_t s, const int32_t* rows, int64_t n, const double* in, double* x);

int64_t grid_rows(int64_t rows);
int64_t grid_elementwise(int64_t n);

}  // namespace mfea
