// capi.hip — the C ABI of include/mfea.h: handle, device memory, the on-device
// step loop (assemble → RHS → PCG in hipGraph-captured chunks → reaction/stress),
// and the multi-partition driver (partition.hpp): one partition per GPU joined
// over RCCL (mfea_dist_init), or several partitions on one device exchanging
// through device copies (mfea_debug_set_parts; the same kernels and the same
// exchange schedule, used to test the partitioned solve on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <deque>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "amg.hpp"
#include "amg_kernels.hpp"
#include "kernels.hpp"
#include "mfea_debug.h"
#include "mfea.h"
#include "partition.hpp"
#include "records.hpp"
#include "symbolic.hpp"

using namespace mfea;

namespace {

thread_local std::string g_err;

// MFEA_BUILD_TIMES=1 (as amg_symbolic.cpp's build split): the host side of a
// new active set on stderr — failed-id tracking, plan build, upload, mask
struct HostLap {
  bool on = std::getenv("MFEA_BUILD_TIMES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what, int64_t n = -1) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    if (n >= 0)
      std::fprintf(stderr, "  host %-26s %8.3f ms  (%lld)\n", what, std::chrono::duration<double, std::milli>(now - t).count(), (long long)n);
    else
      std::fprintf(stderr, "  host %-26s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPC(call)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(MFEA_EDEVICE, std::string(#call) + ": " + hipGetErrorString(e_));       \
  } while (0)

#define NCCLC(call)                                                                       \
  do {                                                                                    \
    ncclResult_t r_ = (call);                                                             \
    if (r_ != ncclSuccess)                                                                \
      return fail(MFEA_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_));        \
  } while (0)

#define RC(call)                  \
  do {                            \
    if (int rc_ = (call)) return rc_; \
  } while (0)

template <class T>
struct DevBuf {
  T* ptr = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= n && ptr) return hipSuccess;
    release();
    n = count;
    return hipMalloc(&ptr, std::max<size_t>(count, 1) * sizeof(T));
  }
};

}  // namespace

// One partition's operator, vectors and solver state on the handle's device.
// Single-GPU handles hold one partition covering the whole mesh.
struct Part {
  int rank = 0;   // partition index = rank in the partitioned solve
  Pattern P;      // local pattern (the whole mesh when not partitioned)
  PartPlan plan;  // partitioned only
  DevBuf<double> xyz_d, val, diag, x, r, p, q, dinv, stress, partials, red;
  DevBuf<double> cg_r1, cg_s0, cg_s1, cg_w0, cg_w1;  // CG-CG double buffers (r0 = r)
  DevBuf<double> cg_part;                            // CG-CG block partials, 2 parities
  DevBuf<int32_t> slice_ptr, row_len, s_col, s_elem, e2n_d;
  DevBuf<uint8_t> active, code, elem_own;
  DevBuf<int32_t> fail_list;  // (owned) elements failed in the last post (any order)
  DevBuf<unsigned> fail_cnt;
  DevBuf<unsigned> tickets;
  // wave-local lane operator (ell.hip); ell_ok = false → SELL kernel
  Ell L;
  bool ell_ok = false;
  bool ell_hc = false;  // compact halo records (ell_op)
  DevBuf<uint32_t> e_code;
  DevBuf<int32_t> e_partner, e_lane_row, e_src_pos, e_nbr_lane, e_hbase;
  DevBuf<uint64_t> e_hmask;
  DevBuf<double> e_f;  // all lane-operator doubles, carved by ell_op / ell_vecs
  DevBuf<Slot> slots;
  DevBuf<SolveState> state, state_mirror;
  SolveState* mirror = nullptr;  // where k_cg_advance publishes the final state
  int64_t G = 0;                 // slots·64
  // partitioned solve: exchange buffers
  DevBuf<double> xrec;  // xs[2] | xr[2] | mr
  DevBuf<double> gbuf;  // gall[2] | gsend | gred
  DevBuf<double> xh;    // displacement halo: send | recv
  DevBuf<int32_t> xsend_rows, xrecv_rows;
  DistVecs dv{};
  double* gred = nullptr;  // [64][4] gathered scalars (RHS norms, reaction, #active)
  double* xh_send = nullptr;
  double* xh_recv = nullptr;
  // SA-AMG preconditioner (amg.hpp): symbolic plan for the active set amg_key
  AmgPlan amg;
  AmgCollapse amg_coll;  // the compact cycle below level kc as one operator (amg_collapse.cpp)
  AmgMerge amg_mplan;    // levels 0 and 1 merged around the collapsed cycle (amg.hpp AmgMerge)
  AmgMergeD amg_mg;
  float* amg_x2 = nullptr;  // level 2's own x / e (the merged cycle points them into amg_mg.B)
  float* amg_e2 = nullptr;
  bool amg_ok = false;
  std::vector<uint8_t> amg_key;
  int64_t amg_gen = 0;               // bumped on every rebuild (captured graphs hold its pointers)
  int amg_last_iters = 0;            // iterations of the last converged GAMG solve (chunk plan)
  // a hierarchy kept over element failures (option amg_reuse): the activity
  // its floating-row mask reflects, the iterations of its first solve, and
  // whether a later solve degraded enough to rebuild
  DevBuf<uint8_t> amg_fmask;         // level-0 rows of floating pieces (kernels.hpp launch_floating)
  const int32_t* amg_row0_inv = nullptr;  // level-0 label of every free row (carved from amg_i)
  DevBuf<int32_t> cc_parent;         // launch_floating's scratch: component links, anchored roots
  DevBuf<uint8_t> cc_anch;
  // element colouring for the element-centric assembly (option asm_kernel 1),
  // built at first use: ec_state 0 not built, 1 usable, -1 not colourable
  ElemColour ec;
  int ec_state = 0;
  DevBuf<int32_t> ec_entry, ec_pos;
  // the plan's key covers the current activity: act_sub_gen when it was
  // built or last compared (failures only ever shrink the set, so it holds
  // until the activity is set explicitly), and its element count
  int64_t amg_sub_gen = -1;
  int64_t amg_key_count = 0;
  int amg_build_iters = -1;
  // the kept hierarchy's rent (option amg_rebuild_rent): the host time its
  // build took, and the time its solves have spent since on iterations above
  // amg_build_iters — a rebuild is bought once the rent paid reaches its price
  double amg_build_s = 0.0;
  double amg_excess_s = 0.0;
  bool amg_stale = false;
  bool amg_reused = false;           // the last ensure_amg kept a hierarchy built for another set
  int64_t amg_seen_gen = -1;         // act_gen at which the plan / mask last matched the activity
  DevBuf<int32_t> amg_i;             // every index array of the plan, carved
  DevBuf<double> amg_d;              // every f64 value / vector array, carved
  DevBuf<float> amg_f;               // the f32 V-cycle copies and vectors, carved
  std::vector<AmgLevD> amg_lev;      // device views
  DevBuf<AmgLevD> amg_levd;          // … and their device copy (the setup tail reads it)
  bool amg_om_own = false;           // the hierarchy is this partition's own (not a split global one)
  bool amg_om_spatial = false;       // ... on Z-ordered labels (level 0's one-pass setup)
  int amg_tail = 0;                  // first level of the single-workgroup tail (0: none)
  int amg_first = 1;                 // first level the four-step tail may start at (not split)
  AmgCg amg_cg;
  // the plan's preconditioner kind: MFEA_PC_GAMG (the hierarchy) or a
  // one-level plan with multicolour sweeps (MFEA_PC_SOR / MFEA_PC_ICC, sweep.hip)
  int amg_kind = MFEA_PC_GAMG;
  SweepPlan sweep;
  SweepD swd;
  DevBuf<int32_t> sw_i;   // the plan's entry arrays and cross lists
  DevBuf<float> sw_f;     // pv | D̃⁻¹ | lov | upv (formed per solve)
  DevBuf<double> sw_y;    // the sweeps' iterate
  const int32_t* amg_a0_ptr = nullptr;
  const int32_t* amg_a0_a = nullptr;
  // partitioned GAMG (amg.hpp AmgHalo): ghost couplings and the u halo
  AmgHalo amg_halo;
  AmgDist amg_dist;
  DevBuf<int32_t> amg_hi;  // send_rows | gptr | gslot | grecv
  DevBuf<double> amg_hd;   // usend | urecv
  // distributed GAMG over the global hierarchy (mfea_handle::gamg): this
  // partition's rows and exchange plans (amg.hpp AmgRank), the plans' item
  // lists on the device and the staging buffers of one exchange
  AmgRank amg_rank;
  PosList g_a0;                 // its level-0 lists over this partition's pattern
  std::vector<int32_t> g_row0;
  int dev_plan = -1;            // which plan the device arrays hold: 0 its own (pt.amg), 1 the global one
  struct XDev {
    const XPlan* x = nullptr;
    const int32_t* s = nullptr;  // sidx
    const int32_t* r = nullptr;  // ridx
  };
  std::vector<XDev> xd_a, xd_r, xd_p, xd_sp, xd_sap;
  XDev xd_g, xd_sg;
  XDev xd_c, xd_spt, xd_sd;  // the compact cycle split at level 0 (AmgRank::compact)
  DevBuf<int32_t> amg_xi;
  DevBuf<double> amg_xs, amg_xr;
};

struct mfea_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  double E = 2500.0, A = 0.0, I = 0.0;
  Material mat{};
  // host-side mesh/BC (original order)
  int64_t N = 0, Ecount = 0;
  std::vector<double> xyz;
  std::vector<int64_t> e2n;
  uint32_t mesh_flags = 0;
  bool planar = false;  // every z == 0 (the whole mesh)
  std::vector<int64_t> top, bot;
  int64_t n_free_global = 0;
  bool has_mesh = false, dirty = true;
  bool assembled = false;  // the operator holds an assembly since the last (re)build
  std::vector<uint8_t> active_host;  // pending upload, original element order (empty = none)
  std::vector<std::unique_ptr<Part>> parts;
  // partitioning: nparts partitions on this device (world == 1), or this
  // process's partition `rank` of `world` (RCCL)
  int nparts = 1, axis = -1;
  int world = 1, rank = 0;
  ncclComm_t comm = nullptr;
  double dist_timeout_s = 60.0;  // per wait; option "dist_timeout_ms"
  SolveState* h_state = nullptr;       // pinned, 2 entries
  SolveState* d_host_state = nullptr;  // device view of h_state (mapped)
  double* h_red = nullptr;             // pinned
  // graph cache (single partition)
  hipGraphExec_t graph = nullptr;
  int graph_chunk = 0, graph_precond = -1, graph_ell = -1;
  hipGraphExec_t graph_big = nullptr;  // GAMG: the planned batch's long chunks
  int graph_big_chunk = 0, graph_big_ell = -1;
  // GAMG: the planned batch's remainder at its exact length, one graph per
  // length (the expected count moves between solves: failures, rebuilds)
  static constexpr int kRemGraphs = 64;
  hipGraphExec_t graph_rem[kRemGraphs] = {};
  int graph_rem_ell = -1;
  // mfea_step (option "batch_graph"): the planned batch as ONE graph of its
  // exact length with the finish and the post kernels behind it, one graph
  // per length, keyed by the plan and the failure strain
  hipGraphExec_t graph_batch[kRemGraphs] = {};
  // ... and (option "combo_graph") behind the numeric setup in the setup's
  // graph: one graph launch per step, one cached graph per batch length
  hipGraphExec_t graph_combo[kRemGraphs] = {};
  uint64_t graph_combo_key[kRemGraphs] = {};
  int graph_batch_ell = -1;
  double graph_batch_strain = 0.0;
  // GAMG: the numeric setup's launches (≈ 30) as one graph, keyed by a hash
  // of every argument they take (the level views, the level-0 operator, reg)
  hipGraphExec_t graph_setup = nullptr;
  uint64_t graph_setup_key = 0;
  hipEvent_t ev[6] = {};
  hipEvent_t ev_setup = nullptr;
  // option "phase_times": record the phase events (mfea_stats t_*_ms).  Off by
  // default: each event recorded between two kernels left the GPU idle for
  // ≈ 5–10 µs (C2 step 0.771 → 0.737 ms, C3 1.665 → 1.635 without them)
  bool opt_phase_times = false;
  bool ev_setup_used = false;  // the last solve recorded ev_setup (GAMG)
  bool in_step = false;        // mfea_step: the solve's end is waited for by post
  // mfea_step's assembly also formed the GAMG solves' RHS for these grip
  // displacements (AsmRhs); the next solve_amg uses it instead of k_amg_rhs
  bool rhs_fused = false;
  double rhs_dy[2] = {0.0, 0.0};
  // mfea_step, one partition (option "spec_post"): the post kernels and
  // their read-back are enqueued behind the solve's planned batch, before the
  // host waits for it, so the one wait covers both — one host round trip per
  // step instead of two.  spec_on: this step may; spec_launched: enqueued
  // behind the last batch (undone by k_unfail when the solve goes on)
  int opt_spec_post = 1;
  // the solve's entry launches (cg_init, first V-cycle, w, update 0) in the
  // captured setup graph (option "setup_entry")
  int opt_setup_entry = 1;
  // mfea_step, one partition, GAMG / SOR / ICC, graphs on, no phase events:
  // the planned batch, the finish and the post as one captured graph
  int opt_batch_graph = 1;
  // mfea_step likewise: the assembly with the fused RHS and the CG start
  // captured at the head of the setup graph, the grip displacements read from
  // pinned h_red[14..15] by a copy node (option "step_graph").  Off: measured
  // 13 µs slower per step at C2 and C3 (profiles/r6/ab_step_graph_wall.log) —
  // an eager assembly runs while the host checks the plan and the setup
  // graph's key; deferred, the GPU waits for that host work
  int opt_step_graph = 0;
  int opt_graph_start = 1;  // the CG start (k_cg_init_finalize) at the setup graph's head
  // with batch_graph: the batch, finish and post behind the setup in one graph
  int opt_combo_graph = 1;
  bool asm_pending = false;  // mfea_step deferred its assembly to solve_amg
  DevBuf<double> d_dy;
  bool spec_on = false;
  bool spec_used = false;  // one speculative post per step: behind the planned batch only
  bool spec_launched = false;
  double spec_strain = 0.0;
  hipEvent_t poll[2] = {};
  int64_t n_active = 0;
  bool act_all = false;  // every element is active on the device (set_active(NULL), no failure since)
  // host view of the element activity (single partition; keys the AMG plan):
  // exact after set_active / a build, stale once a post kernel deactivated
  // elements (then downloaded on demand)
  std::vector<uint8_t> act_host;
  bool act_host_ok = false;
  int64_t act_count = 0;
  // tuning options (mfea_set_option; defaults from the environment at create)
  bool opt_graph = true;       // single-partition chunks replay as hipGraphs
  bool opt_dist_graph = true;  // partitioned chunks too
  int opt_order = kOrderDFS;   // free-row order (symbolic.hpp)
  int opt_lane_dof = 0;        // 0: 2 DOFs per node on planar meshes, 3: always 3
  int opt_cg_kernel = 0;       // Jacobi CG: 0 by density, 1 lanes, 2 SELL
  int opt_ell_block = 256;     // lane kernels: threads per block
  int64_t opt_ell_maxg = 0;    // lane kernels: grid cap (0: kCgMaxG)
  bool opt_ell_compact = true; // lane kernels: compact halo records
  int64_t opt_amg_tail_rows = 2048;  // GAMG: levels of at most this many rows run in one workgroup
  int opt_amg_max_levels = kAmgMaxLevels;  // GAMG: hierarchy depth cap
  int opt_amg_w_block = 0;     // GAMG: w = A u threads per block (0: by size)
  int opt_amg_rlanes = 0;      // GAMG: restriction lanes per coarse row (0: by width)
  int opt_amg_down_split = 0;  // GAMG compact down sweep: R̂ and Ã rows as two launches (experiment)
  int opt_amg_merge = -1;      // GAMG: levels 0 and 1 merged around a level-2 collapse (-1: small networks, 0 off, 1 on)
  int opt_amg_v_lanes = 0;     // GAMG collapsed cycle: lanes per V row (0: by width; 1, 2, 4, 8, 16)
  int64_t opt_amg_small_lanes = 65536;  // GAMG: wide rows of small levels at 16 lanes below this many threads
  int opt_amg_alanes = 0;      // GAMG: operator lanes per row below level 0 (0: by width)
  int opt_amg_tail_lds = 1;    // GAMG: the single-workgroup tail keeps its vectors in LDS
  int opt_amg_collapse = -1;           // GAMG: collapse the compact cycle below the highest level
                                      // within budget (-1), never (0), or from level ≥ k (k ≥ 1)
  int64_t opt_amg_collapse_mb = 32;     // … budget: the collapsed operator's bytes
  int64_t opt_amg_collapse_pairs = 8000000;  // … budget: its setup products' list items
  int opt_amg_spatial = -1;  // GAMG: rows labelled in Z-order (1), depth-first (0), by locality (-1)
  int opt_amg_up_lanes = 0;  // GAMG compact up sweep: lanes per P̃ row (0: by width)
  // GAMG: ρ̂ of the levels below 0 in ppm (ω_l = 4 / (3 ρ̂)); 0: max(2, g_l / 1.45), the
  // Gershgorin-safe value.  A solve that fails with it falls back to the safe
  // value for the handle's lifetime (amg_safe_omega, omega_fallback).
  int64_t opt_amg_coarse_rho_ppm = 1750000;
  int opt_amg_a0_slot = 1;  // level 0's blocks one thread per position (k_amg_a0slot) at a fixed ω
  bool amg_safe_omega = false;
  int64_t opt_amg_x1_rows = 2048;  // GAMG setup: levels of at most this many rows run on one XCD (0: never;
                                   // C3: levels 4-5 gain 1-2 µs per launch, level 3 at 8192 lost as much)
  int opt_amg_big_chunk = 8;  // GAMG: iterations per chunk of a planned batch (drive_sized)
  int opt_sweep_piece = kSweepPieceLen;  // SOR / ICC: rows per chain piece (amg.hpp SweepPlan)
  int opt_amg_fuse_setup = 1;  // GAMG setup: the compact operators fused into the Galerkin chain's launches
  int64_t opt_amg_theta_ppm = 0;  // GAMG: strength threshold θ·10⁶ of the level-0 aggregation (0: all strong)
  int opt_amg_cycle = 1;       // GAMG: 1 the compact V-cycle (two sweeps per level), 0 four steps
  double opt_part_slack = 0.35;  // partition boundaries: min-cut search window (fraction of a strip)
  // GAMG over element failures: 1 keep the hierarchy (floating pieces masked)
  // until a solve needs more than amg_rebuild_pct % of the iterations of the
  // hierarchy's first solve (+2), then rebuild; 0 rebuild on every new active set
  int opt_amg_reuse = 1;
  // assembly: 0 row gather (one launch, fused GAMG RHS), 1 element colours
  // (a launch per colour), 2 element pass + row pass (two launches)
  int opt_asm_kernel = 0;
  int opt_cc_tile = 1024;  // floating rows on the device: rows per LDS tile (512, 1024, 2048, 4096; C3 73 µs at 512-1024, C5 0.6 ms at 1024-2048)
  int opt_amg_rebuild_pct = 800;
  // ... or once the time its solves spent on iterations above that count
  // reaches this % of the time the last build took (0: off).  Rent-or-buy:
  // a C5 rebuild costs 2.4 s of host work — ≈ 80 steps — so a kept hierarchy
  // that needs 40-100 % more iterations is kept; at most twice the cost of
  // the best choice in hindsight (measured)
  int opt_amg_rebuild_rent = 100;
  int opt_amg_dist = -1;          // partitioned GAMG: 1 the global hierarchy (distributed V-cycle), 0 block
                                  // Jacobi over per-partition hierarchies, -1 whichever solves faster (measured)
  int64_t opt_amg_rep_rows = 32768;  // distributed V-cycle: levels of at most this many rows are replicated
  // distributed V-cycle: 1 the compact cycle with level 0 split and every
  // level below replicated (x_0 halo, x_1 all-gather, u halo: three exchange
  // points per iteration), 0 the four-step cycle over the levels of more than
  // amg_rep_rows rows (four exchange points per split level)
  int opt_amg_dist_cycle = 1;
  // GAMG over RCCL: the CG's per-rank partial sums as ONE ncclAllReduce of
  // [world][4] doubles, every rank's buffer zero but its own row (1; the sum
  // is then each row exactly, summed by every rank in rank order as before),
  // or as world − 1 send / receive pairs per rank (0)
  int opt_dist_sums = 1;
  // distributed GAMG (partitioned handles, option "amg_dist" 1): the whole
  // mesh's pattern and node owners (built with the partitions), and ONE
  // global hierarchy for the current global element activity
  Pattern gpat;
  std::vector<int32_t> gowner;
  AmgPlan gamg;
  std::vector<uint8_t> gamg_key;  // the global activity gamg was built for
  // partitioned: the global element activity on the host, exact at act_gen
  // gkey_gen (set by mfea_set_active, moved by the failed-element ids every
  // post exchanges — global_active)
  std::vector<uint8_t> gkey;
  int64_t gkey_gen = -1;
  DevBuf<int32_t> gfail;  // RCCL: failed-id all-gather buffers
  bool gamg_ok = false;
  int64_t gamg_gen = 0;       // bumped on every upload (captured graphs hold its pointers)
  int64_t gamg_plan_gen = 0;  // bumped on every host rebuild (a new active set)
  int64_t act_gen = 1;        // bumped whenever the element activity may have changed
  int64_t act_sub_gen = 1;    // bumped when it changed other than by failures (set_active, a rebuild)
  int64_t gamg_act_gen = 0;   // act_gen the hierarchy was built for
  DevBuf<uint8_t> gact;       // RCCL: the global activity, max-all-reduced
  DevBuf<double> gtime;       // RCCL: a host time, max-all-reduced (amg_dist -1's choice)
  // option "amg_dist" -1: per active set (gamg_plan_gen), the first GAMG
  // solve runs the global hierarchy, the next block Jacobi; the faster
  // (host-timed, plan builds excluded) serves the set's further solves
  struct {
    int64_t gen = -1;
    int choice = -1;
    double t[2] = {-1.0, -1.0};
  } amg_auto;
  // generic CSR path scratch
  DevBuf<int64_t> c_indptr;
  DevBuf<int32_t> c_indices;
  DevBuf<double> c_data, c_kval, c_x, c_r, c_p, c_q, c_dinv;
  DevBuf<uint8_t> c_known;
};

namespace {

constexpr int kMaxChunk = 64;

// lane-operator doubles per lane: V 18, D 6, x 3, p 3, r/s/w × 2 18, M 6; plus per
// compact halo record (ell_vecs): h × 2 18, hM 6
constexpr int64_t kEllDoubles = 18 + 6 + 3 + 3 + 18 + 6 + 18 + 6;
static_assert(kEllNone == kSrcNone && kEllHalo == kSrcHalo, "slot source codes");
static_assert(kGhost == 3, "k_cg_rhs treats code 3 as a ghost free row");
constexpr int kTicketSets = 16;
constexpr int64_t kRecMax = 9, kMMax = 6;  // record / M widths at nd = 3, block Jacobi

Part& part0(mfea_handle* h) { return *h->parts[0]; }
bool partitioned(const mfea_handle* h) { return h->parts.size() > 1 || h->world > 1; }
int nranks(const mfea_handle* h) { return h->world > 1 ? h->world : (int)h->parts.size(); }

// ticket set k (one per reducing kernel kind; see device_util.hpp layout)
unsigned* tix(Part& pt, int k) { return pt.tickets.ptr + (size_t)k * kTicketStride; }
// Host-facing copies and fills on the handle's stream, waited for.  The
// stream is non-blocking: a null-stream hipMemcpy / hipMemset is not ordered
// with it, so a fill of the activity could still be landing while the next
// assembly read it (an intermittent breakdown after set_active(NULL), a
// K assembled from a mix of the old and the new activity).
hipError_t hmemcpy(mfea_handle* h, void* dst, const void* src, size_t n, hipMemcpyKind k) {
  const hipError_t e = hipMemcpyAsync(dst, src, n, k, h->stream);
  return e == hipSuccess ? hipStreamSynchronize(h->stream) : e;
}
hipError_t hmemset(mfea_handle* h, void* dst, int v, size_t n) {
  const hipError_t e = hipMemsetAsync(dst, v, n, h->stream);
  return e == hipSuccess ? hipStreamSynchronize(h->stream) : e;
}

double* cg_part_buf(Part& pt, int par) { return pt.cg_part.ptr + (size_t)par * 4 * kCgMaxPartials; }

void destroy_graph(mfea_handle* h) {
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  if (h->graph_big) (void)hipGraphExecDestroy(h->graph_big);
  h->graph_big = nullptr;
  h->graph_big_chunk = 0;
  h->graph_big_ell = -1;
  for (auto& g : h->graph_rem) {
    if (g) (void)hipGraphExecDestroy(g);
    g = nullptr;
  }
  h->graph_rem_ell = -1;
  for (auto& g : h->graph_batch) {
    if (g) (void)hipGraphExecDestroy(g);
    g = nullptr;
  }
  h->graph_batch_ell = -1;
  // (not the combined graphs: one may be in flight when the solve recaptures
  // its chunk graphs; their keys replace them, mfea_destroy frees them)
  h->graph = nullptr;
  h->graph_chunk = 0;
  h->graph_precond = -1;
  h->graph_ell = -1;
}

int set_device(mfea_handle* h) {
  HIPC(hipSetDevice(h->device));
  return 0;
}

// Row ordering of the free nodes: DFS by default (option "order": -1 DFS,
// 0 natural, > 1 degree sort inside windows of that many rows).
int order_mode(const mfea_handle* h) { return h->opt_order; }

// planar meshes run with 2 DOFs per node (option "lane_dof" 3 forces 3);
// decided on the whole mesh so every partition exchanges records of one width
int lane_dofs(const mfea_handle* h) { return (h->planar && h->opt_lane_dof != 3) ? 2 : 3; }

// Waits for an event.  Partitioned over RCCL: polls with a deadline and the
// communicator's error state, so a lost peer ends the call instead of hanging.
int wait_event(mfea_handle* h, hipEvent_t ev) {
  if (h->world <= 1 || !h->comm) {
    HIPC(hipEventSynchronize(ev));
    return 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) return fail(MFEA_EDEVICE, std::string("hipEventQuery: ") + hipGetErrorString(e));
    ncclResult_t ar = ncclSuccess;
    if (ncclCommGetAsyncError(h->comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress) {
      (void)ncclCommAbort(h->comm);
      h->comm = nullptr;
      return fail(MFEA_ECOMM, std::string("RCCL: ") + ncclGetErrorString(ar));
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > h->dist_timeout_s) {
      (void)ncclCommAbort(h->comm);
      h->comm = nullptr;
      return fail(MFEA_ECOMM, "RCCL: no progress before the deadline (peer lost?)");
    }
    // spin for the first 200 µs (a converged chunk or a step's end is
    // usually that close), then poll every 20 µs
    if (dt > 200e-6) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else std::this_thread::yield();
  }
}

// a phase boundary for mfea_stats (only with option phase_times)
int phase_event(mfea_handle* h, hipEvent_t ev, hipStream_t s) {
  if (h->opt_phase_times) HIPC(hipEventRecord(ev, s));
  return 0;
}

int sync_stream(mfea_handle* h) {
  HIPC(hipEventRecord(h->ev[5], h->stream));
  return wait_event(h, h->ev[5]);
}

// ---------------------------------------------------------------------------
// Build one partition: symbolic pattern + lanes (host), allocate and upload.
// ---------------------------------------------------------------------------
int upload_part(mfea_handle* h, Part& pt, bool dm) {
  const Pattern& P = pt.P;
  const int64_t N = P.n_nodes, E = P.n_elems;
  pt.G = P.n_slots() * kSlice;
  const int64_t maxg = std::max<int64_t>({grid_rows(N), grid_rows(E), 2048, 1});
  HIPC(pt.xyz_d.alloc(3 * N));
  HIPC(pt.val.alloc(6 * pt.G));
  HIPC(pt.diag.alloc(6 * N));
  HIPC(pt.x.alloc(3 * N));
  HIPC(pt.r.alloc(3 * N));
  HIPC(pt.p.alloc(3 * N));
  HIPC(pt.q.alloc(3 * N));
  HIPC(pt.cg_r1.alloc(3 * N));
  HIPC(pt.cg_s0.alloc(3 * N));
  HIPC(pt.cg_s1.alloc(3 * N));
  HIPC(pt.cg_w0.alloc(3 * N));
  HIPC(pt.cg_w1.alloc(3 * N));
  HIPC(pt.cg_part.alloc(2 * 4 * kCgMaxPartials));
  HIPC(pt.dinv.alloc(6 * N));
  HIPC(pt.stress.alloc(E));
  HIPC(pt.partials.alloc(4 * (maxg + 16)));
  HIPC(pt.red.alloc(16));
  HIPC(pt.slice_ptr.alloc(P.slice_ptr.size()));
  HIPC(pt.row_len.alloc(N));
  HIPC(pt.s_col.alloc(pt.G));
  HIPC(pt.s_elem.alloc(pt.G));
  HIPC(pt.e2n_d.alloc(2 * E));
  HIPC(pt.active.alloc(E));
  HIPC(pt.code.alloc(N));
  HIPC(pt.tickets.alloc(kTicketSets * kTicketStride));
  HIPC(pt.slots.alloc(kMaxChunk + 2));
  HIPC(pt.state.alloc(1));
  hipStream_t s = h->stream;
  auto up = [&](void* d, const void* src, size_t bytes) {
    return bytes ? hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
  };
  HIPC(up(pt.xyz_d.ptr, P.xyz_perm.data(), 3 * N * sizeof(double)));
  HIPC(up(pt.slice_ptr.ptr, P.slice_ptr.data(), P.slice_ptr.size() * sizeof(int32_t)));
  HIPC(up(pt.row_len.ptr, P.row_len.data(), N * sizeof(int32_t)));
  HIPC(up(pt.s_col.ptr, P.s_col.data(), pt.G * sizeof(int32_t)));
  HIPC(up(pt.s_elem.ptr, P.s_elem.data(), pt.G * sizeof(int32_t)));
  HIPC(up(pt.e2n_d.ptr, P.e2n_perm.data(), 2 * E * sizeof(int32_t)));
  HIPC(up(pt.code.ptr, P.code.data(), N * sizeof(uint8_t)));
  HIPC(hipMemsetAsync(pt.tickets.ptr, 0, kTicketSets * kTicketStride * sizeof(unsigned), s));
  HIPC(hipMemsetAsync(pt.red.ptr, 0, 16 * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.x.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.p.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.q.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.stress.ptr, 0, E * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.val.ptr, 0, 6 * pt.G * sizeof(double), s));
  HIPC(hipMemsetAsync(pt.diag.ptr, 0, 6 * N * sizeof(double), s));
  std::vector<uint8_t> act;
  if (h->active_host.size() == (size_t)h->Ecount) {
    if (dm) {
      act.resize(E);
      for (int64_t le = 0; le < E; ++le) act[le] = h->active_host[pt.plan.elem_g[le]];
    } else {
      act = h->active_host;
    }
    HIPC(up(pt.active.ptr, act.data(), E));
  } else {
    HIPC(hipMemsetAsync(pt.active.ptr, 1, E, s));
  }
  // wave-local lanes (single partition: falls back to the SELL kernel when a
  // row cannot be placed; partitioned: required)
  const std::string lerr = build_ell(P, pt.L, dm ? &pt.plan.elem_pair : nullptr);
  pt.ell_ok = lerr.empty() && (dm || P.n_free > 0);
  if (dm && !lerr.empty()) return fail(MFEA_EINVAL, "partition " + std::to_string(pt.rank) + ": " + lerr);
  if (pt.ell_ok) {
    const Ell& L = pt.L;
    const int64_t NL = L.n_lanes;
    std::vector<uint32_t> code(NL);
    for (int64_t l = 0; l < NL; ++l)
      code[l] = (L.code[l] & 0xFFFFFFu) | (uint32_t)(uint8_t)(int8_t)L.info[l] << 24;
    HIPC(pt.e_code.alloc(NL));
    HIPC(pt.e_partner.alloc(NL));
    HIPC(pt.e_lane_row.alloc(NL));
    HIPC(pt.e_src_pos.alloc(3 * NL));
    HIPC(pt.e_nbr_lane.alloc(3 * NL));
    HIPC(pt.e_f.alloc((kEllDoubles - 24) * NL + 24 * std::max<int64_t>(NL, L.n_hrec + 1)));
    HIPC(up(pt.e_code.ptr, code.data(), NL * sizeof(uint32_t)));
    // Halo record layout (ell.hip load_lane): compact (measured on one box:
    // C3 21.8 vs 23.7 µs per iteration, C2 41.6 vs 41.7 ms per step) or one
    // per lane (option "ell_compact" 0).  The device partner is the record the lane
    // fills: its mirror lane's record.
    pt.ell_hc = h->opt_ell_compact;
    std::vector<int32_t> push(NL);
    for (int64_t l = 0; l < NL; ++l)
      push[l] = L.partner[l] >= 0 ? (pt.ell_hc ? L.hrec[L.partner[l]] : L.partner[l]) : L.partner[l];
    HIPC(up(pt.e_partner.ptr, push.data(), NL * sizeof(int32_t)));
    HIPC(pt.e_hmask.alloc(NL / 64));
    HIPC(pt.e_hbase.alloc(NL / 64));
    HIPC(up(pt.e_hmask.ptr, L.hmask.data(), NL / 64 * sizeof(uint64_t)));
    HIPC(up(pt.e_hbase.ptr, L.hbase.data(), NL / 64 * sizeof(int32_t)));
    HIPC(up(pt.e_lane_row.ptr, L.lane_row.data(), NL * sizeof(int32_t)));
    HIPC(up(pt.e_src_pos.ptr, L.src_pos.data(), 3 * NL * sizeof(int32_t)));
    HIPC(up(pt.e_nbr_lane.ptr, L.nbr_lane.data(), 3 * NL * sizeof(int32_t)));
    // zero records: a lane without a halo slot reads its neighbour's (unused)
    if (NL) HIPC(hipMemsetAsync(pt.e_f.ptr, 0, pt.e_f.n * sizeof(double), s));
  }
  if (dm) {
    const PartPlan& pl = pt.plan;
    const int64_t NX = std::max<int64_t>(pl.n_pairs, 1);
    HIPC(pt.xrec.alloc(4 * NX * kRecMax + NX * kMMax));
    pt.dv.xs[0] = pt.xrec.ptr;
    pt.dv.xs[1] = pt.xrec.ptr + NX * kRecMax;
    pt.dv.xr[0] = pt.xrec.ptr + 2 * NX * kRecMax;
    pt.dv.xr[1] = pt.xrec.ptr + 3 * NX * kRecMax;
    pt.dv.mr = pt.xrec.ptr + 4 * NX * kRecMax;
    HIPC(hipMemsetAsync(pt.xrec.ptr, 0, pt.xrec.n * sizeof(double), s));
    HIPC(pt.gbuf.alloc(2 * 4 * kMaxRanks + 4 + 4 * kMaxRanks));
    pt.dv.gall[0] = pt.gbuf.ptr;
    pt.dv.gall[1] = pt.gbuf.ptr + 4 * kMaxRanks;
    pt.dv.gsend = pt.gbuf.ptr + 8 * kMaxRanks;
    pt.gred = pt.gbuf.ptr + 8 * kMaxRanks + 4;
    HIPC(hipMemsetAsync(pt.gbuf.ptr, 0, pt.gbuf.n * sizeof(double), s));
    const int64_t ns = (int64_t)pl.xsend_node.size(), nr = (int64_t)pl.xrecv_node.size();
    HIPC(pt.xh.alloc(3 * (ns + nr)));
    pt.xh_send = pt.xh.ptr;
    pt.xh_recv = pt.xh.ptr + 3 * ns;
    std::vector<int32_t> rs(ns), rr(nr);
    for (int64_t i = 0; i < ns; ++i) rs[i] = P.iperm[pl.xsend_node[i]];
    for (int64_t i = 0; i < nr; ++i) rr[i] = P.iperm[pl.xrecv_node[i]];
    HIPC(pt.xsend_rows.alloc(ns));
    HIPC(pt.xrecv_rows.alloc(nr));
    HIPC(up(pt.xsend_rows.ptr, rs.data(), ns * sizeof(int32_t)));
    HIPC(up(pt.xrecv_rows.ptr, rr.data(), nr * sizeof(int32_t)));
    HIPC(pt.elem_own.alloc(E));
    HIPC(up(pt.elem_own.ptr, pl.elem_own.data(), E));
  }
  HIPC(pt.fail_list.alloc(std::max<int64_t>(E, 1)));
  HIPC(pt.fail_cnt.alloc(1));
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// Build the symbolic pattern(s) and (re)allocate + upload device state.
int ensure_built(mfea_handle* h) {
  if (!h->has_mesh) return fail(MFEA_ESTATE, "no mesh: call mfea_set_mesh first");
  if (!h->dirty) return 0;
  destroy_graph(h);
  h->assembled = false;
  h->gkey_gen = -1;
  const bool dm = h->world > 1 || h->nparts > 1;
  const int np = h->world > 1 ? 1 : h->nparts;
  const bool skip = (h->mesh_flags & MFEA_MESH_SKIP_INVALID) != 0;
  h->parts.clear();
  for (int i = 0; i < np; ++i) {
    h->parts.push_back(std::make_unique<Part>());
    Part& pt = *h->parts.back();
    pt.rank = h->world > 1 ? h->rank : i;
    std::string err;
    if (!dm) {
      err = build_pattern(h->N, h->xyz.data(), h->Ecount, h->e2n.data(), skip, h->top, h->bot,
                          order_mode(h), pt.P);
    } else {
      err = build_partition(h->N, h->xyz.data(), h->Ecount, h->e2n.data(), skip, h->top, h->bot,
                            h->world > 1 ? h->world : np, pt.rank, h->axis, h->opt_part_slack, pt.plan);
      if (err.empty())
        err = build_pattern((int64_t)pt.plan.node_g.size(), pt.plan.xyz.data(),
                            (int64_t)pt.plan.elem_g.size(), pt.plan.e2n.data(), false, pt.plan.top,
                            pt.plan.bot, order_mode(h), pt.P, &pt.plan.ghost);
    }
    if (!err.empty()) {
      h->parts.resize(1);
      return fail(MFEA_EINVAL, err);
    }
    if (i == 0) {
      pt.mirror = h->d_host_state;
    } else {
      HIPC(pt.state_mirror.alloc(1));
      pt.mirror = pt.state_mirror.ptr;
    }
    RC(upload_part(h, pt, dm));
  }
  if (dm) {  // distributed GAMG: the whole mesh's pattern and the node owners
    h->gamg_ok = false;
    h->gamg = AmgPlan();
    h->gowner = part0(h).plan.owner;
    const std::string err = build_pattern(h->N, h->xyz.data(), h->Ecount, h->e2n.data(), skip, h->top, h->bot,
                                          order_mode(h), h->gpat);
    if (!err.empty()) return fail(MFEA_EINVAL, err);
  } else {
    h->gpat = Pattern();
  }
  ++h->act_gen;
  ++h->act_sub_gen;
  {  // free DOFs of the whole mesh (reported in mfea_stats)
    std::vector<uint8_t> known(h->N, 0);
    for (int64_t t : h->top) known[t] = 1;
    for (int64_t b : h->bot) known[b] = 1;
    h->n_free_global = h->N - (int64_t)std::count(known.begin(), known.end(), 1);
  }
  if (!dm) {  // the host view of the activity the device now holds
    const int64_t E = part0(h).P.n_elems;
    if (h->active_host.size() == (size_t)h->Ecount) {
      h->act_host.resize(E);
      for (int64_t e = 0; e < E; ++e) h->act_host[e] = h->active_host[e] ? 1 : 0;
    } else {
      h->act_host.assign(E, 1);
    }
    h->act_count = (int64_t)std::count(h->act_host.begin(), h->act_host.end(), (uint8_t)1);
    h->act_host_ok = true;
  }
  h->active_host.clear();
  h->dirty = false;
  return 0;
}

// The lane operator pays off while most rows fit one lane.  Dense networks
// (C5: mean degree 7.5 → 4.5 lanes per free row, most of them helpers that
// move zeros) run the SELL kernel instead: measured 0.94 vs 2.16 ms per
// iteration at 10 M DOF.  The partitioned path always runs lanes.
// Option "cg_kernel" 1 (lanes) / 2 (SELL) forces one (comparison runs).
bool use_ell(const mfea_handle* h, const Part& pt) {
  if (!pt.ell_ok) return false;
  if (h->opt_cg_kernel == 2) return false;
  if (h->opt_cg_kernel == 1) return true;
  return pt.L.n_lanes <= 2 * std::max<int64_t>(pt.P.n_free, 1);
}

mfea_solve_opts default_opts() {
  mfea_solve_opts o;
  o.rtol = 1e-5;
  o.atol = 1e-50;
  o.max_it = 10000;
  o.precond = MFEA_PC_JACOBI;
  o.norm = MFEA_NORM_UNPRECONDITIONED;
  o.chunk = 0;
  o.reg = 1e-12;
  return o;
}

SellOp sell_op(Part& pt) {
  SellOp op;
  op.N = pt.P.n_nodes;
  op.nf = pt.P.n_free;
  op.G = pt.G;
  op.slice_ptr = pt.slice_ptr.ptr;
  op.row_len = pt.row_len.ptr;
  op.s_col = pt.s_col.ptr;
  op.val = pt.val.ptr;
  op.diag = pt.diag.ptr;
  return op;
}

CgVecs cg_vecs(Part& pt) {
  CgVecs v;
  v.x = pt.x.ptr;
  v.p = pt.p.ptr;
  v.r[0] = pt.r.ptr;
  v.r[1] = pt.cg_r1.ptr;
  v.s[0] = pt.cg_s0.ptr;
  v.s[1] = pt.cg_s1.ptr;
  v.w[0] = pt.cg_w0.ptr;
  v.w[1] = pt.cg_w1.ptr;
  v.dinv = pt.dinv.ptr;
  return v;
}

// stride of the halo record arrays: compact records + a spare, or one per lane
int64_t ell_nr(const Part& pt) { return pt.ell_hc ? pt.L.n_hrec + 1 : pt.L.n_lanes; }

EllOp ell_op(const mfea_handle* h, Part& pt) {
  EllOp op;
  const int64_t NL = pt.L.n_lanes;
  op.NL = NL;
  op.nd = lane_dofs(h);
  op.code = pt.e_code.ptr;
  op.partner = pt.e_partner.ptr;
  op.lane_row = pt.e_lane_row.ptr;
  op.src_pos = pt.e_src_pos.ptr;
  op.nbr_lane = pt.e_nbr_lane.ptr;
  op.V = pt.e_f.ptr;
  op.D = op.V + 18 * NL;
  op.hc = pt.ell_hc ? 1 : 0;
  op.NR = ell_nr(pt);
  op.hmask = pt.e_hmask.ptr;
  op.hbase = pt.e_hbase.ptr;
  op.bs = h->opt_ell_block;
  op.maxg = h->opt_ell_maxg;
  return op;
}

EllVecs ell_vecs(Part& pt) {
  EllVecs v;
  const int64_t NL = pt.L.n_lanes;
  double* f = pt.e_f.ptr + 24 * NL;
  auto take = [&](int64_t n) {
    double* p = f;
    f += n * NL;
    return p;
  };
  v.x = take(3);
  v.p = take(3);
  for (int q = 0; q < 2; ++q) {
    v.r[q] = take(3);
    v.s[q] = take(3);
    v.w[q] = take(3);
  }
  v.M = take(6);
  const int64_t NR = ell_nr(pt);
  v.h[0] = f;
  v.h[1] = f + 9 * NR;
  v.hM = f + 18 * NR;
  return v;
}

// ---------------------------------------------------------------------------
// Exchanges of the partitioned solve.  Over RCCL: ONE group of point-to-point
// transfers per exchange point on the handle's stream — the neighbour
// payloads and the 4 partial sums to every other rank (send/recv pairs, not a
// ring all-gather: over xGMI every rank pair has its own link, so the sums
// cost one hop instead of world − 1 ring steps).  The sums travel as copies:
// every rank then adds the same bits in the same (rank) order — never an
// all-reduce, whose summation order may differ per rank.  The producer of
// gsend also writes the rank's own row of gall[q].
// Partitions on one device: device copies on the same stream.
// ---------------------------------------------------------------------------
// inside an open group: gsend → row `rank` of every other rank's gall
int sums_p2p(mfea_handle* h, const double* gsend, double* gall) {
  for (int r = 0; r < h->world; ++r) {
    if (r == h->rank) continue;
    NCCLC(ncclSend(gsend, 4, ncclFloat64, r, h->comm, h->stream));
    NCCLC(ncclRecv(gall + 4 * r, 4, ncclFloat64, r, h->comm, h->stream));
  }
  return 0;
}

// CG records of parity q (xs[q] → the peers' xr[q]); gather: this rank's
// partial sums (gsend) → row `rank` of every rank's gall[q]
int xchg_records(mfea_handle* h, int q, bool gather) {
  const int64_t RW = 3 * lane_dofs(h);
  hipStream_t s = h->stream;
  if (h->world > 1) {
    Part& pt = part0(h);
    const PartPlan& pl = pt.plan;
    if (pl.peers.empty() && !gather) return 0;
    NCCLC(ncclGroupStart());
    for (size_t i = 0; i < pl.peers.size(); ++i) {
      const size_t n = (size_t)(pl.peer_cnt[i] * RW);
      NCCLC(ncclSend(pt.dv.xs[q] + pl.peer_off[i] * RW, n, ncclFloat64, pl.peers[i], h->comm, s));
      NCCLC(ncclRecv(pt.dv.xr[q] + pl.peer_off[i] * RW, n, ncclFloat64, pl.peers[i], h->comm, s));
    }
    if (gather) RC(sums_p2p(h, pt.dv.gsend, pt.dv.gall[q]));
    NCCLC(ncclGroupEnd());
    return 0;
  }
  for (auto& a : h->parts) {
    const PartPlan& pa = a->plan;
    for (size_t i = 0; i < pa.peers.size(); ++i) {
      Part& b = *h->parts[pa.peers[i]];
      const PartPlan& pb = b.plan;
      const auto it = std::lower_bound(pb.peers.begin(), pb.peers.end(), a->rank);
      const size_t jb = (size_t)(it - pb.peers.begin());
      if (it == pb.peers.end() || *it != a->rank || pb.peer_cnt[jb] != pa.peer_cnt[i])
        return fail(MFEA_EINVAL, "internal: asymmetric exchange plan");
      HIPC(hipMemcpyAsync(b.dv.xr[q] + pb.peer_off[jb] * RW, a->dv.xs[q] + pa.peer_off[i] * RW,
                          pa.peer_cnt[i] * RW * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    if (gather)
      for (auto& b : h->parts)
        if (b != a)
          HIPC(hipMemcpyAsync(b->dv.gall[q] + 4 * a->rank, a->dv.gsend, 4 * sizeof(double),
                              hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

// displacement halo: xh_send (packed owned rows) → the peers' xh_recv
int xchg_xhalo(mfea_handle* h) {
  hipStream_t s = h->stream;
  if (h->world > 1) {
    Part& pt = part0(h);
    const PartPlan& pl = pt.plan;
    NCCLC(ncclGroupStart());
    for (size_t i = 0; i < pl.xpeers.size(); ++i) {
      if (pl.xsend_cnt[i])
        NCCLC(ncclSend(pt.xh_send + 3 * pl.xsend_off[i], (size_t)(3 * pl.xsend_cnt[i]), ncclFloat64,
                       pl.xpeers[i], h->comm, s));
      if (pl.xrecv_cnt[i])
        NCCLC(ncclRecv(pt.xh_recv + 3 * pl.xrecv_off[i], (size_t)(3 * pl.xrecv_cnt[i]), ncclFloat64,
                       pl.xpeers[i], h->comm, s));
    }
    NCCLC(ncclGroupEnd());
    return 0;
  }
  for (auto& a : h->parts) {
    const PartPlan& pa = a->plan;
    for (size_t i = 0; i < pa.xpeers.size(); ++i) {
      if (!pa.xsend_cnt[i]) continue;
      Part& b = *h->parts[pa.xpeers[i]];
      const PartPlan& pb = b.plan;
      const auto it = std::lower_bound(pb.xpeers.begin(), pb.xpeers.end(), a->rank);
      const size_t jb = (size_t)(it - pb.xpeers.begin());
      if (it == pb.xpeers.end() || *it != a->rank || pb.xrecv_cnt[jb] != pa.xsend_cnt[i])
        return fail(MFEA_EINVAL, "internal: asymmetric displacement halo");
      HIPC(hipMemcpyAsync(b.xh_recv + 3 * pb.xrecv_off[jb], a->xh_send + 3 * pa.xsend_off[i],
                          3 * pa.xsend_cnt[i] * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
  }
  return 0;
}

// 4 doubles at red + off of every partition → row `rank` of every gred
int gather4(mfea_handle* h, int off) {
  hipStream_t s = h->stream;
  if (h->world > 1) {
    Part& pt = part0(h);
    NCCLC(ncclAllGather(pt.red.ptr + off, pt.gred, 4, ncclFloat64, h->comm, s));
    return 0;
  }
  for (auto& a : h->parts)
    for (auto& b : h->parts)
      HIPC(hipMemcpyAsync(b->gred + 4 * a->rank, a->red.ptr + off, 4 * sizeof(double),
                          hipMemcpyDeviceToDevice, s));
  return 0;
}

// ---------------------------------------------------------------------------
// enqueue one chunk of single-reduction CG iterations (one kernel each)
void enqueue_chunk(mfea_handle* h, int chunk, int precond, bool ell) {
  hipStream_t s = h->stream;
  Part& pt = part0(h);
  if (ell) {
    const EllOp op = ell_op(h, pt);
    const EllVecs v = ell_vecs(pt);
    for (int j = 0; j < chunk; ++j)
      launch_ell_iter(s, j, op, precond, v, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr);
  } else {
    const SellOp op = sell_op(pt);
    const CgVecs v = cg_vecs(pt);
    for (int j = 0; j < chunk; ++j)
      launch_cg_iter(s, j, op, precond, v, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr);
  }
  launch_cg_advance(s, chunk, pt.slots.ptr, pt.state.ptr, pt.mirror);
}

// partitioned: per iteration, every partition's iteration kernel, its partial
// sums, then one exchange of records + sums (launched eagerly)
int enqueue_chunk_dist(mfea_handle* h, int chunk, int precond) {
  hipStream_t s = h->stream;
  for (int j = 0; j < chunk; ++j) {
    const int q = (j & 1) ^ 1;
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_ell_iter(s, j, ell_op(h, pt), precond, ell_vecs(pt), pt.slots.ptr, pt.state.ptr,
                      pt.cg_part.ptr, nullptr, &pt.dv);
    }
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_psum(s, ell_op(h, pt), cg_part_buf(pt, q), pt.dv.gall[q] + 4 * pt.rank, pt.dv.gsend);
    }
    HIPC(hipGetLastError());
    RC(xchg_records(h, q, true));
  }
  for (auto& pp : h->parts) launch_cg_advance(s, chunk, pp->slots.ptr, pp->state.ptr, pp->mirror);
  HIPC(hipGetLastError());
  return 0;
}

// Replays chunks until the device reports done; at most two chunks in flight.
// mirror = true: the chunk's advance kernel writes the final state into the
// mapped pinned h_state[0] itself (CG-CG path); otherwise copy it per chunk.
template <class Enqueue>
int drive_chunks(mfea_handle* h, int chunk, int max_it, Enqueue&& enqueue, SolveState* out,
                 bool mirror = false) {
  hipStream_t s = h->stream;
  Part& pt = part0(h);
  const int64_t max_chunks = (int64_t)max_it / chunk + 3;
  int64_t k = 0;
  bool done = false;
  volatile SolveState* hs = h->h_state;
  if (mirror) hs[0].done = 0;
  while (!done && k < max_chunks) {
    int rc = enqueue();
    if (rc) return rc;
    if (!mirror)
      HIPC(hipMemcpyAsync(&h->h_state[k & 1], pt.state.ptr, sizeof(SolveState),
                          hipMemcpyDeviceToHost, s));
    HIPC(hipEventRecord(h->poll[k & 1], s));
    if (k >= 1) {
      RC(wait_event(h, h->poll[(k - 1) & 1]));
      if (hs[mirror ? 0 : (k - 1) & 1].done) done = true;
    }
    ++k;
  }
  RC(sync_stream(h));
  const SolveState& last = h->h_state[mirror ? 0 : (k - 1) & 1];
  if (!last.done) {
    // should not happen (max_chunks covers max_it); report as maxit
    *out = last;
    out->status = MFEA_EMAXIT;
    out->iters = max_it;
    return 0;
  }
  *out = last;
  return 0;
}

// Replays planned from the expected iteration count (the AMG solves of one
// handle converge in a near-constant number of iterations): enough chunks
// for `expected` iterations are queued back to back with no host wait, then
// one chunk at a time until the device reports done.  A wrong guess costs a
// chunk of early-exiting launches (too high) or one host round trip per
// extra chunk (too low) — never correctness.  `after` is queued behind every
// batch before the host waits (the solve's epilogue: if that batch
// converged, the stream is already past it when the host wakes; if not, the
// next batch's copy supersedes it).
struct NoEpilogue {
  int operator()() const { return 0; }
};
template <class Enqueue, class After = NoEpilogue>
int drive_planned(mfea_handle* h, int chunk, int max_it, int expected, Enqueue&& enqueue,
                  SolveState* out, After&& after = After{}) {
  hipStream_t s = h->stream;
  const int64_t max_chunks = (int64_t)max_it / chunk + 3;
  volatile SolveState* hs = h->h_state;
  hs[0].done = 0;
  int64_t k = 0;
  const int64_t first = std::min<int64_t>(max_chunks, std::max(1, (expected + 1 + chunk - 1) / chunk));
  for (; k < first; ++k) RC(enqueue());
  RC(after());
  HIPC(hipEventRecord(h->poll[0], s));
  RC(wait_event(h, h->poll[0]));
  while (!hs[0].done && k < max_chunks) {
    RC(enqueue());
    RC(after());
    HIPC(hipEventRecord(h->poll[0], s));
    RC(wait_event(h, h->poll[0]));
    ++k;
  }
  RC(sync_stream(h));
  *out = h->h_state[0];
  if (!out->done) {
    out->status = MFEA_EMAXIT;
    out->iters = max_it;
  }
  return 0;
}

// drive_planned with chunks of two sizes: the planned batch (`expected`
// updates) as long chunks of `big` iterations plus short ones of `small` for
// the remainder — one chunk boundary (advance kernel + graph-to-graph gap,
// ≈ 13 µs) per `big` iterations instead of per `small`, while a batch never
// overshoots the expected count by more than small − 1 — then short chunks
// one at a time until the device reports done.  enqueue(size) queues one.
template <class Enqueue, class After = NoEpilogue>
int drive_sized(mfea_handle* h, int big, int small, int max_it, int expected, Enqueue&& enqueue,
                SolveState* out, After&& after = After{}, bool exact_rem = false) {
  hipStream_t s = h->stream;
  volatile SolveState* hs = h->h_state;
  hs[0].done = 0;
  const int need = std::max(1, expected + 1);  // updates the batch assumes, as drive_planned
  const int nbig = big > small ? need / big : 0;
  const int rem = need - nbig * big;
  const int nsmall = (rem + small - 1) / small;
  int64_t done_its = 0;
  for (int k = 0; k < nbig; ++k, done_its += big) RC(enqueue(big));
  if (exact_rem && rem > 0) {  // one chunk of the remainder's own length (drive_rem_chunk)
    RC(enqueue(rem));
    done_its += rem;
  } else {
    for (int k = 0; k < nsmall; ++k, done_its += small) RC(enqueue(small));
  }
  RC(after());
  HIPC(hipEventRecord(h->poll[0], s));
  RC(wait_event(h, h->poll[0]));
  while (!hs[0].done && done_its < (int64_t)max_it + 3 * small) {
    RC(enqueue(small));
    RC(after());
    HIPC(hipEventRecord(h->poll[0], s));
    RC(wait_event(h, h->poll[0]));
    done_its += small;
  }
  RC(sync_stream(h));
  *out = h->h_state[0];
  if (!out->done) {
    out->status = MFEA_EMAXIT;
    out->iters = max_it;
  }
  return 0;
}

// mfea_step's planned batch as one graph (solve_amg, option batch_graph):
// the batch's iterations, the finish and the post; the post counts as the
// step's speculative post (mfea_handle::spec_used), so when the solve goes on
// in small chunks their first batch end undoes its failures (spec_post)
template <class Launch, class Enqueue, class After>
int drive_batch(mfea_handle* h, int small, int max_it, int need, Launch&& launch, Enqueue&& enqueue,
                SolveState* out, After&& after, bool launched = false) {
  hipStream_t s = h->stream;
  volatile SolveState* hs = h->h_state;
  if (!launched) hs[0].done = 0;
  RC(launch());
  h->spec_used = true;
  h->spec_launched = true;
  HIPC(hipEventRecord(h->ev[5], s));  // the post's read-back: the end of the batch
  HIPC(hipEventRecord(h->poll[0], s));
  RC(wait_event(h, h->poll[0]));
  int64_t done_its = need;
  while (!hs[0].done && done_its < (int64_t)max_it + 3 * small) {
    RC(enqueue(small));
    RC(after());
    HIPC(hipEventRecord(h->poll[0], s));
    RC(wait_event(h, h->poll[0]));
    done_its += small;
  }
  RC(sync_stream(h));
  *out = h->h_state[0];
  if (!out->done) {
    out->status = MFEA_EMAXIT;
    out->iters = max_it;
  }
  return 0;
}

// device times of the last solve (its events must have completed)
void solve_times(mfea_handle* h, mfea_stats* st) {
  if (!h->opt_phase_times) return;  // (no phase events recorded: the t_* stay 0)
  float ms = 0;
  (void)hipEventElapsedTime(&ms, h->ev[1], h->ev[2]);
  st->t_rhs_ms = ms;
  (void)hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
  st->t_solve_ms = ms;
  if (h->ev_setup_used) {
    (void)hipEventElapsedTime(&ms, h->ev[2], h->ev_setup);
    st->t_setup_ms = ms;
  }
}

// The solve's end: the status comes from the host copy of the final state
// (drive_chunks / drive_planned waited for it); inside mfea_step the stream
// is not waited for here — post's wait covers it and the times are read then
// (one host round trip less per step).
int finish_solve(mfea_handle* h, const SolveState& fin, mfea_stats* st) {
  if (!h->in_step) {  // (mfea_solve: its end is waited for here)
    HIPC(hipEventRecord(h->ev[3], h->stream));
    RC(wait_event(h, h->ev[3]));
  } else if (!h->spec_launched) {  // (a speculative post recorded it before itself)
    RC(phase_event(h, h->ev[3], h->stream));
  }
  if (st) {
    st->iters = fin.iters;
    st->status = fin.status;
    st->bnorm = std::sqrt(fin.bb0);
    st->relres = fin.res0 > 0 ? std::sqrt(fin.res_final / fin.res0) : 0.0;
    st->n_free = 3 * h->n_free_global;
    if (!h->in_step) solve_times(h, st);
  }
  if (fin.status == -4) return fail(MFEA_EMAXIT, "PCG reached max_it without converging");
  if (fin.status == -5) return fail(MFEA_EBREAKDOWN, "PCG breakdown (p·Ap <= 0 or non-finite)");
  return 0;
}

int solve_chunk_size(const mfea_solve_opts* o) {
  int chunk = o->chunk > 0 ? std::min(o->chunk, kMaxChunk) : 32;
  return chunk + (chunk & 1);  // even: the iteration kernels take the buffer parity from j
}

int solve_impl(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
               mfea_stats* st) {
  Part& pt = part0(h);
  hipStream_t s = h->stream;
  const int precond = o->precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0;
  const int chunk = solve_chunk_size(o);
  const SellOp op = sell_op(pt);
  const CgVecs v = cg_vecs(pt);
  RC(phase_event(h, h->ev[1], s));
  launch_cg_rhs(s, op, pt.code.ptr, dy_top, dy_bot, o->reg, precond, v, pt.partials.ptr, tix(pt, 0),
                pt.red.ptr);
  launch_cg_init_finalize(s, pt.red.ptr, o->rtol, o->atol, o->norm, o->max_it, o->reg,
                          pt.state.ptr,
                          pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
  const bool ell = use_ell(h, pt);
  if (ell) {
    launch_ell_init(s, ell_op(h, pt), op, precond, v, ell_vecs(pt));
    launch_ell_first(s, ell_op(h, pt), o->reg, precond, ell_vecs(pt), pt.slots.ptr, pt.cg_part.ptr);
  } else {
    launch_cg_first(s, op, o->reg, precond, v, pt.slots.ptr, pt.cg_part.ptr);
  }
  HIPC(hipGetLastError());
  RC(phase_event(h, h->ev[2], s));
  // option "graph" 0: launch the chunk kernels eagerly (profilers that do not
  // follow hipGraph replays; same kernels, same order)
  const bool no_graph = !h->opt_graph;
  SolveState fin;
  int rc;
  if (no_graph) {
    rc = drive_chunks(
        h, chunk, o->max_it,
        [&]() -> int {
          enqueue_chunk(h, chunk, precond, ell);
          HIPC(hipGetLastError());
          return 0;
        },
        &fin, /*mirror=*/true);
  } else {
    if (h->graph == nullptr || h->graph_chunk != chunk || h->graph_precond != precond ||
        h->graph_ell != (ell ? lane_dofs(h) : 0)) {
      destroy_graph(h);
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      enqueue_chunk(h, chunk, precond, ell);
      HIPC(hipStreamEndCapture(s, &g));
      hipError_t e = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      h->graph_chunk = chunk;
      h->graph_precond = precond;
      h->graph_ell = ell ? lane_dofs(h) : 0;
    }
    rc = drive_chunks(
        h, chunk, o->max_it,
        [&]() -> int {
          HIPC(hipGraphLaunch(h->graph, s));
          return 0;
        },
        &fin, /*mirror=*/true);
  }
  if (rc) return rc;
  if (ell) {
    launch_ell_finish(s, ell_op(h, pt), ell_vecs(pt), pt.x.ptr);
    HIPC(hipGetLastError());
  }
  return finish_solve(h, fin, st);
}

// ---------------------------------------------------------------------------
// SA-AMG preconditioned CG (amg.hpp / amg.hip), single partition.
// ---------------------------------------------------------------------------
constexpr size_t kAmgAlign = 64;  // elements: every carved array starts 256/512-B aligned
size_t amg_al(size_t n) { return (n + kAmgAlign - 1) / kAmgAlign * kAmgAlign; }

// rows [lo, hi) of a SELL pattern and their positions (amg_kernels.hpp RowRange)
RowRange row_range(const SellPat& S, int64_t lo, int64_t hi) {
  RowRange g;
  g.lo = lo;
  g.hi = hi > lo ? hi : lo;
  if (hi <= lo || S.sptr.size() < 2) return g;
  g.s0 = lo >> 6;
  g.s1 = (hi - 1) >> 6;
  g.p0 = (int64_t)S.sptr[g.s0] * 64;
  g.p1 = (int64_t)S.sptr[g.s1 + 1] * 64;
  g.pf = (int64_t)S.sptr[g.s0 + 1] * 64;
  g.pl = (int64_t)S.sptr[g.s1] * 64;
  return g;
}

// Carves the plan's index arrays and the value / vector arrays out of two
// device allocations and uploads the indices.  Pass 0 sizes, pass 1 carves.
// rk (distributed GAMG): this partition's row ranges, with its own level-0
// lists over ITS pattern (a0, row0) in place of the plan's.
// strength of connection of the level-0 aggregation (option amg_theta_ppm;
// amg.hpp AmgStrength): θ and the bending-to-axial constant 12EI / EA
AmgStrength amg_strength(const mfea_handle* h) {
  AmgStrength st;
  st.theta = h->opt_amg_theta_ppm * 1e-6;
  st.kb_kax = h->mat.EA > 0.0 ? h->mat.EI12 / h->mat.EA : 0.0;
  return st;
}

// w = A u's step width: K = 2 (slices up to 2U blocks in one round trip of
// column loads and gathers, more VGPRs) once level 0's mean slice width
// passes U = 4 blocks, or on a small network, whose launch is one chain of
// dependent loads long and ends with its widest slices (C2 iteration 26.1 →
// 25.4 µs; C3 66.6 vs 66.8, kept at K = 1: profiles/r5/ab_spmv_k.jsonl)
constexpr int64_t kWideSpmvRows = 131072;
static int amg_w_k(const AmgPlan& pl) {
  if (pl.lev.empty() || pl.lev[0].A.sptr.size() < 2) return 1;
  const auto& sp = pl.lev[0].A.sptr;
  const double mean = (double)(sp.back() - sp.front()) / (double)(sp.size() - 1);
  return mean > 4.0 || pl.lev[0].A.n <= kWideSpmvRows ? 2 : 1;
}

// the collapsed cycle's lowest level when chosen automatically: level 1's V
// is dense-ish on small networks (the reference network: 80 blocks per row,
// 0.3 M product pairs, a few ms of host build per rebuild) for one saved
// launch pair; level 2 is what C2 / C3 choose anyway
constexpr int kAmgCollapseAutoLevel = 2;
constexpr int64_t kMergeRows = 131072;  // amg_merge -1: level-0 rows up to which levels 0 and 1 merge

// ρ̂ of the levels below 0 (0: the Gershgorin rule), until a solve has failed
// with it
double coarse_rho(const mfea_handle* h) {
  return h->amg_safe_omega ? 0.0 : (double)h->opt_amg_coarse_rho_ppm * 1e-6;
}

// The smoothing weights of a partition's hierarchy for the handle's current
// mode (DESIGN.md §4.2 "Coarse-level smoothing weight"): over-relaxed — ρ̂_l
// fixed at coarse_rho below level 0 and at 2 (its exact bound) on level 0,
// so no Gershgorin pass and, on an own hierarchy, no coarse D⁻¹ launches
// (fixed_omega) — or, after a fallback, the Gershgorin-safe rule (omega[0] =
// 0: the setup estimates ρ̂_l).  Called at upload and whenever the mode
// changes; the next numeric setup re-forms every ω product.
int apply_coarse_omega(mfea_handle* h, Part& pt) {
  hipStream_t s = h->stream;
  const int nlev = (int)pt.amg_lev.size();
  const double rho = coarse_rho(h);
  static const double kRho0 = 2.0;
  for (int l = 0; l < nlev; ++l) {
    AmgLevD& d = pt.amg_lev[l];
    d.fixed_omega = pt.amg_om_own && l > 0 && rho > 0.0 ? 1 : 0;
    d.a0full = 0;
    d.a0slot = l == 0 ? h->opt_amg_a0_slot : 0;
    HIPC(hipMemsetAsync(d.omega, 0, sizeof(double), s));
    if (l > 0 && rho > 0.0) HIPC(hipMemcpyAsync(d.omega, &rho, sizeof(double), hipMemcpyHostToDevice, s));
  }
  // level 0: its P_0 / Ã_0 then come with A_0 in one row pass (k_amg_a0full)
  // where that measured faster: the Z-ordered plans (C5 setup 4.17 → 3.88
  // ms); on depth-first ones the per-position launch stays (C3 0.401 vs
  // 0.408 ms, C2 0.219 vs 0.224)
  if (pt.amg_om_own && nlev > 1 && rho > 0.0 && pt.amg_lev[0].compact) {
    pt.amg_lev[0].fixed_omega = 1;
    pt.amg_lev[0].a0full = pt.amg_om_spatial ? 1 : 0;
    HIPC(hipMemcpyAsync(pt.amg_lev[0].omega, &kRho0, sizeof(double), hipMemcpyHostToDevice, s));
  }
  if (nlev) {
    HIPC(pt.amg_levd.alloc(nlev));
    HIPC(hipMemcpyAsync(pt.amg_levd.ptr, pt.amg_lev.data(), nlev * sizeof(AmgLevD), hipMemcpyHostToDevice, s));
  }
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// A GAMG solve that failed with the over-relaxed coarse smoothers may have
// met an operator on which they do not give an SPD cycle (ω_l λ_l ≥ 2).  A
// breakdown suggests that; max_it only when the caller's limit is far above
// what this hierarchy needs (`typical` iterations) — a deliberately small
// max_it is not ω's fault.
bool omega_suspect(const mfea_handle* h, int status, int max_it, int typical) {
  if (status == 0 || coarse_rho(h) <= 0.0) return false;
  if (status == -5) return true;
  return status == -4 && max_it > 4 * std::max(typical, 16);
}

// ... then the solve runs once more on the Gershgorin-safe weights, which stay
// for the handle's lifetime only if that solve converges; otherwise the
// over-relaxed ones come back and the retry's failure is returned.
// Partitioned over RCCL every rank sees the same status (the CG scalars are
// all-reduced), so every rank takes this path together.
template <class F>
int omega_retry(mfea_handle* h, F&& again) {
  RC(sync_stream(h));
  h->amg_safe_omega = true;
  for (auto& pp : h->parts) RC(apply_coarse_omega(h, *pp));
  const int rc = again();
  if (rc == MFEA_EMAXIT || rc == MFEA_EBREAKDOWN) {
    h->amg_safe_omega = false;
    for (auto& pp : h->parts) RC(apply_coarse_omega(h, *pp));
  }
  return rc;
}

// the merged cycle on or off (built plans only): level 2's x / e point into
// the merged vector buffer while on
void set_merge(mfea_handle* h, Part& pt) {
  const bool on = pt.amg_mplan.on && h->opt_amg_merge != 0 && pt.amg_lev.size() >= 4 && pt.amg_cg.coll == 2;
  pt.amg_mg.on = on ? 1 : 0;
  if (pt.amg_lev.size() > 2) {
    AmgLevD& L2 = pt.amg_lev[2];
    const int nd = pt.amg.nd;
    L2.x = on ? pt.amg_mg.B + (size_t)nd * pt.amg_mg.n1 : pt.amg_x2;
    L2.e = on ? pt.amg_mg.B + (size_t)nd * (pt.amg_mg.n1 + pt.amg_mg.n2) : pt.amg_e2;
  }
}

int upload_amg(mfea_handle* h, Part& pt, const AmgPlan& pl, const AmgRank* rk = nullptr,
               const PosList* a0 = nullptr, const std::vector<int32_t>* row0 = nullptr) {
  const int nd = pl.nd, nb2 = nd * nd;
  const int nlev = (int)pl.lev.size();
  hipStream_t s = h->stream;
  size_t ni = 0, ndd = 0, nff = 0;
  pt.amg_coll = AmgCollapse();
  // (a distributed plan: collapsed among its replicated levels only)
  if ((!rk || rk->compact) && h->opt_amg_cycle == 1 && h->opt_amg_collapse != 0) {
    const int min_level = h->opt_amg_collapse < 0 ? kAmgCollapseAutoLevel : std::max(1, h->opt_amg_collapse);
    const std::string cerr = build_amg_collapse(pl, h->opt_amg_collapse_mb << 20, h->opt_amg_collapse_pairs,
                                                rk ? std::max(min_level, rk->n_dist) : min_level, pt.amg_coll);
    if (!cerr.empty()) return fail(MFEA_EINVAL, cerr);
  }
  // levels 0 and 1 merged (amg.hpp AmgMerge): where the launches are latency-
  // bound — level 0 under kMergeRows rows (C2: 34 k; C3's 336 k measured
  // slower merged: its c_1 / x_2 / W rows add more bytes than two launches cost)
  pt.amg_mplan = AmgMerge();
  if (!rk && h->opt_amg_merge != 0 && pt.amg_coll.kc == 2 && nlev >= 4 &&
      (h->opt_amg_merge > 0 || pl.lev[0].A.n <= kMergeRows)) {
    const std::string merr = build_amg_merge(pl, pt.amg_coll, pt.amg_mplan);
    if (!merr.empty()) return fail(MFEA_EINVAL, merr);
  }
  // the level-0 label of every free row (the floating mask's scatter, launch_floating)
  std::vector<int32_t> row0_inv;
  if (!rk && nlev > 1) {
    row0_inv.assign(pl.row0.size(), -1);
    for (size_t i = 0; i < pl.row0.size(); ++i) row0_inv[pl.row0[i]] = (int32_t)i;
  }
  int32_t* ip = nullptr;
  double* dp = nullptr;
  float* fp = nullptr;
  int pass = 0;
  hipError_t err = hipSuccess;
  auto I = [&](const std::vector<int32_t>& v) -> const int32_t* {
    if (pass == 0) {
      ni += amg_al(v.size());
      return nullptr;
    }
    int32_t* p = ip;
    ip += amg_al(v.size());
    if (!v.empty() && err == hipSuccess)
      err = hipMemcpyAsync(p, v.data(), v.size() * sizeof(int32_t), hipMemcpyHostToDevice, s);
    return p;
  };
  auto D = [&](size_t n) -> double* {
    if (pass == 0) {
      ndd += amg_al(n);
      return nullptr;
    }
    double* p = dp;
    dp += amg_al(n);
    return p;
  };
  auto F = [&](size_t n) -> float* {
    if (pass == 0) {
      nff += amg_al(n);
      return nullptr;
    }
    float* p = fp;
    fp += amg_al(n);
    return p;
  };
  // vals64: f64 values, vals32: f32 values (the numeric setup stores every
  // hierarchy value in f32 — computing in f64 — and the V-cycle reads them;
  // only A_0's symmetric blocks for the CG's w = A u stay f64)
  std::deque<std::vector<int32_t>> srows;  // alive until the copies below have run (the stream sync at the end)
  auto mat = [&](const SellPat& S, bool vals64, bool vals32) {
    AmgMatD m;
    m.n = S.n;
    m.npos = S.n_pos();
    for (size_t k = 0; k + 1 < S.sptr.size(); ++k) m.wmax = std::max(m.wmax, S.sptr[k + 1] - S.sptr[k]);
    m.sptr = I(S.sptr);
    std::vector<int32_t>& srow = srows.emplace_back(S.sptr.empty() ? 0 : S.sptr.back(), 0);  // slot row → slice
    for (size_t k = 0; k + 1 < S.sptr.size(); ++k)
      for (int32_t t = S.sptr[k]; t < S.sptr[k + 1]; ++t) srow[t] = (int32_t)k;
    m.srow = I(srow);
    m.col = I(S.col);
    m.val = vals64 ? D((size_t)nb2 * m.npos) : nullptr;
    m.val32 = vals32 ? F((size_t)nb2 * m.npos) : nullptr;
    return m;
  };
  for (pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      HIPC(pt.amg_i.alloc(std::max<size_t>(ni, 1)));
      HIPC(pt.amg_d.alloc(std::max<size_t>(ndd, 1)));
      HIPC(pt.amg_f.alloc(std::max<size_t>(nff, 1)));
      HIPC(hipMemsetAsync(pt.amg_d.ptr, 0, pt.amg_d.n * sizeof(double), s));
      HIPC(hipMemsetAsync(pt.amg_f.ptr, 0, pt.amg_f.n * sizeof(float), s));
      ip = pt.amg_i.ptr;
      dp = pt.amg_d.ptr;
      fp = pt.amg_f.ptr;
    }
    pt.amg_lev.assign(nlev, AmgLevD{});
    for (int l = 0; l < nlev; ++l) {
      const AmgLevel& L = pl.lev[l];
      AmgLevD& d = pt.amg_lev[l];
      const int64_t n = L.A.n;
      const int64_t lo = rk ? rk->lo[l] : 0, hi = rk ? rk->hi[l] : n;
      d.A = mat(L.A, false, true);
      d.A.rg = row_range(L.A, lo, hi);
      if (l == 0) {  // A_0: symmetric blocks for the CG and the level-0 V-cycle kernels
        const size_t ns = (size_t)nd * (nd + 1) / 2;
        d.A.sym = D(ns * d.A.npos);
        d.A.sym32 = F(ns * d.A.npos);
      }
      d.dinv = l == 0 && nlev == 1 ? D((size_t)nb2 * n) : nullptr;  // one level: the exact block solve
      d.dinv32 = F((size_t)nb2 * n);
      d.omega = D(2);
      d.b = l ? F((size_t)nd * n) : nullptr;  // level 0 reads the CG's r
      d.x = F((size_t)nd * n);
      d.t = F((size_t)nd * n);
      d.e = l ? F((size_t)nd * n) : nullptr;  // level 0 writes the CG's u
      d.coarsest = L.coarsest ? 1 : 0;
      d.rlanes = h->opt_amg_rlanes;
      d.dsplit = h->opt_amg_down_split;
      d.vlanes = h->opt_amg_v_lanes;
      d.small_lanes = h->opt_amg_small_lanes;
      d.alanes = h->opt_amg_alanes;
      d.tail_lds = h->opt_amg_tail_lds;
      d.ulanes = h->opt_amg_up_lanes;
      d.x1 = !rk && l > 0 && n <= h->opt_amg_x1_rows ? 1 : 0;
      if (!L.coarsest) {
        d.agg = I(L.agg);
        d.P = mat(L.P, false, true);
        d.P.rg = row_range(L.P, lo, hi);
        d.pv_ptr = I(L.pv.ptr);
        d.pv_a = I(L.pv.a);
        const int64_t rlo = rk ? rk->rlo[l] : 0, rhi = rk ? rk->rhi[l] : L.R.n;
        d.R = mat(L.R, false, true);
        d.R.rg = row_range(L.R, rlo, rhi);
        d.ac_rg = row_range(pl.lev[l + 1].A, rlo, rhi);
        d.rp = I(L.rp);
        d.AP = mat(L.AP, false, false);
        d.AP.rg = row_range(L.AP, rk ? rk->aplo[l] : 0, rk ? rk->aphi[l] : L.AP.n);
        d.apval = F((size_t)nb2 * d.AP.npos);
        d.ap_ptr = I(L.ap.ptr);
        d.ap_a = I(L.ap.a);
        d.ap_b = I(L.ap.b);
        d.ac_ptr = I(L.ac.ptr);
        d.ac_a = I(L.ac.a);
        d.ac_b = I(L.ac.b);
        {  // the Galerkin product's lanes per block: its lists run 5–40 pairs (amg.hip ac_body)
          const int64_t np = std::max<int64_t>(1, pl.lev[l + 1].A.n_pos());
          const double mean = L.ac.ptr.empty() ? 0.0 : (double)L.ac.ptr.back() / (double)np;
          d.ac_lanes = mean > 24.0 ? 8 : mean > 12.0 ? 4 : mean > 6.0 ? 2 : 1;
        }
        // the compact cycle's P̃ / R̃: one partition's hierarchy, or a
        // distributed one split at level 0 only (rk->compact: level 0 on this
        // rank's P̃ / R̂ / Ã rows, the replicated levels whole; the four-step
        // distributed cycle exchanges per step instead)
        const bool cmp = !rk || (rk->compact && (l == 0 || l >= rk->n_dist));
        if (cmp && L.PT.n == n) {
          const bool own = rk && l < rk->n_dist;
          d.PT = mat(L.PT, false, true);
          d.A.at32 = F((size_t)nb2 * d.A.npos);
          d.PT.rg = own ? row_range(L.PT, rk->aplo[l], rk->aphi[l]) : row_range(L.PT, 0, n);
          d.pt_row = I(L.pt_row);
          d.pt_ap = I(L.pt_ap);
          d.pt_p = I(L.pt_p);
          d.RT = mat(L.RT, false, true);
          d.RT.rg = own ? row_range(L.RT, rk->rtlo, rk->rthi) : row_range(L.RT, 0, L.RT.n);
          d.rt_pt = I(L.rt_pt);
          d.rt_row = I(L.rt_row);
          d.compact = h->opt_amg_cycle;
        }
        if (pt.amg_coll.kc > 0 && l >= pt.amg_coll.kc) {  // the collapsed operators of this level
          const AmgCollapse::Lev& C = pt.amg_coll.lev[l - pt.amg_coll.kc];
          d.CT = mat(C.T, false, true);
          d.ct_ptr = I(C.tl.ptr);
          d.ct_a = I(C.tl.a);
          d.ct_b = I(C.tl.b);
          d.CV = mat(C.V, false, true);
          d.cv_row = I(C.vrow);
          d.cv_ptr = I(C.vl.ptr);
          d.cv_a = I(C.vl.a);
          d.cv_b = I(C.vl.b);
          d.cv_ext = I(C.va);
          d.cv_diag = I(C.vdiag);
          d.collapsed = 1;
        }
      }
    }
    pt.amg_a0_ptr = I(a0 ? a0->ptr : pl.a0.ptr);
    pt.amg_a0_a = I(a0 ? a0->a : pl.a0.a);
    pt.amg_row0_inv = !rk && nlev > 1 ? I(row0_inv) : nullptr;
    const int64_t nf = nlev ? pl.lev[0].A.n : 0;
    pt.amg_cg.n = nf;
    pt.amg_cg.lo = rk && nlev ? rk->lo[0] : 0;
    pt.amg_cg.hi = rk && nlev ? rk->hi[0] : nf;
    pt.amg_cg.w_block = h->opt_amg_w_block;
    pt.amg_cg.w_k = amg_w_k(pl);
    pt.amg_cg.cycle = h->opt_amg_cycle;
    pt.amg_cg.coll = pt.amg_coll.kc;
    pt.amg_cg.row0 = I(row0 ? *row0 : pl.row0);
    pt.amg_cg.x = D((size_t)nd * nf);
    pt.amg_cg.p = D((size_t)nd * nf);
    pt.amg_cg.s = D((size_t)nd * nf);
    pt.amg_cg.w = D((size_t)nd * nf);
    pt.amg_cg.r = D((size_t)nd * nf);
    pt.amg_cg.u = F((size_t)nd * nf);
    // the merged levels' operators, lists and vector buffer
    pt.amg_mg = AmgMergeD{};
    if (pt.amg_mplan.on) {
      const AmgMerge& M = pt.amg_mplan;
      AmgMergeD& g = pt.amg_mg;
      g.n1 = M.n1;
      g.n2 = M.n2;
      g.DQ = mat(M.DQ, false, true);
      g.DQ.rg = row_range(M.DQ, 0, M.DQ.n);
      g.U = mat(M.U, false, true);
      g.U.rg = row_range(M.U, 0, M.U.n);
      g.dq_dst = I(M.dq_dst);
      g.dq_split = M.dq_split;
      g.dq_ext = I(M.dq_ext);
      g.dq_ptr = I(M.dq_l.ptr);
      g.dq_a = I(M.dq_l.a);
      g.dq_b = I(M.dq_l.b);
      g.u_ext = I(M.u_ext);
      g.u_ptr = I(M.u_l.ptr);
      g.u_a = I(M.u_l.a);
      g.u_b = I(M.u_l.b);
      g.B = F((size_t)nd * (M.n1 + 2 * M.n2 + 1));
    }
  }
  HIPC(err);
  pt.amg_x2 = nlev > 2 ? pt.amg_lev[2].x : nullptr;
  pt.amg_e2 = nlev > 2 ? pt.amg_lev[2].e : nullptr;
  set_merge(h, pt);
  {
    std::vector<int64_t> rows(nlev);
    for (int l = 0; l < nlev; ++l) rows[l] = pl.lev[l].A.n;
    // the single-workgroup tail holds whole levels: never a split one
    const int first = rk ? std::max(1, rk->n_dist) : 1;
    pt.amg_tail = first < nlev ? amg_tail_level(rows.data() + first - 1, nlev - first + 1, h->opt_amg_tail_rows) : 0;
    if (pt.amg_tail > 0) pt.amg_tail += first - 1;
    pt.amg_first = first;
  }
  if (!rk && nlev > 1) {  // the floating-row mask (zero until ensure_amg fills it)
    HIPC(pt.amg_fmask.alloc(std::max<int64_t>(pl.lev[0].A.n, 1)));
    HIPC(hipMemsetAsync(pt.amg_fmask.ptr, 0, pt.amg_fmask.n, s));
    pt.amg_lev[0].fmask = pt.amg_fmask.ptr;
  }
  // the smoothing weights (ρ̂ per level in place of the Gershgorin estimate)
  pt.amg_om_own = !rk;
  pt.amg_om_spatial = pl.spatial;
  HIPC(pt.amg_levd.alloc(std::max(nlev, 1)));
  return apply_coarse_omega(h, pt);
}

// The element activity of the handle's single partition, on the host.
int current_active(mfea_handle* h, Part& pt) {
  if (h->act_host_ok && h->act_host.size() == (size_t)pt.P.n_elems) return 0;
  h->act_host.resize(pt.P.n_elems);
  if (pt.P.n_elems)
    HIPC(hmemcpy(h, h->act_host.data(), pt.active.ptr, pt.P.n_elems, hipMemcpyDeviceToHost));
  h->act_count = (int64_t)std::count(h->act_host.begin(), h->act_host.end(), (uint8_t)1);
  h->act_host_ok = true;
  return 0;
}

// Partitioned GAMG: the halo plan (ghost couplings, u send rows) for the
// plan's active set, uploaded next to the hierarchy.
int upload_amg_halo(mfea_handle* h, Part& pt, const std::vector<uint8_t>& key) {
  const PartPlan& pl = pt.plan;
  const Pattern& P = pt.P;
  std::vector<int32_t> xs(pl.xsend_node.size()), xr(pl.xrecv_node.size());
  for (size_t i = 0; i < xs.size(); ++i) xs[i] = P.iperm[pl.xsend_node[i]];
  for (size_t i = 0; i < xr.size(); ++i) xr[i] = P.iperm[pl.xrecv_node[i]];
  const std::string err = build_amg_halo(P, key, pt.amg, xs, xr, pt.amg_halo);
  if (!err.empty()) return fail(MFEA_EINVAL, "AMG halo: " + err);
  const AmgHalo& hl = pt.amg_halo;
  const int nd = pt.amg.nd;
  const size_t a = hl.send_rows.size(), b = hl.gptr.size(), c = hl.gslot.size();
  HIPC(pt.amg_hi.alloc(a + b + 2 * c + 1));
  HIPC(pt.amg_hd.alloc(nd * (xs.size() + xr.size()) + 1));
  hipStream_t s = h->stream;
  auto up = [&](int32_t* d, const std::vector<int32_t>& v) {
    return v.empty() ? hipSuccess : hipMemcpyAsync(d, v.data(), v.size() * 4, hipMemcpyHostToDevice, s);
  };
  int32_t* ib = pt.amg_hi.ptr;
  HIPC(up(ib, hl.send_rows));
  HIPC(up(ib + a, hl.gptr));
  HIPC(up(ib + a + b, hl.gslot));
  HIPC(up(ib + a + b + c, hl.grecv));
  HIPC(hipMemsetAsync(pt.amg_hd.ptr, 0, pt.amg_hd.n * sizeof(double), s));
  AmgDist& d = pt.amg_dist;
  d = AmgDist{};
  d.rank = pt.rank;
  d.gall[0] = pt.dv.gall[0];
  d.gall[1] = pt.dv.gall[1];
  d.gsend = pt.dv.gsend;
  d.zero_w = h->world > 1 && h->opt_dist_sums == 1 ? h->world : 0;
  d.send_rows = ib;
  d.n_send = (int64_t)a;
  d.gptr = ib + a;
  d.gslot = ib + a + b;
  d.grecv = ib + a + b + c;
  d.sval = pt.val.ptr;
  d.G = pt.G;
  d.usend = pt.amg_hd.ptr;
  d.urecv = pt.amg_hd.ptr + nd * xs.size();
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// The floating-row mask of the device's current activity in level-0 labels
// (one partition's own hierarchy: a partition cannot tell alone what is
// floating): connected components on the device (kernels.hpp
// launch_floating), four launches on the stream, no host pass or wait
int enqueue_fmask(mfea_handle* h, Part& pt) {
  const Pattern& P = pt.P;
  if (P.n_free == 0 || !pt.amg_row0_inv) return 0;
  HIPC(pt.cc_parent.alloc(std::max<int64_t>(P.n_nodes, 1)));
  HIPC(pt.cc_anch.alloc(std::max<int64_t>(P.n_nodes, 1)));
  launch_floating(h->stream, P.n_nodes, P.n_free, P.n_nodes - P.n_ghost, pt.slice_ptr.ptr, pt.row_len.ptr,
                  pt.s_col.ptr, pt.s_elem.ptr, pt.active.ptr, pt.cc_parent.ptr, pt.cc_anch.ptr, pt.amg_row0_inv,
                  pt.amg_fmask.ptr, h->opt_cc_tile);
  HIPC(hipGetLastError());
  return 0;
}

// the multicolour sweep's arrays for a one-level plan (MFEA_PC_SOR / _ICC);
// a GAMG plan: none (amg_cg.sweep = 0)
int upload_sweep(mfea_handle* h, Part& pt, int kind) {
  pt.swd = SweepD{};
  pt.amg_cg.sweep = 0;
  if (kind != MFEA_PC_SOR && kind != MFEA_PC_ICC) return 0;
  const SweepPlan& sp = pt.sweep;
  if (sp.colors > kSweepMaxColors) return fail(MFEA_EINVAL, "sweep plan: too many colours");
  const int nd = pt.amg.nd, nb2 = nd * nd, ns = nd * (nd + 1) / 2;
  const int64_t ne = sp.n_entries();
  const std::vector<int32_t>* iv[] = {&sp.wsteps, &sp.row, &sp.ppos, &sp.dpos, &sp.lo_ptr,
                                      &sp.lo_ent, &sp.lo_pos, &sp.up_ptr, &sp.up_ent, &sp.up_pos};
  size_t ni = 1;
  for (auto* v : iv) ni += v->size();
  HIPC(pt.sw_i.alloc(ni));
  const size_t nlo = sp.lo_ent.size(), nup = sp.up_ent.size();
  HIPC(pt.sw_f.alloc((size_t)ne * (nb2 + ns) + (nlo + nup) * nb2 + 1));
  HIPC(pt.sw_y.alloc((size_t)ne * nd + 1));
  int32_t* ip = pt.sw_i.ptr;
  hipStream_t s = h->stream;
  auto put = [&](const std::vector<int32_t>& v) -> const int32_t* {
    int32_t* p = ip;
    if (!v.empty()) (void)hipMemcpyAsync(p, v.data(), v.size() * 4, hipMemcpyHostToDevice, s);
    ip += v.size();
    return p;
  };
  SweepD& w = pt.swd;
  w.n = sp.n;
  w.ne = ne;
  w.colors = sp.colors;
  w.dic = kind == MFEA_PC_ICC ? 1 : 0;
  for (int c = 0; c <= sp.colors; ++c) w.cw[c] = sp.cwave[c];
  w.wsteps = put(sp.wsteps);
  w.row = put(sp.row);
  w.ppos = put(sp.ppos);
  w.dpos = put(sp.dpos);
  w.lo_ptr = put(sp.lo_ptr);
  w.lo_ent = put(sp.lo_ent);
  w.lo_pos = put(sp.lo_pos);
  w.up_ptr = put(sp.up_ptr);
  w.up_ent = put(sp.up_ent);
  w.up_pos = put(sp.up_pos);
  float* fp = pt.sw_f.ptr;
  w.pv = fp;
  w.dt = fp + (size_t)ne * nb2;
  w.lov = w.dt + (size_t)ne * ns;
  w.upv = w.lov + nlo * nb2;
  // pads and first steps are never written by the setup: zero them once
  HIPC(hipMemsetAsync(fp, 0, pt.sw_f.n * sizeof(float), s));
  w.y = pt.sw_y.ptr;
  HIPC(hipMemsetAsync(w.y, 0, pt.sw_y.n * sizeof(double), s));
  pt.amg_cg.sweep = 1;
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// the preconditioner application u = M r of one PCG iteration (gate: its
// flag; NULL: ungated)
void launch_precond(mfea_handle* h, Part& pt, const int32_t* gate) {
  if (pt.amg_cg.sweep) launch_sweep(h->stream, pt.amg.nd, pt.swd, pt.amg_cg, gate);
  else launch_amg_vcycle(h->stream, pt.amg.nd, pt.amg_lev.data(), (int)pt.amg_lev.size(), pt.amg_cg, pt.amg_tail, gate,
                         0, pt.amg_mg.on ? &pt.amg_mg : nullptr);
}

// (Re)build the hierarchy when the active set differs from the plan's.  One
// partition: the host view of the activity (downloaded only when a post
// kernel changed it); partitioned: each partition's own elements, read back.
int upload_sweep(mfea_handle* h, Part& pt, int kind);

// every element active in `a` is active in `b`: a hierarchy built for b is
// kept for a only then — A_0's slot lists hold b's elements alone, so an
// element that came back since would be missing from the CG's w = A u
// (its couplings absent while the diagonal has them)
static bool active_subset(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
  if (a.size() != b.size()) return false;
  for (size_t e = 0; e < a.size(); ++e)
    if (a[e] && !b[e]) return false;
  return true;
}

// the chain-piece plan with at most kSweepMaxColors colours: shorter pieces
// (fewer couplings per piece) until it fits — pieces of one row are a point
// colouring, max degree + 1 colours at most
std::string build_sweep_bounded(const AmgPlan& plan, int piece_len, SweepPlan& sp) {
  for (int m = piece_len;; m = std::max(1, m / 2)) {
    const std::string err = build_sweep(plan, m, sp);
    if (!err.empty() || sp.colors <= kSweepMaxColors) return err;
    if (m == 1) return "sweep plan: more than 32 colours";
  }
}

int ensure_amg(mfea_handle* h, Part& pt, bool* rebuilt, int kind = MFEA_PC_GAMG) {
  *rebuilt = false;
  if (pt.amg_ok && pt.amg_kind != kind) {  // another preconditioner's plan
    pt.amg_ok = false;
    pt.amg_last_iters = 0;
  }
  const bool dm = partitioned(h);
  // no activity change since the plan / mask last matched it: nothing to do
  // (no O(E) key compares on the hot path)
  if (!dm && pt.amg_ok && !pt.amg_stale && pt.amg_seen_gen == h->act_gen) return 0;
  // the activity moved only by failures since the plan's key was set (post
  // kept the host activity current from the failed ids): keep the hierarchy
  // with no host O(E) pass — the floating mask is recomputed on the device
  if (!dm && pt.amg_ok && !pt.amg_stale && h->opt_amg_reuse && pt.amg_lev.size() > 1 && h->act_host_ok &&
      pt.amg_sub_gen == h->act_sub_gen) {
    RC(enqueue_fmask(h, pt));
    pt.amg_reused = h->act_count != pt.amg_key_count;
    pt.amg_seen_gen = h->act_gen;
    return 0;
  }
  std::vector<uint8_t> local;
  if (dm) {
    local.resize(pt.P.n_elems);
    if (pt.P.n_elems) HIPC(hmemcpy(h, local.data(), pt.active.ptr, pt.P.n_elems, hipMemcpyDeviceToHost));
  } else {
    RC(current_active(h, pt));
  }
  const std::vector<uint8_t>& key = dm ? local : h->act_host;
  pt.amg_reused = false;
  if (!dm && pt.amg_ok && pt.amg_lev.size() > 1 &&
      (pt.amg_key == key || (h->opt_amg_reuse && !pt.amg_stale && active_subset(key, pt.amg_key)))) {
    // keep the hierarchy: the numeric setup re-forms its values from the new
    // K (failed elements are zero slots); only pieces cut off from both grips
    // need care — their P_0 rows are zeroed so they stay exactly at zero
    RC(enqueue_fmask(h, pt));
    pt.amg_reused = pt.amg_key != key;
    pt.amg_seen_gen = h->act_gen;
    pt.amg_sub_gen = h->act_sub_gen;  // key ⊆ amg_key, compared
    return 0;
  }
  if (pt.amg_ok && pt.amg_key == key) {
    if (!dm) pt.amg_seen_gen = h->act_gen;
    if (!dm || pt.dev_plan == 0) return 0;
    destroy_graph(h);  // the device holds the global plan: upload this one again
    RC(upload_amg(h, pt, pt.amg));
    RC(upload_amg_halo(h, pt, key));
    pt.dev_plan = 0;
    ++pt.amg_gen;
    return 0;
  }
  pt.amg_ok = false;
  HostLap clk;
  const auto build_t0 = std::chrono::steady_clock::now();
  AmgLayout lay;
  lay.spatial = h->opt_amg_spatial;
  lay.by_a = h->opt_amg_cycle == 1;
  const bool sweep = kind == MFEA_PC_SOR || kind == MFEA_PC_ICC;
  std::string err = build_amg(pt.P, key, lane_dofs(h), pt.amg, sweep ? 1 : h->opt_amg_max_levels, nullptr,
                              amg_strength(h), lay);
  if (err.empty() && sweep) err = build_sweep_bounded(pt.amg, h->opt_sweep_piece, pt.sweep);
  if (!err.empty()) return fail(MFEA_EINVAL, "AMG setup: " + err);
  clk.lap("plan build");
  destroy_graph(h);
  pt.amg_kind = kind;
  RC(upload_amg(h, pt, pt.amg));
  RC(upload_sweep(h, pt, kind));
  if (dm) RC(upload_amg_halo(h, pt, key));
  clk.lap("plan upload");
  pt.dev_plan = 0;
  pt.amg_key = key;
  pt.amg_ok = true;
  pt.amg_stale = false;
  pt.amg_build_iters = -1;
  pt.amg_excess_s = 0.0;
  pt.amg_build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - build_t0).count();
  pt.amg_reused = false;
  if (!dm && pt.amg_lev.size() > 1) RC(enqueue_fmask(h, pt));
  clk.lap("floating mask");
  if (!dm) pt.amg_seen_gen = h->act_gen;
  pt.amg_sub_gen = dm ? -1 : h->act_sub_gen;
  pt.amg_key_count = (int64_t)std::count(key.begin(), key.end(), (uint8_t)1);
  ++pt.amg_gen;
  *rebuilt = true;
  return 0;
}

void enqueue_amg_iteration(mfea_handle* h, Part& pt, int j, bool profile) {
  hipStream_t s = h->stream;
  const int nd = pt.amg.nd;
  const AmgLevD& L0 = pt.amg_lev[0];
  launch_amg_cg_update(s, nd, j, L0, pt.amg_cg, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr);
  (void)profile;
  launch_precond(h, pt, nullptr);
  launch_amg_cg_w(s, nd, j, profile, L0, pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
}

// ---- partitioned GAMG exchanges -------------------------------------------
// u of the send rows → the peers' urecv (the displacement-halo plan, ND
// doubles per node)
int xchg_u(mfea_handle* h) {
  hipStream_t s = h->stream;
  const int64_t nd = part0(h).amg.nd;
  if (h->world > 1) {
    Part& pt = part0(h);
    const PartPlan& pl = pt.plan;
    if (pl.xpeers.empty()) return 0;
    NCCLC(ncclGroupStart());
    for (size_t i = 0; i < pl.xpeers.size(); ++i) {
      if (pl.xsend_cnt[i])
        NCCLC(ncclSend(pt.amg_dist.usend + nd * pl.xsend_off[i], (size_t)(nd * pl.xsend_cnt[i]), ncclFloat64,
                       pl.xpeers[i], h->comm, s));
      if (pl.xrecv_cnt[i])
        NCCLC(ncclRecv(const_cast<double*>(pt.amg_dist.urecv) + nd * pl.xrecv_off[i],
                       (size_t)(nd * pl.xrecv_cnt[i]), ncclFloat64, pl.xpeers[i], h->comm, s));
    }
    NCCLC(ncclGroupEnd());
    return 0;
  }
  for (auto& a : h->parts) {
    const PartPlan& pa = a->plan;
    for (size_t i = 0; i < pa.xpeers.size(); ++i) {
      if (!pa.xsend_cnt[i]) continue;
      Part& b = *h->parts[pa.xpeers[i]];
      const PartPlan& pb = b.plan;
      const auto it = std::lower_bound(pb.xpeers.begin(), pb.xpeers.end(), a->rank);
      const size_t jb = (size_t)(it - pb.xpeers.begin());
      if (it == pb.xpeers.end() || *it != a->rank || pb.xrecv_cnt[jb] != pa.xsend_cnt[i])
        return fail(MFEA_EINVAL, "internal: asymmetric u halo");
      HIPC(hipMemcpyAsync(const_cast<double*>(b.amg_dist.urecv) + nd * pb.xrecv_off[jb],
                          a->amg_dist.usend + nd * pa.xsend_off[i], nd * pa.xsend_cnt[i] * sizeof(double),
                          hipMemcpyDeviceToDevice, s));
    }
  }
  return 0;
}

// every rank's 4 partial sums (gsend) → row `rank` of every rank's gall[q]
int xchg_sums(mfea_handle* h, int q) {
  hipStream_t s = h->stream;
  if (h->world > 1 && h->opt_dist_sums == 1) {  // one all-reduce: every row but the own zeroed (k_amg_gsum)
    Part& pt = part0(h);
    NCCLC(ncclAllReduce(pt.dv.gall[q], pt.dv.gall[q], (size_t)4 * h->world, ncclFloat64, ncclSum, h->comm, s));
    return 0;
  }
  if (h->world > 1) {
    Part& pt = part0(h);
    NCCLC(ncclGroupStart());
    RC(sums_p2p(h, pt.dv.gsend, pt.dv.gall[q]));
    NCCLC(ncclGroupEnd());
    return 0;
  }
  GallCopy g;  // partitions on one device: one launch for every pair
  for (auto& a : h->parts) {
    if (g.n == 64) return fail(MFEA_EINVAL, "internal: more than 64 partitions");
    g.gsend[g.n] = a->dv.gsend;
    g.gall[g.n] = a->dv.gall[q];
    g.rank[g.n] = a->rank;
    ++g.n;
  }
  launch_gall_copy(s, g);
  HIPC(hipGetLastError());
  return 0;
}

// one partitioned GAMG iteration j on every partition: update (gathered sums)
// → local V-cycle → u halo → w = A u with the ghost couplings → this rank's
// sums → all-gather.  Two exchanges per iteration (the V-cycle output is not
// computable from a neighbour's state, unlike the Jacobi lanes' records).
int enqueue_amg_dist_iteration(mfea_handle* h, int j) {
  hipStream_t s = h->stream;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int nd = pt.amg.nd;
    launch_amg_cg_update(s, nd, j, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr,
                         &pt.amg_dist);
    launch_amg_vcycle(s, nd, pt.amg_lev.data(), (int)pt.amg_lev.size(), pt.amg_cg, pt.amg_tail, nullptr);
    launch_amg_pack_u(s, nd, pt.amg_cg, pt.amg_dist);
  }
  HIPC(hipGetLastError());
  RC(xchg_u(h));
  const int q = (j & 1) ^ 1;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_w(s, pt.amg.nd, j, false, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr,
                    &pt.amg_dist);
    launch_amg_gsum(s, pt.amg_cg, cg_part_buf(pt, q), pt.amg_dist, q);
  }
  HIPC(hipGetLastError());
  return xchg_sums(h, q);
}

int enqueue_amg_dist_chunk(mfea_handle* h, int chunk) {
  for (int j = 0; j < chunk; ++j) RC(enqueue_amg_dist_iteration(h, j));
  for (auto& pp : h->parts) launch_cg_advance(h->stream, chunk, pp->slots.ptr, pp->state.ptr, pp->mirror);
  HIPC(hipGetLastError());
  return 0;
}

// One replayed chunk = `chunk` groups of (V-cycle j, w_j, update j+1): the
// chunk ENDS with an update, so the last planned chunk leaves the device
// knowing whether the solve converged and no chunk of early-exiting launches
// is queued after the converging update (each gated launch still costs
// ≈ 4 µs).  update 0 runs before the first chunk (solve_amg).
void enqueue_amg_chunk(mfea_handle* h, Part& pt, int chunk) {
  hipStream_t s = h->stream;
  const int nd = pt.amg.nd;
  const AmgLevD& L0 = pt.amg_lev[0];
  // The preconditioner and w = A u launches carry no gate: once the update
  // kernel stops the solve (converged, max_it, breakdown) it leaves x, r, p,
  // s and level 0's x unchanged, and every later V-cycle / sweep / w launch
  // is a pure function of those — it rewrites the values it wrote before.  A
  // gate flag cost each launch a load from another XCD's L2 ahead of its
  // first wait (vector loads complete in order), ≈ 1 µs per launch.
  for (int j = 0; j < chunk; ++j) {
    launch_precond(h, pt, nullptr);
    launch_amg_cg_w(s, nd, j, false, L0, pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
    launch_amg_cg_update(s, nd, j + 1, L0, pt.amg_cg, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr);
  }
  launch_cg_advance(s, chunk, pt.slots.ptr, pt.state.ptr, pt.mirror, 1);
}

// hierarchy values for the current K (the per-solve numeric setup)
void enqueue_amg_setup(mfea_handle* h, Part& pt, double reg) {
  hipStream_t s = h->stream;
  const int nd = pt.amg.nd, nlev = (int)pt.amg_lev.size();
  const bool compact = pt.amg_cg.cycle == 1 && nlev > 1 && pt.amg_lev[0].compact;
  const bool fused = compact && h->opt_amg_fuse_setup && !pt.amg_cg.sweep;
  launch_amg_a0(s, nd, pt.amg_lev[0], sell_op(pt), pt.amg_cg.row0, pt.amg_a0_ptr, pt.amg_a0_a, reg,
                fused && pt.amg_lev[0].a0full);
  if (pt.amg_cg.sweep) {
    launch_sweep_setup(s, nd, pt.swd, pt.amg_lev[0]);
    return;
  }
  bool merged_done = false;
  if (fused) {
    merged_done = launch_amg_setup_fused(s, nd, pt.amg_lev.data(), nlev, pt.amg_cg.coll, &pt.amg_mg);
  } else {
    for (int l = 0; l < nlev; ++l)
      launch_amg_level_setup(s, nd, pt.amg_lev[l], l + 1 < nlev ? &pt.amg_lev[l + 1] : nullptr, l == 0);
    launch_amg_compact_setup(s, nd, pt.amg_lev.data(), nlev, compact ? pt.amg_cg.coll : 0);
  }
  if (pt.amg_mg.on && !merged_done) launch_amg_merge_setup(s, nd, pt.amg_lev.data(), pt.amg_mg);
}

// FNV-1a over 8-byte words (then the tail bytes): the setup graph's key is
// hashed on every solve while the GPU runs the assembly, over ≈ 10 KB of level
// views — byte by byte that host work outlasted C2's assembly
uint64_t fnv1a(uint64_t k, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, b + i, 8);
    k = (k ^ w) * 1099511628211ULL;
  }
  for (; i < n; ++i) k = (k ^ b[i]) * 1099511628211ULL;
  return k;
}

void launch_precond(mfea_handle* h, Part& pt, const int32_t* gate);
int enqueue_post_work(mfea_handle* h, double max_strain);

// The solve's entry behind the setup: level-0 b from the CG's r, the first
// preconditioner application, w = A u, update 0 (solve_amg)
void enqueue_amg_entry(mfea_handle* h, Part& pt) {
  hipStream_t s = h->stream;
  const int nd = pt.amg.nd;
  const AmgLevD& L0 = pt.amg_lev[0];
  launch_amg_cg_init(s, nd, L0, pt.amg_cg, cg_vecs(pt).r[0]);
  launch_precond(h, pt, nullptr);
  launch_amg_cg_w(s, nd, 0, true, L0, pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
  launch_amg_cg_update(s, nd, 0, L0, pt.amg_cg, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr);  // update 0
}

// mfea_step's deferred assembly (option step_graph) at the head of the setup
// graph: the grip displacements from pinned h_red[14..15] (a copy node, read
// at replay), the row gather with the fused RHS reading them from d_dy, the
// CG start — k_assemble<true> / k_cg_init_finalize exactly as eager
void enqueue_step_head(mfea_handle* h, Part& pt, const mfea_solve_opts* o) {
  hipStream_t s = h->stream;
  const Pattern& P = pt.P;
  (void)hipMemcpyAsync(h->d_dy.ptr, h->h_red + 14, 2 * sizeof(double), hipMemcpyHostToDevice, s);
  AsmRhs q{};
  q.code = pt.code.ptr;
  q.top_end = P.n_free + P.n_top;
  q.bot_end = P.n_nodes - P.n_ghost;
  q.dyp = h->d_dy.ptr;
  q.nf = P.n_free;
  q.r = pt.r.ptr;
  q.x = pt.x.ptr;
  q.partials = pt.partials.ptr;
  q.ticket = tix(pt, 0);
  q.red_out = pt.red.ptr;
  launch_assemble(s, P.n_nodes, pt.xyz_d.ptr, pt.slice_ptr.ptr, pt.row_len.ptr, pt.s_col.ptr, pt.s_elem.ptr,
                  pt.active.ptr, h->mat, pt.G, pt.val.ptr, pt.diag.ptr, &q);
  launch_cg_init_finalize(s, pt.red.ptr, o->rtol, o->atol, o->norm, o->max_it, o->reg, pt.state.ptr,
                          pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
}

// The numeric setup replayed as one captured graph (single partition): the
// eager launches cost the host ≈ 5–8 µs each (kernel arguments of 1.5–3 KB),
// more than the GPU spends on the deep levels' kernels; recaptured whenever
// anything the launches read changes (the key hashes all of it).  entry: the
// solve's entry launches captured behind the setup (no phase event between
// them); head (non-null): mfea_step's assembly and CG start before it
int launch_amg_setup_graph(mfea_handle* h, Part& pt, double reg, bool entry = false,
                           const mfea_solve_opts* head = nullptr, const mfea_solve_opts* start = nullptr,
                           int tail = 0, int tag = 0) {
  hipStream_t s = h->stream;
  uint64_t k = 1469598103934665603ULL;
  k = fnv1a(k, pt.amg_lev.data(), pt.amg_lev.size() * sizeof(AmgLevD));
  k = fnv1a(k, &pt.amg_mg, sizeof pt.amg_mg);
  const SellOp op = sell_op(pt);
  k = fnv1a(k, &op, sizeof op);
  const void* ptrs[4] = {pt.amg_cg.row0, pt.amg_a0_ptr, pt.amg_a0_a, pt.amg_levd.ptr};
  k = fnv1a(k, ptrs, sizeof ptrs);
  const int ints[5] = {pt.amg.nd, h->opt_amg_fuse_setup, pt.amg_cg.cycle, pt.amg_cg.coll, pt.amg_cg.sweep};
  k = fnv1a(k, &pt.swd, sizeof pt.swd);
  k = fnv1a(k, ints, sizeof ints);
  k = fnv1a(k, &reg, sizeof reg);
  if (entry) {
    const CgVecs v = cg_vecs(pt);
    const void* eptrs[4] = {v.r[0], pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr};
    k = fnv1a(k, eptrs, sizeof eptrs);
    k = fnv1a(k, &pt.amg_cg, sizeof pt.amg_cg);
    k = fnv1a(k, &pt.amg_kind, sizeof pt.amg_kind);
  }
  if (start) {  // the CG start (k_cg_init_finalize) at the graph's head
    const double sd[3] = {start->rtol, start->atol, start->reg};
    const int si[2] = {start->norm, start->max_it};
    const void* sp[3] = {pt.red.ptr, pt.state.ptr, pt.cg_part.ptr};
    k = fnv1a(k ^ 0x5a5a, sd, sizeof sd);
    k = fnv1a(k, si, sizeof si);
    k = fnv1a(k, sp, sizeof sp);
  }
  if (head) {
    const void* hptrs[10] = {pt.xyz_d.ptr, pt.s_elem.ptr, pt.active.ptr, pt.code.ptr, pt.r.ptr,
                             pt.x.ptr, pt.partials.ptr, pt.red.ptr, h->d_dy.ptr, h->h_red};
    k = fnv1a(k, hptrs, sizeof hptrs);
    const double hd[3] = {head->rtol, head->atol, head->reg};
    const int hi[2] = {head->norm, head->max_it};
    k = fnv1a(k, hd, sizeof hd);
    k = fnv1a(k, hi, sizeof hi);
    k = fnv1a(k, &h->mat, sizeof h->mat);
    k = fnv1a(k, &pt.tickets.ptr, sizeof pt.tickets.ptr);
  }
  if (tail > 0) {
    // the step's whole GPU work but the assembly: setup, entry, the planned
    // batch of `tail` iterations, the finish, the post (mfea_step, batch_graph)
    k = fnv1a(k ^ 0xc0b0, &tail, sizeof tail);
    k = fnv1a(k, &tag, sizeof tag);
    k = fnv1a(k, &h->spec_strain, sizeof h->spec_strain);
    hipGraphExec_t& gc = h->graph_combo[tail];
    if (!gc || h->graph_combo_key[tail] != k) {
      if (gc) {
        HIPC(hipStreamSynchronize(s));
        (void)hipGraphExecDestroy(gc);
        gc = nullptr;
      }
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      if (head) enqueue_step_head(h, pt, head);
      if (start)
        launch_cg_init_finalize(s, pt.red.ptr, start->rtol, start->atol, start->norm, start->max_it, start->reg,
                                pt.state.ptr, pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
      enqueue_amg_setup(h, pt, reg);
      enqueue_amg_entry(h, pt);
      enqueue_amg_chunk(h, pt, tail);
      launch_amg_finish(s, pt.amg.nd, pt.amg_cg, pt.x.ptr);
      const int prc = enqueue_post_work(h, h->spec_strain);
      const hipError_t ec = hipStreamEndCapture(s, &g);
      RC(prc);
      HIPC(ec);
      const hipError_t e = hipGraphInstantiate(&gc, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      h->graph_combo_key[tail] = k;
    }
    HIPC(hipGraphLaunch(gc, s));
    return 0;
  }
  if (!h->graph_setup || h->graph_setup_key != k) {
    if (h->graph_setup) {
      HIPC(hipStreamSynchronize(s));  // no replay of the old graph in flight
      (void)hipGraphExecDestroy(h->graph_setup);
      h->graph_setup = nullptr;
    }
    hipGraph_t g;
    HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    if (head) enqueue_step_head(h, pt, head);
    if (start)
      launch_cg_init_finalize(s, pt.red.ptr, start->rtol, start->atol, start->norm, start->max_it, start->reg,
                              pt.state.ptr, pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
    enqueue_amg_setup(h, pt, reg);
    if (entry) enqueue_amg_entry(h, pt);
    HIPC(hipStreamEndCapture(s, &g));
    const hipError_t e = hipGraphInstantiate(&h->graph_setup, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPC(e);
    h->graph_setup_key = k;
  }
  HIPC(hipGraphLaunch(h->graph_setup, s));
  return 0;
}

int spec_post(mfea_handle* h);
int spec_undo(mfea_handle* h);
int assemble_impl(mfea_handle* h, mfea_stats* st, const double* rhs_dy);
int enqueue_post_work(mfea_handle* h, double max_strain);

int solve_amg(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
              mfea_stats* st) {
  Part& pt = part0(h);
  hipStream_t s = h->stream;
  bool rebuilt = false;
  HostLap clk;
  RC(ensure_amg(h, pt, &rebuilt, o->precond));
  clk.lap("ensure_amg");
  const int chunk = o->chunk > 0 ? solve_chunk_size(o) : 2;
  const SellOp op = sell_op(pt);
  const CgVecs v = cg_vecs(pt);
  const int nd = pt.amg.nd;
  // mfea_step's deferred assembly: at the head of the setup graph, or now
  const bool head = h->asm_pending && h->opt_graph && !h->opt_phase_times;
  if (h->asm_pending) {
    h->asm_pending = false;
    if (head) HIPC(h->d_dy.alloc(2));
    else RC(assemble_impl(h, nullptr, h->h_red + 14));
  }
  RC(phase_event(h, h->ev[1], s));
  // the CG start inside the setup graph when no phase event separates them
  const bool start_in_graph = h->opt_graph && h->opt_graph_start && !h->opt_phase_times && !head;
  if (!head) {
    // (mfea_step's assembly formed it for these displacements: AsmRhs)
    const bool rhs_done = h->rhs_fused && h->rhs_dy[0] == dy_top && h->rhs_dy[1] == dy_bot;
    h->rhs_fused = false;
    if (!rhs_done)
      launch_cg_rhs(s, op, pt.code.ptr, dy_top, dy_bot, o->reg, 2, v, pt.partials.ptr, tix(pt, 0), pt.red.ptr);
    if (!start_in_graph)
      launch_cg_init_finalize(s, pt.red.ptr, o->rtol, o->atol, o->norm, o->max_it, o->reg, pt.state.ptr,
                              pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
  }
  RC(phase_event(h, h->ev[2], s));
  // (phase times: the setup's end is an event between the setup and the entry)
  const bool entry = h->opt_graph && h->opt_setup_entry && !h->opt_phase_times;
  const int tag = -1000 - (int)(pt.amg_gen % 1000000);
  // the converging update is iteration `iters`; update 0 ran in the entry, so
  // `expected` more updates = expected / chunk chunks (drive_planned adds one
  // for the update it assumes the chunk starts with: pass expected − 1)
  const int expected = std::max(0, std::min(o->max_it, pt.amg_last_iters > 0 ? pt.amg_last_iters : 16) - 1);
  const int need = std::max(1, expected + 1);
  // mfea_step: the planned batch, the finish and the post as ONE graph of the
  // batch's exact length (option batch_graph), behind the setup in the same
  // graph (option combo_graph)
  const bool batch = h->spec_on && !h->spec_used && h->opt_batch_graph && !h->opt_phase_times &&
                     o->chunk <= 0 && need < mfea_handle::kRemGraphs && h->opt_graph;
  const bool combo = batch && entry && h->opt_combo_graph;
  // (combo: the graph reaches the batch's end and publishes the state; the
  // host's copy of the flag is cleared before it can)
  if (combo) h->h_state[0].done = 0;
  if (h->opt_graph)
    RC(launch_amg_setup_graph(h, pt, o->reg, entry, head ? o : nullptr, start_in_graph ? o : nullptr,
                              combo ? need : 0, tag));
  else enqueue_amg_setup(h, pt, o->reg);
  clk.lap("to the setup graph");
  if (!entry) {
    RC(phase_event(h, h->ev_setup, s));
    h->ev_setup_used = true;
    enqueue_amg_entry(h, pt);
  }
  HIPC(hipGetLastError());
  const bool no_graph = !h->opt_graph;
  SolveState fin;
  int rc;
  const auto drive_t0 = std::chrono::steady_clock::now();
  // x to row order behind every planned batch (see drive_planned)
  auto finish = [&]() -> int {
    launch_amg_finish(s, nd, pt.amg_cg, pt.x.ptr);
    HIPC(hipGetLastError());
    return spec_post(h);  // (mfea_step: the post behind the batch, one wait for both)
  };
  if (no_graph) {
    rc = drive_planned(h, chunk, o->max_it, expected,
                       [&]() -> int {
                         enqueue_amg_chunk(h, pt, chunk);
                         HIPC(hipGetLastError());
                         return 0;
                       },
                       &fin, finish);
  } else {
    auto capture = [&](hipGraphExec_t* ge, int n) -> int {
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      enqueue_amg_chunk(h, pt, n);
      HIPC(hipStreamEndCapture(s, &g));
      hipError_t e = hipGraphInstantiate(ge, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      return 0;
    };
    if (h->graph == nullptr || h->graph_chunk != chunk || h->graph_precond != MFEA_PC_GAMG ||
        h->graph_ell != tag) {
      destroy_graph(h);
      RC(capture(&h->graph, chunk));
      h->graph_chunk = chunk;
      h->graph_precond = MFEA_PC_GAMG;
      h->graph_ell = tag;
    }
    // the planned batch in long chunks (default solves only: a caller's
    // chunk size is kept as given); measured at C3 / C2: chunks of 8 in the
    // batch 2.24 / 1.15 ms per step against 2.36 / 1.20 with chunks of 2
    const int big = o->chunk > 0 ? chunk : h->opt_amg_big_chunk;
    if (big > chunk && (h->graph_big == nullptr || h->graph_big_chunk != big || h->graph_big_ell != tag)) {
      if (h->graph_big) (void)hipGraphExecDestroy(h->graph_big);
      h->graph_big = nullptr;
      RC(capture(&h->graph_big, big));
      h->graph_big_chunk = big;
      h->graph_big_ell = tag;
    }
    // the batch's remainder as ONE chunk of its own length (captured once per
    // length; the AMG iteration kernels keep no state across chunks that
    // depends on the chunk's parity): an odd iteration count no longer runs
    // one gated iteration — which costs as much as a live one — nor two
    // extra chunk boundaries (C3 at 15 iterations: 8 + 7 instead of 8 + 4×2)
    const int rem = big > chunk ? need - (need / big) * big : 0;
    const bool exact_rem = rem > 0 && rem != chunk && rem < mfea_handle::kRemGraphs;
    if (h->graph_rem_ell != tag) {  // another plan: the cached lengths hold its pointers
      for (auto& g : h->graph_rem) {
        if (g) (void)hipGraphExecDestroy(g);
        g = nullptr;
      }
      h->graph_rem_ell = tag;
    }
    // (batch_graph: C2 / C3 two graph launches and four eager ones fewer per step)
    if (batch) {
      if (h->graph_batch_ell != tag || h->graph_batch_strain != h->spec_strain) {
        for (auto& g : h->graph_batch) {
          if (g) (void)hipGraphExecDestroy(g);
          g = nullptr;
        }
        h->graph_batch_ell = tag;
        h->graph_batch_strain = h->spec_strain;
      }
      if (!combo && h->graph_batch[need] == nullptr) {
        hipGraph_t g;
        HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        enqueue_amg_chunk(h, pt, need);
        launch_amg_finish(s, nd, pt.amg_cg, pt.x.ptr);
        const int prc = enqueue_post_work(h, h->spec_strain);
        const hipError_t ec = hipStreamEndCapture(s, &g);
        RC(prc);
        HIPC(ec);
        hipError_t e = hipGraphInstantiate(&h->graph_batch[need], g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        HIPC(e);
      }
      rc = drive_batch(h, chunk, o->max_it, need,
                       [&]() -> int {
                         if (!combo) HIPC(hipGraphLaunch(h->graph_batch[need], s));  // (combo: launched with the setup)
                         return 0;
                       },
                       [&](int n) -> int {
                         HIPC(hipGraphLaunch(h->graph, s));
                         (void)n;
                         return 0;
                       },
                       &fin, finish, combo);
    } else {
      if (exact_rem && h->graph_rem[rem] == nullptr) RC(capture(&h->graph_rem[rem], rem));
      rc = drive_sized(h, big, chunk, o->max_it, expected,
                       [&](int n) -> int {
                         HIPC(hipGraphLaunch(n == chunk ? h->graph : n == big ? h->graph_big : h->graph_rem[n], s));
                         return 0;
                       },
                       &fin, finish, exact_rem);
    }
  }
  if (rc) return rc;
  if (fin.status != 0) RC(spec_undo(h));
  clk.lap("solve (setup + iterations)", fin.iters);
  if (fin.status != 0 && pt.amg_reused) {
    // a hierarchy kept from another active set failed: rebuild for this one
    // before anything else is blamed (the ω retry below would otherwise run
    // on the kept hierarchy)
    pt.amg_stale = true;
    RC(sync_stream(h));
    return solve_amg(h, dy_top, dy_bot, o, st);
  }
  if (pt.amg_lev.size() > 1 && pt.amg_kind == MFEA_PC_GAMG &&
      omega_suspect(h, fin.status, o->max_it, std::max(pt.amg_build_iters, pt.amg_last_iters)))
    return omega_retry(h, [&]() { return solve_amg(h, dy_top, dy_bot, o, st); });
  if (fin.status == 0) pt.amg_last_iters = fin.iters;
  if (fin.status == 0 && !pt.amg_reused) {
    pt.amg_build_iters = fin.iters;  // the hierarchy on the set it was built for
  } else if (pt.amg_reused && pt.amg_build_iters >= 0) {
    // rent or buy: the iterations above the hierarchy's own count cost this
    // solve's time per iteration; once that rent adds up to the last build's
    // time, or one solve needs far more (amg_rebuild_pct), rebuild
    const double t_it = std::chrono::duration<double>(std::chrono::steady_clock::now() - drive_t0).count() /
                        std::max<int64_t>(1, fin.iters + 1);
    if (fin.iters > pt.amg_build_iters) pt.amg_excess_s += (fin.iters - pt.amg_build_iters) * t_it;
    const bool rent_due = h->opt_amg_rebuild_rent > 0 &&
                          pt.amg_excess_s >= pt.amg_build_s * h->opt_amg_rebuild_rent / 100.0;
    if (rent_due || fin.iters > (int64_t)pt.amg_build_iters * h->opt_amg_rebuild_pct / 100 + 2)
      pt.amg_stale = true;  // degraded: the next solve rebuilds for its active set
  }
  rc = finish_solve(h, fin, st);
  if (st) {
    st->amg_levels = (int32_t)pt.amg_lev.size();
    st->amg_rebuilt = rebuilt ? 1 : 0;
  }
  return rc;
}

// ---------------------------------------------------------------------------
// Distributed GAMG over ONE global hierarchy (option "amg_dist" 1, the
// default of partitioned handles).  Every rank builds the same
// hierarchy from the whole mesh — the one-partition hierarchy, so the solve
// needs the one-partition iteration count — and computes only its own rows of
// the split levels (amg.hpp AmgRank); the values a rank's rows read from
// other ranks arrive through the exchanges below.  Levels of at most
// "amg_rep_rows" rows are replicated: every rank holds and computes all of them.
// ---------------------------------------------------------------------------
// The global element activity (original order).  Partitions on one device:
// each partition's own elements; RCCL: a max-all-reduce of E bytes (a rank
// contributes the elements it reports, 0 elsewhere).
int global_active(mfea_handle* h, std::vector<uint8_t>& key) {
  if (h->gkey_gen == h->act_gen && (int64_t)h->gkey.size() == h->Ecount) {
    key = h->gkey;  // kept current by mfea_set_active and the failed-id exchange
    return 0;
  }
  key.assign(h->Ecount, 0);
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int64_t E = pt.P.n_elems;
    std::vector<uint8_t> a(E);
    if (E) HIPC(hmemcpy(h, a.data(), pt.active.ptr, E, hipMemcpyDeviceToHost));
    for (int64_t le = 0; le < E; ++le)
      if (pt.plan.elem_own[le]) key[pt.plan.elem_g[le]] = a[le];
  }
  if (h->world > 1 && h->Ecount) {
    HIPC(h->gact.alloc(h->Ecount));
    HIPC(hipMemcpyAsync(h->gact.ptr, key.data(), h->Ecount, hipMemcpyHostToDevice, h->stream));
    NCCLC(ncclAllReduce(h->gact.ptr, h->gact.ptr, (size_t)h->Ecount, ncclUint8, ncclMax, h->comm, h->stream));
    HIPC(hipMemcpyAsync(key.data(), h->gact.ptr, h->Ecount, hipMemcpyDeviceToHost, h->stream));
    RC(sync_stream(h));
  }
  h->gkey = key;
  h->gkey_gen = h->act_gen;
  return 0;
}

// the partition's exchange plans on the device (item lists carved from one
// allocation) and staging buffers for the largest transfer
int upload_xplans(mfea_handle* h, Part& pt) {
  const AmgRank& rk = pt.amg_rank;
  const int nd = h->gamg.nd;
  size_t items = 0, stage = 1;
  auto size = [&](const XPlan& x, int width_bytes) {
    items += x.sidx.size() + x.ridx.size() + 2;
    stage = std::max(stage, (size_t)std::max(x.n_send(), x.n_recv()) * width_bytes);
  };
  for (const auto& x : rk.xa) size(x, 4 * nd);
  for (const auto& x : rk.xr) size(x, 4 * nd);
  for (const auto& x : rk.xp) size(x, 4 * nd);
  size(rk.xg, 4 * nd);
  for (const auto& x : rk.sp) size(x, 8 * nd * nd);
  for (const auto& x : rk.sap) size(x, 8 * nd * nd);
  size(rk.sg, 8 * nd * nd);
  size(rk.xc, 4 * nd);
  size(rk.spt, 4 * nd * nd);
  size(rk.sd, 4 * nd * nd);
  HIPC(pt.amg_xi.alloc(items));
  HIPC(pt.amg_xs.alloc(stage / 8 + 1));
  HIPC(pt.amg_xr.alloc(stage / 8 + 1));
  int32_t* ip = pt.amg_xi.ptr;
  hipStream_t s = h->stream;
  auto put = [&](const XPlan& x) -> Part::XDev {
    Part::XDev d;
    d.x = &x;
    d.s = ip;
    if (!x.sidx.empty()) (void)hipMemcpyAsync(ip, x.sidx.data(), x.sidx.size() * 4, hipMemcpyHostToDevice, s);
    ip += x.sidx.size() + 1;
    d.r = ip;
    if (!x.ridx.empty()) (void)hipMemcpyAsync(ip, x.ridx.data(), x.ridx.size() * 4, hipMemcpyHostToDevice, s);
    ip += x.ridx.size() + 1;
    return d;
  };
  pt.xd_a.clear();
  pt.xd_r.clear();
  pt.xd_p.clear();
  pt.xd_sp.clear();
  pt.xd_sap.clear();
  for (const auto& x : rk.xa) pt.xd_a.push_back(put(x));
  for (const auto& x : rk.xr) pt.xd_r.push_back(put(x));
  for (const auto& x : rk.xp) pt.xd_p.push_back(put(x));
  pt.xd_g = put(rk.xg);
  for (const auto& x : rk.sp) pt.xd_sp.push_back(put(x));
  for (const auto& x : rk.sap) pt.xd_sap.push_back(put(x));
  pt.xd_sg = put(rk.sg);
  pt.xd_c = put(rk.xc);
  pt.xd_spt = put(rk.spt);
  pt.xd_sd = put(rk.sd);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// the distributed V-cycle in its compact form (option amg_dist_cycle)
bool dist_compact(const mfea_handle* h) { return h->opt_amg_dist_cycle == 1 && h->opt_amg_cycle == 1; }

// (Re)build the global hierarchy (host) when the element activity may have
// changed (act_gen) and actually did.
int ensure_gamg_plan(mfea_handle* h, bool* rebuilt) {
  *rebuilt = false;
  bool host_ok = h->gamg_ok && h->gamg_act_gen == h->act_gen;
  if (!host_ok && h->gamg_ok) {
    std::vector<uint8_t> key;
    RC(global_active(h, key));
    host_ok = key == h->gamg_key;
    if (host_ok) h->gamg_act_gen = h->act_gen;
  }
  if (!host_ok) {
    std::vector<uint8_t> key;
    RC(global_active(h, key));
    h->gamg_ok = false;
    AmgDistSpec spec;
    spec.world = nranks(h);
    const bool compact = dist_compact(h);
    spec.rep_rows = compact ? INT64_MAX : h->opt_amg_rep_rows;
    spec.owner.resize(h->gpat.n_free);
    for (int64_t i = 0; i < h->gpat.n_free; ++i) spec.owner[i] = h->gowner[h->gpat.perm[i]];
    std::string err = build_amg(h->gpat, key, lane_dofs(h), h->gamg, h->opt_amg_max_levels, &spec,
                                amg_strength(h));
    if (!err.empty()) return fail(MFEA_EINVAL, "AMG setup: " + err);
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      err = build_amg_rank(h->gamg, pt.rank, pt.amg_rank);
      if (!compact) pt.amg_rank.compact = false;  // (a four-step plan split at level 0 only)
      if (err.empty())
        err = build_amg_level0(h->gamg, h->gpat, pt.amg_rank, pt.P, pt.plan.node_g, pt.plan.elem_g, key, pt.g_a0,
                               pt.g_row0);
      if (!err.empty()) return fail(MFEA_EINVAL, "AMG setup: " + err);
      pt.dev_plan = -1;
    }
    h->gamg_key = std::move(key);
    h->gamg_ok = true;
    h->gamg_act_gen = h->act_gen;
    ++h->gamg_plan_gen;
    *rebuilt = true;
  }
  return 0;
}

// ... and have the device arrays hold it (they may hold the block-Jacobi plans)
int ensure_gamg(mfea_handle* h, bool* rebuilt) {
  RC(ensure_gamg_plan(h, rebuilt));
  bool up = false;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    if (pt.dev_plan == 1) continue;
    if (!up) destroy_graph(h);
    up = true;
    RC(upload_amg(h, pt, h->gamg, &pt.amg_rank, &pt.g_a0, &pt.g_row0));
    RC(upload_xplans(h, pt));
    AmgDist& d = pt.amg_dist;
    d = AmgDist{};
    d.rank = pt.rank;
    d.gall[0] = pt.dv.gall[0];
    d.gall[1] = pt.dv.gall[1];
    d.gsend = pt.dv.gsend;
    d.zero_w = h->world > 1 && h->opt_dist_sums == 1 ? h->world : 0;
    pt.dev_plan = 1;
  }
  if (up) ++h->gamg_gen;
  return 0;
}

// One exchange of the distributed GAMG on every partition: pack the items of
// plan(pt) from vec(pt) (width scalars of `bytes` each), one RCCL group of
// point-to-point transfers (partitions on one device: device copies), unpack
// into the same array.
template <class GetPlan, class GetVec>
int gx(mfea_handle* h, GetPlan plan, GetVec vec, int width, int bytes) {
  hipStream_t s = h->stream;
  if (h->world <= 1) {  // partitions on one device: every transfer in one launch, array to array
    XPairs pr;
    for (auto& a : h->parts) {
      const Part::XDev& da = plan(*a);
      const XPlan& xa = *da.x;
      for (size_t i = 0; i < xa.peers.size(); ++i) {
        if (!xa.scnt[i]) continue;
        Part& b = *h->parts[xa.peers[i]];
        const Part::XDev& db = plan(b);
        const XPlan& xb = *db.x;
        const auto it = std::lower_bound(xb.peers.begin(), xb.peers.end(), a->rank);
        const size_t jb = (size_t)(it - xb.peers.begin());
        if (it == xb.peers.end() || *it != a->rank || xb.rcnt[jb] != xa.scnt[i])
          return fail(MFEA_EINVAL, "internal: asymmetric GAMG exchange plan");
        if (pr.n == kMaxXPairs) {
          launch_xcopy(s, pr, width, bytes);
          pr = XPairs();
        }
        pr.src[pr.n] = vec(*a);
        pr.dst[pr.n] = vec(b);
        pr.sidx[pr.n] = da.s + xa.soff[i];
        pr.ridx[pr.n] = db.r + xb.roff[jb];
        pr.off[pr.n + 1] = pr.off[pr.n] + xa.scnt[i];
        ++pr.n;
      }
    }
    launch_xcopy(s, pr, width, bytes);
    HIPC(hipGetLastError());
    return 0;
  }
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Part::XDev& d = plan(pt);
    launch_xpack(s, vec(pt), d.s, d.x->n_send(), width, bytes, pt.amg_xs.ptr);
  }
  HIPC(hipGetLastError());
  const size_t item = (size_t)width * bytes;
  if (h->world > 1) {
    Part& pt = part0(h);
    const XPlan& x = *plan(pt).x;
    if (!x.peers.empty()) {
      const ncclDataType_t t = bytes == 8 ? ncclFloat64 : ncclFloat32;
      char* sb = reinterpret_cast<char*>(pt.amg_xs.ptr);
      char* rb = reinterpret_cast<char*>(pt.amg_xr.ptr);
      NCCLC(ncclGroupStart());
      for (size_t i = 0; i < x.peers.size(); ++i) {
        if (x.scnt[i])
          NCCLC(ncclSend(sb + x.soff[i] * item, (size_t)(x.scnt[i] * width), t, x.peers[i], h->comm, s));
        if (x.rcnt[i])
          NCCLC(ncclRecv(rb + x.roff[i] * item, (size_t)(x.rcnt[i] * width), t, x.peers[i], h->comm, s));
      }
      NCCLC(ncclGroupEnd());
    }
  } else {
    for (auto& a : h->parts) {
      const XPlan& xa = *plan(*a).x;
      for (size_t i = 0; i < xa.peers.size(); ++i) {
        if (!xa.scnt[i]) continue;
        Part& b = *h->parts[xa.peers[i]];
        const XPlan& xb = *plan(b).x;
        const auto it = std::lower_bound(xb.peers.begin(), xb.peers.end(), a->rank);
        const size_t jb = (size_t)(it - xb.peers.begin());
        if (it == xb.peers.end() || *it != a->rank || xb.rcnt[jb] != xa.scnt[i])
          return fail(MFEA_EINVAL, "internal: asymmetric GAMG exchange plan");
        HIPC(hipMemcpyAsync(reinterpret_cast<char*>(b.amg_xr.ptr) + xb.roff[jb] * item,
                            reinterpret_cast<const char*>(a->amg_xs.ptr) + xa.soff[i] * item, xa.scnt[i] * item,
                            hipMemcpyDeviceToDevice, s));
      }
    }
  }
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Part::XDev& d = plan(pt);
    launch_xunpack(s, pt.amg_xr.ptr, d.r, d.x->n_recv(), width, bytes, vec(pt));
  }
  HIPC(hipGetLastError());
  return 0;
}

// level l's Gershgorin bound: the maximum over the ranks (every rank then
// takes the same smoother weight ω_l and forms the same P_l)
int bound_max(mfea_handle* h, int l) {
  if (h->world > 1) {
    double* om = part0(h).amg_lev[l].omega + 1;
    NCCLC(ncclAllReduce(om, om, 1, ncclFloat64, ncclMax, h->comm, h->stream));
    return 0;
  }
  std::vector<double*> oms;
  for (auto& pp : h->parts) oms.push_back(pp->amg_lev[l].omega);
  launch_amg_bound_max(h->stream, oms.data(), (int)oms.size());
  HIPC(hipGetLastError());
  return 0;
}

// the per-solve numeric setup, split levels with their exchanges
int enqueue_gamg_setup(mfea_handle* h, double reg) {
  hipStream_t s = h->stream;
  const AmgPlan& pl = h->gamg;
  const int nd = pl.nd, nb2 = nd * nd, nlev = (int)pl.lev.size(), ns = pl.n_dist;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_a0(s, nd, pt.amg_lev[0], sell_op(pt), pt.amg_cg.row0, pt.amg_a0_ptr, pt.amg_a0_a, reg);
  }
  HIPC(hipGetLastError());
  RC(bound_max(h, 0));
  for (int l = 0; l < nlev; ++l) {
    const bool split = l < ns;
    auto stage = [&](int st) -> int {
      for (auto& pp : h->parts) {
        Part& pt = *pp;
        launch_amg_level_setup(s, nd, pt.amg_lev[l], l + 1 < nlev ? &pt.amg_lev[l + 1] : nullptr, l == 0, st);
      }
      HIPC(hipGetLastError());
      return 0;
    };
    if (l > 0) {
      RC(stage(kSetupDinv));
      if (split) RC(bound_max(h, l));
    }
    if (pl.lev[l].coarsest) break;
    RC(stage(kSetupP));
    if (split)
      RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_sp[l]; },
            [l](Part& p) -> void* { return p.amg_lev[l].P.val32; }, nb2, 4));
    RC(stage(kSetupAP));
    if (split)
      RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_sap[l]; },
            [l](Part& p) -> void* { return p.amg_lev[l].apval; }, nb2, 4));
    RC(stage(kSetupAC));
    if (l + 1 == ns && ns < nlev) {  // level ns is replicated: gather its A
      RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_sg; },
            [ns](Part& p) -> void* { return p.amg_lev[ns].A.val32; }, nb2, 4));
    }
  }
  if (part0(h).amg_rank.compact && nlev > 1) {
    // the compact operators: level 0's Ã_0 and P̃_0 on this rank's rows; the
    // P̃_0 blocks and level-0 diagonal blocks other ranks' R̂_0 rows read; its
    // own R̂_0 rows; the replicated levels whole, then their collapse
    for (auto& pp : h->parts)
      launch_amg_compact_level(s, nd, pp->amg_lev.data(), 0, kCompactPT | kCompactAT);
    HIPC(hipGetLastError());
    RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_spt; },
          [](Part& p) -> void* { return p.amg_lev[0].PT.val32; }, nb2, 4));
    RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_sd; },
          [](Part& p) -> void* { return p.amg_lev[0].A.val32; }, nb2, 4));
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_amg_compact_level(s, nd, pt.amg_lev.data(), 0, kCompactRT);
      launch_amg_compact_setup(s, nd, pt.amg_lev.data(), nlev, pt.amg_cg.coll, 1);
    }
    HIPC(hipGetLastError());
  }
  return 0;
}

// One distributed V-cycle on every partition (gate: iteration j's flag;
// j < 0: ungated, the solve's first cycle)
int enqueue_gamg_vcycle(mfea_handle* h, int j) {
  hipStream_t s = h->stream;
  const AmgPlan& pl = h->gamg;
  const int nd = pl.nd, nlev = (int)pl.lev.size(), ns = pl.n_dist;
  if (nlev <= 1) return 0;  // the update's vcycle_entry solved the only level
  if (part0(h).amg_rank.compact) {
    // split at level 0 only: x_0 halo → down_0 (this rank's R̂_0 rows into
    // x_1, its Ã_0 rows into c_0) → x_1 all-gather → the replicated compact
    // cycle from level 1 (collapsed as on one partition) → up_0 on this
    // rank's P̃_0 rows into u.  Three exchange points with the u halo.
    RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_c; }, [](Part& p) -> void* { return p.amg_lev[0].x; },
          nd, 4));
    for (auto& pp : h->parts) launch_amg_down(s, nd, pp->amg_lev[0], pp->amg_lev[1]);
    HIPC(hipGetLastError());
    RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_g; }, [](Part& p) -> void* { return p.amg_lev[1].x; },
          nd, 4));
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_amg_vcycle(s, nd, pt.amg_lev.data(), nlev, pt.amg_cg, 0, nullptr, 1);
      launch_amg_up(s, nd, pt.amg_lev[0], pt.amg_lev[1], pt.amg_cg.u);
    }
    HIPC(hipGetLastError());
    return 0;
  }
  const int top = std::min(ns, nlev - 1);  // split levels with a level below
  (void)j;  // no gate (enqueue_amg_chunk): past the stop every launch rewrites the same values
  auto gate = [](Part&) -> const int32_t* { return nullptr; };
  auto steps = [&](int l, int step) {
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_amg_vstep(s, nd, pt.amg_lev.data(), l, pt.amg_cg, step, gate(pt));
    }
  };
  for (int l = 0; l < top; ++l) {
    RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_a[l]; },
          [l](Part& p) -> void* { return p.amg_lev[l].x; }, nd, 4));
    steps(l, kStepResid);
    HIPC(hipGetLastError());
    RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_r[l]; },
          [l](Part& p) -> void* { return p.amg_lev[l].t; }, nd, 4));
    steps(l, kStepRestrict);
    HIPC(hipGetLastError());
  }
  if (ns < nlev) {  // the replicated levels: gather level ns's b, every rank runs them whole
    RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_g; },
          [ns](Part& p) -> void* { return p.amg_lev[ns].b; }, nd, 4));
    for (auto& pp : h->parts) {
      Part& pt = *pp;
      launch_amg_xinit_rows(s, nd, pt.amg_lev[ns], pt.xd_g.r, pt.xd_g.x->n_recv(), gate(pt));
      launch_amg_vcycle(s, nd, pt.amg_lev.data(), nlev, pt.amg_cg, pt.amg_tail, gate(pt), ns);
    }
    HIPC(hipGetLastError());
  }
  for (int l = top - 1; l >= 0; --l) {
    if (l + 1 < ns) {  // the coarse output of a split level
      const bool co = pl.lev[l + 1].coarsest;
      RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_p[l]; },
            [l, co](Part& p) -> void* { return co ? p.amg_lev[l + 1].x : p.amg_lev[l + 1].e; }, nd, 4));
    }
    steps(l, kStepProlong);
    HIPC(hipGetLastError());
    RC(gx(h, [l](Part& p) -> const Part::XDev& { return p.xd_a[l]; },
          [l](Part& p) -> void* { return p.amg_lev[l].x; }, nd, 4));
    steps(l, kStepPost);
    HIPC(hipGetLastError());
  }
  return 0;
}

// one distributed GAMG iteration j: update (gathered sums) → V-cycle → u halo
// → w = A_0 u → this rank's sums → all-gather of the sums
int enqueue_gamg_iteration(mfea_handle* h, int j) {
  hipStream_t s = h->stream;
  const int nd = h->gamg.nd;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_update(s, nd, j, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.state.ptr, pt.cg_part.ptr,
                         &pt.amg_dist);
  }
  HIPC(hipGetLastError());
  RC(enqueue_gamg_vcycle(h, j));
  RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_a[0]; }, [](Part& p) -> void* { return p.amg_cg.u; },
        nd, 4));
  const int q = (j & 1) ^ 1;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_w(s, nd, j, false, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
    launch_amg_gsum(s, pt.amg_cg, cg_part_buf(pt, q), pt.amg_dist, q);
  }
  HIPC(hipGetLastError());
  return xchg_sums(h, q);
}

int enqueue_gamg_chunk(mfea_handle* h, int chunk) {
  for (int j = 0; j < chunk; ++j) RC(enqueue_gamg_iteration(h, j));
  for (auto& pp : h->parts) launch_cg_advance(h->stream, chunk, pp->slots.ptr, pp->state.ptr, pp->mirror);
  HIPC(hipGetLastError());
  return 0;
}

int solve_gamg_global(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o, mfea_stats* st) {
  hipStream_t s = h->stream;
  bool rebuilt = false;
  RC(ensure_gamg(h, &rebuilt));
  const int chunk = o->chunk > 0 ? solve_chunk_size(o) : 2;
  const int W = nranks(h);
  const int nd = h->gamg.nd;
  RC(phase_event(h, h->ev[1], s));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_cg_rhs(s, sell_op(pt), pt.code.ptr, dy_top, dy_bot, o->reg, 2, cg_vecs(pt), pt.partials.ptr, tix(pt, 0),
                  pt.red.ptr);
  }
  RC(gather4(h, 0));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rank_sum(s, pt.gred, W, pt.red.ptr + 12);
    launch_cg_init_finalize(s, pt.red.ptr + 12, o->rtol, o->atol, o->norm, o->max_it, o->reg, pt.state.ptr,
                            pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
  }
  RC(phase_event(h, h->ev[2], s));
  RC(enqueue_gamg_setup(h, o->reg));
  RC(phase_event(h, h->ev_setup, s));
  h->ev_setup_used = true;
  // iteration 0's u and w: the V-cycle of r₀, ungated
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_init(s, nd, pt.amg_lev[0], pt.amg_cg, cg_vecs(pt).r[0]);
  }
  RC(enqueue_gamg_vcycle(h, -1));
  RC(gx(h, [](Part& p) -> const Part::XDev& { return p.xd_a[0]; }, [](Part& p) -> void* { return p.amg_cg.u; },
        nd, 4));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_w(s, nd, 0, true, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
    launch_amg_gsum(s, pt.amg_cg, cg_part_buf(pt, 0), pt.amg_dist, 0);
  }
  RC(xchg_sums(h, 0));
  HIPC(hipGetLastError());
  const int tag = -3000000 - (int)(h->gamg_gen % 1000000);
  Part& p0 = part0(h);
  const int expected = std::min(o->max_it, p0.amg_last_iters > 0 ? p0.amg_last_iters : 16);
  SolveState fin;
  if (!h->opt_dist_graph) {
    RC(drive_planned(h, chunk, o->max_it, expected, [&]() -> int { return enqueue_gamg_chunk(h, chunk); }, &fin));
  } else {
    if (h->graph == nullptr || h->graph_chunk != chunk || h->graph_precond != MFEA_PC_GAMG || h->graph_ell != tag) {
      destroy_graph(h);
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int rc = enqueue_gamg_chunk(h, chunk);
      const hipError_t ce = hipStreamEndCapture(s, &g);
      if (rc) return rc;
      HIPC(ce);
      hipError_t e = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      h->graph_chunk = chunk;
      h->graph_precond = MFEA_PC_GAMG;
      h->graph_ell = tag;
    }
    RC(drive_planned(h, chunk, o->max_it, expected,
                     [&]() -> int {
                       HIPC(hipGraphLaunch(h->graph, s));
                       return 0;
                     },
                     &fin));
  }
  if (omega_suspect(h, fin.status, o->max_it, p0.amg_last_iters))
    return omega_retry(h, [&]() { return solve_gamg_global(h, dy_top, dy_bot, o, st); });
  if (fin.status == 0) p0.amg_last_iters = fin.iters;
  // x to row order, then the displacement halo (ghost rows of the post kernels)
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_finish(s, nd, pt.amg_cg, pt.x.ptr);
    launch_rows_pack(s, pt.xsend_rows.ptr, (int64_t)pt.plan.xsend_node.size(), pt.x.ptr, pt.xh_send);
  }
  RC(xchg_xhalo(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rows_unpack(s, pt.xrecv_rows.ptr, (int64_t)pt.plan.xrecv_node.size(), pt.xh_recv, pt.x.ptr);
  }
  HIPC(hipGetLastError());
  const int rc = finish_solve(h, fin, st);
  if (st) {
    st->amg_levels = (int32_t)h->gamg.lev.size();
    st->amg_rebuilt = rebuilt ? 1 : 0;
  }
  return rc;
}

// The partitioned GAMG solve: block-Jacobi-over-partitions AMG V-cycles inside
// a global CG (amg.hpp AmgHalo), the exchanges of enqueue_amg_dist_iteration.
int solve_amg_dist(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
                   mfea_stats* st) {
  hipStream_t s = h->stream;
  bool rebuilt = false;
  for (auto& pp : h->parts) {
    bool rb = false;
    RC(ensure_amg(h, *pp, &rb));
    rebuilt = rebuilt || rb;
  }
  const int chunk = o->chunk > 0 ? solve_chunk_size(o) : 2;
  const int W = nranks(h);
  RC(phase_event(h, h->ev[1], s));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_cg_rhs(s, sell_op(pt), pt.code.ptr, dy_top, dy_bot, o->reg, 2, cg_vecs(pt), pt.partials.ptr,
                  tix(pt, 0), pt.red.ptr);
  }
  RC(gather4(h, 0));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rank_sum(s, pt.gred, W, pt.red.ptr + 12);
    launch_cg_init_finalize(s, pt.red.ptr + 12, o->rtol, o->atol, o->norm, o->max_it, o->reg, pt.state.ptr,
                            pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
  }
  RC(phase_event(h, h->ev[2], s));
  for (auto& pp : h->parts) enqueue_amg_setup(h, *pp, o->reg);
  RC(phase_event(h, h->ev_setup, s));
  h->ev_setup_used = true;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int nd = pt.amg.nd;
    launch_amg_cg_init(s, nd, pt.amg_lev[0], pt.amg_cg, cg_vecs(pt).r[0]);
    launch_amg_vcycle(s, nd, pt.amg_lev.data(), (int)pt.amg_lev.size(), pt.amg_cg,
                      pt.amg_tail, nullptr);
    launch_amg_pack_u(s, nd, pt.amg_cg, pt.amg_dist);
  }
  RC(xchg_u(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_cg_w(s, pt.amg.nd, 0, true, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr,
                    &pt.amg_dist);
    launch_amg_gsum(s, pt.amg_cg, cg_part_buf(pt, 0), pt.amg_dist, 0);
  }
  RC(xchg_sums(h, 0));
  HIPC(hipGetLastError());
  int64_t gen = 0;
  for (auto& pp : h->parts) gen = gen * 1000003 + pp->amg_gen;
  const int tag = -2000000 - (int)(gen % 1000000);
  Part& p0 = part0(h);
  const int expected = std::min(o->max_it, p0.amg_last_iters > 0 ? p0.amg_last_iters : 16);
  SolveState fin;
  if (!h->opt_dist_graph) {
    RC(drive_planned(h, chunk, o->max_it, expected, [&]() -> int { return enqueue_amg_dist_chunk(h, chunk); },
                     &fin));
  } else {
    if (h->graph == nullptr || h->graph_chunk != chunk || h->graph_precond != MFEA_PC_GAMG ||
        h->graph_ell != tag) {
      destroy_graph(h);
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int rc = enqueue_amg_dist_chunk(h, chunk);
      const hipError_t ce = hipStreamEndCapture(s, &g);
      if (rc) return rc;
      HIPC(ce);
      hipError_t e = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      h->graph_chunk = chunk;
      h->graph_precond = MFEA_PC_GAMG;
      h->graph_ell = tag;
    }
    RC(drive_planned(h, chunk, o->max_it, expected,
                     [&]() -> int {
                       HIPC(hipGraphLaunch(h->graph, s));
                       return 0;
                     },
                     &fin));
  }
  if (omega_suspect(h, fin.status, o->max_it, p0.amg_last_iters))
    return omega_retry(h, [&]() { return solve_amg_dist(h, dy_top, dy_bot, o, st); });
  if (fin.status == 0) p0.amg_last_iters = fin.iters;
  // x to row order, then the displacement halo (ghost rows of the post kernels)
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_amg_finish(s, pt.amg.nd, pt.amg_cg, pt.x.ptr);
    launch_rows_pack(s, pt.xsend_rows.ptr, (int64_t)pt.plan.xsend_node.size(), pt.x.ptr, pt.xh_send);
  }
  RC(xchg_xhalo(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rows_unpack(s, pt.xrecv_rows.ptr, (int64_t)pt.plan.xrecv_node.size(), pt.xh_recv, pt.x.ptr);
  }
  HIPC(hipGetLastError());
  const int rc = finish_solve(h, fin, st);
  if (st) {
    st->amg_levels = (int32_t)p0.amg_lev.size();
    st->amg_rebuilt = rebuilt ? 1 : 0;
  }
  return rc;
}

// The partitioned solve: the same CG-CG iterations on every partition's lanes,
// with the exchanges of partition.hpp between kernels.
int solve_dist(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
               mfea_stats* st) {
  hipStream_t s = h->stream;
  const int precond = o->precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0;
  const int chunk = solve_chunk_size(o);
  const int W = nranks(h);
  RC(phase_event(h, h->ev[1], s));
  // RHS, M⁻¹ and the global (‖b‖², ‖M⁻¹b‖²)
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_cg_rhs(s, sell_op(pt), pt.code.ptr, dy_top, dy_bot, o->reg, precond, cg_vecs(pt),
                  pt.partials.ptr, tix(pt, 0), pt.red.ptr);
  }
  RC(gather4(h, 0));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rank_sum(s, pt.gred, W, pt.red.ptr + 12);
    launch_cg_init_finalize(s, pt.red.ptr + 12, o->rtol, o->atol, o->norm, o->max_it, o->reg,
                            pt.state.ptr,
                            pt.cg_part.ptr, 2 * 4 * kCgMaxPartials);
    launch_ell_init(s, ell_op(h, pt), sell_op(pt), precond, cg_vecs(pt), ell_vecs(pt));
    launch_ell_pack0(s, ell_op(h, pt), precond, ell_vecs(pt), pt.dv);
  }
  RC(xchg_records(h, 1, false));  // [r₀ | M] of the cut rows
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_ell_first(s, ell_op(h, pt), o->reg, precond, ell_vecs(pt), pt.slots.ptr, pt.cg_part.ptr,
                     &pt.dv);
    launch_psum(s, ell_op(h, pt), cg_part_buf(pt, 0), pt.dv.gall[0] + 4 * pt.rank, pt.dv.gsend);
  }
  RC(xchg_records(h, 0, true));
  HIPC(hipGetLastError());
  RC(phase_event(h, h->ev[2], s));
  // each chunk (kernels + exchanges) replays as one hipGraph (option
  // "dist_graph" 0: eager launches)
  const bool dist_graph = h->opt_dist_graph;
  SolveState fin;
  if (dist_graph) {
    const int tag = -10 - lane_dofs(h);  // graph_ell key of the partitioned chunk
    if (h->graph == nullptr || h->graph_chunk != chunk || h->graph_precond != precond ||
        h->graph_ell != tag) {
      destroy_graph(h);
      hipGraph_t g;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int rc = enqueue_chunk_dist(h, chunk, precond);
      const hipError_t ce = hipStreamEndCapture(s, &g);
      if (rc) return rc;
      HIPC(ce);
      hipError_t e = hipGraphInstantiate(&h->graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPC(e);
      h->graph_chunk = chunk;
      h->graph_precond = precond;
      h->graph_ell = tag;
    }
    RC(drive_chunks(
        h, chunk, o->max_it,
        [&]() -> int {
          HIPC(hipGraphLaunch(h->graph, s));
          return 0;
        },
        &fin, /*mirror=*/true));
  } else {
    RC(drive_chunks(
        h, chunk, o->max_it, [&]() -> int { return enqueue_chunk_dist(h, chunk, precond); }, &fin,
        /*mirror=*/true));
  }
  // x to row order, then the displacement halo (ghost rows of the post kernels)
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_ell_finish(s, ell_op(h, pt), ell_vecs(pt), pt.x.ptr);
    launch_rows_pack(s, pt.xsend_rows.ptr, (int64_t)pt.plan.xsend_node.size(), pt.x.ptr, pt.xh_send);
  }
  RC(xchg_xhalo(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    launch_rows_unpack(s, pt.xrecv_rows.ptr, (int64_t)pt.plan.xrecv_node.size(), pt.xh_recv,
                       pt.x.ptr);
  }
  HIPC(hipGetLastError());
  return finish_solve(h, fin, st);
}

// the element colouring of pt's pattern on the device (symbolic.hpp
// build_elem_colour), once per pattern; false: not colourable (more than 64
// colours, or an element with one row slot) — the row gather runs instead
bool ensure_colour(mfea_handle* h, Part& pt) {
  if (pt.ec_state) return pt.ec_state > 0;
  pt.ec_state = -1;
  if (!build_elem_colour(pt.P, pt.ec).empty()) return false;
  if (pt.ec.entry.empty() && pt.P.n_elems) return false;
  if (pt.ec_entry.alloc(std::max<size_t>(pt.ec.entry.size(), 1)) != hipSuccess ||
      pt.ec_pos.alloc(std::max<size_t>(pt.ec.pos.size(), 1)) != hipSuccess)
    return false;
  if (!pt.ec.entry.empty() &&
      hipMemcpyAsync(pt.ec_entry.ptr, pt.ec.entry.data(), pt.ec.entry.size() * sizeof(int32_t),
                     hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return false;
  if (!pt.ec.pos.empty() && hipMemcpyAsync(pt.ec_pos.ptr, pt.ec.pos.data(), pt.ec.pos.size() * sizeof(int32_t),
                                           hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return false;
  pt.ec_state = 1;
  return true;
}

int assemble_impl(mfea_handle* h, mfea_stats* st, const double* rhs_dy = nullptr) {
  hipStream_t s = h->stream;
  h->assembled = true;
  h->rhs_fused = false;
  RC(phase_event(h, h->ev[0], s));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Pattern& P = pt.P;
    if (h->opt_asm_kernel == 1 && ensure_colour(h, pt)) {
      launch_assemble_colour(s, pt.ec.colors, pt.ec.cstart.data(), pt.ec_entry.ptr, pt.e2n_d.ptr, pt.ec_pos.ptr,
                             pt.xyz_d.ptr, pt.active.ptr, h->mat, pt.G, P.n_nodes, pt.val.ptr, pt.diag.ptr);
      continue;  // (RHS: its own kernel in the solve, rhs_fused stays false)
    }
    if (h->opt_asm_kernel == 2 && ensure_colour(h, pt)) {
      launch_assemble_elems(s, P.n_elems, P.n_nodes, pt.e2n_d.ptr, pt.ec_pos.ptr, pt.xyz_d.ptr, pt.active.ptr,
                            h->mat, pt.slice_ptr.ptr, pt.row_len.ptr, pt.G, pt.val.ptr, pt.diag.ptr);
      continue;
    }
    AsmRhs q{};
    const bool rhs = rhs_dy && h->parts.size() == 1;  // (rhs_dy: a one-partition GAMG / SOR / ICC step)
    if (rhs) {
      q.code = pt.code.ptr;
      q.top_end = P.n_free + P.n_top;
      q.bot_end = P.n_nodes - P.n_ghost;
      q.dy_top = rhs_dy[0];
      q.dy_bot = rhs_dy[1];
      q.nf = P.n_free;
      q.r = pt.r.ptr;
      q.x = pt.x.ptr;
      q.partials = pt.partials.ptr;
      q.ticket = tix(pt, 0);
      q.red_out = pt.red.ptr;
      h->rhs_fused = true;
      h->rhs_dy[0] = rhs_dy[0];
      h->rhs_dy[1] = rhs_dy[1];
    }
    launch_assemble(s, P.n_nodes, pt.xyz_d.ptr, pt.slice_ptr.ptr, pt.row_len.ptr, pt.s_col.ptr,
                    pt.s_elem.ptr, pt.active.ptr, h->mat, pt.G, pt.val.ptr, pt.diag.ptr, rhs ? &q : nullptr);
  }
  HIPC(hipGetLastError());
  RC(phase_event(h, h->ev[1], s));
  if (st && h->opt_phase_times) {
    RC(wait_event(h, h->ev[1]));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    st->t_assemble_ms = ms;
  }
  return 0;
}

// Partitioned: the owned elements that failed in the last post (every
// partition's device list), as global ids, gathered from every rank, cleared
// in the host's global activity.  Over RCCL two all-gathers — the counts,
// then the lists padded to the longest — instead of the E-byte max-reduction
// of the whole activity (C5: 7 MB per failure step per rank).
int apply_failures(mfea_handle* h) {
  std::vector<int32_t> ids;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    unsigned c = 0;
    HIPC(hmemcpy(h, &c, pt.fail_cnt.ptr, sizeof c, hipMemcpyDeviceToHost));
    if (c > (unsigned)pt.P.n_elems) return fail(MFEA_EINVAL, "internal: failed-element list overflow");
    std::vector<int32_t> l(c);
    if (c) HIPC(hmemcpy(h, l.data(), pt.fail_list.ptr, c * sizeof(int32_t), hipMemcpyDeviceToHost));
    for (int32_t le : l) ids.push_back((int32_t)pt.plan.elem_g[le]);
  }
  if (h->world > 1) {
    hipStream_t s = h->stream;
    const int W = h->world;
    HIPC(h->gfail.alloc(2 * (size_t)W));
    int32_t n = (int32_t)ids.size();
    HIPC(hipMemcpyAsync(h->gfail.ptr + h->rank, &n, sizeof n, hipMemcpyHostToDevice, s));
    NCCLC(ncclAllGather(h->gfail.ptr + h->rank, h->gfail.ptr + W, 1, ncclInt32, h->comm, s));
    std::vector<int32_t> cnt(W);
    HIPC(hipMemcpyAsync(cnt.data(), h->gfail.ptr + W, W * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    RC(sync_stream(h));
    const int32_t mx = *std::max_element(cnt.begin(), cnt.end());
    if (mx > 0) {
      HIPC(h->gfail.alloc((size_t)(W + 1) * mx));
      std::vector<int32_t> mine(mx, -1);
      std::copy(ids.begin(), ids.end(), mine.begin());
      HIPC(hipMemcpyAsync(h->gfail.ptr, mine.data(), mx * sizeof(int32_t), hipMemcpyHostToDevice, s));
      NCCLC(ncclAllGather(h->gfail.ptr, h->gfail.ptr + mx, (size_t)mx, ncclInt32, h->comm, s));
      std::vector<int32_t> all((size_t)W * mx);
      HIPC(hipMemcpyAsync(all.data(), h->gfail.ptr + mx, all.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      RC(sync_stream(h));
      ids.clear();
      for (int r = 0; r < W; ++r)
        for (int32_t k = 0; k < cnt[r]; ++k) ids.push_back(all[(size_t)r * mx + k]);
    } else {
      ids.clear();
    }
  }
  for (int32_t g : ids) {
    if (g < 0 || g >= h->Ecount) return fail(MFEA_EINVAL, "internal: failed element id out of range");
    h->gkey[g] = 0;
  }
  return 0;
}

// One partition: the elements that failed in the last post (the stress
// kernel's list) move the host activity — O(failures), no E-byte copy or
// O(E) pass (src/fea_solver.py:283-284: elements only ever fail).  The
// list's counter is cleared for the next post.
unsigned* fail_counter(Part& pt) { return reinterpret_cast<unsigned*>(pt.red.ptr + 6); }

int local_failures(mfea_handle* h, Part& pt, unsigned c) {
  HostLap clk;
  if (c > (unsigned)pt.P.n_elems) return fail(MFEA_EINVAL, "internal: failed-element list overflow");
  std::vector<int32_t> ids(c);
  HIPC(hmemcpy(h, ids.data(), pt.fail_list.ptr, c * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIPC(hipMemsetAsync(fail_counter(pt), 0, sizeof(unsigned), h->stream));
  if (!h->act_host_ok || h->act_host.size() != (size_t)pt.P.n_elems) return 0;
  for (int32_t e : ids) {
    if (e < 0 || e >= pt.P.n_elems || !h->act_host[e]) return fail(MFEA_EINVAL, "internal: bad failed element");
    h->act_host[e] = 0;
  }
  h->act_count -= (int64_t)c;
  clk.lap("failed ids", (int64_t)c);
  if (h->act_count != h->n_active) h->act_host_ok = false;  // cannot happen: fall back to a download
  return 0;
}

// the post kernels (reaction, stress / failures) and the read-back of their
// sums into h_red, ev[5] behind them
int enqueue_post_work(mfea_handle* h, double max_strain);
int enqueue_post(mfea_handle* h, double max_strain) {
  RC(phase_event(h, h->ev[4], h->stream));
  RC(enqueue_post_work(h, max_strain));
  HIPC(hipEventRecord(h->ev[5], h->stream));
  return 0;
}
// the post's kernels and the read-back of their sums into the pinned h_red
// (capturable: the batch graph holds them)
int enqueue_post_work(mfea_handle* h, double max_strain) {
  hipStream_t s = h->stream;
  const bool dm = partitioned(h);
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Pattern& P = pt.P;
    launch_reaction(s, P.n_free, P.n_top, P.n_nodes, pt.slice_ptr.ptr, pt.row_len.ptr, pt.s_col.ptr,
                    pt.val.ptr, pt.diag.ptr, pt.G, pt.x.ptr, pt.partials.ptr, tix(pt, 3),
                    pt.red.ptr + 4);
    if (dm) HIPC(hipMemsetAsync(pt.fail_cnt.ptr, 0, sizeof(unsigned), s));
    // one partition: the counter is red[6] (read back with the force and the
    // count, no copy of its own), zero here — cleared by the host after the
    // last failures were read (local_failures)
    launch_stress(s, P.n_elems, pt.e2n_d.ptr, pt.xyz_d.ptr, pt.x.ptr, h->mat, max_strain,
                  pt.active.ptr, pt.stress.ptr, pt.partials.ptr, tix(pt, 4), pt.red.ptr + 5,
                  dm ? pt.elem_own.ptr : nullptr, pt.fail_list.ptr, dm ? pt.fail_cnt.ptr : fail_counter(pt));
  }
  HIPC(hipGetLastError());
  Part& p0 = part0(h);
  if (dm) {  // (force, #active) of every partition, summed in rank order
    RC(gather4(h, 4));
    launch_rank_sum(s, p0.gred, nranks(h), p0.red.ptr + 12);
    HIPC(hipMemcpyAsync(h->h_red, p0.red.ptr + 12, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
  } else {
    HIPC(hipMemcpyAsync(h->h_red, p0.red.ptr + 4, 3 * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  return 0;
}

// Speculative post (mfea_handle::spec_on), enqueued behind the solve's
// planned batch: the solve's end event, then the post.  At any later batch
// end the solve went on: that post's failures are undone and post runs after
// the solve's wait as usual
int spec_post(mfea_handle* h) {
  if (!h->spec_on) return 0;
  // a later batch end (the planned batch was not the last: SOR / ICC chunks,
  // a first solve): undo, and let post run after the solve as usual
  if (h->spec_used) return spec_undo(h);
  h->spec_used = true;
  RC(phase_event(h, h->ev[3], h->stream));
  RC(enqueue_post(h, h->spec_strain));
  h->spec_launched = true;
  return 0;
}
// the solve did not end with that batch's state: undo its post's failures
int spec_undo(mfea_handle* h) {
  if (!h->spec_launched) return 0;
  Part& pt = part0(h);
  launch_unfail(h->stream, pt.fail_list.ptr, fail_counter(pt), pt.active.ptr);
  HIPC(hipGetLastError());
  h->spec_launched = false;
  return 0;
}

int post_impl(mfea_handle* h, double max_strain, double* total_force, int64_t* n_active,
              mfea_stats* st) {
  const bool dm = partitioned(h);
  if (!h->spec_launched) RC(enqueue_post(h, max_strain));
  h->spec_launched = false;
  Part& p0 = part0(h);
  RC(wait_event(h, h->ev[5]));
  if (!dm && p0.P.n_top == 0) h->h_red[0] = 0.0;
  if (!dm && p0.P.n_elems == 0) h->h_red[1] = 0.0;
  if (total_force) *total_force = h->h_red[0];
  unsigned nfail = 0;  // one partition: the stress kernel's failed-element count
  if (!dm) std::memcpy(&nfail, &h->h_red[2], sizeof nfail);
  // elements only ever fail here
  const bool changed = (int64_t)h->h_red[1] != h->n_active || nfail > 0;
  if (changed) {
    // every rank sees the same global count, so every rank exchanges
    if (dm && h->gkey_gen == h->act_gen) {
      RC(apply_failures(h));
      h->gkey_gen = h->act_gen + 1;
    }
    ++h->act_gen;
  }
  if ((int64_t)h->h_red[1] < h->Ecount) h->act_all = false;
  h->n_active = (int64_t)h->h_red[1];
  if (n_active) *n_active = h->n_active;
  if (!dm && nfail) RC(local_failures(h, p0, nfail));
  else if (!dm && h->act_host_ok && h->n_active != h->act_count) h->act_host_ok = false;
  if (st && h->opt_phase_times) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[4], h->ev[5]);
    st->t_post_ms = ms;
  }
  return 0;
}

// Partitioned GAMG: option "amg_dist" 1 the distributed V-cycle of the
// global hierarchy, 0 block Jacobi over per-partition hierarchies, -1 (the
// default) whichever solved faster: per active set the first solve runs the
// global hierarchy, the second block Jacobi (plan builds and uploads outside
// the clock), later ones the faster of the two.  The block-Jacobi form wins
// where the partition boundaries cut weak couplings (strips between tiles:
// the same iteration count with two exchanges per iteration instead of
// 4·levels + 2); the global form wherever the cut couplings matter (the
// grown networks: 17 iterations instead of 190-310).  A variant that fails
// (max_it, breakdown) hands the step to the other.
// RCCL world: *t ← the maximum of *t over the ranks (collective)
int max_over_ranks(mfea_handle* h, double* t) {
  HIPC(h->gtime.alloc(1));
  HIPC(hipMemcpyAsync(h->gtime.ptr, t, sizeof(double), hipMemcpyHostToDevice, h->stream));
  NCCLC(ncclAllReduce(h->gtime.ptr, h->gtime.ptr, 1, ncclFloat64, ncclMax, h->comm, h->stream));
  HIPC(hipMemcpyAsync(t, h->gtime.ptr, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  return sync_stream(h);
}

int solve_amg_part(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o, mfea_stats* st) {
  auto run = [&](int mode) {
    return mode ? solve_gamg_global(h, dy_top, dy_bot, o, st) : solve_amg_dist(h, dy_top, dy_bot, o, st);
  };
  if (h->opt_amg_dist >= 0) return run(h->opt_amg_dist);
  auto& a = h->amg_auto;
  bool rebuilt = false;
  RC(ensure_gamg_plan(h, &rebuilt));  // the active set's identity (a content compare)
  if (a.gen != h->gamg_plan_gen) {
    a.gen = h->gamg_plan_gen;
    a.choice = -1;
    a.t[0] = a.t[1] = -1.0;
  }
  if (a.choice >= 0) return run(a.choice);
  const int mode = amg_auto_pending(a.t);
  if (mode) {
    RC(ensure_gamg(h, &rebuilt));
  } else {
    for (auto& pp : h->parts) {
      bool rb = false;
      RC(ensure_amg(h, *pp, &rb));
      rebuilt = rebuilt || rb;
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  int rc = run(mode);
  if (rc == 0) rc = sync_stream(h);
  a.t[mode] = rc == 0 ? std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() : 1e300;
  // RCCL: every rank must pick the same form (the two issue different
  // exchanges), so each compares the slowest rank's times, not its own
  if (h->world > 1) RC(max_over_ranks(h, &a.t[mode]));
  if (amg_auto_pending(a.t) < 0) a.choice = amg_auto_choice(a.t);
  if (rc == MFEA_EMAXIT || rc == MFEA_EBREAKDOWN) {
    a.choice = 1 - mode;
    rc = run(a.choice);
  }
  if (st && rebuilt) st->amg_rebuilt = 1;
  return rc;
}

int solve_any(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
              mfea_stats* st) {
  h->ev_setup_used = false;
  if (o->precond == MFEA_PC_GAMG) {
    if (!partitioned(h)) return solve_amg(h, dy_top, dy_bot, o, st);
    return solve_amg_part(h, dy_top, dy_bot, o, st);
  }
  if (o->precond == MFEA_PC_SOR || o->precond == MFEA_PC_ICC) {
    if (partitioned(h)) return fail(MFEA_EINVAL, "MFEA_PC_SOR / MFEA_PC_ICC: one partition per handle");
    return solve_amg(h, dy_top, dy_bot, o, st);
  }
  if (o->precond != MFEA_PC_JACOBI && o->precond != MFEA_PC_BLOCK_JACOBI)
    return fail(MFEA_EINVAL, "unknown preconditioner");
  return partitioned(h) ? solve_dist(h, dy_top, dy_bot, o, st) : solve_impl(h, dy_top, dy_bot, o, st);
}

// current element activity in original order (elements no partition of this
// process holds stay 1)
int gather_active(mfea_handle* h, std::vector<uint8_t>& out) {
  out.assign(h->Ecount, 1);
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int64_t E = pt.P.n_elems;
    std::vector<uint8_t> a(E);
    if (E) HIPC(hmemcpy(h, a.data(), pt.active.ptr, E, hipMemcpyDeviceToHost));
    if (!partitioned(h)) {
      out = a;
      return 0;
    }
    for (int64_t le = 0; le < E; ++le) out[pt.plan.elem_g[le]] = a[le];
  }
  return 0;
}

}  // namespace

extern "C" {

int mfea_abi_version(void) { return MFEA_ABI_VERSION; }

int mfea_last_error(char* buf, size_t n) {
  if (!buf || n == 0) return MFEA_EINVAL;
  std::snprintf(buf, n, "%s", g_err.c_str());
  return 0;
}

int mfea_create(int device, mfea_handle** out) {
  if (!out) return fail(MFEA_EINVAL, "out is NULL");
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) return fail(MFEA_EDEVICE, "no HIP device available");
  if (device < 0 || device >= count) return fail(MFEA_EINVAL, "device index out of range");
  auto* h = new mfea_handle();
  h->device = device;
  HIPC(hipSetDevice(device));
  HIPC(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  for (auto& ev : h->ev) HIPC(hipEventCreate(&ev));
  HIPC(hipEventCreate(&h->ev_setup));
  for (auto& ev : h->poll) HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPC(hipHostMalloc(&h->h_state, 2 * sizeof(SolveState),
                     hipHostMallocMapped | hipHostMallocCoherent));
  HIPC(hipHostGetDevicePointer((void**)&h->d_host_state, h->h_state, 0));
  HIPC(hipHostMalloc(&h->h_red, 16 * sizeof(double), hipHostMallocDefault));
  std::memset(h->h_state, 0, 2 * sizeof(SolveState));
  h->parts.push_back(std::make_unique<Part>());  // scratch of mfea_solve_csr until a mesh is set
  h->parts[0]->mirror = h->d_host_state;
  // reference constants src/fea_solver.py:14-20
  const double d = 0.0002, t = 0.000001;
  const double A = 3.14 * (std::pow(d / 2, 2) - std::pow(d / 2 - t, 2));
  mfea_set_material(h, 2500.0, A, A * 0.001);
  *out = h;
  return 0;
}

int mfea_destroy(mfea_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  destroy_graph(h);
  if (h->graph_setup) (void)hipGraphExecDestroy(h->graph_setup);
  for (auto& g : h->graph_combo)
    if (g) (void)hipGraphExecDestroy(g);
  h->parts.clear();
  if (h->comm) (void)ncclCommDestroy(h->comm);
  for (auto& ev : h->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : h->poll)
    if (ev) (void)hipEventDestroy(ev);
  if (h->ev_setup) (void)hipEventDestroy(h->ev_setup);
  if (h->h_state) (void)hipHostFree(h->h_state);
  if (h->h_red) (void)hipHostFree(h->h_red);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

int mfea_set_material(mfea_handle* h, double E, double A, double I) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  h->E = E;
  h->A = A;
  h->I = I;
  h->mat.EA = E * A;             // src/fea_solver.py:45  (E * A) / L_safe
  h->mat.EI12 = (12.0 * E) * I;  // src/fea_solver.py:58  12 * E * I / L³
  h->mat.E = E;
  return 0;
}

int mfea_set_mesh(mfea_handle* h, int64_t n_nodes, const double* xyz, int64_t n_elems,
                  const int64_t* e2n, uint32_t flags) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (n_nodes < 0 || n_elems < 0) return fail(MFEA_EINVAL, "negative size");
  if ((n_nodes && !xyz) || (n_elems && !e2n)) return fail(MFEA_EINVAL, "NULL mesh array");
  RC(set_device(h));
  h->N = n_nodes;
  h->Ecount = n_elems;
  h->xyz.assign(xyz, xyz + 3 * n_nodes);
  h->e2n.assign(e2n, e2n + 2 * n_elems);
  h->mesh_flags = flags;
  h->has_mesh = true;
  h->dirty = true;
  h->act_all = false;
  h->active_host.clear();
  h->planar = true;
  for (int64_t n = 0; n < n_nodes; ++n)
    if (xyz[3 * n + 2] != 0.0) h->planar = false;
  // validate now so errors surface at the call that caused them
  Pattern tmp;
  std::string err = build_pattern(h->N, h->xyz.data(), h->Ecount, h->e2n.data(),
                                  (flags & MFEA_MESH_SKIP_INVALID) != 0, {}, {}, 0, tmp);
  if (!err.empty()) {
    h->has_mesh = false;
    return fail(MFEA_EINVAL, err);
  }
  return 0;
}

int mfea_set_bc(mfea_handle* h, int64_t n_top, const int64_t* top, int64_t n_bot,
                const int64_t* bot) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (!h->has_mesh) return fail(MFEA_ESTATE, "set the mesh before the boundary conditions");
  if (n_top < 0 || n_bot < 0 || (n_top && !top) || (n_bot && !bot))
    return fail(MFEA_EINVAL, "bad grip node arrays");
  for (int64_t i = 0; i < n_top; ++i)
    if (top[i] < 0 || top[i] >= h->N) return fail(MFEA_EINVAL, "top grip node out of range");
  for (int64_t i = 0; i < n_bot; ++i)
    if (bot[i] < 0 || bot[i] >= h->N) return fail(MFEA_EINVAL, "bottom grip node out of range");
  // keep the current activity across the rebuild
  if (!h->dirty && h->Ecount) RC(gather_active(h, h->active_host));
  h->top.assign(top, top + n_top);
  h->bot.assign(bot, bot + n_bot);
  h->dirty = true;
  return 0;
}

int mfea_set_active(mfea_handle* h, const uint8_t* active) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  // all active already (the benchmark resets every step): nothing changes —
  // no act_gen bump, so a partitioned handle skips its activity all-reduce
  if (!active && h->act_all) return 0;
  ++h->act_gen;
  ++h->act_sub_gen;
  h->act_all = !active;
  if (partitioned(h)) {  // the global activity is known here: no exchange needed for it
    h->gkey.assign(h->Ecount, 1);
    if (active)
      for (int64_t e = 0; e < h->Ecount; ++e) h->gkey[e] = active[e] ? 1 : 0;
    h->gkey_gen = h->act_gen;
  }
  if (h->Ecount == 0) return 0;
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int64_t E = pt.P.n_elems;
    if (!E) continue;
    if (active) {
      std::vector<uint8_t> a(E);
      for (int64_t le = 0; le < E; ++le)
        a[le] = active[partitioned(h) ? pt.plan.elem_g[le] : le] ? 1 : 0;
      HIPC(hmemcpy(h, pt.active.ptr, a.data(), E, hipMemcpyHostToDevice));
      if (!partitioned(h)) h->act_host = std::move(a);
    } else {
      HIPC(hmemset(h, pt.active.ptr, 1, E));
      if (!partitioned(h)) h->act_host.assign(E, 1);
    }
  }
  if (!partitioned(h)) {
    h->act_count = (int64_t)std::count(h->act_host.begin(), h->act_host.end(), (uint8_t)1);
    h->act_host_ok = true;
  }
  return 0;
}

int mfea_assemble(mfea_handle* h) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  RC(assemble_impl(h, nullptr));
  return sync_stream(h);
}

int mfea_solve(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
               mfea_stats* st) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  mfea_solve_opts o = opts ? *opts : default_opts();
  if (st) std::memset(st, 0, sizeof(*st));
  // a (re)build (new mesh / BCs, a layout option) left the operator empty:
  // assemble the current active set first rather than solve a zero operator
  if (!h->assembled) RC(assemble_impl(h, nullptr));
  return solve_any(h, dy_top, dy_bot, &o, st);
}

int mfea_post(mfea_handle* h, double max_strain, double* total_force, int64_t* n_active) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  return post_impl(h, max_strain, total_force, n_active, nullptr);
}

int mfea_step(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
              double max_strain, double* total_force, int64_t* n_active, mfea_stats* st) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  mfea_solve_opts o = opts ? *opts : default_opts();
  if (st) std::memset(st, 0, sizeof(*st));
  // the one-partition GAMG / SOR / ICC solves take their RHS from the
  // assembly's row pass (AsmRhs)
  const bool fuse_rhs = !partitioned(h) && (o.precond == MFEA_PC_GAMG || o.precond == MFEA_PC_SOR ||
                                            o.precond == MFEA_PC_ICC);
  const double dys[2] = {dy_top, dy_bot};
  // one partition, GAMG / SOR / ICC, graphs on, no phase events, the row
  // gather: the assembly rides at the head of the solve's setup graph
  const bool defer = fuse_rhs && h->opt_step_graph && h->opt_graph && !h->opt_phase_times && h->opt_asm_kernel == 0;
  if (defer) {
    h->h_red[14] = dy_top;
    h->h_red[15] = dy_bot;
    h->asm_pending = true;
    h->assembled = true;
    h->rhs_fused = false;
  } else {
    RC(assemble_impl(h, nullptr, fuse_rhs ? dys : nullptr));
  }
  // a solver failure stops the step loop here, as the reference does
  // (src/fea_petsc.cpp:346-354)
  h->in_step = true;
  h->spec_on = fuse_rhs && h->opt_spec_post;
  h->spec_strain = max_strain;
  h->spec_launched = false;
  h->spec_used = false;
  int rc = solve_any(h, dy_top, dy_bot, &o, st);
  h->spec_on = false;
  h->rhs_fused = false;
  if (h->asm_pending) {  // (the solve ended before its assembly: never on success)
    h->asm_pending = false;
    if (rc == 0) rc = assemble_impl(h, nullptr);
    else h->assembled = false;
  }
  if (rc) (void)spec_undo(h);
  if (rc == 0) rc = post_impl(h, max_strain, total_force, n_active, st);
  h->in_step = false;
  if (rc) {
    (void)sync_stream(h);
    return rc;
  }
  if (st && h->opt_phase_times) {  // every event of the step has completed (post waited)
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    st->t_assemble_ms = ms;
    solve_times(h, st);
  }
  return 0;
}

int mfea_get_displacement(mfea_handle* h, double* U) {
  if (!h || !U) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  const bool dm = partitioned(h);
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Pattern& P = pt.P;
    const int64_t N = P.n_nodes;
    std::vector<double> xp(3 * N);
    if (N) HIPC(hmemcpy(h, xp.data(), pt.x.ptr, 3 * N * sizeof(double), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < N; ++i) {
      const int64_t ln = P.perm[i];
      if (dm && pt.plan.ghost[ln]) continue;
      const int64_t g = dm ? pt.plan.node_g[ln] : ln;
      for (int a = 0; a < 3; ++a) U[3 * g + a] = xp[3 * i + a];
    }
  }
  return 0;
}

int mfea_get_stress(mfea_handle* h, double* stress) {
  if (!h || !stress) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int64_t E = pt.P.n_elems;
    if (!E) continue;
    if (!partitioned(h)) {
      HIPC(hmemcpy(h, stress, pt.stress.ptr, E * sizeof(double), hipMemcpyDeviceToHost));
      continue;
    }
    std::vector<double> sl(E);
    HIPC(hmemcpy(h, sl.data(), pt.stress.ptr, E * sizeof(double), hipMemcpyDeviceToHost));
    for (int64_t le = 0; le < E; ++le)
      if (pt.plan.elem_own[le]) stress[pt.plan.elem_g[le]] = sl[le];
  }
  return 0;
}

int mfea_get_active(mfea_handle* h, uint8_t* active) {
  if (!h || !active) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const int64_t E = pt.P.n_elems;
    if (!E) continue;
    if (!partitioned(h)) {
      HIPC(hmemcpy(h, active, pt.active.ptr, E, hipMemcpyDeviceToHost));
      continue;
    }
    std::vector<uint8_t> al(E);
    HIPC(hmemcpy(h, al.data(), pt.active.ptr, E, hipMemcpyDeviceToHost));
    for (int64_t le = 0; le < E; ++le)
      if (pt.plan.elem_own[le]) active[pt.plan.elem_g[le]] = al[le];
  }
  return 0;
}

int mfea_element_stiffness(mfea_handle* h, int64_t n, const double* p1s, const double* p2s,
                           double E, double A, double I, double* Ke, double* L) {
  if (!h || n < 0 || (n && (!p1s || !p2s || !Ke || !L))) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  if (n == 0) return 0;
  Material m;
  m.EA = E * A;
  m.EI12 = (12.0 * E) * I;
  m.E = E;
  DevBuf<double> a, b, k, l;
  HIPC(a.alloc(3 * n));
  HIPC(b.alloc(3 * n));
  HIPC(k.alloc(36 * n));
  HIPC(l.alloc(n));
  HIPC(hipMemcpyAsync(a.ptr, p1s, 3 * n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPC(hipMemcpyAsync(b.ptr, p2s, 3 * n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  launch_element_stiffness(h->stream, n, a.ptr, b.ptr, m, k.ptr, l.ptr);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(Ke, k.ptr, 36 * n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPC(hipMemcpyAsync(L, l.ptr, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  HIPC(hipStreamSynchronize(h->stream));
  return 0;
}

int mfea_export_csr(mfea_handle* h, int64_t* nnz, int64_t* indptr, int32_t* indices,
                    double* data) {
  if (!h || !nnz) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  if (partitioned(h)) return fail(MFEA_ESTATE, "mfea_export_csr: single-partition handles only");
  Part& pt = part0(h);
  const Pattern& P = pt.P;
  const int64_t N = P.n_nodes, E = P.n_elems;
  std::vector<double> diag6(6 * N), val6(6 * pt.G);
  std::vector<uint8_t> act(E);
  if (N) HIPC(hmemcpy(h, diag6.data(), pt.diag.ptr, 6 * N * sizeof(double), hipMemcpyDeviceToHost));
  if (pt.G) HIPC(hmemcpy(h, val6.data(), pt.val.ptr, 6 * pt.G * sizeof(double), hipMemcpyDeviceToHost));
  if (E) HIPC(hmemcpy(h, act.data(), pt.active.ptr, E, hipMemcpyDeviceToHost));
  std::vector<int64_t> ip;
  std::vector<int32_t> ix;
  std::vector<double> dv;
  export_csr(P, act, diag6, val6, ip, ix, dv);
  if (!indptr) {
    *nnz = (int64_t)ix.size();
    return 0;
  }
  if (*nnz < (int64_t)ix.size()) return fail(MFEA_EINVAL, "output arrays too small");
  *nnz = (int64_t)ix.size();
  std::memcpy(indptr, ip.data(), ip.size() * sizeof(int64_t));
  std::memcpy(indices, ix.data(), ix.size() * sizeof(int32_t));
  std::memcpy(data, dv.data(), dv.size() * sizeof(double));
  return 0;
}

int mfea_solve_csr(mfea_handle* h, int64_t n, const int64_t* indptr, const int32_t* indices,
                   const double* data, int64_t n_known, const int64_t* known_dofs,
                   const double* known_vals, const mfea_solve_opts* opts, double* U,
                   mfea_stats* st) {
  if (!h || n < 0 || (n && (!indptr || !U)) || n_known < 0 || (n_known && (!known_dofs || !known_vals)))
    return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  if (h->world > 1) return fail(MFEA_ESTATE, "mfea_solve_csr: not on a partitioned (RCCL) handle");
  mfea_solve_opts o = opts ? *opts : default_opts();
  if (o.precond != MFEA_PC_JACOBI) return fail(MFEA_EINVAL, "CSR path supports Jacobi only");
  if (st) std::memset(st, 0, sizeof(*st));
  if (n == 0) return 0;
  const int64_t nnz = indptr[n];
  for (int64_t t = 0; t < nnz; ++t)
    if (indices[t] < 0 || indices[t] >= n) return fail(MFEA_EINVAL, "column index out of range");
  std::vector<uint8_t> known(n, 0);
  std::vector<double> kval(n, 0.0);
  for (int64_t i = 0; i < n_known; ++i) {
    const int64_t k = known_dofs[i];
    if (k < 0 || k >= n) return fail(MFEA_EINVAL, "known dof out of range");
    known[k] = 1;
    kval[k] = known_vals[i];
  }
  hipStream_t s = h->stream;
  Part& pt = part0(h);  // its reduction scratch, slots and state
  HIPC(h->c_indptr.alloc(n + 1));
  HIPC(h->c_indices.alloc(nnz));
  HIPC(h->c_data.alloc(nnz));
  HIPC(h->c_known.alloc(n));
  HIPC(h->c_kval.alloc(n));
  HIPC(h->c_x.alloc(n));
  HIPC(h->c_r.alloc(n));
  HIPC(h->c_p.alloc(n));
  HIPC(h->c_q.alloc(n));
  HIPC(h->c_dinv.alloc(n));
  const int64_t maxg = std::max<int64_t>(grid_rows(n), 2048);
  if (pt.partials.n < (size_t)(4 * maxg)) HIPC(pt.partials.alloc(4 * (maxg + 16)));
  if (!pt.red.ptr) {
    HIPC(pt.red.alloc(16));
    HIPC(hipMemsetAsync(pt.red.ptr, 0, 16 * sizeof(double), s));
  }
  if (!pt.tickets.ptr) {
    HIPC(pt.tickets.alloc(kTicketSets * kTicketStride));
    HIPC(hipMemsetAsync(pt.tickets.ptr, 0, kTicketSets * kTicketStride * sizeof(unsigned), s));
  }
  HIPC(pt.slots.alloc(kMaxChunk + 2));
  HIPC(pt.state.alloc(1));
  HIPC(hipMemcpyAsync(h->c_indptr.ptr, indptr, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (nnz) {
    HIPC(hipMemcpyAsync(h->c_indices.ptr, indices, nnz * sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(h->c_data.ptr, data, nnz * sizeof(double), hipMemcpyHostToDevice, s));
  }
  HIPC(hipMemcpyAsync(h->c_known.ptr, known.data(), n, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(h->c_kval.ptr, kval.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
  HIPC(hipMemsetAsync(h->c_q.ptr, 0, n * sizeof(double), s));
  HIPC(hipEventRecord(h->ev[1], s));
  launch_csr_rhs_init(s, n, h->c_indptr.ptr, h->c_indices.ptr, h->c_data.ptr, h->c_known.ptr,
                      h->c_kval.ptr, o.reg, h->c_x.ptr, h->c_r.ptr, h->c_p.ptr, h->c_dinv.ptr,
                      pt.partials.ptr, tix(pt, 5), pt.red.ptr);
  launch_init_finalize(s, pt.red.ptr, o.rtol, o.atol, o.norm, o.max_it, o.reg, pt.slots.ptr,
                       pt.state.ptr);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(h->ev[2], s));
  const int chunk = o.chunk > 0 ? std::min(o.chunk, kMaxChunk) : 32;
  SolveState fin;
  int rc = drive_chunks(
      h, chunk, o.max_it,
      [&]() -> int {
        for (int j = 0; j < chunk; ++j) {
          launch_spmv_csr(s, j, n, h->c_indptr.ptr, h->c_indices.ptr, h->c_data.ptr,
                          h->c_known.ptr, o.reg, h->c_p.ptr, h->c_q.ptr, pt.slots.ptr,
                          pt.state.ptr, pt.partials.ptr, tix(pt, 6));
          launch_update(s, j, n, 0, h->c_x.ptr, h->c_r.ptr, h->c_p.ptr, h->c_q.ptr, h->c_dinv.ptr,
                        pt.slots.ptr, pt.state.ptr, pt.partials.ptr, tix(pt, 7));
          launch_direction(s, j, n, 0, h->c_r.ptr, h->c_p.ptr, h->c_dinv.ptr, pt.slots.ptr,
                           pt.state.ptr);
        }
        launch_advance(s, chunk, pt.slots.ptr, pt.state.ptr);
        HIPC(hipGetLastError());
        return 0;
      },
      &fin);
  if (rc) return rc;
  HIPC(hipEventRecord(h->ev[3], s));
  HIPC(hipMemcpyAsync(U, h->c_x.ptr, n * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (st) {
    st->iters = fin.iters;
    st->status = fin.status;
    st->bnorm = std::sqrt(fin.bb0);
    st->relres = fin.res0 > 0 ? std::sqrt(fin.res_final / fin.res0) : 0.0;
    st->n_free = n - (int64_t)std::count(known.begin(), known.end(), 1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
    st->t_solve_ms = ms;
  }
  if (fin.status == -4) return fail(MFEA_EMAXIT, "PCG reached max_it without converging");
  if (fin.status == -5) return fail(MFEA_EBREAKDOWN, "PCG breakdown");
  return 0;
}

int mfea_get_info(mfea_handle* h, mfea_info* info) {
  if (!h || !info) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  Part& pt = part0(h);
  const Pattern& P = pt.P;
  std::memset(info, 0, sizeof(*info));
  info->n_nodes = P.n_nodes;
  info->n_elems = P.n_elems;
  info->n_free_nodes = P.n_free;
  info->n_top = P.n_top;
  info->n_known = P.n_known;
  info->n_slices = P.n_slices();
  info->n_slots = pt.G;
  int64_t inc = 0;
  for (int64_t i = 0; i < P.n_free; ++i) inc += P.row_len[i];
  info->free_incidences = inc;
  info->planar = h->planar ? 1 : 0;
  info->cg_lanes = use_ell(h, pt) ? 1 : 0;
  info->n_lanes = pt.ell_ok ? pt.L.n_lanes : 0;
  int64_t halo = 0;
  if (pt.ell_ok)
    for (int32_t p : pt.L.partner) halo += p != -1;
  info->n_halo = halo;
  info->n_parts = nranks(h);
  info->part = pt.rank;
  info->n_pairs = pt.plan.n_pairs;
  info->n_ghost = P.n_ghost;
  if (pt.ell_ok) {
    info->halo_compact = pt.ell_hc ? 1 : 0;
    info->block_size = ell_block_size(ell_op(h, pt));
    info->grid = ell_grid_size(ell_op(h, pt));
  }
  return 0;
}

// iteration 0 of the active CG kernel of partition 0 (profiling / tracing;
// partitioned handles: the per-GPU kernel without its exchange)
static void launch_iter0(mfea_handle* h, int pc, unsigned long long* trace) {
  Part& pt = part0(h);
  if (use_ell(h, pt))
    launch_ell_iter(h->stream, 0, ell_op(h, pt), pc, ell_vecs(pt), pt.slots.ptr, pt.state.ptr,
                    pt.cg_part.ptr, trace);
  else
    launch_cg_iter(h->stream, 0, sell_op(pt), pc, cg_vecs(pt), pt.slots.ptr, pt.state.ptr,
                   pt.cg_part.ptr, trace);
}

int mfea_profile_spmv(mfea_handle* h, int reps, double* avg_ms) {
  if (!h || !avg_ms || reps <= 0) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  RC(ensure_built(h));
  // partitioned: partition 0's w kernel over its own rows (the plan its device
  // arrays hold: its block-Jacobi hierarchy or its share of the global one)
  Part& pt = part0(h);
  if (!(partitioned(h) ? pt.dev_plan >= 0 : pt.amg_ok)) return fail(MFEA_ESTATE, "profile the SpMV after a GAMG solve");
  hipStream_t s = h->stream;
  const int nd = pt.dev_plan == 1 ? h->gamg.nd : pt.amg.nd;
  hipGraph_t g;
  hipGraphExec_t ge = nullptr;
  HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < reps; ++k) launch_amg_cg_w(s, nd, 0, true, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
  HIPC(hipStreamEndCapture(s, &g));
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  HIPC(e);
  e = hipGraphLaunch(ge, s);  // warm
  if (e == hipSuccess) e = hipEventRecord(h->ev[0], s);
  if (e == hipSuccess) e = hipGraphLaunch(ge, s);
  if (e == hipSuccess) e = hipEventRecord(h->ev[1], s);
  if (e == hipSuccess) e = hipEventSynchronize(h->ev[1]);
  float ms = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
  (void)hipGraphExecDestroy(ge);
  HIPC(e);
  *avg_ms = ms / reps;
  return 0;
}

int mfea_profile_iteration(mfea_handle* h, int precond, int reps, double* avg_ms) {
  if (!h || !avg_ms || reps <= 0) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  RC(ensure_built(h));
  Part& pt = part0(h);
  hipStream_t s = h->stream;
  if (precond == MFEA_PC_GAMG || precond == MFEA_PC_SOR || precond == MFEA_PC_ICC) {
    if (!pt.amg_ok || pt.amg_kind != precond)
      return fail(MFEA_ESTATE, "profile GAMG / SOR / ICC after a solve with that preconditioner");
    // Running state: slots[0] = INIT and real partials from an ungated first
    // w kernel; every rep is update + V-cycle + w(first) — the full work of
    // one PCG iteration, all stores included.
    const int nd = pt.amg.nd;
    launch_amg_cg_w(s, nd, 0, true, pt.amg_lev[0], pt.amg_cg, pt.slots.ptr, pt.cg_part.ptr);
    launch_cg_init_finalize(s, pt.red.ptr + 8, 0.0, 0.0, 0, 1 << 30, 1e-12, pt.state.ptr);
    // the reps iterations replay as one captured graph, as in the solve
    // (eager launches of ≈ 20 short kernels per iteration are host-bound)
    hipGraph_t g;
    hipGraphExec_t ge = nullptr;
    HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < reps; ++k) enqueue_amg_iteration(h, pt, 0, true);
    HIPC(hipStreamEndCapture(s, &g));
    hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPC(e);
    e = hipGraphLaunch(ge, s);  // warm
    if (e == hipSuccess) e = hipEventRecord(h->ev[0], s);
    if (e == hipSuccess) e = hipGraphLaunch(ge, s);
    if (e == hipSuccess) e = hipEventRecord(h->ev[1], s);
    if (e == hipSuccess) e = hipEventSynchronize(h->ev[1]);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    (void)hipGraphExecDestroy(ge);
    HIPC(e);
    *avg_ms = ms / reps;
    return 0;
  }
  const int pc = precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0;
  // Running state with tol 0: slots[0] = INIT and parity-0 partials of 1, so
  // γ = δ = ‖r‖² = ‖u‖² = G > 0, α = 1, β = 0.  Every launch is iteration 0
  // (same parity), so it reads the same buffers and does identical work
  // (including all stores); only x and p drift.
  const double ones[2] = {1.0, 1.0};
  HIPC(hipMemcpyAsync(pt.red.ptr + 8, ones, sizeof(ones), hipMemcpyHostToDevice, s));
  launch_cg_init_finalize(s, pt.red.ptr + 8, 0.0, 0.0, 0, 1 << 30, 1e-12, pt.state.ptr);
  std::vector<double> pones(4 * kCgMaxPartials, 1.0);
  HIPC(hipMemcpyAsync(pt.cg_part.ptr, pones.data(), pones.size() * sizeof(double),
                      hipMemcpyHostToDevice, s));
  Slot s0;
  std::memset(&s0, 0, sizeof(s0));
  s0.flag = kInit;
  HIPC(hipMemcpyAsync(pt.slots.ptr, &s0, sizeof(s0), hipMemcpyHostToDevice, s));
  launch_iter0(h, pc, nullptr);  // warm
  HIPC(hipEventRecord(h->ev[0], s));
  for (int k = 0; k < reps; ++k) launch_iter0(h, pc, nullptr);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(h->ev[1], s));
  HIPC(hipEventSynchronize(h->ev[1]));
  float ms = 0;
  HIPC(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
  *avg_ms = ms / reps;
  return 0;
}

int mfea_debug_trace_iteration(mfea_handle* h, int precond, uint64_t* out, int64_t cap,
                               int64_t* n_waves) {
  if (!h || !out || !n_waves || cap < 0) return fail(MFEA_EINVAL, "bad argument");
  double ms = 0;
  RC(mfea_profile_iteration(h, precond, 20, &ms));  // same running state
  hipStream_t s = h->stream;
  Part& pt = part0(h);
  const bool ell = use_ell(h, pt);
  const int64_t g = ell ? ell_grid_size(ell_op(h, pt)) : cg_grid(pt.P.n_free);
  const int64_t nw = g * ((ell ? ell_block_size(ell_op(h, pt)) : cg_block_size(0)) / 64);
  if (cap < nw * 4) return fail(MFEA_EINVAL, "trace buffer too small");
  unsigned long long* d = nullptr;
  HIPC(hipMalloc(&d, nw * 4 * sizeof(unsigned long long)));
  HIPC(hipMemsetAsync(d, 0, nw * 4 * sizeof(unsigned long long), s));
  launch_iter0(h, precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0, d);
  hipError_t e = hipMemcpyAsync(out, d, nw * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(MFEA_EDEVICE, hipGetErrorString(e));
  *n_waves = nw;
  return 0;
}

int mfea_debug_amg_info(mfea_handle* h, int* n_levels, int64_t* rows, int64_t* blocks,
                        int64_t* pblocks, int cap, int64_t* pair_items, int* nd, int* n_dist,
                        int64_t* ptblocks) {
  if (!h || !n_levels || cap < 0 || (cap && (!rows || !blocks || !pblocks)))
    return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  RC(ensure_built(h));
  bool rebuilt = false;
  if (partitioned(h) && !h->opt_amg_dist) return fail(MFEA_ESTATE, "GAMG block Jacobi: per-partition hierarchies");
  if (partitioned(h)) RC(ensure_gamg(h, &rebuilt));
  else RC(ensure_amg(h, part0(h), &rebuilt));
  const AmgPlan& pl = partitioned(h) ? h->gamg : part0(h).amg;
  if (n_dist) *n_dist = pl.n_dist;
  *n_levels = (int)pl.lev.size();
  for (int l = 0; l < std::min(cap, *n_levels); ++l) {
    const SellPat& A = pl.lev[l].A;
    rows[l] = A.n;
    int64_t nb = 0;
    for (int64_t i = 0; i < A.n; ++i) nb += A.rlen[i];
    blocks[l] = nb;
    int64_t pb = 0;
    for (int32_t r : pl.lev[l].P.rlen) pb += r;
    pblocks[l] = pb;
    if (ptblocks) {
      int64_t tb = 0;
      for (int32_t r : pl.lev[l].PT.rlen) tb += r;
      ptblocks[l] = tb;
    }
  }
  if (pair_items) *pair_items = pl.pair_items;
  if (nd) *nd = pl.nd;
  return 0;
}

int mfea_set_option(mfea_handle* h, const char* name, int64_t value) {
  if (!h || !name) return fail(MFEA_EINVAL, "NULL argument");
  const std::string n(name);
  bool rebuild = false;  // options baked into the symbolic layout
  if (n == "graph") h->opt_graph = value != 0;
  else if (n == "phase_times") h->opt_phase_times = value != 0;
  else if (n == "dist_graph") h->opt_dist_graph = value != 0;
  else if (n == "order") { h->opt_order = (int)value; rebuild = true; }
  else if (n == "lane_dof") { h->opt_lane_dof = (int)value; rebuild = true; }
  else if (n == "cg_kernel") {
    if (value < 0 || value > 2) return fail(MFEA_EINVAL, "cg_kernel: 0 auto, 1 lanes, 2 sell");
    h->opt_cg_kernel = (int)value;
  } else if (n == "ell_block") {
    if (value != 64 && value != 128 && value != 256 && value != 512)
      return fail(MFEA_EINVAL, "ell_block: 64, 128, 256 or 512");
    h->opt_ell_block = (int)value;
  } else if (n == "ell_maxg") h->opt_ell_maxg = value;
  else if (n == "ell_compact") { h->opt_ell_compact = value != 0; rebuild = true; }
  else if (n == "amg_tail_rows") { h->opt_amg_tail_rows = value; rebuild = true; }
  else if (n == "amg_max_levels") {
    if (value < 1 || value > kAmgMaxLevels) return fail(MFEA_EINVAL, "amg_max_levels: 1..32");
    h->opt_amg_max_levels = (int)value;
    rebuild = true;
  }
  else if (n == "amg_restrict_lanes") {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
      return fail(MFEA_EINVAL, "amg_restrict_lanes: 0 (by width), 1, 2, 4, 8 or 16 (16: the compact down sweep)");
    h->opt_amg_rlanes = (int)value;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.rlanes = (int)value;
  }
  else if (n == "amg_v_lanes") {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
      return fail(MFEA_EINVAL, "amg_v_lanes: 0 (by width), 1, 2, 4, 8 or 16");
    h->opt_amg_v_lanes = (int)value;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.vlanes = (int)value;
  }
  else if (n == "amg_small_lanes") {
    if (value < 0 || value > (int64_t(1) << 30)) return fail(MFEA_EINVAL, "amg_small_lanes: 0 .. 2^30");
    h->opt_amg_small_lanes = value;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.small_lanes = value;
  }
  else if (n == "amg_merge") {
    if (value < -1 || value > 1) return fail(MFEA_EINVAL, "amg_merge: -1 (small networks), 0 or 1");
    h->opt_amg_merge = (int)value;
    rebuild = true;
  }
  else if (n == "amg_down_split") {
    h->opt_amg_down_split = value != 0;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.dsplit = (int)(value != 0);
  }
  else if (n == "amg_op_lanes") {
    if (value != 0 && value != 1 && value != 2 && value != 4)
      return fail(MFEA_EINVAL, "amg_op_lanes: 0 (by width), 1, 2 or 4");
    h->opt_amg_alanes = (int)value;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.alanes = (int)value;
  }
  else if (n == "amg_tail_lds") {
    h->opt_amg_tail_lds = value != 0;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.tail_lds = (int)(value != 0);
  }
  else if (n == "amg_collapse" || n == "amg_collapse_mb" || n == "amg_collapse_pairs") {
    if (n == "amg_collapse" ? (value < -1 || value >= kAmgMaxLevels)
        : n == "amg_collapse_mb" ? (value < 0 || value > (int64_t(1) << 40 >> 20))
                                 : (value < 0 || value >= INT32_MAX))
      return fail(MFEA_EINVAL, n + ": out of range");
    if (n == "amg_collapse") h->opt_amg_collapse = (int)value;
    else if (n == "amg_collapse_mb") h->opt_amg_collapse_mb = value;
    else h->opt_amg_collapse_pairs = value;
    rebuild = true;
  }
  else if (n == "amg_spatial") {
    if (value < -1 || value > 1) return fail(MFEA_EINVAL, "amg_spatial: -1 (by locality), 0 or 1");
    h->opt_amg_spatial = (int)value;
    rebuild = true;
  }
  else if (n == "amg_up_lanes") {
    if (value != 0 && value != 1 && value != 2 && value != 4)
      return fail(MFEA_EINVAL, "amg_up_lanes: 0 (by width), 1, 2 or 4");
    h->opt_amg_up_lanes = (int)value;
    for (auto& pp : h->parts)
      for (auto& L : pp->amg_lev) L.ulanes = (int)value;
  }
  else if (n == "amg_coarse_rho_ppm") {
    if (value != 0 && (value < 100000 || value > 100000000))
      return fail(MFEA_EINVAL, "amg_coarse_rho_ppm: 0 (Gershgorin) or 1e5 .. 1e8");
    h->opt_amg_coarse_rho_ppm = value;
    h->amg_safe_omega = false;
    rebuild = true;
  }
  else if (n == "amg_a0_slot") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "amg_a0_slot: 0 or 1");
    h->opt_amg_a0_slot = (int)value;
    rebuild = true;
  }
  else if (n == "sweep_piece") {
    if (value < 1 || value > 64) return fail(MFEA_EINVAL, "sweep_piece: 1..64");
    h->opt_sweep_piece = (int)value;
    rebuild = true;
  }
  else if (n == "amg_fuse_setup") {
    if (value < 0 || value > 1) return fail(MFEA_EINVAL, "amg_fuse_setup: 0 or 1");
    h->opt_amg_fuse_setup = (int)value;
  }
  else if (n == "amg_theta_ppm") {
    if (value < 0 || value > 1000000) return fail(MFEA_EINVAL, "amg_theta_ppm: 0..1000000");
    h->opt_amg_theta_ppm = value;
    rebuild = true;
  }
  else if (n == "amg_cycle") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "amg_cycle: 0 (four steps per level) or 1 (compact)");
    h->opt_amg_cycle = (int)value;
    for (auto& pp : h->parts) {
      pp->amg_cg.cycle = (int)value;
      for (auto& L : pp->amg_lev)
        if (L.PT.n > 0) L.compact = (int)value;
      if (!pp->amg_lev.empty() && pp->amg_levd.n >= pp->amg_lev.size())
        HIPC(hmemcpy(h, pp->amg_levd.ptr, pp->amg_lev.data(), pp->amg_lev.size() * sizeof(AmgLevD),
                       hipMemcpyHostToDevice));
    }
  }
  else if (n == "dist_timeout_ms") h->dist_timeout_s = value / 1e3;
  else if (n == "amg_reuse") {
    if (value < 0 || value > 1) return fail(MFEA_EINVAL, "amg_reuse: 0 (rebuild per active set) or 1");
    h->opt_amg_reuse = (int)value;
    for (auto& pp : h->parts) pp->amg_stale = true;  // the next solve builds for its own set
  }
  else if (n == "amg_rebuild_pct") {
    if (value < 100 || value > 100000) return fail(MFEA_EINVAL, "amg_rebuild_pct: 100 .. 100000");
    h->opt_amg_rebuild_pct = (int)value;
  }
  else if (n == "amg_rebuild_rent") {
    if (value < 0 || value > 100000) return fail(MFEA_EINVAL, "amg_rebuild_rent: 0 .. 100000");
    h->opt_amg_rebuild_rent = (int)value;
  }
  else if (n == "amg_dist") {
    if (value < -1 || value > 1)
      return fail(MFEA_EINVAL, "amg_dist: 0 (block Jacobi over partitions), 1 (global hierarchy), -1 (faster)");
    h->opt_amg_dist = (int)value;
    h->amg_auto.gen = -1;
  }
  else if (n == "amg_rep_rows") {
    if (value < 0) return fail(MFEA_EINVAL, "amg_rep_rows: >= 0");
    h->opt_amg_rep_rows = value;
    h->gamg_ok = false;
  }
  else if (n == "amg_dist_cycle") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "amg_dist_cycle: 0 (four-step) or 1 (compact)");
    h->opt_amg_dist_cycle = (int)value;
    h->gamg_ok = false;
  }
  else if (n == "dist_sums") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "dist_sums: 1 (all-reduce) or 0 (send / receive pairs)");
    h->opt_dist_sums = (int)value;
    for (auto& pp : h->parts) pp->amg_dist.zero_w = value && h->world > 1 ? h->world : 0;
    destroy_graph(h);  // captured chunks hold the old exchange
  }
  else if (n == "combo_graph") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "combo_graph: 0 or 1");
    h->opt_combo_graph = (int)value;
  }
  else if (n == "graph_start") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "graph_start: 0 or 1");
    h->opt_graph_start = (int)value;
  }
  else if (n == "step_graph") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "step_graph: 0 or 1");
    h->opt_step_graph = (int)value;
  }
  else if (n == "batch_graph") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "batch_graph: 0 or 1");
    h->opt_batch_graph = (int)value;
  }
  else if (n == "setup_entry") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "setup_entry: 0 or 1");
    h->opt_setup_entry = (int)value;
  }
  else if (n == "spec_post") {
    if (value != 0 && value != 1) return fail(MFEA_EINVAL, "spec_post: 0 or 1");
    h->opt_spec_post = (int)value;
  }
  else if (n == "asm_kernel") {
    if (value < 0 || value > 2)
      return fail(MFEA_EINVAL, "asm_kernel: 0 (row gather), 1 (element colours), 2 (element pass + row pass)");
    h->opt_asm_kernel = (int)value;
  }
  else if (n == "cc_tile") {
    if (value != 512 && value != 1024 && value != 2048 && value != 4096)
      return fail(MFEA_EINVAL, "cc_tile: 512, 1024, 2048 or 4096");
    h->opt_cc_tile = (int)value;
  }
  else if (n == "part_slack_pct") {
    if (value < 0 || value > 45) return fail(MFEA_EINVAL, "part_slack_pct: 0..45");
    h->opt_part_slack = value / 100.0;
    rebuild = true;
  }
  else return fail(MFEA_EINVAL, "unknown option " + n);
  destroy_graph(h);  // captured graphs hold the old geometry
  if (rebuild) {
    if (!h->dirty && h->Ecount) {  // keep the current activity across the rebuild
      RC(set_device(h));
      RC(gather_active(h, h->active_host));
    }
    h->dirty = true;
  }
  return 0;
}

int mfea_debug_amg_vcycle(mfea_handle* h, const double* r, double* u) {
  if (!h || !r || !u) return fail(MFEA_EINVAL, "NULL argument");
  RC(set_device(h));
  RC(ensure_built(h));
  hipStream_t s = h->stream;
  const bool dm = partitioned(h);
  if (dm && !h->opt_amg_dist) return fail(MFEA_ESTATE, "mfea_debug_amg_vcycle: amg_dist 0 is not one operator");
  bool rebuilt = false;
  if (dm) {
    RC(ensure_gamg(h, &rebuilt));
    RC(enqueue_gamg_setup(h, 1e-12));
  } else {
    RC(ensure_amg(h, part0(h), &rebuilt));
    enqueue_amg_setup(h, part0(h), 1e-12);
  }
  const int nd = dm ? h->gamg.nd : part0(h).amg.nd;
  // r (node order) → each partition's row-order RHS buffer (its q), then
  // the CG init (r, x = ω D⁻¹ r) and one V-cycle
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const Pattern& P = pt.P;
    std::vector<double> b(3 * P.n_nodes, 0.0);
    for (int64_t i = 0; i < P.n_free; ++i) {
      const int64_t g = dm ? pt.plan.node_g[P.perm[i]] : P.perm[i];
      for (int a = 0; a < nd; ++a) b[3 * i + a] = r[nd * g + a];
    }
    HIPC(hmemcpy(h, pt.q.ptr, b.data(), b.size() * sizeof(double), hipMemcpyHostToDevice));
    launch_amg_cg_init(s, nd, pt.amg_lev[0], pt.amg_cg, pt.q.ptr);
  }
  if (dm) {
    RC(enqueue_gamg_vcycle(h, -1));
  } else {
    Part& pt = part0(h);
    launch_amg_vcycle(s, nd, pt.amg_lev.data(), (int)pt.amg_lev.size(), pt.amg_cg, pt.amg_tail, nullptr);
  }
  HIPC(hipGetLastError());
  RC(sync_stream(h));
  std::memset(u, 0, (size_t)h->N * nd * sizeof(double));
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const AmgCg& cg = pt.amg_cg;
    std::vector<float> uf((size_t)nd * cg.n);
    std::vector<int32_t> row0(cg.n);
    if (cg.n) {
      HIPC(hmemcpy(h, uf.data(), cg.u, uf.size() * sizeof(float), hipMemcpyDeviceToHost));
      HIPC(hmemcpy(h, row0.data(), cg.row0, row0.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    }
    for (int64_t i = cg.lo; i < cg.hi; ++i) {
      const int64_t lr = row0[i];
      const int64_t g = dm ? pt.plan.node_g[pt.P.perm[lr]] : pt.P.perm[lr];
      for (int a = 0; a < nd; ++a) u[nd * g + a] = uf[nd * i + a];
    }
  }
  return 0;
}

int mfea_debug_amg_vector(mfea_handle* h, int l, int which, double* out, int64_t cap, int64_t* n) {
  if (!h || !n || which < 0 || which > 6) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  const bool dm = partitioned(h);
  const AmgPlan& pl = dm ? h->gamg : part0(h).amg;
  if (l < 0 || l >= (int)pl.lev.size()) return fail(MFEA_EINVAL, "level out of range");
  const int nd = pl.nd;
  const AmgLevel& L = pl.lev[l];
  *n = L.A.n;
  const int w = which >= 4 && which != 5 ? nd * nd : nd;  // per-row width
  if (!out) return 0;
  // the device must hold the plan pl describes (a partitioned handle may hold
  // the block-Jacobi plans after amg_dist 0 or an automatic choice of it)
  if (dm)
    for (auto& pp : h->parts)
      if (pp->dev_plan != 1) return fail(MFEA_ESTATE, "the device holds the block-Jacobi plans: run amg_vcycle first");
  if (cap < w * L.A.n) return fail(MFEA_EINVAL, "output too small");
  for (auto& pp : h->parts) {
    Part& pt = *pp;
    const AmgLevD& d = pt.amg_lev[l];
    std::vector<double> v((size_t)w * L.A.n, 0.0);
    if (which == 4) {  // D⁻¹ blocks
      std::vector<float> f(v.size());
      HIPC(hmemcpy(h, f.data(), d.dinv32, f.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (size_t k = 0; k < f.size(); ++k) v[k] = f[k];
    } else if (which == 5) {  // the Gershgorin bound g, every row
      double om[2];
      HIPC(hmemcpy(h, om, d.omega, sizeof(om), hipMemcpyDeviceToHost));
      std::fill(v.begin(), v.end(), om[1]);
    } else if (which == 6) {  // diagonal blocks of A (slot 0 of every row)
      std::vector<float> a((size_t)nd * nd * d.A.npos);
      HIPC(hmemcpy(h, a.data(), d.A.val32, a.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < L.A.n; ++i)
        for (int c = 0; c < nd * nd; ++c) v[(size_t)nd * nd * i + c] = a[(size_t)nd * nd * L.A.pos(i, 0) + c];
    } else if (l == 0 && (which == 0 || which == 3)) {
      if (which == 0) {
        HIPC(hmemcpy(h, v.data(), pt.amg_cg.r, v.size() * sizeof(double), hipMemcpyDeviceToHost));
      } else {
        std::vector<float> f(v.size());
        HIPC(hmemcpy(h, f.data(), pt.amg_cg.u, f.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < f.size(); ++k) v[k] = f[k];
      }
    } else {
      const float* src = which == 0 ? d.b : which == 1 ? d.x : which == 2 ? d.t : d.e;
      if (!src) return fail(MFEA_EINVAL, "no such vector on this level");
      std::vector<float> f(v.size());
      HIPC(hmemcpy(h, f.data(), src, f.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (size_t k = 0; k < f.size(); ++k) v[k] = f[k];
    }
    const bool split = dm && l < pl.n_dist;
    const int64_t lo = split ? pt.amg_rank.lo[l] : 0, hi = split ? pt.amg_rank.hi[l] : L.A.n;
    if (!split && pt.rank != 0) continue;
    for (int64_t i = lo; i < hi; ++i)
      for (int a = 0; a < w; ++a) out[(size_t)w * L.nat[i] + a] = v[(size_t)w * i + a];
  }
  return 0;
}

int mfea_get_option(mfea_handle* h, const char* name, int64_t* value) {
  if (!h || !name || !value) return fail(MFEA_EINVAL, "NULL argument");
  const std::string n(name);
  // the read-only plan values need a partition to read them from
  static const char* plan_names[] = {"amg_merged", "amg_merge_dq_blocks", "amg_merge_u_blocks", "sweep_colors",
                                     "sweep_pieces", "amg_reused", "amg_build_iters"};
  for (const char* pn : plan_names)
    if (n == pn && h->parts.empty()) return fail(MFEA_ESTATE, std::string(name) + ": no partition yet");
  if (n == "graph") *value = h->opt_graph;
  else if (n == "phase_times") *value = h->opt_phase_times ? 1 : 0;
  else if (n == "dist_graph") *value = h->opt_dist_graph;
  else if (n == "order") *value = h->opt_order;
  else if (n == "lane_dof") *value = h->opt_lane_dof;
  else if (n == "cg_kernel") *value = h->opt_cg_kernel;
  else if (n == "ell_block") *value = h->opt_ell_block;
  else if (n == "ell_maxg") *value = h->opt_ell_maxg;
  else if (n == "ell_compact") *value = h->opt_ell_compact;
  else if (n == "amg_tail_rows") *value = h->opt_amg_tail_rows;
  else if (n == "amg_max_levels") *value = h->opt_amg_max_levels;
  else if (n == "amg_restrict_lanes") *value = h->opt_amg_rlanes;
  else if (n == "amg_down_split") *value = h->opt_amg_down_split;
  else if (n == "amg_v_lanes") *value = h->opt_amg_v_lanes;
  else if (n == "amg_merge") *value = h->opt_amg_merge;
  else if (n == "amg_merged") *value = part0(h).amg_mg.on;  // read-only: the plan's cycle form
  else if (n == "amg_merge_dq_blocks" || n == "amg_merge_u_blocks") {  // read-only: stored blocks of DQ / U
    const AmgMerge& M = part0(h).amg_mplan;
    int64_t nb = 0;
    if (M.on)
      for (int32_t c : (n == "amg_merge_dq_blocks" ? M.DQ.col : M.U.col)) nb += c >= 0;
    *value = nb;
  }
  else if (n == "amg_small_lanes") *value = h->opt_amg_small_lanes;
  else if (n == "amg_op_lanes") *value = h->opt_amg_alanes;
  else if (n == "amg_tail_lds") *value = h->opt_amg_tail_lds;
  else if (n == "amg_cycle") *value = h->opt_amg_cycle;
  else if (n == "amg_theta_ppm") *value = h->opt_amg_theta_ppm;
  else if (n == "amg_fuse_setup") *value = h->opt_amg_fuse_setup;
  else if (n == "sweep_piece") *value = h->opt_sweep_piece;
  else if (n == "sweep_colors") *value = part0(h).sweep.colors;  // read-only
  else if (n == "sweep_pieces") *value = part0(h).sweep.n_pieces;  // read-only
  else if (n == "amg_up_lanes") *value = h->opt_amg_up_lanes;
  else if (n == "amg_coarse_rho_ppm") *value = h->opt_amg_coarse_rho_ppm;
  else if (n == "amg_a0_slot") *value = h->opt_amg_a0_slot;
  else if (n == "amg_safe_omega") *value = h->amg_safe_omega ? 1 : 0;  // read-only
  else if (n == "amg_spatial") *value = h->opt_amg_spatial;
  else if (n == "amg_collapse") *value = h->opt_amg_collapse;
  else if (n == "amg_collapse_mb") *value = h->opt_amg_collapse_mb;
  else if (n == "amg_collapse_pairs") *value = h->opt_amg_collapse_pairs;
  else if (n == "amg_collapse_level") {  // read-only: partition 0's collapsed level kc (0: none)
    *value = h->parts.empty() ? 0 : h->parts[0]->amg_coll.kc;
  }
  else if (n == "amg_collapse_blocks") {  // read-only: stored blocks of the collapsed V at kc
    int64_t nb = 0;
    if (!h->parts.empty() && h->parts[0]->amg_coll.kc > 0)
      for (int32_t c : h->parts[0]->amg_coll.lev[0].V.col) nb += c >= 0;
    *value = nb;
  }
  else if (n == "amg_spatial_chosen") {  // read-only: partition 0's plan is in Z-order
    *value = h->parts.empty() ? 0 : (h->parts[0]->amg.spatial ? 1 : 0);
  }
  else if (n == "dist_timeout_ms") *value = (int64_t)std::llround(h->dist_timeout_s * 1e3);
  else if (n == "amg_dist") *value = h->opt_amg_dist;
  else if (n == "amg_reuse") *value = h->opt_amg_reuse;
  else if (n == "amg_rebuild_pct") *value = h->opt_amg_rebuild_pct;
  else if (n == "amg_rebuild_rent") *value = h->opt_amg_rebuild_rent;
  else if (n == "amg_reused") *value = part0(h).amg_reused ? 1 : 0;  // read-only: the last solve kept a hierarchy built for another set
  else if (n == "amg_build_iters") *value = part0(h).amg_build_iters;  // read-only
  else if (n == "amg_dist_chosen")  // read-only: the form in use (-1: the automatic choice still undecided)
    *value = h->opt_amg_dist >= 0 ? h->opt_amg_dist : h->amg_auto.choice;
  else if (n == "amg_rep_rows") *value = h->opt_amg_rep_rows;
  else if (n == "cc_tile") *value = h->opt_cc_tile;
  else if (n == "asm_kernel") *value = h->opt_asm_kernel;
  else if (n == "spec_post") *value = h->opt_spec_post;
  else if (n == "setup_entry") *value = h->opt_setup_entry;
  else if (n == "batch_graph") *value = h->opt_batch_graph;
  else if (n == "step_graph") *value = h->opt_step_graph;
  else if (n == "graph_start") *value = h->opt_graph_start;
  else if (n == "combo_graph") *value = h->opt_combo_graph;
  else if (n == "asm_colours") {
    *value = 0;
    for (auto& pp : h->parts) *value = std::max<int64_t>(*value, pp->ec_state > 0 ? pp->ec.colors : 0);
  }
  else if (n == "amg_dist_cycle") *value = h->opt_amg_dist_cycle;
  else if (n == "dist_sums") *value = h->opt_dist_sums;
  else if (n == "part_slack_pct") *value = (int64_t)std::llround(h->opt_part_slack * 100.0);
  else return fail(MFEA_EINVAL, "unknown option " + n);
  return 0;
}

int mfea_debug_global_active(mfea_handle* h, uint8_t* out) {
  if (!h || !out) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  RC(ensure_built(h));
  std::vector<uint8_t> key;
  if (partitioned(h)) RC(global_active(h, key));
  else RC(gather_active(h, key));
  std::copy(key.begin(), key.end(), out);
  return 0;
}

int mfea_debug_floating(mfea_handle* h, uint8_t* out) {
  if (!h || !out) return fail(MFEA_EINVAL, "bad argument");
  RC(set_device(h));
  RC(ensure_built(h));
  if (partitioned(h)) return fail(MFEA_ESTATE, "mfea_debug_floating: one partition");
  Part& pt = part0(h);
  const Pattern& P = pt.P;
  std::memset(out, 0, (size_t)h->N);
  if (P.n_free == 0) return 0;
  DevBuf<uint8_t> mask;
  HIPC(mask.alloc(P.n_free));
  HIPC(pt.cc_parent.alloc(std::max<int64_t>(P.n_nodes, 1)));
  HIPC(pt.cc_anch.alloc(std::max<int64_t>(P.n_nodes, 1)));
  launch_floating(h->stream, P.n_nodes, P.n_free, P.n_nodes - P.n_ghost, pt.slice_ptr.ptr, pt.row_len.ptr,
                  pt.s_col.ptr, pt.s_elem.ptr, pt.active.ptr, pt.cc_parent.ptr, pt.cc_anch.ptr, nullptr, mask.ptr,
                  h->opt_cc_tile);
  HIPC(hipGetLastError());
  std::vector<uint8_t> m(P.n_free);
  HIPC(hipMemcpyAsync(m.data(), mask.ptr, P.n_free, hipMemcpyDeviceToHost, h->stream));
  RC(sync_stream(h));
  for (int64_t r = 0; r < P.n_free; ++r) out[P.perm[r]] = m[r];
  return 0;
}

int mfea_debug_set_parts(mfea_handle* h, int nparts, int axis) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (nparts < 1 || nparts > kMaxRanks) return fail(MFEA_EINVAL, "nparts must be in [1, 64]");
  if (axis < -1 || axis > 1) return fail(MFEA_EINVAL, "axis must be -1, 0 or 1");
  if (h->world > 1 && nparts > 1) return fail(MFEA_ESTATE, "handle already joined an RCCL world");
  h->nparts = nparts;
  h->axis = axis;
  h->dirty = true;
  return 0;
}

int mfea_set_partition_axis(mfea_handle* h, int axis) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (axis < -1 || axis > 1) return fail(MFEA_EINVAL, "axis must be -1, 0 or 1");
  h->axis = axis;
  h->dirty = true;
  return 0;
}

int mfea_write_record_csv(const char* path, int style, int kind, int64_t n_rows, int64_t n_cols,
                          const double* values, const uint8_t* flags, int n_threads) {
  const std::string err =
      write_record_csv(path, style, kind, n_rows, n_cols, values, flags, n_threads);
  return err.empty() ? 0 : fail(MFEA_EINVAL, err);
}

int mfea_write_record_npy(const char* path, int kind, int64_t n_rows, int64_t n_cols, const double* values,
                          const uint8_t* flags) {
  const std::string err = write_record_npy(path, kind, n_rows, n_cols, values, flags);
  return err.empty() ? 0 : fail(MFEA_EINVAL, err);
}

int mfea_dist_unique_id(uint8_t* unique_id) {
  if (!unique_id) return fail(MFEA_EINVAL, "NULL argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  NCCLC(ncclGetUniqueId(&u));
  std::memcpy(unique_id, &u, sizeof(u));
  return 0;
}

int mfea_get_ownership(mfea_handle* h, uint8_t* node_owned, uint8_t* elem_owned) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  if (!partitioned(h)) {
    if (node_owned) std::memset(node_owned, 1, (size_t)h->N);
    if (elem_owned) std::memset(elem_owned, 1, (size_t)h->Ecount);
    return 0;
  }
  if (node_owned) std::memset(node_owned, 0, (size_t)h->N);
  if (elem_owned) std::memset(elem_owned, 0, (size_t)h->Ecount);
  for (auto& pp : h->parts) {
    const PartPlan& pl = pp->plan;
    if (node_owned)
      for (size_t ln = 0; ln < pl.node_g.size(); ++ln)
        if (!pl.ghost[ln]) node_owned[pl.node_g[ln]] = 1;
    if (elem_owned)
      for (size_t le = 0; le < pl.elem_g.size(); ++le)
        if (pl.elem_own[le]) elem_owned[pl.elem_g[le]] = 1;
  }
  return 0;
}

int mfea_gather_results(mfea_handle* h, double* U, double* stress, uint8_t* active) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  RC(set_device(h));
  RC(ensure_built(h));
  const int64_t N = h->N, E = h->Ecount;
  if (h->world <= 1) {
    if (U) RC(mfea_get_displacement(h, U));
    if (stress && E) RC(mfea_get_stress(h, stress));
    if (active && E) RC(mfea_get_active(h, active));
    return 0;
  }
  // this rank's values of its own nodes / elements (ascending global id);
  // every rank knows every rank's counts (the partition is deterministic)
  const int W = h->world, me = h->rank;
  std::vector<double> Ul(3 * N, 0.0), Sl(E, 0.0);
  std::vector<uint8_t> Al(E, 1), nown(N), eown(E);
  RC(mfea_get_displacement(h, Ul.data()));
  if (E) {
    RC(mfea_get_stress(h, Sl.data()));
    RC(mfea_get_active(h, Al.data()));
  }
  auto node_rank = [&](int64_t n) { return h->gowner[n]; };
  auto elem_rank = [&](int64_t e) {
    const int64_t a = h->e2n[2 * e], b = h->e2n[2 * e + 1];
    return (a < 0 || a >= N || b < 0 || b >= N) ? -1 : h->gowner[a];  // skipped elements: nobody's
  };
  std::vector<int64_t> len(W, 0), off(W + 1, 0);
  for (int64_t n = 0; n < N; ++n) len[node_rank(n)] += 3;
  for (int64_t e = 0; e < E; ++e)
    if (elem_rank(e) >= 0) len[elem_rank(e)] += 2;
  for (int p = 0; p < W; ++p) off[p + 1] = off[p] + len[p];
  hipStream_t s = h->stream;
  DevBuf<double> buf;
  if (me != 0) {
    std::vector<double> pk;
    pk.reserve(len[me]);
    for (int64_t n = 0; n < N; ++n)
      if (node_rank(n) == me)
        for (int a = 0; a < 3; ++a) pk.push_back(Ul[3 * n + a]);
    for (int64_t e = 0; e < E; ++e)
      if (elem_rank(e) == me) {
        pk.push_back(Sl[e]);
        pk.push_back(Al[e] ? 1.0 : 0.0);
      }
    HIPC(buf.alloc(pk.size() + 1));
    HIPC(hmemcpy(h, buf.ptr, pk.data(), pk.size() * sizeof(double), hipMemcpyHostToDevice));
    NCCLC(ncclGroupStart());
    if (!pk.empty()) NCCLC(ncclSend(buf.ptr, pk.size(), ncclFloat64, 0, h->comm, s));
    NCCLC(ncclGroupEnd());
    return sync_stream(h);
  }
  HIPC(buf.alloc(off[W] + 1));
  NCCLC(ncclGroupStart());
  for (int p = 1; p < W; ++p)
    if (len[p]) NCCLC(ncclRecv(buf.ptr + off[p], (size_t)len[p], ncclFloat64, p, h->comm, s));
  NCCLC(ncclGroupEnd());
  RC(sync_stream(h));
  std::vector<double> all(off[W]);
  if (off[W]) HIPC(hmemcpy(h, all.data(), buf.ptr, off[W] * sizeof(double), hipMemcpyDeviceToHost));
  std::vector<int64_t> at(off.begin(), off.end() - 1);
  for (int64_t n = 0; n < N; ++n) {
    const int p = node_rank(n);
    for (int a = 0; a < 3; ++a) {
      const double v = p == 0 ? Ul[3 * n + a] : all[at[p]++];
      if (U) U[3 * n + a] = v;
    }
  }
  for (int64_t e = 0; e < E; ++e) {
    const int p = elem_rank(e);
    double sv = Sl[e], av = Al[e];
    if (p > 0) {
      sv = all[at[p]++];
      av = all[at[p]++];
    }
    if (stress) stress[e] = sv;
    if (active) active[e] = av != 0.0 ? 1 : 0;
  }
  return 0;
}

int mfea_dist_init(mfea_handle* h, int rank, int world, const uint8_t* unique_id) {
  if (!h || !unique_id) return fail(MFEA_EINVAL, "NULL argument");
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world)
    return fail(MFEA_EINVAL, "bad rank / world size");
  if (h->comm) return fail(MFEA_ESTATE, "handle already joined an RCCL world");
  if (h->nparts > 1) return fail(MFEA_ESTATE, "handle holds several partitions");
  RC(set_device(h));
  if (world > 1) {
    ncclUniqueId u;
    std::memcpy(&u, unique_id, sizeof(u));
    ncclComm_t c = nullptr;
    NCCLC(ncclCommInitRank(&c, world, u, rank));
    h->comm = c;
  }
  h->world = world;
  h->rank = rank;
  h->dirty = true;
  return 0;
}

}  // extern "C"
