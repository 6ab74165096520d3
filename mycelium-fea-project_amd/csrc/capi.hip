// capi.hip — the C ABI of include/mfea.h: handle, device memory, the on-device
// step loop (assemble → RHS → PCG in hipGraph-captured chunks → reaction/stress).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.hpp"
#include "mfea_debug.h"
#include "mfea.h"
#include "symbolic.hpp"

using namespace mfea;

namespace {

thread_local std::string g_err;

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

template <class T>
struct DevBuf {
  T* ptr = nullptr;
  size_t n = 0;
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

struct mfea_handle {
  int device = 0;
  hipStream_t stream = nullptr;
  double E = 2500.0, A = 0.0, I = 0.0;
  Material mat{};
  // host-side mesh/BC
  int64_t N = 0, Ecount = 0;
  std::vector<double> xyz;
  std::vector<int64_t> e2n;
  uint32_t mesh_flags = 0;
  std::vector<int64_t> top, bot;
  bool has_mesh = false, dirty = true;
  std::vector<uint8_t> active_host;  // pending upload (empty = none)
  Pattern P;
  // device
  DevBuf<double> xyz_d, val, diag, x, r, p, q, dinv, stress, partials, red;
  DevBuf<double> cg_r1, cg_s0, cg_s1, cg_w0, cg_w1;  // CG-CG double buffers (r0 = r)
  DevBuf<double> cg_part;                            // CG-CG block partials, 2 parities
  DevBuf<int32_t> slice_ptr, row_len, s_col, s_elem, e2n_d;
  DevBuf<uint8_t> active, code;
  DevBuf<unsigned> tickets;
  // wave-local lane operator (ell.hip); ell_ok = false → SELL kernel
  Ell L;
  bool ell_ok = false;
  DevBuf<uint32_t> e_code;
  DevBuf<int32_t> e_partner, e_lane_row, e_src_pos, e_nbr_lane;
  DevBuf<double> e_f;  // all lane-operator doubles, carved by ell_op / ell_vecs
  DevBuf<Slot> slots;
  DevBuf<SolveState> state;
  SolveState* h_state = nullptr;  // pinned, 2 entries
  SolveState* d_host_state = nullptr;  // device view of h_state (mapped)
  double* h_red = nullptr;        // pinned
  int64_t G = 0;                  // slots·64
  // graph cache
  hipGraphExec_t graph = nullptr;
  int graph_chunk = 0, graph_precond = -1, graph_ell = -1;
  hipEvent_t ev[6] = {};
  hipEvent_t poll[2] = {};
  int64_t n_active = 0;
  // generic CSR path scratch
  DevBuf<int64_t> c_indptr;
  DevBuf<int32_t> c_indices;
  DevBuf<double> c_data, c_kval, c_x, c_r, c_p, c_q, c_dinv;
  DevBuf<uint8_t> c_known;
};

namespace {

constexpr int kMaxChunk = 64;
// lane-operator doubles per lane: V 18, D 6, x 3, p 3, r/s/w × 2 18, M 6, h × 2 18, hM 6
constexpr int64_t kEllDoubles = 18 + 6 + 3 + 3 + 18 + 6 + 18 + 6;
static_assert(kEllNone == kSrcNone && kEllHalo == kSrcHalo, "slot source codes");
constexpr int kTicketSets = 16;

// ticket set k (one per reducing kernel kind; see device_util.hpp layout)
unsigned* tix(mfea_handle* h, int k) { return h->tickets.ptr + (size_t)k * kTicketStride; }

void destroy_graph(mfea_handle* h) {
  if (h->graph) (void)hipGraphExecDestroy(h->graph);
  h->graph = nullptr;
  h->graph_chunk = 0;
  h->graph_precond = -1;
  h->graph_ell = -1;
}

int set_device(mfea_handle* h) {
  HIPC(hipSetDevice(h->device));
  return 0;
}

// Row ordering of the free nodes: DFS by default; MFEA_ORDER=natural|<window>
// for experiments (original order / degree sort inside windows).
int order_mode() {
  const char* e = std::getenv("MFEA_ORDER");
  if (!e || !*e || std::strcmp(e, "dfs") == 0) return kOrderDFS;
  if (std::strcmp(e, "natural") == 0) return 0;
  return std::atoi(e);
}

// Build the symbolic pattern and (re)allocate + upload device state.
int ensure_built(mfea_handle* h) {
  if (!h->has_mesh) return fail(MFEA_ESTATE, "no mesh: call mfea_set_mesh first");
  if (!h->dirty) return 0;
  destroy_graph(h);
  std::string err = build_pattern(h->N, h->xyz.data(), h->Ecount, h->e2n.data(),
                                  (h->mesh_flags & MFEA_MESH_SKIP_INVALID) != 0, h->top, h->bot,
                                  order_mode(), h->P);
  if (!err.empty()) return fail(MFEA_EINVAL, err);
  const Pattern& P = h->P;
  const int64_t N = P.n_nodes, E = P.n_elems;
  h->G = P.n_slots() * kSlice;
  const int64_t maxg = std::max<int64_t>({grid_rows(N), grid_rows(E), 2048, 1});
  HIPC(h->xyz_d.alloc(3 * N));
  HIPC(h->val.alloc(6 * h->G));
  HIPC(h->diag.alloc(6 * N));
  HIPC(h->x.alloc(3 * N));
  HIPC(h->r.alloc(3 * N));
  HIPC(h->p.alloc(3 * N));
  HIPC(h->q.alloc(3 * N));
  HIPC(h->cg_r1.alloc(3 * N));
  HIPC(h->cg_s0.alloc(3 * N));
  HIPC(h->cg_s1.alloc(3 * N));
  HIPC(h->cg_w0.alloc(3 * N));
  HIPC(h->cg_w1.alloc(3 * N));
  HIPC(h->cg_part.alloc(2 * 4 * kCgMaxPartials));
  HIPC(h->dinv.alloc(6 * N));
  HIPC(h->stress.alloc(E));
  HIPC(h->partials.alloc(4 * (maxg + 16)));
  HIPC(h->red.alloc(16));
  HIPC(h->slice_ptr.alloc(P.slice_ptr.size()));
  HIPC(h->row_len.alloc(N));
  HIPC(h->s_col.alloc(h->G));
  HIPC(h->s_elem.alloc(h->G));
  HIPC(h->e2n_d.alloc(2 * E));
  HIPC(h->active.alloc(E));
  HIPC(h->code.alloc(N));
  HIPC(h->tickets.alloc(kTicketSets * kTicketStride));
  HIPC(h->slots.alloc(kMaxChunk + 2));
  HIPC(h->state.alloc(1));
  hipStream_t s = h->stream;
  auto up = [&](void* d, const void* src, size_t bytes) {
    return bytes ? hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
  };
  HIPC(up(h->xyz_d.ptr, P.xyz_perm.data(), 3 * N * sizeof(double)));
  HIPC(up(h->slice_ptr.ptr, P.slice_ptr.data(), P.slice_ptr.size() * sizeof(int32_t)));
  HIPC(up(h->row_len.ptr, P.row_len.data(), N * sizeof(int32_t)));
  HIPC(up(h->s_col.ptr, P.s_col.data(), h->G * sizeof(int32_t)));
  HIPC(up(h->s_elem.ptr, P.s_elem.data(), h->G * sizeof(int32_t)));
  HIPC(up(h->e2n_d.ptr, P.e2n_perm.data(), 2 * E * sizeof(int32_t)));
  HIPC(up(h->code.ptr, P.code.data(), N * sizeof(uint8_t)));
  HIPC(hipMemsetAsync(h->tickets.ptr, 0, kTicketSets * kTicketStride * sizeof(unsigned), s));
  HIPC(hipMemsetAsync(h->x.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(h->p.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(h->q.ptr, 0, 3 * N * sizeof(double), s));
  HIPC(hipMemsetAsync(h->stress.ptr, 0, E * sizeof(double), s));
  HIPC(hipMemsetAsync(h->val.ptr, 0, 6 * h->G * sizeof(double), s));
  HIPC(hipMemsetAsync(h->diag.ptr, 0, 6 * N * sizeof(double), s));
  if (h->active_host.size() == (size_t)E) {
    HIPC(up(h->active.ptr, h->active_host.data(), E));
  } else {
    HIPC(hipMemsetAsync(h->active.ptr, 1, E, s));
  }
  // wave-local lanes (falls back to the SELL kernel when a row cannot be placed)
  h->ell_ok = build_ell(P, h->L).empty() && P.n_free > 0;
  if (h->ell_ok) {
    const Ell& L = h->L;
    const int64_t NL = L.n_lanes;
    std::vector<uint32_t> code(NL);
    for (int64_t l = 0; l < NL; ++l)
      code[l] = (L.code[l] & 0xFFFFFFu) | (uint32_t)(uint8_t)(int8_t)L.info[l] << 24;
    HIPC(h->e_code.alloc(NL));
    HIPC(h->e_partner.alloc(NL));
    HIPC(h->e_lane_row.alloc(NL));
    HIPC(h->e_src_pos.alloc(3 * NL));
    HIPC(h->e_nbr_lane.alloc(3 * NL));
    HIPC(h->e_f.alloc(kEllDoubles * NL));
    HIPC(up(h->e_code.ptr, code.data(), NL * sizeof(uint32_t)));
    HIPC(up(h->e_partner.ptr, L.partner.data(), NL * sizeof(int32_t)));
    HIPC(up(h->e_lane_row.ptr, L.lane_row.data(), NL * sizeof(int32_t)));
    HIPC(up(h->e_src_pos.ptr, L.src_pos.data(), 3 * NL * sizeof(int32_t)));
    HIPC(up(h->e_nbr_lane.ptr, L.nbr_lane.data(), 3 * NL * sizeof(int32_t)));
    // halo records of lanes without a halo slot are read but never used
    HIPC(hipMemsetAsync(h->e_f.ptr, 0, kEllDoubles * NL * sizeof(double), s));
  }
  HIPC(hipStreamSynchronize(s));
  h->active_host.clear();
  h->dirty = false;
  return 0;
}

// MFEA_CG_KERNEL=sell forces the SELL iteration kernel (comparison runs)
bool use_ell(const mfea_handle* h) {
  const char* e = std::getenv("MFEA_CG_KERNEL");
  return h->ell_ok && !(e && std::strcmp(e, "sell") == 0);
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

SellOp sell_op(mfea_handle* h) {
  SellOp op;
  op.N = h->P.n_nodes;
  op.nf = h->P.n_free;
  op.G = h->G;
  op.slice_ptr = h->slice_ptr.ptr;
  op.row_len = h->row_len.ptr;
  op.s_col = h->s_col.ptr;
  op.val = h->val.ptr;
  op.diag = h->diag.ptr;
  return op;
}

CgVecs cg_vecs(mfea_handle* h) {
  CgVecs v;
  v.x = h->x.ptr;
  v.p = h->p.ptr;
  v.r[0] = h->r.ptr;
  v.r[1] = h->cg_r1.ptr;
  v.s[0] = h->cg_s0.ptr;
  v.s[1] = h->cg_s1.ptr;
  v.w[0] = h->cg_w0.ptr;
  v.w[1] = h->cg_w1.ptr;
  v.dinv = h->dinv.ptr;
  return v;
}

// planar meshes run the lanes with 2 DOFs per node (MFEA_LANE_DOF=3 forces 3)
int lane_dofs(const mfea_handle* h) {
  const char* e = std::getenv("MFEA_LANE_DOF");
  return (h->P.planar && !(e && std::strcmp(e, "3") == 0)) ? 2 : 3;
}

EllOp ell_op(mfea_handle* h) {
  EllOp op;
  const int64_t NL = h->L.n_lanes;
  op.NL = NL;
  op.nd = lane_dofs(h);
  op.code = h->e_code.ptr;
  op.partner = h->e_partner.ptr;
  op.lane_row = h->e_lane_row.ptr;
  op.src_pos = h->e_src_pos.ptr;
  op.nbr_lane = h->e_nbr_lane.ptr;
  op.V = h->e_f.ptr;
  op.D = op.V + 18 * NL;
  return op;
}

EllVecs ell_vecs(mfea_handle* h) {
  EllVecs v;
  const int64_t NL = h->L.n_lanes;
  double* f = h->e_f.ptr + 24 * NL;
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
  v.h[0] = take(9);
  v.h[1] = take(9);
  v.hM = take(6);
  return v;
}

// enqueue one chunk of single-reduction CG iterations (one kernel each)
void enqueue_chunk(mfea_handle* h, int chunk, int precond, bool ell) {
  hipStream_t s = h->stream;
  if (ell) {
    const EllOp op = ell_op(h);
    const EllVecs v = ell_vecs(h);
    for (int j = 0; j < chunk; ++j)
      launch_ell_iter(s, j, op, precond, v, h->slots.ptr, h->state.ptr, h->cg_part.ptr);
  } else {
    const SellOp op = sell_op(h);
    const CgVecs v = cg_vecs(h);
    for (int j = 0; j < chunk; ++j)
      launch_cg_iter(s, j, op, precond, v, h->slots.ptr, h->state.ptr, h->cg_part.ptr);
  }
  launch_cg_advance(s, chunk, h->slots.ptr, h->state.ptr, h->d_host_state);
}

// Replays chunks until the device reports done; at most two chunks in flight.
template <class Enqueue>
// mirror = true: the chunk's advance kernel writes the final state into the
// mapped pinned h_state[0] itself (CG-CG path); otherwise copy it per chunk.
int drive_chunks(mfea_handle* h, int chunk, int max_it, Enqueue&& enqueue, SolveState* out,
                 bool mirror = false) {
  hipStream_t s = h->stream;
  const int64_t max_chunks = (int64_t)max_it / chunk + 3;
  int64_t k = 0;
  bool done = false;
  volatile SolveState* hs = h->h_state;
  if (mirror) hs[0].done = 0;
  while (!done && k < max_chunks) {
    int rc = enqueue();
    if (rc) return rc;
    if (!mirror)
      HIPC(hipMemcpyAsync(&h->h_state[k & 1], h->state.ptr, sizeof(SolveState),
                          hipMemcpyDeviceToHost, s));
    HIPC(hipEventRecord(h->poll[k & 1], s));
    if (k >= 1) {
      HIPC(hipEventSynchronize(h->poll[(k - 1) & 1]));
      if (hs[mirror ? 0 : (k - 1) & 1].done) done = true;
    }
    ++k;
  }
  HIPC(hipStreamSynchronize(s));
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

int finish_solve(mfea_handle* h, const mfea_solve_opts* o, int64_t nf, const SolveState& fin,
                 mfea_stats* st) {
  (void)o;
  HIPC(hipEventRecord(h->ev[3], h->stream));
  HIPC(hipEventSynchronize(h->ev[3]));
  if (st) {
    st->iters = fin.iters;
    st->status = fin.status;
    st->bnorm = std::sqrt(fin.bb0);
    st->relres = fin.res0 > 0 ? std::sqrt(fin.res_final / fin.res0) : 0.0;
    st->n_free = 3 * nf;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[1], h->ev[2]);
    st->t_rhs_ms = ms;
    (void)hipEventElapsedTime(&ms, h->ev[2], h->ev[3]);
    st->t_solve_ms = ms;
  }
  if (fin.status == -4) return fail(MFEA_EMAXIT, "PCG reached max_it without converging");
  if (fin.status == -5) return fail(MFEA_EBREAKDOWN, "PCG breakdown (p·Ap <= 0 or non-finite)");
  return 0;
}

int solve_impl(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* o,
               mfea_stats* st) {
  const Pattern& P = h->P;
  hipStream_t s = h->stream;
  const int64_t nf = P.n_free;
  const int precond = o->precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0;
  int chunk = o->chunk > 0 ? std::min(o->chunk, kMaxChunk) : 32;
  chunk += chunk & 1;  // even: k_cg_iter takes the r/s/w buffer parity from j
  const SellOp op = sell_op(h);
  const CgVecs v = cg_vecs(h);
  HIPC(hipEventRecord(h->ev[1], s));
  launch_cg_rhs(s, op, h->code.ptr, dy_top, dy_bot, o->reg, precond, v, h->partials.ptr,
                tix(h, 0), h->red.ptr);
  launch_cg_init_finalize(s, h->red.ptr, o->rtol, o->atol, o->norm, o->max_it, o->reg,
                          h->state.ptr);
  HIPC(hipMemsetAsync(h->cg_part.ptr, 0, 2 * 4 * kCgMaxPartials * sizeof(double), s));
  const bool ell = use_ell(h);
  if (ell) {
    launch_ell_init(s, ell_op(h), op, precond, v, ell_vecs(h));
    launch_ell_first(s, ell_op(h), o->reg, precond, ell_vecs(h), h->slots.ptr, h->cg_part.ptr);
  } else {
    launch_cg_first(s, op, o->reg, precond, v, h->slots.ptr, h->cg_part.ptr);
  }
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(h->ev[2], s));
  // MFEA_NO_GRAPH=1: launch the chunk kernels eagerly (profilers that do not
  // follow hipGraph replays; same kernels, same order)
  static const bool no_graph = std::getenv("MFEA_NO_GRAPH") != nullptr;
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
    launch_ell_finish(s, ell_op(h), ell_vecs(h), h->x.ptr);
    HIPC(hipGetLastError());
  }
  return finish_solve(h, o, nf, fin, st);
}

int assemble_impl(mfea_handle* h, mfea_stats* st) {
  const Pattern& P = h->P;
  hipStream_t s = h->stream;
  HIPC(hipEventRecord(h->ev[0], s));
  launch_assemble(s, P.n_nodes, h->xyz_d.ptr, h->slice_ptr.ptr, h->row_len.ptr, h->s_col.ptr,
                  h->s_elem.ptr, h->active.ptr, h->mat, h->G, h->val.ptr, h->diag.ptr);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(h->ev[1], s));
  if (st) {
    HIPC(hipEventSynchronize(h->ev[1]));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    st->t_assemble_ms = ms;
  }
  return 0;
}

int post_impl(mfea_handle* h, double max_strain, double* total_force, int64_t* n_active,
              mfea_stats* st) {
  const Pattern& P = h->P;
  hipStream_t s = h->stream;
  HIPC(hipEventRecord(h->ev[4], s));
  launch_reaction(s, P.n_free, P.n_top, P.n_nodes, h->slice_ptr.ptr, h->row_len.ptr, h->s_col.ptr,
                  h->val.ptr, h->diag.ptr, h->G, h->x.ptr, h->partials.ptr, tix(h, 3),
                  h->red.ptr + 4);
  launch_stress(s, P.n_elems, h->e2n_d.ptr, h->xyz_d.ptr, h->x.ptr, h->mat, max_strain,
                h->active.ptr, h->stress.ptr, h->partials.ptr, tix(h, 4), h->red.ptr + 5);
  HIPC(hipGetLastError());
  HIPC(hipMemcpyAsync(h->h_red, h->red.ptr + 4, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPC(hipEventRecord(h->ev[5], s));
  HIPC(hipEventSynchronize(h->ev[5]));
  if (P.n_top == 0) h->h_red[0] = 0.0;
  if (P.n_elems == 0) h->h_red[1] = 0.0;
  if (total_force) *total_force = h->h_red[0];
  h->n_active = (int64_t)h->h_red[1];
  if (n_active) *n_active = h->n_active;
  if (st) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[4], h->ev[5]);
    st->t_post_ms = ms;
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
  for (auto& ev : h->poll) HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPC(hipHostMalloc(&h->h_state, 2 * sizeof(SolveState),
                     hipHostMallocMapped | hipHostMallocCoherent));
  HIPC(hipHostGetDevicePointer((void**)&h->d_host_state, h->h_state, 0));
  HIPC(hipHostMalloc(&h->h_red, 16 * sizeof(double), hipHostMallocDefault));
  std::memset(h->h_state, 0, 2 * sizeof(SolveState));
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
  for (auto& ev : h->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : h->poll)
    if (ev) (void)hipEventDestroy(ev);
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
  if (int rc = set_device(h)) return rc;
  h->N = n_nodes;
  h->Ecount = n_elems;
  h->xyz.assign(xyz, xyz + 3 * n_nodes);
  h->e2n.assign(e2n, e2n + 2 * n_elems);
  h->mesh_flags = flags;
  h->has_mesh = true;
  h->dirty = true;
  h->active_host.clear();
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
  if (!h->dirty && h->Ecount) {
    h->active_host.resize(h->Ecount);
    (void)hipMemcpy(h->active_host.data(), h->active.ptr, h->Ecount, hipMemcpyDeviceToHost);
  }
  h->top.assign(top, top + n_top);
  h->bot.assign(bot, bot + n_bot);
  h->dirty = true;
  return 0;
}

int mfea_set_active(mfea_handle* h, const uint8_t* active) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  if (h->Ecount == 0) return 0;
  if (active) {
    std::vector<uint8_t> a(active, active + h->Ecount);
    for (auto& v : a) v = v ? 1 : 0;
    HIPC(hipMemcpy(h->active.ptr, a.data(), h->Ecount, hipMemcpyHostToDevice));
  } else {
    HIPC(hipMemset(h->active.ptr, 1, h->Ecount));
  }
  return 0;
}

int mfea_assemble(mfea_handle* h) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  if (int rc = assemble_impl(h, nullptr)) return rc;
  HIPC(hipStreamSynchronize(h->stream));
  return 0;
}

int mfea_solve(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
               mfea_stats* st) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  mfea_solve_opts o = opts ? *opts : default_opts();
  if (st) std::memset(st, 0, sizeof(*st));
  return solve_impl(h, dy_top, dy_bot, &o, st);
}

int mfea_post(mfea_handle* h, double max_strain, double* total_force, int64_t* n_active) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  return post_impl(h, max_strain, total_force, n_active, nullptr);
}

int mfea_step(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
              double max_strain, double* total_force, int64_t* n_active, mfea_stats* st) {
  if (!h) return fail(MFEA_EINVAL, "NULL handle");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  mfea_solve_opts o = opts ? *opts : default_opts();
  if (st) std::memset(st, 0, sizeof(*st));
  if (int rc = assemble_impl(h, nullptr)) return rc;
  int rc = solve_impl(h, dy_top, dy_bot, &o, st);
  if (rc && rc != MFEA_EMAXIT && rc != MFEA_EBREAKDOWN) return rc;
  if (rc) return rc;  // the reference stops the step loop here (src/fea_petsc.cpp:346-354)
  if (int rc2 = post_impl(h, max_strain, total_force, n_active, st)) return rc2;
  if (st) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, h->ev[0], h->ev[1]);
    st->t_assemble_ms = ms;
  }
  return 0;
}

int mfea_get_displacement(mfea_handle* h, double* U) {
  if (!h || !U) return fail(MFEA_EINVAL, "NULL argument");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  const int64_t N = h->P.n_nodes;
  std::vector<double> xp(3 * N);
  if (N) HIPC(hipMemcpy(xp.data(), h->x.ptr, 3 * N * sizeof(double), hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < N; ++i)
    for (int a = 0; a < 3; ++a) U[3 * (int64_t)h->P.perm[i] + a] = xp[3 * i + a];
  return 0;
}

int mfea_get_stress(mfea_handle* h, double* stress) {
  if (!h || !stress) return fail(MFEA_EINVAL, "NULL argument");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  if (h->Ecount)
    HIPC(hipMemcpy(stress, h->stress.ptr, h->Ecount * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int mfea_get_active(mfea_handle* h, uint8_t* active) {
  if (!h || !active) return fail(MFEA_EINVAL, "NULL argument");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  if (h->Ecount) HIPC(hipMemcpy(active, h->active.ptr, h->Ecount, hipMemcpyDeviceToHost));
  return 0;
}

int mfea_element_stiffness(mfea_handle* h, int64_t n, const double* p1s, const double* p2s,
                           double E, double A, double I, double* Ke, double* L) {
  if (!h || n < 0 || (n && (!p1s || !p2s || !Ke || !L))) return fail(MFEA_EINVAL, "bad argument");
  if (int rc = set_device(h)) return rc;
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
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  const Pattern& P = h->P;
  const int64_t N = P.n_nodes, E = P.n_elems;
  std::vector<double> diag6(6 * N), val6(6 * h->G);
  std::vector<uint8_t> act(E);
  if (N) HIPC(hipMemcpy(diag6.data(), h->diag.ptr, 6 * N * sizeof(double), hipMemcpyDeviceToHost));
  if (h->G) HIPC(hipMemcpy(val6.data(), h->val.ptr, 6 * h->G * sizeof(double), hipMemcpyDeviceToHost));
  if (E) HIPC(hipMemcpy(act.data(), h->active.ptr, E, hipMemcpyDeviceToHost));
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
  if (int rc = set_device(h)) return rc;
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
  if (h->partials.n < (size_t)(4 * maxg)) HIPC(h->partials.alloc(4 * (maxg + 16)));
  HIPC(h->red.alloc(16));
  HIPC(h->tickets.alloc(kTicketSets * kTicketStride));
  HIPC(h->slots.alloc(kMaxChunk + 2));
  HIPC(h->state.alloc(1));
  if (h->dirty) HIPC(hipMemsetAsync(h->tickets.ptr, 0, kTicketSets * kTicketStride * sizeof(unsigned), s));
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
                      h->partials.ptr, tix(h, 5), h->red.ptr);
  launch_init_finalize(s, h->red.ptr, o.rtol, o.atol, o.norm, o.max_it, o.reg, h->slots.ptr,
                       h->state.ptr);
  HIPC(hipGetLastError());
  HIPC(hipEventRecord(h->ev[2], s));
  const int chunk = o.chunk > 0 ? std::min(o.chunk, kMaxChunk) : 32;
  SolveState fin;
  int rc = drive_chunks(
      h, chunk, o.max_it,
      [&]() -> int {
        for (int j = 0; j < chunk; ++j) {
          launch_spmv_csr(s, j, n, h->c_indptr.ptr, h->c_indices.ptr, h->c_data.ptr,
                          h->c_known.ptr, o.reg, h->c_p.ptr, h->c_q.ptr, h->slots.ptr,
                          h->state.ptr, h->partials.ptr, tix(h, 6));
          launch_update(s, j, n, 0, h->c_x.ptr, h->c_r.ptr, h->c_p.ptr, h->c_q.ptr, h->c_dinv.ptr,
                        h->slots.ptr, h->state.ptr, h->partials.ptr, tix(h, 7));
          launch_direction(s, j, n, 0, h->c_r.ptr, h->c_p.ptr, h->c_dinv.ptr, h->slots.ptr,
                           h->state.ptr);
        }
        launch_advance(s, chunk, h->slots.ptr, h->state.ptr);
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
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  const Pattern& P = h->P;
  std::memset(info, 0, sizeof(*info));
  info->n_nodes = P.n_nodes;
  info->n_elems = P.n_elems;
  info->n_free_nodes = P.n_free;
  info->n_top = P.n_top;
  info->n_known = P.n_known;
  info->n_slices = P.n_slices();
  info->n_slots = h->G;
  int64_t inc = 0;
  for (int64_t i = 0; i < P.n_free; ++i) inc += P.row_len[i];
  info->free_incidences = inc;
  info->planar = P.planar ? 1 : 0;
  info->cg_lanes = use_ell(h) ? 1 : 0;
  info->n_lanes = h->ell_ok ? h->L.n_lanes : 0;
  int64_t halo = 0;
  if (h->ell_ok)
    for (int32_t pt : h->L.partner) halo += pt >= 0;
  info->n_halo = halo;
  return 0;
}

// iteration 0 of the active CG kernel (profiling / tracing)
static void launch_iter0(mfea_handle* h, int pc, unsigned long long* trace) {
  if (use_ell(h))
    launch_ell_iter(h->stream, 0, ell_op(h), pc, ell_vecs(h), h->slots.ptr, h->state.ptr,
                    h->cg_part.ptr, trace);
  else
    launch_cg_iter(h->stream, 0, sell_op(h), pc, cg_vecs(h), h->slots.ptr, h->state.ptr,
                   h->cg_part.ptr, trace);
}

int mfea_profile_iteration(mfea_handle* h, int precond, int reps, double* avg_ms) {
  if (!h || !avg_ms || reps <= 0) return fail(MFEA_EINVAL, "bad argument");
  if (int rc = set_device(h)) return rc;
  if (int rc = ensure_built(h)) return rc;
  hipStream_t s = h->stream;
  const int pc = precond == MFEA_PC_BLOCK_JACOBI ? 1 : 0;
  // Running state with tol 0: slots[0] = INIT and parity-0 partials of 1, so
  // γ = δ = ‖r‖² = ‖u‖² = G > 0, α = 1, β = 0.  Every launch is iteration 0
  // (same parity), so it reads the same buffers and does identical work
  // (including all stores); only x and p drift.
  const double ones[2] = {1.0, 1.0};
  HIPC(hipMemcpyAsync(h->red.ptr + 8, ones, sizeof(ones), hipMemcpyHostToDevice, s));
  launch_cg_init_finalize(s, h->red.ptr + 8, 0.0, 0.0, 0, 1 << 30, 1e-12, h->state.ptr);
  std::vector<double> pones(4 * kCgMaxPartials, 1.0);
  HIPC(hipMemcpyAsync(h->cg_part.ptr, pones.data(), pones.size() * sizeof(double),
                      hipMemcpyHostToDevice, s));
  Slot s0;
  std::memset(&s0, 0, sizeof(s0));
  s0.flag = kInit;
  HIPC(hipMemcpyAsync(h->slots.ptr, &s0, sizeof(s0), hipMemcpyHostToDevice, s));
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
  if (int rc = mfea_profile_iteration(h, precond, 20, &ms)) return rc;  // same running state
  hipStream_t s = h->stream;
  const int64_t g = cg_grid(use_ell(h) ? h->L.n_lanes : h->P.n_free);
  const int64_t nw = g * (cg_block_size(0) / 64);
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

int mfea_dist_unique_id(uint8_t* unique_id) {
  (void)unique_id;
  return fail(MFEA_ESTATE, "multi-GPU path not built in this version");
}

int mfea_dist_init(mfea_handle* h, int rank, int world, const uint8_t* unique_id) {
  (void)h;
  (void)rank;
  (void)world;
  (void)unique_id;
  return fail(MFEA_ESTATE, "multi-GPU path not built in this version");
}

}  // extern "C"
