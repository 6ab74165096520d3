// amg_deep.hip — the deep levels of the SA-AMG V-cycle (amg.hip) in ONE
// persistent launch.
//
// Below level 0 every V-cycle step of a level is a small sweep: at C3
//  the 13 launches of levels 1–3 and the single-workgroup
// tail take ≈ 70 µs of the 116 µs iteration while moving ≈ 12 % of its bytes —
// each launch is a kernel boundary (≈ 1.5 µs) plus its own chain of three
// dependent loads (slice pointer → column → vector gather) behind a cold
// start.  Here the levels [l0, nlev) run as phases of one launch of G
// workgroups (1024 threads, at most one per CU, all resident: G ≤ 256), each
// phase a grid-stride sweep of one level step exactly as the per-level kernels
// compute it (same lanes per row, same slot order, same butterfly: the cycle's
// output is bitwise the per-level launches'), the phases separated by grid
// barriers instead of kernel boundaries:
//   down   t_l = b_l − A_l x_l                       (resid)
//          b_{l+1} = R_l t_l, x_{l+1} = s D⁻¹ b_{l+1}  (restrict)
//   up     x_l += P_l e_{l+1}                       (prolong)
//          e_l = x_l + ω D⁻¹ (b_l − A_l x_l)        (post)
//
// Hand-offs between workgroups (MI355X_MICROARCH.md § visibility, Valid
// forms, the first table row): the V-cycle vectors b, x, t, e of these levels
// are the only bytes written in the launch, and EVERY store of them is an
// agent-scope (sc1, write-through) store and EVERY load of them an agent-scope
// (sc1, L1-bypassing) load; the operators are read-only here and use plain
// loads.  A barrier: every wave drains its stores (s_waitcnt vmcnt(0)), the
// workgroup meets, one lane adds 1 to its shard of an arrival counter (agent
// atomic; 8 shards by blockIdx & 7, so ≈ G/8 arrivals serialise per word), and
// wave 0 polls all shards with sc1 loads until the phase's target; the other
// waves wait at the workgroup barrier it then joins.  The counters count up
// within a launch and are returned to zero by the last workgroup to finish
// (every workgroup has passed its last poll by then); spins are bounded and a
// give-up sets a sticky timeout word (never expected: the grid is resident).
#include "amg_dev.hpp"

namespace mfea {

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned gu32_t;

// A V-cycle vector handed between workgroups inside the launch: loads and
// stores through it are agent-scope (found by ADL from amg_dev.hpp's row
// products, whose gathers take either a plain pointer or this).
struct Coh {
  float* p;
};
template <int ND, class C>
__device__ __forceinline__ void vload(Coh v, int64_t i, C* o) {
  if constexpr (ND == 2) {
    const unsigned long long r =
        __hip_atomic_load((gu64_t*)(v.p + 2 * i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    o[0] = (C)__uint_as_float((unsigned)r);
    o[1] = (C)__uint_as_float((unsigned)(r >> 32));
  } else {
#pragma unroll
    for (int a = 0; a < ND; ++a)
      o[a] = (C)__uint_as_float(
          __hip_atomic_load((gu32_t*)(v.p + ND * i + a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
}
template <int ND, class C>
__device__ __forceinline__ void vstore(Coh v, int64_t i, const C* o) {
  if constexpr (ND == 2) {
    const unsigned long long r = (unsigned long long)__float_as_uint((float)o[0]) |
                                 ((unsigned long long)__float_as_uint((float)o[1]) << 32);
    __hip_atomic_store((gu64_t*)(v.p + 2 * i), r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
#pragma unroll
    for (int a = 0; a < ND; ++a)
      __hip_atomic_store((gu32_t*)(v.p + ND * i + a), __float_as_uint((float)o[a]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

namespace {

constexpr int kDeepBS = 1024;
constexpr unsigned kDeepSpinMax = 1u << 16;  // ≈ 0.1 s of polling
constexpr int kShardWords = 32;              // 128 B between counter words
constexpr int kDoneWord = 8 * kShardWords;
constexpr int kTimeoutWord = kDeepTimeoutWord;
static_assert(kTimeoutWord == 9 * kShardWords && kTimeoutWord < kDeepBarWords, "barrier words");

// the f32 V-cycle operators of one level (SELL-64 pattern + blocks)
struct DeepMat {
  const int32_t* sptr;
  const int32_t* col;
  const float* val;
  int64_t n;
};
struct DeepLev {
  DeepMat A, P, R;  // P, R: not on the coarsest level
  const float* dinv;
  const double* omega;
  float *b, *x, *t, *e;
  int coarsest;
  int sa, sr;  // lanes per row: the operator A (1, 2, 4), the restriction (1, 2, 4, 8)
};
// the levels travel by value in the kernel arguments (their pointers are then
// known to be global, not flat)
struct DeepArgs {
  DeepLev lev[kDeepMaxLev];
  int nl;  // levels: lev[k] = level l0 + k
  const int32_t* gate;
  unsigned* bar;
};

__device__ __forceinline__ void dslice(const DeepMat& M, int64_t row, int64_t& base, int& w) {
  const int s = __builtin_amdgcn_readfirstlane((int)(row >> 6));
  const int a = M.sptr[s], b = M.sptr[s + 1];
  base = (int64_t)a * 64 + (row & 63);
  w = b - a;
}

// the grid barrier (header); target = phases so far × G.  dead: a wait of this
// workgroup (or of an earlier launch on these words) gave up — arrive, never wait
__device__ __forceinline__ void deep_sync(unsigned* bar, unsigned target, bool& dead) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have landed
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (lane == 0)
      __hip_atomic_fetch_add((gu32_t*)(bar + kShardWords * (blockIdx.x & 7)), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spin = 0; !dead; ++spin) {
      unsigned v = lane < 8 ? __hip_atomic_load((gu32_t*)(bar + kShardWords * lane), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : 0u;
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      if ((unsigned)__builtin_amdgcn_readfirstlane(v) >= target) break;
      if (spin >= kDeepSpinMax) {
        if (lane == 0)
          __hip_atomic_store((gu32_t*)(bar + kTimeoutWord), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        dead = true;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // no instruction: keeps the compiler from moving the phase's loads above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}

// the last workgroup past its last barrier zeroes the counters for the next launch
__device__ __forceinline__ void deep_done(unsigned* bar) {
  if (threadIdx.x != 0) return;
  const unsigned old =
      __hip_atomic_fetch_add((gu32_t*)(bar + kDoneWord), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == gridDim.x) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      __hip_atomic_store((gu32_t*)(bar + kShardWords * k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu32_t*)(bar + kDoneWord), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- phases: rows [0, n), S lanes per row, grid-stride; a wave's rows share
// one SELL slice (S divides 64), and a wave leaves together ---------------------
template <int ND, int S>
__device__ __forceinline__ void deep_resid(const DeepLev& L, int64_t tid, int64_t T) {
  const int64_t n = L.A.n;
  for (int64_t t = tid;; t += T) {
    const int64_t i = t / S;
    const int sub = (int)(t % S);
    if (i - (int64_t)((threadIdx.x & 63) / S) >= n) break;
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    dslice(L.A, ii, base, w);
    float y[ND];
    vload<ND>(Coh{L.b}, ii, y);
    if (sub != 0) {
#pragma unroll
      for (int a = 0; a < ND; ++a) y[a] = 0.0f;
    }
    if constexpr (S == 1) sell_mac<ND, true, 2>(L.A.col, L.A.val, 0, base, w, Coh{L.x}, y);
    else sell_mac_sub<ND, S, true>(L.A.col, L.A.val, base, w, sub, Coh{L.x}, y);
    if (i < n && sub == 0) vstore<ND>(Coh{L.t}, i, y);
  }
}

template <int ND, int S>
__device__ __forceinline__ void deep_restrict(const DeepLev& L, const DeepLev& N, int64_t tid, int64_t T) {
  const int64_t n = L.R.n;
  const float sc = N.coarsest ? 1.0f : (float)amg_omega(N.omega);
  for (int64_t t = tid;; t += T) {
    const int64_t I = t / S;
    const int sub = (int)(t % S);
    if (I - (int64_t)((threadIdx.x & 63) / S) >= n) break;
    const int64_t Ic = I < n ? I : n - 1;
    int64_t base;
    int w;
    dslice(L.R, Ic, base, w);
    float Di[ND * ND], bc[ND];
    dinv_load<ND>(N.dinv, Ic, Di);
#pragma unroll
    for (int a = 0; a < ND; ++a) bc[a] = 0.0f;
    if constexpr (S == 1) sell_mac<ND, false, 2>(L.R.col, L.R.val, 0, base, w, Coh{L.t}, bc);
    else sell_mac_sub<ND, S, false>(L.R.col, L.R.val, base, w, sub, Coh{L.t}, bc);
    if (I < n && sub == 0) {
      vstore<ND>(Coh{N.b}, I, bc);
      float xn[ND];
      dinv_mul<ND>(Di, sc, bc, xn);
      vstore<ND>(Coh{N.x}, I, xn);
    }
  }
}

template <int ND>
__device__ __forceinline__ void deep_prolong(const DeepLev& L, const DeepLev& N, int64_t tid, int64_t T) {
  const int64_t n = L.P.n;
  const Coh src{N.coarsest ? N.x : N.e};
  for (int64_t i = tid;; i += T) {
    if (i - (int64_t)(threadIdx.x & 63) >= n) break;
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    dslice(L.P, ii, base, w);
    float x[ND];
    vload<ND>(Coh{L.x}, ii, x);
    sell_mac<ND, false>(L.P.col, L.P.val, 0, base, w, src, x);
    if (i < n) vstore<ND>(Coh{L.x}, i, x);
  }
}

template <int ND, int S>
__device__ __forceinline__ void deep_post(const DeepLev& L, int64_t tid, int64_t T) {
  const int64_t n = L.A.n;
  const float om = (float)amg_omega(L.omega);
  for (int64_t t = tid;; t += T) {
    const int64_t i = t / S;
    const int sub = (int)(t % S);
    if (i - (int64_t)((threadIdx.x & 63) / S) >= n) break;
    const int64_t ii = i < n ? i : n - 1;
    int64_t base;
    int w;
    dslice(L.A, ii, base, w);
    float y[ND], x[ND], d[ND], Di[ND * ND];
    vload<ND>(Coh{L.b}, ii, y);
    vload<ND>(Coh{L.x}, ii, x);
    dinv_load<ND>(L.dinv, ii, Di);
    if (sub != 0) {
#pragma unroll
      for (int a = 0; a < ND; ++a) y[a] = 0.0f;
    }
    if constexpr (S == 1) sell_mac<ND, true, 2>(L.A.col, L.A.val, 0, base, w, Coh{L.x}, y);
    else sell_mac_sub<ND, S, true>(L.A.col, L.A.val, base, w, sub, Coh{L.x}, y);
    dinv_mul<ND>(Di, om, y, d);
#pragma unroll
    for (int a = 0; a < ND; ++a) x[a] += d[a];
    if (i < n && sub == 0) vstore<ND>(Coh{L.e}, i, x);
  }
}

// the lane count is launch-uniform: one branch per phase
template <int ND>
__device__ __forceinline__ void deep_resid_any(const DeepLev& L, int64_t tid, int64_t T) {
  if (L.sa == 4) deep_resid<ND, 4>(L, tid, T);
  else if (L.sa == 2) deep_resid<ND, 2>(L, tid, T);
  else deep_resid<ND, 1>(L, tid, T);
}
template <int ND>
__device__ __forceinline__ void deep_post_any(const DeepLev& L, int64_t tid, int64_t T) {
  if (L.sa == 4) deep_post<ND, 4>(L, tid, T);
  else if (L.sa == 2) deep_post<ND, 2>(L, tid, T);
  else deep_post<ND, 1>(L, tid, T);
}
template <int ND>
__device__ __forceinline__ void deep_restrict_any(const DeepLev& L, const DeepLev& N, int64_t tid, int64_t T) {
  if (L.sr == 8) deep_restrict<ND, 8>(L, N, tid, T);
  else if (L.sr == 4) deep_restrict<ND, 4>(L, N, tid, T);
  else if (L.sr == 2) deep_restrict<ND, 2>(L, N, tid, T);
  else deep_restrict<ND, 1>(L, N, tid, T);
}

template <int ND>
__global__ __launch_bounds__(kDeepBS) void k_amg_deep(const DeepArgs a) {
  if (gated(a.gate)) return;  // converged: the whole grid leaves before any barrier
  const int64_t tid = xcd_block() * kDeepBS + threadIdx.x;
  const int64_t T = (int64_t)gridDim.x * kDeepBS;
  const unsigned G = gridDim.x;
  bool dead = __hip_atomic_load((gu32_t*)(a.bar + kTimeoutWord), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  unsigned ph = 0;
  for (int k = 0; k + 1 < a.nl; ++k) {
    deep_resid_any<ND>(a.lev[k], tid, T);
    deep_sync(a.bar, ++ph * G, dead);
    deep_restrict_any<ND>(a.lev[k], a.lev[k + 1], tid, T);
    deep_sync(a.bar, ++ph * G, dead);
  }
  for (int k = a.nl - 2; k >= 0; --k) {
    deep_prolong<ND>(a.lev[k], a.lev[k + 1], tid, T);
    deep_sync(a.bar, ++ph * G, dead);
    deep_post_any<ND>(a.lev[k], tid, T);
    if (k > 0) deep_sync(a.bar, ++ph * G, dead);
  }
  deep_done(a.bar);
}

DeepMat dmat(const AmgMatD& M) { return DeepMat{M.sptr, M.col, M.val32, M.n}; }
bool whole(const AmgMatD& M) { return M.rg.lo == 0 && M.rg.hi == M.n; }

}  // namespace

bool amg_deep_fits(const AmgLevD* lev, int nlev, int l0) {
  const int nl = nlev - l0;
  if (l0 < 1 || nl < 2 || nl > kDeepMaxLev) return false;
  for (int k = 0; k < nl; ++k) {
    const AmgLevD& L = lev[l0 + k];
    if (!whole(L.A)) return false;  // a level split over ranks: its own launches
    if (!L.coarsest && (!whole(L.P) || !whole(L.R))) return false;
    // the sc1 vector accesses are ND-wide (8 B at ND = 2): aligned rows
    for (const float* v : {L.b, L.x, L.t, L.e})
      if (v && ((uintptr_t)v & 7u)) return false;
  }
  return true;
}

bool launch_amg_deep(hipStream_t s, int nd, const AmgLevD* lev, int nlev, int l0, const AmgCg& cg,
                     const int32_t* gate) {
  if (!cg.deep_bar || !amg_deep_fits(lev, nlev, l0)) return false;
  DeepArgs a{};
  a.nl = nlev - l0;
  a.gate = gate;
  a.bar = cg.deep_bar;
  for (int k = 0; k < a.nl; ++k) {
    const AmgLevD& L = lev[l0 + k];
    DeepLev& d = a.lev[k];
    d.A = dmat(L.A);
    d.dinv = L.dinv32;
    d.omega = L.omega;
    d.b = L.b;
    d.x = L.x;
    d.t = L.t;
    d.e = L.e;
    d.coarsest = L.coarsest;
    d.sa = amg_op_lanes(L);
    if (!L.coarsest) {
      d.P = dmat(L.P);
      d.R = dmat(L.R);
      d.sr = amg_restrict_lanes(L);
    }
  }
  int g = cg.deep_wgs > 0 ? cg.deep_wgs : 128;
  g = g < 8 ? 8 : (g > 256 ? 256 : g);  // at most one 1024-thread workgroup per CU: all resident
  if (nd == 2) hipLaunchKernelGGL(k_amg_deep<2>, dim3(g), dim3(kDeepBS), 0, s, a);
  else hipLaunchKernelGGL(k_amg_deep<3>, dim3(g), dim3(kDeepBS), 0, s, a);
  return true;
}

}  // namespace mfea
