// ubench_chain.hip — the dependent-load chain of one small SELL sweep (the
// V-cycle's deep levels) on MI355X, graph-replayed back to back, each launch
// reading the vector the previous launch wrote:
//   sell : slice pointer (scalar) → column → x gather + block   (the engine's)
//   ell  : column → x gather + block (fixed width, no slice pointer)
//   pre  : block + pre-gathered x at the position (no column, no gather);
//          the producer scatters its outputs into the consumer's positions
// f32 2×2 blocks, W slots per row.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o ubench_chain tools/ubench_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int W = 4;

__global__ __launch_bounds__(256) void k_sell(const int* sptr, const int* col, const float4* val, const float2* x,
                                              float2* y, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i - (threadIdx.x & 63) >= n) return;
  const int s = __builtin_amdgcn_readfirstlane((int)(i >> 6));
  const long base = (long)sptr[s] * 64 + (i & 63);
  const int w = sptr[s + 1] - sptr[s];
  float2 acc = make_float2(0.f, 0.f);
  int c[W];
  for (int k = 0; k < W; ++k) c[k] = k < w ? col[base + 64L * k] : -1;
  float4 m[W];
  float2 xv[W];
  for (int k = 0; k < W; ++k) {
    m[k] = val[base + 64L * k];
    xv[k] = x[c[k] >= 0 ? c[k] : 0];
  }
  for (int k = 0; k < W; ++k)
    if (c[k] >= 0) {
      acc.x += m[k].x * xv[k].x + m[k].y * xv[k].y;
      acc.y += m[k].z * xv[k].x + m[k].w * xv[k].y;
    }
  if (i < n) y[i] = acc;
}

__global__ __launch_bounds__(256) void k_ell(const int* col, const float4* val, const float2* x, float2* y, long n,
                                             long n64) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float2 acc = make_float2(0.f, 0.f);
  int c[W];
  for (int k = 0; k < W; ++k) c[k] = col[i + n64 * k];
  float4 m[W];
  float2 xv[W];
  for (int k = 0; k < W; ++k) {
    m[k] = val[i + n64 * k];
    xv[k] = x[c[k] >= 0 ? c[k] : 0];
  }
  for (int k = 0; k < W; ++k)
    if (c[k] >= 0) {
      acc.x += m[k].x * xv[k].x + m[k].y * xv[k].y;
      acc.y += m[k].z * xv[k].x + m[k].w * xv[k].y;
    }
  y[i] = acc;
}

// pre-gathered: xp[k][i] = x[col[i][k]] written by the producer; this kernel
// scatters its own outputs into the next consumer's positions (tpos: W
// positions per row, -1 none)
__global__ __launch_bounds__(256) void k_pre(const float4* val, const float2* xp, const int* tpos, float2* yp,
                                             long n, long n64) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int tp[W];
  for (int k = 0; k < W; ++k) tp[k] = tpos[i + n64 * k];
  float2 acc = make_float2(0.f, 0.f);
  float4 m[W];
  float2 xv[W];
  for (int k = 0; k < W; ++k) {
    m[k] = val[i + n64 * k];
    xv[k] = xp[i + n64 * k];
  }
  for (int k = 0; k < W; ++k) {
    acc.x += m[k].x * xv[k].x + m[k].y * xv[k].y;
    acc.y += m[k].z * xv[k].x + m[k].w * xv[k].y;
  }
  for (int k = 0; k < W; ++k)
    if (tp[k] >= 0) yp[tp[k]] = acc;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nph = 64;
  for (long n : {1206L, 5273L, 23955L, 96592L}) {
    const long n64 = (n + 63) / 64 * 64, ns = n64 / 64;
    std::vector<int> sptr(ns + 1), col(n64 * W), tpos(n64 * W, -1);
    for (long k = 0; k <= ns; ++k) sptr[k] = (int)(k * W);
    unsigned long long r = 88172645463325252ull;
    std::vector<long> fill(n, 0);
    for (long i = 0; i < n64; ++i)
      for (int k = 0; k < W; ++k) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        long j = i + (long)(r % 64) - 32;
        j = i >= n ? -1 : (j < 0 ? 0 : (j >= n ? n - 1 : j));
        col[(i / 64) * 64 * W + 64L * k + (i & 63)] = (int)j;  // SELL position
      }
    // ELL layout: position i + n64·k; reuse the same columns
    std::vector<int> ecol(n64 * W);
    for (long i = 0; i < n64; ++i)
      for (int k = 0; k < W; ++k) ecol[i + n64 * k] = col[(i / 64) * 64 * W + 64L * k + (i & 63)];
    // transpose positions for the pre-gathered form: row j appears at (i, k)
    std::vector<int> cnt(n, 0);
    for (long i = 0; i < n; ++i)
      for (int k = 0; k < W; ++k) {
        const int j = ecol[i + n64 * k];
        if (j >= 0 && cnt[j] < W) tpos[j + n64 * cnt[j]++] = (int)(i + n64 * k);
      }
    int *d_sptr, *d_col, *d_ecol, *d_tpos;
    float4* d_val;
    float2 *x0, *x1, *p0, *p1;
    CK(hipMalloc(&d_sptr, (ns + 1) * 4));
    CK(hipMalloc(&d_col, n64 * W * 4));
    CK(hipMalloc(&d_ecol, n64 * W * 4));
    CK(hipMalloc(&d_tpos, n64 * W * 4));
    CK(hipMalloc(&d_val, n64 * W * 16));
    CK(hipMalloc(&x0, n64 * 8));
    CK(hipMalloc(&x1, n64 * 8));
    CK(hipMalloc(&p0, n64 * W * 8));
    CK(hipMalloc(&p1, n64 * W * 8));
    CK(hipMemcpy(d_sptr, sptr.data(), (ns + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_col, col.data(), n64 * W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ecol, ecol.data(), n64 * W * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tpos, tpos.data(), n64 * W * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_val, 0, n64 * W * 16));
    CK(hipMemset(x0, 0, n64 * 8));
    CK(hipMemset(x1, 0, n64 * 8));
    CK(hipMemset(p0, 0, n64 * W * 8));
    CK(hipMemset(p1, 0, n64 * W * 8));
    const dim3 g((unsigned)((n + 255) / 256)), b(256);
    float res[3];
    for (int v = 0; v < 3; ++v) {
      hipGraph_t gr;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int p = 0; p < nph; ++p) {
        if (v == 0) hipLaunchKernelGGL(k_sell, g, b, 0, s, d_sptr, d_col, d_val, p & 1 ? x1 : x0, p & 1 ? x0 : x1, n);
        else if (v == 1) hipLaunchKernelGGL(k_ell, g, b, 0, s, d_ecol, d_val, p & 1 ? x1 : x0, p & 1 ? x0 : x1, n, n64);
        else hipLaunchKernelGGL(k_pre, g, b, 0, s, d_val, p & 1 ? p1 : p0, d_tpos, p & 1 ? p0 : p1, n, n64);
      }
      CK(hipStreamEndCapture(s, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int rep = 0; rep < 20; ++rep) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[v] = ms * 1000.f / (20 * nph);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(gr));
    }
    std::printf("n %6ld  sell %.2f  ell %.2f  pre-gathered %.2f us/launch\n", n, res[0], res[1], res[2]);
    hipFree(d_sptr); hipFree(d_col); hipFree(d_ecol); hipFree(d_tpos); hipFree(d_val);
    hipFree(x0); hipFree(x1); hipFree(p0); hipFree(p1);
  }
  return 0;
}
