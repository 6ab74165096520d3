// symbolic.cpp — see symbolic.hpp.  Pure host C++ (no HIP), unit-tested on CPU.
#include "symbolic.hpp"

#include <algorithm>
#include <array>
#include <numeric>

namespace mfea {

std::string build_pattern(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                          bool skip_invalid, const std::vector<int64_t>& top,
                          const std::vector<int64_t>& bot, int sort_window, Pattern& P) {
  if (N < 0 || E < 0) return "negative mesh size";
  if (N > INT32_MAX / 4 || E > INT32_MAX / 4) return "mesh too large for int32 indexing";
  P = Pattern();
  P.n_nodes = N;
  P.n_elems = E;
  P.elem_valid.assign(E, 1);
  for (int64_t e = 0; e < E; ++e) {
    int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a < 0 || a >= N || b < 0 || b >= N) {
      if (!skip_invalid)
        return "element " + std::to_string(e) + " references node out of range [0," +
               std::to_string(N) + ")";
      P.elem_valid[e] = 0;
    }
  }
  // ---- node classes: src/fea_solver.py:226-242 (bottom value overrides top)
  std::vector<uint8_t> code_orig(N, kFree);
  std::vector<uint8_t> in_top(N, 0), in_bot(N, 0);
  for (int64_t t : top) {
    if (t < 0 || t >= N) return "top grip node out of range";
    in_top[t] = 1;
  }
  for (int64_t b : bot) {
    if (b < 0 || b >= N) return "bottom grip node out of range";
    in_bot[b] = 1;
  }
  for (int64_t n = 0; n < N; ++n) code_orig[n] = in_bot[n] ? kBot : (in_top[n] ? kTop : kFree);

  // ---- degree (incident elements, self-loops excluded: they add exactly 0)
  std::vector<int32_t> deg(N, 0);
  for (int64_t e = 0; e < E; ++e) {
    if (!P.elem_valid[e]) continue;
    int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a == b) continue;
    deg[a]++;
    deg[b]++;
  }
  // ---- permutation: free rows first (original order, degree-sorted inside
  // windows of sort_window rows to keep SELL slices uniform), then the top grip
  // rows in top-list order (contiguous → coalesced reaction kernel), then
  // bottom-only rows.
  std::vector<int32_t> free_nodes;
  free_nodes.reserve(N);
  if (sort_window == kOrderDFS) {
    // Depth-first order over the free-node graph: the network is nearly a
    // forest of long hyphal chains, so DFS lays each chain out contiguously
    // and a row's neighbours are mostly rows i±1 — the SpMV gathers of a
    // wavefront then touch a handful of cache lines instead of 64.  (The
    // export order of the growth model interleaves all tips per time step.)
    std::vector<int32_t> aptr(N + 1, 0), adj;
    for (int64_t e = 0; e < E; ++e) {
      if (!P.elem_valid[e]) continue;
      const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
      if (a == b || code_orig[a] != kFree || code_orig[b] != kFree) continue;
      aptr[a + 1]++;
      aptr[b + 1]++;
    }
    for (int64_t n = 0; n < N; ++n) aptr[n + 1] += aptr[n];
    adj.resize(aptr[N]);
    std::vector<int32_t> fp(aptr.begin(), aptr.end() - 1);
    for (int64_t e = 0; e < E; ++e) {
      if (!P.elem_valid[e]) continue;
      const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
      if (a == b || code_orig[a] != kFree || code_orig[b] != kFree) continue;
      adj[fp[a]++] = (int32_t)b;
      adj[fp[b]++] = (int32_t)a;
    }
    std::vector<uint8_t> seen(N, 0);
    std::vector<int32_t> stack;
    for (int64_t s0 = 0; s0 < N; ++s0) {
      if (code_orig[s0] != kFree || seen[s0]) continue;
      stack.push_back((int32_t)s0);
      while (!stack.empty()) {
        const int32_t n = stack.back();
        stack.pop_back();
        if (seen[n]) continue;
        seen[n] = 1;
        free_nodes.push_back(n);
        // push in reverse so the lowest-numbered neighbour is visited first
        for (int32_t q = aptr[n + 1] - 1; q >= aptr[n]; --q)
          if (!seen[adj[q]]) stack.push_back(adj[q]);
      }
    }
  } else {
    for (int64_t n = 0; n < N; ++n)
      if (code_orig[n] == kFree) free_nodes.push_back((int32_t)n);
  }
  if (sort_window > 1) {
    for (size_t w0 = 0; w0 < free_nodes.size(); w0 += sort_window) {
      size_t w1 = std::min(free_nodes.size(), w0 + (size_t)sort_window);
      std::stable_sort(free_nodes.begin() + w0, free_nodes.begin() + w1,
                       [&](int32_t x, int32_t y) { return deg[x] > deg[y]; });
    }
  }
  P.perm = free_nodes;
  P.n_free = (int64_t)free_nodes.size();
  std::vector<uint8_t> placed(N, 0);
  for (int64_t t : top)
    if (!placed[t]) {
      placed[t] = 1;
      P.perm.push_back((int32_t)t);
    }
  P.n_top = (int64_t)P.perm.size() - P.n_free;
  for (int64_t b : bot)
    if (!placed[b] && code_orig[b] != kFree) {
      placed[b] = 1;
      P.perm.push_back((int32_t)b);
    }
  P.n_known = N - P.n_free;
  if ((int64_t)P.perm.size() != N) return "internal: permutation size mismatch";
  P.iperm.assign(N, -1);
  for (int64_t i = 0; i < N; ++i) P.iperm[P.perm[i]] = (int32_t)i;
  P.code.resize(N);
  for (int64_t i = 0; i < N; ++i) P.code[i] = code_orig[P.perm[i]];

  // ---- incidence lists per permuted row, in increasing element id
  // (= the order scipy's csr_matrix sums duplicates, src/fea_solver.py:93-105)
  std::vector<int32_t> ptr(N + 1, 0);
  for (int64_t i = 0; i < N; ++i) ptr[i + 1] = ptr[i] + deg[P.perm[i]];
  std::vector<int32_t> inc(ptr[N]);
  std::vector<int32_t> fill(ptr.begin(), ptr.end() - 1);
  for (int64_t e = 0; e < E; ++e) {
    if (!P.elem_valid[e]) continue;
    int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a == b) continue;
    inc[fill[P.iperm[a]]++] = (int32_t)e;
    inc[fill[P.iperm[b]]++] = (int32_t)e;
  }
  // (elements are visited in increasing id, so each list is already sorted)
  P.row_len.resize(N);
  for (int64_t i = 0; i < N; ++i) P.row_len[i] = ptr[i + 1] - ptr[i];

  // ---- SELL-64 slices
  const int64_t ns = (N + kSlice - 1) / kSlice;
  P.slice_ptr.assign(ns + 1, 0);
  for (int64_t s = 0; s < ns; ++s) {
    int32_t w = 0;
    for (int64_t i = s * kSlice; i < std::min(N, (s + 1) * kSlice); ++i) w = std::max(w, P.row_len[i]);
    P.slice_ptr[s + 1] = P.slice_ptr[s] + w;
  }
  const int64_t G = (int64_t)P.slice_ptr[ns] * kSlice;
  P.s_col.assign(G, -1);
  P.s_elem.assign(G, -1);
  for (int64_t i = 0; i < N; ++i) {
    const int64_t s = i / kSlice, lane = i % kSlice;
    for (int32_t k = 0; k < P.row_len[i]; ++k) {
      const int32_t e = inc[ptr[i] + k];
      const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
      const int64_t other = (P.perm[i] == a) ? b : a;
      const int64_t idx = ((int64_t)P.slice_ptr[s] + k) * kSlice + lane;
      P.s_col[idx] = P.iperm[other];
      P.s_elem[idx] = e;
    }
  }
  P.e2n_perm.assign(2 * E, -1);
  for (int64_t e = 0; e < E; ++e) {
    if (!P.elem_valid[e]) continue;
    P.e2n_perm[2 * e] = P.iperm[e2n[2 * e]];
    P.e2n_perm[2 * e + 1] = P.iperm[e2n[2 * e + 1]];
  }
  P.xyz_perm.resize(3 * N);
  P.planar = true;
  for (int64_t i = 0; i < N; ++i) {
    for (int c = 0; c < 3; ++c) P.xyz_perm[3 * i + c] = xyz[3 * P.perm[i] + c];
    if (xyz[3 * P.perm[i] + 2] != 0.0) P.planar = false;
  }
  return "";
}

// symmetric component index of (a,b): xx xy xz yy yz zz
static inline int sym(int a, int b) {
  if (a > b) std::swap(a, b);
  static const int m[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
  return m[a][b];
}

void export_csr(const Pattern& P, const std::vector<uint8_t>& active,
                const std::vector<double>& diag6, const std::vector<double>& val6,
                std::vector<int64_t>& indptr, std::vector<int32_t>& indices,
                std::vector<double>& data) {
  const int64_t N = P.n_nodes;
  const int64_t G = P.n_slots() * kSlice;
  indptr.assign(3 * N + 1, 0);
  indices.clear();
  data.clear();
  std::vector<std::pair<int32_t, int64_t>> blocks;  // (orig neighbour, slot idx) for one row
  for (int64_t n = 0; n < N; ++n) {
    const int64_t i = P.iperm[n];
    const int64_t s = i / kSlice, lane = i % kSlice;
    blocks.clear();
    bool any_active = false;
    for (int32_t k = 0; k < P.row_len[i]; ++k) {
      const int64_t idx = ((int64_t)P.slice_ptr[s] + k) * kSlice + lane;
      const int32_t e = P.s_elem[idx];
      if (!active[e]) continue;
      any_active = true;
      blocks.emplace_back(P.perm[P.s_col[idx]], idx);
    }
    // merge duplicates (multi-edges) in slot order = element order
    std::stable_sort(blocks.begin(), blocks.end(),
                     [](const auto& x, const auto& y) { return x.first < y.first; });
    // column blocks in ascending node order; the diagonal block goes in its place
    std::vector<std::pair<int32_t, std::array<double, 6>>> merged;
    bool diag_done = !any_active;
    for (size_t q = 0; q < blocks.size();) {
      const int32_t m = blocks[q].first;
      if (!diag_done && m > n) {
        std::array<double, 6> d;
        for (int c = 0; c < 6; ++c) d[c] = diag6[(int64_t)c * N + i];
        merged.emplace_back((int32_t)n, d);
        diag_done = true;
      }
      std::array<double, 6> v;
      for (int c = 0; c < 6; ++c) v[c] = val6[(int64_t)c * G + blocks[q].second];
      size_t r = q + 1;
      for (; r < blocks.size() && blocks[r].first == m; ++r)
        for (int c = 0; c < 6; ++c) v[c] += val6[(int64_t)c * G + blocks[r].second];
      merged.emplace_back(m, v);
      q = r;
    }
    if (!diag_done) {
      std::array<double, 6> d;
      for (int c = 0; c < 6; ++c) d[c] = diag6[(int64_t)c * N + i];
      merged.emplace_back((int32_t)n, d);
    }
    for (int a = 0; a < 3; ++a) {
      for (const auto& bm : merged)
        for (int b = 0; b < 3; ++b) {
          indices.push_back((int32_t)(3 * bm.first + b));
          data.push_back(bm.second[sym(a, b)]);
        }
      indptr[3 * n + a + 1] = (int64_t)indices.size();
    }
  }
}

}  // namespace mfea
