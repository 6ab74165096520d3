// symbolic.cpp — see symbolic.hpp.  Pure host C++ (no HIP), unit-tested on CPU.
#include "symbolic.hpp"

#include <algorithm>
#include <array>
#include <numeric>

namespace mfea {

std::string build_pattern(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                          bool skip_invalid, const std::vector<int64_t>& top,
                          const std::vector<int64_t>& bot, int sort_window, Pattern& P,
                          const std::vector<uint8_t>* ghost) {
  if (N < 0 || E < 0) return "negative mesh size";
  if (ghost && (int64_t)ghost->size() != N) return "internal: ghost mask size mismatch";
  const auto is_ghost = [&](int64_t n) { return ghost && (*ghost)[n]; };
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
  for (int64_t n = 0; n < N; ++n)
    code_orig[n] = in_bot[n] ? kBot : (in_top[n] ? kTop : (is_ghost(n) ? kGhost : kFree));

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
    if (!placed[t] && !is_ghost(t)) {
      placed[t] = 1;
      P.perm.push_back((int32_t)t);
    }
  P.n_top = (int64_t)P.perm.size() - P.n_free;
  for (int64_t b : bot)
    if (!placed[b] && code_orig[b] != kFree && !is_ghost(b)) {
      placed[b] = 1;
      P.perm.push_back((int32_t)b);
    }
  for (int64_t n = 0; n < N; ++n)
    if (is_ghost(n)) {
      P.perm.push_back((int32_t)n);
      P.n_ghost++;
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

// ---------------------------------------------------------------------------
std::string build_ell(const Pattern& P, Ell& L, const std::vector<int32_t>* elem_pair) {
  L = Ell();
  const int64_t nf = P.n_free;
  if (nf == 0) return "";
  const auto pos_of = [&](int64_t i, int k) {
    return ((int64_t)P.slice_ptr[i / kSlice] + k) * kSlice + i % kSlice;
  };
  // a slot to another partition's free node (multi-GPU)
  const auto remote = [&](int64_t pos) {
    const int32_t j = P.s_col[pos];
    return elem_pair && j >= nf && P.code[j] == kGhost;
  };
  // free-neighbour (and remote) slots of every free row, in slot (= element) order
  std::vector<int64_t> fptr(nf + 1, 0);
  for (int64_t i = 0; i < nf; ++i) {
    int c = 0;
    for (int k = 0; k < P.row_len[i]; ++k) c += P.s_col[pos_of(i, k)] < nf || remote(pos_of(i, k));
    fptr[i + 1] = fptr[i] + c;
  }
  std::vector<int64_t> fpos(fptr[nf]);
  for (int64_t i = 0, q = 0; i < nf; ++i)
    for (int k = 0; k < P.row_len[i]; ++k) {
      const int64_t pos = pos_of(i, k);
      if (P.s_col[pos] < nf || remote(pos)) fpos[q++] = pos;
    }
  for (int64_t q = 0; q < fptr[nf]; ++q)
    if (remote(fpos[q]) && (*elem_pair)[P.s_elem[fpos[q]]] < 0)
      return "internal: remote slot without an exchange pair";
  // Waves are filled greedily with consecutive rows: for a candidate wave
  // [a, b) a row's halo slots are exactly its slots to rows outside [a, b),
  // and its group needs max(⌈slots/3⌉, halo slots) lanes.  Take the longest
  // [a, b) whose groups fit 64 lanes (with a short look-ahead, since adding a
  // row can turn earlier halo slots local).
  std::vector<int32_t> need(nf, 1), lane(nf, -1), wave(nf, -1);
  const auto row_need = [&](int64_t i, int32_t w) {
    const int64_t ns = fptr[i + 1] - fptr[i];
    int64_t halo = 0;
    for (int64_t q = fptr[i]; q < fptr[i + 1]; ++q)
      halo += remote(fpos[q]) || wave[P.s_col[fpos[q]]] != w;
    return (int32_t)std::max<int64_t>({1, (ns + kEllSlots - 1) / kEllSlots, halo});
  };
  int64_t n_lanes = 0;
  int32_t w = 0;
  for (int64_t a = 0; a < nf; ++w) {
    int64_t best = -1;
    for (int64_t b = a + 1; b <= nf && b <= a + kSlice; ++b) {
      wave[b - 1] = w;
      int64_t total = 0;
      for (int64_t i = a; i < b; ++i) total += row_need(i, w);
      if (total <= kSlice) best = b;
      else if (best > 0 && b - best >= 8) break;
    }
    if (best < 0) return "a row needs more than 64 lanes (out-of-wave degree too high)";
    for (int64_t i = best; i < nf && i < a + kSlice; ++i) wave[i] = -1;
    int64_t pos = (int64_t)w * kSlice;
    for (int64_t i = a; i < best; ++i) {
      need[i] = row_need(i, w);
      lane[i] = (int32_t)pos;
      pos += need[i];
    }
    a = best;
    n_lanes = (int64_t)(w + 1) * kSlice;
  }
  if (n_lanes > INT32_MAX / 8) return "mesh too large for the lane layout";
  L.n_lanes = n_lanes;
  L.lane_row.assign(n_lanes, -1);
  L.row_lane = lane;
  L.info.assign(n_lanes, 0);
  L.code.assign(n_lanes, kEllNone | kEllNone << 8 | kEllNone << 16);
  L.partner.assign(n_lanes, -1);
  L.src_pos.assign(kEllSlots * n_lanes, -1);
  L.nbr_lane.assign(kEllSlots * n_lanes, -1);
  std::vector<int32_t> lane_of_pos(P.s_col.size(), -1);
  for (int64_t i = 0; i < nf; ++i) {
    const int32_t l0 = lane[i], g = need[i];
    L.lane_row[l0] = (int32_t)i;
    L.info[l0] = g - 1;
    for (int t = 1; t < g; ++t) L.info[l0 + t] = -t;
    // halo slots first (one per lane, slot 0), then the in-wave slots in order
    std::vector<int64_t> halo, local;
    for (int64_t q = fptr[i]; q < fptr[i + 1]; ++q)
      (remote(fpos[q]) || lane[P.s_col[fpos[q]]] / kSlice != l0 / kSlice ? halo : local)
          .push_back(fpos[q]);
    size_t hq = 0, lq = 0;
    for (int t = 0; t < g; ++t) {
      const int32_t l = l0 + t;
      for (int k = 0; k < kEllSlots; ++k) {
        int64_t pos = -1;
        bool is_halo = false;
        if (k == 0 && hq < halo.size()) {
          pos = halo[hq++];
          is_halo = true;
        } else if (lq < local.size()) {
          pos = local[lq++];
        }
        if (pos < 0) continue;
        const int32_t j = P.s_col[pos];
        const uint32_t src = is_halo ? kEllHalo : (uint32_t)(lane[j] % kSlice);
        L.code[l] = (L.code[l] & ~(0xFFu << (8 * k))) | src << (8 * k);
        L.src_pos[(int64_t)k * n_lanes + l] = (int32_t)pos;
        L.nbr_lane[(int64_t)k * n_lanes + l] = remote(pos) ? -1 : lane[j];
        lane_of_pos[pos] = l;
      }
    }
    if (hq != halo.size() || lq != local.size()) return "internal: group too small for its slots";
  }
  // halo partners: the lane holding the mirror slot (same element, seen from j)
  for (int64_t l = 0; l < n_lanes; ++l) {
    if ((L.code[l] & 0xFF) != kEllHalo) continue;
    const int64_t pos = L.src_pos[l];
    const int32_t j = P.s_col[pos], e = P.s_elem[pos];
    if (remote(pos)) {  // the peer rank's lane of the same cut element
      L.partner[l] = -2 - (*elem_pair)[e];
      continue;
    }
    const int32_t i = L.lane_row[l] >= 0 ? L.lane_row[l] : L.lane_row[l + L.info[l]];
    int32_t mirror = -1;
    for (int k = 0; k < P.row_len[j]; ++k) {
      const int64_t pj = pos_of(j, k);
      if (P.s_elem[pj] == e && P.s_col[pj] == i) mirror = lane_of_pos[pj];
    }
    if (mirror < 0 || (L.code[mirror] & 0xFF) != kEllHalo) return "internal: halo mirror missing";
    L.partner[l] = mirror;
  }
  const int64_t nw = n_lanes / kSlice;
  L.hrec.assign(n_lanes, -1);
  L.hmask.assign(nw, 0);
  L.hbase.assign(nw, 0);
  int64_t nr = 0;
  for (int64_t w = 0; w < nw; ++w) {
    L.hbase[w] = (int32_t)nr;
    for (int t = 0; t < kSlice; ++t) {
      const int64_t l = w * kSlice + t;
      if ((L.code[l] & 0xFF) == kEllHalo && L.partner[l] >= 0) {
        L.hmask[w] |= 1ull << t;
        L.hrec[l] = (int32_t)nr++;
      }
    }
  }
  L.n_hrec = nr;
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

std::string build_elem_colour(const Pattern& P, ElemColour& out) {
  out = ElemColour();
  const int64_t E = P.n_elems, N = P.n_nodes;
  out.pos.assign(2 * E, -1);
  for (int64_t r = 0; r < N; ++r) {
    const int64_t base = (int64_t)P.slice_ptr[r >> 6] * kSlice + (r & 63);
    for (int k = 0; k < P.row_len[r]; ++k) {
      const int64_t q = base + (int64_t)k * kSlice;
      const int32_t e = P.s_elem[q];
      if (e < 0) continue;
      const int side = P.e2n_perm[2 * e] == r ? 0 : 1;
      out.pos[2 * e + side] = (int32_t)q;
    }
  }
  for (int64_t e = 0; e < E; ++e)
    if ((out.pos[2 * e] >= 0) != (out.pos[2 * e + 1] >= 0)) return "element colouring: an element with one row slot";
  // elements with both slots, by their first row
  std::vector<std::pair<int64_t, int32_t>> order;
  order.reserve(E);
  for (int64_t e = 0; e < E; ++e)
    if (out.pos[2 * e] >= 0 && out.pos[2 * e + 1] >= 0)
      order.emplace_back(std::min(P.e2n_perm[2 * e], P.e2n_perm[2 * e + 1]), (int32_t)e);
  std::sort(order.begin(), order.end());
  std::vector<uint64_t> used(N, 0);
  std::vector<int8_t> col(E, -1);
  int colors = 0;
  for (const auto& re : order) {
    const int32_t e = re.second, a = P.e2n_perm[2 * e], b = P.e2n_perm[2 * e + 1];
    const uint64_t busy = used[a] | used[b];
    if (~busy == 0) return "element colouring: more than 64 colours";
    const int c = __builtin_ctzll(~busy);
    col[e] = (int8_t)c;
    used[a] |= 1ull << c;
    used[b] |= 1ull << c;
    colors = std::max(colors, c + 1);
  }
  out.colors = colors;
  std::vector<std::vector<int32_t>> by(colors);
  for (const auto& re : order) by[col[re.second]].push_back(re.second);  // (first-row order kept)
  out.cstart.assign(colors + 1, 0);
  for (int c = 0; c < colors; ++c) {
    const int64_t n = (int64_t)by[c].size(), padded = (n + kSlice - 1) / kSlice * kSlice;
    out.cstart[c + 1] = out.cstart[c] + (int32_t)padded;
    out.entry.insert(out.entry.end(), by[c].begin(), by[c].end());
    out.entry.insert(out.entry.end(), (size_t)(padded - n), -1);
  }
  return "";
}

}  // namespace mfea
