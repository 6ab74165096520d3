// amg_collapse.cpp — the compact V-cycle below level kc as ONE explicit
// operator (amg.hpp AmgCollapse).  Host C++, once per hierarchy.
//
// The compact cycle (amg.hip) maps a level's smoothed iterate x_k to its
// output e_k by  e_k = (2I − Ã_k) x_k + P̃_k e_{k+1},  x_{k+1} = R̂_k x_k, so
// the whole cycle below level k is the linear map
//     V_k = (2I − Ã_k) + P̃_k V_{k+1} R̂_k,     V_coarsest = I.
// On the deep levels V_k stays sparse (C3: 15 blocks per row at level 3, 55
// at level 2; C2: 50 at level 2) while the launches it replaces — two per
// level, each ≈ 4.7 µs of latency for kilobytes of data — dominate the
// iteration.  So the setup forms V_kc (through T_k = V_{k+1} R̂_k for every
// k ≥ kc, deepest first) and the cycle applies it with one SpMV.
//
// Here: the patterns of T_k and V_k in the device labels of the plan and the
// fixed-order index lists of their products (amg.hip k_amg_tv / k_amg_vv
// evaluate them every setup: pure gathers, bitwise reproducible).  kc is the
// highest level whose V fits the byte and product budgets.
#include <algorithm>
#include <array>
#include <numeric>

#include "amg.hpp"

namespace mfea {

namespace {

// a SELL pattern read row by row: per row its (column, position) entries in slot order
struct Rows {
  std::vector<int64_t> ptr{0};
  std::vector<int32_t> col, pos;
};
Rows rows_of(const SellPat& S, const std::vector<int32_t>* rowmap = nullptr) {
  const int64_t n = S.n;
  std::vector<int64_t> cnt(n + 1, 0);
  for (int64_t r = 0; r < n; ++r) cnt[(rowmap ? (*rowmap)[r] : r) + 1] += S.rlen[r];
  Rows R;
  R.ptr.assign(n + 1, 0);
  for (int64_t i = 0; i < n; ++i) R.ptr[i + 1] = R.ptr[i] + cnt[i + 1];
  R.col.resize(R.ptr[n]);
  R.pos.resize(R.ptr[n]);
  std::vector<int64_t> fill(R.ptr.begin(), R.ptr.end() - 1);
  for (int64_t r = 0; r < n; ++r) {
    const int64_t i = rowmap ? (*rowmap)[r] : r;
    for (int k = 0; k < S.rlen[r]; ++k) {
      const int64_t q = S.pos(r, k);
      R.col[fill[i]] = S.col[q];
      R.pos[fill[i]++] = (int32_t)q;
    }
  }
  return R;
}

// a product's rows before layout: per row its columns (ascending) and per
// entry the list of (a, b) operand positions in a fixed order
struct Prod {
  int64_t n = 0;
  std::vector<int64_t> ptr{0};
  std::vector<int32_t> col;
  std::vector<int64_t> lptr{0};  // per entry: its pairs [lptr[e], lptr[e+1])
  std::vector<int32_t> a, b;
  std::vector<int32_t> extra;    // per entry: Ã position (V only) or -1
  std::vector<int8_t> diag;      // per entry: on the diagonal (V only)
};

// SELL-64 of a product with rows relabelled by rperm (new = rperm[old]);
// epos[e] = position of entry e
void layout_prod(const Prod& M, const std::vector<int32_t>& rperm, SellPat& S, std::vector<int32_t>& epos) {
  const int64_t n = M.n;
  std::vector<int32_t> inv(n);
  for (int64_t r = 0; r < n; ++r) inv[rperm[r]] = (int32_t)r;
  S = SellPat();
  S.n = n;
  const int64_t ns = (n + 63) / 64;
  S.sptr.assign(ns + 1, 0);
  S.rlen.assign(n, 0);
  int64_t slots = 0;
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t r = 64 * s; r < std::min<int64_t>(n, 64 * s + 64); ++r) {
      const int64_t len = M.ptr[inv[r] + 1] - M.ptr[inv[r]];
      S.rlen[r] = (int32_t)len;
      w = std::max(w, len);
    }
    slots += w;
    S.sptr[s + 1] = (int32_t)slots;
  }
  S.col.assign(slots * 64, -1);
  epos.assign(M.col.size(), -1);
  for (int64_t r = 0; r < n; ++r) {
    const int64_t o = inv[r];
    for (int64_t e = M.ptr[o]; e < M.ptr[o + 1]; ++e) {
      const int64_t q = S.pos(r, (int)(e - M.ptr[o]));
      S.col[q] = M.col[e];
      epos[e] = (int32_t)q;
    }
  }
}

// rows sorted by descending length inside 4096-row windows (SELL-C-σ)
std::vector<int32_t> window_perm(const Prod& M) {
  const int64_t n = M.n;
  std::vector<int32_t> order(n), perm(n);
  std::iota(order.begin(), order.end(), 0);
  for (int64_t w0 = 0; w0 < n; w0 += 4096) {
    const int64_t w1 = std::min(n, w0 + 4096);
    std::stable_sort(order.begin() + w0, order.begin() + w1, [&](int32_t x, int32_t y) {
      return M.ptr[x + 1] - M.ptr[x] > M.ptr[y + 1] - M.ptr[y];
    });
  }
  for (int64_t k = 0; k < n; ++k) perm[order[k]] = (int32_t)k;
  return perm;
}

void to_lists(const Prod& M, const std::vector<int32_t>& epos, int64_t npos, PosList& L) {
  L = PosList();
  L.ptr.assign(npos + 1, 0);
  for (size_t e = 0; e < M.col.size(); ++e) L.ptr[epos[e] + 1] = (int32_t)(M.lptr[e + 1] - M.lptr[e]);
  for (int64_t q = 0; q < npos; ++q) L.ptr[q + 1] += L.ptr[q];
  L.a.resize(L.ptr[npos]);
  L.b.resize(L.ptr[npos]);
  for (size_t e = 0; e < M.col.size(); ++e) {
    int64_t d = L.ptr[epos[e]];
    for (int64_t t = M.lptr[e]; t < M.lptr[e + 1]; ++t, ++d) {
      L.a[d] = M.a[t];
      L.b[d] = M.b[t];
    }
  }
}

// C = X · Y over row lists (X rows: entries (col J, pos); Y rows by J): per
// output (i, j) the pairs (X pos, Y pos) in X-entry order; columns ascending.
// xid: X is the identity (pairs (-1, Y pos)).  mark: scratch of Y's width.
// False (C incomplete) as soon as C holds more than max_pairs pairs or
// max_cols entries: an over-budget level is rejected without being built.
bool spgemm(int64_t n, const Rows* X, const Rows& Y, int64_t /*ncols*/, Prod& C,
            int64_t max_pairs = INT64_MAX, int64_t max_cols = INT64_MAX) {
  C = Prod();
  C.n = n;
  // a row's products as (column, X pos, Y pos) in X-entry order, then a
  // stable sort by column: each output's pairs keep that order
  std::vector<std::array<int32_t, 3>> tr;
  for (int64_t i = 0; i < n; ++i) {
    tr.clear();
    auto add = [&](int32_t xp, int32_t J) {
      for (int64_t t = Y.ptr[J]; t < Y.ptr[J + 1]; ++t)
        if (Y.col[t] >= 0) tr.push_back({Y.col[t], xp, Y.pos[t]});
    };
    if (X) {
      for (int64_t t = X->ptr[i]; t < X->ptr[i + 1]; ++t)
        if (X->col[t] >= 0) add(X->pos[t], X->col[t]);
    } else {
      add(-1, (int32_t)i);
    }
    row_stable_sort(tr.begin(), tr.end(),
                     [](const std::array<int32_t, 3>& x, const std::array<int32_t, 3>& y) { return x[0] < y[0]; });
    for (size_t k = 0; k < tr.size();) {
      const int32_t j = tr[k][0];
      C.col.push_back(j);
      for (; k < tr.size() && tr[k][0] == j; ++k) {
        C.a.push_back(tr[k][1]);
        C.b.push_back(tr[k][2]);
      }
      C.lptr.push_back((int64_t)C.a.size());
    }
    C.ptr.push_back((int64_t)C.col.size());
    if ((int64_t)C.a.size() > max_pairs || (int64_t)C.col.size() > max_cols) return false;
  }
  return true;
}

}  // namespace

std::string build_amg_collapse(const AmgPlan& plan, int64_t max_bytes, int64_t max_pairs, int min_level,
                               AmgCollapse& out) {
  out = AmgCollapse();
  const int nlev = (int)plan.lev.size();
  if (nlev < 2 || plan.n_dist > 0) return "";
  const int nd = plan.nd;
  const int64_t bb = 4LL * nd * nd + 4;  // bytes per stored block (f32 + column)
  // deepest first: V_{c} = I, then V_k for k = c−1, c−2, … while within budget
  std::vector<AmgCollapse::Lev> levs;
  Rows vnext;  // V_{k+1} row by row, in level k+1 labels (positions in its SELL layout)
  bool have_v = false;
  int kc = 0;
  for (int k = nlev - 2; k >= std::max(1, min_level); --k) {
    const AmgLevel& L = plan.lev[k];
    if (L.PT.n != L.A.n || L.RT.n <= 0) break;  // no compact transfers on this level
    AmgCollapse::Lev C;
    C.k = k;
    // T_k = V_{k+1} R̂_k (rows: level k+1, cols: level k)
    const Rows RT = rows_of(L.RT, &L.rt_row);
    Prod T;
    if (!spgemm(L.RT.n, have_v ? &vnext : nullptr, RT, L.A.n, T, max_pairs)) break;
    // V_k = (2I − Ã_k) + P̃_k T_k
    const Rows PT = rows_of(L.PT, &L.pt_row);
    Prod V;
    const bool fits = spgemm(L.A.n, &PT, [&] {
      Rows TR;
      TR.ptr = T.ptr;
      TR.col = T.col;
      TR.pos.resize(T.col.size());
      std::iota(TR.pos.begin(), TR.pos.end(), 0);  // T entry index; mapped to positions below
      return TR;
    }(), L.A.n, V, max_pairs - (int64_t)T.a.size(), max_bytes / bb);
    if (!fits) break;  // over budget (V's merged pattern only grows)
    // merge A_k's pattern (Ã and the diagonal 2I) into V: A ⊆ V's pattern
    // in general, but not always (a row with no coarse coupling): add missing
    const Rows A = rows_of(L.A);
    {
      Prod W;
      W.n = V.n;
      std::vector<int32_t> apos;
      for (int64_t i = 0; i < V.n; ++i) {
        // both sorted ascending in column
        std::vector<std::pair<int32_t, int32_t>> arow;  // (col, A pos)
        for (int64_t t = A.ptr[i]; t < A.ptr[i + 1]; ++t)
          if (A.col[t] >= 0) arow.emplace_back(A.col[t], A.pos[t]);
        std::sort(arow.begin(), arow.end());
        size_t u = 0;
        int64_t e = V.ptr[i];
        while (e < V.ptr[i + 1] || u < arow.size()) {
          const int32_t cv = e < V.ptr[i + 1] ? V.col[e] : INT32_MAX;
          const int32_t ca = u < arow.size() ? arow[u].first : INT32_MAX;
          const int32_t c = std::min(cv, ca);
          W.col.push_back(c);
          W.extra.push_back(ca == c ? arow[u].second : -1);
          W.diag.push_back(c == i ? 1 : 0);
          if (cv == c) {
            for (int64_t t = V.lptr[e]; t < V.lptr[e + 1]; ++t) {
              W.a.push_back(V.a[t]);
              W.b.push_back(V.b[t]);
            }
            ++e;
          }
          if (ca == c) ++u;
          W.lptr.push_back((int64_t)W.a.size());
        }
        W.ptr.push_back((int64_t)W.col.size());
      }
      V = std::move(W);
    }
    const int64_t vbytes = (int64_t)V.col.size() * bb;
    const int64_t pairs = (int64_t)V.a.size() + (int64_t)T.a.size();
    if (!levs.empty() && (vbytes > max_bytes || pairs > max_pairs)) break;
    if (levs.empty() && (vbytes > max_bytes || pairs > max_pairs)) return "";  // not even the deepest fits
    // layouts: T in level k+1 order; V by row length inside windows
    std::vector<int32_t> idT(T.n), eT, eV;
    std::iota(idT.begin(), idT.end(), 0);
    layout_prod(T, idT, C.T, eT);
    const std::vector<int32_t> vperm = window_perm(V);
    layout_prod(V, vperm, C.V, eV);
    C.vrow.assign(V.n, 0);
    for (int64_t i = 0; i < V.n; ++i) C.vrow[vperm[i]] = (int32_t)i;
    // T's pairs: (V_{k+1} position or -1, R̂ position); V's pairs: (P̃ position, T entry → position)
    to_lists(T, eT, C.T.n_pos(), C.tl);
    for (auto& b : V.b) b = eT[b];
    to_lists(V, eV, C.V.n_pos(), C.vl);
    C.va.assign(C.V.n_pos(), -1);
    C.vdiag.assign(C.V.n_pos(), 0);
    for (size_t e = 0; e < V.col.size(); ++e) {
      C.va[eV[e]] = V.extra[e];
      C.vdiag[eV[e]] = V.diag[e] ? 1 : 0;
    }
    // V_k row by row (level k labels, SELL positions) for the level above
    vnext = Rows();
    vnext.ptr = V.ptr;
    vnext.col = V.col;
    vnext.pos.assign(eV.begin(), eV.end());
    have_v = true;
    kc = k;
    levs.push_back(std::move(C));
  }
  if (levs.empty()) return "";
  std::reverse(levs.begin(), levs.end());  // lev[0] = level kc
  out.kc = kc;
  out.lev = std::move(levs);
  return "";
}

// ---- levels 0 and 1 merged (amg.hpp AmgMerge) --------------------------------
namespace {
// Prod M plus, per row, the entries of E (an ext term) merged in by column:
// entries only in E get no pairs; extra[e] = E's position or -1
Prod merge_ext(const Prod& M, const Rows& E) {
  Prod W;
  W.n = M.n;
  for (int64_t i = 0; i < M.n; ++i) {
    std::vector<std::pair<int32_t, int32_t>> er;  // (col, E pos)
    for (int64_t t = E.ptr[i]; t < E.ptr[i + 1]; ++t)
      if (E.col[t] >= 0) er.emplace_back(E.col[t], E.pos[t]);
    std::sort(er.begin(), er.end());
    size_t u = 0;
    int64_t e = M.ptr[i];
    while (e < M.ptr[i + 1] || u < er.size()) {
      const int32_t cm = e < M.ptr[i + 1] ? M.col[e] : INT32_MAX;
      const int32_t ce = u < er.size() ? er[u].first : INT32_MAX;
      const int32_t c = std::min(cm, ce);
      W.col.push_back(c);
      W.extra.push_back(ce == c ? er[u].second : -1);
      if (cm == c) {
        for (int64_t t = M.lptr[e]; t < M.lptr[e + 1]; ++t) {
          W.a.push_back(M.a[t]);
          W.b.push_back(M.b[t]);
        }
        ++e;
      }
      if (ce == c) ++u;
      W.lptr.push_back((int64_t)W.a.size());
    }
    W.ptr.push_back((int64_t)W.col.size());
  }
  return W;
}
}  // namespace

std::string build_amg_merge(const AmgPlan& plan, const AmgCollapse& coll, AmgMerge& out) {
  out = AmgMerge();
  const int nlev = (int)plan.lev.size();
  if (coll.kc != 2 || nlev < 4 || plan.n_dist > 0) return "";
  const AmgLevel &L0 = plan.lev[0], &L1 = plan.lev[1];
  if (L0.PT.n != L0.A.n || L1.PT.n != L1.A.n || L0.RT.n <= 0 || L1.RT.n <= 0) return "";
  const int64_t n0 = L0.A.n, n1 = L1.A.n, n2 = plan.lev[2].A.n;
  const Rows R0 = rows_of(L0.RT, &L0.rt_row);  // level-1 rows → (level-0 col, R̂_0 position)
  const Rows A1 = rows_of(L1.A);               // level-1 rows → (level-1 col, Ã_1 position)
  const Rows R1 = rows_of(L1.RT, &L1.rt_row);  // level-2 rows → (level-1 col, R̂_1 position)
  const Rows P0 = rows_of(L0.PT, &L0.pt_row);  // level-0 rows → (level-1 col, P̃_0 position)
  const Rows P1 = rows_of(L1.PT, &L1.pt_row);  // level-1 rows → (level-2 col, P̃_1 position)
  // c_1 rows: 2 R̂_0 − Ã_1 R̂_0; x_2 rows: R̂_1 R̂_0; U: P̃_0 ∪ P̃_0 P̃_1
  Prod C1, Q, W;
  spgemm(n1, &A1, R0, n0, C1);
  C1 = merge_ext(C1, R0);
  spgemm(n2, &R1, R0, n0, Q);
  Q.extra.assign(Q.col.size(), -1);
  spgemm(n0, &P0, P1, n2, W);
  // U's columns are B indices: c_1 at [0, n1), e_2 at [n1 + n2, n1 + 2 n2)
  for (auto& c : W.col) c += (int32_t)(n1 + n2);
  Prod Uc = merge_ext(W, P0);  // (P̃_0's columns < n1 sort before W's)
  // layouts: c_1 rows and x_2 rows each by length inside windows, the c_1
  // part padded to whole slices (the setup tells the two by position)
  SellPat S1, S2;
  std::vector<int32_t> e1, e2;
  const std::vector<int32_t> p1 = window_perm(C1), p2 = window_perm(Q);
  layout_prod(C1, p1, S1, e1);
  layout_prod(Q, p2, S2, e2);
  const int64_t n1p = (n1 + 63) / 64 * 64, scratch = n1 + 2 * n2;
  SellPat& DQ = out.DQ;
  DQ.n = n1p + n2;
  DQ.sptr = S1.sptr;
  for (size_t k = 1; k < S2.sptr.size(); ++k) DQ.sptr.push_back(S1.sptr.back() + S2.sptr[k]);
  DQ.col = S1.col;
  DQ.col.insert(DQ.col.end(), S2.col.begin(), S2.col.end());
  DQ.rlen.assign(DQ.n, 0);
  for (int64_t r = 0; r < n1; ++r) DQ.rlen[r] = S1.rlen[r];
  for (int64_t r = 0; r < n2; ++r) DQ.rlen[n1p + r] = S2.rlen[r];
  if (DQ.n_pos() > INT32_MAX) return "";
  out.dq_split = S1.n_pos();
  out.dq_dst.assign(DQ.n, (int32_t)scratch);
  for (int64_t J = 0; J < n1; ++J) out.dq_dst[p1[J]] = (int32_t)J;
  for (int64_t J = 0; J < n2; ++J) out.dq_dst[n1p + p2[J]] = (int32_t)(n1 + J);
  for (auto& e : e2) e += (int32_t)out.dq_split;
  // one list set over DQ's positions (C_1's then Q's)
  {
    Prod M;  // C1 and Q as one product for to_lists (rows n1 + n2, entry order kept)
    M.n = n1 + n2;
    M.ptr = C1.ptr;
    for (size_t k = 1; k < Q.ptr.size(); ++k) M.ptr.push_back(C1.ptr.back() + Q.ptr[k]);
    M.col = C1.col;
    M.col.insert(M.col.end(), Q.col.begin(), Q.col.end());
    M.lptr = C1.lptr;
    for (size_t k = 1; k < Q.lptr.size(); ++k) M.lptr.push_back(C1.lptr.back() + Q.lptr[k]);
    M.a = C1.a;
    M.a.insert(M.a.end(), Q.a.begin(), Q.a.end());
    M.b = C1.b;
    M.b.insert(M.b.end(), Q.b.begin(), Q.b.end());
    std::vector<int32_t> ep = e1;
    ep.insert(ep.end(), e2.begin(), e2.end());
    to_lists(M, ep, DQ.n_pos(), out.dq_l);
    out.dq_ext.assign(DQ.n_pos(), -1);
    for (size_t e = 0; e < C1.col.size(); ++e) out.dq_ext[e1[e]] = C1.extra[e];
  }
  // U in P̃_0's row order: SELL row r holds level-0 row pt_row[r]
  {
    std::vector<int32_t> uperm(n0);
    for (int64_t r = 0; r < n0; ++r) uperm[L0.pt_row[r]] = (int32_t)r;
    std::vector<int32_t> eu;
    layout_prod(Uc, uperm, out.U, eu);
    if (out.U.n_pos() > INT32_MAX) return "";
    to_lists(Uc, eu, out.U.n_pos(), out.u_l);
    out.u_ext.assign(out.U.n_pos(), -1);
    for (size_t e = 0; e < Uc.col.size(); ++e) out.u_ext[eu[e]] = Uc.extra[e];
  }
  out.n0 = n0;
  out.n1 = n1;
  out.n2 = n2;
  out.on = true;
  return "";
}

}  // namespace mfea
