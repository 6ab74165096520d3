// amg_symbolic.cpp — host symbolic phase of the SA-AMG preconditioner (amg.hpp).
// Pure host C++ (no HIP), unit-tested on CPU through the debug C ABI.
#include <algorithm>
#include <numeric>

#include "amg.hpp"

namespace mfea {

namespace {

// SELL-64 pattern from per-row column lists (storage order as given)
std::string make_sell(int64_t n, const std::vector<int64_t>& rowptr, const std::vector<int32_t>& cols,
                      SellPat& S) {
  S = SellPat();
  S.n = n;
  const int64_t ns = (n + 63) / 64;
  S.sptr.assign(ns + 1, 0);
  S.rlen.assign(n, 0);
  int64_t slots = 0;
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t r = 64 * s; r < std::min<int64_t>(n, 64 * s + 64); ++r) {
      const int64_t len = rowptr[r + 1] - rowptr[r];
      S.rlen[r] = (int32_t)len;
      w = std::max(w, len);
    }
    slots += w;
    if (slots * 64 > INT32_MAX) return "AMG level too large for int32 positions";
    S.sptr[s + 1] = (int32_t)slots;
  }
  S.col.assign(slots * 64, -1);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) S.col[S.pos(r, (int)(k - rowptr[r]))] = cols[k];
  return "";
}

// list sizes → CSR pointer over positions (checks int32)
std::string finish_ptr(PosList& L, int64_t& items) {
  int64_t run = 0;
  for (size_t q = 0; q + 1 < L.ptr.size(); ++q) {
    const int64_t c = L.ptr[q + 1];
    L.ptr[q + 1] = (int32_t)(run += c);
    if (run > INT32_MAX) return "AMG index lists too large for int32";
  }
  items += run;
  return "";
}

// Standard SA aggregation (PyAMG standard_aggregation) with every coupling
// strong: (1) a node whose neighbours are all unaggregated roots a new
// aggregate with them; (2) a left-over node joins the aggregate of a
// neighbour from pass 1; (3) a node still left roots an aggregate with its
// unaggregated neighbours.  Isolated rows (no off-diagonal) stay out (-1):
// they are decoupled, so the smoother alone solves them up to a scalar.
int64_t aggregate(const SellPat& A, std::vector<int32_t>& agg) {
  const int64_t n = A.n;
  agg.assign(n, -1);
  std::vector<int8_t> pass(n, 0);
  int64_t na = 0;
  auto nbrs = [&](int64_t i, auto&& f) {
    for (int k = 1; k < A.rlen[i]; ++k) f((int64_t)A.col[A.pos(i, k)]);
  };
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.rlen[i] <= 1) continue;
    bool ok = true;
    nbrs(i, [&](int64_t j) { ok = ok && agg[j] < 0; });
    if (!ok) continue;
    agg[i] = (int32_t)na;
    pass[i] = 1;
    nbrs(i, [&](int64_t j) { agg[j] = (int32_t)na; pass[j] = 1; });
    ++na;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.rlen[i] <= 1) continue;
    int32_t a = -1;
    nbrs(i, [&](int64_t j) { if (a < 0 && pass[j] == 1) a = agg[j]; });
    if (a >= 0) {
      agg[i] = a;
      pass[i] = 2;
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.rlen[i] <= 1) continue;
    agg[i] = (int32_t)na;
    pass[i] = 3;
    nbrs(i, [&](int64_t j) {
      if (agg[j] < 0) {
        agg[j] = (int32_t)na;
        pass[j] = 3;
      }
    });
    ++na;
  }
  return na;
}

// One level's P, R, AP and the next level's A pattern with the index lists.
std::string coarsen(AmgLevel& L, SellPat& Anext, int64_t& items) {
  const SellPat& A = L.A;
  const int64_t n = A.n, nc = L.nc;
  std::string err;
  // ---- P: row i → the aggregates of {i} ∪ nbrs(i), sorted; value lists
  std::vector<int64_t> prow(n + 1, 0);
  std::vector<int32_t> pcol;
  std::vector<std::vector<int32_t>> plist;  // per P entry (CSR order): A positions
  {
    std::vector<int32_t> cols;
    for (int64_t i = 0; i < n; ++i) {
      cols.clear();
      for (int k = 0; k < A.rlen[i]; ++k) {
        const int32_t a = L.agg[A.col[A.pos(i, k)]];
        if (a >= 0) cols.push_back(a);
      }
      std::sort(cols.begin(), cols.end());
      cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
      for (int32_t c : cols) {
        pcol.push_back(c);
        std::vector<int32_t> li;
        for (int k = 0; k < A.rlen[i]; ++k)
          if (L.agg[A.col[A.pos(i, k)]] == c) li.push_back((int32_t)A.pos(i, k));
        plist.push_back(std::move(li));
      }
      prow[i + 1] = (int64_t)pcol.size();
    }
  }
  if (!(err = make_sell(n, prow, pcol, L.P)).empty()) return err;
  L.pv.ptr.assign(L.P.n_pos() + 1, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = prow[i]; k < prow[i + 1]; ++k)
      L.pv.ptr[L.P.pos(i, (int)(k - prow[i])) + 1] = (int32_t)plist[k].size();
  if (!(err = finish_ptr(L.pv, items)).empty()) return err;
  L.pv.a.resize(L.pv.ptr.back());
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = prow[i]; k < prow[i + 1]; ++k) {
      const int64_t q = L.P.pos(i, (int)(k - prow[i]));
      std::copy(plist[k].begin(), plist[k].end(), L.pv.a.begin() + L.pv.ptr[q]);
    }
  plist.clear();
  plist.shrink_to_fit();

  // ---- R = Pᵀ: coarse row J → (fine row i, P position), i ascending
  std::vector<int64_t> rrow(nc + 1, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = prow[i]; k < prow[i + 1]; ++k) rrow[pcol[k] + 1]++;
  for (int64_t J = 0; J < nc; ++J) rrow[J + 1] += rrow[J];
  std::vector<int32_t> rcol(rrow[nc]), rpp(rrow[nc]);
  {
    std::vector<int64_t> fill(rrow.begin(), rrow.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = prow[i]; k < prow[i + 1]; ++k) {
        const int64_t t = fill[pcol[k]]++;
        rcol[t] = (int32_t)i;
        rpp[t] = (int32_t)L.P.pos(i, (int)(k - prow[i]));
      }
  }
  if (!(err = make_sell(nc, rrow, rcol, L.R)).empty()) return err;
  L.rp.assign(L.R.n_pos(), -1);
  for (int64_t J = 0; J < nc; ++J)
    for (int64_t t = rrow[J]; t < rrow[J + 1]; ++t) L.rp[L.R.pos(J, (int)(t - rrow[J]))] = rpp[t];

  // ---- AP = A·P (Gustavson, outputs sorted by column)
  std::vector<int64_t> aprow(n + 1, 0);
  std::vector<int32_t> apcol;
  std::vector<int32_t> mark(nc, -1);
  std::vector<std::vector<std::pair<int32_t, int32_t>>> appairs;  // per AP entry (CSR order)
  {
    std::vector<int32_t> cols;
    std::vector<std::vector<std::pair<int32_t, int32_t>>> acc;
    for (int64_t i = 0; i < n; ++i) {
      cols.clear();
      acc.clear();
      for (int k = 0; k < A.rlen[i]; ++k) {
        const int64_t apos = A.pos(i, k);
        const int64_t kk = A.col[apos];
        for (int64_t t = prow[kk]; t < prow[kk + 1]; ++t) {
          const int32_t J = pcol[t];
          if (mark[J] < 0) {
            mark[J] = (int32_t)cols.size();
            cols.push_back(J);
            acc.emplace_back();
          }
          acc[mark[J]].emplace_back((int32_t)apos, (int32_t)L.P.pos(kk, (int)(t - prow[kk])));
        }
      }
      std::vector<int32_t> order(cols.size());
      std::iota(order.begin(), order.end(), 0);
      std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return cols[x] < cols[y]; });
      for (int32_t o : order) {
        apcol.push_back(cols[o]);
        appairs.push_back(std::move(acc[o]));
        mark[cols[o]] = -1;
      }
      aprow[i + 1] = (int64_t)apcol.size();
    }
  }
  if (!(err = make_sell(n, aprow, apcol, L.AP)).empty()) return err;
  L.ap.ptr.assign(L.AP.n_pos() + 1, 0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = aprow[i]; k < aprow[i + 1]; ++k)
      L.ap.ptr[L.AP.pos(i, (int)(k - aprow[i])) + 1] = (int32_t)appairs[k].size();
  if (!(err = finish_ptr(L.ap, items)).empty()) return err;
  L.ap.a.resize(L.ap.ptr.back());
  L.ap.b.resize(L.ap.ptr.back());
  for (int64_t i = 0; i < n; ++i)
    for (int64_t k = aprow[i]; k < aprow[i + 1]; ++k) {
      int64_t q = L.ap.ptr[L.AP.pos(i, (int)(k - aprow[i]))];
      for (auto& pr : appairs[k]) {
        L.ap.a[q] = pr.first;
        L.ap.b[q] = pr.second;
        ++q;
      }
    }
  appairs.clear();
  appairs.shrink_to_fit();

  // ---- A_{l+1} = Pᵀ (AP): coarse row I over R row I; diagonal first
  std::vector<int64_t> crow(nc + 1, 0);
  std::vector<int32_t> ccol;
  std::vector<std::vector<std::pair<int32_t, int32_t>>> cpairs;
  {
    std::vector<int32_t> cols;
    std::vector<std::vector<std::pair<int32_t, int32_t>>> acc;
    for (int64_t I = 0; I < nc; ++I) {
      cols.clear();
      acc.clear();
      mark[I] = 0;
      cols.push_back((int32_t)I);
      acc.emplace_back();
      for (int64_t t = rrow[I]; t < rrow[I + 1]; ++t) {
        const int64_t i = rcol[t];
        for (int64_t k = aprow[i]; k < aprow[i + 1]; ++k) {
          const int32_t J = apcol[k];
          if (mark[J] < 0) {
            mark[J] = (int32_t)cols.size();
            cols.push_back(J);
            acc.emplace_back();
          }
          acc[mark[J]].emplace_back(rpp[t], (int32_t)L.AP.pos(i, (int)(k - aprow[i])));
        }
      }
      std::vector<int32_t> order(cols.size());
      std::iota(order.begin(), order.end(), 0);
      std::sort(order.begin() + 1, order.end(), [&](int32_t x, int32_t y) { return cols[x] < cols[y]; });
      for (int32_t o : order) {
        ccol.push_back(cols[o]);
        cpairs.push_back(std::move(acc[o]));
        mark[cols[o]] = -1;
      }
      crow[I + 1] = (int64_t)ccol.size();
    }
  }
  if (!(err = make_sell(nc, crow, ccol, Anext)).empty()) return err;
  L.ac.ptr.assign(Anext.n_pos() + 1, 0);
  for (int64_t I = 0; I < nc; ++I)
    for (int64_t k = crow[I]; k < crow[I + 1]; ++k)
      L.ac.ptr[Anext.pos(I, (int)(k - crow[I])) + 1] = (int32_t)cpairs[k].size();
  if (!(err = finish_ptr(L.ac, items)).empty()) return err;
  L.ac.a.resize(L.ac.ptr.back());
  L.ac.b.resize(L.ac.ptr.back());
  for (int64_t I = 0; I < nc; ++I)
    for (int64_t k = crow[I]; k < crow[I + 1]; ++k) {
      int64_t q = L.ac.ptr[Anext.pos(I, (int)(k - crow[I]))];
      for (auto& pr : cpairs[k]) {
        L.ac.a[q] = pr.first;
        L.ac.b[q] = pr.second;
        ++q;
      }
    }
  return "";
}

}  // namespace

std::string build_amg(const Pattern& P, const std::vector<uint8_t>& active, int nd, AmgPlan& plan) {
  plan = AmgPlan();
  plan.nd = nd;
  if ((int64_t)active.size() != P.n_elems) return "internal: active size mismatch";
  const int64_t nf = P.n_free;
  std::string err;
  // ---- level 0: free rows, neighbours through active free-free elements
  std::vector<int64_t> rowptr(nf + 1, 0);
  std::vector<int32_t> cols;
  std::vector<std::vector<int32_t>> slots;  // per A_0 entry (CSR order): SELL positions
  {
    std::vector<std::pair<int32_t, int32_t>> nb;  // (neighbour, SELL position)
    for (int64_t i = 0; i < nf; ++i) {
      nb.clear();
      const int64_t base = (int64_t)P.slice_ptr[i >> 6] * 64 + (i & 63);
      for (int t = 0; t < P.row_len[i]; ++t) {
        const int64_t pos = base + (int64_t)t * 64;
        const int32_t j = P.s_col[pos], e = P.s_elem[pos];
        if (j < 0 || j >= nf || e < 0 || !active[e]) continue;
        nb.emplace_back(j, (int32_t)pos);
      }
      std::stable_sort(nb.begin(), nb.end(),
                       [](const auto& x, const auto& y) { return x.first < y.first; });
      cols.push_back((int32_t)i);
      slots.emplace_back();
      for (size_t k = 0; k < nb.size(); ++k) {
        if (k == 0 || nb[k].first != nb[k - 1].first) {
          cols.push_back(nb[k].first);
          slots.emplace_back();
        }
        slots.back().push_back(nb[k].second);
      }
      rowptr[i + 1] = (int64_t)cols.size();
    }
  }
  plan.lev.emplace_back();
  if (!(err = make_sell(nf, rowptr, cols, plan.lev[0].A)).empty()) return err;
  {
    const SellPat& A = plan.lev[0].A;
    plan.a0.ptr.assign(A.n_pos() + 1, 0);
    for (int64_t i = 0; i < nf; ++i)
      for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
        plan.a0.ptr[A.pos(i, (int)(k - rowptr[i])) + 1] = (int32_t)slots[k].size();
    if (!(err = finish_ptr(plan.a0, plan.pair_items)).empty()) return err;
    plan.a0.a.resize(plan.a0.ptr.back());
    for (int64_t i = 0; i < nf; ++i)
      for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
        std::copy(slots[k].begin(), slots[k].end(),
                  plan.a0.a.begin() + plan.a0.ptr[A.pos(i, (int)(k - rowptr[i]))]);
  }
  slots.clear();
  // ---- coarsen until every row is isolated (the coarsest level is then
  // block diagonal and its block-Jacobi inverse is exact)
  for (int l = 0;; ++l) {
    AmgLevel& L = plan.lev[l];
    const int64_t na = aggregate(L.A, L.agg);
    if (na == 0 || l + 1 == kAmgMaxLevels) {
      L.coarsest = true;
      plan.capped = na > 0;  // couplings left: the coarsest block Jacobi is then inexact
      L.nc = 0;
      L.agg.clear();
      break;
    }
    L.nc = na;
    SellPat Anext;
    if (!(err = coarsen(L, Anext, plan.pair_items)).empty()) return err;
    plan.lev.emplace_back();
    plan.lev.back().A = std::move(Anext);
  }
  return "";
}

}  // namespace mfea
