// amg_dist.cpp — one rank's share of the distributed SA-AMG hierarchy
// (amg.hpp AmgRank): its row ranges per level and the exchange plans of the
// V-cycle and of the numeric setup.  Host C++, once per (plan, rank).
//
// Every rank holds the whole (global) plan, so every rank can enumerate what
// every other rank reads: rank q reads the rows its own rows' columns name
// that another rank owns.  Rank r receives from p the items of q = r's list
// owned by p, and sends to q the items of q's list it owns, both in the list's
// order — the two sides of a transfer agree without any negotiation.
#include <algorithm>

#include "amg.hpp"

namespace mfea {

namespace {

struct Need {
  // per reading rank: (item, owner) in enumeration order, items unique
  std::vector<std::vector<std::pair<int32_t, int32_t>>> by_rank;
  explicit Need(int world) : by_rank(world) {}
};

// rows read across ranks: (row, owner) of every column of the listed matrix
// rows, per reading rank, sorted by row and unique
void need_rows(const SellPat& M, const std::vector<int32_t>& row_owner, const std::vector<int32_t>& col_owner,
               Need& nd) {
  for (int64_t i = 0; i < M.n; ++i) {
    const int32_t q = row_owner[i];
    for (int k = 0; k < M.rlen[i]; ++k) {
      const int32_t j = M.col[M.pos(i, k)];
      if (j >= 0 && col_owner[j] != q) nd.by_rank[q].emplace_back(j, col_owner[j]);
    }
  }
  for (auto& v : nd.by_rank) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
  }
}

// the SELL positions of the rows of `rows` (row labels in M's labelling via
// map, or identity), row by row in slot order
void rows_to_pos(const SellPat& M, const std::vector<std::pair<int32_t, int32_t>>& rows,
                 const std::vector<int32_t>* map, std::vector<std::pair<int32_t, int32_t>>& out) {
  out.clear();
  for (const auto& ro : rows) {
    const int64_t r = map ? (*map)[ro.first] : ro.first;
    for (int k = 0; k < M.rlen[r]; ++k) out.emplace_back((int32_t)M.pos(r, k), ro.second);
  }
}

XPlan make_plan(const Need& nd, int r) {
  const int world = (int)nd.by_rank.size();
  std::vector<std::vector<int32_t>> rv(world), sv(world);
  for (const auto& io : nd.by_rank[r]) rv[io.second].push_back(io.first);
  for (int q = 0; q < world; ++q)
    if (q != r)
      for (const auto& io : nd.by_rank[q])
        if (io.second == r) sv[q].push_back(io.first);
  XPlan x;
  for (int p = 0; p < world; ++p) {
    if (p == r || (rv[p].empty() && sv[p].empty())) continue;
    x.peers.push_back(p);
    x.soff.push_back((int64_t)x.sidx.size());
    x.scnt.push_back((int64_t)sv[p].size());
    x.sidx.insert(x.sidx.end(), sv[p].begin(), sv[p].end());
    x.roff.push_back((int64_t)x.ridx.size());
    x.rcnt.push_back((int64_t)rv[p].size());
    x.ridx.insert(x.ridx.end(), rv[p].begin(), rv[p].end());
  }
  return x;
}

// every rank reads every row (or position) it does not own: an all-gather
Need all_others(int world, int64_t n, const std::vector<int32_t>& owner) {
  Need nd(world);
  for (int q = 0; q < world; ++q)
    for (int64_t i = 0; i < n; ++i)
      if (owner[i] != q) nd.by_rank[q].emplace_back((int32_t)i, owner[i]);
  return nd;
}

}  // namespace

std::string build_amg_rank(const AmgPlan& plan, int rank, AmgRank& out) {
  out = AmgRank();
  const int world = plan.world, nlev = (int)plan.lev.size(), nd = plan.n_dist;
  if (nd < 1 || nd > nlev) return "internal: not a distributed AMG plan";
  if (rank < 0 || rank >= world) return "internal: AMG rank out of range";
  out.rank = rank;
  out.world = world;
  out.n_dist = nd;
  for (int l = 0; l <= std::min(nd, nlev - 1); ++l) {
    const AmgLevel& L = plan.lev[l];
    if ((int64_t)L.owner.size() != L.A.n || (int64_t)L.own.size() != world + 1)
      return "internal: AMG owners missing on a split level";
  }
  out.lo.resize(nlev);
  out.hi.resize(nlev);
  out.aplo.resize(nlev);
  out.aphi.resize(nlev);
  out.rlo.resize(nlev);
  out.rhi.resize(nlev);
  for (int l = 0; l < nlev; ++l) {
    const AmgLevel& L = plan.lev[l];
    const bool split = l < nd;
    out.lo[l] = split ? L.own[rank] : 0;
    out.hi[l] = split ? L.own[rank + 1] : L.A.n;
    out.aplo[l] = split && !L.coarsest ? L.ap_own[rank] : 0;
    out.aphi[l] = split && !L.coarsest ? L.ap_own[rank + 1] : L.AP.n;
    if (!L.coarsest) {
      const AmgLevel& N = plan.lev[l + 1];
      out.rlo[l] = split ? N.own[rank] : 0;  // level l+1 ≤ n_dist carries owners
      out.rhi[l] = split ? N.own[rank + 1] : N.A.n;
    }
  }
  std::vector<std::pair<int32_t, int32_t>> pos;
  for (int l = 0; l < nd; ++l) {
    const AmgLevel& L = plan.lev[l];
    Need na(world), nr(world), np(world);
    need_rows(L.A, L.owner, L.owner, na);
    out.xa.push_back(make_plan(na, rank));
    if (L.coarsest) {  // every level split: the coarsest solve is local
      out.xr.emplace_back();
      out.xp.emplace_back();
      out.sp.emplace_back();
      out.sap.emplace_back();
      continue;
    }
    const AmgLevel& N = plan.lev[l + 1];
    need_rows(L.R, N.owner, L.owner, nr);
    out.xr.push_back(make_plan(nr, rank));
    if (l + 1 < nd) need_rows(L.P, L.owner, N.owner, np);
    out.xp.push_back(make_plan(np, rank));
    // setup: P rows read by this rank's A·P rows (A's columns) and by its R
    // rows / A_{l+1} rows (R's columns); A·P rows read by its A_{l+1} rows
    Need sp(world), sap(world);
    for (int q = 0; q < world; ++q) {
      std::vector<std::pair<int32_t, int32_t>> rows = na.by_rank[q];
      rows.insert(rows.end(), nr.by_rank[q].begin(), nr.by_rank[q].end());
      std::sort(rows.begin(), rows.end());
      rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
      rows_to_pos(L.P, rows, nullptr, pos);
      sp.by_rank[q] = pos;
      rows_to_pos(L.AP, nr.by_rank[q], &L.aprow, pos);
      sap.by_rank[q] = pos;
    }
    out.sp.push_back(make_plan(sp, rank));
    out.sap.push_back(make_plan(sap, rank));
  }
  if (nd < nlev) {  // level nd: replicated, its rows produced by their owners
    const AmgLevel& G = plan.lev[nd];
    out.xg = make_plan(all_others(world, G.A.n, G.owner), rank);
    Need sg(world);
    for (int q = 0; q < world; ++q) {
      std::vector<std::pair<int32_t, int32_t>> rows;
      for (int64_t i = 0; i < G.A.n; ++i)
        if (G.owner[i] != q) rows.emplace_back((int32_t)i, G.owner[i]);
      rows_to_pos(G.A, rows, nullptr, pos);
      sg.by_rank[q] = pos;
    }
    out.sg = make_plan(sg, rank);
  }
  // the compact cycle: only level 0 split, its R̂_0 rows owner-major
  const AmgLevel& L0 = plan.lev[0];
  if (nd == 1 && nlev >= 2 && !L0.coarsest && L0.PT.n == L0.A.n && L0.RT.n == plan.lev[1].A.n &&
      (int64_t)L0.rt_own.size() == world + 1 && (int64_t)L0.ap_own.size() == world + 1) {
    out.compact = true;
    out.rtlo = L0.rt_own[rank];
    out.rthi = L0.rt_own[rank + 1];
    std::vector<int32_t> rt_owner(L0.RT.n, 0), pt_owner(L0.PT.n, 0);
    for (int q = 0; q < world; ++q) {
      for (int64_t I = L0.rt_own[q]; I < L0.rt_own[q + 1]; ++I) rt_owner[I] = q;
      for (int64_t a = L0.ap_own[q]; a < L0.ap_own[q + 1]; ++a) pt_owner[a] = q;
    }
    // x_0 halo of the down sweep: the columns of its Ã_0 (A_0's pattern) and R̂_0 rows
    Need nx(world);
    need_rows(L0.A, L0.owner, L0.owner, nx);
    need_rows(L0.RT, rt_owner, L0.owner, nx);
    out.xc = make_plan(nx, rank);
    // P̃_0 positions and level-0 diagonal blocks read by each rank's R̂_0 rows
    std::vector<int32_t> pt_srow(L0.PT.sptr.empty() ? 0 : L0.PT.sptr.back(), 0);
    for (size_t sl = 0; sl + 1 < L0.PT.sptr.size(); ++sl)
      for (int32_t t = L0.PT.sptr[sl]; t < L0.PT.sptr[sl + 1]; ++t) pt_srow[t] = (int32_t)sl;
    Need npt(world), ndg(world);
    for (int64_t I = 0; I < L0.RT.n; ++I) {
      const int32_t q = rt_owner[I];
      for (int k = 0; k < L0.RT.rlen[I]; ++k) {
        const int64_t qq = L0.RT.pos(I, k);
        const int32_t i = L0.RT.col[qq];
        if (i < 0) continue;
        const int32_t pp = L0.rt_pt[qq];
        const int64_t a = 64 * (int64_t)pt_srow[pp >> 6] + (pp & 63);
        if (pt_owner[a] != q) npt.by_rank[q].emplace_back(pp, pt_owner[a]);
        if (L0.owner[i] != q) ndg.by_rank[q].emplace_back((int32_t)L0.A.pos(i, 0), L0.owner[i]);
      }
    }
    for (auto* n : {&npt, &ndg})
      for (auto& v : n->by_rank) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
      }
    out.spt = make_plan(npt, rank);
    out.sd = make_plan(ndg, rank);
  }
  return "";
}

std::string build_amg_level0(const AmgPlan& pl, const Pattern& G, const AmgRank& rk, const Pattern& P,
                             const std::vector<int64_t>& node_g, const std::vector<int64_t>& elem_g,
                             const std::vector<uint8_t>& gkey, PosList& a0, std::vector<int32_t>& row0) {
  const SellPat& A = pl.lev[0].A;
  const int64_t n0 = A.n, lo = rk.lo[0], hi = rk.hi[0];
  const int64_t N = (int64_t)G.perm.size();
  std::vector<int32_t> g2l(N, -1), inv0(G.n_free, -1);
  for (size_t ln = 0; ln < node_g.size(); ++ln) g2l[node_g[ln]] = (int32_t)ln;
  for (int64_t i = 0; i < n0; ++i) inv0[pl.row0[i]] = (int32_t)i;
  row0.assign(n0, 0);
  a0 = PosList();
  a0.ptr.assign(A.n_pos() + 1, 0);
  std::vector<int32_t> slot, qpos;  // per coupling: P's slot, A_0 position (rows in order)
  for (int64_t i = lo; i < hi; ++i) {
    const int32_t ln = g2l[G.perm[pl.row0[i]]];
    if (ln < 0) return "internal: an own level-0 row is not in the partition";
    const int64_t lr = P.iperm[ln];
    if (lr >= P.n_free) return "internal: an own level-0 row is not a free row of the partition";
    row0[i] = (int32_t)lr;
    const int64_t base = (int64_t)P.slice_ptr[lr >> 6] * 64 + (lr & 63);
    for (int t = 0; t < P.row_len[lr]; ++t) {
      const int64_t pos = base + (int64_t)t * 64;
      const int32_t c = P.s_col[pos], e = P.s_elem[pos];
      if (c < 0 || e < 0 || !gkey[elem_g[e]]) continue;
      if (c >= P.n_free && P.code[c] != kGhost) continue;  // a grip neighbour: the RHS, not A_0
      const int64_t gr = G.iperm[node_g[P.perm[c]]];
      if (gr >= G.n_free) return "internal: a free neighbour is a known node globally";
      const int32_t j = inv0[gr];
      int64_t q = -1;
      for (int k = 1; k < A.rlen[i] && q < 0; ++k)
        if (A.col[A.pos(i, k)] == j) q = A.pos(i, k);
      if (q < 0) return "internal: a local coupling is missing from A_0";
      slot.push_back((int32_t)pos);
      qpos.push_back((int32_t)q);
    }
  }
  // CSR over positions; a position's slots in slot order
  for (int32_t q : qpos) a0.ptr[q + 1]++;
  for (int64_t q = 0; q < A.n_pos(); ++q) a0.ptr[q + 1] += a0.ptr[q];
  a0.a.assign(a0.ptr.back(), 0);
  std::vector<int32_t> fill(a0.ptr.begin(), a0.ptr.end() - 1);
  for (size_t k = 0; k < slot.size(); ++k) a0.a[fill[qpos[k]]++] = slot[k];
  return "";
}

}  // namespace mfea
