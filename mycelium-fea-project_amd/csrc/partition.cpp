// partition.cpp — see partition.hpp.  Pure host C++ (no HIP), unit-tested on CPU.
#include "partition.hpp"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <utility>

namespace mfea {

namespace {

// Splits the nodes `ids` into k strips along `axis`: equal FREE-node counts,
// each boundary then moved (by at most slack × the strip size) to the sorted
// position crossed by the fewest elements with both ends in `ids`, so cuts
// fall in the sparse gaps of a network (between tiles) rather than through
// its dense parts — a 1-D min-cut in the spirit of graph partitioners.
// Block-Jacobi-type preconditioners over the strips (partitioned GAMG) need
// this: a boundary through a dense tile costs 10-30x the CG iterations
// (DESIGN.md §5).  Known nodes join the strip around them.  pos: scratch of
// size N, all -1 on entry and on return.  Returns the strip of each ids[i].
std::vector<int32_t> split_strips(const std::vector<int64_t>& ids, const double* xyz, int64_t E,
                                  const int64_t* e2n, int64_t N, const std::vector<uint8_t>& known,
                                  int axis, int k, double slack, std::vector<int64_t>& pos) {
  const int64_t n = (int64_t)ids.size();
  std::vector<int64_t> ord(n);
  std::iota(ord.begin(), ord.end(), (int64_t)0);
  std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
    const double xa = xyz[3 * ids[a] + axis], xb = xyz[3 * ids[b] + axis];
    return xa < xb || (xa == xb && ids[a] < ids[b]);
  });
  std::vector<int32_t> strip(n, 0);
  std::vector<int64_t> fpos;  // sorted position of the s-th free node
  for (int64_t q = 0; q < n; ++q)
    if (!known[ids[ord[q]]]) fpos.push_back(q);
  const int64_t nfree = (int64_t)fpos.size();
  if (k <= 1 || nfree == 0) return strip;
  for (int64_t q = 0; q < n; ++q) pos[ids[ord[q]]] = q;
  std::vector<int64_t> cut(n + 1, 0);  // elements crossing between q and q + 1
  for (int64_t e = 0; e < E; ++e) {
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a < 0 || a >= N || b < 0 || b >= N || a == b || pos[a] < 0 || pos[b] < 0) continue;
    ++cut[std::min(pos[a], pos[b])];
    --cut[std::max(pos[a], pos[b])];
  }
  for (int64_t q = 1; q <= n; ++q) cut[q] += cut[q - 1];
  for (int64_t i : ids) pos[i] = -1;
  const int64_t d = (int64_t)std::floor(std::min(std::max(slack, 0.0), 0.45) * ((double)nfree / k));
  std::vector<int64_t> qcut(k, -1);  // last sorted position of strip j-1
  for (int j = 1; j < k; ++j) {
    const int64_t sj = (j * nfree + k - 1) / k;  // strip j starts at free node ⌈j·nfree/k⌉
    const int64_t q0 = fpos[std::max<int64_t>(sj - 1, 0)];  // the equal-count cut
    int64_t best = std::max(q0, qcut[j - 1] + 1);
    if (d > 0) {
      const int64_t slo = std::max<int64_t>(sj - d, 1), shi = std::min<int64_t>(sj + d, nfree - 1);
      const int64_t qa = std::max(fpos[slo - 1], qcut[j - 1] + 1), qb = fpos[shi] - 1;
      for (int64_t q = qa; q <= qb; ++q) {
        const bool fewer = cut[q] < cut[best];
        const bool tie_closer = cut[q] == cut[best] && std::llabs(q - q0) < std::llabs(best - q0);
        if (fewer || tie_closer) best = q;
      }
    }
    qcut[j] = best;
  }
  int32_t r = 0;
  for (int64_t q = 0; q < n; ++q) {
    while (r + 1 < k && q > qcut[r + 1]) ++r;
    strip[ord[q]] = r;
  }
  return strip;
}

int64_t cut_elements(const std::vector<int32_t>& own, int64_t E, const int64_t* e2n, int64_t N) {
  int64_t c = 0;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a >= 0 && a < N && b >= 0 && b < N && own[a] != own[b]) ++c;
  }
  return c;
}

}  // namespace

std::vector<int32_t> node_owner(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                                const std::vector<int64_t>& top, const std::vector<int64_t>& bot,
                                int world, int axis, double slack, int* axis_used) {
  std::vector<uint8_t> known(N, 0);
  for (int64_t t : top) known[t] = 1;
  for (int64_t b : bot) known[b] = 1;
  std::vector<int64_t> all(N), pos(N, -1);
  std::iota(all.begin(), all.end(), (int64_t)0);
  if (axis == 0 || axis == 1 || world <= 1) {  // strips along one axis
    if (axis_used) *axis_used = axis < 0 ? 0 : axis;
    return split_strips(all, xyz, E, e2n, N, known, axis < 0 ? 0 : axis, world, slack, pos);
  }
  // axis -1: a px × py grid (px strips along x, each cut into py along y) for
  // every factorisation of world; the one with the fewest cut elements wins
  // (ties: fewer x strips)
  std::vector<int32_t> best;
  int64_t best_cut = -1;
  int best_px = 1;
  for (int px = 1; px <= world; ++px) {
    if (world % px) continue;
    const int py = world / px;
    const std::vector<int32_t> sx = split_strips(all, xyz, E, e2n, N, known, 0, px, slack, pos);
    std::vector<std::vector<int64_t>> col(px);
    for (int64_t n = 0; n < N; ++n) col[sx[n]].push_back(n);
    std::vector<int32_t> own(N, 0);
    for (int c = 0; c < px; ++c) {
      const std::vector<int32_t> sy = split_strips(col[c], xyz, E, e2n, N, known, 1, py, slack, pos);
      for (size_t i = 0; i < col[c].size(); ++i) own[col[c][i]] = c * py + sy[i];
    }
    const int64_t cut = cut_elements(own, E, e2n, N);
    if (best_cut < 0 || cut < best_cut) {
      best_cut = cut;
      best = std::move(own);
      best_px = px;
    }
  }
  if (axis_used) *axis_used = best_px == world ? 0 : (best_px == 1 ? 1 : 2);
  return best;
}

std::string build_partition(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                            bool skip_invalid, const std::vector<int64_t>& top,
                            const std::vector<int64_t>& bot, int world, int rank, int axis,
                            double slack, PartPlan& plan) {
  if (world < 1 || rank < 0 || rank >= world) return "bad rank / world size";
  if (N < 0 || E < 0) return "negative mesh size";
  if (N > INT32_MAX / 4 || E > INT32_MAX / 4) return "mesh too large for int32 indexing";
  for (int64_t t : top)
    if (t < 0 || t >= N) return "top grip node out of range";
  for (int64_t b : bot)
    if (b < 0 || b >= N) return "bottom grip node out of range";
  plan = PartPlan();
  plan.world = world;
  plan.rank = rank;
  for (int64_t e = 0; e < E && !skip_invalid; ++e)
    for (int c = 0; c < 2; ++c)
      if (e2n[2 * e + c] < 0 || e2n[2 * e + c] >= N)
        return "element " + std::to_string(e) + " references node out of range [0," + std::to_string(N) + ")";
  plan.owner = node_owner(N, xyz, E, e2n, top, bot, world, axis, slack, &plan.axis);
  const std::vector<int32_t>& own = plan.owner;
  std::vector<uint8_t> known(N, 0);
  for (int64_t t : top) known[t] = 1;
  for (int64_t b : bot) known[b] = 1;

  // ---- local mesh: owned nodes, elements with an owned endpoint, their far ends
  std::vector<uint8_t> valid(E, 1), local_e(E, 0), local_n(N, 0);
  for (int64_t n = 0; n < N; ++n) local_n[n] = own[n] == rank;
  for (int64_t e = 0; e < E; ++e) {
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a < 0 || a >= N || b < 0 || b >= N) {
      if (!skip_invalid)
        return "element " + std::to_string(e) + " references node out of range [0," +
               std::to_string(N) + ")";
      valid[e] = 0;
      continue;
    }
    if (own[a] == rank || own[b] == rank) {
      local_e[e] = 1;
      local_n[a] = local_n[b] = 1;
    }
  }
  std::vector<int64_t> g2l(N, -1);
  for (int64_t n = 0; n < N; ++n) {
    if (!local_n[n]) continue;
    g2l[n] = (int64_t)plan.node_g.size();
    plan.node_g.push_back(n);
    plan.ghost.push_back(own[n] != rank);
    for (int c = 0; c < 3; ++c) plan.xyz.push_back(xyz[3 * n + c]);
  }
  for (int64_t e = 0; e < E; ++e) {
    if (!local_e[e]) continue;
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    plan.elem_g.push_back(e);
    plan.e2n.push_back(g2l[a]);
    plan.e2n.push_back(g2l[b]);
    plan.elem_own.push_back(own[a] == rank);
  }
  for (int64_t t : top)
    if (local_n[t]) plan.top.push_back(g2l[t]);
  for (int64_t b : bot)
    if (local_n[b]) plan.bot.push_back(g2l[b]);

  // ---- CG record pairs: cut elements between two free nodes, (peer, element) order
  const int64_t EL = (int64_t)plan.elem_g.size();
  plan.elem_pair.assign(EL, -1);
  std::vector<std::pair<int32_t, int64_t>> pr;  // (peer, local element)
  for (int64_t le = 0; le < EL; ++le) {
    const int64_t e = plan.elem_g[le];
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a == b || known[a] || known[b] || own[a] == own[b]) continue;
    pr.emplace_back(own[a] == rank ? own[b] : own[a], le);
  }
  // local elements are in ascending global id: a stable sort by peer keeps that order
  std::stable_sort(pr.begin(), pr.end(),
                   [](const auto& x, const auto& y) { return x.first < y.first; });
  for (size_t k = 0; k < pr.size(); ++k) {
    plan.elem_pair[pr[k].second] = (int32_t)k;
    if (plan.peers.empty() || plan.peers.back() != pr[k].first) {
      plan.peers.push_back(pr[k].first);
      plan.peer_off.push_back((int64_t)k);
      plan.peer_cnt.push_back(0);
    }
    plan.peer_cnt.back()++;
  }
  plan.n_pairs = (int64_t)pr.size();

  // ---- displacement halo: A sends B its free nodes adjacent to B's nodes; B
  // receives exactly those as its ghost free nodes.  Both sorted by node id.
  std::vector<std::pair<int32_t, int64_t>> snd, rcv;  // (peer, global node)
  for (int64_t e = 0; e < E; ++e) {
    if (!valid[e]) continue;
    const int64_t a = e2n[2 * e], b = e2n[2 * e + 1];
    if (a == b || own[a] == own[b]) continue;
    for (int s = 0; s < 2; ++s) {
      const int64_t m = s ? b : a, o = s ? a : b;
      if (known[m]) continue;
      if (own[m] == rank) snd.emplace_back(own[o], m);
      if (own[o] == rank) rcv.emplace_back(own[m], m);
    }
  }
  for (auto* v : {&snd, &rcv}) {
    std::sort(v->begin(), v->end());
    v->erase(std::unique(v->begin(), v->end()), v->end());
  }
  std::vector<int32_t> xp;
  for (const auto& s : snd) xp.push_back(s.first);
  for (const auto& r : rcv) xp.push_back(r.first);
  std::sort(xp.begin(), xp.end());
  xp.erase(std::unique(xp.begin(), xp.end()), xp.end());
  plan.xpeers = xp;
  size_t is = 0, ir = 0;
  for (int32_t p : xp) {
    plan.xsend_off.push_back((int64_t)plan.xsend_node.size());
    for (; is < snd.size() && snd[is].first == p; ++is) plan.xsend_node.push_back(g2l[snd[is].second]);
    plan.xsend_cnt.push_back((int64_t)plan.xsend_node.size() - plan.xsend_off.back());
    plan.xrecv_off.push_back((int64_t)plan.xrecv_node.size());
    for (; ir < rcv.size() && rcv[ir].first == p; ++ir) plan.xrecv_node.push_back(g2l[rcv[ir].second]);
    plan.xrecv_cnt.push_back((int64_t)plan.xrecv_node.size() - plan.xrecv_off.back());
  }
  return "";
}

}  // namespace mfea
