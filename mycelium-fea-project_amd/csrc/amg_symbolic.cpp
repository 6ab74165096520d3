// amg_symbolic.cpp — host symbolic phase of the SA-AMG preconditioner (amg.hpp).
// Pure host C++ (no HIP), unit-tested on CPU through tests/native/host_shim.cpp.
//
// Two stages:
//   1. the hierarchy in natural numbering, as row-major (CSR) patterns whose
//      index lists reference CSR entries: aggregation, P, R = Pᵀ, A·P and
//      A_{l+1} = Pᵀ A P (Gustavson, fixed order);
//   2. the device layout: every level's rows are relabelled so that, inside
//      windows of kSortWindow consecutive rows, longer rows come first
//      (SELL-C-σ, C = 64): the 64 rows of a slice then have nearly equal
//      lengths and a slice's width (its longest row) stops padding the
//      others.  Natural (DFS / aggregate) order is kept across windows, so
//      gathers stay local.  Measured on the C3 network: valid positions of
//      the level-0 A / R layouts 52 % / 28 % in natural order, 97 % / 81 %
//      with 4096-row windows.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <thread>

#include "amg.hpp"

namespace mfea {

namespace {

constexpr int64_t kSortWindow = 4096;  // rows per SELL-C-σ sorting window (64 slices)

struct Csr {
  int64_t n = 0;
  std::vector<int64_t> ptr{0};
  std::vector<int32_t> col;
  int64_t len(int64_t r) const { return ptr[r + 1] - ptr[r]; }
};
// index lists per entry of an output matrix (CSR over its entries)
struct Lists {
  std::vector<int64_t> ptr{0};
  std::vector<int32_t> a, b;
};

struct LevelCsr {
  Csr A;
  int64_t nc = 0;
  std::vector<int32_t> agg;
  Csr P, R, AP;
  Lists pv;                // per P entry: A entries
  std::vector<int32_t> rp;  // per R entry: P entry
  Lists ap;                // per AP entry: (A entry, P entry)
  Lists ac;                // per A_{l+1} entry: (P entry, AP entry)
};

// Standard SA aggregation (PyAMG standard_aggregation) with every coupling
// strong: (1) a node whose neighbours are all unaggregated roots a new
// aggregate with them; (2) a left-over node joins the aggregate of a
// neighbour from pass 1; (3) a node still left roots an aggregate with its
// unaggregated neighbours.  Isolated rows (no off-diagonal) stay out (-1):
// they are decoupled, so the smoother alone solves them up to a scalar.
// A's rows hold their diagonal first.  strong (per CSR entry, optional):
// only strong couplings make neighbours; a row whose couplings are all weak
// roots a singleton aggregate in pass 3 (it keeps a coarse representative).
int64_t aggregate(const Csr& A, std::vector<int32_t>& agg, const std::vector<uint8_t>* strong = nullptr) {
  const int64_t n = A.n;
  agg.assign(n, -1);
  std::vector<int8_t> pass(n, 0);
  int64_t na = 0;
  auto nbrs = [&](int64_t i, auto&& f) {
    for (int64_t k = A.ptr[i] + 1; k < A.ptr[i + 1]; ++k)
      if (!strong || (*strong)[k]) f((int64_t)A.col[k]);
  };
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.len(i) <= 1) continue;
    bool ok = true;
    nbrs(i, [&](int64_t j) { ok = ok && agg[j] < 0; });
    if (!ok) continue;
    agg[i] = (int32_t)na;
    pass[i] = 1;
    nbrs(i, [&](int64_t j) { agg[j] = (int32_t)na; pass[j] = 1; });
    ++na;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.len(i) <= 1) continue;
    int32_t a = -1;
    nbrs(i, [&](int64_t j) { if (a < 0 && pass[j] == 1) a = agg[j]; });
    if (a >= 0) {
      agg[i] = a;
      pass[i] = 2;
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    if (agg[i] >= 0 || A.len(i) <= 1) continue;
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

// ---- host threads: the symbolic phase's row loops run over contiguous
// chunks of rows on up to kBuildThreads threads; every output is assembled in
// row order, so the plan is the same bits for any thread count (C5's build
// was 4.9 s on one thread).
constexpr int kBuildThreads = 16;
constexpr int64_t kChunkRows = 8192;

// MFEA_BUILD_TIMES=1: the symbolic phase's split on stderr (host build profile)
struct PhaseClock {
  bool on = std::getenv("MFEA_BUILD_TIMES") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "  build %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

int build_threads() {
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min<unsigned>(h ? h : 1, kBuildThreads));
}

// chunk boundaries of [0, n): T + 1 values
std::vector<int64_t> chunks(int64_t n) {
  const int64_t T = std::max<int64_t>(1, std::min<int64_t>(build_threads(), (n + kChunkRows - 1) / kChunkRows));
  std::vector<int64_t> b(T + 1);
  for (int64_t t = 0; t <= T; ++t) b[t] = n * t / T;
  return b;
}

// f(lo, hi, t) over the chunks of [0, n), one thread each
template <class F>
void par_for(int64_t n, F&& f) {
  const std::vector<int64_t> b = chunks(n);
  const int T = (int)b.size() - 1;
  if (T == 1) {
    f(b[0], b[1], 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back([&, t] { f(b[t], b[t + 1], t); });
  f(b[0], b[1], 0);
  for (auto& x : th) x.join();
}

// One chunk's rows of a CSR with per-entry item lists (P + pv, A·P + ap,
// A_{l+1} + ac, A_0 + a0): entry(c) opens an entry of the current row,
// item(a[, b]) appends to the last entry's list.
struct RowSink {
  std::vector<int64_t> rlen;
  std::vector<int32_t> col, icnt, a, b;
  void begin_row() { rlen.push_back(0); }
  void entry(int32_t c) {
    col.push_back(c);
    icnt.push_back(0);
    ++rlen.back();
  }
  void item(int32_t x) {
    a.push_back(x);
    ++icnt.back();
  }
  void item(int32_t x, int32_t y) {
    a.push_back(x);
    b.push_back(y);
    ++icnt.back();
  }
};

// M (n rows) and its lists from emit(i, sink) per row, rows in parallel
// chunks, merged in row order
template <class Emit>
void produce_rows(int64_t n, Csr& M, Lists& Ls, bool pair, Emit&& emit) {
  const std::vector<int64_t> b = chunks(n);
  const int T = (int)b.size() - 1;
  std::vector<RowSink> sk(T);
  par_for(n, [&](int64_t lo, int64_t hi, int t) {
    RowSink& s = sk[t];
    s.rlen.reserve(hi - lo);
    for (int64_t i = lo; i < hi; ++i) {
      s.begin_row();
      emit(i, s);
    }
  });
  std::vector<int64_t> eoff(T + 1, 0), ioff(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    eoff[t + 1] = eoff[t] + (int64_t)sk[t].col.size();
    ioff[t + 1] = ioff[t] + (int64_t)sk[t].a.size();
  }
  M.n = n;
  M.ptr.assign(n + 1, 0);
  M.col.resize(eoff[T]);
  Ls.ptr.assign(eoff[T] + 1, 0);
  Ls.a.resize(ioff[T]);
  Ls.b.resize(pair ? ioff[T] : 0);
  par_for(n, [&](int64_t lo, int64_t hi, int t) {
    const RowSink& s = sk[t];
    int64_t e = eoff[t];
    for (int64_t i = lo; i < hi; ++i) {
      e += s.rlen[i - lo];
      M.ptr[i + 1] = e;
    }
    std::copy(s.col.begin(), s.col.end(), M.col.begin() + eoff[t]);
    int64_t q = ioff[t];
    for (size_t k = 0; k < s.icnt.size(); ++k) {
      q += s.icnt[k];
      Ls.ptr[eoff[t] + (int64_t)k + 1] = q;
    }
    std::copy(s.a.begin(), s.a.end(), Ls.a.begin() + ioff[t]);
    if (pair) std::copy(s.b.begin(), s.b.end(), Ls.b.begin() + ioff[t]);
  });
}

std::string check32(int64_t v, const char* what) {
  return v > INT32_MAX ? std::string("AMG ") + what + " too large for int32 indices" : std::string();
}

// One level's P, R, AP and the next level's A (natural numbering).
std::string coarsen(LevelCsr& L, Csr& An) {
  const Csr& A = L.A;
  const int64_t n = A.n, nc = L.nc;
  // ---- P: row i → the aggregates of {i} ∪ nbrs(i), ascending; value lists
  produce_rows(n, L.P, L.pv, false, [&](int64_t i, RowSink& s) {
    thread_local std::vector<std::pair<int32_t, int32_t>> t;  // (aggregate, A entry)
    t.clear();
    for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
      const int32_t a = L.agg[A.col[k]];
      if (a >= 0) t.emplace_back(a, (int32_t)k);
    }
    row_stable_sort(t.begin(), t.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (size_t k = 0; k < t.size(); ++k) {
      if (k == 0 || t[k].first != t[k - 1].first) s.entry(t[k].first);
      s.item(t[k].second);
    }
  });
  std::string err;
  if (!(err = check32((int64_t)L.P.col.size(), "prolongator")).empty()) return err;
  // ---- R = Pᵀ: coarse row J → (fine row i ascending, P entry)
  {
    L.R.n = nc;
    L.R.ptr.assign(nc + 1, 0);
    for (int32_t J : L.P.col) L.R.ptr[J + 1]++;
    for (int64_t J = 0; J < nc; ++J) L.R.ptr[J + 1] += L.R.ptr[J];
    L.R.col.resize(L.P.col.size());
    L.rp.resize(L.P.col.size());
    std::vector<int64_t> fill(L.R.ptr.begin(), L.R.ptr.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = L.P.ptr[i]; k < L.P.ptr[i + 1]; ++k) {
        const int64_t t = fill[L.P.col[k]]++;
        L.R.col[t] = (int32_t)i;
        L.rp[t] = (int32_t)k;
      }
  }
  // ---- AP = A·P: per row, (J, A entry, P entry) triples, stable-sorted by J
  {
    struct T3 { int32_t J, a, p; };
    produce_rows(n, L.AP, L.ap, true, [&](int64_t i, RowSink& s) {
      thread_local std::vector<T3> t;
      t.clear();
      for (int64_t k = A.ptr[i]; k < A.ptr[i + 1]; ++k) {
        const int64_t kk = A.col[k];
        for (int64_t q = L.P.ptr[kk]; q < L.P.ptr[kk + 1]; ++q) t.push_back({L.P.col[q], (int32_t)k, (int32_t)q});
      }
      row_stable_sort(t.begin(), t.end(), [](const T3& x, const T3& y) { return x.J < y.J; });
      for (size_t k = 0; k < t.size(); ++k) {
        if (k == 0 || t[k].J != t[k - 1].J) s.entry(t[k].J);
        s.item(t[k].a, t[k].p);
      }
    });
  }
  if (!(err = check32((int64_t)L.AP.col.size(), "A·P")).empty()) return err;
  // ---- A_{l+1} = Pᵀ (AP): coarse row I over R row I, diagonal first
  {
    struct T3 { int32_t J, p, m; };
    An = Csr();
    produce_rows(nc, An, L.ac, true, [&](int64_t I, RowSink& s) {
      thread_local std::vector<T3> t;
      t.clear();
      for (int64_t r = L.R.ptr[I]; r < L.R.ptr[I + 1]; ++r) {
        const int64_t i = L.R.col[r];
        for (int64_t k = L.AP.ptr[i]; k < L.AP.ptr[i + 1]; ++k) t.push_back({L.AP.col[k], L.rp[r], (int32_t)k});
      }
      row_stable_sort(t.begin(), t.end(), [I](const T3& x, const T3& y) {
        const bool dx = x.J == I, dy = y.J == I;  // the diagonal block first, then ascending
        return dx != dy ? dx : x.J < y.J;
      });
      for (size_t k = 0; k < t.size(); ++k) {
        if (k == 0 || t[k].J != t[k - 1].J) s.entry(t[k].J);
        s.item(t[k].p, t[k].m);
      }
    });
  }
  return check32((int64_t)An.col.size(), "coarse operator");
}

// ---- stage 2: relabelled SELL layouts -----------------------------------------
// new = perm[old]: inside windows of kSortWindow rows, rows by descending key
// (stable: ties keep natural order).  own: rows grouped by rank first
// (owner-major, natural order inside a rank), the windows inside each rank's
// segment; bounds (world + 1) receives the segments' first new rows.
std::vector<int32_t> sort_perm(const std::vector<int64_t>& key, const std::vector<int32_t>* own = nullptr,
                               int world = 1, std::vector<int64_t>* bounds = nullptr,
                               const std::vector<int32_t>* base = nullptr) {
  const int64_t n = (int64_t)key.size();
  std::vector<int32_t> order(n), perm(n);
  if (base) order = *base;  // a base order of the rows instead of the natural one (Z-order)
  else std::iota(order.begin(), order.end(), 0);
  std::vector<int64_t> seg{0, n};
  if (own) {
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return (*own)[x] < (*own)[y]; });
    seg.assign(world + 1, 0);
    for (int64_t i = 0; i < n; ++i) seg[(*own)[i] + 1]++;
    for (int r = 0; r < world; ++r) seg[r + 1] += seg[r];
  }
  std::vector<std::pair<int64_t, int64_t>> win;  // the sorting windows, independent
  for (size_t g = 0; g + 1 < seg.size(); ++g)
    for (int64_t w0 = seg[g]; w0 < seg[g + 1]; w0 += kSortWindow) win.emplace_back(w0, std::min(seg[g + 1], w0 + kSortWindow));
  par_for((int64_t)win.size() * kChunkRows / 16, [&](int64_t lo, int64_t hi, int) {
    const int64_t a = lo * 16 / kChunkRows, b = hi * 16 / kChunkRows;
    for (int64_t k = a; k < b && k < (int64_t)win.size(); ++k)
      std::stable_sort(order.begin() + win[k].first, order.begin() + win[k].second,
                       [&](int32_t x, int32_t y) { return key[x] > key[y]; });
  });
  for (int64_t k = 0; k < n; ++k) perm[order[k]] = (int32_t)k;
  if (bounds) *bounds = seg;
  return perm;
}

// Z-order (Morton) of points in the plane / space: 21 bits per axis over the
// bounding box (3-D when any z differs), ties by index
std::vector<int32_t> morton_order(const std::vector<double>& xyz, int64_t n) {
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      lo[c] = std::min(lo[c], xyz[3 * i + c]);
      hi[c] = std::max(hi[c], xyz[3 * i + c]);
    }
  const bool d3 = n > 0 && hi[2] > lo[2];
  double span = 0.0;
  for (int c = 0; c < (d3 ? 3 : 2); ++c) span = std::max(span, hi[c] - lo[c]);
  const double sc = span > 0.0 ? ((1 << 21) - 1) / span : 0.0;
  auto spread = [](uint64_t v, int step) {  // bit b → bit step·b
    uint64_t r = 0;
    for (int b = 0; b < 21; ++b) r |= ((v >> b) & 1ull) << (step * b);
    return r;
  };
  std::vector<uint64_t> key(n);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t k = 0;
    for (int c = 0; c < (d3 ? 3 : 2); ++c)
      k |= spread((uint64_t)((xyz[3 * i + c] - lo[c]) * sc), d3 ? 3 : 2) << c;
    key[i] = k;
  }
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return key[a] < key[b]; });
  return order;
}

// SELL-64 of M with rows relabelled by rperm and columns by cperm; epos[e] =
// position of CSR entry e
std::string layout(const Csr& M, const std::vector<int32_t>& rperm, const std::vector<int32_t>* cperm,
                   SellPat& S, std::vector<int32_t>& epos) {
  const int64_t n = M.n;
  std::vector<int32_t> inv(n);
  par_for(n, [&](int64_t lo, int64_t hi, int) {
    for (int64_t r = lo; r < hi; ++r) inv[rperm[r]] = (int32_t)r;
  });
  S = SellPat();
  S.n = n;
  const int64_t ns = (n + 63) / 64;
  S.sptr.assign(ns + 1, 0);
  S.rlen.assign(n, 0);
  int64_t slots = 0;
  for (int64_t s = 0; s < ns; ++s) {
    int64_t w = 0;
    for (int64_t r = 64 * s; r < std::min<int64_t>(n, 64 * s + 64); ++r) {
      const int64_t len = M.len(inv[r]);
      S.rlen[r] = (int32_t)len;
      w = std::max(w, len);
    }
    slots += w;
    if (slots * 64 > INT32_MAX) return "AMG level too large for int32 positions";
    S.sptr[s + 1] = (int32_t)slots;
  }
  S.col.assign(slots * 64, -1);
  epos.assign(M.col.size(), -1);
  par_for(n, [&](int64_t lo, int64_t hi, int) {  // every row writes its own positions
    for (int64_t r = lo; r < hi; ++r) {
      const int64_t o = inv[r];
      for (int64_t k = M.ptr[o]; k < M.ptr[o + 1]; ++k) {
        const int64_t q = S.pos(r, (int)(k - M.ptr[o]));
        S.col[q] = cperm ? (*cperm)[M.col[k]] : M.col[k];
        epos[k] = (int32_t)q;
      }
    }
  });
  return "";
}

// per-entry lists → per-position lists (items translated by ta / tb)
std::string to_pos(const Lists& L, const std::vector<int32_t>& epos, int64_t npos,
                   const std::vector<int32_t>* ta, const std::vector<int32_t>* tb, bool pair,
                   PosList& out, int64_t& items) {
  out = PosList();
  out.ptr.assign(npos + 1, 0);
  const int64_t ne = (int64_t)L.ptr.size() - 1;
  par_for(ne, [&](int64_t lo, int64_t hi, int) {
    for (int64_t e = lo; e < hi; ++e) out.ptr[epos[e] + 1] = (int32_t)(L.ptr[e + 1] - L.ptr[e]);
  });
  int64_t run = 0;
  for (int64_t q = 0; q < npos; ++q) {
    run += out.ptr[q + 1];
    if (run > INT32_MAX) return "AMG index lists too large for int32";
    out.ptr[q + 1] = (int32_t)run;
  }
  items += run;
  out.a.resize(run);
  if (pair) out.b.resize(run);
  par_for(ne, [&](int64_t lo, int64_t hi, int) {  // every entry fills its own position's list
    for (int64_t e = lo; e < hi; ++e) {
      int64_t d = out.ptr[epos[e]];
      for (int64_t t = L.ptr[e]; t < L.ptr[e + 1]; ++t, ++d) {
        out.a[d] = ta ? (*ta)[L.a[t]] : L.a[t];
        if (pair) out.b[d] = tb ? (*tb)[L.b[t]] : L.b[t];
      }
    }
  });
  return "";
}

}  // namespace

std::string build_amg(const Pattern& P, const std::vector<uint8_t>& active, int nd, AmgPlan& plan,
                      int max_levels, const AmgDistSpec* dist, const AmgStrength& strength,
                      const AmgLayout& lay) {
  max_levels = std::max(1, std::min(max_levels, kAmgMaxLevels));
  plan = AmgPlan();
  plan.nd = nd;
  if ((int64_t)active.size() != P.n_elems) return "internal: active size mismatch";
  const int64_t nf = P.n_free;
  const int world = dist ? dist->world : 1;
  if (dist) {
    if (world < 1 || (int64_t)dist->owner.size() != nf) return "internal: AMG owner size mismatch";
    for (int32_t o : dist->owner)
      if (o < 0 || o >= world) return "internal: AMG owner out of range";
  }
  std::string err;
  PhaseClock clk;
  // ---- stage 1, level 0: free rows, neighbours through active free-free elements
  std::vector<LevelCsr> lv(1);
  Lists a0;  // per A_0 entry: SELL slot positions of the assembled operator
  // level-0 strength (AmgStrength): per A_0 entry Σ ‖S_e‖ of its elements,
  // per row Σ ‖S_e‖ of every active incident element (its diagonal's estimate)
  const bool use_strength = strength.theta > 0.0;
  std::vector<double> w_entry, d_row;
  auto enorm = [&](int64_t i, int64_t j) {
    double v[3], L2 = 0.0;
    for (int c = 0; c < 3; ++c) {
      v[c] = P.xyz_perm[3 * j + c] - P.xyz_perm[3 * i + c];
      L2 += v[c] * v[c];
    }
    const double L = std::max(std::sqrt(L2), 1e-12), q = strength.kb_kax / (L * L);
    return std::sqrt(1.0 + q * q) / L;
  };
  if (use_strength) {
    d_row.assign(nf, 0.0);
    for (int64_t i = 0; i < nf; ++i) {
      const int64_t base = (int64_t)P.slice_ptr[i >> 6] * 64 + (i & 63);
      for (int t = 0; t < P.row_len[i]; ++t) {
        const int64_t pos = base + (int64_t)t * 64;
        const int32_t j = P.s_col[pos], e = P.s_elem[pos];
        if (j < 0 || e < 0 || !active[e]) continue;
        d_row[i] += enorm(i, j);
      }
    }
  }
  // level-0 natural order = the Pattern's (depth-first: hyphal chains
  // contiguous, so a slice's gathers hit few cache lines).  Measured and
  // dropped: a Hilbert-curve order of the nodes (C3: 2× the cache lines per
  // slice) and Cuthill–McKee (C3 21 iterations instead of 16, C5 49 instead
  // of 43 — the greedy aggregation follows the row order — for no gain per
  // iteration).
  auto level0_row = [&](int64_t i, RowSink& s, std::vector<double>* w) {
    thread_local std::vector<std::pair<int32_t, int32_t>> nb;  // (neighbour, SELL position)
    nb.clear();
    const int64_t base = (int64_t)P.slice_ptr[i >> 6] * 64 + (i & 63);
    for (int t = 0; t < P.row_len[i]; ++t) {
      const int64_t pos = base + (int64_t)t * 64;
      const int32_t j = P.s_col[pos], e = P.s_elem[pos];
      if (j < 0 || j >= nf || e < 0 || !active[e]) continue;
      nb.emplace_back(j, (int32_t)pos);
    }
    row_stable_sort(nb.begin(), nb.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    s.entry((int32_t)i);
    if (w) w->push_back(0.0);
    for (size_t t = 0; t < nb.size(); ++t) {
      if (t == 0 || nb[t].first != nb[t - 1].first) {
        s.entry(nb[t].first);
        if (w) w->push_back(0.0);
      }
      s.item(nb[t].second);
      if (w) w->back() += enorm(i, nb[t].first);
    }
  };
  if (!use_strength) {
    produce_rows(nf, lv[0].A, a0, false, [&](int64_t i, RowSink& s) { level0_row(i, s, nullptr); });
  } else {  // the strength weights in row order: one thread
    RowSink s;
    for (int64_t i = 0; i < nf; ++i) {
      s.begin_row();
      level0_row(i, s, &w_entry);
    }
    Csr& A = lv[0].A;
    A.n = nf;
    A.ptr.assign(nf + 1, 0);
    for (int64_t i = 0; i < nf; ++i) A.ptr[i + 1] = A.ptr[i] + s.rlen[i];
    A.col = std::move(s.col);
    a0.ptr.assign(A.col.size() + 1, 0);
    for (size_t k = 0; k < s.icnt.size(); ++k) a0.ptr[k + 1] = a0.ptr[k] + s.icnt[k];
    a0.a = std::move(s.a);
  }
  // ---- coarsen until every row is isolated (the coarsest level is then
  // block diagonal and its block-Jacobi inverse is exact).  The aggregation
  // ignores the ranks: the distributed hierarchy IS the one-partition
  // hierarchy, so the multi-GPU solve needs the one-partition iteration count
  // (an aggregation kept inside each rank's rows, as PETSc's GAMG does, cost
  // 19 → 25 / 28 / 34 iterations at 2 / 4 / 8 ranks on a grown 165k-DOF
  // network: its cut couplings are strong).  Aggregates crossing a cut only
  // widen the halos.
  std::vector<uint8_t> strong0;
  if (use_strength) {
    const Csr& A = lv[0].A;
    strong0.assign(A.col.size(), 1);
    for (int64_t i = 0; i < A.n; ++i)
      for (int64_t k = A.ptr[i] + 1; k < A.ptr[i + 1]; ++k)
        strong0[k] = w_entry[k] >= strength.theta * std::sqrt(d_row[i] * d_row[A.col[k]]);
  }
  clk.lap("level-0 rows");
  for (int l = 0;; ++l) {
    LevelCsr& L = lv[l];
    const int64_t na = aggregate(L.A, L.agg, l == 0 && use_strength ? &strong0 : nullptr);
    clk.lap(l == 0 ? "aggregate l0" : "aggregate l>0");
    if (na == 0 || l + 1 == max_levels) {
      plan.capped = na > 0;  // couplings left: the coarsest block Jacobi is then inexact
      L.agg.clear();
      break;
    }
    L.nc = na;
    Csr An;
    if (!(err = coarsen(L, An)).empty()) return err;
    clk.lap(l == 0 ? "coarsen l0 (P, AP, A1)" : "coarsen l>0");
    lv.emplace_back();
    lv.back().A = std::move(An);
  }
  // ---- distributed: level l stays split while it has more than rep_rows
  // rows (level 0 always); an aggregate belongs to the rank holding most of
  // its rows (ties: the lowest rank).  Level n_dist, the first replicated one,
  // keeps its owners too: each rank restricts into its own rows of it.
  std::vector<std::vector<int32_t>> own;  // natural-order owners of levels [0, n_dist]
  int n_dist = 0;
  if (dist) {
    own.push_back(dist->owner);
    n_dist = 1;
    while (n_dist < (int)lv.size() && lv[n_dist].A.n > dist->rep_rows) ++n_dist;
    for (int l = 0; l < n_dist && l + 1 < (int)lv.size(); ++l) {
      const LevelCsr& L = lv[l];
      std::vector<std::pair<int32_t, int32_t>> ao;  // (aggregate, owner)
      for (int64_t i = 0; i < L.A.n; ++i)
        if (L.agg[i] >= 0) ao.emplace_back(L.agg[i], own[l][i]);
      std::sort(ao.begin(), ao.end());
      std::vector<int32_t> o(L.nc, 0);
      for (size_t a = 0; a < ao.size();) {
        size_t b = a, best = 0;
        int32_t who = ao[a].second;
        while (b < ao.size() && ao[b].first == ao[a].first) {
          size_t c = b;
          while (c < ao.size() && ao[c].first == ao[b].first && ao[c].second == ao[b].second) ++c;
          if (c - b > best) {
            best = c - b;
            who = ao[b].second;
          }
          b = c;
        }
        o[ao[a].first] = who;
        a = b;
      }
      own.push_back(std::move(o));
    }
  }
  plan.world = world;
  plan.n_dist = n_dist;
  clk.lap("owners");
  // ---- stage 2: row labels per level (sort key: the level's A row plus, for
  // a coarse level, its R row — the two SELL matrices its rows index in the
  // V-cycle; equal keys keep their natural order, which is what keeps a
  // slice's gathers local: splitting them further by the A·P length too cost
  // C3's level 0 18 → 31 B of cache lines per 16-B entry)
  const int nlev = (int)lv.size();
  std::vector<std::vector<int32_t>> perm(nlev);
  plan.lev.resize(nlev);
  // Z-order labels (AmgLayout): decided on level 0's natural-order locality
  bool spatial = !dist && lay.spatial > 0;
  if (!dist && lay.spatial < 0) {
    const Csr& A = lv[0].A;
    int64_t off = 0, far = 0;
    for (int64_t i = 0; i < A.n; ++i)
      for (int64_t k = A.ptr[i] + 1; k < A.ptr[i + 1]; ++k) {
        ++off;
        far += std::llabs((long long)A.col[k] - (long long)i) > 4096;
      }
    spatial = off > 0 && (double)far > lay.far_frac * (double)off;
  }
  plan.spatial = spatial;
  std::vector<double> cxyz;  // natural-order coordinates of the current level's rows
  std::vector<std::vector<int32_t>> bases(nlev);  // per level: its Z-order (spatial)
  if (spatial) {
    cxyz.assign(3 * (size_t)nf, 0.0);
    for (int64_t i = 0; i < nf; ++i)
      for (int c = 0; c < 3; ++c) cxyz[3 * i + c] = P.xyz_perm[3 * i + c];
  }
  for (int l = 0; l < nlev; ++l) {
    const int64_t n = lv[l].A.n;
    std::vector<int64_t> key(n);
    for (int64_t i = 0; i < n; ++i) key[i] = lv[l].A.len(i) + (l && !lay.by_a ? lv[l - 1].R.len(i) : 0);
    // levels [0, n_dist] owner-major (level n_dist: its rows are produced by
    // their rank's restriction, then gathered by every rank)
    const bool om = dist && l <= n_dist && l < (int)own.size();
    std::vector<int32_t> base;
    if (spatial) {
      base = morton_order(cxyz, n);
      if (l + 1 < nlev) {  // the next level's coordinates: centroids of the aggregates
        std::vector<double> nx(3 * (size_t)lv[l].nc, 0.0);
        std::vector<int64_t> cnt(lv[l].nc, 0);
        for (int64_t i = 0; i < n; ++i) {
          const int32_t a = lv[l].agg[i];
          if (a < 0) continue;
          ++cnt[a];
          for (int c = 0; c < 3; ++c) nx[3 * a + c] += cxyz[3 * i + c];
        }
        for (int64_t a = 0; a < lv[l].nc; ++a)
          for (int c = 0; c < 3; ++c) nx[3 * a + c] /= (double)std::max<int64_t>(cnt[a], 1);
        cxyz.swap(nx);
      }
    }
    perm[l] = sort_perm(key, om ? &own[l] : nullptr, world, om ? &plan.lev[l].own : nullptr,
                        spatial ? &base : nullptr);
    bases[l] = std::move(base);
    if (om) {
      plan.lev[l].owner.assign(n, 0);
      for (int64_t i = 0; i < n; ++i) plan.lev[l].owner[perm[l][i]] = own[l][i];
    }
  }
  clk.lap("row labels (sort_perm)");
  plan.row0.assign(nf, 0);
  for (int64_t i = 0; i < nf; ++i) plan.row0[perm[0][i]] = (int32_t)i;
  for (int l = 0; l < nlev; ++l) {
    plan.lev[l].nat.assign(lv[l].A.n, 0);
    for (int64_t i = 0; i < lv[l].A.n; ++i) plan.lev[l].nat[perm[l][i]] = (int32_t)i;
  }
  std::vector<std::vector<int32_t>> eA(nlev);
  for (int l = 0; l < nlev; ++l)
    if (!(err = layout(lv[l].A, perm[l], &perm[l], plan.lev[l].A, eA[l])).empty()) return err;
  if (!(err = to_pos(a0, eA[0], plan.lev[0].A.n_pos(), nullptr, nullptr, false, plan.a0, plan.pair_items)).empty())
    return err;
  clk.lap("A layouts + a0 lists");
  for (int l = 0; l < nlev; ++l) {
    AmgLevel& out = plan.lev[l];
    LevelCsr& L = lv[l];
    out.coarsest = l + 1 == nlev;
    if (out.coarsest) continue;
    out.nc = L.nc;
    out.agg.assign(L.A.n, -1);
    for (int64_t i = 0; i < L.A.n; ++i)
      out.agg[perm[l][i]] = L.agg[i] >= 0 ? perm[l + 1][L.agg[i]] : -1;
    std::vector<int32_t> eP, eR, eAP;
    if (!(err = layout(L.P, perm[l], &perm[l + 1], out.P, eP)).empty()) return err;
    if (!(err = layout(L.R, perm[l + 1], &perm[l], out.R, eR)).empty()) return err;
    // A·P is only reached through the setup's index lists, so its rows get a
    // labelling of their own, by A·P length (C3 level 0: 1.69 M → 0.92 M
    // positions)
    std::vector<int32_t> pap;
    {
      std::vector<int64_t> key(L.A.n);
      for (int64_t i = 0; i < L.A.n; ++i) key[i] = L.AP.len(i);
      const bool om = dist && l < n_dist;
      pap = sort_perm(key, om ? &own[l] : nullptr, world, om ? &out.ap_own : nullptr,
                      spatial ? &bases[l] : nullptr);
      if (!(err = layout(L.AP, pap, &perm[l + 1], out.AP, eAP)).empty()) return err;
      if (om) {
        out.aprow.assign(L.A.n, 0);
        for (int64_t i = 0; i < L.A.n; ++i) out.aprow[perm[l][i]] = pap[i];
      }
    }
    // the compact cycle's P̃ on A·P's entries AND layout (its rows by A·P
    // length: C3 level 0 fills 88 % of its positions, 48 % in the level's own
    // row order), pt_row naming each row's level row; R̃ = P̃ᵀ
    {
      std::vector<int32_t> eRT;
      out.PT = out.AP;  // the same pattern and labels as A·P's layout
      const std::vector<int32_t>& ePT = eAP;
      out.pt_row.assign(L.A.n, 0);
      for (int64_t i = 0; i < L.A.n; ++i) out.pt_row[pap[i]] = perm[l][i];
      out.pt_ap.assign(out.PT.n_pos(), -1);
      out.pt_p.assign(out.PT.n_pos(), -1);
      par_for(L.A.n, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {  // both rows ascending in J: merge
          int64_t k = L.P.ptr[i];
          for (int64_t e = L.AP.ptr[i]; e < L.AP.ptr[i + 1]; ++e) {
            out.pt_ap[ePT[e]] = eAP[e];
            while (k < L.P.ptr[i + 1] && L.P.col[k] < L.AP.col[e]) ++k;
            if (k < L.P.ptr[i + 1] && L.P.col[k] == L.AP.col[e]) out.pt_p[ePT[e]] = eP[k];
          }
        }
      });
      Csr RT;  // transpose of A·P: coarse row J → fine rows ascending
      std::vector<int32_t> rt_e(L.AP.col.size());
      RT.n = L.nc;
      RT.ptr.assign(L.nc + 1, 0);
      for (int32_t J : L.AP.col) RT.ptr[J + 1]++;
      for (int64_t J = 0; J < L.nc; ++J) RT.ptr[J + 1] += RT.ptr[J];
      RT.col.resize(L.AP.col.size());
      std::vector<int64_t> fill(RT.ptr.begin(), RT.ptr.end() - 1);
      for (int64_t i = 0; i < L.A.n; ++i)
        for (int64_t e = L.AP.ptr[i]; e < L.AP.ptr[i + 1]; ++e) {
          const int64_t t = fill[L.AP.col[e]]++;
          RT.col[t] = (int32_t)i;
          rt_e[t] = (int32_t)e;
        }
      // R̂'s rows are the down sweep's widest (C5 level 0: 30 blocks on average,
      // 142 at most): their own labelling by R̂ length inside windows, as P̃'s
      // (in the level's order C5 fills 75 % of the padded positions)
      std::vector<int32_t> prt;
      {
        std::vector<int64_t> key(L.nc);
        for (int64_t J = 0; J < L.nc; ++J) key[J] = RT.ptr[J + 1] - RT.ptr[J];
        // distributed: owner-major by the coarse row's owner, so a rank's R̂
        // rows are one range (the compact cycle on a split level)
        const bool om1 = dist && l + 1 <= n_dist && l + 1 < (int)own.size();
        prt = sort_perm(key, om1 ? &own[l + 1] : nullptr, world, om1 ? &out.rt_own : nullptr,
                        spatial ? &bases[l + 1] : nullptr);
      }
      if (!(err = layout(RT, prt, &perm[l], out.RT, eRT)).empty()) return err;
      out.rt_row.assign(L.nc, 0);
      for (int64_t J = 0; J < L.nc; ++J) out.rt_row[prt[J]] = perm[l + 1][J];
      out.rt_pt.assign(out.RT.n_pos(), -1);
      par_for((int64_t)rt_e.size(), [&](int64_t lo, int64_t hi, int) {
        for (int64_t t = lo; t < hi; ++t) out.rt_pt[eRT[t]] = ePT[rt_e[t]];
      });
    }
    if (!(err = to_pos(L.pv, eP, out.P.n_pos(), &eA[l], nullptr, false, out.pv, plan.pair_items)).empty())
      return err;
    out.rp.assign(out.R.n_pos(), -1);
    par_for((int64_t)L.rp.size(), [&](int64_t lo, int64_t hi, int) {
      for (int64_t e = lo; e < hi; ++e) out.rp[eR[e]] = eP[L.rp[e]];
    });
    if (!(err = to_pos(L.ap, eAP, out.AP.n_pos(), &eA[l], &eP, true, out.ap, plan.pair_items)).empty())
      return err;
    if (!(err = to_pos(L.ac, eA[l + 1], plan.lev[l + 1].A.n_pos(), &eP, &eAP, true, out.ac, plan.pair_items))
             .empty())
      return err;
    clk.lap(l == 0 ? "level 0 P/R/AP/RT layouts+lists" : "level>0 layouts+lists");
  }
  return "";
}

std::string build_amg_halo(const Pattern& P, const std::vector<uint8_t>& active, const AmgPlan& plan,
                           const std::vector<int32_t>& xsend_rows, const std::vector<int32_t>& xrecv_rows,
                           AmgHalo& halo) {
  halo = AmgHalo();
  const int64_t nf = P.n_free;
  if ((int64_t)plan.row0.size() != nf) return "internal: AMG plan / pattern mismatch";
  std::vector<int32_t> lev0(P.n_nodes, -1), recv(P.n_nodes, -1);
  for (int64_t i = 0; i < nf; ++i) lev0[plan.row0[i]] = (int32_t)i;
  for (size_t k = 0; k < xrecv_rows.size(); ++k) recv[xrecv_rows[k]] = (int32_t)k;
  for (int32_t r : xsend_rows) {  // a grip (fixed) node travels as zeros: -1
    if (r < 0 || r >= P.n_nodes) return "internal: halo send node out of range";
    halo.send_rows.push_back(r < nf ? lev0[r] : -1);
  }
  halo.gptr.assign(nf + 1, 0);
  for (int64_t i = 0; i < nf; ++i) {  // level-0 row i = Pattern row row0[i]
    const int64_t r = plan.row0[i];
    const int64_t base = (int64_t)P.slice_ptr[r >> 6] * 64 + (r & 63);
    for (int t = 0; t < P.row_len[r]; ++t) {
      const int64_t pos = base + (int64_t)t * 64;
      const int32_t j = P.s_col[pos], e = P.s_elem[pos];
      if (j < nf || e < 0 || !active[e] || P.code[j] != kGhost) continue;
      if (recv[j] < 0) return "internal: a ghost free neighbour is missing from the halo plan";
      halo.gslot.push_back((int32_t)pos);
      halo.grecv.push_back(recv[j]);
    }
    halo.gptr[i + 1] = (int32_t)halo.gslot.size();
  }
  return "";
}

// The chain-piece multicolour order of a one-level plan (amg.hpp SweepPlan).
// PETSc's ICC / SOR run in the natural node order, a sequential triangular
// solve; on this network (mean degree ≈ 2: hyphal chains between branch and
// fusion points) the order that matters is the one along the chains, so the
// pieces keep it where a GPU can: tools/icc_lab.py measured IC(0) to rtol 1e-8
// on the reference network at 395 iterations in the natural order, 392–410 in
// this order with 8–128-row pieces, 639 in a point red-black order (Jacobi:
// 1,262 block / 1,644 point).  Pieces hold at most 64 rows (one wave: the
// sweeps scan a piece across its lanes, sweep.hip).
std::string build_sweep(const AmgPlan& plan, int piece_len, SweepPlan& out) {
  out = SweepPlan();
  piece_len = std::min(64, std::max(1, piece_len));
  out.piece_len = piece_len;
  out.cwave.assign(1, 0);
  out.lo_ptr.assign(1, 0);
  out.up_ptr.assign(1, 0);
  if (plan.lev.empty()) return "";
  const SellPat& A = plan.lev[0].A;
  const int64_t n = A.n;
  out.n = n;
  if (n == 0) return "";
  std::vector<int32_t> nat(n);
  if ((int64_t)plan.lev[0].nat.size() == n) nat = plan.lev[0].nat;
  else std::iota(nat.begin(), nat.end(), 0);
  // A_0's off-diagonal couplings per row, ascending neighbour
  std::vector<int64_t> aptr(n + 1, 0);
  std::vector<std::pair<int32_t, int32_t>> adj;  // (neighbour, A position)
  for (int64_t i = 0; i < n; ++i) {
    const size_t a0 = adj.size();
    for (int k = 1; k < A.rlen[i]; ++k) {
      const int64_t q = A.pos(i, k);
      const int32_t j = A.col[q];
      if (j < 0 || j == i) continue;
      adj.emplace_back(j, (int32_t)q);
    }
    // neighbours in natural (aggregation / depth-first) order, so the pieces
    // do not depend on the level's device labels
    std::sort(adj.begin() + a0, adj.end(), [&](const auto& x, const auto& y) { return nat[x.first] < nat[y.first]; });
    aptr[i + 1] = (int64_t)adj.size();
  }
  std::vector<int32_t> roots(n);
  for (int64_t i = 0; i < n; ++i) roots[nat[i]] = (int32_t)i;
  // depth-first order and tree parents
  std::vector<int32_t> order, parent(n, -1);
  order.reserve(n);
  std::vector<uint8_t> seen(n, 0);
  std::vector<std::pair<int32_t, int64_t>> st;
  for (const int32_t root : roots) {
    if (seen[root]) continue;
    seen[root] = 1;
    order.push_back((int32_t)root);
    st.emplace_back((int32_t)root, aptr[root]);
    while (!st.empty()) {
      const int32_t v = st.back().first;
      const int64_t k = st.back().second;
      if (k == aptr[v + 1]) {
        st.pop_back();
        continue;
      }
      st.back().second = k + 1;
      const int32_t w = adj[k].first;
      if (seen[w]) continue;
      seen[w] = 1;
      parent[w] = v;
      order.push_back(w);
      st.emplace_back(w, aptr[w]);
    }
  }
  // pieces: runs of the order along tree edges, each row coupled inside its
  // piece to its predecessor only
  std::vector<int32_t> piece(n, -1), pstart, plen;
  {
    int32_t cur = -1, last = -1;
    for (size_t t = 0; t < order.size(); ++t) {
      const int32_t v = order[t];
      bool cont = cur >= 0 && plen[cur] < piece_len && parent[v] == last;
      for (int64_t k = aptr[v]; cont && k < aptr[v + 1]; ++k)
        if (adj[k].first != last && piece[adj[k].first] == cur) cont = false;
      if (!cont) {
        cur = (int32_t)pstart.size();
        pstart.push_back((int32_t)t);
        plen.push_back(0);
      }
      piece[v] = cur;
      ++plen[cur];
      last = v;
    }
  }
  const int64_t np = (int64_t)pstart.size();
  out.n_pieces = np;
  // greedy piece colouring in piece (depth-first) order
  std::vector<int32_t> pcol(np, -1);
  for (int64_t p = 0; p < np; ++p) {
    uint64_t used = 0;
    for (int32_t t = pstart[p]; t < pstart[p] + plen[p]; ++t) {
      const int32_t v = order[t];
      for (int64_t k = aptr[v]; k < aptr[v + 1]; ++k) {
        const int32_t q = piece[adj[k].first];
        if (q != p && pcol[q] >= 0) used |= uint64_t(1) << pcol[q];
      }
    }
    int c = 0;
    while (c < 63 && (used >> c & 1)) ++c;
    pcol[p] = c;
    out.colors = std::max(out.colors, c + 1);
  }
  // waves: a colour's pieces packed into the 64 lanes of its waves by
  // best-fit decreasing (longest piece first, into the open wave with the
  // least room that holds it; ties in depth-first order) — a piece's rows on
  // consecutive lanes, never across two waves; the lanes left over are
  // padding.  Depth-first first-fit left C3's colour 1 at 68 % of its lanes.
  std::vector<int64_t> ent0(np);  // entry of a piece's first row
  int64_t ne = 0;
  for (int c = 0; c < out.colors; ++c) {
    std::vector<int32_t> ps;
    for (int64_t p = 0; p < np; ++p)
      if (pcol[p] == c) ps.push_back((int32_t)p);
    std::stable_sort(ps.begin(), ps.end(), [&](int32_t a, int32_t b) { return plen[a] > plen[b]; });
    const int64_t w0 = ne / 64;
    std::vector<int32_t> room, wmax;            // per wave of this colour
    std::vector<std::vector<int32_t>> by_room(65);  // open waves by lanes left
    for (const int32_t p : ps) {
      int32_t w = -1;
      for (int r = plen[p]; r <= 64 && w < 0; ++r) {
        auto& b = by_room[r];
        while (!b.empty() && room[b.back()] != r) b.pop_back();  // stale entries
        if (!b.empty()) {
          w = b.back();
          b.pop_back();
        }
      }
      if (w < 0) {
        w = (int32_t)room.size();
        room.push_back(64);
        wmax.push_back(0);
      }
      ent0[p] = 64 * (w0 + w) + (64 - room[w]);
      room[w] -= plen[p];
      wmax[w] = std::max(wmax[w], plen[p]);
      by_room[room[w]].push_back(w);
    }
    for (size_t w = 0; w < room.size(); ++w) {
      int st = 0;
      while ((1 << st) < wmax[w]) ++st;
      out.wsteps.push_back(st);
    }
    ne += 64 * (int64_t)room.size();
    out.cwave.push_back((int32_t)(ne / 64));
    if (ne > INT32_MAX) return "sweep plan: too many entries";
  }
  out.row.assign(ne, -1);
  out.ppos.assign(ne, -1);
  out.dpos.assign(ne, -1);
  std::vector<int32_t> ent(n);
  for (int64_t p = 0; p < np; ++p)
    for (int32_t s = 0; s < plen[p]; ++s) ent[order[pstart[p] + s]] = (int32_t)(ent0[p] + s);
  auto pos_of = [&](int32_t v, int32_t j) -> int32_t {
    for (int64_t k = aptr[v]; k < aptr[v + 1]; ++k)
      if (adj[k].first == j) return adj[k].second;
    return -1;
  };
  for (int64_t p = 0; p < np; ++p)
    for (int32_t s = 0; s < plen[p]; ++s) {
      const int32_t v = order[pstart[p] + s];
      const int32_t e = ent[v];
      out.row[e] = v;
      out.dpos[e] = (int32_t)A.pos(v, 0);
      if (s > 0) {
        out.ppos[e] = pos_of(v, order[pstart[p] + s - 1]);
        if (out.ppos[e] < 0) return "internal: sweep piece without a predecessor coupling";
      }
    }
  // cross couplings in entry order
  out.lo_ptr.assign(ne + 1, 0);
  out.up_ptr.assign(ne + 1, 0);
  for (int64_t e = 0; e < ne; ++e) {
    const int32_t v = out.row[e];
    if (v >= 0) {
      const int32_t p = piece[v];
      const int32_t s = (int32_t)(e - ent0[p]);
      const int32_t prev = s > 0 ? order[pstart[p] + s - 1] : -1;
      const int32_t next = s + 1 < plen[p] ? order[pstart[p] + s + 1] : -1;
      for (int64_t k = aptr[v]; k < aptr[v + 1]; ++k) {
        const int32_t j = adj[k].first;
        if (j == prev || j == next) continue;
        const int32_t cj = pcol[piece[j]], cv = pcol[p];
        if (cj == cv) return "internal: sweep cross coupling inside one colour";
        (cj < cv ? out.lo_ent : out.up_ent).push_back(ent[j]);
        (cj < cv ? out.lo_pos : out.up_pos).push_back(adj[k].second);
      }
    }
    out.lo_ptr[e + 1] = (int32_t)out.lo_ent.size();
    out.up_ptr[e + 1] = (int32_t)out.up_ent.size();
  }
  return "";
}

}  // namespace mfea
