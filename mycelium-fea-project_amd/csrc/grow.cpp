// Native network producer: the hyphal growth model of the
// reference's C++ simulator, src/mycelium_sim_2D.cpp (process functions
// :236-414, driver loop :529-588, geometry export :477-515), re-laid out for
// networks of millions of segments:
//
//   * segments live in flat arrays (structure of arrays) addressed by a
//     segment id; a hypha is a chain (first/last id + a `next` link), so the
//     reference's hypha-major iteration order ("for h in hyphae, for s in
//     h.segments") is a flattened order array rebuilt once per step;
//   * the spatial hash is a dense voxel grid over the bounding box, built by a
//     stable parallel counting sort (entries within a voxel keep the
//     reference's insertion order), plus per-voxel lists for the entries the
//     anastomosis pass appends (:411);
//   * anastomosis searches run in parallel against the pre-pass state, then a
//     serial pass in hypha order accepts each result unless an earlier
//     anastomosis in the same pass touched one of the tip's 27 voxels (then it
//     re-searches serially) — the outcome is the reference's sequential one;
//   * per-hypha substrate translocation runs in parallel (hyphae are
//     independent; within a hypha the clamp order of :260-264 is kept);
//   * everything the reference computes in a fixed order (the RNG draws, the
//     uptake chain over E, the total-length sum) stays serial in that order,
//     so a run with the reference's parameters and seed writes byte-identical
//     nodes.csv / elements.csv / mycelium_growth_stats.csv / snapshots.
//
// The RNG is std::mt19937_64 + std::uniform_real_distribution<double>, the
// reference's generator (:50-52).  Numbers are written as libstdc++'s
// `ostream << double` does (printf "%g", 6 significant digits) via
// std::to_chars; node identity is the "%.6f_%.6f_%.6f" key of :484.
#include <algorithm>
#include <array>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mfea.h"

namespace mfea {
namespace {

constexpr double kPi = 3.14159265358979323846;  // the simulator's π (:13), not the FEA's 3.14

struct V3 {
  double x, y, z;
};
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 mul(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot3(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double norm3(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

template <class F>
void parallel_for(int64_t n, int threads, F&& f) {
  // f(lo, hi, t) over contiguous chunks; chunk t covers [n·t/T, n·(t+1)/T)
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (n + 4095) / 4096));
  if (T == 1) {
    f((int64_t)0, n, 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T, t); });
  f((int64_t)0, n / T, 0);
  for (auto& x : th) x.join();
}

// printf("%g") of libstdc++'s default ostream precision (6), and "%.6f"
inline char* put_g6(char* p, double v) { return std::to_chars(p, p + 32, v, std::chars_format::general, 6).ptr; }
inline char* put_i64(char* p, int64_t v) { return std::to_chars(p, p + 24, v).ptr; }

// the "%.6f" text of v as an exact integer key (micro-units); "-0.000000"
// (a tiny negative value) is a different key than "0.000000", as in :484
inline int64_t key6(double v) {
  char b[48];
  char* e = std::to_chars(b, b + sizeof(b), v, std::chars_format::fixed, 6).ptr;
  int64_t k = 0;
  bool neg = false;
  for (char* p = b; p < e; ++p) {
    if (*p == '-') neg = true;
    else if (*p != '.') k = k * 10 + (*p - '0');
  }
  if (neg) return k == 0 ? INT64_MIN : -k;
  return k;
}

struct Cuboid {
  V3 c, size;
  bool substrate;
  double E, mu;
  bool contains(V3 p) const {  // :112-117
    const V3 h = mul(size, 0.5);
    return p.x >= (c.x - h.x - 1e-12) && p.x <= (c.x + h.x + 1e-12) && p.y >= (c.y - h.y - 1e-12) &&
           p.y <= (c.y + h.y + 1e-12) && p.z >= (c.z - h.z - 1e-12) && p.z <= (c.z + h.z + 1e-12);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
struct GrowNet {
  mfea_grow_params p{};
  std::mt19937_64 rng;
  int threads = 1;
  // segments (SoA)
  std::vector<double> sx, sy, sz, ex, ey, ez, th, ph, I;
  std::vector<char> st;
  std::vector<int64_t> next;
  // hyphae: chains of segment ids
  std::vector<int64_t> first, last, count;
  int64_t n_sites = 0;
  std::vector<Cuboid> cub;
  // per-step hypha-major order of segment ids, and the stats history
  std::vector<int64_t> ord;
  std::string history;
  // spatial hash (voxel grid over the bounding box of the entries)
  double vs = 0.1;
  int64_t gx0 = 0, gy0 = 0, gz0 = 0, gnx = 0, gny = 0, gnz = 0;
  std::vector<int64_t> vstart, ventry;  // CSR: voxel → entries (segment ids, insertion order)
  struct Geo {
    double sx, sy, sz, ex, ey, ez;
  };
  std::vector<Geo> vgeo;  // each CSR entry's geometry at the rebuild, contiguous per voxel
  double reject2 = 0;     // squared midpoint distance beyond which no entry can be within tol
  double reject2_cur = 0; // the same for the current geometry (tips may have grown by tol)
  std::unordered_map<int64_t, std::vector<int64_t>> vextra;  // entries appended by the anastomosis pass
  std::vector<uint8_t> vdirty;
  std::vector<int32_t> vk, cntbuf;  // rebuild scratch: voxel per entry, per-chunk counts
  std::vector<int64_t> hoff;        // per hypha: first position in ord (build_order)
  std::vector<double> lenbuf;       // stats scratch
  // exported geometry
  std::vector<int64_t> node_of;  // 2 per segment in hypha-major order
  std::vector<double> nxyz;      // first-appearance coordinates
  int64_t n_nodes = 0, n_elems = 0;

  double u01() { return std::uniform_real_distribution<double>(0.0, 1.0)(rng); }
  double urange(double a, double b) { return a + (b - a) * u01(); }
  V3 S(int64_t i) const { return {sx[i], sy[i], sz[i]}; }
  V3 Ee(int64_t i) const { return {ex[i], ey[i], ez[i]}; }
  double len(int64_t i) const { return norm3(sub(Ee(i), S(i))); }
  int64_t add_seg(V3 s, V3 e, double t, double f, double Ii, char state) {
    sx.push_back(s.x), sy.push_back(s.y), sz.push_back(s.z);
    ex.push_back(e.x), ey.push_back(e.y), ez.push_back(e.z);
    th.push_back(t), ph.push_back(f), I.push_back(Ii), st.push_back(state), next.push_back(-1);
    return (int64_t)sx.size() - 1;
  }
  int64_t new_hypha(int64_t s) {
    first.push_back(s), last.push_back(s), count.push_back(1);
    return (int64_t)first.size() - 1;
  }
  void append(int64_t h, int64_t s) {
    next[last[h]] = s;
    last[h] = s;
    ++count[h];
  }

  void build_order() {
    const int64_t H = (int64_t)first.size();
    std::vector<int64_t>& off = hoff;
    off.assign(H + 1, 0);
    for (int64_t h = 0; h < H; ++h) off[h + 1] = off[h] + count[h];
    ord.resize(off[H]);
    parallel_for(H, threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t h = lo; h < hi; ++h) {
        int64_t k = off[h];
        for (int64_t s = first[h]; s >= 0; s = next[s]) ord[k++] = s;
      }
    });
  }

  // :161-181 — H0_per_point straight hyphae per inoculation site
  void init() {
    rng.seed(p.seed);
    const int64_t sites = (int64_t)p.inoc_nx * p.inoc_ny;
    n_sites = sites;
    const double x0 = -(p.inoc_nx - 1) * p.inoc_dist / 2.0, y0 = -(p.inoc_ny - 1) * p.inoc_dist / 2.0;
    const double per_site = p.omega0 / std::max<int64_t>(1, sites);
    for (int i = 0; i < p.inoc_nx; ++i)
      for (int j = 0; j < p.inoc_ny; ++j) {
        const V3 pt{x0 + i * p.inoc_dist, y0 + j * p.inoc_dist, 0.0};  // :143-156
        const double per_seg = per_site / double(p.h0_per_point);
        for (int k = 0; k < p.h0_per_point; ++k) {
          const double t = u01() * kPi;
          const double f = u01() * 2.0 * kPi;
          const V3 d{std::cos(f), std::sin(f), 0.0};
          new_hypha(add_seg(pt, add(pt, mul(d, p.h0)), t, f, per_seg / p.h0, 'A'));
        }
      }
    const double D = p.dish_size, W = p.wall_thickness;
    cub.push_back({{0, 0, 0}, {D, p.substrate_width, 0.1}, true, p.substrate_E, 1e8});  // :546-551
    cub.push_back({{0, D / 2 + W / 2, 0}, {D, W, W}, false, 0.0, 1e8});
    cub.push_back({{0, -D / 2 - W / 2, 0}, {D, W, W}, false, 0.0, 1e8});
    cub.push_back({{D / 2 + W / 2, 0, 0}, {W, D, W}, false, 0.0, 1e8});
    cub.push_back({{-D / 2 - W / 2, 0, 0}, {W, D, W}, false, 0.0, 1e8});
  }

  // :236-265 — exchange with the predecessor; deltas from the pre-step
  // values, applied in the reference's update-list order with clamping
  void translocate() {
    const double dtD = p.dt * p.D, cap = p.M_cap;
    const int64_t H = (int64_t)first.size();
    auto clampI = [cap](double v) {
      if (v < 0.0) v = 0.0;
      if (v > cap) v = cap;
      return v;
    };
    if ((int64_t)hoff.size() != H + 1) build_order();
    parallel_for(H, threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t h = lo; h < hi; ++h) {
        const int64_t* o = ord.data() + hoff[h];
        const int64_t cnt_h = hoff[h + 1] - hoff[h];
        int64_t pr = o[0];
        double pr_old = I[pr], pr_len = len(pr);
        for (int64_t k = 1; k < cnt_h; ++k) {
          const int64_t s = o[k];
          const double s_old = I[s], s_len = len(s);
          const double denom = (s_len + pr_len) / 2.0;
          if (denom > 0.0) {
            const double delta = dtD * (pr_old - s_old) / denom;
            const double new_s = s_old + delta, new_p = pr_old - delta;
            double adj = delta;
            if (new_s < 0) adj = -s_old;
            else if (new_s > cap) adj = cap - s_old;
            else if (new_p < 0) adj = pr_old;
            else if (new_p > cap) adj = cap - pr_old;
            I[s] = clampI(I[s] + adj);    // (s, +adj) ...
            I[pr] = clampI(I[pr] + -adj);  // ... then (pred, −adj)
          }
          pr_old = s_old, pr_len = s_len;
          pr = s;
        }
      }
    });
  }

  std::pair<double, double> rand_dir(double phi) {  // :61-66
    const double dph = (u01() - 0.5) * p.lambda_angle;
    return {kPi / 2.0, phi + dph};
  }

  // :345-386 — serial: the draws follow the hypha order
  void grow() {
    const int64_t H = (int64_t)first.size();
    const double cost = p.c_g * p.h0;
    std::vector<int64_t> children;
    for (int64_t h = 0; h < H; ++h) {
      const int64_t t = last[h];
      if (st[t] != 'A') continue;
      const double L = len(t);
      const double avail = I[t] * L;
      if (avail < cost) continue;
      const bool branch = (u01() < p.P_branch) && (avail >= 2.0 * cost);
      const V3 tip = Ee(t);
      if (branch) {
        I[t] = std::max(0.0, (avail - 2.0 * cost) / L);
        st[t] = 'P';
        const auto a = rand_dir(ph[t]);
        const V3 d0{std::cos(a.second), std::sin(a.second), 0.0};
        const auto b = rand_dir(ph[t]);
        const V3 d1{std::cos(b.second), std::sin(b.second), 0.0};
        const double Ih = 0.5 * I[t];
        append(h, add_seg(tip, add(tip, mul(d0, p.h0)), a.first, a.second, Ih, 'A'));
        children.push_back(add_seg(tip, add(tip, mul(d1, p.h0)), b.first, b.second, Ih, 'A'));
      } else {
        st[t] = 'P';
        I[t] = std::max(0.0, (avail - cost) / L);
        const auto a = rand_dir(ph[t]);
        const V3 d{std::cos(a.second), std::sin(a.second), 0.0};
        append(h, add_seg(tip, add(tip, mul(d, p.h0)), a.first, a.second, 0.5 * I[t], 'A'));
      }
    }
    for (int64_t c : children) new_hypha(c);
  }

  // voxel of a point (:190-195); -1 if outside the grid
  void vox(V3 q, int64_t& ix, int64_t& iy, int64_t& iz) const {
    ix = (int64_t)(int)std::floor(q.x / vs);
    iy = (int64_t)(int)std::floor(q.y / vs);
    iz = (int64_t)(int)std::floor(q.z / vs);
  }
  int64_t vid(int64_t ix, int64_t iy, int64_t iz) const {
    ix -= gx0, iy -= gy0, iz -= gz0;
    if (ix < 0 || iy < 0 || iz < 0 || ix >= gnx || iy >= gny || iz >= gnz) return -1;
    return (iz * gny + iy) * gnx + ix;
  }
  V3 mid(int64_t s) const { return mul(add(S(s), Ee(s)), 0.5); }

  // :209-217 — every segment at its midpoint voxel, hypha-major order
  void rebuild_hash() {
    const int64_t n = (int64_t)ord.size();
    const int T = std::max(1, threads);
    std::vector<std::array<int64_t, 6>> ext(T, {INT64_MAX, INT64_MAX, INT64_MAX, INT64_MIN, INT64_MIN, INT64_MIN});
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int t) {
      auto& e = ext[t];
      for (int64_t k = lo; k < hi; ++k) {
        int64_t x, y, z;
        vox(mid(ord[k]), x, y, z);
        e[0] = std::min(e[0], x), e[1] = std::min(e[1], y), e[2] = std::min(e[2], z);
        e[3] = std::max(e[3], x), e[4] = std::max(e[4], y), e[5] = std::max(e[5], z);
      }
    });
    std::array<int64_t, 6> g = ext[0];
    for (auto& e : ext)
      for (int i = 0; i < 3; ++i) g[i] = std::min(g[i], e[i]), g[i + 3] = std::max(g[i + 3], e[i + 3]);
    gx0 = g[0], gy0 = g[1], gz0 = g[2];
    gnx = g[3] - g[0] + 1, gny = g[4] - g[1] + 1, gnz = g[5] - g[2] + 1;
    const int64_t NV = gnx * gny * gnz;
    // stable counting sort, chunk-parallel: chunk t's entries of voxel v go
    // after chunks < t's entries of v (chunks as parallel_for cuts them)
    const int TT = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (n + 4095) / 4096));
    vk.resize(n);
    cntbuf.resize((size_t)TT * NV);
    parallel_for((int64_t)cntbuf.size(), threads, [&](int64_t lo, int64_t hi, int) {
      std::memset(cntbuf.data() + lo, 0, (size_t)(hi - lo) * sizeof(int32_t));
    });
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int t) {
      int32_t* c = cntbuf.data() + (size_t)t * NV;
      for (int64_t k = lo; k < hi; ++k) {
        int64_t x, y, z;
        vox(mid(ord[k]), x, y, z);
        vk[k] = (int32_t)vid(x, y, z);
        ++c[vk[k]];
      }
    });
    // voxel totals → starts (parallel over voxel ranges, serial scan of the
    // range sums), then each chunk's offset inside its voxel
    vstart.resize(NV + 1);
    const int VT = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (NV + 4095) / 4096));
    std::vector<int64_t> rsum(VT + 1, 0);
    parallel_for(NV, threads, [&](int64_t lo, int64_t hi, int t) {
      int64_t acc = 0;
      for (int64_t v = lo; v < hi; ++v) {
        int64_t tot = 0;
        for (int c = 0; c < TT; ++c) tot += cntbuf[(size_t)c * NV + v];
        vstart[v] = tot;
        acc += tot;
      }
      rsum[t + 1] = acc;
    });
    for (int t = 0; t < VT; ++t) rsum[t + 1] += rsum[t];
    parallel_for(NV, threads, [&](int64_t lo, int64_t hi, int t) {
      int64_t run = rsum[t];
      for (int64_t v = lo; v < hi; ++v) {
        const int64_t tot = vstart[v];
        vstart[v] = run;
        for (int c = 0; c < TT; ++c) {
          int32_t& cc = cntbuf[(size_t)c * NV + v];
          const int32_t x = cc;
          cc = (int32_t)(run - vstart[v]);  // offset inside the voxel
          run += x;
        }
        (void)tot;
      }
    });
    vstart[NV] = n;
    ventry.resize(n);
    vgeo.resize(n);
    std::vector<double> lmax(T, 0.0);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int t) {
      int32_t* c = cntbuf.data() + (size_t)t * NV;
      for (int64_t k = lo; k < hi; ++k) {
        const int64_t sgm = ord[k], at = vstart[vk[k]] + c[vk[k]]++;
        ventry[at] = sgm;
        vgeo[at] = Geo{sx[sgm], sy[sgm], sz[sgm], ex[sgm], ey[sgm], ez[sgm]};
        lmax[t] = std::max(lmax[t], len(sgm));
      }
    });
    // a point within tol of a segment is within L/2 + tol of its midpoint;
    // the bound is padded far above rounding so the exact test decides
    // every case it could accept
    double L = 0;
    for (double v : lmax) L = std::max(L, v);
    const double R = 0.5 * L + p.anastomosis_tol;
    reject2 = R * R * (1.0 + 1e-6) + 1e-18;
    const double Rc = 0.5 * (L + 2 * p.anastomosis_tol) + p.anastomosis_tol;
    reject2_cur = Rc * Rc * (1.0 + 1e-6) + 1e-18;
    vextra.clear();
    vdirty.resize(NV);
    parallel_for(NV, threads, [&](int64_t lo, int64_t hi, int) {
      std::memset(vdirty.data() + lo, 0, (size_t)(hi - lo));
    });
  }

  // :72-82
  static double pseg_dist(V3 q, V3 a, V3 b, V3* proj) {
    const V3 ap = sub(q, a), ab = sub(b, a);
    const double ab2 = dot3(ab, ab);
    if (ab2 < 1e-12) {
      *proj = a;
      return norm3(ap);
    }
    double t = dot3(ap, ab) / ab2;
    if (t < 0.0) t = 0.0;
    if (t > 1.0) t = 1.0;
    *proj = add(a, mul(ab, t));
    return norm3(sub(q, *proj));
  }

  // first entry of the 27 voxels around q (reference order :221-229) within
  // tol of q, skipping segment `self`; -1 if none.  extra: include the
  // entries appended during this pass.
  // current = false: the pre-pass state (the entries' geometry as rebuilt,
  // contiguous); true: the segments' current geometry (after anastomoses of
  // this pass) and the appended entries.
  int64_t search(int64_t self, V3 q, bool current, V3* proj) const {
    const bool extra = current;
    int64_t ix0, iy0, iz0;
    vox(q, ix0, iy0, iz0);
    for (int dx = -1; dx <= 1; ++dx)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dz = -1; dz <= 1; ++dz) {
          const int64_t v = vid(ix0 + dx, iy0 + dy, iz0 + dz);
          if (v < 0) continue;
          for (int64_t k = vstart[v]; k < vstart[v + 1]; ++k) {
            const int64_t s = ventry[k];
            if (s == self) continue;
            V3 a, b;
            if (current) {  // an anastomosed tip may have grown by up to tol
              a = S(s), b = Ee(s);
              const double mx = q.x - 0.5 * (a.x + b.x), my = q.y - 0.5 * (a.y + b.y), mz = q.z - 0.5 * (a.z + b.z);
              if (mx * mx + my * my + mz * mz > reject2_cur) continue;
            } else {
              const Geo& g = vgeo[k];
              a = {g.sx, g.sy, g.sz}, b = {g.ex, g.ey, g.ez};
              const double mx = q.x - 0.5 * (a.x + b.x), my = q.y - 0.5 * (a.y + b.y), mz = q.z - 0.5 * (a.z + b.z);
              if (mx * mx + my * my + mz * mz > reject2) continue;
            }
            if (pseg_dist(q, a, b, proj) <= p.anastomosis_tol) return s;
          }
          if (extra) {
            const auto it = vextra.find(v);
            if (it != vextra.end())
              for (int64_t s : it->second) {
                if (s == self) continue;
                if (pseg_dist(q, S(s), Ee(s), proj) <= p.anastomosis_tol) return s;
              }
          }
        }
    return -1;
  }
  bool near_dirty(V3 q) const {
    int64_t ix0, iy0, iz0;
    vox(q, ix0, iy0, iz0);
    for (int dx = -1; dx <= 1; ++dx)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dz = -1; dz <= 1; ++dz) {
          const int64_t v = vid(ix0 + dx, iy0 + dy, iz0 + dz);
          if (v >= 0 && vdirty[v]) return true;
        }
    return false;
  }

  // :388-414
  void anastomose() {
    const int64_t H = (int64_t)first.size();
    std::vector<int64_t> hit(H, -1);
    std::vector<V3> hp(H);
    parallel_for(H, threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t h = lo; h < hi; ++h) {
        const int64_t t = last[h];
        if (st[t] == 'A') hit[h] = search(t, Ee(t), false, &hp[h]);
      }
    });
    bool any = false;  // any anastomosis so far in this pass
    for (int64_t h = 0; h < H; ++h) {
      const int64_t t = last[h];
      if (st[t] != 'A') continue;
      const V3 q = Ee(t);
      int64_t s = hit[h];
      V3 proj = hp[h];
      if (any && near_dirty(q)) s = search(t, q, true, &proj);
      if (s < 0) continue;
      // the tip's hash entry (old midpoint) now holds new geometry; the
      // re-inserted entry (:411) sits at the new midpoint
      const int64_t v_old = vid_of(mid(t));
      ex[t] = proj.x, ey[t] = proj.y, ez[t] = proj.z;
      st[t] = 'S';
      if (v_old >= 0) vdirty[v_old] = 1;
      int64_t v_new = vid_of(mid(t));
      if (v_new < 0) v_new = grow_grid_for(mid(t));
      vextra[v_new].push_back(t);
      vdirty[v_new] = 1;
      any = true;
    }
  }
  int64_t vid_of(V3 q) const {
    int64_t ix, iy, iz;
    vox(q, ix, iy, iz);
    return vid(ix, iy, iz);
  }
  // a re-inserted midpoint outside the grid: rebuild the grid with a larger
  // box (keeps every list's order); rare (a tip snapping outside the box)
  int64_t grow_grid_for(V3 q) {
    int64_t ix, iy, iz;
    vox(q, ix, iy, iz);
    const int64_t nx0 = std::min(gx0, ix), ny0 = std::min(gy0, iy), nz0 = std::min(gz0, iz);
    const int64_t nnx = std::max(gx0 + gnx - 1, ix) - nx0 + 1, nny = std::max(gy0 + gny - 1, iy) - ny0 + 1,
                  nnz = std::max(gz0 + gnz - 1, iz) - nz0 + 1;
    const int64_t NV = nnx * nny * nnz;
    auto nid = [&](int64_t a, int64_t b, int64_t c) { return ((c - nz0) * nny + (b - ny0)) * nnx + (a - nx0); };
    const int64_t NO = gnx * gny * gnz;
    std::vector<int64_t> map(NO), inv(NV, -1);
    for (int64_t z = 0; z < gnz; ++z)
      for (int64_t y = 0; y < gny; ++y)
        for (int64_t x = 0; x < gnx; ++x) map[(z * gny + y) * gnx + x] = nid(x + gx0, y + gy0, z + gz0);
    for (int64_t o = 0; o < NO; ++o) inv[map[o]] = o;
    std::vector<int64_t> st2(NV + 1, 0), en2;
    std::vector<Geo> ge2;
    std::vector<uint8_t> d2(NV, 0);
    en2.reserve(ventry.size());
    ge2.reserve(vgeo.size());
    for (int64_t v = 0; v < NV; ++v) {
      st2[v] = (int64_t)en2.size();
      const int64_t o = inv[v];
      if (o < 0) continue;
      en2.insert(en2.end(), ventry.begin() + vstart[o], ventry.begin() + vstart[o + 1]);
      ge2.insert(ge2.end(), vgeo.begin() + vstart[o], vgeo.begin() + vstart[o + 1]);
      d2[v] = vdirty[o];
    }
    st2[NV] = (int64_t)en2.size();
    std::unordered_map<int64_t, std::vector<int64_t>> ex2;
    for (auto& kv : vextra) ex2[map[kv.first]] = std::move(kv.second);
    gx0 = nx0, gy0 = ny0, gz0 = nz0, gnx = nnx, gny = nny, gnz = nnz;
    vstart.swap(st2), ventry.swap(en2), vgeo.swap(ge2), vextra.swap(ex2), vdirty.swap(d2);
    return vid(ix, iy, iz);
  }

  // :267-292 — the E chain is serial in hypha-major order
  void uptake() {
    const int64_t n = (int64_t)ord.size();
    std::vector<uint8_t> in(n);
    for (auto& c : cub) {
      if (!c.substrate) continue;
      double E = c.E;
      if (E <= 0.0) continue;
      parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
        for (int64_t k = lo; k < hi; ++k) in[k] = c.contains(Ee(ord[k]));
      });
      const double dtmu = p.dt * c.mu;
      for (int64_t k = 0; k < n; ++k) {
        if (!in[k]) continue;
        double& Ii = I[ord[k]];
        double theta = dtmu * E * Ii;
        const double clamp = std::min(p.M_cap - Ii, E);
        if (theta < 0.0) theta = 0.0;
        if (theta > clamp) theta = clamp;
        Ii += theta;
        E -= theta;
        if (E <= 0.0) break;
      }
      c.E = E;
    }
  }

  // :294-343
  void walls() {
    const int64_t H = (int64_t)first.size();
    for (int64_t h = 0; h < H; ++h) {
      const int64_t t = last[h];
      for (int it = 0; it < 3; ++it) {
        bool pen = false;
        for (const auto& c : cub) {
          if (c.substrate) continue;
          if (!c.contains(Ee(t))) continue;
          pen = true;
          const V3 dl = sub(Ee(t), c.c), hf = mul(c.size, 0.5);
          const double ox = std::fabs(dl.x) - hf.x, oy = std::fabs(dl.y) - hf.y, oz = std::fabs(dl.z) - hf.z;
          int idx = 0;
          double om = ox;
          if (oy > om) om = oy, idx = 1;
          if (oz > om) om = oz, idx = 2;
          V3 nrm{0, 0, 0};
          if (idx == 0) nrm.x = dl.x >= 0 ? 1.0 : -1.0;
          if (idx == 1) nrm.y = dl.y >= 0 ? 1.0 : -1.0;
          if (idx == 2) nrm.z = dl.z >= 0 ? 1.0 : -1.0;
          V3 d = sub(Ee(t), S(t));
          if (norm3(d) < 1e-12) {
            // a zero-length tip (never seen in practice): the reference's
            // Vec3(uniformRange, uniformRange, uniformRange) — GCC evaluates
            // those arguments right to left
            const double rz = urange(-1, 1), ry = urange(-1, 1), rx = urange(-1, 1);
            d = {rx, ry, rz};
          }
          d = normalized(d);
          const double comp = dot3(d, nrm);
          V3 d2 = sub(d, mul(nrm, comp));
          if (norm3(d2) < 1e-12) {
            d2 = d;
            if (idx == 0) d2.x = 0.0;
            else if (idx == 1) d2.y = 0.0;
            else d2.z = 0.0;
          }
          d2 = normalized(d2);
          const V3 ne = add(S(t), mul(d2, len(t)));
          ex[t] = ne.x, ey[t] = ne.y, ez[t] = ne.z;
          th[t] = std::acos(std::max(-1.0, std::min(1.0, d2.z)));
          ph[t] = std::atan2(d2.y, d2.x);
          st[t] = 'A';
          break;
        }
        if (!pen) break;
      }
    }
  }
  static V3 normalized(V3 a) {  // Vec3::normalize (:43)
    const double n = norm3(a);
    if (n > 1e-15) a = {a.x / n, a.y / n, a.z / n};
    return a;
  }

  // :429-445 + the history line of :571
  void stats_line(int step, char* line, double* total) {
    const int64_t segs = (int64_t)ord.size();
    std::vector<std::array<int64_t, 3>> cnt3(std::max(1, threads), {0, 0, 0});
    parallel_for(segs, threads, [&](int64_t lo, int64_t hi, int t) {
      auto& c3 = cnt3[t];
      for (int64_t k = lo; k < hi; ++k) {
        const char c = st[ord[k]];
        c3[0] += c == 'A', c3[1] += c == 'P', c3[2] += c == 'S';
      }
    });
    int64_t A = 0, P = 0, Sg = 0;
    for (auto& c3 : cnt3) A += c3[0], P += c3[1], Sg += c3[2];
    lenbuf.resize(segs);
    parallel_for(segs, threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t k = lo; k < hi; ++k) lenbuf[k] = len(ord[k]);
    });
    double L = 0;  // summed serially in the reference's order (:132-137)
    for (int64_t k = 0; k < segs; ++k) L += lenbuf[k];
    const int64_t hy = (int64_t)first.size();
    char* q = line;
    q = put_i64(q, step), *q++ = ',';
    q = put_i64(q, hy), *q++ = ',';
    q = put_i64(q, segs), *q++ = ',';
    q = put_i64(q, A), *q++ = ',';
    q = put_i64(q, P), *q++ = ',';
    q = put_i64(q, Sg), *q++ = ',';
    q = put_i64(q, std::max<int64_t>(0, hy - n_sites)), *q++ = ',';
    q = put_g6(q, L), *q++ = '\n';
    *q = 0;
    *total = L;
  }

  // :463-475 — chunks formatted in parallel, written in order
  bool write_snapshot(const std::string& path) {
    const int64_t n = (int64_t)ord.size();
    const int T = std::max(1, threads);
    std::vector<std::string> part(T);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int t) {
      std::string& o = part[t];
      o.resize((size_t)(hi - lo) * 80);
      char* q = o.data();
      for (int64_t k = lo; k < hi; ++k) {
        const int64_t s = ord[k];
        q = put_g6(q, sx[s]), *q++ = ',';
        q = put_g6(q, sy[s]), *q++ = ',';
        q = put_g6(q, ex[s]), *q++ = ',';
        q = put_g6(q, ey[s]), *q++ = ',';
        q = put_g6(q, I[s] * len(s)), *q++ = '\n';
      }
      o.resize(q - o.data());
    });
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fputs("x1,y1,x2,y2,intensity\n", f);
    for (auto& o : part) std::fwrite(o.data(), 1, o.size(), f);
    return std::fclose(f) == 0;
  }

  // :477-500 — node identity by the %.6f key, first appearance numbering
  void export_geometry() {
    const int64_t n = (int64_t)ord.size();
    std::vector<int64_t> k(6 * n);
    parallel_for(n, threads, [&](int64_t lo, int64_t hi, int) {
      for (int64_t j = lo; j < hi; ++j) {
        const int64_t s = ord[j];
        int64_t* o = &k[6 * j];
        o[0] = key6(sx[s]), o[1] = key6(sy[s]), o[2] = key6(sz[s]);
        o[3] = key6(ex[s]), o[4] = key6(ey[s]), o[5] = key6(ez[s]);
      }
    });
    // open-addressing table over the 3-int keys
    size_t cap = 16;
    while (cap < (size_t)(4 * n + 16)) cap <<= 1;
    std::vector<int64_t> slot(cap, -1);
    node_of.resize(2 * n);
    nxyz.clear();
    nxyz.reserve(3 * n);
    std::vector<int64_t> nkey;
    nkey.reserve(3 * n);
    auto hsh = [](const int64_t* q) {
      uint64_t h = 1469598103934665603ull;
      for (int i = 0; i < 3; ++i) h = (h ^ (uint64_t)q[i]) * 1099511628211ull, h ^= h >> 29;
      return h;
    };
    for (int64_t j = 0; j < 2 * n; ++j) {
      const int64_t* q = &k[3 * j];
      size_t b = hsh(q) & (cap - 1);
      for (;;) {
        const int64_t id = slot[b];
        if (id < 0) {
          const int64_t s = ord[j / 2];
          const bool end = j & 1;
          slot[b] = (int64_t)(nkey.size() / 3);
          nkey.insert(nkey.end(), q, q + 3);
          nxyz.push_back(end ? ex[s] : sx[s]);
          nxyz.push_back(end ? ey[s] : sy[s]);
          nxyz.push_back(end ? ez[s] : sz[s]);
          node_of[j] = slot[b];
          break;
        }
        if (nkey[3 * id] == q[0] && nkey[3 * id + 1] == q[1] && nkey[3 * id + 2] == q[2]) {
          node_of[j] = id;
          break;
        }
        b = (b + 1) & (cap - 1);
      }
    }
    n_nodes = (int64_t)nxyz.size() / 3;
    n_elems = n;
  }

  bool write_geometry(const std::string& dir) const {
    auto write_parallel = [&](const std::string& path, const char* head, int64_t n, size_t width, auto&& row) {
      const int T = std::max(1, threads);
      std::vector<std::string> part(T);
      parallel_for(n, threads, [&](int64_t lo, int64_t hi, int t) {
        std::string& o = part[t];
        o.resize((size_t)(hi - lo) * width);
        char* q = o.data();
        for (int64_t i = lo; i < hi; ++i) q = row(q, i);
        o.resize(q - o.data());
      });
      FILE* f = std::fopen(path.c_str(), "wb");
      if (!f) return false;
      std::fputs(head, f);
      for (auto& o : part) std::fwrite(o.data(), 1, o.size(), f);
      return std::fclose(f) == 0;
    };
    const bool a = write_parallel(dir + "/nodes.csv", "node_id,x,y,z\n", n_nodes, 96, [&](char* q, int64_t i) {
      q = put_i64(q, i), *q++ = ',';
      q = put_g6(q, nxyz[3 * i]), *q++ = ',';
      q = put_g6(q, nxyz[3 * i + 1]), *q++ = ',';
      q = put_g6(q, nxyz[3 * i + 2]), *q++ = '\n';
      return q;
    });
    const bool b = write_parallel(dir + "/elements.csv", "elem_id,n1,n2\n", n_elems, 64, [&](char* q, int64_t e) {
      q = put_i64(q, e), *q++ = ',';
      q = put_i64(q, node_of[2 * e]), *q++ = ',';
      q = put_i64(q, node_of[2 * e + 1]), *q++ = '\n';
      return q;
    });
    return a && b;
  }
};

}  // namespace mfea

using mfea::GrowNet;

extern "C" {

struct mfea_grow_net : GrowNet {};

void mfea_grow_default_params(mfea_grow_params* p) {
  // src/mycelium_sim_2D.cpp:17-33, 159, 546
  *p = mfea_grow_params{};
  p->seed = 42;
  p->h0 = 0.05;
  p->dt = 0.01;
  p->lambda_angle = mfea::kPi / 6.0;
  p->P_branch = 0.5;
  p->c_g = 1e-7;
  p->D = 3.456;
  p->M_cap = 2e-6;
  p->omega0 = 5e-6;
  p->t_steps = 150;
  p->anastomosis_tol = 1e-3;
  p->wall_thickness = 0.05;
  p->dish_size = 5.0;
  p->h0_per_point = 10;
  p->substrate_width = 5.0;
  p->substrate_E = 2e-6;
  p->inoc_nx = 5;
  p->inoc_ny = 5;
  p->inoc_dist = 0.5;
  p->voxel_size = 0.1;
  p->snapshot_every = 0;
  p->snapshot_dir = nullptr;
  p->verbose = 0;
  p->threads = 0;
}

int mfea_grow(const mfea_grow_params* p, mfea_grow_net** out) {
  if (!p || !out) return MFEA_EINVAL;
  *out = nullptr;
  if (p->inoc_nx < 0 || p->inoc_ny < 0 || p->h0_per_point < 0 || p->t_steps < 0 || !(p->voxel_size > 0))
    return MFEA_EINVAL;
  auto* g = new (std::nothrow) mfea_grow_net();
  if (!g) return MFEA_ENOMEM;
  g->p = *p;
  g->vs = p->voxel_size;
  g->threads = p->threads > 0 ? p->threads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (p->verbose) std::fprintf(stderr, "Seed: %llu\n", (unsigned long long)p->seed);
  g->init();
  g->history = "step,hyphae,segments,active_tips,passive_tips,anastomosed,branches,total_length_mm\n";
  char line[256];
  double tph[8] = {0};
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto lap = [&](int k, std::chrono::steady_clock::time_point& t0) {
    const auto t1 = now();
    tph[k] += std::chrono::duration<double>(t1 - t0).count();
    t0 = t1;
  };
  for (int t = 0; t < p->t_steps; ++t) {  // :561-581
    auto t0 = now();
    g->translocate();
    lap(0, t0);
    g->grow();
    lap(1, t0);
    g->build_order();
    g->rebuild_hash();
    lap(2, t0);
    g->anastomose();
    lap(3, t0);
    g->uptake();
    lap(4, t0);
    g->walls();
    lap(5, t0);
    double L = 0;
    g->stats_line(t, line, &L);
    lap(6, t0);
    g->history += line;
    if (p->snapshot_every > 0 && p->snapshot_dir && (t % p->snapshot_every == 0 || t == p->t_steps - 1)) {
      char fn[64];
      std::snprintf(fn, sizeof(fn), "/step_%04d.csv", t);
      if (!g->write_snapshot(std::string(p->snapshot_dir) + fn)) {
        delete g;
        return MFEA_EINVAL;
      }
    }
    if (p->verbose) {
      char lb[32];
      *mfea::put_g6(lb, L) = 0;
      std::fprintf(stderr, "Step %d: hyphae=%lld segments=%lld total_length=%s\n", t,
                   (long long)g->first.size(), (long long)g->ord.size(), lb);
    }
  }
  g->build_order();
  g->export_geometry();
  if (p->verbose > 1)
    std::fprintf(stderr,
                 "phase s: translocate %.2f grow %.2f order+hash %.2f anastomose %.2f uptake %.2f walls %.2f "
                 "stats %.2f\n",
                 tph[0], tph[1], tph[2], tph[3], tph[4], tph[5], tph[6]);
  *out = g;
  return MFEA_OK;
}

int mfea_grow_info(const mfea_grow_net* g, int64_t* n_nodes, int64_t* n_elems, int64_t* n_hyphae) {
  if (!g) return MFEA_EINVAL;
  if (n_nodes) *n_nodes = g->n_nodes;
  if (n_elems) *n_elems = g->n_elems;
  if (n_hyphae) *n_hyphae = (int64_t)g->first.size();
  return MFEA_OK;
}

int mfea_grow_mesh(const mfea_grow_net* g, double* xyz, int32_t* e2n) {
  if (!g) return MFEA_EINVAL;
  if (xyz) {
    // the coordinates nodes.csv carries (6 significant digits), read back
    mfea::parallel_for(g->n_nodes * 3, g->threads, [&](int64_t lo, int64_t hi, int) {
      char b[40];
      for (int64_t i = lo; i < hi; ++i) {
        char* e = mfea::put_g6(b, g->nxyz[i]);
        std::from_chars(b, e, xyz[i]);
      }
    });
  }
  if (e2n)
    for (int64_t i = 0; i < 2 * g->n_elems; ++i) e2n[i] = (int32_t)g->node_of[i];
  return MFEA_OK;
}

int mfea_grow_write(const mfea_grow_net* g, const char* dir) {
  if (!g || !dir) return MFEA_EINVAL;
  const std::string d(dir);
  if (!g->write_geometry(d)) return MFEA_EINVAL;
  FILE* f = std::fopen((d + "/mycelium_growth_stats.csv").c_str(), "wb");
  if (!f) return MFEA_EINVAL;
  std::fwrite(g->history.data(), 1, g->history.size(), f);
  return std::fclose(f) == 0 ? MFEA_OK : MFEA_EINVAL;
}

void mfea_grow_free(mfea_grow_net* g) { delete g; }

}  // extern "C"
