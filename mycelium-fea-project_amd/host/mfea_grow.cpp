// mfea_grow — command-line drop-in for the reference's growth simulator
// binary (src/mycelium_sim_2D.cpp main, :529-588) over libmfea's native
// producer (mfea_grow_*, csrc/grow.cpp).
//
//   mfea_grow [seed] [--out DIR] [--scale S] [--inoculum NX NY] [--steps T]
//             [--snapshots K] [--threads N] [--quiet]
//
// Without options it behaves as the reference binary: seed 42 (or argv[1]),
// results in ../results/sim_<YYYYmmdd_HHMMSS>/ with snapshots/step_NNNN.csv
// every step, mycelium_growth_stats.csv, nodes.csv, elements.csv, and the
// same stderr progress lines.  --scale S grows an S×-larger dish (inoculum
// grid 5S×5S at the same spacing, substrate and Ω₀ scaled by the area) — the
// large-network mode; --snapshots 0 skips the per-step
// snapshots (at 10 M DOF they would be terabytes).
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <sys/stat.h>

#include "mfea.h"

static int mkdirs(const std::string& path) {
  for (size_t i = 1; i <= path.size(); ++i)
    if (i == path.size() || path[i] == '/') {
      const std::string sub = path.substr(0, i);
      if (mkdir(sub.c_str(), 0755) != 0 && errno != EEXIST) return -1;
    }
  return 0;
}

int main(int argc, char** argv) {
  mfea_grow_params p;
  mfea_grow_default_params(&p);
  p.verbose = 1;
  p.snapshot_every = 1;
  std::string out;
  double scale = 1.0;
  int nx = -1, ny = -1;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto need = [&](int k) {
      if (i + k >= argc) {
        std::fprintf(stderr, "mfea_grow: %s needs %d value(s)\n", a.c_str(), k);
        std::exit(2);
      }
    };
    if (a == "--out") need(1), out = argv[++i];
    else if (a == "--scale") need(1), scale = std::atof(argv[++i]);
    else if (a == "--inoculum") need(2), nx = std::atoi(argv[i + 1]), ny = std::atoi(argv[i + 2]), i += 2;
    else if (a == "--steps") need(1), p.t_steps = std::atoi(argv[++i]);
    else if (a == "--snapshots") need(1), p.snapshot_every = std::atoi(argv[++i]);
    else if (a == "--threads") need(1), p.threads = std::atoi(argv[++i]);
    else if (a == "--quiet") p.verbose = 0;
    else if (a == "--timing") p.verbose = 2;
    else if (a[0] != '-') p.seed = (unsigned)std::atoi(a.c_str());  // :531 (unsigned)atoi
    else {
      std::fprintf(stderr, "mfea_grow: unknown option %s\n", a.c_str());
      return 2;
    }
  }
  if (scale != 1.0) {
    p.dish_size *= scale;
    p.substrate_width *= scale;
    p.substrate_E *= scale * scale;
    p.omega0 *= scale * scale;
    p.inoc_nx = p.inoc_ny = (int)(5 * scale + 0.5);
  }
  if (nx > 0) p.inoc_nx = nx, p.inoc_ny = ny;
  if (out.empty()) {  // :536-540
    char ts[64];
    const std::time_t tt = std::chrono::system_clock::to_time_t(std::chrono::system_clock::now());
    std::tm tmv;
    localtime_r(&tt, &tmv);
    std::strftime(ts, sizeof(ts), "%Y%m%d_%H%M%S", &tmv);
    out = std::string("../results/sim_") + ts;
  }
  const std::string snap = out + "/snapshots";
  if (mkdirs(p.snapshot_every > 0 ? snap : out) != 0) {
    std::fprintf(stderr, "⚠️ Failed to create directory: %s\n", snap.c_str());
    return 1;
  }
  p.snapshot_dir = snap.c_str();
  mfea_grow_net* g = nullptr;
  int rc = mfea_grow(&p, &g);
  if (rc == MFEA_OK) rc = mfea_grow_write(g, out.c_str());
  if (rc != MFEA_OK) {
    std::fprintf(stderr, "mfea_grow: failed (%d)\n", rc);
    mfea_grow_free(g);
    return 1;
  }
  if (p.verbose) {
    std::fprintf(stderr, "✅ Exported geometry to %s\n", out.c_str());
    std::fprintf(stderr, "✅ All results saved under %s\n", out.c_str());
  }
  mfea_grow_free(g);
  return 0;
}
