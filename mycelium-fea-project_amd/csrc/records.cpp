// records.cpp — the driver's CSV record writer (host C++, no device work).
//
// At the end of a run the reference writes its per-step records in one go:
//   src/fea_solver.py:297-316 — pandas DataFrame.to_csv: float64 cells as the
//     shortest round-trip decimal (numpy astype(str): the digits and layout of
//     Python's repr), NaN as an empty field, bools as True/False, and
//     node_displacements.csv headed 0..3N-1 (disp_cols is built but unused);
//   src/fea_petsc.cpp:433-516 — std::ostream << std::setprecision(12)
//     ("%.12g"), actives as 1/0, the node_i_x..node_i_y..node_i_z header over
//     the interleaved DOF values.
// At 1 M DOF node_displacements.csv alone is 40 rows × 3 M cells, so the
// pandas path takes minutes; here each row is formatted in column chunks on
// worker threads and written in order ("record writer at scale").
#include "records.hpp"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "mfea.h"

namespace mfea {

// Python repr of a double (PyOS_double_to_string 'r'): shortest round-trip
// digits; exponent form when the decimal point position is <= -4 or > 16
// (repr(1e-05) = '1e-05', repr(1e16) = '1e+16'), else positional with at
// least one digit after the point ('2.0', '0.0001').  NaN → "" (pandas na_rep).
int format_repr(double v, char* out) {
  char* o = out;
  if (std::isnan(v)) return 0;
  if (std::signbit(v)) *o++ = '-';
  const double a = std::fabs(v);
  if (std::isinf(a)) {
    std::memcpy(o, "inf", 3);
    return (int)(o + 3 - out);
  }
  if (a == 0.0) {
    std::memcpy(o, "0.0", 3);
    return (int)(o + 3 - out);
  }
  char sci[40];
  const auto res = std::to_chars(sci, sci + sizeof(sci) - 1, a, std::chars_format::scientific);
  *res.ptr = '\0';  // to_chars does not terminate; atoi below reads the exponent
  char dig[24] = {};  // shortest digits of d[.ddd]e±XX
  int nd = 0;
  const char* p = sci;
  for (; p < res.ptr && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  const int e10 = std::atoi(p + 1);  // a = d.ddd × 10^e10
  const int decpt = e10 + 1;         // digits before the decimal point
  if (decpt <= -4 || decpt > 16) {
    *o++ = dig[0];
    if (nd > 1) {
      *o++ = '.';
      std::memcpy(o, dig + 1, nd - 1);
      o += nd - 1;
    }
    *o++ = 'e';
    *o++ = e10 < 0 ? '-' : '+';
    const int ae = std::abs(e10);
    if (ae >= 100) *o++ = (char)('0' + ae / 100);
    *o++ = (char)('0' + (ae / 10) % 10);
    *o++ = (char)('0' + ae % 10);
  } else if (decpt <= 0) {
    *o++ = '0';
    *o++ = '.';
    for (int k = 0; k < -decpt; ++k) *o++ = '0';
    std::memcpy(o, dig, nd);
    o += nd;
  } else if (decpt < nd) {
    std::memcpy(o, dig, decpt);
    o += decpt;
    *o++ = '.';
    std::memcpy(o, dig + decpt, nd - decpt);
    o += nd - decpt;
  } else {
    std::memcpy(o, dig, nd);
    o += nd;
    for (int k = nd; k < decpt; ++k) *o++ = '0';
    *o++ = '.';
    *o++ = '0';
  }
  return (int)(o - out);
}

// std::ostream << std::setprecision(12) << v (libstdc++ formats it with "%.*g")
int format_g12(double v, char* out) { return std::snprintf(out, 32, "%.12g", v); }

namespace {

constexpr int kCell = 32;  // upper bound of one formatted cell plus its comma

std::string header(int style, int kind, int64_t n_cols) {
  if (kind == MFEA_REC_FORCE) return "total_displacement,total_force\n";
  std::string h;
  h.reserve((size_t)n_cols * 12 + 8);
  if (kind == MFEA_REC_DISP && style == MFEA_CSV_PETSC) {
    const int64_t n = n_cols / 3;  // src/fea_petsc.cpp:481-491
    for (int c = 0; c < 3; ++c)
      for (int64_t i = 0; i < n; ++i) {
        if (c || i) h += ',';
        h += "node_" + std::to_string(i) + "_" + (char)('x' + c);
      }
  } else {
    for (int64_t i = 0; i < n_cols; ++i) {
      if (i) h += ',';
      if (kind == MFEA_REC_DISP) h += std::to_string(i);
      else h += "elem_" + std::to_string(i);
    }
  }
  h += n_cols ? ",step\n" : "step\n";
  return h;
}

// cells [c0, c1) of one row, each followed by ','
size_t format_cells(int style, int kind, const double* vals, const uint8_t* flags, int64_t c0,
                    int64_t c1, char* buf) {
  char* o = buf;
  for (int64_t c = c0; c < c1; ++c) {
    if (kind == MFEA_REC_ACTIVE) {
      const bool t = flags[c] != 0;
      if (style == MFEA_CSV_PETSC) {
        *o++ = t ? '1' : '0';
      } else {
        std::memcpy(o, t ? "True" : "False", t ? 4 : 5);
        o += t ? 4 : 5;
      }
    } else {
      o += style == MFEA_CSV_PETSC ? format_g12(vals[c], o) : format_repr(vals[c], o);
    }
    *o++ = ',';
  }
  return (size_t)(o - buf);
}

}  // namespace

std::string write_record_csv(const char* path, int style, int kind, int64_t n_rows,
                             int64_t n_cols, const double* values, const uint8_t* flags,
                             int n_threads) {
  if (!path) return "NULL path";
  if (style != MFEA_CSV_PANDAS && style != MFEA_CSV_PETSC) return "unknown CSV style";
  if (kind < MFEA_REC_STRESS || kind > MFEA_REC_FORCE) return "unknown record kind";
  if (n_rows < 0 || n_cols < 0) return "negative record size";
  if (kind == MFEA_REC_FORCE && n_cols != 2) return "force records have 2 columns";
  if (kind == MFEA_REC_DISP && style == MFEA_CSV_PETSC && n_cols % 3)
    return "displacement records need 3 columns per node";
  if (n_rows > 0 && n_cols > 0 && (kind == MFEA_REC_ACTIVE ? !flags : !values))
    return "NULL record array";
  FILE* f = std::fopen(path, "wb");
  if (!f) return std::string("cannot open ") + path;
  const std::string h = header(style, kind, n_cols);
  bool ok = std::fwrite(h.data(), 1, h.size(), f) == h.size();
  const int T = std::max(1, std::min(n_threads, 64));
  const int64_t chunk = std::max<int64_t>(4096, (n_cols + T - 1) / T);
  const int64_t nchunks = (n_cols + chunk - 1) / chunk;
  std::vector<std::vector<char>> bufs((size_t)nchunks);
  std::vector<size_t> lens((size_t)nchunks, 0);
  for (auto& b : bufs) b.resize((size_t)chunk * kCell);
  for (int64_t r = 0; ok && r < n_rows; ++r) {
    const double* rv = values ? values + r * n_cols : nullptr;
    const uint8_t* rf = flags ? flags + r * n_cols : nullptr;
    auto run = [&](int64_t k) {
      const int64_t c0 = k * chunk, c1 = std::min(n_cols, c0 + chunk);
      lens[k] = format_cells(style, kind, rv, rf, c0, c1, bufs[k].data());
    };
    if (nchunks <= 1 || T == 1) {
      for (int64_t k = 0; k < nchunks; ++k) run(k);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < T && t < nchunks; ++t)
        th.emplace_back([&, t] {
          for (int64_t k = t; k < nchunks; k += T) run(k);
        });
      for (auto& x : th) x.join();
    }
    // force rows have no step column: the last cell's comma ends the line
    if (kind == MFEA_REC_FORCE && nchunks) bufs[nchunks - 1][lens[nchunks - 1] - 1] = '\n';
    for (int64_t k = 0; ok && k < nchunks; ++k)
      ok = std::fwrite(bufs[k].data(), 1, lens[k], f) == lens[k];
    if (ok && kind != MFEA_REC_FORCE) ok = std::fprintf(f, "%lld\n", (long long)(r + 1)) > 0;
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? "" : std::string("write failed: ") + path;
}

// NumPy .npy (format 1.0): magic, version, little-endian header length, the
// header dict padded with spaces to a 64-byte boundary and ended by '\n', then
// the C-order data — '<f8' for stress / displacement / force, '|b1' (one byte
// 0/1 per cell) for the activity.  np.load(allow_pickle=False) reads it.
std::string write_record_npy(const char* path, int kind, int64_t n_rows, int64_t n_cols, const double* values,
                             const uint8_t* flags) {
  if (!path) return "NULL path";
  if (kind < MFEA_REC_STRESS || kind > MFEA_REC_FORCE) return "unknown record kind";
  if (n_rows < 0 || n_cols < 0) return "negative record size";
  const bool b1 = kind == MFEA_REC_ACTIVE;
  if (n_rows > 0 && n_cols > 0 && (b1 ? !flags : !values)) return "NULL record array";
  char dict[160];
  const int dn = std::snprintf(dict, sizeof dict, "{'descr': '%s', 'fortran_order': False, 'shape': (%lld, %lld), }",
                               b1 ? "|b1" : "<f8", (long long)n_rows, (long long)n_cols);
  std::string h("\x93NUMPY\x01\x00", 8);
  const size_t total = (10 + (size_t)dn + 1 + 63) / 64 * 64;  // magic 6 + version 2 + length 2
  const size_t hl = total - 10;
  h.push_back((char)(hl & 0xff));
  h.push_back((char)(hl >> 8));
  h.append(dict, (size_t)dn);
  h.append(hl - (size_t)dn - 1, ' ');
  h.push_back('\n');
  FILE* f = std::fopen(path, "wb");
  if (!f) return std::string("cannot open ") + path;
  bool ok = std::fwrite(h.data(), 1, h.size(), f) == h.size();
  const size_t cells = (size_t)n_rows * (size_t)n_cols;
  if (ok && cells) {
    if (b1) {
      std::vector<uint8_t> row((size_t)n_cols);
      for (int64_t r = 0; ok && r < n_rows; ++r) {
        for (int64_t c = 0; c < n_cols; ++c) row[c] = flags[r * n_cols + c] ? 1 : 0;
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
      }
    } else {
      ok = std::fwrite(values, sizeof(double), cells, f) == cells;
    }
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? "" : std::string("write failed: ") + path;
}

}  // namespace mfea
