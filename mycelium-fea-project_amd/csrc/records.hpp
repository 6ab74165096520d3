// records.hpp — CSV record writer of the driver (records.cpp; host only).
#pragma once
#include <cstdint>
#include <string>

namespace mfea {

// Python repr / "%.12g" of one double into out (≥ 32 bytes); returns length.
int format_repr(double v, char* out);
int format_g12(double v, char* out);

// One record file (mfea_write_record_csv in mfea.h).  Returns "" or an error.
std::string write_record_csv(const char* path, int style, int kind, int64_t n_rows,
                             int64_t n_cols, const double* values, const uint8_t* flags,
                             int n_threads);

// The same record as a NumPy .npy sidecar (mfea_write_record_npy in mfea.h).
std::string write_record_npy(const char* path, int kind, int64_t n_rows, int64_t n_cols, const double* values,
                             const uint8_t* flags);

}  // namespace mfea
