// Iman-Conover building blocks (correlation.py:368-425) shared by the C-ABI entry points.
#pragma once

#include "pbh_common.h"
#include "pbh_sort.h"

namespace pbh {

enum RankMode { kModeScores = 0, kModeGather = 1, kModeRanks = 2 };

struct RankOut {
  // kModeScores: S[row] = ndtri(avg / (n + 1)); sorted_x[i] = value at sorted position i
  double* scores;
  double* sorted_x;
  // kModeGather: Y[row * y_rs] = sorted_src[(int64)avg - 1]; idx[row] = (int64)avg - 1
  const double* sorted_src;
  double* y;
  int64_t y_rs;
  int32_t* idx;
  // kModeRanks: ranks[row] = avg
  double* ranks;
};

struct TieBuffers {
  int64_t* first_head;  // per sort tile
  int64_t* last_head;
  int64_t* prev_head;
  int64_t* next_head;
};

size_t tie_workspace_bytes(int64_t n);
void tie_carve(void* ws, int64_t n, TieBuffers& tb);

// Keys of column: keys[i] = f64_to_key(x[i * stride]); sets *flag on NaN / inf.
int load_keys(const double* x, int64_t stride, int64_t n, uint64_t* keys, int32_t* flag, hipStream_t s);

// Given keys sorted ascending with row payload, resolve 'average' tie ranks and emit per mode.
int rank_finish(int mode, const uint64_t* keys, const uint32_t* rows, int64_t n, const TieBuffers& tb,
                const RankOut& out, hipStream_t s);

// Column sums (k columns of length n, column stride ld) into sums[k] (device), fixed order.
int column_means(const double* S, int64_t n, int k, int64_t ld, double* partial, double* means, hipStream_t s);
size_t gram_partials_bytes(int k);
// Centered Gram matrix G = (S - m)^T (S - m), k x k row-major into gram (device), fixed order.
int centered_gram(const double* S, int64_t n, int k, int64_t ld, const double* means, double* partials,
                  double* gram, hipStream_t s);
// In place, per row r: d = forward-substitute(L, s_r) (d_j = (s_j - sum_{m<j} L_jm d_m) * inv_diag_j),
// then cs_j = sum_{m<=j} P_jm d_m.   L, P: k x k row-major device, inv_diag: k.
int apply_decorrelate_correlate(double* S, int64_t n, int k, int64_t ld, const double* L, const double* inv_diag,
                                const double* P, hipStream_t s);

}  // namespace pbh
