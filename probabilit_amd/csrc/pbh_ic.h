// Iman-Conover building blocks (correlation.py:368-425) shared by the C-ABI entry points.
#pragma once

#include "pbh_common.h"
#include "pbh_sort.h"

namespace pbh {

// kModeScoresRank: kModeScores with the scores written in rank order, scores[i] for sorted position
// i (contiguous), for the row placement to put in row order (ic_run's step 1 at large n)
enum RankMode { kModeScores = 0, kModeGather = 1, kModeRanks = 2, kModeScoresRank = 3 };

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
// With eqprev != NULL, ties come from eqprev[i] (element i equals element i - 1) and keys may
// be NULL (gather / ranks modes only).
int rank_finish(int mode, const uint64_t* keys, const uint32_t* rows, int64_t n, const TieBuffers& tb,
                const RankOut& out, hipStream_t s, const uint8_t* eqprev = nullptr);

// 32-bit order-preserving codes of approximately N(0, 1) data: a piecewise-linear map through
// Phi on m uniform segments of [x0, x0 + m w].  code(x) is non-decreasing in x for every
// double (segment index and in-segment offset are both monotone), so sorting by code and
// then ordering equal-code runs by the full value yields the exact float64 order.
struct CodeMap {
  double x0, w, inv_w;
  int m;
  const uint32_t* base;  // m + 1 strictly increasing code bases
  const double* scale;   // m slopes (codes per unit x)
};
constexpr int kCodeSegments = 1024;  // 12 KB: small enough to sit in the LDS of the step-3 kernel
__device__ __forceinline__ uint32_t code_of(double x, const CodeMap& c) {
  double u = (x - c.x0) * c.inv_w;
  if (!(u >= 0.0)) return 0u;
  if (u >= (double)c.m) return 0xFFFFFFFFu;
  int j = (int)u;
  double lo = c.x0 + (double)j * c.w;
  uint32_t b0 = c.base[j], cnt = c.base[j + 1] - b0;
  double off = floor((x - lo) * c.scale[j]);
  uint32_t o = off <= 0.0 ? 0u : (off >= (double)(cnt - 1) ? cnt - 1 : (uint32_t)off);
  return b0 + o;
}
size_t code_map_bytes();
// Host: fill base / scale for N(0, 1)-shaped data into the host buffers.
void code_map_host(uint32_t* base, double* scale, double* x0, double* w);
int make_codes(const double* x, int64_t n, const CodeMap& cm, uint32_t* codes, hipStream_t s);
// Reorders `rows` in place so that every run of equal codes (length <= 16) is ordered by the
// full value x[row]; eqprev[i] = element i equals element i - 1.  flags[0] |= 1 when a run is
// longer (the caller falls back to 64-bit keys), |= 2 when any exact tie exists.
// starts: scratch for n / 2 + 2048 run starts; counts: 2048 per-block counters.
int resolve_code_runs(const uint32_t* codes, uint32_t* rows, const double* x, int64_t n, uint8_t* eqprev,
                      int32_t* flags, uint32_t* starts, uint32_t* counts, hipStream_t s);

// dst = src, then dst[p] = src[s + (e - s) / 2] inside every tie run [s, e] flagged by eqprev:
// the value every member of a tie run receives in step 4 (int of the 'average' rank).
// out (k x n, column-major) = X (n rows of k values, row stride x_rs >= k), and back: Y[r * y_rs + c] =
// in[c * n + r] (tiled through LDS; the operator API's row-major X / Y, k <= 128)
int rows_to_columns(const double* X, int64_t x_rs, int64_t n, int k, double* out, hipStream_t s);
int columns_to_rows(const double* in, int64_t n, int k, double* Y, int64_t y_rs, hipStream_t s);
int tie_fix_values(const uint8_t* eqprev, int64_t n, const double* src, double* dst, hipStream_t s);

// out[c] = (sum of column c) / divisor, k columns of length n (column stride ld), fixed order.
int column_sums(const double* S, int64_t n, int k, int64_t ld, double* partial, double* out, double divisor,
                hipStream_t s);
// Column means (k columns of length n, column stride ld) into means[k] (device), fixed order.
// means[c] = (sum_b partial[c * nb + b]) / divisor, in block order (k_means).
int means_from_partials(const double* partial, int nb, int k, double divisor, double* means, hipStream_t s);
int column_means(const double* S, int64_t n, int k, int64_t ld, double* partial, double* means, hipStream_t s);
size_t gram_partials_bytes(int k);
// Centered Gram matrix G = (S - m)^T (S - m), k x k row-major into gram (device), fixed order.
int centered_gram(const double* S, int64_t n, int k, int64_t ld, const double* means, double* partials,
                  double* gram, hipStream_t s);
// In place, per row r: d = forward-substitute(L, s_r) (d_j = (s_j - sum_{m<j} L_jm d_m) * inv_diag_j),
// then cs_j = sum_{m<=j} P_jm d_m.   L, P: k x k row-major device, inv_diag: k.
// With codes != NULL (and cm), also codes[c * ldc + r] = code_of(CS[r][c]) (step 4's keys).
int apply_decorrelate_correlate(double* S, int64_t n, int k, int64_t ld, const double* L, const double* inv_diag,
                                const double* P, hipStream_t s, uint32_t* codes = nullptr, int64_t ldc = 0,
                                const CodeMap* cm = nullptr);

// ---------------------------------------------------------------- shared orchestration pieces
// Host, step 2 (correlation.py:398-405): G = centered Gram (k x k, row-major) of scores over n
// rows is scaled in place to np.corrcoef (np.cov's 1/(n-1), the two divisions by the standard
// deviations, the clip to [-1, 1]); corr_out (optional) receives it; Lc = cholesky.  Returns
// PBH_ERR_NOT_PD with the reference's message when a pivot is not positive.
int ic_factor(double* G, int64_t n, int k, double* corr_out, double* Lc);

// Step 4 (correlation.py:418-423) for one column, with its workspace.
struct ReorderWs {
  SortBuffers sb;
  TieBuffers tb;
  CodeMap cm;
  uint8_t* eqprev;
  int32_t* flags;
  uint32_t hist_host[8 * 256];
};
size_t reorder_ws_bytes(int64_t n);
// Carves ws and uploads the code map (stream ordered).
int reorder_carve(void* ws, int64_t n, ReorderWs& w, hipStream_t s);
// y[r * y_rs] = sorted_src[rank(cs[r]) - 1]; idx[r] = rank - 1 when idx != NULL.
// codes (optional): code_of(cs) already computed (by the step-3 kernel); not modified.
// code_hist (optional): the codes' byte histograms on the device with the host's decision
// `code_flat` (code_hist_flat), so that the bucket path needs no sync of its own.
// err (optional, device): the placement's look-back failure is OR-ed into *err instead of being
// read back (no host synchronisation after the placement: columns pipelined over streams).
int reorder_column(const double* cs, int64_t n, const double* sorted_src, double* y, int64_t y_rs, int32_t* idx,
                   ReorderWs& w, hipStream_t s, const uint32_t* codes = nullptr, const uint32_t* code_hist = nullptr,
                   int code_flat = 1, int32_t* err = nullptr);

}  // namespace pbh
