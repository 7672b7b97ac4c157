// Native-LHS helpers used by the Iman-Conover orchestrator (pbh_api.hip).
#pragma once

#include "pbh_common.h"

namespace pbh {

// out[t - t0] = ppf of the LHS point in stratum t of column `col`, t in [t0, t0 + nt)
// (scalar parameters only).
// counts != NULL: counts[0] = #ties x[t] == x[t+1], counts[1] = #inversions, inside the segment
// (zeroed first; device counters).
int lhs_sorted_ppf(uint64_t seed, int64_t n, int64_t t0, int64_t nt, int col, int dist, const pbh_param* params,
                   int nparams, double* out, int32_t* flag, hipStream_t s, unsigned long long* counts = nullptr);
// counts[0] = #ties x[t] == x[t+1], counts[1] = #inversions x[t] > x[t+1] (device counters).
int check_sorted(const double* x, int64_t n, unsigned long long* counts, hipStream_t s);
// S[r - row0] = ndtri(rank(r) / (n + 1)) for rows [row0, row0 + nrows): rank(r) = pi(r) + 1, or
// the 'average' rank of the run holding stratum pi(r) when heads != NULL (nheads sorted run
// heads of the whole sorted column, heads[0] == 0).
// partial != NULL: partial[b] = sum of the scores block b wrote (ppf_grid(nrows) blocks).
int perm_scores(uint64_t seed, int64_t n, int col, int64_t row0, int64_t nrows, const uint32_t* heads,
                int64_t nheads, double* S, hipStream_t s, double* partial = nullptr);
// number of partial sums perm_scores writes for nrows rows
unsigned perm_scores_blocks(int64_t nrows);
// perm_scores for a materialised column whose strata (rank - 1 of each row, a permutation of
// [0, n)) are known: S[r] = ndtri(rank / (n + 1)), rank = strata[r] + 1 or its run's average.
int strata_scores(const int32_t* strata, int64_t n, const uint32_t* heads, int64_t nheads, double* S, hipStream_t s);
// sorted[strata[r]] = x[r * stride], then the tie / inversion counts of sorted (counts: 2 device
// u64, as check_sorted).  counts[1] == 0 certifies that sorted is sort(x) and strata its ranks
// (a stratum no row names stays NaN and counts as an inversion).
int strata_sorted(const double* x, int64_t stride, const int32_t* strata, int64_t n, double* sorted,
                  unsigned long long* counts, hipStream_t s);
// Run heads of a sorted segment x[0..m) (see k_heads_write); *count = number written (syncs).
size_t run_heads_ws_bytes(int64_t m);
int run_heads(const double* x, int64_t m, int64_t t0, bool first_is_prev, uint32_t* heads, int64_t* count,
              void* ws, hipStream_t s);

}  // namespace pbh
