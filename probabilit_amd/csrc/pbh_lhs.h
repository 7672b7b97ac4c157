// Native-LHS helpers used by the Iman-Conover orchestrator (pbh_api.hip).
#pragma once

#include "pbh_common.h"

namespace pbh {

// out[t] = ppf of the LHS point in stratum t of column `col` (scalar parameters only).
int lhs_sorted_ppf(uint64_t seed, int64_t n, int col, int dist, const pbh_param* params, int nparams, double* out,
                   int32_t* flag, hipStream_t s);
// counts[0] = #ties x[t] == x[t+1], counts[1] = #inversions x[t] > x[t+1] (device counters).
int check_sorted(const double* x, int64_t n, unsigned long long* counts, hipStream_t s);
// S[r] = ndtri(rank(r) / (n + 1)), rank(r) = pi(r) + 1, or avg[pi(r)] when avg != NULL.
int perm_scores(uint64_t seed, int64_t n, int col, const double* avg, double* S, hipStream_t s);

}  // namespace pbh
