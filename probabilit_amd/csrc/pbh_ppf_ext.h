// Inverse-CDF sweep of the distributions beyond the base set (pbh_ppf_ext.hip); pbh_ppf and
// pbh_lhs_ppf route distribution ids >= PBH_DIST_BETA here.
#pragma once

#include "pbh_common.h"

namespace pbh {

int ppf_ext(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params, int nparams, double* out,
            int32_t* flag, hipStream_t s);
int lhs_ppf_ext(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist, const pbh_param* params,
                int nparams, double* out, int32_t* flag, hipStream_t s);

// Generated columns of these distributions (the Iman-Conover fast path; scalar parameters `val`,
// ext_nparams(dist) of them).  ext_nparams is -1 for an id outside this set.
int ext_nparams(int dist);
bool ext_is_discrete(int dist);  // binom, bernoulli: sorted columns with runs of equal values
// the column in stratum order over [t0, t0 + nt): values (out, optional), tie / inversion counts
// (counts[2], device, optional), run heads appended at heads[*hcur] (< hcap written)
int ext_gen_sorted(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                   int64_t t0, int64_t nt, double* out, int32_t* flag, unsigned long long* counts, uint32_t* heads,
                   uint32_t* hcur, uint32_t hcap, hipStream_t s);
// step 4's placement: y[row * y_rs] = value(p) for the (row << 32 | p) pairs, or (pidx != NULL)
// y[i * y_rs] = value(pidx[i]) for i < rows
int ext_gen_place(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                  const uint64_t* pairs, const uint32_t* pidx, int64_t rows, double* y, int64_t y_rs, int32_t* idx,
                  const int32_t* state, hipStream_t s);
// a column's setup table (stream-ordered allocation, freed with hipFreeAsync; NULL when none):
// beta with scalar (a, b) -> its guide (sfx::BetaGuide)
double* ext_gen_table(int dist, const double* val, int np, hipStream_t s);
// pbh_ppf.hip: the gamma guide of shape a (4 x sf::kGammaGuideM doubles), stream-ordered allocation
double* gamma_guide_table(double a, hipStream_t s);
// the certificate's exact evaluation of the listed pairs (see k_cert_scan / k_cert_eval, pbh_ppf.hip)
int ext_gen_cert_eval(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                      int64_t t0, int64_t nt, const uint32_t* list, uint32_t cap, const uint32_t* count, int32_t* flag,
                      unsigned long long* counts, hipStream_t s);

}  // namespace pbh
