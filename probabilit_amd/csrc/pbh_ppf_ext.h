// Inverse-CDF sweep of the distributions beyond the base set (pbh_ppf_ext.hip); pbh_ppf and
// pbh_lhs_ppf route distribution ids >= PBH_DIST_BETA here.
#pragma once

#include "pbh_common.h"

namespace pbh {

int ppf_ext(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params, int nparams, double* out,
            int32_t* flag, hipStream_t s);
int lhs_ppf_ext(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist, const pbh_param* params,
                int nparams, double* out, int32_t* flag, hipStream_t s);

}  // namespace pbh
