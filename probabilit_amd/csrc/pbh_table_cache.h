// Process-wide cache of inverse-CDF setup tables (pbh_table_cache.hip).
#pragma once

#include <stddef.h>

#include <functional>

#include "pbh_common.h"

namespace pbh {

enum TableKind : int {
  kTabGammaGuide = 1,  // gammainc guide of shape a (gamma, chi, chi2, maxwell, nakagami)
  kTabPoisson = 2,     // pdtr CDF + scipy windows + guide of mean mu
  kTabBetaGuide = 3,   // betainc guide of (a, b)
  kTabDiscrete = 4,    // binom / bernoulli / nbinom CDF + complement (key: dist id, parameters)
};

// The table of (kind, key[0 .. nkey)): built once per process and device by `build` on stream s
// into a persistent allocation of `bytes`, then reused by every later call (s waits for the
// build's completion event).  nullptr when the cache is full or the build fails: the caller then
// builds a table of its own for this call.
double* cached_table(int kind, const double* key, int nkey, size_t bytes, hipStream_t s,
                     const std::function<bool(double*, hipStream_t)>& build);

// The end of a call's use of a table: hipFreeAsync on s unless it belongs to the cache.
void release_table(double* t, hipStream_t s);

}  // namespace pbh
