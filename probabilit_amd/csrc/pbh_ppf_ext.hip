// Inverse CDF of the distributions that distributions.py builds beyond the base set
// (SURVEY.md §8f #3): beta (PERT), truncnorm (TruncatedNormal), binom and bernoulli.
//
//   beta       scipy beta._ppf = Boost ibeta_inv(a, b, q)   -> safeguarded Halley iteration on
//              the Cephes incomplete beta (incbet: power series / two continued fractions)
//   truncnorm  scipy truncnorm._ppf (scipy:stats/_continuous_distns.py): log-space mass and
//              ndtri_exp, left / right cases on the sign of a, _log_gauss_mass's three cases
//   binom      scipy _binom_ppf (Boost quantile, integer_round_up): smallest k in [0, n] with
//              bdtr(k, n, p) >= q, bdtr = Cephes incbet(n - k, k + 1, 1 - p)
//   bernoulli  binom with n = 1
// Parity is to floating-point tolerance (1e-10 relative; discrete outputs exact): scipy's
// beta / binom bodies are Boost's and log_ndtr is Faddeeva's, so the restatements here are
// accurate to a few ulp of the exact function, not bit copies.  FP64-VALU bound.
#include <math.h>

#include "pbh_error.h"
#include "pbh_ppf_ext.h"
#include "pbh_rng.h"
#include "pbh_special.h"
#include "pbh_special_ext.h"
#include "pbh_timing.h"

namespace pbh {


namespace {

struct Params4 {
  const double* ptr[4];
  double val[4];
  __device__ __forceinline__ double at(int j, int64_t i) const { return ptr[j] ? ptr[j][i] : val[j]; }
};

template <int D>
__device__ __forceinline__ double ppf_ext_one(double q, const Params4& p, int64_t i) {
  constexpr double inf = sf::kInf, nan = sf::kNaN;
  if constexpr (D == PBH_DIST_BINOM || D == PBH_DIST_BERNOULLI) {
    const double n = D == PBH_DIST_BINOM ? p.at(0, i) : 1.0;
    const double pp = D == PBH_DIST_BINOM ? p.at(1, i) : p.at(0, i);
    const double loc = D == PBH_DIST_BINOM ? p.at(2, i) : p.at(1, i);
    const bool ok = n >= 0.0 && n == floor(n) && pp >= 0.0 && pp <= 1.0 && loc == loc;
    if (q == 0.0) return -1.0 + loc;  // rv_discrete.ppf places _a - 1 + loc at q == 0 whatever the args
    if (!ok || !(q >= 0.0 && q <= 1.0)) return nan;
    if (q == 1.0) return n + loc;
    return sfx::binom_ppf01(q, n, pp) + loc;
  } else {
    const double a = p.at(0, i), b = p.at(1, i), loc = p.at(2, i), scale = p.at(3, i);
    bool ok = scale > 0.0 && loc == loc;
    double lower, upper;
    if constexpr (D == PBH_DIST_BETA) {
      ok = ok && a > 0.0 && b > 0.0;
      lower = 0.0;
      upper = 1.0;
    } else {  // truncnorm
      ok = ok && a < b;
      lower = a;
      upper = b;
    }
    if (!ok || !(q >= 0.0 && q <= 1.0)) return nan;
    if (q == 0.0) return lower * scale + loc;
    if (q == 1.0) return upper * scale + loc;
    double x;
    if constexpr (D == PBH_DIST_BETA)
      x = sfx::beta_ppf01(q, a, b);
    else
      x = sfx::truncnorm_ppf01(q, a, b);
    (void)inf;
    return x * scale + loc;
  }
}

template <int D>
__global__ __launch_bounds__(256) void k_ppf_ext(const double* __restrict__ q, int64_t q_stride, int64_t n, Params4 prm,
                                                 double* __restrict__ out, int32_t* flag) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double x = ppf_ext_one<D>(q[i * q_stride], prm, i);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

__global__ __launch_bounds__(256) void k_lhs_column(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, uint32_t col,
                                                    double* __restrict__ q) {
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * 256)
    q[i] = lhs_quantile(ph, fp, (uint64_t)(row0 + i), col);
}

}  // namespace

int ppf_ext(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params, int nparams, double* out,
            int32_t* flag, hipStream_t s) {
  const int want = dist == PBH_DIST_BERNOULLI ? 2 : (dist == PBH_DIST_BINOM ? 3 : 4);
  PBH_REQUIRE(nparams == want && params, "ppf: distribution %d takes %d parameters, got %d", dist, want, nparams);
  Params4 prm{};
  for (int j = 0; j < nparams; ++j) {
    prm.ptr[j] = params[j].ptr;
    prm.val[j] = params[j].value;
  }
  if (n == 0) return PBH_OK;
  dim3 g(grid_for(n, 256, 16384)), b(256);
  switch (dist) {
    case PBH_DIST_BETA:
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL(k_ppf_ext<PBH_DIST_BETA>, g, b, 0, s, q, q_stride, n, prm, out, flag));
      break;
    case PBH_DIST_TRUNCNORM:
      PBH_TIMED(kKPpf, s,
                hipLaunchKernelGGL(k_ppf_ext<PBH_DIST_TRUNCNORM>, g, b, 0, s, q, q_stride, n, prm, out, flag));
      break;
    case PBH_DIST_BINOM:
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL(k_ppf_ext<PBH_DIST_BINOM>, g, b, 0, s, q, q_stride, n, prm, out, flag));
      break;
    case PBH_DIST_BERNOULLI:
      PBH_TIMED(kKPpf, s,
                hipLaunchKernelGGL(k_ppf_ext<PBH_DIST_BERNOULLI>, g, b, 0, s, q, q_stride, n, prm, out, flag));
      break;
    default:
      set_error("ppf: unknown distribution id %d", dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// Fused-LHS entry for these distributions: the native LHS column is written to a stream-ordered
// temporary, then swept (16 B per draw instead of 8).
int lhs_ppf_ext(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist, const pbh_param* params,
                int nparams, double* out, int32_t* flag, hipStream_t s) {
  double* q = nullptr;
  PBH_CHECK_HIP(hipMallocAsync((void**)&q, (size_t)nrows * 8, s));
  hipLaunchKernelGGL(k_lhs_column, dim3(grid_for(nrows, 256, 16384)), dim3(256), 0, s, seed, n, row0, nrows,
                     (uint32_t)col, q);
  PBH_CHECK_LAUNCH();
  int st = ppf_ext(dist, q, 1, nrows, params, nparams, out, flag, s);
  PBH_CHECK_HIP(hipFreeAsync(q, s));
  return st;
}

}  // namespace pbh
