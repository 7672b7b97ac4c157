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
//   weibull_min ... chi2 (PBH_DIST_WEIBULL_MIN..CHI2): scipy's closed-form _ppf bodies, one
//              expression each (closed_ppf01), with rv_continuous.ppf's edges: q == 0 / 1 give
//              the support ends, invalid shapes or scale <= 0 give NaN; chi2 = 2 igami(df / 2, q)
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

constexpr bool is_closed(int d) { return d >= PBH_DIST_WEIBULL_MIN && d <= PBH_DIST_CHI2; }

constexpr int closed_shapes(int d) {
  return d == PBH_DIST_LOGUNIFORM ? 2
         : (d == PBH_DIST_WEIBULL_MIN || d == PBH_DIST_WEIBULL_MAX || d == PBH_DIST_PARETO || d == PBH_DIST_LOMAX ||
            d == PBH_DIST_GENEXTREME || d == PBH_DIST_GOMPERTZ || d == PBH_DIST_CHI2)
             ? 1
             : 0;
}

// _argcheck and the support [_a, _b] of scipy's class (rv_continuous default: every shape > 0)
template <int D>
__device__ __forceinline__ bool closed_support(double s0, double s1, double& lo, double& hi) {
  constexpr double inf = sf::kInf;
  lo = -inf;
  hi = inf;
  if constexpr (D == PBH_DIST_WEIBULL_MIN || D == PBH_DIST_RAYLEIGH || D == PBH_DIST_LOMAX ||
                D == PBH_DIST_GOMPERTZ || D == PBH_DIST_CHI2)
    lo = 0.0;
  if constexpr (D == PBH_DIST_WEIBULL_MAX) hi = 0.0;
  if constexpr (D == PBH_DIST_PARETO) lo = 1.0;
  if constexpr (D == PBH_DIST_LOGUNIFORM) {  // loguniform._get_support = (a, b), _argcheck a > 0, b > a
    lo = s0;
    hi = s1;
    return s0 > 0.0 && s1 > s0;
  }
  if constexpr (D == PBH_DIST_GENEXTREME) {  // _argcheck isfinite(c); support from the sign of c
    constexpr double tiny = 2.2250738585072014e-308;  // np.finfo(float).tiny
    if (s0 > 0.0) hi = 1.0 / fmax(s0, tiny);
    if (s0 < 0.0) lo = 1.0 / fmin(s0, -tiny);
    return isfinite(s0);
  }
  if constexpr (closed_shapes(D) == 1) return s0 > 0.0;
  return true;
}

// scipy _ppf for 0 < q < 1
template <int D>
__device__ __forceinline__ double closed_ppf01(double q, double s0, double s1) {
  if constexpr (D == PBH_DIST_WEIBULL_MIN) return pow(-log1p(-q), 1.0 / s0);
  if constexpr (D == PBH_DIST_WEIBULL_MAX) return -pow(-log(q), 1.0 / s0);
  if constexpr (D == PBH_DIST_LOGISTIC) {  // scipy special logit: log1p form on [0.3, 0.65]
    if (q < 0.3 || q > 0.65) return log(q / (1.0 - q));
    const double s = 2.0 * (q - 0.5);
    return log1p(s) - log1p(-s);
  }
  if constexpr (D == PBH_DIST_CAUCHY) {  // Boost cauchy quantile: P in (-0.5, 0.5], -1 / tan(pi P)
    double p = q - floor(q);
    if (p > 0.5) p = p - 1.0;
    if (p == 0.5) return 0.0;
    return -1.0 / tan(sf::kPi * p);
  }
  if constexpr (D == PBH_DIST_LAPLACE) return q > 0.5 ? -log(2.0 * (1.0 - q)) : log(2.0 * q);
  if constexpr (D == PBH_DIST_GUMBEL_R) return -log(-log(q));
  if constexpr (D == PBH_DIST_GUMBEL_L) return log(-log1p(-q));
  if constexpr (D == PBH_DIST_PARETO) return pow(1.0 - q, -1.0 / s0);
  if constexpr (D == PBH_DIST_LOGUNIFORM) return exp(log(s0) + q * (log(s1) - log(s0)));
  if constexpr (D == PBH_DIST_RAYLEIGH) return sqrt(-2.0 * log1p(-q));
  if constexpr (D == PBH_DIST_LOMAX) return expm1(-log1p(-q) / s0);
  if constexpr (D == PBH_DIST_GENEXTREME) {
    const double x = -log(-log(q));
    return (x == x && s0 != 0.0) ? -expm1(-s0 * x) / s0 : x;
  }
  if constexpr (D == PBH_DIST_GOMPERTZ) return log1p(-1.0 / s0 * log1p(-q));
  if constexpr (D == PBH_DIST_CHI2) return 2.0 * sf::igami(s0 / 2.0, q);
  return sf::kNaN;
}

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
  } else if constexpr (is_closed(D)) {
    constexpr int S = closed_shapes(D);
    const double s0 = S > 0 ? p.at(0, i) : 0.0, s1 = S > 1 ? p.at(1, i) : 0.0;
    const double loc = p.at(S, i), scale = p.at(S + 1, i);
    double lo, hi;
    const bool ok = closed_support<D>(s0, s1, lo, hi) && scale > 0.0 && loc == loc;
    if (!ok || !(q >= 0.0 && q <= 1.0)) return nan;
    if (q == 0.0) return lo * scale + loc;
    if (q == 1.0) return hi * scale + loc;
    return closed_ppf01<D>(q, s0, s1) * scale + loc;
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

// one kernel for the swept column (q[i * q_stride]) and the fused native-LHS column (LHS: the
// quantile of row row0 + i generated in registers, 8 B per draw instead of 16)
struct LhsCol {
  uint64_t seed;
  int64_t n, row0;
  uint32_t col;
};

template <int D, bool LHS>
__global__ __launch_bounds__(256) void k_ppf_ext(const double* __restrict__ q, int64_t q_stride, LhsCol lc, int64_t n,
                                                 Params4 prm, double* __restrict__ out, int32_t* flag) {
  Philox ph(lc.seed);
  FeistelPerm fp(ph, (uint64_t)(LHS ? lc.n : 1), lc.col);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double qi = LHS ? lhs_quantile(ph, fp, (uint64_t)(lc.row0 + i), lc.col) : q[i * q_stride];
    const double x = ppf_ext_one<D>(qi, prm, i);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

template <int D>
struct DistTag {
  static constexpr int value = D;
};

// f(DistTag<D>{}) for the distribution ids handled here; false for any other id
template <class F>
bool dispatch_ext(int dist, F&& f) {
  switch (dist) {
#define PBH_EXT(D) \
  case D:          \
    f(DistTag<D>{}); \
    return true;
    PBH_EXT(PBH_DIST_BETA)
    PBH_EXT(PBH_DIST_TRUNCNORM)
    PBH_EXT(PBH_DIST_BINOM)
    PBH_EXT(PBH_DIST_BERNOULLI)
    PBH_EXT(PBH_DIST_WEIBULL_MIN)
    PBH_EXT(PBH_DIST_WEIBULL_MAX)
    PBH_EXT(PBH_DIST_LOGISTIC)
    PBH_EXT(PBH_DIST_CAUCHY)
    PBH_EXT(PBH_DIST_LAPLACE)
    PBH_EXT(PBH_DIST_GUMBEL_R)
    PBH_EXT(PBH_DIST_GUMBEL_L)
    PBH_EXT(PBH_DIST_PARETO)
    PBH_EXT(PBH_DIST_LOGUNIFORM)
    PBH_EXT(PBH_DIST_RAYLEIGH)
    PBH_EXT(PBH_DIST_LOMAX)
    PBH_EXT(PBH_DIST_GENEXTREME)
    PBH_EXT(PBH_DIST_GOMPERTZ)
    PBH_EXT(PBH_DIST_CHI2)
#undef PBH_EXT
    default:
      return false;
  }
}

int launch_ext(int dist, const double* q, int64_t q_stride, const LhsCol* lc, int64_t n, const pbh_param* params,
               int nparams, double* out, int32_t* flag, hipStream_t s) {
  const int want = dist == PBH_DIST_BERNOULLI ? 2
                   : dist == PBH_DIST_BINOM   ? 3
                   : is_closed(dist)          ? closed_shapes(dist) + 2
                                              : 4;
  PBH_REQUIRE(nparams == want && params, "ppf: distribution %d takes %d parameters, got %d", dist, want, nparams);
  Params4 prm{};
  for (int j = 0; j < nparams; ++j) {
    prm.ptr[j] = params[j].ptr;
    prm.val[j] = params[j].value;
  }
  if (n == 0) return PBH_OK;
  dim3 g(grid_for(n, 256, 16384)), b(256);
  const LhsCol l = lc ? *lc : LhsCol{0, 1, 0, 0};
  const bool known = dispatch_ext(dist, [&](auto tag) {
    constexpr int D = decltype(tag)::value;
    if (lc)
      PBH_TIMED(kKLhsPpf, s, hipLaunchKernelGGL((k_ppf_ext<D, true>), g, b, 0, s, q, q_stride, l, n, prm, out, flag));
    else
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL((k_ppf_ext<D, false>), g, b, 0, s, q, q_stride, l, n, prm, out, flag));
  });
  if (!known) {
    set_error("ppf: unknown distribution id %d", dist);
    return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

}  // namespace

int ppf_ext(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params, int nparams, double* out,
            int32_t* flag, hipStream_t s) {
  return launch_ext(dist, q, q_stride, nullptr, n, params, nparams, out, flag, s);
}

// Fused-LHS entry for these distributions: the native LHS quantile is generated in the ppf kernel
int lhs_ppf_ext(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist, const pbh_param* params,
                int nparams, double* out, int32_t* flag, hipStream_t s) {
  const LhsCol lc{seed, n, row0, (uint32_t)col};
  return launch_ext(dist, nullptr, 0, &lc, nrows, params, nparams, out, flag, s);
}

}  // namespace pbh
