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
#include "pbh_glibc.h"
#include "pbh_table_cache.h"
#include "pbh_ppf_ext.h"
#include "pbh_rng.h"
#include "pbh_special.h"
#include "pbh_special_ext.h"
#include "pbh_step4.h"
#include "pbh_timing.h"

namespace pbh {


namespace {

struct Params4 {
  const double* ptr[4];
  double val[4];
  sfx::BetaGuide bg;  // beta with scalar (a, b): the guide table (bg.z == NULL: none)
  sf::GammaGuide gg;  // chi, maxwell, nakagami, chi2 with a scalar shape: gammaincinv's guide (gg.y == NULL: none)
  sf::GammaAux ga;
  const double* dt;   // binom, bernoulli, nbinom with scalar parameters: CDF (dt) and its complement
  int dlen;           // (dt + dlen) of k = 0 .. dlen - 1 (dt == NULL: none)
  int tn_ok;          // truncnorm with scalar (a, b): tn = truncnorm_consts(a, b), set on the host
  double tn[2];
  __device__ __forceinline__ double at(int j, int64_t i) const { return ptr[j] ? ptr[j][i] : val[j]; }
};

// the CDF tables of a scalar-parameter discrete distribution: cdf[k] and its complement for
// k = 0 .. len - 1, by the same functions the per-draw search evaluates (so every lookup answers
// what that search would)
template <int D>
__global__ void k_discrete_table(double s0, double s1, int len, double* __restrict__ cdf, double* __restrict__ ccdf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len) return;
  if constexpr (D == PBH_DIST_NBINOM) {
    cdf[k] = sfx::nbdtr((double)k, s0, s1);
    ccdf[k] = sfx::nbdtrc((double)k, s0, s1);
  } else {  // binom (n, p); bernoulli is binom with n = 1
    const double n = D == PBH_DIST_BINOM ? s0 : 1.0, pp = D == PBH_DIST_BINOM ? s1 : s0;
    cdf[k] = sfx::bdtr((double)k, n, pp);
    ccdf[k] = sfx::bdtrc((double)k, n, pp);
  }
}

// binom_ppf01 / nbinom_ppf01 from the tables: below the median the first k with cdf[k] >= q, above
// it the first k with ccdf[k] <= 1 - q (binary searches); -1 when the answer lies past the table
__device__ __forceinline__ double discrete_from_table(double q, const double* cdf, int len) {
  const double* ccdf = cdf + len;
  int lo = 0, hi = len;  // first index in [lo, hi) satisfying the predicate
  if (q <= 0.5) {
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] >= q)
        hi = mid;
      else
        lo = mid + 1;
    }
  } else {
    const double r = 1.0 - q;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ccdf[mid] <= r)
        hi = mid;
      else
        lo = mid + 1;
    }
  }
  return lo < len ? (double)lo : -1.0;
}

// betabinom (n, a, b) and hypergeom (M, n, N) (round 6): scipy's generic discrete ppf, the smallest k
// of the support with cdf(k) >= q (_drv2_ppfsingle's bisection), cdf(k) the sum of the pmf over
// [lo, k] (rv_discrete._cdf_single; hypergeom._cdf is Boost's sum of its pdf).  Summed here in order
// from lo, by the per-draw loop and the scalar-parameter table alike, so the two answer the same; the
// pmf as scipy's betabinom._logpmf writes it, log C(a, b) = -log(a + 1) - betaln(a - b + 1, b + 1).
// The outputs equal scipy's except where q lies within the summation's rounding (~1e-15) of a CDF value.
PBH_HD inline double lchoose(double a, double b) { return -log(a + 1.0) - sfx::lbeta(a - b + 1.0, b + 1.0); }

// _argcheck and the support [lo, hi]
PBH_HD inline bool sum_bounds(int d, double s0, double s1, double s2, double* lo, double* hi) {
  if (d == PBH_DIST_BETABINOM) {
    *lo = 0.0;
    *hi = s0;
    return s0 >= 0.0 && s0 == floor(s0) && s1 > 0.0 && s2 > 0.0;
  }
  if (d == PBH_DIST_NHYPERGEOM) {  // M, n, r: support [0, n]
    *lo = 0.0;
    *hi = s1;
    return s1 >= 0.0 && s1 <= s0 && s2 >= 0.0 && s2 <= s0 - s1 && s0 == floor(s0) && s1 == floor(s1) &&
           s2 == floor(s2);
  }
  *lo = fmax(s2 - (s0 - s1), 0.0);  // hypergeom: M, n, N
  *hi = fmin(s1, s2);
  return s0 > 0.0 && s1 >= 0.0 && s2 >= 0.0 && s1 <= s0 && s2 <= s0 && s0 == floor(s0) && s1 == floor(s1) &&
         s2 == floor(s2);
}

template <int D>
__device__ __forceinline__ double sum_pmf(double k, double s0, double s1, double s2) {
  if constexpr (D == PBH_DIST_BETABINOM)
    return exp(lchoose(s0, k) + sfx::lbeta(k + s1, s0 - k + s2) - sfx::lbeta(s1, s2));
  else if constexpr (D == PBH_DIST_NHYPERGEOM) {  // scipy nhypergeom._logpmf (M, n, r); 1 at r = k = 0
    if (s2 == 0.0 && k == 0.0) return 1.0;
    const double M = s0, n = s1, r = s2;
    return exp(-sfx::lbeta(k + 1, r) + sfx::lbeta(k + r, 1) - sfx::lbeta(n - k + 1, M - r - n + 1) +
               sfx::lbeta(M - r - k + 1, 1) + sfx::lbeta(n + 1, M - n + 1) - sfx::lbeta(M + 1, 1));
  } else
    return exp(lchoose(s1, k) + lchoose(s0 - s1, s2 - k) - lchoose(s0, s2));
}

// hypergeom above q = 1/2 follows Boost's cdf there, 1 - (the pmf summed from the top down to k + 1):
// the first k with fl(1 - S(k)) >= q, scanned down from hi (summed from lo, the pmf's rounding would
// overshoot 1 by ~1e-13 and move q = 1 - 2^-53's answer by several values)
template <int D>
__device__ __forceinline__ double sum_ppf01(double q, double s0, double s1, double s2, double lo, double hi) {
  if (D == PBH_DIST_HYPERGEOM && q > 0.5) {
    double k = hi, S = 0.0;
    while (k > lo) {
      const double S2 = S + sum_pmf<D>(k, s0, s1, s2);
      if (!(1.0 - S2 >= q)) break;
      S = S2;
      k -= 1.0;
    }
    return k;
  }
  double k = lo, c = sum_pmf<D>(lo, s0, s1, s2);
  while (c < q && k < hi) {
    k += 1.0;
    c += sum_pmf<D>(k, s0, s1, s2);
  }
  return k;
}

// yulesimon(alpha) (round 6): scipy's generic discrete ppf on its closed cdf 1 - k B(k, alpha + 1)
// (support k >= 1), rv_discrete._drv2_ppfsingle step for step: b grows from max(100 q, 10) by doubling
// steps until cdf(b) >= q, then bisection with c = int((a + b) / 2) from a = 1, which returns the
// first c it meets with cdf(c) == q -- near q = 1 the cdf rounds to q over a run of k, and scipy's
// answer is the one its bisection path lands on, not the smallest
__device__ __forceinline__ double yulesimon_cdf(double k, double a) { return 1.0 - k * sfx::beta_fn(k, a + 1.0); }
__device__ __forceinline__ double yulesimon_ppf01(double q, double al) {
  double b = fmax(100.0 * q, 10.0), step = 10.0, qb = 1.0;
  for (int it = 0; it < 1100; ++it) {
    if (!(b < sf::kInf)) {
      qb = 1.0;
      break;
    }
    qb = yulesimon_cdf(b, al);
    if (qb < q) {
      b += step;
      step *= 2.0;
    } else {
      break;
    }
  }
  double a = 1.0, qa = yulesimon_cdf(1.0, al);
  for (int i = 0; i < 2046; ++i) {
    if (qa == q) return a;
    if (qb == q) return b;
    if (b <= a + 1) return qa > q ? a : b;
    const double c = trunc((a + b) / 2.0);
    const double qc = yulesimon_cdf(c, al);
    if (qc < q) {
      a = c;
      qa = qc;
    } else if (qc > q) {
      b = c;
      qb = qc;
    } else {
      return c;
    }
  }
  return sf::kNaN;
}

// zipfian(a, n) (round 6): scipy's generic discrete ppf (_drv2_ppfsingle step for step, the finite
// support [1, n]: no bracket search) on its closed cdf H(k, a) / H(n, a), H the generalized harmonic
// number: zeta(a, 1) - zeta(a, k + 1) for a > 1 (Cephes' Hurwitz zeta, Euler-Maclaurin with its
// twelve Bernoulli terms), else the sum of 1 / i^a from i = k down to 1 -- over glibc's pow restated,
// as scipy's compiled zeta and numpy's power call it, so the cdf is scipy's to the bit
__device__ __forceinline__ double hurwitz_zeta(double x, double q) {
  const double A[12] = {12.0, -720.0, 30240.0, -1209600.0, 47900160.0, -1.8924375803183791606e9, 7.47242496e10,
                        -2.950130727918164224e12, 1.1646782814350067249e14, -4.5979787224074726105e15,
                        1.8152105401943546773e17, -7.1661652561756670113e18};
  constexpr double kMachEp = 1.11022302462515654042e-16;
  if (x == 1.0) return sf::kInf;
  if (q > 1e8) return (1 / (x - 1) + 1 / (2 * q)) * glibc::pow(q, 1 - x);
  double s = glibc::pow(q, -x), a = q, b = 0.0;
  int i = 0;
  while (i < 9 || a <= 9.0) {
    i += 1;
    a += 1.0;
    b = glibc::pow(a, -x);
    s += b;
    if (fabs(b / s) < kMachEp) return s;
  }
  const double w = a;
  s += b * w / (x - 1.0);
  s -= 0.5 * b;
  a = 1.0;
  double k = 0.0;
  for (i = 0; i < 12; ++i) {
    a *= x + k;
    b /= w;
    double t = a * b / A[i];
    s = s + t;
    t = fabs(t / s);
    if (t < kMachEp) return s;
    k += 1.0;
    a *= x + k;
    b /= w;
    k += 1.0;
  }
  return s;
}
__device__ __forceinline__ double gen_harmonic(double k, double a) {
  if (a > 1) return hurwitz_zeta(a, 1.0) - hurwitz_zeta(a, k + 1);
  double out = 0.0;
  for (double i = k; i > 0.0; i -= 1.0) out += 1 / glibc::pow(i, a);
  return out;
}
__device__ __forceinline__ double zipfian_ppf01(double q, double al, double n) {
  const double hn = gen_harmonic(n, al);
  auto cdf = [al, hn](double k) { return gen_harmonic(k, al) / hn; };
  double a = 1.0, qa = cdf(1.0), b = n, qb = 1.0;
  for (int i = 0; i < 2046; ++i) {
    if (qa == q) return a;
    if (qb == q) return b;
    if (b <= a + 1) return qa > q ? a : b;
    const double c = trunc((a + b) / 2.0);
    const double qc = cdf(c);
    if (qc < q) {
      a = c;
      qa = qc;
    } else if (qc > q) {
      b = c;
      qb = qc;
    } else {
      return c;
    }
  }
  return sf::kNaN;
}

// the table of these two: pmf(lo + i) in parallel, then one thread sums them in the per-draw loops'
// orders: cdf[i] from lo up, and the complement the q > 1/2 search compares with 1 - q: 1 - cdf[i],
// or for hypergeom 1 - fl(1 - S(i)) with S summed from the top (exact: fl(1 - S) >= 1/2 there)
template <int D>
__global__ void k_sum_pmf(double s0, double s1, double s2, double lo, int len, double* __restrict__ pmf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < len) pmf[i] = sum_pmf<D>(lo + (double)i, s0, s1, s2);
}
__global__ void k_sum_cdf(int len, int from_top, double* __restrict__ cdf, double* __restrict__ ccdf) {
  if (threadIdx.x || blockIdx.x) return;
  if (from_top) {
    double S = 0.0;
    for (int i = len - 1; i >= 0; --i) {
      ccdf[i] = 1.0 - (1.0 - S);
      S += cdf[i];
    }
  }
  double c = 0.0;
  for (int i = 0; i < len; ++i) {
    c += cdf[i];
    cdf[i] = c;
    if (!from_top) ccdf[i] = 1.0 - c;
  }
}

// the beta guide for scalar (a, b) (sfx::BetaGuide): nodes, then the midpoint check
__global__ void k_beta_guide(double a, double b, double lb, double* z, double* d1, double* d2) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < sfx::kBetaGuideM) sfx::beta_guide_entry(a, b, lb, sfx::kBetaGuideW0 + j * sfx::kBetaGuideH, &z[j], &d1[j], &d2[j]);
}

__global__ void k_beta_guide_check(double a, double b, sfx::BetaGuide T, double* ok) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < sfx::kBetaGuideM) ok[j] = j < sfx::kBetaGuideM - 1 ? sfx::beta_guide_check(a, b, T, j) : 0.0;
}

constexpr int kDiscreteTableMax = 1 << 16;  // CDF entries of a discrete distribution's table

// the shape a of gammaincinv(a, q) behind chi (df / 2), maxwell (1.5), nakagami (nu), chi2 (df / 2),
// and of gammainccinv(a, q) behind invgamma (a)
inline double gamma_family_a(int dist, double s0) {
  return dist == PBH_DIST_MAXWELL ? 1.5 : (dist == PBH_DIST_NAKAGAMI || dist == PBH_DIST_INVGAMMA) ? s0 : 0.5 * s0;
}
constexpr bool is_gamma_family(int d) {
  return d == PBH_DIST_CHI || d == PBH_DIST_MAXWELL || d == PBH_DIST_NAKAGAMI || d == PBH_DIST_CHI2;
}

// the discrete table's length for scalar parameters (0: none): every k up to the answer at the
// largest quantile below 1 for binom / bernoulli (n + 1 values), and for nbinom up to its answer at
// q = 1 - 2^-40 (the rare q beyond take the per-draw search)
int discrete_table_len(int dist, const double* v) {
  if (dist == PBH_DIST_BINOM) {
    if (!(v[0] >= 0.0 && v[0] == floor(v[0]) && v[1] >= 0.0 && v[1] <= 1.0 && v[0] + 1.0 <= kDiscreteTableMax)) return 0;
    return (int)v[0] + 1;
  }
  if (dist == PBH_DIST_BERNOULLI) return (v[0] >= 0.0 && v[0] <= 1.0) ? 2 : 0;
  if (dist == PBH_DIST_BETABINOM || dist == PBH_DIST_HYPERGEOM || dist == PBH_DIST_NHYPERGEOM) {  // v: the three shapes
    double lo, hi;
    if (!sum_bounds(dist, v[0], v[1], v[2], &lo, &hi) || !(hi - lo + 1.0 <= kDiscreteTableMax)) return 0;
    return (int)(hi - lo) + 1;
  }
  if (dist == PBH_DIST_NBINOM) {
    if (!(v[0] > 0.0 && v[1] > 0.0 && v[1] < 1.0 && v[0] < 1e6 && v[1] > 1e-4)) return 0;
    const double top = sfx::nbinom_ppf01(1.0 - 0x1p-40, v[0], v[1]);
    return top + 1.0 <= kDiscreteTableMax ? (int)top + 1 : 0;
  }
  return 0;
}

// the setup table of `dist` with these parameters (stream-ordered allocation, NULL when the
// distribution has none): beta with scalar, valid (a, b) -> its guide; chi / maxwell / nakagami /
// chi2 with a scalar shape -> gammaincinv's guide (pbh_ppf.hip gamma_guide_table); binom /
// bernoulli / nbinom with scalar parameters -> [len, CDF (len), complement (len)]; the process
// cache's (pbh_table_cache.hip) when it has room, callers end with release_table
double* beta_guide_table(double a, double b, hipStream_t s);

double* build_table(int dist, const pbh_param* params, int nparams, hipStream_t s) {
  if (dist == PBH_DIST_T) {  // stdtrit through I^-1(.; df / 2, 1 / 2): beta's guide of (df / 2, 1 / 2)
    if (nparams < 1 || params[0].ptr) return nullptr;
    const double df = params[0].value;
    if (!(df > 0.0 && df < 1e5)) return nullptr;
    return beta_guide_table(0.5 * df, 0.5, s);
  }
  if (is_gamma_family(dist) || dist == PBH_DIST_INVGAMMA) {
    if (dist != PBH_DIST_MAXWELL && (nparams < 1 || params[0].ptr)) return nullptr;
    return gamma_guide_table(gamma_family_a(dist, nparams ? params[0].value : 0.0), s);
  }
  if (dist == PBH_DIST_BETABINOM || dist == PBH_DIST_HYPERGEOM || dist == PBH_DIST_NHYPERGEOM) {
    if (nparams < 3 || params[0].ptr || params[1].ptr || params[2].ptr) return nullptr;
    const double v[3] = {params[0].value, params[1].value, params[2].value};
    const int len = discrete_table_len(dist, v);
    if (len <= 0) return nullptr;
    double lo, hi;
    (void)sum_bounds(dist, v[0], v[1], v[2], &lo, &hi);
    auto build = [=](double* t, hipStream_t st) {
      const double hdr = (double)len;
      if (hipMemcpyAsync(t, &hdr, sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) return false;
      const dim3 g((unsigned)((len + 255) / 256)), b(256);
      if (dist == PBH_DIST_BETABINOM)
        hipLaunchKernelGGL(k_sum_pmf<PBH_DIST_BETABINOM>, g, b, 0, st, v[0], v[1], v[2], lo, len, t + 1);
      else if (dist == PBH_DIST_NHYPERGEOM)
        hipLaunchKernelGGL(k_sum_pmf<PBH_DIST_NHYPERGEOM>, g, b, 0, st, v[0], v[1], v[2], lo, len, t + 1);
      else
        hipLaunchKernelGGL(k_sum_pmf<PBH_DIST_HYPERGEOM>, g, b, 0, st, v[0], v[1], v[2], lo, len, t + 1);
      hipLaunchKernelGGL(k_sum_cdf, dim3(1), dim3(64), 0, st, len, dist == PBH_DIST_HYPERGEOM ? 1 : 0, t + 1,
                         t + 1 + len);
      return hipGetLastError() == hipSuccess;
    };
    const size_t bytes = (size_t)(2 * len + 1) * sizeof(double);
    const double key[4] = {(double)dist, v[0], v[1], v[2]};
    if (double* t = cached_table(kTabDiscrete, key, 4, bytes, s, build)) return t;
    double* t = nullptr;
    if (hipMallocAsync((void**)&t, bytes, s) != hipSuccess) return nullptr;
    if (!build(t, s)) {
      (void)hipFreeAsync(t, s);
      return nullptr;
    }
    return t;
  }
  if (dist == PBH_DIST_BINOM || dist == PBH_DIST_BERNOULLI || dist == PBH_DIST_NBINOM) {
    const int ns = dist == PBH_DIST_BERNOULLI ? 1 : 2;
    if (nparams < ns) return nullptr;
    double v[2] = {0.0, 0.0};
    for (int j = 0; j < ns; ++j) {
      if (params[j].ptr) return nullptr;
      v[j] = params[j].value;
    }
    const int len = discrete_table_len(dist, v);
    if (len <= 0) return nullptr;
    auto build = [=](double* t, hipStream_t st) {
      const double hdr = (double)len;
      if (hipMemcpyAsync(t, &hdr, sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) return false;
      const dim3 g((unsigned)((len + 255) / 256)), b(256);
      if (dist == PBH_DIST_BINOM)
        hipLaunchKernelGGL(k_discrete_table<PBH_DIST_BINOM>, g, b, 0, st, v[0], v[1], len, t + 1, t + 1 + len);
      else if (dist == PBH_DIST_BERNOULLI)
        hipLaunchKernelGGL(k_discrete_table<PBH_DIST_BERNOULLI>, g, b, 0, st, v[0], v[1], len, t + 1, t + 1 + len);
      else
        hipLaunchKernelGGL(k_discrete_table<PBH_DIST_NBINOM>, g, b, 0, st, v[0], v[1], len, t + 1, t + 1 + len);
      return hipGetLastError() == hipSuccess;
    };
    const size_t bytes = (size_t)(2 * len + 1) * sizeof(double);
    const double key[3] = {(double)dist, v[0], v[1]};
    if (double* t = cached_table(kTabDiscrete, key, 3, bytes, s, build)) return t;
    double* t = nullptr;
    if (hipMallocAsync((void**)&t, bytes, s) != hipSuccess) return nullptr;
    if (!build(t, s)) {
      (void)hipFreeAsync(t, s);
      return nullptr;
    }
    return t;
  }
  if (dist != PBH_DIST_BETA || nparams < 2 || params[0].ptr || params[1].ptr) return nullptr;
  return beta_guide_table(params[0].value, params[1].value, s);
}

double* beta_guide_table(double a, double b, hipStream_t s) {
  if (!(a > 0.0 && b > 0.0 && isfinite(a) && isfinite(b))) return nullptr;
  constexpr int m = sfx::kBetaGuideM;
  auto build = [=](double* t, hipStream_t st) {
    const unsigned g = (unsigned)((m + 63) / 64);
    hipLaunchKernelGGL(k_beta_guide, dim3(g), dim3(64), 0, st, a, b, sfx::lbeta(a, b), t, t + m, t + 2 * m);
    const sfx::BetaGuide T{t, t + m, t + 2 * m, t + 3 * m};
    hipLaunchKernelGGL(k_beta_guide_check, dim3(g), dim3(64), 0, st, a, b, T, t + 3 * m);
    return hipGetLastError() == hipSuccess;
  };
  const size_t bytes = (size_t)4 * m * sizeof(double);
  const double key[2] = {a, b};
  if (double* t = cached_table(kTabBetaGuide, key, 2, bytes, s, build)) return t;
  double* t = nullptr;
  if (hipMallocAsync((void**)&t, bytes, s) != hipSuccess) return nullptr;
  if (!build(t, s)) {
    (void)hipFreeAsync(t, s);
    return nullptr;
  }
  return t;
}

sfx::BetaGuide guide_of(const double* t) {
  constexpr int m = sfx::kBetaGuideM;
  return t ? sfx::BetaGuide{t, t + m, t + 2 * m, t + 3 * m} : sfx::BetaGuide{};
}

// Params4's view of build_table's table for `dist` (scalar parameters p.val); truncnorm with
// scalar (a, b) takes its (a, b)-only terms evaluated here once instead of per draw (log_ndtr and
// log_gauss_mass: 0.41 -> 0.24 ms per 1e7, ext_sweep_r5zj.json; within scipy's 1e-10 as before, and the same constants
// reach every kernel of a call, so the sweep, the sorted generator and step 4 agree)
void attach_table(int dist, const double* t, Params4& p) {
  if (dist == PBH_DIST_TRUNCNORM && !p.ptr[0] && !p.ptr[1] && p.val[0] < p.val[1]) {
    sfx::truncnorm_consts(p.val[0], p.val[1], &p.tn[0], &p.tn[1]);
    p.tn_ok = 1;
  }
  if (!t) return;
  if (dist == PBH_DIST_BETA || dist == PBH_DIST_T) {
    p.bg = guide_of(t);
  } else if (is_gamma_family(dist) || dist == PBH_DIST_INVGAMMA) {
    const int m = sf::kGammaGuideM;
    const double a = gamma_family_a(dist, p.val[0]);
    p.gg = sf::GammaGuide{t, t + m, t + 2 * m, t + 3 * m, m, sf::kGammaGuideZ0, sf::kGammaGuideH, 1.0 / sf::kGammaGuideH};
    p.ga = sf::gamma_aux(a);
  } else if (dist == PBH_DIST_BETABINOM || dist == PBH_DIST_HYPERGEOM || dist == PBH_DIST_NHYPERGEOM) {
    p.dlen = discrete_table_len(dist, p.val);
    p.dt = p.dlen > 0 ? t + 1 : nullptr;
  } else if (dist == PBH_DIST_BINOM || dist == PBH_DIST_BERNOULLI || dist == PBH_DIST_NBINOM) {
    const int ns = dist == PBH_DIST_BERNOULLI ? 1 : 2;
    p.dlen = discrete_table_len(dist, p.val);  // the same length the table was built with
    p.dt = p.dlen > 0 ? t + 1 : nullptr;
    (void)ns;
  }
}

constexpr bool is_closed(int d) {
  return (d >= PBH_DIST_WEIBULL_MIN && d <= PBH_DIST_TRAPEZOID) || d == PBH_DIST_INVGAMMA || d == PBH_DIST_T ||
         (d >= PBH_DIST_JOHNSONSU && d <= PBH_DIST_BETAPRIME) || (d >= PBH_DIST_PEARSON3 && d <= PBH_DIST_WALD) || (d >= PBH_DIST_SKEWNORM && d <= PBH_DIST_KSTWOBIGN) || d == PBH_DIST_REL_BREITWIGNER;
}
// discrete distributions beyond binom / bernoulli (round 5): p, loc / low, high, loc / n, p, loc;
// round 6: a, loc (dlaplace) / lambda, loc (planck) / lambda, N, loc (boltzmann)
constexpr bool is_discrete2(int d) {
  return d == PBH_DIST_GEOM || d == PBH_DIST_RANDINT || d == PBH_DIST_NBINOM || d == PBH_DIST_DLAPLACE ||
         d == PBH_DIST_PLANCK || d == PBH_DIST_BOLTZMANN || d == PBH_DIST_BETABINOM || d == PBH_DIST_HYPERGEOM ||
         d == PBH_DIST_NHYPERGEOM || d == PBH_DIST_YULESIMON || d == PBH_DIST_ZIPFIAN;
}

constexpr int closed_shapes(int d) {
  return (d == PBH_DIST_LOGUNIFORM || d == PBH_DIST_BURR || d == PBH_DIST_BURR12 || d == PBH_DIST_EXPONWEIB ||
          d == PBH_DIST_TRAPEZOID || d == PBH_DIST_JOHNSONSU || d == PBH_DIST_JOHNSONSB || d == PBH_DIST_MIELKE ||
          d == PBH_DIST_TRUNCPARETO || d == PBH_DIST_GENGAMMA || d == PBH_DIST_F || d == PBH_DIST_BETAPRIME ||
          d == PBH_DIST_KAPPA4 || d == PBH_DIST_CRYSTALBALL || d == PBH_DIST_POWERLOGNORM || d == PBH_DIST_JF_SKEW_T)
             ? 2
         : (d == PBH_DIST_WEIBULL_MIN || d == PBH_DIST_WEIBULL_MAX || d == PBH_DIST_PARETO || d == PBH_DIST_LOMAX ||
            d == PBH_DIST_GENEXTREME || d == PBH_DIST_GOMPERTZ || d == PBH_DIST_CHI2 || d == PBH_DIST_POWERLAW ||
            d == PBH_DIST_GENPARETO || d == PBH_DIST_FISK || d == PBH_DIST_EXPONPOW || d == PBH_DIST_BRADFORD ||
            d == PBH_DIST_INVWEIBULL || d == PBH_DIST_LOGLAPLACE || d == PBH_DIST_TRUNCEXPON || d == PBH_DIST_CHI ||
            d == PBH_DIST_NAKAGAMI || d == PBH_DIST_DWEIBULL || d == PBH_DIST_KAPPA3 ||
            d == PBH_DIST_GENHALFLOGISTIC || d == PBH_DIST_ALPHA || d == PBH_DIST_FATIGUELIFE ||
            d == PBH_DIST_GENLOGISTIC || d == PBH_DIST_INVGAMMA || d == PBH_DIST_T || d == PBH_DIST_POWERNORM ||
            d == PBH_DIST_LAPLACE_ASYMMETRIC || d == PBH_DIST_TUKEYLAMBDA || d == PBH_DIST_LOGGAMMA ||
            d == PBH_DIST_DGAMMA || d == PBH_DIST_RDIST || d == PBH_DIST_PEARSON3 || d == PBH_DIST_GENNORM ||
            d == PBH_DIST_HALFGENNORM || d == PBH_DIST_WRAPCAUCHY || d == PBH_DIST_SKEWCAUCHY ||
            d == PBH_DIST_FOLDCAUCHY || d == PBH_DIST_FOLDNORM || d == PBH_DIST_INVGAUSS || d == PBH_DIST_SKEWNORM ||
            d == PBH_DIST_RECIPINVGAUSS || d == PBH_DIST_EXPONNORM || d == PBH_DIST_ARGUS ||
            d == PBH_DIST_REL_BREITWIGNER)
             ? 1
             : 0;
}

// scipy.special.boxcox1p (scipy _boxcox.pxd): log1p(x) for a vanishing lambda, else
// expm1(lambda log1p(x)) / lambda
__device__ __forceinline__ double boxcox1p(double x, double lmbda) {
  const double lgx = log1p(x);
  if (fabs(lmbda) < 1e-19 || (fabs(lgx) < 1e-289 && fabs(lmbda) < 1e273)) return lgx;
  return expm1(lmbda * lgx) / lmbda;
}

// scipy.special.boxcox (scipy _boxcox.pxd): log(x) for a vanishing lambda, else
// expm1(lambda log(x)) / lambda
__device__ __forceinline__ double boxcox(double x, double lmbda) {
  if (fabs(lmbda) < 1e-19) return log(x);
  return expm1(lmbda * log(x)) / lmbda;
}

// scipy.special.expit (xsf): 1 / (1 + exp(-x))
__device__ __forceinline__ double expit(double x) { return 1.0 / (1.0 + exp(-x)); }

// scipy.special.powm1 (Boost powm1) for x > 0: expm1(y log x) when that is the accurate form,
// else pow(x, y) - 1
__device__ __forceinline__ double powm1(double x, double y) {
  if (x > 0.0 && (fabs(y * (x - 1.0)) < 0.5 || fabs(y) < 0.2)) {
    const double l = y * log(x);
    if (l < 0.5) return expm1(l);
  }
  return pow(x, y) - 1.0;
}

// trapezoid._cdf(x, c, d) at x = c and x = d (the middle piece), the breaks of its _ppf
__device__ __forceinline__ double trapezoid_mid_cdf(double x, double c, double d) {
  return (c + 2.0 * (x - c)) / (d - c + 1.0);
}

// ---- round 6, third set: quantiles scipy finds by a search (foldcauchy / foldnorm: the generic
// rv_continuous._ppf, brentq on _cdf to xtol 1e-14; invgauss / wald: Boost's inverse_gaussian
// quantile, its complement above q = 1/2; cosine: xsf's cosine_invcdf), each solved here to a few
// ulps by its own method, so they agree with scipy's to its own tolerance

// the x in (lo, hi) with f(x) = t, f increasing (inc) or decreasing (fp(x) its signed derivative): Newton steps kept
// inside the shrinking bracket, bisection when a step leaves it, until a step moves x by <= 4 ulps
template <class F, class Fp>
__device__ __forceinline__ double bracket_newton(F f, Fp fp, double t, double lo, double hi, double x, bool inc) {
  for (int it = 0; it < 200; ++it) {
    const double g = f(x) - t;
    if (g == 0.0) return x;
    if ((g < 0.0) == inc)
      lo = x;
    else
      hi = x;
    double xn = x - g / fp(x);
    if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
    if (fabs(xn - x) <= 4.0 * 2.220446049250313e-16 * fabs(xn) || !(hi > lo)) return xn;
    x = xn;
  }
  return x;
}

// foldcauchy: atan(x - c) + atan(x + c) = pi q, x >= 0, is the positive root of
// sin(th) x^2 + 2 cos(th) x - (1 + c^2) sin(th) = 0, th = pi q (sin / cos of pi q from the nearer
// end, so that they keep their relative precision as q -> 1)
__device__ __forceinline__ double foldcauchy_ppf01(double q, double c) {
  const bool up = q > 0.5;
  const double r = up ? 1.0 - q : q;  // exact for q > 1/2
  const double sn = sin(sf::kPi * r), cs = up ? -cos(sf::kPi * r) : cos(sf::kPi * r);
  const double k = 1.0 + c * c;
  const double root = sqrt(cs * cs + k * sn * sn);
  return cs > 0.0 ? k * sn / (cs + root) : (root - cs) / sn;
}

// foldnorm: scipy's _cdf (0.5 (erf((x - c) / sqrt 2) + erf((x + c) / sqrt 2))) below q = 1/2, its _sf
// (ndtr(c - x) + ndtr(-x - c)) above, the density phi(x - c) + phi(x + c)
__device__ __forceinline__ double foldnorm_ppf01(double q, double c) {
  constexpr double kRs2pi = 0.3989422804014327;  // 1 / sqrt(2 pi)
  auto pdf = [c](double x) { return kRs2pi * (exp(-0.5 * (x - c) * (x - c)) + exp(-0.5 * (x + c) * (x + c))); };
  const double hi = c + 40.0;
  const double x0 = c + fabs(sf::ndtri(0.5 + 0.5 * q));  // the c = 0 answer, shifted
  if (q <= 0.5) {
    auto cdf = [c](double x) { return 0.5 * (sf::erf_((x - c) * sfx::kSqrt1_2) + sf::erf_((x + c) * sfx::kSqrt1_2)); };
    const double xs = fmin(x0, fmax(q / (2.0 * pdf(0.0)), 0.0));
    return bracket_newton(cdf, pdf, q, 0.0, hi, xs > 0.0 ? xs : 0.5 * hi, true);
  }
  auto sfn = [c](double x) { return sfx::ndtr(c - x) + sfx::ndtr(-x - c); };
  auto dsf = [&pdf](double x) { return -pdf(x); };
  return bracket_newton(sfn, dsf, 1.0 - q, 0.0, hi, fmin(x0, 0.5 * hi), false);
}

// invgauss(mu): scipy's _logcdf / _logsf, solved in u = log x (log-concave in u): the quantile below
// q = 1/2, the complement's above (as scipy, whose lower-tail Boost quantile is inaccurate there);
// start: the log-normal with the same mean and variance
__device__ __forceinline__ double invgauss_logcdf(double x, double mu) {
  const double fac = 1.0 / sqrt(x);
  const double a = sfx::log_ndtr(fac * ((x / mu) - 1.0));
  const double b = 2.0 / mu + sfx::log_ndtr(-fac * ((x / mu) + 1.0));
  return a + log1p(exp(b - a));
}
__device__ __forceinline__ double invgauss_logsf(double x, double mu) {
  const double fac = 1.0 / sqrt(x);
  const double a = sfx::log_ndtr(-(fac * ((x / mu) - 1.0)));
  const double b = 2.0 / mu + sfx::log_ndtr(-fac * (x + mu) / mu);
  return a + log1p(-exp(b - a));
}
// the x with cdf(x) = t (upper: sf(x) = t), t <= 1/2
__device__ __forceinline__ double invgauss_solve(double mu, double t, bool upper) {
  // log(x pdf(x)) = -log(2 pi x) / 2 - (x - mu)^2 / (2 x mu^2)
  auto lxpdf = [mu](double x) { return -0.5 * log(2.0 * sf::kPi * x) - (x - mu) * (x - mu) / (2.0 * x * mu * mu); };
  const double s2 = log1p(mu), u0 = log(mu) - 0.5 * s2 + sqrt(s2) * sf::ndtri(upper ? 1.0 - t : t);
  const double lo = -744.0, hi = 709.0;
  const double us = fmin(fmax(u0, lo + 1.0), hi - 1.0);
  double u;
  if (!upper) {
    auto f = [mu](double v) { return invgauss_logcdf(exp(v), mu); };
    auto fp = [mu, &lxpdf](double v) {
      const double x = exp(v);
      return exp(lxpdf(x) - invgauss_logcdf(x, mu));
    };
    u = bracket_newton(f, fp, log(t), lo, hi, us, true);
  } else {
    auto f = [mu](double v) { return invgauss_logsf(exp(v), mu); };
    auto fp = [mu, &lxpdf](double v) {
      const double x = exp(v);
      return -exp(lxpdf(x) - invgauss_logsf(x, mu));
    };
    u = bracket_newton(f, fp, log(t), lo, hi, us, false);
  }
  return exp(u);
}
__device__ __forceinline__ double invgauss_ppf01(double q, double mu) {
  return q <= 0.5 ? invgauss_solve(mu, q, false) : invgauss_solve(mu, 1.0 - q, true);
}
// recipinvgauss(mu) is 1 / invgauss(mu): its q-quantile is 1 / invgauss's (1 - q)-quantile, solved on
// the side that keeps q exact (scipy: brentq on recipinvgauss._cdf)
__device__ __forceinline__ double recipinvgauss_ppf01(double q, double mu) {
  return 1.0 / (q <= 0.5 ? invgauss_solve(mu, q, true) : invgauss_solve(mu, 1.0 - q, false));
}

// exponnorm(K) (scipy: brentq on _cdf): cdf = Phi(x) - exp(e(x)), sf = Phi(-x) + exp(e(x)),
// e(x) = (0.5 / K - x) / K + log_ndtr(x - 1 / K), density exp(e(x)) / K
__device__ __forceinline__ double exponnorm_ppf01(double q, double K) {
  const double invK = 1.0 / K;
  auto e = [invK](double x) { return invK * (0.5 * invK - x) + sfx::log_ndtr(x - invK); };
  auto pdf = [invK, e](double x) { return exp(e(x)) * invK; };
  const double lo = -40.0, hi = 40.0 + 40.0 * K;
  const double x0 = fmin(fmax(sf::ndtri(q) + K, lo + 1.0), hi - 1.0);
  if (q <= 0.5) {
    auto cdf = [e](double x) { return sfx::ndtr(x) - exp(e(x)); };
    return bracket_newton(cdf, pdf, q, lo, hi, x0, true);
  }
  auto sfn = [e](double x) { return sfx::ndtr(-x) + exp(e(x)); };
  auto dsf = [&pdf](double x) { return -pdf(x); };
  return bracket_newton(sfn, dsf, 1.0 - q, lo, hi, x0, false);
}

// argus(chi) (scipy: brentq on _cdf = 1 - _sf): sf = Psi(chi sqrt((1 - x)(1 + x))) / Psi(chi),
// Psi(c) = gammainc(1.5, c^2 / 2) / 2, density from scipy's _logpdf
__device__ __forceinline__ double argus_ppf01(double q, double chi) {
  auto psi = [](double c) { return sf::igam(1.5, c * c / 2) / 2; };
  const double pc = psi(chi);
  const double A = 3 * log(chi) - 0.9189385332046727 - log(pc);  // _norm_pdf_logC = log(sqrt(2 pi))
  auto pdf = [chi, A](double x) { return exp(A + log(x) + 0.5 * log1p(-x * x) - chi * chi * (1.0 - x * x) / 2); };
  auto sfn = [chi, pc, psi](double x) { return psi(chi * sqrt((1 - x) * (1 + x))) / pc; };
  if (q <= 0.5) {
    auto cdf = [&sfn](double x) { return 1.0 - sfn(x); };
    return bracket_newton(cdf, pdf, q, 0.0, 1.0, 0.5, true);
  }
  auto dsf = [&pdf](double x) { return -pdf(x); };
  return bracket_newton(sfn, dsf, 1.0 - q, 0.0, 1.0, 0.5, false);
}

// kstwobign (scipy: kolmogci, the inverse of the Kolmogorov distribution's cdf): below x = 0.82 the
// cdf's theta-function form sqrt(2 pi) / x sum exp(-(2k - 1)^2 pi^2 / (8 x^2)), above it the
// complement 2 sum (-1)^(k - 1) exp(-2 k^2 x^2); the quantile on the side that keeps q exact
__device__ __forceinline__ double kolmog_cdf_small(double x) {
  double s = 0.0;
  const double w = -sf::kPi * sf::kPi / (8.0 * x * x);
  for (int k = 1; k <= 4; ++k) s += exp((2.0 * k - 1) * (2.0 * k - 1) * w);
  return 2.5066282746310002 / x * s;
}
__device__ __forceinline__ double kolmog_sf_large(double x) {
  double s = 0.0, sg = 1.0;
  for (int k = 1; k <= 10; ++k, sg = -sg) s += sg * exp(-2.0 * k * k * x * x);
  return 2.0 * s;
}
__device__ __forceinline__ double kolmog_pdf(double x) {
  if (x < 0.82) {
    const double a = sf::kPi * sf::kPi / 8.0;
    double s = 0.0;
    for (int k = 1; k <= 4; ++k) {
      const double ak = (2.0 * k - 1) * (2.0 * k - 1) * a;
      s += exp(-ak / (x * x)) * (2.0 * ak / (x * x * x * x) - 1.0 / (x * x));
    }
    return 2.5066282746310002 * s;
  }
  double s = 0.0, sg = 1.0;
  for (int k = 1; k <= 10; ++k, sg = -sg) s += sg * k * k * exp(-2.0 * k * k * x * x);
  return 8.0 * x * s;
}
__device__ __forceinline__ double kstwobign_ppf01(double q) {
  auto cdf = [](double x) { return x < 0.82 ? kolmog_cdf_small(x) : 1.0 - kolmog_sf_large(x); };
  auto sfn = [](double x) { return x < 0.82 ? 1.0 - kolmog_cdf_small(x) : kolmog_sf_large(x); };
  auto pdf = [](double x) { return kolmog_pdf(x); };
  auto dsf = [](double x) { return -kolmog_pdf(x); };
  if (q <= 0.5) return bracket_newton(cdf, pdf, q, 0.02, 10.0, 0.8, true);
  return bracket_newton(sfn, dsf, 1.0 - q, 0.02, 10.0, 1.0, false);
}

// cosine: cdf(x) = (pi + x + sin x) / (2 pi), symmetric about 0.  Central q: x + sin x = pi (2 q - 1)
// (exact argument for q in [1/4, 3/4]); tails: y = x + pi for min(q, 1 - q), y - sin y = 2 pi q,
// with its series below y = 1/2 (no cancellation)
__device__ __forceinline__ double cosine_tail_h(double y) {  // y - sin y
  if (y >= 0.5) return y - sin(y);
  const double y2 = y * y;
  double t = y * y2 / 6.0, s = t;
  for (int k = 2; k <= 10; ++k) {
    t *= -y2 / ((2.0 * k) * (2.0 * k + 1.0));
    s += t;
  }
  return s;
}
__device__ __forceinline__ double cosine_ppf01(double q) {
  if (q >= 0.25 && q <= 0.75) {
    const double t = sf::kPi * (2.0 * q - 1.0);
    auto f = [](double x) { return x + sin(x); };
    auto fp = [](double x) { return 1.0 + cos(x); };
    return bracket_newton(f, fp, t, -sf::kPi, sf::kPi, 0.5 * t, true);
  }
  const bool up = q > 0.5;
  const double p = up ? 1.0 - q : q;  // exact for q > 1/2
  auto h = [](double y) { return cosine_tail_h(y); };
  auto hp = [](double y) {
    const double s = sin(0.5 * y);
    return 2.0 * s * s;  // 1 - cos y
  };
  const double y0 = fmin(cbrt(12.0 * sf::kPi * p), sf::kPi);
  const double y = bracket_newton(h, hp, 2.0 * sf::kPi * p, 0.0, sf::kPi, y0, true);
  return up ? sf::kPi - y : y - sf::kPi;
}

// skewnorm(a): scipy's ppf is Boost's skew_normal quantile, Newton on cdf(x) = Phi(x) - 2 T(x, a)
// (T: Owen's function).  Solved here the same way, the complement sf(x) = Phi(-x) + 2 T(x, a) above
// q = 1/2.  Boost's own cdf loses its relative precision in the left tail for a > 0 (scipy's _cdf
// says so and patches it; its _ppf does not), so the two agree to 1e-10 for q in [1e-6, 1 - 1e-6].
// Owen's T(h, a) = (1 / 2 pi) int_0^a exp(-h^2 (1 + x^2) / 2) / (1 + x^2) dx for 0 <= a <= 1 by
// 20-point Gauss-Legendre (the integrand's poles at +-i lie a unit from [0, 1]: ~1e-18 for the h
// where the cdf needs T to full precision), and beyond by Owen's identity
// T(h, a) = (Phi(h) Q(ah) + Phi(ah) Q(h)) / 2 - T(ah, 1 / a), h >= 0 (Q = 1 - Phi, no cancellation).
__device__ __forceinline__ double owens_t01(double h, double a) {
  const double T[10] = {0.07652652113349734, 0.2277858511416451, 0.37370608871541955, 0.5108670019508271,
                        0.636053680726515,   0.7463319064601508, 0.8391169718222188,  0.9122344282513258,
                        0.9639719272779138,  0.9931285991850949};
  const double W[10] = {0.15275338713072578, 0.14917298647260366, 0.14209610931838187, 0.13168863844917653,
                        0.11819453196151825, 0.10193011981724026, 0.08327674157670467, 0.06267204833410944,
                        0.04060142980038622, 0.017614007139153273};
  const double hh = -0.5 * h * h;
  double acc = 0.0;
  for (int i = 0; i < 10; ++i) {
    const double xp = 0.5 * a * (1.0 + T[i]), xm = 0.5 * a * (1.0 - T[i]);
    const double up = 1.0 + xp * xp, um = 1.0 + xm * xm;
    acc += W[i] * (exp(hh * up) / up + exp(hh * um) / um);
  }
  return acc * (0.25 * a / sf::kPi);
}
__device__ __forceinline__ double owens_t(double h, double a) {
  const double sg = a < 0.0 ? -1.0 : 1.0;  // T(h, -a) = -T(h, a), T(-h, a) = T(h, a)
  a = fabs(a);
  h = fabs(h);
  if (a <= 1.0) return sg * owens_t01(h, a);
  const double ah = a * h;
  const double v = 0.5 * (sfx::ndtr(h) * sfx::ndtr(-ah) + sfx::ndtr(ah) * sfx::ndtr(-h)) - owens_t01(ah, 1.0 / a);
  return sg * v;
}
__device__ __forceinline__ double skewnorm_ppf01(double q, double a) {
  constexpr double kRs2pi = 0.3989422804014327;  // 1 / sqrt(2 pi)
  auto pdf = [a](double x) { return 2.0 * kRs2pi * exp(-0.5 * x * x) * sfx::ndtr(a * x); };
  const double x0 = fmin(fmax(sf::ndtri(q) + a / sqrt(1.0 + a * a) * 0.7978845608028654, -39.0), 39.0);
  if (q <= 0.5) {
    auto cdf = [a](double x) { return sfx::ndtr(x) - 2.0 * owens_t(x, a); };
    return bracket_newton(cdf, pdf, q, -40.0, 40.0, x0, true);
  }
  auto sfn = [a](double x) { return sfx::ndtr(-x) + 2.0 * owens_t(x, a); };
  auto dsf = [&pdf](double x) { return -pdf(x); };
  return bracket_newton(sfn, dsf, 1.0 - q, -40.0, 40.0, x0, false);
}

// rel_breitwigner(rho) (scipy: brentq on _cdf): scipy's complex form of the cdf,
// min(2 C Im(sqrt(-1 + i / rho) atan(x / sqrt(-rho (rho + i)))), 1), C = sqrt(2 / (1 + sqrt(1 +
// 1 / rho^2))) / pi, in real arithmetic with the principal branches (sqrt by halves, atan(z) =
// -(i / 2) (log(1 + i z) - log(1 - i z)) away from its cuts: z lies in the first quadrant here);
// density C' / (((x - rho)(x + rho) / rho)^2 + 1)
__device__ __forceinline__ void csqrt_(double re, double im, double* ore, double* oim) {
  const double r = hypot(re, im);
  if (re >= 0.0) {
    const double t = sqrt((r + re) / 2);
    *ore = t;
    *oim = t != 0.0 ? im / (2 * t) : 0.0;
  } else {
    const double t = sqrt((r - re) / 2);
    *ore = fabs(im) / (2 * t);
    *oim = copysign(t, im);
  }
}
__device__ __forceinline__ double rel_breitwigner_cdf(double x, double rho) {
  const double C = sqrt(2 / (1 + sqrt(1 + 1 / (rho * rho)))) / sf::kPi;
  double s1r, s1i, wr, wi;
  csqrt_(-1.0, 1 / rho, &s1r, &s1i);
  csqrt_(-rho * rho, -rho, &wr, &wi);
  const double den = wr * wr + wi * wi;
  const double zr = x * wr / den, zi = -x * wi / den;  // x / w
  const double l1r = log(hypot(1 - zi, zr)), l1i = atan2(zr, 1 - zi);    // log(1 + i z)
  const double l2r = log(hypot(1 + zi, -zr)), l2i = atan2(-zr, 1 + zi);  // log(1 - i z)
  const double ar = (l1i - l2i) / 2, ai = -(l1r - l2r) / 2;             // atan(z)
  return fmin(C * 2 * (s1r * ai + s1i * ar), 1.0);
}
__device__ __forceinline__ double rel_breitwigner_ppf01(double q, double rho) {
  const double C2 = sqrt(2 * (1 + 1 / (rho * rho)) / (1 + sqrt(1 + 1 / (rho * rho)))) * 2 / sf::kPi;
  auto pdf = [rho, C2](double x) {
    const double u = (x - rho) * (x + rho) / rho;
    return C2 / (u * u + 1);
  };
  auto cdf = [rho](double x) { return rel_breitwigner_cdf(x, rho); };
  return bracket_newton(cdf, pdf, q, 0.0, 1e12, rho, true);
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
  if constexpr (D == PBH_DIST_HALFCAUCHY || D == PBH_DIST_HALFLOGISTIC || D == PBH_DIST_HALFNORM ||
                D == PBH_DIST_POWERLAW || D == PBH_DIST_GENPARETO || D == PBH_DIST_FISK || D == PBH_DIST_BURR ||
                D == PBH_DIST_BURR12 || D == PBH_DIST_EXPONWEIB || D == PBH_DIST_EXPONPOW ||
                D == PBH_DIST_BRADFORD || D == PBH_DIST_LEVY || D == PBH_DIST_GIBRAT || D == PBH_DIST_INVWEIBULL ||
                D == PBH_DIST_LOGLAPLACE || D == PBH_DIST_TRUNCEXPON || D == PBH_DIST_CHI ||
                D == PBH_DIST_MAXWELL || D == PBH_DIST_NAKAGAMI || D == PBH_DIST_KAPPA3 ||
                D == PBH_DIST_GENHALFLOGISTIC || D == PBH_DIST_ALPHA || D == PBH_DIST_FATIGUELIFE ||
                D == PBH_DIST_ARCSINE || D == PBH_DIST_TRAPEZOID || D == PBH_DIST_INVGAMMA)
    lo = 0.0;
  if constexpr (D == PBH_DIST_ARCSINE || D == PBH_DIST_POWERLAW || D == PBH_DIST_BRADFORD ||
                D == PBH_DIST_TRAPEZOID)
    hi = 1.0;
  if constexpr (D == PBH_DIST_LEVY_L) hi = 0.0;
  if constexpr (D == PBH_DIST_ANGLIT) {
    lo = -sf::kPi / 4;
    hi = sf::kPi / 4;
  }
  if constexpr (D == PBH_DIST_GENPARETO) {  // _argcheck isfinite(c); support [0, -1 / c) for c < 0
    if (s0 < 0.0) hi = -1.0 / s0;
    return isfinite(s0);
  }
  if constexpr (D == PBH_DIST_TRUNCEXPON) hi = s0;  // support [0, b]
  if constexpr (D == PBH_DIST_GENHALFLOGISTIC) hi = 1.0 / s0;  // support [0, 1 / c]
  if constexpr (D == PBH_DIST_TRAPEZOID) return s0 >= 0.0 && s0 <= 1.0 && s1 >= 0.0 && s1 <= 1.0 && s1 >= s0;
  // round 6
  if constexpr (D == PBH_DIST_JOHNSONSU || D == PBH_DIST_JOHNSONSB) {  // _argcheck (b > 0) & (a == a)
    if constexpr (D == PBH_DIST_JOHNSONSB) {
      lo = 0.0;
      hi = 1.0;
    }
    return s1 > 0.0 && s0 == s0;
  }
  if constexpr (D == PBH_DIST_MIELKE || D == PBH_DIST_F || D == PBH_DIST_BETAPRIME) lo = 0.0;
  if constexpr (D == PBH_DIST_TRUNCPARETO) {  // _argcheck (b > 0) & (c > 1), support [1, c]
    lo = 1.0;
    hi = s1;
    return s0 > 0.0 && s1 > 1.0;
  }
  if constexpr (D == PBH_DIST_TUKEYLAMBDA) {  // _argcheck isfinite(lam); support +-1 / lam for lam > 0
    if (s0 > 0.0) {
      lo = -1.0 / s0;
      hi = 1.0 / s0;
    }
    return isfinite(s0);
  }
  if constexpr (D == PBH_DIST_GENGAMMA) {  // _argcheck (a > 0) & (c != 0), support [0, inf)
    lo = 0.0;
    return s0 > 0.0 && s1 != 0.0;
  }
  if constexpr (D == PBH_DIST_RDIST || D == PBH_DIST_SEMICIRCULAR) {
    lo = -1.0;
    hi = 1.0;
  }
  // round 6, second set
  if constexpr (D == PBH_DIST_PEARSON3) return isfinite(s0);  // _argcheck isfinite(skew)
  if constexpr (D == PBH_DIST_HALFGENNORM) lo = 0.0;
  if constexpr (D == PBH_DIST_WRAPCAUCHY) {  // support [0, 2 pi], _argcheck 0 < c < 1
    lo = 0.0;
    hi = 2.0 * sf::kPi;
    return s0 > 0.0 && s0 < 1.0;
  }
  if constexpr (D == PBH_DIST_SKEWCAUCHY) return fabs(s0) < 1.0;
  if constexpr (D == PBH_DIST_KAPPA4) {  // _argcheck always true; kappa4._get_support's six cases
    const double h = s0, k = s1;
    if (h > 0.0) {
      lo = k == 0.0 ? log(h) : (1.0 - pow(h, -k)) / k;  // np.float_power(h, -k)
      hi = k > 0.0 ? 1.0 / k : inf;
    } else if (h <= 0.0) {
      lo = k < 0.0 ? 1.0 / k : -inf;
      hi = k > 0.0 ? 1.0 / k : inf;
    } else {  // NaN h: no case applies
      lo = hi = sf::kNaN;
    }
    if (k != k) lo = hi = sf::kNaN;
    return true;
  }
  if constexpr (D == PBH_DIST_CRYSTALBALL) return s1 > 1.0 && s0 > 0.0;  // (m > 1) & (beta > 0)
  // round 6, third set
  if constexpr (D == PBH_DIST_POWERLOGNORM || D == PBH_DIST_INVGAUSS || D == PBH_DIST_WALD) lo = 0.0;
  if constexpr (D == PBH_DIST_FOLDCAUCHY || D == PBH_DIST_FOLDNORM) {  // _argcheck c >= 0, support [0, inf)
    lo = 0.0;
    return s0 >= 0.0;
  }
  if constexpr (D == PBH_DIST_SKEWNORM) return isfinite(s0);  // _argcheck isfinite(a)
  if constexpr (D == PBH_DIST_RECIPINVGAUSS || D == PBH_DIST_KSTWOBIGN || D == PBH_DIST_REL_BREITWIGNER) lo = 0.0;
  if constexpr (D == PBH_DIST_ARGUS) {
    lo = 0.0;
    hi = 1.0;
  }
  if constexpr (D == PBH_DIST_COSINE) {
    lo = -sf::kPi;
    hi = sf::kPi;
  }
  if constexpr (closed_shapes(D) == 1) return s0 > 0.0;
  if constexpr (closed_shapes(D) == 2) return s0 > 0.0 && s1 > 0.0;
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
  // round 4 (scipy 1.15 _continuous_distns.py _ppf bodies, operation for operation)
  if constexpr (D == PBH_DIST_HALFCAUCHY) return tan(sf::kPi / 2 * q);
  if constexpr (D == PBH_DIST_HALFLOGISTIC) return 2 * atanh(q);
  if constexpr (D == PBH_DIST_HALFNORM) return sf::ndtri((1 + q) / 2.0);
  if constexpr (D == PBH_DIST_ARCSINE) {
    const double v = sin(sf::kPi / 2.0 * q);
    return v * v;  // ** 2.0: numpy's square
  }
  if constexpr (D == PBH_DIST_HYPSECANT) return log(tan(sf::kPi * q / 2.0));
  if constexpr (D == PBH_DIST_POWERLAW) return pow(q, 1.0 / s0);
  if constexpr (D == PBH_DIST_GENPARETO) return -boxcox1p(-q, -s0);
  if constexpr (D == PBH_DIST_FISK) return pow(1.0 / q - 1, -1.0 / s0);  // q ** -1.0: numpy's reciprocal
  if constexpr (D == PBH_DIST_BURR) return pow(pow(q, -1.0 / s1) - 1, -1.0 / s0);
  if constexpr (D == PBH_DIST_BURR12) return pow(expm1(-1 / s1 * log1p(-q)), 1 / s0);
  if constexpr (D == PBH_DIST_EXPONWEIB) return pow(-log1p(-pow(q, 1.0 / s0)), 1.0 / s1);
  if constexpr (D == PBH_DIST_EXPONPOW) return pow(log1p(-log1p(-q)), 1.0 / s0);
  if constexpr (D == PBH_DIST_BRADFORD) return expm1(q * log1p(s0)) / s0;
  if constexpr (D == PBH_DIST_ANGLIT) return asin(sqrt(q)) - sf::kPi / 4;
  if constexpr (D == PBH_DIST_LEVY) {
    const double v = -sf::ndtri(q / 2);  // _norm_isf(q / 2)
    return 1.0 / (v * v);
  }
  if constexpr (D == PBH_DIST_LEVY_L) {
    const double v = sf::ndtri((q + 1.0) / 2);
    return -1.0 / (v * v);
  }
  if constexpr (D == PBH_DIST_GIBRAT) return exp(sf::ndtri(q));
  if constexpr (D == PBH_DIST_INVWEIBULL) return pow(-log(q), -1.0 / s0);
  if constexpr (D == PBH_DIST_LOGLAPLACE) return q < 0.5 ? pow(2.0 * q, 1.0 / s0) : pow(2 * (1.0 - q), -1.0 / s0);
  if constexpr (D == PBH_DIST_TRUNCEXPON) return -log1p(q * expm1(-s0));
  if constexpr (D == PBH_DIST_CHI) return sqrt(2 * sf::igami(.5 * s0, q));
  if constexpr (D == PBH_DIST_MAXWELL) return sqrt(2 * sf::igami(1.5, q));
  if constexpr (D == PBH_DIST_NAKAGAMI) return sqrt(1.0 / s0 * sf::igami(s0, q));
  if constexpr (D == PBH_DIST_DWEIBULL) {
    double fac = 2. * (q <= 0.5 ? q : 1. - q);
    fac = pow(-log(fac), 1.0 / s0);
    return q > 0.5 ? fac : -fac;
  }
  if constexpr (D == PBH_DIST_KAPPA3) return pow(s0 / (pow(q, -s0) - 1.0), 1.0 / s0);
  if constexpr (D == PBH_DIST_GENHALFLOGISTIC) return 1.0 / s0 * (1 - pow((1.0 - q) / (1.0 + q), s0));
  if constexpr (D == PBH_DIST_ALPHA) return 1.0 / (s0 - sf::ndtri(q * sf::ndtr(s0)));
  if constexpr (D == PBH_DIST_FATIGUELIFE) {
    const double t = s0 * sf::ndtri(q);
    const double u = t + sqrt(t * t + 4);
    return 0.25 * (u * u);
  }
  if constexpr (D == PBH_DIST_GENLOGISTIC) return -log(powm1(q, -1.0 / s0));
  // round 5
  if constexpr (D == PBH_DIST_INVGAMMA) return 1.0 / sf::igamci(s0, q);  // invgamma._ppf
  if constexpr (D == PBH_DIST_T) return sfx::t_ppf01(q, s0);  // t._ppf = stdtrit (cdflib, ~2.5e-11)
  if constexpr (D == PBH_DIST_TRAPEZOID) {
    const double c = s0, d = s1;
    const double qc = trapezoid_mid_cdf(c, c, d), qd = trapezoid_mid_cdf(d, c, d);
    if (q < qc) return sqrt(q * c * (1 + d - c));
    if (q <= qd) return 0.5 * q * (1 + d - c) + 0.5 * c;
    return 1 - sqrt((1 - q) * (d - c + 1) * (1 - d));
  }
  // round 6 (scipy 1.15 _continuous_distns.py _ppf bodies, operation for operation)
  if constexpr (D == PBH_DIST_JOHNSONSU) return sinh((sf::ndtri(q) - s0) / s1);
  if constexpr (D == PBH_DIST_JOHNSONSB) return expit(1.0 / s1 * (sf::ndtri(q) - s0));
  if constexpr (D == PBH_DIST_POWERNORM) return -sf::ndtri(pow(1.0 - q, 1.0 / s0));
  if constexpr (D == PBH_DIST_LAPLACE_ASYMMETRIC) {
    const double kapinv = 1 / s0, kappkapinv = s0 + kapinv;
    return q >= s0 / kappkapinv ? -log((1 - q) * kappkapinv * s0) * kapinv : log(q * kappkapinv / s0) * s0;
  }
  if constexpr (D == PBH_DIST_MIELKE) {
    const double qsk = pow(q, s1 * 1.0 / s0);
    return pow(qsk / (1.0 - qsk), 1.0 / s1);
  }
  if constexpr (D == PBH_DIST_TRUNCPARETO) return pow(1 - (1 - 1 / pow(s1, s0)) * q, -1 / s0);
  if constexpr (D == PBH_DIST_TUKEYLAMBDA) return boxcox(q, s0) - boxcox1p(-q, s0);
  if constexpr (D == PBH_DIST_GENGAMMA) return pow(s1 > 0.0 ? sf::igami(s0, q) : sf::igamci(s0, q), 1.0 / s1);
  if constexpr (D == PBH_DIST_LOGGAMMA) {
    const double g = sf::igami(s0, q);
    return g < 2.2250738585072014e-308 ? (log(q) + sf::lgam(s0 + 1)) / s0 : log(g);  // _XMIN = finfo.tiny
  }
  if constexpr (D == PBH_DIST_DGAMMA) return q > 0.5 ? sf::igami(s0, 2 * q - 1) : -sf::igamci(s0, 2 * q);
  if constexpr (D == PBH_DIST_F) {
    // scipy's fdtri (Cephes fdtr.c) step for step: y = 1 - q first (so q below ~1e-16 reads as 0,
    // and scipy returns 0 there), then the inverse on the side of I_0.5(dfd / 2, dfn / 2) that
    // avoids the cancellation in dfd - dfd w
    const double a = s0, b = s1;
    const double y = 1.0 - q;
    const double w0 = sfx::incbet(0.5 * b, 0.5 * a, 0.5);
    if (w0 > y || y < 0.001) {
      const double w = sfx::beta_ppf01(y, 0.5 * b, 0.5 * a);
      return (b - b * w) / (a * w);
    }
    const double w = sfx::beta_ppf01(1.0 - y, 0.5 * a, 0.5 * b);
    return b * w / (a * (1.0 - w));
  }
  if constexpr (D == PBH_DIST_RDIST) return 2 * sfx::beta_ppf01(q, s0 / 2, s0 / 2) - 1;
  if constexpr (D == PBH_DIST_SEMICIRCULAR) return 2 * sfx::beta_ppf01(q, 1.5, 1.5) - 1;  // rdist._ppf(q, 3)
  if constexpr (D == PBH_DIST_BETAPRIME) {  // r / (1 - r); 1 / beta._isf(p, b, a) - 1 for r > 0.9999
    const double r = sfx::beta_ppf01(q, s0, s1);
    if (r > 0.9999) return 1 / sfx::beta_ppf01(1.0 - q, s1, s0) - 1;
    return r / (1 - r);
  }
  // round 6, second set
  if constexpr (D == PBH_DIST_PEARSON3) {  // pearson3._preprocess / _ppf (loc 0, scale 1 inside)
    if (fabs(s0) < 0.000016) return sf::ndtri(q);  // norm2pearson_transition
    const double beta = 2.0 / (s0 * 1.0), alpha = (1.0 * beta) * (1.0 * beta), zeta = 0.0 - alpha / beta;
    const double qq = beta < 0.0 ? 1.0 - q : q;  // negative skew: gh-17050
    return sf::igami(alpha, qq) / beta + zeta;
  }
  if constexpr (D == PBH_DIST_GENNORM) {
    const double c = q > 0.5 ? 1.0 : (q < 0.5 ? -1.0 : 0.0);  // np.sign(x - 0.5)
    return c * pow(sf::igamci(1.0 / s0, (1.0 + c) - 2.0 * c * q), 1.0 / s0);
  }
  if constexpr (D == PBH_DIST_HALFGENNORM) return pow(sf::igami(1.0 / s0, q), 1.0 / s0);
  if constexpr (D == PBH_DIST_WRAPCAUCHY) {
    const double val = (1.0 - s0) / (1.0 + s0);
    if (q < 1.0 / 2) return 2 * atan(val * tan(sf::kPi * q));
    return 2 * sf::kPi - 2 * atan(val * tan(sf::kPi * (1 - q)));
  }
  if constexpr (D == PBH_DIST_SKEWCAUCHY) {  // i = x < _cdf(0, a) = (1 - a) / 2
    const double a = s0;
    if (q < (1 - a) / 2) return tan(sf::kPi / (1 - a) * (q - (1 - a) / 2)) * (1 - a);
    return tan(sf::kPi / (1 + a) * (q - (1 - a) / 2)) * (1 + a);
  }
  if constexpr (D == PBH_DIST_MOYAL) {  // scipy's erfcinv(y) = -ndtri(0.5 y) / sqrt(2) (cephes erfinv.c)
    const double e = -sf::ndtri(0.5 * q) * 0.7071067811865476;
    return -log(2 * (e * e));
  }
  if constexpr (D == PBH_DIST_KAPPA4) {
    const double h = s0, k = s1;
    if (h != 0.0 && k != 0.0) return 1.0 / k * (1.0 - pow((1.0 - pow(q, h)) / h, k));
    if (h == 0.0 && k != 0.0) return 1.0 / k * (1.0 - pow(-log(q), k));
    if (h != 0.0 && k == 0.0) return -log1p(-pow(q, h)) + log(h);
    if (h == 0.0 && k == 0.0) return -log(-log(q));
    return sf::kNaN;  // _lazyselect's default (a NaN shape)
  }
  if constexpr (D == PBH_DIST_CRYSTALBALL) {
    const double beta = s0, m = s1;
    constexpr double kNormPdfC = 2.5066282746310002;  // np.sqrt(2 * np.pi)
    // above pbeta the quantile is ndtri(ndtr(-beta) + (p / N - C) / sqrt(2 pi)), whose argument nears 1
    // as q does: there an ulp of exp(-beta^2 / 2) (numpy's own SIMD exp in scipy) moves x by ~1e-6
    const double eb = exp(-beta * beta / 2.0);
    const double Phi = sf::ndtr(beta);
    const double N0 = 1.0 / (m / beta / (m - 1) * eb + kNormPdfC * Phi);
    const double pbeta = N0 * (m / beta) * eb / (m - 1);
    const double C = (m / beta) * eb / (m - 1);
    const double N = 1 / (C + kNormPdfC * Phi);
    if (q < pbeta) return m / beta - beta - pow((m - 1) * pow(m / beta, -m) / eb * q / N, 1 / (1 - m));
    return sf::ndtri(sf::ndtr(-beta) + (1 / kNormPdfC) * (q / N - C));
  }
  // round 6, third set
  if constexpr (D == PBH_DIST_POWERLOGNORM) return exp(-sf::ndtri(pow(1.0 - q, 1 / s0)) * s1);  // _isf(1 - q)
  if constexpr (D == PBH_DIST_JF_SKEW_T) {
    const double d1 = sfx::beta_ppf01(q, s0, s1);
    const double d2 = (2 * d1 - 1) * sqrt(s0 + s1);
    const double d3 = 2 * sqrt(d1 * (1 - d1));
    return d2 / d3;
  }
  if constexpr (D == PBH_DIST_FOLDCAUCHY) return foldcauchy_ppf01(q, s0);
  if constexpr (D == PBH_DIST_FOLDNORM) return foldnorm_ppf01(q, s0);
  if constexpr (D == PBH_DIST_COSINE) return cosine_ppf01(q);
  if constexpr (D == PBH_DIST_INVGAUSS) return invgauss_ppf01(q, s0);
  if constexpr (D == PBH_DIST_WALD) return invgauss_ppf01(q, 1.0);
  if constexpr (D == PBH_DIST_SKEWNORM) return skewnorm_ppf01(q, s0);
  if constexpr (D == PBH_DIST_RECIPINVGAUSS) return recipinvgauss_ppf01(q, s0);
  if constexpr (D == PBH_DIST_EXPONNORM) return exponnorm_ppf01(q, s0);
  if constexpr (D == PBH_DIST_ARGUS) return argus_ppf01(q, s0);
  if constexpr (D == PBH_DIST_KSTWOBIGN) return kstwobign_ppf01(q);
  if constexpr (D == PBH_DIST_REL_BREITWIGNER) return rel_breitwigner_ppf01(q, s0);
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
    if (p.dt) {  // scalar (n, p): the CDF tables
      const double k = discrete_from_table(q, p.dt, p.dlen);
      if (k >= 0.0) return k + loc;
    }
    return sfx::binom_ppf01(q, n, pp) + loc;
  } else if constexpr (is_discrete2(D)) {
    // rv_discrete.ppf: q == 0 -> _a - 1 + loc whatever the arguments, q == 1 -> _b + loc for valid
    // ones, NaN otherwise; _a = 1 (geom), low (randint), 0 (nbinom)
    if constexpr (D == PBH_DIST_GEOM) {
      const double pp = p.at(0, i), loc = p.at(1, i);
      if (q == 0.0) return 0.0 + loc;
      if (!(pp > 0.0 && pp <= 1.0 && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return inf + loc;
      return sfx::geom_ppf01(q, pp) + loc;
    } else if constexpr (D == PBH_DIST_RANDINT) {
      const double low = p.at(0, i), high = p.at(1, i), loc = p.at(2, i);
      if (q == 0.0) return low - 1.0 + loc;
      // _argcheck: high > low, both integral (x == np.round(x))
      if (!(high > low && low == rint(low) && high == rint(high) && loc == loc) || !(q >= 0.0 && q <= 1.0))
        return nan;
      if (q == 1.0) return high - 1.0 + loc;
      return sfx::randint_ppf01(q, low, high) + loc;
    } else if constexpr (D == PBH_DIST_DLAPLACE) {  // support (-inf, inf), _argcheck a > 0
      const double a = p.at(0, i), loc = p.at(1, i);
      if (q == 0.0) return -sf::kInf + loc;
      if (!(a > 0.0 && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return inf + loc;
      return sfx::dlaplace_ppf01(q, a) + loc;
    } else if constexpr (D == PBH_DIST_PLANCK) {  // support [0, inf), _argcheck lambda > 0
      const double lam = p.at(0, i), loc = p.at(1, i);
      if (q == 0.0) return -1.0 + loc;
      if (!(lam > 0.0 && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return inf + loc;
      return sfx::planck_ppf01(q, lam) + loc;
    } else if constexpr (D == PBH_DIST_BOLTZMANN) {  // support [0, N - 1], _argcheck lambda > 0, N > 0 integral
      const double lam = p.at(0, i), N = p.at(1, i), loc = p.at(2, i);
      if (q == 0.0) return -1.0 + loc;
      if (!(lam > 0.0 && N > 0.0 && N == floor(N) && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return N - 1.0 + loc;
      return sfx::boltzmann_ppf01(q, lam, N) + loc;
    } else if constexpr (D == PBH_DIST_ZIPFIAN) {  // support [1, n], _argcheck a >= 0, n > 0 integral
      const double a = p.at(0, i), nn = p.at(1, i), loc = p.at(2, i);
      if (q == 0.0) return 0.0 + loc;
      if (!(a >= 0.0 && nn > 0.0 && nn == floor(nn) && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return nn + loc;
      return zipfian_ppf01(q, a, nn) + loc;
    } else if constexpr (D == PBH_DIST_YULESIMON) {  // support [1, inf), _argcheck alpha > 0
      const double a = p.at(0, i), loc = p.at(1, i);
      if (q == 0.0) return 0.0 + loc;
      if (!(a > 0.0 && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return inf + loc;
      return yulesimon_ppf01(q, a) + loc;
    } else if constexpr (D == PBH_DIST_BETABINOM || D == PBH_DIST_HYPERGEOM || D == PBH_DIST_NHYPERGEOM) {
      const double s0 = p.at(0, i), s1 = p.at(1, i), s2 = p.at(2, i), loc = p.at(3, i);
      double lo, hi;
      const bool ok = sum_bounds(D, s0, s1, s2, &lo, &hi) && loc == loc;
      if (q == 0.0) return lo - 1.0 + loc;
      if (!ok || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return hi + loc;
      if (p.dt) {
        const double k = discrete_from_table(q, p.dt, p.dlen);
        if (k >= 0.0) return lo + k + loc;
      }
      return sum_ppf01<D>(q, s0, s1, s2, lo, hi) + loc;
    } else {  // nbinom
      const double n = p.at(0, i), pp = p.at(1, i), loc = p.at(2, i);
      if (q == 0.0) return -1.0 + loc;
      if (!(n > 0.0 && pp > 0.0 && pp <= 1.0 && loc == loc) || !(q >= 0.0 && q <= 1.0)) return nan;
      if (q == 1.0) return inf + loc;
      if (p.dt) {
        const double k = discrete_from_table(q, p.dt, p.dlen);
        if (k >= 0.0) return k + loc;
      }
      return sfx::nbinom_ppf01(q, n, pp) + loc;
    }
  } else if constexpr (is_closed(D)) {
    constexpr int S = closed_shapes(D);
    const double s0 = S > 0 ? p.at(0, i) : 0.0, s1 = S > 1 ? p.at(1, i) : 0.0;
    const double loc = p.at(S, i), scale = p.at(S + 1, i);
    double lo, hi;
    const bool ok = closed_support<D>(s0, s1, lo, hi) && scale > 0.0 && loc == loc;
    if (!ok || !(q >= 0.0 && q <= 1.0)) return nan;
    if (q == 0.0) return lo * scale + loc;
    if (q == 1.0) return hi * scale + loc;
    if constexpr (D == PBH_DIST_INVGAMMA) {
      if (p.gg.y) return 1.0 / sf::igamci_guided(s0, q, &p.ga, p.gg) * scale + loc;  // 1 / gammainccinv
    }
    if constexpr (D == PBH_DIST_T) {
      if (p.bg.z) return sfx::t_ppf_guided(q, s0, p.bg) * scale + loc;
    }
    if constexpr (is_gamma_family(D)) {
      if (p.gg.y) {  // gammaincinv through the guide (igami_guided: within ~1e-12 of igami)
        // the fallbacks behind a call (COLD): inline, with a runtime shape they cost registers
        // and occupancy: chi / nakagami / chi2 0.24 -> 0.14 ms per 1e7 (maxwell, whose shape
        // is a constant, was already 0.14; profiles/r05/ext_cold_ab_r5zh/)
        const double g = sf::igami_guided<true>(D == PBH_DIST_MAXWELL ? 1.5 : D == PBH_DIST_NAKAGAMI ? s0 : .5 * s0, q,
                                                &p.ga, p.gg);
        double x;
        if constexpr (D == PBH_DIST_CHI2)
          x = 2.0 * g;
        else if constexpr (D == PBH_DIST_NAKAGAMI)
          x = sqrt(1.0 / s0 * g);
        else
          x = sqrt(2 * g);
        return x * scale + loc;
      }
    }
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
      x = p.bg.z ? sfx::beta_ppf_guided(q, a, b, p.bg) : sfx::beta_ppf01(q, a, b);
    else
      x = p.tn_ok ? sfx::truncnorm_ppf01_c(q, a, p.tn[0], p.tn[1]) : sfx::truncnorm_ppf01(q, a, b);
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

// binom / bernoulli / nbinom with scalar parameters: a CDF table of at most kExtLdsTab entries
// (and its complement) is staged in LDS, so the binary search reads LDS instead of a cached
// global line per step
constexpr int kExtLdsTab = 512;
template <int D>
constexpr bool ext_table_discrete() {
  return D == PBH_DIST_BINOM || D == PBH_DIST_BERNOULLI || D == PBH_DIST_NBINOM || D == PBH_DIST_BETABINOM ||
         D == PBH_DIST_HYPERGEOM || D == PBH_DIST_NHYPERGEOM;
}

template <int D, bool LHS>
__global__ __launch_bounds__(256) void k_ppf_ext(const double* __restrict__ q, int64_t q_stride, LhsCol lc, int64_t n,
                                                 Params4 prm, double* __restrict__ out, int32_t* flag) {
  if constexpr (ext_table_discrete<D>()) {
    __shared__ double tab[2 * kExtLdsTab];
    if (prm.dt && prm.dlen <= kExtLdsTab) {  // block-uniform
      for (int k = threadIdx.x; k < 2 * prm.dlen; k += 256) tab[k] = prm.dt[k];
      __syncthreads();
      prm.dt = tab;
    }
  }
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
    PBH_EXT(PBH_DIST_HALFCAUCHY)
    PBH_EXT(PBH_DIST_HALFLOGISTIC)
    PBH_EXT(PBH_DIST_HALFNORM)
    PBH_EXT(PBH_DIST_ARCSINE)
    PBH_EXT(PBH_DIST_HYPSECANT)
    PBH_EXT(PBH_DIST_POWERLAW)
    PBH_EXT(PBH_DIST_GENPARETO)
    PBH_EXT(PBH_DIST_FISK)
    PBH_EXT(PBH_DIST_BURR)
    PBH_EXT(PBH_DIST_BURR12)
    PBH_EXT(PBH_DIST_EXPONWEIB)
    PBH_EXT(PBH_DIST_EXPONPOW)
    PBH_EXT(PBH_DIST_BRADFORD)
    PBH_EXT(PBH_DIST_ANGLIT)
    PBH_EXT(PBH_DIST_LEVY)
    PBH_EXT(PBH_DIST_LEVY_L)
    PBH_EXT(PBH_DIST_GIBRAT)
    PBH_EXT(PBH_DIST_INVWEIBULL)
    PBH_EXT(PBH_DIST_LOGLAPLACE)
    PBH_EXT(PBH_DIST_TRUNCEXPON)
    PBH_EXT(PBH_DIST_CHI)
    PBH_EXT(PBH_DIST_MAXWELL)
    PBH_EXT(PBH_DIST_NAKAGAMI)
    PBH_EXT(PBH_DIST_DWEIBULL)
    PBH_EXT(PBH_DIST_KAPPA3)
    PBH_EXT(PBH_DIST_GENHALFLOGISTIC)
    PBH_EXT(PBH_DIST_ALPHA)
    PBH_EXT(PBH_DIST_FATIGUELIFE)
    PBH_EXT(PBH_DIST_GENLOGISTIC)
    PBH_EXT(PBH_DIST_TRAPEZOID)
    PBH_EXT(PBH_DIST_GEOM)
    PBH_EXT(PBH_DIST_RANDINT)
    PBH_EXT(PBH_DIST_NBINOM)
    PBH_EXT(PBH_DIST_INVGAMMA)
    PBH_EXT(PBH_DIST_T)
    PBH_EXT(PBH_DIST_JOHNSONSU)
    PBH_EXT(PBH_DIST_JOHNSONSB)
    PBH_EXT(PBH_DIST_POWERNORM)
    PBH_EXT(PBH_DIST_LAPLACE_ASYMMETRIC)
    PBH_EXT(PBH_DIST_MIELKE)
    PBH_EXT(PBH_DIST_TRUNCPARETO)
    PBH_EXT(PBH_DIST_TUKEYLAMBDA)
    PBH_EXT(PBH_DIST_GENGAMMA)
    PBH_EXT(PBH_DIST_LOGGAMMA)
    PBH_EXT(PBH_DIST_DGAMMA)
    PBH_EXT(PBH_DIST_F)
    PBH_EXT(PBH_DIST_RDIST)
    PBH_EXT(PBH_DIST_SEMICIRCULAR)
    PBH_EXT(PBH_DIST_BETAPRIME)
    PBH_EXT(PBH_DIST_DLAPLACE)
    PBH_EXT(PBH_DIST_PLANCK)
    PBH_EXT(PBH_DIST_BOLTZMANN)
    PBH_EXT(PBH_DIST_PEARSON3)
    PBH_EXT(PBH_DIST_GENNORM)
    PBH_EXT(PBH_DIST_HALFGENNORM)
    PBH_EXT(PBH_DIST_WRAPCAUCHY)
    PBH_EXT(PBH_DIST_SKEWCAUCHY)
    PBH_EXT(PBH_DIST_MOYAL)
    PBH_EXT(PBH_DIST_KAPPA4)
    PBH_EXT(PBH_DIST_CRYSTALBALL)
    PBH_EXT(PBH_DIST_POWERLOGNORM)
    PBH_EXT(PBH_DIST_JF_SKEW_T)
    PBH_EXT(PBH_DIST_FOLDCAUCHY)
    PBH_EXT(PBH_DIST_FOLDNORM)
    PBH_EXT(PBH_DIST_COSINE)
    PBH_EXT(PBH_DIST_INVGAUSS)
    PBH_EXT(PBH_DIST_WALD)
    PBH_EXT(PBH_DIST_BETABINOM)
    PBH_EXT(PBH_DIST_HYPERGEOM)
    PBH_EXT(PBH_DIST_SKEWNORM)
    PBH_EXT(PBH_DIST_RECIPINVGAUSS)
    PBH_EXT(PBH_DIST_EXPONNORM)
    PBH_EXT(PBH_DIST_ARGUS)
    PBH_EXT(PBH_DIST_KSTWOBIGN)
    PBH_EXT(PBH_DIST_NHYPERGEOM)
    PBH_EXT(PBH_DIST_YULESIMON)
    PBH_EXT(PBH_DIST_ZIPFIAN)
    PBH_EXT(PBH_DIST_REL_BREITWIGNER)
#undef PBH_EXT
    default:
      return false;
  }
}

int launch_ext(int dist, const double* q, int64_t q_stride, const LhsCol* lc, int64_t n, const pbh_param* params,
               int nparams, double* out, int32_t* flag, hipStream_t s) {
  const int want = ext_nparams(dist);
  PBH_REQUIRE(want >= 0, "ppf: unknown distribution id %d", dist);
  PBH_REQUIRE(nparams == want && params, "ppf: distribution %d takes %d parameters, got %d", dist, want, nparams);
  Params4 prm{};
  for (int j = 0; j < nparams; ++j) {
    prm.ptr[j] = params[j].ptr;
    prm.val[j] = params[j].value;
  }
  if (n == 0) return PBH_OK;
  double* table = build_table(dist, params, nparams, s);
  attach_table(dist, table, prm);
  dim3 g(grid_for(n, 256, 16384)), b(256);
  const LhsCol l = lc ? *lc : LhsCol{0, 1, 0, 0};
  const bool known = dispatch_ext(dist, [&](auto tag) {
    constexpr int D = decltype(tag)::value;
    if (lc)
      PBH_TIMED(kKLhsPpf, s, hipLaunchKernelGGL((k_ppf_ext<D, true>), g, b, 0, s, q, q_stride, l, n, prm, out, flag));
    else
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL((k_ppf_ext<D, false>), g, b, 0, s, q, q_stride, l, n, prm, out, flag));
  });
  release_table(table, s);  // stream-ordered: after the kernel (cached tables stay)
  if (!known) {
    set_error("ppf: unknown distribution id %d", dist);
    return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// ---------------------------------------------------------------- generated columns
// The Iman-Conover fast path for these distributions (pbh_api.hip ic_run, pbh_ic_owned_*): the
// column in stratum order, value(t) = ppf(lhs_sorted_quantile(t)) -- the quantile of the row
// pi^-1(t), so bit-identical to k_ppf_ext<D, true>'s value for that row -- counted for ties and
// inversions without being stored, and regenerated by step 4's last pass at the sorted position p
// of every row (Y[row] = sort(X)[p]).  The same roles k_lhs_sorted_ppf / k_discrete_heads /
// k_place_gen play for the base set (pbh_ppf.hip).
template <int D>
__device__ __forceinline__ double gen_value(const Philox& ph, int64_t t, uint32_t col, int64_t n, const Params4& p) {
  return ppf_ext_one<D>(lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n), p, 0);
}

// out[i] = value(t0 + i) (out may be NULL); counts[0] += #ties, counts[1] += #inversions over the
// pairs inside the segment; heads: every run head t + 1 (x[t] != x[t + 1]) appended at heads[*hcur].
// Waves advance by 63 strata and overlap by one, so every pair meets inside one wave.
template <int D>
__global__ __launch_bounds__(256) void k_ext_sorted(uint64_t seed, int64_t n, int64_t t0, int64_t nt, uint32_t col,
                                                    Params4 prm, double* __restrict__ out, int32_t* flag,
                                                    unsigned long long* counts, uint32_t* __restrict__ heads,
                                                    uint32_t* __restrict__ hcur, uint32_t hcap) {
  __shared__ unsigned long long sh[2][4];
  Philox ph(seed);
  const int lane = threadIdx.x & 63;
  unsigned long long ties = 0, inv = 0;
  const int64_t waves = (int64_t)gridDim.x * 4;
  const int64_t wid0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t iters = (nt + 63 * waves - 1) / (63 * waves);
  for (int64_t it = 0; it < iters; ++it) {
    const int64_t i = (it * waves + wid0) * 63 + lane;
    const bool valid = i < nt;
    double x = 0.0;
    if (valid) {
      x = gen_value<D>(ph, t0 + i, col, n, prm);
      if (out && lane < 63) out[i] = x;
    }
    flag_nonfinite(flag, valid && lane < 63 && !isfinite(x));
    const double nx = __shfl_down(x, 1, 64);
    const bool has_next = valid && lane < 63 && i + 1 < nt;
    ties += has_next && x == nx;
    inv += has_next && !(x <= nx);
    if (heads) {
      const bool hd = has_next && x != nx;
      const uint64_t m = __ballot(hd);
      if (m) {
        const int leader = __builtin_ctzll(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(hcur, (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        const uint32_t slot = base + (uint32_t)__popcll(m & lt);
        if (hd && slot < hcap) heads[slot] = (uint32_t)(t0 + i + 1);
      }
    }
  }
  if (!counts) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ties += __shfl_xor(ties, o, 64);
    inv += __shfl_xor(inv, o, 64);
  }
  if (lane == 0) {
    sh[0][threadIdx.x >> 6] = ties;
    sh[1][threadIdx.x >> 6] = inv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long a = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    const unsigned long long b = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    if (a) atomicAdd(&counts[0], a);
    if (b) atomicAdd(&counts[1], b);
  }
}

// binom / bernoulli: the run heads of strata [t0, t0 + nt) by one binary search per integer value
// k in (value(t0), value(t0 + nt - 1)] (the strata's quantiles increase strictly and the ppf is
// monotone, so a run boundary is the first stratum whose value reaches k): the heads, the tie count
// nt - 1 - #heads and the inversion count 0 equal k_ext_sorted's, from ~30 evaluations per value
// instead of nt (as k_discrete_heads does for poisson).  Ends that are not finite integers within
// kDiscreteSpan of each other are reported as an inversion: the caller then counts exactly.
constexpr int kExtDiscreteSpan = 4096;

template <int D>
__global__ __launch_bounds__(256) void k_ext_discrete_heads(uint64_t seed, int64_t n, int64_t t0, int64_t nt,
                                                            uint32_t col, Params4 prm, int32_t* flag,
                                                            unsigned long long* counts, uint32_t* __restrict__ heads,
                                                            uint32_t* __restrict__ hcur, uint32_t hcap) {
  __shared__ uint32_t b[kExtDiscreteSpan];
  __shared__ int span, bad;
  __shared__ double vlo;
  __shared__ uint32_t found;
  Philox ph(seed);
  if (threadIdx.x == 0) {
    const double a = gen_value<D>(ph, t0, col, n, prm), z = gen_value<D>(ph, t0 + nt - 1, col, n, prm);
    vlo = a;
    found = 0;
    bad = !(isfinite(a) && isfinite(z) && a == floor(a) && z == floor(z) && z >= a && z - a <= kExtDiscreteSpan);
    span = bad ? 0 : (int)(z - a);
    if (bad) {
      flag_nonfinite(flag, !isfinite(a) || !isfinite(z));
      atomicAdd(&counts[1], 1ull);
    }
  }
  __syncthreads();
  const int m = span;
  for (int i = threadIdx.x; i < m; i += 256) {
    const double k = vlo + 1.0 + (double)i;
    int64_t lo = t0, hi = t0 + nt - 1;  // value(lo) < k <= value(hi)
    while (hi - lo > 1) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      if (gen_value<D>(ph, mid, col, n, prm) >= k)
        hi = mid;
      else
        lo = mid;
    }
    b[i] = (uint32_t)hi;
  }
  __syncthreads();
  uint32_t mine = 0;
  for (int i = threadIdx.x; i < m; i += 256) {
    if (i > 0 && b[i] == b[i - 1]) continue;  // a value no stratum takes
    const uint32_t slot = atomicAdd(hcur, 1u);
    if (slot < hcap) heads[slot] = b[i];
    ++mine;
  }
  if (mine) atomicAdd(&found, mine);
  __syncthreads();
  if (threadIdx.x == 0 && !bad) atomicAdd(&counts[0], (unsigned long long)(nt - 1 - (int64_t)found));
}

// Step 4's last pass: Y[row] = value(p) for the (row << 32 | p) pairs of every block of
// kGenRows consecutive rows, assembled in LDS and written contiguously (BYROW: row r0 + i itself
// with stratum pidx[r0 + i], the row owner's half of a row-sharded step 4).
constexpr int kExtGenRows = 1 << kGenPlaceShift;

template <int D, bool BYROW>
__global__ __launch_bounds__(256) void k_ext_place(const uint64_t* __restrict__ pairs,
                                                   const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                   uint64_t seed, uint32_t col, Params4 prm, double* __restrict__ y,
                                                   int64_t y_rs, int32_t* __restrict__ idx,
                                                   const int32_t* __restrict__ state) {
  if (state && *state) return;
  __shared__ double buf[kExtGenRows];
  if constexpr (ext_table_discrete<D>()) {  // as k_ppf_ext: the small CDF tables from LDS
    __shared__ double tab[2 * kExtLdsTab];
    if (prm.dt && prm.dlen <= kExtLdsTab) {  // block-uniform
      for (int k = threadIdx.x; k < 2 * prm.dlen; k += 256) tab[k] = prm.dt[k];
      __syncthreads();
      prm.dt = tab;
    }
  }
  Philox ph(seed);
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kExtGenRows ? (rows - r0) : kExtGenRows);
    for (int p = threadIdx.x; p < cnt; p += 256) {
      uint32_t t;
      int off;
      if constexpr (BYROW) {
        t = pidx[r0 + p];
        off = p;
      } else {
        const uint64_t pr = pairs[r0 + p];
        t = (uint32_t)pr;
        const int64_t row = (int64_t)(pr >> 32);
        if (idx) idx[row] = (int32_t)t;
        off = (int)(row - r0);
      }
      buf[off] = gen_value<D>(ph, (int64_t)t, col, n, prm);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < cnt; p += 256) y[(r0 + p) * y_rs] = buf[p];
    __syncthreads();
  }
}

// the certificate's exact evaluation (k_cert_eval's role for the base set): the listed pairs
// (t, t + 1) and both ends of the segment, counted for ties / inversions
template <int D>
__global__ __launch_bounds__(256) void k_ext_cert_eval(uint64_t seed, int64_t n, int64_t t0, int64_t nt, uint32_t col,
                                                       Params4 prm, const uint32_t* __restrict__ list, uint32_t cap,
                                                       const uint32_t* __restrict__ count, int32_t* flag,
                                                       unsigned long long* counts) {
  Philox ph(seed);
  const uint32_t m = *count;
  unsigned long long ties = 0, inv = 0;
  if (blockIdx.x == 0 && threadIdx.x < 2) {
    const double x = gen_value<D>(ph, threadIdx.x == 0 ? t0 : t0 + nt - 1, col, n, prm);
    if (!isfinite(x)) {
      if (flag) atomicOr(flag, 1);
      ties += 1;
    }
    if (threadIdx.x == 0 && m > cap) ties += 1;
  }
  const uint32_t mm = m < cap ? m : cap;
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < mm; k += gridDim.x * 256) {
    const int64_t t = t0 + list[k];
    const double a = gen_value<D>(ph, t, col, n, prm), b = gen_value<D>(ph, t + 1, col, n, prm);
    ties += a == b;
    inv += !(a <= b);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ties += __shfl_xor(ties, o, 64);
    inv += __shfl_xor(inv, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && (ties | inv)) {
    atomicAdd(&counts[0], ties);
    atomicAdd(&counts[1], inv);
  }
}

Params4 scalar_params(int dist, const double* val, int np, const double* table) {
  Params4 p{};
  for (int j = 0; j < 4; ++j) p.val[j] = j < np ? val[j] : 0.0;
  attach_table(dist, table, p);
  return p;
}

}  // namespace

int ext_nparams(int dist) {
  if (dist == PBH_DIST_BERNOULLI || dist == PBH_DIST_GEOM || dist == PBH_DIST_DLAPLACE || dist == PBH_DIST_PLANCK ||
      dist == PBH_DIST_YULESIMON)
    return 2;
  if (dist == PBH_DIST_BINOM || dist == PBH_DIST_RANDINT || dist == PBH_DIST_NBINOM || dist == PBH_DIST_BOLTZMANN ||
      dist == PBH_DIST_ZIPFIAN)
    return 3;
  if (dist == PBH_DIST_BETA || dist == PBH_DIST_TRUNCNORM || dist == PBH_DIST_BETABINOM || dist == PBH_DIST_HYPERGEOM || dist == PBH_DIST_NHYPERGEOM)
    return 4;
  if (is_closed(dist)) return closed_shapes(dist) + 2;
  return -1;
}

bool ext_is_discrete(int dist) {
  return dist == PBH_DIST_BINOM || dist == PBH_DIST_BERNOULLI || is_discrete2(dist);
}

namespace {
// An upper bound on the number of distinct values a discrete column takes for quantiles in (0, 1)
// (inf when unknown), and its loc: the binary-search heads need integer values spanning few of them
void discrete_span(int dist, const double* val, double* span, double* loc) {
  const double top = 1.0 - 0x1p-53;  // the largest quantile below 1
  *span = sf::kInf;
  *loc = sf::kNaN;
  switch (dist) {
    case PBH_DIST_BINOM:
      if (val[0] >= 0.0) *span = val[0] + 1.0;
      *loc = val[2];
      break;
    case PBH_DIST_BERNOULLI:
      *span = 2.0;
      *loc = val[1];
      break;
    case PBH_DIST_GEOM:
      if (val[0] > 0.0 && val[0] <= 1.0) *span = sfx::geom_ppf01(top, val[0]) + 1.0;
      *loc = val[1];
      break;
    case PBH_DIST_RANDINT:
      if (val[1] > val[0]) *span = val[1] - val[0] + 1.0;
      *loc = val[2];
      break;
    case PBH_DIST_NBINOM:
      if (val[0] > 0.0 && val[1] > 0.0 && val[1] <= 1.0 && val[0] < 1e6 && val[1] > 1e-6)
        *span = sfx::nbinom_ppf01(top, val[0], val[1]) + 1.0;
      *loc = val[2];
      break;
    case PBH_DIST_DLAPLACE:
      if (val[0] > 0.0) *span = sfx::dlaplace_ppf01(top, val[0]) - sfx::dlaplace_ppf01(0x1p-53, val[0]) + 1.0;
      *loc = val[1];
      break;
    case PBH_DIST_PLANCK:
      if (val[0] > 0.0) *span = sfx::planck_ppf01(top, val[0]) + 1.0;
      *loc = val[1];
      break;
    case PBH_DIST_BOLTZMANN:
      if (val[0] > 0.0 && val[1] > 0.0) *span = val[1];
      *loc = val[2];
      break;
    case PBH_DIST_ZIPFIAN:
      if (val[0] >= 0.0 && val[1] > 0.0) *span = val[1];
      *loc = val[2];
      break;
    case PBH_DIST_BETABINOM:
    case PBH_DIST_HYPERGEOM:
    case PBH_DIST_NHYPERGEOM: {
      double lo, hi;
      if (sum_bounds(dist, val[0], val[1], val[2], &lo, &hi)) *span = hi - lo + 1.0;
      *loc = val[3];
      break;
    }
    default:
      break;
  }
}
}  // namespace

int ext_gen_sorted(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                   int64_t t0, int64_t nt, double* out, int32_t* flag, unsigned long long* counts, uint32_t* heads,
                   uint32_t* hcur, uint32_t hcap, hipStream_t s) {
  const int np = ext_nparams(dist);
  PBH_REQUIRE(np >= 0, "ext_gen_sorted: distribution %d is not an extended one", dist);
  if (nt == 0) return PBH_OK;
  const Params4 prm = scalar_params(dist, val, np, table);
  // binom / bernoulli, counts and heads only: the binary-search heads when the values are integers
  // (an integer loc) spanning few of them (n + 1 at most); any other column (a non-integer loc
  // moves every value off the integers) takes k_ext_sorted, which counts exactly
  if (ext_is_discrete(dist) && counts && heads && !out && nt >= 2) {
    double span, loc;
    discrete_span(dist, val, &span, &loc);
    if (span < (double)kExtDiscreteSpan && isfinite(loc) && loc == floor(loc)) {
      const bool known = dispatch_ext(dist, [&](auto tag) {
        constexpr int D = decltype(tag)::value;
        if constexpr (D == PBH_DIST_BINOM || D == PBH_DIST_BERNOULLI || is_discrete2(D))
          PBH_TIMED(kKLhsSorted, s,
                    hipLaunchKernelGGL(k_ext_discrete_heads<D>, dim3(1), dim3(256), 0, s, seed, n, t0, nt, col, prm,
                                       flag, counts, heads, hcur, hcap));
      });
      (void)known;
      PBH_CHECK_LAUNCH();
      return PBH_OK;
    }
  }
  const dim3 g(grid_for(nt, 256 * 63 / 64 + 1, 8192)), b(256);
  dispatch_ext(dist, [&](auto tag) {
    constexpr int D = decltype(tag)::value;
    PBH_TIMED(kKLhsSorted, s,
              hipLaunchKernelGGL(k_ext_sorted<D>, g, b, 0, s, seed, n, t0, nt, col, prm, out, flag, counts, heads, hcur,
                                 hcap));
  });
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int ext_gen_place(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                  const uint64_t* pairs, const uint32_t* pidx, int64_t rows, double* y, int64_t y_rs, int32_t* idx,
                  const int32_t* state, hipStream_t s) {
  const int np = ext_nparams(dist);
  PBH_REQUIRE(np >= 0, "ext_gen_place: distribution %d is not an extended one", dist);
  const int64_t blocks = (rows + kExtGenRows - 1) / kExtGenRows;
  if (blocks <= 0) return PBH_OK;
  const Params4 prm = scalar_params(dist, val, np, table);
  const dim3 g((unsigned)(blocks < 256 * 8 ? blocks : 256 * 8)), b(256);
  dispatch_ext(dist, [&](auto tag) {
    constexpr int D = decltype(tag)::value;
    if (pidx)
      hipLaunchKernelGGL((k_ext_place<D, true>), g, b, 0, s, pairs, pidx, rows, n, seed, col, prm, y, y_rs, idx,
                         state);
    else
      PBH_TIMED(kKPlaceGen, s,
                hipLaunchKernelGGL((k_ext_place<D, false>), g, b, 0, s, pairs, pidx, rows, n, seed, col, prm, y, y_rs,
                                   idx, state));
  });
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int ext_gen_cert_eval(uint64_t seed, int64_t n, uint32_t col, int dist, const double* val, const double* table,
                      int64_t t0, int64_t nt, const uint32_t* list, uint32_t cap, const uint32_t* count, int32_t* flag,
                      unsigned long long* counts, hipStream_t s) {
  const int np = ext_nparams(dist);
  PBH_REQUIRE(np >= 0, "ext_gen_cert_eval: distribution %d is not an extended one", dist);
  const Params4 prm = scalar_params(dist, val, np, table);
  dispatch_ext(dist, [&](auto tag) {
    constexpr int D = decltype(tag)::value;
    PBH_TIMED(kKLhsSorted, s,
              hipLaunchKernelGGL(k_ext_cert_eval<D>, dim3(512), dim3(256), 0, s, seed, n, t0, nt, col, prm, list, cap,
                                 count, flag, counts));
  });
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

double* ext_gen_table(int dist, const double* val, int np, hipStream_t s) {
  pbh_param prm[4];
  for (int j = 0; j < 4; ++j) prm[j] = pbh_param{nullptr, j < np ? val[j] : 0.0};
  return build_table(dist, prm, np, s);
}

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
