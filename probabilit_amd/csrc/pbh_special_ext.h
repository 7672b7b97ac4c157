// Special functions behind the extended inverse CDFs (pbh_ppf_ext.hip): ndtr, log_ndtr,
// ndtri_exp, the truncnorm log-space mass, the Cephes incomplete beta and its inversion, bdtr.
// __host__ __device__ so tests/native/special_host.cpp can sweep them against scipy on the CPU.
#pragma once

#include "pbh_special.h"

namespace pbh {
namespace sfx {

using namespace sf;

constexpr double kSqrt1_2 = 0.70710678118654752440;
constexpr double kBig = 4.503599627370496e15;
constexpr double kBigInv = 2.22044604925031308085e-16;
constexpr double kMinLog = -7.451332191019412076235e2;

PBH_HD inline double ndtr(double a) {  // Cephes ndtr (xsf/cephes/ndtr.h)
  if (isnan(a)) return a;
  const double x = a * kSqrt1_2;
  const double z = fabs(x);
  if (z < kSqrt1_2) return 0.5 + 0.5 * erf_(x);
  double y = 0.5 * erfc_(z);
  if (x > 0) y = 1.0 - y;
  return y;
}

// erfcx(y) = exp(y^2) erfc(y) for y >= 0: Cephes erfc is exp(-y^2) times a rational function
// for y >= 1, so that rational function is erfcx itself (no underflow).
PBH_HD inline double erfcx_pos(double y) {
  const double P[9] = {2.46196981473530512524e-10, 5.64189564831068821977e-1, 7.46321056442269912687e0,
                       4.86371970985681366614e1,   1.96520832956077098242e2,  5.26445194995477358631e2,
                       9.34528527171957607540e2,   1.02755188689515710272e3,  5.57535335369399327526e2};
  const double Q[8] = {1.32281951154744992508e1, 8.67072140885989742329e1, 3.54937778887819891062e2,
                       9.75708501743205489753e2, 1.82390916687909736289e3, 2.24633760818710981792e3,
                       1.65666309194161350182e3, 5.57535340817727675546e2};
  const double R[6] = {5.64189583547755073984e-1, 1.27536670759978104416e0, 5.01905042251180477414e0,
                       6.16021097993053585195e0,  7.40974269950448939160e0, 2.97886665372100240670e0};
  const double S[6] = {2.26052863220117276590e0, 9.39603524938001434673e0, 1.20489539808096656605e1,
                       1.70814450747565897222e1, 9.60896809063285878198e0, 3.36907645100081516050e0};
  if (y < 1.0) return exp(y * y) * erfc_(y);
  if (y < 8.0) return polevl(y, P, 8) / p1evl(y, Q, 8);
  return polevl(y, R, 5) / p1evl(y, S, 6);
}

// scipy.special.log_ndtr (xsf: log(erfcx(-t) / 2) - t^2 for x < -1, else log1p(-erfc(t) / 2))
PBH_HD inline double log_ndtr(double x) {
  if (isnan(x)) return x;
  const double t = x * kSqrt1_2;
  if (x < -1.0) return log(erfcx_pos(-t) / 2.0) - t * t;
  return log1p(-erfc_(t) / 2.0);
}

// scipy.special.ndtri_exp: ndtri(exp(y)) without underflow (scipy/special/_ndtri_exp.pxd)
PBH_HD inline double ndtri_exp(double y) {
  const double P1[9] = {4.05544892305962419923e0,   3.15251094599893866154e1,  5.71628192246421288162e1,
                        4.40805073893200834700e1,   1.46849561928858024014e1,  2.18663306850790267539e0,
                        -1.40256079171354495875e-1, -3.50424626827848203418e-2, -8.57456785154685413611e-4};
  const double Q1[8] = {1.57799883256466749731e1,   4.53907635128879210584e1,   4.13172038254672030440e1,
                        1.50425385692907503408e1,   2.50464946208309415979e0,   -1.42182922854787788574e-1,
                        -3.80806407691578277194e-2, -9.33259480895457427372e-4};
  const double P2[9] = {3.23774891776946035970e0,  6.91522889068984211695e0,  3.93881025292474443415e0,
                        1.33303460815807542389e0,  2.01485389549179081538e-1, 1.23716634817820021358e-2,
                        3.01581553508235416007e-4, 2.65806974686737550832e-6, 6.23974539184983293730e-9};
  const double Q2[8] = {6.02427039364742014255e0,  3.67983563856160859403e0,  1.37702099489081330271e0,
                        2.16236993594496635890e-1, 1.34204006088543189037e-2, 3.28014464682127739104e-4,
                        2.89247864745380683936e-6, 6.79019408009981274425e-9};
  if (isnan(y)) return y;
  if (y < -1.7976931348623157e308) return -kInf;
  if (y < -2.0) {
    const double x = y >= -1.7976931348623157e308 * 0.5 ? sqrt(-2.0 * y) : sqrt(2.0) * sqrt(-y);
    const double x0 = x - log(x) / x;
    const double z = 1.0 / x;
    const double x1 = x < 8.0 ? z * polevl(z, P1, 8) / p1evl(z, Q1, 8) : z * polevl(z, P2, 8) / p1evl(z, Q2, 8);
    return x1 - x0;
  }
  if (y > -0.14541345786885906) return -ndtri(-expm1(y));  // log1p(-exp(-2))
  return ndtri(exp(y));
}

PBH_HD inline double log_sum(double a, double b) {  // scipy.special.logsumexp([a, b])
  const double m = a > b ? a : b, o = a > b ? b : a;
  if (m == -kInf) return -kInf;
  if (!isfinite(m)) return m + o;
  return log1p(exp(o - m)) + m;
}

PBH_HD inline double log_diff(double a, double b) {  // log(exp(a) - exp(b)), a >= b
  if (b == -kInf) return a;
  return log1p(-exp(b - a)) + a;
}

PBH_HD inline double log_gauss_mass(double a, double b) {  // scipy _log_gauss_mass
  if (b <= 0.0) return log_diff(log_ndtr(b), log_ndtr(a));
  if (a > 0.0) return log_diff(log_ndtr(-a), log_ndtr(-b));
  return log1p(-ndtr(a) - ndtr(-b));
}

PBH_HD inline double truncnorm_ppf01(double q, double a, double b) {  // scipy truncnorm._ppf
  if (a < 0.0) return ndtri_exp(log_sum(log_ndtr(a), log(q) + log_gauss_mass(a, b)));
  return -ndtri_exp(log_sum(log_ndtr(-b), log1p(-q) + log_gauss_mass(a, b)));
}
// The same with the terms that depend on (a, b) alone evaluated once (scalar parameters):
// c0 = log_ndtr(a) for a < 0, else log_ndtr(-b); c1 = log_gauss_mass(a, b)
PBH_HD inline void truncnorm_consts(double a, double b, double* c0, double* c1) {
  *c0 = a < 0.0 ? log_ndtr(a) : log_ndtr(-b);
  *c1 = log_gauss_mass(a, b);
}
PBH_HD inline double truncnorm_ppf01_c(double q, double a, double c0, double c1) {
  if (a < 0.0) return ndtri_exp(log_sum(c0, log(q) + c1));
  return -ndtri_exp(log_sum(c0, log1p(-q) + c1));
}

// ---------------------------------------------------------------- incomplete beta (Cephes)
PBH_HD inline double lbeta(double a, double b) { return lgam(a) + lgam(b) - lgam(a + b); }

PBH_HD inline double beta_fn(double a, double b) {
  if (a + b < kMaxGam && a < kMaxGam && b < kMaxGam) {
    const double y = Gamma(a + b), ga = Gamma(a), gb = Gamma(b);
    if (fabs(fabs(ga) - fabs(y)) > fabs(fabs(gb) - fabs(y))) return (gb / y) * ga;
    return (ga / y) * gb;
  }
  return exp(lbeta(a, b));
}

PBH_HD inline double incbcf(double a, double b, double x) {  // continued fraction #1
  double k1 = a, k2 = a + b, k3 = a, k4 = a + 1.0, k5 = 1.0, k6 = b - 1.0, k7 = k4, k8 = a + 2.0;
  double pkm2 = 0.0, qkm2 = 1.0, pkm1 = 1.0, qkm1 = 1.0, ans = 1.0, r = 1.0;
  const double thresh = 3.0 * kMachEp;
  for (int n = 0; n < 300; ++n) {
    double xk = -(x * k1 * k2) / (k3 * k4);
    double pk = pkm1 + pkm2 * xk, qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1; pkm1 = pk; qkm2 = qkm1; qkm1 = qk;
    xk = (x * k5 * k6) / (k7 * k8);
    pk = pkm1 + pkm2 * xk; qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1; pkm1 = pk; qkm2 = qkm1; qkm1 = qk;
    if (qk != 0.0) r = pk / qk;
    double t;
    if (r != 0.0) {
      t = fabs((ans - r) / r);
      ans = r;
    } else {
      t = 1.0;
    }
    if (t < thresh) break;
    k1 += 1.0; k2 += 1.0; k3 += 2.0; k4 += 2.0; k5 += 1.0; k6 -= 1.0; k7 += 2.0; k8 += 2.0;
    if (fabs(qk) + fabs(pk) > kBig) { pkm2 *= kBigInv; pkm1 *= kBigInv; qkm2 *= kBigInv; qkm1 *= kBigInv; }
    if (fabs(qk) < kBigInv || fabs(pk) < kBigInv) { pkm2 *= kBig; pkm1 *= kBig; qkm2 *= kBig; qkm1 *= kBig; }
  }
  return ans;
}

PBH_HD inline double incbd(double a, double b, double x) {  // continued fraction #2
  double k1 = a, k2 = b - 1.0, k3 = a, k4 = a + 1.0, k5 = 1.0, k6 = a + b, k7 = a + 1.0, k8 = a + 2.0;
  double pkm2 = 0.0, qkm2 = 1.0, pkm1 = 1.0, qkm1 = 1.0, ans = 1.0, r = 1.0;
  const double z = x / (1.0 - x), thresh = 3.0 * kMachEp;
  for (int n = 0; n < 300; ++n) {
    double xk = -(z * k1 * k2) / (k3 * k4);
    double pk = pkm1 + pkm2 * xk, qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1; pkm1 = pk; qkm2 = qkm1; qkm1 = qk;
    xk = (z * k5 * k6) / (k7 * k8);
    pk = pkm1 + pkm2 * xk; qk = qkm1 + qkm2 * xk;
    pkm2 = pkm1; pkm1 = pk; qkm2 = qkm1; qkm1 = qk;
    if (qk != 0.0) r = pk / qk;
    double t;
    if (r != 0.0) {
      t = fabs((ans - r) / r);
      ans = r;
    } else {
      t = 1.0;
    }
    if (t < thresh) break;
    k1 += 1.0; k2 -= 1.0; k3 += 2.0; k4 += 2.0; k5 += 1.0; k6 += 1.0; k7 += 2.0; k8 += 2.0;
    if (fabs(qk) + fabs(pk) > kBig) { pkm2 *= kBigInv; pkm1 *= kBigInv; qkm2 *= kBigInv; qkm1 *= kBigInv; }
    if (fabs(qk) < kBigInv || fabs(pk) < kBigInv) { pkm2 *= kBig; pkm1 *= kBig; qkm2 *= kBig; qkm1 *= kBig; }
  }
  return ans;
}

PBH_HD inline double pseries(double a, double b, double x) {  // power series
  const double ai = 1.0 / a;
  double u = (1.0 - b) * x;
  double v = u / (a + 1.0);
  const double t1 = v;
  double t = u, n = 2.0, s = 0.0;
  const double z = kMachEp * ai;
  while (fabs(v) > z) {
    u = (n - b) * x / n;
    t *= u;
    v = t / (a + n);
    s += v;
    n += 1.0;
  }
  s += t1;
  s += ai;
  u = a * log(x);
  if (a + b < kMaxGam && fabs(u) < kMaxLog) return s * (1.0 / beta_fn(a, b)) * pow(x, a);
  t = -lbeta(a, b) + u + log(s);
  return t < kMinLog ? 0.0 : exp(t);
}

PBH_HD inline double incbet(double aa, double bb, double xx) {  // I_x(a, b)
  if (!(aa > 0.0) || !(bb > 0.0)) return kNaN;
  if (xx <= 0.0 || xx >= 1.0) {
    if (xx == 0.0) return 0.0;
    if (xx == 1.0) return 1.0;
    return kNaN;
  }
  if (bb * xx <= 1.0 && xx <= 0.95) return pseries(aa, bb, xx);
  double w = 1.0 - xx, a, b, x, xc;
  bool flag = false;
  if (xx > aa / (aa + bb)) {
    flag = true;
    a = bb; b = aa; xc = xx; x = w;
  } else {
    a = aa; b = bb; xc = w; x = xx;
  }
  double t;
  if (flag && b * x <= 1.0 && x <= 0.95) {
    t = pseries(a, b, x);
  } else {
    double y = x * (a + b - 2.0) - (a - 1.0);
    w = y < 0.0 ? incbcf(a, b, x) : incbd(a, b, x) / xc;
    y = a * log(x);
    t = b * log(xc);
    if (a + b < kMaxGam && fabs(y) < kMaxLog && fabs(t) < kMaxLog) {
      t = pow(xc, b);
      t *= pow(x, a);
      t /= a;
      t *= w;
      t *= 1.0 / beta_fn(a, b);
    } else {
      y += t - lbeta(a, b);
      y += log(w / a);
      t = y < kMinLog ? 0.0 : exp(y);
    }
  }
  if (flag) t = t <= kMachEp ? 1.0 - kMachEp : 1.0 - t;
  return t;
}

// x in [0, 1] with I_x(a, b) = q, q <= 1/2: bracketed Halley iteration from a normal /
// power-law guess.
PBH_HD inline double beta_ppf_lower(double q, double a, double b) {
  if (q <= 0.0) return 0.0;
  const double lb = lbeta(a, b);
  double x;
  if (a > 1.0 && b > 1.0) {  // Abramowitz & Stegun 26.5.22 (upper-tail deviate)
    const double yp = -ndtri(q);
    const double lam = (yp * yp - 3.0) / 6.0;
    const double h = 2.0 / (1.0 / (2.0 * a - 1.0) + 1.0 / (2.0 * b - 1.0));
    const double w = yp * sqrt(h + lam) / h - (1.0 / (2.0 * b - 1.0) - 1.0 / (2.0 * a - 1.0)) *
                                                  (lam + 5.0 / 6.0 - 2.0 / (3.0 * h));
    x = a / (a + b * exp(2.0 * w));
  } else {  // the tails: I_x ~ x^a / (a B) near 0, 1 - I_x ~ (1 - x)^b / (b B) near 1
    const double lo = exp((log(q) + log(a) + lb) / a);
    const double hi = 1.0 - exp((log1p(-q) + log(b) + lb) / b);
    const double mean = a / (a + b);
    x = incbet(a, b, mean) > q ? lo : hi;
    if (x == 0.0 || x == 1.0) return x;  // the tail root underflows (or rounds to 1)
  }
  if (!(x > 0.0 && x < 1.0)) x = 0.5;
  double lo = 0.0, hi = 1.0;
  for (int it = 0; it < 100; ++it) {
    const double f = incbet(a, b, x) - q;
    if (f == 0.0) break;
    if (f < 0.0)
      lo = x;
    else
      hi = x;
    const double lpdf = (a - 1.0) * log(x) + (b - 1.0) * log1p(-x) - lb;
    const double pdf = exp(lpdf);
    double xn;
    if (pdf > 0.0 && isfinite(pdf)) {
      const double dx = f / pdf;
      const double d2 = (a - 1.0) / x - (b - 1.0) / (1.0 - x);  // (log pdf)'
      const double den = 1.0 - 0.5 * dx * d2;
      xn = x - (den > 0.5 && den < 2.0 ? dx / den : dx);
    } else {
      xn = -1.0;
    }
    if (!(xn > lo && xn < hi)) xn = (lo > 0.0 && hi / lo > 4.0) ? sqrt(lo * hi) : 0.5 * (lo + hi);
    if (fabs(xn - x) <= 2.0 * kMachEp * x) {
      x = xn;
      break;
    }
    if (hi - lo <= 2.0 * kMachEp * lo) break;
    x = xn;
  }
  return x;
}

// x with I_x(a, b) = q.  Above the median the complement I_{1-x}(b, a) = 1 - q is inverted
// instead (1 - q is exact there), as Boost's ibeta_inv does.
PBH_HD inline double beta_ppf01(double q, double a, double b) {
  if (q <= 0.0) return 0.0;
  if (q >= 1.0) return 1.0;
  if (q > 0.5) return 1.0 - beta_ppf_lower(1.0 - q, b, a);
  return beta_ppf_lower(q, a, b);
}

// ---------------------------------------------------------------- beta guide table
// For scalar (a, b) the beta inverse CDF is tabulated as z = logit(x) against w = logit(q) on a
// uniform grid (w in [-60, 40], h = 1/32), with dz/dw and d2z/dw2 from the density:
//   g = dz/dw = q (1 - q) B(a, b) / (x^a (1 - x)^b),  d2z/dw2 = g ((1 - q) - q - (a (1 - x) - b x) g),
// and a draw interpolates the quintic Hermite of its interval (sf::guide_interp_arr, as gamma's
// guide does) -- about 20 FP64 operations plus a log and an exp instead of a Halley iteration
// on the incomplete beta (~40x ndtri's cost).  An interval is used only when the interpolant
// matches the exact inverse at its midpoint to kBetaGuideTol in z (relative 1e-12 in x and in
// 1 - x); the other draws, and any q outside the grid, take beta_ppf01.
constexpr double kBetaGuideW0 = -60.0;
constexpr double kBetaGuideH = 1.0 / 32.0;
constexpr int kBetaGuideM = 3201;
constexpr double kBetaGuideTol = 1e-12;

struct BetaGuide {
  const double* z;   // logit x at w_j = w0 + j h
  const double* d1;  // dz/dw at w_j
  const double* d2;  // d2z/dw2 at w_j
  const double* ok;  // 1.0 when interval [w_j, w_j+1] passed the midpoint check
};

// x and 1 - x of the quantile q = 1 / (1 + e^-w), each to full relative precision
PBH_HD inline void beta_quantile_pair(double w, double a, double b, double* x, double* xc) {
  const double q = 1.0 / (1.0 + exp(-w)), qc = 1.0 / (1.0 + exp(w));
  if (q > 0.5) {
    *xc = beta_ppf_lower(qc, b, a);
    *x = 1.0 - *xc;
  } else {
    *x = beta_ppf_lower(q, a, b);
    *xc = 1.0 - *x;
  }
}

PBH_HD inline void beta_guide_entry(double a, double b, double lb, double w, double* z, double* d1, double* d2) {
  double x, xc;
  beta_quantile_pair(w, a, b, &x, &xc);
  if (!(x > 0.0 && xc > 0.0)) {
    *z = __builtin_nan("");
    *d1 = *d2 = 0.0;
    return;
  }
  const double lx = log(x), lxc = log(xc);
  const double lq = -log1p(exp(-w)), lqc = -log1p(exp(w));
  const double g = exp(lq + lqc + lb - a * lx - b * lxc);
  const double q = exp(lq), qc = exp(lqc);
  *z = lx - lxc;
  *d1 = g;
  *d2 = g * ((qc - q) - (a * xc - b * x) * g);
}

// 1.0 when interval j's interpolant matches the exact z at its midpoint
PBH_HD inline double beta_guide_check(double a, double b, const BetaGuide& T, int j) {
  double x, xc;
  beta_quantile_pair(kBetaGuideW0 + (j + 0.5) * kBetaGuideH, a, b, &x, &xc);
  if (!(x > 0.0 && xc > 0.0)) return 0.0;
  const double exact = log(x) - log(xc);
  const double v = sf::guide_interp_arr(T.z, T.d1, T.d2, kBetaGuideH, j, 0.5);
  return (isfinite(exact) && isfinite(v) && isfinite(T.z[j]) && isfinite(T.z[j + 1]) &&
          fabs(v - exact) <= kBetaGuideTol)
             ? 1.0
             : 0.0;
}

// beta_ppf01 through the guide (q in (0, 1)); lt: log_tab's table (global or an LDS copy)
PBH_HD inline double beta_ppf_guided(double q, double a, double b, const BetaGuide& T) {
  const double w = sf::log_odds_at(q, &sf::pbh_log_tab[0][0]);
  const double u = (w - kBetaGuideW0) * (1.0 / kBetaGuideH);
  if (u >= 0.0 && u < (double)(kBetaGuideM - 1)) {
    const int j = (int)u;
    if (T.ok[j] != 0.0) {
      const double z = sf::guide_interp_arr(T.z, T.d1, T.d2, kBetaGuideH, j, u - (double)j);
      if (z >= 0.0) return 1.0 / (1.0 + exp(-z));
      const double e = exp(z);
      return e / (1.0 + e);
    }
  }
  return beta_ppf01(q, a, b);
}

PBH_HD inline double bdtr(double k, double n, double p) {  // Cephes bdtr, 0 <= k
  if (k >= n) return 1.0;
  const double dn = n - k;
  if (k == 0.0) return pow(1.0 - p, dn);
  return incbet(dn, k + 1.0, 1.0 - p);
}

PBH_HD inline double bdtrc(double k, double n, double p) {  // Cephes bdtrc: P(X > k)
  if (k >= n) return 0.0;
  const double dn = n - k;
  if (k < 0.0) return 1.0;
  if (k == 0.0) return p < 0.01 ? -expm1(dn * log1p(-p)) : 1.0 - pow(1.0 - p, dn);
  return incbet(k + 1.0, dn, p);
}

// smallest k in [0, n] with bdtr(k, n, p) >= q; above the median on the complement,
// bdtrc(k) <= 1 - q (1 - q is exact there), as Boost's discrete quantile does.
PBH_HD inline double binom_ppf01(double q, double n, double p) {
  double k = floor(n * p + sqrt(n * p * (1.0 - p)) * ndtri(q));
  if (!(k >= 0.0)) k = 0.0;
  if (k > n) k = n;
  if (q <= 0.5) {
    if (bdtr(k, n, p) >= q) {
      while (k > 0.0 && bdtr(k - 1.0, n, p) >= q) k -= 1.0;
    } else {
      do {
        k += 1.0;
      } while (k < n && bdtr(k, n, p) < q);
    }
    return k;
  }
  const double r = 1.0 - q;
  if (bdtrc(k, n, p) <= r) {
    while (k > 0.0 && bdtrc(k - 1.0, n, p) <= r) k -= 1.0;
  } else {
    do {
      k += 1.0;
    } while (k < n && bdtrc(k, n, p) > r);
  }
  return k;
}


// ---- round 5: geom, randint, nbinom, t (scipy 1.15 _ppf bodies)

// geom._ppf(q, p) (scipy/stats/_discrete_distns.py), numpy's log1p / expm1 (the C library's):
//   vals = ceil(log1p(-q) / log1p(-p)); temp = _cdf(vals - 1, p) = -expm1(log1p(-p) floor(vals - 1))
//   where((temp >= q) & (vals > 0), vals - 1, vals)
PBH_HD inline double geom_ppf01(double q, double p) {
  const double lp = log1p(-p);
  const double vals = ceil(log1p(-q) / lp);
  const double temp = -expm1(lp * floor(vals - 1.0));
  return (temp >= q && vals > 0.0) ? vals - 1.0 : vals;
}

// randint._ppf(q, low, high): vals = ceil(q (high - low) + low) - 1; vals1 = clip(vals - 1, low, high);
// temp = _cdf(vals1) = (floor(vals1) - low + 1) / (high - low); where(temp >= q, vals1, vals)
PBH_HD inline double randint_ppf01(double q, double low, double high) {
  const double vals = ceil(q * (high - low) + low) - 1.0;
  const double vals1 = fmin(fmax(vals - 1.0, low), high);
  const double temp = (floor(vals1) - low + 1.0) / (high - low);
  return temp >= q ? vals1 : vals;
}

// ---- round 6: dlaplace, planck, boltzmann (scipy 1.15 _discrete_distns.py _ppf / _cdf bodies)

// dlaplace._ppf(q, a): const = 1 + exp(a); vals = ceil(q < 1 / (1 + exp(-a)) ? log(q const) / a - 1
// : -log((1 - q) const) / a); one step down where _cdf(vals - 1, a) >= q, with
// _cdf(k) = 1 - exp(-a k) / (exp(a) + 1) for k >= 0, exp(a (k + 1)) / (exp(a) + 1) below
PBH_HD inline double dlaplace_cdf(double x, double a) {
  const double k = floor(x);
  return k >= 0.0 ? 1.0 - exp(-a * k) / (exp(a) + 1) : exp(a * (k + 1)) / (exp(a) + 1);
}
PBH_HD inline double dlaplace_ppf01(double q, double a) {
  const double cst = 1 + exp(a);
  const double vals = ceil(q < 1.0 / (1 + exp(-a)) ? log(q * cst) / a - 1 : -log((1 - q) * cst) / a);
  const double vals1 = vals - 1;
  return dlaplace_cdf(vals1, a) >= q ? vals1 : vals;
}

// planck._ppf(q, lambda): vals = ceil(-1 / lambda log1p(-q) - 1); vals1 = max(vals - 1, 0);
// _cdf(vals1) = -expm1(-lambda (floor(vals1) + 1)) >= q ? vals1 : vals
PBH_HD inline double planck_ppf01(double q, double lam) {
  const double vals = ceil(-1.0 / lam * log1p(-q) - 1);
  const double vals1 = fmax(vals - 1, 0.0);
  const double temp = -expm1(-lam * (floor(vals1) + 1));
  return temp >= q ? vals1 : vals;
}

// boltzmann._ppf(q, lambda, N): the truncated planck, qnew = q (1 - exp(-lambda N)); vals =
// ceil(-1 / lambda log(1 - qnew) - 1); vals1 = max(vals - 1, 0); _cdf(vals1) = (1 - exp(-lambda
// (floor(vals1) + 1))) / (1 - exp(-lambda N)) >= q ? vals1 : vals
PBH_HD inline double boltzmann_ppf01(double q, double lam, double N) {
  const double qnew = q * (1 - exp(-lam * N));
  const double vals = ceil(-1.0 / lam * log(1 - qnew) - 1);
  const double vals1 = fmax(vals - 1, 0.0);
  const double temp = (1 - exp(-lam * (floor(vals1) + 1))) / (1 - exp(-lam * N));
  return temp >= q ? vals1 : vals;
}

// negative binomial CDF P(X <= k) = I_p(n, k + 1) and its complement I_{1-p}(k + 1, n) (Boost's
// nbinom cdf, the incomplete beta ratio; Cephes incbet restated above)
PBH_HD inline double nbdtr(double k, double n, double p) {
  if (p >= 1.0) return 1.0;
  return incbet(n, k + 1.0, p);
}
PBH_HD inline double nbdtrc(double k, double n, double p) {
  if (p >= 1.0) return 0.0;
  return incbet(k + 1.0, n, 1.0 - p);
}

// scipy nbinom._ppf = Boost's discrete quantile (integer_round_up): the smallest k >= 0 with
// nbdtr(k, n, p) >= q; above the median on the complement, nbdtrc(k) <= 1 - q, as binom_ppf01
PBH_HD inline double nbinom_ppf01(double q, double n, double p) {
  if (p >= 1.0) return 0.0;
  const double m = n * (1.0 - p) / p, sd = sqrt(n * (1.0 - p)) / p;
  double k = floor(m + sd * ndtri(q));
  if (!(k >= 0.0)) k = 0.0;
  if (k > 9.0e15) k = 9.0e15;
  if (q <= 0.5) {
    if (nbdtr(k, n, p) >= q) {
      while (k > 0.0 && nbdtr(k - 1.0, n, p) >= q) k -= 1.0;
    } else {
      do {
        k += 1.0;
      } while (nbdtr(k, n, p) < q && k < 1.0e18);
    }
    return k;
  }
  const double r = 1.0 - q;
  if (nbdtrc(k, n, p) <= r) {
    while (k > 0.0 && nbdtrc(k - 1.0, n, p) <= r) k -= 1.0;
  } else {
    do {
      k += 1.0;
    } while (nbdtrc(k, n, p) > r && k < 1.0e18);
  }
  return k;
}

// Student's t quantile (scipy t._ppf = stdtrit, cdflib's root search, accurate to ~2.5e-11): the
// exact quantile through the incomplete beta.  With pp = 2 min(q, 1 - q) = P(|T| >= |t|):
// below pp = 1/2, x = df / (df + t^2) solves I_x(df / 2, 1 / 2) = pp (x is then at most the
// median, so 1 - x >= ~0.45 / df keeps its relative error below 1e-11 up to df = 1e5); from
// pp = 1/2 on, y = 1 - x solves I_y(1 / 2, df / 2) = 1 - pp, exact there.  Beyond df = 1e5 the
// Cornish-Fisher series in 1 / df (Abramowitz & Stegun 26.7.5, four terms: the next is below
// 1e-15 relative for |z| <= 8.3) from the normal quantile.
PBH_HD inline double t_ppf01(double q, double df) {
  if (isinf(df)) return ndtri(q);
  if (q == 0.5) return 0.0;
  if (df >= 1e5) {
    const double z = ndtri(q), z2 = z * z, u = 1.0 / df;
    const double g1 = (z2 + 1.0) * z / 4.0;
    const double g2 = ((5.0 * z2 + 16.0) * z2 + 3.0) * z / 96.0;
    const double g3 = (((3.0 * z2 + 19.0) * z2 + 17.0) * z2 - 15.0) * z / 384.0;
    const double g4 = ((((79.0 * z2 + 776.0) * z2 + 1482.0) * z2 - 1920.0) * z2 - 945.0) * z / 92160.0;
    return z + (g1 + (g2 + (g3 + g4 * u) * u) * u) * u;
  }
  const double pp = q < 0.5 ? 2.0 * q : 2.0 * (1.0 - q);
  double t2;
  if (pp < 0.5) {
    const double x = beta_ppf01(pp, 0.5 * df, 0.5);
    t2 = df * ((1.0 - x) / x);
  } else {
    const double y = beta_ppf01(1.0 - pp, 0.5, 0.5 * df);
    t2 = df * (y / (1.0 - y));
  }
  const double t = sqrt(t2);
  return q < 0.5 ? -t : t;
}

// t_ppf01 with the incomplete-beta inverse of (df / 2, 1 / 2) read from beta's guide: z = logit x,
// and t^2 = df (1 - x) / x = df e^-z for both of t_ppf01's branches (the upper one inverts the
// complement, y = 1 - x, and y / (1 - y) is the same e^-z), so no 1 - x is ever formed.
PBH_HD inline double t_ppf_guided(double q, double df, const BetaGuide& T) {
  if (q == 0.5 || !(q > 0.0 && q < 1.0) || !(df > 0.0 && df < 1e5)) return t_ppf01(q, df);
  const double pp = q < 0.5 ? 2.0 * q : 2.0 * (1.0 - q);
  const double w = sf::log_odds_at(pp, &sf::pbh_log_tab[0][0]);
  const double u = (w - kBetaGuideW0) * (1.0 / kBetaGuideH);
  if (!(u >= 0.0 && u < (double)(kBetaGuideM - 1))) return t_ppf01(q, df);
  const int j = (int)u;
  if (T.ok[j] == 0.0) return t_ppf01(q, df);
  const double z = sf::guide_interp_arr(T.z, T.d1, T.d2, kBetaGuideH, j, u - (double)j);
  const double t = sqrt(df * exp(-z));
  return q < 0.5 ? -t : t;
}

}  // namespace sfx
}  // namespace pbh
