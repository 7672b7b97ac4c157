// TEST HARNESS: the device special functions of probabilit_amd/csrc/pbh_special.h compiled
// for the HOST (they are __host__ __device__), so that tests/test_special_host.py can sweep
// them against scipy on the CPU.  This never ships in the product library; device results
// are checked separately by tests/test_gpu_ppf.py (libm vs device math may differ by ulps).
#include <vector>

#include "pbh_glibc.h"
#include "pbh_special.h"

using namespace pbh;

extern "C" {

void sfh_log_tab(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::log_tab(x[i]);
}

// log_tab against the C library's log (glibc: what scipy's Cephes calls) on n points
// x = lo * (hi / lo)^u, u from a 64-bit LCG: counts[0] differing results, counts[1] results more
// than 1 ulp apart.
void sfh_log_tab_vs_libm(double lo, double hi, long n, unsigned long long seed, long* counts) {
  long diff = 0, far = 0;
  const double lr = log(hi / lo);
  for (long i = 0; i < n; ++i) {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    const double u = (double)(seed >> 11) * 0x1.0p-53;
    const double x = lo * exp(lr * u);
    const double a = sf::log_tab(x), b = log(x);
    if (a != b) {
      ++diff;
      const long long ia = (long long)__builtin_bit_cast(unsigned long long, a);
      const long long ib = (long long)__builtin_bit_cast(unsigned long long, b);
      if (ia - ib > 1 || ib - ia > 1) ++far;
    }
  }
  counts[0] = diff;
  counts[1] = far;
}

void sfh_exp_tab(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::exp_tab(x[i]);
}

// exp_tab against the C library's exp on n uniform points of [lo, hi): counts as sfh_log_tab_vs_libm
void sfh_exp_tab_vs_libm(double lo, double hi, long n, unsigned long long seed, long* counts) {
  long diff = 0, far = 0;
  for (long i = 0; i < n; ++i) {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    const double y = lo + (hi - lo) * ((double)(seed >> 11) * 0x1.0p-53);
    const double a = sf::exp_tab(y), b = exp(y);
    if (a != b) {
      ++diff;
      const long long ia = (long long)__builtin_bit_cast(unsigned long long, a);
      const long long ib = (long long)__builtin_bit_cast(unsigned long long, b);
      if (ia - ib > 1 || ib - ia > 1) ++far;
    }
  }
  counts[0] = diff;
  counts[1] = far;
}

void sfh_ndtri(const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::ndtri(q[i]);
}

void sfh_ppnd16(const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::ppnd16(q[i]);
}

void sfh_igami(double a, const double* p, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::igami(a, p[i]);
}

void sfh_pdtr(const double* k, double mu, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::pdtr<pbh::glibc::Math>(k[i], mu);
}

// gamma ppf through the scalar-shape guide table, exactly as the device kernels use it.
void sfh_igami_guided(double a, const double* p, long n, double* out) {
  const int m = sf::kGammaGuideM;
  std::vector<double> tb(4 * (size_t)m);
  sf::GammaGuide T{tb.data(), tb.data() + m, tb.data() + 2 * m, tb.data() + 3 * m, m, sf::kGammaGuideZ0,
                   sf::kGammaGuideH, 1.0 / sf::kGammaGuideH};
  for (int j = 0; j < m; ++j) sf::gamma_guide_entry(a, T.z0 + j * T.h, &tb[j], &tb[m + j], &tb[2 * m + j]);
  for (int j = 0; j < m; ++j) tb[3 * m + j] = j < m - 1 ? sf::gamma_guide_check(a, T, j) : 0.0;
  sf::GammaAux aux = sf::gamma_aux(a);
  for (long i = 0; i < n; ++i) out[i] = sf::igami_guided(a, p[i], &aux, T);
}

// fraction of guide intervals that passed the midpoint check
double sfh_guide_ok_fraction(double a) {
  const int m = sf::kGammaGuideM;
  std::vector<double> tb(4 * (size_t)m);
  sf::GammaGuide T{tb.data(), tb.data() + m, tb.data() + 2 * m, tb.data() + 3 * m, m, sf::kGammaGuideZ0,
                   sf::kGammaGuideH, 1.0 / sf::kGammaGuideH};
  for (int j = 0; j < m; ++j) sf::gamma_guide_entry(a, T.z0 + j * T.h, &tb[j], &tb[m + j], &tb[2 * m + j]);
  int ok = 0;
  for (int j = 0; j < m - 1; ++j) ok += sf::gamma_guide_check(a, T, j) != 0.0;
  return (double)ok / (m - 1);
}
}

// ---- extended distributions (pbh_special_ext.h)
#include "pbh_special_ext.h"

extern "C" {
void sfh_log_ndtr(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::log_ndtr(x[i]);
}
void sfh_ndtri_exp(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::ndtri_exp(x[i]);
}
void sfh_truncnorm_ppf(double a, double b, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::truncnorm_ppf01(q[i], a, b);
}
void sfh_incbet(double a, double b, const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::incbet(a, b, x[i]);
}
void sfh_beta_ppf(double a, double b, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::beta_ppf01(q[i], a, b);
}
// beta_ppf_guided with the guide built on the host as k_beta_guide / k_beta_guide_check build it;
// out[n] (one past the draws) receives the fraction of guide intervals that passed the check
void sfh_beta_guided(double a, double b, const double* q, long n, double* out) {
  const int m = sfx::kBetaGuideM;
  std::vector<double> t(4 * (size_t)m);
  const double lb = sfx::lbeta(a, b);
  for (int j = 0; j < m; ++j)
    sfx::beta_guide_entry(a, b, lb, sfx::kBetaGuideW0 + j * sfx::kBetaGuideH, &t[j], &t[m + j], &t[2 * m + j]);
  const sfx::BetaGuide T{t.data(), t.data() + m, t.data() + 2 * m, t.data() + 3 * m};
  double okc = 0.0;
  for (int j = 0; j < m; ++j) {
    t[3 * m + j] = j < m - 1 ? sfx::beta_guide_check(a, b, T, j) : 0.0;
    okc += t[3 * m + j];
  }
  for (long i = 0; i < n; ++i) out[i] = sfx::beta_ppf_guided(q[i], a, b, T);
  out[n] = okc / (m - 1);
}
void sfh_binom_ppf(double nn, double p, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::binom_ppf01(q[i], nn, p);
}
}

// ---- cdflib's pdtrik (pbh_cdflib.h): the poisson ppf's window lanes
#include "pbh_cdflib.h"

extern "C" {
// glibc's exp / log restated (pbh_glibc.h), for the bit-for-bit check against libm
void sfh_glibc_exp(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = pbh::glibc::exp(x[i]);
}
void sfh_glibc_log(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = pbh::glibc::log(x[i]);
}
void sfh_glibc_pow(const double* x, const double* y, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = pbh::glibc::pow(x[i], y[i]);
}
void sfh_pdtrik(double mu, const double* p, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::pdtrik(p[i], mu);
}
void sfh_poisson_ppf_scipy(double mu, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::poisson_ppf_scipy(q[i], mu);
}
// the device's rule given the definition's k (smallest k with pdtr(k, mu) >= q, from the caller)
void sfh_poisson_rule(double mu, const double* q, const double* kdef, long n, double* out) {
  for (long i = 0; i < n; ++i) {
    const double k = kdef[i];
    const bool rare = (k >= 1.0 && q[i] < cdf::poisson_window_hi(k, mu)) || q[i] < cdf::kPoissonDeepTail;
    out[i] = rare ? cdf::poisson_ppf_scipy(q[i], mu) : k;
  }
}
void sfh_poisson_window_hi(double mu, const double* k, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::poisson_window_hi(k[i], mu);
}
// gratio's P(a, x) (out) for x[i]
void sfh_gratio_p(double a, const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) {
    double p, q;
    cdf::gratio(a, x[i], &p, &q);
    out[i] = p;
  }
}
void sfh_gratio_q(double a, const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) {
    double p, q;
    cdf::gratio(a, x[i], &p, &q);
    out[i] = q;
  }
}
void sfh_cdflib_gamma(const double* a, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::gamma_a(a[i]);
}
void sfh_erfc1(double ind, const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::erfc1((int)ind, x[i]);
}
void sfh_rlog(const double* x, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = cdf::rlog(x[i]);
}
}

extern "C" {
// The device's poisson ppf restated on the host (pbh_ppf_core.h poisson_from_table / poisson_rare):
// the definition (smallest k with pdtr(k, mu) >= q) by a search of the CDF table, then scipy's
// pdtrik computation for q in the window win[k] above pdtr(k - 1, mu).  out[i] = NaN-free k.
void sfh_poisson_ppf_device(double mu, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) {
    double k = 0.0;
    if (mu > 0.0) {
      while (sf::pdtr<pbh::glibc::Math>(k, mu) < q[i] && k < 1e7) k += 1.0;
    }
    const bool rare = (k >= 1.0 && q[i] < cdf::poisson_window_hi(k, mu)) || q[i] < cdf::kPoissonDeepTail;
    out[i] = rare ? cdf::poisson_ppf_scipy(q[i], mu) : k;
  }
}
}

extern "C" {
// ---- round 5 distributions (pbh_special_ext.h): scipy's _ppf for 0 < q < 1
void sfh_geom_ppf(double p, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::geom_ppf01(q[i], p);
}
void sfh_randint_ppf(double low, double high, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::randint_ppf01(q[i], low, high);
}
void sfh_nbinom_ppf(double nn, double p, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::nbinom_ppf01(q[i], nn, p);
}
void sfh_t_ppf(double df, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sfx::t_ppf01(q[i], df);
}
void sfh_invgamma_ppf(double a, const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = 1.0 / sf::igamci(a, q[i]);
}
}
