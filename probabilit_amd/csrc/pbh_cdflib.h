// scipy.special.pdtrik as scipy 1.15.3 computes it, for the poisson ppf's rare lanes.
//
// scipy's poisson._ppf (scipy/stats/_discrete_distns.py, reached from the reference's
// Distribution._sample, modeling.py:807) is
//     vals = ceil(pdtrik(q, mu)); vals1 = max(vals - 1, 0); where(pdtr(vals1, mu) >= q, vals1, vals)
// pdtrik comes from cdflib (B. W. Brown, J. Lovato, K. Russell; the "cdfpoi" routine with
// which = 2): it brackets the root in s of cumpoi(s, mu) - p (dinvr: start 5, step 0.5 + 0.5|s|,
// step multiplier 5) and refines it with the Bus-Dekker zero finder (dzror) to a relative
// tolerance of 1e-10 (scipy's setting; measured against scipy.special.pdtrik, see
// tests/test_special_host.py::test_pdtrik_*), so the root is only accurate to ~1e-10 s.  Just
// above each CDF value pdtr(k - 1, mu) the computed root can fall below k - 1, and then scipy
// returns k - 1 where the mathematical definition (smallest k with pdtr(k, mu) >= q) gives k;
// the one-step correction only ever moves the answer down.  The device ppf computes the
// definition from its CDF table everywhere and calls this restatement only for lanes inside
// those windows (poisson_window_hi), so the output equals scipy's bit for bit.
//
// cumpoi(s, mu) is cdflib's cumchi / cumgam, i.e. the regularized incomplete gamma ratio
// Q(s + 1, mu) by gratio (DiDonato & Morris 1986, ACM TOMS 654), restated below for a >= 1
// (the poisson ppf never evaluates a < 1: its bracket starts at s = 0) with the published
// constants; gratio's erfc1, rlog and gamma helpers (A. H. Morris, NSWC library) likewise.
// This is a restatement of published algorithms, not scipy code; host and device share it.
#pragma once

#include <math.h>

#include "pbh_glibc.h"
#include "pbh_special.h"

namespace pbh {
namespace cdf {

constexpr double kEps = 2.220446049250313e-16;  // spmpar(1): smallest e with 1 + e > 1

// erfc1(ind, x): erfc(x) (ind == 0) or exp(x^2) erfc(x) (ind != 0)
PBH_HD inline double erfc1(int ind, double x) {
  const double c = .564189583547756e0;
  const double a0 = .771058495001320e-04, a1 = -.133733772997339e-02, a2 = .323076579225834e-01,
               a3 = .479137145607681e-01, a4 = .128379167095513e+00;
  const double b0 = .301048631703895e-02, b1 = .538971687740286e-01, b2 = .375795757275549e+00;
  const double p[8] = {-1.36864857382717e-07, 5.64195517478974e-01, 7.21175825088309e+00, 4.31622272220567e+01,
                       1.52989285046940e+02,  3.39320816734344e+02, 4.51918953711873e+02, 3.00459261020162e+02};
  const double q[8] = {1.00000000000000e+00, 1.27827273196294e+01, 7.70001529352295e+01, 2.77585444743988e+02,
                       6.38980264465631e+02, 9.31354094850610e+02, 7.90950925327898e+02, 3.00459260956983e+02};
  const double r[5] = {2.10144126479064e+00, 2.62370141675169e+01, 2.13688200555087e+01, 4.65807828718470e+00,
                       2.82094791773523e-01};
  const double s[4] = {9.41537750555460e+01, 1.87114811799590e+02, 9.90191814623914e+01, 1.80124575948747e+01};
  double ax = fabs(x), e, t, top, bot, w, res;
  if (ax <= 0.5) {
    t = x * x;
    top = (((a0 * t + a1) * t + a2) * t + a3) * t + a4 + 1.0;
    bot = ((b0 * t + b1) * t + b2) * t + 1.0;
    res = 0.5 + (0.5 - x * (top / bot));
    if (ind != 0) res = glibc::exp(t) * res;
    return res;
  }
  if (ax <= 4.0) {
    top = ((((((p[0] * ax + p[1]) * ax + p[2]) * ax + p[3]) * ax + p[4]) * ax + p[5]) * ax + p[6]) * ax + p[7];
    bot = ((((((q[0] * ax + q[1]) * ax + q[2]) * ax + q[3]) * ax + q[4]) * ax + q[5]) * ax + q[6]) * ax + q[7];
    res = top / bot;
  } else {
    if (x <= -5.6) return ind != 0 ? 2.0 * glibc::exp(x * x) : 2.0;
    if (ind == 0 && (x > 100.0 || x * x > 708.39641853226408)) return 0.0;  // -exparg(1)
    t = (1.0 / x) * (1.0 / x);
    top = (((r[0] * t + r[1]) * t + r[2]) * t + r[3]) * t + r[4];
    bot = (((s[0] * t + s[1]) * t + s[2]) * t + s[3]) * t + 1.0;
    res = (c - t * (top / bot)) / ax;  // scipy 1.15.3: the ratio first, then times t
  }
  if (ind != 0) {
    if (x < 0.0) res = 2.0 * glibc::exp(x * x) - res;
    return res;
  }
  w = x * x;
  t = w;
  e = w - t;
  res = (0.5 + (0.5 - e)) * glibc::exp(-t) * res;
  if (x < 0.0) res = 2.0 - res;
  return res;
}

// rlog(x) = x - 1 - ln x
PBH_HD inline double rlog(double x) {
  const double a = .566749439387324e-01, b = .456512608815524e-01;
  const double p0 = .333333333333333e0, p1 = -.224696413112536e0, p2 = .620886815375787e-02;
  const double q1 = -.127408923933623e+01, q2 = .354508718369557e0;
  double u, w1;
  if (x < 0.61 || x > 1.57) {
    double r = x - 0.5;
    r -= 0.5;
    return r - glibc::log(x);
  }
  if (x < 0.82) {
    u = x - 0.7;
    u /= 0.7;
    w1 = a - u * 0.3;
  } else if (x > 1.18) {
    u = 0.75 * x - 1.e0;
    w1 = b + u / 3.0;
  } else {
    u = x - 0.5 - 0.5;
    w1 = 0.0;
  }
  const double r = u / (u + 2.0);
  const double t = r * r;
  const double w = ((p2 * t + p1) * t + p0) / ((q2 * t + q1) * t + 1.0);
  return 2.0 * t * (1.0 / (1.0 - r) - r * w) + w1;
}

// Gamma(a) for 1 <= a < 20 (Morris' gamma: a rational Gamma(1 + x) on [0, 1) times the
// recurrence product below 15, the modified Stirling sum from 15 on)
PBH_HD inline double gamma_a(double a) {
  const double d = 0.41893853320467267;  // scipy 1.15.3's value (its C cdflib; see gratio below)
  const double r1 = .820756370353826e-03, r2 = -.595156336428591e-03, r3 = .793650663183693e-03,
               r4 = -.277777777770481e-02, r5 = .833333333333333e-01;
  const double p[7] = {.539637273585445e-03, .261939260042690e-02, .204493667594920e-01, .730981088720487e-01,
                       .279648642639792e+00, .553413866010467e+00, 1.0e0};
  const double q[7] = {-.832979206704073e-03, .470059485860584e-02, .225211131035340e-01, -.170458969313360e+00,
                       -.567902761974940e-01, .113062953091122e+01, 1.0e0};
  double x = a;
  if (fabs(a) < 15.0) {
    double t = 1.0;
    const int m = (int)a - 1;
    for (int j = 1; j <= m; ++j) {
      x -= 1.0;
      t = x * t;
    }
    x -= 1.0;
    double top = p[0], bot = q[0];
    for (int i = 1; i < 7; ++i) {
      top = p[i] + x * top;
      bot = q[i] + x * bot;
    }
    return (top / bot) * t;
  }
  const double t = 1.0 / (x * x);
  double g = ((((r1 * t + r2) * t + r3) * t + r4) * t + r5) / x;
  const double lnx = glibc::log(x);
  g = d + g + (x - 0.5) * (lnx - 1.e0);
  const double w = g;
  const double tt = g - w;
  return glibc::exp(w) * (1.0 + tt);
}

// gratio's Temme coefficients d_k (DiDonato & Morris' d0..d6, to 15 digits), one table
PBH_TABLE double kGratioD0[13] = {.833333333333333e-01,  -.148148148148148e-01, .115740740740741e-02,
                                  .352733686067019e-03,  -.178755144032922e-03, .391926317852244e-04,
                                  -.218544851067999e-05, -.185406221071516e-05, .829671134095309e-06,
                                  -.176659527368261e-06, .670785354340150e-08,  .102618097842403e-07,
                                  -.438203601845335e-08};
PBH_TABLE double kGratioD1[12] = {-.347222222222222e-02, .264550264550265e-02,  -.990226337448560e-03,
                                  .205761316872428e-03,  -.401877572016461e-06, -.180985503344900e-04,
                                  .764916091608111e-05,  -.161209008945634e-05, .464712780280743e-08,
                                  .137863344691572e-06,  -.575254560351770e-07, .119516285997781e-07};
PBH_TABLE double kGratioD2[10] = {-.268132716049383e-02, .771604938271605e-03,  .200938786008230e-05,
                                  -.107366532263652e-03, .529234488291201e-04,  -.127606351886187e-04,
                                  .342357873409614e-07,  .137219573090629e-05,  -.629899213838006e-06,
                                  .142806142060642e-06};
PBH_TABLE double kGratioD3[8] = {.229472093621399e-03,  -.469189494395256e-03, .267720632062839e-03,
                                 -.756180167188398e-04, -.239650511386730e-06, .110826541153473e-04,
                                 -.567495282699160e-05, .142309007324359e-05};
PBH_TABLE double kGratioD4[6] = {.784039221720067e-03,  -.299072480303190e-03, -.146384525788434e-05,
                                 .664149821546512e-04,  -.396836504717943e-04, .113757269706784e-04};
PBH_TABLE double kGratioD5[4] = {-.697281375836586e-04, .277275324495939e-03, -.199325705161888e-03,
                                 .679778047793721e-04};
PBH_TABLE double kGratioD6[2] = {-.592166437353694e-03, .270878209671804e-03};

// ((c[n-1] z + c[n-2]) z + ... + c[0]) z + c00, the order of gratio's unrolled expressions
PBH_HD inline double gratio_poly(const double* c, int n, double z, double c00) {
  double a = c[n - 1];
  for (int i = n - 2; i >= 0; --i) a = a * z + c[i];
  return a * z + c00;
}

// gratio(a, x, ans, qans, ind = 0): P(a, x) and Q(a, x) for a >= 1, x > 0.  Below 1 (where the
// poisson search never goes: its bracket starts at s = 0) it returns gratio's error value.
// Call-free, so that the search around it keeps its registers compact (values live across a call
// occupy the callee-saved VGPR blocks and would size every kernel that reaches the rare path).
PBH_HD inline void gratio(double a, double x, double* ans, double* qans) {
  // scipy 1.15.3's C translation of cdflib carries these four constants to full double precision
  // (read from its compiled gratio; the Fortran's 15-digit literals put P and Q off by ~3 ulp in
  // the a >= 20 branches, which moved dzror's iterates)
  const double alog10 = 2.302585092994046, rt2pin = 0.3989422804014327, rtpi = 1.7724538509055159,
               third = 0.3333333333333333;
  const double d10 = -.185185185185185e-02, d20 = .413359788359788e-02, d30 = .649434156378601e-03,
               d40 = -.861888290916712e-03, d50 = -.336798553366358e-03, d60 = .531307936463992e-03,
               d70 = .344367606892378e-03;
  const double acc = 5.e-15, e = kEps, e0 = .25e-03, x0 = 31.0;  // ind = 0
  double r, t, t1, l, s, z, y, rta, c, w, u, sum, wk[20];
  if (!(a >= 1.0)) goto S430;  // not reached by the poisson search (see above)
  if (a * x == 0.0) goto S420;
  if (a >= 20.0) goto S30;
  if (!(a > x || x >= x0)) {
    const double twoa = a + a;
    const int m = (int)twoa;
    if (twoa == (double)m) {
      const int i = m / 2;
      int n;
      if (a == (double)i) {  // S210: finite sum for integer a
        sum = glibc::exp(-x);
        t = sum;
        n = 1;
        c = 0.0;
      } else {  // S220: half-integer a
        const double rtx = sqrt(x);
        sum = erfc1(0, rtx);
        t = glibc::exp(-x) / (rtpi * rtx);
        n = 0;
        c = -0.5;
      }
      while (n != i) {  // scipy 1.15.3 compiles t *= x / c here (the Fortran's x * t / c rounds differently)
        n += 1;
        c += 1.0;
        t *= (x / c);
        sum += t;
      }
      *qans = sum;
      *ans = 0.5 + (0.5 - *qans);
      return;
    }
  }
  // S20
  t1 = a * glibc::log(x) - x;
  r = glibc::exp(t1) / gamma_a(a);
  goto S40;
S30:
  l = x / a;
  if (l == 0.0) goto S370;
  s = 0.5 + (0.5 - l);
  z = rlog(l);
  if (z >= 700.0 / a) goto S410;
  y = a * z;
  rta = sqrt(a);
  if (fabs(s) <= e0 / rta) {  // S330: Temme expansion for l = 1
    if (a * e * e > 3.28e-3) goto S430;
    c = 0.5 + (0.5 - y);
    w = (0.5 - sqrt(y) * (0.5 + (0.5 - y / 3.0)) / rtpi) / c;
    u = 1.0 / a;
    z = sqrt(z + z);
    if (l < 1.0) z = -z;
    goto S340;
  }
  if (fabs(s) <= 0.4) {  // S270: general Temme expansion
    if (fabs(s) <= 2.0 * e && a * e * e > 3.28e-3) goto S430;
    c = glibc::exp(-y);
    w = 0.5 * erfc1(1, sqrt(y));
    u = 1.0 / a;
    z = sqrt(z + z);
    if (l < 1.0) z = -z;
    if (fabs(s) <= 1.e-3) goto S340;
    {
      const double c0 = gratio_poly(kGratioD0, 13, z, -third);
      const double c1 = gratio_poly(kGratioD1, 12, z, d10);
      const double c2 = gratio_poly(kGratioD2, 10, z, d20);
      const double c3 = gratio_poly(kGratioD3, 8, z, d30);
      const double c4 = gratio_poly(kGratioD4, 6, z, d40);
      const double c5 = gratio_poly(kGratioD5, 4, z, d50);
      const double c6 = gratio_poly(kGratioD6, 2, z, d60);
      t = ((((((d70 * u + c6) * u + c5) * u + c4) * u + c3) * u + c2) * u + c1) * u + c0;
    }
    goto S310;
  }
  t = (1.0 / a) * (1.0 / a);
  t1 = (((0.75 * t - 1.0) * t + 3.5) * t - 105.0) / (a * 1260.0);
  t1 -= y;
  r = rt2pin * rta * glibc::exp(t1);
S40:
  if (r == 0.0) goto S420;
  if (x <= fmax(a, alog10)) {  // S50: Taylor series for P / r
    double apn = a + 1.0;
    t = x / apn;
    wk[0] = t;
    int n;
    for (n = 2; n <= 20; n++) {
      apn += 1.0;
      t *= (x / apn);
      if (t <= 1.e-3) break;
      wk[n - 1] = t;
    }
    // scipy 1.15.3 (its C cdflib, read from the compiled gratio): a loop that never broke leaves
    // n = 21, so all 20 stored terms are summed (the Fortran reset n to 20 and dropped wk(20)),
    // and the tail is a while loop (tested before its first term)
    sum = t;
    const double tol = 0.5 * acc;
    while (t > tol) {
      apn += 1.0;
      t *= (x / apn);
      sum += t;
    }
    const int mx = n - 1;
    for (int m = 1; m <= mx; m++) {
      n -= 1;
      sum += wk[n - 1];
    }
    *ans = r / a * (1.0 + sum);
    *qans = 0.5 + (0.5 - *ans);
    return;
  }
  if (x < x0) {  // S250: continued fraction
    const double tol = fmax(5.0 * e, acc);
    double a2nm1 = 1.0, a2n = 1.0, b2nm1 = x, b2n = x + (1.0 - a), am0, an0;
    c = 1.0;
    do {
      a2nm1 = x * a2n + c * a2nm1;
      b2nm1 = x * b2n + c * b2nm1;
      am0 = a2nm1 / b2nm1;
      c += 1.0;
      const double cma = c - a;
      a2n = a2nm1 + cma * a2n;
      b2n = b2nm1 + cma * b2n;
      an0 = a2n / b2n;
    } while (fabs(an0 - am0) >= tol * an0);
    *qans = r * an0;
    *ans = 0.5 + (0.5 - *qans);
    return;
  }
  {  // S100: asymptotic expansion
    double amn = a - 1.0;
    t = amn / x;
    wk[0] = t;
    int n;
    for (n = 2; n <= 20; n++) {
      amn -= 1.0;
      t *= (amn / x);
      if (fabs(t) <= 1.e-3) break;
      wk[n - 1] = t;
    }
    sum = t;  // (n = 21 after a loop that never broke: all 20 terms, as scipy 1.15.3)
    while (fabs(t) > acc) {
      amn -= 1.0;
      t *= (amn / x);
      sum += t;
    }
    const int mx = n - 1;
    for (int m = 1; m <= mx; m++) {
      n -= 1;
      sum += wk[n - 1];
    }
    *qans = r / x * (1.0 + sum);
    *ans = 0.5 + (0.5 - *qans);
    return;
  }
S340: {
  const double c0 = gratio_poly(kGratioD0, 7, z, -third);
  const double c1 = gratio_poly(kGratioD1, 6, z, d10);
  const double c2 = gratio_poly(kGratioD2, 5, z, d20);
  const double c3 = gratio_poly(kGratioD3, 4, z, d30);
  const double c4 = gratio_poly(kGratioD4, 2, z, d40);
  const double c5 = gratio_poly(kGratioD5, 2, z, d50);
  const double c6 = gratio_poly(kGratioD6, 1, z, d60);
  t = ((((((d70 * u + c6) * u + c5) * u + c4) * u + c3) * u + c2) * u + c1) * u + c0;
}
S310:
  if (l < 1.0) {
    *ans = c * (w - rt2pin * t / rta);
    *qans = 0.5 + (0.5 - *ans);
  } else {
    *qans = c * (w + rt2pin * t / rta);
    *ans = 0.5 + (0.5 - *qans);
  }
  return;
S370:
  *ans = 0.0;
  *qans = 1.0;
  return;
S410:
  if (fabs(s) <= 2.0 * e) goto S430;
S420:
  if (x <= a) goto S370;
  *ans = 1.0;
  *qans = 0.0;
  return;
S430:
  *ans = 2.0;
  *qans = sf::kNaN;
}

// fx of cdfpoi (which = 2) at s: cumpoi(s, mu) = (cum, ccum) by cumchi(2 mu, 2 (s + 1)) ->
// cumgam(mu, s + 1), with cum and ccum swapped; fx = cum - p when p <= q, else ccum - q
struct CumPoi {
  double mu, p, q;
  bool qporq;
  PBH_HD double operator()(double s) const {
    const double df = 2.0 * (s + 1.0);
    const double a = df * 0.5;
    const double x = (2.0 * mu) * 0.5;
    double cg, ccg;
    if (x <= 0.0) {
      cg = 0.0;
      ccg = 1.0;
    } else {
      gratio(a, x, &cg, &ccg);
    }
    return qporq ? ccg - p : cg - q;
  }
};

// pdtrik(p, mu): cdfpoi with which = 2 (dinvr + dzror), NaN outside its domain as scipy returns
PBH_HD inline double pdtrik(double p, double mu) {
  if (p != p || mu != mu) return sf::kNaN;
  const double q = 1.0 - p;
  if (p < 0.0 || p > 1.0 || q <= 0.0 || q > 1.0 || mu < 0.0) return sf::kNaN;
  if (mu == 0.0) return 0.0;  // scipy: pdtrik(p, 0) = 0
  const CumPoi f{mu, p, q, p <= q};
  // dstinv(0, inf = 1e100 (scipy 1.15.3), absstp 0.5, relstp 0.5, stpmul 5, abstol 1e-50, reltol 1e-10), s0 = 5
  const double small = 0.0, big = 1.0e100, absstp = 0.5, relstp = 0.5, stpmul = 5.0, abstol = 1.0e-50,
               reltol = 1.0e-10;
  const double xsave = 5.0;
  const double fsmall = f(small), fbig = f(big);
  const bool qincr = fbig > fsmall;
  // the bound answers: status 1 (qleft) returns 0, status 2 returns inf (pdtrik returns the bound)
  if (qincr) {
    if (fsmall > 0.0) return 0.0;
    if (fbig < 0.0) return big;
  } else {
    if (fsmall < 0.0) return 0.0;
    if (fbig > 0.0) return big;
  }
  double step = fmax(absstp, relstp * fabs(xsave));
  double yy = f(xsave);
  if (yy == 0.0) return xsave;
  const bool qup = (qincr && yy < 0.0) || (!qincr && yy > 0.0);
  double xlb, xub;
  if (qup) {
    xlb = xsave;
    xub = fmin(xlb + step, big);
    bool qbdd, qlim;
    for (;;) {
      yy = f(xub);
      qbdd = (qincr && yy >= 0.0) || (!qincr && yy <= 0.0);
      qlim = xub >= big;
      if (qbdd || qlim) break;
      step = stpmul * step;
      xlb = xub;
      xub = fmin(xlb + step, big);
    }
    if (qlim && !qbdd) return big;
  } else {
    xub = xsave;
    xlb = fmax(xub - step, small);
    bool qbdd, qlim;
    for (;;) {
      yy = f(xlb);
      qbdd = (qincr && yy <= 0.0) || (!qincr && yy >= 0.0);
      qlim = xlb <= small;
      if (qbdd || qlim) break;
      step = stpmul * step;
      xub = xlb;
      xlb = fmax(xub - step, small);
    }
    if (qlim && !qbdd) return small;
  }
  // dzror over [xlb, xub]; note its first tolerance is taken at xhi (xlo = xhi before the loop)
  double xlo = xlb;
  const double xhi = xub;
  double b = xlo, fb = f(b);
  xlo = xhi;
  double a = xlo, fa = f(a);
  if ((fb < 0.0 && fa < 0.0) || (fb > 0.0 && fa > 0.0)) return xlo;  // dzror status -1: dinvr returns xlo
  bool first = true;
  double c = a, fc = fa, d = 0.0, fd = 0.0;
  int ext = 0;
  for (;;) {
    if (fabs(fc) < fabs(fb)) {
      if (c != a) {
        d = a;
        fd = fa;
      }
      a = b;
      fa = fb;
      xlo = c;
      b = xlo;
      fb = fc;
      c = a;
      fc = fa;
    }
    double tol = 0.5 * fmax(abstol, reltol * fabs(xlo));
    const double m = (c + b) * .5;
    const double mb = m - b;
    if (!(fabs(mb) > tol)) break;
    double w;
    if (ext > 3) {
      w = mb;
    } else {
      tol = copysign(tol, mb);
      double pp = (b - a) * fb, qq;
      if (first) {
        qq = fa - fb;
        first = false;
      } else {
        const double fdb = (fd - fb) / (d - b);
        const double fda = (fd - fa) / (d - a);
        pp = fda * pp;
        qq = fdb * fa - fda * fb;
      }
      if (pp < 0.0) {
        pp = -pp;
        qq = -qq;
      }
      if (ext == 3) pp = pp * 2.0;
      if (pp * 1.0 == 0.0 || pp <= qq * tol) {
        w = tol;
      } else if (pp < mb * qq) {
        w = pp / qq;
      } else {
        w = mb;
      }
    }
    d = a;
    fd = fa;
    a = b;
    fa = fb;
    b = b + w;
    xlo = b;
    fb = f(xlo);
    if (fc * fb >= 0.0) {
      c = a;
      fc = fa;
      ext = 0;
    } else if (w == mb) {
      ext = 0;
    } else {
      ext += 1;
    }
  }
  return xlo;
}

// scipy's poisson._ppf(q, mu) for 0 < q < 1, mu >= 0 (before loc)
PBH_HD inline double poisson_ppf_scipy(double q, double mu) {
  const double vals = ceil(pdtrik(q, mu));
  const double vals1 = fmax(vals - 1.0, 0.0);
  return sf::pdtr<glibc::Math>(vals1, mu) >= q ? vals1 : vals;
}

// Below this quantile scipy's answer can leave the definition altogether: cdflib's gratio
// underflows to exactly 0 once a rlog(x / a) >= 700 (Q < ~1e-304), so pdtrik's search meets a
// step instead of the CDF (at mu = 2500, q ~ 1e-308 gives 396 where the smallest k with
// pdtr(k, mu) >= q is 869; such departures reach q ~ 1e-160 for mu up to 1e6).  The device sends such q (never an LHS or uniform draw: those are
// >= 1 / (n + 1)) through the restated search as well, so it returns scipy's number there too.
constexpr double kPoissonDeepTail = 1e-150;

// Upper end of the window above pdtr(k - 1, mu) where scipy's answer can be k - 1 instead of k:
// dzror stops with the root of cdflib's function bracketed in [b, c], |c - b| <= reltol |b|
// (1e-10), and returns b, so the computed s is below k - 1 only if the true root is below
// (k - 1)(1 + 1e-10) (+ the absolute floor).  The bound is taken 25% wider, evaluated as
// Q(k + delta, mu), the continuous cumpoi at s = k - 1 + delta, and widened by 2^-40 relative
// for the difference between gratio's values and the CDF table's (a few ulps, up to ~1e-13 in
// Temme's expansion: q within them of pdtr(k - 1) can fall either way, e.g. at k = 1, where
// gratio's Q(1, mu) is exp(-mu)).  A lane inside costs the restated search (~1e-4 s for its
// wave), so the window is kept as tight as the bound allows.  cdflib's own cumpoi at the same s
// bounds it too: where gratio switches expansions (l = mu / a near 1 +- 0.4) its value can be off
// by far more than an ulp (mu = 2500, k = 1781: scipy's root 1779.9992), and scipy's answer follows
// gratio's root, not the CDF's -- so the window ends at the larger of the two.
PBH_HD inline double poisson_window_hi(double k, double mu) {
  if (k < 1.0) return 0.0;  // the answer 0 is never moved down
  const double delta = 1.25e-10 * (k - 1.0) + 1e-30;
  double P, Q;
  gratio(k + delta, mu, &P, &Q);  // cumpoi(k - 1 + delta, mu) = (Q, P): the searched function
  const double g = Q <= 0.5 ? Q : 1.0 - P;
  const double w = sf::igamc<glibc::Math>(k + delta, mu);
  return (g > w ? g : w) * (1.0 + 0x1p-40);
}

}  // namespace cdf
}  // namespace pbh
