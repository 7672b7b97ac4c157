// glibc 2.35's double exp and log, operation for operation, for the rare lanes that must give
// the reference's bits (the poisson ppf's cdflib search, pbh_cdflib.h).
//
// scipy 1.15.3's cdflib (reached from the reference's Distribution._sample, modeling.py:807, via
// poisson.ppf -> pdtrik) calls libm's exp and log; on x86-64 with FMA + AVX2 (this image and the
// GPU boxes) glibc resolves them to __exp_fma / __log_fma: Szabolcs Nagy's table-driven
// algorithms (N = 128 subintervals, degree-5 polynomials) compiled with fused multiply-adds.
// Both are within ~0.51 ulp, i.e. not always correctly rounded, and pdtrik's bracketing and
// Bus-Dekker steps just above a CDF value turn a last-bit difference into a different integer.
// So these restate the published algorithm exactly: the data tables (pbh_glibc_tables.inc,
// generated from the image's libm by tools/gen_glibc_tables.py) and every fused multiply-add in
// the place the FMA build has it (read from its machine code; noted per line).  The host test
// (tests/test_special_host.py::test_glibc_exp_log_bit_exact) compares them with libm bit for bit.
// Plain IEEE operations and __builtin_fma only, so host and device give the same doubles.
#pragma once

#include <math.h>
#include <stdint.h>

#include "pbh_common.h"

#ifndef PBH_TABLE
#if defined(__HIP_DEVICE_COMPILE__)
#define PBH_TABLE static __constant__ const
#else
#define PBH_TABLE static const
#endif
#endif

namespace pbh {
namespace glibc {

#include "pbh_glibc_tables.inc"

PBH_HD inline uint64_t bits(double x) { return __builtin_bit_cast(uint64_t, x); }
PBH_HD inline double from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }

// exp's large-|x| tail (|x| in [512, 1024)): the scale's exponent would leave the double range
PBH_HD inline double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {  // k > 0
    sbits -= 1009ull << 52;
    const double scale = from_bits(sbits);
    return __builtin_fma(scale, tmp, scale) * 0x1p1009;
  }
  sbits += 1022ull << 52;  // k < 0: careful rounding into the subnormal range
  const double scale = from_bits(sbits);
  const double st = tmp * scale;
  double y = scale + st;
  if (y < 1.0) {
    const double hi = y + 1.0;
    const double lo = (scale - y) + st;
    y = ((((1.0 - hi) + y) + lo) + hi) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return y * 0x1p-1022;
}

PBH_HD inline double exp(double x) {
  const double InvLn2N = kGlibcExpHead[0], Shift = kGlibcExpHead[1], NegLn2hiN = kGlibcExpHead[2],
               NegLn2loN = kGlibcExpHead[3], C2 = kGlibcExpHead[4], C3 = kGlibcExpHead[5], C4 = kGlibcExpHead[6],
               C5 = kGlibcExpHead[7];
  const uint64_t ix = bits(x);
  uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ff;
  if (abstop - 0x3c9u > 0x3eu) {               // |x| < 2^-54 or |x| >= 512 (or inf / nan)
    if ((int32_t)(abstop - 0x3c9u) < 0) return x + 1.0;
    if (abstop > 0x408u) {                     // |x| >= 1024
      if (ix == 0xfff0000000000000ull) return 0.0;
      if (abstop == 0x7ffu) return x + 1.0;
      return (ix >> 63) ? 0.0 : __builtin_inf();
    }
    abstop = 0;                                // exp_special below
  }
  const double kz = __builtin_fma(x, InvLn2N, Shift);  // x * InvLn2N + Shift, one rounding
  const uint64_t ki = bits(kz);
  const double kd = kz - Shift;
  double r = __builtin_fma(kd, NegLn2hiN, x);
  r = __builtin_fma(kd, NegLn2loN, r);
  const uint64_t idx = 2 * (ki & 0x7f);
  const uint64_t top = ki << 45;
  const double p23 = __builtin_fma(r, C3, C2);
  const double tr = r + from_bits(kGlibcExpTab[idx]);
  const uint64_t sbits = kGlibcExpTab[idx + 1] + top;
  const double r2 = r * r;
  const double p45 = __builtin_fma(r, C5, C4);
  const double t = __builtin_fma(p23, r2, tr);
  const double r4 = r2 * r2;
  const double tmp = __builtin_fma(r4, p45, t);
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  const double scale = from_bits(sbits);
  return __builtin_fma(scale, tmp, scale);
}

PBH_HD inline double log(double x) {
  const double Ln2hi = kGlibcLogHead[0], Ln2lo = kGlibcLogHead[1];
  const double* A = kGlibcLogHead + 2;  // A0..A4
  const double* B = kGlibcLogHead + 7;  // B0..B10
  uint64_t ix = bits(x);
  if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {  // x in [1 - 2^-4, 1 + 0x1.09p-4)
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
    double p1 = __builtin_fma(r, B[2], B[1]);
    double p4 = __builtin_fma(r, B[5], B[4]);
    double p7 = __builtin_fma(r, B[8], B[7]);
    const double r2 = r * r;
    p1 = __builtin_fma(r2, B[3], p1);
    p4 = __builtin_fma(r2, B[6], p4);
    const double r3 = r * r2;
    p7 = __builtin_fma(r2, B[9], p7);
    p7 = __builtin_fma(r3, B[10], p7);
    p4 = __builtin_fma(p7, r3, p4);
    p1 = __builtin_fma(p4, r3, p1);
    const double w = __builtin_fma(r, 0x1p27, r);     // r + r 2^27
    const double rhi = __builtin_fma(-0x1p27, r, w);  // (r + w) - w
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = __builtin_fma(rhi2, B[0], r);
    double lo = __builtin_fma(rhi2, B[0], r - hi);
    lo = __builtin_fma(B[0] * rlo, r + rhi, lo);
    const double y = __builtin_fma(p1, r3, lo);
    return hi + y;
  }
  const uint32_t top = (uint32_t)(ix >> 48);
  if (top - 0x10u > 0x7fdfu) {  // zero, subnormal, negative, inf, nan
    if ((ix << 1) == 0) return -__builtin_inf();
    if (ix == 0x7ff0000000000000ull) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return __builtin_nan("");
    ix = bits(x * 0x1p52) - (52ull << 52);  // subnormal: normalise
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 0x7f);
  const int k = (int)((int64_t)tmp >> 52);
  const double z = from_bits(ix - (tmp & 0xfff0000000000000ull));
  const double invc = kGlibcLogTab[2 * i], logc = kGlibcLogTab[2 * i + 1];
  const double kd = (double)k;
  const double r = __builtin_fma(z, invc, -1.0);
  const double w = __builtin_fma(kd, Ln2hi, logc);
  const double p = __builtin_fma(r, A[2], A[1]);
  const double hi = r + w;
  const double r2 = r * r;
  double lo = (w - hi) + r;
  lo = __builtin_fma(kd, Ln2lo, lo);
  const double r3 = r * r2;
  double q = __builtin_fma(r, A[4], A[3]);
  lo = __builtin_fma(r2, A[0], lo);
  q = __builtin_fma(q, r2, p);
  const double y = __builtin_fma(r3, q, lo);
  return y + hi;
}

// pow's log: log(x) as y + tail with ~15 extra bits (e_pow.c log_inline, FMA build)
PBH_HD inline double pow_log(uint64_t ix, double* tail) {
  const double Ln2hi = kGlibcPowHead[0], Ln2lo = kGlibcPowHead[1];
  const double* A = kGlibcPowHead + 2;  // A0 = -0.5 .. A6
  const uint64_t tmp = ix - 0x3fe6955500000000ull;
  const int i = (int)((tmp >> 45) & 0x7f);
  const int k = (int)((int64_t)tmp >> 52);
  const double z = from_bits(ix - (tmp & 0xfff0000000000000ull));
  const double kd = (double)k;
  const double invc = kGlibcPowTab[3 * i], logc = kGlibcPowTab[3 * i + 1], logctail = kGlibcPowTab[3 * i + 2];
  const double t1 = __builtin_fma(kd, Ln2hi, logc);
  const double r = __builtin_fma(z, invc, -1.0);
  const double ar = r * A[0];
  const double lo1 = __builtin_fma(kd, Ln2lo, logctail);
  const double p12 = __builtin_fma(r, A[2], A[1]);
  const double p34 = __builtin_fma(r, A[4], A[3]);
  const double t2 = r + t1;
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double lo3 = __builtin_fma(ar, r, -ar2);
  const double lo2 = (t1 - t2) + r;
  double p56 = __builtin_fma(r, A[6], A[5]);
  const double hi = t2 + ar2;
  p56 = __builtin_fma(p56, ar2, p34);
  const double lo4 = (t2 - hi) + ar2;
  const double p = __builtin_fma(ar2, p56, p12);
  double lo = ((lo1 + lo2) + lo3) + lo4;
  lo = __builtin_fma(ar3, p, lo);
  const double y = hi + lo;
  *tail = (hi - y) + lo;
  return y;
}

// pow's exp: exp(x + xtail) (e_pow.c exp_inline, sign_bias 0, FMA build)
PBH_HD inline double pow_exp(double x, double xtail) {
  const double InvLn2N = kGlibcExpHead[0], Shift = kGlibcExpHead[1], NegLn2hiN = kGlibcExpHead[2],
               NegLn2loN = kGlibcExpHead[3], C2 = kGlibcExpHead[4], C3 = kGlibcExpHead[5], C4 = kGlibcExpHead[6],
               C5 = kGlibcExpHead[7];
  uint32_t abstop = (uint32_t)(bits(x) >> 52) & 0x7ff;
  if (abstop - 0x3c9u > 0x3eu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return x + 1.0;
    if (abstop > 0x408u) return (bits(x) >> 63) ? 0.0 : __builtin_inf();
    abstop = 0;
  }
  const double kz = __builtin_fma(x, InvLn2N, Shift);
  const uint64_t ki = bits(kz);
  const double kd = kz - Shift;
  double r = __builtin_fma(kd, NegLn2hiN, x);
  r = __builtin_fma(kd, NegLn2loN, r);
  r = xtail + r;
  const uint64_t idx = 2 * (ki & 0x7f);
  const uint64_t sbits = kGlibcExpTab[idx + 1] + (ki << 45);
  const double p23 = __builtin_fma(r, C3, C2);
  const double tr = r + from_bits(kGlibcExpTab[idx]);
  const double r2 = r * r;
  const double p45 = __builtin_fma(r, C5, C4);
  const double t = __builtin_fma(p23, r2, tr);
  const double tmp = __builtin_fma(r2 * r2, p45, t);
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  const double scale = from_bits(sbits);
  return __builtin_fma(tmp, scale, scale);
}

// pow(x, y) for x a positive normal double and y with 2^-65 <= |y| < 2^63 (the main path of
// glibc's __pow_fma); any other argument takes the device pow (never reached by the cdflib /
// Cephes restatements that use this: x / fac > 0, 0 < a < 200)
PBH_HD inline double pow(double x, double y) {
  const uint64_t ix = bits(x), iy = bits(y);
  const uint32_t topx = (uint32_t)(ix >> 52), topy = (uint32_t)(iy >> 52) & 0x7ff;
  if (topx - 1u > 0x7fdu || topy - 0x3beu > 0x7fu) return ::pow(x, y);
  double tail;
  const double hi = pow_log(ix, &tail);
  const double ehi = y * hi;
  const double elo = __builtin_fma(y, tail, __builtin_fma(hi, y, -ehi));
  return pow_exp(ehi, elo);
}

// the math of the reference's L0 (scipy's compiled Cephes / cdflib over glibc's libm), for the
// sf:: templates that take a math policy (pbh_special.h)
struct Math {
  PBH_HD static double exp(double x) { return glibc::exp(x); }
  PBH_HD static double log(double x) { return glibc::log(x); }
  PBH_HD static double pow(double x, double y) { return glibc::pow(x, y); }
};

}  // namespace glibc
}  // namespace pbh
