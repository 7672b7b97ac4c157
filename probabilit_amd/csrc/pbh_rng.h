// Counter-based random streams for the native quantile generators.
//
// Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed; the counter carries
// (row, column, purpose), so every (row, column) draw is independent of launch geometry
// and of how rows are sharded across GPUs.
//
// The LHS permutation of column c is a keyed bijection of [0, n): a mixed-radix Feistel
// network on [0, A B) with A B just above n, restricted to [0, n) by cycle walking (Black &
// Rogaway 2002).  Both directions are cheap, so a row's stratum and a stratum's row are
// computed, never stored.
#pragma once

#include <math.h>

#include "pbh_common.h"

namespace pbh {

struct Philox {
  uint32_t k0, k1;
  PBH_HD explicit Philox(uint64_t seed) : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)) {}

  PBH_HD static inline void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
  }

  // 10 rounds on counter c[0..3]; returns 4 words in c.
  PBH_HD inline void operator()(uint32_t c[4]) const {
    uint32_t a0 = k0, a1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      uint32_t hi0, lo0, hi1, lo1;
      mulhilo(0xD2511F53u, c[0], hi0, lo0);
      mulhilo(0xCD9E8D57u, c[2], hi1, lo1);
      uint32_t n0 = hi1 ^ c[1] ^ a0;
      uint32_t n2 = hi0 ^ c[3] ^ a1;
      c[0] = n0;
      c[1] = lo1;
      c[2] = n2;
      c[3] = lo0;
      a0 += 0x9E3779B9u;
      a1 += 0xBB67AE85u;
    }
  }

  // Uniform double in [0, 1) with 53 random bits: (u64 >> 11) * 2^-53 (numpy's next_double).
  PBH_HD inline double uniform(uint64_t row, uint32_t col, uint32_t purpose) const {
    uint32_t c[4] = {(uint32_t)row, (uint32_t)(row >> 32), col, purpose};
    (*this)(c);
    uint64_t u = ((uint64_t)c[1] << 32) | c[0];
    return (double)(u >> 11) * 0x1.0p-53;
  }
};

enum : uint32_t {
  kPurposeLhsU = 0x4C485355u,   // 'LHSU'
  kPurposeFeistel = 0x46454953u,  // 'FEIS'
  kPurposeUniform = 0x50524E47u   // 'PRNG'
};

PBH_HD inline uint32_t mix32(uint32_t x) {  // lowbias32 finalizer
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Keyed bijection of [0, n): an alternating Feistel network over the mixed radix
// Z_A x Z_B (A = ceil(sqrt(n)), B = ceil(n / A), so n <= A B < n + A), with modular addition
// (Black & Rogaway 2002, the FE2 construction of format-preserving encryption): x = L B + R,
// even rounds L <- (L + F(R)) mod A, odd rounds R <- (R + F(L)) mod B.  Every round is a
// bijection of its half, so the network is a bijection of [0, A B); values >= n are cycle-
// walked, which happens with probability < 1 / B (~1e-4 at n = 1e8), so a SIMD lane almost
// never waits on a neighbour's walk -- unlike a power-of-two domain, where 2^b can be ~2n and
// the wave-wide maximum walk count is ~4.  F = lowbias32 of (half XOR round key), reduced to
// the radix by a multiply-high (Lemire): 3 32-bit multiplies (quarter-rate on CDNA) per round,
// 4 rounds (Luby-Rackoff: a pseudo-random permutation from 4 rounds of pseudo-random round
// functions).  The van der Waerden scores kernel evaluates this network once per element and is
// VALU-issue bound (87% VALU-busy with the round-1 network of 6 rounds and a premultiply, 24
// multiplies): the network is most of its instructions.  tests/test_streams_host.py checks the
// permutation statistically on the host (rank correlations across columns, with the row index
// and along rows; the jitter's uniformity).
struct FeistelPerm {
  static constexpr int kRounds = 4;
  uint64_t n;
  uint32_t A, B;
  double inv_b;
  bool small;  // A B < 2^32: split / join in 32 bits
  uint32_t rk[kRounds];

  PBH_HD FeistelPerm(const Philox& ph, uint64_t n_, uint32_t col) : n(n_) {
    uint64_t a = (uint64_t)sqrt((double)n_);  // A = ceil(sqrt(n)): sqrt, then at most a step or two
    if (a == 0) a = 1;
    while (a * a < n_) ++a;
    while (a > 1 && (a - 1) * (a - 1) >= n_) --a;
    A = (uint32_t)a;
    B = (uint32_t)((n_ + A - 1) / A);
    if (B == 0) B = 1;
    inv_b = 1.0 / (double)B;
    small = (uint64_t)A * B + B <= 0xFFFFFFFFull && A < (1u << 24) && B < (1u << 24);  // q B (q off by one) fits too
    uint32_t c[4] = {col, 0u, 0u, kPurposeFeistel};
    ph(c);
    for (int i = 0; i < kRounds; ++i) rk[i] = c[i];
  }

  PBH_HD static inline uint32_t reduce(uint32_t h, uint32_t m) { return (uint32_t)(((uint64_t)h * m) >> 32); }
  PBH_HD inline uint32_t F(uint32_t v, uint32_t k) const { return mix32(v ^ k); }

  PBH_HD static inline uint32_t mul24(uint32_t a, uint32_t b) {  // a, b < 2^24, a b < 2^32
#ifdef __HIP_DEVICE_COMPILE__
    return __umul24(a, b);  // v_mul_u32_u24: full rate (a 32-bit multiply is quarter rate)
#else
    return a * b;
#endif
  }

  PBH_HD inline void split(uint64_t x, uint32_t& L, uint32_t& R) const {
    // x < 2^32 and the product's relative error is ~1e-16, so q is off by at most one:
    // one branch-free correction each way (keeps independent evaluations interleavable)
    if (small) {  // A B < 2^32 (every n < 2^32 but the last ~2^16): 32-bit, 24-bit multiplies
      const uint32_t x32 = (uint32_t)x;
      uint32_t q = (uint32_t)((double)x32 * inv_b);
      uint32_t qb = mul24(q, B);
      const bool lo = qb > x32;
      q -= lo ? 1u : 0u;
      qb -= lo ? B : 0u;
      const bool hi = x32 - qb >= B;
      q += hi ? 1u : 0u;
      qb += hi ? B : 0u;
      L = q;
      R = x32 - qb;
      return;
    }
    uint64_t q = (uint64_t)((double)x * inv_b);
    q -= (q * B > x) ? 1 : 0;
    q += (x - q * B >= B) ? 1 : 0;
    L = (uint32_t)q;
    R = (uint32_t)(x - q * B);
  }

  PBH_HD inline uint64_t join(uint32_t L, uint32_t R) const {
    return small ? (uint64_t)(mul24(L, B) + R) : (uint64_t)L * B + R;
  }

  PBH_HD inline uint64_t round_trip(uint64_t x) const {
    uint32_t L, R;
    split(x, L, R);
#pragma unroll
    for (int i = 0; i < kRounds; ++i) {
      if (i & 1) {
        const uint32_t h = reduce(F(L, rk[i]), B);
        R = R + h >= B ? R + h - B : R + h;
      } else {
        const uint32_t h = reduce(F(R, rk[i]), A);
        L = L + h >= A ? L + h - A : L + h;
      }
    }
    return join(L, R);
  }

  PBH_HD inline uint64_t round_trip_inv(uint64_t y) const {
    uint32_t L, R;
    split(y, L, R);
#pragma unroll
    for (int i = kRounds - 1; i >= 0; --i) {
      if (i & 1) {
        const uint32_t h = reduce(F(L, rk[i]), B);
        R = R >= h ? R - h : R + B - h;
      } else {
        const uint32_t h = reduce(F(R, rk[i]), A);
        L = L >= h ? L - h : L + A - h;
      }
    }
    return join(L, R);
  }

  // Bijection of [0, n) by cycle walking.
  PBH_HD inline uint64_t operator()(uint64_t x) const {
    if (n <= 1) return 0;
    do {
      x = round_trip(x);
    } while (x >= n);
    return x;
  }
  PBH_HD inline uint64_t inverse(uint64_t y) const {
    if (n <= 1) return 0;
    do {
      y = round_trip_inv(y);
    } while (y >= n);
    return y;
  }
};

// q = (perm + 1 - u) / n: scipy's `(perms - samples) / n` with perms in 1..n
// (scipy:stats/_qmc.py LatinHypercube._random_lhs).  The jitter u is keyed by the stratum
// perm (not the row): the point of row r is stratum pi(r) with that stratum's jitter, which
// is as random as a per-row jitter (pi is a random bijection) and lets the stratum-ordered
// (sorted) column be generated without evaluating pi^-1 at all (lhs_sorted_quantile).
//
// The jitter is output t of a SplitMix64 generator (Steele, Lea & Flood, OOPSLA 2014; Java's
// SplittableRandom) whose start is keyed by (seed, column): z = key + (t + 1) * golden gamma,
// then the Stafford "mix13" finalizer.  It is evaluated once per element by the stratum-ordered
// generator and again, in random stratum order, by the step-4 placement, so its cost matters:
// 11 32-bit multiplies (quarter-rate on CDNA) against 40 for a Philox4x32-10 block, whose other
// 75 bits a single jitter would throw away.  The permutation keeps its Feistel network.
PBH_HD inline uint64_t splitmix_finalize(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

PBH_HD inline uint64_t lhs_jitter_key(const Philox& ph, uint32_t col) {
  const uint64_t seed = ((uint64_t)ph.k1 << 32) | ph.k0;
  return splitmix_finalize(seed ^ splitmix_finalize(((uint64_t)col << 32) | kPurposeLhsU));
}

PBH_HD inline double lhs_sorted_quantile(const Philox& ph, uint64_t t, uint32_t col, uint64_t n) {
#ifdef PBH_JITTER_PHILOX  // the round-1 jitter (A/B builds only)
  const double u = ph.uniform(t, col, kPurposeLhsU);
#else
  const uint64_t z = splitmix_finalize(lhs_jitter_key(ph, col) + (t + 1) * 0x9E3779B97F4A7C15ull);
  const double u = (double)(z >> 11) * 0x1.0p-53;
#endif
  return ((double)(t + 1) - u) / (double)n;
}

PBH_HD inline double lhs_quantile(const Philox& ph, const FeistelPerm& fp, uint64_t row, uint32_t col) {
  return lhs_sorted_quantile(ph, fp(row), col, fp.n);
}

}  // namespace pbh
