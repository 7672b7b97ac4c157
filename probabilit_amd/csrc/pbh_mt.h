// numpy's bit generators, restated for index-addressed generation on the GPU.
//
// MT19937 (numpy/random/src/mt19937/mt19937.c, the bit generator behind np.random.RandomState,
// i.e. behind check_random_state(int | None).random((size, d)) at modeling.py:484-486):
//   * key_{b+1} = twist(key_b) (mt19937_gen), output = temper(key_b[pos]);
//   * random_sample: a = next32 >> 5, b = next32 >> 6, (a * 2^26 + b) * 2^-53.
// The untempered word sequence x_g (x_0..x_623 = the key block numpy holds) is an F2-linear
// recurrence on a 19937-bit state (x_g's top bit, x_{g+1..g+623}).  A window
// W_g = (x_g .. x_{g+623}) is moved forward by J words with the jump polynomial
// p_J(x) = x^J mod phi(x) (phi = characteristic polynomial, found here by Berlekamp-Massey;
// Haramoto, Matsumoto, Nishimura, Panneton, L'Ecuyer 2008): W_{g+J} = sum_i p_J[i] W_{g+i}.
// Only the 19937 state bits are exact after a jump, so a jump lands on g - 1 and the caller
// steps once (see mt_fill in pbh_streams.hip).
//
// PCG64 (numpy/random/src/pcg64/pcg64.h): 128-bit LCG s' = s * M + inc, output
// xsl_rr(s') = rotr64(hi ^ lo, s' >> 122) of the new state; next_double = (u64 >> 11) * 2^-53.
// Jump ahead by k draws: s_k = A_k s + C_k, tabulated for k = 2^i.
#pragma once

#include <string.h>

#include <vector>

#include "pbh_common.h"

namespace pbh {
namespace mt {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
constexpr int kDeg = 19937;
constexpr int kPolyWords = 312;              // 19968 bits >= kDeg + 1
constexpr int kChunks = (kDeg + kN - 1) / kN;  // 32 chunks of 624 coefficients
constexpr int kJumpBits = 44;                // jump polynomials x^(2^i), i < 44 (2^44 words)

PBH_HD inline uint32_t temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

// x_{g+624} from x_g (top bit), x_{g+1} (low bits), x_{g+397}
PBH_HD inline uint32_t next_word(uint32_t xg, uint32_t xg1, uint32_t xg397) {
  const uint32_t y = (xg & kUpper) | (xg1 & kLower);
  return xg397 ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
}

// numpy's mt19937_gen on a key block: W_g -> W_{g+624}, in place.
PBH_HD inline void twist(uint32_t* w) {
  for (int i = 0; i < kN; ++i) w[i] = next_word(w[i], w[(i + 1) % kN], w[(i + kM) % kN]);
}

PBH_HD inline double next_double(uint32_t t0, uint32_t t1) {  // tempered words, in draw order
  const uint32_t a = t0 >> 5, b = t1 >> 6;
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

// ---------------------------------------------------------------- host: F2[x] arithmetic
// Polynomials over F2 as little-endian 64-bit words (bit i = coefficient of x^i).
namespace host {

inline void init_genrand(uint32_t s, uint32_t* key) {  // Matsumoto & Nishimura's seeding
  key[0] = s;
  for (int i = 1; i < kN; ++i) key[i] = 1812433253u * (key[i - 1] ^ (key[i - 1] >> 30)) + (uint32_t)i;
}

inline uint64_t get_bits64(const std::vector<uint64_t>& v, int64_t bit) {
  const int64_t w = bit >> 6;
  const int s = (int)(bit & 63);
  const uint64_t lo = w < (int64_t)v.size() ? v[w] : 0;
  if (s == 0) return lo;
  const uint64_t hi = w + 1 < (int64_t)v.size() ? v[w + 1] : 0;
  return (lo >> s) | (hi << (64 - s));
}

// Characteristic polynomial phi (degree kDeg, kPolyWords words) of the word recurrence:
// Berlekamp-Massey on bit 0 of x_{g+1}, g = 0 .. 2 kDeg + 63 (phi is primitive, so any
// nonzero linear functional of the state has minimal polynomial phi).
inline bool charpoly(std::vector<uint64_t>& phi) {
  const int64_t nbits = 2 * (int64_t)kDeg + 64;
  std::vector<uint32_t> key(kN);
  init_genrand(5489u, key.data());
  std::vector<uint8_t> s(nbits);
  int64_t filled = 0;
  int idx = 1;  // x_1 .. x_623 of the first block, then whole blocks
  while (filled < nbits) {
    for (; idx < kN && filled < nbits; ++idx) s[filled++] = key[idx] & 1u;
    twist(key.data());
    idx = 0;
  }
  // reversed sequence: rs bit j = s[nbits - 1 - j]
  const int words = (int)((nbits + 63) / 64) + 2;
  std::vector<uint64_t> rs(words, 0);
  for (int64_t j = 0; j < nbits; ++j)
    if (s[nbits - 1 - j]) rs[j >> 6] |= 1ull << (j & 63);
  const int cw = kPolyWords + 2;
  std::vector<uint64_t> C(cw, 0), B(cw, 0), T(cw);
  C[0] = B[0] = 1;
  int64_t L = 0, m = 1;
  for (int64_t n = 0; n < nbits; ++n) {
    // d = sum_{i=0..L} c_i s_{n-i} = parity(C & rs[nbits-1-n ...])
    const int64_t off = nbits - 1 - n;
    uint64_t acc = 0;
    const int lw = (int)(L >> 6);
    for (int w = 0; w <= lw; ++w) {
      uint64_t cwd = C[w];
      if (w == lw) cwd &= (L & 63) == 63 ? ~0ull : ((2ull << (L & 63)) - 1);
      acc ^= cwd & get_bits64(rs, off + 64 * (int64_t)w);
    }
    if (!__builtin_parityll(acc)) {
      ++m;
      continue;
    }
    const bool grow = 2 * L <= n;
    if (grow) T = C;
    const int ws = (int)(m >> 6), bs = (int)(m & 63);
    for (int w = 0; w + ws < cw; ++w) {
      C[w + ws] ^= B[w] << bs;
      if (bs && w + ws + 1 < cw) C[w + ws + 1] ^= B[w] >> (64 - bs);
    }
    if (grow) {
      L = n + 1 - L;
      B = T;
      m = 1;
    } else {
      ++m;
    }
  }
  if (L != kDeg) return false;
  phi.assign(kPolyWords, 0);
  for (int64_t i = 0; i <= L; ++i)
    if ((C[i >> 6] >> (i & 63)) & 1ull) phi[(L - i) >> 6] |= 1ull << ((L - i) & 63);
  return true;
}

// a^2 mod phi (a: degree < kDeg)
inline void square_mod(const std::vector<uint64_t>& a, const std::vector<uint64_t>& phi, std::vector<uint64_t>& out) {
  std::vector<uint64_t> p(2 * kPolyWords + 2, 0);
  for (int w = 0; w < kPolyWords; ++w) {
    uint64_t v = a[w];
    uint64_t lo = 0, hi = 0;
    for (int b = 0; b < 32; ++b) {
      lo |= ((v >> b) & 1ull) << (2 * b);
      hi |= ((v >> (b + 32)) & 1ull) << (2 * b);
    }
    p[2 * w] = lo;
    p[2 * w + 1] = hi;
  }
  for (int64_t k = 2 * (int64_t)(kDeg - 1); k >= kDeg; --k) {
    if (!((p[k >> 6] >> (k & 63)) & 1ull)) continue;
    const int64_t sh = k - kDeg;
    const int ws = (int)(sh >> 6), bs = (int)(sh & 63);
    for (int w = 0; w < kPolyWords; ++w) {
      p[w + ws] ^= phi[w] << bs;
      if (bs) p[w + ws + 1] ^= phi[w] >> (64 - bs);
    }
  }
  out.assign(p.begin(), p.begin() + kPolyWords);
}

// jump[i] = x^(2^i) mod phi, i < kJumpBits, flattened (kJumpBits x kPolyWords).
inline bool jump_table(std::vector<uint64_t>& table) {
  std::vector<uint64_t> phi;
  if (!charpoly(phi)) return false;
  table.assign((size_t)kJumpBits * kPolyWords, 0);
  std::vector<uint64_t> cur(kPolyWords, 0), nxt;
  cur[0] = 2;  // x
  for (int i = 0; i < kJumpBits; ++i) {
    memcpy(&table[(size_t)i * kPolyWords], cur.data(), kPolyWords * 8);
    square_mod(cur, phi, nxt);
    cur.swap(nxt);
  }
  return true;
}

// W <- sum_i p[i] W_{+i}: the jump as the device kernel computes it (chunked Horner in
// T^624 with the 1248-word extended window), for host tests.
inline void apply_jump(uint32_t* w, const uint64_t* p) {
  uint32_t E[2 * kN], acc[kN];
  memcpy(E, w, kN * 4);
  memcpy(E + kN, w, kN * 4);
  twist(E + kN);
  memset(acc, 0, sizeof(acc));
  for (int q = kChunks - 1; q >= 0; --q) {
    twist(acc);
    for (int r = 0; r < kN; ++r) {
      const int64_t bit = (int64_t)kN * q + r;
      if (!((p[bit >> 6] >> (bit & 63)) & 1ull)) continue;
      for (int m = 0; m < kN; ++m) acc[m] ^= E[r + m];
    }
  }
  memcpy(w, acc, sizeof(acc));
}

}  // namespace host
}  // namespace mt

namespace pcg {

typedef unsigned __int128 u128;
constexpr u128 kMult = ((u128)0x2360ED051FC65DA4ull << 64) | (u128)0x4385DF649FCCF645ull;

PBH_HD inline uint64_t output(u128 s) {
  const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
  const unsigned rot = (unsigned)(s >> 122);
  const uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

PBH_HD inline double to_double(uint64_t v) { return (double)(v >> 11) * (1.0 / 9007199254740992.0); }

// (A, C) for 2^i steps, i < 64: table[2 i] = A, table[2 i + 1] = C
PBH_HD inline void jump_table(u128 inc, u128* table) {
  u128 a = kMult, c = inc;
  for (int i = 0; i < 64; ++i) {
    table[2 * i] = a;
    table[2 * i + 1] = c;
    c = c * (a + 1);
    a = a * a;
  }
}

PBH_HD inline u128 advance(u128 s, uint64_t k, const u128* table) {
  for (int i = 0; k; ++i, k >>= 1)
    if (k & 1) s = table[2 * i] * s + table[2 * i + 1];
  return s;
}

}  // namespace pcg
}  // namespace pbh
