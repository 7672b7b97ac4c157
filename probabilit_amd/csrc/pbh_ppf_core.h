// Device pieces of the inverse-CDF kernels shared by pbh_ppf.hip and pbh_dag.hip: the
// per-element ppf of the base distributions, the ndtri tail queue, and the Sobol' point tables.
#pragma once
#include <math.h>

#include "pbh_cdflib.h"
#include "pbh_error.h"
#include "pbh_special.h"

namespace pbh {
namespace {

constexpr int kPpfBlock = 256;
constexpr double kInf = sf::kInf;
constexpr double kNaN = sf::kNaN;

struct Params {
  const double* ptr[3];
  double val[3];
  PBH_DI double at(int j, int64_t i) const { return ptr[j] ? ptr[j][i] : val[j]; }
};

// Per-launch constants of the distribution (scalar parameters only).
constexpr int kPoissonGuideBits = 11;  // 2048 guide buckets

struct PoissonTable {
  const double* cdf;  // poisson: cdf[j] = pdtr(k_lo + j, mu) for scalar mu, else NULL
  const double* win;  // win[j] = cdf::poisson_window_hi(k_lo + j, mu): scipy's window above cdf[j - 1]
  const int32_t* cdf_guide;  // cdf_guide[b] = first j with cdf[j] >= b / 2^kPoissonGuideBits
  int64_t k_lo;
  int64_t len;
  int has_gamma;      // gamma with scalar a: hoisted GammaAux + z-grid guide
  sf::GammaAux aux;
  sf::GammaGuide guide;
};

// smallest k >= 0 with pdtr(k, mu) >= q, by stepping from a Cornish-Fisher guess.
PBH_DI double poisson_definition_search(double q, double mu) {
  if (mu == 0.0) return 0.0;
  double z = sf::ndtri(q);  // a starting guess only (the search decides k)
  double g = floor(mu + sqrt(mu) * z + (z * z - 1.0) / 6.0);
  if (!(g >= 0.0)) g = 0.0;
  if (g > 9.0e15) g = 9.0e15;
  double k = g;
  if (sf::pdtr<glibc::Math>(k, mu) >= q) {
    while (k > 0.0 && sf::pdtr<glibc::Math>(k - 1.0, mu) >= q) k -= 1.0;
  } else {
    do {
      k += 1.0;
    } while (sf::pdtr<glibc::Math>(k, mu) < q && k < 1.0e18);
  }
  return k;
}

// The rare poisson lanes, one call site per kernel (a real call: its code does not size the
// callers' registers).  k < 0: q lies outside the CDF table (or there is none), so the
// definition is searched first.  Then, when q lies in the window just above pdtr(k - 1, mu) where
// scipy's pdtrik-based ppf can answer k - 1 (pbh_cdflib.h), scipy's computation itself decides.
__attribute__((noinline)) __device__ double poisson_rare(double q, double mu, double k) {
  if (q < cdf::kPoissonDeepTail) return cdf::poisson_ppf_scipy(q, mu);  // scipy's deep tail (pbh_cdflib.h)
  if (k < 0.0) k = poisson_definition_search(q, mu);
  if (k >= 1.0 && q < cdf::poisson_window_hi(k, mu)) return cdf::poisson_ppf_scipy(q, mu);
  return k;
}

// scipy's poisson ppf (before loc) from the CDF table: the first j with cdf[j] >= q by the guide
// table (Chen & Asau 1974: q lies in bucket b = floor(q 2^bits), exact for a power-of-two scale,
// whose guide entry is the answer for q = b / 2^bits <= q, so a short forward scan from it ends at
// the answer -- the same j as a binary search over the table, in ~1 probe instead of log2(len)
// dependent ones), i.e. the smallest k with pdtr(k, mu) >= q; lanes outside the table or inside
// scipy's window above cdf[j - 1] (win[j], a few 1e-10 of the quantile) take poisson_rare.
PBH_DI double poisson_from_table(double q, double mu, const PoissonTable& t) {
  int64_t lo = t.cdf_guide[(int)(q * (double)(1 << kPoissonGuideBits))];
  while (lo < t.len && t.cdf[lo] < q) ++lo;
  const bool outside = lo == t.len || (lo == 0 && t.k_lo > 0);
  double k = (double)(t.k_lo + lo);
  if (outside || q < t.win[lo] || q < cdf::kPoissonDeepTail) k = poisson_rare(q, mu, outside ? -1.0 : k);
  return k;
}

// poisson_from_table without poisson_rare: false when the lane needs it (outside the table, inside
// a window, the deep tail).  The sweep kernels list such lanes for k_ppf_poisson_slow instead of
// calling it, so no call -- and no stack frame for cdflib's search -- sits in their loop (the call
// alone took the 1e8-row sweep at mu = 30 from 0.375 to 0.504 ms, profiles/r06/ppf_sweep_ab_r6pa.log).
PBH_DI bool poisson_table_fast(double q, const PoissonTable& t, double* k) {
  int64_t lo = t.cdf_guide[(int)(q * (double)(1 << kPoissonGuideBits))];
  while (lo < t.len && t.cdf[lo] < q) ++lo;
  const bool outside = lo == t.len || (lo == 0 && t.k_lo > 0);
  if (outside || q < t.win[lo] || q < cdf::kPoissonDeepTail) return false;
  *k = (double)(t.k_lo + lo);
  return true;
}

// log_tab's table staged in LDS without its padding column (3 KiB): ndtri's tail reads two random
// entries per draw, up to 32 cache lines per wave load from the global copy
constexpr int kLog3N = 128 * 3;
PBH_DI void stage_log3(double* lt) {
  for (int k = threadIdx.x; k < kLog3N; k += blockDim.x) lt[k] = (&sf::pbh_log_tab[0][0])[4 * (k / 3) + k % 3];
}
// The normal quantile of norm / lognorm is Wichura's PPND16 (sf::ppnd16: half the FP64 work of
// Cephes' ndtri, within 1.1e-15 of scipy's ndtri).  scale z and exp(s z) scale keep that relative
// error; loc + (those) does not where it cancels -- norm(5, 2) near x = 0 -- so an element whose
// result lies within 2^-12 of its cancelling parts takes Cephes' ndtri instead, bit for bit with
// scipy (normal_guard): the result stays within ~5e-12 of scipy's everywhere, inside the 1e-10
// gate.  The same function in every kernel: the sorted generator, the placement, the certificate
// and the plain ppf agree.
template <int D>
PBH_DI double normal_loc(double p0, double p1) {
  return D == PBH_DIST_NORM ? p0 : p1;
}
PBH_DI bool normal_takes_tail(double q, double /*loc*/) { return sf::ppnd16_takes_tail(q); }
PBH_DI double tail_of(double q, const double* lt) {
#ifdef PBH_NO_LDS_LOGEXP  // A/B build: the global table
  return sf::ppnd16_tail(q);
#else
  return lt ? sf::ppnd16_tail_at<3>(q, lt) : sf::ppnd16_tail(q);
#endif
}
// z = PPND16's quantile, v = its scaled value (scale z, or exp(s z) scale), m = the magnitude its
// error is relative to (|v|, or s |z| |v| for lognorm): true when loc + v keeps that error within
// 2^-12 of itself, i.e. PPND16's result is inside the gate; false sends the element to ndtri
PBH_DI bool normal_guard(double v, double m, double loc) {
  return loc == 0.0 || fabs(v + loc) >= 0x1p-12 * m;
}

// ppf of one element for distribution D; p = (shape..., loc, scale) already resolved.
// PART selects the normal quantile's branch for norm / lognorm (0: whole, 1: centre, 2: tail of
// PPND16; normal_takes_tail; normal_guard's rare elements take ndtri whole),
// for the compacted kernels that know which one an element takes.
// COLD_GAMMA: igami_guided's fallbacks as a call (see igami_guided)
// lt: for PART 2, log_tab's table in LDS with entry stride 3 (stage_log3), else the global table
// ppf_one<PBH_DIST_POISSON> (below) on the table alone: false leaves *x unset and sends the element
// to the slow list (then ppf_one itself evaluates it: the same value)
PBH_DI bool poisson_ppf_fast(double q, double mu, double loc, const PoissonTable& t, double* x) {
  const bool cond0 = (mu >= 0.0) && (loc == loc);
  if (q == 0.0) {
    *x = -1.0 + loc;
  } else if (cond0 && q == 1.0) {
    *x = kInf + loc;
  } else if (cond0 && q > 0.0 && q < 1.0) {
    double k;
    if (!poisson_table_fast(q, t, &k)) return false;
    *x = k + loc;
  } else {
    *x = kNaN;
  }
  return true;
}

template <int D, int PART = 0, bool COLD_GAMMA = false>
PBH_DI double ppf_one(double q, double p0, double p1, double p2, const PoissonTable& pt, const double* lt = nullptr) {
  if constexpr (D == PBH_DIST_POISSON) {
    double mu = p0, loc = p1;
    bool cond0 = (mu >= 0.0) && (loc == loc);
    if (q == 0.0) return -1.0 + loc;
    if (cond0 && q == 1.0) return kInf + loc;
    if (cond0 && q > 0.0 && q < 1.0) {
      double k = pt.cdf ? poisson_from_table(q, mu, pt) : poisson_rare(q, mu, -1.0);
      return k + loc;
    }
    return kNaN;
  } else {
    double shape = 0.0, loc, scale;
    bool arg_ok = true;
    double lower = 0.0, upper = kInf;
    if constexpr (D == PBH_DIST_NORM || D == PBH_DIST_UNIFORM || D == PBH_DIST_EXPON) {
      loc = p0;
      scale = p1;
    } else {
      shape = p0;
      loc = p1;
      scale = p2;
    }
    if constexpr (D == PBH_DIST_NORM) lower = -kInf;
    if constexpr (D == PBH_DIST_UNIFORM || D == PBH_DIST_TRIANG) upper = 1.0;
    if constexpr (D == PBH_DIST_TRIANG) arg_ok = (shape >= 0.0) && (shape <= 1.0);
    if constexpr (D == PBH_DIST_GAMMA || D == PBH_DIST_LOGNORM) arg_ok = shape > 0.0;
    bool cond0 = arg_ok && (scale > 0.0) && (loc == loc);
    if (!cond0) return kNaN;
    if (q == 0.0) return lower * scale + loc;
    if (q == 1.0) return upper * scale + loc;
    if (!(q > 0.0 && q < 1.0)) return kNaN;
    double x;
    if constexpr (D == PBH_DIST_NORM) {
      x = PART == 1 ? sf::ppnd16_centre(q) : PART == 2 ? tail_of(q, lt) : sf::ppnd16(q);
      const bool ok = normal_guard(x * scale, fabs(x * scale), loc);
      if (!sf::wave_all(ok)) {  // cancellation near x = 0: Cephes' ndtri, bit for bit
        if (!ok) x = sf::ndtri(q);
        sf::rare_path_end();
      }
    } else if constexpr (D == PBH_DIST_UNIFORM) {
      x = q;
    } else if constexpr (D == PBH_DIST_EXPON) {
      x = -sf::log1p_(-q);  // scipy expon._ppf: -sc.log1p(-q), the Cephes log1p
    } else if constexpr (D == PBH_DIST_LOGNORM) {
      const double z = PART == 1 ? sf::ppnd16_centre(q) : PART == 2 ? tail_of(q, lt) : sf::ppnd16(q);
      x = exp(shape * z);
      const double v = x * scale;
      const bool ok = normal_guard(v, fabs(v) * (1.0 + shape * fabs(z)), loc);
      if (!sf::wave_all(ok)) {
        if (!ok) x = exp(shape * sf::ndtri(q));
        sf::rare_path_end();
      }
    } else if constexpr (D == PBH_DIST_TRIANG) {
      // np.where(q < c, sqrt(c q), 1 - sqrt((1 - c)(1 - q)))
      x = (q < shape) ? sqrt(shape * q) : 1.0 - sqrt((1.0 - shape) * (1.0 - q));
    } else {  // gamma
      x = pt.has_gamma ? sf::igami_guided<COLD_GAMMA>(shape, q, &pt.aux, pt.guide) : sf::igami(shape, q);
    }
    return x * scale + loc;
  }
}

// ---------------------------------------------------------------- tail compaction
// ndtri (norm / lognorm ppf, the van der Waerden scores) is one rational function for
// min(q, 1 - q) > e^-2 (73% of uniform q) and an expensive tail (two logs, a sqrt, three
// divisions) otherwise.  With q in random order nearly every wave holds both kinds, and a wave
// executes every branch one of its lanes takes, so a plain grid-stride kernel pays centre + tail
// for every element.  The compacted kernels give each thread kCIpt items of a block tile: centre
// items are evaluated at once, tail items are queued in LDS (one LDS atomic per wave) and then
// drained by all lanes of the block together, so the tail costs its 27% share.  Every value is
// computed by the same inline function either way (bit-identical to the plain kernels); the
// results pass through LDS so that the global stores stay coalesced.
constexpr int kCIpt = 8;
constexpr int kCTile = kPpfBlock * kCIpt;

struct TailQueue {
  double arg[kCTile];
  uint16_t pos[kCTile];
  int count;
};

template <class Queue>  // TailQueue, or a smaller queue with the same members
PBH_DI void tail_push(Queue& tq, bool take, double a, int p) {
  const uint64_t m = __ballot(take);
  if (m == 0ull) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if (lane == leader) base = atomicAdd(&tq.count, (int)__popcll(m));
  base = __shfl(base, leader, 64);
  if (take) {
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int slot = base + (int)__popcll(m & lt);
    tq.arg[slot] = a;
    tq.pos[slot] = (uint16_t)p;
  }
}

// x(r) = shift XOR (the direction numbers of the set bits of gray(r) = r ^ (r >> 1)), by four
// 256-entry tables of the XORs over each byte of gray(r) (built in LDS per block): 4 lookups per
// point instead of a loop over ~15 set bits.  Identical values (XOR is associative).
PBH_DI void build_sobol_tables(const uint32_t* sv, uint32_t* T) {
  for (int t = threadIdx.x; t < 256; t += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b)
        if ((t >> b) & 1) v ^= sv[8 * k + b];
      T[k * 256 + t] = v;
    }
  }
}

PBH_DI uint32_t sobol_point(const uint32_t* T, uint32_t shift, uint64_t r) {
  const uint32_t g = (uint32_t)(r ^ (r >> 1));  // r < 2^bits <= 2^32
  return shift ^ T[g & 255u] ^ T[256 + ((g >> 8) & 255u)] ^ T[512 + ((g >> 16) & 255u)] ^ T[768 + (g >> 24)];
}

}  // namespace
}  // namespace pbh
