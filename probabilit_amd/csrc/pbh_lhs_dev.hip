// The reference LHS stream's d Fisher-Yates shuffles decoded on the device (round 5).
//
// scipy's LatinHypercube(d, rng).random(n) (modeling.py:480,488 -> scipy:stats/_qmc.py
// _random_lhs) shuffles d rows of arange(1, n + 1) with numpy's Generator.shuffle: for
// i = n-1 .. 1, j_i = random_interval(i) (draw 32-bit halves of PCG64 outputs until
// (w & mask(i)) <= i), swap x[i], x[j_i].  The rejections make it one sequential stream: a
// draw's fate depends on how many steps came before it.  Here it is decoded in parallel and
// checked exactly:
//
//   classify  every draw (generated in place by PCG64 jump-ahead) against the band of states
//             the column can be in at that draw: the expected steps done +- ksig standard
//             deviations (closed forms over each mask range, band_table).  A draw whose
//             decision is the same for every state of the band is decided; the rest
//             (~1e-3 of the bulk, the whole column tail) are "ambiguous"
//   walk      the ambiguous draws, in order, on the host: state = decided accepts before the
//             draw + ambiguous accepts so far (a few 10^4 per column at n = 1e7)
//   finish    every decision re-checked against the rule at the state its prefix implies
//             (one block scan): all agree <=> the decode is the sequential one, by induction.
//             The accepted draws give the swap targets j_i; the column's last accept gives
//             the next column's first draw.  A disagreement (a state outside its band) retries
//             with a band twice as wide, then hands the call back to the host shuffles.
//
// The swaps themselves are not replayed.  Position p holds p + 1 until the first step (in
// time: the largest i) that targets it; step i writes the value position j_i held just before
// it into x[i], which is final from then on.  With S(i) = the next step after i (in time) with
// the same target and M(q) = the first step to target position q from above, the value q held
// before its own step is V(q) = V(M(q)), or q + 1 when nothing targeted it, and
//   x[i] = V(S(i)) (or j_i + 1 when S(i) is none),   x[0] = V(M(0)) (or 1).
// A stable radix sort of the steps by target (the library's one-sweep passes), one pass to link
// each group, then per row one pointer chase from the position it reads: O(n) work, no
// sequential pass.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "pbh_error.h"
#include "pbh_lhs_dev.h"
#include "pbh_sort.h"
#include "probabilit_hip.h"
#include "pbh_timing.h"

namespace pbh {

// band half-width in standard deviations (pbh_lhs_reference_band) and the last call's record
static double g_band_sigmas = 6.0;
static int32_t g_last_attempts = 0, g_last_device = 0;
static int64_t g_last_ambiguous = 0;

namespace {

using pcg::u128;

constexpr int kT = 256, kPer = 16, kBlk = kT * kPer;  // draws per block
constexpr int kBandLog = 10;                           // band table spacing: 1024 draws
constexpr int kAttempts = 3;
enum : uint8_t { kRej = 0, kAcc = 1, kAmb = 2 };

PBH_HD inline uint32_t mask_of(uint32_t x) {
  x |= x >> 1;
  x |= x >> 2;
  x |= x >> 4;
  x |= x >> 8;
  x |= x >> 16;
  return x;
}

struct DecParams {
  uint64_t s_lo, s_hi, inc_lo, inc_hi;  // PCG64 state before the uniforms; increment
  uint64_t base;                        // 64-bit outputs before the shuffles (the n d uniforms)
  int32_t h;                            // 1: a buffered 32-bit half comes first (has_uint32)
  uint32_t buf32;
  int64_t n;      // steps i = n-1 .. 1 per column
  int64_t tcap;   // draws classified per column (nb * kBlk)
  int64_t nb;     // blocks per column
  int64_t nband;  // band table entries
};

// exclusive scan over a 256-thread block; *total = the block's sum
__device__ __forceinline__ uint32_t scan256(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kT / 64; ++i) {
    const uint32_t t = sh[i];
    pre += i < w ? t : 0u;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

// ---------------------------------------------------------------- scans
// one block per array (blockIdx.x): out[0 .. m] = exclusive prefix of in[0 .. m), out[m] = sum
__global__ __launch_bounds__(1024) void k_scan_small(const uint32_t* __restrict__ in, int64_t m, int64_t in_stride,
                                                     uint32_t* __restrict__ out, int64_t out_stride) {
  __shared__ uint32_t sh[16];
  in += blockIdx.x * in_stride;
  out += blockIdx.x * out_stride;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t per = (m + 1023) / 1024;
  const int64_t a = std::min<int64_t>(m, t * per), b = std::min<int64_t>(m, a + per);
  uint32_t sum = 0;
  for (int64_t i = a; i < b; ++i) sum += in[i];
  uint32_t x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = x;
  __syncthreads();
  uint32_t run = x - sum;
  for (int i = 0; i < w; ++i) run += sh[i];
  for (int64_t i = a; i < b; ++i) {
    const uint32_t v = in[i];
    out[i] = run;
    run += v;
  }
  if (t == 1023) out[m] = run;
}

// ---------------------------------------------------------------- decode
// the band of steps done before draw tau (in i = N1 - steps): false when it lies past the end
__device__ __forceinline__ bool draw_band(const DecParams& pr, const double2* band, int64_t tau, uint32_t* ihi,
                                          uint32_t* ilo) {
  const int64_t N1 = pr.n - 1;
  const int64_t bi = tau >> kBandLog;
  const double f = (double)(tau & ((1 << kBandLog) - 1)) * (1.0 / (1 << kBandLog));
  const double2 b0 = band[bi < pr.nband ? bi : pr.nband - 1];
  const double2 b1 = band[bi + 1 < pr.nband ? bi + 1 : pr.nband - 1];
  const double se = b0.x + (b1.x - b0.x) * f;
  const double e = fmax(b0.y, b1.y) + 2.0;
  const double lo = floor(se - e), hi = ceil(se + e);
  if (lo > (double)(N1 - 1)) return false;
  const int64_t slo = lo < 0.0 ? 0 : (int64_t)lo;
  const int64_t shi = hi > (double)(N1 - 1) ? N1 - 1 : std::max<int64_t>(slo, (int64_t)hi);
  *ihi = (uint32_t)(N1 - slo);
  *ilo = (uint32_t)(N1 - shi);
  return true;
}

// draws tau0 .. tau0 + 15 of column c: PCG64 outputs (one jump-ahead per thread), classified
__global__ __launch_bounds__(kT) void k_dec_classify(DecParams pr, const u128* __restrict__ jt,
                                                     const double2* __restrict__ band, const int64_t* __restrict__ P,
                                                     int c, uint32_t* __restrict__ W, uint8_t* __restrict__ cls,
                                                     uint32_t* __restrict__ tot, int32_t* __restrict__ err) {
  __shared__ uint32_t sh[kT / 64];
  const int64_t p0 = P[c];
  const int64_t tau0 = (int64_t)blockIdx.x * kBlk + (int64_t)threadIdx.x * kPer;
  const int64_t N1 = pr.n - 1;
  uint32_t w[kPer];
  uint8_t cl[kPer];
  uint32_t nacc = 0, namb = 0;
  if (p0 < 0) {  // the previous column did not end inside its classified draws
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      w[j] = 0;
      cl[j] = kRej;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 2);
  } else {
    const u128 s0 = ((u128)pr.s_hi << 64) | pr.s_lo, inc = ((u128)pr.inc_hi << 64) | pr.inc_lo;
    const int64_t tt = p0 + tau0 - pr.h;  // index into the paired 32-bit stream (-1: the buffered half)
    u128 st = pcg::advance(s0, pr.base + (uint64_t)(tt > 0 ? tt >> 1 : 0), jt);
    int64_t kcur = -1;
    uint64_t out = 0;
    for (int j = 0; j < kPer; ++j) {
      const int64_t t2 = tt + j;
      if (t2 < 0) {
        w[j] = pr.buf32;
      } else {
        const int64_t kk = t2 >> 1;
        if (kk != kcur) {
          st = st * pcg::kMult + inc;
          out = pcg::output(st);
          kcur = kk;
        }
        w[j] = (t2 & 1) ? (uint32_t)(out >> 32) : (uint32_t)out;
      }
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      uint32_t ihi, ilo;  // i = N1 - steps done
      uint8_t cj;
      if (!draw_band(pr, band, tau0 + j, &ihi, &ilo)) {
        cj = kRej;  // past the column's end for every state of the band
      } else {
        const uint32_t mh = mask_of(ihi), ml = mask_of(ilo);
        if (mh == ml) {
          const uint32_t v = w[j] & mh;
          cj = v <= ilo ? kAcc : (v > ihi ? kRej : kAmb);
        } else if (mh == 2 * ml + 1) {  // one mask boundary B inside the band
          const uint32_t B = ml + 1, va = w[j] & mh, vb = w[j] & ml;
          const uint8_t da = va <= B ? kAcc : (va > ihi ? kRej : kAmb);
          const uint8_t db = vb <= ilo ? kAcc : kAmb;
          cj = (da == db && da != kAmb) ? da : kAmb;
        } else {
          cj = kAmb;
        }
      }
      cl[j] = cj;
      nacc += cj == kAcc;
      namb += cj == kAmb;
    }
  }
  uint4* w4 = reinterpret_cast<uint4*>(W + tau0);
#pragma unroll
  for (int j = 0; j < kPer / 4; ++j) w4[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
  uint32_t pk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    pk[j] = (uint32_t)cl[4 * j] | ((uint32_t)cl[4 * j + 1] << 8) | ((uint32_t)cl[4 * j + 2] << 16) |
            ((uint32_t)cl[4 * j + 3] << 24);
  *reinterpret_cast<uint4*>(cls + tau0) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  uint32_t total;
  (void)scan256(nacc | (namb << 16), sh, &total);
  if (threadIdx.x == 0) {
    tot[blockIdx.x] = total & 0xFFFFu;
    tot[pr.nb + blockIdx.x] = total >> 16;
  }
}

__device__ __forceinline__ void load_cls(const uint8_t* cls, int64_t tau0, uint8_t* c) {
  const uint4 v = *reinterpret_cast<const uint4*>(cls + tau0);
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < kPer; ++j) c[j] = (uint8_t)(u[j >> 2] >> (8 * (j & 3)));
}

// The ambiguous draws in order, 8 bytes each for the walk.  With A = decided accepts before the
// draw, the walk's state is S = A + extra (extra: the walk's own accepts so far).  Inside one
// mask range the draw is taken iff (w & m) <= N1 - S, i.e. extra < N1 - A - (w & m) + 1 =: x, stored
// as {x (clamped to [0, 2^31)), 0}; a band across a mask boundary stores {A | 2^31, w}.
__global__ __launch_bounds__(kT) void k_dec_compact(DecParams pr, const double2* __restrict__ band,
                                                    const uint32_t* __restrict__ W, const uint8_t* __restrict__ cls,
                                                    const uint32_t* __restrict__ pre, uint2* __restrict__ list,
                                                    int64_t cap) {
  __shared__ uint32_t sh[kT / 64];
  const int64_t tau0 = (int64_t)blockIdx.x * kBlk + (int64_t)threadIdx.x * kPer;
  uint8_t c[kPer];
  load_cls(cls, tau0, c);
  uint32_t nacc = 0, namb = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    nacc += c[j] == kAcc;
    namb += c[j] == kAmb;
  }
  uint32_t total;
  const uint32_t ex = scan256(nacc | (namb << 16), sh, &total);
  uint32_t acc = pre[blockIdx.x] + (ex & 0xFFFFu);
  int64_t amb = (int64_t)pre[pr.nb + 1 + blockIdx.x] + (ex >> 16);
  if (namb == 0) return;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (c[j] == kAmb) {
      if (amb < cap) {
        const uint32_t w = W[tau0 + j];
        uint32_t ihi = 0, ilo = 0;
        const bool in_band = draw_band(pr, band, tau0 + j, &ihi, &ilo);
        const uint32_t m = mask_of(ihi);
        uint2 e = make_uint2(acc | 0x80000000u, w);
        if (in_band && m == mask_of(ilo)) {
          const int64_t x = (pr.n - 1) - (int64_t)acc - (int64_t)(w & m) + 1;
          e = make_uint2((uint32_t)(x < 0 ? 0 : x), 0u);
        }
        list[amb] = e;
      }
      ++amb;
    } else if (c[j] == kAcc) {
      ++acc;
    }
  }
}

// per-draw accept flags: the decided ones and the walk's
__device__ __forceinline__ uint32_t accept_flags(const uint8_t* c, const uint32_t* pre, const uint8_t* dec,
                                                 int64_t nb, uint32_t* sh) {
  uint32_t namb = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) namb += c[j] == kAmb;
  uint32_t total;
  uint32_t amb = pre[nb + 1 + blockIdx.x] + scan256(namb, sh, &total);
  uint32_t bits = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    uint32_t a = c[j] == kAcc;
    if (c[j] == kAmb) a = dec[amb++];
    bits |= a << j;
  }
  return bits;
}

__global__ __launch_bounds__(kT) void k_dec_accsum(DecParams pr, const uint8_t* __restrict__ cls,
                                                   const uint32_t* __restrict__ pre, const uint8_t* __restrict__ dec,
                                                   uint32_t* __restrict__ tot2) {
  __shared__ uint32_t sh[kT / 64];
  const int64_t tau0 = (int64_t)blockIdx.x * kBlk + (int64_t)threadIdx.x * kPer;
  uint8_t c[kPer];
  load_cls(cls, tau0, c);
  const uint32_t bits = accept_flags(c, pre, dec, pr.nb, sh);
  uint32_t total;
  (void)scan256(__popc(bits), sh, &total);
  if (threadIdx.x == 0) tot2[blockIdx.x] = total;
}

// every decision against the rule at the state its prefix implies; the swap targets; the end
__global__ __launch_bounds__(kT) void k_dec_finish(DecParams pr, const uint32_t* __restrict__ W,
                                                   const uint8_t* __restrict__ cls, const uint32_t* __restrict__ pre,
                                                   const uint8_t* __restrict__ dec, const uint32_t* __restrict__ pre2,
                                                   int64_t* __restrict__ P, int c, int32_t* __restrict__ J,
                                                   int32_t* __restrict__ err) {
  __shared__ uint32_t sh[kT / 64];
  const int64_t tau0 = (int64_t)blockIdx.x * kBlk + (int64_t)threadIdx.x * kPer;
  const int64_t N1 = pr.n - 1;
  uint8_t cl[kPer];
  load_cls(cls, tau0, cl);
  const uint32_t bits = accept_flags(cl, pre, dec, pr.nb, sh);
  uint32_t total;
  int64_t S = (int64_t)pre2[blockIdx.x] + scan256(__popc(bits), sh, &total);
  if (S >= N1) return;
  const int64_t p0 = P[c];
  const uint4* w4 = reinterpret_cast<const uint4*>(W + tau0);
  uint32_t w[kPer];
#pragma unroll
  for (int j = 0; j < kPer / 4; ++j) {
    const uint4 v = w4[j];
    w[4 * j] = v.x;
    w[4 * j + 1] = v.y;
    w[4 * j + 2] = v.z;
    w[4 * j + 3] = v.w;
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    if (S < N1) {
      const uint32_t a = (bits >> j) & 1u;
      const uint32_t i = (uint32_t)(N1 - S), v = w[j] & mask_of(i);
      bad |= (uint32_t)(v <= i) != a;
      if (a) {
        J[i] = (int32_t)v;
        if (S == N1 - 1 && p0 >= 0) P[c + 1] = p0 + tau0 + j + 1;
      }
      S += a;
    }
  }
  if (bad) atomicOr(err, 1);
}

// column c checked: no error so far and its end found (read by the column's permutation
// kernels on the side stream, which run while later columns may still fail)
__global__ void k_dec_seal(const int32_t* __restrict__ err, const int64_t* __restrict__ P, int c,
                           int32_t* __restrict__ ok) {
  if (threadIdx.x == 0 && blockIdx.x == 0) ok[c] = (*err == 0 && P[c + 1] >= 0) ? 1 : 0;
}

// ---------------------------------------------------------------- targets -> permutation
// One column at a time, skipped unless the column's decode was sealed.  The steps 1 .. n-1 are
// sorted by target with the library's stable one-sweep radix passes (radix_sort_keys32_async:
// within a target the steps stay ascending), so each target's group is contiguous and in time
// order: S(step) = the next step of its group, M(q) = the group's first step above q.
__global__ __launch_bounds__(256) void k_perm_links(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                                                    int64_t m, int32_t* __restrict__ S, int32_t* __restrict__ M,
                                                    const int32_t* __restrict__ ok) {
  if (!*ok) return;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) {
    const uint32_t t = keys[k];
    const int32_t st = (int32_t)idx[k] + 1;  // key k is J[1 + k]
    const int32_t nx = (k + 1 < m && keys[k + 1] == t) ? (int32_t)idx[k + 1] + 1 : -1;
    S[st] = nx;
    if (k == 0 || keys[k - 1] != t) M[t] = st != (int32_t)t ? st : nx;
  }
}

__global__ void k_flag_if(const uint32_t* __restrict__ word, int32_t* __restrict__ err, int32_t bit) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && *word) atomicOr(err, bit);
}

// V(x) = V(M(x)), or x + 1 at the end of the chain (M(x) > x: it ends)
__device__ __forceinline__ int32_t perm_value(const int32_t* __restrict__ M, int32_t x) {
  int32_t y;
  while ((y = M[x]) >= 0) x = y;
  return x + 1;
}

// q = (perm - u) / n for one column (u in q on entry); strata (optional) = perm - 1.  V is
// followed along M only from the positions a row needs (S(r), or M(0) for row 0) instead of
// being tabulated for every position first (a separate pass of its own, 0.14 ms per 1e7).
__global__ __launch_bounds__(256) void k_perm_combine(const int32_t* __restrict__ J, const int32_t* __restrict__ S,
                                                      const int32_t* __restrict__ M, int64_t n,
                                                      double* __restrict__ q, const int32_t* __restrict__ ok,
                                                      int32_t* __restrict__ strata) {
  if (!*ok) return;
  const double dn = (double)n;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    int32_t v;
    if (r == 0) {
      const int32_t f = M[0];
      v = f >= 0 ? perm_value(M, f) : 1;
    } else {
      const int32_t nx = S[r];
      v = nx >= 0 ? perm_value(M, nx) : J[r] + 1;
    }
    q[r] = ((double)v - q[r]) / dn;  // (perms - samples) / n: subtract, then divide
    if (strata) strata[r] = v - 1;
  }
}

// ---------------------------------------------------------------- host: the band of states
// digamma / trigamma for y >= 1 (recurrence up to 10, then the asymptotic series)
double digamma(double y) {
  double r = 0.0;
  while (y < 10.0) {
    r -= 1.0 / y;
    y += 1.0;
  }
  const double z = 1.0 / (y * y);
  return r + log(y) - 0.5 / y - z * (1.0 / 12 - z * (1.0 / 120 - z / 252));
}

double trigamma(double y) {
  double r = 0.0;
  while (y < 10.0) {
    r += 1.0 / (y * y);
    y += 1.0;
  }
  const double z = 1.0 / (y * y);
  return r + 1.0 / y + z / 2 + z / y * (1.0 / 6 - z * (1.0 / 30 - z / 42));
}

// H(x) = sum_{k <= x} 1/k and its square analogue, continued to real x >= 0 (up to constants)
double harm(double x) { return digamma(x + 1.0); }
double harm2(double x) { return -trigamma(x + 1.0); }

// Band table, one entry per 1024 draws of a column: (expected steps done, half-width in steps).
// Step i needs (m + 1) / (i + 1) draws on average, m = mask(i); over a mask range [lo, hi] the
// draws for steps hi .. x sum to (m + 1) (H(hi + 1) - H(x)), their variance to
// (m + 1)^2 (H2(hi + 1) - H2(x)) - draws.  Returns the draws to classify per column.
int64_t band_table(int64_t n, double ksig, std::vector<double>& band) {
  struct Range {
    double d0, v0;  // draws and variance before the range
    double hi, lo, m1;
  };
  std::vector<Range> rs;
  double dsum = 0.0, vsum = 0.0;
  for (int64_t hi = n - 1; hi >= 1;) {
    const uint32_t m = mask_of((uint32_t)hi);
    const int64_t lo = std::max<int64_t>(1, ((int64_t)m + 1) / 2);
    const double m1 = (double)m + 1.0;
    const double dr = m1 * (harm((double)hi + 1) - harm((double)lo));
    const double vr = m1 * m1 * (harm2((double)hi + 1) - harm2((double)lo)) - dr;
    rs.push_back({dsum, vsum, (double)hi, (double)lo, m1});
    dsum += dr;
    vsum += std::max(vr, 0.0);
    hi = lo - 1;
  }
  const double e_end = ksig * sqrt(vsum) + 16.0;
  const double tneed = dsum + e_end + 4096.0;
  const int64_t tcap = ((int64_t)ceil(tneed) + kBlk - 1) / kBlk * kBlk;
  const int64_t nband = (tcap >> kBandLog) + 2;
  band.assign((size_t)nband * 2, 0.0);
  const double N1 = (double)(n - 1);
  size_t r = 0;
  for (int64_t k = 0; k < nband; ++k) {
    const double tau = (double)k * (1 << kBandLog);
    double s, var, p = 1.0;
    while (r < rs.size() && tau >= rs[r].d0 + rs[r].m1 * (harm(rs[r].hi + 1) - harm(rs[r].lo))) ++r;
    if (r >= rs.size()) {  // past the expected end: the next column's steps would follow
      s = N1 + (tau - dsum);
      var = vsum;
    } else {
      const Range& g = rs[r];
      const double target = harm(g.hi + 1) - (tau - g.d0) / g.m1;  // H(x) = target, x in [lo, hi + 1]
      double x = std::min(g.hi + 1, std::max(g.lo, exp(target + 0.5772156649015329) - 0.5));
      for (int it = 0; it < 8; ++it) {
        x -= (harm(x) - target) / trigamma(x + 1.0);
        x = std::min(g.hi + 1, std::max(g.lo, x));
      }
      s = (N1 - g.hi) + (g.hi + 1 - x);
      var = g.v0 + g.m1 * g.m1 * (harm2(g.hi + 1) - harm2(x)) - (tau - g.d0);
      p = std::min(1.0, x / g.m1);  // acceptance rate at i = x - 1
    }
    // steps done after tau draws: sd = (sd of the draws) x (acceptance rate), renewal theory
    band[2 * k] = s;
    band[2 * k + 1] = ksig * sqrt(std::max(var, 0.0)) * p + 16.0;
  }
  return tcap;
}

// pinned staging of the ambiguous draws and their decisions (kept across calls)
struct Pinned {
  std::mutex mu;
  uint2* list = nullptr;
  uint8_t* dec = nullptr;
  int64_t cap = 0;
  int ensure(int64_t want) {
    if (want <= cap) return PBH_OK;
    if (list) (void)hipHostFree(list);
    if (dec) (void)hipHostFree(dec);
    list = nullptr;
    dec = nullptr;
    cap = 0;
    PBH_CHECK_HIP(hipHostMalloc((void**)&list, (size_t)want * sizeof(uint2), hipHostMallocDefault));
    PBH_CHECK_HIP(hipHostMalloc((void**)&dec, (size_t)want, hipHostMallocDefault));
    cap = want;
    return PBH_OK;
  }
};
Pinned& pinned() {
  static Pinned p;
  return p;
}

struct DevBufs {
  hipStream_t s;
  std::vector<void*> v;
  template <class T>
  int get(T** p, size_t count) {
    void* x = nullptr;
    PBH_CHECK_HIP(hipMallocAsync(&x, std::max<size_t>(count * sizeof(T), 256), s));
    v.push_back(x);
    *p = (T*)x;
    return PBH_OK;
  }
  ~DevBufs() {
    for (void* x : v) (void)hipFreeAsync(x, s);
  }
};

// the stream the permutations are built on, behind the decode (one per process)
hipStream_t perm_stream(hipStream_t fallback) {
  static hipStream_t st = [] {
    hipStream_t x = nullptr;
    if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) x = nullptr;
    return x;
  }();
  return st ? st : fallback;
}

// the caller's stream waits for the side stream on every exit (before DevBufs frees)
struct SideJoin {
  hipStream_t side, main;
  hipEvent_t ev = nullptr;
  ~SideJoin() {
    if (side != main && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
      (void)hipEventRecord(ev, side);
      (void)hipStreamWaitEvent(main, ev, 0);
      (void)hipEventDestroy(ev);
    }
  }
};

struct PermBufs {
  SortBuffers sb;
  int32_t *S, *M;
};

// column c's permutation from its targets (J: n words), combined into q[0 .. n) (u on entry);
// every kernel past the sort exits at once unless ok[0] (k_dec_seal)
int column_to_q(const int32_t* J, int64_t n, PermBufs& pb, const int32_t* ok, int32_t* err, double* q,
                int32_t* strata, hipStream_t s) {
  const int64_t m = n - 1;  // steps 1 .. n-1
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) < n) ++bits;  // targets < n
  int cur = 0;
  uint32_t* stuck = nullptr;
  if (int st = radix_sort_keys32_async(pb.sb, m, (bits + 7) / 8, s, &cur, (const uint32_t*)(J + 1), &stuck)) return st;
  hipLaunchKernelGGL(k_flag_if, dim3(1), dim3(64), 0, s, stuck, err, 4);
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipMemsetAsync(pb.M, 0xFF, (size_t)n * 4, s));  // -1: no step targets q from above
  const unsigned grid = grid_for(n, 256, 1 << 16);
  hipLaunchKernelGGL(k_perm_links, dim3(grid), dim3(256), 0, s, (const uint32_t*)pb.sb.keys[cur], pb.sb.vals[cur], m,
                     pb.S, pb.M, ok);
  PBH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_perm_combine, dim3(grid), dim3(256), 0, s, J, pb.S, pb.M, n, q, ok, strata);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// One attempt with band half-width ksig: u into q, then per column the decode on the caller's
// stream and, once sealed, its permutation on the side stream (overlapping the next column's
// host walk).  *ok: every column passed the check (q complete); otherwise q is to be redone.
int decode_attempt(const DecParams& base, const uint64_t* state_host, const uint64_t* inc_host, const u128* jt_dev,
                   int d, double ksig, double* q, int64_t ldq, int32_t* J, int32_t* strata, int64_t lds,
                   hipStream_t s, bool* ok, int64_t* ambiguous) {
  *ok = false;
  DecParams pr = base;
  const int64_t n = pr.n, N1 = n - 1;
  std::vector<double> band;
  pr.tcap = band_table(n, ksig, band);
  pr.nb = pr.tcap / kBlk;
  pr.nband = (int64_t)band.size() / 2;
  const int64_t cap = std::min<int64_t>(pr.tcap, (int64_t)1 << 22);
  DevBufs b{s};
  uint32_t *W, *tot, *pre, *tot2, *pre2;
  uint8_t *cls, *dec;
  uint2* list;
  double2* band_dev;
  int64_t* P;
  int32_t *err, *okc;
  u128* pcg_ws;
  PermBufs pb;
  char* sort_ws;
  int st;
  if ((st = b.get(&W, pr.tcap)) || (st = b.get(&cls, pr.tcap)) || (st = b.get(&tot, 2 * pr.nb)) ||
      (st = b.get(&pre, 2 * (pr.nb + 1))) || (st = b.get(&tot2, pr.nb)) || (st = b.get(&pre2, pr.nb + 1)) ||
      (st = b.get(&list, cap)) || (st = b.get(&dec, cap)) || (st = b.get(&band_dev, pr.nband)) ||
      (st = b.get(&P, d + 1)) || (st = b.get(&err, 1)) || (st = b.get(&okc, d)) || (st = b.get(&pcg_ws, 128)) ||
      (st = b.get(&pb.S, n)) || (st = b.get(&pb.M, n)) ||
      (st = b.get(&sort_ws, sort_workspace_bytes(n))))
    return st;
  sort_carve(sort_ws, n, pb.sb);
  const hipStream_t side = perm_stream(s);
  SideJoin join{side, s};
  hipEvent_t ev = nullptr;
  PBH_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  struct EvFree {
    hipEvent_t& e;
    ~EvFree() {
      if (e) (void)hipEventDestroy(e);
    }
  } evfree{ev};
  Pinned& pn = pinned();
  std::lock_guard<std::mutex> lock(pn.mu);
  if ((st = pn.ensure(std::max<int64_t>(cap, 1 << 16)))) return st;
  // u = rng.uniform(size=(n, d)), draws 0 .. n d - 1 (rewritten by every attempt)
  if ((st = pbh_pcg64_random(state_host, inc_host, 0, n, d, q, ldq, pcg_ws, 128 * sizeof(u128), s))) return st;
  std::vector<int64_t> p_init(d + 1, -1);
  p_init[0] = 0;
  PBH_CHECK_HIP(hipMemcpyAsync(band_dev, band.data(), band.size() * sizeof(double), hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(P, p_init.data(), (d + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemsetAsync(err, 0, sizeof(int32_t), s));
  const unsigned nb = (unsigned)pr.nb;
  int64_t namb_total = 0;
  for (int c = 0; c < d; ++c) {
    int32_t* Jc = J + (int64_t)c * n;
    hipLaunchKernelGGL(k_dec_classify, dim3(nb), dim3(kT), 0, s, pr, jt_dev, band_dev, P, c, W, cls, tot, err);
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_small, dim3(2), dim3(1024), 0, s, tot, pr.nb, pr.nb, pre, pr.nb + 1);
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_dec_compact, dim3(nb), dim3(kT), 0, s, pr, band_dev, W, cls, pre, list, cap);
    PBH_CHECK_LAUNCH();
    uint32_t namb = 0;
    PBH_CHECK_HIP(hipMemcpyAsync(pn.list, pre + 2 * pr.nb + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    memcpy(&namb, pn.list, sizeof(uint32_t));
    if ((int64_t)namb > cap) return PBH_OK;  // too many to walk: the host shuffles
    namb_total += namb;
    if (namb) {
      PBH_CHECK_HIP(hipMemcpyAsync(pn.list, list, (size_t)namb * sizeof(uint2), hipMemcpyDeviceToHost, s));
      PBH_CHECK_HIP(hipStreamSynchronize(s));
      // the walk (k_dec_compact's encoding); decisions past the column's end are never read
      uint32_t extra = 0;
      const uint2* L = pn.list;
      uint8_t* D = pn.dec;
      for (uint32_t k = 0; k < namb; ++k) {
        const uint32_t x = L[k].x;
        uint32_t a;
        if (!(x >> 31)) {
          a = extra < x;
        } else {
          const int64_t S = (int64_t)(x & 0x7FFFFFFFu) + extra;
          const uint32_t i = S < N1 ? (uint32_t)(N1 - S) : 0u;
          a = S < N1 && (L[k].y & mask_of(i)) <= i;
        }
        D[k] = (uint8_t)a;
        extra += a;
      }
      PBH_CHECK_HIP(hipMemcpyAsync(dec, pn.dec, namb, hipMemcpyHostToDevice, s));
    }
    hipLaunchKernelGGL(k_dec_accsum, dim3(nb), dim3(kT), 0, s, pr, cls, pre, dec, tot2);
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, s, tot2, pr.nb, pr.nb, pre2, pr.nb + 1);
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_dec_finish, dim3(nb), dim3(kT), 0, s, pr, W, cls, pre, dec, pre2, P, c, Jc, err);
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_dec_seal, dim3(1), dim3(64), 0, s, err, P, c, okc);
    PBH_CHECK_LAUNCH();
    if (side != s) {
      PBH_CHECK_HIP(hipEventRecord(ev, s));
      PBH_CHECK_HIP(hipStreamWaitEvent(side, ev, 0));
    }
    if ((st = column_to_q(Jc, n, pb, okc + c, err, q + (int64_t)c * ldq, strata ? strata + (int64_t)c * lds : nullptr,
                          side)))
      return st;
  }
  if (side != s) {  // the permutations' look-back checks land in err before it is read
    PBH_CHECK_HIP(hipEventRecord(ev, side));
    PBH_CHECK_HIP(hipStreamWaitEvent(s, ev, 0));
  }
  int64_t tail = -1;
  int32_t e = 0;
  PBH_CHECK_HIP(hipMemcpyAsync(&tail, P + d, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipMemcpyAsync(&e, err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  *ambiguous = namb_total;
  *ok = e == 0 && tail >= 0;
  return PBH_OK;
}

// n = 1: no shuffle steps, q = (1 - u) / 1
__global__ void k_single_row(double* __restrict__ q, int64_t ldq, int d) {
  for (int c = threadIdx.x; c < d; c += blockDim.x) q[(int64_t)c * ldq] = 1.0 - q[(int64_t)c * ldq];
}

}  // namespace

int lhs_reference_device(const uint64_t* state_host, const uint64_t* inc_host, bool has32, uint32_t buf32, int64_t n,
                         int d, double* q, int64_t ldq, int32_t* targets, hipStream_t s, bool* done, int32_t* strata,
                         int64_t lds) {
  *done = false;
  g_last_attempts = 0;
  g_last_device = 0;
  g_last_ambiguous = 0;
  if (d <= 0 || n <= 0) return PBH_OK;
  PBH_REQUIRE(n < ((int64_t)1 << 31) && ldq >= n && targets, "lhs_reference_device: bad arguments");
  const u128 s0 = ((u128)state_host[1] << 64) | state_host[0];
  const u128 inc = ((u128)inc_host[1] << 64) | inc_host[0];
  int st;
  if (n == 1) {
    DevBufs b{s};
    u128* pcg_ws;
    if ((st = b.get(&pcg_ws, 128))) return st;
    if ((st = pbh_pcg64_random(state_host, inc_host, 0, 1, d, q, ldq, pcg_ws, 128 * sizeof(u128), s))) return st;
    hipLaunchKernelGGL(k_single_row, dim3(1), dim3(256), 0, s, q, ldq, d);
    PBH_CHECK_LAUNCH();
    if (strata)
      for (int c = 0; c < d; ++c) PBH_CHECK_HIP(hipMemsetAsync(strata + (int64_t)c * lds, 0, 4, s));
  } else {
    std::vector<u128> table(128);
    pcg::jump_table(inc, table.data());
    DevBufs b{s};
    u128* jt;
    if ((st = b.get(&jt, 128))) return st;
    PBH_CHECK_HIP(hipMemcpyAsync(jt, table.data(), 128 * sizeof(u128), hipMemcpyHostToDevice, s));
    DecParams pr{};
    pr.s_lo = (uint64_t)s0;
    pr.s_hi = (uint64_t)(s0 >> 64);
    pr.inc_lo = (uint64_t)inc;
    pr.inc_hi = (uint64_t)(inc >> 64);
    pr.base = (uint64_t)(n * (int64_t)d);
    pr.h = has32 ? 1 : 0;
    pr.buf32 = buf32;
    pr.n = n;
    bool ok = false;
    double ksig = g_band_sigmas;
    for (int a = 0; a < kAttempts && !ok; ++a, ksig *= 2.0) {
      int64_t amb = 0;
      ++g_last_attempts;
      if ((st = decode_attempt(pr, state_host, inc_host, jt, d, ksig, q, ldq, targets, strata, lds, s, &ok, &amb)))
        return st;
      g_last_ambiguous = amb;
    }
    if (!ok) return PBH_OK;  // q is to be redone by the caller
  }
  *done = true;
  g_last_device = 1;
  return PBH_OK;
}

}  // namespace pbh

extern "C" int pbh_lhs_reference_band(double sigmas, double* previous) {
  PBH_REQUIRE(sigmas >= 0.0 && sigmas < 1e6, "pbh_lhs_reference_band: bad width");
  if (previous) *previous = pbh::g_band_sigmas;
  if (sigmas > 0.0) pbh::g_band_sigmas = sigmas;
  return PBH_OK;
}

extern "C" int pbh_lhs_reference_stats(int32_t* device, int32_t* attempts, int64_t* ambiguous) {
  PBH_REQUIRE(device && attempts && ambiguous, "pbh_lhs_reference_stats: bad arguments");
  *device = pbh::g_last_device;
  *attempts = pbh::g_last_attempts;
  *ambiguous = pbh::g_last_ambiguous;
  return PBH_OK;
}
