// Quantile generators and the inverse-CDF sweep (the first half of Node.sample,
// modeling.py:478-489 and Distribution._sample, modeling.py:795-807).
//
// Roofline: the ppf sweep moves 16 B per draw (read q 8 + write x 8), the fused
// generator + ppf 8 B per draw (write x only); norm / uniform / expon / triang / lognorm
// are HBM-bound, gamma (igami) and per-element poisson searches are FP64-VALU-bound.
#include <array>
#include <functional>
#include <map>
#include <mutex>
#include <math.h>
#include <stdlib.h>

#include <type_traits>
#include <vector>

#include "pbh_error.h"
#include "pbh_table_cache.h"
#include "pbh_ppf_core.h"
#include "pbh_ppf_ext.h"
#include "pbh_rng.h"
#include "pbh_special.h"
#include "pbh_sort.h"
#include "pbh_step4.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kBlock = 256;
// Register cap of the ppf kernels: gamma / poisson carry their rarely taken fallbacks (igami's
// full iteration, the per-element poisson search) inline, which would otherwise size the
// register allocation of every wave (~256 VGPRs, one wave per SIMD) for code the hot path never
// runs.  Capping at 4 waves per SIMD (128 VGPRs) spills inside those fallbacks instead.
#ifndef PBH_PPF_WAVES
#define PBH_PPF_WAVES 4
#endif
#if PBH_PPF_WAVES > 0
#define PBH_OCC __attribute__((amdgpu_waves_per_eu(PBH_PPF_WAVES)))
#else
#define PBH_OCC
#endif



unsigned compact_grid(int64_t n) { return grid_for(n, kCTile, 256 * 8); }

// Blocks of the gamma slow-list kernels (grid-stride over the list; a few thousand items at a
// time in practice): a grid this size schedules in one wave of the chip even next to the other
// step-4 lanes' kernels.
#ifndef PBH_SLOW_GRID
#define PBH_SLOW_GRID 1024
#endif

bool scalar_params(const Params& prm) { return !prm.ptr[0] && !prm.ptr[1] && !prm.ptr[2]; }

// k_ppf / k_lhs_ppf for D in {norm, lognorm} with tail compaction.  Q(i) gives the quantile of
// tile item i (a strided load, or the fused LHS generator).  SC: every parameter is a scalar
// (no per-row arrays), read once into registers -- with per-item Params::at the norm sweep
// measured 0.78-0.90 ms per 1e8 against 0.60-0.71 (tools/microbench_ppf_c.hip).
template <int D, bool SC, class Q>
PBH_DI void ppf_compacted(int64_t n, const Q& qof, const Params& prm_in, const PoissonTable& pt,
                          double* __restrict__ out, int32_t* flag, TailQueue& tq, double* res,
                          const double* lt = nullptr) {
  Params prm = prm_in;
  if constexpr (SC) prm.ptr[0] = prm.ptr[1] = prm.ptr[2] = nullptr;  // at() folds to the scalars
  bool bad = false;  // a non-finite output, flagged once per thread at the end
  for (int64_t base = (int64_t)blockIdx.x * kCTile; base < n; base += (int64_t)gridDim.x * kCTile) {
    if (threadIdx.x == 0) tq.count = 0;
    __syncthreads();
    // every quantile of the tile first: the loads are issued together, not one per round trip
    // (interleaved with tail_push's LDS atomics they were serialised: 0.82 -> 0.60 ms per 1e8)
    double qa[kCIpt];
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int64_t i = base + j * kBlock + threadIdx.x;
      qa[j] = i < n ? qof(i) : 0.5;
    }
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kBlock + threadIdx.x;
      const int64_t i = base + p;
      const bool valid = i < n;
      const double qv = qa[j];
      const bool tail = valid && normal_takes_tail(qv, normal_loc<D>(prm.at(0, i), prm.at(1, i)));
      if (valid && !tail) res[p] = ppf_one<D, 1>(qv, prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
      tail_push(tq, tail, qv, p);
    }
    __syncthreads();
    const int T = tq.count;
    for (int t = threadIdx.x; t < T; t += kBlock) {
      const int p = tq.pos[t];
      const int64_t i = base + p;
      res[p] = ppf_one<D, 2>(tq.arg[t], prm.at(0, i), prm.at(1, i), prm.at(2, i), pt, lt);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kBlock + threadIdx.x;
      const int64_t i = base + p;
      const double x = i < n ? res[p] : 0.0;
      if (i < n) out[i] = x;
      bad |= !isfinite(x);
    }
  }
  flag_nonfinite(flag, bad);
}

template <int D, bool SC>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_ppf_c(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                  Params prm, PoissonTable pt, double* __restrict__ out,
                                                  int32_t* flag) {
  __shared__ TailQueue tq;
  __shared__ double res[kCTile];
  __shared__ double lt[kLog3N];
  stage_log3(lt);  // (ppf_compacted's first barrier follows)
  ppf_compacted<D, SC>(n, [&](int64_t i) { return q[i * q_stride]; }, prm, pt, out, flag, tq, res, lt);
}

template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_ppf(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                Params prm, PoissonTable pt, double* __restrict__ out,
                                                int32_t* flag) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * kBlock;
  for (; i < n; i += step) {
    double x = ppf_one<D>(q[i * q_stride], prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

// Streaming form of k_ppf for the common case at the sample_from_quantiles boundary: a
// contiguous, 16-byte-aligned q column and scalar parameters.  One wave's 64 lanes can keep
// only one 512-B load in flight per grid-stride step in k_ppf, and with 16 waves per CU that is
// ~2 MB in flight chip-wide, short of the ~12 MB that HBM latency x 6.3 TB/s needs.  Here every
// lane issues kVU independent 16-byte loads (two draws each) before any arithmetic, and writes
// back with non-temporal 16-byte stores (x is written once and not re-read by this launch).
constexpr int kVU = 4;
constexpr int kVTile = kBlock * kVU * 2;  // draws per block step
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_ppf_v(const double* __restrict__ q, int64_t n, Params prm,
                                                  PoissonTable pt, double* __restrict__ out, int32_t* flag) {
  const double p0 = prm.val[0], p1 = prm.val[1], p2 = prm.val[2];
  const int64_t full = n / kVTile;
  bool bad = false;
  for (int64_t t = blockIdx.x; t < full; t += gridDim.x) {
    const f64x2* qv = reinterpret_cast<const f64x2*>(q + t * kVTile);
    f64x2* ov = reinterpret_cast<f64x2*>(out + t * kVTile);
    f64x2 v[kVU];
#pragma unroll
    for (int u = 0; u < kVU; ++u) v[u] = __builtin_nontemporal_load(qv + u * kBlock + threadIdx.x);
#pragma unroll
    for (int u = 0; u < kVU; ++u) {
      f64x2 r;
      r.x = ppf_one<D>(v[u].x, p0, p1, p2, pt);
      r.y = ppf_one<D>(v[u].y, p0, p1, p2, pt);
      bad |= !isfinite(r.x) || !isfinite(r.y);
      __builtin_nontemporal_store(r, ov + u * kBlock + threadIdx.x);
    }
  }
  // ragged end (< kVTile draws): one block, scalar accesses
  if (blockIdx.x == gridDim.x - 1) {
    for (int64_t i = full * kVTile + threadIdx.x; i < n; i += kBlock) {
      const double x = ppf_one<D>(q[i], p0, p1, p2, pt);
      out[i] = x;
      bad |= !isfinite(x);
    }
  }
  flag_nonfinite(flag, bad);
}

template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_lhs_ppf(uint64_t seed, int64_t n, int64_t row0, int64_t nrows,
                                                    uint32_t col, Params prm, PoissonTable pt,
                                                    double* __restrict__ out, int32_t* flag) {
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * kBlock;
  for (; i < nrows; i += step) {
    double q = lhs_quantile(ph, fp, (uint64_t)(row0 + i), col);
    double x = ppf_one<D>(q, prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

template <int D, bool SC>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_lhs_ppf_c(uint64_t seed, int64_t n, int64_t row0, int64_t nrows,
                                                      uint32_t col, Params prm, PoissonTable pt,
                                                      double* __restrict__ out, int32_t* flag) {
  __shared__ TailQueue tq;
  __shared__ double res[kCTile];
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  ppf_compacted<D, SC>(nrows, [&](int64_t i) { return lhs_quantile(ph, fp, (uint64_t)(row0 + i), col); }, prm, pt, out,
                   flag, tq, res);
}

// ---------------------------------------------------------------- gamma: guide table in LDS
// igami_guided reads 7 table values (y, d1, d2 at nodes j and j + 1, ok[j]) at a node chosen by
// the draw.  With q in random order every lane of a wave hits a different cache line, so each of
// those 7 loads costs the texture path ~64 line lookups per wave instruction -- the gamma sweep
// measured 1.3 ms per 1e8 draws, gather-bound.  The whole table (4 x 3841 doubles = 120 KiB)
// fits in a CU's 160 KiB LDS: one 1024-thread workgroup per CU stages it once and then gathers
// from LDS.  The arithmetic and the table values are the same, so results are bit-identical to
// k_ppf / k_lhs_ppf's.
constexpr int kGBlock = 1024;
constexpr int kGTable = 4 * sf::kGammaGuideM;  // y, d1, d2, ok

PBH_DI sf::GammaGuide stage_guide(const sf::GammaGuide& T, double* lds) {
  for (int k = threadIdx.x; k < kGTable; k += kGBlock) lds[k] = T.y[k];  // the four arrays are contiguous
  __syncthreads();
  const int m = sf::kGammaGuideM;
  return sf::GammaGuide{lds, lds + m, lds + 2 * m, lds + 3 * m, m, T.z0, T.h, T.inv_h};
}

PBH_DI double gamma_ppf_lds(double q, const Params& prm, const PoissonTable& pt, const sf::GammaGuide& T) {
  PoissonTable local = pt;  // ppf_one reads the guide through pt
  local.guide = T;
  return ppf_one<PBH_DIST_GAMMA>(q, prm.val[0], prm.val[1], prm.val[2], local);
}


// igami_guided's interpolation branch and ppf_one's gamma wrapper, operation for operation:
// true and *v = the value when the element needs no iteration; false sends it to the slow queue
// (gamma_ppf_lds), so that the hot loops carry no igami code.
// ltab / etab: the log and exp tables staged in LDS (stage_logexp)
PBH_DI bool gamma_fast(double q, const sf::GammaGuide& T, double scale, double loc, bool cond0, double* v,
                       const double* ltab, const double* etab) {
  if (!(cond0 && q > 0.0 && q < 1.0)) return false;
  const double w = sf::log_odds_at(q, ltab);
  const double u = (w - T.z0) * T.inv_h;
  if (!(u >= 0.0 && u < (double)(T.m - 1))) return false;
  const int j = (int)u;
  const double y = sf::guide_interp(T, j, u - (double)j);
  if (!(y >= -680.0 && y <= 700.0 && T.ok[j] != 0.0)) return false;
  *v = sf::exp_tab_at(y, etab) * scale + loc;
  return true;
}

// sf::log_tab's and sf::exp_tab's tables copied into LDS (4 KiB + 2 KiB): their entries are picked
// per lane, so a wave's load from the global copy touches up to 32 / 16 cache lines
constexpr int kLogTabN = 128 * 4, kExpTabN = 128 * 2;
PBH_DI void stage_logexp(double*& ltab, double*& etab) {
#ifdef PBH_NO_LDS_LOGEXP  // A/B build: the global tables
  ltab = const_cast<double*>(&sf::pbh_log_tab[0][0]);
  etab = const_cast<double*>(&sf::pbh_exp_tab[0][0]);
#else
  for (int k = threadIdx.x; k < kLogTabN; k += blockDim.x) ltab[k] = (&sf::pbh_log_tab[0][0])[k];
  for (int k = threadIdx.x; k < kExpTabN; k += blockDim.x) etab[k] = (&sf::pbh_exp_tab[0][0])[k];
#endif
}

__global__ __launch_bounds__(kGBlock) void k_ppf_gamma_lds(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                           Params prm, PoissonTable pt, double* __restrict__ out,
                                                           int32_t* flag) {
  __shared__ double lds[kGTable];
#ifndef PBH_GAMMA_SWEEP_PER
#define PBH_GAMMA_SWEEP_PER 4
#endif
  constexpr int kPer = PBH_GAMMA_SWEEP_PER, kTile = kPer * kGBlock, kQCap = 2048;
  __shared__ uint16_t slowq[kQCap];
  __shared__ int nslow;
  __shared__ double ltab_s[kLogTabN], etab_s[kExpTabN];
  double *ltab = ltab_s, *etab = etab_s;
  stage_logexp(ltab, etab);  // (stage_guide's barrier follows)
  const sf::GammaGuide T = stage_guide(pt.guide, lds);
  const double shape = prm.val[0], loc = prm.val[1], scale = prm.val[2];
  const bool cond0 = (shape > 0.0) && (scale > 0.0) && (loc == loc) && pt.has_gamma;
  bool bad = false;  // a non-finite output, flagged once per thread at the end
  // one workgroup per CU: nothing else on the CU hides a tile's load latency, so the next tile's
  // quantiles are loaded while this one is evaluated (register prefetch)
  const int64_t step = (int64_t)gridDim.x * kTile;
  double qn[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = (int64_t)blockIdx.x * kTile + j * kGBlock + threadIdx.x;
    qn[j] = i < n ? q[i * q_stride] : 0.5;
  }
  for (int64_t base = (int64_t)blockIdx.x * kTile; base < n; base += step) {
    if (threadIdx.x == 0) nslow = 0;
    __syncthreads();
    double qv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
#ifndef PBH_NO_PREFETCH
      qv[j] = qn[j];
      const int64_t i = base + step + j * kGBlock + threadIdx.x;
      qn[j] = i < n ? q[i * q_stride] : 0.5;
#else
      const int64_t i = base + j * kGBlock + threadIdx.x;
      qv[j] = i < n ? q[i * q_stride] : 0.5;
#endif
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = base + j * kGBlock + threadIdx.x;
      if (i >= n) continue;
      double v;
      if (gamma_fast(qv[j], T, scale, loc, cond0, &v, ltab, etab)) {
        out[i] = v;
        bad |= !isfinite(v);
      } else {
        const int slot = atomicAdd(&nslow, 1);
        if (slot < kQCap) slowq[slot] = (uint16_t)(j * kGBlock + threadIdx.x);
      }
    }
    __syncthreads();
    const int ns = nslow;
    const int nd = ns <= kQCap ? ns : kTile;  // queue overflow: the whole tile again
    for (int t = threadIdx.x; t < nd; t += kGBlock) {
      const int64_t i = base + (ns <= kQCap ? slowq[t] : t);
      if (i >= n) continue;
      const double x = gamma_ppf_lds(q[i * q_stride], prm, pt, T);
      out[i] = x;
      bad |= !isfinite(x);
    }
  }
  flag_nonfinite(flag, bad);
}

__global__ __launch_bounds__(kGBlock) void k_lhs_ppf_gamma_lds(uint64_t seed, int64_t n, int64_t row0, int64_t nrows,
                                                               uint32_t col, Params prm, PoissonTable pt,
                                                               double* __restrict__ out, int32_t* flag) {
  __shared__ double lds[kGTable];
  const sf::GammaGuide T = stage_guide(pt.guide, lds);
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  for (int64_t i = (int64_t)blockIdx.x * kGBlock + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * kGBlock) {
    const double x = gamma_ppf_lds(lhs_quantile(ph, fp, (uint64_t)(row0 + i), col), prm, pt, T);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

// scalar shape with a built guide, scalar loc / scale
bool gamma_lds_ok(int dist, const Params& prm, const PoissonTable& pt) {
  return dist == PBH_DIST_GAMMA && pt.has_gamma && pt.guide.m == sf::kGammaGuideM && !prm.ptr[0] &&
         !prm.ptr[1] && !prm.ptr[2];
}

unsigned gamma_lds_grid(int64_t n) { return grid_for(n, kGBlock, 256); }  // one workgroup per CU

// ---------------------------------------------------------------- poisson: CDF table in LDS
// The same gather pattern: poisson_from_table reads guide[floor(q 2^11)] and then cdf[lo..]
// at random positions, two dependent gathers per draw.  The CDF table (32 sd + 53 entries), its
// scipy windows (one double per entry) and the 2048-entry guide are staged in LDS (dynamic,
// <= 56 KiB) when the table is short enough; same table, same search, same result.
constexpr int64_t kPoissonLdsMaxLen = 3072;

PBH_DI PoissonTable stage_poisson(const PoissonTable& pt, double* lds) {
  const int nb = 1 << kPoissonGuideBits;
  int32_t* g = reinterpret_cast<int32_t*>(lds + 2 * pt.len);
  for (int k = threadIdx.x; k < (int)pt.len; k += blockDim.x) {
    lds[k] = pt.cdf[k];
    lds[pt.len + k] = pt.win[k];
  }
  for (int k = threadIdx.x; k < nb; k += blockDim.x) g[k] = pt.cdf_guide[k];
  __syncthreads();
  PoissonTable local = pt;
  local.cdf = lds;
  local.win = lds + pt.len;
  local.cdf_guide = g;
  return local;
}

// one atomic per wave: the lanes with sl set append index i to the global list (slow[0] = count)
__device__ __forceinline__ void append_slow(bool sl, int64_t i, unsigned long long* slow, uint32_t cap) {
  const uint64_t m = __ballot(sl);
  if (!m) return;  // wave-uniform
  const int lane = threadIdx.x & 63, leader = __builtin_ctzll(m);
  unsigned long long b0 = 0;
  if (lane == leader) b0 = atomicAdd(&slow[0], (unsigned long long)__popcll(m));
  b0 = __shfl(b0, leader, 64);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const unsigned long long k = b0 + (unsigned long long)__popcll(m & below);
  if (sl && k < cap) slow[1 + k] = (unsigned long long)i;
}

// The table lookup only (poisson_ppf_fast); the rare lanes -- scipy's windows, outside the table,
// the deep tail -- go to the slow list for k_ppf_poisson_slow
__global__ __launch_bounds__(kBlock) PBH_OCC void k_ppf_poisson_lds(const double* __restrict__ q, int64_t q_stride,
                                                            int64_t n, Params prm, PoissonTable pt,
                                                            double* __restrict__ out, int32_t* flag,
                                                            unsigned long long* __restrict__ slow, uint32_t cap) {
  extern __shared__ double plds[];
  const PoissonTable T = stage_poisson(pt, plds);
  // 4 items per thread per step, their loads issued together (4 independent chains, as in
  // k_place_gen_poisson)
  constexpr int kPer = 4;
  bool bad = false;  // a non-finite output, flagged once per thread at the end
  for (int64_t b = (int64_t)blockIdx.x * kBlock * kPer; b < n; b += (int64_t)gridDim.x * kBlock * kPer) {
    double qv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = b + j * kBlock + threadIdx.x;
      qv[j] = i < n ? q[i * q_stride] : 0.5;
    }
    double x[kPer];
    bool ok[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) ok[j] = poisson_ppf_fast(qv[j], prm.val[0], prm.val[1], T, &x[j]);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = b + j * kBlock + threadIdx.x;
      if (i < n && ok[j]) {
        out[i] = x[j];
        bad |= !isfinite(x[j]);
      }
      append_slow(i < n && !ok[j], i, slow, cap);
    }
  }
  flag_nonfinite(flag, bad);
}

__global__ __launch_bounds__(kBlock) PBH_OCC void k_lhs_ppf_poisson_lds(uint64_t seed, int64_t n, int64_t row0,
                                                                int64_t nrows, uint32_t col, Params prm,
                                                                PoissonTable pt, double* __restrict__ out,
                                                                int32_t* flag, unsigned long long* __restrict__ slow,
                                                                uint32_t cap) {
  extern __shared__ double plds[];
  const PoissonTable T = stage_poisson(pt, plds);
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  bool bad = false;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock; i0 < nrows; i0 += (int64_t)gridDim.x * kBlock) {
    const int64_t i = i0 + threadIdx.x;
    const bool valid = i < nrows;
    double x = 0.0;
    bool ok = true;
    if (valid) {
      const double q = lhs_quantile(ph, fp, (uint64_t)(row0 + i), col);
      ok = poisson_ppf_fast(q, prm.val[0], prm.val[1], T, &x);
      if (ok) {
        out[i] = x;
        bad |= !isfinite(x);
      }
    }
    append_slow(valid && !ok, i, slow, cap);
  }
  flag_nonfinite(flag, bad);
}

// dynamic LDS bytes of the poisson LDS kernels, or 0 when they do not apply
size_t poisson_lds_bytes(int dist, const Params& prm, const PoissonTable& pt) {
  if (dist != PBH_DIST_POISSON || !pt.cdf || !pt.cdf_guide || pt.len <= 0 || pt.len > kPoissonLdsMaxLen ||
      prm.ptr[0] || prm.ptr[1])
    return 0;
  return (size_t)2 * pt.len * sizeof(double) + ((size_t)1 << kPoissonGuideBits) * sizeof(int32_t);
}

// The same LHS column in stratum order: out[t] = ppf(q) for the row pi^-1(t) that holds
// stratum t.  Bit-identical to k_lhs_ppf's value for that row; non-decreasing in t whenever
// the ppf is monotone.  With counts != NULL the kernel also counts, over the pairs (t, t + 1)
// inside the segment, counts[0] += #ties and counts[1] += #inversions (what k_check_sorted
// would find, without re-reading the column): lane l compares with lane l + 1 through a wave
// shuffle, the last lane of a wave evaluates stratum t + 1 itself; one atomic pair per block.
//
// out may be NULL (counts only: the step-4 finish regenerates the values, nothing reads the
// stored column).  With heads != NULL the counting pass also appends, unordered, every run
// head t + 1 with x[t] != x[t + 1] at heads[*hcur] (the caller seeds heads[0] = 0, *hcur = 1
// for t0 = 0); at most hcap are written, *hcur counts them all (k_sort_heads orders them).
template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_lhs_sorted_ppf(uint64_t seed, int64_t n, int64_t t0, int64_t nt,
                                                           uint32_t col, Params prm, PoissonTable pt,
                                                           double* __restrict__ out, int32_t* flag,
                                                           unsigned long long* counts, uint32_t* __restrict__ heads,
                                                           uint32_t* __restrict__ hcur, uint32_t hcap) {
  __shared__ unsigned long long sh[2][kBlock / 64];
  Philox ph(seed);
  auto value = [&](int64_t t) {  // stratum t's point: no permutation needed (lhs_sorted_quantile)
    const double q = lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n);
    return ppf_one<D, 0, true>(q, prm.val[0], prm.val[1], prm.val[2], pt);
  };
  const int lane = threadIdx.x & 63;
  unsigned long long ties = 0, inv = 0;
  if (!counts) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nt; i += (int64_t)gridDim.x * kBlock) {
      const double x = value(t0 + i);
      out[i] = x;
      flag_nonfinite(flag, !isfinite(x));
    }
  } else {
    // waves advance by 63 strata and overlap by one: lane 63 evaluates the stratum the next
    // wave writes from its lane 0, so every pair (t, t + 1) meets inside one wave (a divergent
    // extra evaluation by one lane would cost the whole wave a second pass).
    const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
    const int64_t wid0 = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t iters = (nt + 63 * waves - 1) / (63 * waves);  // uniform trip count
    for (int64_t it = 0; it < iters; ++it) {
      const int64_t i = (it * waves + wid0) * 63 + lane;
      const bool valid = i < nt;
      double x = 0.0;
      if (valid) {
        x = value(t0 + i);
        if (out && lane < 63) out[i] = x;
      }
      flag_nonfinite(flag, valid && lane < 63 && !isfinite(x));
      const double nx = __shfl_down(x, 1, 64);
      const bool has_next = valid && lane < 63 && i + 1 < nt;
      ties += has_next && x == nx;
      inv += has_next && !(x <= nx);
      if (heads) {
        const bool hd = has_next && x != nx;
        const uint32_t ht = (uint32_t)(t0 + i + 1);
        const uint64_t m = __ballot(hd);
        if (m) {  // wave-uniform
          const int leader = __builtin_ctzll(m);
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(hcur, (uint32_t)__popcll(m));
          base = __shfl(base, leader, 64);
          const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
          const uint32_t slot = base + (uint32_t)__popcll(m & lt);
          if (hd && slot < hcap) heads[slot] = ht;
        }
      }
    }
  }
  if (counts) {
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
      unsigned long long a = 0, b = 0;
      for (int w = 0; w < kBlock / 64; ++w) {
        a += sh[0][w];
        b += sh[1][w];
      }
      if (a) atomicAdd(&counts[0], a);
      if (b) atomicAdd(&counts[1], b);
    }
  }
}

// ---------------------------------------------------------------- tie / inversion certificate
// The deferred tie / inversion check of a continuous column (pbh_api.hip, PBH_DEFER_COUNTS) without
// evaluating the inverse CDF at every stratum.  Adjacent strata t, t + 1 have quantiles
// q_t < q_t+1 (the LHS jitter u lies in [0, 1)), and the exact inverse CDF F is strictly increasing
// on the support, with F(q_t+1) - F(q_t) = dq / f(xi) by the mean value theorem.  The device's F
// differs from the exact one by at most eps (|loc| + scale |y|) (y the standardised value; eps
// per family, gen_cert_gap), so the two computed values are strictly ordered whenever
// dq > 2 eps sup_y f0(y) (|loc| / scale + |y|) =: T.  k_cert_scan lists the pairs with dq <= T (a
// fraction (T n)^2 / 2 of them: ~1e-3 for norm(0, 1) at N = 1e8) from the quantiles alone (one
// SplitMix64 per stratum, no inverse CDF); k_cert_eval evaluates only those pairs exactly and
// counts their ties / inversions, plus both ends of the segment (a non-finite end sets the flag;
// monotone and finite at both ends means finite throughout).  Any count, a list overflow or a
// non-finite end is reported as a tie, and the caller redoes the call with the exact counts
// (k_lhs_sorted_ppf): the certificate can only confirm "no tie, no inversion".
__global__ __launch_bounds__(kBlock) PBH_OCC void k_cert_scan(uint64_t seed, int64_t n, int64_t t0, int64_t nt, uint32_t col,
                                                      double T, uint32_t* __restrict__ list, uint32_t cap,
                                                      uint32_t* __restrict__ count) {
  // candidates gather in LDS and leave with one global atomic per block flush: one atomic per
  // wave on the single counter serialised ~4 ms per column at a 1% candidate rate
  constexpr int kBuf = 2048;
  __shared__ uint32_t buf[kBuf];
  __shared__ uint32_t nbuf, gbase;
  Philox ph(seed);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) nbuf = 0;
  __syncthreads();
  auto flush = [&]() {  // block-uniform call
    __syncthreads();
    const uint32_t m = nbuf < kBuf ? nbuf : kBuf;
    if (threadIdx.x == 0) gbase = m ? atomicAdd(count, m) : 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < m; k += kBlock)
      if (gbase + k < cap) list[gbase + k] = buf[k];
    __syncthreads();
    if (threadIdx.x == 0) nbuf = 0;
    __syncthreads();
  };
  const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t wid0 = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int64_t iters = (nt + 63 * waves - 1) / (63 * waves);  // waves advance by 63 and overlap by one
  for (int64_t it = 0; it < iters; ++it) {
    const int64_t i = (it * waves + wid0) * 63 + lane;
    const bool valid = i < nt;
    const double q = valid ? lhs_sorted_quantile(ph, (uint64_t)(t0 + i), col, (uint64_t)n) : 0.0;
    const double nq = __shfl_down(q, 1, 64);
    const bool cand = valid && lane < 63 && i + 1 < nt && !(nq - q > T);
    const uint64_t m = __ballot(cand);
    if (m) {
      const int leader = __builtin_ctzll(m);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&nbuf, (uint32_t)__popcll(m));
      base = __shfl(base, leader, 64);
      const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
      const uint32_t slot = base + (uint32_t)__popcll(m & lt);
      if (cand && slot < kBuf) buf[slot] = (uint32_t)i;  // offset in the segment
      if (cand && slot >= kBuf && slot - kBuf < cap) {     // (LDS full: straight out, rare)
        const uint32_t g = atomicAdd(count, 1u);
        if (g < cap) list[g] = (uint32_t)i;
      }
    }
    // block-uniform decision: every wave reads nbuf between two barriers (an iteration appends at
    // most 4 x 63 < kBlock entries, so the buffer cannot overflow before the next check)
    __syncthreads();
    const bool full = nbuf >= kBuf - kBlock;
    __syncthreads();
    if (full) flush();
  }
  flush();
}

template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_cert_eval(uint64_t seed, int64_t n, int64_t t0, int64_t nt, uint32_t col,
                                                      Params prm, PoissonTable pt, const uint32_t* __restrict__ list,
                                                      uint32_t cap, const uint32_t* __restrict__ count, int32_t* flag,
                                                      unsigned long long* counts) {
  Philox ph(seed);
  auto value = [&](int64_t t) {
    return ppf_one<D, 0, true>(lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n), prm.val[0], prm.val[1],
                               prm.val[2], pt);
  };
  const uint32_t m = *count;
  unsigned long long ties = 0, inv = 0;
  if (blockIdx.x == 0 && threadIdx.x < 2) {  // the segment's ends
    const double x = value(threadIdx.x == 0 ? t0 : t0 + nt - 1);
    if (!isfinite(x)) {
      if (flag) atomicOr(flag, 1);
      ties += 1;
    }
    if (threadIdx.x == 0 && m > cap) ties += 1;  // unlisted candidates: not certified
  }
  const uint32_t mm = m < cap ? m : cap;
  for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < mm; k += gridDim.x * kBlock) {
    const int64_t t = t0 + list[k];
    const double a = value(t), b = value(t + 1);
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

// ---------------------------------------------------------------- step-4 placement, generated columns
// The last pass of Iman-Conover step 4 for a generated column (pbh_step4.hip): the pairs
// (row << 32 | p) of every block of 4096 consecutive rows are together, and Y[row] = sort(X)[p]
// is this column's value in stratum p, regenerated here (lhs_sorted_quantile + ppf_one: the
// same function k_lhs_sorted_ppf evaluates, so bit-identical to the stored sorted column)
// instead of being carried through the placement passes.  The block is assembled in LDS and
// written out contiguously.  norm / lognorm compact ndtri's tail per wave (k_place_gen_w);
// gamma / poisson stage their tables in LDS (random p: table gathers); a discrete column with its
// runs reads each run's value (k_place_gen_runs).
constexpr int kGenRows = 1 << kGenPlaceShift;

// BYROW (the row owner of a row-sharded run, pbh_lhs_values_at): the item at position p of a block
// is row r0 + p itself, its stratum pidx[r0 + p] -- the sorted positions the column's owner sent
// back -- for `rows` rows of an n-row design; otherwise the (row << 32 | p) pairs, rows == n.
template <int D, bool BYROW = false>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_place_gen(const uint64_t* __restrict__ pairs,
                                                      const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                      uint64_t seed, uint32_t col, Params prm, PoissonTable pt,
                                                      double* __restrict__ y, int64_t y_rs, int32_t* __restrict__ idx,
                                                      const int32_t* __restrict__ state) {
  static_assert(D != PBH_DIST_NORM && D != PBH_DIST_LOGNORM, "norm / lognorm: k_place_gen_w");
  if (state && *state) return;
  __shared__ double buf[kGenRows];
  Philox ph(seed);
  const double p0 = prm.val[0], p1 = prm.val[1], p2 = prm.val[2];
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    for (int h = 0; h < kGenRows; h += kCTile) {
      // every pair of the tile first (loads issued together)
      uint64_t pa[kCIpt];
#pragma unroll
      for (int j = 0; j < kCIpt; ++j) {
        const int p = h + j * kBlock + threadIdx.x;
        pa[j] = p >= cnt ? 0ull : BYROW ? (uint64_t)pidx[r0 + p] : pairs[r0 + p];
      }
#pragma unroll
      for (int j = 0; j < kCIpt; ++j) {
        const int p = h + j * kBlock + threadIdx.x;
        if (p >= cnt) continue;
        uint32_t t;
        int off;
        if constexpr (BYROW) {
          t = (uint32_t)pa[j];
          off = p;
        } else {
          const uint64_t pr = pa[j];
          t = (uint32_t)pr;
          const int64_t row = (int64_t)(pr >> 32);
          if (idx) idx[row] = (int32_t)t;
          off = (int)(row - r0);
        }
        buf[off] = ppf_one<D>(lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n), p0, p1, p2, pt);
      }
    }
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// norm / lognorm placement with ndtri's tail compacted per WAVE (as k_perm_scores): wave w takes
// items [1024 w, 1024 w + 1024) of the 4096-row block, 8 per lane per step, puts the centre values
// into the block's LDS image and pushes the tail arguments onto its own stack, which it drains 64
// at a time (full width) after each half-step; the last < 64 go before the block's one barrier.
// k_place_gen's block-wide queue spent two barriers and a ragged drain on every 2048 items.
constexpr int kPGQ = 192;  // a wave's tail stack: at most 63 left over + 2 x 64 pushed in a quarter-step
constexpr int kPGStep = 2;  // items per lane between two drains (the stacks keep 4 blocks per CU)

template <int D, bool BYROW = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_place_gen_w(const uint64_t* __restrict__ pairs,
                                                        const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                        uint64_t seed, uint32_t col, Params prm, PoissonTable pt,
                                                        double* __restrict__ y, int64_t y_rs,
                                                        int32_t* __restrict__ idx, const int32_t* __restrict__ state) {
  static_assert(D == PBH_DIST_NORM || D == PBH_DIST_LOGNORM, "norm / lognorm only");
  if (state && *state) return;
  __shared__ double buf[kGenRows];
  __shared__ double qarg[kBlock / 64][kPGQ];
  __shared__ uint16_t qpos[kBlock / 64][kPGQ];
  Philox ph(seed);
  const double p0 = prm.val[0], p1 = prm.val[1], p2 = prm.val[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  double* qa = qarg[w];
  uint16_t* qp = qpos[w];
  constexpr int kPerWave = kGenRows / (kBlock / 64);
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    int qc = 0;  // wave-uniform
    for (int h = w * kPerWave; h < (w + 1) * kPerWave; h += 512) {
      uint64_t pa[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = h + j * 64 + lane;
        pa[j] = p >= cnt ? 0ull : BYROW ? (uint64_t)pidx[r0 + p] : pairs[r0 + p];
      }
#pragma unroll
      for (int part = 0; part < 8 / kPGStep; ++part) {
#pragma unroll
        for (int jj = 0; jj < kPGStep; ++jj) {
          const int j = part * kPGStep + jj;
          const int p = h + j * 64 + lane;
          const bool valid = p < cnt;
          double q = 0.5;
          int off = 0;
          if (valid) {
            uint32_t t;
            if constexpr (BYROW) {
              t = (uint32_t)pa[j];
              off = p;
            } else {
              const uint64_t pr = pa[j];
              t = (uint32_t)pr;
              const int64_t row = (int64_t)(pr >> 32);
              if (idx) idx[row] = (int32_t)t;
              off = (int)(row - r0);
            }
            q = lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n);
          }
          const bool tail = valid && normal_takes_tail(q, normal_loc<D>(p0, p1));
          if (valid && !tail) buf[off] = ppf_one<D, 1>(q, p0, p1, p2, pt);
          const uint64_t m = __ballot(tail);
          if (tail) {
            const int slot = qc + (int)__popcll(m & lt);
            qa[slot] = q;
            qp[slot] = (uint16_t)off;
          }
          qc += (int)__popcll(m);
        }
        // the stack is written by some lanes and read by others of the same wave: keep the
        // compiler from moving LDS accesses across the push / drain boundary (no instruction)
        __builtin_amdgcn_wave_barrier();
        while (qc >= 64) {  // full-width batches off the top of the stack
          qc -= 64;
          buf[qp[qc + lane]] = ppf_one<D, 2>(qa[qc + lane], p0, p1, p2, pt);
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (lane < qc) buf[qp[lane]] = ppf_one<D, 2>(qa[lane], p0, p1, p2, pt);
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// gamma with the guide table in LDS (120 KiB) next to the block (32 KiB): one 1024-thread
// workgroup per CU
template <bool BYROW = false>
__global__ __launch_bounds__(kGBlock) void k_place_gen_gamma(const uint64_t* __restrict__ pairs,
                                                             const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                             uint64_t seed, uint32_t col, Params prm, PoissonTable pt,
                                                             double* __restrict__ y, int64_t y_rs,
                                                             int32_t* __restrict__ idx,
                                                             const int32_t* __restrict__ state) {
  if (state && *state) return;
  __shared__ double lds[kGTable];
  __shared__ double buf[kGenRows];
  // items whose value needs igami's own iteration (outside the grid, an interval that failed its
  // check, q at 0 or 1, invalid parameters): queued by position in the block and evaluated by
  // gamma_ppf_lds after the interpolated ones -- so the hot loop carries no igami code (inlined,
  // it sized the registers of the whole kernel and spilled, 1.6 GB of scratch reloads per launch)
  constexpr int kQCap = 2048;
  __shared__ uint16_t slowq[kQCap];
  __shared__ int nslow;
  const sf::GammaGuide T = stage_guide(pt.guide, lds);
  Philox ph(seed);
  const double shape = prm.val[0], loc = prm.val[1], scale = prm.val[2];
  const bool cond0 = (shape > 0.0) && (scale > 0.0) && (loc == loc) && pt.has_gamma;
  constexpr int kPer = kGenRows / kGBlock;
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    if (threadIdx.x == 0) nslow = 0;
    __syncthreads();
    uint64_t pr[kPer];  // BYROW: the same (row << 32 | p) form, built from the row and pidx
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int p = j * kGBlock + threadIdx.x;
      if constexpr (BYROW)
        pr[j] = p < cnt ? ((uint64_t)(r0 + p) << 32) | pidx[r0 + p] : ~0ull;
      else
        pr[j] = p < cnt ? pairs[r0 + p] : ~0ull;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool valid = pr[j] != ~0ull;
      const double q = lhs_sorted_quantile(ph, (uint64_t)(uint32_t)pr[j], col, (uint64_t)n);
      // igami_guided's interpolation branch, operation for operation
      bool fast = valid && cond0 && q > 0.0 && q < 1.0;
      double v = 0.0;
      if (fast) {
        const double w = sf::log_tab(q / (1.0 - q));
        const double u = (w - T.z0) * T.inv_h;
        fast = u >= 0.0 && u < (double)(T.m - 1);
        if (fast) {
          const int jj = (int)u;
          const double yy = sf::guide_interp(T, jj, u - (double)jj);
          fast = yy >= -680.0 && yy <= 700.0 && T.ok[jj] != 0.0;
          if (fast) v = sf::exp_tab(yy) * scale + loc;
        }
      }
      if (valid) {
        const int64_t row = (int64_t)(pr[j] >> 32);
        if (!BYROW && idx) idx[row] = (int32_t)(uint32_t)pr[j];
        if (fast) {
          buf[row - r0] = v;
        } else {
          const int slot = atomicAdd(&nslow, 1);
          if (slot < kQCap) slowq[slot] = (uint16_t)(j * kGBlock + threadIdx.x);
        }
      }
    }
    __syncthreads();
    const int ns = nslow;
    const int nd = ns <= kQCap ? ns : cnt;  // queue overflow: recompute the whole block
    for (int i = threadIdx.x; i < nd; i += kGBlock) {
      const int p = ns <= kQCap ? slowq[i] : i;
      const uint64_t prr = BYROW ? ((uint64_t)(r0 + p) << 32) | pidx[r0 + p] : pairs[r0 + p];
      buf[(int64_t)(prr >> 32) - r0] =
          gamma_ppf_lds(lhs_sorted_quantile(ph, (uint64_t)(uint32_t)prr, col, (uint64_t)n), prm, pt, T);
    }
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kGBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kGBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// gamma with a window of the guide table in LDS: a column of n strata draws its quantiles from
// [~1 / n, 1 - ~1 / n], i.e. w = log(q / (1 - q)) within about +-log n, a third of the table's
// [-80, 40] at n = 1e8 (1280 nodes: 40 KiB next to the 32 KiB block).  Two 512-thread workgroups
// per CU then take the place of one 1024-thread one (k_place_gen_gamma), so one workgroup's
// barriers and loads overlap the other's arithmetic.  The interpolation is guide_interp's
// arithmetic on the same node values, so every value is bit-identical.  An item the window
// cannot interpolate (its interval outside the window -- a quantile within 1 / (4 n) of 0 or 1 --
// or an interval without the midpoint check, q at 0 or 1, invalid parameters) is appended to a
// global list instead, and k_place_gen_gamma_slow evaluates the list with ppf_one and the global
// table (the same function and values as gamma_ppf_lds) after the placement: igami's iteration
// is not in this kernel at all, whose registers it would otherwise size (80+ VGPRs of spills on
// the hot path, 0.4 GB of scratch traffic per launch).  A list that overflows (a shape whose guide
// leaves many intervals unchecked) makes the second kernel evaluate every row of the column.
constexpr int kGWBlock = 512;
constexpr int kGWin = 1280;  // window nodes of the step-4 placement

// nodes [*j0, *j0 + *jn) of the guide cover w in [-wl, wl]; false when more than cap nodes
// PBH_GAMMA_WIN=0: the whole table in LDS, one 1024-thread workgroup per CU
bool gamma_win_on() {
  static const bool on = [] {
    const char* e = getenv("PBH_GAMMA_WIN");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool gamma_window_w(double wl, const sf::GammaGuide& T, int cap, int* j0, int* jn) {
  const int lo = (int)floor((-wl - T.z0) * T.inv_h) - 1, hi = (int)ceil((wl - T.z0) * T.inv_h) + 2;
  *j0 = lo < 0 ? 0 : lo;
  const int h = hi > T.m ? T.m : hi;
  *jn = h - *j0;
  return *jn >= 2 && *jn <= cap;
}

bool gamma_window(int64_t n, const sf::GammaGuide& T, int* j0, int* jn) {
  return gamma_window_w(log(4.0 * (double)n), T, kGWin, j0, jn);  // q in [1 / (4 n), 1 - 1 / (4 n)]
}

template <bool BYROW = false>
__global__ __launch_bounds__(kGWBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_place_gen_gamma_w(const uint64_t* __restrict__ pairs,
                                                                const uint32_t* __restrict__ pidx, int64_t rows,
                                                                int64_t n, uint64_t seed, uint32_t col, Params prm,
                                                                PoissonTable pt, double* __restrict__ y, int64_t y_rs,
                                                                int32_t* __restrict__ idx,
                                                                const int32_t* __restrict__ state, int j0, int jn,
                                                                unsigned long long* __restrict__ slow, uint32_t cap) {
  if (state && *state) return;
  __shared__ double win[4 * kGWin];  // y, d1, d2, ok of nodes j0 .. j0 + jn - 1
  __shared__ double buf[kGenRows];
  __shared__ double ltab_s[kLogTabN], etab_s[kExpTabN];
  double *ltab = ltab_s, *etab = etab_s;
  stage_logexp(ltab, etab);  // (the window's barrier follows)
  const sf::GammaGuide& G = pt.guide;
  for (int k = threadIdx.x; k < 4 * jn; k += kGWBlock) {
    const int a = k / jn, i = k - a * jn;
    win[a * kGWin + i] = G.y[(int64_t)a * G.m + j0 + i];  // the four global arrays are contiguous
  }
  __syncthreads();
  Philox ph(seed);
  const double shape = prm.val[0], loc = prm.val[1], scale = prm.val[2];
  const bool cond0 = (shape > 0.0) && (scale > 0.0) && (loc == loc) && pt.has_gamma;
  constexpr int kPer = kGenRows / kGWBlock;
  // the next block's pairs are loaded while this one is evaluated (register prefetch)
  auto load = [&](int64_t b, uint64_t* pr) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = r0 < rows ? (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows) : 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int p = j * kGWBlock + threadIdx.x;
      if constexpr (BYROW)
        pr[j] = p < cnt ? ((uint64_t)(r0 + p) << 32) | pidx[r0 + p] : ~0ull;
      else
        pr[j] = p < cnt ? pairs[r0 + p] : ~0ull;
    }
  };
  uint64_t pn[kPer];
  load(blockIdx.x, pn);
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    uint64_t pr[kPer];
#ifndef PBH_NO_PREFETCH
#pragma unroll
    for (int j = 0; j < kPer; ++j) pr[j] = pn[j];
    load(b + gridDim.x, pn);
#else
    load(b, pr);
#endif
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool valid = pr[j] != ~0ull;
      const double q = lhs_sorted_quantile(ph, (uint64_t)(uint32_t)pr[j], col, (uint64_t)n);
      // igami_guided's interpolation branch, operation for operation, on the window
      bool fast = valid && cond0 && q > 0.0 && q < 1.0;
      double v = 0.0;
      if (fast) {
        const double w = sf::log_odds_at(q, ltab);
        const double u = (w - G.z0) * G.inv_h;
        fast = u >= 0.0 && u < (double)(G.m - 1);
        if (fast) {
          const int jj = (int)u;
          const int jl = jj - j0;
          fast = jl >= 0 && jl < jn - 1;
          if (fast) {
            const double yy = sf::guide_interp_arr(win, win + kGWin, win + 2 * kGWin, G.h, jl, u - (double)jj);
            fast = yy >= -680.0 && yy <= 700.0 && win[3 * kGWin + jl] != 0.0;
            if (fast) v = sf::exp_tab_at(yy, etab) * scale + loc;
          }
        }
      }
      if (valid) {
        const int64_t row = (int64_t)(pr[j] >> 32);
        if (!BYROW && idx) idx[row] = (int32_t)(uint32_t)pr[j];
        buf[row - r0] = v;  // a slow item's value is written again by k_place_gen_gamma_slow
        if (!fast) {
          const unsigned long long k = atomicAdd(&slow[0], 1ull);
          if (k < cap) slow[1 + k] = pr[j];
        }
      }
    }
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kGWBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kGWBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// The window kernel's slow list: y[row] = ppf_one (igami with the global guide) for every listed
// (row << 32 | p), or, when the list overflowed, for every row of the column
template <bool BYROW = false>
__global__ __launch_bounds__(256) void k_place_gen_gamma_slow(const uint64_t* __restrict__ pairs,
                                                              const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                              uint64_t seed, uint32_t col, Params prm, PoissonTable pt,
                                                              double* __restrict__ y, int64_t y_rs,
                                                              const int32_t* __restrict__ state,
                                                              const unsigned long long* __restrict__ slow,
                                                              uint32_t cap) {
  if (state && *state) return;
  Philox ph(seed);
  const unsigned long long count = slow[0];
  const bool all = count > cap;
  const int64_t m = all ? rows : (int64_t)count;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) {
    uint64_t pr;
    if (!all)
      pr = slow[1 + i];
    else if constexpr (BYROW)
      pr = ((uint64_t)i << 32) | pidx[i];
    else
      pr = pairs[i];
    const int64_t row = (int64_t)(pr >> 32);
    y[row * y_rs] = ppf_one<PBH_DIST_GAMMA>(lhs_sorted_quantile(ph, (uint64_t)(uint32_t)pr, col, (uint64_t)n),
                                            prm.val[0], prm.val[1], prm.val[2], pt);
  }
}

// ---------------------------------------------------------------- gamma sweep on a guide window
// (round 5) k_ppf_gamma_lds stages the whole 120 KiB guide, so one 1024-thread workgroup runs per
// CU, with two block barriers per 4096-item tile around its LDS slow queue and igami's iteration
// inline (128 VGPRs with spills): latency-bound (wave_active 0.28).  These kernels stage the window
// of the guide that quantiles in [2.3e-9, 1 - 2.3e-9] reach (|w| <= 19.9: 1275 nodes, 40 KiB, as
// the step-4 placement does), take no barrier after the staging, and append every item the window
// cannot interpolate (a quantile beyond the window, an interval without the midpoint check, q at 0
// or 1, invalid parameters) to a global list, one atomic per wave; k_ppf_gamma_slow then evaluates
// the list with ppf_one and the global table -- the same function and values as gamma_ppf_lds, so
// every value is bit-identical -- or every row when the list overflowed.
constexpr double kGSweepW = 19.9;
#ifndef PBH_GSWEEP_PER
#define PBH_GSWEEP_PER 4
#endif
#ifndef PBH_GSWEEP_BLOCK
#define PBH_GSWEEP_BLOCK 512
#endif
#ifndef PBH_GSWEEP_WAVES
#define PBH_GSWEEP_WAVES 6
#endif
constexpr int kGSweepPer = PBH_GSWEEP_PER;  // items per thread per tile, their quantiles loaded a tile ahead
constexpr int kGSBlock = PBH_GSWEEP_BLOCK;  // 512: three workgroups per CU (46 KiB of LDS each), 80 VGPRs

struct GammaLhs {  // the fused native-LHS column (LHS = true): quantile of row row0 + i
  uint64_t seed;
  int64_t n, row0;
  uint32_t col;
};

template <bool LHS>
__global__ __launch_bounds__(kGSBlock) __attribute__((amdgpu_waves_per_eu(PBH_GSWEEP_WAVES))) void k_ppf_gamma_w(
    const double* __restrict__ q, int64_t q_stride, int64_t n, GammaLhs lc, Params prm, PoissonTable pt,
    double* __restrict__ out, int32_t* flag, int j0, int jn, unsigned long long* __restrict__ slow, uint32_t cap) {
  __shared__ double win[4 * kGWin];  // y, d1, d2, ok of nodes j0 .. j0 + jn - 1
  __shared__ double ltab_s[kLogTabN], etab_s[kExpTabN];
  double *ltab = ltab_s, *etab = etab_s;
  stage_logexp(ltab, etab);
  const sf::GammaGuide& G = pt.guide;
  for (int k = threadIdx.x; k < 4 * jn; k += kGSBlock) {
    const int a = k / jn, i = k - a * jn;
    win[a * kGWin + i] = G.y[(int64_t)a * G.m + j0 + i];  // the four global arrays are contiguous
  }
  __syncthreads();
  Philox ph(lc.seed);
  FeistelPerm fp(ph, (uint64_t)(LHS ? lc.n : 1), lc.col);
  const double shape = prm.val[0], loc = prm.val[1], scale = prm.val[2];
  const bool cond0 = (shape > 0.0) && (scale > 0.0) && (loc == loc) && pt.has_gamma;
  constexpr int kTile = kGSweepPer * kGSBlock;
  const int64_t step = (int64_t)gridDim.x * kTile;
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  auto quantile = [&](int64_t i) -> double {
    if constexpr (LHS)
      return lhs_quantile(ph, fp, (uint64_t)(lc.row0 + i), lc.col);
    else
      return q[i * q_stride];
  };
  double qn[kGSweepPer];
  if constexpr (!LHS) {
#pragma unroll
    for (int j = 0; j < kGSweepPer; ++j) {
      const int64_t i = (int64_t)blockIdx.x * kTile + j * kGSBlock + threadIdx.x;
      qn[j] = i < n ? q[i * q_stride] : 0.5;
    }
  }
  bool bad = false;
  for (int64_t base = (int64_t)blockIdx.x * kTile; base < n; base += step) {
    double qv[kGSweepPer];
#pragma unroll
    for (int j = 0; j < kGSweepPer; ++j) {
      if constexpr (LHS) {
        const int64_t i = base + j * kGSBlock + threadIdx.x;
        qv[j] = i < n ? quantile(i) : 0.5;
      } else {
        qv[j] = qn[j];
        const int64_t i = base + step + j * kGSBlock + threadIdx.x;
        qn[j] = i < n ? q[i * q_stride] : 0.5;
      }
    }
#pragma unroll
    for (int j = 0; j < kGSweepPer; ++j) {
      const int64_t i = base + j * kGSBlock + threadIdx.x;
      const bool valid = i < n;
      const double qq = qv[j];
      // igami_guided's interpolation branch and ppf_one's gamma wrapper, operation for operation
      bool fast = valid && cond0 && qq > 0.0 && qq < 1.0;
      double v = 0.0;
      if (fast) {
        const double w = sf::log_odds_at(qq, ltab);
        const double u = (w - G.z0) * G.inv_h;
        fast = u >= 0.0 && u < (double)(G.m - 1);
        if (fast) {
          const int jj = (int)u;
          const int jl = jj - j0;
          fast = jl >= 0 && jl < jn - 1;
          if (fast) {
            const double yy = sf::guide_interp_arr(win, win + kGWin, win + 2 * kGWin, G.h, jl, u - (double)jj);
            fast = yy >= -680.0 && yy <= 700.0 && win[3 * kGWin + jl] != 0.0;
            if (fast) v = sf::exp_tab_at(yy, etab) * scale + loc;
          }
        }
      }
      if (fast) {
        out[i] = v;
        bad |= !isfinite(v);
      }
      const bool sl = valid && !fast;
      const uint64_t m = __ballot(sl);
      if (m) {  // wave-uniform
        const int leader = __builtin_ctzll(m);
        unsigned long long b0 = 0;
        if (lane == leader) b0 = atomicAdd(&slow[0], (unsigned long long)__popcll(m));
        b0 = __shfl(b0, leader, 64);
        const unsigned long long k = b0 + (unsigned long long)__popcll(m & below);
        if (sl && k < cap) slow[1 + k] = (unsigned long long)i;
      }
    }
  }
  flag_nonfinite(flag, bad);
}

template <bool LHS>
__global__ __launch_bounds__(256) void k_ppf_gamma_slow(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                        GammaLhs lc, Params prm, PoissonTable pt,
                                                        double* __restrict__ out, int32_t* flag,
                                                        const unsigned long long* __restrict__ slow, uint32_t cap) {
  const unsigned long long count = slow[0];
  if (count == 0) return;
  const bool all = count > cap;
  const int64_t m = all ? n : (int64_t)count;
  Philox ph(lc.seed);
  FeistelPerm fp(ph, (uint64_t)(LHS ? lc.n : 1), lc.col);
  bool bad = false;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) {
    const int64_t i = all ? k : (int64_t)slow[1 + k];
    double qi;
    if constexpr (LHS)
      qi = lhs_quantile(ph, fp, (uint64_t)(lc.row0 + i), lc.col);
    else
      qi = q[i * q_stride];
    const double x = ppf_one<PBH_DIST_GAMMA>(qi, prm.val[0], prm.val[1], prm.val[2], pt);
    out[i] = x;
    bad |= !isfinite(x);
  }
  flag_nonfinite(flag, bad);
}

// The poisson sweeps' slow list: ppf_one (poisson_rare included) on the global table for the listed
// rows, or every row when the list overflowed -- the same function as the table lookup, so the same
// values.  LHS: the fused native-LHS column (the quantile of row row0 + i regenerated).
template <bool LHS>
__global__ __launch_bounds__(256) void k_ppf_poisson_slow(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                          GammaLhs lc, Params prm, PoissonTable pt,
                                                          double* __restrict__ out, int32_t* flag,
                                                          const unsigned long long* __restrict__ slow, uint32_t cap) {
  const unsigned long long count = slow[0];
  if (count == 0) return;
  const bool all = count > cap;
  const int64_t m = all ? n : (int64_t)count;
  Philox ph(lc.seed);
  FeistelPerm fp(ph, (uint64_t)(LHS ? lc.n : 1), lc.col);
  bool bad = false;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < m; k += (int64_t)gridDim.x * 256) {
    const int64_t i = all ? k : (int64_t)slow[1 + k];
    double qi;
    if constexpr (LHS)
      qi = lhs_quantile(ph, fp, (uint64_t)(lc.row0 + i), lc.col);
    else
      qi = q[i * q_stride];
    const double x = ppf_one<PBH_DIST_POISSON>(qi, prm.val[0], prm.val[1], prm.val[2], pt);
    out[i] = x;
    bad |= !isfinite(x);
  }
  flag_nonfinite(flag, bad);
}

// The poisson LDS sweep and its slow list (pbh_ppf: q given; pbh_lhs_ppf: lc, the fused LHS)
int launch_poisson_lds(const double* q, int64_t qs, int64_t n, const GammaLhs* lc, size_t pl, const Params& prm,
                       const PoissonTable& pt, double* out, int32_t* flag, hipStream_t s) {
  if (n <= 0) return PBH_OK;
  const uint32_t cap = (uint32_t)((n >> 10) + 4096 < (1u << 30) ? (n >> 10) + 4096 : (1u << 30));
  unsigned long long* slow = nullptr;
  PBH_CHECK_HIP(hipMallocAsync((void**)&slow, ((size_t)cap + 1) * 8, s));
  struct Free {
    unsigned long long* p;
    hipStream_t s;
    ~Free() { (void)hipFreeAsync(p, s); }  // stream-ordered: after the slow kernel
  } fr{slow, s};
  PBH_CHECK_HIP(hipMemsetAsync(slow, 0, 8, s));
  const GammaLhs l = lc ? *lc : GammaLhs{0, 1, 0, 0};
  const dim3 b(kBlock);
  if (lc) {
    PBH_TIMED(kKLhsPpf, s, {
      hipLaunchKernelGGL(k_lhs_ppf_poisson_lds, dim3(grid_for(n, kBlock, 256 * 8)), b, pl, s, l.seed, l.n, l.row0, n,
                         l.col, prm, pt, out, flag, slow, cap);
      hipLaunchKernelGGL(k_ppf_poisson_slow<true>, dim3(PBH_SLOW_GRID), dim3(256), 0, s, q, qs, n, l, prm, pt, out,
                         flag, slow, cap);
    });
  } else {
    PBH_TIMED(kKPpf, s, {
      hipLaunchKernelGGL(k_ppf_poisson_lds, dim3(grid_for(n, kBlock, 256 * 8)), b, pl, s, q, qs, n, prm, pt, out,
                         flag, slow, cap);
      hipLaunchKernelGGL(k_ppf_poisson_slow<false>, dim3(PBH_SLOW_GRID), dim3(256), 0, s, q, qs, n, l, prm, pt, out,
                         flag, slow, cap);
    });
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// The windowed gamma sweep (pbh_ppf / pbh_lhs_ppf with scalar a, loc, scale): false when it does not
// apply (PBH_GAMMA_WIN=0, no guide, a window wider than kGWin)
bool launch_gamma_w(const double* q, int64_t qs, int64_t n, const GammaLhs* lc, const Params& prm,
                    const PoissonTable& pt, double* out, int32_t* flag, hipStream_t s, int* status) {
  int j0 = 0, jn = 0;
  *status = PBH_OK;
  if (!gamma_win_on() || !gamma_window_w(kGSweepW, pt.guide, kGWin, &j0, &jn)) return false;
  if (n <= 0) return true;
  const uint32_t cap = (uint32_t)((n >> 8) + 4096 < (1u << 30) ? (n >> 8) + 4096 : (1u << 30));
  unsigned long long* slow = nullptr;
  if (hipMallocAsync((void**)&slow, ((size_t)cap + 1) * 8, s) != hipSuccess) {
    *status = PBH_ERR_HIP;
    set_error("pbh_ppf: hipMallocAsync of the gamma slow list failed");
    return true;
  }
  if (hipMemsetAsync(slow, 0, 8, s) != hipSuccess) {
    (void)hipFreeAsync(slow, s);
    *status = PBH_ERR_HIP;
    set_error("pbh_ppf: hipMemsetAsync failed");
    return true;
  }
  const GammaLhs l = lc ? *lc : GammaLhs{0, 1, 0, 0};
  const unsigned gw = grid_for(n, kGSweepPer * kGSBlock, 256 * 3 * 512 / kGSBlock), gs = PBH_SLOW_GRID;
  if (lc) {
    PBH_TIMED(kKLhsPpf, s, {
      hipLaunchKernelGGL(k_ppf_gamma_w<true>, dim3(gw), dim3(kGSBlock), 0, s, q, qs, n, l, prm, pt, out, flag, j0, jn,
                         slow, cap);
      hipLaunchKernelGGL(k_ppf_gamma_slow<true>, dim3(gs), dim3(256), 0, s, q, qs, n, l, prm, pt, out, flag, slow, cap);
    });
  } else {
    PBH_TIMED(kKPpf, s, {
      hipLaunchKernelGGL(k_ppf_gamma_w<false>, dim3(gw), dim3(kGSBlock), 0, s, q, qs, n, l, prm, pt, out, flag, j0,
                         jn, slow, cap);
      hipLaunchKernelGGL(k_ppf_gamma_slow<false>, dim3(gs), dim3(256), 0, s, q, qs, n, l, prm, pt, out, flag, slow,
                         cap);
    });
  }
  if (hipGetLastError() != hipSuccess) *status = PBH_ERR_HIP;
  (void)hipFreeAsync(slow, s);  // stream-ordered: after the slow kernel
  return true;
}

// poisson with the CDF table + guide in (dynamic) LDS
template <bool BYROW = false>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_place_gen_poisson(const uint64_t* __restrict__ pairs,
                                                              const uint32_t* __restrict__ pidx, int64_t rows,
                                                              int64_t n, uint64_t seed, uint32_t col, Params prm,
                                                              PoissonTable pt, double* __restrict__ y, int64_t y_rs,
                                                              int32_t* __restrict__ idx,
                                                              const int32_t* __restrict__ state) {
  if (state && *state) return;
  extern __shared__ double plds[];
  __shared__ double buf[kGenRows];
  const PoissonTable T = stage_poisson(pt, plds);
  Philox ph(seed);
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    for (int h = 0; h < kGenRows; h += 4 * kBlock) {  // 4 independent chains per thread
      uint64_t pr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = h + j * kBlock + threadIdx.x;
        if constexpr (BYROW)
          pr[j] = p < cnt ? ((uint64_t)(r0 + p) << 32) | pidx[r0 + p] : ~0ull;
        else
          pr[j] = p < cnt ? pairs[r0 + p] : ~0ull;
      }
      double v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = ppf_one<PBH_DIST_POISSON>(lhs_sorted_quantile(ph, (uint64_t)(uint32_t)pr[j], col, (uint64_t)n),
                                         prm.val[0], prm.val[1], prm.val[2], T);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (pr[j] != ~0ull) {
          const int64_t row = (int64_t)(pr[j] >> 32);
          if (!BYROW && idx) idx[row] = (int32_t)(uint32_t)pr[j];
          buf[row - r0] = v[j];
        }
      }
    }
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// A discrete column's placement from its runs (gen_set_runs): the sorted column is constant on
// each run [heads[i], heads[i + 1]) of strata, so the value of stratum p is vals[run of p] --
// bit-identical to evaluating it, by the definition of the heads (every stratum whose value
// differs from its predecessor's) -- found through a guide over p >> shift (most cells lie in
// one run: one compare) instead of the jitter hash and the CDF-table search of every row.  The
// runs, their values and the guide sit in (dynamic) LDS next to the 4096-row block.
constexpr int kRunsGuideMax = 2048;
constexpr int64_t kRunsLdsMax = 1024;  // runs staged in LDS (12 B each)

__device__ __forceinline__ int runs_guide_shift(int64_t n) {
  int sh = 0;
  while (((n - 1) >> sh) + 1 > kRunsGuideMax) ++sh;
  return sh;
}

template <bool BYROW = false>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_place_gen_runs(const uint64_t* __restrict__ pairs,
                                                           const uint32_t* __restrict__ pidx, int64_t rows, int64_t n,
                                                           const uint32_t* __restrict__ heads,
                                                           const double* __restrict__ vals, int nruns,
                                                           double* __restrict__ y, int64_t y_rs,
                                                           int32_t* __restrict__ idx,
                                                           const int32_t* __restrict__ state) {
  if (state && *state) return;
  extern __shared__ double rlds[];
  __shared__ double buf[kGenRows];
  double* lv = rlds;                                   // nruns values
  uint32_t* lh = (uint32_t*)(rlds + nruns);            // nruns heads
  uint32_t* lg = lh + nruns;                           // guide
  const int sh = runs_guide_shift(n);
  const int ng = (int)(((n - 1) >> sh) + 1);
  for (int i = threadIdx.x; i < nruns; i += kBlock) {
    lv[i] = vals[i];
    lh[i] = heads[i];
  }
  __syncthreads();
  for (int g = threadIdx.x; g < ng; g += kBlock) {  // guide[g] = the run holding stratum g << sh
    const uint32_t t = (uint32_t)((int64_t)g << sh);
    int lo = 0, hi = nruns;  // first head > t
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lh[mid] <= t)
        lo = mid + 1;
      else
        hi = mid;
    }
    lg[g] = (uint32_t)(lo - 1);
  }
  __syncthreads();
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < rows; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((rows - r0) < kGenRows ? (rows - r0) : kGenRows);
    for (int h = 0; h < kGenRows; h += 4 * kBlock) {  // 4 independent chains per thread
      uint64_t pr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = h + j * kBlock + threadIdx.x;
        if constexpr (BYROW)
          pr[j] = p < cnt ? ((uint64_t)(r0 + p) << 32) | pidx[r0 + p] : ~0ull;
        else
          pr[j] = p < cnt ? pairs[r0 + p] : ~0ull;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (pr[j] != ~0ull) {
          const uint32_t t = (uint32_t)pr[j];
          uint32_t r = lg[t >> sh];
          while (r + 1 < (uint32_t)nruns && lh[r + 1] <= t) ++r;
          const int64_t row = (int64_t)(pr[j] >> 32);
          if (!BYROW && idx) idx[row] = (int32_t)t;
          buf[row - r0] = lv[r];
        }
      }
    }
    __syncthreads();
    if (y_rs == 1) {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[r0 + p] = buf[p];
    } else {
      for (int p = threadIdx.x; p < cnt; p += kBlock) y[(r0 + p) * y_rs] = buf[p];
    }
    __syncthreads();
  }
}

// counts[0] += #(x[t] == x[t+1]), counts[1] += #(x[t] > x[t+1] or unordered)
// (kCheckU pairs per thread and step, their loads issued together: one pair per step left each
// wave a single load in flight, 111 us per 1e7)
constexpr int kCheckU = 4;
__global__ __launch_bounds__(kBlock) void k_check_sorted(const double* __restrict__ x, int64_t n,
                                                         unsigned long long* counts) {
  unsigned long long ties = 0, inv = 0;
  for (int64_t base = (int64_t)blockIdx.x * kBlock * kCheckU; base + 1 < n;
       base += (int64_t)gridDim.x * kBlock * kCheckU) {
    double a[kCheckU], b[kCheckU];
#pragma unroll
    for (int u = 0; u < kCheckU; ++u) {
      const int64_t t = base + u * kBlock + threadIdx.x;
      const bool in = t + 1 < n;
      a[u] = in ? x[t] : 0.0;
      b[u] = in ? x[t + 1] : 1.0;
    }
#pragma unroll
    for (int u = 0; u < kCheckU; ++u) {
      ties += (a[u] == b[u]);
      inv += !(a[u] <= b[u]);
    }
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

// Run heads appended out of order by k_lhs_sorted_ppf, sorted in place: one 1024-thread block,
// bitonic network over the next power of two (<= kHeadsCap entries, padded with 0xFFFFFFFF) in LDS.
__global__ __launch_bounds__(1024) void k_sort_heads(uint32_t* __restrict__ heads, int nh, int np2) {
  __shared__ uint32_t v[kHeadsCap];
  for (int i = threadIdx.x; i < np2; i += 1024) v[i] = i < nh ? heads[i] : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += 1024) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const uint32_t a = v[i], b = v[p];
          if ((a > b) == up) {
            v[i] = b;
            v[p] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < nh; i += 1024) heads[i] = v[i];
}

// 'average' rank of stratum t given the run heads (sorted, heads[0] = 0) of the sorted
// column: the run [s, e] holding t has ranks s+1 .. e+1, average s + 1 + (e - s) / 2
// (scipy _rankdata; the same formula as k_rank_finish).
__device__ __forceinline__ double run_average_rank(const uint32_t* __restrict__ heads, int64_t nheads, int64_t n,
                                                   int64_t t) {
  int64_t lo = 0, hi = nheads;  // first head > t
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)heads[mid] <= t)
      lo = mid + 1;
    else
      hi = mid;
  }
  const int64_t s = heads[lo - 1];
  const int64_t e = (lo < nheads ? (int64_t)heads[lo] : n) - 1;
  return (double)(s + 1) + (double)(e - s) / 2.0;
}

constexpr int64_t kLdsHeads = 4096;  // run heads staged in LDS by k_perm_scores (16 KiB)

// Van der Waerden scores of an LHS column, rows [row0, row0 + nrows), in row order: the rank
// of row r is pi(r) + 1 (untied), or the run average of stratum pi(r) (heads != NULL), so
// S[r] = Phi^-1(rank / (n + 1)) (correlation.py:394-395; sf::ppnd16) without sorting anything.
// Ranks of consecutive rows are random, so the tail (15% of the ranks, ~3x the centre's cost) is
// compacted per WAVE: each wave takes 512 consecutive rows per step (8 a lane), writes its centre
// scores straight to S (coalesced), and pushes the tail arguments onto its own LDS stack; at the
// end of the step it evaluates them 64 at a time (full width) and scatters them into S (rows of
// its recent steps: merged in L2).  No block barrier after the heads' staging, no LDS staging of
// the results, no ragged drain: round 3's block-wide queue spent ~50 VALU instructions per score
// on its bookkeeping and idled at four barriers per 2048-row tile (r4e PMC pass of
// tools/microbench_feistel.hip; interleaved A/B r4f: 22.4-22.7 against 24.3-25.1 ms per step).
// With partial != NULL each wave writes the sum of its scores to partial[wave] (the column mean of
// step 2 without re-reading S; summed in a fixed order by k_means): formed in a fixed order, since
// the queue order is the lanes' order (ballots, no atomics), so the result is deterministic.
constexpr int kWaveQ = 576;  // a wave's tail stack: at most 63 left over + 8 x 64 pushed in a step

// STRATA: the strata come from an array (strata[row0 + i], a materialised LHS column's known
// permutation, e.g. the reference stream's decoded shuffles) instead of the Feistel permutation.
template <bool STRATA>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_perm_scores(uint64_t seed, int64_t n, uint32_t col, int64_t row0,
                                                          int64_t nrows, const uint32_t* __restrict__ heads,
                                                          int64_t nheads, double* __restrict__ S,
                                                          double* __restrict__ partial,
                                                          const int32_t* __restrict__ strata) {
  __shared__ double qarg[kBlock / 64][kWaveQ];
  __shared__ uint32_t qrow[kBlock / 64][kWaveQ];
  extern __shared__ uint32_t lheads[];
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  const double np1 = (double)(n + 1);
  if (heads && nheads <= kLdsHeads) {
    for (int64_t i = threadIdx.x; i < nheads; i += kBlock) lheads[i] = heads[i];
    __syncthreads();
    heads = lheads;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  double* qa = qarg[w];
  uint32_t* qr = qrow[w];
  double sum = 0.0;
  int qc = 0;  // wave-uniform: queued tail arguments
  const int64_t gw = (int64_t)blockIdx.x * (kBlock / 64) + w, W = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t base = gw * 512; base < nrows; base += W * 512) {
    uint64_t tt[8];
    if constexpr (STRATA) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = base + j * 64 + lane;
        tt[j] = i < nrows ? (uint64_t)(uint32_t)strata[row0 + i] : 0;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t i = base + j * 64 + lane;
        tt[j] = n > 1 && i < nrows ? fp.round_trip((uint64_t)(row0 + i)) : 0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        while (tt[j] >= (uint64_t)n) tt[j] = fp.round_trip(tt[j]);
    }
#pragma unroll 2
    for (int j = 0; j < 8; ++j) {
      const int64_t i = base + j * 64 + lane;
      const bool valid = i < nrows;
      double y = 0.5;
      if (valid) {
        const uint64_t t = tt[j];
        const double rank = heads ? run_average_rank(heads, nheads, n, (int64_t)t) : (double)(t + 1);
        y = rank / np1;
      }
      const bool tail = valid && sf::ppnd16_takes_tail(y);
      if (valid && !tail) {
        const double v = sf::ppnd16_centre(y);
        S[i] = v;
        sum += v;
      }
      const uint64_t m = __ballot(tail);
      if (tail) {
        const int slot = qc + (int)__popcll(m & lt);
        qa[slot] = y;
        qr[slot] = (uint32_t)i;
      }
      qc += (int)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();  // pushes by some lanes, reads by others: no reordering across
    while (qc >= 64) {  // full-width batches off the top of the stack (the step's strata are dead here)
      qc -= 64;
      const double a = qa[qc + lane];
      const uint32_t r = qr[qc + lane];
      const double v = sf::ppnd16_tail(a);
      S[r] = v;
      sum += v;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane < qc) {  // the leftover (< 64): once per wave
    const double v = sf::ppnd16_tail(qa[lane]);
    S[qr[lane]] = v;
    sum += v;
  }
  if (partial) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) partial[gw] = sum;
  }
}

// Run heads of a sorted segment x[0..m): position p is a head when p == 0 (unless x[0] is
// the value before the segment, first_is_prev) or x[p] != x[p - 1]; heads are reported as
// t0 + p (t0 - 1 + p with first_is_prev).  Two passes: per-tile counts, then ordered writes.
constexpr int kHeadTile = kBlock * 16;

__device__ __forceinline__ bool is_head(const double* __restrict__ x, int64_t p, bool first_is_prev) {
  return p == 0 ? !first_is_prev : x[p] != x[p - 1];
}

__global__ __launch_bounds__(kBlock) void k_heads_count(const double* __restrict__ x, int64_t m, int first_is_prev,
                                                        uint32_t* __restrict__ counts) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kHeadTile;
  uint32_t c = 0;
  for (int j = 0; j < 16; ++j) {
    const int64_t p = base + j * kBlock + threadIdx.x;
    c += (p < m && is_head(x, p, first_is_prev)) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(kBlock) void k_heads_write(const double* __restrict__ x, int64_t m, int first_is_prev,
                                                        int64_t t0, const uint32_t* __restrict__ offsets,
                                                        uint32_t* __restrict__ heads) {
  __shared__ uint32_t wcount[kBlock / 64];
  __shared__ uint32_t running;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kHeadTile;
  const int64_t shift = first_is_prev ? t0 - 1 : t0;
  if (threadIdx.x == 0) running = offsets[blockIdx.x];
  __syncthreads();
  for (int j = 0; j < 16; ++j) {  // tile order = position order: row j of 256 positions
    const int64_t p = base + j * kBlock + threadIdx.x;
    const bool h = p < m && is_head(x, p, first_is_prev);
    const uint64_t bal = __ballot(h);
    const uint32_t below = (uint32_t)__popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (lane == 0) wcount[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t off = running;
    for (int v = 0; v < w; ++v) off += wcount[v];
    if (h) heads[off + below] = (uint32_t)(shift + p);
    __syncthreads();
    if (threadIdx.x == 0) running += wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
  }
}

__global__ void k_gamma_guide(double a, sf::GammaGuide T, double* y, double* d1, double* d2) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < T.m) sf::gamma_guide_entry(a, T.z0 + j * T.h, &y[j], &d1[j], &d2[j]);
}

__global__ void k_gamma_guide_check(double a, sf::GammaGuide T, double* ok) {
  int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < T.m) ok[j] = (j < T.m - 1) ? sf::gamma_guide_check(a, T, j) : 0.0;
}

// cdf[j] = pdtr(k_lo + j, mu); win[j] = the end of scipy's window above cdf[j - 1] (pbh_cdflib.h)
__global__ void k_poisson_table(double mu, int64_t k_lo, int64_t len, double* cdf, double* win) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < len) {
    cdf[j] = sf::pdtr<glibc::Math>((double)(k_lo + j), mu);  // scipy's pdtr bit for bit (pbh_glibc.h)
    win[j] = cdf::poisson_window_hi((double)(k_lo + j), mu);
  }
}

// guide[b] = first j with cdf[j] >= b / 2^kPoissonGuideBits (len when none)
__global__ void k_poisson_guide(const double* __restrict__ cdf, int64_t len, int32_t* __restrict__ guide) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (1 << kPoissonGuideBits)) return;
  const double v = (double)b / (double)(1 << kPoissonGuideBits);
  int64_t lo = 0, hi = len;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cdf[mid] >= v)
      hi = mid;
    else
      lo = mid + 1;
  }
  guide[b] = (int32_t)lo;
}

// ---------------------------------------------------------------- generators
__global__ __launch_bounds__(kBlock) void k_fill_lhs(uint64_t seed, int64_t n, int64_t row0, int64_t nrows,
                                                     int col0, double* __restrict__ q, int64_t ldq) {
  const uint32_t col = (uint32_t)(col0 + blockIdx.y);
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, col);
  double* qc = q + (int64_t)blockIdx.y * ldq;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * kBlock)
    qc[i] = lhs_quantile(ph, fp, (uint64_t)(row0 + i), col);
}

__global__ __launch_bounds__(kBlock) void k_fill_uniform(uint64_t seed, int64_t row0, int64_t nrows, int col0,
                                                         double* __restrict__ q, int64_t ldq) {
  const uint32_t col = (uint32_t)(col0 + blockIdx.y);
  Philox ph(seed);
  double* qc = q + (int64_t)blockIdx.y * ldq;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * kBlock)
    qc[i] = ph.uniform((uint64_t)(row0 + i), col, kPurposeUniform);
}

constexpr int kSobolColsPerLaunch = 16;
struct SobolArgs {
  uint32_t sv[kSobolColsPerLaunch][32];
  uint32_t shift[kSobolColsPerLaunch];
};


__global__ __launch_bounds__(kBlock) void k_fill_sobol(SobolArgs a, double scale, int64_t row0, int64_t nrows,
                                                       double* __restrict__ q, int64_t ldq) {
  __shared__ uint32_t T[1024];
  const int c = blockIdx.y;
  build_sobol_tables(a.sv[c], T);
  __syncthreads();
  double* qc = q + (int64_t)c * ldq;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * kBlock) {
    const uint32_t x = sobol_point(T, a.shift[c], (uint64_t)(row0 + i));
    qc[i] = (double)x * scale;
  }
}

// One scrambled Sobol' column fused into the inverse CDF (the "sobol" method of Node.sample,
// modeling.py:482,488): the quantile never goes through HBM.  norm / lognorm take the tail-
// compacted form.  Same points as k_fill_sobol, same values as pbh_ppf on them.
struct SobolCol {
  uint32_t sv[32];
  uint32_t shift;
  double scale;
};

template <int D, bool SC>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_sobol_ppf_c(SobolCol sc, int64_t row0, int64_t nrows, Params prm,
                                                               PoissonTable pt, double* __restrict__ out,
                                                               int32_t* flag) {
  __shared__ TailQueue tq;
  __shared__ double res[kCTile];
  __shared__ uint32_t T[1024];
  build_sobol_tables(sc.sv, T);
  __syncthreads();
  ppf_compacted<D, SC>(nrows, [&](int64_t i) { return (double)sobol_point(T, sc.shift, (uint64_t)(row0 + i)) * sc.scale; },
                   prm, pt, out, flag, tq, res);
}

template <int D>
__global__ __launch_bounds__(kBlock) PBH_OCC void k_sobol_ppf(SobolCol sc, int64_t row0, int64_t nrows, Params prm,
                                                             PoissonTable pt, double* __restrict__ out, int32_t* flag) {
  __shared__ uint32_t T[1024];
  build_sobol_tables(sc.sv, T);
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nrows; i += (int64_t)gridDim.x * kBlock) {
    const double q = (double)sobol_point(T, sc.shift, (uint64_t)(row0 + i)) * sc.scale;
    const double x = ppf_one<D>(q, prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
    out[i] = x;
    flag_nonfinite(flag, !isfinite(x));
  }
}

unsigned ppf_grid(int64_t n) { return grid_for(n, kBlock, 256 * 16); }

int launch_ppf(int dist, const double* q, int64_t qs, int64_t n, const Params& prm, const PoissonTable& pt,
               double* out, int32_t* flag, hipStream_t s) {
  dim3 g(ppf_grid(n)), b(kBlock);
  // k_ppf_v: contiguous 16-byte-aligned q and x, scalar parameters
  // (uniform / triang / expon: the draws whose arithmetic is light enough for HBM to bound them;
  // unrolling gamma's / poisson's code kVU x 2 times measured 1.7x / 1.25x slower)
  const bool light = dist == PBH_DIST_UNIFORM || dist == PBH_DIST_TRIANG || dist == PBH_DIST_EXPON;
  const bool streamable = light && qs == 1 && !prm.ptr[0] && !prm.ptr[1] && !prm.ptr[2] &&
                          ((uintptr_t)q & 15) == 0 && ((uintptr_t)out & 15) == 0;
  dim3 gv(grid_for(n, kVTile, 256 * 8));
  if (gamma_lds_ok(dist, prm, pt)) {
    int st = PBH_OK;
    if (launch_gamma_w(q, qs, n, nullptr, prm, pt, out, flag, s, &st)) return st;
    PBH_TIMED(kKPpf, s, hipLaunchKernelGGL(k_ppf_gamma_lds, dim3(gamma_lds_grid(n)), dim3(kGBlock), 0, s, q, qs, n,
                                           prm, pt, out, flag));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  if (const size_t pl = poisson_lds_bytes(dist, prm, pt)) return launch_poisson_lds(q, qs, n, nullptr, pl, prm, pt, out, flag, s);
  switch (dist) {
#define PBH_CASE(D) \
  case D:           \
    if ((D == PBH_DIST_NORM || D == PBH_DIST_LOGNORM))                                                  \
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL((scalar_params(prm) ? k_ppf_c<D, true> : k_ppf_c<D, false>),            \
                                             dim3(grid_for(n, kCTile, 8192)), b, 0, s, q, qs, n, prm, pt, out,  \
                                             flag));                                                            \
    else if (streamable)                                                                                        \
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL(k_ppf_v<D>, gv, b, 0, s, q, n, prm, pt, out, flag));               \
    else                                                                                                        \
      PBH_TIMED(kKPpf, s, hipLaunchKernelGGL(k_ppf<D>, g, b, 0, s, q, qs, n, prm, pt, out, flag));              \
    break;
    PBH_CASE(PBH_DIST_NORM)
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_LOGNORM)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
    PBH_CASE(PBH_DIST_POISSON)
#undef PBH_CASE
    default:
      set_error("pbh_ppf: unsupported distribution id %d", dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int launch_lhs_ppf(int dist, uint64_t seed, int64_t n, int64_t row0, int64_t nrows, uint32_t col,
                   const Params& prm, const PoissonTable& pt, double* out, int32_t* flag, hipStream_t s) {
  dim3 g(ppf_grid(nrows)), b(kBlock);
  if (gamma_lds_ok(dist, prm, pt)) {
    int st = PBH_OK;
    const GammaLhs lc{seed, n, row0, col};
    if (launch_gamma_w(nullptr, 0, nrows, &lc, prm, pt, out, flag, s, &st)) return st;
    PBH_TIMED(kKLhsPpf, s, hipLaunchKernelGGL(k_lhs_ppf_gamma_lds, dim3(gamma_lds_grid(nrows)), dim3(kGBlock), 0, s,
                                              seed, n, row0, nrows, col, prm, pt, out, flag));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  if (const size_t pl = poisson_lds_bytes(dist, prm, pt)) {
    const GammaLhs lc{seed, n, row0, col};
    return launch_poisson_lds(nullptr, 0, nrows, &lc, pl, prm, pt, out, flag, s);
  }
  switch (dist) {
#define PBH_CASE(D) \
  case D:           \
    if ((D == PBH_DIST_NORM || D == PBH_DIST_LOGNORM))                                                  \
      PBH_TIMED(kKLhsPpf, s,                                                                                    \
                hipLaunchKernelGGL((scalar_params(prm) ? k_lhs_ppf_c<D, true> : k_lhs_ppf_c<D, false>),            \
                                   dim3(compact_grid(nrows)), b, 0, s, seed, n, row0, nrows, col, prm, pt, out, \
                                   flag));                                                                      \
    else                                                                                                        \
      PBH_TIMED(kKLhsPpf, s,                                                                                    \
                hipLaunchKernelGGL(k_lhs_ppf<D>, g, b, 0, s, seed, n, row0, nrows, col, prm, pt, out, flag));   \
    break;
    PBH_CASE(PBH_DIST_NORM)
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_LOGNORM)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
    PBH_CASE(PBH_DIST_POISSON)
#undef PBH_CASE
    default:
      set_error("pbh_lhs_ppf: unsupported distribution id %d", dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int expected_nparams(int dist) {
  switch (dist) {
    case PBH_DIST_NORM:
    case PBH_DIST_UNIFORM:
    case PBH_DIST_EXPON:
    case PBH_DIST_POISSON:
      return 2;
    case PBH_DIST_LOGNORM:
    case PBH_DIST_TRIANG:
    case PBH_DIST_GAMMA:
      return 3;
    default:
      return -1;
  }
}

// Scalar-mu poisson: build the CDF table pdtr(k, mu), k in [k_lo, k_lo + len), in a
// stream-ordered allocation; elements outside its coverage fall back to the search.
int with_params(int dist, const pbh_param* params, int nparams, Params& prm, PoissonTable& pt, double** table,
                hipStream_t s) {
  int want = expected_nparams(dist);
  if (want < 0) {
    set_error("unsupported distribution id %d", dist);
    return PBH_ERR_UNSUPPORTED;
  }
  PBH_REQUIRE(nparams == want, "distribution %d expects %d parameters, got %d", dist, want, nparams);
  PBH_REQUIRE(params != nullptr, "params must not be NULL");
  for (int j = 0; j < 3; ++j) {
    prm.ptr[j] = j < nparams ? params[j].ptr : nullptr;
    prm.val[j] = j < nparams ? params[j].value : 0.0;
  }
  pt = PoissonTable{};
  *table = nullptr;
  if (dist == PBH_DIST_GAMMA && params[0].ptr == nullptr && params[0].value > 0.0 && isfinite(params[0].value)) {
    const double a = params[0].value;
    const int m = sf::kGammaGuideM;
    *table = gamma_guide_table(a, s);
    if (!*table) {
      set_error("gamma guide table for a = %g failed", a);
      return PBH_ERR_HIP;
    }
    double* tb = *table;
    pt.has_gamma = 1;
    pt.aux = sf::gamma_aux(a);
    pt.guide = sf::GammaGuide{tb, tb + m, tb + 2 * m, tb + 3 * m, m, sf::kGammaGuideZ0, sf::kGammaGuideH,
                              1.0 / sf::kGammaGuideH};
  }
  if (dist == PBH_DIST_POISSON && params[0].ptr == nullptr) {
    double mu = params[0].value;
    if (mu > 0.0 && mu < 1.0e12) {
      double sd = sqrt(mu);
      double lo = floor(mu - 12.0 * sd - 12.0);
      int64_t k_lo = lo > 0.0 ? (int64_t)lo : 0;
      int64_t k_hi = (int64_t)ceil(mu + 20.0 * sd + 40.0);
      int64_t len = k_hi - k_lo + 1;
      const int nb = 1 << kPoissonGuideBits;
      const size_t bytes = (size_t)2 * len * sizeof(double) + (size_t)nb * 4;
      auto build = [=](double* t, hipStream_t st) {
        hipLaunchKernelGGL(k_poisson_table, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, st, mu, k_lo, len, t,
                           t + len);
        hipLaunchKernelGGL(k_poisson_guide, dim3((unsigned)(nb / 256)), dim3(256), 0, st, t, len,
                           (int32_t*)(t + 2 * len));
        return hipGetLastError() == hipSuccess;
      };
      *table = cached_table(kTabPoisson, &mu, 1, bytes, s, build);
      if (!*table) {
        PBH_CHECK_HIP(hipMallocAsync((void**)table, bytes, s));
        if (!build(*table, s)) {
          set_error("poisson table launch failed");
          return PBH_ERR_HIP;
        }
      }
      pt.cdf = *table;
      pt.win = *table + len;
      pt.cdf_guide = (int32_t*)(*table + 2 * len);
      pt.k_lo = k_lo;
      pt.len = len;
    }
  }
  return PBH_OK;
}

}  // namespace

// The gamma guide of shape a (4 x kGammaGuideM doubles: y, d1, d2, ok), for gamma (with_params)
// and the extended distributions whose ppf is gammaincinv (chi, maxwell, nakagami, chi2:
// pbh_ppf_ext.hip): the process cache's (pbh_table_cache.hip), or a fresh stream-ordered
// allocation when the cache is full; callers end with release_table.  NULL for an invalid a.
double* gamma_guide_table(double a, hipStream_t s) {
  if (!(a > 0.0 && isfinite(a))) return nullptr;
  const int m = sf::kGammaGuideM;
  auto build = [=](double* tb, hipStream_t st) {
    sf::GammaGuide T{tb, tb + m, tb + 2 * m, tb + 3 * m, m, sf::kGammaGuideZ0, sf::kGammaGuideH, 1.0 / sf::kGammaGuideH};
    const unsigned g = (unsigned)((m + 63) / 64);
    hipLaunchKernelGGL(k_gamma_guide, dim3(g), dim3(64), 0, st, a, T, tb, tb + m, tb + 2 * m);
    hipLaunchKernelGGL(k_gamma_guide_check, dim3(g), dim3(64), 0, st, a, T, tb + 3 * m);
    return hipGetLastError() == hipSuccess;
  };
  const size_t bytes = (size_t)4 * m * sizeof(double);
  if (double* t = cached_table(kTabGammaGuide, &a, 1, bytes, s, build)) return t;
  double* tb = nullptr;
  if (hipMallocAsync((void**)&tb, bytes, s) != hipSuccess) return nullptr;
  if (!build(tb, s)) {
    (void)hipFreeAsync(tb, s);
    return nullptr;
  }
  return tb;
}

struct GenColumn {
  uint64_t seed;
  int64_t n;
  uint32_t col;
  int dist;
  Params prm;
  PoissonTable pt;
  double* table;
  bool ext;        // an extended distribution (pbh_ppf_ext.hip): its kernels take xval
  double xval[4];
  const uint32_t* rheads = nullptr;  // a discrete column's sorted run heads (gen_set_runs)
  double* rvals = nullptr;           // the value of each run
  int64_t nruns = 0;
};

int gen_create(uint64_t seed, int64_t n, int col, int dist, const pbh_param* params, int nparams, GenColumn** out,
               hipStream_t s) {
  for (int j = 0; j < nparams; ++j)
    PBH_REQUIRE(params[j].ptr == nullptr, "stratum-ordered LHS generation needs scalar parameters");
  GenColumn* g = new GenColumn{};
  g->seed = seed;
  g->n = n;
  g->col = (uint32_t)col;
  g->dist = dist;
  if (const int want = ext_nparams(dist); want >= 0) {
    if (nparams != want || (nparams && !params)) {
      delete g;
      set_error("distribution %d expects %d parameters, got %d", dist, want, nparams);
      return PBH_ERR_INVALID;
    }
    g->ext = true;
    for (int j = 0; j < nparams; ++j) g->xval[j] = params[j].value;
    g->table = ext_gen_table(dist, g->xval, nparams, s);
    *out = g;
    return PBH_OK;
  }
  int st = with_params(dist, params, nparams, g->prm, g->pt, &g->table, s);
  if (st != PBH_OK) {
    delete g;
    return st;
  }
  *out = g;
  return PBH_OK;
}

void gen_destroy(GenColumn* g, hipStream_t s) {
  if (!g) return;
  release_table(g->table, s);
  if (g->rvals) (void)hipFreeAsync(g->rvals, s);
  delete g;
}

// The counts and run heads of a poisson column's strata [t0, t0 + nt) without evaluating every
// stratum: q_t = (t + 1 - u_t) / n increases strictly with t and the poisson ppf is monotone in q,
// so the values are non-decreasing and a run boundary is the first stratum whose value reaches
// some integer k.  One thread per k in (value(t0), value(t0 + nt - 1)] binary-searches it with
// the same value() k_lhs_sorted_ppf evaluates (the same SplitMix64 jitter, the same CDF table
// and comparisons), so the heads, the tie count (nt - 1 - #heads) and the inversion count (0)
// equal that kernel's exactly, from ~30 evaluations per distinct value instead of nt.  The host
// takes this path only when the last value is finite and the values span at most kDiscreteSpan.
constexpr int kDiscreteSpan = 4096;

__global__ __launch_bounds__(256) PBH_OCC void k_discrete_heads(uint64_t seed, int64_t n, int64_t t0, int64_t nt, uint32_t col,
                                                        Params prm, PoissonTable pt, int32_t* flag,
                                                        unsigned long long* counts, uint32_t* __restrict__ heads,
                                                        uint32_t* __restrict__ hcur, uint32_t hcap) {
  __shared__ uint32_t b[kDiscreteSpan];
  __shared__ int span, bad;
  __shared__ double vlo;
  __shared__ uint32_t found;
  Philox ph(seed);
  auto value = [&](int64_t t) {
    const double q = lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n);
    return ppf_one<PBH_DIST_POISSON, 0, true>(q, prm.val[0], prm.val[1], prm.val[2], pt);
  };
  if (threadIdx.x == 0) {
    const double a = value(t0), z = value(t0 + nt - 1);
    vlo = a;
    found = 0;
    // not the case this kernel covers (non-finite or non-integer ends, too many values): the
    // caller checked the parameters, so this is a guard; the counts then say "not certified"
    bad = !(isfinite(a) && isfinite(z) && a == floor(a) && z == floor(z) && z >= a && z - a <= kDiscreteSpan);
    span = bad ? 0 : (int)(z - a);
    if (bad) {
      flag_nonfinite(flag, !isfinite(a) || !isfinite(z));
      atomicAdd(&counts[1], 1ull);  // read as an inversion: the caller redoes the column exactly
    }
  }
  __syncthreads();
  const int m = span;
  for (int i = threadIdx.x; i < m; i += 256) {  // k = vlo + 1 + i
    const double k = vlo + 1.0 + (double)i;
    int64_t lo = t0, hi = t0 + nt - 1;  // value(lo) < k <= value(hi)
    while (hi - lo > 1) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      if (value(mid) >= k)
        hi = mid;
      else
        lo = mid;
    }
    b[i] = (uint32_t)hi;
    // scipy's window above pdtr(k - 1, mu) (PoissonTable::win): its strata take k - 1 or k, so
    // the search (which needs non-decreasing values) is exact unless the window holds two strata
    // whose values decrease.  q_t lies in (t / n, (t + 1) / n], so the window's strata are within
    // [c n - 1, w n] (padded by 1); when two or more of their quantiles fall in it, their values
    // are checked here and a decrease is counted as an inversion (the caller then counts the
    // column exactly).  At cfg3 (N = 1e8, mu <= 30) a window is narrower than a stratum.
    const int64_t j = (int64_t)k - pt.k_lo;
    if (j >= 1 && j < pt.len && pt.win[j] > pt.cdf[j - 1]) {
      const double c = pt.cdf[j - 1], w = pt.win[j];
      const int64_t ta = max(t0, (int64_t)floor(c * (double)n) - 2);
      const int64_t tb = min(t0 + nt - 1, (int64_t)floor(w * (double)n) + 1);
      int inside = 0;
      for (int64_t t = ta; t <= tb && inside < 2 && tb - ta <= 256; ++t) {
        const double qt = lhs_sorted_quantile(ph, (uint64_t)t, col, (uint64_t)n);
        inside += qt >= c && qt < w;
      }
      if (tb - ta > 256) {
        atomicAdd(&counts[1], 1ull);
      } else if (inside >= 2) {
        double prev = value(ta);
        for (int64_t t = ta + 1; t <= tb; ++t) {
          const double v = value(t);
          if (v < prev) {
            atomicAdd(&counts[1], 1ull);
            break;
          }
          prev = v;
        }
      }
    }
  }
  __syncthreads();
  uint32_t mine = 0;
  for (int i = threadIdx.x; i < m; i += 256) {
    if (i > 0 && b[i] == b[i - 1]) continue;  // a value no stratum takes: the same boundary
    const uint32_t slot = atomicAdd(hcur, 1u);
    if (slot < hcap) heads[slot] = b[i];
    ++mine;
  }
  if (mine) atomicAdd(&found, mine);
  __syncthreads();
  if (threadIdx.x == 0 && !bad) atomicAdd(&counts[0], (unsigned long long)(nt - 1 - (int64_t)found));
}

int gen_sorted(const GenColumn* g, int64_t t0, int64_t nt, double* out, int32_t* flag, unsigned long long* counts,
               hipStream_t s, uint32_t* heads, uint32_t* hcur, uint32_t hcap) {
  const int64_t n = g->n;
  PBH_REQUIRE(t0 >= 0 && nt >= 0 && t0 + nt <= n, "lhs_sorted_ppf: strata [%lld, %lld) outside [0, %lld)",
              (long long)t0, (long long)(t0 + nt), (long long)n);
  PBH_REQUIRE(out || counts, "gen_sorted: neither an output column nor counts");
  PBH_REQUIRE(!heads || (counts && hcur && hcap >= 1), "gen_sorted: run heads need counts");
  if (counts) PBH_CHECK_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(unsigned long long), s));
  if (heads && t0 == 0) {  // stratum 0 heads the first run
    PBH_CHECK_HIP(hipMemsetAsync(heads, 0, sizeof(uint32_t), s));
    PBH_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)hcur, 1, 1, s));
  } else if (heads) {  // a later segment: its first stratum is the previous shard's last one
    PBH_CHECK_HIP(hipMemsetAsync(hcur, 0, sizeof(uint32_t), s));
  }
  if (nt == 0) return PBH_OK;
  if (g->ext)
    return ext_gen_sorted(g->seed, n, g->col, g->dist, g->xval, g->table, t0, nt, out, flag, counts, heads, hcur, hcap,
                          s);
  static const bool fast_heads = [] {  // PBH_DISCRETE_SCAN=1: evaluate every stratum
    const char* e = getenv("PBH_DISCRETE_SCAN");
    return !(e && e[0] == '1');
  }();
  const double mu = g->prm.val[0];
  if (fast_heads && g->dist == PBH_DIST_POISSON && counts && heads && !out && nt >= 2 && g->pt.cdf &&
      isfinite(mu) && mu > 0.0 && mu + 40.0 * sqrt(mu) + 100.0 < (double)kDiscreteSpan) {
    PBH_TIMED(kKLhsSorted, s,
              hipLaunchKernelGGL(k_discrete_heads, dim3(1), dim3(256), 0, s, g->seed, n, t0, nt, g->col, g->prm, g->pt,
                                 flag, counts, heads, hcur, hcap));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  dim3 gr(ppf_grid(nt)), b(kBlock);
  switch (g->dist) {
#define PBH_CASE(D)                                                                                            \
  case D:                                                                                                      \
    PBH_TIMED(kKLhsSorted, s,                                                                                  \
              hipLaunchKernelGGL(k_lhs_sorted_ppf<D>, gr, b, 0, s, g->seed, n, t0, nt, g->col, g->prm, g->pt, out, \
                                 flag, counts, heads, hcur, hcap));                                            \
    break;
    PBH_CASE(PBH_DIST_NORM)
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_LOGNORM)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
    PBH_CASE(PBH_DIST_POISSON)
#undef PBH_CASE
    default:
      set_error("unsupported distribution id %d", g->dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// T of the certificate (k_cert_scan) for a column's family and scalar parameters, or 0 when it
// does not apply (discrete, a parameter outside the family's domain, or sup f0 (|loc| / scale + |y|)
// unbounded).  eps: the assumed bound of the device inverse CDF's error relative to |loc| + scale |y|
// -- 1e-12 for the closed forms and Cephes' ndtri (errors of a few ulp), 1e-9 for gamma's guided
// interpolation (checked to 1e-12 per interval when the guide is built) -- 10^3 to 10^4 times the
// largest difference from scipy measured over 10^6 strata per column at N = 1e8
// (tests/test_gpu_scale_values.py).  The supremum is taken over a dense grid of y and widened by
// half for the grid's resolution and for xi between the two strata.
static double cert_gap(int dist, const double* v);

double gen_cert_gap(const GenColumn* g) {
  // cached per (family, parameters): the supremum scan costs ~4 ms of host time
  static std::mutex mu;
  static std::map<std::array<double, 5>, double> cache;
  const double* v = g->ext ? g->xval : g->prm.val;
  const std::array<double, 5> key = {(double)g->dist, v[0], v[1], v[2], g->ext ? v[3] : 0.0};
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const double T = cert_gap(g->dist, v);
  cache[key] = T;
  return T;
}

static double cert_gap(int dist, const double* v) {
  double loc = 0.0, scale = 1.0, eps = 1e-12;
  std::function<double(double)> f0;
  double lo = 0.0, hi = 1.0;
  bool logy = false;
  switch (dist) {
    case PBH_DIST_NORM:
      loc = v[0], scale = v[1];
      f0 = [](double y) { return 0.3989422804014327 * exp(-0.5 * y * y); };
      lo = -40.0, hi = 40.0;
      break;
    case PBH_DIST_UNIFORM:
      loc = v[0], scale = v[1];
      f0 = [](double) { return 1.0; };
      break;
    case PBH_DIST_EXPON:
      loc = v[0], scale = v[1];
      f0 = [](double y) { return exp(-y); };
      hi = 800.0;
      break;
    case PBH_DIST_TRIANG: {
      const double c = v[0];
      loc = v[1], scale = v[2];
      if (!(c >= 0.0 && c <= 1.0)) return 0.0;
      f0 = [c](double y) { return y < c ? 2.0 * y / c : (c < 1.0 ? 2.0 * (1.0 - y) / (1.0 - c) : 0.0); };
      break;
    }
    case PBH_DIST_GAMMA: {
      const double a = v[0];
      loc = v[1], scale = v[2], eps = 1e-9;
      if (!(a > 0.0)) return 0.0;
      if (a < 1.0 && loc != 0.0) return 0.0;  // f0 unbounded at 0 with |loc| > 0: no finite bound
      const double lg = lgamma(a);
      f0 = [a, lg](double y) { return y > 0.0 ? exp((a - 1.0) * log(y) - y - lg) : (a == 1.0 ? 1.0 : 0.0); };
      lo = 1e-300, hi = 100.0 * (a + 10.0), logy = true;
      break;
    }
    case PBH_DIST_LOGNORM: {
      const double sg = v[0];
      loc = v[1], scale = v[2];
      if (!(sg > 0.0)) return 0.0;
      eps = 1e-12 * (1.0 + 40.0 * sg);  // exp(s z) amplifies z's error by s |z|
      f0 = [sg](double y) {
        if (!(y > 0.0)) return 0.0;
        const double z = log(y) / sg;
        return 0.3989422804014327 * exp(-0.5 * z * z) / (sg * y);
      };
      lo = 1e-300, hi = 1e300, logy = true;
      break;
    }
    case PBH_DIST_BETA: {  // the guided inverse (sfx::beta_ppf_guided) is within ~1e-12 of the exact one
      const double a = v[0], b = v[1];
      loc = v[2], scale = v[3], eps = 1e-9;
      if (!(a >= 1.0 && b >= 1.0 && isfinite(a) && isfinite(b))) return 0.0;  // f0 bounded on [0, 1]
      const double lb = lgamma(a) + lgamma(b) - lgamma(a + b);
      f0 = [a, b, lb](double y) {
        if (!(y > 0.0 && y < 1.0)) return (a == 1.0 && y == 0.0) || (b == 1.0 && y == 1.0) ? exp(-lb) : 0.0;
        return exp((a - 1.0) * log(y) + (b - 1.0) * log1p(-y) - lb);
      };
      break;
    }
    case PBH_DIST_TRUNCNORM: {  // phi(y) / (Phi(b) - Phi(a)) on [a, b]; a log-space inverse, few-ulp accurate
      const double a = v[0], b = v[1];
      loc = v[2], scale = v[3], eps = 1e-9;
      if (!(a < b) || !isfinite(a) || !isfinite(b)) return 0.0;
      const double mass = 0.5 * (erfc(-b / sqrt(2.0)) - erfc(-a / sqrt(2.0)));
      if (!(mass > 1e-300)) return 0.0;
      f0 = [a, b, mass](double y) {
        return y >= a && y <= b ? 0.3989422804014327 * exp(-0.5 * y * y) / mass : 0.0;
      };
      lo = a, hi = b;
      break;
    }
    default:
      return 0.0;
  }
  if (!(scale > 0.0) || !isfinite(scale) || !isfinite(loc)) return 0.0;
  const double L = fabs(loc) / scale;
  double B = 0.0;
  const int m = 400000;
  for (int i = 0; i <= m; ++i) {
    const double y = logy ? exp(log(lo) + (log(hi) - log(lo)) * i / m) : lo + (hi - lo) * i / m;
    const double b = f0(y) * (L + fabs(y));
    if (!isfinite(b)) return 0.0;
    B = b > B ? b : B;
  }
  return 2.0 * eps * B * 1.5;
}

bool gen_cert_plan(const GenColumn* g, int64_t nt, double* T, uint32_t* cap) {
  const char* forced = getenv("PBH_CERT_T");  // tests: a given gap, the cost check skipped
  *T = forced ? atof(forced) : gen_cert_gap(g);
  if (!(*T > 0.0) || nt < 2) return false;
  const double n = (double)g->n;
  const double frac = std::min(1.0, 0.5 * (*T * n) * (*T * n));  // P(gap < T): gap = (1 - u' + u) / n
  if (!forced && frac > 0.05) return false;  // as costly as counting every stratum
  *cap = (uint32_t)std::min<double>((double)nt, std::max(65536.0, 8.0 * frac * (double)nt + 4096.0));
  return true;
}

int gen_certify(const GenColumn* g, int64_t t0, int64_t nt, double T, uint32_t* list, uint32_t cap, uint32_t* count,
                int32_t* flag, unsigned long long* counts, hipStream_t s) {
  PBH_REQUIRE(T > 0.0 && nt >= 1 && t0 >= 0 && t0 + nt <= g->n, "gen_certify: bad arguments");
  PBH_CHECK_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(unsigned long long), s));
  PBH_CHECK_HIP(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_cert_scan, dim3(ppf_grid(nt)), dim3(kBlock), 0, s, g->seed, g->n, t0, nt, g->col, T, list, cap,
                     count);
  PBH_CHECK_LAUNCH();
  if (g->ext)
    return ext_gen_cert_eval(g->seed, g->n, g->col, g->dist, g->xval, g->table, t0, nt, list, cap, count, flag, counts,
                             s);
  switch (g->dist) {
#define PBH_CASE(D)                                                                                               \
  case D:                                                                                                         \
    PBH_TIMED(kKLhsSorted, s,                                                                                     \
              hipLaunchKernelGGL(k_cert_eval<D>, dim3(512), dim3(kBlock), 0, s, g->seed, g->n, t0, nt, g->col, g->prm, \
                                 g->pt, list, cap, count, flag, counts));                                         \
    break;
    PBH_CASE(PBH_DIST_NORM)
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_LOGNORM)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
#undef PBH_CASE
    default:
      set_error("gen_certify: distribution %d has no certificate", g->dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

template <bool BYROW>
static int place_launch(const GenColumn* g, const uint64_t* pairs, const uint32_t* pidx, int64_t rows, double* y,
                        int64_t y_rs, int32_t* idx, const int32_t* state, hipStream_t s) {
  const int64_t n = g->n;
  if (g->rvals) {  // a discrete column with its runs: values from the run table
    const int64_t blocks = (rows + kGenRows - 1) / kGenRows;
    if (blocks <= 0) return PBH_OK;
    int sh = 0;
    while (((n - 1) >> sh) + 1 > kRunsGuideMax) ++sh;
    const size_t lds = (size_t)g->nruns * 12 + (size_t)(((n - 1) >> sh) + 1) * 4;
    PBH_TIMED(kKPlaceGen, s,
              hipLaunchKernelGGL(k_place_gen_runs<BYROW>, dim3((unsigned)(blocks < 256 * 8 ? blocks : 256 * 8)),
                                 dim3(kBlock), lds, s, pairs, pidx, rows, n, g->rheads, g->rvals, (int)g->nruns, y,
                                 y_rs, idx, state));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  if (g->ext)
    return ext_gen_place(g->seed, n, g->col, g->dist, g->xval, g->table, pairs, BYROW ? pidx : nullptr, rows, y, y_rs,
                         idx, state, s);
  const int64_t blocks = (rows + kGenRows - 1) / kGenRows;
  if (blocks <= 0) return PBH_OK;
  int j0 = 0, jn = 0;
  if (gamma_win_on() && gamma_lds_ok(g->dist, g->prm, g->pt) && gamma_window(n, g->pt.guide, &j0, &jn)) {
    // the slow list: a counter and cap entries (stream-ordered, freed after the second kernel)
    const uint32_t cap = (uint32_t)(rows / 64 + 1024 < (1 << 20) ? rows / 64 + 1024 : (1 << 20));
    unsigned long long* slow = nullptr;
    PBH_CHECK_HIP(hipMallocAsync((void**)&slow, ((size_t)cap + 1) * 8, s));
    PBH_CHECK_HIP(hipMemsetAsync(slow, 0, 8, s));
    PBH_TIMED(kKPlaceGen, s,
              hipLaunchKernelGGL(k_place_gen_gamma_w<BYROW>, dim3((unsigned)(blocks < 512 ? blocks : 512)),
                                 dim3(kGWBlock), 0, s, pairs, pidx, rows, n, g->seed, g->col, g->prm, g->pt, y, y_rs,
                                 idx, state, j0, jn, slow, cap));
    PBH_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_place_gen_gamma_slow<BYROW>, dim3(PBH_SLOW_GRID), dim3(256), 0, s, pairs, pidx, rows, n, g->seed,
                       g->col, g->prm, g->pt, y, y_rs, state, slow, cap);
    PBH_CHECK_LAUNCH();
    PBH_CHECK_HIP(hipFreeAsync(slow, s));
    return PBH_OK;
  }
  if (gamma_lds_ok(g->dist, g->prm, g->pt)) {
    PBH_TIMED(kKPlaceGen, s,
              hipLaunchKernelGGL(k_place_gen_gamma<BYROW>, dim3((unsigned)(blocks < 256 ? blocks : 256)), dim3(kGBlock),
                                 0, s, pairs, pidx, rows, n, g->seed, g->col, g->prm, g->pt, y, y_rs, idx, state));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  const unsigned gr = (unsigned)(blocks < 256 * 8 ? blocks : 256 * 8);
  if (g->dist == PBH_DIST_NORM || g->dist == PBH_DIST_LOGNORM) {
#define PBH_WCASE(D)                                                                                   \
  PBH_TIMED(kKPlaceGen, s,                                                                             \
            hipLaunchKernelGGL((k_place_gen_w<D, BYROW>), dim3(gr), dim3(kBlock), 0, s, pairs, pidx, rows, n, \
                               g->seed, g->col, g->prm, g->pt, y, y_rs, idx, state))
    if (g->dist == PBH_DIST_NORM)
      PBH_WCASE(PBH_DIST_NORM);
    else
      PBH_WCASE(PBH_DIST_LOGNORM);
#undef PBH_WCASE
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  if (const size_t pl = poisson_lds_bytes(g->dist, g->prm, g->pt)) {
    PBH_TIMED(kKPlaceGen, s,
              hipLaunchKernelGGL(k_place_gen_poisson<BYROW>, dim3(gr), dim3(kBlock), pl, s, pairs, pidx, rows, n,
                                 g->seed, g->col, g->prm, g->pt, y, y_rs, idx, state));
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  switch (g->dist) {
#define PBH_CASE(D)                                                                                          \
  case D:                                                                                                    \
    PBH_TIMED(kKPlaceGen, s,                                                                                 \
              hipLaunchKernelGGL((k_place_gen<D, BYROW>), dim3(gr), dim3(kBlock), 0, s, pairs, pidx, rows, n,  \
                                 g->seed, g->col, g->prm, g->pt, y, y_rs, idx, state));                      \
    break;
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
    PBH_CASE(PBH_DIST_POISSON)
#undef PBH_CASE
    default:
      set_error("unsupported distribution id %d", g->dist);
      return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int gen_place(const GenColumn* g, const uint64_t* pairs, int64_t n, double* y, int64_t y_rs, int32_t* idx,
              const int32_t* state, hipStream_t s) {
  PBH_REQUIRE(n == g->n, "gen_place: %lld rows for a column of %lld", (long long)n, (long long)g->n);
  return place_launch<false>(g, pairs, nullptr, n, y, y_rs, idx, state, s);
}

int gen_values_at(const GenColumn* g, const uint32_t* p, int64_t m, double* y, int64_t y_rs, hipStream_t s) {
  return place_launch<true>(g, nullptr, p, m, y, y_rs, nullptr, nullptr, s);
}

int gen_set_runs(GenColumn* g, const uint32_t* heads, int64_t nh, hipStream_t s) {
  static const bool on = [] {  // PBH_PLACE_RUNS=0 (A/B): every row through the inverse CDF
    const char* e = getenv("PBH_PLACE_RUNS");
    return !(e && e[0] == '0');
  }();
  if (!on || !gen_discrete(g->dist) || nh < 1 || nh > kRunsLdsMax || g->n < 1) return PBH_OK;
  double* v = nullptr;
  PBH_CHECK_HIP(hipMallocAsync((void**)&v, (size_t)nh * 8, s));
  const int st = gen_values_at(g, heads, nh, v, 1, s);  // the value of each run: its head's
  if (st != PBH_OK) {
    (void)hipFreeAsync(v, s);
    return st;
  }
  if (g->rvals) (void)hipFreeAsync(g->rvals, s);
  g->rvals = v;
  g->rheads = heads;
  g->nruns = nh;
  return PBH_OK;
}

int lhs_sorted_ppf(uint64_t seed, int64_t n, int64_t t0, int64_t nt, int col, int dist, const pbh_param* params,
                   int nparams, double* out, int32_t* flag, hipStream_t s, unsigned long long* counts) {
  PBH_REQUIRE(t0 >= 0 && nt >= 0 && t0 + nt <= n, "lhs_sorted_ppf: strata [%lld, %lld) outside [0, %lld)",
              (long long)t0, (long long)(t0 + nt), (long long)n);
  if (nt == 0) return PBH_OK;
  GenColumn* g = nullptr;
  int st = gen_create(seed, n, col, dist, params, nparams, &g, s);
  if (st != PBH_OK) return st;
  st = gen_sorted(g, t0, nt, out, flag, counts, s);
  gen_destroy(g, s);
  return st;
}

int sort_heads(uint32_t* heads, int64_t nh, hipStream_t s) {
  PBH_REQUIRE(nh >= 1 && nh <= kHeadsCap, "sort_heads: %lld heads outside [1, %d]", (long long)nh, kHeadsCap);
  int np2 = 1;
  while (np2 < nh) np2 <<= 1;
  hipLaunchKernelGGL(k_sort_heads, dim3(1), dim3(1024), 0, s, heads, (int)nh, np2);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int check_sorted(const double* x, int64_t n, unsigned long long* counts, hipStream_t s) {
  PBH_CHECK_HIP(hipMemsetAsync(counts, 0, 2 * sizeof(unsigned long long), s));
  hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(n, kBlock * kCheckU, 4096)), dim3(kBlock), 0, s, x, n, counts);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// blocks of the scores kernel; its partial sums: one per wave
static unsigned scores_grid(int64_t nrows) { return compact_grid(nrows); }
unsigned perm_scores_blocks(int64_t nrows) { return scores_grid(nrows) * (kBlock / 64); }

int perm_scores(uint64_t seed, int64_t n, int col, int64_t row0, int64_t nrows, const uint32_t* heads,
                int64_t nheads, double* S, hipStream_t s, double* partial) {
  PBH_REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= n, "perm_scores: rows outside [0, n)");
  if (nrows == 0) return PBH_OK;
  const size_t lds = heads && nheads <= kLdsHeads ? (size_t)nheads * 4 : 0;
  PBH_TIMED(kKPermScores, s,
            hipLaunchKernelGGL(k_perm_scores<false>, dim3(scores_grid(nrows)), dim3(kBlock), lds, s, seed, n,
                               (uint32_t)col, row0, nrows, heads, nheads, S, partial, nullptr));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int strata_scores(const int32_t* strata, int64_t n, const uint32_t* heads, int64_t nheads, double* S, hipStream_t s) {
  if (n == 0) return PBH_OK;
  const size_t lds = heads && nheads <= kLdsHeads ? (size_t)nheads * 4 : 0;
  PBH_TIMED(kKPermScores, s,
            hipLaunchKernelGGL(k_perm_scores<true>, dim3(scores_grid(n)), dim3(kBlock), lds, s, 0ull, n, 0u, 0ll, n,
                               heads, nheads, S, nullptr, strata));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// sorted[strata[r]] = x[r * stride]: a materialised column put in order by its known strata
// (sorted is NaN-filled first, so a stratum no row names reads as an inversion in check_sorted)
__global__ __launch_bounds__(kBlock) void k_strata_scatter(const double* __restrict__ x, int64_t stride,
                                                           const int32_t* __restrict__ strata, int64_t n,
                                                           double* __restrict__ sorted) {
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n; r += (int64_t)gridDim.x * kBlock) {
    const uint32_t t = (uint32_t)strata[r];
    if (t < (uint64_t)n) sorted[t] = x[r * stride];
  }
}

int strata_sorted(const double* x, int64_t stride, const int32_t* strata, int64_t n, double* sorted,
                  unsigned long long* counts, hipStream_t s) {
  PBH_CHECK_HIP(hipMemsetAsync(sorted, 0xFF, (size_t)n * 8, s));  // all-ones: a NaN
  hipLaunchKernelGGL(k_strata_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, x, stride, strata, n,
                     sorted);
  PBH_CHECK_LAUNCH();
  return check_sorted(sorted, n, counts, s);
}

size_t run_heads_ws_bytes(int64_t m) {
  const int64_t nb = (m + kHeadTile - 1) / kHeadTile;
  return ((size_t)nb * 4 + 255) / 256 * 256 + ((size_t)scan_partials_count(nb) * 4 + 255) / 256 * 256 + 256;
}

int run_heads(const double* x, int64_t m, int64_t t0, bool first_is_prev, uint32_t* heads, int64_t* count,
              void* ws, hipStream_t s) {
  if (m <= 0) {
    *count = 0;
    return PBH_OK;
  }
  const int64_t nb = (m + kHeadTile - 1) / kHeadTile;
  uint32_t* counts = (uint32_t*)ws;
  uint32_t* partials = (uint32_t*)((char*)ws + ((size_t)nb * 4 + 255) / 256 * 256);
  hipLaunchKernelGGL(k_heads_count, dim3((unsigned)nb), dim3(kBlock), 0, s, x, m, (int)first_is_prev, counts);
  PBH_CHECK_LAUNCH();
  uint32_t last = 0, last_off = 0;
  PBH_CHECK_HIP(hipMemcpyAsync(&last, counts + nb - 1, 4, hipMemcpyDeviceToHost, s));
  int st = exclusive_scan_u32(counts, nb, partials, s);
  if (st) return st;
  PBH_CHECK_HIP(hipMemcpyAsync(&last_off, counts + nb - 1, 4, hipMemcpyDeviceToHost, s));
  hipLaunchKernelGGL(k_heads_write, dim3((unsigned)nb), dim3(kBlock), 0, s, x, m, (int)first_is_prev, t0, counts,
                     heads);
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  *count = (int64_t)last_off + last;
  return PBH_OK;
}

}  // namespace pbh

using namespace pbh;

extern "C" int pbh_ppf(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params,
                       int nparams, double* out, int32_t* nonfinite_flag, void* stream) {
  PBH_REQUIRE(n >= 0, "pbh_ppf: n must be >= 0");
  if (n == 0) return PBH_OK;
  PBH_REQUIRE(q != nullptr && out != nullptr, "pbh_ppf: q and out must be device pointers");
  hipStream_t s = as_stream(stream);
  if (dist >= PBH_DIST_BETA) return ppf_ext(dist, q, q_stride, n, params, nparams, out, nonfinite_flag, s);
  Params prm;
  PoissonTable pt;
  double* table = nullptr;
  int st = with_params(dist, params, nparams, prm, pt, &table, s);
  if (st != PBH_OK) return st;
  st = launch_ppf(dist, q, q_stride, n, prm, pt, out, nonfinite_flag, s);
  release_table(table, s);
  return st;
}

extern "C" int pbh_lhs_ppf(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist,
                           const pbh_param* params, int nparams, double* out, int32_t* nonfinite_flag,
                           void* stream) {
  PBH_REQUIRE(n >= 1 && row0 >= 0 && nrows >= 0 && row0 + nrows <= n, "pbh_lhs_ppf: bad row range");
  PBH_REQUIRE(col >= 0, "pbh_lhs_ppf: bad column");
  if (nrows == 0) return PBH_OK;
  hipStream_t s = as_stream(stream);
  if (dist >= PBH_DIST_BETA)
    return lhs_ppf_ext(seed, n, row0, nrows, col, dist, params, nparams, out, nonfinite_flag, s);
  Params prm;
  PoissonTable pt;
  double* table = nullptr;
  int st = with_params(dist, params, nparams, prm, pt, &table, s);
  if (st != PBH_OK) return st;
  st = launch_lhs_ppf(dist, seed, n, row0, nrows, (uint32_t)col, prm, pt, out, nonfinite_flag, s);
  release_table(table, s);
  return st;
}

// Every column of a graph's uncorrelated native-LHS leaves in one call (round 5, cfg2): each
// column's inverse-CDF setup (gamma guide, poisson / binom CDF tables, beta guide: latency-bound
// kernels of 10-100 us) and its fused LHS + ppf kernel run on one of the step-4 lanes' streams,
// so the columns' setups overlap one another instead of queueing on the caller's stream; the
// caller's stream then waits for every lane.  Values are the per-column pbh_lhs_ppf's, bit for bit.
extern "C" int pbh_lhs_ppf_columns(const pbh_ic_column* cols, int32_t k, int64_t n, int64_t row0, int64_t nrows,
                                   double* out, int64_t ld, void* stream) {
  PBH_REQUIRE(cols && k >= 1 && n >= 1 && row0 >= 0 && nrows >= 0 && row0 + nrows <= n && out && ld >= nrows,
              "pbh_lhs_ppf_columns: bad arguments");
  if (nrows == 0) return PBH_OK;
  hipStream_t s = as_stream(stream);
  const int nts = step4_streams();  // 1 in the serial measurement mode
  hipStream_t ts[kStep4MaxStreams];
  std::vector<hipEvent_t> ev;
  struct Cleanup {
    std::vector<hipEvent_t>& v;
    bool joined = false;
    ~Cleanup() {
      if (!joined) step4_sync_side_streams();  // an error return: no lane may still read a table
      for (hipEvent_t e : v) (void)hipEventDestroy(e);
    }
  } cleanup{ev};
  auto order = [&](hipStream_t from, hipStream_t to) -> int {
    if (from == to) return PBH_OK;
    hipEvent_t e = nullptr;
    PBH_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev.push_back(e);
    PBH_CHECK_HIP(hipEventRecord(e, from));
    PBH_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
    return PBH_OK;
  };
  // below 2^20 rows a column's kernel is a few microseconds: the lanes' events (create, record,
  // wait, destroy on each side) would cost more host time than the overlap saves, and the setup
  // tables are cached after the first call, so the columns go on the caller's stream in order
  const int nl = nrows < ((int64_t)1 << 20) ? 1 : (nts < k ? nts : k);
  for (int i = 0; i < nl; ++i) {
    ts[i] = nl > 1 ? step4_side_stream(i) : s;
    if (!ts[i]) ts[i] = s;
    if (int st = order(s, ts[i])) return st;
  }
  for (int c = 0; c < k; ++c) {
    pbh_param prm[4];
    for (int j = 0; j < 4; ++j) prm[j] = pbh_param{nullptr, cols[c].params[j]};
    if (int st = pbh_lhs_ppf(cols[c].seed, n, row0, nrows, cols[c].lhs_col, cols[c].dist, prm, cols[c].nparams,
                             out + (int64_t)c * ld, cols[c].nonfinite_flag, ts[c % nl]))
      return st;
  }
  for (int i = 0; i < nl; ++i)
    if (int st = order(ts[i], s)) return st;
  cleanup.joined = true;
  return PBH_OK;
}

extern "C" int pbh_fill_lhs(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col0, int ncols,
                            double* q, int64_t ldq, void* stream) {
  PBH_REQUIRE(n >= 1 && row0 >= 0 && nrows >= 0 && row0 + nrows <= n, "pbh_fill_lhs: bad row range");
  PBH_REQUIRE(ncols >= 0 && col0 >= 0 && ncols <= 65535, "pbh_fill_lhs: bad column range");
  PBH_REQUIRE(ldq >= nrows, "pbh_fill_lhs: ldq < nrows");
  if (nrows == 0 || ncols == 0) return PBH_OK;
  dim3 g(grid_for(nrows, kBlock, 4096), (unsigned)ncols);
  hipLaunchKernelGGL(k_fill_lhs, g, dim3(kBlock), 0, as_stream(stream), seed, n, row0, nrows, col0, q, ldq);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

extern "C" int pbh_fill_uniform(uint64_t seed, int64_t row0, int64_t nrows, int col0, int ncols, double* q,
                                int64_t ldq, void* stream) {
  PBH_REQUIRE(row0 >= 0 && nrows >= 0, "pbh_fill_uniform: bad row range");
  PBH_REQUIRE(ncols >= 0 && col0 >= 0 && ncols <= 65535, "pbh_fill_uniform: bad column range");
  PBH_REQUIRE(ldq >= nrows, "pbh_fill_uniform: ldq < nrows");
  if (nrows == 0 || ncols == 0) return PBH_OK;
  dim3 g(grid_for(nrows, kBlock, 4096), (unsigned)ncols);
  hipLaunchKernelGGL(k_fill_uniform, g, dim3(kBlock), 0, as_stream(stream), seed, row0, nrows, col0, q, ldq);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

extern "C" int pbh_fill_sobol(const uint32_t* sv_host, const uint32_t* shift_host, int d, int bits, int64_t row0,
                              int64_t nrows, int col0, int ncols, double* q, int64_t ldq, void* stream) {
  PBH_REQUIRE(sv_host && shift_host, "pbh_fill_sobol: sv/shift must be host arrays");
  PBH_REQUIRE(bits >= 1 && bits <= 32, "pbh_fill_sobol: bits must be in [1, 32]");
  PBH_REQUIRE(col0 >= 0 && ncols >= 0 && col0 + ncols <= d, "pbh_fill_sobol: bad column range");
  PBH_REQUIRE(row0 >= 0 && nrows >= 0 && (row0 + nrows) <= (int64_t)1 << bits, "pbh_fill_sobol: rows exceed 2^bits");
  PBH_REQUIRE(ldq >= nrows, "pbh_fill_sobol: ldq < nrows");
  if (nrows == 0 || ncols == 0) return PBH_OK;
  const double scale = 1.0 / (double)((uint64_t)1 << bits);
  for (int c0 = 0; c0 < ncols; c0 += kSobolColsPerLaunch) {
    int nc = ncols - c0 < kSobolColsPerLaunch ? ncols - c0 : kSobolColsPerLaunch;
    SobolArgs a = {};
    for (int c = 0; c < nc; ++c) {
      int col = col0 + c0 + c;
      for (int b = 0; b < bits; ++b) a.sv[c][b] = sv_host[(int64_t)col * bits + b];
      a.shift[c] = shift_host[col];
    }
    dim3 g(grid_for(nrows, kBlock, 4096), (unsigned)nc);
    hipLaunchKernelGGL(k_fill_sobol, g, dim3(kBlock), 0, as_stream(stream), a, scale, row0, nrows,
                       q + (int64_t)c0 * ldq, ldq);
    PBH_CHECK_LAUNCH();
  }
  return PBH_OK;
}

extern "C" int pbh_sobol_ppf(const uint32_t* sv_host, const uint32_t* shift_host, int d, int bits, int64_t row0,
                             int64_t nrows, int col, int dist, const pbh_param* params, int nparams, double* out,
                             int32_t* nonfinite_flag, void* stream) {
  PBH_REQUIRE(sv_host && shift_host && out, "pbh_sobol_ppf: null pointer");
  PBH_REQUIRE(bits >= 1 && bits <= 32, "pbh_sobol_ppf: bits must be in [1, 32]");
  PBH_REQUIRE(col >= 0 && col < d, "pbh_sobol_ppf: bad column");
  PBH_REQUIRE(row0 >= 0 && nrows >= 0 && (row0 + nrows) <= (int64_t)1 << bits, "pbh_sobol_ppf: rows exceed 2^bits");
  if (nrows == 0) return PBH_OK;
  if (dist < 0 || dist >= PBH_DIST_BETA) {
    set_error("pbh_sobol_ppf: distribution %d has no fused Sobol' kernel (use pbh_fill_sobol + pbh_ppf)", dist);
    return PBH_ERR_UNSUPPORTED;
  }
  hipStream_t s = as_stream(stream);
  SobolCol sc = {};
  for (int b = 0; b < bits; ++b) sc.sv[b] = sv_host[(int64_t)col * bits + b];
  sc.shift = shift_host[col];
  sc.scale = 1.0 / (double)((uint64_t)1 << bits);
  Params prm;
  PoissonTable pt;
  double* table = nullptr;
  int st = with_params(dist, params, nparams, prm, pt, &table, s);
  if (st != PBH_OK) return st;
  dim3 g(ppf_grid(nrows)), b(kBlock);
  switch (dist) {
#define PBH_CASE(D)                                                                                               \
  case D:                                                                                                         \
    if ((D == PBH_DIST_NORM || D == PBH_DIST_LOGNORM))                                                          \
      PBH_TIMED(kKPpf, s,                                                                                         \
                hipLaunchKernelGGL((scalar_params(prm) ? k_sobol_ppf_c<D, true> : k_sobol_ppf_c<D, false>),         \
                                   dim3(compact_grid(nrows)), b, 0, s, sc, row0, nrows, prm, pt, out,             \
                                   nonfinite_flag));                                                              \
    else                                                                                                          \
      PBH_TIMED(kKPpf, s,                                                                                         \
                hipLaunchKernelGGL(k_sobol_ppf<D>, g, b, 0, s, sc, row0, nrows, prm, pt, out, nonfinite_flag));  \
    break;
    PBH_CASE(PBH_DIST_NORM)
    PBH_CASE(PBH_DIST_UNIFORM)
    PBH_CASE(PBH_DIST_EXPON)
    PBH_CASE(PBH_DIST_LOGNORM)
    PBH_CASE(PBH_DIST_TRIANG)
    PBH_CASE(PBH_DIST_GAMMA)
    PBH_CASE(PBH_DIST_POISSON)
#undef PBH_CASE
    default:
      break;
  }
  PBH_CHECK_LAUNCH();
  release_table(table, s);
  return PBH_OK;
}
