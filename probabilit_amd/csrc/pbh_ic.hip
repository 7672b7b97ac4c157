// Iman-Conover device kernels (correlation.py:368-425).
//
//   rank_finish   : 'average' tie ranks of a sorted column (scipy _rankdata semantics:
//                   ordinal(first of run) + (count - 1) / 2) -> scores / gather / ranks
//   centered_gram : (S - mean)^T (S - mean), the np.cov inside np.corrcoef (:398)
//   apply         : per row, forward substitution with L = cholesky(E) (the
//                   solve_triangular of :409-411) and the multiply by P^T (:414)
#include <math.h>

#include <stdlib.h>
#include <string.h>

#include "pbh_error.h"
#include "pbh_ic.h"
#include "pbh_special.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int T = kSortThreads;  // 256
constexpr int IPT = kSortItems;  // 16
constexpr int TILE = kSortTile;  // 4096
constexpr int64_t kNoHead = INT64_MAX;

__device__ __forceinline__ int pad(int p) { return p + (p >> 4); }

template <bool IsMax>
__device__ __forceinline__ int64_t comb(int64_t a, int64_t b) {
  return IsMax ? (a > b ? a : b) : (a < b ? a : b);
}

// Exclusive scan across the 256 threads of a block (forward for max, or reverse when Rev).
template <bool IsMax, bool Rev>
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t identity, int64_t* sh /*>= 8*/) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t y = Rev ? __shfl_down(x, o, 64) : __shfl_up(x, o, 64);
    bool ok = Rev ? (lane + o < 64) : (lane >= o);
    if (ok) x = comb<IsMax>(x, y);
  }
  // x = inclusive scan within the wave (from the left, or from the right when Rev)
  if (Rev ? lane == 0 : lane == 63) sh[w] = x;
  int64_t excl = Rev ? __shfl_down(x, 1, 64) : __shfl_up(x, 1, 64);
  if (Rev ? lane == 63 : lane == 0) excl = identity;
  __syncthreads();
  int64_t other = identity;
  if (Rev) {
    for (int i = w + 1; i < 4; ++i) other = comb<IsMax>(other, sh[i]);
  } else {
    for (int i = 0; i < w; ++i) other = comb<IsMax>(other, sh[i]);
  }
  __syncthreads();
  return comb<IsMax>(excl, other);
}

__global__ __launch_bounds__(T) void k_load_keys(const double* __restrict__ x, int64_t stride, int64_t n,
                                                uint64_t* __restrict__ keys, int32_t* flag) {
  for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < n; i += (int64_t)gridDim.x * T) {
    double v = x[i * stride];
    keys[i] = f64_to_key(v);
    flag_nonfinite(flag, isnan(v));  // +-inf sort fine; NaN ranks are undefined (ValueError)
  }
}

__global__ __launch_bounds__(T) void k_head_bounds(const uint64_t* __restrict__ keys, const uint8_t* __restrict__ eqprev,
                                                  int64_t n, int64_t* __restrict__ first_head,
                                                  int64_t* __restrict__ last_head) {
  __shared__ int64_t sh[8];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  int64_t f = kNoHead, l = -1;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int64_t i = base + j * T + threadIdx.x;
    if (i < n) {
      bool head = (i == 0) || (eqprev ? !eqprev[i] : keys[i] != keys[i - 1]);
      if (head) {
        f = i < f ? i : f;
        l = i > l ? i : l;
      }
    }
  }
  // block min / max
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t fo = __shfl_xor(f, o, 64), lo = __shfl_xor(l, o, 64);
    f = fo < f ? fo : f;
    l = lo > l ? lo : l;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w] = f;
    sh[4 + w] = l;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t ff = sh[0], ll = sh[4];
    for (int i = 1; i < 4; ++i) {
      ff = sh[i] < ff ? sh[i] : ff;
      ll = sh[4 + i] > ll ? sh[4 + i] : ll;
    }
    first_head[blockIdx.x] = ff;
    last_head[blockIdx.x] = ll;
  }
}

// prev_head[t] = max(last_head[0..t-1]) (or -1); next_head[t] = min(first_head[t+1..]) (or n).
__global__ __launch_bounds__(T) void k_head_prefix(const int64_t* __restrict__ first_head,
                                                  const int64_t* __restrict__ last_head, int64_t ntiles, int64_t n,
                                                  int64_t* __restrict__ prev_head, int64_t* __restrict__ next_head) {
  __shared__ int64_t sh[8];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = -1;
  __syncthreads();
  for (int64_t b0 = 0; b0 < ntiles; b0 += T) {
    int64_t i = b0 + threadIdx.x;
    int64_t v = i < ntiles ? last_head[i] : -1;
    int64_t ex = block_excl_scan<true, false>(v, -1, sh);
    int64_t c = carry;
    if (i < ntiles) prev_head[i] = ex > c ? ex : c;
    __syncthreads();
    if (threadIdx.x == T - 1) {
      int64_t tot = comb<true>(ex, v);
      carry = tot > c ? tot : c;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) carry = n;
  __syncthreads();
  for (int64_t e0 = ntiles; e0 > 0; e0 -= T) {
    int64_t i = e0 - T + threadIdx.x;  // may be negative in the last chunk
    int64_t v = i >= 0 ? first_head[i] : kNoHead;
    int64_t ex = block_excl_scan<false, true>(v, kNoHead, sh);
    int64_t c = carry;
    if (i >= 0) next_head[i] = ex < c ? ex : c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t tot = comb<false>(ex, v);
      carry = tot < c ? tot : c;
    }
    __syncthreads();
  }
}

template <int MODE>
__global__ __launch_bounds__(T) void k_rank_finish(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ rows,
                                                  const uint8_t* __restrict__ eqprev, int64_t n,
                                                  const int64_t* __restrict__ prev_head,
                                                  const int64_t* __restrict__ next_head, RankOut out) {
  __shared__ uint64_t sk[TILE + TILE / 16];
  __shared__ uint32_t sr[TILE + TILE / 16];
  __shared__ int64_t sh[8];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const int cnt = (int)((n - base) < TILE ? (n - base) : TILE);
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int p = j * T + t;
    if (p < cnt) {
      // with eqprev the key slot carries the "equals previous" flag instead of the key
      sk[pad(p)] = eqprev ? (uint64_t)eqprev[base + p] : keys[base + p];
      sr[pad(p)] = rows ? rows[base + p] : (uint32_t)(base + p);  // NULL payload: identity
    }
  }
  const uint64_t before = (base > 0 && !eqprev) ? keys[base - 1] : 0ull;
  __syncthreads();

  // blocked view: thread t owns positions t*16 .. t*16+15 of the tile
  uint64_t k[IPT];
  bool head[IPT];
  int64_t first_local = kNoHead, last_local = -1;
#pragma unroll
  for (int q = 0; q < IPT; ++q) {
    int p = t * IPT + q;
    if (p < cnt) {
      k[q] = sk[pad(p)];
      if (eqprev) {
        head[q] = (base + p == 0) || k[q] == 0;
      } else {
        uint64_t prev = (p == 0) ? before : sk[pad(p - 1)];
        head[q] = (base + p == 0) || (k[q] != prev);
      }
      if (head[q]) {
        int64_t g = base + p;
        first_local = g < first_local ? g : first_local;
        last_local = g;
      }
    } else {
      k[q] = 0;
      head[q] = false;
    }
  }
  int64_t start = block_excl_scan<true, false>(last_local, -1, sh);
  start = comb<true>(start, prev_head[blockIdx.x]);
  int64_t nxt = block_excl_scan<false, true>(first_local, kNoHead, sh);
  nxt = comb<false>(nxt, next_head[blockIdx.x]);

  int64_t next_after[IPT];
#pragma unroll
  for (int q = IPT - 1; q >= 0; --q) {
    next_after[q] = nxt;
    if (head[q]) nxt = base + t * IPT + q;
  }
  const double np1 = (double)(n + 1);
#pragma unroll
  for (int q = 0; q < IPT; ++q) {
    int p = t * IPT + q;
    if (p >= cnt) continue;
    int64_t g = base + p;
    if (head[q]) start = g;
    int64_t end = next_after[q] - 1;  // next_after == n when no later head
    double avg = (double)(start + 1) + (double)(end - start) / 2.0;
    uint32_t row = sr[pad(p)];
    if constexpr (MODE == kModeScores) {
      out.scores[row] = sf::ppnd16(avg / np1);  // the scores of k_perm_scores (sf::ppnd16)
    } else if constexpr (MODE == kModeScoresRank) {
      out.scores[g] = sf::ppnd16(avg / np1);
      (void)row;
    } else if constexpr (MODE == kModeGather) {
      int64_t idx = (int64_t)avg - 1;
      out.y[(int64_t)row * out.y_rs] = out.sorted_src[idx];
      if (out.idx) out.idx[row] = (int32_t)idx;
    } else {
      out.ranks[row] = avg;
    }
  }
  if constexpr (MODE == kModeScores || MODE == kModeScoresRank) {
    if (out.sorted_x) {
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        int p = j * T + t;
        if (p < cnt) out.sorted_x[base + p] = key_to_f64(sk[pad(p)]);
      }
    }
  }
}

// ---------------------------------------------------------------- column means
constexpr int kRedThreads = 256;

__device__ __forceinline__ double block_sum(double v, double* sh /*4*/) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = ((sh[0] + sh[1]) + (sh[2] + sh[3]));
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kRedThreads) void k_colsum(const double* __restrict__ S, int64_t n, int64_t ld,
                                                       int64_t chunk, double* __restrict__ partial) {
  __shared__ double sh[4];
  const int c = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  int64_t r1 = r0 + chunk;
  if (r1 > n) r1 = n;
  double s = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += kRedThreads) s += S[(int64_t)c * ld + r];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[(int64_t)c * gridDim.x + blockIdx.x] = s;
}

// means[c] = (sum of the nb partials of column c) / divisor: one 256-thread block per column, each
// thread summing a stride-256 subset in order, then a fixed tree in LDS -- a fixed order
// (deterministic) without one thread walking thousands of dependent loads (the per-wave partials
// of the scores kernel: 8192 per column at N = 1e8 took 0.8 ms per step sequentially)
__global__ __launch_bounds__(256) void k_means(const double* __restrict__ partial, int nb, int k, double divisor,
                                               double* __restrict__ means) {
  __shared__ double sh[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double s = 0.0;
  for (int b = t; b < nb; b += 256) s += partial[(int64_t)c * nb + b];
  sh[t] = s;
  __syncthreads();
#pragma unroll
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) sh[t] += sh[t + o];
    __syncthreads();
  }
  if (t == 0) means[c] = sh[0] / divisor;
}

// ---------------------------------------------------------------- centered Gram
constexpr int GT = 32;     // Gram tile (columns)
constexpr int GROWS = 64;  // rows staged per step
constexpr int kGramBlocksMax = 768;  // 3 blocks per CU: the register prefetch of k_gram_mfma allows 3 waves per SIMD

__global__ __launch_bounds__(256) void k_gram(const double* __restrict__ S, int64_t n, int k, int64_t ld,
                                             const double* __restrict__ means, int64_t chunk,
                                             double* __restrict__ partials) {
  __shared__ double A[GROWS][GT + 1];  // +1 pad: conflict-free column-wise staging writes
  __shared__ double B[GROWS][GT + 1];
  __shared__ double red[4][GT * GT / 4];  // reused for the 4-group reduction in quarters
  const int t = threadIdx.x, g = t >> 6, l = t & 63;
  // tile pair (ti <= tj) from blockIdx.y
  const int nt = (k + GT - 1) / GT;
  int pair = blockIdx.y, ti = 0;
  while (pair >= nt - ti) {
    pair -= nt - ti;
    ++ti;
  }
  const int tj = ti + pair;
  const int i0 = (l >> 3) * 4, j0 = (l & 7) * 4;
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;

  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  int64_t r1 = r0 + chunk;
  if (r1 > n) r1 = n;
  for (int64_t rb = r0; rb < r1; rb += GROWS) {
#pragma unroll
    for (int m = 0; m < (GROWS * GT) / 256; ++m) {
      int idx = t + 256 * m;
      int col = idx / GROWS, row = idx % GROWS;
      int64_t r = rb + row;
      int ca = ti * GT + col, cb = tj * GT + col;
      A[row][col] = (r < r1 && ca < k) ? S[(int64_t)ca * ld + r] - means[ca] : 0.0;
      B[row][col] = (r < r1 && cb < k) ? S[(int64_t)cb * ld + r] - means[cb] : 0.0;
    }
    __syncthreads();
#pragma unroll 4
    for (int row = g; row < GROWS; row += 4) {
      double a[4], b[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        a[x] = A[row][i0 + x];
        b[x] = B[row][j0 + x];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = __builtin_fma(a[x], b[y], acc[x][y]);
    }
    __syncthreads();
  }
  // reduce the 4 row groups: group g writes its 16 values; group 0 sums in fixed order
  double* out = partials + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (GT * GT);
  for (int q = 0; q < 4; ++q) {  // quarter q of the 1024 entries handled via red[4][256]
    // thread l of group g holds entries (i0+x, j0+y); map entry to slot within quarter
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        int e = (i0 + x) * GT + (j0 + y);
        if ((e >> 8) == q) red[g][e & 255] = acc[x][y];
      }
    __syncthreads();
    {
      int e = t;  // 256 threads cover the quarter
      double v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
      out[q * 256 + e] = v;
    }
    __syncthreads();
  }
}

__global__ void k_gram_reduce(const double* __restrict__ partials, int nb, int k, double* __restrict__ gram) {
  const int nt = (k + GT - 1) / GT;
  int pair = blockIdx.y, ti = 0;
  while (pair >= nt - ti) {
    pair -= nt - ti;
    ++ti;
  }
  const int tj = ti + pair;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= GT * GT) return;
  const int i = ti * GT + e / GT, j = tj * GT + e % GT;
  if (i >= k || j >= k) return;
  const double* p = partials + (int64_t)blockIdx.y * nb * (GT * GT) + e;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += p[(int64_t)b * (GT * GT)];
  gram[(int64_t)i * k + j] = s;
  gram[(int64_t)j * k + i] = s;
}

// Gram for K <= 32 on the f64 matrix cores.  A block stages GM_ROWS rows x 32 columns of the
// centered scores in LDS (one coalesced 512-byte column load per wave instruction, zero
// padding for columns >= k and rows past the chunk), then every wave feeds row quads to
// v_mfma_f64_16x16x4_f64: with A[m][q] = B[q][m] = S[row q][16 I + m], the three tiles
// (0,0), (0,1), (1,1) of the 32 x 32 upper block triangle accumulate in 12 registers.
// The four waves' tiles are summed through LDS in a fixed order at the end (deterministic).
// partials[(block * 32 + i) * 32 + j] for i <= j, as k_gram_rows_reduce<32> expects.
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));
constexpr int GM_ROWS = 128;

__global__ __launch_bounds__(256) void k_gram_mfma(const double* __restrict__ S, int64_t n, int k, int64_t ld,
                                                  const double* __restrict__ means, int64_t chunk,
                                                  double* __restrict__ partials) {
  __shared__ double smem[GM_ROWS * 33];  // staging tile [row][col], reused for the wave reduction
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  const int64_t r1 = (r0 + chunk) < n ? (r0 + chunk) : n;
  double mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) mu[j] = (w * 8 + j) < k ? means[w * 8 + j] : 0.0;
  f64x4 c00 = {0.0, 0.0, 0.0, 0.0}, c01 = c00, c11 = c00;
  // the next chunk's loads are issued before this chunk's MFMAs (register prefetch); with
  // `pair` (ld even, S 16-byte aligned: the host checks) a lane reads rows 2 l and 2 l + 1 of a
  // column in one 16-byte access, half the load instructions of one row per lane
  static_assert(GM_ROWS == 128, "one 16-byte pair per lane and column");
  double pre[2][8];
  const bool pair = (ld % 2 == 0) && ((uintptr_t)S % 16 == 0);
  auto load = [&](int64_t rb) {
    const int64_t r = rb + 2 * lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = w * 8 + j;
      double a = 0.0, b = 0.0;
      if (c < k) {
        const double* src = &S[(int64_t)c * ld + r];
        if (pair && r + 1 < r1) {
          const v2d t = __builtin_nontemporal_load((const v2d*)src);
          a = t.x;
          b = t.y;
        } else {
          a = r < r1 ? src[0] : 0.0;
          b = r + 1 < r1 ? src[1] : 0.0;
        }
      }
      pre[0][j] = a;
      pre[1][j] = b;
    }
  };
  if (r0 < r1) load(r0);
  for (int64_t rb = r0; rb < r1; rb += GM_ROWS) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 2 * lane + h;
      const int64_t r = rb + row;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = w * 8 + j;
        smem[row * 33 + c] = (c < k && r < r1) ? pre[h][j] - mu[j] : 0.0;
      }
    }
    __syncthreads();
    if (rb + GM_ROWS < r1) load(rb + GM_ROWS);
#pragma unroll
    for (int qi = 0; qi < GM_ROWS / 16; ++qi) {
      const int row = (w + 4 * qi) * 4 + (lane >> 4);
      const double a0 = smem[row * 33 + (lane & 15)];
      const double a1 = smem[row * 33 + 16 + (lane & 15)];
      c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, a0, c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, a1, c01, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, a1, c11, 0, 0, 0);
    }
    __syncthreads();
  }
  // wave reduction: red[w][tile][reg][lane]
  double* red = smem;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    red[((w * 3 + 0) * 4 + g) * 64 + lane] = c00[g];
    red[((w * 3 + 1) * 4 + g) * 64 + lane] = c01[g];
    red[((w * 3 + 2) * 4 + g) * 64 + lane] = c11[g];
  }
  __syncthreads();
  double* out = partials + (int64_t)blockIdx.x * 32 * 32;
  for (int e = t; e < 3 * 4 * 64; e += 256) {  // e = (tile * 4 + reg) * 64 + lane
    const int tile = e / 256, g = (e >> 6) & 3, l = e & 63;
    const double v = ((red[((0 * 3 + tile) * 4 + g) * 64 + l] + red[((1 * 3 + tile) * 4 + g) * 64 + l]) +
                      red[((2 * 3 + tile) * 4 + g) * 64 + l]) +
                     red[((3 * 3 + tile) * 4 + g) * 64 + l];
    const int i = (l >> 4) + 4 * g + (tile == 2 ? 16 : 0);
    const int j = (l & 15) + (tile >= 1 ? 16 : 0);
    if (i <= j) out[i * 32 + j] = v;
  }
}

// gram[i][j] = gram[j][i] = sum over blocks (in order) of partials[b][min][max]
template <int KC>
__global__ void k_gram_rows_reduce(const double* __restrict__ partials, int nb, int k, double* __restrict__ gram) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= k * k) return;
  int i = e / k, j = e % k;
  if (i > j) {
    const int t = i;
    i = j;
    j = t;
  }
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += partials[(int64_t)b * KC * KC + i * KC + j];
  gram[e] = s;
}

// ---------------------------------------------------------------- decorrelate + correlate
template <int KMAX>
__global__ __launch_bounds__(256) void k_apply(double* __restrict__ S, int64_t n, int k, int64_t ld,
                                              const double* __restrict__ L, const double* __restrict__ inv_diag,
                                              const double* __restrict__ P, uint32_t* __restrict__ codes,
                                              int64_t ldc, CodeMap cm) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    double v[KMAX];
#pragma unroll
    for (int m = 0; m < KMAX; ++m) v[m] = (m < k) ? S[(int64_t)m * ld + r] : 0.0;
    // D = S L^-T : forward substitution, row by row of L
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      if (j < k) {
        double acc = v[j];
#pragma unroll
        for (int m = 0; m < j; ++m) acc = __builtin_fma(-L[j * k + m], v[m], acc);
        v[j] = acc * inv_diag[j];
      }
    }
    // CS = D P^T (P lower triangular), in place from the last column down
#pragma unroll
    for (int j = KMAX - 1; j >= 0; --j) {
      if (j < k) {
        double acc = 0.0;
#pragma unroll
        for (int m = 0; m <= j; ++m) acc = __builtin_fma(v[m], P[j * k + m], acc);
        v[j] = acc;
      }
    }
#pragma unroll
    for (int m = 0; m < KMAX; ++m)
      if (m < k) S[(int64_t)m * ld + r] = v[m];
    if (codes) {  // step 4's sort keys, while the row is in registers
#pragma unroll
      for (int m = 0; m < KMAX; ++m)
        if (m < k) codes[(int64_t)m * ldc + r] = code_of(v[m], cm);
    }
  }
}

// ---------------------------------------------------------------- step 3 on the matrix cores
// For K <= 32 the two triangular factors fold into one 32 x 32 matrix M = L^-T P^T (zero padded),
// CS = S M, and the N x 32 by 32 x 32 product runs on v_mfma_f64_16x16x4_f64.  The vector
// kernel above is latency bound (one row per lane: 32 loads, ~1000 dependent FMAs, 64 stores,
// 150 VGPRs); here a wave multiplies 64-row tiles with the whole of M held as B operands in
// registers, and the result goes through LDS so that every column store is 512 contiguous
// bytes.  M is computed on the device from L by column-wise forward substitution (f64); the
// product differs from substitution-then-multiply in the last bits only, as the reference's
// own dtrsm + dgemm order does from either.
__global__ void k_transform_matrix(const double* __restrict__ L, const double* __restrict__ inv_diag,
                                   const double* __restrict__ P, int k, double* __restrict__ M) {
  __shared__ double Linv[32][33];  // Linv[i][c] = (L^-1)[i][c]
  const int c = threadIdx.x;  // column c of L^-1: solve L x = e_c
  if (c < 32) {
    for (int i = 0; i < 32; ++i) {
      double v = 0.0;
      if (i < k && c < k && i >= c) {
        double acc = (i == c) ? 1.0 : 0.0;
        for (int m = c; m < i; ++m) acc = __builtin_fma(-L[i * k + m], Linv[m][c], acc);
        v = acc * inv_diag[i];
      }
      Linv[i][c] = v;
    }
  }
  __syncthreads();
  // M[m][j] = sum_q Linv[q][m] P[j][q]  (q in [m, j]: both triangular)
  for (int e = threadIdx.x; e < 32 * 32; e += blockDim.x) {
    const int m = e >> 5, j = e & 31;
    double acc = 0.0;
    if (m < k && j < k)
      for (int q = m; q <= j; ++q) acc = __builtin_fma(Linv[q][m], P[j * k + q], acc);
    M[e] = acc;
  }
}

// AM_ROWS rows per wave tile: 32 (default: 148 registers with the prefetch and 46 KiB of LDS, 3
// waves per SIMD; each store instruction writes two columns' 256-byte halves) or 64
// (PBH_APPLY_ROWS=64: 218 registers and 80 KiB, 2 waves per SIMD)
// NT: non-temporal loads of S and stores of CS and the codes (PBH_APPLY_NT=1; streaming, no reuse)
template <int AM_ROWS, bool NT = false>
__global__ __launch_bounds__(256) void k_apply_mfma(double* __restrict__ S, int64_t n, int k, int64_t ld,
                                                   const double* __restrict__ M, uint32_t* __restrict__ codes,
                                                   int64_t ldc, CodeMap cm) {
  __shared__ double tile[4][AM_ROWS * 33];
  __shared__ uint32_t cbase[kCodeSegments + 1];  // the code map in LDS: two lookups per code
  __shared__ double cscale[kCodeSegments];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* tl = tile[w];
  if (codes) {
    for (int j = threadIdx.x; j <= cm.m; j += 256) cbase[j] = cm.base[j];
    for (int j = threadIdx.x; j < cm.m; j += 256) cscale[j] = cm.scale[j];
    cm.base = cbase;
    cm.scale = cscale;
  }
  __syncthreads();
  const int q = lane >> 4, m16 = lane & 15;
  double b[8][2];  // B operands: M[4 s + q][16 J + m16]
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int J = 0; J < 2; ++J) b[s][J] = M[(4 * s + q) * 32 + 16 * J + m16];
  const int64_t tiles = (n + AM_ROWS - 1) / AM_ROWS;
  // A operands of the wave's next 64-row tile, loaded while the current tile's columns are
  // stored (register prefetch: the loads of tile t + 1 overlap the LDS transpose and the stores
  // of tile t; rows of different tiles never alias, so the in-place update is unaffected)
  double pa[AM_ROWS / 16][8];
  auto load = [&](int64_t bt) {
    const int64_t tw = bt * 4 + w;
#pragma unroll
    for (int rb = 0; rb < AM_ROWS / 16; ++rb) {
      const int64_t r = tw * AM_ROWS + rb * 16 + m16;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int c = 4 * s + q;
        pa[rb][s] = (tw < tiles && c < k && r < n)
                        ? (NT ? __builtin_nontemporal_load(&S[(int64_t)c * ld + r]) : S[(int64_t)c * ld + r])
                        : 0.0;
      }
    }
  };
  if ((int64_t)blockIdx.x * 4 < tiles) load(blockIdx.x);
  for (int64_t bt = blockIdx.x; bt * 4 < tiles; bt += gridDim.x) {  // uniform trip count per block
    const int64_t tw = bt * 4 + w;
    const int64_t r0 = tw * AM_ROWS;
    if (tw < tiles) {
#pragma unroll
      for (int rb = 0; rb < AM_ROWS / 16; ++rb) {
        f64x4 c0 = {0.0, 0.0, 0.0, 0.0}, c1 = c0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[rb][s], b[s][0], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[rb][s], b[s][1], c1, 0, 0, 0);
        }
        // C[i][j]: register g of lane l holds row i = (l >> 4) + 4 g, column j = l & 15
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = rb * 16 + q + 4 * g;
          tl[row * 33 + m16] = c0[g];
          tl[row * 33 + 16 + m16] = c1[g];
        }
      }
    }
    if ((bt + gridDim.x) * 4 < tiles) load(bt + gridDim.x);
    __syncthreads();
    const int rl = lane % AM_ROWS, c0 = lane / AM_ROWS;  // row in the tile, first column
    const int64_t r = r0 + rl;
    if (tw < tiles && r < n) {
      for (int c = c0; c < k; c += 64 / AM_ROWS) {
        const double v = tl[rl * 33 + c];
        if constexpr (NT) {
          __builtin_nontemporal_store(v, &S[(int64_t)c * ld + r]);
          if (codes) __builtin_nontemporal_store(code_of(v, cm), &codes[(int64_t)c * ldc + r]);
        } else {
          S[(int64_t)c * ld + r] = v;
          if (codes) codes[(int64_t)c * ldc + r] = code_of(v, cm);
        }
      }
    }
    __syncthreads();
  }
}

// Paired-row variant (PBH_APPLY_W2=1): 32-row wave tiles as in k_apply_mfma<32>, but each lane
// loads and stores two consecutive rows of a column with one 16-byte access (codes: 8 bytes), so
// a tile takes half the memory instructions.  The even rows of the tile feed the first 16-row
// MFMA block and the odd rows the second; the LDS transpose puts them back in row order.
// Needs ld, ldc even and S / codes 16- / 8-byte aligned (checked on the host).  The default step 3
// (interleaved A/B, profiles/r04/README_ab.md: 13.5-13.6 against 15.0-15.1 ms per cfg3 step).
// NT: non-temporal accesses as well (streaming: S, CS and the codes are not re-read by this kernel).
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ __launch_bounds__(256) void k_apply_mfma_w2(double* __restrict__ S, int64_t n, int k, int64_t ld,
                                                       const double* __restrict__ M, uint32_t* __restrict__ codes,
                                                       int64_t ldc, CodeMap cm) {
  constexpr int R = 32;
  __shared__ double tile[4][R * 33];
  __shared__ uint32_t cbase[kCodeSegments + 1];
  __shared__ double cscale[kCodeSegments];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* tl = tile[w];
  if (codes) {
    for (int j = threadIdx.x; j <= cm.m; j += 256) cbase[j] = cm.base[j];
    for (int j = threadIdx.x; j < cm.m; j += 256) cscale[j] = cm.scale[j];
    cm.base = cbase;
    cm.scale = cscale;
  }
  __syncthreads();
  const int q = lane >> 4, m16 = lane & 15;
  double b[8][2];
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int J = 0; J < 2; ++J) b[s][J] = M[(4 * s + q) * 32 + 16 * J + m16];
  const int64_t tiles = (n + R - 1) / R;
  double pa[2][8];  // [row parity][s]: rows r0 + 2 m16 (+1) of column 4 s + q
  auto load = [&](int64_t bt) {
    const int64_t tw = bt * 4 + w;
    const int64_t r = tw * R + 2 * m16;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int c = 4 * s + q;
      double2 v = {0.0, 0.0};
      if (tw < tiles && c < k) {
        const double* src = &S[(int64_t)c * ld + r];
        if (r + 1 < n) {
          const v2d t = NT ? __builtin_nontemporal_load((const v2d*)src) : *(const v2d*)src;
          v = double2{t.x, t.y};
        } else if (r < n) {
          v.x = src[0];
        }
      }
      pa[0][s] = v.x;
      pa[1][s] = v.y;
    }
  };
  if ((int64_t)blockIdx.x * 4 < tiles) load(blockIdx.x);
  for (int64_t bt = blockIdx.x; bt * 4 < tiles; bt += gridDim.x) {
    const int64_t tw = bt * 4 + w;
    const int64_t r0 = tw * R;
    if (tw < tiles) {
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        f64x4 c0 = {0.0, 0.0, 0.0, 0.0}, c1 = c0;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[par][s], b[s][0], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[par][s], b[s][1], c1, 0, 0, 0);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 2 * (q + 4 * g) + par;  // MFMA row i = q + 4 g is tile row 2 i + parity
          tl[row * 33 + m16] = c0[g];
          tl[row * 33 + 16 + m16] = c1[g];
        }
      }
    }
    if ((bt + gridDim.x) * 4 < tiles) load(bt + gridDim.x);
    __syncthreads();
    const int rp = lane & 15, c0 = lane >> 4;  // rows 2 rp, 2 rp + 1; first column
    const int64_t r = r0 + 2 * rp;
    if (tw < tiles && r < n) {
      for (int c = c0; c < k; c += 4) {
        const double v0 = tl[(2 * rp) * 33 + c], v1 = tl[(2 * rp + 1) * 33 + c];
        double* dst = &S[(int64_t)c * ld + r];
        if (r + 1 < n) {
          const v2d t = {v0, v1};
          if (NT)
            __builtin_nontemporal_store(t, (v2d*)dst);
          else
            *(v2d*)dst = t;
          if (codes) {
            const v2u cc = {code_of(v0, cm), code_of(v1, cm)};
            if (NT)
              __builtin_nontemporal_store(cc, (v2u*)&codes[(int64_t)c * ldc + r]);
            else
              *(v2u*)&codes[(int64_t)c * ldc + r] = cc;
          }
        } else {
          dst[0] = v0;
          if (codes) codes[(int64_t)c * ldc + r] = code_of(v0, cm);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace

size_t tie_workspace_bytes(int64_t n) {
  int64_t nt = sort_tiles(n);
  return 4 * (((size_t)nt * 8 + 255) & ~(size_t)255);
}

void tie_carve(void* ws, int64_t n, TieBuffers& tb) {
  int64_t nt = sort_tiles(n);
  size_t stride = ((size_t)nt * 8 + 255) & ~(size_t)255;
  char* p = (char*)ws;
  tb.first_head = (int64_t*)(p);
  tb.last_head = (int64_t*)(p + stride);
  tb.prev_head = (int64_t*)(p + 2 * stride);
  tb.next_head = (int64_t*)(p + 3 * stride);
}

int load_keys(const double* x, int64_t stride, int64_t n, uint64_t* keys, int32_t* flag, hipStream_t s) {
  PBH_TIMED(kKLoadKeys, s,
            hipLaunchKernelGGL(k_load_keys, dim3(grid_for(n, T, 8192)), dim3(T), 0, s, x, stride, n, keys, flag));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int rank_finish(int mode, const uint64_t* keys, const uint32_t* rows, int64_t n, const TieBuffers& tb,
                const RankOut& out, hipStream_t s, const uint8_t* eqprev) {
  const int64_t nt = sort_tiles(n);
  PBH_TIMED(kKHeadBounds, s,
            hipLaunchKernelGGL(k_head_bounds, dim3((unsigned)nt), dim3(T), 0, s, keys, eqprev, n, tb.first_head,
                               tb.last_head);
            hipLaunchKernelGGL(k_head_prefix, dim3(1), dim3(T), 0, s, tb.first_head, tb.last_head, nt, n,
                               tb.prev_head, tb.next_head));
  switch (mode) {
    case kModeScores:
      PBH_TIMED(kKRankScores, s,
                hipLaunchKernelGGL(k_rank_finish<kModeScores>, dim3((unsigned)nt), dim3(T), 0, s, keys, rows, eqprev, n,
                                   tb.prev_head, tb.next_head, out));
      break;
    case kModeScoresRank:
      PBH_TIMED(kKRankScores, s,
                hipLaunchKernelGGL(k_rank_finish<kModeScoresRank>, dim3((unsigned)nt), dim3(T), 0, s, keys, rows, eqprev,
                                   n, tb.prev_head, tb.next_head, out));
      break;
    case kModeGather:
      PBH_TIMED(kKRankGather, s,
                hipLaunchKernelGGL(k_rank_finish<kModeGather>, dim3((unsigned)nt), dim3(T), 0, s, keys, rows, eqprev, n,
                                   tb.prev_head, tb.next_head, out));
      break;
    default:
      hipLaunchKernelGGL(k_rank_finish<kModeRanks>, dim3((unsigned)nt), dim3(T), 0, s, keys, rows, eqprev, n, tb.prev_head,
                         tb.next_head, out);
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

static int64_t red_blocks(int64_t n, int64_t* chunk) {
  int64_t nb = (n + 4095) / 4096;
  if (nb > kGramBlocksMax) nb = kGramBlocksMax;
  if (nb < 1) nb = 1;
  int64_t c = (n + nb - 1) / nb;
  c = (c + GROWS - 1) / GROWS * GROWS;
  *chunk = c;
  return (n + c - 1) / c;
}

size_t gram_partials_bytes(int k) {
  int nt = (k + GT - 1) / GT;
  int pairs = nt * (nt + 1) / 2;
  size_t a = (size_t)pairs * kGramBlocksMax * GT * GT * 8;
  size_t b = (size_t)k * kGramBlocksMax * 8;
  return a > b ? a : b;
}

int column_sums(const double* S, int64_t n, int k, int64_t ld, double* partial, double* out, double divisor,
                hipStream_t s) {
  int64_t chunk;
  int64_t nb = red_blocks(n, &chunk);
  hipLaunchKernelGGL(k_colsum, dim3((unsigned)nb, (unsigned)k), dim3(kRedThreads), 0, s, S, n, ld, chunk, partial);
  hipLaunchKernelGGL(k_means, dim3((unsigned)k), dim3(256), 0, s, partial, (int)nb, k, divisor, out);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int means_from_partials(const double* partial, int nb, int k, double divisor, double* means, hipStream_t s) {
  hipLaunchKernelGGL(k_means, dim3((unsigned)k), dim3(256), 0, s, partial, nb, k, divisor, means);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int column_means(const double* S, int64_t n, int k, int64_t ld, double* partial, double* means, hipStream_t s) {
  return column_sums(S, n, k, ld, partial, means, (double)n, s);
}

int centered_gram(const double* S, int64_t n, int k, int64_t ld, const double* means, double* partials,
                  double* gram, hipStream_t s) {
  if (k <= 32) {
    int64_t nb = kGramBlocksMax;
    int64_t chunk = ((n + nb - 1) / nb + GM_ROWS - 1) / GM_ROWS * GM_ROWS;
    nb = (n + chunk - 1) / chunk;
    PBH_TIMED(kKGram, s,
              hipLaunchKernelGGL(k_gram_mfma, dim3((unsigned)nb), dim3(256), 0, s, S, n, k, ld, means, chunk,
                                 partials));
    hipLaunchKernelGGL(k_gram_rows_reduce<32>, dim3((k * k + 255) / 256), dim3(256), 0, s, partials, (int)nb, k,
                       gram);
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  int64_t chunk;
  int64_t nb = red_blocks(n, &chunk);
  int nt = (k + GT - 1) / GT;
  int pairs = nt * (nt + 1) / 2;
  PBH_TIMED(kKGram, s,
            hipLaunchKernelGGL(k_gram, dim3((unsigned)nb, (unsigned)pairs), dim3(256), 0, s, S, n, k, ld, means,
                               chunk, partials));
  hipLaunchKernelGGL(k_gram_reduce, dim3((GT * GT + 255) / 256, (unsigned)pairs), dim3(256), 0, s, partials, (int)nb,
                     k, gram);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int apply_decorrelate_correlate(double* S, int64_t n, int k, int64_t ld, const double* L, const double* inv_diag,
                                const double* P, hipStream_t s, uint32_t* codes, int64_t ldc, const CodeMap* cm) {
  dim3 g(grid_for(n, 256, 8192)), b(256);
  CodeMap c = cm ? *cm : CodeMap{};
  if (!cm) codes = nullptr;
  if (k <= 32) {
    double* M = nullptr;
    PBH_CHECK_HIP(hipMallocAsync((void**)&M, 32 * 32 * sizeof(double), s));
    hipLaunchKernelGGL(k_transform_matrix, dim3(1), dim3(64), 0, s, L, inv_diag, P, k, M);
    PBH_CHECK_LAUNCH();
    static const int rows = [] {  // 32 (default): 15.1 against 15.3-15.7 ms per step with 64
      const char* e = getenv("PBH_APPLY_ROWS");
      return e && atoi(e) == 64 ? 64 : 32;
    }();
    const int64_t tiles = (n + rows - 1) / rows;
    const unsigned gb = (unsigned)((tiles + 3) / 4 < 8192 ? (tiles + 3) / 4 : 8192);
    static const bool nt = [] {  // PBH_APPLY_NT=0: cached accesses (r4e A/B: 12.8 against 13.2 ms per step)
      const char* e = getenv("PBH_APPLY_NT");
      return !(e && atoi(e) == 0);
    }();
    static const bool w2 = [] {  // PBH_APPLY_W2=0: the one-row kernel (variant tests)
      const char* e = getenv("PBH_APPLY_W2");
      return !(e && atoi(e) == 0);
    }();
    const bool w2_ok = w2 && rows == 32 && ld % 2 == 0 && ((uintptr_t)S & 15) == 0 &&
                       (!codes || (ldc % 2 == 0 && ((uintptr_t)codes & 7) == 0));
    if (w2_ok && nt)
      PBH_TIMED(kKApply, s,
                hipLaunchKernelGGL(k_apply_mfma_w2<true>, dim3(gb > 0 ? gb : 1), b, 0, s, S, n, k, ld, M, codes, ldc,
                                   c));
    else if (w2_ok)
      PBH_TIMED(kKApply, s,
                hipLaunchKernelGGL(k_apply_mfma_w2<false>, dim3(gb > 0 ? gb : 1), b, 0, s, S, n, k, ld, M, codes, ldc,
                                   c));
    else if (rows == 32 && nt)
      PBH_TIMED(kKApply, s,
                hipLaunchKernelGGL((k_apply_mfma<32, true>), dim3(gb > 0 ? gb : 1), b, 0, s, S, n, k, ld, M, codes, ldc,
                                   c));
    else if (rows == 32)
      PBH_TIMED(kKApply, s,
                hipLaunchKernelGGL(k_apply_mfma<32>, dim3(gb > 0 ? gb : 1), b, 0, s, S, n, k, ld, M, codes, ldc, c));
    else
      PBH_TIMED(kKApply, s,
                hipLaunchKernelGGL(k_apply_mfma<64>, dim3(gb > 0 ? gb : 1), b, 0, s, S, n, k, ld, M, codes, ldc, c));
    PBH_CHECK_LAUNCH();
    PBH_CHECK_HIP(hipFreeAsync(M, s));
    return PBH_OK;
  }
  if (k <= 8)
    PBH_TIMED(kKApply, s, hipLaunchKernelGGL(k_apply<8>, g, b, 0, s, S, n, k, ld, L, inv_diag, P, codes, ldc, c));
  else if (k <= 16)
    PBH_TIMED(kKApply, s, hipLaunchKernelGGL(k_apply<16>, g, b, 0, s, S, n, k, ld, L, inv_diag, P, codes, ldc, c));
  else if (k <= 32)
    PBH_TIMED(kKApply, s, hipLaunchKernelGGL(k_apply<32>, g, b, 0, s, S, n, k, ld, L, inv_diag, P, codes, ldc, c));
  else if (k <= 64)
    PBH_TIMED(kKApply, s, hipLaunchKernelGGL(k_apply<64>, g, b, 0, s, S, n, k, ld, L, inv_diag, P, codes, ldc, c));
  else if (k <= 128)
    PBH_TIMED(kKApply, s,
              hipLaunchKernelGGL(k_apply<128>, g, b, 0, s, S, n, k, ld, L, inv_diag, P, codes, ldc, c));
  else {
    set_error("Iman-Conover: K = %d exceeds the supported maximum of 128 variables", k);
    return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// ---------------------------------------------------------------- 32-bit codes of the scores
static __global__ __launch_bounds__(256) void k_make_codes(const double* __restrict__ x, int64_t n, CodeMap cm,
                                                          uint32_t* __restrict__ codes) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    codes[i] = code_of(x[i], cm);
}

constexpr int kMaxRun = 16;

// Runs of equal codes, two phases.  Phase 1 streams the sorted codes with 16-byte loads:
// block b owns the contiguous positions [b * chunk, (b + 1) * chunk) and appends the start of
// every run of equal codes in it (~1% of positions for N(0, 1) scores at N = 1e8) to its own
// region of `starts` (a run has >= 2 members, so <= chunk / 2 + 1 entries), one LDS atomic per
// wave and no global atomics: the single global counter of a previous version serialised
// ~4e5 atomics per column at N = 1e8 (4 ms).  Phase 2 takes one run per thread and reorders it
// in place: a member's place in its run is the number of members before it in (value, position)
// order; ties with an earlier member are flagged in eqprev.
// flags: bit 0 = a run longer than kMaxRun (caller falls back to 64-bit keys), bit 1 = a tie.
constexpr int kRunBlocks = 2048;

static inline int64_t run_chunk(int64_t n, int64_t* nb) {
  int64_t c = (n + kRunBlocks - 1) / kRunBlocks;
  c = (c + 1023) / 1024 * 1024;
  *nb = (n + c - 1) / c;
  return c;
}
// run starts a block can hold: a run has >= 2 members, so <= min(chunk, n) / 2 + 1
PBH_HD inline int64_t run_stride(int64_t n, int64_t chunk) { return (chunk < n ? chunk : n) / 2 + 1; }

static __global__ __launch_bounds__(256) void k_runs_scan(const uint32_t* __restrict__ code, int64_t n, int64_t chunk,
                                                         uint32_t* __restrict__ starts,
                                                         uint32_t* __restrict__ counts) {
  __shared__ uint32_t cnt_sh;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) cnt_sh = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  uint32_t* out = starts + (int64_t)blockIdx.x * run_stride(n, chunk);
  for (int64_t q0 = lo; q0 < hi; q0 += 1024) {
    const int64_t p0 = q0 + 4 * (int64_t)threadIdx.x;
    uint32_t found = 0;  // bit i: position p0 + i starts a run
    if (p0 + 4 <= hi) {
      const uint4 c = *(const uint4*)(code + p0);
      const uint32_t cprev = p0 > 0 ? code[p0 - 1] : ~c.x;
      const uint32_t cnext = p0 + 4 < n ? code[p0 + 4] : ~c.w;
      found = (uint32_t)(c.x == c.y && cprev != c.x) | ((uint32_t)(c.y == c.z && c.x != c.y) << 1) |
              ((uint32_t)(c.z == c.w && c.y != c.z) << 2) | ((uint32_t)(c.w == cnext && c.z != c.w) << 3);
    } else {
      for (int64_t p = p0; p < hi; ++p) {
        const bool start = p + 1 < n && code[p + 1] == code[p] && (p == 0 || code[p - 1] != code[p]);
        found |= (uint32_t)start << (p - p0);
      }
    }
    const int cnt = __popc(found);
    int excl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(excl, o, 64);
      if (lane >= o) excl += y;
    }
    const int total = __shfl(excl, 63, 64);
    excl -= cnt;
    uint32_t base = 0;
    if (lane == 0 && total) base = atomicAdd(&cnt_sh, (uint32_t)total);
    base = __shfl(base, 0, 64);
    uint32_t k = base + (uint32_t)excl;
    for (int i = 0; i < 4; ++i)
      if (found & (1u << i)) out[k++] = (uint32_t)(p0 + i);
  }
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = cnt_sh;
}

static __global__ __launch_bounds__(256) void k_runs_resolve(const uint32_t* __restrict__ code,
                                                            uint32_t* __restrict__ rows,
                                                            const double* __restrict__ x, int64_t n, int64_t chunk,
                                                            const uint32_t* __restrict__ starts,
                                                            const uint32_t* __restrict__ counts,
                                                            uint8_t* __restrict__ eqprev, int32_t* flags) {
  const uint32_t m = counts[blockIdx.x];
  const uint32_t* st = starts + (int64_t)blockIdx.x * run_stride(n, chunk);
  for (uint32_t i = threadIdx.x; i < m; i += 256) {
    const int64_t s = st[i];
    const uint32_t c = code[s];
    int64_t e = s + 1;
    while (e + 1 < n && code[e + 1] == c && e - s + 1 <= kMaxRun) ++e;
    if (e - s + 1 > kMaxRun) {
      atomicOr(flags, 1);
      continue;
    }
    const int len = (int)(e - s + 1);
    // fully unrolled over kMaxRun with predicates: the run stays in registers (no scratch)
    uint32_t r[kMaxRun];
    double v[kMaxRun];
#pragma unroll
    for (int j = 0; j < kMaxRun; ++j) {
      r[j] = j < len ? rows[s + j] : 0u;
      v[j] = j < len ? x[r[j]] : 0.0;
    }
    bool any_tie = false;
#pragma unroll
    for (int p = 0; p < kMaxRun; ++p) {
      int pos = 0;
      bool tie = false;
#pragma unroll
      for (int j = 0; j < kMaxRun; ++j) {
        const bool other = j < len && j != p;
        pos += (other && (v[j] < v[p] || (v[j] == v[p] && j < p))) ? 1 : 0;
        tie |= other && v[j] == v[p] && j < p;
      }
      if (p < len) {
        rows[s + pos] = r[p];
        if (tie) {
          eqprev[s + pos] = 1;
          any_tie = true;
        }
      }
    }
    if (any_tie) atomicOr(flags, 2);
  }
}

// dst[p] = src[s + (e - s) / 2] for every position p of a tie run [s, e] (eqprev marks the
// non-head members): the int('average' rank) - 1 of correlation.py:422 that all members of
// the run share.  dst already holds src elsewhere.  16 positions per thread.
static __global__ __launch_bounds__(256) void k_tie_fix(const uint8_t* __restrict__ eqprev, int64_t n,
                                                       const double* __restrict__ src, double* __restrict__ dst) {
  const int64_t nq = (n + 15) / 16;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (int64_t)gridDim.x * 256) {
    const int64_t p0 = q * 16;
    bool any = false;
    if (p0 + 16 <= n) {
      const uint4 v = *(const uint4*)(eqprev + p0);
      any = (v.x | v.y | v.z | v.w) != 0u || (p0 + 16 < n && eqprev[p0 + 16] != 0);
    } else {
      for (int64_t p = p0; p < n; ++p) any |= eqprev[p] != 0;
    }
    if (!any) continue;
    for (int64_t p = p0; p < p0 + 16 && p < n; ++p) {
      const bool member = eqprev[p] != 0 || (p + 1 < n && eqprev[p + 1] != 0);
      if (!member) continue;
      int64_t st = p, e = p;
      while (st > 0 && eqprev[st] != 0) --st;
      while (e + 1 < n && eqprev[e + 1] != 0) ++e;
      dst[p] = src[st + (e - st) / 2];
    }
  }
}

int tie_fix_values(const uint8_t* eqprev, int64_t n, const double* src, double* dst, hipStream_t s) {
  PBH_CHECK_HIP(hipMemcpyAsync(dst, src, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(k_tie_fix, dim3(grid_for((n + 15) / 16, 256, 4096)), dim3(256), 0, s, eqprev, n, src, dst);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

size_t code_map_bytes() { return ((kCodeSegments + 1) * 4 + 255) / 256 * 256 + kCodeSegments * 8; }

void code_map_host(uint32_t* base, double* scale, double* x0, double* w) {
  const int m = kCodeSegments;
  *x0 = -8.5;
  *w = 17.0 / m;
  const double span = 4294967295.0 - m;
  for (int j = 0; j <= m; ++j) {
    double lo = *x0 + (double)j * (*w);
    double phi = 0.5 * erfc(-lo * 0.70710678118654752440);
    double b = floor(phi * span) + j;
    base[j] = (uint32_t)(b > 4294967295.0 ? 4294967295.0 : b);
  }
  for (int j = 0; j < m; ++j) scale[j] = (double)(base[j + 1] - base[j]) / (*w);
}

int make_codes(const double* x, int64_t n, const CodeMap& cm, uint32_t* codes, hipStream_t s) {
  PBH_TIMED(kKMakeCodes, s,
            hipLaunchKernelGGL(k_make_codes, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, x, n, cm, codes));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int resolve_code_runs(const uint32_t* codes, uint32_t* rows, const double* x, int64_t n, uint8_t* eqprev,
                      int32_t* flags, uint32_t* starts, uint32_t* counts, hipStream_t s) {
  int64_t nb;
  const int64_t chunk = run_chunk(n, &nb);
  PBH_TIMED(kKCodeRuns, s,
            (void)hipMemsetAsync(eqprev, 0, (size_t)n, s);
            hipLaunchKernelGGL(k_runs_scan, dim3((unsigned)nb), dim3(256), 0, s, codes, n, chunk, starts, counts);
            hipLaunchKernelGGL(k_runs_resolve, dim3((unsigned)nb), dim3(256), 0, s, codes, rows, x, n, chunk, starts,
                               counts, eqprev, flags));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// ---------------------------------------------------------------- row-major <-> column-major
// The operator API's X and Y are (n, k) row-major (correlation.py:368: numpy C order); every phase
// reads and writes whole columns.  Read strided, a column costs a 64-byte line per 8-byte value
// (k_load_keys 2.7 ms per 1e8-row column at k = 32); one tiled transpose of the whole block costs
// ~2 x 8 n k bytes, once.  A tile of kTRows rows x k columns passes through LDS (row pitch k + 1:
// conflict-free both ways): rows read contiguously, columns written contiguously.
constexpr int kTRows = 64;

__global__ __launch_bounds__(256) void k_rows_to_columns(const double* __restrict__ X, int64_t x_rs, int64_t n, int k,
                                                         double* __restrict__ out) {
  extern __shared__ double tile[];
  const int pitch = k + 1;
  for (int64_t r0 = (int64_t)blockIdx.x * kTRows; r0 < n; r0 += (int64_t)gridDim.x * kTRows) {
    const int rows = (int)((n - r0) < kTRows ? (n - r0) : kTRows);
    const int m = rows * k;
    for (int e = threadIdx.x; e < m; e += 256) {
      const int r = e / k, c = e - r * k;
      tile[r * pitch + c] = X[(r0 + r) * x_rs + c];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kTRows * k; e += 256) {
      const int c = e / kTRows, r = e - c * kTRows;
      if (r < rows) out[(int64_t)c * n + r0 + r] = tile[r * pitch + c];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_columns_to_rows(const double* __restrict__ in, int64_t n, int k,
                                                         double* __restrict__ Y, int64_t y_rs) {
  extern __shared__ double tile[];
  const int pitch = k + 1;
  for (int64_t r0 = (int64_t)blockIdx.x * kTRows; r0 < n; r0 += (int64_t)gridDim.x * kTRows) {
    const int rows = (int)((n - r0) < kTRows ? (n - r0) : kTRows);
    for (int e = threadIdx.x; e < kTRows * k; e += 256) {
      const int c = e / kTRows, r = e - c * kTRows;
      if (r < rows) tile[r * pitch + c] = in[(int64_t)c * n + r0 + r];
    }
    __syncthreads();
    const int m = rows * k;
    for (int e = threadIdx.x; e < m; e += 256) {
      const int r = e / k, c = e - r * k;
      Y[(r0 + r) * y_rs + c] = tile[r * pitch + c];
    }
    __syncthreads();
  }
}

int rows_to_columns(const double* X, int64_t x_rs, int64_t n, int k, double* out, hipStream_t s) {
  PBH_REQUIRE(k >= 1 && k <= 128 && x_rs >= k, "rows_to_columns: bad shape");
  const size_t lds = (size_t)kTRows * (k + 1) * sizeof(double);
  PBH_TIMED(kKTranspose, s,
            hipLaunchKernelGGL(k_rows_to_columns, dim3(grid_for(n, kTRows, 8192)), dim3(256), lds, s, X, x_rs, n, k,
                               out));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int columns_to_rows(const double* in, int64_t n, int k, double* Y, int64_t y_rs, hipStream_t s) {
  PBH_REQUIRE(k >= 1 && k <= 128 && y_rs >= k, "columns_to_rows: bad shape");
  const size_t lds = (size_t)kTRows * (k + 1) * sizeof(double);
  PBH_TIMED(kKTranspose, s,
            hipLaunchKernelGGL(k_columns_to_rows, dim3(grid_for(n, kTRows, 8192)), dim3(256), lds, s, in, n, k, Y,
                               y_rs));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

}  // namespace pbh
