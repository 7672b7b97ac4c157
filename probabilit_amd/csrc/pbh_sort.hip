#include <stdlib.h>
#include <string.h>

#include "pbh_error.h"
#include "pbh_sort.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int T = kSortThreads;
constexpr int IPT = kSortItems;
constexpr int TILE = kSortTile;

// ------------------------------------------------------------------ full digit histogram
template <typename K>
__global__ __launch_bounds__(256) void k_digit_hist(const K* __restrict__ keys, int64_t n,
                                                    uint32_t* __restrict__ hist) {
  constexpr int NB = sizeof(K);
  __shared__ uint32_t h[NB][256];
  for (int i = threadIdx.x; i < NB * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  // A byte every lane of the wave shares (the sign / exponent bytes of data within a binade) is
  // counted by one atomic of the wave's count instead of 64 atomics on one LDS word, which the LDS
  // serialises (k_digit_hist<u64> took 0.91 ms per 1e8 keys, 0.88 TB/s, pmc_valu_r6v.json).
  const int lane = threadIdx.x & 63;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    K k = keys[i];
    const uint64_t active = __ballot(true);
    const int leader = __builtin_ctzll(active);
#pragma unroll
    for (int p = 0; p < NB; ++p) {
      const uint32_t d = (uint32_t)(k >> (8 * p)) & 255u;
      const uint32_t d0 = (uint32_t)__shfl((int)d, leader, 64);
      if (__ballot(d == d0) == active) {
        if (lane == leader) atomicAdd(&h[p][d0], (uint32_t)__popcll(active));
      } else {
        atomicAdd(&h[p][d], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NB * 256; i += 256) {
    uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(&hist[i], v);
  }
}

// ------------------------------------------------------------------ upsweep
template <typename K>
__global__ __launch_bounds__(T) void k_upsweep(const K* __restrict__ keys, int64_t n, int shift,
                                              uint32_t* __restrict__ counts, int64_t ntiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * TILE;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int64_t i = base + j * T + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  counts[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// ------------------------------------------------------------------ exclusive scan (uint32)
__device__ __forceinline__ uint32_t block_exclusive_scan_256(uint32_t v, uint32_t* sh, uint32_t* total) {
  // 256 threads; sh has >= 256 + 8 entries
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[256 + w] = x;
  __syncthreads();
  uint32_t wprefix = 0;
  for (int i = 0; i < w; ++i) wprefix += sh[256 + i];
  if (total) *total = sh[256] + sh[257] + sh[258] + sh[259];
  __syncthreads();
  return wprefix + x - v;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ a, int64_t m,
                                                     uint32_t* __restrict__ partials) {
  __shared__ uint32_t sh[264];
  const int64_t base = (int64_t)blockIdx.x * 2048;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int64_t i = base + j * 256 + threadIdx.x;
    if (i < m) s += a[i];
  }
  uint32_t tot;
  block_exclusive_scan_256(s, sh, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_partials(uint32_t* __restrict__ partials, int64_t np) {
  __shared__ uint32_t sh[264];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t b0 = 0; b0 < np; b0 += 256) {
    int64_t i = b0 + threadIdx.x;
    uint32_t v = i < np ? partials[i] : 0;
    uint32_t tot;
    uint32_t ex = block_exclusive_scan_256(v, sh, &tot);
    uint32_t c = carry;
    if (i < np) partials[i] = c + ex;
    __syncthreads();
    if (threadIdx.x == 0) carry = c + tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_scan_down(uint32_t* __restrict__ a, int64_t m,
                                                   const uint32_t* __restrict__ partials) {
  __shared__ uint32_t sh[264];
  const int64_t base = (int64_t)blockIdx.x * 2048;
  // blocked: thread t owns elements base + t*8 .. +7
  uint32_t v[8];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int64_t i = base + threadIdx.x * 8 + j;
    v[j] = i < m ? a[i] : 0;
    s += v[j];
  }
  uint32_t ex = block_exclusive_scan_256(s, sh, nullptr) + partials[blockIdx.x];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int64_t i = base + threadIdx.x * 8 + j;
    if (i < m) a[i] = ex;
    ex += v[j];
  }
}


}  // namespace

int exclusive_scan_u32(uint32_t* a, int64_t m, uint32_t* partials, hipStream_t s) {
  int64_t np = scan_partials_count(m);
  PBH_TIMED(kKScan, s, hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)np), dim3(256), 0, s, a, m, partials);
            hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, s, partials, np);
            hipLaunchKernelGGL(k_scan_down, dim3((unsigned)np), dim3(256), 0, s, a, m, partials));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

namespace {

// ------------------------------------------------------------------ stable scatter
template <typename K, typename V = uint32_t>
__global__ __launch_bounds__(T) void k_scatter(const K* __restrict__ kin, const V* __restrict__ vin,
                                              K* __restrict__ kout, V* __restrict__ vout, int64_t n,
                                              int shift, const uint32_t* __restrict__ offsets, int64_t ntiles) {
  __shared__ K skeys[TILE];
  __shared__ V svals[TILE];
  __shared__ uint32_t run[256];
  __shared__ uint32_t chunk[2][4][256];  // double-buffered by item parity
  __shared__ uint32_t dstart[256 + 8];
  __shared__ uint32_t gbase[256];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * TILE;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  K key[IPT];
  uint32_t rank[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int64_t i = base + j * T + t;
    key[j] = i < n ? kin[i] : (K)0;
  }
  run[t] = 0;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    uint32_t(*ck)[256] = chunk[j & 1];
    ck[w][lane] = 0;
    ck[w][lane + 64] = 0;
    ck[w][lane + 128] = 0;
    ck[w][lane + 192] = 0;
    __syncthreads();
    const int64_t i = base + j * T + t;
    const bool valid = i < n;
    const uint32_t d = (uint32_t)(key[j] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      uint64_t bb = __ballot(valid && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    uint32_t below = (uint32_t)__popcll(peers & lanemask_lt);
    if (valid && below == 0) ck[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t r = run[d] + below;
      for (int ww = 0; ww < w; ++ww) r += ck[ww][d];
      rank[j] = r;
    }
    __syncthreads();
    run[t] += ck[0][t] + ck[1][t] + ck[2][t] + ck[3][t];
  }
  __syncthreads();
  uint32_t hist_t = run[t];
  uint32_t ex = block_exclusive_scan_256(hist_t, dstart, nullptr);
  dstart[t] = ex;  // safe: scan helper only uses dstart[256..259] after its final barrier
  gbase[t] = offsets[(int64_t)t * ntiles + tile];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int64_t i = base + j * T + t;
    if (i < n) {
      uint32_t d = (uint32_t)(key[j] >> shift) & 255u;
      uint32_t lp = dstart[d] + rank[j];
      skeys[lp] = key[j];
      svals[lp] = vin ? vin[i] : (V)i;  // NULL payload: the identity (row index)
    }
  }
  __syncthreads();
  const int64_t cnt = (n - base) < TILE ? (n - base) : TILE;
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int p = j * T + t;
    if (p < cnt) {
      K k = skeys[p];
      uint32_t d = (uint32_t)(k >> shift) & 255u;
      int64_t o = (int64_t)gbase[d] + (p - (int64_t)dstart[d]);
      kout[o] = k;
      vout[o] = svals[p];
    }
  }
}

// ------------------------------------------------------------------ one-sweep scatter
// One launch per digit pass, no upsweep / scan: every tile ranks its keys per wave (one
// wave-private digit counter array, no block barrier inside the ranking loop), publishes its
// digit counts, and finds the count of each digit in all earlier tiles by decoupled
// look-back over the published (flag | count) words (Merrill & Garland's single-pass scan,
// as in Adinets & Merrill's Onesweep).  Global digit bases come from the one up-front
// histogram.  Tile ids are taken from an atomic counter, so a tile only ever waits on tiles
// that started before it: the look-back always terminates.
// Every word carries its pass's epoch (bits 40..61): a word left by an earlier pass reads as "not
// yet published", so the words are cleared once per workspace (sweep_begin) instead of by a fill
// before every pass, and the tile counter runs on across passes (tile = counter - tile_base).
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62, kFlagMask = 3ull << 62;
constexpr uint64_t kCountMask = (1ull << 40) - 1;
constexpr int kEpochShift = 40;
constexpr uint32_t kEpochMax = (1u << 22) - 1;

template <typename K, typename V, int IPTT>
__global__ __launch_bounds__(T) void k_onesweep(const K* __restrict__ kin, const V* __restrict__ vin,
                                               K* __restrict__ kout, V* __restrict__ vout, int64_t n, int shift,
                                               const uint32_t* __restrict__ digit_base, uint64_t* status,
                                               uint32_t* tile_counter, uint32_t epoch, uint32_t tile_base) {
  constexpr int IPT = IPTT;
  constexpr int TILE = T * IPTT;
  __shared__ K skeys[TILE];
  __shared__ V svals[TILE];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t dstart[256 + 8];
  __shared__ int64_t gbase[256];
  __shared__ uint32_t tile_sh;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) tile_sh = atomicAdd(tile_counter, 1u) - tile_base;
#pragma unroll
  for (int q = 0; q < 4; ++q) wcnt[w][lane + 64 * q] = 0;
  __syncthreads();
  const int64_t tile = tile_sh;
  const int64_t base = tile * TILE;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  // wave w owns tile positions [w * 1024, (w + 1) * 1024), item-major: j * 64 + lane
  K key[IPT];
  V val[IPT];
  uint32_t rank[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int64_t i = base + w * (IPT * 64) + j * 64 + lane;
    const bool valid = i < n;
    key[j] = valid ? kin[i] : (K)0;
    val[j] = valid ? (vin ? vin[i] : (V)i) : (V)0;
  }
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int64_t i = base + w * (IPT * 64) + j * 64 + lane;
    const bool valid = i < n;
    const uint32_t d = (uint32_t)(key[j] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lanemask_lt);
    const uint32_t c = valid ? wcnt[w][d] : 0u;
    rank[j] = c + below;
    if (valid && below == 0) wcnt[w][d] = c + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // thread t = digit t
  const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
  const uint32_t tot = c0 + c1 + c2 + c3;
  uint64_t* my = status + tile * 256 + t;
  const uint64_t etag = (uint64_t)epoch << kEpochShift;
  if (tile == 0)
    __hip_atomic_store(my, kFlagInc | etag | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    __hip_atomic_store(my, kFlagAgg | etag | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t ex = block_exclusive_scan_256(tot, dstart, nullptr);
  uint64_t excl = 0;
  if (tile > 0) {
    int64_t tp = tile - 1;
    uint32_t spins = 0;
    while (true) {
      const uint64_t sv = __hip_atomic_load(status + tp * 256 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t flag = (sv & ~kFlagMask & ~kCountMask) == etag ? sv & kFlagMask : 0ull;
      if (flag == 0) {  // tile tp has not published in this pass yet
        if (++spins > (1u << 26)) {  // cannot happen (see above); never hang the device on a bug
          atomicOr(tile_counter + 1, 1u);
          break;
        }
        continue;
      }
      excl += sv & kCountMask;
      if (flag == kFlagInc) break;
      --tp;
    }
    __hip_atomic_store(my, kFlagInc | etag | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  dstart[t] = ex;
  wcnt[0][t] = 0;
  wcnt[1][t] = c0;
  wcnt[2][t] = c0 + c1;
  wcnt[3][t] = c0 + c1 + c2;
  gbase[t] = (int64_t)digit_base[t] + (int64_t)excl - (int64_t)ex;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int64_t i = base + w * (IPT * 64) + j * 64 + lane;
    if (i < n) {
      const uint32_t d = (uint32_t)(key[j] >> shift) & 255u;
      const uint32_t lp = dstart[d] + wcnt[w][d] + rank[j];
      skeys[lp] = key[j];
      svals[lp] = val[j];
    }
  }
  __syncthreads();
  const int cnt = (int)((n - base) < TILE ? (n - base) : TILE);
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * T + t;
    if (p < cnt) {
      const K k = skeys[p];
      const uint32_t d = (uint32_t)(k >> shift) & 255u;
      const int64_t o = gbase[d] + p;
      kout[o] = k;
      vout[o] = svals[p];
    }
  }
}

// bases[p * 256 + d] = exclusive scan over digits of hist[p * 256 + d], for np byte positions
__global__ __launch_bounds__(256) void k_digit_bases(const uint32_t* __restrict__ hist, uint32_t* __restrict__ bases) {
  __shared__ uint32_t sh[264];
  const uint32_t v = hist[blockIdx.x * 256 + threadIdx.x];
  bases[blockIdx.x * 256 + threadIdx.x] = block_exclusive_scan_256(v, sh, nullptr);
}

// digit bases of the row keys of place_by_row: rows are a permutation of [0, n), so digit d at
// `shift` counts the rows r < n with (r >> shift) & 255 == d, in closed form.
__global__ __launch_bounds__(256) void k_place_bases(int64_t n, int shift, uint32_t* __restrict__ bases) {
  __shared__ uint32_t sh[264];
  const uint32_t d = threadIdx.x;
  const int64_t span = (int64_t)1 << shift;
  uint64_t count = 0;
  for (int64_t h = 0;; ++h) {
    const int64_t lo = ((h << 8) + d) << shift;
    if (lo >= n) break;
    count += (uint64_t)((n - lo) < span ? (n - lo) : span);
  }
  bases[d] = block_exclusive_scan_256((uint32_t)count, sh, nullptr);
}

// Items per thread of the one-sweep scatter (tile = 256 x items).  Measured on MI355X
// (profiles/r01/bench_r14_*, bench_r40_*, bench_r41_*): 32-bit key + 32-bit payload passes take 36
// items (9216-key tiles: ~36 keys per digit bucket, whole 128-byte lines per burst; 72 KB of LDS,
// 2 tiles per CU; 0.59 ms per 1e8-key pass against 0.62 with 32, 0.69 with 24); the 32-bit key +
// 64-bit value passes of the row placement with 24
// (72 KB, still 2 tiles per CU: 0.75 ms per 1e8-row pass against 0.91 with 16).
int onesweep_items(size_t item_bytes_minus_key4) {
  return item_bytes_minus_key4 <= 4 ? 36 : 24;  // item_bytes (key + value) 8 -> 36, 12 -> 24: ~79 KB of LDS either way
}

// The next pass's epoch and tile base; the words and the counter are cleared (one fill) on a
// workspace's first pass and when the epoch or the counter would wrap.
int sweep_begin(SweepState& sw, uint64_t* status, int64_t nt, hipStream_t s, uint32_t* epoch, uint32_t* tile_base) {
  if (sw.epoch == 0 || sw.epoch >= kEpochMax || (uint64_t)sw.tile_base + (uint64_t)nt >= (1ull << 31)) {
    PBH_CHECK_HIP(hipMemsetAsync(status, 0, sw.bytes, s));  // words, tile counter, stuck flag
    sw.epoch = 0;
    sw.tile_base = 0;
  }
  *epoch = ++sw.epoch;
  *tile_base = sw.tile_base;
  sw.tile_base += (uint32_t)nt;
  return PBH_OK;
}

// counter: the tile counter (the stuck flag is the word after it), at status + 256 * sort_tiles(n)
template <typename K, typename V, int IPT_>
int launch_onesweep_ipt(const K* kin, const V* vin, K* kout, V* vout, int64_t n, int shift, const uint32_t* bases,
                        uint64_t* status, uint32_t* counter, SweepState& sw, hipStream_t s) {
  const int64_t nt = (n + T * IPT_ - 1) / (T * IPT_);
  uint32_t epoch = 0, tile_base = 0;
  if (int st = sweep_begin(sw, status, nt, s, &epoch, &tile_base)) return st;
  hipLaunchKernelGGL((k_onesweep<K, V, IPT_>), dim3((unsigned)nt), dim3(T), 0, s, kin, vin, kout, vout, n, shift,
                     bases, status, counter, epoch, tile_base);
  return PBH_OK;
}

template <typename K, typename V>
int launch_onesweep(const K* kin, const V* vin, K* kout, V* vout, int64_t n, int shift, const uint32_t* bases,
                    uint64_t* status, uint32_t* counter, SweepState& sw, hipStream_t s) {
  if (onesweep_items(sizeof(K) + sizeof(V) - 4) == 36)  // u64 key + u32 row sizes like u32 + f64
    return launch_onesweep_ipt<K, V, 36>(kin, vin, kout, vout, n, shift, bases, status, counter, sw, s);
  return launch_onesweep_ipt<K, V, 24>(kin, vin, kout, vout, n, shift, bases, status, counter, sw, s);
}

// ------------------------------------------------------------------ row placement
__global__ void k_or_flag(const uint32_t* __restrict__ word, int32_t* __restrict__ err) {
  if (threadIdx.x == 0 && *word) atomicOr(err, 1);
}

// Bucket b = rows [b * kPlaceRows, (b + 1) * kPlaceRows).  Because `rows` is a permutation,
// after the bucket passes bucket b occupies exactly positions [b * kPlaceRows, ...) of the
// staging arrays; one workgroup assembles its bucket in LDS and writes it out contiguously.
__global__ __launch_bounds__(T) void k_place(const uint32_t* __restrict__ rows, const double* __restrict__ v,
                                            int64_t n, double* __restrict__ y, int64_t y_rs) {
  __shared__ double buf[kPlaceRows];
  const int64_t r0 = (int64_t)blockIdx.x * kPlaceRows;
  const int cnt = (int)((n - r0) < kPlaceRows ? (n - r0) : kPlaceRows);
  for (int p = threadIdx.x; p < cnt; p += T) buf[rows[r0 + p] - (uint32_t)r0] = v[r0 + p];
  __syncthreads();
  if (y_rs == 1) {
    for (int p = threadIdx.x; p < cnt; p += T) y[r0 + p] = buf[p];
  } else {
    for (int p = threadIdx.x; p < cnt; p += T) y[(r0 + p) * y_rs] = buf[p];
  }
}

// ------------------------------------------------------------------ top-16-bit code buckets
// Step 4's 32-bit code sort in three launches instead of four one-sweep passes plus the run
// fix-up: two one-sweep passes on bytes 2 and 3 leave the (code, row) pairs sorted by the top
// 16 code bits, stable in row order; every top-16 bucket (~n / 65536 pairs: the codes are
// Phi-uniformised, so ~1500 at n = 1e8) is then finished by one wave in LDS -- two stable
// counting passes on bytes 0 and 1, and the ordering of equal-code runs by the full value with
// the exact-tie flags, as resolve_code_runs does (equal codes share their bucket).
// A bucket larger than kBucketCap, or a run longer than kBucketMaxRun, sets flags bit 0 and the
// caller falls back to the 64-bit sort, exactly like a long run of the four-pass path.
constexpr int kBucketCap = 2048;  // pairs per bucket (one wave)
constexpr int kBucketMaxRun = 16;
constexpr uint32_t kNoStart = 0xFFFFFFFFu;

// start[b] = first position of bucket b (keys sorted by their top 16 bits); untouched (kNoStart)
// for empty buckets.
__global__ __launch_bounds__(256) void k_bucket_starts(const uint32_t* __restrict__ keys, int64_t n,
                                                      uint32_t* __restrict__ start) {
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
    const uint32_t b = keys[p] >> 16;
    if (p == 0 || (keys[p - 1] >> 16) != b) start[b] = (uint32_t)p;
  }
}

// Every wave finishes one bucket on its own (no block barriers): the bucket's low 16 code bits
// and rows sit in registers (32 items per lane, position order j * 64 + lane); the low byte pass
// ranks with LDS atomics (see wave_count_pass), the stable high byte pass with ballot peer
// matching against LDS digit counters; each pass
// scans the 256 counters across the wave, and scatters into the wave's LDS arrays, which are
// read back in position order for the next pass.  ~15 KB of LDS per wave.  (Measured
// alternatives, profiles/r01/: one block-wide bucket per workgroup was 2x slower; a non-stable
// atomic grouping + per-group insertion sort was slower on columns with equal-code runs, its
// insertion chains being LDS-latency bound.)
constexpr int kWBItems = kBucketCap / 64;

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WaveBucket {
  uint16_t key[kBucketCap];
  uint32_t row[kBucketCap];
  uint8_t eq[kBucketCap];
  uint32_t cnt[256];
  uint16_t runs[256];
};

// one stable pass on the byte of k at `shift` (0 or 8); k / r: this lane's items in position order
__device__ __forceinline__ void wave_radix_pass(uint32_t (&k)[kWBItems], uint32_t (&r)[kWBItems], int len,
                                                int shift, WaveBucket& B) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int q = 0; q < 4; ++q) B.cnt[lane * 4 + q] = 0;
  wave_sync();
  uint32_t rank[kWBItems];
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    const bool valid = j * 64 + lane < len;
    const uint32_t d = (k[j] >> shift) & 255u;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t below = (uint32_t)__popcll(peers & lt);
    const uint32_t c = valid ? B.cnt[d] : 0u;  // LDS is in order within a wave
    rank[j] = c + below;
    if (valid && below == 0) B.cnt[d] = c + (uint32_t)__popcll(peers);
  }
  wave_sync();
  // exclusive scan of the 256 counters: lane l owns digits 4 l .. 4 l + 3
  uint32_t v[4], sum = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = B.cnt[lane * 4 + q];
    sum += v[q];
  }
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  uint32_t run = incl - sum;
  wave_sync();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    B.cnt[lane * 4 + q] = run;
    run += v[q];
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    if (j * 64 + lane < len) {
      const uint32_t lp = B.cnt[(k[j] >> shift) & 255u] + rank[j];
      B.key[lp] = (uint16_t)k[j];
      B.row[lp] = r[j];
    }
  }
  wave_sync();
}

// The first (low byte) pass need not be stable: pairs that tie on the low byte and then on the
// high byte have equal codes, i.e. they form a run, which is put in value order afterwards.  So
// it ranks with one LDS atomic per item instead of the ballot matching.
__device__ __forceinline__ void wave_count_pass(uint32_t (&k)[kWBItems], uint32_t (&r)[kWBItems], int len,
                                                WaveBucket& B) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < 4; ++q) B.cnt[lane * 4 + q] = 0;
  wave_sync();
  uint32_t rank[kWBItems];
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;
    rank[j] = (j * 64 + lane < len) ? atomicAdd(&B.cnt[k[j] & 255u], 1u) : 0u;
  }
  wave_sync();
  uint32_t v[4], sum = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = B.cnt[lane * 4 + q];
    sum += v[q];
  }
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  uint32_t run = incl - sum;
  wave_sync();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    B.cnt[lane * 4 + q] = run;
    run += v[q];
  }
  wave_sync();
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    if (j * 64 + lane < len) {
      const uint32_t lp = B.cnt[k[j] & 255u] + rank[j];
      B.key[lp] = (uint16_t)k[j];
      B.row[lp] = r[j];
    }
  }
  wave_sync();
}

// Stable value order of the run [p, p + L) of equal codes (L <= R), with the exact-tie flags:
// member q lands after every member of smaller value and every earlier member of equal value.
template <int R>
__device__ __forceinline__ bool resolve_run(WaveBucket& B, int p, int L, const double* __restrict__ x) {
  uint32_t rr[R];
  double v[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    rr[j] = j < L ? B.row[p + j] : 0u;
    v[j] = j < L ? x[rr[j]] : 0.0;
  }
  bool any_tie = false;
#pragma unroll
  for (int q = 0; q < R; ++q) {
    int pos = 0;
    bool tie = false;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const bool other = j < L && j != q;
      pos += (other && (v[j] < v[q] || (v[j] == v[q] && j < q))) ? 1 : 0;
      tie |= other && v[j] == v[q] && j < q;
    }
    if (q < L) {
      B.row[p + pos] = rr[q];
      B.eq[p + pos] = tie ? 1 : 0;
      any_tie |= tie;
    }
  }
  return any_tie;
}

constexpr int kCBWaves = 2;  // waves (buckets) per block: ~31 KB of LDS

__global__ __launch_bounds__(64 * kCBWaves) void k_code_buckets(const uint32_t* __restrict__ keys,
                                                               uint32_t* __restrict__ rows,
                                                               const double* __restrict__ x, int64_t n,
                                                               const uint32_t* __restrict__ start,
                                                               uint8_t* __restrict__ eqprev, int32_t* flags) {
  __shared__ WaveBucket wb[kCBWaves];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  WaveBucket& B = wb[w];
  const int bkt = blockIdx.x * kCBWaves + w;
  if (bkt >= 65536) return;
  const uint32_t s0 = start[bkt];
  if (s0 == kNoStart) return;  // empty bucket (wave-uniform)
  // end: the first non-empty bucket after this one, 64 candidates per probe
  int64_t e = n;
  for (int c0 = bkt + 1; c0 < 65536; c0 += 64) {
    const int c = c0 + lane;
    const uint32_t v = c < 65536 ? start[c] : kNoStart;
    const uint64_t m = __ballot(v != kNoStart);
    if (m) {
      e = __shfl(v, __builtin_ctzll(m), 64);
      break;
    }
  }
  const int64_t s = s0;
  if (e - s > kBucketCap) {
    if (lane == 0) atomicOr(flags, 1);
    return;
  }
  const int len = __builtin_amdgcn_readfirstlane((int)(e - s));
  uint32_t k[kWBItems], r[kWBItems];
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    const int p = j * 64 + lane;
    k[j] = p < len ? (keys[s + p] & 0xFFFFu) : 0u;
    r[j] = p < len ? rows[s + p] : 0u;
  }
  wave_count_pass(k, r, len, B);
#pragma unroll
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    const int p = j * 64 + lane;
    k[j] = p < len ? B.key[p] : 0u;
    r[j] = p < len ? B.row[p] : 0u;
  }
  wave_sync();
  wave_radix_pass(k, r, len, 8, B);
  // runs of equal codes (equal low 16 bits inside a bucket), compacted into B.runs
  int nrun = 0;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll 4
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    const int p = j * 64 + lane;
    bool st = false;
    if (p < len) {
      const uint16_t c = B.key[p];
      st = p + 1 < len && B.key[p + 1] == c && (p == 0 || B.key[p - 1] != c);
      B.eq[p] = 0;
    }
    const uint64_t m = __ballot(st);
    const int slot = nrun + (int)__popcll(m & lt);
    if (st && slot < 256) B.runs[slot] = (uint16_t)p;
    nrun += (int)__popcll(m);
  }
  wave_sync();
  if (nrun > 256) {
    if (lane == 0) atomicOr(flags, 1);
    return;
  }
  bool any_tie = false;
  for (int i = lane; i < nrun; i += 64) {  // as k_runs_resolve: stable order by value, ties flagged
    const int p = B.runs[i];
    const uint16_t c = B.key[p];
    int L = 2;
    while (p + L < len && B.key[p + L] == c && L <= kBucketMaxRun) ++L;
    if (L > kBucketMaxRun) {
      atomicOr(flags, 1);
      continue;
    }
    if (L <= 4)  // nearly every run: a 4-wide register version; 16-wide only when some lane needs it
      any_tie |= resolve_run<4>(B, p, L, x);
    else
      any_tie |= resolve_run<kBucketMaxRun>(B, p, L, x);
  }
  if (__ballot(any_tie) && lane == 0) atomicOr(flags, 2);
  wave_sync();
#pragma unroll 4
  for (int j = 0; j < kWBItems; ++j) {
    if (j * 64 >= len) break;  // wave-uniform: a small bucket skips the empty item slots
    const int p = j * 64 + lane;
    if (p < len) {
      rows[s + p] = B.row[p];
      eqprev[s + p] = B.eq[p];
    }
  }
}

}  // namespace

int place_by_row(const uint32_t* rows, const double* v, int64_t n, double* y, int64_t y_rs, const PlaceBuffers& pb,
                 hipStream_t s, int32_t* err) {
  PBH_REQUIRE(n >= 1 && n < ((int64_t)1 << 32), "place_by_row: n out of range");
  int bits = 0;
  while (((int64_t)1 << bits) < n) ++bits;
  const int64_t nt = sort_tiles(n);
  const uint32_t* rin = rows;
  const double* vin = v;
  int cur = 0;
  for (int shift = kPlaceShift; shift < bits; shift += 8) {
    hipLaunchKernelGGL(k_place_bases, dim3(1), dim3(256), 0, s, n, shift, pb.bases);
    PBH_CHECK_LAUNCH();
    int st = PBH_OK;
    PBH_TIMED(kKPlaceScatter, s,
              st = launch_onesweep<uint32_t, double>(rin, vin, pb.rows[cur], pb.vals[cur], n, shift, pb.bases,
                                                     pb.status, (uint32_t*)(pb.status + nt * 256), *pb.sweep, s));
    if (st) return st;
    PBH_CHECK_LAUNCH();
    rin = pb.rows[cur];
    vin = pb.vals[cur];
    cur ^= 1;
  }
  const int64_t nb = (n + kPlaceRows - 1) / kPlaceRows;
  PBH_TIMED(kKPlace, s, hipLaunchKernelGGL(k_place, dim3((unsigned)nb), dim3(T), 0, s, rin, vin, n, y, y_rs));
  PBH_CHECK_LAUNCH();
  if (bits > kPlaceShift && err) {
    hipLaunchKernelGGL(k_or_flag, dim3(1), dim3(64), 0, s, (const uint32_t*)(pb.status + nt * 256) + 1, err);
    PBH_CHECK_LAUNCH();
  } else if (bits > kPlaceShift) {
    uint32_t stuck = 0;
    PBH_CHECK_HIP(hipMemcpyAsync(&stuck, (uint32_t*)(pb.status + nt * 256) + 1, 4, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    if (stuck) {
      set_error("row placement: one-sweep look-back did not complete");
      return PBH_ERR_HIP;
    }
  }
  return PBH_OK;
}

bool code_buckets_enabled(int64_t n) {
  const char* e = getenv("PBH_STEP4");  // read per call: "buckets" forces, "lsd" disables
  if (e && strcmp(e, "buckets") == 0) return n >= 2 && n < ((int64_t)1 << 32);
  if (e && strcmp(e, "lsd") == 0) return false;
  return n >= ((int64_t)1 << 22) && n <= (int64_t)110000000;  // mean bucket <= ~1700 of the 2048 cap
}

bool code_hist_flat(const uint32_t* hist4, int64_t n) {
  const char* force = getenv("PBH_STEP4");
  if (force && strcmp(force, "buckets") == 0) return true;  // tests: exercise the kernel and its safety net
  uint32_t top_max = 0;
  for (int d = 0; d < 256; ++d) top_max = hist4[3 * 256 + d] > top_max ? hist4[3 * 256 + d] : top_max;
  return (double)top_max <= 1.5 * (double)n / 256.0 + 64.0;
}

int code_hist(const uint32_t* codes, int64_t n, uint32_t* hist4, hipStream_t s) {
  PBH_CHECK_HIP(hipMemsetAsync(hist4, 0, 4 * 256 * 4, s));
  PBH_TIMED(kKSortDigitHist32, s,
            hipLaunchKernelGGL(k_digit_hist<uint32_t>, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, codes, n, hist4));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int code_sort_buckets(SortBuffers& b, int64_t n, const uint32_t* codes, const double* x, uint8_t* eqprev,
                      int32_t* flags, hipStream_t s, int* out_buf, const uint32_t* hist_dev, int flat) {
  PBH_REQUIRE(n >= 2 && n < ((int64_t)1 << 32), "code_sort_buckets: n out of range");
  const int64_t nt = sort_tiles(n);
  uint32_t* keys[2] = {(uint32_t*)b.keys[0], (uint32_t*)b.keys[1]};
  if (!hist_dev) {
    int st = code_hist(codes, n, b.hist, s);
    if (st) return st;
    hist_dev = b.hist;
    // A column whose top-byte histogram is far from flat (a mixture with discrete spikes, e.g.
    // a poisson-dominated correlated score) would overflow top-16 buckets: leave it to the four
    // passes (*out_buf = -1).  The kernel's overflow flag stays the safety net.
    PBH_CHECK_HIP(hipMemcpyAsync(b.hist_host, b.hist, 4 * 256 * 4, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    flat = code_hist_flat(b.hist_host, n) ? 1 : 0;
  }
  if (!flat) {
    *out_buf = -1;
    return PBH_OK;
  }
  hipLaunchKernelGGL(k_digit_bases, dim3(4), dim3(256), 0, s, hist_dev, b.bases);
  PBH_CHECK_LAUNCH();
  int cur = 0;
  for (int ip = 0; ip < 2; ++ip) {
    const int byte = 2 + ip;
    int st = PBH_OK;
    PBH_TIMED(kKSortScatter32, s,
              st = launch_onesweep<uint32_t, uint32_t>(ip == 0 ? codes : keys[cur], ip == 0 ? nullptr : b.vals[cur],
                                                       keys[cur ^ 1], b.vals[cur ^ 1], n, 8 * byte,
                                                       b.bases + byte * 256, b.status,
                                                       (uint32_t*)(b.status + nt * 256), b.sweep, s));
    if (st) return st;
    PBH_CHECK_LAUNCH();
    cur ^= 1;
  }
  // 65536 bucket starts: in `counts` (256 * sort_tiles(n) words) when it is large enough
  uint32_t* start = b.counts;
  const bool own = (int64_t)256 * nt < 65536;
  if (own) PBH_CHECK_HIP(hipMallocAsync((void**)&start, 65536 * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(start, 0xFF, 65536 * 4, s));
  PBH_TIMED(kKCodeRuns, s,
            hipLaunchKernelGGL(k_bucket_starts, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, keys[cur], n, start);
            hipLaunchKernelGGL(k_code_buckets, dim3(65536 / kCBWaves), dim3(64 * kCBWaves), 0, s, keys[cur], b.vals[cur], x, n, start,
                               eqprev, flags));
  PBH_CHECK_LAUNCH();
  if (own) PBH_CHECK_HIP(hipFreeAsync(start, s));
  *out_buf = cur;
  return PBH_OK;
}

size_t sort_workspace_bytes(int64_t n) {
  int64_t nt = sort_tiles(n);
  int64_t m = 256 * nt;
  size_t b = 0;
  auto add = [&](size_t bytes) { b += (bytes + 255) & ~(size_t)255; };
  add((size_t)n * 8);
  add((size_t)n * 8);
  add((size_t)n * 4);
  add((size_t)n * 4);
  add((size_t)m * 4);
  add((size_t)scan_partials_count(m) * 4);
  add(8 * 256 * 4);
  add((size_t)m * 8 + 256);  // one-sweep status words + tile counter
  add(8 * 256 * 4);          // digit bases
  return b;
}

void sort_carve(void* ws, int64_t n, SortBuffers& sb) {
  int64_t nt = sort_tiles(n);
  int64_t m = 256 * nt;
  char* p = (char*)ws;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~(size_t)255;
    return (void*)r;
  };
  sb.keys[0] = (uint64_t*)take((size_t)n * 8);
  sb.keys[1] = (uint64_t*)take((size_t)n * 8);
  sb.vals[0] = (uint32_t*)take((size_t)n * 4);
  sb.vals[1] = (uint32_t*)take((size_t)n * 4);
  sb.counts = (uint32_t*)take((size_t)m * 4);
  sb.partials = (uint32_t*)take((size_t)scan_partials_count(m) * 4);
  sb.hist = (uint32_t*)take(8 * 256 * 4);
  sb.status = (uint64_t*)take((size_t)m * 8 + 256);
  sb.sweep = SweepState{0, 0, (size_t)m * 8 + 256};  // cleared by the first pass (sweep_begin)
  sb.bases = (uint32_t*)take(8 * 256 * 4);
}

template <typename K>
int radix_sort_impl(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf, const K* in = nullptr,
                    int skip_low = 0, bool* low_varies = nullptr) {
  constexpr int NB = sizeof(K);
  PBH_REQUIRE(n >= 1 && n < ((int64_t)1 << 32), "radix sort: n out of range");
  const int64_t nt = sort_tiles(n);
  K* keys[2] = {(K*)b.keys[0], (K*)b.keys[1]};
  const K* first = in ? in : keys[0];  // pass 0 reads here and writes keys[1]
  // which byte positions vary?
  PBH_CHECK_HIP(hipMemsetAsync(b.hist, 0, 8 * 256 * 4, s));
  PBH_TIMED(NB == 8 ? kKSortDigitHist : kKSortDigitHist32, s,
            hipLaunchKernelGGL(k_digit_hist<K>, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, first, n, b.hist));
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipMemcpyAsync(b.hist_host, b.hist, NB * 256 * 4, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  int passes[8], npass = 0;
  if (low_varies) *low_varies = false;
  for (int p = 0; p < NB; ++p) {
    int nonzero = 0;
    for (int d = 0; d < 256; ++d) nonzero += b.hist_host[p * 256 + d] != 0;
    if (nonzero > 1 && p < skip_low) {
      *low_varies = true;  // left to the caller's fix-up
      continue;
    }
    if (nonzero > 1) passes[npass++] = p;
  }
  if (npass == 0) passes[npass++] = 0;  // all keys equal: one pass yields the identity payload
  int cur = 0;
  hipLaunchKernelGGL(k_digit_bases, dim3(NB), dim3(256), 0, s, b.hist, b.bases);
  PBH_CHECK_LAUNCH();
  for (int ip = 0; ip < npass; ++ip) {
    const int shift = 8 * passes[ip];
    int st = PBH_OK;
    PBH_TIMED(NB == 8 ? kKSortScatter : kKSortScatter32, s,
              st = launch_onesweep<K, uint32_t>(ip == 0 ? first : keys[cur], ip == 0 ? nullptr : b.vals[cur],
                                                keys[cur ^ 1], b.vals[cur ^ 1], n, shift, b.bases + passes[ip] * 256,
                                                b.status, (uint32_t*)(b.status + nt * 256), b.sweep, s));
    if (st) return st;
    PBH_CHECK_LAUNCH();
    cur ^= 1;
  }
  uint32_t stuck = 0;
  PBH_CHECK_HIP(hipMemcpyAsync(&stuck, (uint32_t*)(b.status + nt * 256) + 1, 4, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  if (stuck) {
    set_error("radix sort: one-sweep look-back did not complete");
    return PBH_ERR_HIP;
  }
  *out_buf = cur;
  return PBH_OK;
}

int radix_sort_keys32_async(SortBuffers& b, int64_t n, int npass, hipStream_t s, int* out_buf, const uint32_t* in,
                            uint32_t** stuck) {
  PBH_REQUIRE(n >= 1 && n < ((int64_t)1 << 32) && npass >= 1 && npass <= 4 && in,
              "radix_sort_keys32_async: bad arguments");
  const int64_t nt = sort_tiles(n);
  uint32_t* keys[2] = {(uint32_t*)b.keys[0], (uint32_t*)b.keys[1]};
  PBH_CHECK_HIP(hipMemsetAsync(b.hist, 0, 8 * 256 * 4, s));
  hipLaunchKernelGGL(k_digit_hist<uint32_t>, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, in, n, b.hist);
  PBH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_digit_bases, dim3(4), dim3(256), 0, s, b.hist, b.bases);
  PBH_CHECK_LAUNCH();
  int cur = 0;
  for (int ip = 0; ip < npass; ++ip) {
    if (int st = launch_onesweep<uint32_t, uint32_t>(ip == 0 ? in : keys[cur], ip == 0 ? nullptr : b.vals[cur],
                                                     keys[cur ^ 1], b.vals[cur ^ 1], n, 8 * ip, b.bases + ip * 256,
                                                     b.status, (uint32_t*)(b.status + nt * 256), b.sweep, s))
      return st;
    PBH_CHECK_LAUNCH();
    cur ^= 1;
  }
  *out_buf = cur;
  *stuck = (uint32_t*)(b.status + nt * 256) + 1;
  return PBH_OK;
}

int radix_sort_keys(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf) {
  return radix_sort_impl<uint64_t>(b, n, s, out_buf);
}

namespace {
// After the passes over bytes 2..7 only: keys equal in their top 48 bits form runs still in row
// order; the head of each run orders it by the whole key (insertion sort, rows along).  Runs are
// rare and short for continuous data (48 bits resolve 2^-36 of a binade); a run longer than
// kFixCap sets *long_run and the caller sorts the column again with every byte.
constexpr int64_t kFixCap = 64;
__global__ __launch_bounds__(256) void k_fix_low16(uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                   int64_t n, uint32_t* __restrict__ long_run) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t hk = keys[i] >> 16;
    if (i > 0 && (keys[i - 1] >> 16) == hk) continue;   // not a run head
    if (i + 1 >= n || (keys[i + 1] >> 16) != hk) continue;  // alone in its top 48 bits
    int64_t j = i + 1;
    while (j < n && (keys[j] >> 16) == hk && j - i <= kFixCap) ++j;
    if (j - i > kFixCap) {
      atomicOr(long_run, 1u);
      continue;
    }
    for (int64_t a = i + 1; a < j; ++a) {  // stable insertion sort by the whole key
      const uint64_t k = keys[a];
      const uint32_t v = vals[a];
      int64_t b = a;
      while (b > i && keys[b - 1] > k) {
        keys[b] = keys[b - 1];
        vals[b] = vals[b - 1];
        --b;
      }
      keys[b] = k;
      vals[b] = v;
    }
  }
}
}  // namespace

int radix_sort_keys_top48(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf, bool* redo) {
  *redo = false;
  bool low = false;
  int st = radix_sort_impl<uint64_t>(b, n, s, out_buf, nullptr, 2, &low);
  if (st || !low) return st;
  uint32_t* flag = (uint32_t*)b.hist;  // the histogram is read back already; one word of it
  PBH_CHECK_HIP(hipMemsetAsync(flag, 0, 4, s));
  hipLaunchKernelGGL(k_fix_low16, dim3(grid_for(n, 256, 8192)), dim3(256), 0, s, b.keys[*out_buf],
                     b.vals[*out_buf], n, flag);
  PBH_CHECK_LAUNCH();
  uint32_t h = 0;
  PBH_CHECK_HIP(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  *redo = h != 0;
  return PBH_OK;
}

int radix_sort_keys32(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf, const uint32_t* in) {
  return radix_sort_impl<uint32_t>(b, n, s, out_buf, in);
}

}  // namespace pbh
