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
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    K k = keys[i];
#pragma unroll
    for (int p = 0; p < NB; ++p) atomicAdd(&h[p][(k >> (8 * p)) & 255u], 1u);
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

int exclusive_scan_u32(uint32_t* a, int64_t m, uint32_t* partials, hipStream_t s) {
  int64_t np = scan_partials_count(m);
  PBH_TIMED(kKScan, s, hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)np), dim3(256), 0, s, a, m, partials);
            hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(256), 0, s, partials, np);
            hipLaunchKernelGGL(k_scan_down, dim3((unsigned)np), dim3(256), 0, s, a, m, partials));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

// ------------------------------------------------------------------ stable scatter
template <typename K>
__global__ __launch_bounds__(T) void k_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                              K* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n,
                                              int shift, const uint32_t* __restrict__ offsets, int64_t ntiles) {
  __shared__ K skeys[TILE];
  __shared__ uint32_t svals[TILE];
  __shared__ uint32_t run[256];
  __shared__ uint32_t chunk[2][4][256];  // double-buffered by item parity
  __shared__ uint32_t dstart[256 + 8];
  __shared__ uint32_t gbase[256];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * TILE;
  const uint64_t lanemask_lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  K key[IPT];
  uint32_t val[IPT];
  uint32_t rank[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    int64_t i = base + j * T + t;
    bool valid = i < n;
    key[j] = valid ? kin[i] : (K)0;
    val[j] = valid ? (vin ? vin[i] : (uint32_t)i) : 0u;
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
      svals[lp] = val[j];
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

}  // namespace

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
}

template <typename K>
int radix_sort_impl(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf) {
  constexpr int NB = sizeof(K);
  PBH_REQUIRE(n >= 1 && n < ((int64_t)1 << 32), "radix sort: n out of range");
  const int64_t nt = sort_tiles(n);
  K* keys[2] = {(K*)b.keys[0], (K*)b.keys[1]};
  // which byte positions vary?
  PBH_CHECK_HIP(hipMemsetAsync(b.hist, 0, 8 * 256 * 4, s));
  PBH_TIMED(NB == 8 ? kKSortDigitHist : kKSortDigitHist32, s,
            hipLaunchKernelGGL(k_digit_hist<K>, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, keys[0], n, b.hist));
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipMemcpyAsync(b.hist_host, b.hist, NB * 256 * 4, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  int passes[8], npass = 0;
  for (int p = 0; p < NB; ++p) {
    int nonzero = 0;
    for (int d = 0; d < 256; ++d) nonzero += b.hist_host[p * 256 + d] != 0;
    if (nonzero > 1) passes[npass++] = p;
  }
  if (npass == 0) passes[npass++] = 0;  // all keys equal: one pass yields the identity payload
  int cur = 0;
  for (int ip = 0; ip < npass; ++ip) {
    const int shift = 8 * passes[ip];
    PBH_TIMED(NB == 8 ? kKSortUpsweep : kKSortUpsweep32, s,
              hipLaunchKernelGGL(k_upsweep<K>, dim3((unsigned)nt), dim3(T), 0, s, keys[cur], n, shift, b.counts, nt));
    PBH_CHECK_LAUNCH();
    int st = exclusive_scan_u32(b.counts, 256 * nt, b.partials, s);
    if (st != PBH_OK) return st;
    PBH_TIMED(NB == 8 ? kKSortScatter : kKSortScatter32, s,
              hipLaunchKernelGGL(k_scatter<K>, dim3((unsigned)nt), dim3(T), 0, s, keys[cur],
                                 ip == 0 ? nullptr : b.vals[cur], keys[cur ^ 1], b.vals[cur ^ 1], n, shift, b.counts,
                                 nt));
    PBH_CHECK_LAUNCH();
    cur ^= 1;
  }
  *out_buf = cur;
  return PBH_OK;
}

int radix_sort_keys(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf) {
  return radix_sort_impl<uint64_t>(b, n, s, out_buf);
}

int radix_sort_keys32(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf) {
  return radix_sort_impl<uint32_t>(b, n, s, out_buf);
}

}  // namespace pbh
