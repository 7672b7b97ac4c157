// Microbenchmark (timing only): one one-sweep radix pass (u32 key + u32 / f64 payload, 10^8
// elements) with and without the decoupled look-back, to see whether the look-back chain or
// the memory traffic bounds the pass.  Kernel body copied from probabilit_amd/csrc/pbh_sort.hip.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_onesweep.hip -o tools/gpu/mbos
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
constexpr int T = 256;
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

constexpr uint64_t kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62, kCountMask = (1ull << 62) - 1;

template <typename K, typename V, int IPTT, bool LB, int W = 1>
__global__ __launch_bounds__(T) void k_onesweep(const K* __restrict__ kin, const V* __restrict__ vin,
                                               K* __restrict__ kout, V* __restrict__ vout, int64_t n, int shift,
                                               const uint32_t* __restrict__ digit_base, uint64_t* status,
                                               uint32_t* tile_counter) {
  constexpr int IPT = IPTT;
  constexpr int TILE = T * IPTT;
  __shared__ K skeys[TILE];
  __shared__ V svals[TILE];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t dstart[256 + 8];
  __shared__ int64_t gbase[256];
  __shared__ uint32_t tile_sh;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) tile_sh = atomicAdd(tile_counter, 1u);
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
  if (tile == 0)
    __hip_atomic_store(my, kFlagInc | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    __hip_atomic_store(my, kFlagAgg | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t ex = block_exclusive_scan_256(tot, dstart, nullptr);
  uint64_t excl = 0;
  if (LB && tile > 0) {
    // windowed look-back: up to W predecessor words loaded at once, consumed in order
    int64_t tp = tile - 1;
    uint32_t spins = 0;
    while (true) {
      uint64_t sv[W];
#pragma unroll
      for (int w = 0; w < W; ++w)
        sv[w] = (tp - w >= 0) ? __hip_atomic_load(status + (tp - w) * 256 + t, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                              : 0ull;
      int used = 0;
      bool done = false;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        if (done || used != w) continue;
        const uint64_t flag = sv[w] & ~kCountMask;
        if (flag == 0) continue;  // not yet published: stop consuming here
        excl += sv[w] & kCountMask;
        ++used;
        if (flag == kFlagInc) done = true;
      }
      if (done) break;
      tp -= used;
      if (used == 0 && ++spins > (1u << 26)) {
        atomicOr(tile_counter + 1, 1u);
        break;
      }
    }
    __hip_atomic_store(my, kFlagInc | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!LB) excl = (uint64_t)tile * (TILE / 256);  // the real write layout, no dependency
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


__global__ void k_fill(uint32_t* k, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 0x9E3779B1u;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
    k[i] = h;
  }
}
__global__ void k_bases(uint32_t* b, int64_t n) { b[threadIdx.x] = (uint32_t)((n / 256) * threadIdx.x); }

template <typename V, int IPT, bool LB, int W = 1>
float run(const uint32_t* kin, const V* vin, uint32_t* kout, V* vout, int64_t n, int shift, uint32_t* bases,
          uint64_t* status, int reps) {
  const int64_t nt = (n + T * IPT - 1) / (T * IPT);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float tot = 0;
  for (int r = 0; r < reps + 1; ++r) {
    hipMemsetAsync(status, 0, (size_t)nt * 256 * 8 + 256);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_onesweep<uint32_t, V, IPT, LB, W>), dim3((unsigned)nt), dim3(T), 0, 0, kin, vin, kout, vout, n,
                       shift, bases, status, (uint32_t*)(status + nt * 256));
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    if (r) tot += ms;
  }
  return tot / reps;
}

int main() {
  const int64_t n = 100000000;
  uint32_t *k0, *k1, *bases; uint32_t *v0, *v1; double *d0, *d1; uint64_t* status;
  const int64_t slack = 1 << 22;  // the fake digit bases can run past n by a few thousand
  hipMalloc(&k0, n * 4); hipMalloc(&k1, (n + slack) * 4); hipMalloc(&v0, n * 4); hipMalloc(&v1, (n + slack) * 4);
  hipMalloc(&d0, n * 8); hipMalloc(&d1, (n + slack) * 8); hipMalloc(&bases, 1024);
  hipMalloc(&status, ((n + 4095) / 4096) * 256 * 8 + 256);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k0, n);
  hipLaunchKernelGGL(k_bases, dim3(1), dim3(256), 0, 0, bases, n);
  hipMemset(v0, 0, n * 4); hipMemset(d0, 0, n * 8);
  for (int shift : {0, 24}) {
    printf("shift %d\n", shift);
    printf("  u32/u32 IPT32 W1  %.4f ms\n", run<uint32_t, 32, true, 1>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT32 W4  %.4f ms\n", run<uint32_t, 32, true, 4>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT32 W8  %.4f ms\n", run<uint32_t, 32, true, 8>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT32 W16 %.4f ms\n", run<uint32_t, 32, true, 16>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT32 none %.4f ms\n", run<uint32_t, 32, false>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT16 W1  %.4f ms\n", run<uint32_t, 16, true, 1>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT16 W8  %.4f ms\n", run<uint32_t, 16, true, 8>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/u32 IPT16 W16 %.4f ms\n", run<uint32_t, 16, true, 16>(k0, v0, k1, v1, n, shift, bases, status, 5));
    printf("  u32/f64 IPT16 W1  %.4f ms\n", run<double, 16, true, 1>(k0, d0, k1, d1, n, shift, bases, status, 5));
    printf("  u32/f64 IPT16 W8  %.4f ms\n", run<double, 16, true, 8>(k0, d0, k1, d1, n, shift, bases, status, 5));
    printf("  u32/f64 IPT16 W16 %.4f ms\n", run<double, 16, true, 16>(k0, d0, k1, d1, n, shift, bases, status, 5));
    printf("  u32/f64 IPT16 none %.4f ms\n", run<double, 16, false>(k0, d0, k1, d1, n, shift, bases, status, 5));
  }
  return 0;
}
