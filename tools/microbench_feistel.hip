// Microbenchmark: the van der Waerden scores kernel (k_perm_scores) with candidate LHS
// permutations, N = 1e8 rows, best of 5 launches:
//   perm_<P>   S[r] = (pi(r) + 1) / (n + 1)            (the permutation alone, 8 chains a thread)
//   full_<P>   S[r] = ndtri((pi(r) + 1) / (n + 1))     (the production structure: tail compaction)
//   full_hash  the same with pi(r) replaced by a one-multiply hash (ndtri + compaction alone)
//   write      S[r] = r
// P: cur = FeistelPerm (pbh_rng.h: lowbias32 rounds, 32-bit multiplies), f24 = FeistelPerm's
// round function on 24-bit multiplies (v_mul_u32_u24 / v_mul_hi_u32_u24, full rate).
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I probabilit_amd/csrc -I include \
//         tools/microbench_feistel.hip -o gpurun_out/mbfeistel && gpurun_out/mbfeistel
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "pbh_ppf_core.h"
#include "pbh_rng.h"
#include "pbh_special.h"

using namespace pbh;

constexpr int kB = 256;

struct PermCur {
  FeistelPerm fp;
  __device__ PermCur(const Philox& ph, uint64_t n, uint32_t col) : fp(ph, n, col) {}
  __device__ uint64_t rt(uint64_t x) const { return fp.round_trip(x); }
  __device__ uint64_t n() const { return fp.n; }
};

// round function on 24-bit multiplies: h = (v ^ k0) * M1 (low 32), h ^= h >> 15, h = (h ^ k1) * M2
// (low 24 bits of the operand), h ^= h >> 16, then the top 24 bits scaled to [0, m) by one
// v_mul_hi_u32_u24 against m << 8 (m < 2^16 in the 32-bit domain)
struct PermF24 {
  FeistelPerm fp;
  uint32_t k0[4], k1[4], a8, b8;
  __device__ PermF24(const Philox& ph, uint64_t n, uint32_t col) : fp(ph, n, col) {
    for (int i = 0; i < 4; ++i) {
      k0[i] = fp.rk[i] & 0xFFFFFFu;
      k1[i] = (fp.rk[i] >> 8) & 0xFFFFFFu;
    }
    a8 = fp.A << 8;
    b8 = fp.B << 8;
  }
  static __device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return __umul24(a, b); }
  static __device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
  }
  __device__ __forceinline__ uint32_t F(uint32_t v, int i, uint32_t m8) const {
    uint32_t h = mul24(v ^ k0[i], 0xE5B4A3u);
    h ^= h >> 15;
    h = mul24(h ^ k1[i], 0x9E3779u);
    h ^= h >> 16;
    return mulhi24(h >> 8, m8);
  }
  __device__ uint64_t rt(uint64_t x) const {
    uint32_t L, R;
    fp.split(x, L, R);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i & 1) {
        const uint32_t h = F(L, i, b8);
        R = R + h >= fp.B ? R + h - fp.B : R + h;
      } else {
        const uint32_t h = F(R, i, a8);
        L = L + h >= fp.A ? L + h - fp.A : L + h;
      }
    }
    return fp.join(L, R);
  }
  __device__ uint64_t n() const { return fp.n; }
};

template <class P>
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(4))) void k_perm(uint64_t seed, int64_t n,
                                                                                      double* __restrict__ S) {
  Philox ph(seed);
  P pm(ph, (uint64_t)n, 3u);
  const double np1 = (double)(n + 1);
  for (int64_t base = (int64_t)blockIdx.x * kCTile; base < n; base += (int64_t)gridDim.x * kCTile) {
    uint64_t tt[kCIpt];
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int64_t i = base + j * kB + threadIdx.x;
      tt[j] = i < n ? pm.rt((uint64_t)i) : 0;
    }
#pragma unroll
    for (int j = 0; j < kCIpt; ++j)
      while (tt[j] >= (uint64_t)n) tt[j] = pm.rt(tt[j]);
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int64_t i = base + j * kB + threadIdx.x;
      if (i < n) S[i] = (double)(tt[j] + 1) / np1;
    }
  }
}

struct PermHash {  // not a permutation: ndtri's cost with a one-multiply rank
  __device__ PermHash(const Philox&, uint64_t n, uint32_t) : nn(n) {}
  uint64_t nn;
  __device__ uint64_t rt(uint64_t x) const {
    return (uint64_t)(((uint64_t)(uint32_t)(x * 2654435761u) * nn) >> 32);
  }
  __device__ uint64_t n() const { return nn; }
};

template <class P>
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(4))) void k_full(uint64_t seed, int64_t n,
                                                                                      double* __restrict__ S) {
  __shared__ TailQueue tq;
  __shared__ double res[kCTile];
  Philox ph(seed);
  P pm(ph, (uint64_t)n, 3u);
  const double np1 = (double)(n + 1);
  for (int64_t base = (int64_t)blockIdx.x * kCTile; base < n; base += (int64_t)gridDim.x * kCTile) {
    if (threadIdx.x == 0) tq.count = 0;
    __syncthreads();
    uint64_t tt[kCIpt];
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int64_t i = base + j * kB + threadIdx.x;
      tt[j] = i < n ? pm.rt((uint64_t)i) : 0;
    }
#pragma unroll
    for (int j = 0; j < kCIpt; ++j)
      while (tt[j] >= (uint64_t)n) tt[j] = pm.rt(tt[j]);
#pragma unroll 2
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kB + threadIdx.x;
      const bool valid = base + p < n;
      const double y = valid ? (double)(tt[j] + 1) / np1 : 0.5;
      const bool tail = valid && sf::ndtri_takes_tail(y);
      if (valid && !tail) res[p] = sf::ndtri_centre(y);
      tail_push(tq, tail, y, p);
    }
    __syncthreads();
    const int T = tq.count;
    for (int t = threadIdx.x; t < T; t += kB) res[tq.pos[t]] = sf::ndtri_tail(tq.arg[t]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kB + threadIdx.x;
      if (base + p < n) S[base + p] = res[p];
    }
  }
}

// ndtri's branches alone over y = (hash(r) + 1) / (n + 1): MODE 1 every element through ndtri_centre
// (y folded into the centre), MODE 2 every element through ndtri_tail (y folded into the tail)
template <int MODE>
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(4))) void k_branch(int64_t n,
                                                                                        double* __restrict__ S) {
  const double np1 = (double)(n + 1);
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < n; r += (int64_t)gridDim.x * kB) {
    const double u = (double)((((uint64_t)(uint32_t)(r * 2654435761u)) * (uint64_t)n) >> 32) / np1;
    double v;
    if (MODE == 1) v = sf::ndtri_centre(0.1354 + 0.729 * u);
    if (MODE == 2) v = sf::ndtri_tail(u < 0.5 ? u * 0.27 : 1.0 - (1.0 - u) * 0.27);
    S[r] = v;
  }
}

__global__ void k_write(int64_t n, double* __restrict__ S) {
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < n; r += (int64_t)gridDim.x * kB) S[r] = (double)r;
}

// distinct strata, checked on the device: every stratum hit once
__global__ void k_hits(const double* __restrict__ S, int64_t n, unsigned* hits) {
  const double np1 = (double)(n + 1);
  for (int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x; r < n; r += (int64_t)gridDim.x * kB) {
    const int64_t t = (int64_t)__builtin_rint(S[r] * np1) - 1;
    if (t >= 0 && t < n) atomicAdd(&hits[t], 1u);
  }
}

template <class F>
float best(F&& launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float m = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    m = ms < m ? ms : m;
  }
  return m;
}

int main() {
  const int64_t n = 100000000;
  double* S;
  unsigned* hits;
  if (hipMalloc(&S, n * 8) != hipSuccess || hipMalloc(&hits, n * 4) != hipSuccess) return 1;
  const unsigned grid = 256 * 8;
  auto bad_strata = [&]() {
    hipMemset(hits, 0, n * 4);
    hipLaunchKernelGGL(k_hits, dim3(8192), dim3(kB), 0, 0, S, n, hits);
    unsigned* h = new unsigned[n];
    hipMemcpy(h, hits, n * 4, hipMemcpyDeviceToHost);
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += h[i] != 1;
    delete[] h;
    return bad;
  };
  const float pc = best([&] { hipLaunchKernelGGL(k_perm<PermCur>, dim3(grid), dim3(kB), 0, 0, 7ull, n, S); });
  const int64_t bc = bad_strata();
  const float p24 = best([&] { hipLaunchKernelGGL(k_perm<PermF24>, dim3(grid), dim3(kB), 0, 0, 7ull, n, S); });
  const int64_t b24 = bad_strata();
  const float fc = best([&] { hipLaunchKernelGGL(k_full<PermCur>, dim3(grid), dim3(kB), 0, 0, 7ull, n, S); });
  const float f24 = best([&] { hipLaunchKernelGGL(k_full<PermF24>, dim3(grid), dim3(kB), 0, 0, 7ull, n, S); });
  const float fh = best([&] { hipLaunchKernelGGL(k_full<PermHash>, dim3(grid), dim3(kB), 0, 0, 7ull, n, S); });
  const float w = best([&] { hipLaunchKernelGGL(k_write, dim3(8192), dim3(kB), 0, 0, n, S); });
  const float brc = best([&] { hipLaunchKernelGGL(k_branch<1>, dim3(grid * 8), dim3(kB), 0, 0, n, S); });
  const float brt = best([&] { hipLaunchKernelGGL(k_branch<2>, dim3(grid * 8), dim3(kB), 0, 0, n, S); });
  printf("{\"centre_all\": %.4f, \"tail_all\": %.4f}\n", brc, brt);
  printf("{\"n\": %lld, \"perm_cur\": %.4f, \"perm_f24\": %.4f, \"full_cur\": %.4f, \"full_f24\": %.4f, "
         "\"full_hash\": %.4f, \"write\": %.4f, \"bad_strata_cur\": %lld, \"bad_strata_f24\": %lld}\n",
         (long long)n, pc, p24, fc, f24, fh, w, (long long)bc, (long long)b24);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
