// Microbenchmark of the tail-compacted norm ppf sweep (k_ppf_c<norm>, pbh_ppf.hip) against
// variants of its tile structure, 10^8 random-order quantiles per launch, 16 B per draw:
//   base    : the production structure (centre results and the tail queue in LDS, results
//             copied out of LDS after the drain, two barriers per tile)
//   direct  : centre results stored straight from registers, tail results stored at their
//             positions by the draining lanes (no result buffer in LDS)
//   prefetch: direct + the next tile's quantiles loaded before the tail drain
// with items per thread IPT and a waves-per-SIMD cap W (0: none), plus reference points (copy
// through the same tiles, centre formula for every item).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I ../probabilit_amd/csrc -I ../include
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "pbh_ppf_core.h"

using namespace pbh;

namespace {

constexpr int kB = 256;

template <int IPT>
struct Queue {
  double arg[kB * IPT];
  uint16_t pos[kB * IPT];
  int count;
};

template <int W>
struct Occ;

PBH_DI double centre(double q) { return ppf_one<PBH_DIST_NORM, 1>(q, 0.0, 1.0, 0.0, PoissonTable{}); }
PBH_DI double tail(double q) { return ppf_one<PBH_DIST_NORM, 2>(q, 0.0, 1.0, 0.0, PoissonTable{}); }

// ndtri's tail with the math library's log (before sf::log_tab), for the A/B
PBH_DI double tail_libm(double y0) {
  const double P1[9] = {4.05544892305962419923e0, 3.15251094599893866154e1, 5.71628192246421288162e1,
                        4.40805073893200834700e1, 1.46849561928858024014e1, 2.18663306850790267539e0,
                        -1.40256079171354495875e-1, -3.50424626827848203418e-2, -8.57456785154685413611e-4};
  const double Q1[8] = {1.57799883256466749731e1, 4.53907635128879210584e1, 4.13172038254672030440e1,
                        1.50425385692907503408e1, 2.50464946208309415979e0, -1.42182922854787788574e-1,
                        -3.80806407691578277194e-2, -9.33259480895457427372e-4};
  const double P2[9] = {3.23774891776946035970e0, 6.91522889068984211695e0, 3.93881025292474443415e0,
                        1.33303460815807542389e0, 2.01485389549179081538e-1, 1.23716634817820021358e-2,
                        3.01581553508235416007e-4, 2.65806974686737550832e-6, 6.23974539184983293730e-9};
  const double Q2[8] = {6.02427039364742014255e0, 3.67983563856160859403e0, 1.37702099489081330271e0,
                        2.16236993594496635890e-1, 1.34204006088543189037e-2, 3.28014464682127739104e-4,
                        2.89247864745380683936e-6, 6.79019408009981274425e-9};
  bool negate = true;
  double y = y0;
  if (y > (1.0 - sf::kNdtriExpM2)) {
    y = 1.0 - y;
    negate = false;
  }
  double x = sqrt(-2.0 * log(y));
  const double x0 = x - log(x) / x;
  const double z = 1.0 / x;
  double x1;
  if (x < 8.0)
    x1 = z * sf::polevl(z, P1, 8) / sf::p1evl(z, Q1, 8);
  else
    x1 = z * sf::polevl(z, P2, 8) / sf::p1evl(z, Q2, 8);
  x = x0 - x1;
  return negate ? -x : x;
}

__global__ void k_cmp(const double* a, const double* b, int64_t n, unsigned long long* bad) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    if (__builtin_bit_cast(uint64_t, a[i]) != __builtin_bit_cast(uint64_t, b[i])) atomicAdd(bad, 1ull);
}

#define KATTR(W) __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(W == 0 ? 1 : W)))

// MODE 0 base, 1 direct, 2 prefetch, 3 copy, 4 centre for all, 5 base with the libm-log tail
template <int MODE, int IPT, int W>
__global__ KATTR(W) void k_norm(const double* __restrict__ q, int64_t n, double* __restrict__ out) {
  constexpr int kT = kB * IPT;
  __shared__ Queue<IPT> tq;
  __shared__ double res[(MODE == 0 || MODE == 5 || MODE == 6) ? kT : 1];
  const int64_t stride = (int64_t)gridDim.x * kT;
  int64_t base = (int64_t)blockIdx.x * kT;
  double qn[IPT];
  if (MODE == 2) {
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + j * kB + threadIdx.x;
      qn[j] = i < n ? q[i] : 0.5;
    }
  }
  for (; base < n; base += stride) {
    if (MODE <= 2 || MODE >= 5) {
      if (threadIdx.x == 0) tq.count = 0;
      __syncthreads();
    }
    double qv[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + j * kB + threadIdx.x;
      if (MODE == 2)
        qv[j] = qn[j];
      else
        qv[j] = i < n ? q[i] : 0.5;
    }
    if (MODE == 3 || MODE == 4) {
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const int64_t i = base + j * kB + threadIdx.x;
        if (i < n) out[i] = MODE == 3 ? qv[j] : centre(qv[j]);
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int p = j * kB + threadIdx.x;
      const int64_t i = base + p;
      const bool valid = i < n;
      const bool tl = valid && sf::ndtri_takes_tail(qv[j]);
      if (valid && !tl) {
        const double x = centre(qv[j]);
        if (MODE == 0 || MODE == 5 || MODE == 6)
          res[p] = x;
        else
          out[i] = x;
      }
      tail_push(tq, tl, qv[j], p);
    }
    if (MODE == 2) {
      const int64_t nb = base + stride;
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const int64_t i = nb + j * kB + threadIdx.x;
        qn[j] = i < n ? q[i] : 0.5;
      }
    }
    __syncthreads();
    const int T = tq.count;
    if (MODE == 6) {  // two tail items per lane per round: two independent chains
      for (int t = threadIdx.x; t < T; t += 2 * kB) {
        const bool two = t + kB < T;
        const double a0 = tq.arg[t], a1 = two ? tq.arg[t + kB] : 0.01;
        const double x0 = tail(a0), x1 = tail(a1);
        res[tq.pos[t]] = x0;
        if (two) res[tq.pos[t + kB]] = x1;
      }
    } else {
      for (int t = threadIdx.x; t < T; t += kB) {
        const int p = tq.pos[t];
        const double x = MODE == 5 ? tail_libm(tq.arg[t]) : tail(tq.arg[t]);
        if (MODE == 0 || MODE == 5 || MODE == 6)
          res[p] = x;
        else
          out[base + p] = x;
      }
    }
    __syncthreads();
    if (MODE == 0 || MODE == 5 || MODE == 6) {
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const int p = j * kB + threadIdx.x;
        const int64_t i = base + p;
        if (i < n) out[i] = res[p];
      }
    }
  }
}

// the production k_ppf_c<norm> body (pbh_ppf.hip ppf_compacted) with its Params / flag arguments;
// FLAG = false drops the per-item non-finite flag
// VAR 0: per-item Params::at; 1: scalars in registers (runtime loc / scale); 2: scalars, no
// cond0 / q edge checks (the centre formula times scale plus loc); 3: compile-time loc 0, scale 1
template <bool FLAG, int VAR = 0>
__global__ __launch_bounds__(kB) __attribute__((amdgpu_waves_per_eu(4))) void k_prod(const double* __restrict__ q,
                                                                                     int64_t n, Params prm_in,
                                                                                     PoissonTable pt,
                                                                                     double* __restrict__ out,
                                                                                     int32_t* flag) {
  Params prm = prm_in;
  if (VAR >= 1) prm.ptr[0] = prm.ptr[1] = prm.ptr[2] = nullptr;
  if (VAR == 3) {
    prm.val[0] = 0.0;
    prm.val[1] = 1.0;
  }
  __shared__ TailQueue tq;
  __shared__ double res[kCTile];
  for (int64_t base = (int64_t)blockIdx.x * kCTile; base < n; base += (int64_t)gridDim.x * kCTile) {
    if (threadIdx.x == 0) tq.count = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kB + threadIdx.x;
      const int64_t i = base + p;
      const bool valid = i < n;
      const double qv = valid ? q[i] : 0.5;
      const bool tail = valid && sf::ndtri_takes_tail(qv);
      if (valid && !tail) {
        if (VAR == 2)
          res[p] = sf::ndtri_centre(qv) * prm.val[1] + prm.val[0];
        else
          res[p] = ppf_one<PBH_DIST_NORM, 1>(qv, prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
      }
      tail_push(tq, tail, qv, p);
    }
    __syncthreads();
    const int T = tq.count;
    for (int t = threadIdx.x; t < T; t += kB) {
      const int p = tq.pos[t];
      const int64_t i = base + p;
      if (VAR == 2)
        res[p] = sf::ndtri_tail(tq.arg[t]) * prm.val[1] + prm.val[0];
      else
        res[p] = ppf_one<PBH_DIST_NORM, 2>(tq.arg[t], prm.at(0, i), prm.at(1, i), prm.at(2, i), pt);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCIpt; ++j) {
      const int p = j * kB + threadIdx.x;
      const int64_t i = base + p;
      const double x = i < n ? res[p] : 0.0;
      if (i < n) out[i] = x;
      if (FLAG) flag_nonfinite(flag, !isfinite(x));
    }
  }
}

// wave-private tiles: each wave owns 64 x IPT items, queues its tail items in its own LDS slice
// and drains them itself (no block barrier); centre results stored from registers; the next
// tile's quantiles are loaded before the drain when PF.
template <int IPT, int W, bool PF>
__global__ KATTR(W) void k_norm_wave(const double* __restrict__ q, int64_t n, double* __restrict__ out) {
  constexpr int kWT = 64 * IPT;
  __shared__ double qarg[kB / 64][kWT];
  __shared__ uint16_t qpos[kB / 64][kWT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* const arg = qarg[wv];
  uint16_t* const pos = qpos[wv];
  const int64_t nw = (int64_t)gridDim.x * (kB / 64);
  const int64_t stride = nw * kWT;
  int64_t base = ((int64_t)blockIdx.x * (kB / 64) + wv) * kWT;
  double qn[IPT];
  if (PF) {
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + j * 64 + lane;
      qn[j] = i < n ? q[i] : 0.5;
    }
  }
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (; base < n; base += stride) {
    double qv[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int64_t i = base + j * 64 + lane;
      qv[j] = PF ? qn[j] : (i < n ? q[i] : 0.5);
    }
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const int p = j * 64 + lane;
      const int64_t i = base + p;
      const bool valid = i < n;
      const bool tl = valid && sf::ndtri_takes_tail(qv[j]);
      if (valid && !tl) out[i] = centre(qv[j]);
      const uint64_t m = __ballot(tl);
      if (tl) {
        const int slot = cnt + (int)__popcll(m & lt);
        arg[slot] = qv[j];
        pos[slot] = (uint16_t)p;
      }
      cnt += (int)__popcll(m);
    }
    if (PF) {
      const int64_t nb = base + stride;
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const int64_t i = nb + j * 64 + lane;
        qn[j] = i < n ? q[i] : 0.5;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = lane; t < cnt; t += 64) out[base + pos[t]] = tail(arg[t]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <int IPT, int W, bool PF>
void run_wave(const char* name, const double* q, double* out, const double* ref, int64_t n, unsigned long long* bad,
              int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipMemset(out, 0, n * 8);
  hipLaunchKernelGGL((k_norm_wave<IPT, W, PF>), dim3(grid), dim3(kB), 0, 0, q, n, out);
  hipMemset(bad, 0, 8);
  hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, out, ref, n, bad);
  unsigned long long nb = 0;
  hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
  hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((k_norm_wave<IPT, W, PF>), dim3(grid), dim3(kB), 0, 0, q, n, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  printf("%-28s grid %7d  %.4f ms  %7.1f GB/s  differ from the libm-log ndtri: %llu\n", name, grid, ms, 16e-6 * n / ms, nb);
}

__global__ void k_fill(double* q, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    q[i] = ((double)(h >> 11) + 0.5) * 0x1.0p-53;
  }
}

__global__ void k_ref(const double* q, int64_t n, double* out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = sf::ndtri_takes_tail(q[i]) ? tail_libm(q[i]) : centre(q[i]);
}


}  // namespace

template <int MODE, int IPT, int W>
void run(const char* name, const double* q, double* out, const double* ref, int64_t n, unsigned long long* bad,
         int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipMemset(out, 0, n * 8);
  hipLaunchKernelGGL((k_norm<MODE, IPT, W>), dim3(grid), dim3(kB), 0, 0, q, n, out);
  hipMemset(bad, 0, 8);
  hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, out, ref, n, bad);
  unsigned long long nb = 0;
  hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
  hipEventRecord(a);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((k_norm<MODE, IPT, W>), dim3(grid), dim3(kB), 0, 0, q, n, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  printf("%-28s grid %7d  %.4f ms  %7.1f GB/s  differ from the libm-log ndtri: %llu\n", name, grid, ms, 16e-6 * n / ms,
         (MODE == 3 || MODE == 4) ? 0 : nb);
}

int main() {
  const int64_t n = 100000000;
  double *q, *out, *ref;
  unsigned long long* bad;
  hipMalloc(&q, n * 8);
  hipMalloc(&out, n * 8);
  hipMalloc(&ref, n * 8);
  hipMalloc(&bad, 8);
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, q, n);
  hipLaunchKernelGGL(k_ref, dim3(8192), dim3(256), 0, 0, q, n, ref);
  hipDeviceSynchronize();
  int32_t* flag;
  hipMalloc(&flag, 4);
  hipMemset(flag, 0, 4);
  Params prm{};
  prm.val[0] = 0.0;
  prm.val[1] = 1.0;
  for (int rep = 0; rep < 2; ++rep) {
    for (int g : {2048, 8192}) {
      run<0, 8, 4>("base ipt8 w4 (replica)", q, out, ref, n, bad, g);
      for (int f = 0; f < 6; ++f) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        for (int r = 0; r < 10; ++r) {
          switch (f) {
            case 0: hipLaunchKernelGGL((k_prod<true, 0>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
            case 1: hipLaunchKernelGGL((k_prod<true, 1>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
            case 2: hipLaunchKernelGGL((k_prod<false, 1>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
            case 3: hipLaunchKernelGGL((k_prod<true, 2>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
            case 4: hipLaunchKernelGGL((k_prod<false, 2>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
            default: hipLaunchKernelGGL((k_prod<false, 3>), dim3(g), dim3(kB), 0, 0, q, n, prm, PoissonTable{}, out, flag); break;
          }
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const char* nm[6] = {"prod: at(), flag", "prod: scalars, flag", "prod: scalars", "prod: bare ndtri, flag",
                             "prod: bare ndtri", "prod: const 0/1"};
        printf("%-28s grid %7d  %.4f ms\n", nm[f], g, ms / 10);
      }
    }
  }
  return 0;
}
