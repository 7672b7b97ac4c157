// Microbenchmark: where does k_perm_scores spend its time?  Variants over N = 1e8 rows:
//   full      S[r] = ndtri((pi(r) + 1) / (n + 1))            (the production kernel's work)
//   perm      S[r] = (pi(r) + 1) / (n + 1)                   (Feistel permutation only)
//   ndtri     S[r] = ndtri((r + 1) / (n + 1))                (ndtri, no divergence)
//   ndtri_rnd S[r] = ndtri(hash(r) / (n + 1))                (ndtri, divergent like `full`)
//   write     S[r] = r                                        (store bandwidth)
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I probabilit_amd/csrc -I include \
//         tools/microbench_scores.hip -o tools/gpu/mbscores && tools/gpu/mbscores
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "pbh_rng.h"
#include "pbh_special.h"

using namespace pbh;

template <int V>
__global__ __launch_bounds__(256) void k_var(uint64_t seed, int64_t n, double* __restrict__ S) {
  Philox ph(seed);
  FeistelPerm fp(ph, (uint64_t)n, 3u);
  const double np1 = (double)(n + 1);
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    double v;
    if (V == 0) v = sf::ndtri((double)(fp((uint64_t)r) + 1) / np1);
    if (V == 1) v = (double)(fp((uint64_t)r) + 1) / np1;
    if (V == 2) v = sf::ndtri((double)(r + 1) / np1);
    if (V == 3) v = sf::ndtri((double)((mix32((uint32_t)r) % (uint32_t)n) + 1) / np1);
    if (V == 4) v = (double)r;
    S[r] = v;
  }
}

template <int V>
float run(int64_t n, double* S, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(k_var<V>, dim3(grid), dim3(256), 0, 0, 7ull, n, S);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  const int64_t n = 100000000;
  double* S;
  if (hipMalloc(&S, n * 8) != hipSuccess) return 1;
  for (int grid : {4096, 16384, 65536}) {
    printf("{\"grid\": %d, \"full\": %.3f, \"perm\": %.3f, \"ndtri\": %.3f, \"ndtri_rnd\": %.3f, \"write\": %.3f}\n",
           grid, run<0>(n, S, grid), run<1>(n, S, grid), run<2>(n, S, grid), run<3>(n, S, grid),
           run<4>(n, S, grid));
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
