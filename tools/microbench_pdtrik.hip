// Microbenchmark: latency of the poisson ppf's rare lanes (scipy's pdtrik search restated in
// pbh_cdflib.h), the cost a wave pays when one of its lanes falls in a window above a CDF value.
//   capped   one wave, every lane in a window, through poisson_rare (the product's call, under
//            the ppf kernels' 4-waves-per-SIMD register cap)
//   free     the same without the cap
//   one      a single lane (the common case: one window lane in a wave)
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I probabilit_amd/csrc -I include \
//         tools/microbench_pdtrik.hip -o tools/gpu/mbpdtrik && tools/gpu/mbpdtrik
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "pbh_ppf_core.h"

using namespace pbh;

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_capped(const double* q, double mu,
                                                                                      double* out, int lanes) {
  const int i = threadIdx.x;
  if (i < lanes) out[i] = poisson_rare(q[i], mu, -1.0);
}
__global__ __launch_bounds__(64) void k_free(const double* q, double mu, double* out, int lanes) {
  const int i = threadIdx.x;
  if (i < lanes) out[i] = cdf::poisson_ppf_scipy(q[i], mu);
}

int main() {
  const double mus[3] = {4.0, 30.0, 250.0};
  double *q, *out;
  hipMalloc(&q, 64 * sizeof(double));
  hipMalloc(&out, 64 * sizeof(double));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("{");
  for (int m = 0; m < 3; ++m) {
    const double mu = mus[m];
    double hq[64];
    for (int i = 0; i < 64; ++i) {  // just above pdtr(k - 1) for k around mu
      const double k = floor(mu) + (i % 5) - 2.0;
      hq[i] = sf::pdtr(k - 1.0, mu) * (1.0 + 1e-13 * (1 + i));
    }
    hipMemcpy(q, hq, sizeof(hq), hipMemcpyHostToDevice);
    for (int v = 0; v < 3; ++v) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(a, 0);
        if (v == 0) hipLaunchKernelGGL(k_capped, dim3(1), dim3(64), 0, 0, q, mu, out, 64);
        if (v == 1) hipLaunchKernelGGL(k_free, dim3(1), dim3(64), 0, 0, q, mu, out, 64);
        if (v == 2) hipLaunchKernelGGL(k_capped, dim3(1), dim3(64), 0, 0, q, mu, out, 1);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("%s\"mu%g_%s_us\": %.1f", (m || v) ? ", " : "", mu, v == 0 ? "capped" : v == 1 ? "free" : "one",
             best * 1000.0f);
    }
  }
  printf("}\n");
  return 0;
}
