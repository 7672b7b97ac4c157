// Microbenchmark of the fp64 building blocks of ndtri on gfx950 (10^8 elements per launch):
// centre-only and tail-only ndtri, log, division, sqrt, and a Horner chain, each writing one
// double per element.  Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I ../probabilit_amd/csrc
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "pbh_special.h"

using namespace pbh;

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, int64_t n, double lo, double hi) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    // a cheap scrambled q in [lo, hi)
    uint32_t h = (uint32_t)i * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    const double q = lo + (hi - lo) * ((double)h * 2.3283064365386963e-10);
    double x;
    if (MODE == 0) x = sf::ndtri(q);
    else if (MODE == 1) x = log(q);
    else if (MODE == 2) x = 1.0 / q;
    else if (MODE == 3) x = sqrt(q);
    else if (MODE == 4) {
      double a = q;
#pragma unroll
      for (int j = 0; j < 16; ++j) a = a * q + 0.37;
      x = a;
    } else x = q;
    out[i] = x;
  }
}

template <int MODE>
float run(double* out, int64_t n, double lo, double hi, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, n, lo, hi);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, n, lo, hi);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int64_t n = 100000000;
  double* out;
  hipMalloc(&out, n * 8);
  for (int grid : {4096, 16384, 390625}) {
    printf("grid %d\n", grid);
    printf("  store only        %.3f ms\n", run<9>(out, n, 0.2, 0.8, grid));
    printf("  ndtri centre only %.3f ms\n", run<0>(out, n, 0.2, 0.8, grid));
    printf("  ndtri tail only   %.3f ms\n", run<0>(out, n, 1e-6, 0.13, grid));
    printf("  ndtri uniform     %.3f ms\n", run<0>(out, n, 1e-9, 1.0 - 1e-9, grid));
    printf("  log               %.3f ms\n", run<1>(out, n, 1e-6, 0.13, grid));
    printf("  1/q               %.3f ms\n", run<2>(out, n, 1e-6, 0.13, grid));
    printf("  sqrt              %.3f ms\n", run<3>(out, n, 1e-6, 0.13, grid));
    printf("  horner16 (mul+add) %.3f ms\n", run<4>(out, n, 1e-6, 0.13, grid));
  }
  hipFree(out);
  return 0;
}
