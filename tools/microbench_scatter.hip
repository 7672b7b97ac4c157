// Microbenchmark: cost of a permutation scatter y[dst(i)] = src[i] (8-byte elements) on
// MI355X as a function of the destination footprint that is live at one time.
//
// This decides the design of the Iman-Conover step-4 write (Y[row] = sorted_x[rank - 1]):
// a plain scatter over the whole column, or a bucket pass followed by a scatter whose live
// footprint fits the Infinity Cache (256 MiB) or one XCD's L2 (4 MiB).
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_scatter.hip -o /tmp/mbs && /tmp/mbs
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// destination of staging element i: a bijection inside its region of 2^rlog rows
__device__ __forceinline__ int64_t dst_of(int64_t i, int rlog) {
  const int64_t mask = ((int64_t)1 << rlog) - 1;
  const uint64_t within = (uint64_t)(i & mask);
  return (i & ~mask) | (int64_t)((within * 0x2545F4914F6CDD1Dull) & (uint64_t)mask);  // odd multiplier
}

// plain: blocks sweep the staging order together (live footprint ~ the region size)
__global__ __launch_bounds__(256) void k_plain(const double* __restrict__ src, double* __restrict__ y, int64_t n,
                                               int rlog) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    y[dst_of(i, rlog)] = src[i];
}

// xcd: blocks b, b+8, ... (one XCD under round-robin placement) sweep their own eighth
__global__ __launch_bounds__(256) void k_xcd(const double* __restrict__ src, double* __restrict__ y, int64_t n,
                                             int rlog) {
  const int x = blockIdx.x & 7;
  const int64_t per = (n + 7) / 8;
  const int64_t lo = x * per, hi = (lo + per) < n ? (lo + per) : n;
  const int64_t nb = gridDim.x / 8;
  for (int64_t i = lo + (int64_t)(blockIdx.x >> 3) * 256 + threadIdx.x; i < hi; i += nb * 256)
    y[dst_of(i, rlog)] = src[i];
}

__global__ __launch_bounds__(256) void k_copy(const double* __restrict__ src, double* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = src[i];
}

int main() {
  const int64_t n = (int64_t)1 << 27;  // 134M doubles = 1 GiB per buffer
  double *src, *y;
  CHECK(hipMalloc(&src, n * 8));
  CHECK(hipMalloc(&y, n * 8));
  CHECK(hipMemset(src, 0, n * 8));
  CHECK(hipMemset(y, 0, n * 8));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int grids[] = {2048, 8192};
  printf("{\n");
  // copy reference
  {
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, src, y, n);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    printf("  \"copy\": {\"ms\": %.4f, \"GBps\": %.1f},\n", best, 16.0 * n / (best * 1e-3) / 1e9);
  }
  const int rlogs[] = {17, 18, 19, 21, 23, 24, 25, 27};
  for (int g : grids)
    for (int mode = 0; mode < 2; ++mode)
      for (int rl : rlogs) {
        float best = 1e30f;
        for (int r = 0; r < 4; ++r) {
          CHECK(hipEventRecord(a));
          if (mode == 0)
            hipLaunchKernelGGL(k_plain, dim3(g), dim3(256), 0, 0, src, y, n, rl);
          else
            hipLaunchKernelGGL(k_xcd, dim3(g), dim3(256), 0, 0, src, y, n, rl);
          CHECK(hipGetLastError());
          CHECK(hipEventRecord(b));
          CHECK(hipEventSynchronize(b));
          float ms;
          CHECK(hipEventElapsedTime(&ms, a, b));
          best = ms < best ? ms : best;
        }
        printf("  \"%s_g%d_region%.1fMiB\": {\"ms\": %.4f, \"Gelem_per_s\": %.2f},\n", mode ? "xcd" : "plain", g,
               (double)((int64_t)8 << rl) / 1048576.0, best, n / (best * 1e-3) / 1e9);
      }
  printf("  \"n\": %lld\n}\n", (long long)n);
  return 0;
}
