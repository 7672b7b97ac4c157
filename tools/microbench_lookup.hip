// Microbenchmark: random small reads on MI355X, to decide the step-4 design of Iman-Conover.
//
// A "rank lookup" step 4 would rank every row in row order by looking its 32-bit code up in
// per-bucket tables (a 65536 x 256 table of 16-bit offsets, 32 MB, and a 1-byte-per-row list of
// sorted low bytes, 100 MB at N = 1e8) instead of moving (row, value) pairs through two bucket
// passes and an LDS assembly.  Whether that wins depends on the rate of random 2-byte / 1-byte
// reads from tables that may or may not stay in the Infinity Cache next to the streamed
// traffic of the same kernel.  Also: the HBM copy ceiling with plain vs non-temporal 16-byte
// accesses (the bench's measured peak).
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_lookup.hip -o /tmp/mbl && /tmp/mbl
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

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// per row: code = hash(row); bucket b = code >> 16, h = (code >> 8) & 255;
// o0, o1 = off[b][h], off[b][h + 1]; count list bytes in [start[b] + o0, start[b] + o1) below code & 255
template <int MODE>
__global__ __launch_bounds__(256) void k_lookup(const uint32_t* __restrict__ start, const uint16_t* __restrict__ off,
                                                const uint8_t* __restrict__ list, uint64_t list_mask, int64_t n,
                                                double* __restrict__ out, uint32_t tmask) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t code = mix32((uint32_t)i * 2654435761u + 12345u);
    const uint32_t b = (code >> 16) & tmask, h = (code >> 8) & 255u;
    double r = 0.0;
    if (MODE >= 1) {
      const uint32_t o = *(const uint32_t*)(off + ((size_t)b * 256 + (h & ~1u)));  // the pair (off[h], off[h+1])
      const uint32_t o0 = (h & 1) ? (o >> 16) : (o & 0xFFFF);
      r = (double)o0;
      if (MODE >= 2) {
        const uint64_t base = ((uint64_t)start[b] + o0) & list_mask;
        const uint64_t w = *(const uint64_t*)(list + (base & ~7ull));
        const uint32_t low = code & 255u;
        int c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) c += ((w >> (8 * j)) & 255u) < low;
        r += (double)c;
      }
    }
    out[i] = r;
  }
}

// random 8-byte gather from a large table (the sorted_x[rank] read of a row-order step 4)
__global__ __launch_bounds__(256) void k_gather8(const double* __restrict__ t, uint64_t tmask, int64_t n,
                                                 double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint64_t j = (((uint64_t)mix32((uint32_t)i) << 32) | mix32((uint32_t)i ^ 0x9E3779B9u)) & tmask;
    out[i] = t[j];
  }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT, int U>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = NT ? __builtin_nontemporal_load(src + i + j * stride) : src[i + j * stride];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (NT)
        __builtin_nontemporal_store(v[j], dst + i + j * stride);
      else
        dst[i + j * stride] = v[j];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// blocked copy: each block moves one contiguous 64 KB chunk per iteration (4 x 16 B per lane)
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_blocked(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                      int64_t n16) {
  const int64_t chunk = 256 * 16;
  for (int64_t c0 = (int64_t)blockIdx.x * chunk; c0 < n16; c0 += (int64_t)gridDim.x * chunk) {
    u32x4 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t i = c0 + j * 256 + threadIdx.x;
      if (i < n16) v[j] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t i = c0 + j * 256 + threadIdx.x;
      if (i < n16) {
        if (NT)
          __builtin_nontemporal_store(v[j], dst + i);
        else
          dst[i] = v[j];
      }
    }
  }
}

int main() {
  const int64_t n = 100000000;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto timeit = [&](auto launch, int reps) -> float {
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
  };
  printf("{\n");
  // ---- copy ceiling
  {
    const size_t bytes = (size_t)4 << 30;
    void *s, *d;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(s, 1, bytes));
    const int64_t n16 = bytes / 16;
    for (int g : {1024, 2048, 4096, 8192}) {
      float t1 = timeit([&] { hipLaunchKernelGGL((k_copy<false, 4>), dim3(g), dim3(256), 0, 0, (const u32x4*)s, (u32x4*)d, n16); }, 5);
      float t2 = timeit([&] { hipLaunchKernelGGL((k_copy<true, 4>), dim3(g), dim3(256), 0, 0, (const u32x4*)s, (u32x4*)d, n16); }, 5);
      float t3 = timeit([&] { hipLaunchKernelGGL((k_copy<false, 1>), dim3(g), dim3(256), 0, 0, (const u32x4*)s, (u32x4*)d, n16); }, 5);
      float t4 = timeit([&] { hipLaunchKernelGGL((k_copy_blocked<false>), dim3(g), dim3(256), 0, 0, (const u32x4*)s, (u32x4*)d, n16); }, 5);
      float t5 = timeit([&] { hipLaunchKernelGGL((k_copy_blocked<true>), dim3(g), dim3(256), 0, 0, (const u32x4*)s, (u32x4*)d, n16); }, 5);
      printf("  \"copy_g%d\": {\"plain_u4_GBps\": %.1f, \"nt_u4_GBps\": %.1f, \"plain_u1_GBps\": %.1f, \"blocked_GBps\": %.1f, \"blocked_nt_GBps\": %.1f},\n",
             g, 2.0 * bytes / (t1 / 1e3) / 1e9, 2.0 * bytes / (t2 / 1e3) / 1e9, 2.0 * bytes / (t3 / 1e3) / 1e9,
             2.0 * bytes / (t4 / 1e3) / 1e9, 2.0 * bytes / (t5 / 1e3) / 1e9);
    }
    CHECK(hipFree(s));
    CHECK(hipFree(d));
  }
  // ---- lookups
  double* out;
  CHECK(hipMalloc(&out, n * 8));
  uint32_t* start;
  CHECK(hipMalloc(&start, 65536 * 4));
  CHECK(hipMemset(start, 0, 65536 * 4));
  uint16_t* off;
  CHECK(hipMalloc(&off, (size_t)65536 * 256 * 2 + 64));
  CHECK(hipMemset(off, 0, (size_t)65536 * 256 * 2 + 64));
  uint8_t* list;
  const size_t list_bytes = (size_t)1 << 27;  // 128 MB
  CHECK(hipMalloc(&list, list_bytes + 64));
  CHECK(hipMemset(list, 7, list_bytes + 64));
  const unsigned grid = 256 * 16;
  float tw = timeit([&] { hipLaunchKernelGGL((k_lookup<0>), dim3(grid), dim3(256), 0, 0, start, off, list, list_bytes - 1, n, out, 0xFFFFu); }, 5);
  printf("  \"write_only_1e8_ms\": %.4f,\n", tw);
  for (uint32_t tm : {0xFFu, 0xFFFu, 0x3FFFu, 0xFFFFu}) {  // off-table footprint 128 KB .. 32 MB
    float t1 = timeit([&] { hipLaunchKernelGGL((k_lookup<1>), dim3(grid), dim3(256), 0, 0, start, off, list, list_bytes - 1, n, out, tm); }, 5);
    printf("  \"offset_lookup_table%uKB_1e8_ms\": %.4f,\n", (tm + 1) * 512 / 1024, t1);
  }
  for (size_t lb : {(size_t)1 << 20, (size_t)1 << 24, (size_t)1 << 26, (size_t)1 << 27}) {
    float t2 = timeit([&] { hipLaunchKernelGGL((k_lookup<2>), dim3(grid), dim3(256), 0, 0, start, off, list, lb - 1, n, out, 0xFFFFu); }, 5);
    printf("  \"two_level_off32MB_list%zuMB_1e8_ms\": %.4f,\n", lb >> 20, t2);
  }
  double* tab;
  const size_t tb = (size_t)1 << 27;  // 2^27 doubles = 1 GB
  CHECK(hipMalloc(&tab, tb * 8));
  CHECK(hipMemset(tab, 0, tb * 8));
  for (size_t tsz : {(size_t)1 << 17, (size_t)1 << 22, (size_t)1 << 25, (size_t)1 << 27}) {
    float t = timeit([&] { hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(256), 0, 0, tab, (uint64_t)(tsz - 1), n, out); }, 5);
    printf("  \"gather8_table%zuMB_1e8_ms\": %.4f,\n", (tsz * 8) >> 20, t);
  }
  printf("  \"n\": %lld\n}\n", (long long)n);
  return 0;
}
