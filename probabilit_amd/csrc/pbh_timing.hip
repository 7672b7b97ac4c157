#include <vector>

#include "pbh_error.h"
#include "pbh_timing.h"

namespace pbh {

bool g_timing_on = false;

namespace {
struct Slot {
  std::vector<hipEvent_t> start, stop;
};
Slot g_slots[kKCount];
std::vector<hipEvent_t> g_pool;

const char* kNames[kKCount] = {"k_lhs_ppf", "k_ppf", "k_scatter", "k_upsweep", "k_digit_hist", "k_rank_finish<scores>",
                               "k_rank_finish<gather>", "k_load_keys", "k_gram", "k_apply", "k_elementwise",
                               "k_head_bounds", "k_scan", "k_lhs_sorted_ppf", "k_perm_scores", "k_code_runs",
                               "k_make_codes", "k_scatter<u32>", "k_upsweep<u32>", "k_digit_hist<u32>",
                               "k_upsweep<place>", "k_scatter<place>", "k_place", "k_streams", "k_affine", "k_table_ppf",
                               "k_permcorr", "k_hbm_copy", "k_hist16", "k_msd1", "k_msd2", "k_finish",
                               "k_place_msd", "k_place_gen", "k_dag", "k_transpose"};

hipEvent_t take_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}
}  // namespace

void timing_before(int id, hipStream_t s) {
  hipEvent_t e = take_event();
  (void)hipEventRecord(e, s);
  g_slots[id].start.push_back(e);
}

void timing_after(int id, hipStream_t s) {
  hipEvent_t e = take_event();
  (void)hipEventRecord(e, s);
  g_slots[id].stop.push_back(e);
}

// HBM copy ceiling of the box (bench.py's measured peak next to the 8 TB/s spec).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// variant 0: grid-stride, 16-byte non-temporal loads and stores, four in flight per lane
__global__ __launch_bounds__(256) void k_hbm_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(src + i + j * stride);
#pragma unroll
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(v[j], dst + i + j * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// variants 1-4: one block per contiguous tile of 256 x U 16-byte vectors (no grid stride: many
// more blocks than CUs), U loads in flight per lane before the stores; NT: non-temporal
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_hbm_copy_tile(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       int64_t n16) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int64_t i = base + (int64_t)j * 256;
    if (i < n16) v[j] = NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int64_t i = base + (int64_t)j * 256;
    if (i < n16) {
      if (NT)
        __builtin_nontemporal_store(v[j], dst + i);
      else
        dst[i] = v[j];
    }
  }
}

}  // namespace pbh

using namespace pbh;

extern "C" int pbh_hbm_copy(const void* src, void* dst, size_t bytes, int variant, void* stream) {
  PBH_REQUIRE(src && dst && bytes % 16 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
              "pbh_hbm_copy: 16-byte aligned buffers and size required");
  PBH_REQUIRE(variant >= 0 && variant <= 4, "pbh_hbm_copy: variant %d outside [0, 4]", variant);
  hipStream_t s = as_stream(stream);
  const int64_t n16 = (int64_t)(bytes / 16);
  const auto tiles = [&](int u) { return dim3((unsigned)((n16 + 256 * u - 1) / (256 * u))); };
  switch (variant) {
    case 0:
      PBH_TIMED(kKHbmCopy, s,
                hipLaunchKernelGGL(k_hbm_copy, dim3(grid_for(n16, 256, 256 * 16)), dim3(256), 0, s, (const u32x4*)src,
                                   (u32x4*)dst, n16));
      break;
    case 1: PBH_TIMED(kKHbmCopy, s, hipLaunchKernelGGL((k_hbm_copy_tile<4, false>), tiles(4), dim3(256), 0, s,
                                                       (const u32x4*)src, (u32x4*)dst, n16)); break;
    case 2: PBH_TIMED(kKHbmCopy, s, hipLaunchKernelGGL((k_hbm_copy_tile<8, false>), tiles(8), dim3(256), 0, s,
                                                       (const u32x4*)src, (u32x4*)dst, n16)); break;
    case 3: PBH_TIMED(kKHbmCopy, s, hipLaunchKernelGGL((k_hbm_copy_tile<4, true>), tiles(4), dim3(256), 0, s,
                                                       (const u32x4*)src, (u32x4*)dst, n16)); break;
    default: PBH_TIMED(kKHbmCopy, s, hipLaunchKernelGGL((k_hbm_copy_tile<8, true>), tiles(8), dim3(256), 0, s,
                                                        (const u32x4*)src, (u32x4*)dst, n16)); break;
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

extern "C" int pbh_timing_enable(int on) {
  g_timing_on = on != 0;
  return PBH_OK;
}

extern "C" int pbh_timing_reset(void) {
  for (auto& s : g_slots) {
    for (auto e : s.start) g_pool.push_back(e);
    for (auto e : s.stop) g_pool.push_back(e);
    s.start.clear();
    s.stop.clear();
  }
  return PBH_OK;
}

extern "C" const char* pbh_kernel_name(int id) { return (id >= 0 && id < kKCount) ? kNames[id] : ""; }

extern "C" int pbh_timing_read(int id, double* total_ms, int64_t* launches) {
  PBH_REQUIRE(id >= 0 && id < kKCount && total_ms && launches, "pbh_timing_read: bad arguments");
  Slot& s = g_slots[id];
  double tot = 0.0;
  for (size_t i = 0; i < s.start.size() && i < s.stop.size(); ++i) {
    PBH_CHECK_HIP(hipEventSynchronize(s.stop[i]));
    float ms = 0.f;
    PBH_CHECK_HIP(hipEventElapsedTime(&ms, s.start[i], s.stop[i]));
    tot += ms;
  }
  *total_ms = tot;
  *launches = (int64_t)s.start.size();
  return PBH_OK;
}
