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
                               "k_permcorr"};

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

}  // namespace pbh

using namespace pbh;

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
