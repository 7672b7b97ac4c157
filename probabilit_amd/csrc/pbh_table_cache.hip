// Inverse-CDF setup tables kept for the process (round 5, cfg2).  A graph sampled again with the
// same scalar parameters -- the reference's usual loop of .sample() calls -- would otherwise
// rebuild the gamma / beta guides and the poisson / binom CDF tables on every call: latency-bound
// kernels of 10-100 us each (k_gamma_guide + check ~110 us at a = 2), which at N = 1e7 cost as
// much as the inverse CDF itself.  Entries are never evicted; past kCacheBytes the tables are
// built per call again.
#include <string.h>

#include <mutex>
#include <vector>

#include "pbh_error.h"
#include "pbh_table_cache.h"
#include "probabilit_hip.h"

namespace pbh {
namespace {

constexpr size_t kCacheBytes = (size_t)1 << 30;
constexpr size_t kCacheEntries = 4096;

struct Entry {
  int kind, nkey, device;
  double key[4];
  double* ptr;
  size_t bytes;
  hipEvent_t ready;
};

}  // namespace

struct TableCache {
  std::mutex mu;
  std::vector<Entry> entries;
  size_t bytes = 0;
  int64_t hits = 0;
};

static TableCache& cache() {
  static TableCache c;
  return c;
}

double* cached_table(int kind, const double* key, int nkey, size_t bytes, hipStream_t s,
                     const std::function<bool(double*, hipStream_t)>& build) {
  if (nkey < 0 || nkey > 4) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  TableCache& c = cache();
  std::lock_guard<std::mutex> lock(c.mu);
  for (const Entry& e : c.entries) {
    if (e.kind == kind && e.nkey == nkey && e.device == dev && memcmp(e.key, key, (size_t)nkey * 8) == 0) {
      if (hipStreamWaitEvent(s, e.ready, 0) != hipSuccess) return nullptr;
      ++c.hits;
      return e.ptr;
    }
  }
  if (c.bytes + bytes > kCacheBytes || c.entries.size() >= kCacheEntries) return nullptr;
  Entry e{kind, nkey, dev, {0, 0, 0, 0}, nullptr, bytes, nullptr};
  memcpy(e.key, key, (size_t)nkey * 8);
  if (hipMalloc((void**)&e.ptr, bytes) != hipSuccess) return nullptr;
  if (!build(e.ptr, s) || hipEventCreateWithFlags(&e.ready, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamSynchronize(s);
    (void)hipFree(e.ptr);
    return nullptr;
  }
  if (hipEventRecord(e.ready, s) != hipSuccess) {
    (void)hipStreamSynchronize(s);
    (void)hipEventDestroy(e.ready);
    (void)hipFree(e.ptr);
    return nullptr;
  }
  c.entries.push_back(e);
  c.bytes += bytes;
  return e.ptr;
}

void release_table(double* t, hipStream_t s) {
  if (!t) return;
  {
    TableCache& c = cache();
    std::lock_guard<std::mutex> lock(c.mu);
    for (const Entry& e : c.entries)
      if (e.ptr == t) return;
  }
  (void)hipFreeAsync(t, s);
}

}  // namespace pbh

extern "C" int pbh_table_cache_stats(int64_t* entries, int64_t* bytes, int64_t* hits) {
  PBH_REQUIRE(entries && bytes && hits, "pbh_table_cache_stats: bad arguments");
  pbh::TableCache& c = pbh::cache();
  std::lock_guard<std::mutex> lock(c.mu);
  *entries = (int64_t)c.entries.size();
  *bytes = (int64_t)c.bytes;
  *hits = c.hits;
  return PBH_OK;
}
