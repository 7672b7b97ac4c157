// Inverse-CDF setup tables kept for the process (round 5, cfg2).  A graph sampled again with the
// same scalar parameters -- the reference's usual loop of .sample() calls -- would otherwise
// rebuild the gamma / beta guides and the poisson / binom CDF tables on every call: latency-bound
// kernels of 10-100 us each (k_gamma_guide + check ~110 us at a = 2), which at N = 1e7 cost as
// much as the inverse CDF itself.  A table larger than kEntryMaxBytes (a poisson table at a huge
// mean) is never cached; past kCacheBytes or kCacheEntries the least recently used entry that no
// call holds is evicted (after the last kernel that read it), and pbh_table_cache_clear frees
// every entry no call holds.
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
constexpr size_t kEntryMaxBytes = (size_t)64 << 20;

struct Entry {
  int kind, nkey, device;
  double key[4];
  double* ptr;
  size_t bytes;
  hipEvent_t ready;     // the build's completion
  hipEvent_t last_use;  // recorded by release_table: the last kernel of a call that read it
  int refs;             // calls between cached_table and release_table
  uint64_t stamp;       // last acquisition (LRU order)
};

// Frees e once the kernels that read it are done (its events first).
void free_entry(Entry& e) {
  if (e.last_use) (void)hipEventSynchronize(e.last_use);
  (void)hipEventSynchronize(e.ready);
  (void)hipFree(e.ptr);
  if (e.last_use) (void)hipEventDestroy(e.last_use);
  (void)hipEventDestroy(e.ready);
}

}  // namespace

struct TableCache {
  std::mutex mu;
  std::vector<Entry> entries;
  size_t bytes = 0;
  int64_t hits = 0;
  int64_t evictions = 0;
  uint64_t clock = 0;
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
  for (Entry& e : c.entries) {
    if (e.kind == kind && e.nkey == nkey && e.device == dev && memcmp(e.key, key, (size_t)nkey * 8) == 0) {
      if (hipStreamWaitEvent(s, e.ready, 0) != hipSuccess) return nullptr;
      ++c.hits;
      ++e.refs;
      e.stamp = ++c.clock;
      return e.ptr;
    }
  }
  if (bytes > kEntryMaxBytes) return nullptr;
  // make room: evict the least recently used entries no call holds
  while (c.bytes + bytes > kCacheBytes || c.entries.size() >= kCacheEntries) {
    size_t victim = c.entries.size();
    for (size_t i = 0; i < c.entries.size(); ++i)
      if (c.entries[i].refs == 0 && (victim == c.entries.size() || c.entries[i].stamp < c.entries[victim].stamp))
        victim = i;
    if (victim == c.entries.size()) return nullptr;  // every entry is in use: build per call
    c.bytes -= c.entries[victim].bytes;
    free_entry(c.entries[victim]);
    c.entries.erase(c.entries.begin() + (ptrdiff_t)victim);
    ++c.evictions;
  }
  Entry e{kind, nkey, dev, {0, 0, 0, 0}, nullptr, bytes, nullptr, nullptr, 1, ++c.clock};
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
    for (Entry& e : c.entries)
      if (e.ptr == t) {
        if (!e.last_use) (void)hipEventCreateWithFlags(&e.last_use, hipEventDisableTiming);
        if (e.last_use) (void)hipEventRecord(e.last_use, s);
        if (e.refs > 0) --e.refs;
        return;
      }
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

extern "C" int pbh_table_cache_clear(int64_t* freed, int64_t* kept) {
  pbh::TableCache& c = pbh::cache();
  std::lock_guard<std::mutex> lock(c.mu);
  int64_t f = 0;
  std::vector<pbh::Entry> keep;
  for (pbh::Entry& e : c.entries) {
    if (e.refs > 0) {
      keep.push_back(e);
      continue;
    }
    c.bytes -= e.bytes;
    pbh::free_entry(e);
    ++f;
  }
  c.entries.swap(keep);
  if (freed) *freed = f;
  if (kept) *kept = (int64_t)c.entries.size();
  return PBH_OK;
}
