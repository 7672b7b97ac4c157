// Device radix sort of one column of float64 keys with a uint32 row payload.
//
// This is the "argsort" inside scipy.stats.rankdata (scipy:stats/_stats_py.py _rankdata,
// reached from correlation.py:394 and :422) and the np.sort of correlation.py:423.
// Stable LSD radix sort over the order-preserving 64-bit image of the doubles, 8-bit
// digits, tiles of 4096 keys per 256-thread workgroup:
//   upsweep  : per-tile digit histogram                       (read 8 B/key)
//   scan     : exclusive scan of the [digit][tile] count table
//   scatter  : stable in-tile ranking with wave64 ballots, LDS-staged so that every
//              digit run leaves the tile as one contiguous burst (read 12, write 12 B/key)
// Byte positions on which every key agrees are skipped (one histogram pass up front).
#pragma once

#include "pbh_common.h"

namespace pbh {

// the one-sweep look-back words' pass state (host side, one per workspace): the words carry the
// pass's epoch, so they are cleared once (the first pass) rather than before every pass
struct SweepState {
  uint32_t epoch;      // of the last pass; 0: the words are not cleared yet
  uint32_t tile_base;  // the tile counter's value before the next pass
  size_t bytes;        // the words, the tile counter and the stuck flag
};

struct SortBuffers {
  uint64_t* keys[2];
  uint32_t* vals[2];
  uint32_t* counts;    // 256 * ntiles
  uint32_t* partials;  // scan partials
  uint32_t* hist;      // 8 * 256 digit histogram
  uint32_t* hist_host; // pinned host mirror of hist (8 * 256)
  uint64_t* status;    // one-sweep look-back words (256 * ntiles) + tile counter
  uint32_t* bases;     // one-sweep global digit bases (8 * 256)
  SweepState sweep;    // set by sort_carve
};

constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortThreads * kSortItems;  // 4096

inline int64_t sort_tiles(int64_t n) { return (n + kSortTile - 1) / kSortTile; }
inline int64_t scan_partials_count(int64_t m) { return (m + 2047) / 2048; }

// Workspace (bytes) for sorting n keys, excluding nothing: keys x2, vals x2, counts,
// partials, histogram.
size_t sort_workspace_bytes(int64_t n);
void sort_carve(void* ws, int64_t n, SortBuffers& b);

// Sorts keys in b.keys[0] (payload: row index, generated) and returns the index (0/1) of
// the buffer holding the sorted keys / payload.  `stream` ordered; synchronises once to read
// the digit histogram (pass skipping).  Returns < 0 and sets the last error on failure.
int radix_sort_keys(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf);
// The same over bytes 2..7 only, then each run of keys equal in their top 48 bits ordered by the
// whole key: the same result with two passes fewer when the low bytes vary.  *redo: a run was
// longer than the fix-up takes (the keys are left partly ordered: load them again and sort with
// radix_sort_keys).  Synchronises once more than radix_sort_keys.
int radix_sort_keys_top48(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf, bool* redo);
// In-place exclusive scan of m uint32 counts (partials: scan_partials_count(m) entries).
int exclusive_scan_u32(uint32_t* a, int64_t m, uint32_t* partials, hipStream_t s);
// The same on uint32 keys stored in b.keys[0] (reinterpreted), or read from `in` (left
// unmodified): at most 4 passes.
int radix_sort_keys32(SortBuffers& b, int64_t n, hipStream_t s, int* out_buf, const uint32_t* in = nullptr);
// The stable LSD passes of radix_sort_keys32 over the low npass bytes of the keys read from `in`
// (payload: their index), with no host synchronisation: every pass runs (a constant byte is a
// copy), and *stuck points at the device word a failed look-back sets (the caller checks it).
int radix_sort_keys32_async(SortBuffers& b, int64_t n, int npass, hipStream_t s, int* out_buf, const uint32_t* in,
                            uint32_t** stuck);
// Step 4's code sort for 2^22 <= n <= 2^27 (see k_code_buckets): codes -> rows in final rank
// order in b.vals[*out_buf] plus eqprev / flags exactly as resolve_code_runs leaves them (flags
// bit 0: fall back to 64-bit keys; bit 1: exact ties).  flags must be zeroed by the caller.
// hist_dev (optional): the four byte histograms of `codes` already on the device (code_hist),
// with `flat` the host's code_hist_flat decision for them; without it the function computes
// both (one stream sync).
bool code_buckets_enabled(int64_t n);
bool code_hist_flat(const uint32_t* hist4_host, int64_t n);
int code_hist(const uint32_t* codes, int64_t n, uint32_t* hist4, hipStream_t s);
int code_sort_buckets(SortBuffers& b, int64_t n, const uint32_t* codes, const double* x, uint8_t* eqprev,
                      int32_t* flags, hipStream_t s, int* out_buf, const uint32_t* hist_dev = nullptr, int flat = 1);

// Y[rows[p] * y_rs] = v[p] for a permutation `rows` of [0, n): the inverse-permutation write
// of Iman-Conover step 4 (correlation.py:423) without random 8-byte stores.  LSD bucket passes
// on row >> kPlaceShift (the stable scatter above, payload = value) bring every block of
// kPlaceRows consecutive rows together; k_place then assembles each block in LDS and writes it
// out as one contiguous run.  rows/vals: two ping-pong staging pairs of n entries each.
constexpr int kPlaceShift = 13;
constexpr int kPlaceRows = 1 << kPlaceShift;  // 8192 rows = 64 KB of LDS per block
struct PlaceBuffers {
  uint32_t* rows[2];
  double* vals[2];
  uint32_t* counts;    // 256 * sort_tiles(n)
  uint32_t* partials;  // scan partials
  uint64_t* status;    // one-sweep look-back words
  uint32_t* bases;     // 256 digit bases
  SweepState* sweep;   // the SortBuffers' pass state whose status words these are
};
// err (optional, device): a look-back failure is OR-ed into *err on the stream instead of being
// read back with a synchronisation
int place_by_row(const uint32_t* rows, const double* v, int64_t n, double* y, int64_t y_rs, const PlaceBuffers& pb,
                 hipStream_t s, int32_t* err = nullptr);

}  // namespace pbh
