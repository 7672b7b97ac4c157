// Iman-Conover step 4 for generated LHS columns (pbh_step4.hip): MSD code passes with atomic
// cursors, a per-bucket LDS finish that emits (row, sorted position) pairs, MSD row-placement
// passes and the final assembly (gen_place, pbh_ppf.hip) that regenerates sort(X)[p].
#pragma once

#include "pbh_common.h"

namespace pbh {

constexpr int kGenPlaceShift = 12;  // final placement blocks of 4096 rows (32 KB of LDS)

// per-call state of all k columns (device): histograms, bucket starts, cursors, tile maps,
// state[c] (bit 0 counter overflow, bit 1 bucket above the finish capacity: the column is not
// flat) and flags[c] (bit 0: a run of equal codes too long for the finish; bit 2: the column is
// still not flat after the adaptive code map -- every later pass skips it, and it is redone by
// the general path after the others).  A column that is not flat under the fixed N(0, 1) code
// map (a score dominated by a discrete column: a mixture of narrow peaks) is re-coded once with
// a code map built from its own histogram (retry[c] = 1; seghist, amap) and re-counted.
constexpr int kAdaptSegments = 4096;  // adaptive code map: segments of [-8.5, 8.5]
struct Step4Shared {
  int k;
  uint32_t* hist;
  uint32_t* start;
  uint32_t* cur1;
  uint32_t* cur2;
  uint32_t* curF;  // fused finish: cursors of the top row-placement level
  uint32_t* cls;     // per column: top-byte counts of each msd1 tile class (8 x 256)
  uint32_t* cstart;  // per column: each class's start in every top-byte group (8 x 256)
  uint32_t* tpre;
  uint32_t* seghist;  // per column: kAdaptSegments counts of CS (adaptive code map)
  uint32_t* amap;     // per column: adaptive code map, kAdaptMapWords words (bases, then slopes)
  int32_t* state;
  int32_t* flags;
  int32_t* retry;
};
// words of one column's adaptive code map: kAdaptSegments + 1 bases (padded to 8 bytes), then
// kAdaptSegments double slopes
constexpr int kAdaptBaseWords = (kAdaptSegments + 2) & ~1;
constexpr int kAdaptMapWords = kAdaptBaseWords + 2 * kAdaptSegments;
// one column's staging (reused column after column)
struct Step4Column {
  uint32_t* keys32;
  uint32_t* rows1;
  uint16_t* keys16;
  uint32_t* rows2;
  uint64_t* pairs[2];
  uint32_t* pcur[2];
};

size_t step4_gen_shared_bytes(int k);
size_t step4_gen_column_bytes(int64_t n);
void step4_gen_carve_shared(void* ws, int k, Step4Shared& sh);
void step4_gen_carve_column(void* ws, int64_t n, Step4Column& cb);
bool step4_gen_enabled(int64_t n);
// columns of step 4 run concurrently on this many streams (PBH_STEP4_STREAMS, default 3, at
// most kStep4MaxStreams), each with its own Step4Column staging, so that one column's VALU- or
// latency-bound kernels (bucket finish, gen_place) overlap another's bandwidth-bound passes
constexpr int kStep4MaxStreams = 4;
int step4_streams();            // lanes in use now (1 in the serial measurement mode)
int step4_lanes_configured();   // lanes a workspace is sized for (>= step4_streams() always)
extern int g_serial;  // pbh_set_serial (measurement mode: one lane, counts not deferred)
// the side streams of this device, created once (thread-safe) and kept for the process
hipStream_t step4_side_stream(int i);
void step4_sync_side_streams();
// top-16 histograms, bucket starts and flatness of the code columns c0 .. c0 + kk - 1 (column c
// at codes + (c - c0) * ldc).  With cs (column c at cs + (c - c0) * ldcs),
// a column that is not flat is re-coded with its adaptive code map and counted again, all on
// the device (the codes are rewritten in place); state / flags then hold the final verdict.
int step4_gen_hist(uint32_t* codes, int64_t ldc, const double* cs, int64_t ldcs, int64_t n, const Step4Shared& sh,
                   int c0, int kk, hipStream_t s);
// the adaptive re-code alone (after step4_gen_hist without cs): a column's lane runs it, so the
// rare re-coded column's passes overlap the other lanes; ~6 launches that exit at once otherwise
int step4_gen_adapt(uint32_t* codes, int64_t ldc, const double* cs, int64_t ldcs, int64_t n, const Step4Shared& sh,
                    int c0, int kk, hipStream_t s);
// code passes and bucket finish of column c: (row << 32 | p') pairs in cb.pairs[0], grouped by
// the top row-placement level
int step4_gen_column(int c, const uint32_t* codes, const double* cs, int64_t n, const Step4Shared& sh,
                     const Step4Column& cb, hipStream_t s);
// row-placement MSD passes on cb.pairs[0]; *out_buf = the pairs buffer grouped by 4096-row block
int step4_gen_place_passes(int c, int64_t n, const Step4Shared& sh, const Step4Column& cb, hipStream_t s, int* out_buf);

// A generated LHS column's inverse-CDF setup (scalar parameters; gamma guide / poisson CDF
// tables built once), shared by the stratum-ordered generator and the final placement.
struct GenColumn;
// a distribution whose generated sorted column has runs of equal values (poisson, binom, bernoulli,
// geom, randint, nbinom): step 1 takes its tie count and run heads up front (never deferred)
inline bool gen_discrete(int dist) {
  return dist == PBH_DIST_POISSON || dist == PBH_DIST_BINOM || dist == PBH_DIST_BERNOULLI ||
         dist == PBH_DIST_GEOM || dist == PBH_DIST_RANDINT || dist == PBH_DIST_NBINOM ||
         dist == PBH_DIST_DLAPLACE || dist == PBH_DIST_PLANCK || dist == PBH_DIST_BOLTZMANN ||
         dist == PBH_DIST_BETABINOM || dist == PBH_DIST_HYPERGEOM || dist == PBH_DIST_NHYPERGEOM ||
         dist == PBH_DIST_YULESIMON || dist == PBH_DIST_ZIPFIAN;
}
int gen_create(uint64_t seed, int64_t n, int col, int dist, const pbh_param* params, int nparams, GenColumn** out,
               hipStream_t s);
void gen_destroy(GenColumn* g, hipStream_t s);
// out[t - t0] = the column's value in stratum t (see lhs_sorted_ppf); out may be NULL when
// counts (ties, inversions) is given.  heads: the run heads, unordered, at most hcap of them --
// every t in (t0, t0 + nt) whose value differs from stratum t - 1's, and t0 itself when t0 = 0;
// *hcur = their number (= nt - ties when t0 = 0 and there is no inversion).
constexpr int kHeadsCap = 16384;
int gen_sorted(const GenColumn* g, int64_t t0, int64_t nt, double* out, int32_t* flag, unsigned long long* counts,
               hipStream_t s, uint32_t* heads = nullptr, uint32_t* hcur = nullptr, uint32_t hcap = 0);
// The tie / inversion certificate of a continuous column's strata [t0, t0 + nt) (k_cert_scan /
// k_cert_eval, pbh_ppf.hip): counts[0] > 0 unless certified free of ties and inversions (an
// uncertified column is recounted exactly by the caller).  T = gen_cert_gap(g) > 0 required;
// list: cap candidate slots, count: one device word.
double gen_cert_gap(const GenColumn* g);
// whether the certificate applies to strata segments of nt of column g, with its gap T and list
// capacity (8 x the expected candidates; false when no bound exists or it would list > 5%)
bool gen_cert_plan(const GenColumn* g, int64_t nt, double* T, uint32_t* cap);
int gen_certify(const GenColumn* g, int64_t t0, int64_t nt, double T, uint32_t* list, uint32_t cap, uint32_t* count,
                int32_t* flag, unsigned long long* counts, hipStream_t s);
// heads[0 .. nh) in increasing order (nh <= kHeadsCap)
int sort_heads(uint32_t* heads, int64_t nh, hipStream_t s);
// y[row * y_rs] = value of stratum p for every pair (row << 32 | p) of `pairs`, grouped by
// 4096-row block (block b = positions [b << 12, ...)); idx[row] = p when idx != NULL.
// state (optional device word): skip when non-zero.
int gen_place(const GenColumn* g, const uint64_t* pairs, int64_t n, double* y, int64_t y_rs, int32_t* idx,
              const int32_t* state, hipStream_t s);
// y[i * y_rs] = value of stratum p[i] for i < m (the row owner of a row-sharded run: the sorted
// positions of its rows, sent back by the column's owner; the same kernels as gen_place)
int gen_values_at(const GenColumn* g, const uint32_t* p, int64_t m, double* y, int64_t y_rs, hipStream_t s);
// A discrete column's sorted run heads (heads[0] == 0, increasing, no inversion in the column):
// its placement then reads each run's value from a table (k_place_gen_runs) instead of evaluating
// the inverse CDF per row.  heads must stay valid while g is placed.  No-op unless the column is
// discrete with 1 <= nh <= 1024 runs (or with PBH_PLACE_RUNS=0).
int gen_set_runs(GenColumn* g, const uint32_t* heads, int64_t nh, hipStream_t s);
// p_out[row] = p for every pair (row << 32 | p) of `pairs` grouped by 4096-row block, the block
// assembled in LDS and written contiguously (the owner's step-4 output of a row-sharded run);
// state (optional device word): skip when non-zero
int place_positions(const uint64_t* pairs, int64_t n, uint32_t* p_out, const int32_t* state, hipStream_t s);

}  // namespace pbh
