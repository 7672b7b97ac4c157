// Iman-Conover step 4 for GENERATED columns (correlation.py:418-423):
//     idx = rankdata(CS[:, k]).astype(int) - 1;  Y[:, k] = sort(X[:, k])[idx]
// where sort(X[:, k]) is the stratum-ordered native LHS column, so its value at sorted
// position p is regenerated from p (pbh_ppf.hip gen_place) and only the permutation moves:
//
//   hist16   top-16-bit histogram of the 32-bit codes (written by step 3), its prefix = the
//            start of every top-16 bucket, a per-column flatness check        (read 4 B)
//   msd1     (code, row) scattered by the top code byte                       (read 4, write 8)
//   msd2     (low 16 code bits, row) scattered into the top-16 buckets        (read 8, write 6)
//   finish   one wave per bucket (~1500 items): sort by the low 16 bits in LDS, order runs of
//            equal codes by the full CS value (exact ties flagged), emit (row, p') packed in a
//            u64 with p' = the sorted position, or the tie group's 'average' position  (read 6, write 8)
//   place    MSD passes on the row of (row, p') until every 4096-row block is together (read 8,
//            write 8 per pass; 2 passes at N = 1e8), then gen_place assembles each block in
//            LDS, regenerating sort(X)[p'] (write 8)
//
// Every scatter is an MSD pass with per-destination cursors advanced by one global atomic per
// (tile, digit): no decoupled look-back, no status words, no host round trip.  Stability is not
// needed anywhere: the bucket finish orders every bucket completely, and the row placement
// writes each value at its own row.  Host decisions are batched: one readback after hist16 for
// all columns (flatness), one at the end (buckets that met a run longer than kRunCap), whose
// columns are redone by the general path (pbh_phases.hip reorder_column).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "pbh_error.h"
#include "pbh_ic.h"
#include "pbh_step4.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kT = 256;
constexpr int kIptP = 16;
constexpr int kTileP = kT * kIptP;  // placement tiles: 4096 pairs (divides every group size 2^s >= 2^12)
constexpr int kBucketCap2 = 2048;   // items per top-16 bucket a wave can finish
constexpr int kRunCap = 16;         // longest run of equal codes the finish orders
// Cursor spacing (u32 words) of the code-pass and finish cursors: one 64-byte line each.
static int cur_pad() { return 16; }

__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sh /* >= 256 + waves */) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[256 + w] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int i = 0; i < w; ++i) pre += sh[256 + i];
  __syncthreads();
  return pre + x - v;
}

// ---------------------------------------------------------------- hist16
// One 1024-thread block per (chunk, column): 65536 16-bit counters packed two per LDS word
// (128 KiB), flushed with one global add per non-empty counter.  A counter reaching 65535 in
// one block (a spike: a discrete-dominated correlated score) sets the column's state bit 0,
// which routes it to the general path; so does a bucket above kBucketCap2 (k_hist16_scan).
//
// It also counts, per column, the top code byte of every tile class x = (row >> tlog) mod 8
// (cls[x][byte]; 2^tlog = msd1's tile): k_msd1x tile i runs as block i, and blocks b and b + 8
// share an XCD, so the code pass gives each class its own cursors and sub-ranges (see k_msd1x).
__global__ __launch_bounds__(1024) void k_hist16(const uint32_t* __restrict__ codes, int64_t ld, int64_t n,
                                                 uint32_t* __restrict__ hist, uint32_t* __restrict__ cls,
                                                 int32_t* __restrict__ state, const int32_t* __restrict__ gate,
                                                 int tlog) {
  __shared__ uint32_t w[32768];
  __shared__ uint32_t cw[8 * 256];
  __shared__ int ovf;
  const int c = blockIdx.y;
  if (gate && !gate[c]) return;  // the adaptive re-count: only the re-coded columns
  const uint32_t* cc = codes + (int64_t)c * ld;
  for (int i = threadIdx.x; i < 32768; i += 1024) w[i] = 0;
  for (int i = threadIdx.x; i < 8 * 256; i += 1024) cw[i] = 0;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  const int64_t chunk = ((n + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  bool bad = false;
  auto add = [&](uint32_t code, int64_t row) {
    const uint32_t b = code >> 16, sh = (b & 1u) * 16u;
    const uint32_t old = atomicAdd(&w[b >> 1], 1u << sh);
    bad |= ((old >> sh) & 0xFFFFu) == 0xFFFFu;
    atomicAdd(&cw[(((uint32_t)(row >> tlog) & 7u) << 8) | (code >> 24)], 1u);
  };
  if ((((uintptr_t)(cc + lo)) & 15) == 0) {
    const int64_t n4 = (hi - lo) / 4;
    const uint4* v4 = reinterpret_cast<const uint4*>(cc + lo);
    for (int64_t i = threadIdx.x; i < n4; i += 1024) {
      const uint4 v = v4[i];
      const int64_t r = lo + 4 * i;
      add(v.x, r);
      add(v.y, r + 1);
      add(v.z, r + 2);
      add(v.w, r + 3);
    }
    for (int64_t i = lo + 4 * n4 + threadIdx.x; i < hi; i += 1024) add(cc[i], i);
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += 1024) add(cc[i], i);
  }
  if (bad) ovf = 1;
  __syncthreads();
  uint32_t* hc = hist + (int64_t)c * 65536;
  for (int j = threadIdx.x; j < 32768; j += 1024) {
    const uint32_t v = w[j];
    if (v & 0xFFFFu) atomicAdd(&hc[2 * j], v & 0xFFFFu);
    if (v >> 16) atomicAdd(&hc[2 * j + 1], v >> 16);
  }
  for (int j = threadIdx.x; j < 8 * 256; j += 1024)
    if (cw[j]) atomicAdd(&cls[(int64_t)c * 2048 + j], cw[j]);
  if (threadIdx.x == 0 && ovf) atomicOr(&state[c], 1);
}

// k_hist16 in class-major order (gridDim.x a multiple of 8, the default 64 blocks per column): block
// b counts only tiles of class x = b mod 8 (a contiguous share of them), so its tile-class top-byte
// counts are the sums of its own 65536 counters over each top byte -- formed once at the flush
// instead of one more LDS atomic per code (half of the kernel's atomics) -- and each thread keeps
// four 16-byte loads in flight.  Same counts as k_hist16.
__global__ __launch_bounds__(1024) void k_hist16c(const uint32_t* __restrict__ codes, int64_t ld, int64_t n,
                                                  uint32_t* __restrict__ hist, uint32_t* __restrict__ cls,
                                                  int32_t* __restrict__ state, const int32_t* __restrict__ gate,
                                                  int tlog) {
  __shared__ uint32_t w[32768];
  __shared__ uint32_t cw[256];
  __shared__ int ovf;
  const int c = blockIdx.y;
  if (gate && !gate[c]) return;
  const uint32_t* cc = codes + (int64_t)c * ld;
  for (int i = threadIdx.x; i < 32768; i += 1024) w[i] = 0;
  if (threadIdx.x < 256) cw[threadIdx.x] = 0;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  const int x = blockIdx.x & 7, sub = blockIdx.x >> 3, nsub = gridDim.x >> 3;
  const int64_t T = (int64_t)1 << tlog;
  const int64_t ntiles = (n + T - 1) >> tlog;
  const int64_t nct = ntiles > x ? (ntiles - x + 7) >> 3 : 0;  // tiles of class x
  const int64_t j0 = nct * sub / nsub, j1 = nct * (sub + 1) / nsub;
  bool bad = false;
  auto add = [&](uint32_t code) {
    const uint32_t b = code >> 16, sh = (b & 1u) * 16u;
    const uint32_t old = atomicAdd(&w[b >> 1], 1u << sh);
    bad |= ((old >> sh) & 0xFFFFu) == 0xFFFFu;
  };
  // the full tiles as one stream of 16-byte units: unit u -> tile x + 8 (j0 + u / q4), offset u % q4
  const bool partial_last = (n & (T - 1)) != 0 && j1 > j0 && x + 8 * (j1 - 1) == ntiles - 1;
  const int64_t jf = partial_last ? j1 - 1 : j1;  // full tiles [j0, jf)
  const int64_t q4 = T >> 2;
  if ((((uintptr_t)cc) & 15) == 0 && tlog >= 2) {
    const uint4* v4 = reinterpret_cast<const uint4*>(cc);
    const int64_t units = (jf - j0) * q4;
    for (int64_t u0 = threadIdx.x; u0 < units; u0 += 4 * 1024) {
      uint4 v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int64_t u = u0 + m * 1024;
        if (u < units) {
          const int64_t j = j0 + (u >> (tlog - 2));  // q4 = 2^(tlog - 2) units per tile
          v[m] = v4[((x + 8 * j) << (tlog - 2)) + (u & (q4 - 1))];
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (u0 + m * 1024 < units) {
          add(v[m].x);
          add(v[m].y);
          add(v[m].z);
          add(v[m].w);
        }
      }
    }
  } else {
    for (int64_t j = j0; j < jf; ++j)
      for (int64_t i = threadIdx.x; i < T; i += 1024) add(cc[((x + 8 * j) << tlog) + i]);
  }
  if (partial_last) {
    const int64_t r0 = (x + 8 * (j1 - 1)) << tlog;
    for (int64_t i = r0 + threadIdx.x; i < n; i += 1024) add(cc[i]);
  }
  if (bad) ovf = 1;
  __syncthreads();
  uint32_t* hc = hist + (int64_t)c * 65536;
  for (int j = threadIdx.x; j < 32768; j += 1024) {
    const uint32_t v = w[j];
    if (v & 0xFFFFu) atomicAdd(&hc[2 * j], v & 0xFFFFu);
    if (v >> 16) atomicAdd(&hc[2 * j + 1], v >> 16);
    // the top byte of the counters in word j is j >> 7; a wave's 64 words share it
    uint32_t sum = (v & 0xFFFFu) + (v >> 16);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0 && sum) atomicAdd(&cw[j >> 7], sum);
  }
  __syncthreads();
  if (threadIdx.x < 256 && cw[threadIdx.x]) atomicAdd(&cls[(int64_t)c * 2048 + (x << 8) + threadIdx.x], cw[threadIdx.x]);
  if (threadIdx.x == 0 && ovf) atomicOr(&state[c], 1);
}

// The gated re-count of k_hist16 (the adaptive code map's second count): the same counts in four
// quarters of the 65536 buckets (blockIdx.z), 16-bit packed in 32 KiB of LDS instead of 128 KiB --
// the gate is only known on the device, so every column's blocks are dispatched, and a no-op block
// holding 136 KiB of LDS would wait for an almost empty CU; the tile-class counts in quarter 0.
__global__ __launch_bounds__(1024) void k_hist16_q(const uint32_t* __restrict__ codes, int64_t ld, int64_t n,
                                                   uint32_t* __restrict__ hist, uint32_t* __restrict__ cls,
                                                   int32_t* __restrict__ state, const int32_t* __restrict__ gate,
                                                   int tlog) {
  __shared__ uint32_t w[8192];
  __shared__ uint32_t cw[8 * 256];
  __shared__ int ovf;
  const int c = blockIdx.y;
  if (!gate[c]) return;
  const uint32_t q = blockIdx.z;
  const uint32_t* cc = codes + (int64_t)c * ld;
  for (int i = threadIdx.x; i < 8192; i += 1024) w[i] = 0;
  for (int i = threadIdx.x; i < 8 * 256; i += 1024) cw[i] = 0;
  if (threadIdx.x == 0) ovf = 0;
  __syncthreads();
  const int64_t chunk = ((n + gridDim.x - 1) / gridDim.x + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  bool bad = false;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 1024) {
    const uint32_t code = cc[i];
    const uint32_t b = code >> 16;
    if (q == 0) atomicAdd(&cw[(((uint32_t)(i >> tlog) & 7u) << 8) | (code >> 24)], 1u);
    if ((b >> 14) != q) continue;
    const uint32_t l = b & 16383u, sh = (l & 1u) * 16u;
    const uint32_t old = atomicAdd(&w[l >> 1], 1u << sh);
    bad |= ((old >> sh) & 0xFFFFu) == 0xFFFFu;
  }
  if (bad) ovf = 1;
  __syncthreads();
  uint32_t* hc = hist + (int64_t)c * 65536 + q * 16384;
  for (int j = threadIdx.x; j < 8192; j += 1024) {
    const uint32_t v = w[j];
    if (v & 0xFFFFu) atomicAdd(&hc[2 * j], v & 0xFFFFu);
    if (v >> 16) atomicAdd(&hc[2 * j + 1], v >> 16);
  }
  if (q == 0)
    for (int j = threadIdx.x; j < 8 * 256; j += 1024)
      if (cw[j]) atomicAdd(&cls[(int64_t)c * 2048 + j], cw[j]);
  if (threadIdx.x == 0 && ovf) atomicOr(&state[c], 1);
}

// One 1024-thread block per column: start[b] = exclusive prefix of the 65536 bucket counts
// (start[65536] = n), the msd2 tile map (tiles of 2^tlog inside every top-byte group: tpre[g]
// = tiles before group g), and state bit 1 when a bucket exceeds kBucketCap2.
// cstart[x][g] = start of top byte g + the counts of classes < x in it (k_msd1's sub-ranges).
__global__ __launch_bounds__(1024) void k_hist16_scan(const uint32_t* __restrict__ hist, int64_t n,
                                                      uint32_t* __restrict__ start, uint32_t* __restrict__ tpre,
                                                      const uint32_t* __restrict__ cls, uint32_t* __restrict__ cstart,
                                                      int32_t* __restrict__ state, int32_t* __restrict__ flags,
                                                      const int32_t* __restrict__ gate, int tlog) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t gsize[256];
  __shared__ uint32_t gstart[256];
  __shared__ int big;
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (gate && !gate[c]) return;
  const uint32_t* hc = hist + (int64_t)c * 65536;
  uint32_t* sc = start + (int64_t)c * 65537;
  if (t == 0) big = 0;
  uint32_t v[64], s = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    v[j] = hc[t * 64 + j];
    s += v[j];
    mx = v[j] > mx ? v[j] : mx;
  }
  uint32_t x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int i = 0; i < wv; ++i) pre += wsum[i];
  uint32_t run = pre + x - s;
  if ((t & 3) == 0) gstart[t >> 2] = run;  // start of top byte t / 4 (= bucket 64 t)
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    sc[t * 64 + j] = run;
    run += v[j];
  }
  if (t == 1023) sc[65536] = run;
  if (mx > (uint32_t)kBucketCap2) big = 1;
  if ((t & 3) == 0) gsize[t >> 2] = 0;
  __syncthreads();
  atomicAdd(&gsize[t >> 2], s);  // top-byte group g = threads 4 g .. 4 g + 3 (256 buckets)
  __syncthreads();
  if (t < 256) {
    uint32_t r = gstart[t];
    for (int xc = 0; xc < 8; ++xc) {
      cstart[(int64_t)c * 2048 + xc * 256 + t] = r;
      r += cls[(int64_t)c * 2048 + xc * 256 + t];
    }
  }
  if (t == 0) {
    uint32_t acc = 0;
    for (int g = 0; g < 256; ++g) {
      tpre[(int64_t)c * 257 + g] = acc;
      acc += (gsize[g] + (1u << tlog) - 1) >> tlog;
    }
    tpre[(int64_t)c * 257 + 256] = acc;
    if (big) atomicOr(&state[c], 2);
    // not flat (this kernel's verdict or k_hist16's counter overflow): the placement passes and
    // gen_place, which test flags, skip the column as the code passes and the finish do on state
    if (big || state[c]) atomicOr(&flags[c], 4);
  }
}

// ---------------------------------------------------------------- adaptive code map
// A column that is not flat under the fixed map (code_of: Phi of an N(0, 1) score) gets a map
// built from its own distribution: kAdaptSegments equal segments of [-8.5, 8.5], segment j's
// codes [base_j, base_j+1) in proportion to its share of the column.  code(x) stays
// non-decreasing in x (bases strictly increasing, offsets monotone and clamped), so sorting by
// code and ordering equal-code runs by value is still the exact float64 order.
constexpr double kAdaptX0 = -8.5;
constexpr double kAdaptW = 17.0 / kAdaptSegments;

// one block per column: retry[c] = (state[c] != 0); a retried column's histograms, cursors and
// verdict words are cleared for the second count
__global__ __launch_bounds__(1024) void k_adapt_reset(int32_t* __restrict__ state, int32_t* __restrict__ flags,
                                                      int32_t* __restrict__ retry, uint32_t* __restrict__ hist,
                                                      uint32_t* __restrict__ cur1, uint32_t* __restrict__ cur2,
                                                      uint32_t* __restrict__ curF, uint32_t* __restrict__ cls,
                                                      uint32_t* __restrict__ seghist, int cpad) {
  const int c = blockIdx.x, t = threadIdx.x;
  const bool again = state[c] != 0;
  __syncthreads();  // every thread has read state[c] before thread 0 clears it
  if (!again) {
    if (t == 0) retry[c] = 0;
    return;
  }
  for (int i = t; i < 65536; i += 1024) {
    hist[(int64_t)c * 65536 + i] = 0u;
    cur2[(int64_t)c * 65536 + i] = 0u;
  }
  for (int i = t; i < 8 * 256 * cpad; i += 1024) {
    cur1[(int64_t)c * 8 * 256 * cpad + i] = 0u;
    curF[(int64_t)c * 8 * 256 * cpad + i] = 0u;
  }
  for (int i = t; i < 2048; i += 1024) cls[(int64_t)c * 2048 + i] = 0u;
  for (int i = t; i < kAdaptSegments; i += 1024) seghist[(int64_t)c * kAdaptSegments + i] = 0u;
  if (t == 0) {
    state[c] = 0;
    flags[c] = 0;
    retry[c] = 1;
  }
}

// segment counts of the retried columns' CS values (values outside [-8.5, 8.5] are not counted:
// they take code 0 / 0xFFFFFFFF)
__global__ __launch_bounds__(1024) void k_seg_hist(const double* __restrict__ cs, int64_t ld, int64_t n,
                                                   const int32_t* __restrict__ retry, uint32_t* __restrict__ seghist) {
  __shared__ uint32_t h[kAdaptSegments];
  const int c = blockIdx.y;
  if (!retry[c]) return;
  for (int i = threadIdx.x; i < kAdaptSegments; i += 1024) h[i] = 0u;
  __syncthreads();
  const double* x = cs + (int64_t)c * ld;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 1024) {
    const double u = (x[i] - kAdaptX0) * (1.0 / kAdaptW);
    if (u >= 0.0 && u < (double)kAdaptSegments) atomicAdd(&h[(int)u], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kAdaptSegments; i += 1024)
    if (h[i]) atomicAdd(&seghist[(int64_t)c * kAdaptSegments + i], h[i]);
}

// one block per retried column: bases from the exclusive prefix of the segment counts
// (base_j = floor(cum_j span / total) + j: strictly increasing), slopes = codes per unit x
__global__ __launch_bounds__(1024) void k_seg_map(const uint32_t* __restrict__ seghist, const int32_t* __restrict__ retry,
                                                  uint32_t* __restrict__ amap) {
  constexpr int kPer = kAdaptSegments / 1024;
  __shared__ uint32_t sh[1024 + 16];
  __shared__ uint32_t bs[kAdaptSegments + 1];
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (!retry[c]) return;
  const uint32_t* h = seghist + (int64_t)c * kAdaptSegments;
  uint32_t v[kPer], sum = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    v[q] = h[t * kPer + q];
    sum += v[q];
  }
  uint32_t x = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[1024 + wv] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int i = 0; i < wv; ++i) pre += sh[1024 + i];
  uint32_t run = pre + x - sum;
  if (t == 1023) sh[0] = run + sum;  // the total (read after the barrier below)
  __syncthreads();
  const double total = sh[0] ? (double)sh[0] : 1.0;
  const double span = 4294967295.0 - kAdaptSegments;
  uint32_t* base = amap + (int64_t)c * kAdaptMapWords;
  double* slope = (double*)(base + kAdaptBaseWords);
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int j = t * kPer + q;
    bs[j] = (uint32_t)floor((double)run * span / total) + (uint32_t)j;
    run += v[q];
  }
  if (t == 1023) bs[kAdaptSegments] = 4294967295u;  // floor(total span / total) + m
  __syncthreads();
  for (int j = t; j <= kAdaptSegments; j += 1024) base[j] = bs[j];
  for (int j = t; j < kAdaptSegments; j += 1024) slope[j] = (double)(bs[j + 1] - bs[j]) * (1.0 / kAdaptW);
}

// codes of the retried columns under their adaptive maps (staged in LDS), rewritten in place
__global__ __launch_bounds__(256) void k_make_codes_adapt(const double* __restrict__ cs, int64_t ld, int64_t n,
                                                          const int32_t* __restrict__ retry,
                                                          const uint32_t* __restrict__ amap,
                                                          uint32_t* __restrict__ codes, int64_t ldc) {
  __shared__ uint32_t lb[kAdaptSegments + 1];
  __shared__ double ls[kAdaptSegments];
  const int c = blockIdx.y;
  if (!retry[c]) return;
  const uint32_t* base = amap + (int64_t)c * kAdaptMapWords;
  const double* slope = (const double*)(base + kAdaptBaseWords);
  for (int j = threadIdx.x; j <= kAdaptSegments; j += 256) lb[j] = base[j];
  for (int j = threadIdx.x; j < kAdaptSegments; j += 256) ls[j] = slope[j];
  __syncthreads();
  CodeMap cm;
  cm.x0 = kAdaptX0;
  cm.w = kAdaptW;
  cm.inv_w = 1.0 / kAdaptW;
  cm.m = kAdaptSegments;
  cm.base = lb;
  cm.scale = ls;
  const double* x = cs + (int64_t)c * ld;
  uint32_t* out = codes + (int64_t)c * ldc;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = code_of(x[i], cm);
}

// ---------------------------------------------------------------- code passes
// msd1: tiles of NT x IPT consecutive rows; digit = top code byte.  msd2: tiles of the same size
// inside each top-byte group (tile map tpre); digit = code byte 2; destination = the group's
// top-16 bucket (g << 8 | digit); writes the low 16 code bits.
//
// Both stage through one 32-bit LDS array, used twice (codes, then rows).  A slot's LDS position
// (digit start + rank) replaces its code and rank once the digit starts are known, so the code is
// dead after the first staging round and the rows round reuses the slots and the destinations:
// every configuration stays within 64 VGPRs, 8 waves per SIMD (round 2's 256-thread kernels held
// code, rank and destination at once: 83-84 VGPRs, 5 waves, msd1 16.4 against 11 ms per step).
// PBH_MSD_TILE picks the tile: 8192 rows over 1024 threads (default: a tile's run for one digit is
// 32 items, 128 bytes of codes) or 4096 over 256 (msd1) / 512 (msd2) threads (64-byte runs).
// XCD: msd1's tile class x = blockIdx.x mod 8 appends to its own sub-range of every top-byte
// group through its own cursor (cstart, cur + x * 256): 1/8 of the tiles contend on a cursor,
// and the runs of one sub-range are all written from one XCD (its L2 merges the lines); k_hist16
// counts the classes with the same tile size.
template <int NT, int IPT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8))) void k_msd1x(
    const uint32_t* __restrict__ codes, int64_t n, const uint32_t* __restrict__ start, uint32_t* __restrict__ cur,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ rout, const uint32_t* __restrict__ cstart, int cpad,
    const int32_t* __restrict__ state) {
  constexpr int kTile = NT * IPT;
  if (*state) return;  // uniform: this column takes the general path
  __shared__ uint32_t cnt[256], lst[256 + NT / 64], gb[256];
  __shared__ uint32_t sk[kTile];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int m = (int)((n - base) < kTile ? (n - base) : kTile);
  if (t < 256) cnt[t] = 0;
  __syncthreads();
  uint32_t key[IPT], slot[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    key[j] = p < m ? codes[base + p] : 0u;
  }
#pragma unroll
  for (int j = 0; j < IPT; ++j) slot[j] = (j * NT + t < m) ? atomicAdd(&cnt[key[j] >> 24], 1u) : 0u;
  __syncthreads();
  const uint32_t my = t < 256 ? cnt[t] : 0u;
  const uint32_t ex = block_excl_scan256(my, lst);  // waves past the fourth add nothing
  // the cursor add's round trip overlaps the first LDS scatter: its result is stored to gb only
  // after that scatter (the barrier that follows publishes it)
  uint32_t myb = 0u;
  if (t < 256) {
    lst[t] = ex;
    if (cstart) {
      const uint32_t xc = blockIdx.x & 7u;
      myb = my ? cstart[(xc << 8) + t] + atomicAdd(&cur[((xc << 8) + t) * cpad], my) : 0u;
    } else {
      myb = my ? start[t << 8] + atomicAdd(&cur[t * cpad], my) : 0u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    if (j * NT + t < m) {
      slot[j] += lst[key[j] >> 24];
      sk[slot[j]] = key[j];
    }
  }
  if (t < 256) gb[t] = myb;
  __syncthreads();
  uint32_t dst[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    if (p < m) {
      const uint32_t k = sk[p], d = k >> 24;
      dst[j] = gb[d] + ((uint32_t)p - lst[d]);
      kout[dst[j]] = k;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j)
    if (j * NT + t < m) sk[slot[j]] = (uint32_t)(base + j * NT + t);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    if (p < m) rout[dst[j]] = sk[p];
  }
}

template <int NT, int IPT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(8))) void k_msd2x(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ rin, const uint32_t* __restrict__ start,
    const uint32_t* __restrict__ tpre, uint32_t* __restrict__ cur, uint16_t* __restrict__ kout,
    uint32_t* __restrict__ rout, const int32_t* __restrict__ state) {
  constexpr int kTile = NT * IPT;
  if (*state) return;
  const uint32_t tile = blockIdx.x;
  if (tile >= tpre[256]) return;
  __shared__ uint32_t cnt[256], lst[256 + NT / 64], gb[256];
  __shared__ uint32_t sk[kTile];
  __shared__ int gsh;
  const int t = threadIdx.x;
  if (t == 0) {  // the group holding this tile: last g with tpre[g] <= tile
    int lo = 0, hi = 256;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tpre[mid] <= tile)
        lo = mid;
      else
        hi = mid - 1;
    }
    while (lo < 255 && tpre[lo + 1] <= tile) ++lo;  // skip empty groups
    gsh = lo;
  }
  if (t < 256) cnt[t] = 0;
  __syncthreads();
  const int g = gsh;
  const int64_t gs = start[g << 8], ge = start[(g + 1) << 8];
  const int64_t base = gs + (int64_t)(tile - tpre[g]) * kTile;
  const int m = (int)((ge - base) < kTile ? (ge - base) : kTile);
  uint32_t key[IPT], row[IPT], slot[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    key[j] = p < m ? kin[base + p] : 0u;
    row[j] = p < m ? rin[base + p] : 0u;
  }
#pragma unroll
  for (int j = 0; j < IPT; ++j) slot[j] = (j * NT + t < m) ? atomicAdd(&cnt[(key[j] >> 16) & 255u], 1u) : 0u;
  __syncthreads();
  const uint32_t my = t < 256 ? cnt[t] : 0u;
  const uint32_t ex = block_excl_scan256(my, lst);
  uint32_t myb = 0u;
  if (t < 256) {
    lst[t] = ex;
    const uint32_t b = ((uint32_t)g << 8) | (uint32_t)t;
    myb = my ? start[b] + atomicAdd(&cur[b], my) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    if (j * NT + t < m) {
      slot[j] += lst[(key[j] >> 16) & 255u];
      sk[slot[j]] = key[j];
    }
  }
  if (t < 256) gb[t] = myb;
  __syncthreads();
  uint32_t dst[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    if (p < m) {
      const uint32_t kk = sk[p], d = (kk >> 16) & 255u;
      dst[j] = gb[d] + ((uint32_t)p - lst[d]);
      kout[dst[j]] = (uint16_t)kk;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j)
    if (j * NT + t < m) sk[slot[j]] = row[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int p = j * NT + t;
    if (p < m) rout[dst[j]] = sk[p];
  }
}

// ---------------------------------------------------------------- counting finish, fused row pass
// One 512-thread block finishes two consecutive top-16 buckets, one after the other, and then
// scatters their (row << 32 | p') pairs straight into the groups of the first row-placement level
// (row >> s_top; group g at positions [g << s_top, ...), closed form since the rows are a
// permutation), so the pairs never exist in position order.  Per bucket:
//   * a non-stable LDS-atomic counting pass on the top 11 of the 16 low code bits (2048 bins,
//     ~0.75 items per bin at 1500 items per bucket) puts every bin together;
//   * every item counts, inside its bin, the items below it: lt = #{smaller low bits} +
//     #{equal code (a run), smaller CS value}, eq = #{equal code, equal CS} (exact ties);
//   * p' = bucket start + bin start + lt + eq / 2: the sorted position, or for a group of exact
//     ties [a, a + eq] its 'average' rank minus one, truncated (rankdata(...).astype(int) - 1).
// No order inside a bin is ever materialised, so neither pass needs to be stable.  A bin above
// kBinCap items (far from the expected: a discrete spike) flags the column for the general path.
constexpr int kBinCap = 32;

// The counting finish over 512 threads: 4 items of each bucket per thread, so it fits 64 VGPRs
// and 8 waves per SIMD (the 256-thread form needed ~100-120 VGPRs: 4 waves), which hides its
// latency far better (r3 A/B: 23-24 against 28-30 ms per step).  The bin loop counts by code alone and marks the members of
// runs of equal codes; a second loop orders each run by CS value.  With Q the run members' CS
// values are first loaded together into an LDS queue (one round trip per bucket instead of one
// per item; a bucket whose runs hold more than kFQCap items reads the rest from global memory):
// faster standalone, but the default without it measured ~2 ms per step faster in the pipeline.
constexpr int kFQCap = 512;
#ifndef PBH_FINISH_BINS
#define PBH_FINISH_BINS 2048  // counting bins of k_finish_q (4096: 113.8-114.4 against 113.5-114.8 ms per
                              // step, no gain: profiles/r06/ab_finish_bins_r6fb.log)
#endif
#ifndef PBH_FINISH_NT
#define PBH_FINISH_NT 512  // threads of k_finish_q; 1024 (two items of each bucket per thread, 16-wave
                           // barriers) measured 120 against 113-116 ms per step (profiles/r06/ab_finish_nt_r6fn.log)
#endif

template <int BINS, int FB>
union FinishQLds {
  struct {
    uint32_t cnt[BINS + 1];
    uint16_t key[kBucketCap2];
    uint16_t qi[kBucketCap2];  // a run member's queue slot, by its position in the bin order
    uint32_t row[kBucketCap2];
    double qx[kFQCap];
  } a;
  uint64_t sv[FB * kBucketCap2];
};

// NT threads per block (256: 8 items of each bucket per thread, 4 waves per SIMD; 512: 4 items, 8)
// Q = false: no queue, the run members read the CS values of their run from global memory in
// pass 2 (as k_finish_ah does in its one loop)
template <int BINS, int NT, bool Q = true>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT >= 512 ? 8 : 4))) void k_finish_q(
    const uint16_t* __restrict__ keys, const uint32_t* __restrict__ rows, const double* __restrict__ x,
    const uint32_t* __restrict__ start, int s_top, uint32_t* __restrict__ gcur, int cpad, uint64_t* __restrict__ out,
    int32_t* __restrict__ flags, const int32_t* __restrict__ state) {
  if (*state) return;
  constexpr int FB = 2;  // buckets per block (one per block measured 24 -> 42 ms per step)
  constexpr int kShift = 16 - __builtin_ctz(BINS);
  constexpr int kPer = BINS / NT;
  constexpr int kIt = kBucketCap2 / NT;  // items of a bucket per thread
  __shared__ FinishQLds<BINS, FB> L;
  __shared__ uint32_t gcnt[256], goff[256 + NT / 64], gbase[256];
  __shared__ int bad;
  __shared__ uint32_t nq;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  if (t < 256) gcnt[t] = 0;
  uint32_t kk[FB][kIt], rr[FB][kIt], grk[FB * kIt];
  int64_t s0[FB];
  int l0[FB];
#pragma unroll
  for (int bb = 0; bb < FB; ++bb) {
    const int bkt = blockIdx.x * FB + bb;
    s0[bb] = start[bkt];
    l0[bb] = (int)((int64_t)start[bkt + 1] - s0[bb]);
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
      const int p = j * NT + t;
      kk[bb][j] = p < l0[bb] ? (uint32_t)keys[s0[bb] + p] : 0u;
      rr[bb][j] = p < l0[bb] ? rows[s0[bb] + p] : 0u;
    }
  }
  __syncthreads();
#pragma unroll
  for (int bb = 0; bb < FB; ++bb)
#pragma unroll
    for (int j = 0; j < kIt; ++j)
      grk[bb * kIt + j] = (j * NT + t < l0[bb]) ? atomicAdd(&gcnt[rr[bb][j] >> s_top], 1u) : 0u;
  __syncthreads();
  const uint32_t my = t < 256 ? gcnt[t] : 0u;
  const uint32_t gex = block_excl_scan256(my, goff);  // waves past 4 add nothing
  if (t < 256) goff[t] = gex;
  const uint32_t mybase = my ? (uint32_t)(((uint64_t)t << s_top) + atomicAdd(&gcur[t * cpad], my)) : 0u;
  uint64_t pr[FB * kIt];
  int total = 0;
#pragma unroll
  for (int bb = 0; bb < FB; ++bb) {
    const int64_t s = s0[bb];
    const int len = l0[bb];
    for (int i = t; i <= BINS; i += NT) L.a.cnt[i] = 0;
    if (t == 0) nq = 0;
    __syncthreads();
    uint32_t rk[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j)
      rk[j] = (j * NT + t < len) ? atomicAdd(&L.a.cnt[kk[bb][j] >> kShift], 1u) : 0u;
    __syncthreads();
    uint32_t cb[kPer], sum = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      cb[q] = L.a.cnt[kPer * t + q];
      sum += cb[q];
    }
    uint32_t run = block_excl_scan256(sum, goff);  // scratch goff[256..259]; goff[0..255] kept
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      L.a.cnt[kPer * t + q] = run;
      run += cb[q];
    }
    if (t == NT - 1) L.a.cnt[BINS] = run;
    __syncthreads();
    uint32_t pos[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
      if (j * NT + t < len) {
        pos[j] = L.a.cnt[kk[bb][j] >> kShift] + rk[j];
        L.a.key[pos[j]] = (uint16_t)kk[bb][j];
        L.a.row[pos[j]] = rr[bb][j];
      }
    }
    __syncthreads();
    // pass 1: the bin's items by code alone; members of runs of equal codes are marked
    uint32_t lt[kIt], runs = 0;
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
      lt[j] = 0;
      if (j * NT + t >= len) continue;
      const uint32_t kj = kk[bb][j];
      const uint32_t bs = L.a.cnt[kj >> kShift], be = L.a.cnt[(kj >> kShift) + 1];
      if (be - bs > 1) {
        if (be - bs > (uint32_t)kBinCap) bad = 1;
        bool member = false;
        for (uint32_t m = bs; m < be; ++m) {
          const uint32_t km = L.a.key[m];
          lt[j] += km < kj;
          member |= km == kj && m != pos[j];
        }
        runs |= (uint32_t)member << j;
      }
      lt[j] += bs;
    }
    // the run members' CS values: queue slots, then every load issued before any is waited on
    uint32_t slot[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) slot[j] = kFQCap;
    if constexpr (Q) {
#pragma unroll
      for (int j = 0; j < kIt; ++j) {
        if ((runs >> j) & 1u) {
          slot[j] = atomicAdd(&nq, 1u);
          L.a.qi[pos[j]] = (uint16_t)(slot[j] < (uint32_t)kFQCap ? slot[j] : 0xFFFFu);
        }
      }
      double v[kIt];
#pragma unroll
      for (int j = 0; j < kIt; ++j) v[j] = slot[j] < (uint32_t)kFQCap ? x[rr[bb][j]] : 0.0;
#pragma unroll
      for (int j = 0; j < kIt; ++j)
        if (slot[j] < (uint32_t)kFQCap) L.a.qx[slot[j]] = v[j];
      __syncthreads();
    }
    // pass 2: a run member counts the smaller / equal CS values of its run (from LDS)
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
      const int sl = bb * kIt + j;
      if (j * NT + t >= len) {
        pr[sl] = ~0ull;
        continue;
      }
      uint32_t eq = 0;
      if ((runs >> j) & 1u) {
        const uint32_t kj = kk[bb][j];
        const uint32_t bs = L.a.cnt[kj >> kShift], be = L.a.cnt[(kj >> kShift) + 1];
        const double xv = slot[j] < (uint32_t)kFQCap ? L.a.qx[slot[j]] : x[rr[bb][j]];
        for (uint32_t m = bs; m < be; ++m) {
          if (L.a.key[m] != kj || m == pos[j]) continue;
          const uint32_t qm = Q ? L.a.qi[m] : 0xFFFFu;
          const double xm = qm < (uint32_t)kFQCap ? L.a.qx[qm] : x[L.a.row[m]];
          lt[j] += xm < xv;
          eq += xm == xv;
        }
      }
      const uint32_t p = (uint32_t)s + lt[j] + eq / 2;
      pr[sl] = ((uint64_t)rr[bb][j] << 32) | (uint64_t)p;
    }
    total += len;
    __syncthreads();
  }
  if (t < 256) gbase[t] = mybase;
  __syncthreads();
#pragma unroll
  for (int sl = 0; sl < FB * kIt; ++sl)
    if (pr[sl] != ~0ull) L.sv[goff[(uint32_t)(pr[sl] >> (32 + s_top))] + grk[sl]] = pr[sl];
  __syncthreads();
  for (int p = t; p < total; p += NT) {
    const uint64_t v2 = L.sv[p];
    const uint32_t g = (uint32_t)(v2 >> (32 + s_top));
    out[gbase[g] + ((uint32_t)p - goff[g])] = v2;
  }
  __syncthreads();
  if (t == 0 && bad) atomicOr(flags, 1);
}

// ---------------------------------------------------------------- row placement passes
// Input grouped by row >> s_in (closed-form groups: rows are a permutation of [0, n), so group
// g occupies positions [g << s_in, ...)); tiles of kTileP never straddle a group.  Digit =
// (row >> s_out) within the group; destination = positions (row >> s_out) << s_out.
// A 4096-pair tile over 512 threads of 8 pairs each, 8 waves per SIMD (the 256-thread form of 16
// pairs needed 100 VGPRs: 4 waves; 13.4 against 13.1 ms per step).  The low halves are staged
// first and read back in position order, then the high halves (rows), which give the
// destination; the pair is written whole.
constexpr int kTO = 512;
constexpr int kIptO = kTileP / kTO;
__global__ __launch_bounds__(kTO) __attribute__((amdgpu_waves_per_eu(8))) void k_place_msdo(
    const uint64_t* __restrict__ in, int64_t n, int s_out, uint32_t* __restrict__ cur, uint64_t* __restrict__ out,
    const int32_t* __restrict__ state) {
  if (state && *state) return;
  __shared__ uint32_t cnt[256], lst[264], gb[256];
  __shared__ uint32_t sh32[kTileP];
  __shared__ uint32_t gfirst;
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kTileP;
  const int m = (int)((n - base) < kTileP ? (n - base) : kTileP);
  if (t < 256) cnt[t] = 0;
  if (t == 0) gfirst = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t hi[kIptO], lo[kIptO], slot[kIptO];
#pragma unroll
  for (int j = 0; j < kIptO; ++j) {
    const int p = j * kTO + t;
    const uint64_t v = p < m ? in[base + p] : 0ull;
    hi[j] = (uint32_t)(v >> 32);
    lo[j] = (uint32_t)v;
  }
  uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
  for (int j = 0; j < kIptO; ++j)
    if (j * kTO + t < m) mn = min(mn, hi[j] >> s_out);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor(mn, o, 64));
  if ((t & 63) == 0) atomicMin(&gfirst, mn);
  __syncthreads();
  const uint32_t g0 = gfirst;
#pragma unroll
  for (int j = 0; j < kIptO; ++j) slot[j] = (j * kTO + t < m) ? atomicAdd(&cnt[(hi[j] >> s_out) - g0], 1u) : 0u;
  __syncthreads();
  const uint32_t my = t < 256 ? cnt[t] : 0u;
  const uint32_t ex = block_excl_scan256(my, lst);  // waves 4-7 add nothing (lst[256..263] scratch)
  uint32_t myb = 0u;
  if (t < 256) {
    lst[t] = ex;
    myb = my ? (uint32_t)(((uint64_t)(g0 + t) << s_out) + atomicAdd(&cur[g0 + t], my)) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kIptO; ++j) {
    if (j * kTO + t < m) {
      slot[j] += lst[(hi[j] >> s_out) - g0];
      sh32[slot[j]] = lo[j];
    }
  }
  if (t < 256) gb[t] = myb;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kIptO; ++j) lo[j] = sh32[j * kTO + t];  // low halves in position order
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kIptO; ++j)
    if (j * kTO + t < m) sh32[slot[j]] = hi[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kIptO; ++j) {
    const int p = j * kTO + t;
    if (p < m) {
      const uint32_t h = sh32[p], d = (h >> s_out) - g0;
      out[gb[d] + ((uint32_t)p - lst[d])] = ((uint64_t)h << 32) | lo[j];
    }
  }
}

// p_out[row] = p of the pairs (row << 32 | p) of every 4096-row block, assembled in LDS and
// written contiguously: a row-sharded run's owner sends these sorted positions back (4 bytes a
// row instead of the 8 of Y; the row owner regenerates sort(X)[p], gen_values_at)
__global__ __launch_bounds__(256) void k_place_positions(const uint64_t* __restrict__ pairs, int64_t n,
                                                         uint32_t* __restrict__ p_out,
                                                         const int32_t* __restrict__ state) {
  if (state && *state) return;
  constexpr int kRows = 1 << kGenPlaceShift;
  __shared__ uint32_t buf[kRows];
  for (int64_t b = blockIdx.x; (b << kGenPlaceShift) < n; b += gridDim.x) {
    const int64_t r0 = b << kGenPlaceShift;
    const int cnt = (int)((n - r0) < kRows ? (n - r0) : kRows);
    for (int p = threadIdx.x; p < cnt; p += 256) {
      const uint64_t pr = pairs[r0 + p];
      buf[(int64_t)(pr >> 32) - r0] = (uint32_t)pr;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < cnt; p += 256) p_out[r0 + p] = buf[p];
    __syncthreads();
  }
}

}  // namespace

int place_positions(const uint64_t* pairs, int64_t n, uint32_t* p_out, const int32_t* state, hipStream_t s) {
  const int64_t blocks = (n + (1 << kGenPlaceShift) - 1) >> kGenPlaceShift;
  if (blocks <= 0) return PBH_OK;
  PBH_TIMED(kKPlaceGen, s,
            hipLaunchKernelGGL(k_place_positions, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, s,
                               pairs, n, p_out, state));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

size_t step4_gen_shared_bytes(int k) {
  // per column: hist 65536 + start 65537 + cur1 8 x 256 * pad + cur2 65536 + curF 256 * pad +
  // cls 2048 + cstart 2048 + tpre 257 + seghist + amap (u32), state / flags / retry
  const size_t pad = (size_t)cur_pad();
  return (size_t)k * ((65536 + 65537 + 8 * 256 * pad + 65536 + 8 * 256 * pad + 2048 + 2048 + 257 + kAdaptSegments +
                       kAdaptMapWords) * 4 + 64) + 512;
}

size_t step4_gen_column_bytes(int64_t n) {
  // keys32 + rows (msd1 out) | keys16 + rows (msd2 out) | pairs x 2 | placement cursors
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const int64_t ncur = (n >> kGenPlaceShift) + 2;
  return al((size_t)n * 4) * 2 + al((size_t)n * 2) + al((size_t)n * 4) + al((size_t)n * 8) +
         al((size_t)n * 8) + al((size_t)ncur * 4) * 2 + al(2049 * 4);
}

void step4_gen_carve_shared(void* ws, int k, Step4Shared& sh) {
  char* p = (char*)ws;
  sh.k = k;
  sh.hist = (uint32_t*)p;
  p += (size_t)k * 65536 * 4;
  sh.start = (uint32_t*)p;
  p += (size_t)k * 65537 * 4;
  sh.cur1 = (uint32_t*)p;
  p += (size_t)k * 8 * 256 * cur_pad() * 4;
  sh.cur2 = (uint32_t*)p;
  p += (size_t)k * 65536 * 4;
  sh.curF = (uint32_t*)p;
  p += (size_t)k * 8 * 256 * cur_pad() * 4;
  sh.cls = (uint32_t*)p;
  p += (size_t)k * 2048 * 4;
  sh.cstart = (uint32_t*)p;
  p += (size_t)k * 2048 * 4;
  sh.tpre = (uint32_t*)p;
  p += (size_t)k * 257 * 4;
  sh.seghist = (uint32_t*)p;
  p += (size_t)k * kAdaptSegments * 4;
  p = (char*)(((uintptr_t)p + 63) & ~(uintptr_t)63);
  sh.amap = (uint32_t*)p;  // 8-byte aligned slopes: kAdaptBaseWords is even
  p += (size_t)k * kAdaptMapWords * 4;
  p = (char*)(((uintptr_t)p + 63) & ~(uintptr_t)63);
  sh.state = (int32_t*)p;   // k words: bit 0 counter overflow, bit 1 bucket over cap
  sh.flags = sh.state + k;  // k words: bit 0 long run / too many runs in a bucket, bit 2 not flat
  sh.retry = sh.flags + k;  // k words: re-coded with the adaptive map
}

void step4_gen_carve_column(void* ws, int64_t n, Step4Column& cb) {
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* p = (char*)ws;
  cb.keys32 = (uint32_t*)p;
  p += al((size_t)n * 4);
  cb.rows1 = (uint32_t*)p;
  p += al((size_t)n * 4);
  cb.keys16 = (uint16_t*)p;
  p += al((size_t)n * 2);
  cb.rows2 = (uint32_t*)p;
  p += al((size_t)n * 4);
  cb.pairs[0] = (uint64_t*)p;
  p += al((size_t)n * 8);
  cb.pairs[1] = (uint64_t*)p;
  p += al((size_t)n * 8);
  const int64_t ncur = (n >> kGenPlaceShift) + 2;
  cb.pcur[0] = (uint32_t*)p;
  p += al((size_t)ncur * 4);
  cb.pcur[1] = (uint32_t*)p;
  p += al((size_t)ncur * 4);
}

int g_serial = 0;  // pbh_set_serial: one lane, no deferred counts (standalone kernel durations)

int step4_lanes_configured() {  // PBH_STEP4_STREAMS (default 3): the workspaces hold this many lanes
  static const int v = [] {
    const char* e = getenv("PBH_STEP4_STREAMS");
    int x = e ? atoi(e) : 3;
    return x < 1 ? 1 : (x > kStep4MaxStreams ? kStep4MaxStreams : x);
  }();
  return v;
}

int step4_streams() { return g_serial ? 1 : step4_lanes_configured(); }

hipStream_t step4_side_stream(int i) {
  // created once per device and kept for the life of the process (non-blocking: no implicit
  // ordering with the legacy default stream; the caller orders them with events).  Creation is
  // serialised: two host threads may reach it at once (calls on one device are not otherwise
  // concurrent: probabilit_hip.h).
  static hipStream_t streams[64][kStep4MaxStreams] = {};
  static std::mutex mu;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64 || i < 0 || i >= kStep4MaxStreams) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!streams[dev][i]) (void)hipStreamCreateWithFlags(&streams[dev][i], hipStreamNonBlocking);
  return streams[dev][i];
}

void step4_sync_side_streams() {
  for (int i = 0; i < kStep4MaxStreams; ++i) {  // every one (the deferred counts use the last)
    hipStream_t x = step4_side_stream(i);
    if (x) (void)hipStreamSynchronize(x);
  }
}

// PBH_MSD_TILE: the code passes' tile, 8192 rows (default) or 4096 (k_msd1x / k_msd2x)
static bool hist_class_major() {  // PBH_HIST_CLASS=0: k_hist16 (one more LDS atomic per code) everywhere
  static const bool on = [] {
    const char* e = getenv("PBH_HIST_CLASS");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int msd_tile_log() {
  static const int v = [] {
    const char* e = getenv("PBH_MSD_TILE");
    return e && atoi(e) == 4096 ? 12 : 13;
  }();
  return v;
}



// MSD levels of the row placement: shifts from kGenPlaceShift up, at most 8 bits per level
// With two levels the top one (the finish's scatter) takes 8 bits and the MSD pass the rest (at
// N = 1e8: 191 groups of 2^19 rows, 128 digits per placement tile, 32-item runs: place_msd 13.2 ->
// 11.3 ms per step, the finish +0.5); PBH_PLACE_TOP=0: the MSD pass takes 8 (96 groups of 2^20,
// 256 digits)
static int place_levels(int64_t n, int* shifts) {
  static const bool top = [] {
    const char* e = getenv("PBH_PLACE_TOP");
    return !(e && e[0] == '0');
  }();
  int bits = 0;
  while (((int64_t)1 << bits) < n) ++bits;
  int nl = 0;
  for (int sh = kGenPlaceShift; sh < bits; sh += 8) shifts[nl++] = sh;
  if (top && nl == 2 && bits - 8 > shifts[0]) shifts[1] = bits - 8;
  return nl;
}

bool step4_gen_enabled(int64_t n) {
  const char* e = getenv("PBH_STEP4");  // "lsd" / "legacy": the general path for every column
  if (e && (strcmp(e, "lsd") == 0 || strcmp(e, "legacy") == 0)) return false;
  return n >= 2 && n < ((int64_t)1 << 32);
}


int step4_gen_hist(uint32_t* codes, int64_t ldc, const double* cs, int64_t ldcs, int64_t n, const Step4Shared& sh,
                   int c0, int kk, hipStream_t s) {
  PBH_REQUIRE(c0 >= 0 && kk >= 1 && c0 + kk <= sh.k, "step4_gen_hist: columns [%d, %d) outside [0, %d)", c0, c0 + kk,
              sh.k);
  const int cpad = cur_pad();
  const size_t cw = (size_t)8 * 256 * cpad;
  uint32_t* hist = sh.hist + (int64_t)c0 * 65536;
  uint32_t* cls = sh.cls + (int64_t)c0 * 2048;
  int32_t* state = sh.state + c0;
  int32_t* flags = sh.flags + c0;
  PBH_CHECK_HIP(hipMemsetAsync(hist, 0, (size_t)kk * 65536 * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(sh.cur1 + c0 * cw, 0, kk * cw * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(sh.cur2 + (int64_t)c0 * 65536, 0, (size_t)kk * 65536 * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(sh.curF + c0 * cw, 0, kk * cw * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(cls, 0, (size_t)kk * 2048 * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(state, 0, (size_t)kk * 4, s));
  PBH_CHECK_HIP(hipMemsetAsync(flags, 0, (size_t)kk * 4, s));
  // >= 64 K codes per block and at most 64 blocks per column: every block flushes its non-empty
  // counters with global atomics (~64 K each), which the PMC pass counted as ~2 GB of writes at
  // 256 blocks per column (pmc_traffic_r72_ck1.json).  32 and 128 blocks measured no better
  // (profiles/r04/README_ab.md).
  constexpr int64_t cap = 64;
  int64_t blocks = (n + 65535) / 65536;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (blocks >= 8) blocks &= ~(int64_t)7;  // k_hist16c: 8 tile classes
  if (blocks % 8 == 0 && hist_class_major())
    PBH_TIMED(kKHist16, s,
              hipLaunchKernelGGL(k_hist16c, dim3((unsigned)blocks, (unsigned)kk), dim3(1024), 0, s, codes, ldc, n,
                                 hist, cls, state, nullptr, msd_tile_log()));
  else
    PBH_TIMED(kKHist16, s,
              hipLaunchKernelGGL(k_hist16, dim3((unsigned)blocks, (unsigned)kk), dim3(1024), 0, s, codes, ldc, n, hist,
                                 cls, state, nullptr, msd_tile_log()));
  PBH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_hist16_scan, dim3((unsigned)kk), dim3(1024), 0, s, hist, n, sh.start + (int64_t)c0 * 65537,
                     sh.tpre + (int64_t)c0 * 257, cls, sh.cstart + (int64_t)c0 * 2048, state, flags, nullptr,
                     msd_tile_log());
  PBH_CHECK_LAUNCH();
  if (!cs) return PBH_OK;
  return step4_gen_adapt(codes, ldc, cs, ldcs, n, sh, c0, kk, s);
}

int step4_gen_adapt(uint32_t* codes, int64_t ldc, const double* cs, int64_t ldcs, int64_t n, const Step4Shared& sh,
                    int c0, int kk, hipStream_t s) {
  PBH_REQUIRE(c0 >= 0 && kk >= 1 && c0 + kk <= sh.k, "step4_gen_adapt: columns [%d, %d) outside [0, %d)", c0,
              c0 + kk, sh.k);
  const int cpad = cur_pad();
  const size_t cw = (size_t)8 * 256 * cpad;
  uint32_t* hist = sh.hist + (int64_t)c0 * 65536;
  uint32_t* cls = sh.cls + (int64_t)c0 * 2048;
  int32_t* state = sh.state + c0;
  int32_t* flags = sh.flags + c0;
  int32_t* retry = sh.retry + c0;
  int64_t blocks = (n + 65535) / 65536;
  if (blocks > 64) blocks = 64;
  if (blocks < 1) blocks = 1;
  if (blocks >= 8) blocks &= ~(int64_t)7;  // k_hist16c: 8 tile classes
  // the re-code of the columns that are not flat: every kernel exits at once for the others
  hipLaunchKernelGGL(k_adapt_reset, dim3((unsigned)kk), dim3(1024), 0, s, state, flags, retry, hist,
                     sh.cur1 + c0 * cw, sh.cur2 + (int64_t)c0 * 65536, sh.curF + c0 * cw, cls,
                     sh.seghist + (int64_t)c0 * kAdaptSegments, cpad);
  PBH_CHECK_LAUNCH();
  // one column (a lane's re-code, kk = 1): enough blocks to fill the chip; all columns: 64 each
  const unsigned sblocks = kk == 1 ? 512u : 64u;
  hipLaunchKernelGGL(k_seg_hist, dim3(sblocks, (unsigned)kk), dim3(1024), 0, s, cs, ldcs, n, retry,
                     sh.seghist + (int64_t)c0 * kAdaptSegments);
  PBH_CHECK_LAUNCH();
  uint32_t* amap = sh.amap + (int64_t)c0 * kAdaptMapWords;
  hipLaunchKernelGGL(k_seg_map, dim3((unsigned)kk), dim3(1024), 0, s, sh.seghist + (int64_t)c0 * kAdaptSegments, retry,
                     amap);
  PBH_CHECK_LAUNCH();
  const int64_t cb = (n + 256 * 16 - 1) / (256 * 16);
  hipLaunchKernelGGL(k_make_codes_adapt, dim3((unsigned)(cb < 1024 ? (cb < 1 ? 1 : cb) : 1024), (unsigned)kk),
                     dim3(256), 0, s, cs, ldcs, n, retry, amap, codes, ldc);
  PBH_CHECK_LAUNCH();
  // (not timed as k_hist16: a re-count, where k_hist16's bytes per launch are all the columns.)
  // One column: the full-LDS count (the column read once; k_hist16_q's four quarters read it four
  // times), on as many blocks as k_hist16 gives a column (each flushes ~64 K counters with global
  // atomics); several: k_hist16_q, whose no-op blocks for the columns that need no re-count hold
  // 32 KiB instead of 136 (the gate is only known on the device)
  if (kk == 1) {
    if (blocks % 8 == 0 && hist_class_major())
      hipLaunchKernelGGL(k_hist16c, dim3((unsigned)blocks, 1), dim3(1024), 0, s, codes, ldc, n, hist, cls, state,
                         retry, msd_tile_log());
    else
      hipLaunchKernelGGL(k_hist16, dim3((unsigned)blocks, 1), dim3(1024), 0, s, codes, ldc, n, hist, cls, state, retry,
                         msd_tile_log());
  } else {
    hipLaunchKernelGGL(k_hist16_q, dim3((unsigned)blocks, (unsigned)kk, 4), dim3(1024), 0, s, codes, ldc, n, hist, cls,
                       state, retry, msd_tile_log());
  }
  PBH_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_hist16_scan, dim3((unsigned)kk), dim3(1024), 0, s, hist, n, sh.start + (int64_t)c0 * 65537,
                     sh.tpre + (int64_t)c0 * 257, cls, sh.cstart + (int64_t)c0 * 2048, state, flags, retry,
                     msd_tile_log());
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int step4_gen_column(int c, const uint32_t* codes, const double* cs, int64_t n, const Step4Shared& sh,
                     const Step4Column& cb, hipStream_t s) {
  const uint32_t* start = sh.start + (int64_t)c * 65537;
  const int32_t* state = sh.state + c;
  const int tlog = msd_tile_log();
  const int64_t t1 = (n + ((int64_t)1 << tlog) - 1) >> tlog;
  const uint32_t* cst = sh.cstart + (int64_t)c * 2048;  // per tile class cursors (k_msd1x)
  uint32_t* cur1 = sh.cur1 + (int64_t)c * 8 * 256 * cur_pad();
  uint32_t* cur2 = sh.cur2 + (int64_t)c * 65536;
  const uint32_t* tp = sh.tpre + (int64_t)c * 257;
  if (tlog == 13) {
    PBH_TIMED(kKMsd1, s,
              hipLaunchKernelGGL((k_msd1x<1024, 8>), dim3((unsigned)t1), dim3(1024), 0, s, codes, n, start, cur1,
                                 cb.keys32, cb.rows1, cst, cur_pad(), state));
    PBH_CHECK_LAUNCH();
    PBH_TIMED(kKMsd2, s,
              hipLaunchKernelGGL((k_msd2x<1024, 8>), dim3((unsigned)(t1 + 256)), dim3(1024), 0, s, cb.keys32, cb.rows1,
                                 start, tp, cur2, cb.keys16, cb.rows2, state));
  } else {
    PBH_TIMED(kKMsd1, s,
              hipLaunchKernelGGL((k_msd1x<256, 16>), dim3((unsigned)t1), dim3(256), 0, s, codes, n, start, cur1,
                                 cb.keys32, cb.rows1, cst, cur_pad(), state));
    PBH_CHECK_LAUNCH();
    PBH_TIMED(kKMsd2, s,
              hipLaunchKernelGGL((k_msd2x<512, 8>), dim3((unsigned)(t1 + 256)), dim3(512), 0, s, cb.keys32, cb.rows1,
                                 start, tp, cur2, cb.keys16, cb.rows2, state));
  }
  PBH_CHECK_LAUNCH();
  {
    int shifts[4];
    const int nl = place_levels(n, shifts);
    const int s_top = nl ? shifts[nl - 1] : kGenPlaceShift;
    // k_finish_q over 512 threads, 2048 bins, the run members' CS values read in pass 2 (r4s-r4u:
    // 23.2-23.6 against 23.9-24.5 ms per step with 1024 bins; 512 bins 25.7-26.2; the 256-thread
    // form, the LDS-queued CS reads, both buckets' phases in one pass and the XCD-class segmented
    // output were measured and removed: profiles/r03/, r04/README_ab.md)
    uint32_t* gc = sh.curF + (int64_t)c * 8 * 256 * cur_pad();
    PBH_TIMED(kKFinish, s,
              hipLaunchKernelGGL((k_finish_q<PBH_FINISH_BINS, PBH_FINISH_NT, false>), dim3(65536 / 2), dim3(PBH_FINISH_NT), 0, s, cb.keys16,
                                 cb.rows2, cs, start, s_top, gc, cur_pad(), cb.pairs[0], sh.flags + c, state));
  }
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

int step4_gen_place_passes(int c, int64_t n, const Step4Shared& sh, const Step4Column& cb, hipStream_t s,
                           int* out_buf) {
  int32_t* state = sh.flags + c;
  int shifts[4];
  int nl = place_levels(n, shifts);
  if (nl > 0) --nl;  // the finish scattered the top level
  int cur = 0;
  const int64_t tiles = (n + kTileP - 1) / kTileP;
  for (int l = nl - 1; l >= 0; --l) {
    const int64_t ncur = (n >> shifts[l]) + 1;
    uint32_t* cr = cb.pcur[l & 1];
    PBH_CHECK_HIP(hipMemsetAsync(cr, 0, (size_t)ncur * 4, s));
    PBH_TIMED(kKPlaceMsd, s,
              hipLaunchKernelGGL(k_place_msdo, dim3((unsigned)tiles), dim3(kTO), 0, s, cb.pairs[cur], n, shifts[l], cr,
                                 cb.pairs[cur ^ 1], state));
    PBH_CHECK_LAUNCH();
    cur ^= 1;
  }
  *out_buf = cur;
  return PBH_OK;
}

}  // namespace pbh
