// scipy.stats.qmc.LatinHypercube(d, rng).random(n) bit for bit: the reference's own LHS stream
// (modeling.py:480,488 -> scipy:stats/_qmc.py LatinHypercube._random_lhs), as an opt-in parity
// mode next to the native counter-based design of pbh_ppf.hip.
//
//   u     = rng.uniform(size=(n, d))                 draws 0 .. n d - 1 of the engine's PCG64,
//                                                    row-major: on the device (pbh_pcg64_random)
//   perms = d shuffles of arange(1, n + 1)           numpy Generator.shuffle: for i = n-1 .. 1,
//                                                    j = random_interval(i) (masked rejection on
//                                                    buffered 32-bit halves), swap: on the device
//                                                    (pbh_lhs_dev.hip), host threads as fallback
//   q     = (perms.T - u) / n                        on the device (k_lhs_combine)
//
// The shuffles are one sequential stream (a column's rejections decide where the next column's
// draws start).  pbh_lhs_reference decodes them on the device (pbh_lhs_dev.hip: banded parallel
// classification, a host walk of the ambiguous draws, an exact check of every decision); the
// host shuffles here are its fallback and pbh_lhs_reference_perms: a counting pass walks the
// stream once to find each column's starting state, then the columns are shuffled in parallel
// threads, each replaying its own stretch of the stream with the swap targets prefetched.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "pbh_error.h"
#include "pbh_lhs_dev.h"
#include "pbh_mt.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

using pcg::u128;

// numpy's PCG64 bit generator with the 32-bit buffer of next_uint32 (numpy/random/src/pcg64).
struct Pcg64 {
  u128 s, inc;
  bool has32;
  uint32_t buf;
  uint64_t next64() {
    s = s * pcg::kMult + inc;
    return pcg::output(s);
  }
  uint32_t next32() {
    if (has32) {
      has32 = false;
      return buf;
    }
    const uint64_t v = next64();
    has32 = true;
    buf = (uint32_t)(v >> 32);
    return (uint32_t)v;
  }
  // numpy's random_interval(bitgen, max) for 0 < max <= 0xFFFFFFFF
  uint32_t interval32(uint32_t mx) {
    uint32_t mask = mx;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    while ((v = (next32() & mask)) > mx) {
    }
    return v;
  }
};

// One column's shuffle of arange(1, n + 1) (Generator.shuffle -> _shuffle_raw, i = n - 1 .. 1).
void shuffle_column(Pcg64& g, int64_t n, int32_t* perm) {
  for (int64_t i = 0; i < n; ++i) perm[i] = (int32_t)(i + 1);
  constexpr int kAhead = 32;  // swap targets drawn and prefetched this far ahead of the swaps
  uint32_t js[kAhead];
  int64_t i = n - 1;
  while (i >= 1) {
    const int m = (int)std::min<int64_t>(kAhead, i);
    for (int b = 0; b < m; ++b) {
      js[b] = g.interval32((uint32_t)(i - b));
      __builtin_prefetch(perm + js[b], 1);
    }
    for (int b = 0; b < m; ++b) {
      const int64_t a = i - b;
      const int32_t t = perm[a];
      perm[a] = perm[js[b]];
      perm[js[b]] = t;
    }
    i -= m;
  }
}

// The stream walk of one column without the array: only the draws it consumes.
void skip_column(Pcg64& g, int64_t n) {
  for (int64_t i = n - 1; i >= 1; --i) (void)g.interval32((uint32_t)i);
}

int worker_count(int d) {
  int hw = (int)std::thread::hardware_concurrency();
  if (hw <= 0) hw = 1;
  int cap = 16;  // the GPU box's CPU share per GPU
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) cap = std::min(cap, v);
  }
  return std::max(1, std::min({d, hw, cap}));
}

__global__ __launch_bounds__(256) void k_lhs_combine(const int32_t* __restrict__ perms, double* __restrict__ q,
                                                     int64_t n, int d, int64_t ldq, int32_t* __restrict__ strata,
                                                     int64_t lds) {
  const double dn = (double)n;
  const int64_t total = n * (int64_t)d;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int64_t c = e / n, r = e - c * n;
    double* p = q + c * ldq + r;
    *p = ((double)perms[e] - *p) / dn;  // (perms - samples) / n: subtract, then divide
    if (strata) strata[c * lds + r] = perms[e] - 1;
  }
}

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_lhs_reference_perms(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32,
                                       uint32_t buf32, int64_t n, int32_t d, int32_t* perms_host,
                                       uint64_t* state_out_host) {
  PBH_REQUIRE(state_host && inc_host && n >= 1 && n < ((int64_t)1 << 31) && d >= 0 && (d == 0 || perms_host),
              "pbh_lhs_reference_perms: bad arguments");
  Pcg64 g{((u128)state_host[1] << 64) | state_host[0], ((u128)inc_host[1] << 64) | inc_host[0], has32 != 0, buf32};
  const int workers = worker_count(d);
  if (workers <= 1) {
    for (int c = 0; c < d; ++c) shuffle_column(g, n, perms_host + (int64_t)c * n);
  } else {
    std::vector<Pcg64> start(d);
    for (int c = 0; c < d; ++c) {  // counting pass: each column's starting state
      start[c] = g;
      skip_column(g, n);
    }
    std::vector<std::thread> pool;
    for (int w = 0; w < workers; ++w)
      pool.emplace_back([&, w] {
        for (int c = w; c < d; c += workers) {
          Pcg64 gc = start[c];
          shuffle_column(gc, n, perms_host + (int64_t)c * n);
        }
      });
    for (auto& t : pool) t.join();
  }
  if (state_out_host) {
    state_out_host[0] = (uint64_t)g.s;
    state_out_host[1] = (uint64_t)(g.s >> 64);
    state_out_host[2] = g.has32 ? 1u : 0u;
    state_out_host[3] = g.buf;
  }
  return PBH_OK;
}

extern "C" int pbh_lhs_reference_workspace_size(int64_t n, int32_t d, size_t* bytes) {
  PBH_REQUIRE(bytes && n >= 0 && d >= 0, "pbh_lhs_reference_workspace_size: bad arguments");
  *bytes = (((size_t)n * d * 4 + 255) & ~(size_t)255) + 128 * sizeof(u128);
  return PBH_OK;
}

extern "C" int pbh_lhs_reference(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32, uint32_t buf32,
                                 int64_t n, int32_t d, double* q, int64_t ldq, void* ws, size_t ws_bytes,
                                 void* stream) {
  return pbh_lhs_reference_strata(state_host, inc_host, has32, buf32, n, d, q, ldq, nullptr, 0, ws, ws_bytes, stream);
}

extern "C" int pbh_lhs_reference_strata(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32,
                                        uint32_t buf32, int64_t n, int32_t d, double* q, int64_t ldq, int32_t* strata,
                                        int64_t lds, void* ws, size_t ws_bytes, void* stream) {
  PBH_REQUIRE(state_host && inc_host && n >= 1 && n < ((int64_t)1 << 31) && d >= 1 && q && ldq >= n && ws &&
                  (!strata || lds >= n),
              "pbh_lhs_reference: bad arguments");
  size_t need = 0;
  pbh_lhs_reference_workspace_size(n, d, &need);
  if (ws_bytes < need) {
    set_error("pbh_lhs_reference: workspace %zu < %zu bytes", ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  int32_t* perms_dev = (int32_t*)ws;
  void* pcg_ws = (char*)ws + (((size_t)n * d * 4 + 255) & ~(size_t)255);
  // u and the shuffles on the device (pbh_lhs_dev.hip), or, when its check fails, u again and
  // the shuffles on the host: draws 0 .. n d - 1 row-major into q's column-major layout; the
  // shuffles continue the stream after the n d doubles (uniform() leaves the 32-bit buffer)
  bool done = false;
  int st = lhs_reference_device(state_host, inc_host, has32 != 0, buf32, n, d, q, ldq, perms_dev, s, &done, strata,
                                lds);
  if (st || done) return st;
  st = pbh_pcg64_random(state_host, inc_host, 0, n, d, q, ldq, pcg_ws, 128 * sizeof(u128), stream);
  if (st) return st;
  u128 s0 = ((u128)state_host[1] << 64) | state_host[0];
  const u128 inc = ((u128)inc_host[1] << 64) | inc_host[0];
  std::vector<u128> table(128);
  pcg::jump_table(inc, table.data());
  s0 = pcg::advance(s0, (uint64_t)(n * (int64_t)d), table.data());
  const uint64_t s_after[2] = {(uint64_t)s0, (uint64_t)(s0 >> 64)};
  std::vector<int32_t> perms((size_t)n * d);
  st = pbh_lhs_reference_perms(s_after, inc_host, has32, buf32, n, d, perms.data(), nullptr);
  if (st) return st;
  PBH_CHECK_HIP(hipMemcpyAsync(perms_dev, perms.data(), perms.size() * 4, hipMemcpyHostToDevice, s));
  PBH_TIMED(kKStreams, s,
            hipLaunchKernelGGL(k_lhs_combine, dim3(grid_for(n * (int64_t)d, 256, 65536)), dim3(256), 0, s, perms_dev,
                               q, n, (int)d, ldq, strata, lds));
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // `perms` is pageable and goes out of scope
  return PBH_OK;
}
