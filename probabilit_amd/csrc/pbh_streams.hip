// numpy's MT19937 and PCG64 streams generated on the GPU, bit for bit.
//
//   pbh_mt19937_random : RandomState.random((nrows, d))   check_random_state(int | None | RandomState)
//                        (modeling.py:484-486) -- np.random.RandomState's MT19937
//   pbh_pcg64_random   : Generator.random((nrows, d))     random_state=np.random.Generator
//                        (modeling.py:484-486), and the uniform draws of scipy's
//                        LatinHypercube._random_lhs (rng.uniform(size=(n, d)))
//
// MT19937: one workgroup per segment of J output words.  A workgroup moves numpy's key block
// to its segment with the jump polynomials x^(2^i) mod phi (pbh_mt.h), then twists forward in
// LDS (624 lanes, three dependency phases per twist) and writes tempered words; a second
// kernel pairs words into doubles in the caller's column-major layout.
// PCG64: each lane jumps its 128-bit LCG state to its row's first draw (tabulated 2^i
// strides) and steps d times.
#include <mutex>
#include <vector>

#include "pbh_error.h"
#include "pbh_mt.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kMtBlock = 640;  // lanes 0..623 own one word of the 624-word window

// W_g -> W_{g+624} on the LDS window a[0..623] (numpy's mt19937_gen, three parallel phases:
// words 0..226 read only old words, 227..453 need phase-1 words, 454..623 phase-2 words).
__device__ void twist_lds(uint32_t* a) {
  const int m = threadIdx.x;
  uint32_t v = 0;
  if (m < 227) v = mt::next_word(a[m], a[m + 1], a[m + 397]);
  __syncthreads();
  if (m < 227) a[m] = v;
  __syncthreads();
  if (m >= 227 && m < 454) v = mt::next_word(a[m], a[m + 1], a[m - 227]);
  __syncthreads();
  if (m >= 227 && m < 454) a[m] = v;
  __syncthreads();
  if (m >= 454 && m < mt::kN) v = mt::next_word(a[m], a[m == mt::kN - 1 ? 0 : m + 1], a[m - 227]);
  __syncthreads();
  if (m >= 454 && m < mt::kN) a[m] = v;
  __syncthreads();
}

// E[0..623] <- sum_i p[i] W_{+i}.  Chunked Horner in T^624: with E[624..1247] = the next 624
// words, T^r W = E[r .. r + 623] for r < 624, so chunk q of p contributes
// acc[m] ^= E[r + m] for every set coefficient 624 q + r.  The coefficient loop is uniform
// across the workgroup (scalar loads of p, no divergence).
__device__ void jump_lds(uint32_t* E, uint32_t* acc, const uint64_t* __restrict__ p) {
  const int m = threadIdx.x;
  const int mm = m < mt::kN ? m : 0;
  if (m < mt::kN) {
    E[mt::kN + m] = E[m];
    acc[m] = 0;
  }
  __syncthreads();
  twist_lds(E + mt::kN);
  for (int q = mt::kChunks - 1; q >= 0; --q) {
    if (q < mt::kChunks - 1) twist_lds(acc);
    uint32_t x = acc[mm];
    const int b0 = mt::kN * q, b1 = b0 + mt::kN;  // coefficient range [b0, b1)
    for (int w = b0 >> 6; w <= (b1 - 1) >> 6; ++w) {
      uint64_t bits = p[w];
      const int lo = w * 64;
      if (lo < b0) bits &= ~0ull << (b0 - lo);
      if (lo + 64 > b1) bits &= (b1 - lo) >= 64 ? ~0ull : ((1ull << (b1 - lo)) - 1);
      while (bits) {
        const int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        x ^= E[lo + b - b0 + mm];
      }
    }
    __syncthreads();
    if (m < mt::kN) acc[m] = x;
    __syncthreads();
  }
  if (m < mt::kN) E[m] = acc[m];
  __syncthreads();
}

// Window W_{target - 1} (exact in its 19937 state bits) from numpy's key block (W_0).
__device__ void window_before(uint32_t* E, uint32_t* acc, const uint32_t* __restrict__ key0, int64_t target,
                              const uint64_t* __restrict__ jt) {
  const int m = threadIdx.x;
  if (m < mt::kN) E[m] = key0[m];
  __syncthreads();
  const int64_t D = target - 1;
  for (int i = 0; i < mt::kJumpBits; ++i)
    if ((D >> i) & 1) jump_lds(E, acc, jt + (size_t)i * mt::kPolyWords);
}

// Tempered words g in [pos + o0, pos + o1) of the sequence, out[g - pos]; segment = blockIdx.
// `pos` = absolute word of out[0].
__global__ __launch_bounds__(kMtBlock) void k_mt_words(const uint32_t* __restrict__ key0, int64_t pos, int64_t total,
                                                       int64_t seg, const uint64_t* __restrict__ jt,
                                                       uint32_t* __restrict__ out) {
  __shared__ uint32_t E[2 * mt::kN];
  __shared__ uint32_t acc[mt::kN];
  const int m = threadIdx.x;
  const int64_t o0 = (int64_t)blockIdx.x * seg;
  const int64_t o1 = o0 + seg < total ? o0 + seg : total;
  const int64_t g0 = pos + o0, g1 = pos + o1;
  int64_t wstart = 0;
  if (g0 > 0) {
    window_before(E, acc, key0, g0, jt);
    wstart = g0 - 1;  // word 0's low bits are not state bits: never emitted (g >= g0)
  } else {
    if (m < mt::kN) E[m] = key0[m];
    __syncthreads();
  }
  while (true) {
    if (m < mt::kN) {
      const int64_t g = wstart + m;
      if (g >= g0 && g < g1) out[g - pos] = mt::temper(E[m]);
    }
    if (wstart + mt::kN >= g1) break;
    twist_lds(E);
    wstart += mt::kN;
  }
}

// numpy's key block b (x_{624 b} .. x_{624 b + 623}) for the state write-back.
__global__ __launch_bounds__(kMtBlock) void k_mt_block(const uint32_t* __restrict__ key0, int64_t b,
                                                       const uint64_t* __restrict__ jt, uint32_t* __restrict__ key_out) {
  __shared__ uint32_t E[2 * mt::kN];
  __shared__ uint32_t acc[mt::kN];
  const int m = threadIdx.x;
  if (b == 0) {
    if (m < mt::kN) key_out[m] = key0[m];
    return;
  }
  window_before(E, acc, key0, (int64_t)mt::kN * b, jt);
  if (m < mt::kN) key_out[m] = m < mt::kN - 1 ? E[m + 1] : mt::next_word(E[0], E[1], E[mt::kM]);
}

// q[c * ldq + r] = double from words 2 t, 2 t + 1 with t = r * d + c (row-major draws).
__global__ __launch_bounds__(256) void k_mt_doubles(const uint32_t* __restrict__ w, int64_t nrows, int d,
                                                    double* __restrict__ q, int64_t ldq) {
  const int64_t total = nrows * d;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t c = i / nrows, r = i - c * nrows;
    const int64_t t = r * d + c;
    q[c * ldq + r] = mt::next_double(w[2 * t], w[2 * t + 1]);
  }
}

// ---------------------------------------------------------------- PCG64
__global__ __launch_bounds__(256) void k_pcg_random(const pcg::u128* __restrict__ table, uint64_t s_lo, uint64_t s_hi,
                                                    uint64_t inc_lo, uint64_t inc_hi, int64_t draw0, int64_t nrows,
                                                    int d, double* __restrict__ q, int64_t ldq) {
  const pcg::u128 inc = ((pcg::u128)inc_hi << 64) | inc_lo;
  const pcg::u128 s0 = ((pcg::u128)s_hi << 64) | s_lo;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * 256) {
    pcg::u128 s = pcg::advance(s0, (uint64_t)(draw0 + r * d), table);
    for (int c = 0; c < d; ++c) {
      s = s * pcg::kMult + inc;
      q[(int64_t)c * ldq + r] = pcg::to_double(pcg::output(s));
    }
  }
}

// ---------------------------------------------------------------- scrambled Halton
// scipy.stats.qmc.Halton._random -> van_der_corput(scramble=True) per dimension
// (scipy:stats/_qmc.py; the loop of scipy:stats/_qmc_cy.pyx): for index i,
//   s = 0; b2r = 1/base; repeat count times: s += perm[j][i % base] * b2r; b2r /= base; i /= base
// with count = ceil(54 / log2(base)) - 1 (every digit permuted, zeros included).  b2r comes
// from a host table built by the same repeated IEEE divisions; each += rounds separately
// (-ffp-contract=off), so the points are bit-identical.
struct HaltonDim {
  int32_t base, count;
  int64_t perm_off, b2r_off;
};

__global__ __launch_bounds__(256) void k_fill_halton(const HaltonDim* __restrict__ dims,
                                                     const int32_t* __restrict__ perms,
                                                     const double* __restrict__ b2r, int64_t row0, int64_t nrows,
                                                     int col0, int ncols, double* __restrict__ q, int64_t ldq) {
  const int c = blockIdx.y;
  const HaltonDim hd = dims[col0 + c];
  const int32_t* P = perms + hd.perm_off;
  const double* B = b2r + hd.b2r_off;
  const uint64_t base = (uint64_t)hd.base;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * 256) {
    uint64_t idx = (uint64_t)(row0 + r);
    double s = 0.0;
    for (int j = 0; j < hd.count; ++j) {
      uint64_t quo, rem;
      if (idx <= 0xFFFFFFFFull) {
        const uint32_t i32 = (uint32_t)idx;
        quo = i32 / (uint32_t)base;
        rem = i32 - (uint32_t)quo * (uint32_t)base;
      } else {
        quo = idx / base;
        rem = idx - quo * base;
      }
      s = s + (double)P[j * hd.base + rem] * B[j];
      idx = quo;
    }
    q[(int64_t)c * ldq + r] = s;
  }
}

// ---------------------------------------------------------------- host
struct JumpTable {
  std::vector<uint64_t> words;
  bool ok = false;
};

const JumpTable& jump_table() {
  static JumpTable t;
  static std::once_flag once;
  std::call_once(once, [] { t.ok = mt::host::jump_table(t.words); });
  return t;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
constexpr size_t kJtBytes = (size_t)mt::kJumpBits * mt::kPolyWords * 8;

int64_t mt_segment(int64_t total) {
  int64_t seg = 4096;
  while (seg * 2048 < total) seg *= 2;
  return seg;
}

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_mt19937_workspace_size(int64_t nrows, int32_t d, size_t* bytes) {
  PBH_REQUIRE(bytes && nrows >= 0 && d >= 0, "pbh_mt19937_workspace_size: bad arguments");
  *bytes = align256(kJtBytes) + align256(mt::kN * 4) * 2 + align256((size_t)2 * nrows * d * 4 + 8);
  return PBH_OK;
}

namespace pbh {
namespace {
// Uploads the jump table and key block into the workspace; returns the carved pointers.
int mt_setup(const uint32_t* key_host, void* ws, size_t ws_bytes, size_t need, hipStream_t s, uint64_t** jt_dev,
             uint32_t** key_dev, uint32_t** key_out_dev, uint32_t** words) {
  if (ws_bytes < need) {
    set_error("MT19937: workspace %zu < %zu bytes", ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  const JumpTable& jt = jump_table();
  if (!jt.ok) {
    set_error("MT19937: characteristic polynomial not found (Berlekamp-Massey)");
    return PBH_ERR_INVALID;
  }
  char* p = (char*)ws;
  *jt_dev = (uint64_t*)p;
  p += align256(kJtBytes);
  *key_dev = (uint32_t*)p;
  p += align256(mt::kN * 4);
  *key_out_dev = (uint32_t*)p;
  p += align256(mt::kN * 4);
  *words = (uint32_t*)p;
  PBH_CHECK_HIP(hipMemcpyAsync(*jt_dev, jt.words.data(), kJtBytes, hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(*key_dev, key_host, mt::kN * 4, hipMemcpyHostToDevice, s));
  return PBH_OK;
}
}  // namespace
}  // namespace pbh

extern "C" int pbh_mt19937_random(const uint32_t* key_host, int32_t pos, int64_t row0, int64_t nrows, int32_t d,
                                  double* q, int64_t ldq, void* ws, size_t ws_bytes, void* stream) {
  PBH_REQUIRE(key_host && ws && row0 >= 0 && nrows >= 0 && d >= 0 && pos >= 0 && pos <= mt::kN,
              "pbh_mt19937_random: bad arguments");
  PBH_REQUIRE(nrows * (int64_t)d == 0 || (q && ldq >= nrows), "pbh_mt19937_random: bad output");
  size_t need = 0;
  pbh_mt19937_workspace_size(nrows, d, &need);
  hipStream_t s = as_stream(stream);
  uint64_t* jt_dev;
  uint32_t *key_dev, *key_out_dev, *words;
  int st = mt_setup(key_host, ws, ws_bytes, need, s, &jt_dev, &key_dev, &key_out_dev, &words);
  if (st) return st;
  const int64_t total = 2 * nrows * (int64_t)d;
  if (total > 0) {
    const int64_t seg = mt_segment(total);
    const int64_t nseg = (total + seg - 1) / seg;
    const int64_t start = (int64_t)pos + 2 * row0 * (int64_t)d;  // absolute word of the shard's first draw
    PBH_TIMED(kKStreams, s,
              hipLaunchKernelGGL(k_mt_words, dim3((unsigned)nseg), dim3(kMtBlock), 0, s, key_dev, start, total, seg,
                                 jt_dev, words);
              hipLaunchKernelGGL(k_mt_doubles, dim3(grid_for(nrows * d, 256, 65536)), dim3(256), 0, s, words, nrows,
                                 (int)d, q, ldq));
    PBH_CHECK_LAUNCH();
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // key_host / jump table copies are pageable
  return PBH_OK;
}

extern "C" int pbh_mt19937_advance(const uint32_t* key_host, int32_t pos, int64_t nwords, uint32_t* key_out_host,
                                   int32_t* pos_out, void* ws, size_t ws_bytes, void* stream) {
  PBH_REQUIRE(key_host && key_out_host && pos_out && ws && nwords >= 0 && pos >= 0 && pos <= mt::kN,
              "pbh_mt19937_advance: bad arguments");
  size_t need = 0;
  pbh_mt19937_workspace_size(0, 0, &need);
  hipStream_t s = as_stream(stream);
  uint64_t* jt_dev;
  uint32_t *key_dev, *key_out_dev, *words;
  int st = mt_setup(key_host, ws, ws_bytes, need, s, &jt_dev, &key_dev, &key_out_dev, &words);
  if (st) return st;
  int64_t b = 0, np = pos;
  if (nwords > 0) {  // numpy holds the block of the last word drawn, pos in [1, 624]
    b = (pos + nwords - 1) / mt::kN;
    np = pos + nwords - (int64_t)mt::kN * b;
  }
  hipLaunchKernelGGL(k_mt_block, dim3(1), dim3(kMtBlock), 0, s, key_dev, b, jt_dev, key_out_dev);
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipMemcpyAsync(key_out_host, key_out_dev, mt::kN * 4, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  *pos_out = (int32_t)np;
  return PBH_OK;
}

extern "C" int pbh_pcg64_workspace_size(size_t* bytes) {
  PBH_REQUIRE(bytes, "pbh_pcg64_workspace_size: bad arguments");
  *bytes = 128 * sizeof(pcg::u128);
  return PBH_OK;
}

extern "C" int pbh_pcg64_random(const uint64_t* state_host, const uint64_t* inc_host, int64_t draw0, int64_t nrows,
                                int32_t d, double* q, int64_t ldq, void* ws, size_t ws_bytes, void* stream) {
  PBH_REQUIRE(state_host && inc_host && ws && nrows >= 0 && d >= 0 && draw0 >= 0, "pbh_pcg64_random: bad arguments");
  PBH_REQUIRE(nrows * (int64_t)d == 0 || (q && ldq >= nrows), "pbh_pcg64_random: bad output");
  PBH_REQUIRE(ws_bytes >= 128 * sizeof(pcg::u128), "pbh_pcg64_random: workspace too small");
  hipStream_t s = as_stream(stream);
  const pcg::u128 inc = ((pcg::u128)inc_host[1] << 64) | inc_host[0];
  std::vector<pcg::u128> table(128);
  pcg::jump_table(inc, table.data());
  PBH_CHECK_HIP(hipMemcpyAsync(ws, table.data(), 128 * sizeof(pcg::u128), hipMemcpyHostToDevice, s));
  if (nrows * (int64_t)d > 0) {
    PBH_TIMED(kKStreams, s,
              hipLaunchKernelGGL(k_pcg_random, dim3(grid_for(nrows, 256, 65536)), dim3(256), 0, s,
                                 (const pcg::u128*)ws, state_host[0], state_host[1], inc_host[0], inc_host[1], draw0,
                                 nrows, (int)d, q, ldq));
    PBH_CHECK_LAUNCH();
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // `table` is pageable and goes out of scope
  return PBH_OK;
}

extern "C" int pbh_halton_workspace_size(const int32_t* bases_host, const int32_t* counts_host, int d, size_t* bytes) {
  PBH_REQUIRE(bases_host && counts_host && bytes && d >= 0, "pbh_halton_workspace_size: bad arguments");
  size_t perm = 0, b2r = 0;
  for (int c = 0; c < d; ++c) {
    perm += (size_t)counts_host[c] * bases_host[c];
    b2r += (size_t)counts_host[c];
  }
  *bytes = align256((size_t)d * sizeof(HaltonDim)) + align256(perm * 4) + align256(b2r * 8);
  return PBH_OK;
}

extern "C" int pbh_fill_halton(const int32_t* bases_host, const int32_t* counts_host, const int32_t* perms_host, int d,
                               int64_t row0, int64_t nrows, int col0, int ncols, double* q, int64_t ldq, void* ws,
                               size_t ws_bytes, void* stream) {
  PBH_REQUIRE(bases_host && counts_host && perms_host && ws && d >= 0 && row0 >= 0 && nrows >= 0,
              "pbh_fill_halton: bad arguments");
  PBH_REQUIRE(col0 >= 0 && ncols >= 0 && col0 + ncols <= d && (nrows * ncols == 0 || (q && ldq >= nrows)),
              "pbh_fill_halton: bad output range");
  size_t need = 0;
  pbh_halton_workspace_size(bases_host, counts_host, d, &need);
  if (ws_bytes < need) {
    set_error("pbh_fill_halton: workspace %zu < %zu bytes", ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  std::vector<HaltonDim> dims(d);
  std::vector<double> b2r;
  int64_t poff = 0;
  for (int c = 0; c < d; ++c) {
    PBH_REQUIRE(bases_host[c] >= 2 && counts_host[c] >= 1, "pbh_fill_halton: base < 2 or no permutation");
    dims[c] = HaltonDim{bases_host[c], counts_host[c], poff, (int64_t)b2r.size()};
    double v = 1.0 / (double)bases_host[c];
    for (int j = 0; j < counts_host[c]; ++j) {
      b2r.push_back(v);
      v /= (double)bases_host[c];
    }
    poff += (int64_t)counts_host[c] * bases_host[c];
  }
  hipStream_t s = as_stream(stream);
  char* p = (char*)ws;
  HaltonDim* dims_dev = (HaltonDim*)p;
  p += align256((size_t)d * sizeof(HaltonDim));
  int32_t* perms_dev = (int32_t*)p;
  p += align256((size_t)poff * 4);
  double* b2r_dev = (double*)p;
  if (d > 0) {
    PBH_CHECK_HIP(hipMemcpyAsync(dims_dev, dims.data(), (size_t)d * sizeof(HaltonDim), hipMemcpyHostToDevice, s));
    PBH_CHECK_HIP(hipMemcpyAsync(perms_dev, perms_host, (size_t)poff * 4, hipMemcpyHostToDevice, s));
    PBH_CHECK_HIP(hipMemcpyAsync(b2r_dev, b2r.data(), b2r.size() * 8, hipMemcpyHostToDevice, s));
  }
  if (nrows > 0 && ncols > 0) {
    PBH_TIMED(kKStreams, s,
              hipLaunchKernelGGL(k_fill_halton, dim3(grid_for(nrows, 256, 16384), (unsigned)ncols), dim3(256), 0, s,
                                 dims_dev, perms_dev, b2r_dev, row0, nrows, col0, ncols, q, ldq));
    PBH_CHECK_LAUNCH();
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // host tables are pageable and go out of scope
  return PBH_OK;
}
