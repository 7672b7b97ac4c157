// PermutationCorrelator's randomized hill climb on the device (correlation.py:650-700, with
// CorrelationMatrix.update_column / commit, :875-921, and _error, :582-586).
//
// The loop is sequential across steps (each accept decision changes the state the next step
// reads) and tiny within a step (2 s rows of K values, s <= log2(iterations) + 1), so it runs
// as ONE persistent workgroup of one wave: the K x K correlation matrix lives in LDS, the
// measured columns X_ (K x N, column-major) stay in HBM and are read / swapped in place, and
// the swap index lists of a whole chunk of steps are precomputed by the host (they do not
// depend on the accept decisions: SwapIndexGenerator consumes its permutation identically
// whatever happens).  One launch replaces ~K x iterations Python round trips of the reference.
//
// Bit-exact with numpy: every sum the reference forms is reproduced in numpy's association
// order -- the axis-0 sum over swap pairs sequentially from the first pair, np.average's and
// np.sum's contiguous reductions by numpy's pairwise summation -- and the file is compiled with
// -ffp-contract=off, so on the same initial state and swap lists the decisions, the final
// matrix and the permuted data equal the restatement's (oracle/permcorr.py) bit for bit.
#include "pbh_error.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kMaxK = 128;  // K x K doubles in LDS (128 KB) + 4 K-vectors

// numpy's pairwise_sum over a contiguous run of n values get(lo..lo+n): fewer than 8 values
// sequentially from 0.0; up to 128 values in 8 interleaved partial sums combined as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the tail; longer runs split at n / 2
// rounded down to a multiple of 8, left half + right half.
template <class F>
__device__ double pw_leaf(F& get, int64_t lo, int64_t n) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += get(lo + i);
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = get(lo + j);
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += get(lo + i + j);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += get(lo + i);
  return res;
}

template <class F>
__device__ double pairwise(F& get, int64_t n) {
  struct Frame {
    int64_t lo, n;
    int stage;
    double left;
  };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Frame& f = st[sp];
    if (f.n <= 128) {
      ret = pw_leaf(get, f.lo, f.n);
      --sp;
      continue;
    }
    int64_t n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.stage == 0) {
      f.stage = 1;
      st[sp + 1] = {f.lo, n2, 0, 0.0};
      ++sp;
    } else if (f.stage == 1) {
      f.left = ret;
      f.stage = 2;
      st[sp + 1] = {f.lo + n2, f.n - n2, 0, 0.0};
      ++sp;
    } else {
      ret = f.left + ret;
      --sp;
    }
  }
  return ret;
}

// the weighted squared residuals of the strict upper triangle in np.triu_indices order,
// addressed by flat index (sequential access advances a cursor; a jump re-derives (a, b))
struct TriuTerms {
  const double* corr;
  const double* C;
  const double* W;
  int k;
  int64_t at = -1;
  int a = 0, b = 0;
  __device__ double operator()(int64_t idx) {
    if (idx == at + 1 && at >= 0) {
      if (++b == k) {
        ++a;
        b = a + 1;
      }
    } else {
      a = 0;
      int64_t rem = idx;
      while (rem >= k - 1 - a) {
        rem -= k - 1 - a;
        ++a;
      }
      b = a + 1 + (int)rem;
    }
    at = idx;
    const double d = corr[a * k + b] - C[a * k + b];  // (observed - target) ** 2.0
    return W[a * k + b] * (d * d);
  }
};

struct LdsVec {
  const double* v;
  __device__ double operator()(int64_t i) const { return v[i]; }
};

// One wave.  Step t works on variable col = t % k (every chunk starts at a col-0 step); its
// swap lists are swaps[off[t] .. off[t] + s) (rows i) and the next s entries (rows j).
__global__ __launch_bounds__(64) void k_permcorr(double* __restrict__ xs, double* __restrict__ xo, int64_t ldx,
                                                 int64_t m, int k, double* __restrict__ corr_g,
                                                 const double* __restrict__ prm, const int64_t* __restrict__ swaps,
                                                 const int64_t* __restrict__ off, int64_t nsteps, double tol,
                                                 double* __restrict__ errlog, int64_t* __restrict__ state) {
  extern __shared__ double lds[];
  double* corr = lds;         // k x k, row-major
  double* eo = corr + k * k;  // weighted squared residuals of the old column
  double* en = eo + k;        // ... of the new column
  double* dcol = en + k;      // delta of column col
  double* scl = dcol + k;     // sum of weights row c (np.average's scale)
  __shared__ int accept_sh, stop_sh;
  const double* den = prm;
  const double* C = prm + k;
  const double* W = prm + k + k * k;
  const int lane = threadIdx.x;

  for (int i = lane; i < k * k; i += 64) corr[i] = corr_g[i];
  for (int c = lane; c < k; c += 64) {
    LdsVec row{W + c * k};
    scl[c] = pairwise(row, k);
  }
  if (lane == 0) stop_sh = 0;
  __syncthreads();

  const double mf = (double)m;
  int64_t t = 0;
  for (; t < nsteps; ++t) {
    const int col = (int)(t % k);
    const int64_t o = off[t];
    const int s = (int)((off[t + 1] - o) / 2);
    const int64_t* I = swaps + o;
    const int64_t* J = I + s;
    const double* xcol = xs + (int64_t)col * ldx;
    // delta_numerator (:890-897) and the two weighted residual vectors (:683-687)
    for (int c = lane; c < k; c += 64) {
      const double* xc = xs + (int64_t)c * ldx;
      double acc = 0.0;
      for (int u = 0; u < s; ++u) {
        const double term = (xc[I[u]] - xc[J[u]]) * (xcol[J[u]] - xcol[I[u]]);
        acc = u == 0 ? term : acc + term;
      }
      if (c == col) acc = 0.0;
      const double dc = acc / ((mf * den[c]) * den[col]);
      dcol[c] = dc;
      const double tc = C[col * k + c], w = W[col * k + c];
      const double a = tc - corr[col * k + c];         // target - old (row col)
      const double b = tc - (corr[c * k + col] + dc);  // target - new (column col + delta)
      eo[c] = (a * a) * w;
      en[c] = (b * b) * w;
    }
    __syncthreads();
    if (lane == 0) {
      LdsVec vo{eo}, vn{en};
      const double e_old = pairwise(vo, k) / scl[col];
      const double e_new = pairwise(vn, k) / scl[col];
      accept_sh = e_new < e_old;
    }
    __syncthreads();
    if (accept_sh) {  // commit (:860-873): column col, then row col, then swap the data
      for (int c = lane; c < k; c += 64) corr[c * k + col] += dcol[c];
      __syncthreads();
      for (int c = lane; c < k; c += 64) corr[col * k + c] += dcol[c];
      double* xw = xs + (int64_t)col * ldx;
      for (int u = lane; u < s; u += 64) {
        const double vi = xw[I[u]], vj = xw[J[u]];
        xw[I[u]] = vj;
        xw[J[u]] = vi;
        if (xo) {
          double* xq = xo + (int64_t)col * ldx;
          const double qi = xq[I[u]], qj = xq[J[u]];
          xq[I[u]] = qj;
          xq[J[u]] = qi;
        }
      }
      __threadfence_block();
      __syncthreads();
    }
    if (col == 0) {  // convergence check once per cycle through the variables (:693-700)
      if (lane == 0) {
        TriuTerms terms{corr, C, W, k};
        const double err = sqrt(pairwise(terms, (int64_t)k * (k - 1) / 2));
        errlog[t / k] = err;
        stop_sh = err < tol;
      }
      __syncthreads();
      if (stop_sh) {
        ++t;
        break;
      }
    }
  }
  for (int i = lane; i < k * k; i += 64) corr_g[i] = corr[i];
  if (lane == 0) {
    state[0] = t;
    state[1] = stop_sh;
  }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
size_t prm_bytes(int k) { return align256((size_t)(k + 2 * k * k) * 8); }

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_permcorr_workspace_size(int32_t k, size_t* bytes) {
  PBH_REQUIRE(bytes && k >= 1 && k <= kMaxK, "pbh_permcorr_workspace_size: 1 <= k <= 128");
  *bytes = prm_bytes(k);
  return PBH_OK;
}

extern "C" int pbh_permcorr_climb(double* xs, double* xo, int64_t n, int32_t k, int64_t ldx, double* corr,
                                  const double* den_host, const double* target_host, const double* weights_host,
                                  const int64_t* swaps, const int64_t* offsets, int64_t nsteps, double tol,
                                  double* errlog, int64_t* state, void* ws, size_t ws_bytes, void* stream) {
  PBH_REQUIRE(k >= 1 && k <= kMaxK && n >= 2 && ldx >= n && nsteps >= 0,
              "pbh_permcorr_climb: bad sizes (1 <= k <= 128, n >= 2, ldx >= n)");
  PBH_REQUIRE(xs && corr && den_host && target_host && weights_host && errlog && state && ws,
              "pbh_permcorr_climb: null pointer");
  PBH_REQUIRE(nsteps == 0 || (swaps && offsets), "pbh_permcorr_climb: null swap lists");
  PBH_REQUIRE(nsteps % k == 0, "pbh_permcorr_climb: steps must be whole cycles through the k variables");
  PBH_REQUIRE(ws_bytes >= prm_bytes(k), "pbh_permcorr_climb: workspace too small");
  hipStream_t s = as_stream(stream);
  double* prm = (double*)ws;
  PBH_CHECK_HIP(hipMemcpyAsync(prm, den_host, (size_t)k * 8, hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(prm + k, target_host, (size_t)k * k * 8, hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(prm + k + k * k, weights_host, (size_t)k * k * 8, hipMemcpyHostToDevice, s));
  const size_t lds = (size_t)(k * k + 4 * k) * 8;
  if (lds > 65536)
    PBH_CHECK_HIP(hipFuncSetAttribute((const void*)k_permcorr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PBH_TIMED(kKPermCorr, s,
            hipLaunchKernelGGL(k_permcorr, dim3(1), dim3(64), lds, s, xs, xo, ldx, n, (int)k, corr, prm, swaps,
                               offsets, nsteps, tol, errlog, state));
  PBH_CHECK_LAUNCH();
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // the host buffers above were sources of async copies
  return PBH_OK;
}
