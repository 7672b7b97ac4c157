// Inverse CDF of the table-driven distribution nodes (modeling.py:825-927), q -> x on the device:
//
//   PBH_TABLE_INTERP    CumulativeDistribution._sample  np.interp(q, xp, fp)
//                       (numpy compiled_base.c arr_interp: j with xp[j] <= q < xp[j+1],
//                       slope * (q - xp[j]) + fp[j], the NaN retry from the right end, clamps
//                       to fp[0] / fp[-1] outside [xp[0], xp[-1]])
//   PBH_TABLE_QUANTILE  EmpiricalDistribution._sample   np.quantile(data, q, method=...)
//                       on the sorted data (numpy lib/_function_base_impl.py _quantile:
//                       virtual index (m - 1) q, _get_indexes clamping, _lerp with its
//                       t >= 0.5 branch); methods linear / lower / higher / nearest / midpoint
//   PBH_TABLE_SEARCH    DiscreteDistribution._sample    values[searchsorted(cumsum(p), q, 'right')]
//                       (index m -- q at or above the last cumulative -- is flagged: the
//                       reference raises IndexError there)
//
// One element per lane, the table read through L1/L2 (tables are small and shared by every
// lane); HBM bound at 16 B per draw (read q, write x).
#include <math.h>

#include <type_traits>

#include "pbh_error.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

// first index j in [0, m) with t[j] > v (searchsorted side='right'), m if none
__device__ __forceinline__ int64_t upper_bound(const double* __restrict__ t, int64_t m, double v) {
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (t[mid] <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__device__ __forceinline__ double interp_one(double x, const double* __restrict__ xp, const double* __restrict__ fp,
                                             int64_t m) {
  if (isnan(x)) return x;
  if (m == 1) return fp[0];
  const double left = fp[0], right = fp[m - 1];
  if (x < xp[0]) return left;
  if (x > xp[m - 1]) return right;
  if (x == xp[m - 1]) return right;
  const int64_t j = upper_bound(xp, m, x) - 1;  // xp[j] <= x < xp[j + 1]
  const double slope = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]);
  double r = slope * (x - xp[j]) + fp[j];
  if (isnan(r)) {
    r = slope * (x - xp[j + 1]) + fp[j + 1];
    if (isnan(r) && fp[j] == fp[j + 1]) r = fp[j];
  }
  return r;
}

enum QuantileMethod { kLinear = 0, kLower = 1, kHigher = 2, kNearest = 3, kMidpoint = 4 };

__device__ __forceinline__ double quantile_one(double q, const double* __restrict__ a, int64_t m, int method) {
  if (isnan(a[m - 1])) return a[m - 1];  // numpy: any NaN in the data makes every quantile NaN
  const double vi = (double)(m - 1) * q;
  if (method == kLower || method == kHigher || method == kNearest) {
    double k = method == kLower ? floor(vi) : (method == kHigher ? ceil(vi) : rint(vi));
    int64_t i = (int64_t)k;
    i = i < 0 ? 0 : (i > m - 1 ? m - 1 : i);
    return a[i];
  }
  // linear / midpoint: _get_indexes then _lerp
  const double fl = floor(vi);
  int64_t prev = (int64_t)fl, next = prev + 1;
  double gamma = vi - fl;
  if (vi >= (double)(m - 1)) {
    prev = next = m - 1;  // numpy uses index -1 for both: the last element
  } else if (vi < 0.0) {
    prev = next = 0;
  }
  if (method == kMidpoint) gamma = gamma == 0.0 ? 0.0 : 0.5;
  const double lo = a[prev], hi = a[next];
  const double diff = hi - lo;
  if (gamma >= 0.5) return hi - diff * (1.0 - gamma);
  return lo + diff * gamma;
}

template <int KIND, typename OUT>
__global__ __launch_bounds__(256) void k_table_ppf(const double* __restrict__ q, int64_t q_stride, int64_t n,
                                                   const double* __restrict__ t0, const void* __restrict__ t1,
                                                   int64_t m, int method, OUT* __restrict__ out, int32_t* flag) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double x = q[i * q_stride];
    if constexpr (KIND == PBH_TABLE_INTERP) {
      const double r = interp_one(x, t0, (const double*)t1, m);
      out[i] = (OUT)r;
      flag_nonfinite(flag, !isfinite(r));
    } else if constexpr (KIND == PBH_TABLE_QUANTILE) {
      const double r = quantile_one(x, t0, m, method);
      out[i] = (OUT)r;
      flag_nonfinite(flag, !isfinite(r));
    } else {
      int64_t j = upper_bound(t0, m, x);
      const bool oob = !(j < m);
      if (oob) j = m - 1;
      if (t1)
        out[i] = ((const OUT*)t1)[j];
      else
        out[i] = (OUT)j;
      if (flag) {
        const unsigned long long b = __ballot(oob);
        if (b && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(b)) atomicOr(flag, 4);
      }
      if constexpr (std::is_floating_point<OUT>::value) flag_nonfinite(flag, !isfinite((double)out[i]));
    }
  }
}

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_table_ppf(int kind, const double* q, int64_t q_stride, int64_t n, const double* t0, const void* t1,
                             int64_t m, int method, int out_dtype, void* out, int32_t* flag, void* stream) {
  PBH_REQUIRE(n >= 0 && m >= 1 && t0 && (n == 0 || (q && out)), "pbh_table_ppf: bad arguments (empty table?)");
  PBH_REQUIRE(kind >= PBH_TABLE_INTERP && kind <= PBH_TABLE_SEARCH, "pbh_table_ppf: unknown kind %d", kind);
  PBH_REQUIRE(kind != PBH_TABLE_INTERP || t1, "pbh_table_ppf: interp needs fp");
  PBH_REQUIRE(method >= 0 && method <= 4, "pbh_table_ppf: unknown quantile method %d", method);
  PBH_REQUIRE(out_dtype == PBH_FLOAT64 || (kind == PBH_TABLE_SEARCH && out_dtype == PBH_INT64),
              "pbh_table_ppf: output dtype");
  if (n == 0) return PBH_OK;
  hipStream_t s = as_stream(stream);
  dim3 g(grid_for(n, 256, 16384)), b(256);
  PBH_TIMED(kKTable, s, {
    if (kind == PBH_TABLE_INTERP)
      hipLaunchKernelGGL((k_table_ppf<PBH_TABLE_INTERP, double>), g, b, 0, s, q, q_stride, n, t0, t1, m, method,
                         (double*)out, flag);
    else if (kind == PBH_TABLE_QUANTILE)
      hipLaunchKernelGGL((k_table_ppf<PBH_TABLE_QUANTILE, double>), g, b, 0, s, q, q_stride, n, t0, t1, m, method,
                         (double*)out, flag);
    else if (out_dtype == PBH_INT64)
      hipLaunchKernelGGL((k_table_ppf<PBH_TABLE_SEARCH, int64_t>), g, b, 0, s, q, q_stride, n, t0, t1, m, method,
                         (int64_t*)out, flag);
    else
      hipLaunchKernelGGL((k_table_ppf<PBH_TABLE_SEARCH, double>), g, b, 0, s, q, q_stride, n, t0, t1, m, method,
                         (double*)out, flag);
  });
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}
