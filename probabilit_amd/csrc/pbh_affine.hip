// Affine row transform Y = offset + ((X - shift) / scale) @ M on the device: the N-sized part
// of the Cholesky correlator (correlation.py:271-285) and of decorrelate
// (correlation.py:745-754).  Their K x K algebra (covariance from the centered Gram of
// pbh_centered_gram, Cholesky factors, triangular solves) runs on the host.
//
// One row per lane, the row held in registers (K <= 128), M / shift / scale / offset read
// with uniform (scalar) loads.  HBM bound: 8 K bytes read + 8 K written per row.
#include <vector>

#include "pbh_error.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

template <int KMAX>
__global__ __launch_bounds__(256) void k_affine(const double* __restrict__ X, int64_t n, int k, int64_t x_rs,
                                                int64_t x_cs, const double* __restrict__ prm, double* __restrict__ Y,
                                                int64_t y_rs, int64_t y_cs) {
  const double* shift = prm;
  const double* scale = prm + k;
  const double* offset = prm + 2 * k;
  const double* M = prm + 3 * k;  // row-major k x k
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < n; r += (int64_t)gridDim.x * 256) {
    double v[KMAX];
#pragma unroll
    for (int i = 0; i < KMAX; ++i) v[i] = i < k ? (X[r * x_rs + i * x_cs] - shift[i]) / scale[i] : 0.0;
#pragma unroll 4
    for (int j = 0; j < k; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < KMAX; ++i)
        if (i < k) acc = acc + v[i] * M[i * k + j];
      Y[r * y_rs + j * y_cs] = offset[j] + acc;
    }
  }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_affine_workspace_size(int32_t k, size_t* bytes) {
  PBH_REQUIRE(bytes && k >= 1 && k <= 128, "pbh_affine_workspace_size: 1 <= k <= 128");
  *bytes = align256((size_t)(3 * k + k * k) * 8);
  return PBH_OK;
}

extern "C" int pbh_affine_rows(const double* X, int64_t n, int32_t k, int64_t x_rs, int64_t x_cs,
                               const double* shift_host, const double* scale_host, const double* offset_host,
                               const double* M_host, double* Y, int64_t y_rs, int64_t y_cs, void* ws, size_t ws_bytes,
                               void* stream) {
  PBH_REQUIRE(shift_host && offset_host && M_host && ws && n >= 0 && k >= 1 && k <= 128,
              "pbh_affine_rows: bad arguments (1 <= k <= 128)");
  PBH_REQUIRE(n == 0 || (X && Y), "pbh_affine_rows: null data pointer");
  PBH_REQUIRE(ws_bytes >= align256((size_t)(3 * k + k * k) * 8), "pbh_affine_rows: workspace too small");
  hipStream_t s = as_stream(stream);
  std::vector<double> prm((size_t)3 * k + (size_t)k * k);
  for (int i = 0; i < k; ++i) {
    prm[i] = shift_host[i];
    prm[k + i] = scale_host ? scale_host[i] : 1.0;
    prm[2 * k + i] = offset_host[i];
  }
  for (int i = 0; i < k * k; ++i) prm[3 * k + i] = M_host[i];
  PBH_CHECK_HIP(hipMemcpyAsync(ws, prm.data(), prm.size() * 8, hipMemcpyHostToDevice, s));
  if (n > 0) {
    dim3 g(grid_for(n, 256, 16384)), b(256);
    const double* p = (const double*)ws;
    if (k <= 8)
      PBH_TIMED(kKAffine, s, hipLaunchKernelGGL(k_affine<8>, g, b, 0, s, X, n, k, x_rs, x_cs, p, Y, y_rs, y_cs));
    else if (k <= 32)
      PBH_TIMED(kKAffine, s, hipLaunchKernelGGL(k_affine<32>, g, b, 0, s, X, n, k, x_rs, x_cs, p, Y, y_rs, y_cs));
    else
      PBH_TIMED(kKAffine, s, hipLaunchKernelGGL(k_affine<128>, g, b, 0, s, X, n, k, x_rs, x_cs, p, Y, y_rs, y_cs));
    PBH_CHECK_LAUNCH();
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // `prm` is pageable and goes out of scope
  return PBH_OK;
}
