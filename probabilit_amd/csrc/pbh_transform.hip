// Elementwise Transform nodes (modeling.py:933-1169) with numpy semantics, plus the
// Avg reduction (modeling.py:986-990) and an LDS-tiled transpose.
//
// The host decides numpy's result dtype and passes (compute dtype, output dtype); the
// kernel is HBM-bound (8 B per float64 operand vector read, 8 B written per element).
#include <math.h>

#include "pbh_error.h"
#include "pbh_ops.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kBlock = 256;

PBH_DI double ld_f(const pbh_operand& o, int64_t i) {
  if (!o.ptr) return o.dtype == PBH_FLOAT64 ? o.f : (double)o.i;
  switch (o.dtype) {
    case PBH_FLOAT64:
      return ((const double*)o.ptr)[i];
    case PBH_INT64:
      return (double)((const int64_t*)o.ptr)[i];
    default:
      return ((const uint8_t*)o.ptr)[i] ? 1.0 : 0.0;
  }
}

PBH_DI int64_t ld_i(const pbh_operand& o, int64_t i) {
  if (!o.ptr) return o.dtype == PBH_FLOAT64 ? (int64_t)o.f : o.i;
  switch (o.dtype) {
    case PBH_FLOAT64:
      return (int64_t)((const double*)o.ptr)[i];
    case PBH_INT64:
      return ((const int64_t*)o.ptr)[i];
    default:
      return ((const uint8_t*)o.ptr)[i] ? 1 : 0;
  }
}


PBH_DI int64_t i_floordiv(int64_t a, int64_t b) {
  if (b == 0) return 0;
  if (a == INT64_MIN && b == -1) return INT64_MIN;
  int64_t q = a / b;
  if (((a % b) != 0) && ((a < 0) != (b < 0))) q -= 1;
  return q;
}
PBH_DI int64_t i_mod(int64_t a, int64_t b) {
  if (b == 0) return 0;
  if (b == -1) return 0;
  int64_t r = a % b;
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}
PBH_DI int64_t i_pow(int64_t a, int64_t b) {
  uint64_t r = 1, base = (uint64_t)a;
  while (b > 0) {
    if (b & 1) r *= base;
    base *= base;
    b >>= 1;
  }
  return (int64_t)r;
}


PBH_DI int64_t i_binary(int op, int64_t a, int64_t b, bool* neg_pow) {
  switch (op) {
    case PBH_OP_ADD: return (int64_t)((uint64_t)a + (uint64_t)b);
    case PBH_OP_SUB: return (int64_t)((uint64_t)a - (uint64_t)b);
    case PBH_OP_MUL: return (int64_t)((uint64_t)a * (uint64_t)b);
    case PBH_OP_FLOORDIV: return i_floordiv(a, b);
    case PBH_OP_MOD: return i_mod(a, b);
    case PBH_OP_POW:
      if (b < 0) *neg_pow = true;
      return i_pow(a, b);
    case PBH_OP_MAX: return a > b ? a : b;
    case PBH_OP_MIN: return a < b ? a : b;
    case PBH_OP_AND: return (a != 0 && b != 0);
    case PBH_OP_OR: return (a != 0 || b != 0);
    case PBH_OP_EQ: return a == b;
    case PBH_OP_NE: return a != b;
    case PBH_OP_LT: return a < b;
    case PBH_OP_LE: return a <= b;
    case PBH_OP_GT: return a > b;
    case PBH_OP_GE: return a >= b;
    default: return 0;
  }
}

PBH_DI int64_t i_unary(int op, int64_t a) {
  switch (op) {
    case PBH_OP_NEG: return (int64_t)(0ull - (uint64_t)a);
    case PBH_OP_ABS: return a < 0 ? (int64_t)(0ull - (uint64_t)a) : a;
    case PBH_OP_SIGN: return (a > 0) - (a < 0);
    case PBH_OP_SQUARE: return (int64_t)((uint64_t)a * (uint64_t)a);
    case PBH_OP_FLOOR:
    case PBH_OP_CEIL:
    default: return a;  // CAST
  }
}

PBH_DI void flag_bits(int32_t* flag, bool cond, int bit) {
  if (flag == nullptr) return;
  unsigned long long m = __ballot(cond);
  if (m != 0ull && (threadIdx.x & 63) == (unsigned)__builtin_ctzll(m)) atomicOr(flag, bit);
}

__global__ __launch_bounds__(kBlock) void k_elementwise(int op, int cdt, int odt, pbh_operand a, pbh_operand b,
                                                        void* __restrict__ out, int64_t n, int32_t* flag) {
  const bool unary = op >= PBH_OP_NEG;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    bool bad = false, negpow = false;
    if (cdt == PBH_FLOAT64) {
      double x = unary ? f_unary(op, ld_f(a, i)) : f_binary(op, ld_f(a, i), ld_f(b, i));
      if (odt == PBH_FLOAT64) {
        ((double*)out)[i] = x;
        bad = !isfinite(x);
      } else if (odt == PBH_INT64) {
        ((int64_t*)out)[i] = (int64_t)x;
      } else {
        ((uint8_t*)out)[i] = x != 0.0;
      }
    } else {  // INT64 or BOOL compute: integer arithmetic on 0/1 for bool
      int64_t x;
      if (unary) {
        x = i_unary(op, ld_i(a, i));
      } else {
        int64_t u = ld_i(a, i), v = ld_i(b, i);
        if (cdt == PBH_BOOL) {  // numpy bool arithmetic: + is or, * is and
          if (op == PBH_OP_ADD) op = PBH_OP_OR;
          if (op == PBH_OP_MUL) op = PBH_OP_AND;
        }
        x = i_binary(op, u, v, &negpow);
      }
      if (odt == PBH_FLOAT64)
        ((double*)out)[i] = (double)x;
      else if (odt == PBH_INT64)
        ((int64_t*)out)[i] = x;
      else
        ((uint8_t*)out)[i] = x != 0;
    }
    flag_bits(flag, bad, 1);
    flag_bits(flag, negpow, 2);
  }
}

// Fast path for the arithmetic that dominates DAG transforms (the README mutual fund is 20
// multiplies and 20 adds per row): float64 +, -, *, / of float64 vectors and scalars, one
// template instance per (op, vector/scalar) shape so that no other operator's code sizes the
// registers of the wave.  4 elements per thread per iteration, 16-byte loads and stores when
// the vectors are 16-byte aligned.  Same IEEE operations as f_binary (-ffp-contract=off).
template <int OP>
PBH_DI double arith(double a, double b) {
  if constexpr (OP == PBH_OP_ADD) return a + b;
  if constexpr (OP == PBH_OP_SUB) return a - b;
  if constexpr (OP == PBH_OP_MUL) return a * b;
  return a / b;
}

template <int OP, bool AV, bool BV>
__global__ __launch_bounds__(kBlock) void k_arith_f64(const double* __restrict__ a, double as,
                                                     const double* __restrict__ b, double bs,
                                                     double* __restrict__ out, int64_t n, int32_t* flag) {
  const int64_t nq = n / 4;
  bool bad = false;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += (int64_t)gridDim.x * kBlock) {
    double2 x0, x1, y0, y1;
    if constexpr (AV) {
      x0 = ((const double2*)a)[2 * q];
      x1 = ((const double2*)a)[2 * q + 1];
    } else {
      x0 = x1 = double2{as, as};
    }
    if constexpr (BV) {
      y0 = ((const double2*)b)[2 * q];
      y1 = ((const double2*)b)[2 * q + 1];
    } else {
      y0 = y1 = double2{bs, bs};
    }
    double2 r0{arith<OP>(x0.x, y0.x), arith<OP>(x0.y, y0.y)}, r1{arith<OP>(x1.x, y1.x), arith<OP>(x1.y, y1.y)};
    ((double2*)out)[2 * q] = r0;
    ((double2*)out)[2 * q + 1] = r1;
    bad |= !isfinite(r0.x) || !isfinite(r0.y) || !isfinite(r1.x) || !isfinite(r1.y);
  }
  if (blockIdx.x == 0) {  // tail
    const int64_t i = nq * 4 + threadIdx.x;
    if (i < n) {
      const double r = arith<OP>(AV ? a[i] : as, BV ? b[i] : bs);
      out[i] = r;
      bad |= !isfinite(r);
    }
  }
  flag_bits(flag, bad, 1);
}

template <int OP>
void launch_arith(const pbh_operand& a, const pbh_operand& b, double* out, int64_t n, int32_t* flag, hipStream_t s) {
  const double as = a.ptr ? 0.0 : (a.dtype == PBH_FLOAT64 ? a.f : (double)a.i);
  const double bs = b.ptr ? 0.0 : (b.dtype == PBH_FLOAT64 ? b.f : (double)b.i);
  const double* ap = (const double*)a.ptr;
  const double* bp = (const double*)b.ptr;
  dim3 g(grid_for((n + 3) / 4, kBlock, 8192)), blk(kBlock);
  if (ap && bp)
    hipLaunchKernelGGL((k_arith_f64<OP, true, true>), g, blk, 0, s, ap, as, bp, bs, out, n, flag);
  else if (ap)
    hipLaunchKernelGGL((k_arith_f64<OP, true, false>), g, blk, 0, s, ap, as, bp, bs, out, n, flag);
  else
    hipLaunchKernelGGL((k_arith_f64<OP, false, true>), g, blk, 0, s, ap, as, bp, bs, out, n, flag);
}

bool arith_fast_path(int op, int cdt, int odt, const pbh_operand& a, const pbh_operand& b, const void* out) {
  if (!(op == PBH_OP_ADD || op == PBH_OP_SUB || op == PBH_OP_MUL || op == PBH_OP_TRUEDIV)) return false;
  if (cdt != PBH_FLOAT64 || odt != PBH_FLOAT64) return false;
  if (!a.ptr && !b.ptr) return false;
  auto ok = [](const pbh_operand& o) {
    return o.ptr ? (o.dtype == PBH_FLOAT64 && ((uintptr_t)o.ptr & 15) == 0) : true;
  };
  return ok(a) && ok(b) && ((uintptr_t)out & 15) == 0;
}

struct AvgArgs {
  const double* p[32];
};

__global__ __launch_bounds__(kBlock) void k_average(AvgArgs args, int m, int64_t n, double* __restrict__ out,
                                                    int32_t* flag) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    double s = args.p[0][i];
    for (int j = 1; j < m; ++j) s += args.p[j][i];
    double x = s / (double)m;
    out[i] = x;
    flag_bits(flag, !isfinite(x), 1);
  }
}

constexpr int TT = 32;
__global__ __launch_bounds__(TT * 8) void k_transpose(const double* __restrict__ in, int64_t rows, int64_t cols,
                                                      int64_t ld_in, double* __restrict__ out, int64_t ld_out) {
  // in: rows x cols, element (r, c) at in[r * ld_in + c]; out(c, r) at out[c * ld_out + r]
  __shared__ double tile[TT][TT + 1];
  const int64_t r0 = (int64_t)blockIdx.x * TT, c0 = (int64_t)blockIdx.y * TT;
  for (int y = threadIdx.y; y < TT; y += 8) {
    int64_t r = r0 + y, c = c0 + threadIdx.x;
    if (r < rows && c < cols) tile[y][threadIdx.x] = in[r * ld_in + c];
  }
  __syncthreads();
  for (int y = threadIdx.y; y < TT; y += 8) {
    int64_t c = c0 + y, r = r0 + threadIdx.x;
    if (r < rows && c < cols) out[c * ld_out + r] = tile[threadIdx.x][y];
  }
}

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_elementwise(int op, int compute_dtype, int out_dtype, const pbh_operand* a, const pbh_operand* b,
                               void* out, int64_t n, int32_t* nonfinite_flag, void* stream) {
  PBH_REQUIRE(a != nullptr && out != nullptr, "pbh_elementwise: a and out required");
  PBH_REQUIRE(compute_dtype >= PBH_BOOL && compute_dtype <= PBH_FLOAT64, "pbh_elementwise: bad compute dtype");
  PBH_REQUIRE(out_dtype >= PBH_BOOL && out_dtype <= PBH_FLOAT64, "pbh_elementwise: bad output dtype");
  const bool unary = op >= PBH_OP_NEG;
  PBH_REQUIRE((op >= PBH_OP_ADD && op <= PBH_OP_ARCTAN2) || (op >= PBH_OP_NEG && op <= PBH_OP_ARCTANH) ||
                  op == PBH_OP_CAST,
              "pbh_elementwise: unknown op %d", op);
  PBH_REQUIRE(unary || b != nullptr, "pbh_elementwise: binary op needs b");
  if (n <= 0) return PBH_OK;
  pbh_operand bb = unary ? *a : *b;
  hipStream_t s = as_stream(stream);
  if (!unary && arith_fast_path(op, compute_dtype, out_dtype, *a, bb, out)) {
    switch (op) {
      case PBH_OP_ADD: PBH_TIMED(kKElementwise, s, launch_arith<PBH_OP_ADD>(*a, bb, (double*)out, n, nonfinite_flag, s)); break;
      case PBH_OP_SUB: PBH_TIMED(kKElementwise, s, launch_arith<PBH_OP_SUB>(*a, bb, (double*)out, n, nonfinite_flag, s)); break;
      case PBH_OP_MUL: PBH_TIMED(kKElementwise, s, launch_arith<PBH_OP_MUL>(*a, bb, (double*)out, n, nonfinite_flag, s)); break;
      default: PBH_TIMED(kKElementwise, s, launch_arith<PBH_OP_TRUEDIV>(*a, bb, (double*)out, n, nonfinite_flag, s)); break;
    }
    PBH_CHECK_LAUNCH();
    return PBH_OK;
  }
  PBH_TIMED(kKElementwise, s,
            hipLaunchKernelGGL(k_elementwise, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, s, op, compute_dtype,
                               out_dtype, *a, bb, out, n, nonfinite_flag));
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

extern "C" int pbh_average(const double* const* parents_host, int m, int64_t n, double* out, int32_t* nonfinite_flag,
                           void* stream) {
  PBH_REQUIRE(m >= 1 && m <= 32, "pbh_average: 1 <= m <= 32 parents supported");
  PBH_REQUIRE(parents_host && out, "pbh_average: null pointer");
  if (n <= 0) return PBH_OK;
  AvgArgs a = {};
  for (int j = 0; j < m; ++j) a.p[j] = parents_host[j];
  hipLaunchKernelGGL(k_average, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, as_stream(stream), a, m, n, out,
                     nonfinite_flag);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}

extern "C" int pbh_transpose(const double* in, int64_t rows, int64_t cols, int64_t ld_in, double* out,
                             int64_t ld_out, void* stream) {
  PBH_REQUIRE(in && out, "pbh_transpose: null pointer");
  PBH_REQUIRE(ld_in >= cols && ld_out >= rows, "pbh_transpose: bad leading dimension");
  if (rows <= 0 || cols <= 0) return PBH_OK;
  PBH_REQUIRE((cols + TT - 1) / TT <= 65535, "pbh_transpose: too many columns per launch");
  dim3 g((unsigned)((rows + TT - 1) / TT), (unsigned)((cols + TT - 1) / TT)), b(TT, 8);
  hipLaunchKernelGGL(k_transpose, g, b, 0, as_stream(stream), in, rows, cols, ld_in, out, ld_out);
  PBH_CHECK_LAUNCH();
  return PBH_OK;
}
