// float64 operators of the Transform nodes with numpy semantics (modeling.py:933-1169), shared
// by the per-node kernels (pbh_transform.hip) and the fused DAG program (pbh_dag.hip).
#pragma once
#include <math.h>

#include "pbh_error.h"

namespace pbh {
namespace {

// numpy npy_divmod / npy_floor_divide / npy_remainder for float64
PBH_DI double np_divmod(double a, double b, double* modp) {
  double mod = fmod(a, b);
  if (b == 0.0) {
    *modp = mod;
    return a / b;
  }
  double div = (a - mod) / b;
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) {
      mod += b;
      div -= 1.0;
    }
  } else {
    mod = copysign(0.0, b);
  }
  double floordiv;
  if (div != 0.0) {
    floordiv = floor(div);
    if (div - floordiv > 0.5) floordiv += 1.0;
  } else {
    floordiv = copysign(0.0, a / b);
  }
  *modp = mod;
  return floordiv;
}
PBH_DI double np_floordiv(double a, double b) {
  if (b == 0.0) return a / b;
  double m;
  return np_divmod(a, b, &m);
}
PBH_DI double np_remainder(double a, double b) {
  if (b == 0.0) return fmod(a, b);
  double m;
  np_divmod(a, b, &m);
  return m;
}

PBH_DI double f_binary(int op, double a, double b) {
  switch (op) {
    case PBH_OP_ADD: return a + b;
    case PBH_OP_SUB: return a - b;
    case PBH_OP_MUL: return a * b;
    case PBH_OP_TRUEDIV: return a / b;
    case PBH_OP_FLOORDIV: return np_floordiv(a, b);
    case PBH_OP_MOD: return np_remainder(a, b);
    case PBH_OP_POW: return pow(a, b);
    case PBH_OP_MAX: return (a >= b || isnan(a)) ? a : b;
    case PBH_OP_MIN: return (a <= b || isnan(a)) ? a : b;
    case PBH_OP_ARCTAN2: return atan2(a, b);
    case PBH_OP_AND: return (a != 0.0 && b != 0.0) ? 1.0 : 0.0;
    case PBH_OP_OR: return (a != 0.0 || b != 0.0) ? 1.0 : 0.0;
    case PBH_OP_EQ: return a == b;
    case PBH_OP_NE: return a != b;
    case PBH_OP_LT: return a < b;
    case PBH_OP_LE: return a <= b;
    case PBH_OP_GT: return a > b;
    case PBH_OP_GE: return a >= b;
    case PBH_OP_ISCLOSE: {  // np.isclose(a, b) with rtol=1e-5, atol=1e-8, equal_nan=False
      bool fin = isfinite(a) && isfinite(b);
      return fin ? (fabs(a - b) <= 1e-08 + 1e-05 * fabs(b)) : (a == b);
    }
    default: return __builtin_nan("");
  }
}

PBH_DI double f_unary(int op, double a) {
  switch (op) {
    case PBH_OP_NEG: return -a;
    case PBH_OP_ABS: return fabs(a);
    case PBH_OP_LOG: return log(a);
    case PBH_OP_EXP: return exp(a);
    case PBH_OP_FLOOR: return floor(a);
    case PBH_OP_CEIL: return ceil(a);
    case PBH_OP_SIGN: return a > 0.0 ? 1.0 : (a < 0.0 ? -1.0 : (a == 0.0 ? 0.0 : a));
    case PBH_OP_SQRT: return sqrt(a);
    case PBH_OP_SQUARE: return a * a;
    case PBH_OP_LOG10: return log10(a);
    case PBH_OP_SIN: return sin(a);
    case PBH_OP_COS: return cos(a);
    case PBH_OP_TAN: return tan(a);
    case PBH_OP_ARCSIN: return asin(a);
    case PBH_OP_ARCCOS: return acos(a);
    case PBH_OP_ARCTAN: return atan(a);
    case PBH_OP_SINH: return sinh(a);
    case PBH_OP_COSH: return cosh(a);
    case PBH_OP_TANH: return tanh(a);
    case PBH_OP_ARCSINH: return asinh(a);
    case PBH_OP_ARCCOSH: return acosh(a);
    case PBH_OP_ARCTANH: return atanh(a);
    default: return a;  // CAST
  }
}

}  // namespace
}  // namespace pbh
