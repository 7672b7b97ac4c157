// Status / last-error plumbing for the C-ABI (no exception crosses extern "C").
#pragma once

#include <stdarg.h>
#include <stdio.h>

#include "pbh_common.h"

namespace pbh {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace pbh

#define PBH_CHECK_HIP(expr)                                                              \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      pbh::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,    \
                     __LINE__);                                                          \
      return PBH_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define PBH_CHECK_LAUNCH() PBH_CHECK_HIP(hipGetLastError())

#define PBH_REQUIRE(cond, ...)        \
  do {                                \
    if (!(cond)) {                    \
      pbh::set_error(__VA_ARGS__);    \
      return PBH_ERR_INVALID;         \
    }                                 \
  } while (0)
