// Shared definitions for the probabilit MI355X (gfx950) native library.
//
// Everything in csrc/ is compiled by hipcc for gfx950 only, with -ffp-contract=off so that
// every multiply and add rounds separately, as in scipy/numpy's x86-64 builds (no FMA).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/probabilit_hip.h"

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
#define PBH_HD __host__ __device__
#else
#define PBH_HD
#endif

#define PBH_DI __device__ __forceinline__

namespace pbh {

constexpr int kWave = 64;  // CDNA wavefront width

// Order-preserving map of a finite double to an unsigned key (ascending doubles <->
// ascending keys).  -0.0 is folded onto +0.0 first so that the two compare equal, as
// they do for numpy's argsort / rankdata tie detection.
PBH_HD inline uint64_t f64_to_key(double x) {
  x = x + 0.0;  // -0.0 + 0.0 == +0.0
  uint64_t b = __builtin_bit_cast(uint64_t, x);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

PBH_HD inline double key_to_f64(uint64_t k) {
  uint64_t b = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
  return __builtin_bit_cast(double, b);
}

inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// Sets *flag to 1 (one atomic per wave) when any active lane saw a non-finite value.
PBH_DI void flag_nonfinite(int32_t* flag, bool bad) {
  if (flag == nullptr) return;
  unsigned long long m = __ballot(bad);
  if (m != 0ull && (threadIdx.x & (kWave - 1)) == (unsigned)__builtin_ctzll(m)) atomicOr(flag, 1);
}

}  // namespace pbh
