// Device decode of the reference LHS stream's shuffles (pbh_lhs_dev.hip), called by
// pbh_lhs_reference (pbh_lhs_ref.hip), which keeps the host shuffles as its fallback.
#pragma once

#include <stdint.h>

#include "pbh_common.h"
#include "pbh_mt.h"

namespace pbh {

// u = rng.uniform(size=(n, d)) and the d shuffles of arange(1, n + 1) that numpy's
// Generator.shuffle makes from the same PCG64 stream (state / inc: {low, high} words before the
// uniforms; has32 / buf32: the 32-bit buffer of next_uint32), combined into q (column-major,
// ldq) as (perms.T - u) / n, the whole thing on the device.  targets: d * n int32 of scratch.
// *done = false: the decode failed its own check at every band width; q then holds nothing
// usable (the caller draws u again and shuffles on the host).  strata (optional, column c at
// strata + c * lds): each row's stratum perms - 1.
int lhs_reference_device(const uint64_t* state_host, const uint64_t* inc_host, bool has32, uint32_t buf32, int64_t n,
                         int d, double* q, int64_t ldq, int32_t* targets, hipStream_t s, bool* done,
                         int32_t* strata = nullptr, int64_t lds = 0);

}  // namespace pbh
