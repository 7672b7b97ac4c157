// Per-kernel launch timing with HIP events on the launching stream (for bench.py's roofline:
// average device duration of one launch of a given kernel inside the timed region).
#pragma once

#include "pbh_common.h"

namespace pbh {

enum KernelId {
  kKLhsPpf = 0,
  kKPpf,
  kKSortScatter,
  kKSortUpsweep,
  kKSortDigitHist,
  kKRankScores,
  kKRankGather,
  kKLoadKeys,
  kKGram,
  kKApply,
  kKElementwise,
  kKHeadBounds,
  kKScan,
  kKLhsSorted,
  kKPermScores,
  kKCodeRuns,
  kKMakeCodes,
  kKSortScatter32,
  kKSortUpsweep32,
  kKSortDigitHist32,
  kKPlaceUpsweep,
  kKPlaceScatter,
  kKPlace,
  kKStreams,
  kKAffine,
  kKTable,
  kKPermCorr,
  kKHbmCopy,
  kKHist16,
  kKMsd1,
  kKMsd2,
  kKFinish,
  kKPlaceMsd,
  kKPlaceGen,
  kKDag,
  kKTranspose,
  kKCount
};

extern bool g_timing_on;
void timing_before(int id, hipStream_t s);
void timing_after(int id, hipStream_t s);

}  // namespace pbh

#define PBH_TIMED(id, s, ...)                     \
  do {                                            \
    if (pbh::g_timing_on) pbh::timing_before(id, s); \
    __VA_ARGS__;                                  \
    if (pbh::g_timing_on) pbh::timing_after(id, s);  \
  } while (0)
