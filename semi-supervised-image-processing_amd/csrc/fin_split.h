// Split of a BatchNorm finalize over several workgroups per channel (host and
// device constants shared by bn_common.h and the partial-buffer sizing in
// conv.hip / stem.hip / bn.hip).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>

namespace {

constexpr int FIN_NT = 256;  // threads of a finalize workgroup
constexpr int FIN_PT = 8;
constexpr int FIN_SMAX = 64;

// (one-wave LDS-free finalize workgroups, SSIP_FIN64=1: 6.52 vs 6.48 ms/step
// in round 3, -0.55 % / +0.8 % on two boxes in round 5; bn.hip)
static inline int fin_splits(long tiles) {
  long s = (tiles + (long)FIN_NT * FIN_PT - 1) / ((long)FIN_NT * FIN_PT);
  return (int)(s < 1 ? 1 : (s > FIN_SMAX ? FIN_SMAX : s));
}
// floats the split finalize needs behind `records` floats of records (vals
// fp64 values per (channel, split)); 0 when one workgroup per channel suffices
static inline int64_t fin_scratch_floats(int C, long tiles, int vals) {
  const int S = fin_splits(tiles);
  return S > 1 ? 2 + (int64_t)C * S * vals * 2 : 0;
}
static inline double* fin_scratch(float* partial, int64_t records) {
  uintptr_t p = (uintptr_t)(partial + records);
  return (double*)((p + 7) & ~(uintptr_t)7);
}

}  // namespace
