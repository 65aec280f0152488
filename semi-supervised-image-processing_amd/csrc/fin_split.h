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

// (SSIP_FIN_NT=64: one-wave, LDS-free finalize workgroups, an A/B option:
// 6.52 vs 6.48 ms/step, 3 + 3 runs, the blocking in the step trace is the
// halo kernels' register files, not their LDS)
static inline int fin_nt() {
  static const int nt = getenv("SSIP_FIN_NT") && atoi(getenv("SSIP_FIN_NT")) == 64 ? 64 : FIN_NT;
  return nt;
}
// (SSIP_FIN_PT: records per thread before a split, a tuning override)
static inline int fin_splits(long tiles) {
  static const long pt = getenv("SSIP_FIN_PT") ? std::max(1, atoi(getenv("SSIP_FIN_PT"))) : FIN_PT;
  long s = (tiles + fin_nt() * pt - 1) / (fin_nt() * pt);
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
