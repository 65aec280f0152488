// BatchNorm backward finalize shared by bn.hip and stem.hip: per-channel sums
// of dout and dout*xhat from [C][blocks][2] (or [blocks][C][2]) partials
// (fixed-order fp64 tree)
// -> dgamma/dbeta and the apply coefficients
//   dy = coef[c] * dout + coef[C+c] * y + coef[2C+c].
#pragma once
#include "ssip_common.h"

namespace {

// sums of up to three values over a 1024-thread workgroup in fp64 with one
// LDS round (wave butterflies, then the 16 wave totals in fixed order)
template <int V>
__device__ __forceinline__ void block_sums_f64_1024(double (&v)[V], double* sh) {
#pragma unroll
  for (int k = 0; k < V; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < V; ++k) sh[k * 16 + (threadIdx.x >> 6)] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < V; ++k) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) t += sh[k * 16 + w];
    v[k] = t;
  }
}

// One 1024-thread workgroup per channel: sums of dout and dout*xhat over the
// partials (threads take blocks t = tid, tid + 1024, ...); cmajor: [C][blocks][2]
// (each channel's records contiguous), else [blocks][C][2].
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(int C, int blocks, long M, int cmajor,
                                                               const float* __restrict__ partial,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd, float* dgamma,
                                                               float* dbeta, int accumulate, float* coef) {
  __shared__ double sh[2 * 16];
  const int c = blockIdx.x;
  double ab[2] = {0.0, 0.0};
  const long cs = cmajor ? 2 : (long)C * 2;
  const float* pc = partial + (cmajor ? (long)c * blocks * 2 : (long)c * 2);
  for (int t = threadIdx.x; t < blocks; t += 1024) {
    ab[0] += pc[t * cs + 0];
    ab[1] += pc[t * cs + 1];
  }
  block_sums_f64_1024<2>(ab, sh);
  const double sum_d = ab[0], sum_dx = ab[1];
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = (float)(accumulate ? dgamma[c] + sum_dx : sum_dx);
    if (dbeta) dbeta[c] = (float)(accumulate ? dbeta[c] + sum_d : sum_d);
    const double g = gamma ? gamma[c] : 1.0;
    const double is = invstd[c];
    const double A = g * is;
    const double k0 = -A * sum_d / (double)M;
    const double k1 = -A * sum_dx / (double)M * is;
    coef[c] = (float)A;                           // * dout
    coef[C + c] = (float)k1;                      // * y
    coef[2 * C + c] = (float)(k0 - k1 * mean[c]);  // constant
  }
}

static inline int bn_bwd_finalize_grid(int C) { return C; }

}  // namespace
