// BatchNorm backward finalize shared by bn.hip and stem.hip: per-channel sums
// of dout and dout*xhat from [blocks][C][2] partials (fixed-order fp64 tree)
// -> dgamma/dbeta and the apply coefficients
//   dy = coef[c] * dout + coef[C+c] * y + coef[2C+c].
#pragma once
#include "ssip_common.h"

namespace {

// sum over a 1024-thread workgroup in fp64: wave butterflies, then the 16
// wave totals in fixed order (every thread returns the total)
__device__ __forceinline__ double block_sum_f64_1024(double v, double* sh16) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh16[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += sh16[w];
  __syncthreads();
  return t;
}

// One 1024-thread workgroup per channel: sums of dout and dout*xhat over the
// [blocks][C][2] partials (threads take blocks t = tid, tid + 1024, ...).
__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(int C, int blocks, long M,
                                                               const float* __restrict__ partial,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd, float* dgamma,
                                                               float* dbeta, int accumulate, float* coef) {
  __shared__ double sh[2][16];
  const int c = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (int t = threadIdx.x; t < blocks; t += 1024) {
    a += partial[((long)t * C + c) * 2 + 0];
    b += partial[((long)t * C + c) * 2 + 1];
  }
  const double sum_d = block_sum_f64_1024(a, sh[0]);
  const double sum_dx = block_sum_f64_1024(b, sh[1]);
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
