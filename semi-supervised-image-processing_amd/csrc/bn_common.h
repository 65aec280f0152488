// BatchNorm backward finalize shared by bn.hip and stem.hip: per-channel sums
// of dout and dout*xhat from [blocks][C][2] partials (fixed-order fp64 tree)
// -> dgamma/dbeta and the apply coefficients
//   dy = coef[c] * dout + coef[C+c] * y + coef[2C+c].
#pragma once
#include "ssip_common.h"

namespace {

__global__ void __launch_bounds__(1024) bn_bwd_finalize_kernel(int C, int blocks, long M,
                                                               const float* __restrict__ partial,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd, float* dgamma,
                                                               float* dbeta, int accumulate, float* coef) {
  const int c = blockIdx.x;
  __shared__ double r0[1024], r1[1024];
  double a = 0.0, b = 0.0;
  for (int t = threadIdx.x; t < blocks; t += blockDim.x) {
    a += partial[((long)t * C + c) * 2 + 0];
    b += partial[((long)t * C + c) * 2 + 1];
  }
  r0[threadIdx.x] = a;
  r1[threadIdx.x] = b;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      r0[threadIdx.x] += r0[threadIdx.x + o];
      r1[threadIdx.x] += r1[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double sum_d = r0[0], sum_dx = r1[0];
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

}  // namespace
