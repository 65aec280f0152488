// Fused AdamW over the flat fp32 parameter arena, and the per-step weight
// preparation (fp32 torchvision KCRS master -> compute-dtype KRSC for the
// forward GEMM and CRSK for the data-gradient GEMM).
//
// AdamW semantics follow torch.optim.AdamW (the optimizer the reference
// builds at src/training/semi_supervised.py:115-122,265-272,291-298 and
// src/training/supervised.py:71-78; stepped at src/training/common.py:383):
//   p *= 1 - lr*wd
//   m  = lerp(m, g, 1-b1)          (torch lerp: m + w*(g-m) for w < 0.5)
//   v  = b2*v + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
#include "ssip_common.h"

namespace {

__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, float lr, float b1, float b2, float eps, float wd, float step_size,
                             float bc2_sqrt, float grad_scale) {
  const float decay = 1.f - lr * wd;
  const float w1 = 1.f - b1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * grad_scale;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = (w1 < 0.5f) ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// w (KCRS, f32) -> out_krsc[K][R][Sp][Cp] and out_crsk[Cp][R][Sp][K] (zero padded)
template <typename T>
__global__ void weight_prep_kernel(int K, int C, int R, int S, int Cp, int Sp, const float* __restrict__ w,
                                   T* __restrict__ krsc, T* __restrict__ crsk) {
  const long total = (long)K * R * Sp * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    long t = i / Cp;
    const int s = (int)(t % Sp);
    t /= Sp;
    const int r = (int)(t % R);
    const int k = (int)(t / R);
    const float v = (c < C && s < S) ? w[(((long)k * C + c) * R + r) * S + s] : 0.f;
    const T tv = from_f32<T>(v);
    if (krsc) krsc[i] = tv;
    if (crsk) crsk[(((long)c * R + r) * Sp + s) * K + k] = tv;
  }
}

}  // namespace

extern "C" {

int ssip_adamw(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float lr, float beta1,
               float beta2, float eps, float weight_decay, int64_t step, float grad_scale, void* stream) {
  SSIP_REQUIRE(n > 0 && param && grad && exp_avg && exp_avg_sq && step >= 1, SSIP_ERR_ARG, "ssip_adamw: bad arguments");
  // host-side scalars in double, as torch computes them in Python floats
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adamw_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (long)n, param, grad, exp_avg,
                     exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, grad_scale);
  return ::ssip::check_launch("adamw");
}

int ssip_weight_prep(int dtype, int K, int C, int R, int S, int Cp, int Sp, const float* w_kcrs, void* w_krsc,
                     void* w_crsk, void* stream) {
  SSIP_REQUIRE(K > 0 && C > 0 && R > 0 && S > 0 && Cp >= C && Sp >= S && w_kcrs && (w_krsc || w_crsk), SSIP_ERR_ARG,
               "ssip_weight_prep: bad arguments");
  const long total = (long)K * R * Sp * Cp;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(weight_prep_kernel<T>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, K, C, R, S, Cp, Sp,
                       w_kcrs, (T*)w_krsc, (T*)w_crsk);
  });
  return ::ssip::check_launch("weight_prep");
}

}  // extern "C"
