// The stem's BN -> ReLU -> max-pool, fused (torchvision resnet `bn1 -> relu ->
// maxpool` inside `model(inputs)`, src/training/common.py:380, and the
// matching backward reached by `loss.backward()`, common.py:382).
//
// Forward: the pooled map is computed straight from the pre-BN conv output y:
//   z = T(relu(fma(y, scale, shift)))   (bit-identical to ssip_bn_apply)
//   out/idx = max-pool of z with torch's first-max tie break
// so the full-resolution z (411 MB at batch 256 bf16) is never written or
// read back.  Backward recomputes what it needs from y, the pooled gradient
// and the argmax bytes:
//   dz(h,w)   = sum of dpool over the windows whose argmax is (h,w)  (gather)
//   dpre      = dz * (fma(y, scale, shift) > 0)                      (ReLU mask)
//   sums      = sum dpre, sum dpre * (y - mean) * invstd             (pass 1)
//   dy        = A * dpre + B * y + C                                 (pass 2)
// replacing ssip_maxpool_bwd + ssip_bn_bwd's three full-resolution passes.
#include "ssip_common.h"

namespace {

__device__ __forceinline__ float bn_relu(float y, float sc, float sh) {
  const float t = __builtin_fmaf(y, sc, sh);
  return t > 0.f ? t : 0.f;
}

template <typename T>
__global__ void stem_bn_pool_fwd_kernel(int N, int H, int W, int C, int P, int Q, int k, int s, int pad,
                                        const T* __restrict__ y, const float* __restrict__ scale,
                                        const float* __restrict__ shift, T* __restrict__ out,
                                        uint8_t* __restrict__ idx) {
  const int cpr = C / 8;
  const long total = (long)N * P * Q * cpr;
  // the grid stride is a multiple of cpr (blockDim 256, cpr | 256): fixed chunk per thread
  const long start = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int cc = (int)(start % cpr);
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = scale[cc * 8 + j]; sh[j] = shift[cc * 8 + j]; }
  for (long i = start; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i / cpr;
    const int q = t % Q;
    t /= Q;
    const int p = t % P;
    const int n = (int)(t / P);
    float best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = -1; }
    for (int r = 0; r < k; ++r) {
      const int h = p * s - pad + r;
      if (h < 0 || h >= H) continue;
      for (int u = 0; u < k; ++u) {
        const int w = q * s - pad + u;
        if (w < 0 || w >= W) continue;
        Vec8<T> v;
        v.load(y + (((long)n * H + h) * W + w) * C + cc * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // the value ssip_bn_apply would have stored
          const float f = to_f32(from_f32<T>(bn_relu(v.get(j), sc[j], sh[j])));
          if (bi[j] < 0 || f > best[j] || f != f) { best[j] = f; bi[j] = r * k + u; }
        }
      }
    }
    Vec8<T> o;
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o.set(j, best[j]);
      packed |= (uint64_t)(uint8_t)bi[j] << (8 * j);
    }
    o.store(out + i * 8);
    *reinterpret_cast<uint64_t*>(idx + i * 8) = packed;
  }
}

// dz at (n, h, w, chunk): pooled gradients of the windows that chose (h, w),
// summed in output order (p, q ascending) like ssip_maxpool_bwd.
template <typename T>
__device__ __forceinline__ void pool_grad_gather(int n, int h, int w, int cc, int C, int P, int Q, int k, int s,
                                                 int pad, const T* __restrict__ dpool,
                                                 const uint8_t* __restrict__ idx, float (&acc)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int plo = h + pad - k + 1;
  plo = plo <= 0 ? 0 : (plo + s - 1) / s;
  int phi = (h + pad) / s;
  if (phi > P - 1) phi = P - 1;
  int qlo = w + pad - k + 1;
  qlo = qlo <= 0 ? 0 : (qlo + s - 1) / s;
  int qhi = (w + pad) / s;
  if (qhi > Q - 1) qhi = Q - 1;
  for (int p = plo; p <= phi; ++p) {
    const int r = h - (p * s - pad);
    for (int q = qlo; q <= qhi; ++q) {
      const int u = w - (q * s - pad);
      const int pos = r * k + u;
      const long o = (((long)n * P + p) * Q + q) * C + cc * 8;
      const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
      // skip the gradient load when no channel of this chunk chose (h, w)
      bool any = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) any |= (int)((packed >> (8 * j)) & 0xff) == pos;
      if (!any) continue;
      Vec8<T> g;
      g.load(dpool + o);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((int)((packed >> (8 * j)) & 0xff) == pos) acc[j] += g.get(j);
    }
  }
}

// pass 1: per-(row block, channel) {sum dpre, sum dpre*xhat}; layout
// [blocks][C][2] as ssip_bn_bwd's reduction (finalized by the same kernel).
template <typename T>
__global__ void stem_pool_bn_bwd_reduce_kernel(int N, int H, int W, int C, int P, int Q, int k, int s, int pad,
                                               int rows_per_block, const T* __restrict__ dpool,
                                               const uint8_t* __restrict__ idx, const T* __restrict__ y,
                                               const float* __restrict__ scale, const float* __restrict__ shift,
                                               const float* __restrict__ mean, const float* __restrict__ invstd,
                                               float* __restrict__ partial) {
  const int cpr = C / 8;
  const int rpi = 256 / cpr;
  const int chunk = threadIdx.x % cpr;
  const int rsub = threadIdx.x / cpr;
  const int c0 = chunk * 8;
  const long M = (long)N * H * W;
  const long r0 = (long)blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float sd[8], sx[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sd[j] = 0.f; sx[j] = 0.f;
    mu[j] = mean[c0 + j]; is[j] = invstd[c0 + j];
    sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j];
  }
  if (rsub < rpi) {
    for (long r = r0 + rsub; r < r1; r += rpi) {
      const int w = (int)(r % W);
      const long t = r / W;
      const int h = (int)(t % H);
      const int n = (int)(t / H);
      float dz[8];
      pool_grad_gather<T>(n, h, w, chunk, C, P, Q, k, s, pad, dpool, idx, dz);
      Vec8<T> yy;
      yy.load(y + r * C + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float yv = yy.get(j);
        const float d = bn_relu(yv, sc[j], sh[j]) > 0.f ? dz[j] : 0.f;
        sd[j] += d;
        sx[j] += d * ((yv - mu[j]) * is[j]);
      }
    }
  }
  __shared__ float red[2][256][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x][j] = sd[j];
    red[1][threadIdx.x][j] = sx[j];
  }
  __syncthreads();
  if (threadIdx.x < cpr) {
    float* o = partial + ((long)blockIdx.x * C + c0) * 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f, b = 0.f;
      for (int q = 0; q < rpi; ++q) {
        a += red[0][q * cpr + threadIdx.x][j];
        b += red[1][q * cpr + threadIdx.x][j];
      }
      o[2 * j] = a;
      o[2 * j + 1] = b;
    }
  }
}

__global__ void stem_bwd_finalize_kernel(int C, int blocks, long M, const float* __restrict__ partial,
                                         const float* __restrict__ gamma, const float* __restrict__ mean,
                                         const float* __restrict__ invstd, float* dgamma, float* dbeta,
                                         int accumulate, float* coef) {
  const int c = blockIdx.x;
  __shared__ double r0[256], r1[256];
  double a = 0.0, b = 0.0;
  for (int t = threadIdx.x; t < blocks; t += blockDim.x) {
    a += partial[((long)t * C + c) * 2 + 0];
    b += partial[((long)t * C + c) * 2 + 1];
  }
  r0[threadIdx.x] = a;
  r1[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
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
    coef[c] = (float)A;
    coef[C + c] = (float)k1;
    coef[2 * C + c] = (float)(k0 - k1 * mean[c]);
  }
}

// pass 2: dy = A * dpre + B * y + C, dpre recomputed by the same gather
template <typename T>
__global__ void stem_pool_bn_bwd_apply_kernel(int N, int H, int W, int C, int P, int Q, int k, int s, int pad,
                                              const T* __restrict__ dpool, const uint8_t* __restrict__ idx,
                                              const T* __restrict__ y, const float* __restrict__ scale,
                                              const float* __restrict__ shift, const float* __restrict__ coef,
                                              T* __restrict__ dy) {
  const int cpr = C / 8;
  const long total = (long)N * H * W * cpr;
  const long start = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int cc = (int)(start % cpr);
  const int c0 = cc * 8;
  float ca[8], cb[8], ck[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = coef[c0 + j]; cb[j] = coef[C + c0 + j]; ck[j] = coef[2 * C + c0 + j];
    sc[j] = scale[c0 + j]; sh[j] = shift[c0 + j];
  }
  for (long i = start; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr;
    const int w = (int)(r % W);
    const long t = r / W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float dz[8];
    pool_grad_gather<T>(n, h, w, cc, C, P, Q, k, s, pad, dpool, idx, dz);
    Vec8<T> yy, o;
    yy.load(y + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float yv = yy.get(j);
      const float d = bn_relu(yv, sc[j], sh[j]) > 0.f ? dz[j] : 0.f;
      o.set(j, ca[j] * d + cb[j] * yv + ck[j]);
    }
    o.store(dy + i * 8);
  }
}

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

static int rows_per_block(long M, int C) {
  const int rpi = 256 / (C / 8);
  long rows = (M + 1023) / 1024;
  if (rows < rpi) rows = rpi;
  rows = ((rows + rpi - 1) / rpi) * rpi;
  return (int)rows;
}

}  // namespace

extern "C" {

int ssip_stem_bn_pool_fwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* y,
                          const float* scale, const float* shift, void* out, uint8_t* idx, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && 256 % (C / 8) == 0 && k > 0 && k * k <= 255 && s > 0 &&
                   y && scale && shift && out && idx,
               SSIP_ERR_ARG, "ssip_stem_bn_pool_fwd: bad arguments");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  const long total = (long)N * P * Q * (C / 8);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(stem_bn_pool_fwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, H,
                       W, C, P, Q, k, s, pad, (const T*)y, scale, shift, (T*)out, idx);
  });
  return ::ssip::check_launch("stem_bn_pool_fwd");
}

int64_t ssip_stem_pool_bn_bwd_partial_floats(int N, int H, int W, int C) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || 256 % (C / 8)) return -1;
  const long M = (long)N * H * W;
  const int rows = rows_per_block(M, C);
  return ((M + rows - 1) / rows) * (int64_t)C * 2;
}

int ssip_stem_pool_bn_bwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* dpool,
                          const uint8_t* idx, const void* y, const float* mean, const float* invstd,
                          const float* scale, const float* shift, const float* gamma, float* dgamma, float* dbeta,
                          int accumulate, void* dy, float* partial, float* coef, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && 256 % (C / 8) == 0 && k > 0 && k * k <= 255 && s > 0 &&
                   dpool && idx && y && mean && invstd && scale && shift && dy && partial && coef,
               SSIP_ERR_ARG, "ssip_stem_pool_bn_bwd: bad arguments");
  const long M = (long)N * H * W;
  SSIP_REQUIRE(M * C / 8 < (1l << 31), SSIP_ERR_ARG, "ssip_stem_pool_bn_bwd: too large");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  const int rows = rows_per_block(M, C);
  const int blocks = (int)((M + rows - 1) / rows);
  hipStream_t st = (hipStream_t)stream;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    hipLaunchKernelGGL(stem_pool_bn_bwd_reduce_kernel<T>, dim3(blocks), dim3(256), 0, st, N, H, W, C, P, Q, k, s,
                       pad, rows, (const T*)dpool, idx, (const T*)y, scale, shift, mean, invstd, partial);
    hipLaunchKernelGGL(stem_bwd_finalize_kernel, dim3(C), dim3(256), 0, st, C, blocks, M, partial, gamma, mean,
                       invstd, dgamma, dbeta, accumulate, coef);
    hipLaunchKernelGGL(stem_pool_bn_bwd_apply_kernel<T>, dim3(grid_for(M * C / 8)), dim3(256), 0, st, N, H, W, C, P,
                       Q, k, s, pad, (const T*)dpool, idx, (const T*)y, scale, shift, coef, (T*)dy);
  });
  return ::ssip::check_launch("stem_pool_bn_bwd");
}

}  // extern "C"
