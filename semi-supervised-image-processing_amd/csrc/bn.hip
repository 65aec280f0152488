// BatchNorm2d (training + eval) for NHWC activations, with the ReLU and the
// BasicBlock residual add fused into the elementwise passes.
//
// Reference semantics (torchvision resnet18 BatchNorm2d, used through
// `model(inputs)` at src/training/common.py:380 and `model.train()` at :371):
// batch mean / biased variance normalise, running_var gets the unbiased
// variance, momentum 0.1, eps 1e-5.  In the frozen-backbone pretrain stage
// (src/training/semi_supervised.py:260-285) BN still runs in train mode, so
// the running statistics keep updating even though gamma/beta are frozen.
//
// Statistics: the conv FWD epilogue already produced per-(tile, channel)
// {count, sum, M2} records; `bn_finalize` merges them in fixed order in
// fp64 (two-pass: global mean, then sum of M2_t + n_t (mean_t - mean)^2).
// Backward: `bn_bwd_reduce` computes per-(row-block, channel) partial sums
// of dout and dout*xhat (dout = dz masked by the following ReLU), the
// finalize merges them in fp64, `bn_bwd_apply` writes
// dy = A*dout + B*y + Cc  (per-channel A, B, Cc) and optionally dout itself
// (the gradient that flows down the identity branch).
#include "ssip_common.h"
#include "bn_common.h"

namespace {

struct BnFwdFin {
  const float *gamma, *beta;
  float *running_mean, *running_var;
  float momentum, eps;
  int update_running;
  float *mean_out, *invstd_out, *scale_out, *shift_out;
};

__device__ __forceinline__ void bn_fin_write(int c, const BnFwdFin& f, double N, double mu, double m2) {
  const double var = N > 0.0 ? m2 / N : 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float g = f.gamma ? f.gamma[c] : 1.f, b = f.beta ? f.beta[c] : 0.f;
  const float scale = g * invstd;
  f.mean_out[c] = (float)mu;
  f.invstd_out[c] = invstd;
  f.scale_out[c] = scale;
  f.shift_out[c] = b - (float)mu * scale;
  if (f.update_running) {
    const double unbiased = N > 1 ? m2 / (N - 1) : var;
    f.running_mean[c] = (float)((1.0 - f.momentum) * f.running_mean[c] + f.momentum * mu);
    f.running_var[c] = (float)((1.0 - f.momentum) * f.running_var[c] + f.momentum * unbiased);
  }
}

// Workgroup (s, c): split s of channel c's per-tile {count, sum,
// M2-about-tile-mean} records in fp64, shifted by the split's first record's
// mean K (the shifted-data form of the pairwise merge):
//   n = sum n_t,  s = sum n_t (mean_t - K),  q = sum M2_t + n_t (mean_t - K)^2
//   mean = K + s / n,  M2 = q - s^2 / n.
// Threads take FIN_PT records at a time, NT apart, in increasing order; wave
// butterflies and (NT = 256) a 4-entry LDS combine in fixed order keep the
// result reproducible.  S == 1 writes the statistics; otherwise {n, mean, M2}
// of the split go to scratch[c][s] for bn_finalize_merge_kernel.
template <int NT>
__global__ void __launch_bounds__(NT) bn_finalize_kernel(int C, int tiles, int S, const float* __restrict__ partial,
                                                        double* scratch, BnFwdFin f) {
  const int c = blockIdx.y, s = blockIdx.x;
  const float* rec = partial + (long)c * tiles * 3;
  const int L = (tiles + S - 1) / S;
  const int t0 = s * L, t1 = min(tiles, t0 + L);
  double K = 0.0;
  if (t0 < t1) {
    const double n0 = rec[(long)t0 * 3];
    K = n0 > 0.0 ? (double)rec[(long)t0 * 3 + 1] / n0 : 0.0;
  }
  double v[3] = {0.0, 0.0, 0.0};
  for (int base = t0 + threadIdx.x; base < t1; base += NT * FIN_PT) {
    float r[FIN_PT][3];
#pragma unroll
    for (int i = 0; i < FIN_PT; ++i) {
      const int t = base + i * NT;
      const bool ok = t < t1;
      r[i][0] = ok ? rec[(long)t * 3] : 0.f;
      r[i][1] = ok ? rec[(long)t * 3 + 1] : 0.f;
      r[i][2] = ok ? rec[(long)t * 3 + 2] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FIN_PT; ++i) {
      const double nb = r[i][0];
      if (nb > 0.0) {
        const double d = (double)r[i][1] / nb - K;
        v[0] += nb;
        v[1] += nb * d;
        v[2] += (double)r[i][2] + nb * d * d;
      }
    }
  }
  if constexpr (NT == 64) {
    wave_sums_f64<3>(v);
  } else {
    __shared__ double sh[3 * 4];
    block_sums_f64_256<3>(v, sh);
  }
  if (threadIdx.x == 0) {
    const double N = v[0];
    const double mu = N > 0.0 ? K + v[1] / N : 0.0;
    const double m2 = N > 0.0 ? fmax(v[2] - v[1] * v[1] / N, 0.0) : 0.0;
    if (S == 1) {
      bn_fin_write(c, f, N, mu, m2);
    } else {
      double* o = scratch + ((long)c * S + s) * 3;
      o[0] = N;
      o[1] = mu;
      o[2] = m2;
    }
  }
}

// split finalize, second pass: one wave per channel merges the S split
// {n, mean, M2} in a fixed butterfly, shifted by split 0's mean
__global__ void __launch_bounds__(FIN_NT) bn_finalize_merge_kernel(int C, int S, const double* __restrict__ scratch,
                                                                   BnFwdFin f) {
  const int c = blockIdx.x * (FIN_NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const double* in = scratch + (long)c * S * 3;
  const double K = in[1];  // split 0's mean (0 when it is empty)
  double v[3] = {0.0, 0.0, 0.0};
  if (lane < S && in[lane * 3] > 0.0) {
    const double n = in[lane * 3], d = in[lane * 3 + 1] - K;
    v[0] = n;
    v[1] = n * d;
    v[2] = in[lane * 3 + 2] + n * d * d;
  }
  wave_sums_f64<3>(v);
  if (lane == 0) {
    const double N = v[0];
    const double mu = N > 0.0 ? K + v[1] / N : 0.0;
    const double m2 = N > 0.0 ? fmax(v[2] - v[1] * v[1] / N, 0.0) : 0.0;
    bn_fin_write(c, f, N, mu, m2);
  }
}

__global__ void bn_eval_coeffs_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                      float eps, float* mean_out, float* invstd_out, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * invstd;
  shift[c] = b - rm[c] * g * invstd;
  if (mean_out) mean_out[c] = rm[c];
  if (invstd_out) invstd_out[c] = invstd;
}

// z = act(y*scale + shift (+ residual)), 8 channels per thread.  The grid
// stride is a multiple of C/8 (blockDim 256, C/8 | 256), so each thread keeps
// one channel chunk and its scale/shift in registers; the grid is sized so a
// thread handles several vectors (the per-channel loads are amortised), two
// of them in flight per iteration.  DUAL: the residual is itself a BatchNorm
// output, res*scale2 + shift2, formed in registers (ssip_bn_apply2).
template <typename T, bool DUAL>
__global__ void __launch_bounds__(256) bn_apply_kernel(int total8, int C, const T* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       const float* __restrict__ scale2,
                                                       const float* __restrict__ shift2, int relu,
                                                       T* __restrict__ z, uint8_t* __restrict__ mbits) {
  const int cpr = C >> 3;
  const int start = blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (start % cpr) * 8;
  float sc[8], sh[8], sc2[8], sh2[8];
  load_f8(sc, scale + c0);
  load_f8(sh, shift + c0);
  if constexpr (DUAL) {
    load_f8(sc2, scale2 + c0);
    load_f8(sh2, shift2 + c0);
  }
  const int stride = gridDim.x * blockDim.x;
  auto one = [&](const Vec8<T>& v, const Vec8<T>& r, int i) {
    Vec8<T> o;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = __builtin_fmaf(v.get(j), sc[j], sh[j]);  // the stem's fused kernels repeat this exactly
      if constexpr (DUAL) t += __builtin_fmaf(r.get(j), sc2[j], sh2[j]);
      else if (res) t += r.get(j);
      if (relu) t = t > 0.f ? t : 0.f;
      o.set(j, t);
      bits |= (o.get(j) > 0.f ? 1u : 0u) << j;  // the stored value's sign: the backward's ReLU mask
    }
    o.store(z + (long)i * 8);
    if (mbits) mbits[i] = (uint8_t)bits;
  };
  int i = start;
  for (; i + stride < total8; i += 2 * stride) {
    Vec8<T> v0, v1, r0, r1;
    v0.load(y + (long)i * 8);
    v1.load(y + (long)(i + stride) * 8);
    if (res) {
      r0.load(res + (long)i * 8);
      r1.load(res + (long)(i + stride) * 8);
    }
    one(v0, r0, i);
    one(v1, r1, i + stride);
  }
  if (i < total8) {
    Vec8<T> v0, r0;
    v0.load(y + (long)i * 8);
    if (res) r0.load(res + (long)i * 8);
    one(v0, r0, i);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(int total8, int C, const T* __restrict__ dz,
                                                           const T* __restrict__ zmask,
                                                           const uint8_t* __restrict__ mbits, const T* __restrict__ y,
                                                           const float* __restrict__ coef, T* __restrict__ dy,
                                                           T* __restrict__ dpre, const float* __restrict__ mscale,
                                                           const float* __restrict__ mshift) {
  const int cpr = C >> 3;
  const int start = blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (start % cpr) * 8;
  float ca[8], cb[8], cc[8], msc[8], msh[8];
  const bool amask = mscale != nullptr;
  load_f8(ca, coef + c0);
  load_f8(cb, coef + C + c0);
  load_f8(cc, coef + 2 * C + c0);
  if (amask) {
    load_f8(msc, mscale + c0);
    load_f8(msh, mshift + c0);
  }
  const int stride = gridDim.x * blockDim.x;
  auto one = [&](const Vec8<T>& g, const Vec8<T>& zz, const Vec8<T>& yy, int i) {
    Vec8<T> o, p;
    const uint32_t mb = mbits ? mbits[i] : 0xFFu;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = g.get(j);
      if (zmask) d = zz.get(j) > 0.f ? d : 0.f;
      if (amask) d = __builtin_fmaf(yy.get(j), msc[j], msh[j]) > 0.f ? d : 0.f;
      d = ((mb >> j) & 1u) ? d : 0.f;
      p.set(j, d);
      o.set(j, ca[j] * d + cb[j] * yy.get(j) + cc[j]);
    }
    o.store(dy + (long)i * 8);
    if (dpre) p.store(dpre + (long)i * 8);
  };
  int i = start;
  for (; i + stride < total8; i += 2 * stride) {
    Vec8<T> g0, g1, z0, z1, y0, y1;
    g0.load(dz + (long)i * 8);
    g1.load(dz + (long)(i + stride) * 8);
    y0.load(y + (long)i * 8);
    y1.load(y + (long)(i + stride) * 8);
    if (zmask) {
      z0.load(zmask + (long)i * 8);
      z1.load(zmask + (long)(i + stride) * 8);
    }
    one(g0, z0, y0, i);
    one(g1, z1, y1, i + stride);
  }
  if (i < total8) {
    Vec8<T> g0, z0, y0;
    g0.load(dz + (long)i * 8);
    y0.load(y + (long)i * 8);
    if (zmask) z0.load(zmask + (long)i * 8);
    one(g0, z0, y0, i);
  }
}

// Backward of z = relu(BN_a(ya) + BN_b(yb)): dout = dz * (zmask > 0) is the
// gradient of both BN outputs.  Per-(row block, channel) sums of dout,
// dout*xhat_a and dout*xhat_b, written as two [C][blocks][2] partial sets
// (sum dout duplicated) that the ordinary finalize consumes.
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_dual_kernel(long M, int C, int rows_per_block,
                                                                 const T* __restrict__ dz,
                                                                 const T* __restrict__ zmask,
                                                                 const uint8_t* __restrict__ mbits,
                                                                 const T* __restrict__ ya, const T* __restrict__ yb,
                                                                 const float* __restrict__ mean_a,
                                                                 const float* __restrict__ invstd_a,
                                                                 const float* __restrict__ mean_b,
                                                                 const float* __restrict__ invstd_b,
                                                                 float* __restrict__ partial_a,
                                                                 float* __restrict__ partial_b) {
  const int cpr = C / 8;
  const int rpi = 256 / cpr;
  const int chunk = threadIdx.x % cpr;
  const int rsub = threadIdx.x / cpr;
  const int c0 = chunk * 8;
  const long r0 = (long)blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float sd[8], sa[8], sb[8], mua[8], isa[8], mub[8], isb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sd[j] = 0.f; sa[j] = 0.f; sb[j] = 0.f; }
  load_f8(mua, mean_a + c0);
  load_f8(isa, invstd_a + c0);
  load_f8(mub, mean_b + c0);
  load_f8(isb, invstd_b + c0);
  auto acc = [&](const Vec8<T>& g, const Vec8<T>& zz, uint32_t mb, const Vec8<T>& a, const Vec8<T>& b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool on = mbits ? ((mb >> j) & 1u) != 0 : zz.get(j) > 0.f;
      const float d = on ? g.get(j) : 0.f;
      sd[j] += d;
      sa[j] += d * ((a.get(j) - mua[j]) * isa[j]);
      sb[j] += d * ((b.get(j) - mub[j]) * isb[j]);
    }
  };
  if (rsub < rpi) {
    // four rows in flight per thread, accumulated in plain-walk order
    constexpr int U = 4;
    long r = r0 + rsub;
    for (; r + (U - 1) * rpi < r1; r += U * rpi) {
      Vec8<T> g[U], z[U], av[U], bv[U];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + (long)u * rpi;
        g[u].load(dz + rr * C + c0);
        mb[u] = 0;
        if (mbits) mb[u] = mbits[rr * cpr + chunk];
        else z[u].load(zmask + rr * C + c0);
        av[u].load(ya + rr * C + c0);
        bv[u].load(yb + rr * C + c0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc(g[u], z[u], mb[u], av[u], bv[u]);
    }
    for (; r < r1; r += rpi) {
      Vec8<T> g0, z0, a0, b0;
      uint32_t m0 = 0;
      g0.load(dz + r * C + c0);
      if (mbits) m0 = mbits[r * cpr + chunk];
      else z0.load(zmask + r * C + c0);
      a0.load(ya + r * C + c0);
      b0.load(yb + r * C + c0);
      acc(g0, z0, m0, a0, b0);
    }
  }
  __shared__ float red[256][25];
  float v[3][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[0][j] = sd[j];
    v[1][j] = sa[j];
    v[2][j] = sb[j];
  }
  chunk_sums<3>(v, cpr, red);
  if (threadIdx.x < cpr) {
    const long o = ((long)c0 * gridDim.x + blockIdx.x) * 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long oj = o + (long)j * gridDim.x * 2;
      partial_a[oj] = v[0][j];
      partial_a[oj + 1] = v[1][j];
      partial_b[oj] = v[0][j];
      partial_b[oj + 1] = v[2][j];
    }
  }
}

// dy_a = A_a*dout + B_a*ya + C_a,  dy_b = A_b*dout + B_b*yb + C_b
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_apply_dual_kernel(int total8, int C, const T* __restrict__ dz,
                                                                const T* __restrict__ zmask,
                                                                const uint8_t* __restrict__ mbits,
                                                                const T* __restrict__ ya, const T* __restrict__ yb,
                                                                const float* __restrict__ coef_a,
                                                                const float* __restrict__ coef_b,
                                                                T* __restrict__ dya, T* __restrict__ dyb) {
  const int cpr = C >> 3;
  const int start = blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (start % cpr) * 8;
  float aa[8], ab[8], ac[8], ba[8], bb[8], bc[8];
  load_f8(aa, coef_a + c0);
  load_f8(ab, coef_a + C + c0);
  load_f8(ac, coef_a + 2 * C + c0);
  load_f8(ba, coef_b + c0);
  load_f8(bb, coef_b + C + c0);
  load_f8(bc, coef_b + 2 * C + c0);
  const int stride = gridDim.x * blockDim.x;
  for (int i = start; i < total8; i += stride) {
    Vec8<T> g, zz, a, b, oa, ob;
    uint32_t mb = 0;
    g.load(dz + (long)i * 8);
    if (mbits) mb = mbits[i];
    else zz.load(zmask + (long)i * 8);
    a.load(ya + (long)i * 8);
    b.load(yb + (long)i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool on = mbits ? ((mb >> j) & 1u) != 0 : zz.get(j) > 0.f;
      const float d = on ? g.get(j) : 0.f;
      oa.set(j, aa[j] * d + ab[j] * a.get(j) + ac[j]);
      ob.set(j, ba[j] * d + bb[j] * b.get(j) + bc[j]);
    }
    oa.store(dya + (long)i * 8);
    ob.store(dyb + (long)i * 8);
  }
}

// dst = src * (mask > 0)  (ReLU backward as a standalone pass)
template <typename T>
__global__ void relu_bwd_kernel(long total8, const T* __restrict__ g, const T* __restrict__ z, T* __restrict__ out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total8; i += (long)gridDim.x * blockDim.x) {
    Vec8<T> a, m, o;
    a.load(g + i * 8);
    m.load(z + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) o.set(j, m.get(j) > 0.f ? a.get(j) : 0.f);
    o.store(out + i * 8);
  }
}

static int grid_for(long n, int per_block = 256) {
  long b = (n + per_block - 1) / per_block;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

// elementwise BN passes: >= 4 vectors per thread where the tensor allows,
// at most 2048 workgroups (8 per CU)
static int bn_elem_grid(long total8) {
  long b = (total8 + 1023) / 1024;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}


}  // namespace

extern "C" {

int ssip_bn_finalize(int C, int tiles, float* partial, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int update_running,
                     float* mean_out, float* invstd_out, float* scale_out, float* shift_out, void* stream) {
  SSIP_REQUIRE(C > 0 && tiles > 0 && partial && mean_out && invstd_out && scale_out && shift_out, SSIP_ERR_ARG,
               "ssip_bn_finalize: bad arguments");
  SSIP_REQUIRE(!update_running || (running_mean && running_var), SSIP_ERR_ARG, "running stats required");
  hipStream_t st = (hipStream_t)stream;
  const BnFwdFin f{gamma, beta, running_mean, running_var, momentum, eps, update_running,
                   mean_out, invstd_out, scale_out, shift_out};
  const int S = fin_splits(tiles);
  double* scratch = fin_scratch(partial, (int64_t)C * tiles * 3);
  // SSIP_FIN64=1: one-wave, LDS-free workgroups where one per channel
  // suffices.  They fit beside a persistent kernel that holds a CU's whole LDS
  // (the other stream's layer-1 halo conv), where a 256-thread workgroup with
  // its 96-B combine waits for it to finish: layer-1 finalize 42 -> 20 us in
  // the step trace, but the step moved -0.55 % on one box and +0.8 % on
  // another (round 5): off by default.
  static const bool nt64 = [] {
    const char* e = getenv("SSIP_FIN64");
    return e != nullptr && e[0] == '1';
  }();
  if (nt64 && S == 1)
    SSIP_KLAUNCH(bn_finalize_kernel<64>, dim3(S, C), dim3(64), 0, st, C, tiles, S, (const float*)partial,
                       scratch, f);
  else
    SSIP_KLAUNCH(bn_finalize_kernel<FIN_NT>, dim3(S, C), dim3(FIN_NT), 0, st, C, tiles, S,
                       (const float*)partial, scratch, f);
  if (S > 1)
    SSIP_KLAUNCH(bn_finalize_merge_kernel, dim3((C + FIN_NT / 64 - 1) / (FIN_NT / 64)), dim3(FIN_NT), 0, st,
                       C, S, (const double*)scratch, f);
  return ::ssip::check_launch("bn_finalize");
}

int64_t ssip_bn_finalize_scratch_floats(int C, int tiles) {
  if (C <= 0 || tiles <= 0) return -1;
  return fin_scratch_floats(C, tiles, 3);
}

int ssip_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float* mean_out, float* invstd_out, float* scale_out,
                        float* shift_out, void* stream) {
  SSIP_REQUIRE(C > 0 && running_mean && running_var && scale_out && shift_out, SSIP_ERR_ARG,
               "ssip_bn_eval_coeffs: bad arguments");
  SSIP_KLAUNCH(bn_eval_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C, gamma, beta,
                     running_mean, running_var, eps, mean_out, invstd_out, scale_out, shift_out);
  return ::ssip::check_launch("bn_eval_coeffs");
}

int ssip_bn_apply(int dtype, int64_t M, int C, const void* y, const float* scale, const float* shift,
                  const void* residual, int relu, void* z, uint8_t* mask_bits, void* stream) {
  SSIP_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && y && scale && shift && z, SSIP_ERR_ARG, "ssip_bn_apply: bad arguments");
  SSIP_REQUIRE(M * C / 8 < (1l << 31) && 256 % (C / 8) == 0, SSIP_ERR_ARG, "ssip_bn_apply: unsupported size");
  const int total8 = (int)(M * C / 8);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH((bn_apply_kernel<T, false>), dim3(bn_elem_grid(total8)), dim3(256), 0, (hipStream_t)stream,
                       total8, C, (const T*)y, scale, shift, (const T*)residual, (const float*)nullptr,
                       (const float*)nullptr, relu, (T*)z, mask_bits);
  });
  return ::ssip::check_launch("bn_apply");
}

int ssip_bn_apply2(int dtype, int64_t M, int C, const void* y, const float* scale, const float* shift,
                   const void* y2, const float* scale2, const float* shift2, int relu, void* z, uint8_t* mask_bits,
                   void* stream) {
  SSIP_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && y && scale && shift && y2 && scale2 && shift2 && z, SSIP_ERR_ARG,
               "ssip_bn_apply2: bad arguments");
  SSIP_REQUIRE(M * C / 8 < (1l << 31) && 256 % (C / 8) == 0, SSIP_ERR_ARG, "ssip_bn_apply2: unsupported size");
  const int total8 = (int)(M * C / 8);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH((bn_apply_kernel<T, true>), dim3(bn_elem_grid(total8)), dim3(256), 0, (hipStream_t)stream,
                       total8, C, (const T*)y, scale, shift, (const T*)y2, scale2, shift2, relu, (T*)z, mask_bits);
  });
  return ::ssip::check_launch("bn_apply2");
}

int64_t ssip_bn_bwd_dual_partial_floats(int64_t M, int C) {
  if (M <= 0 || C <= 0 || C % 8 || C > 2048) return -1;
  const int rows = bwd_rows_per_block(M, C);
  const long blocks = (M + rows - 1) / rows;
  return 2 * (blocks * (int64_t)C * 2 + fin_scratch_floats(C, blocks, 2));
}

int ssip_bn_bwd_dual(int dtype, int64_t M, int C, const void* dz, const void* zmask, const uint8_t* mask_bits,
                     const void* ya,
                     const float* mean_a, const float* invstd_a, const float* gamma_a, float* dgamma_a,
                     float* dbeta_a, const void* yb, const float* mean_b, const float* invstd_b,
                     const float* gamma_b, float* dgamma_b, float* dbeta_b, int accumulate, void* dy_a, void* dy_b,
                     float* partial, float* coef, void* stream) {
  SSIP_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && C <= 2048 && dz && (zmask || mask_bits) && ya && yb && mean_a && invstd_a &&
                   mean_b && invstd_b && dy_a && dy_b && partial && coef,
               SSIP_ERR_ARG, "ssip_bn_bwd_dual: bad arguments");
  SSIP_REQUIRE(M * C / 8 < (1l << 31) && 256 % (C / 8) == 0, SSIP_ERR_ARG, "ssip_bn_bwd_dual: unsupported size");
  hipStream_t st = (hipStream_t)stream;
  const int rows = bwd_rows_per_block(M, C);
  const int blocks = (int)((M + rows - 1) / rows);
  const int total8 = (int)(M * C / 8);
  float* pa = partial;
  float* pb = partial + (long)blocks * C * 2;
  double* scratch = fin_scratch(partial, 2 * (int64_t)blocks * C * 2);
  const int S = fin_splits(blocks);
  BnBwdFin f;
  f.set[0] = bn_bwd_fin_set(pa, gamma_a, mean_a, invstd_a, dgamma_a, dbeta_a, coef, scratch);
  f.set[1] = bn_bwd_fin_set(pb, gamma_b, mean_b, invstd_b, dgamma_b, dbeta_b, coef + 3 * C,
                            scratch + (int64_t)C * S * 2);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(bn_bwd_reduce_dual_kernel<T>, dim3(blocks), dim3(256), 0, st, (long)M, C, rows, (const T*)dz,
                       (const T*)zmask, mask_bits, (const T*)ya, (const T*)yb, mean_a, invstd_a, mean_b, invstd_b, pa,
                       pb);
    launch_bn_bwd_finalize(st, C, blocks, (long)M, 1, 2, f, accumulate);
    SSIP_KLAUNCH(bn_bwd_apply_dual_kernel<T>, dim3(bn_elem_grid(total8)), dim3(256), 0, st, total8, C,
                       (const T*)dz, (const T*)zmask, mask_bits, (const T*)ya, (const T*)yb, coef, coef + 3 * C, (T*)dy_a,
                       (T*)dy_b);
  });
  return ::ssip::check_launch("bn_bwd_dual");
}

int64_t ssip_bn_bwd_partial_floats(int64_t M, int C) {
  if (M <= 0 || C <= 0 || C % 8 || C > 2048) return -1;
  const int rows = bwd_rows_per_block(M, C);
  const long blocks = (M + rows - 1) / rows;
  return blocks * (int64_t)C * 2 + fin_scratch_floats(C, blocks, 2);
}

static int bn_bwd_impl(int dtype, int64_t M, int C, const void* dz, const void* zmask, const uint8_t* mbits,
                       const float* mscale,
                       const float* mshift, const void* y, const float* mean, const float* invstd,
                       const float* gamma, float* dgamma, float* dbeta, int accumulate, void* dy, void* dpre,
                       float* partial, float* coef, void* stream) {
  SSIP_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && C <= 2048 && dz && y && mean && invstd && dy && partial && coef,
               SSIP_ERR_ARG, "ssip_bn_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int rows = bwd_rows_per_block(M, C);
  const int blocks = (int)((M + rows - 1) / rows);
  SSIP_REQUIRE(M * C / 8 < (1l << 31) && 256 % (C / 8) == 0, SSIP_ERR_ARG, "ssip_bn_bwd: unsupported size");
  const int total8 = (int)(M * C / 8);
  // (64-VGPR 4-channel forms that fit beside a resident wgrad made the step
  // slower, 6.70 vs 6.50 ms: r3-variants branch)
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(bn_bwd_reduce_kernel<T>, dim3(blocks), dim3(256), 0, st, (long)M, C, rows, (const T*)dz,
                       (const T*)zmask, mbits, (const T*)y, mean, invstd, mscale, mshift, partial);
    BnBwdFin f;
    f.set[0] = bn_bwd_fin_set(partial, gamma, mean, invstd, dgamma, dbeta, coef,
                              fin_scratch(partial, (int64_t)blocks * C * 2));
    launch_bn_bwd_finalize(st, C, blocks, (long)M, 1, 1, f, accumulate);
    SSIP_KLAUNCH(bn_bwd_apply_kernel<T>, dim3(bn_elem_grid(total8)), dim3(256), 0, st, total8, C,
                       (const T*)dz, (const T*)zmask, mbits, (const T*)y, coef, (T*)dy, (T*)dpre, mscale, mshift);
  });
  return ::ssip::check_launch("bn_bwd");
}

int ssip_bn_bwd_from_partials(int dtype, int64_t M, int C, int tiles, float* partial, const void* dout,
                              const void* y, const float* mean, const float* invstd, const float* gamma,
                              float* dgamma, float* dbeta, int accumulate, void* dy, float* coef, void* stream) {
  SSIP_REQUIRE(M > 0 && C > 0 && C % 8 == 0 && tiles > 0 && partial && dout && y && mean && invstd && dy && coef,
               SSIP_ERR_ARG, "ssip_bn_bwd_from_partials: bad arguments");
  SSIP_REQUIRE(M * C / 8 < (1l << 31) && 256 % (C / 8) == 0, SSIP_ERR_ARG,
               "ssip_bn_bwd_from_partials: unsupported size");
  hipStream_t st = (hipStream_t)stream;
  const int total8 = (int)(M * C / 8);
  BnBwdFin f;
  f.set[0] = bn_bwd_fin_set(partial, gamma, mean, invstd, dgamma, dbeta, coef,
                            fin_scratch(partial, (int64_t)tiles * C * 2));
  launch_bn_bwd_finalize(st, C, tiles, (long)M, 1, 1, f, accumulate);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(bn_bwd_apply_kernel<T>, dim3(bn_elem_grid(total8)), dim3(256), 0, st, total8, C, (const T*)dout,
                       (const T*)nullptr, (const uint8_t*)nullptr, (const T*)y, coef, (T*)dy, (T*)nullptr,
                       (const float*)nullptr,
                       (const float*)nullptr);
  });
  return ::ssip::check_launch("bn_bwd_from_partials");
}

int ssip_bn_bwd(int dtype, int64_t M, int C, const void* dz, const void* zmask, const uint8_t* mask_bits,
                const void* y, const float* mean,
                const float* invstd, const float* gamma, float* dgamma, float* dbeta, int accumulate, void* dy,
                void* dpre, float* partial, float* coef, void* stream) {
  return bn_bwd_impl(dtype, M, C, dz, zmask, mask_bits, nullptr, nullptr, y, mean, invstd, gamma, dgamma, dbeta,
                     accumulate, dy,
                     dpre, partial, coef, stream);
}

int ssip_bn_relu_bwd(int dtype, int64_t M, int C, const void* dz, const void* y, const float* mean,
                     const float* invstd, const float* scale, const float* shift, const float* gamma, float* dgamma,
                     float* dbeta, int accumulate, void* dy, float* partial, float* coef, void* stream) {
  SSIP_REQUIRE(scale && shift, SSIP_ERR_ARG, "ssip_bn_relu_bwd: scale/shift required");
  return bn_bwd_impl(dtype, M, C, dz, nullptr, nullptr, scale, shift, y, mean, invstd, gamma, dgamma, dbeta,
                     accumulate, dy,
                     nullptr, partial, coef, stream);
}

int ssip_relu_bwd(int dtype, int64_t n, const void* g, const void* z, void* out, void* stream) {
  SSIP_REQUIRE(n > 0 && n % 8 == 0 && g && z && out, SSIP_ERR_ARG, "ssip_relu_bwd: bad arguments");
  const long total8 = n / 8;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(relu_bwd_kernel<T>, dim3(grid_for(total8)), dim3(256), 0, (hipStream_t)stream, total8,
                       (const T*)g, (const T*)z, (T*)out);
  });
  return ::ssip::check_launch("relu_bwd");
}

}  // extern "C"
