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
#include "bn_common.h"

namespace {

__device__ __forceinline__ float bn_relu(float y, float sc, float sh) {
  const float t = __builtin_fmaf(y, sc, sh);
  return t > 0.f ? t : 0.f;
}

// One workgroup per pooled output row (n, p); threads walk (q, channel chunk)
// with a fixed chunk per thread (blockDim % (C/8) == 0): no 64-bit index math.
template <typename T>
__global__ void __launch_bounds__(256) stem_bn_pool_fwd_kernel(int H, int W, int C, int P, int Q, int k, int s,
                                                               int pad, const T* __restrict__ y,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, T* __restrict__ out,
                                                               uint8_t* __restrict__ idx, T* __restrict__ ymax) {
  const int cpr = C >> 3;
  const int row = blockIdx.x;  // n * P + p
  const int n = row / P, p = row - (row / P) * P;
  const int cc = threadIdx.x % cpr;
  float sc[8], sh[8];
  load_f8(sc, scale + cc * 8);
  load_f8(sh, shift + cc * 8);
  const T* yb = y + (long)n * H * W * C + cc * 8;
  if (k == 3) {
    // all nine window loads issued before the first compare (out-of-image
    // taps are skipped by the ok mask, in the same r, u order)
    for (int e = threadIdx.x; e < Q * cpr; e += blockDim.x) {
      const int q = e / cpr;
      Vec8<T> v[9];
      bool ok[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int h = p * s - pad + r, w = q * s - pad + u;
          ok[r * 3 + u] = h >= 0 && h < H && w >= 0 && w < W;
          v[r * 3 + u].load(yb + (ok[r * 3 + u] ? (h * W + w) * C : 0));
        }
      float best[8], ysel[8];
      int bi[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = -1; ysel[j] = 0.f; }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = to_f32(from_f32<T>(bn_relu(v[t].get(j), sc[j], sh[j])));
          if (bi[j] < 0 || f > best[j] || f != f) { best[j] = f; bi[j] = t; ysel[j] = v[t].get(j); }
        }
      }
      Vec8<T> o, ym;
      uint64_t packed = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o.set(j, best[j]);
        ym.set(j, ysel[j]);
        packed |= (uint64_t)(uint8_t)bi[j] << (8 * j);
      }
      const long oi = ((long)row * Q + q) * C + cc * 8;
      o.store(out + oi);
      if (idx) *reinterpret_cast<uint64_t*>(idx + oi) = packed;
      if (ymax) ym.store(ymax + oi);
    }
    return;
  }
  for (int e = threadIdx.x; e < Q * cpr; e += blockDim.x) {
    const int q = e / cpr;
    float best[8], ysel[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = -1; ysel[j] = 0.f; }
    for (int r = 0; r < k; ++r) {
      const int h = p * s - pad + r;
      if (h < 0 || h >= H) continue;
      for (int u = 0; u < k; ++u) {
        const int w = q * s - pad + u;
        if (w < 0 || w >= W) continue;
        Vec8<T> v;
        v.load(yb + (h * W + w) * C);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // the value ssip_bn_apply would have stored
          const float f = to_f32(from_f32<T>(bn_relu(v.get(j), sc[j], sh[j])));
          if (bi[j] < 0 || f > best[j] || f != f) { best[j] = f; bi[j] = r * k + u; ysel[j] = v.get(j); }
        }
      }
    }
    Vec8<T> o, ym;
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o.set(j, best[j]);
      ym.set(j, ysel[j]);
      packed |= (uint64_t)(uint8_t)bi[j] << (8 * j);
    }
    const long oi = ((long)row * Q + q) * C + cc * 8;
    o.store(out + oi);
    if (idx) *reinterpret_cast<uint64_t*>(idx + oi) = packed;
    if (ymax) ym.store(ymax + oi);
  }
}

// dz at (h, w, chunk) of image n: pooled gradients of the windows that chose
// (h, w), summed in output order (p, q ascending) like ssip_maxpool_bwd.
// dpool/idx point at (n, 0, 0, chunk).  With at most 2x2 windows per input
// pixel (k <= 2s) all argmax bytes and gradients are loaded up front,
// predicated instead of branched, so every load of a pixel is in flight at
// once (the branchy form is a chain of dependent round trips).
template <typename T>
__device__ __forceinline__ void pool_grad_gather(int h, int w, int C, int P, int Q, int k, int s, int pad,
                                                 int plo, int phi, const T* __restrict__ dpool,
                                                 const uint8_t* __restrict__ idx, float (&acc)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int qlo = w + pad - k + 1;
  qlo = qlo <= 0 ? 0 : (qlo + s - 1) / s;
  int qhi = (w + pad) / s;
  if (qhi > Q - 1) qhi = Q - 1;
  if (k <= 2 * s) {
    uint64_t pk[2][2];
    Vec8<T> g[2][2];
    int pos[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int p = plo + a, q = qlo + b;
        const bool ok = p <= phi && q <= qhi;
        const int o = ok ? (p * Q + q) * C : 0;
        pos[a][b] = ok ? (h - (p * s - pad)) * k + (w - (q * s - pad)) : -1;
        pk[a][b] = *reinterpret_cast<const uint64_t*>(idx + o);
        g[a][b].load(dpool + o);
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((int)((pk[a][b] >> (8 * j)) & 0xff) == pos[a][b]) acc[j] += g[a][b].get(j);
    return;
  }
  for (int p = plo; p <= phi; ++p) {
    const int r = h - (p * s - pad);
    for (int q = qlo; q <= qhi; ++q) {
      const int u = w - (q * s - pad);
      const int pos = r * k + u;
      const int o = (p * Q + q) * C;
      const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
      Vec8<T> g;
      g.load(dpool + o);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((int)((packed >> (8 * j)) & 0xff) == pos) acc[j] += g.get(j);
    }
  }
}

__device__ __forceinline__ void pool_rows(int h, int P, int k, int s, int pad, int& plo, int& phi) {
  plo = h + pad - k + 1;
  plo = plo <= 0 ? 0 : (plo + s - 1) / s;
  phi = (h + pad) / s;
  if (phi > P - 1) phi = P - 1;
}

// pass 1: per-(row block, channel) {sum dpre, sum dpre*xhat}; layout
// [blocks][C][2] as ssip_bn_bwd's reduction.  A workgroup owns `rows`
// consecutive (n, h) rows of the full-resolution map.
template <typename T>
__global__ void __launch_bounds__(128) stem_pool_bn_bwd_reduce_kernel(
    int N, int H, int W, int C, int P, int Q, int k, int s, int pad, int rows, const T* __restrict__ dpool,
    const uint8_t* __restrict__ idx, const T* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ mean, const float* __restrict__ invstd,
    float* __restrict__ partial) {
  const int cpr = C >> 3;
  const int chunk = threadIdx.x % cpr;
  const int c0 = chunk * 8;
  float sd[8], sx[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sd[j] = 0.f; sx[j] = 0.f; }
  load_f8(mu, mean + c0);
  load_f8(is, invstd + c0);
  load_f8(sc, scale + c0);
  load_f8(sh, shift + c0);
  const int row0 = blockIdx.x * rows;
  const int row1 = min(row0 + rows, N * H);
  for (int row = row0; row < row1; ++row) {
    const int n = row / H, h = row - (row / H) * H;
    int plo, phi;
    pool_rows(h, P, k, s, pad, plo, phi);
    const T* dp = dpool + (long)n * P * Q * C + c0;
    const uint8_t* ix = idx + (long)n * P * Q * C + c0;
    const T* yr = y + (long)row * W * C + c0;
    for (int e = threadIdx.x; e < W * cpr; e += blockDim.x) {
      const int w = e / cpr;
      float dz[8];
      pool_grad_gather<T>(h, w, C, P, Q, k, s, pad, plo, phi, dp, ix, dz);
      Vec8<T> yy;
      yy.load(yr + w * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float yv = yy.get(j);
        const float d = bn_relu(yv, sc[j], sh[j]) > 0.f ? dz[j] : 0.f;
        sd[j] += d;
        sx[j] += d * ((yv - mu[j]) * is[j]);
      }
    }
  }
  __shared__ float red[2][128][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x][j] = sd[j];
    red[1][threadIdx.x][j] = sx[j];
  }
  __syncthreads();
  const int rpi = blockDim.x / cpr;
  if (threadIdx.x < cpr) {
    float* o = partial + ((long)c0 * gridDim.x + blockIdx.x) * 2;  // [C][blocks][2]
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f, b = 0.f;
      for (int q = 0; q < rpi; ++q) {
        a += red[0][q * cpr + threadIdx.x][j];
        b += red[1][q * cpr + threadIdx.x][j];
      }
      o[(long)j * gridDim.x * 2] = a;
      o[(long)j * gridDim.x * 2 + 1] = b;
    }
  }
}

// pass 2: dy = A * dpre + B * y + C, dpre recomputed by the same gather; one
// workgroup per full-resolution row (n, h).
template <typename T>
__global__ void __launch_bounds__(128) stem_pool_bn_bwd_apply_kernel(
    int H, int W, int C, int P, int Q, int k, int s, int pad, const T* __restrict__ dpool,
    const uint8_t* __restrict__ idx, const T* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, T* __restrict__ dy) {
  const int cpr = C >> 3;
  const int row = blockIdx.x;
  const int n = row / H, h = row - (row / H) * H;
  const int cc = threadIdx.x % cpr;
  const int c0 = cc * 8;
  float ca[8], cb[8], ck[8], sc[8], sh[8];
  load_f8(ca, coef + c0);
  load_f8(cb, coef + C + c0);
  load_f8(ck, coef + 2 * C + c0);
  load_f8(sc, scale + c0);
  load_f8(sh, shift + c0);
  int plo, phi;
  pool_rows(h, P, k, s, pad, plo, phi);
  const T* dp = dpool + (long)n * P * Q * C + c0;
  const uint8_t* ix = idx + (long)n * P * Q * C + c0;
  const T* yr = y + (long)row * W * C + c0;
  T* dr = dy + (long)row * W * C + c0;
  for (int e = threadIdx.x; e < W * cpr; e += blockDim.x) {
    const int w = e / cpr;
    float dz[8];
    pool_grad_gather<T>(h, w, C, P, Q, k, s, pad, plo, phi, dp, ix, dz);
    Vec8<T> yy, o;
    yy.load(yr + w * C);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float yv = yy.get(j);
      const float d = bn_relu(yv, sc[j], sh[j]) > 0.f ? dz[j] : 0.f;
      o.set(j, ca[j] * d + cb[j] * yv + ck[j]);
    }
    o.store(dr + w * C);
  }
}

// The ResNet stem's case (bf16, C = 64, 3x3 / 2 / pad 1, even H and W), VALU-
// lean: the generic kernel above spends ~10 VALU ops per window tap and channel
// (bf16 -> f32, BN, ReLU, rounding, a float compare and three selects) and
// recomputes every z 2.25 times (overlapping windows): ~825 ops per 8-channel
// output, which made it VALU-bound (180 us at batch 256, 3.7 TB/s).  Here
//  * each thread walks R pooled rows of one (column q, 8-channel chunk),
//    carrying input row 2p+1 into the next pooled row's window (row 2p-1):
//    6 new taps per output instead of 9;
//  * z is formed on channel pairs: one packed fma, one packed bf16 rounding,
//    then ReLU in the integer domain: a saturating +0x7f and a signed max with
//    0x7f map every negative value, -0.0 and NaN to 0x7f -- the code of 0 --
//    and keep every z >= 0 in order (z + 0x7f <= 0x7fff): the same order and
//    ties as bf16(relu(fma(y, scale, shift))) with the generic kernel's
//    `t > 0 ? t : 0` (NaN -> 0), i.e. ssip_bn_apply's stored value;
//  * the window max with torch's first-max tie break is one signed 32-bit
//    max over keys (z' << 16) | (15 - t): equal z prefer the smaller tap index
//    t, and a padding tap (all ones) is negative and never wins.  The argmax
//    and the pre-BN y there follow the winning key.
// Bit-identical outputs, argmax bytes and ymax to the generic kernel
// (tests/test_gpu_stem_pool.py; bench geometry: tests/test_gpu_bench_geometry.py).
namespace stem_pool {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

// z' = z + 0x7f per channel of a pair (0x7f = relu'd zero, NaN or negative)
__device__ __forceinline__ uint32_t zpair(uint32_t ydw, f2 sc, f2 sh) {
  f2 yv;
  yv.x = __builtin_bit_cast(float, ydw << 16);
  yv.y = __builtin_bit_cast(float, ydw & 0xffff0000u);
  const f2 t = __builtin_elementwise_fma(yv, sc, sh);
  const bf2 b = __builtin_convertvector(t, bf2);
  const u2 a = __builtin_elementwise_add_sat(__builtin_bit_cast(u2, b), (u2){0x7f, 0x7f});
  const s2 r = __builtin_elementwise_max(__builtin_bit_cast(s2, a), (s2){0x7f, 0x7f});
  return __builtin_bit_cast(uint32_t, r);
}

}  // namespace stem_pool

// YMAX 0: no ymax; 1: ymax follows the winning key (a compare + select per
// tap); 2: the nine taps' y go to the thread's own LDS slots and ymax is read
// back at the argmax (no per-tap select)
template <int YMAX>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
stem_bn_pool_fwd_k3s2_kernel(int H, int W, int P, int Q, int R,
                                                                    const __bf16* __restrict__ y,
                                                                    const float* __restrict__ scale,
                                                                    const float* __restrict__ shift,
                                                                    __bf16* __restrict__ out,
                                                                    uint8_t* __restrict__ idx,
                                                                    __bf16* __restrict__ ymax) {
  using namespace stem_pool;
  constexpr int C = 64;
  // blockIdx.y: a group of 64 pooled columns (one workgroup row covers Q <= 64)
  const int q = (int)blockIdx.y * 64 + (threadIdx.x >> 3), cc = threadIdx.x & 7;
  if (q >= Q) return;
  const int groups = (P + R - 1) / R;
  const int n = blockIdx.x / groups, p0 = (blockIdx.x - n * groups) * R;
  const int p1 = p0 + R < P ? p0 + R : P;
  f2 sc[4], sh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sc[i] = *reinterpret_cast<const f2*>(scale + cc * 8 + 2 * i);
    sh[i] = *reinterpret_cast<const f2*>(shift + cc * 8 + 2 * i);
  }
  const char* yb = reinterpret_cast<const char*>(y + (long)n * H * W * C + cc * 8);
  const bool left = q == 0;  // column 2q - 1 is padding
  const long c0 = (long)(left ? 0 : 2 * q - 1) * C * 2, c1 = (long)(2 * q) * C * 2, c2 = c1 + C * 2;
  auto load_row = [&](int h, uint4 (&v)[3]) {
    const char* rp = yb + (long)h * W * C * 2;
    v[0] = *reinterpret_cast<const uint4*>(rp + c0);
    v[1] = *reinterpret_cast<const uint4*>(rp + c1);
    v[2] = *reinterpret_cast<const uint4*>(rp + c2);
  };
  // z' pairs of one input row's three taps (padding column: all ones)
  auto z_row = [&](const uint4 (&v)[3], uint32_t (&z)[3][4]) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t zz = zpair(d[i], sc[i], sh[i]);
        z[u][i] = (u == 0 && left) ? 0xffffffffu : zz;
      }
    }
  };
  int32_t best[8];
  uint32_t ysel[8];
  __shared__ uint4 ylds[YMAX == 2 ? 512 * 9 : 1];
  uint4* mine = ylds + (YMAX == 2 ? threadIdx.x * 9 : 0);
  // fold one input row (window row r) into the running keys
  auto fold = [&](const uint32_t (&z)[3][4], const uint4 (&v)[3], int r) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const uint32_t yd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      const uint32_t lo = 15 - (r * 3 + u);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t zd = z[u][j >> 1];
        const int32_t key = (int32_t)((j & 1) ? ((zd & 0xffff0000u) | lo) : ((zd << 16) | lo));
        if (YMAX == 1) {
          const bool gt = key > best[j];
          best[j] = gt ? key : best[j];
          ysel[j] = gt ? yd[j >> 1] : ysel[j];
        } else {
          best[j] = key > best[j] ? key : best[j];
        }
      }
    }
  };
  uint32_t zt[3][4];  // window row 0 (input row 2p - 1)
  uint4 vt[3];
  if (p0 == 0) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      vt[u] = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) zt[u][i] = 0xffffffffu;
    }
  } else {
    load_row(2 * p0 - 1, vt);
    z_row(vt, zt);
  }
  uint4 a[3], b[3];
  load_row(2 * p0, a);
  load_row(2 * p0 + 1, b);
  for (int p = p0; p < p1; ++p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = 0; ysel[j] = 0; }
    if (YMAX == 2) {
#pragma unroll
      for (int u = 0; u < 3; ++u) { mine[u] = vt[u]; mine[3 + u] = a[u]; mine[6 + u] = b[u]; }
    }
    fold(zt, vt, 0);
    uint32_t zm[3][4];
    z_row(a, zm);
    fold(zm, a, 1);
    z_row(b, zt);  // window row 2 now, row 0 of the next pooled row
#pragma unroll
    for (int u = 0; u < 3; ++u) vt[u] = b[u];
    if (p + 1 < p1) {  // the next pooled row's two new input rows, in flight during the selection
      load_row(2 * p + 2, a);
      load_row(2 * p + 3, b);
    }
    fold(zt, vt, 2);
    uint4 o, ym;
    uint32_t od[4], yd[4];
    uint32_t ilo = 0, ihi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t zz = ((uint32_t)best[2 * i] >> 16) | ((uint32_t)best[2 * i + 1] & 0xffff0000u);
      od[i] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u2, zz) - (u2){0x7f, 0x7f});
      if (YMAX == 1) yd[i] = (ysel[2 * i] & 0xffffu) | (ysel[2 * i + 1] & 0xffff0000u);
    }
    if (YMAX == 2) {
      const uint16_t* m16 = reinterpret_cast<const uint16_t*>(mine);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t e0 = m16[(15u - ((uint32_t)best[2 * i] & 15u)) * 8 + 2 * i];
        const uint32_t e1 = m16[(15u - ((uint32_t)best[2 * i + 1] & 15u)) * 8 + 2 * i + 1];
        yd[i] = e0 | (e1 << 16);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t t = 15u - ((uint32_t)best[j] & 15u);
      if (j < 4) ilo |= t << (8 * j); else ihi |= t << (8 * (j - 4));
    }
    o.x = od[0]; o.y = od[1]; o.z = od[2]; o.w = od[3];
    ym.x = yd[0]; ym.y = yd[1]; ym.z = yd[2]; ym.w = yd[3];
    const long oi = (((long)n * P + p) * Q + q) * C + cc * 8;
    *reinterpret_cast<uint4*>(out + oi) = o;
    if (YMAX || idx) *reinterpret_cast<uint2*>(idx + oi) = make_uint2(ilo, ihi);
    if (YMAX) *reinterpret_cast<uint4*>(ymax + oi) = ym;
  }
}

// full-resolution rows (n, h) per reduction workgroup: ~8192 workgroups
// (each thread's gather chain is serial: parallelism comes from workgroups)
static int rows_per_block(int N, int H) {
  const int rows = (N * H + 8191) / 8192;
  return rows < 1 ? 1 : rows;
}

}  // namespace

extern "C" {

// the pooled-forward kernel ssip_stem_bn_pool_fwd takes for a shape: 2 / 1 / 0
// = stem_bn_pool_fwd_k3s2_kernel<ymax from LDS / per-tap ymax / no ymax>,
// -1 = the generic stem_bn_pool_fwd_kernel
static int pool_fwd_variant(int dtype, int H, int W, int C, int k, int s, int pad, bool ymax) {
  const char* pr = std::getenv("SSIP_POOL_ROWS");  // pooled rows per workgroup of the k3s2 kernel; 0: generic
  const int pool_rows = pr ? std::atoi(pr) : 4;
  if (!(dtype == SSIP_BF16 && C == 64 && k == 3 && s == 2 && pad == 1 && H % 2 == 0 && W % 2 == 0 && pool_rows > 0))
    return -1;
  const char* lm = std::getenv("SSIP_POOL_LDS");  // ymax from LDS slots (default) or per-tap selects
  return !ymax ? 0 : ((lm == nullptr || std::atoi(lm) != 0) ? 2 : 1);
}

int ssip_stem_bn_pool_kernel_name(int dtype, int N, int H, int W, int C, int k, int s, int pad, int has_ymax,
                                  char* buf, int buflen) {
  SSIP_REQUIRE(buf && buflen > 0 && N > 0 && H > 0 && W > 0 && k > 0 && s > 0, SSIP_ERR_ARG,
               "ssip_stem_bn_pool_kernel_name: bad arguments");
  const int v = pool_fwd_variant(dtype, H, W, C, k, s, pad, has_ymax != 0);
  if (v < 0) snprintf(buf, buflen, "stem_bn_pool_fwd<generic>");
  else snprintf(buf, buflen, "stem_bn_pool_fwd_k3s2<%d>", v);
  return SSIP_OK;
}

int ssip_stem_bn_pool_fwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* y,
                          const float* scale, const float* shift, void* out, uint8_t* idx, void* ymax, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && 256 % (C / 8) == 0 && k > 0 && k * k <= 255 && s > 0 &&
                   y && scale && shift && out && (idx || !ymax),
               SSIP_ERR_ARG, "ssip_stem_bn_pool_fwd: bad arguments");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  SSIP_REQUIRE((long)N * H * W * C < (1l << 31), SSIP_ERR_ARG, "ssip_stem_bn_pool_fwd: too large");
  const int variant = pool_fwd_variant(dtype, H, W, C, k, s, pad, ymax != nullptr);
  if (variant >= 0) {
    const char* pr = std::getenv("SSIP_POOL_ROWS");
    const int pool_rows = pr ? std::atoi(pr) : 4;
    const int groups = (P + pool_rows - 1) / pool_rows;
    const dim3 grid(N * groups, (Q + 63) / 64), block(Q >= 64 ? 512 : (Q * 8 + 63) / 64 * 64);
    if (variant == 2)
      SSIP_KLAUNCH(stem_bn_pool_fwd_k3s2_kernel<2>, grid, block, 0, (hipStream_t)stream, H, W, P, Q, pool_rows,
                   (const __bf16*)y, scale, shift, (__bf16*)out, idx, (__bf16*)ymax);
    else if (variant == 1)
      SSIP_KLAUNCH(stem_bn_pool_fwd_k3s2_kernel<1>, grid, block, 0, (hipStream_t)stream, H, W, P, Q, pool_rows,
                   (const __bf16*)y, scale, shift, (__bf16*)out, idx, (__bf16*)ymax);
    else
      SSIP_KLAUNCH(stem_bn_pool_fwd_k3s2_kernel<0>, grid, block, 0, (hipStream_t)stream, H, W, P, Q, pool_rows,
                   (const __bf16*)y, scale, shift, (__bf16*)out, idx, (__bf16*)nullptr);
    return ::ssip::check_launch("stem_bn_pool_fwd");
  }
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(stem_bn_pool_fwd_kernel<T>, dim3(N * P), dim3(256), 0, (hipStream_t)stream, H, W, C, P, Q,
                       k, s, pad, (const T*)y, scale, shift, (T*)out, idx, (T*)ymax);
  });
  return ::ssip::check_launch("stem_bn_pool_fwd");
}

int64_t ssip_stem_pool_bn_bwd_partial_floats(int N, int H, int W, int C) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || 256 % (C / 8)) return -1;
  const int rows = rows_per_block(N, H);
  const long full = (N * H + rows - 1) / rows;
  // the pooled-grid reduction (ymax given): any pooled size <= the full-resolution one
  const long Mp = (long)N * H * W;
  const int prow = bwd_rows_per_block(Mp, C);
  const long blocks = std::max<long>(full, (Mp + prow - 1) / prow);
  // + the split finalize's scratch (bn_common.h)
  return blocks * C * 2 + fin_scratch_floats(C, blocks, 2);
}

int ssip_stem_pool_bn_bwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* dpool,
                          const uint8_t* idx, const void* y, const void* ymax, const float* mean, const float* invstd,
                          const float* scale, const float* shift, const float* gamma, float* dgamma, float* dbeta,
                          int accumulate, void* dy, float* partial, float* coef, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && 128 % (C / 8) == 0 && k > 0 && k * k <= 255 && s > 0 &&
                   dpool && idx && y && mean && invstd && scale && shift && partial && coef,
               SSIP_ERR_ARG, "ssip_stem_pool_bn_bwd: bad arguments");
  const long M = (long)N * H * W;
  SSIP_REQUIRE(M * C / 8 < (1l << 31), SSIP_ERR_ARG, "ssip_stem_pool_bn_bwd: too large");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  hipStream_t st = (hipStream_t)stream;
  const int rows = rows_per_block(N, H);
  const int blocks = (N * H + rows - 1) / rows;
  // with ymax (the pre-BN value at each window's argmax, from the forward)
  // the sums run over the pooled grid: every full-resolution pixel's masked
  // gradient is the sum of the pooled gradients of the windows that chose it,
  // so sum d = sum_windows mask(ymax) dpool and likewise for d * xhat
  const long Mp = (long)N * P * Q;
  const int prow = ymax ? bwd_rows_per_block(Mp, C) : 0;
  const int red_blocks = ymax ? (int)((Mp + prow - 1) / prow) : blocks;
  SSIP_REQUIRE(!ymax || 256 % (C / 8) == 0, SSIP_ERR_ARG, "ssip_stem_pool_bn_bwd: unsupported C");
  SSIP_DISPATCH_DTYPE(dtype, T, {
    if (ymax)
      SSIP_KLAUNCH(bn_bwd_reduce_kernel<T>, dim3(red_blocks), dim3(256), 0, st, Mp, C, prow, (const T*)dpool,
                         (const T*)nullptr, (const uint8_t*)nullptr, (const T*)ymax, mean, invstd, scale, shift,
                         partial);
    else
      SSIP_KLAUNCH(stem_pool_bn_bwd_reduce_kernel<T>, dim3(blocks), dim3(128), 0, st, N, H, W, C, P, Q, k, s,
                         pad, rows, (const T*)dpool, idx, (const T*)y, scale, shift, mean, invstd, partial);
    BnBwdFin f;
    f.set[0] = bn_bwd_fin_set(partial, gamma, mean, invstd, dgamma, dbeta, coef,
                              fin_scratch(partial, (int64_t)red_blocks * C * 2));
    launch_bn_bwd_finalize(st, C, red_blocks, M, 1, 1, f, accumulate);
    if (dy)  // dy == nullptr: only dgamma/dbeta/coef (ssip_stem_bwd_wgrad forms dy on the fly)
      SSIP_KLAUNCH(stem_pool_bn_bwd_apply_kernel<T>, dim3(N * H), dim3(128), 0, st, H, W, C, P, Q, k, s, pad,
                         (const T*)dpool, idx, (const T*)y, scale, shift, coef, (T*)dy);
  });
  return ::ssip::check_launch("stem_pool_bn_bwd");
}

}  // extern "C"
