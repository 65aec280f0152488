// Stem max-pool, global-average-pool + fc head, and the classification
// losses of the train / pseudo-label / consistency steps.
//
// Reference call sites:
//   maxpool 3x3/2 and AdaptiveAvgPool2d(1) + fc (512->C): torchvision
//     resnet18 forward inside `model(inputs)` (src/training/common.py:380);
//     the avgpool output is the 512-D embedding of
//     src/feature_extraction.py:224,291-293 (`children()[:-1]` + flatten).
//   nn.CrossEntropyLoss (mean): src/training/common.py:381,
//     src/training/semi_supervised.py:111.
//   softmax / max / >= threshold pseudo-labelling:
//     src/training/semi_supervised.py:57-66.
//   softmax + P(pos) + argmax/threshold for evaluation:
//     src/training/common.py:452-484.
#include "ssip_common.h"

namespace {

// ---------------------------------------------------------------------------
// max pool (NHWC), first-max-wins tie break like torch (scan kh then kw).
// idx[] keeps the in-window position (0..kh*kw-1) of the max per element.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_fwd_kernel(int N, int H, int W, int C, int P, int Q, int k, int s, int pad,
                                   const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx) {
  const long total = (long)N * P * Q * (C / 8);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % (C / 8));
    long t = i / (C / 8);
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
        v.load(x + (((long)n * H + h) * W + w) * C + cc * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = v.get(j);
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
    o.store(y + i * 8);
    *reinterpret_cast<uint64_t*>(idx + i * 8) = packed;
  }
}

// gather form: each input element sums the grads of the outputs that chose it,
// in output order (p, q ascending) like torch's scatter-add over outputs.
template <typename T>
__global__ void maxpool_bwd_kernel(int N, int H, int W, int C, int P, int Q, int k, int s, int pad,
                                   const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx) {
  const long total = (long)N * H * W * (C / 8);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % (C / 8));
    long t = i / (C / 8);
    const int w = t % W;
    t /= W;
    const int h = t % H;
    const int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // outputs p with p*s - pad <= h <= p*s - pad + k - 1
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
        Vec8<T> g;
        g.load(dy + o);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((int)((packed >> (8 * j)) & 0xff) == pos) acc[j] += g.get(j);
      }
    }
    Vec8<T> out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out.set(j, acc[j]);
    out.store(dx + i * 8);
  }
}

// ---------------------------------------------------------------------------
// global average pool + fc:  feat[b][c] = mean_pq z[b][pq][c]; logits = feat W^T + bias
// one block (256 threads) per image
// ---------------------------------------------------------------------------
template <typename T>
__global__ void avgpool_fc_fwd_kernel(int PQ, int C, int J, const T* __restrict__ z, const float* __restrict__ w,
                                      const float* __restrict__ bias, float* __restrict__ feat,
                                      float* __restrict__ logits) {
  const int b = blockIdx.x;
  extern __shared__ float sfeat[];  // [C] + [256]
  float* red = sfeat + C;
  const T* zb = z + (long)b * PQ * C;
  const float inv = 1.f / (float)PQ;
  const int cpr = C >> 3;
  if ((C & 7) == 0 && cpr <= 256 && 256 % cpr == 0) {
    // 16-B vectors: thread (group g, chunk k) sums rows g, g + G, ... of its
    // 8 channels; the G group partials are combined in order through LDS
    const int G = 256 / cpr, k = threadIdx.x % cpr, g = threadIdx.x / cpr;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int i = g; i < PQ; i += G) {
      Vec8<T> v;
      v.load(zb + (long)i * C + k * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v.get(j);
    }
    float* part = red;  // [G][C] after sfeat[C]
#pragma unroll
    for (int j = 0; j < 8; ++j) part[g * C + k * 8 + j] = acc[j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float t = 0.f;
      for (int q = 0; q < G; ++q) t += part[q * C + c];
      const float f = t * inv;
      sfeat[c] = f;
      if (feat) feat[(long)b * C + c] = f;
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float t = 0.f;
      for (int i = 0; i < PQ; ++i) t += to_f32<T>(zb[(long)i * C + c]);
      const float f = t * inv;
      sfeat[c] = f;
      if (feat) feat[(long)b * C + c] = f;
    }
  }
  __syncthreads();
  if (!logits) return;
  for (int j = 0; j < J; ++j) {
    float part = 0.f;
    for (int c = threadIdx.x; c < C; c += blockDim.x) part += sfeat[c] * w[(long)j * C + c];
    red[threadIdx.x] = part;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) logits[(long)b * J + j] = red[0] + (bias ? bias[j] : 0.f);
    __syncthreads();
  }
}

// dz[b][pq][c] = (sum_j dlogits[b][j] w[j][c]) / PQ
template <typename T>
__global__ void avgpool_fc_bwd_data_kernel(int PQ, int C, int J, const float* __restrict__ dlogits,
                                           const float* __restrict__ w, T* __restrict__ dz) {
  const int b = blockIdx.x;
  const float inv = 1.f / (float)PQ;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float g = 0.f;
    for (int j = 0; j < J; ++j) g += dlogits[(long)b * J + j] * w[(long)j * C + c];
    const T v = from_f32<T>(g * inv);
    T* zb = dz + (long)b * PQ * C;
    for (int i = 0; i < PQ; ++i) zb[(long)i * C + c] = v;
  }
}

// dW[j][c] (+)= sum_b dlogits[b][j] feat[b][c];  dbias[j] (+)= sum_b dlogits[b][j]
// block = 64 output elements x 16 batch groups; fixed-order LDS combine.
__global__ void __launch_bounds__(1024) fc_bwd_weight_kernel(int B, int C, int J, const float* __restrict__ dlogits,
                                                             const float* __restrict__ feat, float* dw, float* dbias,
                                                             int accumulate) {
  __shared__ float red[16][65];
  const int cl = threadIdx.x & 63, bg = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + cl;
  float a = 0.f;
  if (i < J * C) {
    const int j = i / C, c = i % C;
    // four batch rows' loads in flight per trip (a serial load chain was
    // 21 us on the main stream at batch 256); the sum keeps the b order
    int b = bg;
    for (; b + 48 < B; b += 64) {
      const float d0 = dlogits[(long)b * J + j], d1 = dlogits[(long)(b + 16) * J + j];
      const float d2 = dlogits[(long)(b + 32) * J + j], d3 = dlogits[(long)(b + 48) * J + j];
      const float f0 = feat[(long)b * C + c], f1 = feat[(long)(b + 16) * C + c];
      const float f2 = feat[(long)(b + 32) * C + c], f3 = feat[(long)(b + 48) * C + c];
      a += d0 * f0;
      a += d1 * f1;
      a += d2 * f2;
      a += d3 * f3;
    }
    for (; b < B; b += 16) a += dlogits[(long)b * J + j] * feat[(long)b * C + c];
  }
  red[bg][cl] = a;
  __syncthreads();
  if (bg == 0 && i < J * C) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][cl];
    dw[i] = accumulate ? dw[i] + t : t;
  }
  if (dbias && blockIdx.x == 0) {
    // the 16 batch groups' partial sums (b = bg mod 16, in order), combined in
    // fixed order: no single-thread chain over the whole batch
    for (int j0 = 0; j0 < J; j0 += 64) {
      const int j = j0 + cl;
      float t = 0.f;
      if (j < J)
        for (int b = bg; b < B; b += 16) t += dlogits[(long)b * J + j];
      __syncthreads();
      red[bg][cl] = t;
      __syncthreads();
      if (bg == 0 && j < J) {
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < 16; ++g) s += red[g][cl];
        dbias[j] = accumulate ? dbias[j] + s : s;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// losses.  One block of 256 threads; deterministic fixed-order reductions.
// ---------------------------------------------------------------------------
__device__ void row_softmax(const float* z, int J, float* p, float& lse, int& amax, float& pmax) {
  float m = z[0];
  amax = 0;
  for (int j = 1; j < J; ++j)
    if (z[j] > m) { m = z[j]; amax = j; }
  float s = 0.f;
  for (int j = 0; j < J; ++j) s += expf(z[j] - m);
  lse = m + logf(s);
  pmax = 0.f;
  for (int j = 0; j < J; ++j) {
    p[j] = expf(z[j] - lse);
  }
  pmax = p[amax];
}

__device__ float block_sum(float v, float* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

constexpr int MAXJ = 16;

// mean CE over B rows; dlogits = grad_scale * (softmax - onehot) / B
__global__ void cross_entropy_kernel(int B, int J, const float* __restrict__ logits, const int64_t* __restrict__ labels,
                                     float grad_scale, float* loss, float* dlogits, int64_t* pred) {
  __shared__ float red[256];
  float part = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float p[MAXJ], lse, pmax;
    int am;
    row_softmax(logits + (long)b * J, J, p, lse, am, pmax);
    const int y = (int)labels[b];
    part += lse - logits[(long)b * J + y];
    if (dlogits)
      for (int j = 0; j < J; ++j) dlogits[(long)b * J + j] = grad_scale * (p[j] - (j == y ? 1.f : 0.f)) / (float)B;
    if (pred) pred[b] = am;
  }
  const float tot = block_sum(part, red);
  if (threadIdx.x == 0 && loss) loss[0] = tot / (float)B;
}

// FixMatch-style consistency:  L = CE(z_l, y_l) + lambda * mean_u[ 1(max p_w >= tau) CE(z_s, argmax z_w) ]
// out[0] = total, out[1] = L_l, out[2] = L_u, out[3] = mask count
__global__ void semi_loss_kernel(int Bl, int Bu, int J, const float* __restrict__ zl, const int64_t* __restrict__ yl,
                                 const float* __restrict__ zw, const float* __restrict__ zs, float tau, float lambda_u,
                                 float* out, float* dzl, float* dzs, int64_t* pseudo, uint8_t* mask) {
  __shared__ float red[256];
  float pl = 0.f;
  for (int b = threadIdx.x; b < Bl; b += blockDim.x) {
    float p[MAXJ], lse, pmax;
    int am;
    row_softmax(zl + (long)b * J, J, p, lse, am, pmax);
    const int y = (int)yl[b];
    pl += lse - zl[(long)b * J + y];
    for (int j = 0; j < J; ++j) dzl[(long)b * J + j] = (p[j] - (j == y ? 1.f : 0.f)) / (float)Bl;
  }
  float pu = 0.f, pm = 0.f;
  for (int b = threadIdx.x; b < Bu; b += blockDim.x) {
    float pw[MAXJ], lsew, pmaxw;
    int amw;
    row_softmax(zw + (long)b * J, J, pw, lsew, amw, pmaxw);
    const bool keep = pmaxw >= tau;
    float ps[MAXJ], lses, pmaxs;
    int ams;
    row_softmax(zs + (long)b * J, J, ps, lses, ams, pmaxs);
    if (keep) {
      pu += lses - zs[(long)b * J + amw];
      pm += 1.f;
    }
    for (int j = 0; j < J; ++j)
      dzs[(long)b * J + j] = keep ? lambda_u * (ps[j] - (j == amw ? 1.f : 0.f)) / (float)Bu : 0.f;
    if (pseudo) pseudo[b] = amw;
    if (mask) mask[b] = keep ? 1 : 0;
  }
  const float Ll = block_sum(pl, red) / (float)(Bl > 0 ? Bl : 1);
  const float Lu = block_sum(pu, red) / (float)(Bu > 0 ? Bu : 1);
  const float cnt = block_sum(pm, red);
  if (threadIdx.x == 0) {
    out[0] = Ll + lambda_u * Lu;
    out[1] = Ll;
    out[2] = Lu;
    out[3] = cnt;
  }
}

// softmax / max / threshold (pseudo labels, eval probabilities)
__global__ void softmax_select_kernel(int B, int J, const float* __restrict__ logits, float threshold, int pos_col,
                                      float* probs, float* conf, int64_t* pred, uint8_t* keep, float* pos_prob) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float p[MAXJ], lse, pmax;
  int am;
  row_softmax(logits + (long)b * J, J, p, lse, am, pmax);
  if (probs)
    for (int j = 0; j < J; ++j) probs[(long)b * J + j] = p[j];
  if (conf) conf[b] = pmax;
  if (pred) pred[b] = am;
  if (keep) keep[b] = pmax >= threshold ? 1 : 0;
  if (pos_prob) pos_prob[b] = p[pos_col];
}

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

int ssip_maxpool_fwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* x, void* y,
                     uint8_t* idx, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && k > 0 && k * k <= 255 && s > 0 && x && y && idx,
               SSIP_ERR_ARG, "ssip_maxpool_fwd: bad arguments");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  const long total = (long)N * P * Q * (C / 8);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(maxpool_fwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C,
                       P, Q, k, s, pad, (const T*)x, (T*)y, idx);
  });
  return ::ssip::check_launch("maxpool_fwd");
}

int ssip_maxpool_bwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* dy,
                     const uint8_t* idx, void* dx, void* stream) {
  SSIP_REQUIRE(N > 0 && H > 0 && W > 0 && C % 8 == 0 && k > 0 && s > 0 && dy && idx && dx, SSIP_ERR_ARG,
               "ssip_maxpool_bwd: bad arguments");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  const long total = (long)N * H * W * (C / 8);
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(maxpool_bwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, H, W, C,
                       P, Q, k, s, pad, (const T*)dy, idx, (T*)dx);
  });
  return ::ssip::check_launch("maxpool_bwd");
}

int ssip_avgpool_fc_fwd(int dtype, int B, int PQ, int C, int J, const void* z, const float* w, const float* bias,
                        float* feat, float* logits, void* stream) {
  SSIP_REQUIRE(B > 0 && PQ > 0 && C > 0 && z && (feat || logits), SSIP_ERR_ARG, "ssip_avgpool_fc_fwd: bad arguments");
  SSIP_REQUIRE(!logits || (w && J > 0), SSIP_ERR_ARG, "ssip_avgpool_fc_fwd: fc weight required");
  const size_t shm = (size_t)(C + 2048) * sizeof(float);  // sfeat[C] + the group partials (<= 2048)
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(avgpool_fc_fwd_kernel<T>, dim3(B), dim3(256), shm, (hipStream_t)stream, PQ, C, J, (const T*)z,
                       w, bias, feat, logits);
  });
  return ::ssip::check_launch("avgpool_fc_fwd");
}

int ssip_avgpool_fc_bwd(int dtype, int B, int PQ, int C, int J, const float* dlogits, const float* w,
                        const float* feat, void* dz, float* dw, float* dbias, int accumulate, void* stream) {
  SSIP_REQUIRE(B > 0 && PQ > 0 && C > 0 && J > 0 && dlogits && w, SSIP_ERR_ARG, "ssip_avgpool_fc_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (dz) {
    SSIP_DISPATCH_DTYPE(dtype, T, {
      SSIP_KLAUNCH(avgpool_fc_bwd_data_kernel<T>, dim3(B), dim3(256), 0, st, PQ, C, J, dlogits, w, (T*)dz);
    });
  }
  if (dw) {
    SSIP_REQUIRE(feat, SSIP_ERR_ARG, "ssip_avgpool_fc_bwd: feat required for dw");
    SSIP_REQUIRE(J <= 256, SSIP_ERR_ARG, "ssip_avgpool_fc_bwd: J <= 256");
    SSIP_KLAUNCH(fc_bwd_weight_kernel, dim3((J * C + 63) / 64), dim3(1024), 0, st, B, C, J, dlogits, feat, dw,
                       dbias, accumulate);
  }
  return ::ssip::check_launch("avgpool_fc_bwd");
}

int ssip_cross_entropy(int B, int J, const float* logits, const int64_t* labels, float grad_scale, float* loss,
                       float* dlogits, int64_t* pred, void* stream) {
  SSIP_REQUIRE(B > 0 && J > 0 && J <= MAXJ && logits && labels, SSIP_ERR_ARG, "ssip_cross_entropy: bad arguments");
  SSIP_KLAUNCH(cross_entropy_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, B, J, logits, labels,
                     grad_scale, loss, dlogits, pred);
  return ::ssip::check_launch("cross_entropy");
}

int ssip_semi_loss(int Bl, int Bu, int J, const float* zl, const int64_t* yl, const float* zw, const float* zs,
                   float tau, float lambda_u, float* out4, float* dzl, float* dzs, int64_t* pseudo, uint8_t* mask,
                   void* stream) {
  SSIP_REQUIRE(Bl >= 0 && Bu >= 0 && Bl + Bu > 0 && J > 0 && J <= MAXJ && out4 && (Bl == 0 || (zl && yl && dzl)) &&
                   (Bu == 0 || (zw && zs && dzs)),
               SSIP_ERR_ARG, "ssip_semi_loss: bad arguments");
  SSIP_KLAUNCH(semi_loss_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, Bl, Bu, J, zl, yl, zw, zs, tau,
                     lambda_u, out4, dzl, dzs, pseudo, mask);
  return ::ssip::check_launch("semi_loss");
}

int ssip_softmax_select(int B, int J, const float* logits, float threshold, int pos_col, float* probs, float* conf,
                        int64_t* pred, uint8_t* keep, float* pos_prob, void* stream) {
  SSIP_REQUIRE(B > 0 && J > 0 && J <= MAXJ && logits && pos_col >= 0 && pos_col < J, SSIP_ERR_ARG,
               "ssip_softmax_select: bad arguments");
  SSIP_KLAUNCH(softmax_select_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, B, J, logits,
                     threshold, pos_col, probs, conf, pred, keep, pos_prob);
  return ::ssip::check_launch("softmax_select");
}

}  // extern "C"
