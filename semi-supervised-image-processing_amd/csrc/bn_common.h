// BatchNorm backward finalize shared by bn.hip and stem.hip: per-channel sums
// of dout and dout*xhat from [C][blocks][2] (or [blocks][C][2]) partials
// (fixed-order fp64 tree)
// -> dgamma/dbeta and the apply coefficients
//   dy = coef[c] * dout + coef[C+c] * y + coef[2C+c].
#pragma once
#include "ssip_common.h"
#include "fin_split.h"

namespace {

// Finalize workgroups: 256 threads (one wave per SIMD), so a finalize
// launched beside a running convolution finds room as soon as any conv
// workgroup retires (a 1024-thread workgroup waited for a whole CU).  A
// channel whose records would take more than FIN_PT per thread is split over
// S workgroups (fin_splits); their fp64 partial results go to a scratch area
// behind the records (fin_scratch) and a one-wave-per-channel merge finishes
// them.  (Round 3 measured one-wave finalize workgroups without LDS slower;
// that variant and its SSIP_FIN_NT knob are gone.)
// sums of up to three values over a 256-thread workgroup in fp64 with one
// LDS round (wave butterflies, then the 4 wave totals in fixed order)
template <int V>
__device__ __forceinline__ void block_sums_f64_256(double (&v)[V], double* sh) {
#pragma unroll
  for (int k = 0; k < V; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < V; ++k) sh[k * 4 + (threadIdx.x >> 6)] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < V; ++k) v[k] = ((sh[k * 4] + sh[k * 4 + 1]) + sh[k * 4 + 2]) + sh[k * 4 + 3];
}

// sums of V values over one wave (every lane ends with the same bits)
template <int V>
__device__ __forceinline__ void wave_sums_f64(double (&v)[V]) {
#pragma unroll
  for (int k = 0; k < V; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
}

// One BatchNorm's backward finalize operands
struct BnBwdFinSet {
  const float *partial, *gamma, *mean, *invstd;
  float *dgamma, *dbeta, *coef;
  double* scratch;  // [C][S][2] when S > 1
};
struct BnBwdFin {
  BnBwdFinSet set[2];
};

__device__ __forceinline__ void bn_bwd_fin_write(int c, int C, long M, const BnBwdFinSet& f, int accumulate,
                                                 double sum_d, double sum_dx) {
  if (f.dgamma) f.dgamma[c] = (float)(accumulate ? f.dgamma[c] + sum_dx : sum_dx);
  if (f.dbeta) f.dbeta[c] = (float)(accumulate ? f.dbeta[c] + sum_d : sum_d);
  const double g = f.gamma ? f.gamma[c] : 1.0;
  const double is = f.invstd[c];
  const double A = g * is;
  const double k0 = -A * sum_d / (double)M;
  const double k1 = -A * sum_dx / (double)M * is;
  f.coef[c] = (float)A;                             // * dout
  f.coef[C + c] = (float)k1;                        // * y
  f.coef[2 * C + c] = (float)(k0 - k1 * f.mean[c]);  // constant
}

// Workgroup (s, set * C + c): sums of dout and dout*xhat over split s of the
// channel's partials (threads take FIN_PT records at a time, FIN_NT apart, in
// increasing order); cmajor: [C][blocks][2] (each channel's records
// contiguous), else [blocks][C][2].  S == 1 writes the outputs directly.
template <int NT>
__global__ void __launch_bounds__(NT) bn_bwd_finalize_kernel(int C, int blocks, int S, long M, int cmajor,
                                                            BnBwdFin fin, int accumulate) {
  const int set = blockIdx.y >= C ? 1 : 0;
  const int c = blockIdx.y - set * C, s = blockIdx.x;
  const BnBwdFinSet& f = fin.set[set];
  const int L = (blocks + S - 1) / S;
  const int t0 = s * L, t1 = min(blocks, t0 + L);
  const long cs = cmajor ? 2 : (long)C * 2;
  const float* pc = f.partial + (cmajor ? (long)c * blocks * 2 : (long)c * 2);
  double ab[2] = {0.0, 0.0};
  for (int base = t0 + threadIdx.x; base < t1; base += NT * FIN_PT) {
    float r[FIN_PT][2];
#pragma unroll
    for (int i = 0; i < FIN_PT; ++i) {
      const int t = base + i * NT;
      r[i][0] = t < t1 ? pc[t * cs + 0] : 0.f;
      r[i][1] = t < t1 ? pc[t * cs + 1] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FIN_PT; ++i) {
      ab[0] += r[i][0];
      ab[1] += r[i][1];
    }
  }
  if constexpr (NT == 64) {
    wave_sums_f64<2>(ab);
  } else {
    __shared__ double sh[2 * 4];
    block_sums_f64_256<2>(ab, sh);
  }
  if (threadIdx.x == 0) {
    if (S == 1) {
      bn_bwd_fin_write(c, C, M, f, accumulate, ab[0], ab[1]);
    } else {
      f.scratch[((long)c * S + s) * 2 + 0] = ab[0];
      f.scratch[((long)c * S + s) * 2 + 1] = ab[1];
    }
  }
}

// split finalize, second pass: one wave per (set, channel) adds the S split
// sums in a fixed butterfly
__global__ void __launch_bounds__(FIN_NT) bn_bwd_finalize_merge_kernel(int C, int sets, int S, long M, BnBwdFin fin,
                                                                       int accumulate) {
  const int w = blockIdx.x * (FIN_NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= sets * C) return;
  const int set = w >= C ? 1 : 0;
  const int c = w - set * C;
  const BnBwdFinSet& f = fin.set[set];
  double ab[2] = {0.0, 0.0};
  if (lane < S) {
    ab[0] = f.scratch[((long)c * S + lane) * 2 + 0];
    ab[1] = f.scratch[((long)c * S + lane) * 2 + 1];
  }
  wave_sums_f64<2>(ab);
  if (lane == 0) bn_bwd_fin_write(c, C, M, f, accumulate, ab[0], ab[1]);
}

// host: launch the (split) backward finalize of `sets` BatchNorms whose
// records are `blocks` per channel
static inline void launch_bn_bwd_finalize(hipStream_t st, int C, int blocks, long M, int cmajor, int sets,
                                          const BnBwdFin& fin, int accumulate) {
  const int S = fin_splits(blocks);
  SSIP_KLAUNCH(bn_bwd_finalize_kernel<FIN_NT>, dim3(S, sets * C), dim3(FIN_NT), 0, st, C, blocks, S, M,
                     cmajor, fin, accumulate);
  if (S > 1)
    SSIP_KLAUNCH(bn_bwd_finalize_merge_kernel, dim3((sets * C + FIN_NT / 64 - 1) / (FIN_NT / 64)),
                       dim3(FIN_NT), 0, st, C, sets, S, M, fin, accumulate);
}

static inline BnBwdFinSet bn_bwd_fin_set(const float* partial, const float* gamma, const float* mean,
                                         const float* invstd, float* dgamma, float* dbeta, float* coef,
                                         double* scratch) {
  BnBwdFinSet f;
  f.partial = partial;
  f.gamma = gamma;
  f.mean = mean;
  f.invstd = invstd;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.coef = coef;
  f.scratch = scratch;
  return f;
}

// Totals of V per-thread [8]-vectors over the threads that share a channel
// chunk (tid % cpr, 256-thread block): a butterfly over the lane bits above
// log2(cpr) inside each wave, then at most 4 groups through LDS in fixed
// order.  Threads tid < cpr hold the totals on return.  Deterministic (the
// butterfly leaves identical bits in every lane of a group).
template <int V>
__device__ __forceinline__ void chunk_sums(float (&v)[V][8], int cpr, float (*red)[V * 8 + 1]) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (cpr < 64) {
    for (int o = cpr; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < V; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += __shfl_xor(v[k][j], o, 64);
  }
  const int groups = cpr < 64 ? 4 : 256 / cpr;
  const bool writer = cpr < 64 ? lane < cpr : true;
  const int slot = cpr < 64 ? (tid >> 6) * cpr + lane : tid;
  if (writer)
#pragma unroll
    for (int k = 0; k < V; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[slot][k * 8 + j] = v[k][j];
  __syncthreads();
  if (tid < cpr) {
#pragma unroll
    for (int k = 0; k < V; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = 0.f;
        for (int g = 0; g < groups; ++g) t += red[g * cpr + tid][k * 8 + j];
        v[k][j] = t;
      }
  }
}

// per-(row block, channel) sums of dout and dout*xhat.
// Block: 256 threads; each thread owns an 8-channel chunk; threads/row = C/8.
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(long M, int C, int rows_per_block, const T* __restrict__ dz,
                                     const T* __restrict__ zmask, const uint8_t* __restrict__ mbits,
                                     const T* __restrict__ y,
                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                     const float* __restrict__ mscale, const float* __restrict__ mshift,
                                     float* __restrict__ partial) {
  const int cpr = C / 8;               // chunks per row
  const int rpi = 256 / cpr;           // rows per iteration (>= 1 since C <= 2048)
  const int chunk = threadIdx.x % cpr;
  const int rsub = threadIdx.x / cpr;
  const int c0 = chunk * 8;
  const long r0 = (long)blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float sd[8], sx[8], mu[8], is[8], msc[8], msh[8];
  const bool amask = mscale != nullptr;  // ReLU mask recomputed from y (no z read)
#pragma unroll
  for (int j = 0; j < 8; ++j) { sd[j] = 0.f; sx[j] = 0.f; msc[j] = 0.f; msh[j] = 0.f; }
  load_f8(mu, mean + c0);
  load_f8(is, invstd + c0);
  if (amask) {
    load_f8(msc, mscale + c0);
    load_f8(msh, mshift + c0);
  }
  auto acc = [&](const Vec8<T>& g, const Vec8<T>& zz, uint32_t mb, const Vec8<T>& yy) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = g.get(j);
      if (zmask) d = zz.get(j) > 0.f ? d : 0.f;
      if (amask) d = __builtin_fmaf(yy.get(j), msc[j], msh[j]) > 0.f ? d : 0.f;
      d = ((mb >> j) & 1u) ? d : 0.f;
      const float xh = (yy.get(j) - mu[j]) * is[j];
      sd[j] += d;
      sx[j] += d * xh;
    }
  };
  if (rsub < rpi) {
    // four rows in flight per thread (one memory round trip covers a small
    // tensor's whole share); rows accumulate in the same order as a plain
    // r += rpi walk, so the sums do not depend on the unroll
    constexpr int U = 4;
    long r = r0 + rsub;
    for (; r + (U - 1) * rpi < r1; r += U * rpi) {
      Vec8<T> g[U], z[U], yv[U];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + (long)u * rpi;
        g[u].load(dz + rr * C + c0);
        yv[u].load(y + rr * C + c0);
        if (zmask) z[u].load(zmask + rr * C + c0);
        mb[u] = mbits ? (uint32_t)mbits[rr * cpr + chunk] : 0xFFu;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc(g[u], z[u], mb[u], yv[u]);
    }
    for (; r < r1; r += rpi) {
      Vec8<T> g0, z0, y0;
      uint32_t m0 = 0xFFu;
      g0.load(dz + r * C + c0);
      y0.load(y + r * C + c0);
      if (zmask) z0.load(zmask + r * C + c0);
      if (mbits) m0 = mbits[r * cpr + chunk];
      acc(g0, z0, m0, y0);
    }
  }
  __shared__ float red[256][17];
  float v[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[0][j] = sd[j];
    v[1][j] = sx[j];
  }
  chunk_sums<2>(v, cpr, red);
  if (threadIdx.x < cpr) {
    // [C][blocks][2]: each channel's records contiguous for the finalize
    float* out = partial + ((long)c0 * gridDim.x + blockIdx.x) * 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      out[(long)j * gridDim.x * 2] = v[0][j];
      out[(long)j * gridDim.x * 2 + 1] = v[1][j];
    }
  }
}

static inline int bwd_rows_per_block(long M, int C) {
  // aim for ~512 blocks (2 per CU), at least eight iterations of rows (fewer,
  // longer blocks: 38.1 vs 43.8 us at layer1 batch 256, 15.6 vs 19.5 at layer3,
  // tools/time_bn_bwd.py)
  constexpr long nb = 512, it = 8;
  const int rpi = 256 / (C / 8);
  long rows = (M + nb - 1) / nb;
  if (rows < it * rpi) rows = it * rpi;
  if (rows < rpi) rows = rpi;
  rows = ((rows + rpi - 1) / rpi) * rpi;
  return (int)rows;
}

}  // namespace
