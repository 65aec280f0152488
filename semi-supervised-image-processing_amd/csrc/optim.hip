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

// One element of the update (the same fp32 operations in every code path, so
// the vector and scalar paths below agree bit for bit).
struct AdamC {
  float decay, w1, b2, eps, step_size, bc2_sqrt, grad_scale;
};

__device__ __forceinline__ void adamw_math(float& pi, float& mi, float& vi, float graw, const AdamC& c) {
  // no fused multiply-adds: the compiler would contract the scalar and the
  // packed (v_pk_*) forms differently, and a run must not depend on its offset
#pragma clang fp contract(off)
  const float gi = graw * c.grad_scale;
  pi = pi * c.decay;
  mi = (c.w1 < 0.5f) ? mi + c.w1 * (gi - mi) : gi - (gi - mi) * (1.f - c.w1);
  vi = vi * c.b2 + (1.f - c.b2) * gi * gi;
  const float denom = sqrtf(vi) / c.bc2_sqrt + c.eps;
  pi = pi - c.step_size * (mi / denom);
}

__device__ __forceinline__ void adamw_scalar(long i, float* __restrict__ p, const float* __restrict__ g,
                                             float* __restrict__ m, float* __restrict__ v, const AdamC& c) {
  float pi = p[i], mi = m[i], vi = v[i];
  adamw_math(pi, mi, vi, g[i], c);
  p[i] = pi;
  m[i] = mi;
  v[i] = vi;
}

// Grid-stride over [0, n): 16-B vectors (4 elements per lane, four loads of
// 16 B in flight instead of four of 4 B) where the four arrays share their
// 16-B alignment (the arena's parameter / gradient / moment tensors do, at any
// run offset), scalar head and tail around them.  HBM-bound: 28 B / element.
__device__ __forceinline__ void adamw_range(long n, float* __restrict__ p, const float* __restrict__ g,
                                            float* __restrict__ m, float* __restrict__ v, const AdamC& c) {
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x, nt = (long)gridDim.x * blockDim.x;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p) & 15;
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == a && (reinterpret_cast<uintptr_t>(m) & 15) == a &&
                   (reinterpret_cast<uintptr_t>(v) & 15) == a && (a & 3) == 0;
  const long head = vec ? min(n, (long)(((16 - a) & 15) >> 2)) : n;
  for (long i = tid; i < head; i += nt) adamw_scalar(i, p, g, m, v, c);
  if (!vec) return;
  const long nv = (n - head) >> 2;
  float4* __restrict__ p4 = reinterpret_cast<float4*>(p + head);
  const float4* __restrict__ g4 = reinterpret_cast<const float4*>(g + head);
  float4* __restrict__ m4 = reinterpret_cast<float4*>(m + head);
  float4* __restrict__ v4 = reinterpret_cast<float4*>(v + head);
  // two vectors per lane per trip, all eight 16-B loads issued before any
  // math (the compiler otherwise sinks the moment loads below the first
  // update and pays two HBM round trips per trip)
  for (long j = tid; j < nv; j += 2 * nt) {
    const long j1 = j + nt < nv ? j + nt : j;
    float4 pp[2] = {p4[j], p4[j1]}, mm[2] = {m4[j], m4[j1]}, vv[2] = {v4[j], v4[j1]};
    const float4 gg[2] = {g4[j], g4[j1]};
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      adamw_math(pp[u].x, mm[u].x, vv[u].x, gg[u].x, c);
      adamw_math(pp[u].y, mm[u].y, vv[u].y, gg[u].y, c);
      adamw_math(pp[u].z, mm[u].z, vv[u].z, gg[u].z, c);
      adamw_math(pp[u].w, mm[u].w, vv[u].w, gg[u].w, c);
    }
    p4[j] = pp[0];
    m4[j] = mm[0];
    v4[j] = vv[0];
    if (j1 != j) {
      p4[j1] = pp[1];
      m4[j1] = mm[1];
      v4[j1] = vv[1];
    }
  }
  for (long i = head + (nv << 2) + tid; i < n; i += nt) adamw_scalar(i, p, g, m, v, c);
}

__global__ void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, float lr, float b1, float b2, float eps, float wd, float step_size,
                             float bc2_sqrt, float grad_scale) {
  const AdamC c{1.f - lr * wd, 1.f - b1, b2, eps, step_size, bc2_sqrt, grad_scale};
  adamw_range(n, p, g, m, v, c);
}

// Device-resident schedule (graph-replayable step): sched = {lr, t, lr/(1-b1^t),
// sqrt(1-b2^t)} in fp64.  One thread advances t and the bias corrections
// (the same double arithmetic the host path does); the update kernel reads
// them, so a captured step needs no host-side scalars that change per step.
__global__ void adamw_sched_kernel(double* sched, double b1, double b2) {
  const double t = sched[1] + 1.0;
  sched[1] = t;
  sched[2] = sched[0] / (1.0 - pow(b1, t));
  sched[3] = sqrt(1.0 - pow(b2, t));
  sched[5] = 1.0 - pow(b1, t + 1.0);  // staged for the next advancing launch
  sched[6] = sqrt(1.0 - pow(b2, t + 1.0));
}

// advance != 0: this launch also advances the schedule (t + 1 and the bias
// corrections, computed per workgroup from sched[0..1] exactly as
// adamw_sched_kernel does), and the last workgroup to finish (an arrival
// count in sched[4], left at zero) writes them back -- every workgroup has
// read sched[1] by then.  Saves the one-thread schedule launch per step.
__global__ void adamw_dev_kernel(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, double* sched, float b1, float b2, float eps, float wd,
                                 float grad_scale, int advance) {
  // wave-uniform schedule values, no LDS: this launch shares the CUs with the
  // stem wgrad, which holds all of their LDS (conv_stem_bwd_wgrad_kernel)
  double t = sched[1], ss = sched[2], bc = sched[3];
  if (advance) {
    t += 1.0;
    const double c1 = sched[5];
    if (c1 != 0.0) {  // staged by the previous step (the same doubles as below)
      ss = sched[0] / c1;
      bc = sched[6];
    } else {  // a fresh or host-reset schedule: every thread evaluates them once
      ss = sched[0] / (1.0 - pow((double)b1, t));
      bc = sqrt(1.0 - pow((double)b2, t));
    }
  }
  const float lr = (float)sched[0];
  const AdamC c{1.f - lr * wd, 1.f - b1, b2, eps, (float)ss, (float)bc, grad_scale};
  adamw_range(n, p, g, m, v, c);
  if (advance) {
    // A workgroup counts as arrived once every one of its waves has read the
    // schedule: those loads have returned (their values were consumed before
    // the barrier), so the arrival needs no release -- and a release at agent
    // scope writes back the XCD's L2 (full of this launch's p / m / v lines)
    // for each of the 2048 workgroups: 129 vs 52 us for ResNet-18's 11.7 M
    // parameters (tools/time_adamw.py).  Nothing else this kernel writes is
    // ordered against the count; the last arriver's schedule stores reach the
    // next launch at the kernel boundary.
    __syncthreads();
    if (threadIdx.x != 0) return;
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(sched + 4);
    const unsigned long long old = __hip_atomic_fetch_add(cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      sched[1] = t;
      sched[2] = ss;
      sched[3] = bc;
      sched[5] = 1.0 - pow((double)b1, t + 1.0);  // the next step's, by one thread
      sched[6] = sqrt(1.0 - pow((double)b2, t + 1.0));
      __hip_atomic_store(cnt, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
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

// Batched preparation: one workgroup per (item, 64-k tile, 64-c tile, r, s);
// the 64x64 K x C slice is staged through LDS so both outputs are written as
// contiguous rows (KRSC rows run over c, CRSK rows over k).  One slice per
// workgroup keeps every load independent (a per-workgroup (r, s) loop
// serialises ~R*S HBM round trips: 0.36 ms for ResNet-18).
struct WprepTable {
  ssip_wprep it[SSIP_WPREP_MAX];
  int tile_start[SSIP_WPREP_MAX + 1];
  int count;
  int xcd;
};

template <typename T>
__global__ void __launch_bounds__(256) weight_prep_batch_kernel(const WprepTable tab) {
  __shared__ float tile[64][65];
  // XCD-aware order: the hardware deals workgroups round-robin to the 8 XCDs;
  // remap so each XCD runs a contiguous range, which puts the R*Sp tap slices
  // of one 64x64 (k, c) tile on one XCD: they read the same KCRS cache lines
  // (a 36-B lane stride), fetched into that XCD's L2 once instead of by up
  // to nine XCDs.
  int b = blockIdx.x, idx = 0;
  if (tab.xcd) {
    const int nb = gridDim.x, xcd = b & 7, q = nb >> 3, r = nb & 7;
    b = xcd * q + min(xcd, r) + (b >> 3);
  }
  while (idx + 1 < tab.count && b >= tab.tile_start[idx + 1]) ++idx;
  const ssip_wprep& e = tab.it[idx];
  b -= tab.tile_start[idx];
  const int rs = b % (e.R * e.Sp);
  b /= e.R * e.Sp;
  const int r = rs / e.Sp, s = rs - r * e.Sp;
  const int ctiles = (e.Cp + 63) / 64;
  const int k0 = (b / ctiles) * 64, c0 = (b % ctiles) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  T* krsc = static_cast<T*>(e.w_krsc);
  T* crsk = static_cast<T*>(e.w_crsk);
  // all sixteen loads of a thread in flight before the first LDS store (a
  // partly unrolled loop paid several HBM round trips per workgroup)
  float vals[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = k0 + ty + 4 * q, c = c0 + tx;
    vals[q] = (k < e.K && c < e.C && s < e.S) ? e.w_kcrs[(((long)k * e.C + c) * e.R + r) * e.S + s] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = k0 + ty + 4 * q;
    float v = vals[q];
    // only in-range elements take the folded BN scale: a padding zero times a
    // negative scale would store -0.0 where ssip_weight_prep stores +0.0
    if (e.kscale && k < e.K && c0 + tx < e.C && s < e.S) v *= e.kscale[k];
    tile[ty + 4 * q][tx] = v;
  }
  __syncthreads();
  if (krsc) {
    for (int kk = ty; kk < 64; kk += 4) {
      const int k = k0 + kk, c = c0 + tx;
      if (k < e.K && c < e.Cp) krsc[(((long)k * e.R + r) * e.Sp + s) * e.Cp + c] = from_f32<T>(tile[kk][tx]);
    }
  }
  if (crsk) {
    for (int cc = ty; cc < 64; cc += 4) {
      const int c = c0 + cc, k = k0 + tx;
      if (k < e.K && c < e.Cp) crsk[(((long)c * e.R + r) * e.Sp + s) * e.K + k] = from_f32<T>(tile[tx][cc]);
    }
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
  long blocks = (n + 1023) / 1024;  // 4 elements per lane
  if (blocks > 8192) blocks = 8192;
  SSIP_KLAUNCH(adamw_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (long)n, param, grad, exp_avg,
                     exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt, grad_scale);
  return ::ssip::check_launch("adamw");
}

int ssip_adamw_sched_step(double* sched, float beta1, float beta2, void* stream) {
  SSIP_REQUIRE(sched, SSIP_ERR_ARG, "ssip_adamw_sched_step: null schedule");
  SSIP_KLAUNCH(adamw_sched_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, sched, (double)beta1,
                     (double)beta2);
  return ::ssip::check_launch("adamw_sched");
}

int ssip_adamw_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, double* sched,
                   float beta1, float beta2, float eps, float weight_decay, float grad_scale, int advance,
                   void* stream) {
  SSIP_REQUIRE(n > 0 && param && grad && exp_avg && exp_avg_sq && sched, SSIP_ERR_ARG,
               "ssip_adamw_dev: bad arguments");
  long blocks = (n + 1023) / 1024;  // 4 elements per lane
  if (blocks > 2048) blocks = 2048;  // grid-stride: each wave computes the schedule scalars once
  SSIP_KLAUNCH(adamw_dev_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (long)n, param, grad,
                     exp_avg, exp_avg_sq, sched, beta1, beta2, eps, weight_decay, grad_scale, advance ? 1 : 0);
  return ::ssip::check_launch("adamw_dev");
}

int ssip_weight_prep(int dtype, int K, int C, int R, int S, int Cp, int Sp, const float* w_kcrs, void* w_krsc,
                     void* w_crsk, void* stream) {
  SSIP_REQUIRE(K > 0 && C > 0 && R > 0 && S > 0 && Cp >= C && Sp >= S && w_kcrs && (w_krsc || w_crsk), SSIP_ERR_ARG,
               "ssip_weight_prep: bad arguments");
  const long total = (long)K * R * Sp * Cp;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(weight_prep_kernel<T>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, K, C, R, S, Cp, Sp,
                       w_kcrs, (T*)w_krsc, (T*)w_crsk);
  });
  return ::ssip::check_launch("weight_prep");
}

}  // extern "C"

extern "C" int ssip_weight_prep_batch(int dtype, int count, const ssip_wprep* items, void* stream) {
  SSIP_REQUIRE(count >= 0 && count <= SSIP_WPREP_MAX && (count == 0 || items), SSIP_ERR_ARG,
               "ssip_weight_prep_batch: count must be 0..%d", SSIP_WPREP_MAX);
  if (count == 0) return SSIP_OK;
  WprepTable tab;
  memset(&tab, 0, sizeof(tab));
  tab.count = count;
  int tiles = 0;
  for (int i = 0; i < count; ++i) {
    const ssip_wprep& e = items[i];
    SSIP_REQUIRE(e.K > 0 && e.C > 0 && e.R > 0 && e.S > 0 && e.Cp >= e.C && e.Sp >= e.S && e.w_kcrs &&
                     (e.w_krsc || e.w_crsk),
                 SSIP_ERR_ARG, "ssip_weight_prep_batch: bad item %d", i);
    tab.it[i] = e;
    tab.tile_start[i] = tiles;
    tiles += ((e.K + 63) / 64) * ((e.Cp + 63) / 64) * e.R * e.Sp;
  }
  tab.tile_start[count] = tiles;
  tab.xcd = 1;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(weight_prep_batch_kernel<T>, dim3(tiles), dim3(256), 0, (hipStream_t)stream, tab);
  });
  return ::ssip::check_launch("weight_prep_batch");
}

// ---------------------------------------------------------------------------
// BatchNorm num_batches_tracked += delta for every BN layer in one launch
// ---------------------------------------------------------------------------
namespace {
struct CounterTable {
  int64_t* p[SSIP_COUNTERS_MAX];
};

__global__ void counters_add_kernel(CounterTable t, int count, int64_t delta) {
  const int i = threadIdx.x;
  if (i < count) t.p[i][0] += delta;
}
}  // namespace

extern "C" int ssip_counters_add(int count, int64_t* const* ptrs, int64_t delta, void* stream) {
  SSIP_REQUIRE(count >= 0 && count <= SSIP_COUNTERS_MAX && (count == 0 || ptrs), SSIP_ERR_ARG,
               "ssip_counters_add: count must be 0..%d", SSIP_COUNTERS_MAX);
  if (count == 0) return SSIP_OK;
  CounterTable t;
  for (int i = 0; i < count; ++i) {
    SSIP_REQUIRE(ptrs[i], SSIP_ERR_ARG, "ssip_counters_add: null counter %d", i);
    t.p[i] = ptrs[i];
  }
  SSIP_KLAUNCH(counters_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, t, count, delta);
  return ::ssip::check_launch("counters_add");
}
