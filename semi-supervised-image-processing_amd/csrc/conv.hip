// Implicit-GEMM convolution for gfx950 (CDNA4), NHWC activations.
//
// Replaces the torchvision/MIOpen convolutions that ResNet-18 runs inside
// `model(inputs)` / `loss.backward()` in the reference hot loop
// (reference: src/training/common.py:380-382; model built at :299-304).
//
// Three GEMM views of one conv (M x N x K, all fp32-accumulated on MFMA):
//   FWD   : Y[m=(n,p,q)][k]        = sum_{(r,s,c)} X[n,p*st-pd+r,q*st-pd+s,c] * W[k][r][s][c]
//   DGRAD : dX[m=(n,h,w)][c]       = sum_{(r,s,k)} dY[n,(h+pd-r)/st,(w+pd-s)/st,k] * WT[c][r][s][k]
//   WGRAD : dW[k][(r,s,c)]         = sum_{m=(n,p,q)} dY[m][k] * X[n,p*st-pd+r,q*st-pd+s,c]
// FWD/DGRAD stage A/B as [rows][32] k-contiguous LDS tiles (16-B slot XOR
// swizzle); WGRAD stages both operands m-major ([32][cols], as they lie in
// HBM) and reads fragments with ds_read_b64_tr_b16 (bf16) — no register
// transposes.  bf16 uses v_mfma_f32_16x16x32_bf16; the f32 parity path uses
// v_mfma_f32_16x16x4_f32 on the same tiles (8 MFMAs per 32-deep k step).
//
// FWD also emits per-(M-tile, channel) BatchNorm partial statistics
// {count, sum, M2-about-tile-mean} from the fp32 accumulators so the BN
// batch statistics need no extra pass over Y.  WGRAD is split over the m
// reduction into fp32 slabs that a second kernel sums in fixed order
// (bitwise reproducible, no atomics).
#include "ssip_common.h"

namespace {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct FastDiv {  // n / d for 0 <= n < 2^31, 1 <= d < 2^31 (round-up multiplier)
  uint32_t d, mul, shr;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) { f.mul = 0; f.shr = 0; return f; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;            // l = ceil(log2 d) >= 1
  const uint64_t p = 31 + l;
  f.mul = (uint32_t)(((1ull << p) + d - 1) / d);  // < 2^32
  f.shr = (uint32_t)(p - 32);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return f.mul ? (__umulhi(n, f.mul) >> f.shr) : n;
}

struct ConvArgs {
  int N, H, W, C, K, R, S, stride, pad, P, Q;
  int M;        // GEMM rows (FWD: N*P*Q, DGRAD: N*H*W, WGRAD: K)
  int Ng;       // GEMM cols (FWD: K, DGRAD: C, WGRAD: R*S*C)
  int Kg;       // reduction length (FWD: R*S*C, DGRAD: R*S*K)
  int Mred;     // WGRAD: N*P*Q
  int ksteps;   // k steps per block (WGRAD: per split)
  int tiles_n;
  FastDiv div_pq, div_q, div_hw, div_w;
  const void* A;
  const void* B;
  void* out;
  const void* add;
  float* partial;
};

// ---------------------------------------------------------------------------
// LDS addressing
// ---------------------------------------------------------------------------
// FWD/DGRAD tiles: [rows][32 elems].  bf16 rows are 64 B (4 x 16-B slots);
// slot' = slot ^ g(row) keeps every ds_read_b128 lane group conflict-free.
template <typename T> struct KTile;
template <> struct KTile<__bf16> {
  static constexpr int ROW_BYTES = 64;
  __device__ static __forceinline__ int off(int row, int slot) {
    const int g = (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // [0,2,3,1][(row>>2)&3]
    return row * 64 + ((slot ^ g) << 4);
  }
};
template <> struct KTile<float> {
  static constexpr int ROW_BYTES = 144;  // 128 B + 16 B pad
  __device__ static __forceinline__ int off(int row, int slot) { return row * 144 + (slot << 4); }
};

// WGRAD tiles: [32 m-rows][COLS elems], cols contiguous (as in HBM).
template <typename T, int COLS> struct MTile;
template <int COLS> struct MTile<__bf16, COLS> {
  static constexpr int ROW_BYTES = COLS * 2;
  static constexpr int UNITS = COLS / 4;  // 8-byte units per row
  __device__ static __forceinline__ int swz(int row) {
    int h = (row & 3) | (((row >> 3) & 1) << 2);
    return (h * 4) & (UNITS - 1) & ~3;
  }
  // byte offset of element `col` (multiple of 4) in row
  __device__ static __forceinline__ int off(int row, int col) {
    return row * ROW_BYTES + ((((col >> 2) ^ swz(row))) << 3);
  }
};
template <int COLS> struct MTile<float, COLS> {
  static constexpr int ROW_BYTES = COLS * 4 + 16;
  __device__ static __forceinline__ int off(int row, int col) { return row * ROW_BYTES + col * 4; }
};

// ---------------------------------------------------------------------------
// MFMA step over one 32-deep k slice for a FMxFN grid of 16x16 blocks
// ---------------------------------------------------------------------------
template <typename T> struct Frag;
template <> struct Frag<__bf16> { bf16x8 v; };
template <> struct Frag<float> { float v[8]; };

__device__ __forceinline__ void mma(f32x4& acc, const Frag<__bf16>& a, const Frag<__bf16>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f32x4& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[e], b.v[e], acc, 0, 0, 0);
}

// k-contiguous fragment: lane holds rows (l&15), k = 8*(l>>4) .. +7
__device__ __forceinline__ void read_kfrag(Frag<__bf16>& f, const char* base, int row, int kq) {
  f.v = *reinterpret_cast<const bf16x8*>(base + KTile<__bf16>::off(row, kq));
}
__device__ __forceinline__ void read_kfrag(Frag<float>& f, const char* base, int row, int kq) {
  const f32x4 lo = *reinterpret_cast<const f32x4*>(base + KTile<float>::off(row, 2 * kq));
  const f32x4 hi = *reinterpret_cast<const f32x4*>(base + KTile<float>::off(row, 2 * kq + 1));
  f.v[0] = lo[0]; f.v[1] = lo[1]; f.v[2] = lo[2]; f.v[3] = lo[3];
  f.v[4] = hi[0]; f.v[5] = hi[1]; f.v[6] = hi[2]; f.v[7] = hi[3];
}

// m-major fragment (WGRAD): lane l gets column col0 + (l&15), m = 8*(l>>4) .. +7
template <int COLS>
__device__ __forceinline__ void read_mfrag(Frag<__bf16>& f, const char* base, int col0, int lane) {
  typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = 8 * g + q;
  const char* a0 = base + MTile<__bf16, COLS>::off(r0, col0 + 4 * p);
  const char* a1 = base + MTile<__bf16, COLS>::off(r0 + 4, col0 + 4 * p);
  v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a0));
  v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a1));
  f.v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
template <int COLS>
__device__ __forceinline__ void read_mfrag(Frag<float>& f, const char* base, int col0, int lane) {
  const int g = lane >> 4, col = col0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    f.v[j] = *reinterpret_cast<const float*>(base + MTile<float, COLS>::off(8 * g + j, col));
}

// 4-element (one padded pixel) vector load helpers for the conv1 layout (C == 4)
template <typename T> struct Vec4;
template <> struct Vec4<__bf16> {
  typedef __attribute__((ext_vector_type(2))) int raw;
  raw v;
};
template <> struct Vec4<float> {
  typedef i32x4 raw;
  raw v;
};

template <typename T>
__device__ __forceinline__ void load_v8(Vec8<T>& d, const T* p, bool ok) {
  if (ok) d.load(p); else d.zero();
}
// two pixels of 4 channels each
template <typename T>
__device__ __forceinline__ void load_2px(Vec8<T>& d, const T* p0, bool ok0, const T* p1, bool ok1);
template <>
__device__ __forceinline__ void load_2px<__bf16>(Vec8<__bf16>& d, const __bf16* p0, bool ok0, const __bf16* p1, bool ok1) {
  typedef __attribute__((ext_vector_type(2))) int i2;
  i2 a = ok0 ? *reinterpret_cast<const i2*>(p0) : (i2){0, 0};
  i2 b = ok1 ? *reinterpret_cast<const i2*>(p1) : (i2){0, 0};
  d.v = (i32x4){a[0], a[1], b[0], b[1]};
}
template <>
__device__ __forceinline__ void load_2px<float>(Vec8<float>& d, const float* p0, bool ok0, const float* p1, bool ok1) {
  d.v0 = ok0 ? *reinterpret_cast<const i32x4*>(p0) : (i32x4){0, 0, 0, 0};
  d.v1 = ok1 ? *reinterpret_cast<const i32x4*>(p1) : (i32x4){0, 0, 0, 0};
}

template <typename T>
__device__ __forceinline__ void store_kchunk(char* base, int row, int kc, const Vec8<T>& v);
template <>
__device__ __forceinline__ void store_kchunk<__bf16>(char* base, int row, int kc, const Vec8<__bf16>& v) {
  *reinterpret_cast<i32x4*>(base + KTile<__bf16>::off(row, kc)) = v.v;
}
template <>
__device__ __forceinline__ void store_kchunk<float>(char* base, int row, int kc, const Vec8<float>& v) {
  *reinterpret_cast<i32x4*>(base + KTile<float>::off(row, 2 * kc)) = v.v0;
  *reinterpret_cast<i32x4*>(base + KTile<float>::off(row, 2 * kc + 1)) = v.v1;
}
template <typename T, int COLS>
__device__ __forceinline__ void store_mchunk(char* base, int row, int col, const Vec8<T>& v);
template <int COLS>
__device__ __forceinline__ void store_mchunk(char* base, int row, int col, const Vec8<__bf16>& v) {
  *reinterpret_cast<i32x4*>(base + MTile<__bf16, COLS>::off(row, col)) = v.v;
}
template <int COLS>
__device__ __forceinline__ void store_mchunk(char* base, int row, int col, const Vec8<float>& v) {
  *reinterpret_cast<i32x4*>(base + MTile<float, COLS>::off(row, col)) = v.v0;
  *reinterpret_cast<i32x4*>(base + MTile<float, COLS>::off(row, col + 4)) = v.v1;
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
template <int MODE, typename T, int BM, int BN, bool CONV1>
__global__ void __launch_bounds__(256) conv_gemm_kernel(const ConvArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr bool WG = (MODE == MODE_WGRAD);
  constexpr int A_BYTES = WG ? 32 * MTile<T, BM>::ROW_BYTES : BM * KTile<T>::ROW_BYTES;
  constexpr int B_BYTES = WG ? 32 * MTile<T, BN>::ROW_BYTES : BN * KTile<T>::ROW_BYTES;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ITA = BM * 4 / 256;  // 8-element chunks per thread per k step
  constexpr int ITB = BN * 4 / 256;
  static_assert(ITA >= 1 && ITB >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  const int tn = blockIdx.x % a.tiles_n;
  const int tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const T* __restrict__ Ag = static_cast<const T*>(a.A);
  const T* __restrict__ Bg = static_cast<const T*>(a.B);

  // ---------------- per-thread loader state ----------------
  // FWD/DGRAD A: chunk (row, kc) with row = (tid + it*256) >> 2, kc = tid & 3
  // B (FWD/DGRAD): same mapping over BN rows of the [Ng][Kg] weight matrix
  // WGRAD A: [32 m][BM cols]: m_local = id / (BM/8), col chunk = id % (BM/8)
  // WGRAD B: [32 m][BN cols]: m_local = id / (BN/8), col chunk = id % (BN/8)
  int a_base[ITA], a_h[ITA], a_w[ITA];
  bool a_ok[ITA];
  int b_r = 0, b_s = 0, b_c = 0;
  bool b_colok = true;
  const int kc = tid & 3;

  // uniform k-step counters (FWD/DGRAD):  k = ((r*S)+s)*Cred + cb
  int kr = 0, ks_ = 0, kcb = 0;
  const int Cred = (MODE == MODE_FWD) ? a.C : a.K;  // contiguous reduction channels

  long mstart = 0, mend = 0;
  if constexpr (!WG) {
#pragma unroll
    for (int it = 0; it < ITA; ++it) {
      const int row = (tid + it * 256) >> 2;
      const int m = m0 + row;
      a_ok[it] = m < a.M;
      const int mm = a_ok[it] ? m : 0;
      if constexpr (MODE == MODE_FWD) {
        const int n = fdiv(mm, a.div_pq);
        const int rem = mm - n * a.P * a.Q;
        const int p = fdiv(rem, a.div_q);
        const int q = rem - p * a.Q;
        a_base[it] = n * a.H * a.W;
        a_h[it] = p * a.stride - a.pad;
        a_w[it] = q * a.stride - a.pad;
      } else {
        const int n = fdiv(mm, a.div_hw);
        const int rem = mm - n * a.H * a.W;
        const int h = fdiv(rem, a.div_w);
        const int w = rem - h * a.W;
        a_base[it] = n * a.P * a.Q;
        a_h[it] = h + a.pad;
        a_w[it] = w + a.pad;
      }
    }
  } else {
    mstart = (long)blockIdx.y * a.ksteps * 32;
    mend = mstart + (long)a.ksteps * 32;
    if (mend > a.Mred) mend = a.Mred;
    // B column info (fixed per thread): col chunk nc = tid % (BN/8)
    const int nc = tid % (BN / 8);
    const int col = n0 + nc * 8;
    b_colok = col < a.Ng;
    const int cc = b_colok ? col : 0;
    if constexpr (CONV1) {
      b_r = cc / (a.S * a.C);
      const int rem = cc - b_r * a.S * a.C;
      b_s = rem / a.C;
      b_c = 0;
    } else {
      const int rs = cc / a.C;
      b_c = cc - rs * a.C;
      b_r = rs / a.S;
      b_s = rs - b_r * a.S;
    }
  }

  Vec8<T> ra[ITA], rb[ITB];

  auto load_tiles = [&](int ks) {
    if constexpr (MODE == MODE_FWD) {
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        if constexpr (CONV1) {
          // k step == filter row r; chunk kc = pixels s = 2kc, 2kc+1 (4 channels each)
          const int hin = a_h[it] + ks;
          const int w0 = a_w[it] + 2 * kc;
          const bool rowok = a_ok[it] && hin >= 0 && hin < a.H;
          const bool ok0 = rowok && w0 >= 0 && w0 < a.W;
          const bool ok1 = rowok && (w0 + 1) >= 0 && (w0 + 1) < a.W;
          const T* p0 = Ag + ((long)(a_base[it] + hin * a.W + w0)) * 4;
          load_2px<T>(ra[it], p0, ok0, p0 + 4, ok1);
        } else {
          const int hin = a_h[it] + kr, win = a_w[it] + ks_;
          const bool ok = a_ok[it] && hin >= 0 && hin < a.H && win >= 0 && win < a.W;
          const T* p = Ag + ((long)(a_base[it] + hin * a.W + win)) * a.C + kcb + kc * 8;
          load_v8<T>(ra[it], p, ok);
        }
      }
    } else if constexpr (MODE == MODE_DGRAD) {
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        const int hp = a_h[it] - kr, wp = a_w[it] - ks_;
        int p = hp, q = wp;
        bool ok = a_ok[it] && hp >= 0 && wp >= 0;
        if (a.stride != 1) {
          ok = ok && (hp % a.stride == 0) && (wp % a.stride == 0);
          p = hp / a.stride;
          q = wp / a.stride;
        }
        ok = ok && p < a.P && q < a.Q;
        const T* ptr = Ag + ((long)(a_base[it] + p * a.Q + q)) * a.K + kcb + kc * 8;
        load_v8<T>(ra[it], ptr, ok);
      }
    }
    if constexpr (!WG) {
      // B: [Ng][Kg] rows
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int row = (tid + it * 256) >> 2;
        const int n = n0 + row;
        const bool ok = n < a.Ng;
        const T* p = Bg + (long)(ok ? n : 0) * a.Kg + ks * 32 + kc * 8;
        load_v8<T>(rb[it], p, ok);
      }
    } else {
      // A: dY[m][K] chunk along k;  B: X gathered chunk along (r,s,c)
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        const int id = tid + it * 256;
        const int ml = id / (BM / 8), cch = id % (BM / 8);
        const long m = mstart + (long)ks * 32 + ml;
        const int k = m0 + cch * 8;
        const bool ok = m < mend && k < a.K;
        const T* p = Ag + (ok ? m : 0) * (long)a.K + (ok ? k : 0);
        load_v8<T>(ra[it], p, ok);
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int id = tid + it * 256;
        const int ml = id / (BN / 8);
        const long m = mstart + (long)ks * 32 + ml;
        const bool mok = m < mend && b_colok;
        const int mm = mok ? (int)m : 0;
        const int n = fdiv(mm, a.div_pq);
        const int rem = mm - n * a.P * a.Q;
        const int p = fdiv(rem, a.div_q);
        const int q = rem - p * a.Q;
        const int hin = p * a.stride - a.pad + b_r;
        if constexpr (CONV1) {
          const int w0 = q * a.stride - a.pad + b_s;
          const bool rowok = mok && hin >= 0 && hin < a.H;
          const bool ok0 = rowok && w0 >= 0 && w0 < a.W;
          const bool ok1 = rowok && (w0 + 1) >= 0 && (w0 + 1) < a.W;
          const T* p0 = Bg + ((long)((n * a.H + hin) * a.W + w0)) * 4;
          load_2px<T>(rb[it], p0, ok0, p0 + 4, ok1);
        } else {
          const int win = q * a.stride - a.pad + b_s;
          const bool ok = mok && hin >= 0 && hin < a.H && win >= 0 && win < a.W;
          const T* ptr = Bg + ((long)((n * a.H + hin) * a.W + win)) * a.C + b_c;
          load_v8<T>(rb[it], ptr, ok);
        }
      }
    }
  };

  auto advance_k = [&]() {  // uniform (r, s, cb) counters for FWD/DGRAD
    if constexpr (!WG && !CONV1) {
      kcb += 32;
      if (kcb >= Cred) {
        kcb = 0;
        if (++ks_ >= a.S) { ks_ = 0; ++kr; }
      }
    }
  };

  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
    if constexpr (!WG) {
#pragma unroll
      for (int it = 0; it < ITA; ++it) store_kchunk<T>(As, (tid + it * 256) >> 2, kc, ra[it]);
#pragma unroll
      for (int it = 0; it < ITB; ++it) store_kchunk<T>(Bs, (tid + it * 256) >> 2, kc, rb[it]);
    } else {
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        const int id = tid + it * 256;
        store_mchunk<BM>(As, id / (BM / 8), (id % (BM / 8)) * 8, ra[it]);
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int id = tid + it * 256;
        store_mchunk<BN>(Bs, id / (BN / 8), (id % (BN / 8)) * 8, rb[it]);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  int nsteps = a.ksteps;
  if constexpr (WG) {
    const long rem = mend - mstart;
    nsteps = rem > 0 ? (int)((rem + 31) / 32) : 0;
  }

  if (nsteps > 0) {
    load_tiles(0);
    advance_k();
    store_tiles(0);
    __syncthreads();
  }
  for (int ks = 0; ks < nsteps; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nsteps) {
      load_tiles(ks + 1);
      advance_k();
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    Frag<T> fa[FM], fb[FN];
    if constexpr (!WG) {
#pragma unroll
      for (int i = 0; i < FM; ++i) read_kfrag(fa[i], As, wm * WM + i * 16 + (lane & 15), lane >> 4);
#pragma unroll
      for (int j = 0; j < FN; ++j) read_kfrag(fb[j], Bs, wn * WN + j * 16 + (lane & 15), lane >> 4);
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i) read_mfrag<BM>(fa[i], As, wm * WM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) read_mfrag<BN>(fb[j], Bs, wn * WN + j * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[i], fb[j]);
    if (ks + 1 < nsteps) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  const int rbase = wm * WM + (lane >> 4) * 4;
  const int cbase = wn * WN + (lane & 15);
  if constexpr (MODE == MODE_WGRAD) {
    float* slab = static_cast<float*>(a.out) + (long)blockIdx.y * a.M * a.Ng;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + cbase + j * 16;
        if (n >= a.Ng) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + rbase + i * 16 + e;
          if (m < a.M) slab[(long)m * a.Ng + n] = acc[i][j][e];
        }
      }
    return;
  }

  // Out and Add may alias (in-place residual-gradient add): no __restrict__
  T* Out = static_cast<T*>(a.out);
  const T* Add = static_cast<const T*>(a.add);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + cbase + j * 16;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + rbase + i * 16 + e;
        if (m < a.M && n < a.Ng) {
          float v = acc[i][j][e];
          if constexpr (MODE == MODE_DGRAD) {
            if (Add) v += to_f32<T>(Add[(long)m * a.Ng + n]);
          }
          Out[(long)m * a.Ng + n] = from_f32<T>(v);
        }
      }
    }

  if constexpr (MODE == MODE_FWD) {
    if (a.partial == nullptr) return;
    // BatchNorm partial statistics over this tile's valid rows.
    float* red = reinterpret_cast<float*>(smem);  // [2][BN]  (main loop finished: safe to reuse)
    float* mean_t = red + 2 * BN;                  // [BN]
    const int cnt = min(BM, a.M - m0);
    float s[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase + i * 16 + e;
          t += (row < cnt) ? acc[i][j][e] : 0.f;
        }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      s[j] = t;
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) red[wm * BN + cbase + j * 16] = s[j];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) mean_t[c] = (red[c] + red[BN + c]) / (float)cnt;
    __syncthreads();
    float q2[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const float mu = mean_t[cbase + j * 16];
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase + i * 16 + e;
          const float d = acc[i][j][e] - mu;
          t += (row < cnt) ? d * d : 0.f;
        }
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      q2[j] = t;
    }
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) red[wm * BN + cbase + j * 16] = q2[j];
    }
    // sums were overwritten: recompute from mean
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      const int n = n0 + c;
      if (n < a.Ng) {
        const int tiles_m = gridDim.x / a.tiles_n;
        float* rec = a.partial + ((long)n * tiles_m + tm) * 3;  // [C][tiles][3]
        rec[0] = (float)cnt;
        rec[1] = mean_t[c] * (float)cnt;
        rec[2] = red[c] + red[BN + c];
      }
    }
  }
}

// WGRAD slab reduction:  dW[k][c][r][s] (torchvision KCRS, fp32) =
//   (accumulate ? dW : 0) + sum_split slab[split][k][(r*Sp + s)*Cp + c]
// Threads walk the slab in its own (k, col) order so every split's read is
// coalesced; padded columns (s >= S or c >= C) are skipped.
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K, int Ng, int C, int R,
                                    int S, int Cp, int Sp, float* __restrict__ dw, int accumulate) {
  const long total = (long)K * Ng;
  const long sstride = (long)K * Ng;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int col = (int)(idx % Ng);
    const int k = (int)(idx / Ng);
    const int c = col % Cp;
    const int rs = col / Cp;
    const int s = rs % Sp;
    const int r = rs / Sp;
    if (c >= C || s >= S) continue;
    float acc = 0.f;
    const float* p = slab + idx;
    for (int sp = 0; sp < splits; ++sp) acc += p[sp * sstride];
    const long o = (((long)k * C + c) * R + r) * S + s;
    dw[o] = accumulate ? dw[o] + acc : acc;
  }
}

// ---------------------------------------------------------------------------
// host-side planning
// ---------------------------------------------------------------------------
struct Plan {
  int mode;
  int bm, bn;
  bool conv1;
  ConvArgs args;
  dim3 grid;
  int splits;
};

static bool desc_ok(const ssip_conv_desc* d) {
  return d && d->N > 0 && d->H > 0 && d->W > 0 && d->C > 0 && d->K > 0 && d->R > 0 && d->S > 0 &&
         d->stride > 0 && d->pad >= 0 && d->P > 0 && d->Q > 0;
}

static void fill_common(ConvArgs& a, const ssip_conv_desc* d) {
  memset(&a, 0, sizeof(a));
  a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C; a.K = d->K; a.R = d->R; a.S = d->S;
  a.stride = d->stride; a.pad = d->pad; a.P = d->P; a.Q = d->Q;
  a.div_pq = make_fastdiv((uint32_t)(d->P * d->Q));
  a.div_q = make_fastdiv((uint32_t)d->Q);
  a.div_hw = make_fastdiv((uint32_t)(d->H * d->W));
  a.div_w = make_fastdiv((uint32_t)d->W);
}

static int plan_conv(int mode, const ssip_conv_desc* d, Plan& pl) {
  SSIP_REQUIRE(desc_ok(d), SSIP_ERR_ARG, "bad conv descriptor");
  // output size must match the conv formula
  pl.mode = mode;
  pl.conv1 = (d->C == 4);
  // the padded stem stores S = 8 columns for a real 7-wide filter
  const int s_real = pl.conv1 ? d->S - 1 : d->S;
  SSIP_REQUIRE(d->P == (d->H + 2 * d->pad - d->R) / d->stride + 1 && d->Q == (d->W + 2 * d->pad - s_real) / d->stride + 1,
               SSIP_ERR_ARG, "P/Q inconsistent with H/W/R/S/stride/pad");
  SSIP_REQUIRE(pl.conv1 ? (d->S == 8) : (d->C % 32 == 0), SSIP_ERR_ARG,
               "conv input channels must be a multiple of 32 (or 4 with S padded to 8); got C=%d S=%d", d->C, d->S);
  SSIP_REQUIRE(d->K % 32 == 0, SSIP_ERR_ARG, "conv output channels must be a multiple of 32; got K=%d", d->K);
  const long NPQ = (long)d->N * d->P * d->Q, NHW = (long)d->N * d->H * d->W;
  SSIP_REQUIRE(NPQ < (1l << 31) && NHW * d->C < (1l << 31) && NPQ * d->K < (1l << 31), SSIP_ERR_ARG,
               "tensor too large for 32-bit indexing");
  ConvArgs& a = pl.args;
  fill_common(a, d);
  pl.splits = 1;
  if (mode == MODE_FWD) {
    a.M = (int)NPQ; a.Ng = d->K; a.Kg = d->R * d->S * d->C;
    a.ksteps = a.Kg / 32;
    pl.bm = 128; pl.bn = (d->K % 128 == 0) ? 128 : 64;
  } else if (mode == MODE_DGRAD) {
    SSIP_REQUIRE(!pl.conv1, SSIP_ERR_ARG, "dgrad of the C=4 stem conv is not supported (input needs no grad)");
    a.M = (int)NHW; a.Ng = d->C; a.Kg = d->R * d->S * d->K;
    a.ksteps = a.Kg / 32;
    pl.bm = 128; pl.bn = (d->C % 128 == 0) ? 128 : 64;
  } else {
    a.M = d->K; a.Ng = d->R * d->S * d->C; a.Kg = 0;
    a.Mred = (int)NPQ;
    pl.bm = (d->K % 128 == 0) ? 128 : 64;
    pl.bn = 128;
    if (a.Ng % 128 != 0 && a.Ng % 64 == 0 && pl.bm == 128) pl.bn = 64;
    const int tiles = ceil_div(a.M, pl.bm) * ceil_div(a.Ng, pl.bn);
    const int total_ks = ceil_div(a.Mred, 32);
    // ~1024 blocks (4 per CU), slab <= 64 MiB (stays in the Infinity Cache),
    // >= 8 k-steps per split
    int splits = ceil_div(1024, tiles);
    const long slab_split = (long)a.M * a.Ng * 4;
    const int cap_bytes = (int)std::max<long>(1, (64l << 20) / slab_split);
    if (splits > cap_bytes) splits = cap_bytes;
    const int max_splits = ceil_div(total_ks, 8);
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    a.ksteps = ceil_div(total_ks, splits);
    splits = ceil_div(total_ks, a.ksteps);
    pl.splits = splits;
  }
  a.tiles_n = ceil_div(a.Ng, pl.bn);
  const int tiles_m = ceil_div(a.M, pl.bm);
  pl.grid = dim3(tiles_m * a.tiles_n, pl.splits, 1);
  return SSIP_OK;
}

template <int MODE, typename T>
static int launch_conv(const Plan& pl, hipStream_t st) {
#define SSIP_LAUNCH(BM_, BN_, C1_) \
  { hipLaunchKernelGGL((conv_gemm_kernel<MODE, T, BM_, BN_, C1_>), pl.grid, dim3(256), 0, st, pl.args); }
  const bool c1 = pl.conv1;
  if (pl.bm == 128 && pl.bn == 128) {
    if constexpr (MODE != MODE_DGRAD) { if (c1) SSIP_LAUNCH(128, 128, true) else SSIP_LAUNCH(128, 128, false) }
    else SSIP_LAUNCH(128, 128, false)
  } else if (pl.bm == 128 && pl.bn == 64) {
    if constexpr (MODE != MODE_DGRAD) { if (c1) SSIP_LAUNCH(128, 64, true) else SSIP_LAUNCH(128, 64, false) }
    else SSIP_LAUNCH(128, 64, false)
  } else if (pl.bm == 64 && pl.bn == 128 && MODE == MODE_WGRAD) {
    if (c1) SSIP_LAUNCH(64, 128, true) else SSIP_LAUNCH(64, 128, false)
  } else {
    ::ssip::set_error("no kernel for tile %dx%d", pl.bm, pl.bn);
    return SSIP_ERR_ARG;
  }
#undef SSIP_LAUNCH
  return ::ssip::check_launch("conv_gemm");
}

}  // namespace

extern "C" {

int64_t ssip_conv_fwd_partial_floats(const ssip_conv_desc* d) {
  Plan pl;
  if (plan_conv(MODE_FWD, d, pl) != SSIP_OK) return -1;
  return (int64_t)ceil_div(pl.args.M, pl.bm) * d->K * 3;
}

int ssip_conv_fwd(const ssip_conv_desc* d, int dtype, const void* x, const void* w_krsc, void* y, float* bn_partial,
                  void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_FWD, d, pl);
  if (rc) return rc;
  SSIP_REQUIRE(x && w_krsc && y, SSIP_ERR_ARG, "ssip_conv_fwd: null pointer");
  pl.args.A = x; pl.args.B = w_krsc; pl.args.out = y; pl.args.partial = bn_partial;
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_FWD, T>(pl, (hipStream_t)stream));
}

int ssip_conv_dgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, void* dx,
                    const void* dx_add, void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_DGRAD, d, pl);
  if (rc) return rc;
  SSIP_REQUIRE(dy && w_crsk && dx, SSIP_ERR_ARG, "ssip_conv_dgrad: null pointer");
  pl.args.A = dy; pl.args.B = w_crsk; pl.args.out = dx; pl.args.add = dx_add;
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_DGRAD, T>(pl, (hipStream_t)stream));
}

int64_t ssip_conv_wgrad_workspace_bytes(const ssip_conv_desc* d) {
  Plan pl;
  if (plan_conv(MODE_WGRAD, d, pl) != SSIP_OK) return -1;
  return (int64_t)pl.splits * pl.args.M * pl.args.Ng * 4;
}

int ssip_conv_wgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* x, float* dw_kcrs, int c_real,
                    int s_real, int accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_WGRAD, d, pl);
  if (rc) return rc;
  SSIP_REQUIRE(dy && x && dw_kcrs && workspace, SSIP_ERR_ARG, "ssip_conv_wgrad: null pointer");
  const int64_t need = (int64_t)pl.splits * pl.args.M * pl.args.Ng * 4;
  SSIP_REQUIRE(workspace_bytes >= need, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
               (long long)workspace_bytes, (long long)need);
  SSIP_REQUIRE(c_real >= 1 && c_real <= d->C && s_real >= 1 && s_real <= d->S, SSIP_ERR_ARG, "bad c_real/s_real");
  pl.args.A = dy; pl.args.B = x; pl.args.out = workspace;
  hipStream_t st = (hipStream_t)stream;
  SSIP_DISPATCH_DTYPE(dtype, T, rc = launch_conv<MODE_WGRAD, T>(pl, st));
  if (rc) return rc;
  const long total = (long)d->K * pl.args.Ng;
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)workspace, pl.splits, d->K,
                     pl.args.Ng, c_real, d->R, s_real, d->C, d->S, dw_kcrs, accumulate);
  return ::ssip::check_launch("wgrad_reduce");
}

}  // extern "C"
