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
//
// Block = WMW x WNW waves (64-wide), tile BM x BN, k-step BK = 128 bytes of
// reduction per row (64 bf16 / 32 f32).  FWD/DGRAD stage A/B as
// [rows][128 B] k-contiguous LDS tiles (16-B slot XOR swizzle, conflict-free
// ds_read_b128 fragment reads); WGRAD stages both operands m-major
// ([BK][cols], as they lie in HBM) and reads fragments with
// ds_read_b64_tr_b16 (bf16) — no register transposes.  Global->LDS staging
// is register double-buffered (issue k+1 loads before the MFMAs of k, write
// them to the other LDS buffer after), one barrier per k-step.
// bf16: v_mfma_f32_16x16x32_bf16; f32 parity path: v_mfma_f32_16x16x4_f32 on
// the same tiles.  Epilogue goes through LDS so global stores (and the
// residual-gradient add of DGRAD) are 16-B per lane, row-contiguous.
//
// FWD also emits per-(channel, M-tile) BatchNorm partial statistics
// {count, sum, M2-about-tile-mean} from the fp32 accumulators so the BN
// batch statistics need no extra pass over Y.  WGRAD is split over the m
// reduction into fp32 slabs that a second kernel sums in fixed order
// (bitwise reproducible, no atomics).
#include <algorithm>
#include <cstdio>
#include <vector>
#include "ssip_common.h"
#include "fin_split.h"

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

struct PhaseInfo {
  int M, tiles_m, ksteps;     // rows (N * Hph * Wph), M-tiles, k-steps of this phase
  int r0, s0, nr, ns, bh, bw;  // first tap, tap counts, dy offsets
  int ph, pw, Wph;
  FastDiv div_hw, div_w;       // / (Hph * Wph), / Wph
};

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
  const void* add;     // DGRAD: residual-gradient add; FWD: residual (ssip_conv_fwd_bias)
  float* partial;
  const float* bias;   // FWD: per-output-channel bias (a folded eval-mode BatchNorm), nullable
  int relu;            // FWD: ReLU on the output (after bias and residual)
  // DGRAD post-op (BN backward of the layer that produced this conv's input):
  // out = (dgrad + add) * relu_mask; per-(channel, tile) sums of out and
  // out * (py - pmean) * pinvstd into partial [Ng][tiles_m][2].  The ReLU
  // mask: pmask > 0 (z), else bit n & 7 of pbits[m * Ng / 8 + n / 8], else
  // fma(py, pmscale, pmshift) > 0 (the forward's sign for a BN+ReLU with no
  // residual).  Active when pmean != nullptr.
  const void* pmask;
  const uint8_t* pbits;
  const float* pmscale;
  const float* pmshift;
  const void* py;
  const float* pmean;
  const float* pinvstd;
  // DGRAD stride-2 phase split (LDS-DMA kernel): blockIdx.y = phase
  // (ph, pw) = output rows h = 2i+ph, columns w = 2j+pw; only the taps
  // r = r0 + 2*ri, s = s0 + 2*si reach them, at dy row p = i + bh - ri.
  int phased;
  PhaseInfo phase[4];
  // phase order (2 bits each, heaviest first): workgroup t of an XCD's
  // contiguous run takes phase (phase_order >> 2*(t & 3)) & 3 of tile t >> 2,
  // so every XCD gets the same mix of long and short phases
  int phase_order;
  // DGRAD of a stride-2 3x3 conv fused with its block's 1x1 / stride-2
  // downsample (ssip_conv_dgrad_ds): phase (0, 0) -- the only one the
  // downsample reaches, at the same dy pixel as its single tap -- runs
  // ds_from own k-steps, then K/64 more over dY_ds (A2) and W_ds [C][K] (B2)
  const void* A2;
  const void* B2;
  uint32_t a2_bytes, b2_bytes;
  int ds_from;
  int xcd_remap;  // 1: XCD-aware workgroup -> tile order (LDS-DMA kernel)
  int dma_mid;  // LDS-DMA ring: the next stage's pieces after the k-step's reads, before its second MFMA half (SSIP_DMA_MID)
  int stagger;  // LDS-DMA ring: waves NW/2.. run each k-step's second MFMA half after the next barrier (SSIP_STAGGER)
  // INBN (LDS-DMA ring, FWD's A / WGRAD's B operand): the conv input is
  // relu(fma(y, in_scale[c], in_shift[c])) of the layer below, formed in place
  // in the ring after each wave's own pieces land (ssip_conv_*_bnrelu_in)
  const float* in_scale;
  const float* in_shift;
  // INBN FWD of a 1x1 / stride-1 conv (nullable): the n-tile-0 workgroups
  // also store each transformed piece to zout (same layout as A), so the
  // weight gradient takes relu(bn(y)) as a plain input
  void* zout;
  // FWD of a 3x3 / stride-s conv fused with its block's 1x1 / stride-s
  // downsample (ssip_conv_fwd_ds): workgroups >= fwd_tiles1 compute the
  // downsample's tiles -- its input pixel is the conv's tap (1, 1) pixel, so
  // they run only that tap's C/64 k-steps, with W_ds [K][C] as B -- into
  // out_ds / partial_ds.  0: no downsample.
  int fwd_tiles1;
  const void* Bds;
  void* out_ds;
  float* partial_ds;
  uint32_t bds_bytes;
  int stat_tiles_m;  // BN record tiles per channel when the grid is not tiles_m x tiles_n (0: from the grid)
  uint32_t a_bytes, b_bytes;  // operand extents (LDS-DMA kernel buffer resources)
  // WGRAD x-gather walk: a 64-row k-step advances each row's output pixel
  // (n, p, q) by (dn, dp, dq); its input byte offset by k0, plus e1 when q
  // wraps into the next row and e2 when p wraps into the next image
  int wg_dn, wg_dp, wg_dq, wg_k0, wg_e1, wg_e2;
};

template <typename T> struct Traits;
template <> struct Traits<__bf16> { static constexpr int BK = 64; };
template <> struct Traits<float> { static constexpr int BK = 32; };

// ---------------------------------------------------------------------------
// LDS addressing
// ---------------------------------------------------------------------------
// FWD/DGRAD tiles: [rows][128 B] (8 x 16-B slots).  slot' = slot ^ ((row>>1)&7)
// makes every 16-lane group of a ds_read_b128 fragment read (rows l&15,
// slot 4h + (l>>4) for bf16; slots 2(l>>4)+{0,1} for f32) hit 16 distinct
// 16-B bank slots.
__device__ __forceinline__ int ktile_off(int row, int slot) { return row * 128 + ((slot ^ ((row >> 1) & 7)) << 4); }

// WGRAD tiles: [BK m-rows][COLS elems], cols contiguous (as in HBM).
template <typename T, int COLS> struct MTile;
// 16-B chunk XOR of row `row` in a 64-column (128-B row) MTile: a transposed
// fragment read (read_mfrag / read_tfrag) touches rows r0 + {0..3, 8..11} in
// one 32-lane half, and two rows of equal parity share the 32 banks of one
// 128-B half-line -- so the four equal-parity rows need four different 32-B
// column groups for every r0.  Row bits 1 and 3 pick the group (the former
// row & 3 selector repeated every 8 rows: rows r and r + 8 collided, a 2-way
// conflict on every read, SQ_LDS_BANK_CONFLICT = 0.50 of the active LDS
// cycles of conv_halo_wgrad_kernel).
__device__ __forceinline__ int mt64_chunk_xor(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

template <int COLS> struct MTile<__bf16, COLS> {
  static constexpr int ROW_BYTES = COLS * 2;
  static constexpr int UNITS = COLS / 4;  // 8-byte units per row
  __device__ static __forceinline__ int swz(int row) {
    if constexpr (COLS == 64) return mt64_chunk_xor(row) << 1;
    int h = (row & 3) | (((row >> 3) & 1) << 2);
    return (h * 4) & (UNITS - 1) & ~3;
  }
  __device__ static __forceinline__ int off(int row, int col) {  // col multiple of 4
    return row * ROW_BYTES + ((((col >> 2) ^ swz(row))) << 3);
  }
};
template <int COLS> struct MTile<float, COLS> {
  static constexpr int ROW_BYTES = COLS * 4 + 16;
  __device__ static __forceinline__ int off(int row, int col) { return row * ROW_BYTES + col * 4; }
};

// ---------------------------------------------------------------------------
// fragments and MFMA
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

// k-contiguous fragment for 32-deep sub-step h: lane holds row (l&15), k = 32h + 8(l>>4) .. +7
__device__ __forceinline__ void read_kfrag(Frag<__bf16>& f, const char* base, int row, int kq, int h) {
  f.v = *reinterpret_cast<const bf16x8*>(base + ktile_off(row, 4 * h + kq));
}
__device__ __forceinline__ void read_kfrag(Frag<float>& f, const char* base, int row, int kq, int) {
  const f32x4 lo = *reinterpret_cast<const f32x4*>(base + ktile_off(row, 2 * kq));
  const f32x4 hi = *reinterpret_cast<const f32x4*>(base + ktile_off(row, 2 * kq + 1));
  f.v[0] = lo[0]; f.v[1] = lo[1]; f.v[2] = lo[2]; f.v[3] = lo[3];
  f.v[4] = hi[0]; f.v[5] = hi[1]; f.v[6] = hi[2]; f.v[7] = hi[3];
}

// m-major fragment (WGRAD) for sub-step h: lane l gets column col0 + (l&15),
// m = 32h + 8(l>>4) .. +7
template <int COLS>
__device__ __forceinline__ void read_mfrag(Frag<__bf16>& f, const char* base, int col0, int lane, int h) {
  typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = 32 * h + 8 * g + q;
  const char* a0 = base + MTile<__bf16, COLS>::off(r0, col0 + 4 * p);
  const char* a1 = base + MTile<__bf16, COLS>::off(r0 + 4, col0 + 4 * p);
  v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a0));
  v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a1));
  f.v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
template <int COLS>
__device__ __forceinline__ void read_mfrag(Frag<float>& f, const char* base, int col0, int lane, int h) {
  const int g = lane >> 4, col = col0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 8; ++j)
    f.v[j] = *reinterpret_cast<const float*>(base + MTile<float, COLS>::off(32 * h + 8 * g + j, col));
}

template <typename T>
__device__ __forceinline__ void load_v8(Vec8<T>& d, const T* p, bool ok) {
  if (ok) d.load(p); else d.zero();
}
// two padded pixels of 4 channels each (stem layout)
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

// 8-element chunk kc (0..KC-1) of a k-tile row
__device__ __forceinline__ void store_kchunk(char* base, int row, int kc, const Vec8<__bf16>& v) {
  *reinterpret_cast<i32x4*>(base + ktile_off(row, kc)) = v.v;
}
__device__ __forceinline__ void store_kchunk(char* base, int row, int kc, const Vec8<float>& v) {
  *reinterpret_cast<i32x4*>(base + ktile_off(row, 2 * kc)) = v.v0;
  *reinterpret_cast<i32x4*>(base + ktile_off(row, 2 * kc + 1)) = v.v1;
}
template <int COLS>
__device__ __forceinline__ void store_mchunk(char* base, int row, int col, const Vec8<__bf16>& v) {
  *reinterpret_cast<i32x4*>(base + MTile<__bf16, COLS>::off(row, col)) = v.v;
}
template <int COLS>
__device__ __forceinline__ void store_mchunk(char* base, int row, int col, const Vec8<float>& v) {
  *reinterpret_cast<i32x4*>(base + MTile<float, COLS>::off(row, col)) = v.v0;
  *reinterpret_cast<i32x4*>(base + MTile<float, COLS>::off(row, col + 4)) = v.v1;
}

template <int MODE, typename T, int BM, int BN>
struct Smem {
  static constexpr int BK = Traits<T>::BK;
  static constexpr bool WG = (MODE == MODE_WGRAD);
  static constexpr int A_BYTES = WG ? BK * MTile<T, BM>::ROW_BYTES : BM * 128;
  static constexpr int B_BYTES = WG ? BK * MTile<T, BN>::ROW_BYTES : BN * 128;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int EPI = WG ? 0 : BM * (BN * (int)sizeof(T) + 16);
  static constexpr int BYTES = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
};

// ---------------------------------------------------------------------------
// shared epilogue: WGRAD -> fp32 slab; FWD/DGRAD -> LDS-staged 16-B stores
// (+ residual-gradient add for DGRAD, + BN partial statistics for FWD)
// ---------------------------------------------------------------------------
// DGRAD epilogue with the BatchNorm-backward reduction fused in (the tile is
// already staged in LDS as T).  Each thread owns one 8-channel chunk (NT is a
// multiple of BN/8), so its sums stay in registers; the NT/(BN/8) partial
// sums per chunk are combined in fixed order through LDS.
// The epilogue operands of the fused BN backward (mask z, pre-BN y and the
// residual-gradient add) for the rows this thread stores; the LDS-DMA kernel
// loads them before its main loop so the epilogue never waits on HBM.
template <typename T, int BM, int BN, int NT>
struct BnPostRegs {
  static constexpr int CPR = BN / 8;
  static constexpr int RPI = NT / CPR;  // rows per pass
  static constexpr int ROWS = BM / RPI;
  static_assert(NT % CPR == 0 && BM % RPI == 0, "thread count must cover whole rows");
  Vec8<T> z[ROWS], y[ROWS], add[ROWS];
  uint32_t mb[ROWS];  // mask byte (pbits) of the thread's 8-channel chunk

  __device__ __forceinline__ void load(const ConvArgs& a, int m0, int n0) {
    const int tid = threadIdx.x;
    const int ch = tid % CPR, rsub = tid / CPR;
    const int n = n0 + ch * 8;
    if (n >= a.Ng) return;
    const T* Zm = static_cast<const T*>(a.pmask);
    const T* Yp = static_cast<const T*>(a.py);
    const T* Add = static_cast<const T*>(a.add);
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int m = m0 + rsub + k * RPI;
      if (m < a.M) {
        const long off = (long)m * a.Ng + n;
        if (Zm) z[k].load(Zm + off);
        else if (a.pbits) mb[k] = a.pbits[off >> 3];
        y[k].load(Yp + off);
        if (Add) add[k].load(Add + off);
      }
    }
  }
};

template <typename T, int BM, int BN, int NT>
__device__ __forceinline__ void dgrad_bn_post(const ConvArgs& a, char* smem, int m0, int n0, int tm,
                                              const BnPostRegs<T, BM, BN, NT>& pr) {
  constexpr int CPR = BN / 8;
  constexpr int RPI = NT / CPR;  // rows per pass
  constexpr int ROWS = BM / RPI;
  constexpr int EROW = BN * (int)sizeof(T) + 16;
  const int tid = threadIdx.x;
  const int ch = tid % CPR, rsub = tid / CPR;
  const int n = n0 + ch * 8;
  T* Out = static_cast<T*>(a.out);
  const bool has_add = a.add != nullptr;
  float sd[8], sx[8], mu[8], is[8], msc[8], msh[8];
  const bool nok = n < a.Ng;
  const int mode = a.pmask ? 0 : (a.pbits ? 1 : 2);  // mask source (ConvArgs)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sd[j] = 0.f;
    sx[j] = 0.f;
    mu[j] = nok ? a.pmean[n + j] : 0.f;
    is[j] = nok ? a.pinvstd[n + j] : 0.f;
    msc[j] = (nok && mode == 2) ? a.pmscale[n + j] : 0.f;
    msh[j] = (nok && mode == 2) ? a.pmshift[n + j] : 0.f;
  }
  if (nok) {
#pragma unroll
    for (int k = 0; k < ROWS; ++k) {
      const int row = rsub + k * RPI;
      const int m = m0 + row;
      if (m >= a.M) break;
      Vec8<T> v;
      const char* src = smem + row * EROW + ch * 8 * (int)sizeof(T);
      if constexpr (sizeof(T) == 2) {
        v.v = *reinterpret_cast<const i32x4*>(src);
      } else {
        reinterpret_cast<Vec8<float>&>(v).v0 = reinterpret_cast<const i32x4*>(src)[0];
        reinterpret_cast<Vec8<float>&>(v).v1 = reinterpret_cast<const i32x4*>(src)[1];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = v.get(j);
        if (has_add) d += pr.add[k].get(j);
        const bool keep = mode == 0 ? pr.z[k].get(j) > 0.f
                                    : (mode == 1 ? ((pr.mb[k] >> j) & 1u) != 0u
                                                 : __builtin_fmaf(pr.y[k].get(j), msc[j], msh[j]) > 0.f);
        d = keep ? d : 0.f;
        v.set(j, d);
        const float dq = v.get(j);  // the stored (rounded) value feeds the sums
        sd[j] += dq;
        sx[j] += dq * ((pr.y[k].get(j) - mu[j]) * is[j]);
      }
      v.store(Out + (long)m * a.Ng + n);
    }
  }
  // lanes l, l+CPR, ... of a wave share a chunk: butterfly over the lane
  // bits above log2(CPR), then combine the waves in fixed order via LDS.
  static_assert(CPR == 8 || CPR == 16 || CPR == 32, "chunk count per row");
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sd[j] += __shfl_xor(sd[j], o, 64);
      sx[j] += __shfl_xor(sx[j], o, 64);
    }
  }
  __syncthreads();
  constexpr int NW = NT / 64;
  float* red = reinterpret_cast<float*>(smem);  // [NW][CPR][16]
  const int lane = tid & 63, wave = tid >> 6;
  if (lane < CPR) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * CPR + lane) * 16 + j] = sd[j];
      red[(wave * CPR + lane) * 16 + 8 + j] = sx[j];
    }
  }
  __syncthreads();
  if (tid < CPR * 16) {
    const int c8 = tid >> 4, v = tid & 15;  // chunk, value (0-7 sum d, 8-15 sum d*xhat)
    const int nn = n0 + c8 * 8;
    if (nn < a.Ng) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += red[(w * CPR + c8) * 16 + v];
      const int tiles_m = (a.M + BM - 1) / BM;  // [Ng][tiles_m][2]: each channel's records contiguous
      a.partial[((long)(nn + (v & 7)) * tiles_m + tm) * 2 + (v >> 3)] = t;
    }
  }
}

// GEMM row -> output row (identity, or the phase's strided rows of dx)
struct RowMap {
  int M;
  bool phased;  // false: identity
  int H, W, ph, pw, Wph;
  FastDiv div_hw, div_w;
  __device__ __forceinline__ long row(int m) const {
    if (!phased) return m;
    const int n = fdiv(m, div_hw);
    const int rem = m - n * (int)div_hw.d;
    const int i = fdiv(rem, div_w);
    const int j = rem - i * Wph;
    return ((long)n * H + 2 * i + ph) * W + 2 * j + pw;
  }
};

template <int MODE, typename T, int BM, int BN, int WMW, int WNW, int FM, int FN, bool ALLOW_POST = true,
          bool FOLD = false>
__device__ __forceinline__ void conv_epilogue_impl(const ConvArgs& a, f32x4 (&acc)[FM][FN], char* smem, int m0,
                                                   int n0, int tm, const BnPostRegs<T, BM, BN, 64 * WMW * WNW>& pre,
                                                   bool pre_loaded, const RowMap& rmap, int split,
                                                   void* out_alt = nullptr, float* partial_alt = nullptr) {
  constexpr int NT = 64 * WMW * WNW;
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WNW, wn = wave % WNW;
  const int rbase = wm * WTM + (lane >> 4) * 4;
  const int cbase = wn * WTN + (lane & 15);
  if constexpr (MODE == MODE_WGRAD) {
    float* slab = static_cast<float*>(a.out) + (long)split * a.M * a.Ng;
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

  // stage the tile through LDS (main loop finished: the staging buffers are free)
  constexpr int EROW = BN * (int)sizeof(T) + 16;  // padded row (bytes)
  {
    float bcol[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + cbase + j * 16;
      bcol[j] = (FOLD && n < a.Ng) ? a.bias[n] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase + i * 16 + e;
          const int col = cbase + j * 16;
          *reinterpret_cast<T*>(smem + row * EROW + col * (int)sizeof(T)) =
              from_f32<T>(FOLD ? acc[i][j][e] + bcol[j] : acc[i][j][e]);
        }
  }
  __syncthreads();
  if constexpr (MODE == MODE_DGRAD && ALLOW_POST) {
    if (a.pmean != nullptr) {
      if (pre_loaded) {
        dgrad_bn_post<T, BM, BN, NT>(a, smem, m0, n0, tm, pre);
      } else {
        BnPostRegs<T, BM, BN, NT> pr;
        pr.load(a, m0, n0);
        dgrad_bn_post<T, BM, BN, NT>(a, smem, m0, n0, tm, pr);
      }
      return;
    }
  }
  {
    // each thread moves 8-element chunks: BN/8 chunks per row
    constexpr int CPR = BN / 8;
    T* Out = static_cast<T*>(out_alt ? out_alt : a.out);   // may alias Add (in-place residual-gradient add)
    const T* Add = static_cast<const T*>(a.add);
    for (int id = tid; id < BM * CPR; id += NT) {
      const int row = id / CPR, ch = id % CPR;
      const int m = m0 + row, n = n0 + ch * 8;
      if (m >= rmap.M || n >= a.Ng) continue;
      const long orow = rmap.row(m);
      Vec8<T> v;
      const char* src = smem + row * EROW + ch * 8 * (int)sizeof(T);
      if constexpr (sizeof(T) == 2) {
        v.v = *reinterpret_cast<const i32x4*>(src);
      } else {
        reinterpret_cast<Vec8<float>&>(v).v0 = reinterpret_cast<const i32x4*>(src)[0];
        reinterpret_cast<Vec8<float>&>(v).v1 = reinterpret_cast<const i32x4*>(src)[1];
      }
      if constexpr (MODE == MODE_DGRAD) {
        if (Add) {
          // the unrounded accumulator would be better; the LDS copy is already in T
          Vec8<T> r;
          r.load(Add + orow * a.Ng + n);
#pragma unroll
          for (int j = 0; j < 8; ++j) v.set(j, v.get(j) + r.get(j));
        }
      }
      if constexpr (MODE == MODE_FWD && FOLD) {  // folded eval BN: + residual, ReLU (bias already in)
        {
          Vec8<T> r;
          if (Add) r.load(Add + orow * a.Ng + n);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = v.get(j);
            if (Add) t += r.get(j);
            if (a.relu) t = t > 0.f ? t : 0.f;
            v.set(j, t);
          }
        }
      }
      v.store(Out + orow * a.Ng + n);
    }
  }

  if constexpr (MODE == MODE_FWD) {
    float* const partial = partial_alt ? partial_alt : a.partial;
    if (partial == nullptr) return;
    __syncthreads();
    // BatchNorm partial statistics over this tile's valid rows (from fp32 accumulators).
    float* red = reinterpret_cast<float*>(smem);  // [WMW][BN]
    float* mean_t = red + WMW * BN;               // [BN]
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
    for (int c = tid; c < BN; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WMW; ++w) t += red[w * BN + c];
      mean_t[c] = t / (float)cnt;
    }
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
    __syncthreads();
    const int tiles_m = a.stat_tiles_m > 0 ? a.stat_tiles_m : (int)(gridDim.x / a.tiles_n);
    for (int c = tid; c < BN; c += NT) {
      const int n = n0 + c;
      if (n < a.Ng) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WMW; ++w) t += red[w * BN + c];
        float* rec = partial + ((long)n * tiles_m + tm) * 3;  // [C][tiles][3]
        rec[0] = (float)cnt;
        rec[1] = mean_t[c] * (float)cnt;
        rec[2] = t;
      }
    }
  }
}

template <int MODE, typename T, int BM, int BN, int WMW, int WNW, int FM, int FN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[FM][FN], char* smem, int m0, int n0,
                                              int tm) {
  BnPostRegs<T, BM, BN, 64 * WMW * WNW> none;
  RowMap rmap;
  rmap.M = a.M;
  rmap.phased = false;
  if (MODE == MODE_FWD && a.bias != nullptr)  // ssip_conv_fwd_bias on the register-staged kernel
    conv_epilogue_impl<MODE, T, BM, BN, WMW, WNW, FM, FN, true, true>(a, acc, smem, m0, n0, tm, none, false, rmap,
                                                                      (int)blockIdx.y);
  else
    conv_epilogue_impl<MODE, T, BM, BN, WMW, WNW, FM, FN>(a, acc, smem, m0, n0, tm, none, false, rmap,
                                                          (int)blockIdx.y);
}

template <int MODE, typename T, int BM, int BN, int WMW, int WNW, int FM, int FN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[FM][FN], char* smem, int m0, int n0,
                                              int tm, const BnPostRegs<T, BM, BN, 64 * WMW * WNW>& pre,
                                              const RowMap& rmap, int split) {
  conv_epilogue_impl<MODE, T, BM, BN, WMW, WNW, FM, FN>(a, acc, smem, m0, n0, tm, pre, true, rmap, split);
}

// ---------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------
template <int MODE, typename T, int BM, int BN, int WMW, int WNW, bool CONV1>
__global__ void __launch_bounds__(64 * WMW * WNW) conv_gemm_kernel(const ConvArgs a) {
  constexpr int NT = 64 * WMW * WNW;
  constexpr int BK = Traits<T>::BK;
  constexpr int KC = BK / 8;                 // 8-element chunks per k-tile row
  constexpr int NSUB = BK / 32;              // 32-deep MFMA sub-steps per k step
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr bool WG = (MODE == MODE_WGRAD);
  typedef Smem<MODE, T, BM, BN> SM;
  constexpr int ITA = WG ? (BK * BM / 8) / NT : (BM * KC) / NT;
  constexpr int ITB = WG ? (BK * BN / 8) / NT : (BN * KC) / NT;
  static_assert(ITA >= 1 && ITB >= 1 && FM >= 1 && FN >= 1, "tile too small");
  static_assert(!WG || ((BK * BM / 8) % NT == 0 && (BK * BN / 8) % NT == 0), "bad WGRAD tile");
  __shared__ __attribute__((aligned(16))) char smem[SM::BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WNW, wn = wave % WNW;

  const int tn = blockIdx.x % a.tiles_n;
  const int tm = blockIdx.x / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const T* __restrict__ Ag = static_cast<const T*>(a.A);
  const T* __restrict__ Bg = static_cast<const T*>(a.B);

  // ---------------- per-thread loader state ----------------
  // FWD/DGRAD: chunk id = tid + it*NT -> (row = id / KC, kc = id % KC); KC | NT so kc is fixed per thread
  // WGRAD A: [BK m][BM cols]: ml = id / (BM/8), col chunk = id % (BM/8) (fixed per thread)
  // WGRAD B: [BK m][BN cols]: ml = id / (BN/8), col chunk = id % (BN/8) (fixed per thread)
  int a_base[ITA], a_h[ITA], a_w[ITA];
  bool a_ok[ITA];
  int b_r = 0, b_s = 0, b_c = 0;
  bool b_colok = true;
  const int kc = tid % KC;

  // uniform k-step counters (FWD/DGRAD):  k = ((r*S)+s)*Cred + cb
  int kr = 0, ks_ = 0, kcb = 0;
  const int Cred = (MODE == MODE_FWD) ? a.C : a.K;

  long mstart = 0, mend = 0;
  if constexpr (!WG) {
#pragma unroll
    for (int it = 0; it < ITA; ++it) {
      const int row = (tid + it * NT) / KC;
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
    mstart = (long)blockIdx.y * a.ksteps * BK;
    mend = mstart + (long)a.ksteps * BK;
    if (mend > a.Mred) mend = a.Mred;
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
          // k = ks*BK + kc*8: filter row r = k / 32, pixel pair s = (k % 32) / 4, 4 channels each
          const int k = ks * BK + kc * 8;
          const int r = k >> 5;
          const int s0 = (k & 31) >> 2;
          const int hin = a_h[it] + r;
          const int w0 = a_w[it] + s0;
          const bool rowok = a_ok[it] && r < a.R && hin >= 0 && hin < a.H;
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
          ok = ok && ((hp | wp) & (a.stride - 1)) == 0;  // stride is a power of two (host-checked)
          p = hp >> (a.stride >> 1);
          q = wp >> (a.stride >> 1);
        }
        ok = ok && p < a.P && q < a.Q;
        const T* ptr = Ag + ((long)(a_base[it] + p * a.Q + q)) * a.K + kcb + kc * 8;
        load_v8<T>(ra[it], ptr, ok);
      }
    }
    if constexpr (!WG) {
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int row = (tid + it * NT) / KC;
        const int n = n0 + row;
        const int k = ks * BK + kc * 8;
        const bool ok = n < a.Ng && k < a.Kg;
        const T* p = Bg + (long)(ok ? n : 0) * a.Kg + (ok ? k : 0);
        load_v8<T>(rb[it], p, ok);
      }
    } else {
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        const int id = tid + it * NT;
        const int ml = id / (BM / 8), cch = id % (BM / 8);
        const long m = mstart + (long)ks * BK + ml;
        const int k = m0 + cch * 8;
        const bool ok = m < mend && k < a.K;
        const T* p = Ag + (ok ? m : 0) * (long)a.K + (ok ? k : 0);
        load_v8<T>(ra[it], p, ok);
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int id = tid + it * NT;
        const int ml = id / (BN / 8);
        const long m = mstart + (long)ks * BK + ml;
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
      kcb += BK;
      if (kcb >= Cred) {
        kcb = 0;
        if (++ks_ >= a.S) { ks_ = 0; ++kr; }
      }
    }
  };

  auto store_tiles = [&](int buf) {
    char* As = smem + buf * SM::STAGE;
    char* Bs = As + SM::A_BYTES;
    if constexpr (!WG) {
#pragma unroll
      for (int it = 0; it < ITA; ++it) store_kchunk(As, (tid + it * NT) / KC, kc, ra[it]);
#pragma unroll
      for (int it = 0; it < ITB; ++it) store_kchunk(Bs, (tid + it * NT) / KC, kc, rb[it]);
    } else {
#pragma unroll
      for (int it = 0; it < ITA; ++it) {
        const int id = tid + it * NT;
        store_mchunk<BM>(As, id / (BM / 8), (id % (BM / 8)) * 8, ra[it]);
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int id = tid + it * NT;
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
    nsteps = rem > 0 ? (int)((rem + BK - 1) / BK) : 0;
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
    const char* As = smem + cur * SM::STAGE;
    const char* Bs = As + SM::A_BYTES;
#pragma unroll
    for (int h = 0; h < NSUB; ++h) {
      Frag<T> fa[FM], fb[FN];
      if constexpr (!WG) {
#pragma unroll
        for (int i = 0; i < FM; ++i) read_kfrag(fa[i], As, wm * WTM + i * 16 + (lane & 15), lane >> 4, h);
#pragma unroll
        for (int j = 0; j < FN; ++j) read_kfrag(fb[j], Bs, wn * WTN + j * 16 + (lane & 15), lane >> 4, h);
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i) read_mfrag<BM>(fa[i], As, wm * WTM + i * 16, lane, h);
#pragma unroll
        for (int j = 0; j < FN; ++j) read_mfrag<BN>(fb[j], Bs, wn * WTN + j * 16, lane, h);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[i], fb[j]);
    }
    if (ks + 1 < nsteps) store_tiles(cur ^ 1);
    __syncthreads();
  }

  conv_epilogue<MODE, T, BM, BN, WMW, WNW>(a, acc, smem, m0, n0, tm);
}

// ---------------------------------------------------------------------------
// bf16 fast path: LDS-DMA (global_load_lds_dwordx4) 3-stage ring.
// Each wave-instruction moves 64 x 16 B = 1 KiB straight into LDS (no VGPR
// staging, no ds_write); the XOR swizzle is applied to the per-lane SOURCE
// chunk so the LDS image is the same one the register-staged kernel builds.
// Padded / out-of-range taps read a 16-byte zero block.  Prefetch distance
// 2: the loop waits with a counted vmcnt (one stage left in flight) and a
// raw s_barrier, never vmcnt(0) until the last step.
// ---------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) int g_zero16[4];


__device__ __forceinline__ void glds16(const void* src, char* lds_block) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_block, 16, 0, 0);
}

// Buffer-resource LDS-DMA: a raw buffer over the whole operand, per-lane
// 32-bit byte offsets.  An offset past the extent reads zeros (the padding /
// out-of-tile taps), so a gather step costs a mask test and one add per lane
// instead of 64-bit address arithmetic and a select against a zero page.
constexpr uint32_t SSIP_OOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, char* lds_block) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_block, 16, voff, 0, 0, 0);
}

// relu(fma(v, scale, shift)) over the 8 channels c0 .. c0 + 7 of one LDS
// chunk, in place -- bn_apply_kernel's arithmetic exactly, so a conv over the
// transformed tile equals the conv of the materialised BN+ReLU output
__device__ __forceinline__ bf16x8 bnrelu8(bf16x8 v, const float (&sc)[8], const float (&sh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = __builtin_fmaf((float)v[j], sc[j], sh[j]);
    t = t > 0.f ? t : 0.f;
    v[j] = (__bf16)t;
  }
  return v;
}
__device__ __forceinline__ void bnrelu_chunk(char* p, const float (&sc)[8], const float (&sh)[8]) {
  bf16x8 v = *reinterpret_cast<bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = __builtin_fmaf((float)v[j], sc[j], sh[j]);
    t = t > 0.f ? t : 0.f;
    v[j] = (__bf16)t;
  }
  *reinterpret_cast<bf16x8*>(p) = v;
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
// the same with every LDS read of this wave retired first: with the stagger a
// lagging wave's second-half fragments are read before the barrier but used
// after it, and nothing else keeps those reads ahead of the next refill of
// their ring slot, which other waves issue right after the barrier
template <int N>
__device__ __forceinline__ void wait_vm_lgkm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Waves per SIMD the LDS budget allows; asking the compiler for that many
// keeps the register count from costing a resident workgroup.
constexpr int glds_min_waves(int bm, int bn, int nw, int nstage, bool wg) {
  const int stage = wg ? 64 * (bm + bn) * 2 : (bm + bn) * 128;
  const int blocks = 163840 / (nstage * stage);
  const int w = blocks * nw / 4;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// C4: the stem conv on a pre-padded 4-channel image (pad 0, S padded to 8,
// even W): a 16-B chunk is a pixel pair (s, s+1) of one filter row, so a
// 64-deep k-step covers filter rows 2ks and 2ks+1; k >= R*S*4 reads zeros.
// POST: DGRAD with the BN-backward epilogue (ssip_conv_dgrad_bn); its
// operand registers are only allocated in that instantiation.
// (Round 3's timing ablations of this k-loop, its 5- and 8-phase ping-pong
// schedules and the persistent row-balanced halo kernel conv_hb -- all
// measured no faster in the step -- live on the r3-variants branch.)
// INBN: FWD / WGRAD over relu(bn(y)) of the layer below (ConvArgs::in_scale),
// the transform applied to each wave's own landed pieces before the k-step's
// barrier (2-stage ring; input channels <= GLDS_INBN_C).
constexpr int GLDS_INBN_C = 512;
template <int MODE, int BM, int BN, int WMW, int WNW, int NSTAGE, bool C4 = false, bool POST = false,
          bool FOLD = false, bool INBN = false>
__global__ void __launch_bounds__(64 * WMW * WNW, glds_min_waves(BM, BN, WMW * WNW, NSTAGE, MODE == 2))
    conv_glds_kernel(const ConvArgs a) {
  typedef __bf16 T;
  constexpr int NW = WMW * WNW, BK = 64;
  constexpr int WTM = BM / WMW, WTN = BN / WNW;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr bool WG = (MODE == MODE_WGRAD);
  constexpr int A_BYTES = WG ? BK * BM * 2 : BM * 128;
  constexpr int B_BYTES = WG ? BK * BN * 2 : BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  static_assert(NSTAGE == 2 || NSTAGE == 3, "2 or 3 LDS stages");
  constexpr int NBUF = NSTAGE;
  constexpr int IA = A_BYTES / 1024, IB = B_BYTES / 1024;
  constexpr int LA = IA / NW, LB = IB / NW;
  constexpr int L = LA + LB;
  static_assert(IA % NW == 0 && IB % NW == 0 && LA >= 1 && LB >= 1, "bad glds tile");
  static_assert(FM >= 1 && FN >= 1, "bad wave tile");
  constexpr int EPI = WG ? 0 : BM * (BN * 2 + 16);
  constexpr int SMEM = (NBUF * STAGE > EPI) ? NBUF * STAGE : EPI;
  static_assert(!INBN || (NSTAGE == 2 && !C4 && !POST && !FOLD && MODE != MODE_DGRAD), "INBN: FWD / WGRAD, 2 stages");
  __shared__ __attribute__((aligned(16))) char smem[SMEM + (INBN ? 2 * GLDS_INBN_C * 4 : 0)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  // XCD-aware order: the hardware deals workgroups round-robin to the 8 XCDs
  // (each with its own L2); remap so every XCD owns a contiguous run of
  // tiles (same split/phase, neighbouring M-tiles sharing im2col rows and the
  // whole weight panel) instead of every 8th tile.
  int bx, by;
  bool ds = false;  // FWD: a fused downsample tile (ConvArgs::fwd_tiles1)
  {
    const int nb = gridDim.x * gridDim.y;
    const int lin = blockIdx.x + blockIdx.y * gridDim.x;
    const int xcd = lin & 7, q = nb >> 3, r = nb & 7;
    const int t = a.xcd_remap ? xcd * q + min(xcd, r) + (lin >> 3) : lin;
    if (MODE == MODE_DGRAD && a.phased) {  // gridDim.y == 4: all phases of a tile together, heaviest first
      bx = t >> 2;
      by = (a.phase_order >> (2 * (t & 3))) & 3;
    } else {
      bx = t % gridDim.x;
      by = t / gridDim.x;
    }
    if (MODE == MODE_FWD && a.fwd_tiles1 > 0) {
      // fused downsample: the conv's tiles first in dispatch order, then the
      // short downsample tiles (they fill the last round), each group remapped
      // XCD-contiguously on its own
      ds = lin >= a.fwd_tiles1;
      const int base = ds ? a.fwd_tiles1 : 0, cnt = ds ? nb - a.fwd_tiles1 : a.fwd_tiles1;
      const int l = lin - base, x8 = l & 7, q8 = cnt >> 3, r8 = cnt & 7;
      bx = a.xcd_remap ? x8 * q8 + min(x8, r8) + (l >> 3) : l;
      by = 0;
    }
  }
  const int tn = bx % a.tiles_n;
  const int tm = bx / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const T* __restrict__ Ag = static_cast<const T*>(a.A);
  const T* __restrict__ Bg = static_cast<const T*>(a.B);
  // stride-2 DGRAD phase (uniform per workgroup); surplus M-tiles of the
  // shorter phases leave before touching memory or a barrier
  // (field-wise constant-index selects: a dynamic index into the kernel
  // argument struct, or a pointer into a copy, lands it in scratch)
  const bool phased = (MODE == MODE_DGRAD) && a.phased;
  const int f = phased ? by : 0;
#define SSIP_PSEL(fld) \
  (f == 0 ? a.phase[0].fld : f == 1 ? a.phase[1].fld : f == 2 ? a.phase[2].fld : a.phase[3].fld)
  RowMap rmap;
  rmap.phased = phased;
  rmap.H = a.H;
  rmap.W = a.W;
  int ph_nr = a.R, ph_ns = a.S, ph_r0 = 0, ph_s0 = 0, ph_bh = 0, ph_bw = 0,
      ph_ksteps = (MODE == MODE_FWD && ds) ? a.C / 64 : a.ksteps;
  if (phased) {
    if (tm >= SSIP_PSEL(tiles_m)) return;
    // a phase no tap reaches (1x1 stride-2 dgrad: 3 of 4) adds nothing: with
    // the residual gradient accumulated in place there is nothing to write
    if (!POST && SSIP_PSEL(ksteps) == 0 && a.add == a.out) return;
    rmap.M = SSIP_PSEL(M);
    rmap.ph = SSIP_PSEL(ph);
    rmap.pw = SSIP_PSEL(pw);
    rmap.Wph = SSIP_PSEL(Wph);
    rmap.div_hw.d = SSIP_PSEL(div_hw.d);
    rmap.div_hw.mul = SSIP_PSEL(div_hw.mul);
    rmap.div_hw.shr = SSIP_PSEL(div_hw.shr);
    rmap.div_w.d = SSIP_PSEL(div_w.d);
    rmap.div_w.mul = SSIP_PSEL(div_w.mul);
    rmap.div_w.shr = SSIP_PSEL(div_w.shr);
    ph_nr = SSIP_PSEL(nr);
    ph_ns = SSIP_PSEL(ns);
    ph_r0 = SSIP_PSEL(r0);
    ph_s0 = SSIP_PSEL(s0);
    ph_bh = SSIP_PSEL(bh);
    ph_bw = SSIP_PSEL(bw);
    ph_ksteps = SSIP_PSEL(ksteps);
  } else {
    rmap.M = a.M;
  }
#undef SSIP_PSEL
  const int Mrows = rmap.M;

  // ---------------- per-lane source state ----------------
  // FWD/DGRAD: instruction j = wave + NW*t covers k-tile rows 8j..8j+7;
  //   lane -> row 8j + lane/8, LDS slot lane%8 holds logical chunk (lane%8) ^ ((row>>1)&7)
  // WGRAD: rows of CPR = cols/8 chunks; instruction j covers 64/CPR rows.
  int a_base[LA], a_h[LA], a_w[LA], a_c[LA];
  bool a_ok[LA];
  const T* b_ptr[LB];
  int b_r[LB], b_s[LB], b_c[LB], b_row[LB];
  bool b_ok[LB];
  int kr = 0, ks_ = 0, kcb = 0;
  if (MODE == MODE_FWD && ds) { kr = 1; ks_ = 1; }  // the downsample's pixel is the conv's tap (1, 1)
  const int Cred = (MODE == MODE_FWD) ? a.C : a.K;
  long mstart = 0, mend = 0;

  if constexpr (!WG) {
#pragma unroll
    for (int t = 0; t < LA; ++t) {
      const int row = 8 * (wave + NW * t) + (lane >> 3);
      a_c[t] = (lane & 7) ^ ((row >> 1) & 7);
      const int m = m0 + row;
      a_ok[t] = m < Mrows;
      const int mm = a_ok[t] ? m : 0;
      if constexpr (MODE == MODE_FWD) {
        const int n = fdiv(mm, a.div_pq);
        const int rem = mm - n * a.P * a.Q;
        const int p = fdiv(rem, a.div_q);
        const int q = rem - p * a.Q;
        a_base[t] = n * a.H * a.W;
        a_h[t] = p * a.stride - a.pad;
        a_w[t] = q * a.stride - a.pad;
      } else if (phased) {
        const int n = fdiv(mm, rmap.div_hw);
        const int rem = mm - n * (int)rmap.div_hw.d;
        const int i = fdiv(rem, rmap.div_w);
        const int j = rem - i * rmap.Wph;
        a_base[t] = n * a.P * a.Q;
        a_h[t] = i + ph_bh;  // dy row for tap ri: a_h - ri
        a_w[t] = j + ph_bw;
      } else {
        const int n = fdiv(mm, a.div_hw);
        const int rem = mm - n * a.H * a.W;
        const int h = fdiv(rem, a.div_w);
        const int w = rem - h * a.W;
        a_base[t] = n * a.P * a.Q;
        a_h[t] = h + a.pad;
        a_w[t] = w + a.pad;
      }
    }
#pragma unroll
    for (int t = 0; t < LB; ++t) {
      const int row = 8 * (wave + NW * t) + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int n = n0 + row;
      b_ok[t] = n < a.Ng;
      b_c[t] = c;
      b_ptr[t] = Bg + (long)(b_ok[t] ? n : 0) * a.Kg + c * 8;
    }
  } else {
    mstart = (long)by * a.ksteps * BK;
    mend = mstart + (long)a.ksteps * BK;
    if (mend > a.Mred) mend = a.Mred;
    constexpr int CPA = BM / 8, RPA = 64 / CPA;
    constexpr int CPB = BN / 8, RPB = 64 / CPB;
#pragma unroll
    for (int t = 0; t < LA; ++t) {
      const int row = RPA * (wave + NW * t) + lane / CPA;
      const int lc = (lane % CPA) ^ (MTile<T, BM>::swz(row) >> 1);
      a_h[t] = row;                       // m-row within the k-step
      a_c[t] = m0 + lc * 8;               // output-channel column
      a_ok[t] = a_c[t] < a.K;
    }
#pragma unroll
    for (int t = 0; t < LB; ++t) {
      const int row = RPB * (wave + NW * t) + lane / CPB;
      const int lc = (lane % CPB) ^ (MTile<T, BN>::swz(row) >> 1);
      const int col = n0 + lc * 8;
      b_row[t] = row;
      b_ok[t] = col < a.Ng;
      const int cc = b_ok[t] ? col : 0;
      const int rs = cc / a.C;
      b_c[t] = cc - rs * a.C;
      b_r[t] = rs / a.S;
      b_s[t] = rs - b_r[t] * a.S;
    }
  }

  // buffer-resource state (FWD except the stem, DGRAD stride 1 / phase-split,
  // WGRAD's dY operand): byte offset of the lane's chunk at tap 0 and the
  // taps (bit r*S + s) whose source pixel lies inside the image.
  constexpr bool BUF_A = !C4;
  uint32_t a_off[LA], a_msk[LA], b_off[LB];
  __amdgpu_buffer_rsrc_t rsA = make_rsrc(Ag, a.a_bytes),
                         rsB = (MODE == MODE_FWD && ds) ? make_rsrc(a.Bds, a.bds_bytes) : make_rsrc(Bg, a.b_bytes);
  const int b_stride = (MODE == MODE_FWD && ds) ? a.C : a.Kg;  // B row length (W_ds: [K][C])
  const bool dsx = (MODE == MODE_DGRAD) && phased && f == 0 && a.A2 != nullptr;
  if constexpr (!WG && BUF_A) {
    const int nr = phased ? ph_nr : a.R, ns = phased ? ph_ns : a.S;
#pragma unroll
    for (int t = 0; t < LA; ++t) {
      // valid taps: rows [lr, hr) x columns [ls, hs) of the (nr x ns) filter
      int lr, hr, ls, hs;
      long pix;
      if constexpr (MODE == MODE_FWD) {  // input pixel (a_h + r, a_w + s)
        lr = max(0, -a_h[t]); hr = min(nr, a.H - a_h[t]);
        ls = max(0, -a_w[t]); hs = min(ns, a.W - a_w[t]);
        pix = (long)a_base[t] + (long)a_h[t] * a.W + a_w[t];
        a_off[t] = (uint32_t)((pix * a.C + a_c[t] * 8) * 2);
      } else {  // dY pixel (a_h - r, a_w - s)
        lr = max(0, a_h[t] - a.P + 1); hr = min(nr, a_h[t] + 1);
        ls = max(0, a_w[t] - a.Q + 1); hs = min(ns, a_w[t] + 1);
        pix = (long)a_base[t] + (long)a_h[t] * a.Q + a_w[t];
        a_off[t] = (uint32_t)((pix * a.K + a_c[t] * 8) * 2);
      }
      const uint32_t cbits = hs > ls ? ((1u << hs) - 1u) & ~((1u << ls) - 1u) : 0u;
      uint32_t msk = 0;
      for (int r = 0; r < nr; ++r) msk |= (r >= lr && r < hr) ? cbits << (r * ns) : 0u;
      a_msk[t] = a_ok[t] ? msk : 0u;
    }
#pragma unroll
    for (int t = 0; t < LB; ++t) {
      const int row = 8 * (wave + NW * t) + (lane >> 3);
      b_off[t] = b_ok[t] ? (uint32_t)(((long)(n0 + row) * b_stride + b_c[t] * 8) * 2) : 0xF0000000u;
    }
  } else if constexpr (WG) {
#pragma unroll
    for (int t = 0; t < LA; ++t) a_off[t] = (uint32_t)(((mstart + a_h[t]) * a.K + a_c[t]) * 2);
  }
  // WGRAD x gather: per slot the output pixel (p, q) of its row, the byte
  // offset of its tap's input pixel (+ channel chunk), and the p / q ranges
  // for which that tap lies inside the image (fixed: the slot's tap is fixed)
  int w_p[LB], w_q[LB], w_plo[LB], w_pn[LB], w_qlo[LB], w_qn[LB];
  uint32_t w_pix[LB];
  if constexpr (WG) {
#pragma unroll
    for (int t = 0; t < LB; ++t) {
      const int m = (int)min(mstart + b_row[t], (long)a.Mred - 1);
      const int n = fdiv(m, a.div_pq);
      const int rem = m - n * a.P * a.Q;
      const int pp = fdiv(rem, a.div_q);
      const int qq = rem - pp * a.Q;
      w_p[t] = pp;
      w_q[t] = qq;
      const int hin = pp * a.stride - a.pad + b_r[t], win = qq * a.stride - a.pad + b_s[t];
      w_pix[t] = (uint32_t)(((((long)n * a.H + hin) * a.W + win) * a.C + b_c[t]) * 2);
      // hin = p*stride - pad + r in [0, H)  <=>  p in [plo, plo + pn)
      const int r0 = a.pad - b_r[t], s0 = a.pad - b_s[t];
      const int plo = r0 > 0 ? (r0 + a.stride - 1) / a.stride : 0;
      const int phi = min(a.P, (a.H - 1 + r0) >= 0 ? (a.H - 1 + r0) / a.stride + 1 : 0);
      const int qlo = s0 > 0 ? (s0 + a.stride - 1) / a.stride : 0;
      const int qhi = min(a.Q, (a.W - 1 + s0) >= 0 ? (a.W - 1 + s0) / a.stride + 1 : 0);
      w_plo[t] = plo;
      w_pn[t] = b_ok[t] ? max(0, phi - plo) : 0;
      w_qlo[t] = qlo;
      w_qn[t] = max(0, qhi - qlo);
    }
  }

  // INBN: per ring stage, which of this wave's pieces read real input (bit t;
  // padding taps, rows past the grid and split tails stay zero) and, FWD, the
  // channel offset of the k-step
  uint32_t inb_v0 = 0, inb_v1 = 0;
  int inb_k0 = 0, inb_k1 = 0;
  auto issue = [&](int ks, int stage) {
    char* As = smem + stage * STAGE;
    char* Bs = As + A_BYTES;
    uint32_t inb_v = 0;
    if constexpr (MODE == MODE_FWD && C4) {
#pragma unroll
      for (int t = 0; t < LA; ++t) {
        const int k = ks * BK + a_c[t] * 8;
        const int hin = a_h[t] + 2 * ks + (a_c[t] >> 2), win = a_w[t] + 2 * (a_c[t] & 3);
        const bool ok = a_ok[t] && k < a.Kg && hin >= 0 && hin < a.H && win >= 0 && win + 1 < a.W;
        const T* src = ok ? Ag + ((long)(a_base[t] + hin * a.W + win)) * 4
                          : reinterpret_cast<const T*>(g_zero16);
        glds16(src, As + (wave + NW * t) * 1024);
      }
    } else if constexpr (MODE == MODE_FWD) {
      const int tp = kr * a.S + ks_;
      const uint32_t toff = (uint32_t)(((kr * a.W + ks_) * a.C + kcb) * 2);
#pragma unroll
      for (int t = 0; t < LA; ++t) {
        const bool ok = (a_msk[t] >> tp) & 1u;
        blds16(rsA, ok ? a_off[t] + toff : SSIP_OOB, As + (wave + NW * t) * 1024);
        if constexpr (INBN) inb_v |= (ok ? 1u : 0u) << t;
      }
      if constexpr (INBN) {
        if (stage == 0) { inb_v0 = inb_v; inb_k0 = kcb; } else { inb_v1 = inb_v; inb_k1 = kcb; }
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      if (dsx && ks == a.ds_from) {
        // switch to the fused downsample: its dY_ds pixel is this phase's tap-0
        // pixel (same a_off / mask bit 0), its weights are [C][K]
        rsA = make_rsrc(a.A2, a.a2_bytes);
        rsB = make_rsrc(a.B2, a.b2_bytes);
#pragma unroll
        for (int t = 0; t < LB; ++t) {
          const int row = 8 * (wave + NW * t) + (lane >> 3);
          b_off[t] = b_ok[t] ? (uint32_t)(((long)(n0 + row) * a.K + b_c[t] * 8) * 2) : 0xF0000000u;
        }
        kr = 0; ks_ = 0; kcb = 0; ph_r0 = 0; ph_s0 = 0; ph_ns = 1;
      }
      const int tp = kr * ph_ns + ks_;
      const uint32_t toff = (uint32_t)((kcb - (kr * a.Q + ks_) * a.K) * 2);
#pragma unroll
      for (int t = 0; t < LA; ++t) {
        const bool ok = (a_msk[t] >> tp) & 1u;
        blds16(rsA, ok ? a_off[t] + toff : SSIP_OOB, As + (wave + NW * t) * 1024);
      }
    }
    if constexpr (!WG) {
#pragma unroll
      for (int t = 0; t < LB; ++t) {
        int koff = ks * BK;
        if constexpr (MODE == MODE_DGRAD) {
          if (phased) koff = ((ph_r0 + 2 * kr) * a.S + ph_s0 + 2 * ks_) * a.K + kcb;
        }
        if constexpr (BUF_A) {
          blds16(rsB, b_off[t] + (uint32_t)(koff * 2), Bs + (wave + NW * t) * 1024);
        } else {
          bool ok = b_ok[t];
          if constexpr (C4) ok = ok && ks * BK + b_c[t] * 8 < a.Kg;
          const T* src = ok ? b_ptr[t] + koff : reinterpret_cast<const T*>(g_zero16);
          glds16(src, Bs + (wave + NW * t) * 1024);
        }
      }
    } else {
      const int mlim = (int)(mend - mstart) - ks * BK;  // rows of this k-step inside the split
      const uint32_t moff = (uint32_t)(ks * BK * a.K * 2);
#pragma unroll
      for (int t = 0; t < LA; ++t) {
        const bool ok = a_ok[t] && a_h[t] < mlim;
        blds16(rsA, ok ? a_off[t] + moff : SSIP_OOB, As + (wave + NW * t) * 1024);
      }
#pragma unroll
      for (int t = 0; t < LB; ++t) {
        const bool ok = b_row[t] < mlim && (uint32_t)(w_p[t] - w_plo[t]) < (uint32_t)w_pn[t] &&
                        (uint32_t)(w_q[t] - w_qlo[t]) < (uint32_t)w_qn[t];
        blds16(rsB, ok ? w_pix[t] : SSIP_OOB, Bs + (wave + NW * t) * 1024);
        if constexpr (INBN) inb_v |= (ok ? 1u : 0u) << t;
        // advance the slot's row by the 64 rows of a k-step
        int q = w_q[t] + a.wg_dq;
        const bool c1 = q >= a.Q;
        q = c1 ? q - a.Q : q;
        int pp = w_p[t] + a.wg_dp + (c1 ? 1 : 0);
        const bool c2 = pp >= a.P;
        pp = c2 ? pp - a.P : pp;
        w_q[t] = q;
        w_p[t] = pp;
        w_pix[t] += (uint32_t)(a.wg_k0 + (c1 ? a.wg_e1 : 0) + (c2 ? a.wg_e2 : 0));
      }
      if constexpr (INBN) {
        if (stage == 0) inb_v0 = inb_v; else inb_v1 = inb_v;
      }
    }
    if constexpr (!WG) {
      kcb += BK;
      if (kcb >= Cred) {
        kcb = 0;
        if (++ks_ >= ph_ns) { ks_ = 0; ++kr; }
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  int nsteps = ph_ksteps;
  if constexpr (WG) {
    const long rem = mend - mstart;
    nsteps = rem > 0 ? (int)((rem + BK - 1) / BK) : 0;
  }
  // NSTAGE-deep ring, NSTAGE-1 k-steps in flight.  Step ks: retire stage ks
  // with a counted vmcnt (the later in-flight steps stay outstanding across
  // the raw barrier), then refill the slot every wave finished reading in
  // step ks-1.
  // fused-BN epilogue operands: issued first, landed long before the epilogue
  BnPostRegs<T, BM, BN, 64 * WMW * WNW> post;
  if constexpr (MODE == MODE_DGRAD && POST) post.load(a, m0, n0);
  float* const inb_sc = reinterpret_cast<float*>(smem + SMEM);
  float* const inb_sh = inb_sc + GLDS_INBN_C;
  // INBN FWD z_out (1x1 / stride 1: a piece's byte offset at tap 0 + the
  // k-step's channel offset is its input offset, so z has A's layout); only
  // the n-tile-0 workgroups store (every n-tile reads the same pieces)
  const bool zst = INBN && MODE == MODE_FWD && a.zout != nullptr && tn == 0;
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(zst ? a.zout : nullptr, zst ? a.a_bytes : 0);
  if constexpr (INBN) {
    for (int c = tid; c < a.C; c += 64 * NW) {
      inb_sc[c] = a.in_scale[c];
      inb_sh[c] = a.in_shift[c];
    }
    __syncthreads();
  }
  // INBN: this wave's landed pieces of `stage` become relu(fma(y, scale, shift))
  // in place (bn_apply_kernel's arithmetic: fp32 fma, ReLU, one bf16 rounding),
  // so the k-step's fragment reads see the conv input itself
  auto inbn_xform = [&](int stage) {
    if constexpr (INBN) {
      const uint32_t vb = stage == 0 ? inb_v0 : inb_v1;
      char* const base = smem + stage * STAGE + (WG ? A_BYTES : 0);
      constexpr int LP = WG ? LB : LA;
#pragma unroll
      for (int t = 0; t < LP; ++t) {
        if ((vb >> t) & 1u) {
          int c0;
          if constexpr (WG) c0 = b_c[t];
          else c0 = (stage == 0 ? inb_k0 : inb_k1) + a_c[t] * 8;
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(inb_sc + c0);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(inb_sc + c0 + 4);
          const f32x4 h0 = *reinterpret_cast<const f32x4*>(inb_sh + c0);
          const f32x4 h1 = *reinterpret_cast<const f32x4*>(inb_sh + c0 + 4);
          const float sc8[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
          const float sh8[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
          bnrelu_chunk(base + (wave + NW * t) * 1024 + lane * 16, sc8, sh8);
          if constexpr (!WG) {
            if (zst) {
              typedef __attribute__((ext_vector_type(4))) unsigned int zv4u;
              const zv4u v = *reinterpret_cast<const zv4u*>(base + (wave + NW * t) * 1024 + lane * 16);
              __builtin_amdgcn_raw_buffer_store_b128(
                  v, rsZ, a_off[t] + (uint32_t)((stage == 0 ? inb_k0 : inb_k1) * 2), 0, 0);
            }
          }
        }
      }
    }
  };
  if (nsteps > 0) issue(0, 0);
  if (NSTAGE == 3 && nsteps > 1) issue(1, 1);
  int stage = 0;
  Frag<T> fa[2][FM], fb[2][FN];
  // Stagger (MI355X_MICROARCH "two waves per SIMD" item 9): waves w and
  // w + NW/2 share a SIMD and run this loop in lockstep -- both issue their
  // LDS-DMA pieces and fragment reads right after the barrier with the SIMD's
  // matrix pipe idle, then both multiply (round 3's ablation: the DMA and MFMA
  // phases add).  The second half of the workgroup runs each k-step's second
  // MFMA half after the next barrier instead, from fragments it already holds
  // in registers, so its matrix work fills the interval in which its partner
  // issues the ring refill and reads.  LDS is untouched by the deferred half;
  // the accumulation order h0(ks), h1(ks), h0(ks+1), ... is unchanged, so the
  // results are the same bits.
  const bool lag = a.stagger != 0 && wave >= NW / 2;
  for (int ks = 0; ks < nsteps; ++ks) {
    bool deferred = lag && ks > 0;
    if constexpr (INBN) {
      // own pieces landed -> transform them -> publish (LDS writes, barrier);
      // the lagging half's deferred MFMAs (registers only) go first, beside
      // the leading half's transform
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (deferred) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[1][i], fb[1][j]);
        deferred = false;
      }
      inbn_xform(stage);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (a.stagger) {
      if (NSTAGE == 3 && ks + 1 < nsteps) wait_vm_lgkm_barrier<L>(); else wait_vm_lgkm_barrier<0>();
    } else if (NSTAGE == 3 && ks + 1 < nsteps) {
      wait_vm_barrier<L>();
    } else {
      wait_vm_barrier<0>();
    }
    if (deferred) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[1][i], fb[1][j]);
    }
    const bool refill = ks + NSTAGE - 1 < nsteps;
    if (refill && !a.dma_mid) issue(ks + NSTAGE - 1, stage == 0 ? NSTAGE - 1 : stage - 1);
    const char* As = smem + stage * STAGE;
    const char* Bs = As + A_BYTES;
    // both k-halves' fragments are requested before the first MFMA, so the
    // second half's LDS reads overlap the first half's matrix work
    // (wave tiles of more than 8 fragments read one k-half at a time)
    constexpr bool BOTH = FM + FN <= 8;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!BOTH && h == 1) break;
      if constexpr (!WG) {
#pragma unroll
        for (int i = 0; i < FM; ++i) read_kfrag(fa[h][i], As, wm * WTM + i * 16 + (lane & 15), lane >> 4, h);
#pragma unroll
        for (int j = 0; j < FN; ++j) read_kfrag(fb[h][j], Bs, wn * WTN + j * 16 + (lane & 15), lane >> 4, h);
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i) read_mfrag<BM>(fa[h][i], As, wm * WTM + i * 16, lane, h);
#pragma unroll
        for (int j = 0; j < FN; ++j) read_mfrag<BN>(fb[h][j], Bs, wn * WTN + j * 16, lane, h);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (!BOTH && h == 1) {
        if constexpr (!WG) {
#pragma unroll
          for (int i = 0; i < FM; ++i) read_kfrag(fa[1][i], As, wm * WTM + i * 16 + (lane & 15), lane >> 4, 1);
#pragma unroll
          for (int j = 0; j < FN; ++j) read_kfrag(fb[1][j], Bs, wn * WTN + j * 16 + (lane & 15), lane >> 4, 1);
        } else {
#pragma unroll
          for (int i = 0; i < FM; ++i) read_mfrag<BM>(fa[1][i], As, wm * WTM + i * 16, lane, 1);
#pragma unroll
          for (int j = 0; j < FN; ++j) read_mfrag<BN>(fb[1][j], Bs, wn * WTN + j * 16, lane, 1);
        }
      }
      // (dma_mid: after every fragment read of the step, so no read follows
      // the DMA into the ring before the next step's barrier)
      if (h == 1 && refill && a.dma_mid) issue(ks + NSTAGE - 1, stage == 0 ? NSTAGE - 1 : stage - 1);
      if (h == 1 && lag) break;  // deferred past the next barrier
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[h][i], fb[h][j]);
    }
    stage = stage == NSTAGE - 1 ? 0 : stage + 1;
  }
  if (lag && nsteps > 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) mma(acc[i][j], fa[1][i], fb[1][j]);
  }
  __syncthreads();
  if constexpr (MODE == MODE_DGRAD && POST)
    conv_epilogue<MODE, T, BM, BN, WMW, WNW>(a, acc, smem, m0, n0, tm, post, rmap, by);
  else
    conv_epilogue_impl<MODE, T, BM, BN, WMW, WNW, FM, FN, false, FOLD>(
        a, acc, smem, m0, n0, tm, post, false, rmap, by, (MODE == MODE_FWD && ds) ? a.out_ds : nullptr,
        (MODE == MODE_FWD && ds) ? a.partial_ds : nullptr);
}

// WGRAD slab reduction:  dW[k][c][r][s] (torchvision KCRS, fp32) =
//   (accumulate ? dW : 0) + sum_split slab[split][k][(r*Sp + s)*Cp + c]
// A thread owns one 16-B vector (4 consecutive columns) in one of G split
// groups (G a power of two, chosen so the grid has ~1024 workgroups); a
// group sums its contiguous split range in order, then the G partials are
// combined in fixed order through LDS: bitwise reproducible.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int K,
                                                           int Ng, int C, int R, int S, int Cp, int Sp,
                                                           float* __restrict__ dw, int accumulate, int lg) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  __shared__ f4 red[256];
  const int G = 1 << lg, V = 256 >> lg;
  const int v = threadIdx.x & (V - 1), grp = threadIdx.x >> (8 - lg);
  const long total4 = (long)K * Ng / 4;
  const long idx4 = (long)blockIdx.x * V + v;
  const long sstride4 = total4;
  const int per = (splits + G - 1) / G;
  const int s0 = grp * per;
  const int s1 = min(splits, s0 + per);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  if (idx4 < total4) {
    const f4* p = reinterpret_cast<const f4*>(slab) + idx4;
    int sp = s0;
    for (; sp + 4 <= s1; sp += 4) {
      const f4 a0 = p[(long)sp * sstride4], a1 = p[(long)(sp + 1) * sstride4];
      const f4 a2 = p[(long)(sp + 2) * sstride4], a3 = p[(long)(sp + 3) * sstride4];
      acc += a0;
      acc += a1;
      acc += a2;
      acc += a3;
    }
    for (; sp < s1; ++sp) acc += p[(long)sp * sstride4];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (grp == 0 && idx4 < total4) {
    f4 t = red[v];
    for (int g = 1; g < G; ++g) t += red[g * V + v];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long idx = idx4 * 4 + e;
      const int col = (int)(idx % Ng);
      const int k = (int)(idx / Ng);
      const int c = col % Cp;
      const int rs = col / Cp;
      const int s = rs % Sp;
      const int r = rs / Sp;
      if (c < C && s < S) {
        const long o = (((long)k * C + c) * R + r) * S + s;
        dw[o] = accumulate ? dw[o] + t[e] : t[e];
      }
    }
  }
}

// The same reduction with coalesced KCRS stores, for few splits over many
// output rows (C % 64 == 0, no channel / tap padding): one workgroup per
// (k, 64-channel block) sums the block's R*S segments of 64 columns (16-B
// vectors, splits in order) into LDS as [c][rs] and writes dW[k][c0 ..
// c0+63][r][s] -- 64 R S contiguous floats -- as 16-B vectors.  (The kernel
// above stores 4-B values R*S floats apart, a partial line per lane.)
constexpr int WGR_T_MAXRS = 9;

__global__ void __launch_bounds__(256) wgrad_reduce_t_kernel(const float* __restrict__ slab, int splits, int K,
                                                             int Ng, int C, int RS, float* __restrict__ dw,
                                                             int accumulate) {
  typedef __attribute__((ext_vector_type(4))) float f4;
  __shared__ float tile[64 * WGR_T_MAXRS];
  const int cblocks = C >> 6;
  const int k = blockIdx.x / cblocks, c0 = (blockIdx.x - k * cblocks) << 6;
  const long sstride4 = (long)K * Ng / 4;
  for (int u = threadIdx.x; u < RS * 16; u += blockDim.x) {
    const int rs = u >> 4, cv = u & 15;
    const f4* p = reinterpret_cast<const f4*>(slab) + ((long)k * Ng + (long)rs * C + c0 + cv * 4) / 4;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    int sp = 0;
    for (; sp + 4 <= splits; sp += 4) {
      const f4 a0 = p[(long)sp * sstride4], a1 = p[(long)(sp + 1) * sstride4];
      const f4 a2 = p[(long)(sp + 2) * sstride4], a3 = p[(long)(sp + 3) * sstride4];
      acc += a0;
      acc += a1;
      acc += a2;
      acc += a3;
    }
    for (; sp < splits; ++sp) acc += p[(long)sp * sstride4];
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[(cv * 4 + e) * RS + rs] = acc[e];
  }
  __syncthreads();
  f4* o = reinterpret_cast<f4*>(dw + ((long)k * C + c0) * RS);
  for (int i = threadIdx.x; i < 16 * RS; i += blockDim.x) {
    f4 t = {tile[4 * i], tile[4 * i + 1], tile[4 * i + 2], tile[4 * i + 3]};
    if (accumulate) t += o[i];
    o[i] = t;
  }
}

// ---------------------------------------------------------------------------
// Halo-resident 3x3 / stride 1 / pad 1 convolution over 64 reduction
// channels: every forward conv of ResNet layer1 and every stride-1 DGRAD
// whose reduction is 64 channels (the same conv of dy with the taps flipped).
//
// The implicit-GEMM kernel above gathers the A operand once per tap (each
// input pixel crosses L2 -> LDS nine times) and pays a barrier per k-step.
// Here a persistent workgroup (one per CU) keeps the whole 64-column weight
// panel (9 taps x 64 x 64 bf16 = 72 KiB) resident in LDS and stages, per
// tile of TR whole output rows (TR*W <= 256 pixels of one image), the
// (TR+2) x (W+2) zero-haloed input rows once.  Tap (r, s) of output pixel
// (j, q) is LDS pixel (j + r)(W+2) + q + s, a uniform offset from tap (0, 0),
// so the nine taps are nine shifted fragment reads of one LDS image and the
// 18 MFMA k-steps of a tile run with no barrier.  The input rows are double
// buffered: tile u+1's rows are DMA'd while tile u computes, and tile u's
// epilogue stages its output through its own (then idle) buffer.  The wait
// for the next rows is a counted vmcnt that leaves the epilogue's stores in
// flight (vector-memory ops retire in issue order; the epilogue issues a
// fixed number of them per thread through buffer ops, rows past the tile
// going to an out-of-range offset).  LDS pixels use ktile_off's 16-B slot
// swizzle (conflict-free ds_read_b128 over 16 consecutive pixels).  Each
// MFMA k-step is one weight tap's 64 channels, in tap order, exactly as in
// conv_glds_kernel: the outputs are the same bits.
//
// FWD epilogue: bf16 y plus the BatchNorm statistics of the workgroup's
// tiles merged in fixed order (Chan) into one {count, sum, M2} record per
// (channel, workgroup): [Ncols][G][3].  DGRAD epilogue: dx (+ add, which may
// alias dx).
// ---------------------------------------------------------------------------
// BatchNorm statistics of a wave's output rows over the tiles of a
// persistent workgroup: per lane (one column, the rows (l >> 4) * 4 + e of
// each 16x16 fragment) a count and sums shifted by the lane's first value;
// wave_merge turns them into {n, mean, M2} per column and combines the four
// lane groups in fixed order (Chan).  Deterministic.
template <int FM, int FN>
struct WaveStats {
  float n, k[FN], s1[FN], s2[FN];
  __device__ __forceinline__ void reset() {
    n = 0.f;
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) k[jj] = s1[jj] = s2[jj] = 0.f;
  }
  __device__ __forceinline__ void tile(const f32x4 (&acc)[FM][FN], uint32_t vmask) {
    if (n == 0.f)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) k[jj] = acc[0][jj][0];
#pragma unroll
    for (int jj = 0; jj < FN; ++jj)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = ((vmask >> (i * 4 + e)) & 1) ? acc[i][jj][e] - k[jj] : 0.f;
          s1[jj] += d;
          s2[jj] = __builtin_fmaf(d, d, s2[jj]);
        }
    n += (float)__builtin_popcount(vmask);
  }
  // tile() one row group at a time (i = 0 first): the same sums in the same order
  __device__ __forceinline__ void rows(const f32x4 (&acc)[FM][FN], uint32_t vmask, int i) {
    if (i == 0) {
      if (n == 0.f)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) k[jj] = acc[0][jj][0];
      n += (float)__builtin_popcount(vmask);
    }
#pragma unroll
    for (int jj = 0; jj < FN; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = ((vmask >> (i * 4 + e)) & 1) ? acc[i][jj][e] - k[jj] : 0.f;
        s1[jj] += d;
        s2[jj] = __builtin_fmaf(d, d, s2[jj]);
      }
  }
  __device__ __forceinline__ void wave_merge(float& nw, float (&mean)[FN], float (&m2)[FN]) const {
    nw = n;
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      mean[jj] = n > 0.f ? k[jj] + s1[jj] / n : 0.f;
      m2[jj] = n > 0.f ? fmaxf(s2[jj] - s1[jj] * s1[jj] / n, 0.f) : 0.f;
    }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float nb = __shfl_xor(nw, off, 64);
      const float nn = nw + nb;
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const float mb = __shfl_xor(mean[jj], off, 64), qb = __shfl_xor(m2[jj], off, 64);
        // combine in a fixed order (lower lane group first) so every lane gets the same bits
        const bool lo = (threadIdx.x & off) == 0;
        const float na_ = lo ? nw : nb, ma = lo ? mean[jj] : mb, qa = lo ? m2[jj] : qb;
        const float nb_ = lo ? nb : nw, mb_ = lo ? mb : mean[jj], qb_ = lo ? qb : m2[jj];
        const float d = mb_ - ma;
        mean[jj] = nn > 0.f ? ma + d * (nb_ / nn) : 0.f;
        m2[jj] = nn > 0.f ? qa + qb_ + d * d * (na_ * nb_ / nn) : 0.f;
      }
      nw = nn;
    }
  }
};

struct HaloArgs {
  const __bf16* X;    // [N][H][W][64]   (FWD: x, DGRAD: dy)
  const __bf16* Wt;   // [Ncols][9][64]  (FWD: w_krsc, DGRAD: w_crsk)
  __bf16* out;        // [N][H][W][Ncols]
  const __bf16* add;  // DGRAD residual gradient / FWD residual (nullable, may alias out)
  float* partial;     // FWD BN records (nullable)
  const float* bias;  // FWD per-channel bias (folded eval BN), nullable
  int relu;           // FWD ReLU after bias and residual
  uint32_t x_bytes, w_bytes, o_bytes;
  int N, H, W, Ncols, TR, tiles, units, flip;
  // DGRAD BN-backward post-op (conv_halo_kernel<..., BNPOST>, ssip_conv_dgrad_bn):
  // out = (dgrad + add) * relu_mask, and per-(channel, workgroup, wave row)
  // sums {out, out * (y - mean) * invstd} into partial [Ncols][G][HALO_WMW][2].
  // Mask: bit c & 7 of pbits[pixel * Ncols / 8 + c / 8], or (pbits null)
  // fma(y, mscale, mshift) > 0.
  const __bf16* py;
  const uint8_t* pbits;
  const float *pmean, *pinvstd, *pmscale, *pmshift;
  uint32_t bits_bytes;
  // INBN (FWD): the input is y of the BN+ReLU below; x = relu(fma(y, in_scale,
  // in_shift)) is formed in LDS (ssip_conv_fwd_bnrelu_in)
  const float *in_scale, *in_shift;
  __bf16* zout;  // INBN (nullable): the transformed input's own tile rows written out (the wgrad's x)
  unsigned long long* stamps;  // STAMP instances only (SSIP_HALO_DIAG 128): per wave and tile 3 s_memtime stamps;
                               // with it, 1 = no output stores, 2 = no MFMAs (compile-time forms, results wrong)
  int diag;  // timing ablations only (SSIP_HALO_DIAG, results wrong): 4 no input-row DMA after the
             // first tile, 8 no BN statistics (round 5's 1 = no stores / 2 = no MFMAs: r5_halo_lab.txt);
             // 16 (results right): the next tile's rows issued before the MFMAs, not among them;
             // 32 (results right, INBN): the BN+ReLU transform after the k-loop, not inside it;
             // 64 (INBN, results wrong): no transform
};

constexpr int HALO_XBUF = 44 * 1024;
constexpr int HALO_WMW = 8;  // BN records per (channel, workgroup) of the halo / stem forwards (>= wave rows)

// X-row LDS image: pixel px's 128-B row, 16-B slot s at s ^ 2((px >> 1) & 3).
// Fragment reads start at any pixel (tap shifts); with this swizzle the 16
// lanes of every ds_read_b128 lane group ({0-3,12-15,20-27}, ...: rows
// r0..r0+15 across two k-slots) hit 16 distinct 16-B bank slots for every r0
// (ktile_off's swizzle is conflict-free only for r0 = 0 mod 16).
__device__ __forceinline__ int xtile_off(int px, int slot) { return px * 128 + ((slot ^ (((px >> 1) & 3) << 1)) << 4); }  // wave rows of every conv_halo_kernel instantiation (BN record count)

// LDS-only workgroup barrier: __syncthreads() would also drain vmcnt, i.e.
// wait for the next tile's rows in flight and this tile's output stores
__device__ __forceinline__ void halo_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }  // one input-row buffer: (TR + 2) * (W + 2) <= 352 pixels

// diagnostic phase stamp (conv_halo_kernel<..., STAMP>): one asm statement with
// its own lgkmcnt(0) (s_memtime returns out of order with LDS reads), fenced
__device__ __forceinline__ unsigned long long halo_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// conv_halo_kernel's DGRAD epilogue with the BN-backward reduction of the
// BN+ReLU below fused in (ssip_conv_dgrad_bn): per row-fragment i, the
// residual-gradient add, y and the mask bytes of the lane's 4 x FN elements
// are loaded together, then d = relu_mask ? bf16(bf16(acc) + add) : 0 is
// stored and summed (d, d * (y - mean) * invstd) into the lane's columns.
// Padded-grid rows (vmask clear) store nothing and add nothing.
template <int FM, int FN, int BATCH, bool YONLY>
__device__ __forceinline__ void halo_bnpost_epilogue(const HaloArgs& a, const f32x4 (&acc)[FM][FN],
                                                     __amdgpu_buffer_rsrc_t rsO, __amdgpu_buffer_rsrc_t rsA,
                                                     __amdgpu_buffer_rsrc_t rsY, __amdgpu_buffer_rsrc_t rsM, int tile,
                                                     int rows, int col0, const uint32_t (&rowoff)[FM][4],
                                                     uint32_t vmask, int cbase, float (&bsd)[FN], float (&bsx)[FN],
                                                     const short (*pre_y)[FN][4] = nullptr) {
  typedef __bf16 T;
  static_assert(FM % BATCH == 0, "row-group batches");
  const uint32_t obase = (uint32_t)(((long)tile * rows * a.Ncols + col0) * 2);
  float mu[FN], is[FN], msc[FN], msh[FN];
  const bool bits = !YONLY && a.pbits != nullptr;  // YONLY: no add, mask from the BN affine
  const bool has_add = !YONLY && a.add != nullptr;
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) {
    const int c = col0 + cbase + jj * 16;
    mu[jj] = a.pmean[c];
    is[jj] = a.pinvstd[c];
    msc[jj] = bits ? 0.f : a.pmscale[c];
    msh[jj] = bits ? 0.f : a.pmshift[c];
  }
  const int cbit = cbase & 7;  // column c's bit in its mask byte (jj * 16 keeps c & 7)
  // the operands of BATCH row groups per round trip (all FM in one where the
  // registers allow: each batch is a dependent HBM round trip per tile)
#pragma unroll
  for (int i0 = 0; i0 < FM; i0 += BATCH) {
    short ra[BATCH][FN][4], ry[BATCH][FN][4];
    uint32_t rm[BATCH][FN][4];
#pragma unroll
    for (int b = 0; b < BATCH; ++b)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = i0 + b;
          const uint32_t off = obase + rowoff[i][e] + jj * 32;
          const bool valid = (vmask >> (i * 4 + e)) & 1u;
          ry[b][jj][e] = pre_y ? pre_y[i][jj][e] : __builtin_amdgcn_raw_buffer_load_b16(rsY, off, 0, 0);
          ra[b][jj][e] = has_add ? __builtin_amdgcn_raw_buffer_load_b16(rsA, off, 0, 0) : (short)0;
          rm[b][jj][e] =
              bits ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsM, valid ? off >> 4 : SSIP_OOB, 0, 0) : 0u;
        }
#pragma unroll
    for (int b = 0; b < BATCH; ++b)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = i0 + b;
          const uint32_t off = obase + rowoff[i][e] + jj * 32;
          const bool valid = (vmask >> (i * 4 + e)) & 1u;
          const float yv = to_f32(__builtin_bit_cast(T, ry[b][jj][e]));
          float t = to_f32(from_f32<T>(acc[i][jj][e]));
          if (has_add) t += to_f32(__builtin_bit_cast(T, ra[b][jj][e]));
          const bool keep = bits ? ((rm[b][jj][e] >> cbit) & 1u) != 0u : __builtin_fmaf(yv, msc[jj], msh[jj]) > 0.f;
          const T o = from_f32<T>(keep ? t : 0.f);
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(short, o), rsO, off, 0, 0);
          const float dq = valid ? to_f32(o) : 0.f;
          bsd[jj] += dq;
          bsx[jj] += dq * ((yv - mu[jj]) * is[jj]);
        }
  }
}

// BNPOST: 0 = none; 1 = the BN-backward post-op with no residual add and the
// mask from the BN affine (y is the only extra operand: one load batch per
// tile); 2 = any other post-op operand set (one load batch per row group:
// the registers hold no more without spilling)
template <int WMW, int WNW, bool FOLD = false, int BNPOST = 0, bool ADD = false, bool INBN = false, int STAMP = 0>
__global__ void __launch_bounds__(64 * WMW * WNW, (WMW * WNW) / 4) conv_halo_kernel(const HaloArgs a) {
  typedef __bf16 T;
  constexpr int NW = WMW * WNW, NT = 64 * NW;
  constexpr int BM = 256, BN = 64;
  constexpr int WTM = BM / WMW, WTN = BN / WNW, FM = WTM / 16, FN = WTN / 16;
  constexpr int B_BYTES = 9 * BN * 128;
  static_assert(FM >= 1 && FN >= 1 && (NW == 4 || NW == 8 || NW == 16) && WMW <= HALO_WMW, "bad halo wave tile");
  static_assert(B_BYTES + 2 * HALO_XBUF <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[B_BYTES + 2 * HALO_XBUF];
  char* const Bs = smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int G = gridDim.x, g = blockIdx.x;
  const int u0 = (int)((long)g * a.units / G), u1 = (int)((long)(g + 1) * a.units / G);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(a.X, a.x_bytes), rsW = make_rsrc(a.Wt, a.w_bytes);
  const __amdgpu_buffer_rsrc_t rsO = make_rsrc(a.out, a.o_bytes), rsA = make_rsrc(a.add, a.o_bytes);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(a.zout, a.zout ? a.x_bytes : 0);
  typedef __attribute__((ext_vector_type(4))) unsigned int hv4u;
  const int Wp = a.W + 2;
  const int npx = (a.TR + 2) * Wp;
  const int nxi = (npx + 7) >> 3;  // X DMA wave-instructions per tile (8 pixels each)
  const int rows = a.TR * a.W;     // output pixels per tile
  const int mrows = a.TR * Wp;     // GEMM rows per tile: the padded grid (q = W, W+1 are discarded)

  // one 1-KiB LDS-DMA piece (8 pixels) of tile (n, p0)'s input rows
  auto issue_x_piece = [&](int n, int p0, int i, char* Xs) {
    const int px = i * 8 + (lane >> 3);
    const int sr = px / Wp, sc = px - sr * Wp;
    const int pin = p0 - 1 + sr, win = sc - 1;
    const int ch = (lane & 7) ^ (((px >> 1) & 3) << 1);  // xtile_off's swizzle
    const bool ok = px < npx && pin >= 0 && pin < a.H && win >= 0 && win < a.W;
    const uint32_t off = (uint32_t)(((((long)n * a.H + pin) * a.W + win) * 64 + ch * 8) * 2);
    blds16(rsX, ok ? off : SSIP_OOB, Xs + i * 1024);
  };
  auto issue_x = [&](int tile, char* Xs) {
    const int R0 = tile * a.TR;
    const int n = R0 / a.H, p0 = R0 - n * a.H;
    for (int i = wave; i < nxi; i += NW) issue_x_piece(n, p0, i, Xs);
  };
  constexpr int XPW = (HALO_XBUF / 1024 + NW - 1) / NW;  // most pieces per wave and tile
  // INBN: this wave's pieces of `tile` (landed: after its vmcnt(0)) become
  // relu(bn(y)) in place; halo and out-of-image pixels stay zero.  Every
  // wave transforms only what it DMA'd, so the next barrier publishes it.
  // A lane's LDS chunk is (lane & 7) ^ xtile swizzle of px = 8 i + lane / 8,
  // i.e. ((px >> 1) & 3) = (lane >> 4) & 3 for every piece i: the lane's
  // eight channels, and so its scale / shift, are fixed for the whole kernel
  // (loaded once here; per piece they were a dependent L2 round trip each)
  float isc[8], ish[8];
  if constexpr (INBN) {
    const int c0 = ((lane & 7) ^ (((lane >> 4) & 3) << 1)) * 8;
    load_f8(isc, a.in_scale + c0);
    load_f8(ish, a.in_shift + c0);
  }
  auto xform_x = [&](int tile, char* Xs, bool zst) {
    if (a.diag & 64) return;  // ablation: no transform (results wrong)
    const int R0 = tile * a.TR;
    const int n = R0 / a.H, p0 = R0 - n * a.H;
    for (int i = wave; i < nxi; i += NW) {
      const int px = i * 8 + (lane >> 3);
      const int sr = px / Wp, sc = px - sr * Wp;
      const int pin = p0 - 1 + sr, win = sc - 1;
      const bool ok = px < npx && pin >= 0 && pin < a.H && win >= 0 && win < a.W;
      if (ok) {
        char* const q = Xs + i * 1024 + lane * 16;
        bnrelu_chunk(q, isc, ish);
        if (zst && sr >= 1 && sr <= a.TR) {
          const int ch = (lane & 7) ^ (((px >> 1) & 3) << 1);
          const uint32_t off = (uint32_t)(((((long)n * a.H + pin) * a.W + win) * 64 + ch * 8) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hv4u, *reinterpret_cast<const bf16x8*>(q)),
                                                 rsZ, off, 0, 0);
        }
      }
    }
  };
  // INBN register staging of the next tile's pieces (XLAG + 1 slots)
  constexpr int XLAG = 2;
  bf16x8 xr[XLAG + 1];
  bool xok[XLAG + 1];
  uint32_t xzo[XLAG + 1];  // z_out offset of the piece (SSIP_OOB: halo row, padding or no z_out)
  auto xreg_load = [&](int n, int p0, int i, int slot, bool zst_tile) {
    const int px = i * 8 + (lane >> 3);
    const int sr = px / Wp, sc = px - sr * Wp;
    const int pin = p0 - 1 + sr, win = sc - 1;
    const int ch = (lane & 7) ^ (((px >> 1) & 3) << 1);  // xtile_off's swizzle
    const bool ok = px < npx && pin >= 0 && pin < a.H && win >= 0 && win < a.W;
    const uint32_t off = (uint32_t)(((((long)n * a.H + pin) * a.W + win) * 64 + ch * 8) * 2);
    xr[slot] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsX, ok ? off : SSIP_OOB, 0, 0));
    xok[slot] = ok;
    xzo[slot] = (ok && zst_tile && sr >= 1 && sr <= a.TR) ? off : SSIP_OOB;
  };
  auto xreg_store = [&](int i, int slot, char* Xs) {
    bf16x8 v = xr[slot];
    if (xok[slot]) v = bnrelu8(v, isc, ish);
    *reinterpret_cast<bf16x8*>(Xs + i * 1024 + lane * 16) = v;
    if (a.zout) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(hv4u, v), rsZ, xzo[slot], 0, 0);
  };
  auto issue_w = [&](int jn) {
    for (int i = wave; i < 72; i += NW) {
      const int tw = i >> 3, col = ((i & 7) << 3) + (lane >> 3);
      const int ch = (lane & 7) ^ ((col >> 1) & 7);
      const uint32_t off = (uint32_t)(((((long)jn * 64 + col) * 9 + tw) * 64 + ch * 8) * 2);
      blds16(rsW, off, Bs + i * 1024);
    }
  };

  // per-lane fragment bases: A rows (LDS pixel of tap (0, 0)), B columns
  int pxb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wm * WTM + i * 16 + (lane & 15);
    pxb[i] = m < mrows ? m : 0;  // row m of the padded grid reads LDS pixel m + tap offset
  }
  const int kq = lane >> 4;
  // A-fragment LDS offsets of the first 32-channel half, per row group and
  // k-step tap (DGRAD: flipped), fixed for all tiles: 9 FM registers.  The
  // second half is the same pixel at slot ^ 4, i.e. offset ^ 64 (xtile_off's
  // swizzle only XORs the slot, and the buffer bases are multiples of 128):
  // one v_xor per read instead of 9 FM more hoisted offsets.
  uint32_t offA[FM][9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int tt = a.flip ? 8 - t : t;
    const int toff = (tt / 3) * Wp + (tt % 3);
#pragma unroll
    for (int i = 0; i < FM; ++i) offA[i][t] = (uint32_t)xtile_off(pxb[i] + toff, kq);
  }
  int boff[FN][2];
#pragma unroll
  for (int jj = 0; jj < FN; ++jj)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) boff[jj][kh] = ktile_off(wn * WTN + jj * 16 + (lane & 15), 4 * kh + kq);

  // BN records [Ncols][G][WMW][3]: one per (channel, workgroup, wave row);
  // zero this workgroup's, then lanes < 16 of each wave keep the running
  // {n, mean, M2} of their FN columns over the wave's rows of every tile
  constexpr int RV = BNPOST ? 2 : 3;  // floats per record
  if (a.partial) {
    for (int c = tid; c < a.Ncols * HALO_WMW; c += NT) {
      float* rec = a.partial + ((long)(c / HALO_WMW) * G * HALO_WMW + (long)g * HALO_WMW + c % HALO_WMW) * RV;
#pragma unroll
      for (int v = 0; v < RV; ++v) rec[v] = 0.f;
    }
  }
  // BNPOST: this lane's running sums {d, d * xhat} of its FN columns
  float bsd[FN], bsx[FN];
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) bsd[jj] = bsx[jj] = 0.f;
  const __amdgpu_buffer_rsrc_t rsY = make_rsrc(a.py, BNPOST ? a.o_bytes : 0);
  const __amdgpu_buffer_rsrc_t rsM = make_rsrc(a.pbits, BNPOST ? a.bits_bytes : 0);
  WaveStats<FM, FN> ws;
  ws.reset();
  // this lane's output rows (rbase + 16 i + e): byte offset within a tile's
  // output block and validity (q < W of the padded grid), fixed for all tiles
  const int rbase = wm * WTM + kq * 4, cbase = wn * WTN + (lane & 15);
  uint32_t rowoff[FM][4];
  uint32_t vmask = 0;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = rbase + i * 16 + e;
      const int j = m / Wp, q = m - j * Wp;
      const bool v = m < mrows && q < a.W;
      rowoff[i][e] = v ? (uint32_t)(((j * a.W + q) * a.Ncols + cbase) * 2) : 0x80000000u;  // + jj*32 stays out of range
      vmask |= (v ? 1u : 0u) << (i * 4 + e);
    }
  int wrows = 0;  // valid rows of this wave in a tile (uniform)
  for (int r = wm * WTM; r < wm * WTM + WTM; ++r) wrows += (r < mrows && r % Wp < a.W) ? 1 : 0;

  if (u0 < u1) {
    const int jn = u0 / a.tiles;
    issue_w(jn);
    issue_x(u0 - jn * a.tiles, smem + B_BYTES);
  }
  const bool stats = a.partial && wrows > 0 && !(a.diag & 8);
  constexpr bool has_add = ADD;  // BNPOST == 0: out += add (BNPOST reads a.add itself)
  // The epilogue of one row group i of a finished tile: BN statistics over the
  // fp32 accumulators of its valid rows, then 16-bit stores straight from the
  // accumulators (lane: 4 rows x 1 column per fragment; padded-grid rows go to
  // an out-of-range offset), with the residual (ra, loaded beforehand) and the
  // folded eval BN bias / ReLU applied.  Round 5 measured the stores at 3 us
  // of a 78 us layer-1 forward and a transposed tile with 16-B row stores at
  // 93 us (profiles/r5_halo_lab.txt): the 32-B pieces do not bound the kernel.
  auto epi_rows = [&](const f32x4 (&ac)[FM][FN], int i, int etile, int ejn, const short (&ra)[FM][FN][4]) {
    if (stats) ws.rows(ac, vmask, i);
    const uint32_t obase = (uint32_t)(((long)etile * rows * a.Ncols + ejn * BN) * 2);
    const float lo = (FOLD && a.relu) ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      const float bcol = FOLD ? a.bias[ejn * BN + cbase + jj * 16] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t off = obase + rowoff[i][e] + jj * 32;
        float t = FOLD ? ac[i][jj][e] + bcol : ac[i][jj][e];
        if (has_add) t = to_f32(from_f32<T>(t)) + to_f32(__builtin_bit_cast(T, ra[i][jj][e]));
        const T o = from_f32<T>(FOLD ? fmaxf(t, lo) : t);
        if constexpr (!(STAMP & 4)) __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(short, o), rsO, off, 0, 0);
      }
    }
  };
  auto epi_load = [&](int etile, int ejn, short (&ra)[FM][FN][4]) {
    const uint32_t obase = (uint32_t)(((long)etile * rows * a.Ncols + ejn * BN) * 2);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          ra[i][jj][e] = __builtin_amdgcn_raw_buffer_load_b16(rsA, obase + rowoff[i][e] + jj * 32, 0, 0);
  };
  // panel / range end: the wave's BN sums -> records [c][g][wm]
  auto stats_flush = [&](int ejn) {
    float n, mean[FN], m2[FN];
    ws.wave_merge(n, mean, m2);
    if (lane < 16) {
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const int c = ejn * BN + cbase + jj * 16;
        float* rec = a.partial + ((long)c * G * HALO_WMW + (long)g * HALO_WMW + wm) * 3;
        rec[0] = n;
        rec[1] = mean[jj] * n;
        rec[2] = m2[jj];
      }
    }
    ws.reset();
  };

  // One barrier per tile: after it every wave has finished the previous
  // tile's fragment reads (so that buffer may take the next rows) and has
  // seen its own share of this tile's rows land (the vmcnt(0) each wave
  // issues after its MFMAs, by which time the prefetch has had the whole
  // MFMA phase).  The epilogue writes straight from the accumulators with
  // 16-bit buffer stores and needs no LDS, so a wave that finishes its MFMAs
  // early runs its epilogue while the other waves still compute, and its
  // stores stay in flight into the next tile.  (Round 5 deferred each tile's
  // epilogue into the next tile's MFMAs, one row group per 4 k-steps: the 32
  // accumulators it keeps push the kernel past 256 VGPRs into spills, 132 vs
  // 82 us; profiles/r5_halo_lab.txt.)
  short rap[FM][FN][4];
  bool first = true;
  for (int u = u0; u < u1; ++u) {
    const int jn = u / a.tiles, tile = u - jn * a.tiles;
    char* const Xs = smem + B_BYTES + ((u - u0) & 1) * HALO_XBUF;
    char* const Xn = smem + B_BYTES + ((u - u0 + 1) & 1) * HALO_XBUF;
    if (first) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (INBN) xform_x(tile, Xs, a.zout != nullptr && jn == 0);
    }
    first = false;
    halo_lds_barrier();
    unsigned long long st0 = 0, st1 = 0;
    if constexpr (STAMP) st0 = halo_stamp();
    const int un = u + 1;
    const bool more = un < u1;
    const int jn_next = more ? un / a.tiles : jn;
    const bool prefetch = more && jn_next == jn;
    // this tile's epilogue operands (the residual; BNPOST 1: y) are requested
    // now and land during the MFMAs: loaded after them, each tile paid a
    // dependent HBM round trip before its stores
    if constexpr (BNPOST == 0 && has_add) epi_load(tile, jn, rap);
    if constexpr (BNPOST == 1) {
      const uint32_t ob = (uint32_t)(((long)tile * rows * a.Ncols + jn * BN) * 2);  // the epilogue's obase
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rap[i][jj][e] = __builtin_amdgcn_raw_buffer_load_b16(rsY, ob + rowoff[i][e] + jj * 32, 0, 0);
    }
    // the next tile's rows go to tile u-1's buffer (every wave is past its
    // reads): one piece per wave after every other k-step's MFMAs, so the
    // DMA issue (~60-185 cycles a piece) runs beside the matrix pipe instead
    // of ahead of it with the partner wave's in the same place
    const bool spread = prefetch && !(a.diag & 4) && !(a.diag & 16);
    const int nR0 = (un - jn * a.tiles) * a.TR;
    const int nn = nR0 / a.H, np0 = nR0 - nn * a.H;
    if (prefetch && !(a.diag & 4) && (a.diag & 16)) issue_x(un - jn * a.tiles, Xn);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // 18 k-steps (weight tap t, 32-channel half kh) in weight-tap order, as
    // conv_glds_kernel; DGRAD's tap t reads dy at the flipped shift 8 - t.
    // Fragments are read one k-step ahead (register double buffer) so the
    // LDS latency hides behind the previous step's MFMAs.
    Frag<T> fa[2][FM], fb[2][FN];
    const uint32_t xbase = (uint32_t)(Xs - smem);
    uint32_t m64 = 64;  // opaque per tile: keeps offA ^ 64 from being hoisted into 9 FM more registers
    asm volatile("" : "+s"(m64));
    uint32_t xa[FM];
    auto load_step = [&](int st, Frag<T>(&ra)[FM], Frag<T>(&rb)[FN]) {
      const int t = st >> 1, kh = st & 1;
      const char* bt = Bs + t * (BN * 128);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        xa[i] = kh ? xa[i] ^ m64 : xbase + offA[i][t];
        ra[i].v = *reinterpret_cast<const bf16x8*>(smem + xa[i]);
      }
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) rb[jj].v = *reinterpret_cast<const bf16x8*>(bt + boff[jj][kh]);
    };
    load_step(0, fa[0], fb[0]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      if (st + 1 < 18) load_step(st + 1, fa[(st + 1) & 1], fb[(st + 1) & 1]);
      // step st + 1's fragment reads go out before step st's MFMAs: with the
      // k-loop one basic block the scheduler otherwise sinks each read to just
      // before its first use (lgkmcnt(0) ahead of most MFMAs)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
          if constexpr (!(STAMP & 2)) mma(acc[i][jj], fa[st & 1][i], fb[st & 1][jj]);
      if (st % 2 == 0 && st / 2 < XPW) {
        const int i = wave + (st / 2) * NW;
        if constexpr (INBN) {
          // INBN: the piece comes through registers -- a buffer load now, the
          // BN+ReLU and one LDS store XLAG pieces later (by then it has
          // landed) -- so the transform needs no LDS read-modify-write pass and
          // its VALU work sits between k-steps beside the partner wave's MFMAs
          // (issued unconditionally -- an unneeded piece reads the OOB zero --
          // so the compiler can count the loads in flight: vmcnt(XLAG) before
          // a store instead of vmcnt(0))
          xreg_load(nn, np0, i, (st / 2) % (XLAG + 1), a.zout != nullptr && jn == 0);
          if ((a.diag & 32) && spread && i < nxi) issue_x_piece(nn, np0, i, Xn);
        } else {
          if (spread && i < nxi) issue_x_piece(nn, np0, i, Xn);
        }
      }
      if constexpr (INBN) {
        if (st % 2 == 0 && st / 2 >= XLAG && st / 2 - XLAG < XPW) {
          const int k = st / 2 - XLAG, i = wave + k * NW;
          if (spread && !(a.diag & 32) && i < nxi) xreg_store(i, k % (XLAG + 1), Xn);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next tile's rows (issued before the MFMAs) and this wave's older
    // stores retire here; nothing younger is in flight
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (STAMP) st1 = halo_stamp();
    if constexpr (INBN) {
      // pieces staged too late for the k-loop's stores (XPW + XLAG > 9)
#pragma unroll
      for (int k = 9 - XLAG; k < XPW; ++k) {
        const int i = wave + k * NW;
        if (spread && !(a.diag & 32) && k >= 0 && i < nxi) xreg_store(i, k % (XLAG + 1), Xn);
      }
      // DMA'd pieces (diag 32, or the non-spread order) are transformed in place
      if (prefetch && !(a.diag & 4) && ((a.diag & 32) || !spread))
        xform_x(un - jn * a.tiles, Xn, a.zout != nullptr && jn == 0);
    }

    // ---- epilogue
    if constexpr (BNPOST) {
      halo_bnpost_epilogue<FM, FN, BNPOST == 1 ? FM : 1, BNPOST == 1>(
          a, acc, rsO, rsA, rsY, rsM, tile, rows, jn * BN, rowoff, vmask, cbase, bsd, bsx,
          BNPOST == 1 ? rap : nullptr);
      if (!prefetch) {
        // panel / range end: the wave's column sums -> records [c][g][wm]
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
#pragma unroll
          for (int off = 16; off <= 32; off <<= 1) {
            bsd[jj] += __shfl_xor(bsd[jj], off, 64);
            bsx[jj] += __shfl_xor(bsx[jj], off, 64);
          }
        if (lane < 16) {
#pragma unroll
          for (int jj = 0; jj < FN; ++jj) {
            const int c = jn * BN + cbase + jj * 16;
            float* rec = a.partial + ((long)c * G * HALO_WMW + (long)g * HALO_WMW + wm) * 2;
            rec[0] = bsd[jj];
            rec[1] = bsx[jj];
          }
        }
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) bsd[jj] = bsx[jj] = 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i) epi_rows(acc, i, tile, jn, rap);
      if (stats && !prefetch) stats_flush(jn);
    }
    if constexpr (STAMP) {
      const unsigned long long st2 = halo_stamp();
      if (lane == 0 && u - u0 < 32) {
        unsigned long long* sp = a.stamps + (((long)g * NW + wave) * 32 + (u - u0)) * 3;
        sp[0] = st0;
        sp[1] = st1;
        sp[2] = st2;
      }
    }
    if (more && !prefetch) {
      // panel change: new weights and the next tile's rows, loaded once every
      // wave is past this tile's MFMAs
      halo_lds_barrier();
      issue_w(jn_next);
      issue_x(un - jn_next * a.tiles, Xn);
      first = true;
    }
  }
}

// ---------------------------------------------------------------------------
// The stem conv (7x7 / stride 2 over the pre-padded 4-channel image, pad 0,
// S padded to 8) in the same persistent, LDS-resident form.  A tile is
// STEM_TR = 2 output rows; their 9 input rows (2 p0 .. 2 p0 + 8) are one
// contiguous run of the NHWC4 image, DMA'd linearly into a double buffer.
// Output pixel (j, q), filter row r reads the 8 pixels 2q .. 2q+7 of input
// row 2j + r: 64 contiguous bytes = one 32-deep MFMA k-step (s = 7 carries a
// zero weight), so a tile is 7 k-steps with no barrier.  GEMM rows are the
// output rows padded to STEM_QP = 128 (q >= Q discarded).  The weight panel
// (64 filters x 7 rows x 32) stays resident.  Epilogue as conv_halo_kernel:
// 16-bit stores from the accumulators, per-wave BN records [K][G][4][3].
// The k-order differs from conv_glds_kernel's C4 path (which pairs two filter
// rows per 64-deep step), so outputs agree to fp32 rounding, not bitwise.
// ---------------------------------------------------------------------------
struct StemArgs {
  const __bf16* X;    // [N][H][W][4]   pre-padded image
  const __bf16* Wt;   // [Ncols][7][8][4]
  __bf16* out;        // [N][P][Q][Ncols]
  float* partial;     // BN records (nullable)
  uint32_t x_bytes, w_bytes, o_bytes;
  int N, H, W, P, Q, Ncols, tiles, units;
  int diag;  // timing ablations only (SSIP_STEM_DIAG, results wrong): 1 no output stores, 8 no BN statistics
};

constexpr int STEM_QP = 128, STEM_TR = 2, STEM_XROWS = 2 * STEM_TR + 5;
constexpr int STEM_XBUF = 17 * 1024;  // 9 rows x W x 8 B, W <= 240

template <int WMW, int WNW>
__global__ void __launch_bounds__(64 * WMW * WNW, (WMW * WNW) / 2) conv_stem_halo_kernel(const StemArgs a) {
  typedef __bf16 T;
  constexpr int NW = WMW * WNW, NT = 64 * NW;
  constexpr int BM = STEM_TR * STEM_QP, BN = 64;
  constexpr int WTM = BM / WMW, WTN = BN / WNW, FM = WTM / 16, FN = WTN / 16;
  constexpr int B_BYTES = 7 * BN * 64;  // [r][col][32 k], 16-B slot s at s ^ 2((col >> 3) & 1)
  static_assert(FM >= 1 && FN >= 1, "bad stem wave tile");
  __shared__ __attribute__((aligned(16))) char smem[B_BYTES + 2 * STEM_XBUF];
  char* const Bs = smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;
  const int G = gridDim.x, g = blockIdx.x;
  const int u0 = (int)((long)g * a.units / G), u1 = (int)((long)(g + 1) * a.units / G);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(a.X, a.x_bytes), rsW = make_rsrc(a.Wt, a.w_bytes);
  const __amdgpu_buffer_rsrc_t rsO = make_rsrc(a.out, a.o_bytes);
  const int xpitch = a.W * 8;                  // one input row (4 channels bf16)
  const int xrun = STEM_XROWS * xpitch;        // bytes of a tile's input rows
  const int nxi = (xrun + 1023) >> 10;         // 1-KiB DMA wave-instructions

  auto issue_x = [&](int tile, char* Xs) {
    const int R0 = tile * STEM_TR;
    const int n = R0 / a.P, p0 = R0 - n * a.P;
    const uint32_t base = (uint32_t)((((long)n * a.H + 2 * p0) * a.W) * 8);
    for (int i = wave; i < nxi; i += NW) {
      const int b = i * 1024 + lane * 16;
      blds16(rsX, b < xrun ? base + (uint32_t)b : SSIP_OOB, Xs + i * 1024);
    }
  };
  auto issue_w = [&](int jn) {
    // 7 x 64 x 64 B = 28 KiB: instruction i covers rows r = i / 4, cols 16 (i % 4) .. +16
    for (int i = wave; i < 28; i += NW) {
      const int r = i >> 2, col = ((i & 3) << 4) + (lane >> 2);
      const int sl = (lane & 3) ^ (((col >> 3) & 1) << 1);
      const uint32_t off = (uint32_t)(((((long)jn * 64 + col) * 7 + r) * 32 + sl * 8) * 2);
      blds16(rsW, off, Bs + i * 1024);
    }
  };

  const int kq = lane >> 4;
  const int rbase = wm * WTM + kq * 4, cbase = wn * WTN + (lane & 15);
  // A fragment bases: GEMM row m = j * QP + q reads input row 2j + r, pixel 2q + 2kq
  int abase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wm * WTM + i * 16 + (lane & 15);
    const int j = m / STEM_QP, q = m - j * STEM_QP;
    abase[i] = q < a.Q ? 2 * j * xpitch + (2 * q + 2 * kq) * 8 : 0;
  }
  int boff[FN];
#pragma unroll
  for (int jj = 0; jj < FN; ++jj) {
    const int col = wn * WTN + jj * 16 + (lane & 15);
    boff[jj] = col * 64 + ((kq ^ (((col >> 3) & 1) << 1)) << 4);
  }
  uint32_t rowoff[FM][4];
  uint32_t vmask = 0;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = rbase + i * 16 + e;
      const int j = m / STEM_QP, q = m - j * STEM_QP;
      const bool v = q < a.Q;
      rowoff[i][e] = v ? (uint32_t)(((j * a.Q + q) * a.Ncols + cbase) * 2) : 0x80000000u;
      vmask |= (v ? 1u : 0u) << (i * 4 + e);
    }
  int wrows = 0;
  for (int r = wm * WTM; r < wm * WTM + WTM; ++r) wrows += (r % STEM_QP < a.Q) ? 1 : 0;

  if (a.partial) {
    for (int c = tid; c < a.Ncols * HALO_WMW; c += NT) {
      float* rec = a.partial + ((long)(c / HALO_WMW) * G * HALO_WMW + (long)g * HALO_WMW + c % HALO_WMW) * 3;
      rec[0] = 0.f;
      rec[1] = 0.f;
      rec[2] = 0.f;
    }
  }
  WaveStats<FM, FN> ws;
  ws.reset();

  if (u0 < u1) {
    const int jn = u0 / a.tiles;
    issue_w(jn);
    issue_x(u0 - jn * a.tiles, smem + B_BYTES);
  }
  bool first = true;
  for (int u = u0; u < u1; ++u) {
    const int jn = u / a.tiles, tile = u - jn * a.tiles;
    char* const Xs = smem + B_BYTES + ((u - u0) & 1) * STEM_XBUF;
    char* const Xn = smem + B_BYTES + ((u - u0 + 1) & 1) * STEM_XBUF;
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    first = false;
    halo_lds_barrier();
    const int un = u + 1;
    const bool more = un < u1;
    const int jn_next = more ? un / a.tiles : jn;
    const bool prefetch = more && jn_next == jn;
    if (prefetch) issue_x(un - jn * a.tiles, Xn);

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    Frag<T> fa[2][FM], fb[2][FN];
    auto load_step = [&](int r, Frag<T>(&ra)[FM], Frag<T>(&rb)[FN]) {
#pragma unroll
      for (int i = 0; i < FM; ++i) ra[i].v = *reinterpret_cast<const bf16x8*>(Xs + abase[i] + r * xpitch);
#pragma unroll
      for (int jj = 0; jj < FN; ++jj)
        rb[jj].v = *reinterpret_cast<const bf16x8*>(Bs + r * (BN * 64) + boff[jj]);
    };
    load_step(0, fa[0], fb[0]);
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      if (r + 1 < 7) load_step(r + 1, fa[(r + 1) & 1], fb[(r + 1) & 1]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) mma(acc[i][jj], fa[r & 1][i], fb[r & 1][jj]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    if (a.partial && wrows > 0 && !(a.diag & 8)) {
      // per-lane shifted sums over the fp32 accumulators of the valid rows;
      // merged across the wave (and written) when the panel or range ends
      ws.tile(acc, vmask);
      if (!prefetch) {
        float n, mean[FN], m2[FN];
        ws.wave_merge(n, mean, m2);
        if (lane < 16) {
#pragma unroll
          for (int jj = 0; jj < FN; ++jj) {
            const int c = jn * BN + cbase + jj * 16;
            float* rec = a.partial + ((long)c * G * HALO_WMW + (long)g * HALO_WMW + wm) * 3;
            rec[0] = n;
            rec[1] = mean[jj] * n;
            rec[2] = m2[jj];
          }
        }
        ws.reset();
      }
    }
    if (!(a.diag & 1)) {
      const uint32_t obase = (uint32_t)(((long)tile * STEM_TR * a.Q * a.Ncols + jn * BN) * 2);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(short, from_f32<T>(acc[i][jj][e])), rsO,
                                                  obase + rowoff[i][e] + jj * 32, 0, 0);
    }
    if (more && !prefetch) {
      halo_lds_barrier();
      issue_w(jn_next);
      issue_x(un - jn_next * a.tiles, Xn);
      first = true;
    }
  }
}

// ---------------------------------------------------------------------------
// WGRAD of the same 3x3 / stride 1 / pad 1 convs with C = K = 64 (layer1):
//   dW[k][(t, c)] = sum_m dy[m][k] * x_pad[m + toff(t)][c]
// over the padded-grid rows m = j (W+2) + q of each tile (dy is zero at
// q >= W).  A persistent workgroup (one per CU) stages per tile the input
// rows (as conv_halo_kernel, with the m-major MTile swizzle) and the tile's
// dy rows, both double-buffered, and keeps the whole 64 x 576 fp32 result in
// registers across its tiles (waves: 2 k-halves x 4 quarters of the 36
// (tap, 16-channel) column blocks); the nine taps are shifted transposed
// fragment reads of the one input image.  At the end each workgroup writes
// its partial dW as one fp32 slab; wgrad_reduce_kernel sums the slabs in
// fixed order (deterministic).
// ---------------------------------------------------------------------------
struct HaloWgArgs {
  const __bf16* X;   // [N][H][W][64]
  const __bf16* DY;  // [N][H][W][64]
  float* slab;       // [G][64][576]
  uint32_t x_bytes;
  int N, H, W, TR, tiles;
  int spread;        // the next tile's pieces among the k-steps' MFMAs (SSIP_HWG_SPREAD=0: ahead of them)
  // INBN: X is y of the BN+ReLU below; relu(fma(y, in_scale, in_shift)) is
  // formed in LDS (ssip_conv_wgrad_bnrelu_in)
  const float *in_scale, *in_shift;
};

constexpr int HWG_XBUF = 48 * 1024;  // 384 input-image rows x 128 B
constexpr int HWG_DBUF = 32 * 1024;  // 256 dy rows x 128 B

// transposed (m-major) fragment of a [rows][64] bf16 MTile image: lane l gets
// column col0 + (l & 15), rows row0 + 8 (l >> 4) .. +7
__device__ __forceinline__ void read_tfrag(Frag<__bf16>& f, const char* base, int row0, int col0, int lane) {
  typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = row0 + 8 * g + q;
  const char* a0 = base + MTile<__bf16, 64>::off(r0, col0 + 4 * p);
  const char* a1 = base + MTile<__bf16, 64>::off(r0 + 4, col0 + 4 * p);
  v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a0));
  v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a1));
  f.v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <bool INBN = false>
__global__ void __launch_bounds__(512, 2) conv_halo_wgrad_kernel(const HaloWgArgs a) {
  typedef __bf16 T;
  constexpr int NW = 8;
  // the two tile buffers as two objects: the tile loop runs unrolled by two,
  // so the compiler sees that this tile's fragment reads and the next tile's
  // LDS-DMA never alias (one array: a vmcnt(0) wait for the DMA ahead of every
  // read that followed it)
  __shared__ __attribute__((aligned(16))) char smem0[HWG_XBUF + HWG_DBUF];
  __shared__ __attribute__((aligned(16))) char smem1[HWG_XBUF + HWG_DBUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // k rows 32 wm .. +31; column blocks 9 wn .. 9 wn + 8
  const int G = gridDim.x, g = blockIdx.x;
  const int u0 = (int)((long)g * a.tiles / G), u1 = (int)((long)(g + 1) * a.tiles / G);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(a.X, a.x_bytes), rsD = make_rsrc(a.DY, a.x_bytes);
  const int Wp = a.W + 2;
  const int npx = (a.TR + 2) * Wp, mrows = a.TR * Wp;

  // LDS-DMA pieces of a tile: all 48 of the input image's (the k-loop reads
  // rows up to 255 + 2 Wp + 2: dy is zero at m >= mrows, but 0 x garbage in
  // an unfilled row is NaN), then all 32 of dy's
  constexpr int nxp = HWG_XBUF / 1024, npieces = nxp + HWG_DBUF / 1024;
  auto issue_piece = [&](int n, int p0, int i, char* Xs, char* Ds) {
    if (i < nxp) {  // input image: 8 rows per instruction
      const int px = i * 8 + (lane >> 3);
      const int sr = px / Wp, sc = px - sr * Wp;
      const int pin = p0 - 1 + sr, win = sc - 1;
      const int ch = (lane & 7) ^ mt64_chunk_xor(px);  // MTile<64>
      const bool ok = px < npx && pin >= 0 && pin < a.H && win >= 0 && win < a.W;
      const uint32_t off = (uint32_t)(((((long)n * a.H + pin) * a.W + win) * 64 + ch * 8) * 2);
      blds16(rsX, ok ? off : SSIP_OOB, Xs + i * 1024);
    } else {  // dy rows of the padded grid
      const int m = (i - nxp) * 8 + (lane >> 3);
      const int j = m / Wp, q = m - j * Wp;
      const int ch = (lane & 7) ^ mt64_chunk_xor(m);
      const bool ok = m < mrows && q < a.W;
      const uint32_t off = (uint32_t)(((((long)n * a.H + p0 + j) * a.W + q) * 64 + ch * 8) * 2);
      blds16(rsD, ok ? off : SSIP_OOB, Ds + (i - nxp) * 1024);
    }
  };
  auto issue = [&](int tile, char* Xs, char* Ds) {
    const int R0 = tile * a.TR;
    const int n = R0 / a.H, p0 = R0 - n * a.H;
    for (int i = wave; i < npieces; i += NW) issue_piece(n, p0, i, Xs, Ds);
  };
  // INBN: this wave's input-image pieces of `tile` (landed) become
  // relu(bn(y)) in place; padding and out-of-image pixels stay zero
  // (a lane's chunk, (lane & 7) ^ mt64_chunk_xor(8 i + lane / 8), depends on i
  // only through i & 1 = wave & 1: one scale / shift load per call, not per piece)
  auto xform_x = [&](int tile, char* Xs) {
    const int R0 = tile * a.TR;
    const int n = R0 / a.H, p0 = R0 - n * a.H;
    (void)n;
    float isc[8], ish[8];
    const int c0 = ((lane & 7) ^ mt64_chunk_xor(wave * 8 + (lane >> 3))) * 8;
    load_f8(isc, a.in_scale + c0);
    load_f8(ish, a.in_shift + c0);
    for (int i = wave; i < nxp; i += NW) {
      const int px = i * 8 + (lane >> 3);
      const int sr = px / Wp, sc = px - sr * Wp;
      const int pin = p0 - 1 + sr, win = sc - 1;
      const bool ok = px < npx && pin >= 0 && pin < a.H && win >= 0 && win < a.W;
      if (ok) bnrelu_chunk(Xs + i * 1024 + lane * 16, isc, ish);
    }
  };
  // This wave's pieces of every tile -- i = wave + 8 k: k < 6 input image, k >= 6
  // dy -- as tile-independent byte offsets from the tile's first pixel, with
  // the input piece's row (0 .. TR + 1) in bits 0-2 and bit 3 set where the
  // piece lane is always out of range; only the input rows above / below the
  // image depend on the tile.  The k-loop issues them two per k-step, beside
  // the MFMAs, without the division of issue_piece.
  static_assert(nxp == 6 * NW && npieces == 10 * NW, "piece map");
  int pc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    if (k < 6) {
      const int px = (wave + NW * k) * 8 + (lane >> 3);
      const int sr = px / Wp, sc = px - sr * Wp, win = sc - 1;
      const int ch = (lane & 7) ^ mt64_chunk_xor(px);
      const bool ok = px < npx && win >= 0 && win < a.W;
      pc[k] = ((((sr - 1) * a.W + win) * 64 + ch * 8) * 2) | (sr & 7) | (ok ? 0 : 8);
    } else {
      const int m = (wave + NW * (k - 6)) * 8 + (lane >> 3);
      const int j = m / Wp, q = m - j * Wp;
      const int ch = (lane & 7) ^ mt64_chunk_xor(m);
      const bool ok = m < mrows && q < a.W;
      pc[k] = (((j * a.W + q) * 64 + ch * 8) * 2) | (ok ? 0 : 8);
    }
  }
  auto issue_pc = [&](int k, int base, int p0, char* Xs, char* Ds) {
    const int v = pc[k];
    bool ok = (v & 8) == 0;
    if (k < 6) {
      const int pin = p0 - 1 + (v & 7);
      ok = ok && pin >= 0 && pin < a.H;
    }
    const uint32_t off = (uint32_t)(base + (v & ~15));
    if (k < 6)
      blds16(rsX, ok ? off : SSIP_OOB, Xs + (wave + NW * k) * 1024);
    else
      blds16(rsD, ok ? off : SSIP_OOB, Ds + (wave + NW * (k - 6)) * 1024);
  };

  f32x4 acc[2][9];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int b = 0; b < 9; ++b) acc[x][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // column block b of this wave: tap t = (9 wn + b) / 4, channels 16 ((9 wn + b) % 4) ..
  // Per-lane LDS byte offsets of the transposed fragment reads at k-step 0
  // (read_tfrag's rows r0 and r0 + 4): a k-step adds 32 rows = 4096 B and
  // leaves row bits 1 and 3 -- the swizzle's -- unchanged.
  int xo[9][2], dof[2][2];
  {
    const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3;
#pragma unroll
    for (int b = 0; b < 9; ++b) {
      const int nb = 9 * wn + b, t = nb >> 2;
      const int toff = (t / 3) * Wp + (t % 3), ccol = (nb & 3) * 16;
      xo[b][0] = MTile<__bf16, 64>::off(toff + 8 * tg + tq, ccol + 4 * tp);
      xo[b][1] = MTile<__bf16, 64>::off(toff + 8 * tg + tq + 4, ccol + 4 * tp);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      dof[x][0] = MTile<__bf16, 64>::off(8 * tg + tq, (2 * wm + x) * 16 + 4 * tp);
      dof[x][1] = MTile<__bf16, 64>::off(8 * tg + tq + 4, (2 * wm + x) * 16 + 4 * tp);
    }
  }
  auto tfrag_at = [](Frag<T>& f, const char* a0, const char* a1) {
    typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
    v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a0));
    v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a1));
    f.v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  if (u0 < u1) issue(u0, smem0, smem0 + HWG_XBUF);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (INBN) {
    if (u0 < u1) xform_x(u0, smem0);
  }
  auto run_tile = [&](int u, char* const Xs, char* const Xn) {
    char* const Ds = Xs + HWG_XBUF;
    halo_lds_barrier();
    // the next tile's pieces: two per wave after each of k-steps 0-4's MFMAs
    // (beside the matrix pipe instead of ahead of it, where both waves of a
    // SIMD issued theirs at once; SSIP_HWG_SPREAD=0: ahead, as before)
    const bool nxt = u + 1 < u1;
    if (nxt && !a.spread) issue(u + 1, Xn, Xn + HWG_XBUF);
    const int nR0 = (u + 1) * a.TR;
    const int nn = nR0 / a.H, np0 = nR0 - nn * a.H;
    const int nbase = (nn * a.H + np0) * a.W * 128;
    const bool spread = nxt && a.spread;
    Frag<T> fa[2][2], fb[2][9];
    auto load_step = [&](int ks, Frag<T>(&ra)[2], Frag<T>(&rb)[9]) {
#pragma unroll
      for (int x = 0; x < 2; ++x) tfrag_at(ra[x], Ds + 4096 * ks + dof[x][0], Ds + 4096 * ks + dof[x][1]);
#pragma unroll
      for (int b = 0; b < 9; ++b) tfrag_at(rb[b], Xs + 4096 * ks + xo[b][0], Xs + 4096 * ks + xo[b][1]);
    };
    load_step(0, fa[0], fb[0]);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 1 < 8) load_step(ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int b = 0; b < 9; ++b) mma(acc[x][b], fa[ks & 1][x], fb[ks & 1][b]);
      if (ks < 5 && spread) {
        issue_pc(2 * ks, nbase, np0, Xn, Xn + HWG_XBUF);
        issue_pc(2 * ks + 1, nbase, np0, Xn, Xn + HWG_XBUF);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's rows land before the barrier
    if constexpr (INBN) {
      if (nxt) xform_x(u + 1, Xn);
    }
  };
  for (int u = u0; u < u1; u += 2) {
    run_tile(u, smem0, smem1);
    if (u + 1 < u1) run_tile(u + 1, smem1, smem0);
  }
  // this workgroup's partial dW: slab[g][k][(t, c)]
  float* sl = a.slab + (long)g * 64 * 576;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int b = 0; b < 9; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = (2 * wm + x) * 16 + 4 * (lane >> 4) + e;
        const int col = (9 * wn + b) * 16 + (lane & 15);
        sl[(long)k * 576 + col] = acc[x][b][e];
      }
}

// ---------------------------------------------------------------------------
// WGRAD of the stem conv (7x7 / stride 2 over the pre-padded NHWC4 image):
//   dW[k][(r, s, c)] = sum_m dy[m][k] * x[2p + r][2q + s][c]
// Per tile of STEM_TR output rows (GEMM rows m = j * QP + q, dy zero for
// q >= Q) a persistent workgroup stages the 9 contiguous input rows (as
// conv_stem_halo_kernel) and the tile's dy rows (m-major MTile image), both
// double-buffered, and keeps the 64 x 224 fp32 result in registers across
// its tiles.  The x operand of column block (r, 16 of the 32 (s, c)) for
// row m is the 64-B run at input row 2j + r, pixel 2q: transposed fragment
// reads with per-lane row addresses (overlapping runs).  One fp32 slab per
// workgroup, summed by wgrad_reduce_kernel.
// ---------------------------------------------------------------------------
struct StemWgArgs {
  const __bf16* X;   // [N][H][W][4]
  const __bf16* DY;  // [N][P][Q][64]
  float* slab;       // [G][64][224]
  uint32_t x_bytes, dy_bytes;
  int N, H, W, P, Q, tiles;
};

constexpr int SWG_DBUF = 32 * 1024;  // 256 dy rows x 128 B

__global__ void __launch_bounds__(512, 2) conv_stem_wgrad_kernel(const StemWgArgs a) {
  typedef __bf16 T;
  typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
  constexpr int NW = 8, NB = 14;  // 224 / 16 column blocks
  __shared__ __attribute__((aligned(16))) char smem[2 * (STEM_XBUF + SWG_DBUF)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // k rows 32 wm .. +31; column blocks wn, wn + 4, ...
  const int G = gridDim.x, g = blockIdx.x;
  const int u0 = (int)((long)g * a.tiles / G), u1 = (int)((long)(g + 1) * a.tiles / G);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(a.X, a.x_bytes), rsD = make_rsrc(a.DY, a.dy_bytes);
  const int xpitch = a.W * 8;
  const int xrun = STEM_XROWS * xpitch;
  const int nxi = (xrun + 1023) >> 10;

  auto issue = [&](int tile, char* Xs, char* Ds) {
    const int R0 = tile * STEM_TR;
    const int n = R0 / a.P, p0 = R0 - n * a.P;
    const uint32_t xbase = (uint32_t)((((long)n * a.H + 2 * p0) * a.W) * 8);
    for (int i = wave; i < nxi; i += NW) {
      const int b = i * 1024 + lane * 16;
      blds16(rsX, b < xrun ? xbase + (uint32_t)b : SSIP_OOB, Xs + i * 1024);
    }
    for (int i = wave; i < SWG_DBUF / 1024; i += NW) {
      const int m = i * 8 + (lane >> 3);
      const int j = m / STEM_QP, q = m - j * STEM_QP;
      const int ch = (lane & 7) ^ mt64_chunk_xor(m);  // MTile<64> swizzle
      const bool ok = q < a.Q;
      const uint32_t off = (uint32_t)(((((long)n * a.P + p0 + j) * a.Q + q) * 64 + ch * 8) * 2);
      blds16(rsD, ok ? off : SSIP_OOB, Ds + i * 1024);
    }
  };

  const int nbw = wn < NB - 12 ? 4 : 3;  // column blocks of this wave: wn + 4 b, b < nbw
  f32x4 acc[2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[x][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // x fragment addressing: lane (g, q, p) reads rows m = row0 + 8 g + q (+4),
  // columns 4p .. 4p+3 of its block; row m's run starts at (2j + r) xpitch + 16 q_m
  const int lg = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;

  if (u0 < u1) issue(u0, smem, smem + STEM_XBUF);
  bool first = true;
  for (int u = u0; u < u1; ++u) {
    char* const Xs = smem + ((u - u0) & 1) * (STEM_XBUF + SWG_DBUF);
    char* const Ds = Xs + STEM_XBUF;
    char* const Xn = smem + ((u - u0 + 1) & 1) * (STEM_XBUF + SWG_DBUF);
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    first = false;
    halo_lds_barrier();
    if (u + 1 < u1) issue(u + 1, Xn, Xn + STEM_XBUF);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      Frag<T> fa[2], fb[4];
#pragma unroll
      for (int x = 0; x < 2; ++x) read_tfrag(fa[x], Ds, 32 * ks, (2 * wm + x) * 16, lane);
      // the lane's two rows (lo: +0, hi: +4) of this k-step
      const int m_lo = 32 * ks + 8 * lg + lq, m_hi = m_lo + 4;
      const int jl = m_lo / STEM_QP, ql = m_lo - jl * STEM_QP;
      const int jh = m_hi / STEM_QP, qh = m_hi - jh * STEM_QP;
      const int base_lo = 2 * jl * xpitch + (ql < a.Q ? ql : 0) * 16;  // rows past Q meet dy = 0
      const int base_hi = 2 * jh * xpitch + (qh < a.Q ? qh : 0) * 16;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (b < nbw) {
          const int nb = wn + 4 * b, r = nb >> 1, cofs = ((nb & 1) * 16 + 4 * lp) * 2;
          const char* a0 = Xs + base_lo + r * xpitch + cofs;
          const char* a1 = Xs + base_hi + r * xpitch + cofs;
          v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a0));
          v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) v4bf*)(a1));
          fb[b].v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (b < nbw) mma(acc[x][b], fa[x], fb[b]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float* sl = a.slab + (long)g * 64 * 224;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (b < nbw)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = (2 * wm + x) * 16 + 4 * (lane >> 4) + e;
          const int col = (wn + 4 * b) * 16 + (lane & 15);
          sl[(long)k * 224 + col] = acc[x][b][e];
        }
}

// ---------------------------------------------------------------------------
// Stem backward tail fused: the BN(+ReLU, through the 3x3/2/1 max-pool)
// backward apply pass and the stem wgrad in one persistent kernel, so the
// full-resolution dy never goes through HBM.  Per tile of 2 conv-output
// rows (h0 = 2T, 2T+1) a workgroup DMAs (double-buffered) the 9 input rows,
// the 2 pre-BN rows y, and pooled rows T, T+1 of dpool and the argmax bytes;
// then forms dy = A*d + B*y + C in LDS (d = the argmax-gathered pooled
// gradient masked by relu(fma(y, scale, shift)) > 0, exactly as
// stem_pool_bn_bwd_apply_kernel) as an m-major MTile image over the 224
// output pixels, and runs conv_stem_wgrad_kernel's MFMA loop on it.
// ---------------------------------------------------------------------------
struct StemBwArgs {
  const __bf16* X;      // [N][H][W][4]   pre-padded image
  const __bf16* Y;      // [N][P][Q][64]  pre-BN stem conv output
  const __bf16* DP;     // [N][P2][Q2][64] pooled gradient
  const uint8_t* IX;    // [N][P2][Q2][64] argmax bytes
  const float* scale;   // BN affine (ReLU mask)
  const float* shift;
  const float* coef;    // [3][64] from the BN-backward finalize
  float* slab;          // [G][64][224]
  uint32_t x_bytes, y_bytes, dp_bytes, ix_bytes;
  int N, H, W, P, Q, P2, Q2, tiles;
};

constexpr int SBW_Y = 28 * 1024, SBW_DP = 14 * 1024, SBW_IX = 7 * 1024;
constexpr int SBW_IN = STEM_XBUF + SBW_Y + SBW_DP + SBW_IX;  // one input buffer (66 KiB)

// The two halves of the work are specialised (tools/time_stem_bw.py on
// round 2's form, where every wave ran both behind a barrier -- r3-variants
// branch: DMA + sync alone 133 us, the dy pass +72, the MFMAs +74, and the
// two did not overlap): waves 0-7 form dy (two per SIMD,
// 4 channels x one 2x2 block per thread), waves 8-11 multiply (one per SIMD,
// all 64 k x 3-4 column blocks).  A tile's 224 GEMM rows are cut into half A (output columns
// 0-63 of both rows: 128 rows, 4 k-steps) and half B (columns 64-111: 96
// rows, 3 k-steps), GEMM row = 16 columns x 2 rows per 32-row chunk (the
// 2x2 pixel blocks of 8 pooled windows).  Phase (u, A): the dy waves form
// (u, B) while the MFMA waves run (u, A); phase (u, B): the dy waves form
// (u+1, A) while the MFMA waves run (u, B); one barrier per phase, each half
// in its own slot, so on every SIMD one wave's VALU work runs beside its
// partner's MFMAs.  The input regions are refilled as soon as their last
// reader is done, two phases ahead of their next reader: x of tile u+1 at
// (u, A) (x of u-1 was last read at (u-1, B)); y, the pooled gradient and
// the argmax of tile u+2 at (u, B) (those of u were last read at (u, A)).
// The dy waves issue every LDS-DMA, a fixed count per wave per region, and
// retire each region with a counted vmcnt before the barrier ahead of its
// first reader.  Same dy formula and (p, q)-ascending window order as above;
// the MFMA k-order within a tile differs (column chunks), so results agree
// to fp32 rounding.
constexpr int SBW2_SA = 128 * 128, SBW2_SB = 96 * 128;  // dy slots of half A / B

__global__ void __launch_bounds__(768, 1) conv_stem_bwd_wgrad2_kernel(const StemBwArgs a) {
  typedef __bf16 T;
  typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
  constexpr int NB = 14;
  constexpr int NVW = 8;  // dy waves (2 per SIMD); waves 8-11 run the MFMAs
  static_assert(STEM_XBUF / 1024 >= NVW && (SBW_Y + SBW_DP + SBW_IX) / 1024 >= NVW, "padding re-issues block i - NVW");
  static_assert(2 * SBW_IN + SBW2_SA + SBW2_SB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * SBW_IN + SBW2_SA + SBW2_SB];
  char* const SA = smem + 2 * SBW_IN;
  char* const SB = SA + SBW2_SA;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool vw = wave < NVW;
  const int G = gridDim.x, g = blockIdx.x;
  const int u0 = (int)((long)g * a.tiles / G), u1 = (int)((long)(g + 1) * a.tiles / G);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(a.X, a.x_bytes), rsY = make_rsrc(a.Y, a.y_bytes);
  const __amdgpu_buffer_rsrc_t rsP = make_rsrc(a.DP, a.dp_bytes), rsI = make_rsrc(a.IX, a.ix_bytes);
  const int xpitch = a.W * 8;
  const int xrun = STEM_XROWS * xpitch;
  const int yrun = 2 * a.Q * 128, prow = a.Q2 * 128, irow = a.Q2 * 64;
  auto buf = [&](int tile) { return smem + ((tile - u0) & 1) * SBW_IN; };

  // x rows of a tile (ceil(STEM_XBUF / NVW KiB) instructions per dy wave; a
  // tile past the range issues zero-fill so every wave's count is fixed)
  auto issue_x = [&](int tile) {
    char* B = buf(tile);
    const bool ok = tile < u1;
    const int R0 = tile * 2;
    const int n = R0 / a.P, h0 = R0 - n * a.P;
    const uint32_t xb = (uint32_t)((((long)n * a.H + 2 * h0) * a.W) * 8);
#pragma unroll
    for (int k = 0; k < (STEM_XBUF / 1024 + NVW - 1) / NVW; ++k) {
      // past the region: the wave's previous block again (same bytes to the same place)
      const int i = wave + NVW * k - (wave + NVW * k < STEM_XBUF / 1024 ? 0 : NVW);
      const int b = i * 1024 + lane * 16;
      blds16(rsX, ok && b < xrun ? xb + (uint32_t)b : SSIP_OOB, B + i * 1024);
    }
  };
  // y (whole 1-KiB runs), pooled gradient rows and argmax rows of a tile
  auto issue_ypi = [&](int tile) {
    char* B = buf(tile);
    const bool ok = tile < u1;
    const int R0 = tile * 2;
    const int n = R0 / a.P, h0 = R0 - n * a.P, T0 = h0 >> 1;
    const uint32_t yb = (uint32_t)((((long)n * a.P + h0) * a.Q) * 128);
    const int prows = (T0 + 1 < a.P2) ? 2 : 1;
    const uint32_t pb = (uint32_t)((((long)n * a.P2 + T0) * a.Q2) * 128);
    const uint32_t ib = (uint32_t)((((long)n * a.P2 + T0) * a.Q2) * 64);
    constexpr int NY = SBW_Y / 1024, NP = SBW_DP / 1024, NI = SBW_IX / 1024;
#pragma unroll
    for (int k = 0; k < (NY + NP + NI + NVW - 1) / NVW; ++k) {
      // past the regions: the wave's previous block again (same bytes to the same place)
      const int i = wave + NVW * k - (wave + NVW * k < NY + NP + NI ? 0 : NVW);
      const int b = (i < NY ? i : (i < NY + NP ? i - NY : i - NY - NP)) * 1024 + lane * 16;
      if (i < NY) {
        blds16(rsY, ok && b < yrun ? yb + (uint32_t)b : SSIP_OOB, B + STEM_XBUF + i * 1024);
      } else if (i < NY + NP) {
        blds16(rsP, ok && b < prows * prow ? pb + (uint32_t)b : SSIP_OOB, B + STEM_XBUF + i * 1024);
      } else {
        blds16(rsI, ok && b < prows * irow ? ib + (uint32_t)b : SSIP_OOB, B + STEM_XBUF + i * 1024);
      }
    }
  };
  constexpr int CX = (STEM_XBUF / 1024 + NVW - 1) / NVW;
  constexpr int CY = ((SBW_Y + SBW_DP + SBW_IX) / 1024 + NVW - 1) / NVW;

  // ---- dy waves: thread = (block lb, 4-channel quad c4) of a half
  const int lb = tid >> 4, c4 = tid & 15, ch0 = c4 * 4;
  float sc[4], sh[4], ca[4], cb[4], ck[4];
  if (vw) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sc[e] = a.scale[ch0 + e];
      sh[e] = a.shift[ch0 + e];
      ca[e] = a.coef[ch0 + e];
      cb[e] = a.coef[64 + ch0 + e];
      ck[e] = a.coef[128 + ch0 + e];
    }
  }
  // half h of tile `tile` into slot D (GEMM row of pixel (j, q) = chunk * 32 + j * 16 + q % 16,
  // chunk = (q - q0) / 16 with q0 the half's first column)
  auto produce = [&](int tile, int h, char* D) {
    const int nblk = h == 0 ? 32 : 24;
    if (lb >= nblk) return;
    const int R0 = tile * 2;
    const int h0 = R0 - (R0 / a.P) * a.P, T0 = h0 >> 1;
    const char* B = buf(tile);
    const char* Ys = B + STEM_XBUF;
    const char* Ps = Ys + SBW_Y;
    const char* Is = Ps + SBW_DP;
    const int l = (h == 0 ? 0 : 32) + lb;  // pooled window column: output columns 2l, 2l+1
    const bool q1 = l + 1 < a.Q2, p1 = T0 + 1 < a.P2;
    const uint32_t NOHIT = ~0u;  // no argmax byte is 255
    uint32_t k00, k01 = NOHIT, k10 = NOHIT, k11 = NOHIT;
    v4bf g00, g01, g10, g11;
    const v4bf z4 = (v4bf){(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
    k00 = *reinterpret_cast<const uint32_t*>(Is + l * 64 + ch0);
    g00 = *reinterpret_cast<const v4bf*>(Ps + l * 128 + ch0 * 2);
    g01 = g10 = g11 = z4;
    if (q1) {
      k01 = *reinterpret_cast<const uint32_t*>(Is + (l + 1) * 64 + ch0);
      g01 = *reinterpret_cast<const v4bf*>(Ps + (l + 1) * 128 + ch0 * 2);
    }
    if (p1) {
      k10 = *reinterpret_cast<const uint32_t*>(Is + (a.Q2 + l) * 64 + ch0);
      g10 = *reinterpret_cast<const v4bf*>(Ps + (a.Q2 + l) * 128 + ch0 * 2);
      if (q1) {
        k11 = *reinterpret_cast<const uint32_t*>(Is + (a.Q2 + l + 1) * 64 + ch0);
        g11 = *reinterpret_cast<const v4bf*>(Ps + (a.Q2 + l + 1) * 128 + ch0 * 2);
      }
    }
    float dz[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int b00 = (int)((k00 >> (8 * e)) & 0xff), b01 = (int)((k01 >> (8 * e)) & 0xff);
      const int b10 = (int)((k10 >> (8 * e)) & 0xff), b11 = (int)((k11 >> (8 * e)) & 0xff);
      const float v00 = (float)g00[e], v01 = (float)g01[e], v10 = (float)g10[e], v11 = (float)g11[e];
      float d;
      d = 0.f; if (b00 == 4) d += v00;
      dz[0][e] = d;
      d = 0.f; if (b00 == 5) d += v00; if (b01 == 3) d += v01;
      dz[1][e] = d;
      d = 0.f; if (b00 == 7) d += v00; if (b10 == 1) d += v10;
      dz[2][e] = d;
      d = 0.f; if (b00 == 8) d += v00; if (b01 == 6) d += v01; if (b10 == 2) d += v10; if (b11 == 0) d += v11;
      dz[3][e] = d;
    }
    const int q0 = h == 0 ? 0 : 64;
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int q = 2 * l + (px & 1), j = px >> 1;
      const int m = j * a.Q + q;                                      // pixel within the tile
      const int r = ((q - q0) >> 4) * 32 + j * 16 + ((q - q0) & 15);  // GEMM row within the half
      const v4bf yy = *reinterpret_cast<const v4bf*>(Ys + m * 128 + ch0 * 2);
      v4bf o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float yv = (float)yy[e];
        const float t = __builtin_fmaf(yv, sc[e], sh[e]);
        const float d = (t > 0.f ? t : 0.f) > 0.f ? dz[px][e] : 0.f;
        o[e] = (__bf16)(ca[e] * d + cb[e] * yv + ck[e]);
      }
      *reinterpret_cast<v4bf*>(D + r * 128 + (((c4 >> 1) ^ mt64_chunk_xor(r)) << 4) + (c4 & 1) * 8) = o;
    }
  };

  // ---- MFMA waves: wave mw = wave - NVW owns column blocks mw + 4 b (b < nbw) x all 64 k
  const int mw = wave - NVW;
  const int nbw = mw < NB - 12 ? 4 : 3;
  const int lg = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;
  auto consume = [&](f32x4 (&acc)[4][4], int tile, int h, const char* D) {
    const char* Xs = buf(tile);
    const int nks = h == 0 ? 4 : 3, q0 = h == 0 ? 0 : 64;
    for (int ks = 0; ks < nks; ++ks) {
      Frag<T> fa[4], fb[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) read_tfrag(fa[x], D, 32 * ks, x * 16, lane);
      // the lane's rows (lo, hi = lo + 4) of this chunk: output row >> 4, column q0 + 16 ks + (row & 15)
      const int m_lo = 8 * lg + lq, m_hi = m_lo + 4;
      const int base_lo = 2 * (m_lo >> 4) * xpitch + (q0 + 16 * ks + (m_lo & 15)) * 16;
      const int base_hi = 2 * (m_hi >> 4) * xpitch + (q0 + 16 * ks + (m_hi & 15)) * 16;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (b < nbw) {
          const int nb = mw + 4 * b, r = nb >> 1, cofs = ((nb & 1) * 16 + 4 * lp) * 2;
          v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (__attribute__((address_space(3))) v4bf*)(Xs + base_lo + r * xpitch + cofs));
          v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (__attribute__((address_space(3))) v4bf*)(Xs + base_hi + r * xpitch + cofs));
          fb[b].v = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (b < nbw) mma(acc[x][b], fa[x], fb[b]);
    }
  };

  // the two roles run separate loops (so neither holds the other's registers)
  // with the same barrier sequence: 2 in the prologue, 2 per tile
  if (vw) {
    if (u0 < u1) {
      // prologue: inputs of the first tile (+ y / pooled / argmax of the second), its half A
      issue_ypi(u0);
      issue_x(u0);
      issue_ypi(u0 + 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CY) : "memory");
      halo_lds_barrier();
      produce(u0, 0, SA);
      halo_lds_barrier();
    }
    for (int u = u0; u < u1; ++u) {
      // phase (u, A): dy (u, B) beside the MFMAs of (u, A); x of u+1 into its buffer
      issue_x(u + 1);
      produce(u, 1, SB);
      // y / pooled / argmax of u+1 (issued at (u-1, B)) land before the barrier
      // ahead of phase (u, B), whose dy waves form (u+1, A); younger: x of u+1
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CX) : "memory");
      halo_lds_barrier();
      // phase (u, B): dy (u+1, A) beside the MFMAs of (u, B); y / pooled / argmax of u+2
      issue_ypi(u + 2);
      if (u + 1 < u1) produce(u + 1, 0, SA);
      // x of u+1 (issued at (u, A)) lands before the barrier ahead of (u+1, A);
      // younger: this phase's y / pooled / argmax of u+2
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CY) : "memory");
      halo_lds_barrier();
    }
    // the zero-fill issues past the range land before the LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    f32x4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[x][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (u0 < u1) {
      halo_lds_barrier();
      halo_lds_barrier();
    }
    for (int u = u0; u < u1; ++u) {
      consume(acc, u, 0, SA);
      halo_lds_barrier();
      consume(acc, u, 1, SB);
      halo_lds_barrier();
    }
    float* sl = a.slab + (long)g * 64 * 224;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (b < nbw)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int kk = x * 16 + 4 * (lane >> 4) + e;
            const int col = (mw + 4 * b) * 16 + (lane & 15);
            sl[(long)kk * 224 + col] = acc[x][b][e];
          }
  }
}

// ---------------------------------------------------------------------------
// host-side planning
// ---------------------------------------------------------------------------
struct Plan {
  int mode;
  int bm, bn, wmw, wnw;
  int stages;  // 2/3: LDS-DMA ring kernel (bf16); 0: register-staged kernel
  bool conv1;
  bool stem_glds;  // conv1 on a pre-padded image (pad 0, even W): LDS-DMA capable
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

static void pick_tile(int M, int Ng, int elem_bytes, Plan& pl) {
  // bf16: 256-row tiles (8 waves) when the grid still fills the chip twice over
  const int bn = (Ng % 128 == 0) ? 128 : 64;
  const long blocks256 = (long)ceil_div(M, 256) * ceil_div(Ng, bn);
  if (elem_bytes == 2 && blocks256 >= 512) {
    pl.bm = 256; pl.bn = bn; pl.wmw = 4; pl.wnw = 2;
  } else {
    pl.bm = 128; pl.bn = bn; pl.wmw = 2; pl.wnw = 2;
  }
}

static bool glds_has(int mode, bool stem, int bm, int bn, int wm, int wn, int st);
static int device_cus();
// SSIP_WGRAD_BIG (a wgrad with a budget, i.e. on the side stream): 0 = the
// full-grid tiles; 1 = 16-wave 256-column tiles for every 3x3 wgrad, 2 = only
// the 256x256 ones (K % 256 == 0) -- round 5: faster alone, slower in the step
// (6.34 vs 6.19 ms), a 16-wave workgroup holding every register of its CU
// keeps the main stream's dgrad / BN chain off it; 3 = 8-wave 256x256 tiles
// for those; 4 (default) = those and 8-wave 128x256 tiles where 128 <= K <
// 256, both on SSIP_WGRAD_BIG_CUS (default 62) percent of the budget's CUs,
// the rest of the chip left to the main stream.  Round 6, with the stagger
// (tools/gpu_r6_{i,j,k}.sh, alternated runs on one box each, ms/step): mode 4
// on 62 % of the CUs 5.937 vs 6.013 (4 + 4; 56 % 5.969, 70 % 5.979, 80 %
// 6.083), 5.933 vs 6.018 on another box; mode 3 at 62 % 5.985; mode 3 on
// every CU 5.98 vs 5.87 (profiles/r6_wgrad_big_ab.txt)
static int wgrad_big_mode() {
  const char* e = getenv("SSIP_WGRAD_BIG");
  return e ? atoi(e) : 4;
}

// Default LDS-DMA configuration for a bf16 GEMM view (M x Ng, reduction Kg).
// Chosen from tools/tune_conv.py over the ResNet-18 train-step shapes
// (profiles/r1_conv_tune.txt): two LDS stages and 8-16 waves per workgroup
// beat deeper rings at one workgroup per CU on every shape; 2-3 workgroups
// per CU hide each other's barriers and epilogues.
static void choose_glds(int mode, const ConvArgs& a, Plan& pl) {
  pl.stages = 2;
  if (mode == MODE_WGRAD) {
    // 8 waves of 32x64 (profiles/r2_wgrad_tiles.txt: 3-6 % over 16 waves of 32x32,
    // whose fragment reads load the LDS as much as the MFMAs)
    if (a.M % 128 == 0) { pl.bm = 128; pl.bn = 128; pl.wmw = 4; pl.wnw = 2; }
    else { pl.bm = 64; pl.bn = 128; pl.wmw = 2; pl.wnw = 4; }
    return;
  }
  pl.bm = 128; pl.wmw = 4; pl.wnw = 2;
  pl.bn = (a.Ng % 128 == 0) ? 128 : 64;
  // 256x256 tiles (8 waves of 64x128) where a forward or stride-1 dgrad still
  // has >= 160 of them (ResNet-18 layer3: fwd 62.7 vs 69.1 us,
  // profiles/r1_conv_tune.txt; dgrad 62.4 vs 67.8 us, profiles/r3_tune_fd.txt)
  if ((mode == MODE_FWD || (mode == MODE_DGRAD && a.stride == 1)) && a.Ng % 256 == 0 &&
      (long)ceil_div(a.M, 256) * (a.Ng / 256) >= 160) {
    pl.bm = 256; pl.bn = 256;
  } else if (mode == MODE_FWD && a.Ng % 128 == 0 && (long)ceil_div(a.M, 128) * (a.Ng / 128) <= device_cus()) {
    // at most one 128x128 tile per CU (the weak forward's layer4 at batch 128:
    // 196 tiles): one workgroup of 16 waves (32x32 wave tiles) and a 3-deep
    // ring per CU instead of 8 waves that leave every second slot empty
    // (l4.3x3 42.4 vs 50.2 us, l4.3x3s2 24.1 vs 26.7, profiles/r2_tune_fwd_b128.txt)
    pl.wnw = 4; pl.stages = 3;
  }
}

// Tuning override: SSIP_CONV_FORCE="<f|d|w>,bm,bn,waves_m,waves_n,stages"
// (stages 0 = register-staged kernel) applies to the named pass only.
static int apply_force(int mode, int elem_bytes, Plan& pl) {
  const char* e = getenv("SSIP_CONV_FORCE");
  if (!e || !e[0]) return SSIP_OK;
  const char want = mode == MODE_FWD ? 'f' : mode == MODE_DGRAD ? 'd' : 'w';
  if (e[0] != want || (pl.conv1 && !pl.stem_glds)) return SSIP_OK;
  int bm, bn, wm, wn, st;
  SSIP_REQUIRE(sscanf(e + 1, ",%d,%d,%d,%d,%d", &bm, &bn, &wm, &wn, &st) == 5, SSIP_ERR_ARG,
               "bad SSIP_CONV_FORCE '%s'", e);
  if (st > 0) {
    SSIP_REQUIRE(elem_bytes == 2 && glds_has(mode, pl.conv1, bm, bn, wm, wn, st), SSIP_ERR_ARG,
                 "SSIP_CONV_FORCE: no LDS-DMA kernel %s", e);
  } else {
    const bool ok = mode == MODE_WGRAD ? (wm == 2 && wn == 2 && (bm == 128 || bm == 64))
                                       : ((bm == 256 && wm == 4 && wn == 2 && elem_bytes == 2) ||
                                          (bm == 128 && wm == 2 && wn == 2));
    SSIP_REQUIRE(ok && (bn == 128 || bn == 64), SSIP_ERR_ARG, "SSIP_CONV_FORCE: no register-staged kernel %s", e);
  }
  pl.bm = bm; pl.bn = bn; pl.wmw = wm; pl.wnw = wn; pl.stages = st;
  return SSIP_OK;
}

// SSIP_STAGGER (read per plan, so a lab can flip it in one process): a
// bit mask over the passes whose LDS-DMA ring kernels run the stagger
// (conv_glds_kernel: waves NW/2.. one MFMA half behind), 1 fwd, 2 dgrad,
// 4 wgrad; 0 off; default 7 (round 6, tools/stagger_lab.py, batch 256, same
// bits: the layer 2-4 launches -3.8 % in sum, the 256x256 layer-3 fwd /
// dgrad -11 to -13 %, the side stream's one-workgroup-per-CU wgrads -4 to
// -6 %; step 6.076 -> 6.045 ms, 3 + 3 alternated runs,
// profiles/r6_stagger_lab.txt).
static int stagger_for(int mode, const Plan& pl) {
  if (pl.stages <= 0 || pl.conv1) return 0;
  const char* e = getenv("SSIP_STAGGER");
  const int m = e != nullptr ? atoi(e) : 7;
  return (m >> mode) & 1;
}

static int plan_conv(int mode, const ssip_conv_desc* d, int elem_bytes, Plan& pl, int wg_budget = 0,
                     bool allow_big = true) {
  SSIP_REQUIRE(desc_ok(d), SSIP_ERR_ARG, "bad conv descriptor");
  pl.mode = mode;
  pl.conv1 = (d->C == 4);
  // the padded stem stores S = 8 columns for a real 7-wide filter
  const int s_real = pl.conv1 ? d->S - 1 : d->S;
  SSIP_REQUIRE(d->P == (d->H + 2 * d->pad - d->R) / d->stride + 1 && d->Q == (d->W + 2 * d->pad - s_real) / d->stride + 1,
               SSIP_ERR_ARG, "P/Q inconsistent with H/W/R/S/stride/pad");
  const int BK = elem_bytes == 2 ? 64 : 32;
  SSIP_REQUIRE(pl.conv1 ? (d->S == 8) : (d->C % BK == 0), SSIP_ERR_ARG,
               "conv input channels must be a multiple of %d (or 4 with S padded to 8); got C=%d S=%d", BK, d->C,
               d->S);
  SSIP_REQUIRE(d->K % BK == 0, SSIP_ERR_ARG, "conv output channels must be a multiple of %d; got K=%d", BK, d->K);
  const long NPQ = (long)d->N * d->P * d->Q, NHW = (long)d->N * d->H * d->W;
  SSIP_REQUIRE(NPQ < (1l << 31) && NHW * d->C < (1l << 31) && NPQ * d->K < (1l << 31), SSIP_ERR_ARG,
               "tensor too large for 32-bit indexing");
  ConvArgs& a = pl.args;
  fill_common(a, d);
  pl.splits = 1;
  if (mode == MODE_FWD) {
    a.M = (int)NPQ; a.Ng = d->K; a.Kg = d->R * d->S * d->C;
    a.ksteps = ceil_div(a.Kg, BK);
    pick_tile(a.M, a.Ng, elem_bytes, pl);
  } else if (mode == MODE_DGRAD) {
    SSIP_REQUIRE(!pl.conv1, SSIP_ERR_ARG, "dgrad of the C=4 stem conv is not supported (input needs no grad)");
    SSIP_REQUIRE(d->stride == 1 || d->stride == 2 || d->stride == 4, SSIP_ERR_ARG, "dgrad stride must be 1, 2 or 4");
    a.M = (int)NHW; a.Ng = d->C; a.Kg = d->R * d->S * d->K;
    a.ksteps = a.Kg / BK;
    pick_tile(a.M, a.Ng, elem_bytes, pl);
  } else {
    a.M = d->K; a.Ng = d->R * d->S * d->C; a.Kg = 0;
    a.Mred = (int)NPQ;
    pl.wmw = 2; pl.wnw = 2;
    pl.bm = (d->K % 128 == 0) ? 128 : 64;
    pl.bn = 128;
    if (a.Ng % 128 != 0 && a.Ng % 64 == 0 && pl.bm == 128) pl.bn = 64;
  }
  pl.stages = 0;
  pl.stem_glds = pl.conv1 && d->pad == 0 && d->W % 2 == 0 && d->S == 8;
  if (elem_bytes == 2 && (!pl.conv1 || pl.stem_glds)) choose_glds(mode, a, pl);
  // a wgrad sharing the chip at one workgroup per CU (ssip_conv_wgrad_budget):
  // 8-wave 128x128 workgroups alone on a CU wait on their own barriers and
  // LDS-DMA (18 % MFMA busy, 59 % of wave cycles parked); 16-wave
  // workgroups of 256 columns hide that and halve the DMA bytes per FLOP
  // (tools/wgrad_lab.py at the 256-workgroup budget, profiles/r5_wgrad_lab.txt:
  // l2.3x3 110.9 -> 89.1 us with 128x256, l3.3x3 109.9 -> 73.9 and l4.3x3
  // 101.4 -> 75.4 with 256x256) -- but not in the step (wgrad_big_mode)
  const int bigm = (mode == MODE_WGRAD && allow_big) ? wgrad_big_mode() : 0;
  // (round 5 also measured 8-wave 128x256 tiles at the budget -- two waves
  // per SIMD, 96 KiB of LDS, so not the whole CU: 517.6 -> 461.1 us over the
  // six layer 2-4 wgrads, but the step 6.14 -> 6.43 ms, 4 + 4 runs)
  if (mode == MODE_WGRAD && wg_budget > 0 && pl.stages > 0 && !pl.conv1 && bigm > 0) {
    // (the 1x1 downsample wgrads, Ng <= 256, keep their many-tile grids)
    if (a.M % 256 == 0 && a.Ng % 256 == 0 && a.Ng >= 512) {
      // 3, 4: the 8-wave 256x256 tile (with the stagger: l3 / l4 3x3 wgrads
      // at the budget 98 -> 73 us, profiles/r6_tile_lab.txt)
      pl.bm = 256; pl.bn = 256; pl.wmw = 4; pl.wnw = bigm >= 3 ? 2 : 4;
    } else if (bigm == 1 && a.M % 128 == 0 && a.Ng >= 512) {
      pl.bm = 128; pl.bn = 256; pl.wmw = 4; pl.wnw = 4;  // a partial last tile where Ng % 256 != 0
    } else if (bigm == 4 && a.M % 128 == 0 && a.Ng >= 512) {
      pl.bm = 128; pl.bn = 256; pl.wmw = 2; pl.wnw = 4;  // 8 waves, 96 KiB of LDS
    }
    if (bigm >= 3 && pl.bn == 256) {
      // on SSIP_WGRAD_BIG_CUS percent of the budget's CUs, the rest left to the
      // main stream (measured: profiles/r6_tile_lab.txt)
      const char* e = getenv("SSIP_WGRAD_BIG_CUS");
      const int pc = e ? std::max(1, std::min(100, atoi(e))) : 62;
      wg_budget = std::max(1, wg_budget * pc / 100);
    }
  }
  if (int rc = apply_force(mode, elem_bytes, pl)) return rc;
  if (mode == MODE_WGRAD) {
    const int tiles = ceil_div(a.M, pl.bm) * ceil_div(a.Ng, pl.bn);
    const int total_ks = ceil_div(a.Mred, BK);
    // split count: every split is one more fp32 slab written here and read by
    // the reduce; the grid should end on a full wave of resident workgroups
    // (a launch of 540 workgroups on 512 slots runs two waves for 5 % more
    // work).  Cost in k-step times: waves * k-steps per split + the slab
    // round trip (~0.27 k-step per MiB, tools/tune_wgrad_splits.py);
    // slab <= 64 MiB, >= 16 k-steps per split.
    const long slab_split = (long)a.M * a.Ng * 4;
    const int cap_bytes = (int)std::max<long>(1, (64l << 20) / slab_split);
    const int max_splits = std::max(1, std::min(cap_bytes, total_ks / 16));
    int splits = 1;
    if (const char* e = getenv("SSIP_WGRAD_BLOCKS"); e && e[0]) {  // tuning override: target workgroup count
      splits = std::min(max_splits, ceil_div(std::max(1, atoi(e)), tiles));
    } else if (pl.stages > 0 && wg_budget > 0) {
      // a wgrad sharing the chip (ssip_conv_wgrad_budget): ResNet-18 train
      // step with the side-stream wgrads at one workgroup per CU, two A/Bs of
      // 3 + 3 alternated runs: 6.341 vs 6.369 and 6.431 vs 6.490 ms/step
      // (the main stream's BN-backward passes wait less for wgrad workgroups
      // to retire, and half the split slabs move through HBM)
      // a kernel that fits one workgroup per CU (LDS > 80 KiB): at most
      // `budget` workgroups (one more would run a second round on its CU);
      // the 2-per-CU tiles round up (an extra workgroup shares a CU)
      const int lds = std::max(2, pl.stages) * 64 * (pl.bm + pl.bn) * 2;
      splits = std::min(max_splits, lds > 81920 ? std::max(1, wg_budget / tiles) : ceil_div(wg_budget, tiles));
    } else if (pl.stages > 0) {
      const int nt = 64 * pl.wmw * pl.wnw;
      const int nbuf = std::max(2, pl.stages);
      const int lds = nbuf * 64 * (pl.bm + pl.bn) * 2;
      const int per_cu = std::max(1, std::min(2048 / nt, 163840 / lds));
      const long slots = (long)device_cus() * per_cu;
      double best = 1e30;
      for (int s = 1; s <= max_splits; ++s) {
        const long waves = ((long)tiles * s + slots - 1) / slots;
        const double cost = (double)waves * ceil_div(total_ks, s) + 0.27 * s * (double)slab_split / (1 << 20);
        if (cost < best - 1e-9) { best = cost; splits = s; }
      }
    } else {
      splits = std::min(max_splits, ceil_div(1024, tiles));
    }
    if (splits < 1) splits = 1;
    a.ksteps = ceil_div(total_ks, splits);
    splits = ceil_div(total_ks, a.ksteps);
    pl.splits = splits;
  }
  a.tiles_n = ceil_div(a.Ng, pl.bn);
  const int tiles_m = ceil_div(a.M, pl.bm);
  pl.grid = dim3(tiles_m * a.tiles_n, pl.splits, 1);
  a.xcd_remap = 1;
  {
    // SSIP_DMA_MID: 0 never, 1 every LDS-DMA ring, 2 the 256x256 tiles only
    static const int mid = [] {
      const char* e = getenv("SSIP_DMA_MID");
      return e != nullptr ? atoi(e) : 0;
    }();
    a.dma_mid = mid == 1 || (mid == 2 && pl.bm == 256 && pl.bn == 256);
  }
  a.stagger = stagger_for(mode, pl);
  return SSIP_OK;
}

// LDS-DMA ring kernel configurations (bm, bn, waves_m, waves_n, stages):
// the ones choose_glds() selects (round 3's wider tuning sets are on the
// r3-variants branch, with tools/tune_conv.py's lists)
#define SSIP_GLDS_FD(X) X(128, 128, 4, 2, 2) X(128, 64, 4, 2, 2) X(256, 256, 4, 2, 2) X(128, 128, 4, 4, 3)
// (the first two: the full-grid tiles; the two 16-wave ones: the side-stream
// budget's; the rest are tools/wgrad_lab.py comparison points)
#define SSIP_GLDS_WG(X)                                                                                     \
  X(128, 128, 4, 2, 2) X(64, 128, 2, 4, 2) X(256, 256, 4, 4, 2) X(128, 256, 4, 4, 2) X(128, 256, 2, 4, 2)    \
  X(256, 256, 4, 2, 2) X(128, 128, 4, 4, 2)
#define SSIP_GLDS_POST(X) X(128, 128, 4, 2, 2) X(128, 64, 4, 2, 2)
#define SSIP_GLDS_FOLD(X) SSIP_GLDS_FD(X)
#define SSIP_GLDS_STEM(X) X(128, 64, 4, 2, 2)

static bool glds_has(int mode, bool stem, int bm, int bn, int wm, int wn, int st) {
#define SSIP_GLDS_EQ(BM_, BN_, WM_, WN_, ST_) \
  if (bm == BM_ && bn == BN_ && wm == WM_ && wn == WN_ && st == ST_) return true;
  if (mode == MODE_WGRAD) {
    SSIP_GLDS_WG(SSIP_GLDS_EQ)
  } else if (mode == MODE_FWD && stem) {
    SSIP_GLDS_STEM(SSIP_GLDS_EQ)
  } else {
    SSIP_GLDS_FD(SSIP_GLDS_EQ)
  }
#undef SSIP_GLDS_EQ
  return false;
}

// the LDS-DMA ring configurations with the BN+ReLU-in operand transform
#define SSIP_GLDS_INBN_FD(X) X(128, 128, 4, 2, 2) X(128, 64, 4, 2, 2) X(256, 256, 4, 2, 2)
#define SSIP_GLDS_INBN_WG(X) X(128, 128, 4, 2, 2)

template <int MODE>
static int launch_glds(const Plan& pl, hipStream_t st) {
  if constexpr (MODE != MODE_DGRAD) {
    if (pl.args.in_scale != nullptr) {
#define SSIP_GLDS_GOI(BM_, BN_, WM_, WN_, ST_)                                                                \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_) {                   \
    SSIP_KLAUNCH((conv_glds_kernel<MODE, BM_, BN_, WM_, WN_, ST_, false, false, false, true>), pl.grid,      \
                 dim3(64 * WM_ * WN_), 0, st, pl.args);                                                       \
    return ::ssip::check_launch("conv_glds_inbn");                                                            \
  }
      if constexpr (MODE == MODE_WGRAD) {
        SSIP_GLDS_INBN_WG(SSIP_GLDS_GOI)
      } else {
        SSIP_GLDS_INBN_FD(SSIP_GLDS_GOI)
      }
#undef SSIP_GLDS_GOI
      ::ssip::set_error("no BN+ReLU-in conv kernel for %dx%d/%dx%d/%d", pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages);
      return SSIP_ERR_ARG;
    }
  }
#define SSIP_GLDS_GO(BM_, BN_, WM_, WN_, ST_)                                                                 \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_) {                   \
    SSIP_KLAUNCH((conv_glds_kernel<MODE, BM_, BN_, WM_, WN_, ST_>), pl.grid, dim3(64 * WM_ * WN_), 0,   \
                       st, pl.args);                                                                          \
    return ::ssip::check_launch("conv_glds");                                                                 \
  }
  if constexpr (MODE == MODE_WGRAD) {
    SSIP_GLDS_WG(SSIP_GLDS_GO)
  } else {
    if constexpr (MODE == MODE_DGRAD) {
      if (pl.args.pmean != nullptr) {  // fused BN-backward epilogue: default tiles only
#define SSIP_GLDS_GOP(BM_, BN_, WM_, WN_, ST_)                                                                \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_) {                   \
    SSIP_KLAUNCH((conv_glds_kernel<MODE, BM_, BN_, WM_, WN_, ST_, false, true>), pl.grid,               \
                       dim3(64 * WM_ * WN_), 0, st, pl.args);                                                 \
    return ::ssip::check_launch("conv_glds_bnpost");                                                          \
  }
        SSIP_GLDS_POST(SSIP_GLDS_GOP)
#undef SSIP_GLDS_GOP
        ::ssip::set_error("no fused-BN dgrad kernel for %dx%d/%dx%d/%d", pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages);
        return SSIP_ERR_ARG;
      }
    }
    if constexpr (MODE == MODE_FWD) {
      if (pl.args.bias != nullptr) {  // folded eval BN epilogue: the default tiles only
#define SSIP_GLDS_GOF(BM_, BN_, WM_, WN_, ST_)                                                                \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_) {                   \
    SSIP_KLAUNCH((conv_glds_kernel<MODE, BM_, BN_, WM_, WN_, ST_, false, false, true>), pl.grid,        \
                       dim3(64 * WM_ * WN_), 0, st, pl.args);                                                 \
    return ::ssip::check_launch("conv_glds_fold");                                                            \
  }
        SSIP_GLDS_FOLD(SSIP_GLDS_GOF)
#undef SSIP_GLDS_GOF
        ::ssip::set_error("no folded-BN conv kernel for %dx%d/%dx%d/%d", pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages);
        return SSIP_ERR_ARG;
      }
      if (pl.conv1) {
#define SSIP_GLDS_GO4(BM_, BN_, WM_, WN_, ST_)                                                                \
  if (pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_) {                   \
    SSIP_KLAUNCH((conv_glds_kernel<MODE, BM_, BN_, WM_, WN_, ST_, true>), pl.grid, dim3(64 * WM_ * WN_), \
                       0, st, pl.args);                                                                       \
    return ::ssip::check_launch("conv_glds_stem");                                                            \
  }
        SSIP_GLDS_STEM(SSIP_GLDS_GO4)
#undef SSIP_GLDS_GO4
        ::ssip::set_error("no LDS-DMA stem kernel for %dx%d/%dx%d/%d", pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages);
        return SSIP_ERR_ARG;
      }
    }
    SSIP_GLDS_FD(SSIP_GLDS_GO)
  }
#undef SSIP_GLDS_GO
  ::ssip::set_error("no LDS-DMA conv kernel for %dx%d/%dx%d/%d", pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages);
  return SSIP_ERR_ARG;
}

template <int MODE, typename T>
static int launch_conv(const Plan& pl, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    if (pl.stages > 0) return launch_glds<MODE>(pl, st);
  }
#define SSIP_LAUNCH(BM_, BN_, WM_, WN_, C1_)                                                                  \
  {                                                                                                           \
    SSIP_KLAUNCH((conv_gemm_kernel<MODE, T, BM_, BN_, WM_, WN_, C1_>), pl.grid, dim3(64 * WM_ * WN_), 0, \
                       st, pl.args);                                                                          \
  }
  const bool c1 = pl.conv1;
  if constexpr (MODE == MODE_WGRAD) {
    if (pl.bm == 128 && pl.bn == 128) {
      if (c1) SSIP_LAUNCH(128, 128, 2, 2, true) else SSIP_LAUNCH(128, 128, 2, 2, false)
    } else if (pl.bm == 128 && pl.bn == 64) {
      if (c1) SSIP_LAUNCH(128, 64, 2, 2, true) else SSIP_LAUNCH(128, 64, 2, 2, false)
    } else if (pl.bm == 64 && pl.bn == 128) {
      if (c1) SSIP_LAUNCH(64, 128, 2, 2, true) else SSIP_LAUNCH(64, 128, 2, 2, false)
    } else {
      ::ssip::set_error("no wgrad kernel for tile %dx%d", pl.bm, pl.bn);
      return SSIP_ERR_ARG;
    }
  } else if constexpr (MODE == MODE_FWD) {
    if (sizeof(T) == 2 && pl.bm == 256 && pl.bn == 128) {
      if constexpr (sizeof(T) == 2) { if (c1) SSIP_LAUNCH(256, 128, 4, 2, true) else SSIP_LAUNCH(256, 128, 4, 2, false) }
    } else if (sizeof(T) == 2 && pl.bm == 256 && pl.bn == 64) {
      if constexpr (sizeof(T) == 2) { if (c1) SSIP_LAUNCH(256, 64, 4, 2, true) else SSIP_LAUNCH(256, 64, 4, 2, false) }
    } else if (pl.bm == 128 && pl.bn == 128) {
      if (c1) SSIP_LAUNCH(128, 128, 2, 2, true) else SSIP_LAUNCH(128, 128, 2, 2, false)
    } else if (pl.bm == 128 && pl.bn == 64) {
      if (c1) SSIP_LAUNCH(128, 64, 2, 2, true) else SSIP_LAUNCH(128, 64, 2, 2, false)
    } else {
      ::ssip::set_error("no fwd kernel for tile %dx%d", pl.bm, pl.bn);
      return SSIP_ERR_ARG;
    }
  } else {
    if (sizeof(T) == 2 && pl.bm == 256 && pl.bn == 128) {
      if constexpr (sizeof(T) == 2) SSIP_LAUNCH(256, 128, 4, 2, false)
    } else if (sizeof(T) == 2 && pl.bm == 256 && pl.bn == 64) {
      if constexpr (sizeof(T) == 2) SSIP_LAUNCH(256, 64, 4, 2, false)
    } else if (pl.bm == 128 && pl.bn == 128) SSIP_LAUNCH(128, 128, 2, 2, false)
    else if (pl.bm == 128 && pl.bn == 64) SSIP_LAUNCH(128, 64, 2, 2, false)
    else {
      ::ssip::set_error("no dgrad kernel for tile %dx%d", pl.bm, pl.bn);
      return SSIP_ERR_ARG;
    }
  }
#undef SSIP_LAUNCH
  return ::ssip::check_launch("conv_gemm");
}

static int elem_bytes_of(int dtype) { return dtype == SSIP_BF16 ? 2 : 4; }

// Register-staged kernel for a FWD/DGRAD GEMM view the LDS-DMA kernel does not
// address: the strided DGRAD without its phase split, filters of > 32 taps.
static void fallback_regstaged(Plan& pl) {
  ConvArgs& a = pl.args;
  pl.stages = 0;
  a.phased = 0;
  pick_tile(a.M, a.Ng, 2, pl);
  a.tiles_n = ceil_div(a.Ng, pl.bn);
  pl.grid = dim3(ceil_div(a.M, pl.bm) * a.tiles_n, 1, 1);
}

// phases by k-steps, descending (ties in phase order): the kernel hands them
// out in this order within each tile, so the long phases start first
static void set_phase_order(ConvArgs& a) {
  int ord[4] = {0, 1, 2, 3};
  std::stable_sort(ord, ord + 4, [&](int x, int y) { return a.phase[x].ksteps > a.phase[y].ksteps; });
  a.phase_order = ord[0] | (ord[1] << 2) | (ord[2] << 4) | (ord[3] << 6);
}

// Stride-2 DGRAD as four dense sub-problems, one per output parity phase:
// phase (ph, pw) only meets the taps r = r0 + 2*ri, s = s0 + 2*si, so the
// k-loop skips the 3/4 of (tap, pixel) pairs the plain implicit GEMM would
// gather as zeros.  blockIdx.y = phase; grid.x covers the largest phase.
static void phase_split(Plan& pl, const ssip_conv_desc* d) {
  if (pl.stages == 0 || pl.conv1 || d->stride != 2) return;
  ConvArgs& a = pl.args;
  int max_tiles = 0;
  for (int f = 0; f < 4; ++f) {
    PhaseInfo& P = a.phase[f];
    P.ph = f >> 1;
    P.pw = f & 1;
    const int Hph = (d->H - P.ph + 1) / 2, Wph = (d->W - P.pw + 1) / 2;
    P.r0 = (P.ph + d->pad) % 2;
    P.s0 = (P.pw + d->pad) % 2;
    P.nr = P.r0 < d->R ? (d->R - P.r0 + 1) / 2 : 0;
    P.ns = P.s0 < d->S ? (d->S - P.s0 + 1) / 2 : 0;
    P.bh = (P.ph + d->pad - P.r0) / 2;
    P.bw = (P.pw + d->pad - P.s0) / 2;
    P.Wph = Wph;
    P.M = d->N * Hph * Wph;
    P.tiles_m = ceil_div(P.M, pl.bm);
    P.ksteps = P.nr * P.ns * (d->K / 64);
    P.div_hw = make_fastdiv((uint32_t)std::max(1, Hph * Wph));
    P.div_w = make_fastdiv((uint32_t)std::max(1, Wph));
    max_tiles = std::max(max_tiles, P.tiles_m);
  }
  a.phased = 1;
  set_phase_order(a);
  pl.grid = dim3(std::max(1, max_tiles) * a.tiles_n, 4, 1);
}

// ---- halo path (conv_halo_kernel): 3x3 / stride 1 / pad 1, 64 reduction
// channels, bf16.  SSIP_HALO=0 turns it off; an SSIP_CONV_FORCE for the pass
// selects the implicit-GEMM kernels instead (tools/tune_conv.py).
struct HaloPlan {
  int TR, tiles, units, G, cols;
};

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    cus = (hipGetDevice(&dev) == hipSuccess &&
           hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
              ? v
              : 256;
  }
  return cus;
}

static bool halo_plan(int mode, const ssip_conv_desc* d, int dtype, HaloPlan& hp) {
  const char* e = getenv("SSIP_HALO");
  if (e && e[0] == '0') return false;
  const char* f = getenv("SSIP_CONV_FORCE");
  if (f && f[0] == (mode == MODE_FWD ? 'f' : 'd')) return false;
  if (dtype != SSIP_BF16 || !desc_ok(d) || d->R != 3 || d->S != 3 || d->stride != 1 || d->pad != 1 ||
      d->P != d->H || d->Q != d->W)
    return false;
  const int redc = mode == MODE_FWD ? d->C : d->K;
  const int cols = mode == MODE_FWD ? d->K : d->C;
  if (redc != 64 || cols % 64 != 0) return false;
  int TR = 0;
  for (int tr = std::min(d->H, 256 / (d->W + 2)); tr >= 1; --tr)  // TR (W+2) GEMM rows <= 256
    if (d->H % tr == 0 && (tr + 2) * (d->W + 2) <= HALO_XBUF / 128) {
      TR = tr;
      break;
    }
  if (TR == 0 || TR * d->W < 128) return false;  // short tiles: the implicit-GEMM kernels do better
  const long pix = (long)d->N * d->H * d->W;
  if (pix * 64 * 2 >= (1l << 31) || pix * cols * 2 >= (1l << 31)) return false;
  hp.TR = TR;
  hp.cols = cols;
  hp.tiles = (int)((long)d->N * d->H / TR);
  hp.units = hp.tiles * (cols / 64);
  // persistent: one workgroup per CU
  hp.G = std::min(hp.units, device_cus());
  return true;
}

// ---- stem path (conv_stem_halo_kernel): the pre-padded 7x7 / stride 2 stem
static bool stem_plan(const ssip_conv_desc* d, int dtype, HaloPlan& hp) {
  const char* e = getenv("SSIP_HALO");
  if (e && e[0] == '0') return false;
  const char* f = getenv("SSIP_CONV_FORCE");
  if (f && f[0] == 'f') return false;
  if (dtype != SSIP_BF16 || !desc_ok(d) || d->C != 4 || d->R != 7 || d->S != 8 || d->stride != 2 || d->pad != 0 ||
      d->K % 64 != 0 || d->Q > STEM_QP || d->P % STEM_TR != 0 || d->W % 2 != 0 ||
      STEM_XROWS * d->W * 8 > STEM_XBUF || d->H < 2 * (d->P - 1) + 7)
    return false;
  const long ib = (long)d->N * d->H * d->W * 8, ob = (long)d->N * d->P * d->Q * d->K * 2;
  if (ib >= (1l << 31) || ob >= (1l << 31)) return false;
  hp.TR = STEM_TR;
  hp.cols = d->K;
  hp.tiles = d->N * d->P / STEM_TR;
  hp.units = hp.tiles * (d->K / 64);
  hp.G = std::min(hp.units, 2 * device_cus());  // 62 KiB of LDS: two workgroups per CU
  return true;
}

static int launch_stem_halo(const ssip_conv_desc* d, const HaloPlan& hp, const void* X, const void* Wt, void* out,
                            float* partial, hipStream_t st) {
  StemArgs s;
  s.X = static_cast<const __bf16*>(X);
  s.Wt = static_cast<const __bf16*>(Wt);
  s.out = static_cast<__bf16*>(out);
  s.partial = partial;
  s.x_bytes = (uint32_t)((long)d->N * d->H * d->W * 8);
  s.w_bytes = (uint32_t)((long)d->K * 7 * 8 * 4 * 2);
  s.o_bytes = (uint32_t)((long)d->N * d->P * d->Q * d->K * 2);
  s.N = d->N; s.H = d->H; s.W = d->W; s.P = d->P; s.Q = d->Q; s.Ncols = d->K;
  s.tiles = hp.tiles; s.units = hp.units;
  s.diag = 0;
  if (const char* dg = getenv("SSIP_STEM_DIAG")) s.diag = atoi(dg);
  SSIP_KLAUNCH((conv_stem_halo_kernel<4, 2>), dim3(hp.G), dim3(512), 0, st, s);
  return ::ssip::check_launch("conv_stem_halo");
}

// ---- halo WGRAD (conv_halo_wgrad_kernel): 3x3 / stride 1 / pad 1, C = K = 64, bf16
static bool halo_wg_plan(const ssip_conv_desc* d, int dtype, HaloPlan& hp) {
  const char* e = getenv("SSIP_HALO");
  if (e && e[0] == '0') return false;
  const char* f = getenv("SSIP_CONV_FORCE");
  if (f && f[0] == 'w') return false;
  if (dtype != SSIP_BF16 || !desc_ok(d) || d->R != 3 || d->S != 3 || d->stride != 1 || d->pad != 1 ||
      d->P != d->H || d->Q != d->W || d->C != 64 || d->K != 64)
    return false;
  const int Wp = d->W + 2;
  if (256 + 2 * Wp + 2 > HWG_XBUF / 128) return false;  // shifted reads stay inside the input image
  int TR = 0;
  for (int tr = std::min(d->H, 256 / Wp); tr >= 1; --tr)
    if (d->H % tr == 0 && (tr + 2) * Wp <= HWG_XBUF / 128) {
      TR = tr;
      break;
    }
  if (TR == 0 || TR * d->W < 128) return false;
  if ((long)d->N * d->H * d->W * 64 * 2 >= (1l << 31)) return false;
  hp.TR = TR;
  hp.cols = 576;
  hp.tiles = d->N * d->H / TR;
  hp.units = hp.tiles;
  hp.G = std::min(hp.tiles, device_cus());
  return true;
}

// ---- stem WGRAD (conv_stem_wgrad_kernel)
static bool stem_wg_plan(const ssip_conv_desc* d, int dtype, HaloPlan& hp) {
  const char* e = getenv("SSIP_HALO");
  if (e && e[0] == '0') return false;
  const char* f = getenv("SSIP_CONV_FORCE");
  if (f && f[0] == 'w') return false;
  if (!stem_plan(d, dtype, hp) || d->K != 64) return false;  // same geometry as the forward's kernel
  hp.G = std::min(hp.tiles, device_cus());
  hp.units = hp.tiles;
  return true;
}

struct HaloBnPost {
  const void* y;
  const uint8_t* bits;
  const float *mean, *invstd, *mscale, *mshift;
};

static int launch_halo(int mode, const ssip_conv_desc* d, const HaloPlan& hp, const void* X, const void* Wt,
                       void* out, const void* add, float* partial, hipStream_t st, const float* bias = nullptr,
                       int relu = 0, const HaloBnPost* bp = nullptr, const float* in_scale = nullptr,
                       const float* in_shift = nullptr, void* zout = nullptr) {
  HaloArgs h;
  memset(&h, 0, sizeof(h));
  if (bp) {
    h.py = static_cast<const __bf16*>(bp->y);
    h.pbits = bp->bits;
    h.pmean = bp->mean; h.pinvstd = bp->invstd; h.pmscale = bp->mscale; h.pmshift = bp->mshift;
    h.bits_bytes = (uint32_t)((long)d->N * d->H * d->W * hp.cols / 8);
  }
  h.bias = bias;
  h.relu = relu;
  h.X = static_cast<const __bf16*>(X);
  h.Wt = static_cast<const __bf16*>(Wt);
  h.out = static_cast<__bf16*>(out);
  h.add = static_cast<const __bf16*>(add);
  h.partial = partial;
  h.x_bytes = (uint32_t)((long)d->N * d->H * d->W * 64 * 2);
  h.w_bytes = (uint32_t)((long)hp.cols * 9 * 64 * 2);
  h.o_bytes = (uint32_t)((long)d->N * d->H * d->W * hp.cols * 2);
  h.N = d->N; h.H = d->H; h.W = d->W; h.Ncols = hp.cols;
  h.TR = hp.TR; h.tiles = hp.tiles; h.units = hp.units;
  h.flip = mode == MODE_DGRAD ? 1 : 0;
  if (const char* dg = getenv("SSIP_HALO_DIAG")) h.diag = atoi(dg);
  // 8 waves of 64x32 (16 waves of 32x32 were ~10 % faster in isolation but 3 %
  // slower in the step, where the side streams' kernels run beside them; 4
  // waves of 64x64 slower still: r3-variants branch)
  h.in_scale = in_scale;
  h.in_shift = in_shift;
  h.zout = static_cast<__bf16*>(zout);
  if (in_scale != nullptr)  // FWD over relu(bn(y)) of the layer below, formed in LDS
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, false, true>), dim3(hp.G), dim3(512), 0, st, h);
  else if (bp != nullptr && add == nullptr && bp->bits == nullptr)  // DGRAD + BN-backward reduction
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 1>), dim3(hp.G), dim3(512), 0, st, h);
  else if (bp != nullptr)
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 2>), dim3(hp.G), dim3(512), 0, st, h);
  else if (bias != nullptr && add != nullptr)  // folded eval BN epilogue
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, true, 0, true>), dim3(hp.G), dim3(512), 0, st, h);
  else if (bias != nullptr)
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, true>), dim3(hp.G), dim3(512), 0, st, h);
  else if (add != nullptr)
    SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, true>), dim3(hp.G), dim3(512), 0, st, h);
  else if (h.diag & 128) {
    // phase stamps (lab only): per workgroup, wave and tile {after the tile's
    // barrier, after the k-loop's vmcnt(0), after the epilogue}, written to
    // SSIP_HALO_STAMP_OUT as raw u64 [G][8][32][3]
    static unsigned long long* buf = nullptr;
    const size_t n = (size_t)hp.G * 8 * 32 * 3;
    if (buf == nullptr && hipMalloc(&buf, n * 8) != hipSuccess) return SSIP_ERR_LAUNCH;
    (void)hipMemsetAsync(buf, 0, n * 8, st);
    h.stamps = buf;
    // compile-time ablations (timing only, results wrong): diag 2 no MFMAs, diag 1 no output stores
    if ((h.diag & 3) == 3)
      SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, false, false, 7>), dim3(hp.G), dim3(512), 0, st, h);
    else if (h.diag & 2)
      SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, false, false, 3>), dim3(hp.G), dim3(512), 0, st, h);
    else if (h.diag & 1)
      SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, false, false, 5>), dim3(hp.G), dim3(512), 0, st, h);
    else
      SSIP_KLAUNCH((conv_halo_kernel<4, 2, false, 0, false, false, 1>), dim3(hp.G), dim3(512), 0, st, h);
    std::vector<unsigned long long> host(n);
    if (hipMemcpyAsync(host.data(), buf, n * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return SSIP_ERR_LAUNCH;
    const char* path = getenv("SSIP_HALO_STAMP_OUT");
    if (FILE* f = fopen(path ? path : "/tmp/halo_stamps.bin", "wb")) {
      fwrite(host.data(), 8, n, f);
      fclose(f);
    }
  } else
    SSIP_KLAUNCH((conv_halo_kernel<4, 2>), dim3(hp.G), dim3(512), 0, st, h);
  return ::ssip::check_launch("conv_halo");
}

// layer-1 WGRAD on conv_halo_wgrad_kernel + its slab reduce (in_scale: the
// input is y of the BN+ReLU below, transformed in LDS)
static int launch_halo_wgrad(const ssip_conv_desc* d, HaloPlan hp, const void* dy, const void* x, float* dw_kcrs,
                             int c_real, int s_real, int accumulate, void* workspace, int64_t workspace_bytes,
                             int max_workgroups, hipStream_t st, const float* in_scale, const float* in_shift) {
  if (max_workgroups > 0) hp.G = std::min(hp.G, max_workgroups);  // persistent: fewer CUs, more tiles each
  const int64_t hneed = (int64_t)hp.G * 64 * 576 * 4;
  SSIP_REQUIRE(workspace_bytes >= hneed, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
               (long long)workspace_bytes, (long long)hneed);
  HaloWgArgs h;
  h.X = static_cast<const __bf16*>(x);
  h.DY = static_cast<const __bf16*>(dy);
  h.slab = static_cast<float*>(workspace);
  h.x_bytes = (uint32_t)((long)d->N * d->H * d->W * 64 * 2);
  h.N = d->N; h.H = d->H; h.W = d->W; h.TR = hp.TR; h.tiles = hp.tiles;
  static const int spread = [] {
    const char* e = getenv("SSIP_HWG_SPREAD");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  h.spread = spread;
  h.in_scale = in_scale;
  h.in_shift = in_shift;
  if (in_scale != nullptr)
    SSIP_KLAUNCH(conv_halo_wgrad_kernel<true>, dim3(hp.G), dim3(512), 0, st, h);
  else
    SSIP_KLAUNCH(conv_halo_wgrad_kernel<false>, dim3(hp.G), dim3(512), 0, st, h);
  int rc = ::ssip::check_launch("conv_halo_wgrad");
  if (rc) return rc;
  const long total4 = 64L * 576 / 4;
  int lg = 0;
  while (lg < 6 && (2 << lg) <= hp.G && ((total4 << (lg + 1)) + 255) / 256 <= 1024) ++lg;
  const long blocks = (total4 + (256 >> lg) - 1) / (256 >> lg);
  SSIP_KLAUNCH(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)workspace, hp.G, 64, 576,
               c_real, 3, s_real, 64, 3, dw_kcrs, accumulate, lg);
  return ::ssip::check_launch("wgrad_reduce");
}

}  // namespace

extern "C" {

int64_t ssip_conv_fwd_partial_floats(const ssip_conv_desc* d) {
  // the partial-buffer size must not depend on dtype: size for the smaller (128-row) tiles
  Plan pl;
  if (plan_conv(MODE_FWD, d, 4, pl) != SSIP_OK) {
    if (plan_conv(MODE_FWD, d, 2, pl) != SSIP_OK) return -1;
  }
  int64_t n = (int64_t)ceil_div(pl.args.M, 128) * d->K * 3;
  HaloPlan hp;  // one record per (channel, workgroup) on the halo path
  if (halo_plan(MODE_FWD, d, SSIP_BF16, hp)) n = std::max(n, (int64_t)hp.G * HALO_WMW * d->K * 3);
  if (stem_plan(d, SSIP_BF16, hp)) n = std::max(n, (int64_t)hp.G * HALO_WMW * d->K * 3);
  // + the scratch of ssip_bn_finalize's split pass (the most records any
  // plan writes bounds the splits; the scratch starts behind the records)
  return n + fin_scratch_floats(d->K, n / (3 * d->K), 3);
}

int ssip_conv_fwd(const ssip_conv_desc* d, int dtype, const void* x, const void* w_krsc, void* y, float* bn_partial,
                  void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_FWD, d, elem_bytes_of(dtype), pl);
  if (rc) return rc;
  if (pl.stages > 0 && !pl.conv1 && d->R * d->S > 32) fallback_regstaged(pl);
  SSIP_REQUIRE(x && w_krsc && y, SSIP_ERR_ARG, "ssip_conv_fwd: null pointer");
  HaloPlan hp;
  if (halo_plan(MODE_FWD, d, dtype, hp))
    return launch_halo(MODE_FWD, d, hp, x, w_krsc, y, nullptr, bn_partial, (hipStream_t)stream);
  if (stem_plan(d, dtype, hp)) return launch_stem_halo(d, hp, x, w_krsc, y, bn_partial, (hipStream_t)stream);
  pl.args.A = x; pl.args.B = w_krsc; pl.args.out = y; pl.args.partial = bn_partial;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->H * d->W * d->C * 2);
  pl.args.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_FWD, T>(pl, (hipStream_t)stream));
}

// A 3x3 / pad-1 / stride-s conv and its block's 1x1 / pad-0 / stride-s
// downsample over the same input and output grid: one LDS-DMA launch when the
// conv takes a 2- or 3-stage ring kernel (else false: two launches).
static bool fwd_ds_plan(const ssip_conv_desc* d, const ssip_conv_desc* dds, int dtype, Plan& pl) {
  if (dtype != SSIP_BF16 || !desc_ok(d) || !desc_ok(dds) || getenv("SSIP_NO_FWD_DSFUSE")) return false;
  if (d->R != 3 || d->S != 3 || d->pad != 1 || dds->R != 1 || dds->S != 1 || dds->pad != 0 ||
      dds->stride != d->stride || dds->N != d->N || dds->H != d->H || dds->W != d->W || dds->C != d->C ||
      dds->K != d->K || dds->P != d->P || dds->Q != d->Q || d->C % 64 != 0)
    return false;
  HaloPlan hp;
  if (halo_plan(MODE_FWD, d, dtype, hp) || stem_plan(d, dtype, hp)) return false;
  if (plan_conv(MODE_FWD, d, 2, pl) != SSIP_OK || pl.conv1) return false;
  return pl.stages == 2 || pl.stages == 3;
}

int ssip_conv_fwd_ds_partial_tiles(const ssip_conv_desc* d, const ssip_conv_desc* dds, int dtype) {
  Plan pl;
  if (fwd_ds_plan(d, dds, dtype, pl)) return ceil_div(pl.args.M, pl.bm);
  return ssip_conv_fwd_partial_tiles(dds, dtype);
}

int ssip_conv_fwd_ds(const ssip_conv_desc* d, const ssip_conv_desc* dds, int dtype, const void* x, const void* w_krsc,
                     void* y, float* bn_partial, const void* wds_kc, void* y_ds, float* bn_partial_ds, void* stream) {
  SSIP_REQUIRE(x && w_krsc && y && wds_kc && y_ds, SSIP_ERR_ARG, "ssip_conv_fwd_ds: null pointer");
  Plan pl;
  if (!fwd_ds_plan(d, dds, dtype, pl)) {  // two launches
    int rc = ssip_conv_fwd(d, dtype, x, w_krsc, y, bn_partial, stream);
    if (rc) return rc;
    return ssip_conv_fwd(dds, dtype, x, wds_kc, y_ds, bn_partial_ds, stream);
  }
  SSIP_REQUIRE((bn_partial == nullptr) == (bn_partial_ds == nullptr), SSIP_ERR_ARG,
               "ssip_conv_fwd_ds: both or neither BN partial buffers");
  ConvArgs& a = pl.args;
  a.A = x; a.B = w_krsc; a.out = y; a.partial = bn_partial;
  a.a_bytes = (uint32_t)((long)d->N * d->H * d->W * d->C * 2);
  a.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  const int T1 = (int)pl.grid.x;
  a.fwd_tiles1 = T1;
  a.Bds = wds_kc; a.out_ds = y_ds; a.partial_ds = bn_partial_ds;
  a.bds_bytes = (uint32_t)((long)d->K * d->C * 2);
  a.stat_tiles_m = ceil_div(a.M, pl.bm);
  pl.grid = dim3(2 * T1, 1, 1);
  return launch_conv<MODE_FWD, __bf16>(pl, (hipStream_t)stream);
}

int ssip_conv_fwd_partial_tiles(const ssip_conv_desc* d, int dtype) {
  HaloPlan hp;
  if (halo_plan(MODE_FWD, d, dtype, hp)) return hp.G * HALO_WMW;
  if (stem_plan(d, dtype, hp)) return hp.G * HALO_WMW;
  Plan pl;
  if (plan_conv(MODE_FWD, d, elem_bytes_of(dtype), pl) != SSIP_OK) return -1;
  if (pl.stages > 0 && !pl.conv1 && d->R * d->S > 32) fallback_regstaged(pl);
  return ceil_div(pl.args.M, pl.bm);
}

int ssip_conv_fwd_bias(const ssip_conv_desc* d, int dtype, const void* x, const void* w_krsc, const float* bias,
                       const void* residual, int relu, void* y, void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_FWD, d, elem_bytes_of(dtype), pl);
  if (rc) return rc;
  SSIP_REQUIRE(!pl.conv1, SSIP_ERR_ARG, "ssip_conv_fwd_bias: not for the C = 4 stem");
  SSIP_REQUIRE(x && w_krsc && bias && y, SSIP_ERR_ARG, "ssip_conv_fwd_bias: null pointer");
  if (pl.stages > 0 && d->R * d->S > 32) fallback_regstaged(pl);
  HaloPlan hp;
  if (halo_plan(MODE_FWD, d, dtype, hp))
    return launch_halo(MODE_FWD, d, hp, x, w_krsc, y, residual, nullptr, (hipStream_t)stream, bias, relu ? 1 : 0);
  pl.args.A = x; pl.args.B = w_krsc; pl.args.out = y; pl.args.partial = nullptr;
  pl.args.add = residual; pl.args.bias = bias; pl.args.relu = relu ? 1 : 0;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->H * d->W * d->C * 2);
  pl.args.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_FWD, T>(pl, (hipStream_t)stream));
}

int ssip_conv_dgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, void* dx,
                    const void* dx_add, void* stream) {
  Plan pl;
  int rc = plan_conv(MODE_DGRAD, d, elem_bytes_of(dtype), pl);
  if (rc) return rc;
  phase_split(pl, d);
  if (pl.stages > 0 && ((d->stride != 1 && !pl.args.phased) || d->R * d->S > 32)) fallback_regstaged(pl);
  SSIP_REQUIRE(dy && w_crsk && dx, SSIP_ERR_ARG, "ssip_conv_dgrad: null pointer");
  HaloPlan hp;
  if (halo_plan(MODE_DGRAD, d, dtype, hp))
    return launch_halo(MODE_DGRAD, d, hp, dy, w_crsk, dx, dx_add, nullptr, (hipStream_t)stream);
  pl.args.A = dy; pl.args.B = w_crsk; pl.args.out = dx; pl.args.add = dx_add;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->P * d->Q * d->K * 2);
  pl.args.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_DGRAD, T>(pl, (hipStream_t)stream));
}

int ssip_conv_dgrad_ds(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, const void* dy_ds,
                       const void* wds_ck, void* dx, void* stream) {
  SSIP_REQUIRE(desc_ok(d) && dy && w_crsk && dy_ds && wds_ck && dx, SSIP_ERR_ARG, "ssip_conv_dgrad_ds: bad arguments");
  SSIP_REQUIRE(d->H % d->stride == 0 && d->W % d->stride == 0 && d->P * d->stride == d->H &&
                   d->Q * d->stride == d->W, SSIP_ERR_ARG,
               "ssip_conv_dgrad_ds: the 1x1 downsample's output grid must equal the conv's (H, W divisible by stride)");
  ssip_conv_desc dd = *d;  // the block's 1x1 / stride downsample: same input, same output grid
  dd.R = 1; dd.S = 1; dd.pad = 0;
  Plan pl;
  int rc = plan_conv(MODE_DGRAD, d, elem_bytes_of(dtype), pl);
  if (rc) return rc;
  phase_split(pl, d);
  const bool fuse = pl.stages > 0 && pl.args.phased && d->R == 3 && d->S == 3 && d->pad == 1 && d->stride == 2;
  if (!fuse) {  // two passes: the conv's dgrad, then the downsample's accumulated in place
    rc = ssip_conv_dgrad(d, dtype, dy, w_crsk, dx, nullptr, stream);
    if (rc) return rc;
    return ssip_conv_dgrad(&dd, dtype, dy_ds, wds_ck, dx, dx, stream);
  }
  ConvArgs& a = pl.args;
  a.A = dy; a.B = w_crsk; a.out = dx; a.add = nullptr;
  a.a_bytes = (uint32_t)((long)d->N * d->P * d->Q * d->K * 2);
  a.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  a.A2 = dy_ds; a.B2 = wds_ck;
  a.a2_bytes = a.a_bytes;
  a.b2_bytes = (uint32_t)((long)d->K * d->C * 2);
  // phase (0, 0): h = 2i, w = 2j meet tap (1, 1) at dy pixel (i, j) -- the downsample's pixel
  SSIP_REQUIRE(a.phase[0].nr == 1 && a.phase[0].ns == 1 && a.phase[0].bh == 0 && a.phase[0].bw == 0, SSIP_ERR_ARG,
               "ssip_conv_dgrad_ds: unexpected phase (0, 0) geometry");
  a.ds_from = a.phase[0].ksteps;
  a.phase[0].ksteps += d->K / 64;
  set_phase_order(a);
  return launch_conv<MODE_DGRAD, __bf16>(pl, (hipStream_t)stream);
}

int64_t ssip_conv_dgrad_bn_partial_floats(const ssip_conv_desc* d) {
  Plan pl;
  if (plan_conv(MODE_DGRAD, d, 4, pl) != SSIP_OK) {
    if (plan_conv(MODE_DGRAD, d, 2, pl) != SSIP_OK) return -1;
  }
  long tiles = ceil_div(pl.args.M, 128);  // the LDS-DMA / register-staged paths: >= 128-row tiles
  HaloPlan hp;
  if (halo_plan(MODE_DGRAD, d, SSIP_BF16, hp)) tiles = std::max<long>(tiles, (long)hp.G * HALO_WMW);
  return tiles * d->C * 2 + fin_scratch_floats(d->C, tiles, 2);  // + ssip_bn_bwd_from_partials' split scratch
}

static int wgrad_implicit(Plan& pl, const ssip_conv_desc* d, int dtype, const void* dy, const void* x,
                          float* dw_kcrs, int c_real, int s_real, int accumulate, void* workspace, hipStream_t st);

// ssip_conv_*_bnrelu_in beyond the layer-1 halo geometry: the LDS-DMA ring
// kernels with the INBN operand transform, for bf16 stride-1 convs with
// 64 <= C <= GLDS_INBN_C input channels -- 1x1 / pad 0 (the ResNet-50
// bottleneck's conv3 over relu(bn2(y2))) with SSIP_BNRELU_GLDS bit 0, 3x3 /
// pad 1 with bit 1.  The transform keeps padding taps, rows past the grid
// and split tails zero.
// SSIP_BNRELU_GLDS: bit 0 the 1x1 / stride-1 form (default on: config 5,
// 60.23 vs 60.60 ms/step with the forward's z_out, profiles/r6_bnrelu_in_glds_lab.txt),
// bit 1 the 3x3 form (off: slower in both steps)
static int bnrelu_glds_mask() {
  const char* e = getenv("SSIP_BNRELU_GLDS");
  return e != nullptr ? atoi(e) : 1;
}

static bool glds_inbn_plan(int mode, const ssip_conv_desc* d, int dtype, Plan& pl, int budget = 0) {
  if (dtype != SSIP_BF16 || !desc_ok(d) || d->stride != 1 || d->C % 64 || d->C > GLDS_INBN_C || d->K % 64)
    return false;
  const int m = bnrelu_glds_mask();
  // the 1x1 form pays where the apply pass it removes is large: per launch it
  // wins at ResNet-50 layers 1-2 (>= 262,144 rows) and loses at layers 3-4,
  // where the conv is short and the in-ring transform is not hidden
  // (profiles/r6_bnrelu_in_glds_lab.txt); SSIP_BNRELU_GLDS_MINM overrides
  const char* me = getenv("SSIP_BNRELU_GLDS_MINM");
  const long min_rows = me != nullptr ? atol(me) : 262144l;
  if (d->R == 1 && (long)d->N * d->H * d->W < min_rows) return false;
  const bool g1 = d->R == 1 && d->S == 1 && d->pad == 0 && (m & 1);
  const bool g3 = d->R == 3 && d->S == 3 && d->pad == 1 && (m & 2);
  if (!g1 && !g3) return false;
  HaloPlan hp;
  if (halo_plan(MODE_FWD, d, dtype, hp)) return false;
  // (the wide budget tiles of SSIP_WGRAD_BIG have no INBN form: the budget's plain tiles)
  if (plan_conv(mode, d, 2, pl, budget, false) != SSIP_OK || pl.conv1 || pl.stages != 2) return false;
  bool ok = false;
#define SSIP_GLDS_INBN_EQ(BM_, BN_, WM_, WN_, ST_) \
  ok |= pl.bm == BM_ && pl.bn == BN_ && pl.wmw == WM_ && pl.wnw == WN_ && pl.stages == ST_;
  if (mode == MODE_WGRAD) {
    SSIP_GLDS_INBN_WG(SSIP_GLDS_INBN_EQ)
  } else {
    SSIP_GLDS_INBN_FD(SSIP_GLDS_INBN_EQ)
  }
#undef SSIP_GLDS_INBN_EQ
  return ok;
}

// the kernel ssip_conv_dgrad_bn runs: the halo kernel where it applies, else
// the implicit-GEMM kernels at their 128-row tiles (no phase split)
static int dgrad_bn_plan(const ssip_conv_desc* d, int dtype, Plan& pl, HaloPlan& hp, bool& halo) {
  int rc = plan_conv(MODE_DGRAD, d, elem_bytes_of(dtype), pl);
  if (rc) return rc;
  halo = halo_plan(MODE_DGRAD, d, dtype, hp);
  if (halo) return SSIP_OK;
  if (pl.stages > 0 && (d->stride != 1 || d->R * d->S > 32)) fallback_regstaged(pl);  // not phase-split here
  if (pl.stages > 0 && !getenv("SSIP_CONV_FORCE")) {  // the fused epilogue is built for the 128-row tiles only
    pl.bm = 128; pl.wmw = 4; pl.wnw = 2; pl.stages = 2;
    pl.bn = (pl.args.Ng % 128 == 0) ? 128 : 64;
    pl.args.tiles_n = ceil_div(pl.args.Ng, pl.bn);
    pl.grid = dim3(ceil_div(pl.args.M, pl.bm) * pl.args.tiles_n, 1, 1);
  }
  SSIP_REQUIRE(pl.bm >= 128, SSIP_ERR_ARG, "ssip_conv_dgrad_bn: partial sizing assumes >= 128-row tiles");
  return SSIP_OK;
}

int ssip_conv_dgrad_bn_partial_tiles(const ssip_conv_desc* d, int dtype) {
  Plan pl;
  HaloPlan hp;
  bool halo = false;
  if (dgrad_bn_plan(d, dtype, pl, hp, halo) != SSIP_OK) return -1;
  return halo ? hp.G * HALO_WMW : ceil_div(pl.args.M, pl.bm);
}

int ssip_conv_dgrad_bn(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, const void* dx_add,
                       const void* zmask, const uint8_t* mask_bits, const float* mscale, const float* mshift,
                       const void* y, const float* mean, const float* invstd, void* dpre, float* partial,
                       void* stream) {
  Plan pl;
  HaloPlan hp;
  bool halo = false;
  int rc = dgrad_bn_plan(d, dtype, pl, hp, halo);
  if (rc) return rc;
  SSIP_REQUIRE(dy && w_crsk && y && mean && invstd && dpre && partial, SSIP_ERR_ARG,
               "ssip_conv_dgrad_bn: null pointer");
  SSIP_REQUIRE(zmask || mask_bits || (mscale && mshift), SSIP_ERR_ARG,
               "ssip_conv_dgrad_bn: one ReLU-mask source (zmask, mask_bits or mscale+mshift) is required");
  SSIP_REQUIRE(d->C % 8 == 0, SSIP_ERR_ARG, "ssip_conv_dgrad_bn: C must be a multiple of 8");
  if (halo) {
    SSIP_REQUIRE(!zmask || mask_bits || (mscale && mshift), SSIP_ERR_ARG,
                 "ssip_conv_dgrad_bn: the halo kernel takes mask bits or the BN affine, not z");
    HaloBnPost bp;
    bp.y = y; bp.bits = mask_bits; bp.mean = mean; bp.invstd = invstd;
    bp.mscale = mask_bits ? nullptr : mscale; bp.mshift = mask_bits ? nullptr : mshift;
    return launch_halo(MODE_DGRAD, d, hp, dy, w_crsk, dpre, dx_add, partial, (hipStream_t)stream, nullptr, 0, &bp);
  }
  pl.args.A = dy; pl.args.B = w_crsk; pl.args.out = dpre; pl.args.add = dx_add;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->P * d->Q * d->K * 2);
  pl.args.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  pl.args.pmask = zmask; pl.args.pbits = zmask ? nullptr : mask_bits;
  pl.args.pmscale = (zmask || mask_bits) ? nullptr : mscale; pl.args.pmshift = (zmask || mask_bits) ? nullptr : mshift;
  pl.args.py = y; pl.args.pmean = mean; pl.args.pinvstd = invstd; pl.args.partial = partial;
  SSIP_DISPATCH_DTYPE(dtype, T, return launch_conv<MODE_DGRAD, T>(pl, (hipStream_t)stream));
}

int64_t ssip_conv_wgrad_workspace_bytes_budget(const ssip_conv_desc* d, int max_workgroups) {
  // max over dtypes so one workspace serves both
  Plan p2, p4;
  int64_t b = -1;
  if (max_workgroups < 0) return -1;
  if (plan_conv(MODE_WGRAD, d, 2, p2, max_workgroups) == SSIP_OK) b = (int64_t)p2.splits * p2.args.M * p2.args.Ng * 4;
  if (max_workgroups > 0 && plan_conv(MODE_WGRAD, d, 2, p2, max_workgroups, false) == SSIP_OK)  // the INBN form's plan
    b = std::max<int64_t>(b, (int64_t)p2.splits * p2.args.M * p2.args.Ng * 4);
  if (plan_conv(MODE_WGRAD, d, 4, p4, max_workgroups) == SSIP_OK)
    b = std::max<int64_t>(b, (int64_t)p4.splits * p4.args.M * p4.args.Ng * 4);
  HaloPlan hp;
  if (b >= 0 && halo_wg_plan(d, SSIP_BF16, hp)) b = std::max<int64_t>(b, (int64_t)hp.G * 64 * 576 * 4);
  if (b >= 0 && stem_wg_plan(d, SSIP_BF16, hp)) b = std::max<int64_t>(b, (int64_t)hp.G * 64 * 224 * 4);
  return b;
}

int64_t ssip_conv_wgrad_workspace_bytes(const ssip_conv_desc* d) { return ssip_conv_wgrad_workspace_bytes_budget(d, 0); }

int ssip_conv_wgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* x, float* dw_kcrs, int c_real,
                    int s_real, int accumulate, void* workspace, int64_t workspace_bytes, void* stream) {
  return ssip_conv_wgrad_budget(d, dtype, dy, x, dw_kcrs, c_real, s_real, accumulate, workspace, workspace_bytes, 0,
                                stream);
}

int ssip_conv_wgrad_budget(const ssip_conv_desc* d, int dtype, const void* dy, const void* x, float* dw_kcrs,
                           int c_real, int s_real, int accumulate, void* workspace, int64_t workspace_bytes,
                           int max_workgroups, void* stream) {
  SSIP_REQUIRE(max_workgroups >= 0, SSIP_ERR_ARG, "ssip_conv_wgrad_budget: negative budget");
  Plan pl;
  int rc = plan_conv(MODE_WGRAD, d, elem_bytes_of(dtype), pl, max_workgroups);
  if (rc) return rc;
  SSIP_REQUIRE(dy && x && dw_kcrs && workspace, SSIP_ERR_ARG, "ssip_conv_wgrad: null pointer");
  const int64_t need = (int64_t)pl.splits * pl.args.M * pl.args.Ng * 4;
  SSIP_REQUIRE(workspace_bytes >= need, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
               (long long)workspace_bytes, (long long)need);
  SSIP_REQUIRE(c_real >= 1 && c_real <= d->C && s_real >= 1 && s_real <= d->S, SSIP_ERR_ARG, "bad c_real/s_real");
  {
    HaloPlan hp;
    if (stem_wg_plan(d, dtype, hp)) {
      if (max_workgroups > 0) hp.G = std::min(hp.G, max_workgroups);
      const int64_t sneed = (int64_t)hp.G * 64 * 224 * 4;
      SSIP_REQUIRE(workspace_bytes >= sneed, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
                   (long long)workspace_bytes, (long long)sneed);
      StemWgArgs h;
      h.X = static_cast<const __bf16*>(x);
      h.DY = static_cast<const __bf16*>(dy);
      h.slab = static_cast<float*>(workspace);
      h.x_bytes = (uint32_t)((long)d->N * d->H * d->W * 8);
      h.dy_bytes = (uint32_t)((long)d->N * d->P * d->Q * 64 * 2);
      h.N = d->N; h.H = d->H; h.W = d->W; h.P = d->P; h.Q = d->Q; h.tiles = hp.tiles;
      hipStream_t st = (hipStream_t)stream;
      SSIP_KLAUNCH(conv_stem_wgrad_kernel, dim3(hp.G), dim3(512), 0, st, h);
      rc = ::ssip::check_launch("conv_stem_wgrad");
      if (rc) return rc;
      const long total4 = 64L * 224 / 4;
      int lg = 0;
      while (lg < 6 && (2 << lg) <= hp.G && ((total4 << (lg + 1)) + 255) / 256 <= 1024) ++lg;
      const long blocks = (total4 + (256 >> lg) - 1) / (256 >> lg);
      SSIP_KLAUNCH(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)workspace,
                         hp.G, 64, 224, c_real, d->R, s_real, d->C, d->S, dw_kcrs, accumulate, lg);
      return ::ssip::check_launch("wgrad_reduce");
    }
    if (halo_wg_plan(d, dtype, hp))
      return launch_halo_wgrad(d, hp, dy, x, dw_kcrs, c_real, s_real, accumulate, workspace, workspace_bytes,
                               max_workgroups, (hipStream_t)stream, nullptr, nullptr);
  }
  return wgrad_implicit(pl, d, dtype, dy, x, dw_kcrs, c_real, s_real, accumulate, workspace, (hipStream_t)stream);
}

// the split-K implicit-GEMM wgrad of a planned conv + its fixed-order slab
// reduce (ssip_conv_wgrad_budget; ssip_conv_wgrad_bnrelu_in with in_scale set)
static int wgrad_implicit(Plan& pl, const ssip_conv_desc* d, int dtype, const void* dy, const void* x,
                          float* dw_kcrs, int c_real, int s_real, int accumulate, void* workspace, hipStream_t st) {
  int rc;
  pl.args.A = dy; pl.args.B = x; pl.args.out = workspace;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->P * d->Q * d->K * 2);
  pl.args.b_bytes = (uint32_t)((long)d->N * d->H * d->W * d->C * 2);
  {
    const int PQ = d->P * d->Q, BKr = 64;  // LDS-DMA k-step rows (bf16)
    const int dn = BKr / PQ, rem = BKr % PQ;
    ConvArgs& g = pl.args;
    g.wg_dn = dn;
    g.wg_dp = rem / d->Q;
    g.wg_dq = rem % d->Q;
    g.wg_k0 = (dn * d->H * d->W + g.wg_dp * d->stride * d->W + g.wg_dq * d->stride) * d->C * 2;
    g.wg_e1 = (d->stride * d->W - d->Q * d->stride) * d->C * 2;
    g.wg_e2 = (d->H * d->W - d->P * d->stride * d->W) * d->C * 2;
  }
  SSIP_DISPATCH_DTYPE(dtype, T, rc = launch_conv<MODE_WGRAD, T>(pl, st));
  if (rc) return rc;
  const int RS = d->R * d->S;
  if (c_real == d->C && s_real == d->S && d->C % 64 == 0 && RS <= WGR_T_MAXRS && pl.args.Ng == RS * d->C &&
      pl.splits <= 32 && (long)d->K * (d->C / 64) >= 256 && (reinterpret_cast<uintptr_t>(dw_kcrs) & 15) == 0) {
    SSIP_KLAUNCH(wgrad_reduce_t_kernel, dim3((unsigned)(d->K * (d->C / 64))), dim3(256), 0, st,
                       (const float*)workspace, pl.splits, d->K, pl.args.Ng, d->C, RS, dw_kcrs, accumulate);
    return ::ssip::check_launch("wgrad_reduce_t");
  }
  const long total4 = (long)d->K * pl.args.Ng / 4;  // Ng = R*S*C: C % 32 == 0, or the stem's 7x8x4
  int lg = 0;  // split groups: double while splits allow and the grid stays within ~1024 workgroups
  while (lg < 6 && (2 << lg) <= pl.splits && ((total4 << (lg + 1)) + 255) / 256 <= 1024) ++lg;
  const long blocks = (total4 + (256 >> lg) - 1) / (256 >> lg);
  SSIP_KLAUNCH(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)workspace,
                     pl.splits, d->K, pl.args.Ng, c_real, d->R, s_real, d->C, d->S, dw_kcrs, accumulate, lg);
  return ::ssip::check_launch("wgrad_reduce");
}

int ssip_stem_bwd_wgrad_supported(const ssip_conv_desc* d, int dtype) {
  HaloPlan hp;
  return (stem_wg_plan(d, dtype, hp) && d->Q * 2 == 224 && d->P % 2 == 0) ? 1 : 0;
}

int ssip_stem_bwd_wgrad(const ssip_conv_desc* d, int dtype, const void* dpool, const uint8_t* idx, const void* y,
                        const void* x, const float* scale, const float* shift, const float* coef, float* dw_kcrs,
                        int c_real, int s_real, int accumulate, void* workspace, int64_t workspace_bytes,
                        void* stream) {
  HaloPlan hp;
  SSIP_REQUIRE(ssip_stem_bwd_wgrad_supported(d, dtype) && stem_wg_plan(d, dtype, hp), SSIP_ERR_ARG,
               "ssip_stem_bwd_wgrad: unsupported geometry");
  SSIP_REQUIRE(dpool && idx && y && x && scale && shift && coef && dw_kcrs && workspace, SSIP_ERR_ARG,
               "ssip_stem_bwd_wgrad: null pointer");
  SSIP_REQUIRE(c_real >= 1 && c_real <= d->C && s_real >= 1 && s_real <= d->S, SSIP_ERR_ARG, "bad c_real/s_real");
  const int64_t need = (int64_t)hp.G * 64 * 224 * 4;
  SSIP_REQUIRE(workspace_bytes >= need, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
               (long long)workspace_bytes, (long long)need);
  const int P2 = (d->P + 2 - 3) / 2 + 1, Q2 = (d->Q + 2 - 3) / 2 + 1;  // the 3x3 / 2 / 1 max-pool
  StemBwArgs h;
  h.X = static_cast<const __bf16*>(x);
  h.Y = static_cast<const __bf16*>(y);
  h.DP = static_cast<const __bf16*>(dpool);
  h.IX = idx;
  h.scale = scale; h.shift = shift; h.coef = coef;
  h.slab = static_cast<float*>(workspace);
  h.x_bytes = (uint32_t)((long)d->N * d->H * d->W * 8);
  h.y_bytes = (uint32_t)((long)d->N * d->P * d->Q * 64 * 2);
  h.dp_bytes = (uint32_t)((long)d->N * P2 * Q2 * 64 * 2);
  h.ix_bytes = (uint32_t)((long)d->N * P2 * Q2 * 64);
  h.N = d->N; h.H = d->H; h.W = d->W; h.P = d->P; h.Q = d->Q; h.P2 = P2; h.Q2 = Q2; h.tiles = hp.tiles;
  hipStream_t st = (hipStream_t)stream;
  SSIP_KLAUNCH(conv_stem_bwd_wgrad2_kernel, dim3(hp.G), dim3(768), 0, st, h);
  int rc = ::ssip::check_launch("conv_stem_bwd_wgrad");
  if (rc) return rc;
  const long total4 = 64L * 224 / 4;
  int lg = 0;
  while (lg < 6 && (2 << lg) <= hp.G && ((total4 << (lg + 1)) + 255) / 256 <= 1024) ++lg;
  const long blocks = (total4 + (256 >> lg) - 1) / (256 >> lg);
  SSIP_KLAUNCH(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)workspace, hp.G,
                     64, 224, c_real, d->R, s_real, d->C, d->S, dw_kcrs, accumulate, lg);
  return ::ssip::check_launch("wgrad_reduce");
}


int ssip_conv_bnrelu_in_supported(const ssip_conv_desc* d, int dtype) {
  HaloPlan hp, hw;
  if (halo_plan(MODE_FWD, d, dtype, hp) && halo_wg_plan(d, dtype, hw)) return 1;
  Plan pf, pw;
  return (glds_inbn_plan(MODE_FWD, d, dtype, pf) && glds_inbn_plan(MODE_WGRAD, d, dtype, pw)) ? 1 : 0;
}

int ssip_conv_fwd_bnrelu_in(const ssip_conv_desc* d, int dtype, const void* y_in, const float* in_scale,
                            const float* in_shift, const void* w_krsc, void* y, float* bn_partial, void* z_out,
                            void* stream) {
  HaloPlan hp;
  SSIP_REQUIRE(ssip_conv_bnrelu_in_supported(d, dtype), SSIP_ERR_ARG,
               "ssip_conv_fwd_bnrelu_in: unsupported geometry (ssip_conv_bnrelu_in_supported)");
  SSIP_REQUIRE(y_in && in_scale && in_shift && w_krsc && y, SSIP_ERR_ARG, "ssip_conv_fwd_bnrelu_in: null pointer");
  if (halo_plan(MODE_FWD, d, dtype, hp))
    return launch_halo(MODE_FWD, d, hp, y_in, w_krsc, y, nullptr, bn_partial, (hipStream_t)stream, nullptr, 0,
                       nullptr, in_scale, in_shift, z_out);
  Plan pl;
  SSIP_REQUIRE(glds_inbn_plan(MODE_FWD, d, dtype, pl), SSIP_ERR_ARG,
               "ssip_conv_fwd_bnrelu_in: no LDS-DMA BN+ReLU-in plan");
  SSIP_REQUIRE(z_out == nullptr || (d->R == 1 && d->S == 1 && d->pad == 0), SSIP_ERR_ARG,
               "ssip_conv_fwd_bnrelu_in: z_out on the halo geometry and 1x1 convs only");
  pl.args.zout = z_out;
  pl.args.A = y_in; pl.args.B = w_krsc; pl.args.out = y; pl.args.partial = bn_partial;
  pl.args.a_bytes = (uint32_t)((long)d->N * d->H * d->W * d->C * 2);
  pl.args.b_bytes = (uint32_t)((long)d->K * d->R * d->S * d->C * 2);
  pl.args.in_scale = in_scale; pl.args.in_shift = in_shift;
  return launch_glds<MODE_FWD>(pl, (hipStream_t)stream);
}

int ssip_conv_wgrad_bnrelu_in(const ssip_conv_desc* d, int dtype, const void* dy, const void* y_in,
                              const float* in_scale, const float* in_shift, float* dw_kcrs, int accumulate,
                              void* workspace, int64_t workspace_bytes, int max_workgroups, void* stream) {
  HaloPlan hp;
  SSIP_REQUIRE(ssip_conv_bnrelu_in_supported(d, dtype), SSIP_ERR_ARG,
               "ssip_conv_wgrad_bnrelu_in: unsupported geometry (ssip_conv_bnrelu_in_supported)");
  SSIP_REQUIRE(dy && y_in && in_scale && in_shift && dw_kcrs && workspace && max_workgroups >= 0, SSIP_ERR_ARG,
               "ssip_conv_wgrad_bnrelu_in: bad arguments");
  if (halo_wg_plan(d, dtype, hp))
    return launch_halo_wgrad(d, hp, dy, y_in, dw_kcrs, d->C, d->S, accumulate, workspace, workspace_bytes,
                             max_workgroups, (hipStream_t)stream, in_scale, in_shift);
  Plan pl;
  SSIP_REQUIRE(glds_inbn_plan(MODE_WGRAD, d, dtype, pl, max_workgroups), SSIP_ERR_ARG,
               "ssip_conv_wgrad_bnrelu_in: no LDS-DMA BN+ReLU-in plan under this budget");
  const int64_t need = (int64_t)pl.splits * pl.args.M * pl.args.Ng * 4;
  SSIP_REQUIRE(workspace_bytes >= need, SSIP_ERR_WORKSPACE, "wgrad workspace too small: %lld < %lld",
               (long long)workspace_bytes, (long long)need);
  pl.args.in_scale = in_scale; pl.args.in_shift = in_shift;
  return wgrad_implicit(pl, d, dtype, dy, y_in, dw_kcrs, d->C, d->S, accumulate, workspace, (hipStream_t)stream);
}

/* Which kernel a conv pass selects for this geometry (tests / tuning): writes a
 * NUL-terminated name such as "glds<fwd,256x256,4x2,2>" or "halo<fwd>" into buf. */
int ssip_conv_kernel_name(int mode, const ssip_conv_desc* d, int dtype, char* buf, int buflen) {
  return ssip_conv_kernel_name_budget(mode, d, dtype, 0, buf, buflen);
}

int ssip_conv_kernel_name_budget(int mode, const ssip_conv_desc* d, int dtype, int max_workgroups, char* buf,
                                 int buflen) {
  SSIP_REQUIRE(buf && buflen > 0, SSIP_ERR_ARG, "ssip_conv_kernel_name: no buffer");
  SSIP_REQUIRE(max_workgroups >= 0, SSIP_ERR_ARG, "ssip_conv_kernel_name_budget: negative budget");
  SSIP_REQUIRE(mode >= 0 && mode <= 2, SSIP_ERR_ARG, "ssip_conv_kernel_name: mode must be 0 (fwd), 1 (dgrad), 2 (wgrad)");
  static const char* mname[3] = {"fwd", "dgrad", "wgrad"};
  const int m = mode == 0 ? MODE_FWD : mode == 1 ? MODE_DGRAD : MODE_WGRAD;
  HaloPlan hp;
  if (m == MODE_FWD && halo_plan(MODE_FWD, d, dtype, hp)) {
    snprintf(buf, buflen, "halo<fwd,TR=%d,G=%d>", hp.TR, hp.G);
    return SSIP_OK;
  }
  if (m == MODE_FWD && stem_plan(d, dtype, hp)) {
    snprintf(buf, buflen, "stem_halo<fwd,G=%d>", hp.G);
    return SSIP_OK;
  }
  if (m == MODE_DGRAD && halo_plan(MODE_DGRAD, d, dtype, hp)) {
    snprintf(buf, buflen, "halo<dgrad,TR=%d,G=%d>", hp.TR, hp.G);
    return SSIP_OK;
  }
  if (m == MODE_WGRAD && stem_wg_plan(d, dtype, hp)) {
    snprintf(buf, buflen, "stem_wgrad<G=%d>", max_workgroups > 0 ? std::min(hp.G, max_workgroups) : hp.G);
    return SSIP_OK;
  }
  if (m == MODE_WGRAD && halo_wg_plan(d, dtype, hp)) {
    snprintf(buf, buflen, "halo_wgrad<TR=%d,G=%d>", hp.TR, max_workgroups > 0 ? std::min(hp.G, max_workgroups) : hp.G);
    return SSIP_OK;
  }
  Plan pl;
  int rc = plan_conv(m, d, elem_bytes_of(dtype), pl, m == MODE_WGRAD ? max_workgroups : 0);
  if (rc) return rc;
  if (m == MODE_FWD && pl.stages > 0 && !pl.conv1 && d->R * d->S > 32) fallback_regstaged(pl);
  if (m == MODE_DGRAD) {
    phase_split(pl, d);
    if (pl.stages > 0 && ((d->stride != 1 && !pl.args.phased) || d->R * d->S > 32)) fallback_regstaged(pl);
  }
  snprintf(buf, buflen, "%s<%s,%dx%d,%dx%d,%d%s%s,splits=%d>", pl.stages > 0 ? "glds" : "regstaged", mname[mode],
           pl.bm, pl.bn, pl.wmw, pl.wnw, pl.stages, pl.conv1 ? ",stem" : "", pl.args.phased ? ",phased" : "",
           pl.splits);
  return SSIP_OK;
}

}  // extern "C"
