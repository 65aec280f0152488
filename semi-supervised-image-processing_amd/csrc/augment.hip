// Image input pipeline on the GPU: PIL-exact resize -> flip -> rotate ->
// ToTensor -> Normalize, writing the stem conv's NHWC4 input directly.
//
// Reference transforms (run on CPU DataLoader workers in the reference):
//   train: Resize((S,S)) -> RandomHorizontalFlip -> RandomRotation(10)
//          -> ToTensor -> Normalize(ImageNet)   src/training/common.py:96-119
//   eval : Resize((S,S)) -> ToTensor -> Normalize            (same file)
//   extraction: Resize(256) -> CenterCrop(224) -> ToTensor -> Normalize
//                                           src/feature_extraction.py:184-207
// The arithmetic is Pillow's (torchvision delegates PIL images to it):
//   * Resize BILINEAR = separable antialiased triangle filter with 22-bit
//     fixed-point coefficients, horizontal pass first, uint8 clip between
//     passes (the coefficient tables are built on the host, bit-identical to
//     Pillow's precompute_coeffs/normalize_coeffs_8bpc);
//   * rotate(NEAREST, expand=False, fill 0) = Pillow's 16.16 fixed-point
//     affine walk (coefficients a0,a1,a3,a4,xo,yo computed on the host);
//   * ToTensor = u8 / 255 (f32), Normalize = (x - mean) / std (f32).
// With T = float the output is bit-identical to torchvision's CPU pipeline.
// Optional per-sample photometric jitter and cutout implement the "strong"
// view of the consistency step (a build extension; identity by default).
#include "ssip_common.h"

namespace {

template <typename T>
struct __attribute__((aligned(4 * sizeof(T)))) Vec4Px {
  T v[4];
};

// tmp[b][row][xo][ch] = clip8(sum_t src[b][row][xmin+t][ch] * k[xo][t] >> 22)
__global__ void resize_h_kernel(int B, const uint8_t* __restrict__ src, long src_bstride, int Hs, int Ws, int Wo,
                                int ksize, const int* __restrict__ bounds, const int* __restrict__ coeffs,
                                uint8_t* __restrict__ tmp) {
  const long total = (long)B * Hs * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int xo = (int)(i % Wo);
    const long t = i / Wo;
    const int row = (int)(t % Hs);
    const int b = (int)(t / Hs);
    const int xmin = bounds[2 * xo], xn = bounds[2 * xo + 1];
    const uint8_t* s = src + b * src_bstride + ((long)row * Ws + xmin) * 3;
    const int* k = coeffs + (long)xo * ksize;
    int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int x = 0; x < xn; ++x) {
      const int kx = k[x];
      s0 += (int)s[3 * x + 0] * kx;
      s1 += (int)s[3 * x + 1] * kx;
      s2 += (int)s[3 * x + 2] * kx;
    }
    uint8_t* o = tmp + i * 3;
    o[0] = (uint8_t)min(max(s0 >> 22, 0), 255);
    o[1] = (uint8_t)min(max(s1 >> 22, 0), 255);
    o[2] = (uint8_t)min(max(s2 >> 22, 0), 255);
  }
}

constexpr int AUG_ROWS = 4;  // output rows per workgroup (round 2: 46.7 -> 34.2 us per launch vs one row)

template <typename T>
__global__ void augment_kernel(int B, const uint8_t* __restrict__ src, long src_bstride, int src_h, int src_w,
                               int Hr, int Wr, int Ho, int Wo, int cx, int cy, int ksize_v,
                               const int* __restrict__ bounds_v, const int* __restrict__ coeffs_v,
                               const ssip_aug_param* __restrict__ params, float m0, float m1, float m2, float s0,
                               float s1, float s2, int opad, int rows, T* __restrict__ out) {
  // `rows` output rows per workgroup (grid ceil(Hp / rows) x B): sample index
  // and row are workgroup-uniform (the sample's parameters are scalar loads),
  // no 64-bit index division per pixel; several rows per workgroup amortise
  // the wave launch over more than one pixel per thread
  const int Hp = Ho + 2 * opad, Wp = Wo + 2 * opad;
  const int b = (int)blockIdx.y;
  const ssip_aug_param pa = params ? params[b] : ssip_aug_param{};
  const int yp0 = (int)blockIdx.x * rows;
  const int yp1 = min(Hp, yp0 + rows);
  // ToTensor (+ photometric jitter, cutout) + Normalize of one in-image pixel
  auto emit = [&](long i, bool inside, int u0, int u1, int u2, int xr, int yr) {
    float v[3] = {0.f, 0.f, 0.f};
    if (inside) {
      v[0] = (float)u0 / 255.f;
      v[1] = (float)u1 / 255.f;
      v[2] = (float)u2 / 255.f;
    }
    if (pa.photometric) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float w = v[c] * pa.brightness;
        w = (w - 0.5f) * pa.contrast + 0.5f;
        v[c] = fminf(fmaxf(w, 0.f), 1.f);
      }
    }
    if (xr >= pa.cut_x0 && xr < pa.cut_x1 && yr >= pa.cut_y0 && yr < pa.cut_y1) v[0] = v[1] = v[2] = 0.5f;
    Vec4Px<T> o;
    o.v[0] = from_f32<T>((v[0] - m0) / s0);
    o.v[1] = from_f32<T>((v[1] - m1) / s1);
    o.v[2] = from_f32<T>((v[2] - m2) / s2);
    o.v[3] = from_f32<T>(0.f);
    *reinterpret_cast<Vec4Px<T>*>(out + i * 4) = o;
  };
  auto zero = [&](long i) {  // the zero border of a pre-padded stem input
    Vec4Px<T> z;
#pragma unroll
    for (int c = 0; c < 4; ++c) z.v[c] = from_f32<T>(0.f);
    *reinterpret_cast<Vec4Px<T>*>(out + i * 4) = z;
  };
  const uint8_t* sb = src + b * src_bstride;
  if (ksize_v == 0 && rows == AUG_ROWS) {
    // no vertical filter (the resize is the identity or horizontal only):
    // the source bytes of all of a thread's rows are loaded before any
    // arithmetic, so their round trips overlap instead of running one per row
    for (int xp = threadIdx.x; xp < Wp; xp += blockDim.x) {
      const int x = xp - opad;
      int u[AUG_ROWS][3], xrs[AUG_ROWS], yrs[AUG_ROWS];
      bool ins[AUG_ROWS], brd[AUG_ROWS];
#pragma unroll
      for (int r = 0; r < AUG_ROWS; ++r) {
        const int yp = yp0 + r, y = yp - opad;
        brd[r] = yp >= yp1 || x < 0 || x >= Wo || y < 0 || y >= Ho;
        const int xr = x + cx, yr = y + cy;
        int xin = xr, yin = yr;
        bool inside = !brd[r];
        if (pa.rotate) {
          const int xx = pa.xo + yr * pa.a1 + xr * pa.a0;
          const int yy = pa.yo + yr * pa.a4 + xr * pa.a3;
          xin = xx >> 16;
          yin = yy >> 16;
          inside = inside && xin >= 0 && xin < Wr && yin >= 0 && yin < Hr;
        }
        const int xs = pa.flip ? (Wr - 1 - xin) : xin;
        const uint8_t* q = sb + (inside ? ((long)yin * src_w + xs) * 3 : 0);
        u[r][0] = q[0];
        u[r][1] = q[1];
        u[r][2] = q[2];
        ins[r] = inside;
        xrs[r] = xr;
        yrs[r] = yr;
      }
#pragma unroll
      for (int r = 0; r < AUG_ROWS; ++r) {
        const int yp = yp0 + r;
        if (yp >= yp1) continue;
        const long i = ((long)b * Hp + yp) * Wp + xp;
        if (brd[r]) zero(i);
        else emit(i, ins[r], u[r][0], u[r][1], u[r][2], xrs[r], yrs[r]);
      }
    }
    return;
  }
  for (int yp = yp0; yp < yp1; ++yp)
  for (int xp = threadIdx.x; xp < Wp; xp += blockDim.x) {
    const int y = yp - opad;
    const long i = ((long)b * Hp + yp) * Wp + xp;
    const int x = xp - opad;
    if (x < 0 || x >= Wo || y < 0 || y >= Ho) {
      zero(i);
      continue;
    }
    const int xr = x + cx, yr = y + cy;
    int xin = xr, yin = yr;
    bool inside = true;
    if (pa.rotate) {
      const int xx = pa.xo + yr * pa.a1 + xr * pa.a0;
      const int yy = pa.yo + yr * pa.a4 + xr * pa.a3;
      xin = xx >> 16;
      yin = yy >> 16;
      inside = xin >= 0 && xin < Wr && yin >= 0 && yin < Hr;
    }
    int u[3] = {0, 0, 0};
    if (inside) {
      const int xs = pa.flip ? (Wr - 1 - xin) : xin;
      if (ksize_v > 0) {
        const int ymin = bounds_v[2 * yin], yn = bounds_v[2 * yin + 1];
        const int* k = coeffs_v + (long)yin * ksize_v;
        int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
        for (int q = 0; q < yn; ++q) {
          const uint8_t* p = sb + ((long)(ymin + q) * src_w + xs) * 3;
          a0 += (int)p[0] * k[q];
          a1 += (int)p[1] * k[q];
          a2 += (int)p[2] * k[q];
        }
        u[0] = min(max(a0 >> 22, 0), 255);
        u[1] = min(max(a1 >> 22, 0), 255);
        u[2] = min(max(a2 >> 22, 0), 255);
      } else {
        const uint8_t* p = sb + ((long)yin * src_w + xs) * 3;
        u[0] = p[0]; u[1] = p[1]; u[2] = p[2];
      }
    }
    emit(i, inside, u[0], u[1], u[2], xr, yr);
  }
  (void)src_h;
}

// f32 NCHW -> T NHWC with channel padding (zeros)
template <typename T>
__global__ void nchw_to_nhwc_kernel(int B, int C, int H, int W, int Cp, int opad, const float* __restrict__ x,
                                    T* __restrict__ out) {
  const int Hp = H + 2 * opad, Wp = W + 2 * opad;
  const long total = (long)B * Hp * Wp * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long t = i / Cp;
    const int w = (int)(t % Wp) - opad;
    const long t2 = t / Wp;
    const int h = (int)(t2 % Hp) - opad;
    const int b = (int)(t2 / Hp);
    const bool in = c < C && h >= 0 && h < H && w >= 0 && w < W;
    const float v = in ? x[(((long)b * C + c) * H + h) * W + w] : 0.f;
    out[i] = from_f32<T>(v);
  }
}

static int grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

int ssip_resize_h_u8(int B, const uint8_t* src, int64_t src_batch_stride, int Hs, int Ws, int Wo, int ksize,
                     const int* bounds, const int* coeffs, uint8_t* tmp, void* stream) {
  SSIP_REQUIRE(B > 0 && src && Hs > 0 && Ws > 0 && Wo > 0 && ksize > 0 && bounds && coeffs && tmp, SSIP_ERR_ARG,
               "ssip_resize_h_u8: bad arguments");
  const long total = (long)B * Hs * Wo;
  SSIP_KLAUNCH(resize_h_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, src,
                     (long)src_batch_stride, Hs, Ws, Wo, ksize, bounds, coeffs, tmp);
  return ::ssip::check_launch("resize_h_u8");
}

int ssip_augment_u8(int dtype, int B, const uint8_t* src, int64_t src_batch_stride, int src_h, int src_w, int Hr,
                    int Wr, int Ho, int Wo, int crop_x, int crop_y, int ksize_v, const int* bounds_v,
                    const int* coeffs_v, const ssip_aug_param* params, const float* mean3, const float* std3,
                    int out_pad, void* out, void* stream) {
  SSIP_REQUIRE(B > 0 && src && Hr > 0 && Wr > 0 && Ho > 0 && Wo > 0 && mean3 && std3 && out, SSIP_ERR_ARG,
               "ssip_augment_u8: bad arguments");
  SSIP_REQUIRE(crop_x >= 0 && crop_y >= 0 && crop_x + Wo <= Wr && crop_y + Ho <= Hr, SSIP_ERR_ARG,
               "ssip_augment_u8: crop window outside the resized image");
  SSIP_REQUIRE(src_w == Wr && (ksize_v > 0 ? (bounds_v && coeffs_v) : src_h == Hr), SSIP_ERR_ARG,
               "ssip_augment_u8: source geometry does not match the resize plan");
  SSIP_REQUIRE(out_pad >= 0 && out_pad <= 8, SSIP_ERR_ARG, "ssip_augment_u8: out_pad must be 0..8");
  SSIP_REQUIRE((long)B * (Ho + 2 * out_pad) < 65536l * 65536l && B < 65536, SSIP_ERR_ARG,
               "ssip_augment_u8: batch too large");
  const int wp = Wo + 2 * out_pad, hp = Ho + 2 * out_pad;
  const int rows = AUG_ROWS;
  const dim3 grid((unsigned)((hp + rows - 1) / rows), (unsigned)B);
  const dim3 block((unsigned)(wp >= 256 ? 256 : ((wp + 63) / 64) * 64));
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(augment_kernel<T>, grid, block, 0, (hipStream_t)stream, B, src,
                       (long)src_batch_stride, src_h, src_w, Hr, Wr, Ho, Wo, crop_x, crop_y, ksize_v, bounds_v,
                       coeffs_v, params, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], out_pad, rows,
                       (T*)out);
  });
  return ::ssip::check_launch("augment_u8");
}

int ssip_nchw_to_nhwc(int dtype, int B, int C, int H, int W, int Cp, int out_pad, const float* x, void* out,
                      void* stream) {
  SSIP_REQUIRE(B > 0 && C > 0 && Cp >= C && H > 0 && W > 0 && out_pad >= 0 && out_pad <= 8 && x && out,
               SSIP_ERR_ARG, "ssip_nchw_to_nhwc: bad arguments");
  const long total = (long)B * (H + 2 * out_pad) * (W + 2 * out_pad) * Cp;
  SSIP_DISPATCH_DTYPE(dtype, T, {
    SSIP_KLAUNCH(nchw_to_nhwc_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B, C, H, W,
                       Cp, out_pad, x, (T*)out);
  });
  return ::ssip::check_launch("nchw_to_nhwc");
}

}  // extern "C"
