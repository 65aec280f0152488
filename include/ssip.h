/*
 * ssip.h — C ABI of libssip_hip.so, the MI355X (gfx950) kernels behind the
 * semi-supervised ResNet-18 train / pseudo-label / eval / embedding path of
 * Septimus4/semi-supervised-image-processing.
 *
 * The reference has no FFI layer: its hot path is torchvision/torch ops
 * called from Python.  Each entry point below replaces the op the reference
 * reaches at the cited call site (paths relative to the reference repo):
 *
 *   model(inputs) / loss.backward()        src/training/common.py:380-382
 *     -> ssip_conv_fwd / _dgrad / _dgrad_bn / _wgrad, ssip_bn_*,
 *        ssip_stem_bn_pool_fwd / ssip_stem_pool_bn_bwd (bn1 -> relu -> maxpool),
 *        ssip_maxpool_*, ssip_avgpool_fc_*   (torchvision resnet18, :299-304)
 *     -> ssip_weight_prep_batch            (the conv weights each forward reads)
 *   criterion(outputs, labels)             src/training/common.py:381
 *     -> ssip_cross_entropy                (nn.CrossEntropyLoss, semi_supervised.py:111)
 *   optimizer.step()                       src/training/common.py:383
 *     -> ssip_adamw                        (optim.AdamW, semi_supervised.py:115-122)
 *   transform(PIL.Image)                   src/training/common.py:96-119,145,172,192
 *                                          src/feature_extraction.py:184-207,233-240
 *     -> ssip_resize_h_u8 + ssip_augment_u8
 *   softmax/max/threshold pseudo-labels    src/training/semi_supervised.py:57-66
 *     -> ssip_softmax_select
 *   (build extension, no reference) weak/strong consistency loss
 *     -> ssip_semi_loss
 *
 * Conventions
 *   - Every pointer is a device pointer unless documented otherwise; the
 *     caller owns all memory (kernels never allocate).  Scratch comes from a
 *     caller buffer sized by the matching *_workspace_bytes / *_floats query.
 *   - Activations are NHWC, element type selected by `dtype`
 *     (SSIP_F32 = parity path, SSIP_BF16 = throughput path); all
 *     accumulation, BatchNorm statistics, weight gradients, optimizer state
 *     and logits are fp32.
 *   - `stream` is a hipStream_t (NULL = default stream).  Calls are
 *     stream-ordered, do no host synchronisation and are safe to capture in
 *     a hipGraph.
 *   - Return 0 on success or a negative SSIP_ERR_* code;
 *     ssip_last_error() returns a thread-local message.  Nothing throws.
 */
#ifndef SSIP_H_
#define SSIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SSIP_ABI_VERSION 14

enum ssip_dtype { SSIP_F32 = 0, SSIP_BF16 = 1 };
enum ssip_status { SSIP_OK = 0, SSIP_ERR_ARG = -1, SSIP_ERR_LAUNCH = -2, SSIP_ERR_WORKSPACE = -3 };

const char* ssip_last_error(void);
int ssip_version(void);

/* ------------------------------------------------------------------------
 * Convolution as implicit GEMM on MFMA (torchvision nn.Conv2d, bias=False).
 * x: [N][H][W][C], y/dy: [N][P][Q][K].  C and K must be multiples of 64
 * (bf16) / 32 (f32), or C == 4 with S == 8 (the padded 7x7 stem: channel 3
 * and filter column 7 are zero).
 * ---------------------------------------------------------------------- */
typedef struct ssip_conv_desc {
  int N, H, W, C; /* input (C = stored channels)          */
  int K;          /* output channels (multiple of 32)      */
  int R, S;       /* filter rows / stored filter columns   */
  int stride, pad;
  int P, Q;       /* output spatial size                   */
} ssip_conv_desc;

/* floats needed for the BatchNorm partial-statistics buffer of ssip_conv_fwd */
int64_t ssip_conv_fwd_partial_floats(const ssip_conv_desc* d);
/* number of M-tiles (records per channel) ssip_conv_fwd writes for this dtype */
int ssip_conv_fwd_partial_tiles(const ssip_conv_desc* d, int dtype);
/* y = conv(x, w); w_krsc: [K][R][S][C] in dtype.  bn_partial (nullable):
 * fp32 {count, sum, M2} per (channel, M-tile) consumed by ssip_bn_finalize. */
int ssip_conv_fwd(const ssip_conv_desc* d, int dtype, const void* x, const void* w_krsc, void* y, float* bn_partial,
                  void* stream);
/* dx = conv_transpose(dy, w) (+ dx_add, nullable); w_crsk: [C][R][S][K] */
int ssip_conv_dgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, void* dx,
                    const void* dx_add, void* stream);
/* dx = conv_transpose(dy, w) + conv_transpose_1x1/stride(dy_ds, w_ds): the
 * input gradient of a downsampling BasicBlock (conv1 3x3/2 and the 1x1/2
 * downsample share the block input; torchvision BasicBlock.forward).  wds_ck:
 * [C][K] (the downsample's CRSK copy).  The bf16 stride-2 3x3 case runs as ONE
 * phase-split launch (the downsample adds k-steps to the (even, even) phase);
 * anything else runs the two dgrads back to back. */
int ssip_conv_dgrad_ds(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, const void* dy_ds,
                       const void* wds_ck, void* dx, void* stream);
/* DGRAD with the next-lower BatchNorm's backward reduction fused into the
 * epilogue (replaces ssip_conv_dgrad + the reduce pass of ssip_bn_bwd):
 *   dpre = (dgrad(dy) + dx_add) * relu_mask                 [N][H][W][C]
 *   partial[c][tile] = { sum dpre, sum dpre * (y - mean[c]) * invstd[c] }
 * relu_mask (ABI 9: one source, first non-null wins): zmask > 0; bit c & 7 of
 * mask_bits[pixel * C / 8 + c / 8] (ssip_bn_apply's mask bits); or
 * fma(y, mscale, mshift) > 0 (a BN+ReLU with no residual: the forward's sign).
 * y / mean / invstd belong to the BN+ReLU that produced this conv's input;
 * dx_add (nullable) may alias dpre.  The 3x3 / stride-1 / 64-channel halo
 * kernel takes mask_bits or mscale+mshift (not zmask); its records are one per
 * (channel, workgroup, wave row).  Records per channel:
 * ssip_conv_dgrad_bn_partial_tiles; ssip_conv_dgrad_bn_partial_floats sizes the
 * buffer (records + the split finalize's scratch). */
int64_t ssip_conv_dgrad_bn_partial_floats(const ssip_conv_desc* d);
int ssip_conv_dgrad_bn_partial_tiles(const ssip_conv_desc* d, int dtype);
int ssip_conv_dgrad_bn(const ssip_conv_desc* d, int dtype, const void* dy, const void* w_crsk, const void* dx_add,
                       const void* zmask, const uint8_t* mask_bits, const float* mscale, const float* mshift,
                       const void* y, const float* mean, const float* invstd, void* dpre, float* partial,
                       void* stream);
/* Forward of a downsampling block's first conv (3x3, pad 1, stride s) and its
 * 1x1 / stride-s downsample (torchvision BasicBlock conv1 + downsample[0],
 * both `model(inputs)` at src/training/common.py:380) over the same input x:
 * one launch (ABI 8) -- the downsample's GEMM is the conv's tap-(1,1) column
 * block with W_ds [K][C] (KRSC of a 1x1 filter), so its short tiles run as
 * extra workgroups of the conv's grid.  Outputs and BN partial records as two
 * ssip_conv_fwd calls; the downsample's records per channel are
 * ssip_conv_fwd_ds_partial_tiles(d, dds, dtype) (both buffers sized by
 * ssip_conv_fwd_partial_floats of their own descriptor).  Falls back to two
 * launches where the conv does not take the LDS-DMA ring kernel. */
int ssip_conv_fwd_ds_partial_tiles(const ssip_conv_desc* d, const ssip_conv_desc* dds, int dtype);
int ssip_conv_fwd_ds(const ssip_conv_desc* d, const ssip_conv_desc* dds, int dtype, const void* x, const void* w_krsc,
                     void* y, float* bn_partial, const void* wds_kc, void* y_ds, float* bn_partial_ds, void* stream);
/* Eval-mode conv + folded BatchNorm (+ residual) (+ ReLU), one launch:
 *   y = act(conv(x, w') + bias[k] (+ residual)),  w' = w * scale[k] (ssip_wprep.kscale)
 * (torchvision BasicBlock / Bottleneck in eval mode: bn(conv(x)) with running
 * statistics is an affine map per output channel).  Not for the C == 4 stem. */
int ssip_conv_fwd_bias(const ssip_conv_desc* d, int dtype, const void* x, const void* w_krsc, const float* bias,
                       const void* residual, int relu, void* y, void* stream);
int64_t ssip_conv_wgrad_workspace_bytes(const ssip_conv_desc* d);
/* dw_kcrs (fp32, torchvision layout [K][c_real][R][s_real]) (+)= dW */
int ssip_conv_wgrad(const ssip_conv_desc* d, int dtype, const void* dy, const void* x, float* dw_kcrs, int c_real,
                    int s_real, int accumulate, void* workspace, int64_t workspace_bytes, void* stream);
/* The same with a workgroup budget for the split-K grid of the LDS-DMA wgrad
 * (ABI 10), for a wgrad that shares the chip with another stream's kernels
 * (the backward's side stream beside the dgrad / BN-backward chain); 0 =
 * ssip_conv_wgrad's full-chip grid.  By default a budget keeps the full-grid
 * tiles and sets their split count to ceil(max_workgroups / output tiles).
 * Only with $SSIP_WGRAD_BIG=1 (or 2: the K % 256 == 0 shapes only) does the
 * bf16 wgrad take 16-wave 256x256 / 128x256 tiles that fit one workgroup per
 * CU, at most max_workgroups of them (split count = floor(max_workgroups /
 * output tiles)); they measured faster alone but slower in the step.  The persistent
 * layer-1 and stem wgrads (one workgroup per CU, all of its LDS) run on at
 * most max_workgroups CUs.  Same result up to the fp32 order of the split /
 * slab sum (fixed for a budget).  The workspace a budget needs:
 * ssip_conv_wgrad_workspace_bytes_budget (ABI 12; budget 0 =
 * ssip_conv_wgrad_workspace_bytes) -- a budget may need more slab bytes than
 * the full-grid plan. */
int64_t ssip_conv_wgrad_workspace_bytes_budget(const ssip_conv_desc* d, int max_workgroups);
int ssip_conv_wgrad_budget(const ssip_conv_desc* d, int dtype, const void* dy, const void* x, float* dw_kcrs,
                           int c_real, int s_real, int accumulate, void* workspace, int64_t workspace_bytes,
                           int max_workgroups, void* stream);

/* ABI 13: a conv whose input is the ReLU(BatchNorm) of the layer below,
 * formed in the conv's LDS tile instead of a separate apply pass:
 *   x = relu(fma(y_in, in_scale[c], in_shift[c]))   (ssip_bn_apply's arithmetic)
 * Replaces the bn1 -> relu -> conv2 sequence of a torchvision BasicBlock /
 * Bottleneck (model(inputs) at src/training/common.py:380) where conv2 is the
 * layer-1 3x3 / stride 1 / pad 1, 64 -> 64 conv (the halo kernels); the
 * weight gradient of the same conv takes the same input.  Bit-identical to
 * ssip_bn_apply followed by ssip_conv_fwd / ssip_conv_wgrad.  z_out
 * (nullable, [N][H][W][C]): the forward also writes the transformed input
 * there (= ssip_bn_apply's output, each row once) for a later plain
 * ssip_conv_wgrad, which is cheaper than ssip_conv_wgrad_bnrelu_in beside
 * another stream.
 * ABI 14: also bf16 stride-1 convs on the LDS-DMA ring kernels with 64 <= C
 * <= 512 input channels -- 1x1 / pad 0 (the ResNet-50 Bottleneck's conv3 over
 * relu(bn2(y2)), $SSIP_BNRELU_GLDS bit 0, on by default from
 * $SSIP_BNRELU_GLDS_MINM = 262144 rows N*H*W up) and 3x3 / pad 1
 * (bit 1, off: slower in the steps): each wave transforms
 * the input pieces it DMA'd once they land, before the k-step's barrier;
 * padding taps and rows past the grid stay zero.  Same bits as ssip_bn_apply
 * + the plain conv.  z_out: also for the 1x1 form (the n-tile-0 workgroups
 * store each transformed piece), NULL for the 3x3 form. */
int ssip_conv_bnrelu_in_supported(const ssip_conv_desc* d, int dtype);
int ssip_conv_fwd_bnrelu_in(const ssip_conv_desc* d, int dtype, const void* y_in, const float* in_scale,
                            const float* in_shift, const void* w_krsc, void* y, float* bn_partial, void* z_out,
                            void* stream);
int ssip_conv_wgrad_bnrelu_in(const ssip_conv_desc* d, int dtype, const void* dy, const void* y_in,
                              const float* in_scale, const float* in_shift, float* dw_kcrs, int accumulate,
                              void* workspace, int64_t workspace_bytes, int max_workgroups, void* stream);

/* Name of the kernel a pass selects for this geometry (mode 0 = fwd,
 * 1 = dgrad, 2 = wgrad), e.g. "glds<fwd,256x256,4x2,2,splits=1>" or
 * "halo<dgrad,TR=4,G=256>": lets tests assert that a shape exercises the
 * production kernel the benchmark runs. */
int ssip_conv_kernel_name(int mode, const ssip_conv_desc* d, int dtype, char* buf, int buflen);
/* ABI 12: the kernel ssip_conv_wgrad_budget selects with that budget (mode 2;
 * fwd / dgrad ignore the budget) */
int ssip_conv_kernel_name_budget(int mode, const ssip_conv_desc* d, int dtype, int max_workgroups, char* buf,
                                 int buflen);

/* ------------------------------------------------------------------------
 * BatchNorm2d (train / eval) fused with ReLU and the residual add.
 * ---------------------------------------------------------------------- */
/* Batch statistics from `tiles` {count, sum, M2} records per channel
 * ([C][tiles][3], as ssip_conv_fwd writes them) -> mean / invstd / scale /
 * shift (+ the running statistics).  More than 2048 records per channel are
 * split over several workgroups (ABI 9) whose fp64 partial results use
 * ssip_bn_finalize_scratch_floats(C, tiles) floats behind the records (the
 * records themselves are not modified); ssip_conv_fwd_partial_floats
 * includes that tail. */
int64_t ssip_bn_finalize_scratch_floats(int C, int tiles);
int ssip_bn_finalize(int C, int tiles, float* partial, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, float momentum, float eps, int update_running,
                     float* mean_out, float* invstd_out, float* scale_out, float* shift_out, void* stream);
int ssip_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float* mean_out, float* invstd_out, float* scale_out,
                        float* shift_out, void* stream);
/* z = (relu)(y*scale[c] + shift[c] (+ residual)); M rows of C channels.
 * mask_bits (nullable): bit j of byte i = (z[8i + j] > 0), the ReLU mask the
 * backward reads instead of z (1/16 of its bytes in bf16). */
int ssip_bn_apply(int dtype, int64_t M, int C, const void* y, const float* scale, const float* shift,
                  const void* residual, int relu, void* z, uint8_t* mask_bits, void* stream);
/* z = (relu)(y*scale[c] + shift[c] + (y2*scale2[c] + shift2[c])): a block output
 * whose residual is the downsample's BN (bn2(conv2) + bn_ds(ds)) in one pass. */
int ssip_bn_apply2(int dtype, int64_t M, int C, const void* y, const float* scale, const float* shift,
                   const void* y2, const float* scale2, const float* shift2, int relu, void* z, uint8_t* mask_bits,
                   void* stream);
int64_t ssip_bn_bwd_partial_floats(int64_t M, int C);
/* dout = dz * (zmask > 0), or * mask bit (mask_bits as ssip_bn_apply writes them);
 * both NULL = no ReLU; dgamma/dbeta (+)= ...; dy = dBN(dout); dpre (nullable)
 * = dout.  coef: 3*C floats scratch. */
int ssip_bn_bwd(int dtype, int64_t M, int C, const void* dz, const void* zmask, const uint8_t* mask_bits,
                const void* y, const float* mean,
                const float* invstd, const float* gamma, float* dgamma, float* dbeta, int accumulate, void* dy,
                void* dpre, float* partial, float* coef, void* stream);
/* ssip_bn_bwd for a BN+ReLU without residual: the ReLU mask is recomputed
 * from y as fma(y, scale, shift) > 0 (bit-identical to ssip_bn_apply's
 * output sign), so the activation z is never read. */
int ssip_bn_relu_bwd(int dtype, int64_t M, int C, const void* dz, const void* y, const float* mean,
                     const float* invstd, const float* scale, const float* shift, const float* gamma, float* dgamma,
                     float* dbeta, int accumulate, void* dy, float* partial, float* coef, void* stream);
/* Finish a BN backward whose reduction came from ssip_conv_dgrad_bn's partials
 * ([C][tiles][2] sums of dout and dout*xhat, as ssip_conv_dgrad_bn writes
 * them (ABI 9; was [tiles][C][2]); dout already ReLU-masked):
 * dgamma/dbeta (+)= ..., dy = dBN(dout).  The split finalize's scratch sits
 * behind the records (ssip_conv_dgrad_bn_partial_floats includes it). */
int ssip_bn_bwd_from_partials(int dtype, int64_t M, int C, int tiles, float* partial, const void* dout,
                              const void* y, const float* mean, const float* invstd, const float* gamma,
                              float* dgamma, float* dbeta, int accumulate, void* dy, float* coef, void* stream);
int ssip_relu_bwd(int dtype, int64_t n, const void* g, const void* z, void* out, void* stream);
/* Backward of z = relu(BN_a(ya) + BN_b(yb)) (ssip_bn_apply2's forward):
 * dout = dz * (zmask > 0) (or the mask bits) feeds both BatchNorms; one
 * reduction pass over (dz, mask, ya, yb), one apply pass writing dy_a and dy_b (dout itself is
 * never stored).  partial: ssip_bn_bwd_dual_partial_floats(M, C) floats;
 * coef: 6*C floats scratch. */
int64_t ssip_bn_bwd_dual_partial_floats(int64_t M, int C);
int ssip_bn_bwd_dual(int dtype, int64_t M, int C, const void* dz, const void* zmask, const uint8_t* mask_bits,
                     const void* ya,
                     const float* mean_a, const float* invstd_a, const float* gamma_a, float* dgamma_a,
                     float* dbeta_a, const void* yb, const float* mean_b, const float* invstd_b,
                     const float* gamma_b, float* dgamma_b, float* dbeta_b, int accumulate, void* dy_a, void* dy_b,
                     float* partial, float* coef, void* stream);

/* ------------------------------------------------------------------------
 * Stem BN -> ReLU -> max-pool, fused (torchvision bn1/relu/maxpool).
 * Forward: out/idx = maxpool(T(relu(fma(y, scale, shift)))) without writing
 * the full-resolution activation (bit-identical to ssip_bn_apply followed by
 * ssip_maxpool_fwd).  Backward: dy = BN-backward of the ReLU-masked gathered
 * pool gradient (replaces ssip_maxpool_bwd + ssip_bn_bwd); y is the pre-BN
 * conv output [N][H][W][C]; partial sized by ..._partial_floats; coef 3*C;
 * dy may be NULL (dgamma / dbeta / coef only: see ssip_stem_bwd_wgrad).
 * ymax (nullable, pooled shape): the forward stores each window's pre-BN
 * argmax value there, and the backward then reduces over the pooled grid
 * (dpool + ymax) instead of gathering the full-resolution map twice.
 * idx may be NULL when no backward follows (a no-grad forward): the argmax
 * bytes are then not written.
 * ---------------------------------------------------------------------- */
int ssip_stem_bn_pool_fwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* y,
                          const float* scale, const float* shift, void* out, uint8_t* idx, void* ymax, void* stream);
/* ABI 14: the kernel ssip_stem_bn_pool_fwd launches for that shape (has_ymax:
 * a ymax output is passed), as a NUL-terminated name into buf:
 * "stem_bn_pool_fwd_k3s2<2|1|0>" (bf16, C = 64, 3x3 / stride 2 / pad 1, even
 * H and W; 2 = ymax from LDS, 1 = per-tap ymax, 0 = no ymax) or
 * "stem_bn_pool_fwd<generic>".  For tests and profiles; no launch. */
int ssip_stem_bn_pool_kernel_name(int dtype, int N, int H, int W, int C, int k, int s, int pad, int has_ymax,
                                  char* buf, int buflen);
int64_t ssip_stem_pool_bn_bwd_partial_floats(int N, int H, int W, int C);
/* The stem backward tail fused (bf16, 224x224 input): dW (+)= wgrad of the
 * stem conv with dy = BN-backward apply of the ReLU-masked, argmax-gathered
 * pooled gradient, formed per tile in LDS (never written).  coef: the 3*64
 * apply coefficients from ssip_stem_pool_bn_bwd called with dy = NULL (which
 * then only produces dgamma / dbeta / coef).  d describes the stem conv
 * (pre-padded NHWC4 input x); y its pre-BN output; dpool / idx pooled.
 * Workspace: ssip_conv_wgrad_workspace_bytes(d). */
int ssip_stem_bwd_wgrad_supported(const ssip_conv_desc* d, int dtype);
int ssip_stem_bwd_wgrad(const ssip_conv_desc* d, int dtype, const void* dpool, const uint8_t* idx, const void* y,
                        const void* x, const float* scale, const float* shift, const float* coef, float* dw_kcrs,
                        int c_real, int s_real, int accumulate, void* workspace, int64_t workspace_bytes,
                        void* stream);
int ssip_stem_pool_bn_bwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* dpool,
                          const uint8_t* idx, const void* y, const void* ymax, const float* mean,
                          const float* invstd,
                          const float* scale, const float* shift, const float* gamma, float* dgamma, float* dbeta,
                          int accumulate, void* dy, float* partial, float* coef, void* stream);

/* ------------------------------------------------------------------------
 * Pooling, head, losses
 * ---------------------------------------------------------------------- */
int ssip_maxpool_fwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* x, void* y,
                     uint8_t* idx, void* stream);
int ssip_maxpool_bwd(int dtype, int N, int H, int W, int C, int k, int s, int pad, const void* dy,
                     const uint8_t* idx, void* dx, void* stream);
/* feat[b][c] = mean over PQ; logits[b][j] = feat . w[j] + bias[j]  (both fp32, either nullable) */
int ssip_avgpool_fc_fwd(int dtype, int B, int PQ, int C, int J, const void* z, const float* w, const float* bias,
                        float* feat, float* logits, void* stream);
int ssip_avgpool_fc_bwd(int dtype, int B, int PQ, int C, int J, const float* dlogits, const float* w,
                        const float* feat, void* dz, float* dw, float* dbias, int accumulate, void* stream);
/* mean CE; dlogits = grad_scale*(softmax - onehot)/B; pred = argmax (each output nullable) */
int ssip_cross_entropy(int B, int J, const float* logits, const int64_t* labels, float grad_scale, float* loss,
                       float* dlogits, int64_t* pred, void* stream);
/* out4 = {total, L_l, L_u, mask_count}:  CE(zl, yl) + lambda * mean_u[1(max softmax zw >= tau) CE(zs, argmax zw)] */
int ssip_semi_loss(int Bl, int Bu, int J, const float* zl, const int64_t* yl, const float* zw, const float* zs,
                   float tau, float lambda_u, float* out4, float* dzl, float* dzs, int64_t* pseudo, uint8_t* mask,
                   void* stream);
int ssip_softmax_select(int B, int J, const float* logits, float threshold, int pos_col, float* probs, float* conf,
                        int64_t* pred, uint8_t* keep, float* pos_prob, void* stream);

/* ------------------------------------------------------------------------
 * Input pipeline (Pillow-exact).  Images are uint8 RGB [B][H][W][3].
 * ---------------------------------------------------------------------- */
typedef struct ssip_aug_param {
  int32_t flip;                       /* horizontal flip before rotation             */
  int32_t rotate;                     /* 1: Pillow 16.16 affine walk below           */
  int32_t a0, a1, a3, a4, xo, yo;     /* ImagingTransformAffine fixed-point terms    */
  int32_t photometric;                /* 1: brightness/contrast jitter (strong view) */
  float brightness, contrast;
  int32_t cut_x0, cut_y0, cut_x1, cut_y1; /* cutout box set to 0.5 (empty if x1<=x0) */
  int32_t reserved;
} ssip_aug_param;

/* horizontal resample pass: tmp [B][Hs][Wo][3]; bounds [Wo][2] = {xmin, count}; coeffs [Wo][ksize] (22-bit) */
int ssip_resize_h_u8(int B, const uint8_t* src, int64_t src_batch_stride, int Hs, int Ws, int Wo, int ksize,
                     const int* bounds, const int* coeffs, uint8_t* tmp, void* stream);
/* vertical pass (ksize_v > 0) or none, then flip/rotate/photometric/cutout in the Hr x Wr frame,
 * crop (crop_x, crop_y, Wo, Ho), ToTensor + Normalize -> out [B][Ho+2p][Wo+2p][4] (channel 3 = 0,
 * a zero border of p = out_pad pixels: the stem conv's padding, pre-applied so the stem reads
 * aligned pixel pairs with no bounds checks).
 * mean3/std3 are HOST pointers; params (nullable) is a device array of B entries. */
int ssip_augment_u8(int dtype, int B, const uint8_t* src, int64_t src_batch_stride, int src_h, int src_w, int Hr,
                    int Wr, int Ho, int Wo, int crop_x, int crop_y, int ksize_v, const int* bounds_v,
                    const int* coeffs_v, const ssip_aug_param* params, const float* mean3, const float* std3,
                    int out_pad, void* out, void* stream);
/* f32 NCHW (the nn.Module input contract) -> NHWC with Cp >= C channels and an out_pad zero border */
int ssip_nchw_to_nhwc(int dtype, int B, int C, int H, int W, int Cp, int out_pad, const float* x, void* out,
                      void* stream);

/* ------------------------------------------------------------------------
 * Optimizer and weight preparation
 * ---------------------------------------------------------------------- */
int ssip_adamw(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float lr, float beta1,
               float beta2, float eps, float weight_decay, int64_t step, float grad_scale, void* stream);
/* Graph-replayable AdamW (same update as ssip_adamw): the schedule lives on the
 * device, sched = {lr, t, lr / (1 - beta1^t), sqrt(1 - beta2^t), counter,
 * 1 - beta1^(t+1), sqrt(1 - beta2^(t+1))} (7 fp64; slot 4 is an arrival
 * counter, zero between launches; slots 5-6 stage the next step's bias
 * corrections, 0 = not staged).
 * ssip_adamw_sched_step advances t and the bias corrections (one thread);
 * ssip_adamw_dev applies the update reading them -- or, with advance != 0,
 * advances them itself (ABI 8: the first update launch of a step; no
 * separate schedule launch) -- so no per-step host scalar is baked into a
 * captured hipGraph or launch plan.  ABI 11: the advancing launch reads the
 * staged corrections (every thread used to evaluate the fp64 pow()s: 131 vs
 * 52 us for ResNet-18's 11.7 M parameters) and its last workgroup stages the
 * next ones.  (torch.optim.AdamW, semi_supervised.py:115-122) */
int ssip_adamw_sched_step(double* sched, float beta1, float beta2, void* stream);
int ssip_adamw_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, double* sched,
                   float beta1, float beta2, float eps, float weight_decay, float grad_scale, int advance,
                   void* stream);
/* w_kcrs (fp32 torchvision layout) -> w_krsc [K][R][Sp][Cp] and/or w_crsk [Cp][R][Sp][K] in dtype */
int ssip_weight_prep(int dtype, int K, int C, int R, int S, int Cp, int Sp, const float* w_kcrs, void* w_krsc,
                     void* w_crsk, void* stream);
/* Batched form: every stale conv weight of a model in one launch (per step).
 * krsc or crsk may be NULL per item; count <= SSIP_WPREP_MAX per call.
 * kscale (nullable): per-output-channel factor applied before the conversion,
 * w'[k] = w[k] * kscale[k] -- an eval-mode BatchNorm folded into the conv
 * (bias = its shift, ssip_bn_eval_coeffs). */
#define SSIP_WPREP_MAX 32
typedef struct ssip_wprep {
  int K, C, R, S, Cp, Sp;
  const float* w_kcrs;
  void* w_krsc;
  void* w_crsk;
  const float* kscale;
} ssip_wprep;
int ssip_weight_prep_batch(int dtype, int count, const ssip_wprep* items, void* stream);

/* num_batches_tracked += delta for `count` int64 device counters (the BN
 * layers' num_batches_tracked, torch.nn.BatchNorm2d train-mode forward);
 * ptrs is a HOST array of count <= SSIP_COUNTERS_MAX device pointers. */
#define SSIP_COUNTERS_MAX 64
int ssip_counters_add(int count, int64_t* const* ptrs, int64_t delta, void* stream);

/* ------------------------------------------------------------------------
 * Launch plans: a recorded sequence of the stream-ordered entry points
 * above, replayed from C++ (the host-side counterpart of a hipGraph that
 * keeps multi-stream concurrency: HIP executes a graph's parallel branches
 * one after another).  The Python engine records one step while running it
 * (ssip/plan.py); a replay then enqueues the same launches, with the same
 * device pointers, on the same streams, with no Python in the loop.
 *   - a call records the function (index from ssip_plan_fn_index) and one
 *     64-bit slot per argument: integers and device pointers as their value,
 *     floats as their bit pattern; an argument with blob_len[i] > 0 is a HOST
 *     pointer to blob_len[i] bytes, copied into the plan at record time (conv
 *     descriptors, weight-prep tables, mean/std triples, counter tables);
 *   - events order streams: ssip_plan_add_event records an event on a stream,
 *     ssip_plan_add_wait makes another stream wait for it;
 *   - markers cut the plan into segments so the caller can run host work
 *     (collective launches) between them: ssip_plan_run(plan, seg).
 * Only functions whose last parameter is the stream can be recorded. */
typedef struct ssip_plan ssip_plan;
ssip_plan* ssip_plan_create(void);
void ssip_plan_destroy(ssip_plan* plan);
int ssip_plan_fn_index(const char* name);
int ssip_plan_add_call(ssip_plan* plan, int fn, int nargs, const uint64_t* slots, const int64_t* blob_len,
                       const void* blob_data);
int ssip_plan_add_event(ssip_plan* plan, void* stream);
int ssip_plan_add_wait(ssip_plan* plan, void* stream, int event);
int ssip_plan_add_marker(ssip_plan* plan);
int ssip_plan_segments(const ssip_plan* plan);
int64_t ssip_plan_num_ops(const ssip_plan* plan);
int ssip_plan_run(ssip_plan* plan, int segment);

#ifdef __cplusplus
}
#endif
#endif /* SSIP_H_ */
