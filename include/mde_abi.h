/*
 * mde_abi.h — C ABI of libmde_hip.so, the MI355X (gfx950) kernels of the
 * dense-depth training hot path.
 *
 * The reference (LuizGuzzo/Monocular_Depth_Estimation) has no FFI: its boundary
 * is the PyTorch nn.Module / callable API.  Every entry point below replaces
 * one ATen call site (or a fused group of them) on that path; the citation on
 * each entry names the reference file:line it stands in for.  The Python
 * mirror of the reference interface (monocular_depth_estimation_amd/) binds
 * these with ctypes.
 *
 * Conventions
 *  - Plain pointers to DEVICE memory; the caller owns every buffer.
 *  - Tensors are dense NCHW, element type selected by `dtype`: MDE_F32
 *    everywhere; MDE_BF16 (activation / gradient storage, fp32 statistics and
 *    accumulation) for the BatchNorm, pointwise, skip_reduce(_bn), se_bn and
 *    exact-x2 bilinear entry points (list: INTEGRATION.md "Element types");
 *    other entry points return MDE_ERR_UNSUPPORTED for it.
 *  - Small parameter/statistics tensors (weights, scales, loss scalars,
 *    min/max) are always fp32.
 *  - `stream` is a hipStream_t (NULL = default stream).  No entry point
 *    synchronises the host, allocates memory or keeps global mutable state
 *    except the opt-in timing registry at the end of this file.
 *  - Ops that need scratch take a `workspace` of at least the byte count the
 *    matching mde_*_workspace() query returns.
 *  - Return value: 0 on success, a positive hipError_t on a HIP failure, a
 *    negative MDE_ERR_* on argument errors.  Nothing is launched when an
 *    argument error is returned.
 */
#ifndef MDE_ABI_H
#define MDE_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDE_ABI_VERSION 1

#define MDE_F32 0
#define MDE_BF16 1

#define MDE_OK 0
#define MDE_ERR_INVALID_ARG (-1)
#define MDE_ERR_UNSUPPORTED (-2)

int mde_abi_version(void);
const char* mde_status_string(int status);

/* ---------------------------------------------------------------------------
 * Resizes.  scale_h / scale_w are the SOURCE-per-DESTINATION scales ATen uses
 * (area_pixel_compute_scale): 1/scale_factor when F.interpolate got a
 * scale_factor, in/out when it got a size.  The host computes them in fp32.
 * ------------------------------------------------------------------------- */

/* Bilinear resize, arbitrary ratio, align_corners 0/1.
 * Replaces F.interpolate(mode='bilinear') at
 *   src/GuideDepth/model/GuideDepth.py:49,52,55 (x2 decoder upsamples),
 *   src/GuideDepth/model/DDRNet_23_slim.py:182,185,188,191,332,342,348 (resizes
 *   to explicit sizes, non-integer ratios), and
 *   src/model_mobileV3_large_newCRFs.py:55-58,124 (x4 head upsample). */
int mde_bilinear_fwd(const void* x, void* y, int64_t n, int64_t c, int64_t hi,
                     int64_t wi, int64_t ho, int64_t wo, float scale_h,
                     float scale_w, int align_corners, int dtype, void* stream);
/* Gradient w.r.t. x (gather formulation, no atomics; gx fully overwritten). */
int mde_bilinear_bwd(const void* gy, void* gx, int64_t n, int64_t c,
                     int64_t hi, int64_t wi, int64_t ho, int64_t wo,
                     float scale_h, float scale_w, int align_corners,
                     int dtype, void* stream);
/* x2 backward for an output read by two consumers whose gradients arrive
 * separately (GuideDepth.py:49,52,55 -> the block's feature_conv and its skip
 * fusion, modules.py:89,100): gx = adjoint(gy + gy2) with the sum formed on
 * load.  Only the x2 column-pair shape (align_corners 0, scales 0.5, even wi);
 * mde_bilinear_bwd2_supported says whether a shape is one. */
int mde_bilinear_bwd2_supported(int64_t n, int64_t c, int64_t hi, int64_t wi, int64_t ho,
                                int64_t wo, float scale_h, float scale_w, int align_corners);
int mde_bilinear_bwd2(const void* gy, const void* gy2, void* gx, int64_t n, int64_t c,
                      int64_t hi, int64_t wi, int64_t ho, int64_t wo, float scale_h,
                      float scale_w, int align_corners, int dtype, void* stream);

/* Nearest resize (PyTorch 'nearest': src = min(floor(dst*scale), in-1)).
 * Replaces F.interpolate(x, scale_factor=.5 / .25) at
 *   src/GuideDepth/model/GuideDepth.py:46-47. */
int mde_nearest_fwd(const void* x, void* y, int64_t n, int64_t c, int64_t hi,
                    int64_t wi, int64_t ho, int64_t wo, float scale_h,
                    float scale_w, int dtype, void* stream);
/* Gradient w.r.t. x (gx fully overwritten). */
int mde_nearest_bwd(const void* gy, void* gx, int64_t n, int64_t c, int64_t hi,
                    int64_t wi, int64_t ho, int64_t wo, float scale_h,
                    float scale_w, int dtype, void* stream);
/* Both guides of GuideDepth.py:46-47 in one pass over the image: half =
 * nearest x0.5 of x [n,c,h/2,w/2], quarter = nearest x0.25 [n,c,h/4,w/4]
 * (bit-identical to the two mde_nearest_fwd calls: pure copies).  fp32,
 * h % 4 == 0 and w % 8 == 0 (mde_nearest_pyramid_supported). */
int mde_nearest_pyramid_supported(int64_t n, int64_t c, int64_t h, int64_t w);
int mde_nearest_pyramid(const void* x, void* half, void* quarter, int64_t n, int64_t c, int64_t h,
                        int64_t w, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Squeeze-excitation over a channel concatenation (cat fused away).
 * Replaces torch.cat([x, y], 1) at src/GuideDepth/model/modules.py:90 and
 * SELayer.forward (modules.py:21-25; reduction=1 -> two bias-free CxC
 * Linear layers, ReLU, Sigmoid):
 *   xy = cat(xa[n,ca,h,w], xb[n,cb,h,w]);  m = mean_hw(xy)
 *   s  = sigmoid(W2 relu(W1 m));  out = xy * s
 * W1: [cr, c], W2: [c, cr] with c = ca + cb (row-major, as nn.Linear.weight).
 * Saved for backward: s [n,c], hidden = relu(W1 m) [n,cr], mean [n,c].
 * xb may be NULL with cb = 0 (plain SELayer).
 * ------------------------------------------------------------------------- */
size_t mde_se_workspace(int64_t n, int64_t c, int64_t cr, int64_t h,
                        int64_t w);
int mde_se_fwd(const void* xa, int64_t ca, const void* xb, int64_t cb,
               const float* w1, const float* w2, int64_t cr, void* out,
               float* s, float* hidden, float* mean, int64_t n, int64_t h,
               int64_t w, void* workspace, int dtype, void* stream);
/* Gradients: gxa, gxb (may be NULL when not needed), gw1 [cr,c], gw2 [c,cr]
 * (overwritten, not accumulated). */
int mde_se_bwd(const void* gout, const void* xa, int64_t ca, const void* xb,
               int64_t cb, const float* w1, const float* w2, int64_t cr,
               const float* s, const float* hidden, const float* mean,
               void* gxa, void* gxb, float* gw1, float* gw2, int64_t n,
               int64_t h, int64_t w, void* workspace, int dtype, void* stream);
/* Gated variant: torchvision SqueezeExcitation of the MobileNetV3-Large
 * blocks (features[4-6, 11-15], src/model_mobileV3_large_newCRFs.py:165):
 *   s = gate(W2 relu(W1 mean(x) + b1) + b2), gate 0 = sigmoid,
 *   1 = hardsigmoid (clamp(z/6 + 1/2, 0, 1)).  b1 [cr], b2 [c] nullable;
 * gb1 / gb2 (nullable) receive their gradients.  mde_se_fwd / mde_se_bwd
 * are this with no biases and gate 0.  Same workspace. */
int mde_se_gate_fwd(const void* xa, int64_t ca, const void* xb, int64_t cb,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    int64_t cr, int gate, void* out, float* s, float* hidden, float* mean,
                    int64_t n, int64_t h, int64_t w, void* workspace, int dtype,
                    void* stream);
int mde_se_gate_bwd(const void* gout, const void* xa, int64_t ca, const void* xb,
                    int64_t cb, const float* w1, const float* w2, const float* b2,
                    int64_t cr, int gate, const float* s, const float* hidden,
                    const float* mean, void* gxa, void* gxb, float* gw1, float* gb1,
                    float* gw2, float* gb2, int64_t n, int64_t h, int64_t w,
                    void* workspace, int dtype, void* stream);
/* SE over two BatchNorm + ReLU outputs (the guided-upsampling blocks: the
 * last `BatchNorm2d -> ReLU` of feature_conv and guide_conv, modules.py:49,59,
 * their torch.cat at modules.py:90 and SELayer.forward, modules.py:21-25):
 *   out = SELayer(cat(relu(sa*ya + ha), relu(sb*yb + hb)))
 * from the BatchNorms' RAW inputs ya [n,ca,h,w], yb [n,cb,h,w] (the 1x1 convs'
 * outputs without their folded bias); scale / shift [ca+cb] are the two BNs'
 * coefficients (mde_batchnorm_fwd_coef / _coef_stats) concatenated.  The BN +
 * ReLU outputs are never written.  Saved: s, hidden, mean as mde_se_fwd.
 * Replaces (per block) two BN apply passes, the SE squeeze and scale. */
size_t mde_se_bn_workspace(int64_t n, int64_t c, int64_t cr, int64_t h, int64_t w);
int mde_se_bn_fwd(const void* ya, int64_t ca, const void* yb, int64_t cb, const float* scale,
                  const float* shift, const float* w1, const float* w2, int64_t cr, void* out,
                  float* s, float* hidden, float* mean, int64_t n, int64_t h, int64_t w,
                  void* workspace, int dtype, void* stream);
/* Backward through SE, both ReLUs and both BatchNorms: gya / gyb = d/dya,
 * d/dyb; ggamma / gbeta [ca+cb] (concatenated, nullable) the BN parameter
 * gradients; gw1 / gw2 as mde_se_bwd.  bn_mean / bn_invstd [ca+cb]: the BNs'
 * save_mean (of the raw input) / save_invstd; training 0 = eval-mode BN
 * (running statistics: no batch-statistics terms).  The folded conv bias has
 * zero gradient through a training-mode BN (the caller supplies zeros). */
int mde_se_bn_bwd(const void* gout, const void* ya, int64_t ca, const void* yb, int64_t cb,
                  const float* scale, const float* shift, const float* bn_mean,
                  const float* bn_invstd, int training, const float* w1, const float* w2,
                  int64_t cr, const float* s, const float* hidden, const float* mean, void* gya,
                  void* gyb, float* ggamma, float* gbeta, float* gw1, float* gw2, int64_t n,
                  int64_t h, int64_t w, void* workspace, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Skip fusion: residual add + 1x1 conv with bias.
 * Replaces `self.reduce(residual + depth)` at src/GuideDepth/model/modules.py:100
 * (+ modules.py:76-78 nn.Conv2d(in, out, 1)):
 *   out[n,o,p] = b[o] + sum_c W[o,c] (r[n,c,p] + d[n,c,p])
 * Supported (cin, cout): cin in {1..64}, cout in {1..64}.
 * ------------------------------------------------------------------------- */
int mde_skip_reduce_fwd(const void* r, const void* d, const float* wt,
                        const float* b, void* out, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, int dtype,
                        void* stream);
size_t mde_skip_reduce_workspace(int64_t n, int64_t cin, int64_t cout,
                                 int64_t h, int64_t w);
/* gs = dL/d(r+d) (the gradient of BOTH r and d), gw [cout,cin], gb [cout]
 * (gw, gb overwritten). */
int mde_skip_reduce_bwd(const void* gout, const void* r, const void* d,
                        const float* wt, void* gs, float* gw, float* gb,
                        int64_t n, int64_t cin, int64_t cout, int64_t h,
                        int64_t w, void* workspace, int dtype, void* stream);
/* Skip fusion over the comb_conv's last BatchNorm + ReLU (modules.py:72-73,
 * 100): r is that BN's RAW input (the 1x1 conv output without its folded
 * bias), in_scale / in_shift [cin] its coefficients (mde_batchnorm_fwd_coef*):
 *   out = b + W (relu(in_scale r + in_shift) + d)
 * -- the BN + ReLU output is never written.  Backward: gs = W^T g (the
 * gradient of d and of the ReLU output), gw, gb as mde_skip_reduce_bwd, and
 * with in_sums [cin][2] (nullable) the BN backward's sums (sum e, sum e (r -
 * in_mean)), e = gs [in_scale r + in_shift > 0], for mde_batchnorm_bwd_apply.
 * mde_skip_reduce_bn_supported(.., sums): 1 if the shape runs (with sums). */
int mde_skip_reduce_bn_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int sums);
size_t mde_skip_reduce_bn_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w);
int mde_skip_reduce_bn_fwd(const void* r, const void* d, const float* in_scale,
                           const float* in_shift, const float* wt, const float* b, void* out,
                           int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                           void* stream);
int mde_skip_reduce_bn_bwd(const void* gout, const void* r, const void* d, const float* in_scale,
                           const float* in_shift, const float* in_mean, const float* wt, void* gs,
                           float* gw, float* gb, float* in_sums, int64_t n, int64_t cin,
                           int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                           void* stream);

/* ---------------------------------------------------------------------------
 * DepthNorm, src/utils.py:7-8: (d - d.min()) / (d.max() - d.min()), min/max
 * over the whole batch tensor (train.py:89).
 * ------------------------------------------------------------------------- */
size_t mde_minmax_workspace(int64_t numel);
/* minmax[0] = min(x), minmax[1] = max(x). */
int mde_minmax(const void* x, int64_t numel, float* minmax, void* workspace,
               int dtype, void* stream);
int mde_depthnorm_apply(const void* x, const float* minmax, void* y,
                        int64_t numel, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * SSIM (3x3 box, ReflectionPad2d(1), C1=1e-4, C2=9e-4; src/loss.py:57-88)
 * fused with nn.L1Loss (src/train.py:53,94) and, optionally, DepthNorm of the
 * target (train.py:89).  b = N*C images of h x w.
 *   t      = target_minmax ? (target - mn)/(mx - mn) : target
 *   l_ssim = mean(clamp((1 - S)/2, 0, 1));  l_l1 = mean|pred - t|
 *   loss[0] = w_ssim*l_ssim + w_l1*l_l1, loss[1] = l_ssim, loss[2] = l_l1
 * grad_pred (nullable) receives d loss[0] / d pred; grad_target (nullable)
 * d loss[0] / d t.  Requires h, w >= 2 (reflection pad).
 * ------------------------------------------------------------------------- */
size_t mde_ssim3_l1_workspace(int64_t b, int64_t h, int64_t w);
int mde_ssim3_l1_fwd(const void* pred, const void* target,
                     const float* target_minmax, float w_ssim, float w_l1,
                     float* loss, void* grad_pred, void* grad_target,
                     int64_t b, int64_t h, int64_t w, void* workspace,
                     int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Depth_Loss (src/GuideDepth/losses.py:15-127):
 *   alpha*L1 + beta*clamp((1 - SSIM11)*0.5, 0, 1) + gamma*grad
 * SSIM11: Gaussian window sigma 1.5 of size min(11,h,w), zero padding 5,
 * C1=(0.01 L)^2, C2=(0.03 L)^2, L = max_depth, mean over the map.
 * grad: forward differences, last column/row zero (losses.py:82-115).
 * masked mode (beta == gamma == 0): L1 over depth > 0 only (losses.py:26-31).
 * out[0] = loss, out[1] = l1, out[2] = clamped ssim term, out[3] = grad term,
 * out[4] = raw ssim mean, out[5] = element count used by L1.
 * The forward leaves the SSIM gradient coefficients in `workspace` (full
 * 11x11 window); pass the SAME workspace, unmodified, to the backward, which
 * reads them and the forward's device scalars (fwd_out); gout is a device
 * fp32 scalar.
 * ------------------------------------------------------------------------- */
size_t mde_depth_loss_workspace(int64_t b, int64_t h, int64_t w);
int mde_depth_loss_fwd(const void* pred, const void* gt, float alpha,
                       float beta, float gamma, float max_depth, float* out,
                       int64_t b, int64_t h, int64_t w, void* workspace,
                       int dtype, void* stream);
int mde_depth_loss_bwd(const void* pred, const void* gt, float alpha,
                       float beta, float gamma, float max_depth,
                       const float* fwd_out, const float* gout,
                       void* grad_pred, int64_t b, int64_t h, int64_t w,
                       void* workspace, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * BatchNorm2d with the preceding conv bias, the following activation and a
 * residual add fused (NCHW).
 * Replaces nn.BatchNorm2d — plus the bias add of the conv feeding it and the
 * ReLU / `out += residual; relu(out)` that follows it — at the 73 BN sites of
 * GuideDepth: src/GuideDepth/model/modules.py:43-49,53-59,68-74 and
 * src/GuideDepth/model/DDRNet_23_slim.py:46-72,80-113,118-172,201-210,
 * 229-265,294-298.
 *   z = x + prebias[c]                              (prebias nullable)
 *   y = act(gamma*(z - mean)/sqrt(var + eps) + beta + residual)
 *   act: 0 = identity, 1 = ReLU, 2 = Hardswish; residual nullable; gamma/beta/stats fp32 [c].
 * Training: batch mean / biased variance of z over (n,h,w); running stats
 * (nullable together) updated with `momentum` and the unbiased variance;
 * *num_batches_tracked += 1 (nullable).  Eval: running statistics.
 * save_mean (mean of the RAW x, i.e. without prebias) and save_invstd [c]
 * are written for the backward in both modes.
 * ------------------------------------------------------------------------- */
size_t mde_batchnorm_workspace(int64_t n, int64_t c, int64_t h, int64_t w);
int mde_batchnorm_fwd_train(const void* x, const float* gamma, const float* beta,
                            const float* prebias, float* running_mean,
                            float* running_var, int64_t* num_batches_tracked,
                            float momentum, float eps, const void* residual,
                            void* y, float* save_mean, float* save_invstd,
                            int64_t n, int64_t c, int64_t h, int64_t w, int act,
                            void* workspace, int dtype, void* stream);
int mde_batchnorm_fwd_eval(const void* x, const float* gamma, const float* beta,
                           const float* prebias, const float* running_mean,
                           const float* running_var, float eps,
                           const void* residual, void* y, float* save_mean,
                           float* save_invstd, int64_t n, int64_t c, int64_t h,
                           int64_t w, int act, int dtype, void* stream);
/* Training-mode statistics (or, training = 0, the running statistics) turned
 * into per-channel coefficients only: y = x * scale[c] + shift[c] is the BN
 * output (conv bias `prebias` folded), for a consumer that applies it while
 * loading (mde_pointwise_fwd in_scale / in_shift).  Running statistics,
 * num_batches_tracked and save_mean / save_invstd as mde_batchnorm_fwd_train;
 * the backward is mde_batchnorm_bwd with the consumer's input gradient. */
int mde_batchnorm_fwd_coef(const void* x, const float* gamma, const float* beta,
                           const float* prebias, float* running_mean, float* running_var,
                           int64_t* num_batches_tracked, float momentum, float eps,
                           int training, float* scale, float* shift, float* save_mean,
                           float* save_invstd, int64_t n, int64_t c, int64_t h, int64_t w,
                           void* workspace, int dtype, void* stream);
/* Backward.  `training` selects batch-statistics gradients.  The activation
 * mask is recomputed from x (and residual), so y need not be kept.
 * gresidual (nullable) receives d/d residual; with act == 0 it equals gy and
 * may be left NULL.  ggamma / gbeta / gprebias (nullable) are overwritten;
 * gprebias = sum over (n,h,w) of d/dz (the folded conv bias gradient). */
int mde_batchnorm_bwd(const void* gy, const void* x, const void* residual,
                      const float* gamma, const float* beta, const float* mean,
                      const float* invstd, int training, void* gx,
                      void* gresidual, float* ggamma, float* gbeta,
                      float* gprebias, int64_t n, int64_t c, int64_t h,
                      int64_t w, int act, void* workspace, int dtype,
                      void* stream);
/* Training forward / coefficients with the statistics emitted by the
 * producing convolution's epilogue (mde_pointwise_fwd_stats,
 * mde_conv3x3_fwd_stats): stats = DEVICE fp32 [c][stats_blocks][4] =
 * (shift, count, sum (x - shift), sum (x - shift)^2) per channel and
 * producer block of the RAW x, merged here in a fixed order (double) -- the
 * separate statistics pass over x is skipped.  Otherwise as mde_batchnorm_fwd_train / _fwd_coef (training, fp32
 * x); workspace = mde_batchnorm_workspace bytes. */
int mde_batchnorm_fwd_train_stats(const void* x, const float* gamma, const float* beta,
                                  const float* prebias, float* running_mean, float* running_var,
                                  int64_t* num_batches_tracked, float momentum, float eps,
                                  const void* residual, void* y, float* save_mean,
                                  float* save_invstd, int64_t n, int64_t c, int64_t h, int64_t w,
                                  int act, const float* stats, int64_t stats_blocks,
                                  void* workspace, int dtype, void* stream);
int mde_batchnorm_fwd_coef_stats(const void* x, const float* gamma, const float* beta,
                                 const float* prebias, float* running_mean, float* running_var,
                                 int64_t* num_batches_tracked, float momentum, float eps,
                                 float* scale, float* shift, float* save_mean, float* save_invstd,
                                 int64_t n, int64_t c, int64_t h, int64_t w, const float* stats,
                                 int64_t stats_blocks, void* workspace, int dtype, void* stream);
/* mde_batchnorm_bwd without its reduction pass: `sums` (DEVICE fp32 [c][2])
 * holds sum dy' and sum dy' * (x - mean) over (n,h,w), dy' = dy * act'(...),
 * as computed by a fused producer (mde_pointwise_bwd_bn's in_sums). */
int mde_batchnorm_bwd_apply(const void* gy, const void* x, const void* residual,
                            const float* gamma, const float* beta, const float* mean,
                            const float* invstd, int training, const float* sums, void* gx,
                            void* gresidual, float* ggamma, float* gbeta, float* gprebias,
                            int64_t n, int64_t c, int64_t h, int64_t w, int act, int dtype,
                            void* stream);

/* ---------------------------------------------------------------------------
 * NewCRF shifted-window attention (head dim 32, window <= 8), fp32 on MFMA.
 * Replaces, per CRFBlock (src/newcrf_layers.py:195-257), the pad / roll /
 * window_partition / WindowAttention core / window_reverse / roll / crop
 * sequence (:212-251, :30-59, :110-146) — everything between the qk Linear
 * and the proj Linear:
 *   qk      [b, h*w, 2c]  qk Linear output of the REAL tokens (q | k halves)
 *   qk_bias [2c]          that Linear's bias = q, k of zero-padded tokens
 *   v       [b, h, w, c]  value tokens (not projected; split into c/32 heads)
 *   v_bias  [c] or NULL   v of a zero-padded token: NULL = 0 (NewCRF, v is not
 *                         projected); SAM's cross-window attention
 *                         (src/SAM.py:111-144, 195-244) projects v with the kv
 *                         Linear after padding, so its padded v is that bias
 *   table   [(2*window-1)^2, heads] relative position bias table
 *   out     [b, h*w, c]   attention output in token order (before proj)
 * shift = 0 (W-MSA) or window/2 (SW-MSA, with the -100 region mask).
 * ------------------------------------------------------------------------- */
size_t mde_window_attn_workspace(int64_t b, int64_t h, int64_t w, int64_t c,
                                 int64_t heads, int64_t window);
int mde_window_attn_fwd(const void* qk, const float* qk_bias, const void* v,
                        const float* v_bias, const float* table, void* out, int64_t b,
                        int64_t h, int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, int dtype, void* stream);
/* gqk [b,h*w,2c] and gv [b,h,w,c] are fully overwritten; gtable and gqk_bias
 * (the contribution of the padded tokens only: q half 0, k half = sum of the
 * padded keys' gradients) are overwritten; gv_bias (nullable, needs v_bias)
 * receives the padded values' gradient sum. */
int mde_window_attn_bwd(const void* gout, const void* qk, const float* qk_bias,
                        const void* v, const float* v_bias, const float* table, void* gqk,
                        void* gv, float* gtable, float* gqk_bias, float* gv_bias, int64_t b,
                        int64_t h, int64_t w, int64_t c, int64_t heads, int64_t window,
                        int64_t shift, void* workspace, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Token-major Linear backward helpers (fp32), the NewCRF blocks' qk / proj /
 * fc1 / fc2 Linears (src/newcrf_layers.py:9-27,110-149) whose GEMMs stay on
 * hipBLASLt.  g / dh / a / da are row-major [t_rows, n] with n % 4 == 0.
 *   mde_colsum:          gb[n] = sum_t g[t, n]   (the Linear's bias gradient,
 *                        replacing autograd's `grad.sum(0)`)
 *   mde_gelu_bwd_colsum: da = dh * GELU'(a) (nn.GELU, erf form, a = fc1's
 *                        output) AND gb = sum_t da -- fc1's bias gradient in
 *                        the GELU backward's own pass
 * Fixed-order two-level reductions (bitwise reproducible); workspace bytes
 * from mde_colsum_workspace (0 = unsupported shape).
 * ------------------------------------------------------------------------- */
size_t mde_colsum_workspace(int64_t t_rows, int64_t n);
int mde_colsum(const void* g, float* gb, int64_t t_rows, int64_t n, void* workspace, int dtype,
               void* stream);
int mde_gelu_bwd_colsum(const void* dh, const void* a, void* da, float* gb, int64_t t_rows,
                        int64_t n, void* workspace, int dtype, void* stream);

/* Token-major Linear weight gradient (fp32): gw[m][n] = sum_t g[t][m] x[t][n]
 * (the `g.t() @ x` of src/newcrf_layers.py's Linear backwards, :9-27,110-149,
 * which autograd runs as one hipBLASLt GEMM) and, when gb is non-null, the
 * bias gradient gb[m] = sum_t g[t][m] from the same reads.  g [t_rows, m], x
 * [t_rows, n] row-major; t_rows % 16 == 0, m % 128 == 0, n % 128 == 0.
 * Split-K over token ranges on v_mfma_f32_16x16x4_f32, partials summed in a
 * fixed order (bitwise reproducible).  Workspace bytes from
 * mde_linear_wgrad_workspace (0 = unsupported shape). */
size_t mde_linear_wgrad_workspace(int64_t t_rows, int64_t m, int64_t n);
int mde_linear_wgrad(const void* g, const void* x, float* gw, float* gb, int64_t t_rows,
                     int64_t m, int64_t n, void* workspace, int dtype, void* stream);

/* Per-channel sums of an NCHW fp32 tensor, gb[c] = sum_{n,p} g[n][c][p] (a
 * biased conv's bias gradient: autograd's grad.sum((0, 2, 3)) behind the
 * NewCRF projections' `y + bias`, src/newcrf_layers.py:384-392); hw % 4 == 0.
 * Fixed-order two-level reduction; workspace bytes from mde_chansum_workspace
 * (0 = unsupported shape). */
size_t mde_chansum_workspace(int64_t n, int64_t c, int64_t hw);
int mde_chansum(const void* g, float* gb, int64_t n, int64_t c, int64_t hw, void* workspace,
                int dtype, void* stream);

/* 3x3 / stride-1 / pad-1 convolution with ONE output channel, NCHW fp32 (the
 * NewCRF decoder's depth head, src/model_mobileV3_large_newCRFs.py:81,123
 * Decoder.conv1 = nn.Conv2d(128, 1, 3, padding=1)): y = b + conv(x) (bias
 * nullable), gx, gw (fixed-order reduction; workspace from
 * mde_head_conv_wgrad_workspace).  w % 4 == 0. */
int mde_head_conv_supported(int64_t n, int64_t c, int64_t h, int64_t w);
int mde_head_conv_fwd(const void* x, const float* weight, const float* bias, void* y, int64_t n,
                      int64_t c, int64_t h, int64_t w, int dtype, void* stream);
int mde_head_conv_dgrad(const void* gy, const float* weight, void* gx, int64_t n, int64_t c,
                        int64_t h, int64_t w, int dtype, void* stream);
size_t mde_head_conv_wgrad_workspace(int64_t n, int64_t c, int64_t h, int64_t w);
int mde_head_conv_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t c,
                        int64_t h, int64_t w, void* workspace, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * Bias-free 1x1 convolution, NCHW: y[n,o,p] = sum_c W[o,c] x[n,c,p].  The
 * guided-upsampling blocks' 1x1 convs (`nn.Conv2d(E, E/2, 1)`, `(E, in, 1)`,
 * src/GuideDepth/model/modules.py:43-74) whose bias is folded into the
 * following BatchNorm.  Supported (cin, cout): (16,8) (16,16) (16,32) (32,16)
 * (32,32) (32,64) (64,32) with h*w % 64 == 0 (query with
 * mde_pointwise_supported); others return MDE_ERR_UNSUPPORTED.
 * Backward: gx (nullable) = W^T gy; gw [cout,cin] overwritten.
 * ------------------------------------------------------------------------- */
int mde_pointwise_supported(int64_t cin, int64_t cout, int64_t h, int64_t w);
size_t mde_pointwise_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w);
/* in_scale / in_shift (nullable, both or neither, fp32 [cin]): the input is
 * relu(x * in_scale[c] + in_shift[c]) — the producer's BatchNorm + ReLU
 * (`nn.BatchNorm2d(E), nn.ReLU()` before this conv, modules.py:44-47,54-57,
 * 69-72) fused into the operand load, coefficients from
 * mde_batchnorm_fwd_coef.  Backward then recomputes that input for gweight
 * and gx is the gradient w.r.t. it (the BN backward applies the ReLU mask). */
int mde_pointwise_fwd(const void* x, const float* in_scale, const float* in_shift,
                      const float* weight, void* y, int64_t n, int64_t cin, int64_t cout,
                      int64_t h, int64_t w, int dtype, void* stream);
int mde_pointwise_bwd(const void* gy, const void* x, const float* in_scale,
                      const float* in_shift, const float* weight, void* gx, float* gweight,
                      int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                      void* workspace, int dtype, void* stream);
/* mde_pointwise_fwd that also emits the output's per-channel shifted sums
 * per block -- the following BatchNorm's statistics (stats = DEVICE fp32
 * [cout][blocks][4] = (shift, count, s1, s2), blocks =
 * mde_pointwise_stats_blocks(...); 0 = unsupported shape).  Consumed by
 * mde_batchnorm_fwd_train_stats / _coef_stats. */
int mde_pointwise_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w);
int mde_pointwise_fwd_stats(const void* x, const float* in_scale, const float* in_shift,
                            const float* weight, void* y, float* stats, int64_t n, int64_t cin,
                            int64_t cout, int64_t h, int64_t w, int dtype, void* stream);
/* mde_pointwise_bwd with the fused BN + ReLU input (in_scale / in_shift
 * required) that ALSO computes that BatchNorm's backward reductions in its
 * epilogue: in_sums (DEVICE fp32 [cin][2]) = sum e, sum e * (x - in_mean[c])
 * with e = gx * [x * in_scale + in_shift > 0] -- the input of
 * mde_batchnorm_bwd_apply (act = ReLU, gy = gx), so the BN reduce pass over
 * (gx, x) is skipped.  in_mean = the BN's save_mean.  cin <= 32 (others
 * return MDE_ERR_UNSUPPORTED: the sums' registers cost more than the pass). */
int mde_pointwise_bwd_bn(const void* gy, const void* x, const float* in_scale,
                         const float* in_shift, const float* in_mean, const float* weight,
                         void* gx, float* gweight, float* in_sums, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                         void* stream);

/* ---------------------------------------------------------------------------
 * Bias-free 3x3 convolution, stride 1, zero padding 1, dilation 1, NCHW fp32
 * (MFMA).  The kxk first layers of the guided-upsampling blocks' feature_conv,
 * guide_conv and comb_conv (`nn.Conv2d(in, E, kernel_size=3, padding=1)`,
 * src/GuideDepth/model/modules.py:43-74), bias folded into the following
 * BatchNorm.  x [n,cin,h,w], weight [cout,cin,3,3], y [n,cout,h,w].
 * mde_conv3x3_supported(cin, cout, pass, dtype): pass 0 forward, 1 data
 * gradient, 2 weight gradient.  MDE_F32 (v_mfma_f32_16x16x4_f32): forward
 * (3,16) (3,32) (3,64) (16,16) (32,32); data gradient (16,16) (32,32);
 * weight gradient all five plus every cin % 32 == 0, cout % 64 == 0 pair (the
 * 64 / 128 / 256-channel convs of DDRNet's BasicBlocks and the decoder,
 * src/GuideDepth/model/DDRNet_23_slim.py:41-72, NCHW, no NHWC transposes).
 * MDE_BF16 (autocast, v_mfma_f32_16x16x32_bf16,
 * fp32 accumulation; x / gy / y / gx bf16, the fp32 weight rounded to bf16
 * on load, the weight gradient fp32; w % 4 == 0): (16,16) and (32,32), every
 * pass.  Others return MDE_ERR_UNSUPPORTED.
 * bwd_data: gx [n,cin,h,w] = conv_transpose(gy, weight), overwritten.
 * wgrad: gweight [cout,cin,3,3] overwritten (deterministic block partials +
 * fixed-order reduction in mde_conv3x3_wgrad_workspace bytes).
 * ------------------------------------------------------------------------- */
int mde_conv3x3_supported(int64_t cin, int64_t cout, int pass, int dtype);
int mde_conv3x3_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                    int64_t cout, int64_t h, int64_t w, int dtype, void* stream);
/* mde_conv3x3_fwd that also emits y's per-channel shifted sums per block,
 * the following BatchNorm's statistics (stats = DEVICE fp32
 * [cout][blocks][4] = (shift, count, s1, s2), blocks =
 * mde_conv3x3_stats_blocks(...)). */
int mde_conv3x3_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                             int dtype);
int mde_conv3x3_fwd_stats(const void* x, const float* weight, void* y, float* stats, int64_t n,
                          int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                          void* stream);
int mde_conv3x3_bwd_data(const void* gy, const float* weight, void* gx, int64_t n,
                         int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                         void* stream);
size_t mde_conv3x3_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int dtype);
int mde_conv3x3_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                      void* stream);

/* Stride-2 3x3 weight gradient: the DDRNet stem convolutions
 * (`nn.Conv2d(3, 32, 3, stride=2, padding=1)`, `nn.Conv2d(32, 32, 3, 2, 1)`,
 * src/GuideDepth/model/DDRNet_23_slim.py:229-236, bias folded into the BN).
 * x [n,cin,h,w] (w even), gy [n,cout,(h-1)/2+1,(w-1)/2+1], fp32 (MDE_F32);
 * (cin, cout) = (3, 32) or (32, 32).  gweight [cout,cin,3,3] overwritten
 * (block partials + fixed-order reduction in the workspace: deterministic). */
int mde_conv3x3s2_supported(int64_t cin, int64_t cout, int dtype);
size_t mde_conv3x3s2_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                     int dtype);
int mde_conv3x3s2_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, void* workspace, int dtype,
                        void* stream);

/* ---------------------------------------------------------------------------
 * Depthwise convolution (groups == channels, square k = 3 or 5, stride 1 or
 * 2, zero padding `pad`, dilation 1, no bias), NCHW.  Replaces the
 * depthwise Conv2d of every MobileNetV3-Large inverted-residual block
 * (torchvision mobilenet_v3_large().features[1..15], called at
 * src/model_mobileV3_large_newCRFs.py:165,178-182).
 *   x [n,c,h,w], weight [c,1,k,k] fp32, y [n,c,ho,wo],
 *   ho = (h + 2 pad - k) / stride + 1 (same for wo).  n*c <= 65535.
 * Backward: gx (nullable) and gweight (nullable, fp32 [c,k,k]) are
 * overwritten; gweight needs x and a workspace of mde_dwconv_workspace bytes
 * (workspace may be NULL when that size is 0).
 * ------------------------------------------------------------------------- */
size_t mde_dwconv_workspace(int64_t n, int64_t c, int64_t h, int64_t w, int64_t k,
                            int64_t stride, int64_t pad);
int mde_dwconv_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t c,
                   int64_t h, int64_t w, int64_t k, int64_t stride, int64_t pad, int dtype,
                   void* stream);
/* A channel's weight gradient split over several blocks is summed in a fixed
 * order by the launch that follows (deterministic; round 3 dropped the
 * round-2 `counters` argument and its in-kernel last-block hand-off). */
int mde_dwconv_bwd(const void* gy, const void* x, const float* weight, void* gx,
                   float* gweight, int64_t n, int64_t c, int64_t h, int64_t w, int64_t k,
                   int64_t stride, int64_t pad, void* workspace, int dtype, void* stream);

/* ---------------------------------------------------------------------------
 * LayerNorm over the last axis of a token-major [rows, c] tensor (c a
 * multiple of 64, <= 1024; larger multiples return MDE_ERR_UNSUPPORTED),
 * nn.LayerNorm semantics (biased variance, eps inside the sqrt).  Replaces
 * norm1 / norm2 of every CRFBlock and NewCRF.norm_crf
 * (src/newcrf_layers.py:197,212,233,419-434).
 *   mean / rstd [rows] fp32 are written by the forward and read by the
 *   backward; ggamma / gbeta [c] are overwritten; workspace of
 *   mde_layernorm_workspace bytes.
 * ------------------------------------------------------------------------- */
size_t mde_layernorm_workspace(int64_t rows, int64_t c);
int mde_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y,
                      float* mean, float* rstd, int64_t rows, int64_t c, float eps, int dtype,
                      void* stream);
int mde_layernorm_bwd(const void* gy, const void* x, const float* gamma, const float* mean,
                      const float* rstd, void* gx, float* ggamma, float* gbeta, int64_t rows,
                      int64_t c, void* workspace, int dtype, void* stream);
/* The residual add in front of a LayerNorm (CRFBlock's `x + attn(..)` /
 * `x + mlp(..)` and the next norm2 / norm1 / norm_crf,
 * src/newcrf_layers.py:229-257,434): sum = x + r is written and normalised in
 * one pass; the backward takes the gradient the sum's residual branch carries
 * (gres) and adds it in its epilogue: gx = gres + LayerNorm'(gy), the
 * gradient of both x and r. */
int mde_layernorm_add_fwd(const void* x, const void* r, const float* gamma, const float* beta,
                          void* sum, void* y, float* mean, float* rstd, int64_t rows, int64_t c,
                          float eps, int dtype, void* stream);
int mde_layernorm_bwd_res(const void* gy, const void* x, const void* gres, const float* gamma,
                          const float* mean, const float* rstd, void* gx, float* ggamma,
                          float* gbeta, int64_t rows, int64_t c, void* workspace, int dtype,
                          void* stream);

/* Batched 2-D transpose y[b][j][i] = x[b][i][j] of x [batch, m, n]: the
 * NCHW <-> token-major conversions around the NewCRF layers
 * (x.flatten(2).transpose(1, 2), v.permute(0, 2, 3, 1), and the
 * permute(0, 3, 1, 2).contiguous() of src/newcrf_layers.py:425-434).
 * batch <= 65535, ceil(m / 64) <= 65535. */
int mde_transpose(const void* x, void* y, int64_t batch, int64_t m, int64_t n, int dtype,
                  void* stream);

/* ---------------------------------------------------------------------------
 * NYU-Depth-V2 batch augmentation (data pipeline).
 * Replaces the host transforms RandomHorizontalFlip / RandomChannelSwap /
 * ToTensor of src/data.py:16-46,100-168 for a decoded uint8 batch:
 *   image [n, h, w, 3] uint8 (HWC, PIL order), depth [n, dh, dw] uint8
 *   (depth_bits 8: 'L' PNG, divided by 255) or int16 (depth_bits 16: 'I;16'
 *   PNG viewed as np.int16, not scaled), flags DEVICE int32 [n, 2] =
 *   {flip, k}: flip != 0 mirrors both maps, k in 0..5 permutes the image's
 *   channels by itertools.permutations(range(3))[k] (k = -1: none).
 *   image_out [n, 3, h, w], depth_out [n, 1, dh, dw] fp32 (bit-exact with
 *   the reference's ToTensor).
 * ------------------------------------------------------------------------- */
int mde_nyu_augment(const void* image, const void* depth, const int32_t* flags, float* image_out,
                    float* depth_out, int64_t n, int64_t h, int64_t w, int64_t dh, int64_t dw,
                    int depth_bits, void* stream);

/* ---------------------------------------------------------------------------
 * Depth-evaluation error sums (evaluation).  Replaces the
 * host numpy path of src/test.py:96-124 (pred clamp :105-108, range mask
 * :110, Eigen crop :114-117, utils.compute_errors src/utils.py:45-66) and the
 * FastDepth Result.evaluate of src/GuideDepth/metrics.py:41-62.
 *   pred, gt [n, h, w] fp32 (a [n,1,h,w] map is the same memory).
 *   mode bit 0: pred clamped to [min_depth, max_depth] (NaN -> min_depth) and
 *               only pixels with min_depth < gt < max_depth counted;
 *   mode bit 1: only rows [crop[0], crop[1]) x cols [crop[2], crop[3]) counted
 *               (crop is a HOST int32[4]; NULL when bit 1 is clear).
 *   sums: DEVICE double[16] = count, #(delta < 1.25^k) k=1..3, sum (g-p)^2,
 *   sum (ln g - ln p)^2, sum |g-p|/g, sum (g-p)^2/g, sum (ln p - ln g),
 *   sum |log10 p - log10 g|, sum |g-p|, sum (log10 p - log10 g)^2,
 *   sum |1/p - 1/g|, sum (1/p - 1/g)^2, 0, 0 -- every metric of both
 *   reference functions is a closed form of these.  Deterministic.
 * ------------------------------------------------------------------------- */
size_t mde_eval_workspace(int64_t n, int64_t h, int64_t w);
int mde_eval_sums(const void* pred, const void* gt, int64_t n, int64_t h, int64_t w,
                  float min_depth, float max_depth, int mode, const int32_t* crop,
                  void* workspace, double* sums, int dtype, void* stream);

/* The guide convs under bf16 autocast (src/GuideDepth/model/modules.py:52-54,
 * GuideDepth.py:46-47 feeding them the image): y = conv3x3(bf16(x), bf16(w))
 * with fp32 accumulation, stored as bf16 -- autocast's conv semantics -- from
 * the fp32 image, so neither an fp32 output nor a cast pass exists.  cout 16,
 * 32 or 64.  stats (nullable) [cout][blocks][4], blocks =
 * mde_conv3x3_guide_bf16_stats_blocks(...), the statistics of the stored
 * (rounded) y for the BatchNorm that follows.  The weight gradient is
 * mde_conv3x3_wgrad (fp32). */
int mde_conv3x3_guide_bf16_stats_blocks(int64_t n, int64_t cout, int64_t h, int64_t w);
int mde_conv3x3_guide_bf16_fwd(const float* x, const float* weight, void* y, float* stats,
                               int64_t n, int64_t cout, int64_t h, int64_t w, void* stream);

/* ---------------------------------------------------------------------------
 * Wide 1x1 convolutions (NCHW fp32, bias-free, stride 1 or 2, padding 0):
 * DDRNet's Bottleneck conv1 / conv3, the residual downsample, compression3 /
 * compression4 and DAPPM's 1x1 convs
 * (src/GuideDepth/model/DDRNet_23_slim.py:79,84,121-171,245,250,294-296),
 * which MIOpen runs as NHWC implicit GEMMs behind NCHW <-> NHWC transposes.
 * cin, cout multiples of 32; ho * wo a multiple of 4 (ho = (h-1)/stride+1);
 * stride 2 needs an even w.  mde_conv1x1_supported says whether a shape is
 * one.  fwd: y[n,cout,ho,wo]; bwd_data: gx[n,cin,h,w] fully overwritten
 * (zeros at the odd positions of a stride-2 conv); wgrad: gweight[cout,cin]
 * overwritten, deterministic (workspace from mde_conv1x1_wgrad_workspace).
 * ------------------------------------------------------------------------- */
int mde_conv1x1_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int stride,
                          int dtype);
int mde_conv1x1_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                    int64_t cout, int64_t h, int64_t w, int stride, int dtype, void* stream);
int mde_conv1x1_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int stride, int dtype,
                         void* stream);
size_t mde_conv1x1_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int stride, int dtype);
int mde_conv1x1_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, int stride, void* workspace, int dtype,
                      void* stream);

/* ---------------------------------------------------------------------------
 * Wide stride-2 3x3 convolutions (padding 1, bias-free, NCHW fp32): forward
 * and data gradient.  DDRNet's stem conv (32 -> 32), the first BasicBlock conv
 * of layer2 / 3 / 4, down3 / down4 and layer5's Bottleneck conv2
 * (src/GuideDepth/model/DDRNet_23_slim.py:80,232-233,254-265 and :41-72 via
 * _make_layer :291-309), which MIOpen runs as Winograd or NHWC implicit GEMMs
 * behind transposes.  h, w: input sizes (w even); cin, cout multiples of 32;
 * the *_supported queries say whether a shape has a kernel.  fwd:
 * y[n,cout,(h-1)/2+1,(w-1)/2+1]; bwd_data: gx[n,cin,h,w] fully overwritten.
 * The weight gradient is mde_conv3x3s2_wgrad (above).
 * ------------------------------------------------------------------------- */
int mde_conv3x3s2_fwd_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype);
int mde_conv3x3s2_dgrad_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype);
int mde_conv3x3s2_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                      int64_t cout, int64_t h, int64_t w, int dtype, void* stream);
int mde_conv3x3s2_bwd_data(const void* gy, const float* weight, void* gx, int64_t n, int64_t cin,
                           int64_t cout, int64_t h, int64_t w, int dtype, void* stream);

/* Stride-1 counterparts for the 64 / 128 / 256-channel 3x3 convs of the
 * BasicBlocks (DDRNet_23_slim.py:41-72), which MIOpen runs as Winograd:
 * pass 0 = forward, 1 = data gradient (the weight gradient is
 * mde_conv3x3_wgrad).  cin, cout multiples of 32; the query says whether the
 * (channels, h, w) geometry has a kernel. */
int mde_conv3x3_wide_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int pass,
                               int dtype);
int mde_conv3x3_wide_fwd(const void* x, const float* weight, void* y, int64_t n, int64_t cin,
                         int64_t cout, int64_t h, int64_t w, int dtype, void* stream);
int mde_conv3x3_wide_bwd_data(const void* gy, const float* weight, void* gx, int64_t n,
                              int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype,
                              void* stream);

/* Winograd F(2x2, 3x3) for the same stride-1 convs (wino.hip): 16 GEMMs of
 * (cout x cin) x (cin x tiles) per 2x2 output tile instead of 36 MACs per
 * (cout, cin) pair and tile.  mde_wino_weight transforms the forward conv's
 * [cout][cin][3][3] filter into u (mde_wino_weight_bytes); flip = 1 gives the
 * data-gradient transform (the conv cout -> cin on gy).  mde_wino_conv runs a
 * stride-1 / pad-1 conv x[n][cin][h][w] -> y[n][cout][h][w] from such a u
 * (for the data gradient: x = gy, cin = the forward's cout, cout = its cin);
 * pass 0 / 1 only selects the timing id.  cin % 16 == 0, cout % 32 == 0,
 * w even (mde_wino_supported). */
/* Which Winograd kernel the activation-heavy passes (no XCD split) take: bit
 * 0 = 0 one tile block a workgroup (the default), 1 the persistent one
 * (blocks walk runs of tile blocks with one chunk pipeline across them;
 * MDE_WINO_P=1 at load); bit 1 = the one-block kernel's B operands read one
 * transform position ahead into registers (default on; MDE_WINO_BPRE=0 at
 * load turns it off); bit 2 = 32-channel blocks with the 16 transform
 * positions split across waves (MDE_WINO_X=1 at load; its two halves are
 * summed in another order: float64-tested, not bitwise the other kernels).
 * Both compute the same products in the same order (bitwise equal).  mode < 0
 * only queries.  Returns the previous mode. */
int mde_wino_mode(int mode);
int mde_wino_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int dtype);
size_t mde_wino_weight_bytes(int64_t cin, int64_t cout);
int mde_wino_weight(const float* weight, float* u, int64_t cin, int64_t cout, int flip,
                    void* stream);
/* Both transforms of the filter in one launch: u (flip 0) and u_flip (flip 1). */
int mde_wino_weight2(const float* weight, float* u, float* u_flip, int64_t cin, int64_t cout,
                     void* stream);
int mde_wino_conv(const float* x, const float* u, float* y, int64_t n, int64_t cin, int64_t cout,
                  int64_t h, int64_t w, int pass, int dtype, void* stream);
/* mde_wino_conv with y = add + conv(x) (add [n,cout,h,w] fp32, read once in the
 * epilogue; must not overlap y): the data gradient of a BasicBlock's first conv summed
 * with the residual path's gradient of the same input (DDRNet_23_slim.py:61-72,
 * `out += residual`), where autograd would run a separate accumulation add. */
int mde_wino_conv_acc(const float* x, const float* u, const float* add, float* y, int64_t n,
                      int64_t cin, int64_t cout, int64_t h, int64_t w, int pass, int dtype,
                      void* stream);
/* Every Winograd filter transform of a forward in one launch (the per-conv
 * mde_wino_weight2 launches of a step, one table): table [rows][8] int64 on
 * the device, row = {weight ptr, u ptr, u_flip ptr (0: none), cin, cout,
 * first block, 0, 0} of a FORWARD conv (cout x cin), first block = the sum of
 * mde_wino_weight_blocks(cin, cout, u_flip != 0) over earlier rows; blocks =
 * that sum over all rows; pairs = sum of cin x cout (accounting only).  The
 * same values as mde_wino_weight2 / mde_wino_weight. */
int64_t mde_wino_weight_blocks(int64_t cin, int64_t cout, int both);
int mde_wino_weight_table(const int64_t* table, int rows, int64_t blocks, int64_t pairs,
                          void* stream);
/* The same with the following BatchNorm's statistics of y from the epilogue
 * (stats [cout][mde_wino_stats_blocks][4] = (shift, count, s1, s2), the format
 * of mde_batchnorm_fwd_train_stats; NULL stats = mde_wino_conv). */
int mde_wino_conv_stats(const float* x, const float* u, float* y, float* stats, int64_t n,
                        int64_t cin, int64_t cout, int64_t h, int64_t w, int pass, int dtype,
                        void* stream);
int mde_wino_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w);

/* ---------------------------------------------------------------------------
 * Captured-graph repair (no reference counterpart: the reference runs its step
 * eagerly, src/train.py:83-114; the build replays it from a hipGraph).
 * `graph` is a hipGraph_t that has been captured but not instantiated.  On
 * this ROCm stack a captured hipMemsetAsync is only correct on the graph's
 * first replay (graph.hip header); mde_graph_replace_memsets swaps every
 * memset node for a fill-kernel node with the same dependencies and reports
 * how many it replaced.
 * ------------------------------------------------------------------------- */
int mde_graph_count_memsets(void* graph, int64_t* count);
/* counts[6] = {all nodes, kernel, memcpy, memset, event record / wait, other
 * (child graphs, host nodes, ...)} of a captured graph: the data-parallel
 * tests use it to see the RCCL collectives captured into the step graph. */
int mde_graph_node_counts(void* graph, int64_t* counts);
/* counts[16]: nodes per hipGraphNodeType value 0..14 (kernel, memcpy, memset,
 * host, child graph, empty, wait event, event record, ext-semaphore signal /
 * wait, mem alloc / free, memcpy from / to symbol, batch mem op), [15] any
 * other type.  Diagnostic census of what a captured collective contributes. */
int mde_graph_node_types(void* graph, int64_t* counts);
/* hipGraphDebugDotPrint (verbose) of a captured graph to `path`. */
int mde_graph_dot(void* graph, const char* path);
int mde_graph_replace_memsets(void* graph, int64_t* replaced);

/* Which storage types the one-launch small-tensor BatchNorm kernels serve
 * (n * h * w <= 16384; the others take the statistics + apply launches):
 * 0 none, 1 fp32, 2 fp32 and bf16 (default).  mode < 0 only queries.
 * Returns the previous mode. */
int mde_bn_chan_mode(int mode);

/* How mde_batchnorm_fwd_train_stats uses a producer's statistics records for
 * this shape: 0 not at all (the one-launch small-tensor kernel runs), 1 merged
 * by the apply kernel itself (plane mode, stats_blocks <= 256), 2 one merge
 * launch before the apply; -1 invalid arguments. */
int mde_batchnorm_stats_route(int64_t n, int64_t c, int64_t h, int64_t w, int64_t stats_blocks,
                              int dtype);

/* ---------------------------------------------------------------------------
 * bf16 convolutions, NCHW, any cin / cout multiple of 32, 3x3 (padding 1) or
 * 1x1 (padding 0), stride 1 or 2, input width even (v_mfma_f32_32x32x16_bf16,
 * fp32 accumulation): DDRNet-23-slim's BasicBlock / Bottleneck / stem / down /
 * compression / DAPPM convolutions (src/GuideDepth/model/DDRNet_23_slim.py:
 * 41-113, 121-171, 230-263) under bf16 autocast -- the `F.conv2d` /
 * `conv.weight.grad` of each, with autocast's semantics: bf16 x / y / gy / gx,
 * the fp32 weight rounded to bf16 (RNE), fp32 weight gradient.
 * x [n,cin,h,w]; y [n,cout,ho,wo], ho = (h + 2p - k) / s + 1.
 * mde_convbf_supported(cin, cout, h, w, ks, stride, pass): pass 0 forward, 1
 * data gradient, 2 weight gradient (shape and LDS-capacity rules).
 * mde_convbf_pack: the filter of one pass as packed bf16 [cin/32][ks*ks][cout]
 * [32] (transpose = 0, the forward) or of the data gradient (transpose = 1:
 * channels swapped, taps flipped), mde_convbf_pack_elems elements;
 * mde_convbf_pack_both: both in one launch (either output nullable);
 * mde_convbf_pack_table: every filter of a table in one launch.
 * mde_convbf_fwd: y from x and the forward pack; stats (nullable) receives the
 * following BatchNorm's per-block shifted sums [cout][blocks][4] (blocks =
 * mde_convbf_stats_blocks).  mde_convbf_bwd_data: gx [n,cin,h,w] from gy and
 * the transposed pack (stride 2: gy zero-inserted, stride-1 convolution),
 * overwritten.  mde_convbf_wgrad: gweight [cout,cin,ks,ks] fp32 (cout % 64 ==
 * 0), overwritten, from deterministic block partials in
 * mde_convbf_wgrad_workspace bytes + a fixed-order reduction.
 * ------------------------------------------------------------------------- */
int mde_convbf_supported(int64_t cin, int64_t cout, int64_t h, int64_t w, int ks, int stride,
                         int pass);
/* mde_convbf_supported at batch n: also false when the launch for this batch
 * would refuse it (n x patches >= 2^22, the kernels' exact-division range),
 * so a caller can fall back before the step instead of failing inside it. */
int mde_convbf_supported_n(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                           int stride, int pass);
/* The algorithmic FLOPs (2 per MAC) the timing registry credits a pass with:
 * 2 n Ho Wo cin cout ks^2 over the FORWARD output plane for all three passes
 * (the stride-2 data gradient included: not its full-resolution output plane,
 * nor the products of the zero-inserted form).  0 for an unsupported shape. */
double mde_convbf_flops(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                        int stride, int pass);
size_t mde_convbf_pack_elems(int64_t cin, int64_t cout, int ks, int transpose);
int mde_convbf_pack(const float* weight, void* packed, int64_t cin, int64_t cout, int ks,
                    int transpose, void* stream);
int mde_convbf_pack_both(const float* weight, void* packed, void* packed_t, int64_t cin,
                         int64_t cout, int ks, void* stream);
/* Many filters in one launch: table [rows][8] int64 on the device, row =
 * {weight ptr, packed ptr, packed_t ptr (0: none), cin, cout, ks, first
 * block, 0}, first block = the sum over earlier rows of
 * ceil(max(pack elems, transposed pack elems) / 256); blocks = that sum over
 * all rows; elems = the total packed elements (launch accounting only). */
int mde_convbf_pack_table(const int64_t* table, int rows, int64_t blocks, int64_t elems,
                          void* stream);
int mde_convbf_stats_blocks(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w, int ks,
                            int stride);
int mde_convbf_fwd(const void* x, const void* packed, void* y, float* stats, int64_t n,
                   int64_t cin, int64_t cout, int64_t h, int64_t w, int ks, int stride,
                   void* stream);
int mde_convbf_bwd_data(const void* gy, const void* packed_t, void* gx, int64_t n, int64_t cin,
                        int64_t cout, int64_t h, int64_t w, int ks, int stride, void* stream);
size_t mde_convbf_wgrad_workspace(int64_t n, int64_t cin, int64_t cout, int64_t h, int64_t w,
                                   int ks, int stride);
int mde_convbf_wgrad(const void* gy, const void* x, float* gweight, int64_t n, int64_t cin,
                     int64_t cout, int64_t h, int64_t w, int ks, int stride, void* workspace,
                     void* stream);

/* ---------------------------------------------------------------------------
 * DDRNet-23-slim's stem convolution under bf16 autocast (src/GuideDepth/model/
 * DDRNet_23_slim.py:230-233, conv1[0]): 3 -> cout (32 or 64) channels, 3x3,
 * stride 2, padding 1, on the fp32 image x [n,3,h,w] (w % 4 == 0), the image
 * and weight [cout,3,3,3] rounded to bf16 (RNE) as autocast does, fp32
 * accumulation.  mde_stem_bf16_fwd: y [n,cout,ho,wo] bf16, ho = (h-1)/2+1.
 * mde_stem_bf16_wgrad: gweight [cout,3,3,3] fp32 (overwritten) from gy bf16
 * and x, via deterministic block partials in mde_stem_bf16_wgrad_workspace
 * bytes.  The image takes no gradient.  Replaces MIOpen's NHWC bf16 solvers
 * (and their transposes / zero fills) for this conv.
 * ------------------------------------------------------------------------- */
int mde_stem_bf16_supported(int64_t cin, int64_t cout, int64_t h, int64_t w);
int mde_stem_bf16_fwd(const float* x, const float* weight, void* y, int64_t n, int64_t cout,
                      int64_t h, int64_t w, void* stream);
size_t mde_stem_bf16_wgrad_workspace(int64_t n, int64_t cout, int64_t h, int64_t w);
int mde_stem_bf16_wgrad(const void* gy, const float* x, float* gweight, int64_t n, int64_t cout,
                        int64_t h, int64_t w, void* workspace, void* stream);
/* The guide convs' weight gradient under bf16 autocast (3 -> 16 / 32 / 64,
 * 3x3, stride 1, padding 1 on the image; src/GuideDepth/model/modules.py:
 * 52-54): gweight [cout,3,3,3] fp32 (overwritten) from gy [n,cout,h,w] bf16
 * read as such and the fp32 image rounded to bf16 (w % 4 == 0), same kernel
 * family and determinism as mde_stem_bf16_wgrad (stem.hip). */
size_t mde_conv3x3_guide_bf16_wgrad_workspace(int64_t n, int64_t cout, int64_t h, int64_t w);
int mde_conv3x3_guide_bf16_wgrad(const void* gy, const float* x, float* gweight, int64_t n,
                                 int64_t cout, int64_t h, int64_t w, void* workspace,
                                 void* stream);

/* ---------------------------------------------------------------------------
 * Opt-in kernel timing registry (measurement only; off by default).
 * When enabled, every launch made through this ABI is bracketed by hipEvents
 * on the stream it is launched on, and its algorithmic HBM bytes (SURVEY
 * §8(d) formulas) are accumulated.  Launches made while the stream is being
 * captured into a hipGraph record their events as external event nodes: each
 * replay re-records them, and mde_timing_collect (called once after each
 * replay) adds that replay's times, keeping the events until
 * mde_timing_reset.
 * ------------------------------------------------------------------------- */
int mde_timing_enable(int on);
int mde_timing_reset(void);
/* Resolves pending events (synchronises on them) into per-kernel totals. */
int mde_timing_collect(void);
int mde_kernel_count(void);
const char* mde_kernel_name(int kid);
int mde_timing_query(int kid, double* total_ms, int64_t* launches,
                     double* bytes);
/* Algorithmic FLOPs (2 per multiply-accumulate) of the MFMA kernels
 * (conv3x3, pointwise / skip fusion, window attention); 0 for the others. */
int mde_timing_query_flops(int kid, double* flops);

#ifdef __cplusplus
}
#endif

#endif /* MDE_ABI_H */
