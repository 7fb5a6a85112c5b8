/*
 * posfeat_hip.h -- C ABI of libposfeat_hip.so, the MI355X (gfx950) engine for
 * the PoSFeat extraction + correlation hot path.
 *
 * The reference (The-Learning-And-Vision-Atelier-LAVA/PoSFeat) has no FFI: its
 * hot path is duck-typed Python over PyTorch ATen.  Each entry point below
 * replaces the ATen work behind one reference Python surface (cited), and the
 * Python shims in posfeat_amd/ (networks/, losses/, managers/) keep those
 * surfaces' names, argument meanings and error behaviour.
 *
 * Conventions
 *   - All pointers are device pointers unless stated; all tensors are
 *     caller-owned (the library never allocates device memory except inside
 *     posfeat_model_create, which allocates nothing either: the caller passes
 *     workspace).  Scratch comes from a caller workspace sized by *_workspace.
 *   - `stream` is a hipStream_t passed as void*; every call is stream-ordered
 *     and never synchronises the host (graph-capturable), except where noted.
 *   - Return 0 on success or a negative POSFEAT_E_* code; posfeat_strerror()
 *     describes it.  No C++ exception crosses the ABI.
 *   - Feature maps inside the engine are NHWC fp32 with an explicit pixel
 *     stride (`*_cstride`, in floats) so channel concatenation is free.
 */
#ifndef POSFEAT_HIP_H
#define POSFEAT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POSFEAT_OK 0
#define POSFEAT_E_INVALID (-1)     /* bad argument / unsupported shape     */
#define POSFEAT_E_HIP (-2)         /* a HIP runtime call failed            */
#define POSFEAT_E_WORKSPACE (-3)   /* workspace too small                  */
#define POSFEAT_E_UNSUPPORTED (-4) /* option the engine does not implement */

#define POSFEAT_ACT_NONE 0
#define POSFEAT_ACT_RELU 1
#define POSFEAT_ACT_ELU 2

const char *posfeat_strerror(int code);
int posfeat_abi_version(void);
/* 1 if a gfx950 device is visible and the code object loads on it. */
int posfeat_device_ok(void);

/* ------------------------------------------------------------------------
 * Fused convolution (implicit GEMM on v_mfma_f32_32x32x2_f32).
 * Replaces: nn.Conv2d + eval BatchNorm2d + ReLU/ELU (+ residual add) of
 *   networks/DescNet.py:167-179 (conv), 182-190 (upconv's conv) and the
 *   torchvision Bottleneck convs behind DescNet.py:27-35; and the bias-only
 *   convs of networks/DeteNet.py:11-21.
 * x: NHWC, pixel stride x_cstride >= cin (cin multiple of 4); cout, y/res
 *    strides multiple of 4 and x/w/y/res/bias 16-B aligned (vector epilogue).
 * w: packed [cout][Kpad], K ordered (kh, kw, cin), Kpad = roundup(K, 32),
 *    zero-padded (posfeat_conv_packed_k).  BN already folded into w/bias.
 * y[p, c] = act(sum + bias[c] + res[p, c])   (res may be NULL)
 * ------------------------------------------------------------------------ */
typedef struct {
  int n, h, w;       /* input batch / height / width                      */
  int cin;           /* input channels, multiple of 4                     */
  int x_cstride;     /* floats between consecutive input pixels           */
  int cout, kh, kw, stride, pad;
  int y_cstride;     /* floats between consecutive output pixels          */
  int res_cstride;   /* floats between consecutive residual pixels        */
  int act;           /* POSFEAT_ACT_*                                     */
} posfeat_conv_desc;

int posfeat_conv_packed_k(int cin, int kh, int kw); /* returns Kpad */
/* Product arithmetic of the row-tile convolutions (1x1, strided, the batched
 * Winograd / tap GEMMs); returns the previous mode.  0: fp32-input MFMA
 * (v_mfma_f32_32x32x2_f32, exact fp32 fmaf chains).  1 (default): "bf16x6" --
 * each fp32 operand split exactly into three bf16 terms (h + m + l, residual
 * <= 2^-27 relative) and the six products of order >= 2^-16 accumulated in
 * fp32 on v_mfma_f32_32x32x16_bf16 (16x the fp32-MFMA rate): per-product error
 * ~2e-8 relative, below an fp32 fmaf's own rounding -- fp32-accurate results
 * (tests/test_gpu_precision.py), not a reduced-precision mode.  2: as 1, with
 * the Winograd / tap GEMM operands split by their producers (A/B only).
 * 3x3 stride-1 convs with Cin % 32 == 0 and weight planes (the extraction
 * engine's) run the bf16x6 gathered-tap tile in modes >= 1; the fp32 halo
 * kernel is kept for convs without planes and inside the training
 * instances' scopes.  Modes >= 1 also switch DiskLoss's flash passes
 * (posfeat_disk_loss, posfeat_disk_flash_lse) to bf16x6 similarity products.
 * Instances created afterwards plan with the new mode.  mode = -1: query
 * only. */
int posfeat_set_conv_precision(int mode);
/* 1 when this library is the A/B build (`make ab`, libposfeat_hip_ab.so),
 * which reads the POSFEAT_* environment switches that select the non-default
 * paths kept for A/B tests; 0 for the shipped library, which ignores them. */
int posfeat_ab_build(void);
int posfeat_conv2d_nhwc(const posfeat_conv_desc *d, const float *x, const float *w,
                        const float *bias, const float *res, float *y, void *stream);
/* Same, allowed to split K over workgroups (deterministic: fp32 partial slabs
 * summed in split order by a second kernel) when the tile count would leave
 * the last wave of workgroups underfilled.  Scratch: *_workspace bytes
 * (0 = this shape never splits). */
size_t posfeat_conv2d_workspace(const posfeat_conv_desc *d);
int posfeat_conv2d_nhwc_ws(const posfeat_conv_desc *d, const float *x, const float *w,
                           const float *bias, const float *res, float *y, void *ws,
                           size_t ws_bytes, void *stream);
/* Same as posfeat_conv2d_nhwc_ws with the weights ALSO given as their three
 * bf16 planes (h, m, l of the packed [cout][Kpad] array, plane stride wplane
 * elements, >= cout * posfeat_conv_packed_k(cin, kh, kw) or POSFEAT_E_INVALID;
 * h = RNE_bf16(w), m = RNE_bf16(w - h), l = RNE_bf16(w - h - m)),
 * as the engine passes them: the pre-split tiles run (dense 1x1 convs: the
 * 16x16x32 conv_bf6x_kernel; others: conv_bf6d_kernel).  tile: -1 for the
 * default plan, else a tile id the engine's autotuner may pick (ignored where
 * illegal) -- every legal tile of a conv gives bit-identical results.
 * Replaces the same reference convs as posfeat_conv2d_nhwc
 * (networks/DescNet.py:167-190). */
int posfeat_conv2d_nhwc_planes(const posfeat_conv_desc *d, const float *x, const float *w,
                               const unsigned short *wb, long long wplane, const float *bias,
                               const float *res, float *y, void *ws, size_t ws_bytes, int tile,
                               void *stream);
/* A torchvision Bottleneck's conv3 + downsample branch as ONE GEMM (the
 * reference's ResUNet encoder, networks/DescNet.py:29-35, through torchvision's
 * Bottleneck: relu(bn3(conv3(t)) + bn_ds(conv_ds(x))) with both BatchNorms
 * folded; replaces conv3 and the downsample conv of layer1.0 / layer2.0 /
 * layer3.0): y[n][oh][ow] = act(x1[n][oh][ow] . W1^T + x2[n][oh*s2][ow*s2] .
 * W2^T + bias), K = k1 + k2, bf16x6 products on the 16x16x32 tiles.  x1: rows
 * of k1 channels (pitch x1cs), x2: an h2 x w2 map of k2 channels (pitch x2cs),
 * wb: the three bf16 planes of the [cout][k1 + k2] weights (plane stride
 * cout * (k1 + k2)), bias: the two biases summed.  k1, k2 % 32 == 0,
 * cout % 128 == 0, 16-B aligned pointers, else POSFEAT_E_INVALID. */
int posfeat_conv1x1_dual(int n, int oh, int ow, const float *x1, int x1cs, int k1,
                         const float *x2, int x2cs, int h2, int w2, int s2, int k2, int cout,
                         const unsigned short *wb, const float *bias, int act, float *y, int ycs,
                         void *stream);
/* Conv (no residual, no activation) whose epilogue also reduces per-tile
 * channel sums for InstanceNorm2d (networks/DeteNet.py:12-22): writes y and
 * mean/rstd [n][cout] of y over each image (biased var, rstd=1/sqrt(var+eps)).
 * Needs out-height*out-width >= 128 (returns POSFEAT_E_UNSUPPORTED otherwise). */
size_t posfeat_conv2d_stats_workspace(const posfeat_conv_desc *d);
int posfeat_conv2d_nhwc_stats(const posfeat_conv_desc *d, const float *x, const float *w,
                              const float *bias, float *y, void *ws, size_t ws_bytes,
                              float *mean, float *rstd, float eps, void *stream);

/* KeypointDet's conv2 over cat[F.interpolate(L, x4, bilinear,
 * align_corners=False), G] + InstanceNorm statistics, without materialising
 * the upsampled map.  Replaces networks/DeteNet.py:109-112 (interpolate, cat,
 * conv2, the statistics of norm2).  L: n x H/4 x W/4 x 192 (pitch lcs), the
 * already normalised PReLU(IN(conv1)); G: n x H x W x 64 (pitch gcs),
 * IN(convimg); w_packed/bias: conv2 (256 -> 128, 3x3) packed as for
 * posfeat_conv2d_nhwc (only read by posfeat_conv2_up4_weights);
 * wph: posfeat_conv2_up4_weights_floats() floats (16 phase-combined weight
 * sets + transposed border taps) built from w_packed (rebuild after changing
 * the weights).
 * Writes y (n x H x W x 128, pitch ycs; bias added, no activation) and
 * mean/rstd [n][128] of y (biased var).  H, W multiples of 4, >= 16. */
size_t posfeat_conv2_up4_weights_floats(void);
size_t posfeat_conv2_up4_workspace(int n, int H, int W);
int posfeat_conv2_up4_weights(const float *w_packed, float *wph, void *stream);
int posfeat_conv2_up4(int n, int H, int W, const float *L, int lcs, const float *G, int gcs,
                      const float *wph, const float *w_packed, const float *bias, float *y,
                      int ycs, void *ws, size_t ws_bytes, float *mean, float *rstd, float eps,
                      void *stream);

/* ------------------------------------------------------------------------
 * Keypoint selection.
 * Replaces: losses/preprocess_utils.py:215-278 generate_kpts_single
 *   (stable=True) with nms (449-464), threshold (232-240), 3x3 soft-argmax
 *   refine + 3x3 max score (242-247), num_pts clamp (249-261), topk+gather
 *   (263-267).
 * kp_map: b x h x w fp32 (the 1-channel local_point).  Tie rule: NMS keeps
 *   p iff S[p] > every earlier and >= every later element of its
 *   reflect-padded window (row-major); top-k orders by (score desc, inner
 *   flat index asc).
 * thr_mode: 0 = no threshold (thr=False), 1 = 'abs', 2 = 'max', 3 = 'mean'.
 * num_pts <= 0 means "all survivors" (num_pts=False).
 * Outputs (capacity `cap` rows per image, cap >= max(num_pts,128) or h*w):
 *   idx [b][cap] int32 inner flat index, coord [b][cap][2] normalised (x,y),
 *   score [b][cap], n_sel[1] (device int32) = rows valid per image (same for
 *   all images, as in the reference), counts[b] (device int32) survivors.
 * ------------------------------------------------------------------------ */
int posfeat_detect_workspace(int b, int h, int w, int cap, size_t *bytes);
int posfeat_detect(const float *kp_map, int b, int h, int w, int nms_radius, int use_nms,
                   int thr_mode, float thr, int num_pts, int cap, int32_t *idx, float *coord,
                   float *score, int32_t *n_sel, int32_t *counts, void *ws, size_t ws_bytes,
                   void *stream);

/* posfeat_detect with every image of the batch selected as if it were
 * detected alone: n_sel[b] (device int32), n_sel[i] = clamp(min(num_pts,
 * counts[i]), 128) -- the reference's extraction loop, which runs
 * generate_kpts_single on one image at a time (extractor.py:336-342 with
 * batch_size 1), for a group of same-size images in one call. */
int posfeat_detect_each(const float *kp_map, int b, int h, int w, int nms_radius, int use_nms,
                        int thr_mode, float thr, int num_pts, int cap, int32_t *idx,
                        float *coord, float *score, int32_t *n_sel, int32_t *counts, void *ws,
                        size_t ws_bytes, void *stream);

/* NMS mask alone (losses/preprocess_utils.py:449-464 nms): mask[b][h][w] = 1
 * iff the pixel is its reflect-padded (2r+1)^2 window's first-occurrence max. */
int posfeat_nms_mask(const float *score, int b, int h, int w, int radius, uint8_t *mask,
                     void *stream);

/* ------------------------------------------------------------------------
 * Descriptor sampling.
 * Replaces: losses/preprocess_utils.py:40-53 sample_feat_by_coord
 *   (grid_sample bilinear, zeros padding, align_corners=False, then
 *   F.normalize p=2 dim=1 eps 1e-12 when `normalize`).
 * fmap: NHWC [b][h][w] with pixel stride cstride, c channels (c <= 1024).
 * coord: [b][npts][2] normalised (x, y); n_valid: optional device int32
 *   (rows beyond *n_valid are written as zeros); out: [b][npts][c].
 * ------------------------------------------------------------------------ */
int posfeat_sample_desc(const float *fmap, int b, int c, int h, int w, int cstride,
                        const float *coord, int npts, const int32_t *n_valid, int normalize,
                        float *out, void *stream);

/* posfeat_sample_desc with one valid-row count per image: n_valid[b] (device
 * int32, required), e.g. posfeat_detect_each's n_sel. */
int posfeat_sample_desc_each(const float *fmap, int b, int c, int h, int w, int cstride,
                             const float *coord, int npts, const int32_t *n_valid, int normalize,
                             float *out, void *stream);

/* NCHW <-> NHWC helpers used at the API boundary (torch tensors are NCHW). */
int posfeat_nchw_to_nhwc(const float *x, int n, int c, int h, int w, int cstride_out,
                         float *y, void *stream);
int posfeat_nhwc_to_nchw(const float *x, int n, int c, int h, int w, int cstride_in,
                         float *y, void *stream);

/* Extraction input on the device.  Replaces the per-image host transform of
 *   datasets/hpatches.py:14-17 / aachen.py / ETH_local_feature.py
 *   (transforms.ToTensor + Normalize(ImageNet mean/std)) so only the uint8
 *   image crosses PCIe: src uint8 [b][h][w][3] (row pitch src_pitch bytes),
 *   dst float [b][3][h][w] = ((u / 255) - mean) / std, bit-identical to the
 *   host's fp32 numpy/torch computation. */
int posfeat_normalize_rgb8(const unsigned char *src, int b, int h, int w, int src_pitch,
                           float *dst, void *stream);

/* ------------------------------------------------------------------------
 * Training-side dense correlation (forward values).
 * Replaces: losses/preprocess.py:27-121 Preprocess_Line2Window.forward with
 *   generate_kpts_regular_grid_random (preprocess_utils.py:598-659, identity
 *   map), epipolar_line_search (661-694, use_nn, loc_rand), get_endpoints
 *   (696-719), get_expected_correspondence_within_window (721-758); and
 *   losses/epipolarloss.py:38-101 EpipolarLoss_full.forward.
 * xf1/xf2: NHWC local maps [b][H/4][W/4] (128 channels, pixel stride cs).
 * F1/F2: [b][3][3].  sel1/sel2: [b][n] Categorical draw (0..grid^2-1) per
 * grid cell; rand1/rand2: [b][n][2] U(0,1) (loc_rand jitter).  The caller owns
 * the RNG; n = (H/grid)*(W/grid).  Outputs (caller buffers, [b][n][...]):
 * ------------------------------------------------------------------------ */
typedef struct {
  float *coord1, *coord2;       /* grid points, pixels [b][n][2]             */
  float *g1, *g2;               /* feat{1,2}g_corloc, pixels                 */
  float *g1_std, *g2_std;       /* feat{1,2}g_std [b][n]                     */
  float *l1_exp_n, *l2_exp_n;   /* line expectation + jitter, normalised     */
  float *l1_org_n, *l2_org_n;   /* line expectation before jitter, normalised*/
  uint8_t *valid1, *valid2;     /* valid_epi{1,2}                            */
  float *w1, *w2;               /* feat{1,2}w_corloc, pixels                 */
  float *w1_std, *w2_std;       /* feat{1,2}w_std                            */
} posfeat_l2w_out;

size_t posfeat_line2window_workspace(int b, int H1, int W1, int H2, int W2, int grid);
int posfeat_line2window(const float *xf1, int cs1, const float *xf2, int cs2, int b, int H1,
                        int W1, int H2, int W2, const float *F1, const float *F2,
                        const int32_t *sel1, const int32_t *sel2, const float *rand1,
                        const float *rand2, float temperature, int grid, float window_size,
                        int line_step, posfeat_l2w_out *out, void *ws, size_t ws_bytes,
                        void *stream);
/* out[7] = {loss, loss_g1, loss_w1, loss_g2, loss_w2, percent_g, percent_w} */
int posfeat_epipolar_loss(int b, int n, const float *F1, const float *F2, const float *c1,
                          const float *c2, const float *g1, const float *g2, const float *w1,
                          const float *w2, const float *sg1, const float *sg2, const float *sw1,
                          const float *sw2, const uint8_t *v1, const uint8_t *v2,
                          float short_edge, float grid_thr, float win_thr, float weight_grid,
                          float weight_window, float *out, void *stream);

/* Backward of the descriptor loss (configs/train_desc.yaml: weight_grid 0,
 * weight_window 1, use_std_as_weight): dL/d local_map for both images, i.e.
 * what loss.backward() sends from losses/epipolarloss.py:38-101 through
 * losses/preprocess.py:98-101 (window expectation, preprocess_utils.py:
 * 721-758) and the query descriptors (sample_feat_by_coord, 40-53) into the
 * backbone (managers/trainer.py:331).  The std weights are detached
 * (epipolarloss.py:29-31) and the line search runs under no_grad
 * (preprocess_utils.py:661), so no other path carries gradient.
 * Call after posfeat_line2window on the SAME fwd_ws with its outputs `fwd`
 * (coord*, l*_exp_n, w*, w*_std, valid* are read).  dxf1/dxf2: NHWC
 * [b][H/4][W/4] (pixel stride dcs, 128 channels), overwritten.  Scatters
 * accumulate in 64-bit fixed point, so the result is deterministic.
 * Invariant the query-descriptor gradient relies on: fwd->coord1 / coord2
 * are the forward's own grid points, point i inside its own grid cell i =
 * cy (W / grid) + cx (n = (H / grid)(W / grid) points, one per cell, as
 * posfeat_line2window draws them): each map pixel gathers its gradient from
 * the cells whose sample can have it as a bilinear corner, so a point moved
 * outside its cell between the two calls would lose its gradient (the
 * descriptor-training step never edits them).
 * weight_grid != 0 returns POSFEAT_E_UNSUPPORTED. */
size_t posfeat_line2window_backward_workspace(int b, int H1, int W1, int H2, int W2, int grid);
int posfeat_line2window_backward(const float *xf1, int cs1, const float *xf2, int cs2, int b,
                                 int H1, int W1, int H2, int W2, const float *F1,
                                 const float *F2, const posfeat_l2w_out *fwd, const void *fwd_ws,
                                 float temperature, int grid, float window_size,
                                 float short_edge, float grid_thr, float win_thr,
                                 float weight_grid, float weight_window, float *dxf1, int dcs1,
                                 float *dxf2, int dcs2, void *ws, size_t ws_bytes, void *stream);

/* DiskLoss forward (losses/kploss.py:132-197, constant_reward, grid 8):
 * kp1/kp2 [b][H][W] score maps, xf1/xf2 NHWC local maps [b][H/4][W/4] (pixel
 * stride cs), F1/F2 [b][3][3].  Either prop1,prop2,acc1,acc2 ([b][n] Categorical proposal
 * 0..63 and Bernoulli acceptance) are given, or uni1/uni2 ([b][n][65] U(0,1):
 * 64 Gumbel-max uniforms + 1 acceptance uniform) and the kernel samples.
 * out[4] = {loss, reinforce, kp_penalty, n_kps}. */
size_t posfeat_disk_loss_workspace(int b, int H, int W);
int posfeat_disk_loss(const float *kp1, const float *kp2, const float *xf1, int cs1,
                      const float *xf2, int cs2, int b, int H, int W, const float *F1,
                      const float *F2, const int32_t *prop1, const int32_t *prop2,
                      const uint8_t *acc1, const uint8_t *acc2, const float *uni1,
                      const float *uni2, float temperature, float reward_thr, float good_reward,
                      float bad_reward, float kp_penalty, float *out, void *ws, size_t ws_bytes,
                      void *stream);

/* DiskLoss forward + gradient w.r.t. both score maps (the backward of
 * losses/kploss.py:132-197 with cor_detach=True, match_grad=False as in
 * configs/train_kp.yaml:69-73: only the keypoint log-probabilities of
 * point_distribution (20-35) carry gradient).  Same arguments as
 * posfeat_disk_loss plus dkp1/dkp2 [b][H][W] (overwritten). */
size_t posfeat_disk_loss_grad_workspace(int b, int H, int W);
int posfeat_disk_loss_grad(const float *kp1, const float *kp2, const float *xf1, int cs1,
                           const float *xf2, int cs2, int b, int H, int W, const float *F1,
                           const float *F2, const int32_t *prop1, const int32_t *prop2,
                           const uint8_t *acc1, const uint8_t *acc2, const float *uni1,
                           const float *uni2, float temperature, float reward_thr,
                           float good_reward, float bad_reward, float kp_penalty, float *out,
                           float *dkp1, float *dkp2, void *ws, size_t ws_bytes, void *stream);

/* Weight gradient of a stride-1 "same" conv (the autograd conv2d weight/bias
 * backward behind managers/trainer.py:331): dw [cout][Kpad] in the packed K
 * order of posfeat_conv2d_nhwc (so it lines up with the packed weights),
 * db [cout] (may be NULL).  dy: NHWC [n][h][w] pitch dy_cstride; x: NHWC
 * input pitch x_cstride; cin % 32 == 0 or cin == 4; cout % 32 == 0; odd
 * square kernel.  Deterministic (pixel-split partials summed in order). */
size_t posfeat_conv_wgrad_workspace(int n, int h, int w, int cin, int cout, int kh, int kw);
int posfeat_conv_wgrad(const float *dy, int dy_cstride, const float *x, int x_cstride, int n,
                       int h, int w, int cin, int cout, int kh, int kw, float *dw, float *db,
                       void *ws, size_t ws_bytes, void *stream);

/* Winograd 3x3 stride-1 pad-1 conv (the decoder layers,
 * networks/DescNet.py:41-45, as the engine runs them): F(4x4,3x3) when h and w
 * are multiples of 4 (36 transformed weight matrices), else F(2x2,3x3) (16).
 * U ([36][cout][cin] floats) from the engine-packed weights by
 * posfeat_wino_weights for the same (h, w); then input transform -> the
 * transform-domain GEMMs (one launch) -> output transform + bias + act into y
 * (pixel stride y_cstride).  h, w even; cin % 32 == 0.  Same result as
 * posfeat_conv2d_nhwc within fp32 rounding (transform-grown). */
size_t posfeat_wino_workspace(int n, int h, int w, int cin, int cout);
int posfeat_wino_weights(const float *w_packed, int cout, int cin, int h, int w, float *U,
                         void *stream);
int posfeat_conv3x3_wino(const float *x, int x_cstride, int n, int h, int w, int cin,
                         const float *U, const float *bias, int cout, int act, float *y,
                         int y_cstride, void *ws, size_t ws_bytes, void *stream);

/* The same conv by Winograd F(6x6,3x3) (the extraction engine's decoder and
 * head.conv1, networks/DescNet.py:41-45 and DeteNet.py:102-121): 64
 * transformed weight matrices U ([64][cout][cin] floats, posfeat_wino6_weights),
 * 6x6 output tiles (the last tile row / column cut at h, w), 1.27x fewer
 * transform-domain MACs than F(4x4).  Any h, w; cin % 32 == 0, cout % 4 == 0,
 * even pitches.  Same result as posfeat_conv2d_nhwc within fp32 rounding
 * grown by the transforms (B^T, A^T exact; G in ninths). */
size_t posfeat_wino6_workspace(int n, int h, int w, int cin, int cout);
int posfeat_wino6_weights(const float *w_packed, int cout, int cin, float *U, void *stream);
int posfeat_conv3x3_wino6(const float *x, int x_cstride, int n, int h, int w, int cin,
                          const float *U, const float *bias, int cout, int act, float *y,
                          int y_cstride, void *ws, size_t ws_bytes, void *stream);
/* The engine's variants of the same conv: planes = 1 -- U as three bf16
 * planes (96 x cout x cin halves, posfeat_wino6_weights_planes; cout % 64 ==
 * 0), the GEMM splitting V on the fly (bf16x6); up2 = 1 -- x is the (h/2, w/2)
 * map and the conv reads its x2 bilinear upsample (align_corners = True,
 * DescNet.py:182-190 upconv), formed inside the input transform (h, w even).
 * posfeat_wino6_weights_floats: the U size in floats for those arguments. */
size_t posfeat_wino6_weights_floats(int cin, int cout, int planes);
int posfeat_wino6_weights_planes(const float *w_packed, int cout, int cin, int planes, float *U,
                                 void *stream);
int posfeat_conv3x3_wino6_ex(const float *x, int x_cstride, int n, int h, int w, int cin,
                             const float *U, int planes, int up2, const float *bias, int cout,
                             int act, float *y, int y_cstride, void *ws, size_t ws_bytes,
                             void *stream);
/* Weight gradient of the same conv by F(6x6) (the training step's decoder,
 * behind managers/trainer.py:331): dM = A dY A^T, 64 transform-domain GEMMs,
 * dw = G^T dU G in the packed K order; db (may be NULL) = sum of dy.  Any h,
 * w; cin, cout % 128 == 0.  Deterministic. */
size_t posfeat_wino6_wgrad_workspace(int n, int h, int w, int cin, int cout);
int posfeat_conv3x3_wino6_wgrad(const float *dy, int dy_cstride, const float *x, int x_cstride,
                                int n, int h, int w, int cin, int cout, float *dw, float *db,
                                void *ws, size_t ws_bytes, void *stream);

/* Weight gradient of the same decoder convs by F(4x4,3x3) (the autograd
 * conv2d weight/bias backward behind managers/trainer.py:331 for
 * networks/DescNet.py:41-45): dM = A dY A^T per 4x4 output tile, the 36
 * transform-domain GEMMs dU_xi = sum_tiles dM_xi (x) V_xi (one launch, split
 * over tiles), dw = G^T dU G written in the packed K order of
 * posfeat_conv2d_nhwc; db (may be NULL) = sum of dy.  h, w % 4 == 0;
 * cin, cout % 128 == 0.  Deterministic. */
size_t posfeat_wino_wgrad_workspace(int n, int h, int w, int cin, int cout);
int posfeat_conv3x3_wino_wgrad(const float *dy, int dy_cstride, const float *x, int x_cstride,
                               int n, int h, int w, int cin, int cout, float *dw, float *db,
                               void *ws, size_t ws_bytes, void *stream);

/* torch.optim.SGD step without momentum/weight decay (train_kp.yaml:11-13,
 * managers/trainer.py:118-119, 356): w -= lr * g over n floats. */
int posfeat_sgd(float *w, const float *g, long long n, float lr, void *stream);

/* ------------------------------------------------------------------------
 * Whole-model extraction engine.
 * Replaces: networks/PoSFeat_model.py:91-134 PoSFeat.extract for the
 *   effective model ResUNet(resnet50, 128/128) + KeypointDet(192, 1,
 *   'identity', 'Softplus') (configs/train_desc.yaml:16-31), i.e.
 *   networks/DescNet.py:64-84 and networks/DeteNet.py:102-121.
 * Weights: one packed fp32 blob; layer i occupies w_off/b_off floats (from
 *   posfeat_model_conv_spec).  The spec named "head.prelu" holds the shared
 *   PReLU scalar at b_off.
 * ------------------------------------------------------------------------ */
typedef struct posfeat_model posfeat_model;

typedef struct {
  float *local_map;       /* [b][128][h/4][w/4]  NCHW (may be NULL)        */
  float *global_map;      /* [b][128][h/16][w/16] NCHW (may be NULL)       */
  float *global_feat;     /* [b][128]                 (may be NULL)        */
  float *local_point;     /* [b][1][h][w]                                  */
  float *local_map_small; /* [b][64][h/4][w/4]  NCHW (may be NULL)         */
  const float *local_map_nhwc; /* OUT: engine-internal NHWC local_map     */
  int local_map_cstride;       /* OUT: its pixel stride in floats          */
} posfeat_extract_out;

int posfeat_model_num_specs(void);
int posfeat_model_conv_spec(int i, const char **name, int *cout, int *cin, int *kh, int *kw,
                            long long *w_off, long long *b_off);
long long posfeat_model_weight_floats(void);
int posfeat_model_create(int batch, int h, int w, const float *weights, posfeat_model **out);
/* The same, sharing the derived-weight store of `share` (an extraction
 * instance made from the same `weights` pointer; NULL: a store of its own):
 * the blob's bf16 planes and the Winograd-domain weights (F(4x4) and F(2x2)
 * slots) are built once for every instance of an engine, whatever image
 * sizes they serve, and destroying one instance frees no device memory while
 * another still uses the store (Extractor over many image sizes,
 * managers/extractor.py:357-382 with datasets/hpatches.py:35-38's crops).
 * Instances sharing a store may run on different streams: a forward orders
 * itself after the forward that last built derived weights.  They also share
 * one side stream and its fork / join events (KeypointDet's image branch):
 * instances sharing a store must be driven from ONE host thread (their
 * forwards then serialise on that side stream, as the Extractor's loop
 * does); give concurrent host threads separate stores (share = NULL). */
int posfeat_model_create_shared(int batch, int h, int w, const float *weights,
                                posfeat_model *share, posfeat_model **out);
/* An extraction instance (posfeat_model_create) builds its derived weights --
 * the blob's bf16 planes and the Winograd-domain weights -- once, in device
 * memory of its store (allocated by its first forward), by the first forward
 * that needs them.  A caller that rewrites the weight blob in place calls
 * this before the next forward: every instance sharing the store rebuilds
 * (training instances rebuild them every forward and ignore it). */
int posfeat_model_weights_changed(posfeat_model *m);
size_t posfeat_model_workspace(const posfeat_model *m);
/* The process-wide conv tile choices (the engine's autotuner: tiles never
 * change results, only speed) as text, one "<descriptor class>|<n>/<h>/<w>
 * <tile>" line each: export writes them into buf (cap bytes; *len = bytes
 * needed incl. the NUL; buf NULL: size query), import adds lines not yet
 * known and returns how many.  A tuning database kept between processes
 * (records/tile_db.txt): a new image size within 25 % of a stored GEMM M
 * reuses its tile instead of timing every candidate. */
int posfeat_tile_cache_export(char *buf, size_t cap, size_t *len);
int posfeat_tile_cache_import(const char *text);
int posfeat_model_extract(posfeat_model *m, const float *img_nchw, posfeat_extract_out *out,
                          void *ws, size_t ws_bytes, void *stream);
/* ResUNet.forward alone (networks/DescNet.py:64-84): fills out->local_map,
 * global_map, local_map_small (and global_feat) when non-NULL; local_point is
 * not touched.  Eval-mode BatchNorm (folded), as PoSFeat.extract uses it. */
int posfeat_model_backbone(posfeat_model *m, const float *img_nchw, posfeat_extract_out *out,
                           void *ws, size_t ws_bytes, void *stream);
/* KeypointDet.forward([x, img]) alone (networks/DeteNet.py:102-121):
 * x_nchw = cat[local_map, local_map_small] [b][192][h/4][w/4] (the input
 * PoSFeat.extract builds, PoSFeat_model.py:97-102), img_nchw [b][3][h][w];
 * writes local_point [b][1][h][w]. */
int posfeat_model_keypointdet(posfeat_model *m, const float *x_nchw, const float *img_nchw,
                              float *local_point, void *ws, size_t ws_bytes, void *stream);
/* Optional per-kernel timing: when enabled, extract() records hipEvents
 * around every launch; posfeat_model_timing() returns the summed ms of the
 * last call for launches whose label starts with `prefix`. */
int posfeat_model_set_timing(posfeat_model *m, int enable);
int posfeat_model_timing(posfeat_model *m, const char *prefix, double *ms, double *flops,
                         int *launches);
/* The i-th timed launch of the last call (diagnostic; host-synchronises):
 * its label (valid until the next call on m), duration and the FLOPs the
 * engine counts for it.  POSFEAT_E_INVALID past the last launch. */
int posfeat_model_timing_event(posfeat_model *m, int i, const char **label, double *ms,
                               double *flops);
/* the arithmetic of the i-th timed label's MFMA launches: a mask of 1 (fp32
 * MFMA) and 2 (bf16x6, fp32-exact products on the bf16 matrix cores); 0 for a
 * label without MFMA work.  Diagnostics for bench.py's rooflines (no
 * reference counterpart). */
int posfeat_model_timing_event_arith(posfeat_model *m, int i);
void posfeat_model_destroy(posfeat_model *m);

/* Keypoint-head training (config 5, configs/train_kp.yaml: optimal_modules
 * ['localheader'], backbone frozen and detached, PoSFeat_model.py:97-102).
 * A model made by posfeat_model_create_train keeps in its workspace what the
 * backward needs (it materialises head.conv2's input instead of the phase
 * path; results identical within fp32 rounding).
 * posfeat_model_head_backward: given dL/d local_point [b][h][w] of the LAST
 * extract() on the same workspace, writes dL/d(head parameters) into grad
 * (posfeat_model_head_floats() floats, laid out exactly like the weight blob
 * from float posfeat_model_head_offset() on: conv1, convimg, conv2, conv3,
 * prelu).  Replaces the autograd backward of networks/DeteNet.py:102-121
 * (managers/trainer.py:330-331). */
int posfeat_model_create_train(int batch, int h, int w, const float *weights,
                               posfeat_model **out);
long long posfeat_model_head_offset(void);
long long posfeat_model_head_floats(void);
int posfeat_model_head_backward(posfeat_model *m, const float *dlocal_point, float *grad,
                                void *ws, size_t ws_bytes, void *stream);

/* ------------------------------------------------------------------------
 * Descriptor training (config 3, configs/train_desc.yaml: optimal_modules
 * ['backbone'], Adam lr 1e-4).  Train-mode ResUNet (BatchNorm with batch
 * statistics and running-stat update) forward and backward.
 * Replaces: the autograd forward/backward of networks/DescNet.py:64-84 under
 *   backbone.train() (managers/trainer.py:293-297, 330-331) and
 *   torch.optim.Adam.step (trainer.py:118-119, 356).
 * Layout: one packed fp32 parameter blob (per layer: conv weight [cout][Kpad]
 *   as the engine packs it, conv bias when the layer has one, BN weight, BN
 *   bias -- offsets from posfeat_bbtrain_layer offs[0..3]); the gradient blob
 *   has the same layout; running mean / var live in a second blob
 *   (offs[4], offs[5]).  Layer names follow posfeat_model_conv_spec.
 * Workspaces: forward() fills `act` (posfeat_bbtrain_act_bytes, one per image
 *   batch: im1 and im2 keep separate BN statistics, PoSFeat_model.py:144-145);
 *   backward() reads the same `act`; `scratch` is shared.  All 256-B aligned.
 * forward: img [b][3][h][w] NCHW; *local_map_nhwc = the NHWC local map
 *   [b][h/4][w/4][128] inside `act`.  stats may be NULL (no running update).
 * backward: dlocal_map NHWC (pixel stride dcs); grad = (accumulate ? grad : 0)
 *   + dL/d params.  h and w must be multiples of 16.  An accumulate = 0 call
 *   derives every layer's input-gradient weights (transposed / phase weights,
 *   their bf16 planes, the Winograd U) into `scratch`; an accumulate = 1 call
 *   reuses them, so it must follow an accumulate = 0 call with the SAME params
 *   and scratch (the second image batch of one step, as the trainer does).
 * posfeat_adam: torch.optim.Adam (no amsgrad) on n floats; g is scaled by
 *   grad_scale first (1/world after a summing all-reduce = DDP's mean). */
typedef struct posfeat_bbtrain posfeat_bbtrain;

/* SyncBatchNorm groups (group.hip).  Replaces the SyncBatchNorm conversion of
 *   networks/PoSFeat_model.py:48-55 (PoSFeat.set_parallel): with a group set
 *   (posfeat_bbtrain_set_group), every BatchNorm of the train-mode backbone
 *   sums its statistics over the group's ranks -- forward (sum y, sum y^2,
 *   count) and backward (sum g, sum g x^) -- as torch's SyncBatchNorm does;
 *   dgamma / dbeta stay per rank (DDP averages them with the other grads).
 * RCCL: rank 0 calls posfeat_group_unique_id (128 bytes), the host broadcasts
 *   them (torch.distributed), every rank calls posfeat_group_create_rccl.
 * local: `world` ranks that are threads of one process on one device (the
 *   one-GPU test of the cross-rank semantics).
 * host: a process group without RCCL (torch.distributed over gloo, e.g. ranks
 *   that share one device): each exchange copies the n doubles to the host
 *   (the stream is synchronised), calls allreduce(buf, n, user) -- which must
 *   sum buf in place over the ranks and return 0 -- and copies them back. */
typedef struct posfeat_group posfeat_group;
typedef struct posfeat_local_group posfeat_local_group;
typedef int (*posfeat_host_allreduce_fn)(double *buf, int n, void *user);
int posfeat_group_unique_id(void *out128);
int posfeat_group_create_rccl(int world, int rank, const void *id128, posfeat_group **out);
int posfeat_group_create_host(int world, int rank, posfeat_host_allreduce_fn allreduce,
                              void *user, posfeat_group **out);
int posfeat_local_group_create(int world, int max_doubles, posfeat_local_group **out);
int posfeat_group_create_local(posfeat_local_group *L, int rank, posfeat_group **out);
void posfeat_group_destroy(posfeat_group *g);
void posfeat_local_group_destroy(posfeat_local_group *L);
int posfeat_bbtrain_set_group(posfeat_bbtrain *m, posfeat_group *g);
int posfeat_bbtrain_num_layers(void);
int posfeat_bbtrain_layer(int i, const char **name, int *cin, int *cout, int *k, int *stride,
                          int *has_bias, long long *offs /* [6] */);
long long posfeat_bbtrain_param_floats(void);
long long posfeat_bbtrain_stat_floats(void);
int posfeat_bbtrain_create(int batch, int h, int w, posfeat_bbtrain **out);
size_t posfeat_bbtrain_act_bytes(const posfeat_bbtrain *m);
size_t posfeat_bbtrain_scratch_bytes(const posfeat_bbtrain *m);
int posfeat_bbtrain_forward(posfeat_bbtrain *m, const float *params, float *stats, float momentum,
                            const float *img_nchw, void *act, void *scratch,
                            float **local_map_nhwc, void *stream);
int posfeat_bbtrain_backward(posfeat_bbtrain *m, const float *params, const void *act,
                             const float *dlocal_map_nhwc, int dcs, float *grad, int accumulate,
                             void *scratch, void *stream);
int posfeat_bbtrain_set_timing(posfeat_bbtrain *m, int enable);
int posfeat_bbtrain_timing(posfeat_bbtrain *m, const char *prefix, double *ms, double *flops,
                           int *launches);
/* The i-th timed launch of the last timed step (labels "fwd:conv:<layer>",
 * "bwd:wgrad:<layer>", "bwd:dgrad:<layer>", "fwd:bn", ...): label, ms, flops;
 * POSFEAT_E_INVALID past the last.  Host-synchronises. */
int posfeat_bbtrain_timing_event(posfeat_bbtrain *m, int i, const char **label, double *ms,
                                 double *flops);
/* as posfeat_model_timing_event_arith, for the training step's labels */
int posfeat_bbtrain_timing_event_arith(posfeat_bbtrain *m, int i);
void posfeat_bbtrain_destroy(posfeat_bbtrain *m);
int posfeat_adam(float *p, const float *g, float *m, float *v, long long n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, long long step, float grad_scale,
                 void *stream);

/* DiskLoss's flash LSE pass alone (kploss.py:160-166: the normaliser of
 * Categorical(logits=affinity)): lse[b][j] = logsumexp_i(T <fa_i, fb_j> - T) over
 * the n rows of fa for each row j of fb, fa/fb [b][n][128]; the n x n
 * similarity is recomputed by fp32 MFMA and never stored. */
size_t posfeat_disk_flash_lse_workspace(int b, int n);
int posfeat_disk_flash_lse(const float *fa, const float *fb, int b, int n, float T, float *lse,
                           void *ws, size_t ws_bytes, void *stream);

/* ---- evaluation matchers ---------------------------------
 * Replaces mnn_matcher (losses/preprocess_utils.py:795-803 =
 * evaluations/hpatches/evaluation.py:28-38), mutual_nn_matcher / ratio_matcher /
 * mutual_nn_ratio_matcher (evaluations/aachen/matchers.py:5-75, the same code
 * as evaluations/ETH_local_feature/custom_matcher.py) for L2-normalised
 * descriptors d1 [n1][dim], d2 [n2][dim] (dim == 128, 16-B aligned).
 * mode: 0 mutual NN, 1 symmetric Lowe ratio, 2 mutual NN + ratio.
 * matches: int32 [n1][2] capacity, written in ascending first index;
 * *count (device) = number written.  Tie rule: the first (lowest) index wins
 * an arg-max tie; the second-best similarity is the 2nd largest value with
 * multiplicity (torch.topk(2)).  sim = d1 d2^T is never materialised. */
size_t posfeat_match_workspace(int n1, int n2);
int posfeat_match(const float *d1, int n1, const float *d2, int n2, int dim, int mode, float ratio,
                  int32_t *matches, int32_t *count, void *ws, size_t ws_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* POSFEAT_HIP_H */
