// fmap.h -- internal (non-ABI) launchers shared by the engine.
#pragma once
#include <functional>
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../../include/posfeat_hip.h"

int pf_nchw_to_nhwc(const float* x, int n, int c, int h, int w, int cso, float* y, hipStream_t st);
int pf_nhwc_to_nchw(const float* x, int n, int c, int h, int w, int csi, float* y, hipStream_t st);
int pf_maxpool3s2(const float* x, int n, int h, int w, int c, int csi, float* y, int cso,
                  hipStream_t st);
int pf_upsample2x_ac(const float* x, int n, int h, int w, int c, int csi, float* y, int cso,
                     hipStream_t st);
size_t pf_in_stats_ws_bytes(int n, int hw, int C);
int pf_in_stats(const float* x, int n, int hw, int C, int cs, float* mean, float* rstd,
                double* part, hipStream_t st);
int pf_in_apply(float* x, int n, int hw, int C, int cs, const float* mean, const float* rstd,
                const float* prelu_slope, hipStream_t st);
int pf_norm_prelu_upsample(const float* x, int n, int h, int w, int C, int csi, const float* mean,
                           const float* rstd, const float* slope, int OH, int OW, float* y,
                           int cso, hipStream_t st);
int pf_head_tail(const float* x, int n, int hw, int cs, const float* mean, const float* rstd,
                 const float* slope, const float* w3, const float* b3, float* yraw, float* out,
                 float* mean1, float* rstd1, double* part, hipStream_t st);
int pf_global_feat(const float* g, int n, int hw, int cs, float* out, hipStream_t st);

// head.conv2 by bilinear phases, step by step (conv.hip; see posfeat_conv2_up4)
int pf_up4_gconv(int n, int H, int W, const float* G, int gcs, const float* wph,
                 const float* bias, float* y, int ycs, hipStream_t st);
int pf_up4_border(int n, int H, int W, const float* L, int lcs, const float* wph, float* y,
                  int ycs, hipStream_t st);
int pf_up4_main(int n, int H, int W, const float* L, int lcs, const float* wph, float* y, int ycs,
                void* ws, size_t ws_bytes, float* mean, float* rstd, float eps, hipStream_t st);

// conv tile control (conv.hip): legal tile ids for a shape, and runs with a
// given tile (-1 = default).  All tiles of one shape give bit-identical results.
// wplanes / wb: the weights also exist as three bf16 planes of w's layout
// (plane stride wplane elements): enables the pre-split bf16x6 tiles
int pf_conv_candidates(const posfeat_conv_desc* d, int* tiles, int max, bool wplanes = false);
int pf_conv_run_tile(const posfeat_conv_desc* d, const float* x, const float* w,
                     const float* bias, const float* res, float* y, void* ws, size_t ws_bytes,
                     int tile, hipStream_t st, const unsigned short* wb = nullptr,
                     long long wplane = 0);
// a bottleneck's conv3 + downsample as one two-source GEMM (conv.hip), and its
// weights: the [cout][k1 + k2] bf16 planes (plane stride cout * (k1 + k2)) from
// the two layers' planes (source plane stride sp) and the summed biases
int pf_conv_dual(int n, int oh, int ow, const float* x1, int x1cs, int k1, const float* x2,
                 int x2cs, int h2, int w2, int s2, int k2, int cout,
                 const unsigned short* wb, long long wplane, const float* bias, int act, float* y,
                 int ycs, hipStream_t st);
// head.conv2's tap GEMM on the weight-stationary persistent kernel (conv.hip)
int pf_tap_gemm_ws(const float* x, int lda, int M, const unsigned short* wb, long long wplane,
                   int N, float* y, int ldc, hipStream_t st);
// the same kernel for a short-K dense 1x1 conv (y = act(x W^T + bias (+ res)));
// pf_ws_gemm_ok(K, N): a shape it is instantiated for
bool pf_ws_gemm_ok(int K, int N);
// ... and the stem (7x7, 4-channel NHWC image, N = 64, kpad = 224)
int pf_gemm_ws_stem(const float* x, int n, int H, int W, int OH, int OW, int stride, int pad,
                    const unsigned short* wb, long long wplane, int kpad, int N, const float* bias,
                    int act, float* y, int ldc, hipStream_t st);
int pf_gemm_ws(const float* x, int lda, int M, int K, const unsigned short* wb, long long wplane,
               int N, const float* bias, const float* res, int rcs, int act, float* y, int ldc,
               hipStream_t st);
// a dense 1x1 GEMM with A normalised on load: PReLU((x - mean) * rstd) per
// image / channel (the 128 x 128 bf6x tile only, else POSFEAT_E_UNSUPPORTED)
int pf_conv_run_tile_np(const posfeat_conv_desc* d, const float* x, const float* w,
                        float* y, int tile, hipStream_t st, const unsigned short* wb,
                        long long wplane, const float* mean, const float* rstd,
                        const float* slope);
int pf_dual_weights(const unsigned short* w1, int k1, const unsigned short* w2, int k2,
                    long long sp, int cout, const float* b1, const float* b2,
                    unsigned short* dst, float* bdst, hipStream_t st);
// the same with the train-mode BatchNorm partial sums from the epilogue
// (conv.hip; *nparts = 0: not produced, run the statistics pass)
int pf_conv_run_tile_bn(const posfeat_conv_desc* d, const float* x, const float* w,
                        const float* bias, float* y, void* ws, size_t ws_bytes, int tile,
                        hipStream_t st, const unsigned short* wb, long long wplane, double* part,
                        size_t part_bytes, int* nparts);
// engine.hip: run(tile) with the process-wide autotuned tile of this conv
int pf_conv_tuned_run(const posfeat_conv_desc* d, bool res, bool wplanes, hipStream_t st,
                      const std::function<int(int)>& run);
size_t pf_conv_stats_ws_max(const posfeat_conv_desc* d);
int pf_conv_stats_run_tile(const posfeat_conv_desc* d, const float* x, const float* w,
                           const float* bias, float* y, void* ws, size_t ws_bytes, float* mean,
                           float* rstd, float eps, int tile, hipStream_t st,
                           const unsigned short* wb = nullptr, long long wplane = 0);

// batched GEMM on the conv engine (conv.hip): C[z] = A[z] x B[z]^T, z < nb
// Bb: B also as three bf16 planes (plane stride bplane; batch stride sb)
int pf_gemm_batched(const float* A, int lda, long long sa, const float* B, long long sb, float* C,
                    int ldc, long long sc, int nb, int M, int N, int K, hipStream_t st,
                    const unsigned short* Bb = nullptr, long long bplane = 0);
// Winograd F(2x2,3x3) (wino.hip): U = [16][Cout][Cin] transformed weights
size_t pf_wino_ws_bytes(int n, int h, int w, int Cin, int Cout);
size_t pf_wino_weights_floats(int Cin, int Cout);
int pf_wino_weights(const float* wpk, int Cout, int Cin, float* U, hipStream_t st);  // F(2x2)
// U for the variant pf_wino_conv picks at (h, w): F(4x4) if h, w % 4 == 0
// bf6p (weights): U written as three bf16 planes (F(4x4), Cout % 128 == 0);
// U then needs pf_wino_weights_floats_bf6p floats.  pf_wino_conv planes: 0
// fp32 U, 1 U planes (pre-split-weight bf16x6 tiles), 2 U and V planes
// (gemm6.hip)
int pf_wino_weights_hw(const float* wpk, int Cout, int Cin, int h, int w, float* U,
                       hipStream_t st, bool bf6p = false);
size_t pf_wino_weights_floats_bf6p(int Cin, int Cout);
// stages: bit 0 input transform, bit 1 the batched GEMMs, bit 2 output transform
// up2: x is the (h/2, w/2) map; the conv input is its x2 align_corners
// upsample, interpolated inside the input transform (F(4x4) only)
int pf_wino_conv(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                 const float* bias, int Cout, int act, float* y, int ycs, void* ws, size_t ws_bytes,
                 hipStream_t st, int stages = 7, int planes = 0, int up2 = 0);
// Winograd F(6x6,3x3) (wino.hip): U = [64][Cout][Cin] (planes: three bf16
// planes, Cout % 64 == 0, 96 floats per pair); tiles ceil(h/6) x ceil(w/6);
// pf_wino6_conv planes 0 / 1 as pf_wino_conv's, stages and up2 likewise
size_t pf_wino6_ws_bytes(int n, int h, int w, int Cin, int Cout);
size_t pf_wino6_weights_floats(int Cin, int Cout, bool planes);
int pf_wino6_weights(const float* wpk, int Cout, int Cin, float* U, hipStream_t st, bool planes);
// vkeep: V ([64][T][Cin] fp32, pf_wino6_v_floats) goes there instead of ws,
// for the weight gradient of the same x (pf_wino6_wgrad's vpre)
// stats (act none, Cout % 64 == 0): the output transform also writes the
// instance-norm partial sums of y, stats[b][g][Cout][2] fp64 (sum, sum of
// squares) over tile group g = 4 consecutive tiles of image b
// (pf_wino6_stats_groups per image: pf_in_finalize's unshifted chunks)
int pf_wino6_conv(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                  const float* bias, int Cout, int act, float* y, int ycs, void* ws,
                  size_t ws_bytes, hipStream_t st, int stages = 7, int planes = 0, int up2 = 0,
                  float* vkeep = nullptr, double* stats = nullptr);
inline int pf_wino6_stats_groups(int h, int w) { return (((h + 5) / 6) * ((w + 5) / 6) + 3) / 4; }
inline size_t pf_wino6_v_floats(int n, int h, int w, int Cin) {
  return (size_t)64 * n * ((h + 5) / 6) * ((w + 5) / 6) * Cin;
}
// F(6x6) weight gradient (any h, w; Cin, Cout % 128 == 0), as pf_wino_wgrad;
// vpre: x's V from the forward (skips the input transform)
size_t pf_wino6_wgrad_ws_bytes(int n, int h, int w, int Cin, int Cout);
int pf_wino6_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int h, int w, int Cin,
                   int Cout, float* dw, float* db, int acc, void* ws, size_t ws_bytes,
                   hipStream_t st, const float* vpre = nullptr);
// head.conv2's G part as one per-image 5x5 conv of the image (gfuse.hip)
size_t pf_gfuse_weights_floats(int n);
int pf_gfuse_weights(const float* w2_packed, const float* b2, const float* w1_packed,
                     const float* b1, const float* mean, const float* rstd, int n, float* wc,
                     float* bc, hipStream_t st);
// c: the raw convimg output for the border ring, or nullptr: recompute those
// values from the image with w1_packed / b1
int pf_gfuse_conv(const float* img4, const float* c, int ccs, int n, int H, int W,
                  const float* wc, const float* bc, const float* mean, const float* rstd,
                  const float* w2_packed, const float* b2, float* y, int ycs, hipStream_t st,
                  const float* w1_packed = nullptr, const float* b1 = nullptr,
                  unsigned short* wplanes = nullptr);
// scratch of the pre-split K = 80 weights (gfuse_conv5_k80_kernel)
size_t pf_gfuse_wplanes_bytes(int n);
// the fused head (pf_up4tap_gcombine): weight planes + the border ring's G
// values ring[b][r][128], r in pf_ring_index order
size_t pf_gfuse_ring_floats(int n, int H, int W);
// one image's border-ring floats (the ring part of pf_gfuse_ring_floats is image-major)
size_t pf_gfuse_ring_image_floats(int H, int W);
int pf_gfuse_prep(const float* img4, const float* c, int ccs, int n, int H, int W,
                  const float* wc, const float* bc, const float* mean, const float* rstd,
                  const float* b2, const float* w1_packed, const float* b1,
                  unsigned short* wplanes, float* ring, hipStream_t st);
// ring index of border pixel (Y, X) of an H x W image: the top row, the
// bottom row, then the left and right columns without the corners
__host__ __device__ inline int pf_ring_index(int Y, int X, int H, int W) {
  if (Y == 0) return X;
  if (Y == H - 1) return W + X;
  return 2 * W + (X == 0 ? 0 : H - 2) + (Y - 1);
}
// convimg's instance-norm statistics from the image's tap moments (no conv)
size_t pf_gfuse_imgstats_ws_bytes(int n, int H);
int pf_gfuse_imgstats(const float* img4, int n, int H, int W, const float* w1_packed,
                      const float* b1, float* mean, float* rstd, void* ws, size_t ws_bytes,
                      hipStream_t st, double* gram = nullptr);
size_t pf_wino_wgrad_ws_bytes(int n, int h, int w, int Cin, int Cout);
int pf_wino_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int h, int w, int Cin,
                  int Cout, float* dw, float* db, int acc, void* ws, size_t ws_bytes,
                  hipStream_t st);
size_t pf_up4_wino_weights_floats();
size_t pf_up4_wino_ws_bytes(int n, int H, int W);
int pf_up4_wino_weights(const float* wph, float* U, hipStream_t st);
int pf_up4_wino(int n, int H, int W, const float* L, int lcs, const float* U, float* y, int ycs,
                void* ws, size_t ws_bytes, hipStream_t st, int stages = 7, float* mean = nullptr,
                float* rstd = nullptr);
int pf_in_finalize(const double* part, int n, int nchunk, int hw, int C, float* mean, float* rstd,
                   hipStream_t st);
// head.conv2's upsampled part with the channel mixing on the low-res grid (up4tap.hip)
size_t pf_up4tap_weights_floats();
size_t pf_up4tap_p_floats(int n, int H, int W);
size_t pf_up4tap_part_bytes(int n, int H, int W);
int pf_up4tap_weights(const float* w2_packed, float* wt, hipStream_t st);
int pf_up4tap_combine(int n, int H, int W, const float* P, float* y, int ycs, double* part,
                      float* mean, float* rstd, hipStream_t st);
// the combine with head.conv2's G part computed in the same kernel (no G pass)
int pf_up4tap_gcombine(int n, int H, int W, const float* P, const float* img4,
                       const unsigned short* wp, const float* bc, const float* ring, float* y,
                       int ycs, double* part, float* mean, float* rstd, hipStream_t st);
// training: D = the combine's adjoint of dy (dL/dP), and the transposed tap
// weights WtT [192][1152] (dL = D . WtT^T)
int pf_up4tap_adjoint(int n, int H, int W, const float* dy, int dycs, float* D, hipStream_t st);
int pf_up4tap_weights_t(const float* w2_packed, float* wt, hipStream_t st);
// keypoint-head training, the image branch (headgrad.hip): X32[p] = the 27
// zero-padded 3x3 image taps of p (gfuse's moment order), 1, 0 x 4
int pf_img_taps32(const float* img4, int n, int H, int W, float* x32, hipStream_t st);
// per image z: A[z][co][t*32 + j] = the 3x3 weight gradient of dy against X32
// over image z alone (halo wgrad, image-aligned splits)
size_t pf_conv_wgrad_per_image_ws_bytes(int n, int H, int W, int Cin, int Cout);
int pf_conv_wgrad_per_image(const float* dy, int ldy, const float* x, int xcs, int n, int H, int W,
                            int Cin, int Cout, float* dw, void* ws, size_t ws_bytes,
                            hipStream_t st);
// gradients of head.conv2's image slice, convimg's weights and bias, and
// conv2's bias from A, the convimg IN statistics and the image moments, plus
// the tap-weight gradient dWtap [1152][192] -> the packed head gradient
size_t pf_imgbr_grad_ws_bytes(int n);
int pf_imgbr_grad(const float* A, int n, int HW, const float* w2p, const float* w1p,
                  const float* b1, const float* meanI, const float* rstdI, const double* gram,
                  const float* dwtap, float* g_w2, float* g_b2, float* g_w1, float* g_b1, void* ws,
                  size_t ws_bytes, hipStream_t st);

// conv product arithmetic: 0 fp32 MFMA, 1 bf16x6, 2 bf16x6 + pre-split GEMMs
int pf_conv_precision();
// the calling thread's tile arithmetic (conv.hip): the 16x16x32 dense tiles and the
// bf16x6 halo tiles are on unless a training scope turned them off
bool pf_bf6x_on();
bool pf_halo_bf6_on();
// while alive, this thread's 3x3 stride-1 (halo) convs use fp32 MFMA tiles
// (and the dense GEMMs the 32x32x16 bf6d tiles, the stem fp32 MFMA).
// halo_fp32 = false keeps the latter two but leaves the halo convs on their
// bf16x6 tiles (POSFEAT_TRAIN_HALO_BF6=1, A/B build: bbtrain.hip)
struct PfHaloFp32Scope {
  explicit PfHaloFp32Scope(bool halo_fp32 = true);
  ~PfHaloFp32Scope();
  PfHaloFp32Scope(const PfHaloFp32Scope&) = delete;
  PfHaloFp32Scope& operator=(const PfHaloFp32Scope&) = delete;
  bool halo_;
};
// While alive (and `on`), the calling thread's dense pre-split GEMMs run the
// 32x32x16 bf6d tiles instead of the 16x16x32 conv_bf6x_kernel: the training
// steps' forward / backward keep the arithmetic their fp64-pinned fixtures
// validated (PfHaloFp32Scope implies it).
// The convs run in this scope also write their output NCHW ([n][cout][oh*ow],
// fp32) to `dst` from the epilogue (conv_epilogue_t; not for split-K plans):
// conv_fine's local_map without the layout pass.  done() says whether the last
// conv in the scope did.
struct PfNchwSink {
  explicit PfNchwSink(float* dst);
  ~PfNchwSink();
  bool done() const;
  PfNchwSink(const PfNchwSink&) = delete;
  PfNchwSink& operator=(const PfNchwSink&) = delete;
};
struct PfDense32Scope {
  explicit PfDense32Scope(bool on);
  ~PfDense32Scope();
  PfDense32Scope(const PfDense32Scope&) = delete;
  PfDense32Scope& operator=(const PfDense32Scope&) = delete;
  bool on_;
};
// bf16x6 GEMMs on pre-split operands (gemm6.hip).  POSFEAT_BF6=2 turns them on
// for the Winograd transform-domain GEMMs and head.conv2's low-res tap GEMM.
bool pf_bf6p_on();
int pf_split3_rows(const float* x, long long rows, int cols, int ldx, unsigned short* out,
                   hipStream_t st);
int pf_gemm_batched_pre(const unsigned short* Ab, int lda, long long pa, long long sa,
                        const unsigned short* Bb, long long bplane, long long sb, float* C, int ldc,
                        long long sc, int nb, int M, int N, int K, hipStream_t st);
int pf_gemm_bf6p(const unsigned short* A, int lda, long long pa, long long sa,
                 const unsigned short* B, int ldb, long long pb, long long sb, float* C, int ldc,
                 long long sc, int nb, int M, int N, int K, hipStream_t st);
