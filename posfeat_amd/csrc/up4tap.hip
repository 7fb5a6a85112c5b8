// up4tap.hip -- head.conv2's x4-upsampled part with the channel mixing at LOW
// resolution (networks/DeteNet.py:108-112).
//
// KeypointDet feeds conv2 (3x3, 256 -> 128) with cat[up4(L), G] where
// up4 = F.interpolate(x4, bilinear, align_corners=False) of the 192-channel
// L = PReLU(IN(conv1)) at h x w = H/4 x W/4.  Both the interpolation and the
// conv are linear, and the interpolation acts per channel, so for each tap
// k = (ky, kx) of the 3x3 kernel
//
//   W_k . up4(L)(p + k - 1) = sum_q c(p + k - 1, q) (W_k . L(q)),
//
// i.e. the channel mixing P_k(q) = W_k[:, :192] . L(q) (a 1x1 conv 192 -> 128
// per tap) can run on the h x w grid: one GEMM [B h w] x 192 x (9 x 128),
// 2 * 9 * 128 * 192 FLOP per LOW-RES pixel = 1/16 of the reference layer's
// 2 * 128 * 192 * 9 per FULL-RES pixel (and 1/4 of the low-res Winograd
// F(4x4) form).  The interpolation is then applied to the nine 128-channel
// maps P_k and summed over the taps (up4tap_combine_kernel): per output pixel
// and channel 9 taps x 2 x 2 bilinear weights, evaluated separably (x first,
// then y) with a sliding window over the low-res rows.  The conv's zero
// padding is exact: a tap whose upsampled position p + k - 1 lies outside the
// H x W image contributes nothing (no border correction pass); inside, the
// bilinear source rows/cols are the replicate-clamped ones ATen uses
// (area_pixel_compute_source_index, align_corners=False: src = (dst + .5)/4 -
// .5 clamped at 0, second index clamped at h-1; weights 3/8, 5/8 / 1/8, 7/8 /
// 7/8, 1/8 / 5/8, 3/8 by phase).
//
// The combine adds the result to y, which already holds the G part + conv2's
// bias (gfuse.hip), and reduces the instance-norm statistics of the finished
// conv2 output (fp64 block partials, fixed order -> pf_in_finalize).
#include "common.h"
#include "fmap.h"

namespace {

constexpr int TAP_CU = 192;              // upsampled input channels of head.conv2
constexpr int TAP_CO = 128;              // head.conv2 output channels
constexpr int TAP_N = 9 * TAP_CO;        // P channels: tap-major, channel-minor
constexpr int TAP_KP2 = 256 * 9;         // head.conv2 packed K (Cin 256, 3x3)
constexpr int TQ = 4;                    // low-res rows per combine block
constexpr int TXC = 4;                   // full-res columns per combine block

// Wt[k * 128 + co][ci] = W2[co][ci][ky][kx] for ci < 192, from the engine's
// packed conv2 weights (K order (cin/32, kh, kw, cin%32), conv.hip).
__global__ void up4tap_weights_kernel(const float* __restrict__ w2p, float* __restrict__ wt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TAP_N * TAP_CU) return;
  const int o = i / TAP_CU, ci = i - o * TAP_CU;
  const int k = o / TAP_CO, co = o - k * TAP_CO;
  wt[i] = w2p[(long long)co * TAP_KP2 + (ci >> 5) * 288 + k * 32 + (ci & 31)];
}

// bilinear x4 (align_corners=False) of output offset d = r + k - 1 in
// [-1, 4] relative to low-res index q: taps (q + lo, q + lo + 1) with weights
// (wa, wb), lo = -1 for d in {-1, 0, 1} (d = -1 is phase 3 of q - 1), lo = 0
// for d in {2, 3, 4} (d = 4 is phase 0 of q + 1)
__device__ __forceinline__ void up4_w(int d, int& lo, float& wa, float& wb) {
  switch (d) {
    case -1: lo = -1; wa = 0.625f; wb = 0.375f; break;
    case 0: lo = -1; wa = 0.375f; wb = 0.625f; break;
    case 1: lo = -1; wa = 0.125f; wb = 0.875f; break;
    case 2: lo = 0; wa = 0.875f; wb = 0.125f; break;
    case 3: lo = 0; wa = 0.625f; wb = 0.375f; break;
    default: lo = 0; wa = 0.375f; wb = 0.625f; break;
  }
}

// Block = (4 full-res columns, 4 low-res rows = 16 full-res rows, image);
// wave = one column X = 4 qx + rx, lane = 2 channels (64 lanes x 8 B = one
// 512-B pixel row: every P / y access of a wave is one contiguous row).  The
// thread forms R_ky(iy) = sum_kx [X + kx - 1 in image] (wa P_k[iy][ia] +
// wb P_k[iy][ib]) for the three low-res rows iy = q-1, q, q+1 of a sliding
// window, then y[4q + r][X] += sum_ky [4q + r + ky - 1 in image]
// (wa R_ky(q+lo) + wb R_ky(q+lo+1)).  Two channels per lane keep the window,
// the 18 in-flight tap loads and the fp64 statistics under 128 VGPRs
// (>= 4 waves per SIMD: the kernel is HBM-bound on the y read-modify-write).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void up4tap_combine_kernel(const float* __restrict__ P, int h,
                                                             int w, float* __restrict__ y, int ycs,
                                                             double* __restrict__ part) {
  __shared__ double red[TXC][64][4];
  const int H = 4 * h, W = 4 * w;
  const int c2 = threadIdx.x & 63, xl = threadIdx.x >> 6;
  const int X = blockIdx.x * TXC + xl;
  const int q0 = blockIdx.y * TQ;
  const int b = blockIdx.z;
  const int qx = X >> 2, rx = X & 3;
  // column taps: source columns (clamped) and weights, 0 weight for padding
  int cola[3], colb[3];
  float wxa[3], wxb[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    int lo;
    up4_w(rx + kx - 1, lo, wxa[kx], wxb[kx]);
    const int u = X + kx - 1;
    if (u < 0 || u >= W) wxa[kx] = wxb[kx] = 0.f;
    cola[kx] = min(max(qx + lo, 0), w - 1) * TAP_N;
    colb[kx] = min(max(qx + lo + 1, 0), w - 1) * TAP_N;
  }
  const float* Pb = P + (long long)b * h * w * TAP_N + c2 * 2;
  auto rowR = [&](int iy, f32x2 (&R)[3]) {
    iy = min(max(iy, 0), h - 1);
    const float* pr = Pb + (long long)iy * w * TAP_N;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      f32x2 s = {0.f, 0.f};
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int k = ky * 3 + kx;
        const f32x2 pa = *reinterpret_cast<const f32x2*>(pr + cola[kx] + k * TAP_CO);
        const f32x2 pb = *reinterpret_cast<const f32x2*>(pr + colb[kx] + k * TAP_CO);
        s += wxa[kx] * pa + wxb[kx] * pb;
      }
      R[ky] = s;
    }
  };
  // all 16 y values of this thread are loaded up front: the HBM latency of
  // the read-modify-write is paid once per block, under the tap loads
  float* yb = y + (long long)b * H * W * ycs + (long long)X * ycs + c2 * 2;
  const long long yrow = (long long)W * ycs;
  f32x2 o[TQ][4];
#pragma unroll
  for (int i = 0; i < TQ; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      o[i][r] = *reinterpret_cast<const f32x2*>(yb + (4 * (q0 + i) + r) * yrow);
  f32x2 Rm[3], R0[3], Rp[3];
  rowR(q0 - 1, Rm);
  rowR(q0, R0);
  double s1[2] = {0, 0}, s2[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    const int q = q0 + i;
    rowR(q + 1, Rp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int Y = 4 * q + r;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int v = Y + ky - 1;
        if (v < 0 || v >= H) continue;
        int lo;
        float wa, wb;
        up4_w(r + ky - 1, lo, wa, wb);
        if (lo < 0)
          o[i][r] += wa * Rm[ky] + wb * R0[ky];
        else
          o[i][r] += wa * R0[ky] + wb * Rp[ky];
      }
      *reinterpret_cast<f32x2*>(yb + Y * yrow) = o[i][r];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        s1[j] += (double)o[i][r][j];
        s2[j] += (double)o[i][r][j] * (double)o[i][r][j];
      }
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      Rm[ky] = R0[ky];
      R0[ky] = Rp[ky];
    }
  }
  if (!part) return;
  red[xl][c2][0] = s1[0];
  red[xl][c2][1] = s1[1];
  red[xl][c2][2] = s2[0];
  red[xl][c2][3] = s2[1];
  __syncthreads();
  if (xl != 0) return;
  double a[4] = {0, 0, 0, 0};
  for (int r = 0; r < TXC; ++r)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += red[r][c2][k];
  const long long chunk = (long long)blockIdx.y * gridDim.x + blockIdx.x;
  const long long nchunk = (long long)gridDim.x * gridDim.y;
  double* dst = part + (((long long)b * nchunk + chunk) * TAP_CO + c2 * 2) * 2;
  dst[0] = a[0];
  dst[1] = a[2];
  dst[2] = a[1];
  dst[3] = a[3];
}

}  // namespace

size_t pf_up4tap_weights_floats() { return (size_t)TAP_N * TAP_CU; }
size_t pf_up4tap_p_floats(int n, int H, int W) { return (size_t)n * (H / 4) * (W / 4) * TAP_N; }
size_t pf_up4tap_part_bytes(int n, int H, int W) {
  return (size_t)n * ((H / 4) / TQ) * (W / TXC) * TAP_CO * 2 * sizeof(double);
}

int pf_up4tap_weights(const float* w2_packed, float* wt, hipStream_t st) {
  hipLaunchKernelGGL(up4tap_weights_kernel, dim3((TAP_N * TAP_CU + 255) / 256), dim3(256), 0, st,
                     w2_packed, wt);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// y (n x H x W x 128, pitch ycs) += the upsampled part of head.conv2 from the
// nine tap maps P (n x H/4 x W/4 x 1152); mean/rstd (optional) = the
// instance-norm statistics of the resulting y.  H/4 % 4 == 0, W % 8 == 0.
int pf_up4tap_combine(int n, int H, int W, const float* P, float* y, int ycs, double* part,
                      float* mean, float* rstd, hipStream_t st) {
  const int h = H / 4, w = W / 4;
  if (H % 16 || W % TXC || ycs % 4 || n <= 0) return POSFEAT_E_INVALID;
  if (mean && !part) return POSFEAT_E_INVALID;
  const dim3 grid(W / TXC, h / TQ, n);
  hipLaunchKernelGGL(up4tap_combine_kernel, grid, dim3(256), 0, st, P, h, w, y, ycs,
                     mean ? part : nullptr);
  PF_CHECK_LAUNCH();
  if (mean) PF_TRY(pf_in_finalize(part, n, (int)(grid.x * grid.y), H * W, TAP_CO, mean, rstd, st));
  return POSFEAT_OK;
}
