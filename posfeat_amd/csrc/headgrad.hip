// headgrad.hip -- the image branch of the keypoint-head backward (config 5,
// configs/train_kp.yaml) WITHOUT the full-resolution G map or its gradient.
//
// KeypointDet (networks/DeteNet.py:102-121) feeds head.conv2's channels
// 192..255 with G = IN(convimg(img)): per image b and convimg channel c,
// X[p][c] = b1_c + sum_i w1[c][i] x_i(p) with x(p) the 27 zero-padded 3x3 x
// 3-channel image taps (gfuse.hip's moment order i = tap*3 + ci), and
// G = (X - mu_c) rho_c.  With dY = dL/d(conv2 out) (full res, 128 ch) every
// gradient the reference's autograd produces for this branch is a
// contraction of ONE per-image quantity
//
//   A_b[co][t][j] = sum_p dY[p][co] X32(p + t - 1)[j],
//
// X32 = (x_0 .. x_26, 1, 0, 0, 0, 0) zero outside the image -- a 3x3 weight
// gradient of dY against the 32-channel tap image (pf_conv_wgrad_per_image,
// MFMA) -- with the image moments E_b[i][j] = mean_p x_i x_j (gfuse's Gram,
// kept by the forward) and the convimg IN statistics:
//
//   S[co][t]        = A[co][t][27]                 (sum of dY over the taps' valid pixels)
//   dW2[co][c][t]   = rho_c ((b1_c - mu_c) S[co][t] + sum_i w1[c][i] A[co][t][i])
//   sum_p dG[p][c]  = sum_{co,t} W2[co][192+c][t] S[co][t]            (= HW e1)
//   sum_p dG G      = sum_{co,t} W2[co][192+c][t] dW2[co][c][t]       (= HW e2)
//   sum_p dG x_i    = sum_{co,t} W2[co][192+c][t] A[co][t][i]         (= Q_i)
//   sum_p G x_i     = rho_c HW ((b1_c - mu_c) m_i + sum_j w1[c][j] E[j][i])
//   dW1[c][i]       = rho_c (Q_i - e1 HW m_i - e2 sum_p G x_i)   (IN backward, then convimg dW)
//   db1[c]          = rho_c (HW e1 - HW e1 - e2 sum_p G)
//   db2[co]         = S[co][centre]
//
// (dG = the conv2 input gradient, never formed: conv2's image slice costs no
// input-gradient conv and no G-map weight gradient -- 2 x 725 GFLOP at 16
// images of 480x640 -- only the 32-channel A, 362 GFLOP.)  Exact in real
// arithmetic; the borders are exact because X32 is zero outside the image
// exactly where conv2's padding zeroes G.
#include "common.h"
#include "fmap.h"

namespace {

constexpr int HG_CO = 128, HG_C = 64, HG_T = 27, HG_CU = 192, HG_KP2 = 2304;

// x32[b][p][j]: float4 per thread (8 per pixel)
__global__ void img_taps32_kernel(const float* __restrict__ img4, int n, int H, int W,
                                  float* __restrict__ x32) {
  const long long total = (long long)n * H * W * 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i & 7);
    const long long pix = i >> 3;
    const int x = (int)(pix % W);
    const long long r = pix / W;
    const int y = (int)(r % H);
    const long long b = r / H;
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = q * 4 + e;
      float s = 0.f;
      if (j < HG_T) {
        const int t = j / 3, ci = j - t * 3;
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
          s = img4[((b * H + yy) * W + xx) * 4 + ci];
      } else if (j == HG_T) {
        s = 1.f;
      }
      v[e] = s;
    }
    *reinterpret_cast<f32x4*>(x32 + pix * 32 + q * 4) = v;
  }
}

// one block per (convimg channel c, image z); thread = conv2 output channel co
__global__ __launch_bounds__(128) void imgbr_image_kernel(
    const float* __restrict__ A, const float* __restrict__ w2p, const float* __restrict__ w1p,
    int k1pad, const float* __restrict__ b1, const float* __restrict__ meanI,
    const float* __restrict__ rstdI, const double* __restrict__ gram, int HW,
    float* __restrict__ dw2i, double* __restrict__ dwi) {
  const int c = blockIdx.x, z = blockIdx.y, co = threadIdx.x;
  __shared__ double wi[HG_T];
  __shared__ double red[HG_CO][HG_T + 3];
  if (co < HG_T) wi[co] = (double)w1p[c * k1pad + (co / 3) * 4 + co % 3];
  __syncthreads();
  const double mu = meanI[z * HG_C + c], rho = rstdI[z * HG_C + c], bb = b1[c];
  const float* a = A + ((long long)z * HG_CO + co) * 288;
  double e1 = 0.0, e2 = 0.0, Q[HG_T];
#pragma unroll
  for (int i = 0; i < HG_T; ++i) Q[i] = 0.0;
  for (int t = 0; t < 9; ++t) {
    const double w2 = w2p[(long long)co * HG_KP2 + (6 + (c >> 5)) * 288 + t * 32 + (c & 31)];
    const double S = a[t * 32 + HG_T];
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < HG_T; ++i) {
      const double av = a[t * 32 + i];
      s += wi[i] * av;
      Q[i] += w2 * av;
    }
    const double g = rho * ((bb - mu) * S + s);
    dw2i[(((long long)z * HG_CO + co) * HG_C + c) * 9 + t] = (float)g;
    e1 += w2 * S;
    e2 += w2 * g;
  }
#pragma unroll
  for (int i = 0; i < HG_T; ++i) red[co][i] = Q[i];
  red[co][HG_T] = e1;
  red[co][HG_T + 1] = e2;
  __syncthreads();
  for (int o = HG_CO / 2; o > 0; o >>= 1) {  // fixed-order tree over co
    if (co < o)
      for (int i = 0; i < HG_T + 2; ++i) red[co][i] += red[co + o][i];
    __syncthreads();
  }
  if (co > HG_T) return;
  const double E1 = red[0][HG_T] / HW, E2 = red[0][HG_T + 1] / HW;
  const double* G = gram + (long long)z * 32 * 32;
  double* o = dwi + ((long long)z * HG_C + c) * 28;
  if (co < HG_T) {
    double s = 0.0;
    for (int j = 0; j < HG_T; ++j) s += wi[j] * G[j * 32 + co];
    const double m = G[HG_T * 32 + co];
    const double gx = rho * HW * ((bb - mu) * m + s);  // sum_p G x_i
    o[co] = rho * (red[0][co] - E1 * HW * m - E2 * gx);
  } else {
    double s = 0.0;
    for (int j = 0; j < HG_T; ++j) s += wi[j] * G[HG_T * 32 + j];
    const double sg = rho * HW * ((bb - mu) + s);  // sum_p G (0 up to the rounding of mu)
    o[HG_T] = rho * (red[0][HG_T] - HW * E1 - E2 * sg);
  }
}

// the packed head gradient: conv2 weights (tap part from dWtap, image slice
// summed over images in order), conv2 bias, convimg weights and bias
__global__ void imgbr_assemble_kernel(const float* __restrict__ A, const float* __restrict__ dw2i,
                                      const double* __restrict__ dwi,
                                      const float* __restrict__ dwtap, int n, int k1pad,
                                      float* __restrict__ g_w2, float* __restrict__ g_b2,
                                      float* __restrict__ g_w1, float* __restrict__ g_b1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nw2 = HG_CO * HG_KP2, nw1 = HG_C * k1pad;
  if (i < nw2) {
    const int co = i / HG_KP2, k = i - co * HG_KP2;
    const int slab = k / 288, rem = k - slab * 288, t = rem >> 5, cl = rem & 31;
    if (slab < HG_CU / 32) {
      g_w2[i] = dwtap[(t * HG_CO + co) * HG_CU + slab * 32 + cl];
    } else {
      const int c = (slab - HG_CU / 32) * 32 + cl;
      double s = 0.0;
      for (int z = 0; z < n; ++z) s += dw2i[(((long long)z * HG_CO + co) * HG_C + c) * 9 + t];
      g_w2[i] = (float)s;
    }
    return;
  }
  int j = i - nw2;
  if (j < HG_CO) {
    double s = 0.0;
    for (int z = 0; z < n; ++z) s += A[((long long)z * HG_CO + j) * 288 + 4 * 32 + HG_T];
    g_b2[j] = (float)s;
    return;
  }
  j -= HG_CO;
  if (j < nw1) {
    const int c = j / k1pad, k = j - c * k1pad, t = k >> 2, ci = k & 3;
    double s = 0.0;
    if (t < 9 && ci < 3)
      for (int z = 0; z < n; ++z) s += dwi[((long long)z * HG_C + c) * 28 + t * 3 + ci];
    g_w1[j] = (float)s;
    return;
  }
  j -= nw1;
  if (j < HG_C) {
    double s = 0.0;
    for (int z = 0; z < n; ++z) s += dwi[((long long)z * HG_C + j) * 28 + HG_T];
    g_b1[j] = (float)s;
  }
}

}  // namespace

int pf_img_taps32(const float* img4, int n, int H, int W, float* x32, hipStream_t st) {
  if (n <= 0 || H <= 0 || W <= 0) return POSFEAT_E_INVALID;
  const long long total = (long long)n * H * W * 8;
  long long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(img_taps32_kernel, dim3((unsigned)g), dim3(256), 0, st, img4, n, H, W, x32);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

size_t pf_imgbr_grad_ws_bytes(int n) {
  return pf_align((size_t)n * HG_CO * HG_C * 9 * sizeof(float), 256) +
         pf_align((size_t)n * HG_C * 28 * sizeof(double), 256);
}

int pf_imgbr_grad(const float* A, int n, int HW, const float* w2p, const float* w1p,
                  const float* b1, const float* meanI, const float* rstdI, const double* gram,
                  const float* dwtap, float* g_w2, float* g_b2, float* g_w1, float* g_b1, void* ws,
                  size_t ws_bytes, hipStream_t st) {
  if (n <= 0 || !ws || ws_bytes < pf_imgbr_grad_ws_bytes(n)) return POSFEAT_E_WORKSPACE;
  float* dw2i = static_cast<float*>(ws);
  double* dwi = reinterpret_cast<double*>(static_cast<char*>(ws) +
                                          pf_align((size_t)n * HG_CO * HG_C * 9 * sizeof(float), 256));
  const int k1pad = posfeat_conv_packed_k(3, 3, 3);
  hipLaunchKernelGGL(imgbr_image_kernel, dim3(HG_C, n), dim3(HG_CO), 0, st, A, w2p, w1p, k1pad, b1,
                     meanI, rstdI, gram, HW, dw2i, dwi);
  PF_CHECK_LAUNCH();
  const int total = HG_CO * HG_KP2 + HG_CO + HG_C * k1pad + HG_C;
  hipLaunchKernelGGL(imgbr_assemble_kernel, dim3((total + 255) / 256), dim3(256), 0, st, A, dw2i,
                     dwi, dwtap, n, k1pad, g_w2, g_b2, g_w1, g_b1);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
