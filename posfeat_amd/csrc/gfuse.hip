// gfuse.hip -- KeypointDet's image branch folded into one 5x5 conv.
//
// head.conv2 reads cat[up4(L), G] with G = IN(convimg(img)) (DeteNet.py:
// 108-112).  Its G part, conv3x3(G; W2[:, 192:]), is linear in the raw
// convimg output c = convimg(img) + b1:  G = rstd (c - mean) per image and
// channel, so away from the image border
//
//   conv3x3(G)[p] = sum_t W2[t] rstd (sum_s W1[s] img[p+t+s-2] + b1 - mean)
//                 = conv5x5(img; Wc_b)[p] + const_b
//
// with per-image composite weights Wc_b = sum_k W2[:,k] (*) rstd_b[k] W1[k]
// (a 3x3 (*) 3x3 = 5x5 kernel over the 3 image channels) -- 2·HW·128·4·25
// instead of 2·HW·128·64·9 MACs (5.8x less), and the IN apply pass over G
// disappears.  Both convs zero-pad their own input, so the identity holds
// exactly wherever the 3x3 window of conv2 stays inside the image; the
// one-pixel border ring (where conv2 sees G's zero padding, not the
// continuation of c) is recomputed directly from the raw c.
#include "common.h"
#include "fmap.h"

namespace {

constexpr int GF_COUT = 128, GF_CG = 64, GF_CL = 192;  // conv2 out, G channels, L channels
constexpr int GF_KPAD = 128;                            // 5*5*4 = 100 -> 128

// W2's G slice transposed for the ring kernel: w2t[t][k][co]
__global__ __launch_bounds__(128) void gfuse_w2t_kernel(const float* __restrict__ w2, int k2pad,
                                                        float* __restrict__ w2t) {
  const int t = blockIdx.x / GF_CG, k = blockIdx.x % GF_CG, co = threadIdx.x;
  const int ci = GF_CL + k;
  w2t[((size_t)t * GF_CG + k) * GF_COUT + co] =
      w2[(size_t)co * k2pad + ((ci >> 5) * 9 + t) * 32 + (ci & 31)];
}

// Wc[b][co][(u*5+v)*4 + ci] (ci < 3; zero-padded to 128), bc[b][co]
__global__ __launch_bounds__(128) void gfuse_weights_kernel(
    const float* __restrict__ w2, int k2pad, const float* __restrict__ b2,
    const float* __restrict__ w1, int k1pad, const float* __restrict__ b1,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ wc,
    float* __restrict__ bc) {
  const int co = blockIdx.x, b = blockIdx.y, e = threadIdx.x;
  const float* mb = mean + (size_t)b * GF_CG;
  const float* rb = rstd + (size_t)b * GF_CG;
  const float* w2r = w2 + (size_t)co * k2pad;
  // W2 packed K index of channel 192 + k, tap t: ((ci/32)*9 + t)*32 + ci%32
  auto w2at = [&](int k, int t) {
    const int ci = GF_CL + k;
    return w2r[((ci >> 5) * 9 + t) * 32 + (ci & 31)];
  };
  float v = 0.f;
  if (e < 100) {
    const int ci = e & 3, uv = e >> 2, u = uv / 5, vv = uv - u * 5;
    if (ci < 3) {
      for (int ty = 0; ty < 3; ++ty) {
        const int sy = u - ty;
        if (sy < 0 || sy > 2) continue;
        for (int tx = 0; tx < 3; ++tx) {
          const int sx = vv - tx;
          if (sx < 0 || sx > 2) continue;
          const int t = ty * 3 + tx, s = sy * 3 + sx;
          float acc = 0.f;
          for (int k = 0; k < GF_CG; ++k)
            acc += w2at(k, t) * rb[k] * w1[(size_t)k * k1pad + s * 4 + ci];
          v += acc;
        }
      }
    }
  }
  wc[((size_t)b * GF_COUT + co) * GF_KPAD + e] = v;
  if (e == 0) {
    float acc = b2[co];
    for (int t = 0; t < 9; ++t)
      for (int k = 0; k < GF_CG; ++k) acc += w2at(k, t) * rb[k] * (b1[k] - mb[k]);
    bc[(size_t)b * GF_COUT + co] = acc;
  }
}

// Border ring: y[p] = b2 + sum_t sum_k W2[:, 192+k, t] G[p+t-1][k], G = rstd (c - mean)
// inside the image, 0 outside (conv2's zero padding).  One workgroup = RP ring
// pixels x 128 couts; the G taps go through LDS, W2 (transposed, w2t[t][k][co])
// is read coalesced across couts and reused for the RP pixels.
constexpr int GF_RP = 8;
__global__ __launch_bounds__(GF_COUT) void gfuse_ring_kernel(
    const float* __restrict__ c, int ccs, int H, int W, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ w2t, const float* __restrict__ b2,
    float* __restrict__ y, int ycs) {
  const int b = blockIdx.y, co = threadIdx.x;
  const int nring = 2 * W + 2 * (H - 2);
  __shared__ float g[GF_RP][9][GF_CG];
  __shared__ int pys[GF_RP], pxs[GF_RP];
  if (threadIdx.x < GF_RP) {
    int r = blockIdx.x * GF_RP + threadIdx.x, py = -1, px = -1;
    if (r < nring) {
      if (r < W) {
        py = 0;
        px = r;
      } else if ((r -= W) < W) {
        py = H - 1;
        px = r;
      } else if ((r -= W) < H - 2) {
        py = 1 + r;
        px = 0;
      } else {
        py = 1 + (r - (H - 2));
        px = W - 1;
      }
    }
    pys[threadIdx.x] = py;
    pxs[threadIdx.x] = px;
  }
  __syncthreads();
  const float* mb = mean + (size_t)b * GF_CG;
  const float* rb = rstd + (size_t)b * GF_CG;
  for (int i = threadIdx.x; i < GF_RP * 9 * GF_CG; i += blockDim.x) {
    const int j = i / (9 * GF_CG), rem = i - j * 9 * GF_CG, t = rem / GF_CG, k = rem - t * GF_CG;
    const int py = pys[j], px = pxs[j];
    const int qy = py + t / 3 - 1, qx = px + t % 3 - 1;
    float v = 0.f;
    if (py >= 0 && (unsigned)qy < (unsigned)H && (unsigned)qx < (unsigned)W)
      v = (c[(((size_t)b * H + qy) * W + qx) * ccs + k] - mb[k]) * rb[k];
    g[j][t][k] = v;
  }
  __syncthreads();
  float acc[GF_RP];
#pragma unroll
  for (int j = 0; j < GF_RP; ++j) acc[j] = b2[co];
  for (int tk = 0; tk < 9 * GF_CG; ++tk) {
    const float wv = w2t[(size_t)tk * GF_COUT + co];
#pragma unroll
    for (int j = 0; j < GF_RP; ++j) acc[j] += wv * (&g[j][0][0])[tk];
  }
#pragma unroll
  for (int j = 0; j < GF_RP; ++j)
    if (pys[j] >= 0) y[(((size_t)b * H + pys[j]) * W + pxs[j]) * ycs + co] = acc[j];
}

}  // namespace

// wc (n*128*128) | bc (n*128) | w2t (9*64*128)
size_t pf_gfuse_weights_floats(int n) {
  return (size_t)n * GF_COUT * (GF_KPAD + 1) + (size_t)9 * GF_CG * GF_COUT;
}

// wc: n * 128 * 128 floats (packed 5x5 weights over 4 channels), bc: n * 128,
// followed by the transposed W2 G slice the ring kernel reads
int pf_gfuse_weights(const float* w2_packed, const float* b2, const float* w1_packed,
                     const float* b1, const float* mean, const float* rstd, int n, float* wc,
                     float* bc, hipStream_t st) {
  const int k2pad = posfeat_conv_packed_k(GF_CL + GF_CG, 3, 3);
  const int k1pad = posfeat_conv_packed_k(3, 3, 3);
  hipLaunchKernelGGL(gfuse_weights_kernel, dim3(GF_COUT, n), dim3(128), 0, st, w2_packed, k2pad,
                     b2, w1_packed, k1pad, b1, mean, rstd, wc, bc);
  hipLaunchKernelGGL(gfuse_w2t_kernel, dim3(9 * GF_CG), dim3(GF_COUT), 0, st, w2_packed, k2pad,
                     bc + (size_t)n * GF_COUT);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// y (n x H x W x 128, pitch ycs) = G part of head.conv2 + b2 for every pixel:
// per-image 5x5 conv of img4 (pitch 4) with the composite weights, then the
// exact border ring from the raw convimg output c (pitch ccs)
int pf_gfuse_conv(const float* img4, const float* c, int ccs, int n, int H, int W,
                  const float* wc, const float* bc, const float* mean, const float* rstd,
                  const float* w2_packed, const float* b2, float* y, int ycs, hipStream_t st) {
  posfeat_conv_desc d{};
  d.n = 1;
  d.h = H;
  d.w = W;
  d.cin = 4;
  d.x_cstride = 4;
  d.cout = GF_COUT;
  d.kh = d.kw = 5;
  d.stride = 1;
  d.pad = 2;
  d.y_cstride = ycs;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  for (int b = 0; b < n; ++b)
    PF_TRY(pf_conv_run_tile(&d, img4 + (size_t)b * H * W * 4, wc + (size_t)b * GF_COUT * GF_KPAD,
                            bc + (size_t)b * GF_COUT, nullptr, y + (size_t)b * H * W * ycs, nullptr,
                            0, -1, st));
  (void)w2_packed;
  const int nring = 2 * W + 2 * (H - 2);
  hipLaunchKernelGGL(gfuse_ring_kernel, dim3((nring + GF_RP - 1) / GF_RP, n), dim3(GF_COUT), 0, st,
                     c, ccs, H, W, mean, rstd, bc + (size_t)n * GF_COUT, b2, y, ycs);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
