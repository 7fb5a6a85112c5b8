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
#include <algorithm>

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

// Wc[b][co][(u*5+v)*4 + ci] (ci < 3; zero-padded to 128), bc[b][co].  One
// block per (co, image): the block's W2 row slice (9 taps x 64 G channels,
// times rstd -- the product the sums below take first) and convimg's weights
// are staged in LDS once, so each of the 100 composite taps reads its operands
// from LDS instead of three dependent global loads per term (310 -> ~20 us
// per 32-image step, r16d; the side stream's kernels slow the main stream
// almost one for one).  Same terms in the same order: t outer,
// k inner, (w2 rstd) w1 -- bit-identical to the round-5 kernel.
constexpr int GW_W1S = 37;  // floats per k row of W1 in LDS (36 used: 9 taps x 4 channels)
__global__ __launch_bounds__(128) void gfuse_weights_kernel(
    const float* __restrict__ w2, int k2pad, const float* __restrict__ b2,
    const float* __restrict__ w1, int k1pad, const float* __restrict__ b1,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ wc,
    float* __restrict__ bc) {
  const int co = blockIdx.x, b = blockIdx.y, e = threadIdx.x;
  __shared__ float a_s[9][GF_CG];          // W2[co][192 + k][t] * rstd[k]
  __shared__ float w1_s[GF_CG][GW_W1S];    // W1[k][s * 4 + ci]
  __shared__ float d_s[GF_CG];             // b1[k] - mean[k]
  const float* mb = mean + (size_t)b * GF_CG;
  const float* rb = rstd + (size_t)b * GF_CG;
  const float* w2r = w2 + (size_t)co * k2pad;
  for (int i = e; i < 9 * GF_CG; i += blockDim.x) {
    const int t = i / GF_CG, k = i - t * GF_CG;
    const int ci = GF_CL + k;  // W2 packed K index of channel 192 + k, tap t
    a_s[t][k] = w2r[((ci >> 5) * 9 + t) * 32 + (ci & 31)] * rb[k];
  }
  for (int i = e; i < GF_CG * 36; i += blockDim.x) {
    const int k = i / 36, j = i - k * 36;
    w1_s[k][j] = w1[(size_t)k * k1pad + j];
  }
  if (e < GF_CG) d_s[e] = b1[e] - mb[e];
  __syncthreads();
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
          const int t = ty * 3 + tx, s4 = (sy * 3 + sx) * 4 + ci;
          float acc = 0.f;
          for (int k = 0; k < GF_CG; ++k) acc += a_s[t][k] * w1_s[k][s4];
          v += acc;
        }
      }
    }
  }
  wc[((size_t)b * GF_COUT + co) * GF_KPAD + e] = v;
  if (e == 0) {
    float acc = b2[co];
    for (int t = 0; t < 9; ++t)
      for (int k = 0; k < GF_CG; ++k) acc += a_s[t][k] * d_s[k];
    bc[(size_t)b * GF_COUT + co] = acc;
  }
}

// Border ring: y[p] = b2 + sum_t sum_k W2[:, 192+k, t] G[p+t-1][k], G = rstd (c - mean)
// inside the image, 0 outside (conv2's zero padding).  One workgroup = RP ring
// pixels x 128 couts; W2 (transposed, w2t[t][k][co], 295 KB) is read coalesced
// across couts once per block and reused for the RP pixels, so RP sets the
// weight traffic: 64 pixels per block (16 before: 4480 blocks re-read 1.3 GB of
// w2t from L2 per 32-image step, 1.06 ms).  The G taps go through LDS one
// conv2 tap t at a time (g[RP][64], 16 KB): the sums run in the same order as
// before -- t outer, k inner -- so the values are bit-identical.  y == nullptr:
// into the ring buffer ring[b][r][128] instead (r = the ring index below, the
// order pf_ring_index in fmap.h restates), for up4tap_gcombine_kernel.
constexpr int GF_RP = 64;  // ring pixels per block
__global__ __launch_bounds__(2 * GF_COUT) PF_NO_PK_FP32 void gfuse_ring_kernel(
    const float* __restrict__ c, int ccs, const float* __restrict__ img4,
    const float* __restrict__ w1, int k1pad, const float* __restrict__ b1, int H, int W,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ w2t,
    const float* __restrict__ b2, float* __restrict__ y, int ycs, float* __restrict__ ring) {
  const int b = blockIdx.y, co = threadIdx.x % GF_COUT;
  const int nring = 2 * W + 2 * (H - 2);
  __shared__ __attribute__((aligned(16))) float g[GF_RP][GF_CG];
  // convimg's input taps at every ring pixel's position q = p + t - 1 of the
  // current conv2 tap, loaded once per block (the 64 channel threads share
  // them): xs[j][s * 3 + ch]
  __shared__ float xs[GF_RP][27];
  __shared__ float w1s[GF_CG][27];
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
  if (!c) {
    for (int i = threadIdx.x; i < GF_CG * 27; i += blockDim.x) {
      const int k = i / 27, e = i - k * 27;
      w1s[k][e] = w1[(size_t)k * k1pad + (e / 3) * 4 + e % 3];
    }
  }
  const float* mb = mean + (size_t)b * GF_CG;
  const float* rb = rstd + (size_t)b * GF_CG;
  // two halves of the block take GF_RP / 2 ring pixels each (same cout)
  constexpr int HP = GF_RP / 2;
  const int j0 = (threadIdx.x / GF_COUT) * HP;
  float acc[HP];
  const float bias = b2[co];
#pragma unroll
  for (int j = 0; j < HP; ++j) acc[j] = bias;
  for (int t = 0; t < 9; ++t) {
    pf_syncthreads();  // pys / w1s written; the previous tap's g and xs read
    if (!c) {  // zero-padded image taps around q (0 outside the image)
      for (int i = threadIdx.x; i < GF_RP * 27; i += blockDim.x) {
        const int jj = i / 27, e = i - jj * 27;
        const int s9 = e / 3, ch = e - s9 * 3;
        const int qy = pys[jj] + t / 3 - 1, qx = pxs[jj] + t % 3 - 1;
        const int iy = qy + s9 / 3 - 1, ix = qx + s9 % 3 - 1;
        float v = 0.f;
        if (pys[jj] >= 0 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
          v = img4[(((size_t)b * H + iy) * W + ix) * 4 + ch];
        xs[jj][e] = v;
      }
      pf_syncthreads();
    }
    for (int i = threadIdx.x; i < GF_RP * GF_CG; i += blockDim.x) {
      const int jj = i / GF_CG, k = i - jj * GF_CG;
      const int py = pys[jj], px = pxs[jj];
      const int qy = py + t / 3 - 1, qx = px + t % 3 - 1;
      float v = 0.f;
      if (py >= 0 && (unsigned)qy < (unsigned)H && (unsigned)qx < (unsigned)W) {
        float cv;
        if (c) {
          cv = c[(((size_t)b * H + qy) * W + qx) * ccs + k];
        } else {  // convimg at q, the conv's own tap order (zero taps add +0: exact)
          cv = b1[k];
          for (int s9 = 0; s9 < 9; ++s9) {
            const float* xv = &xs[jj][s9 * 3];
            const float* wk = &w1s[k][s9 * 3];
            cv += wk[0] * xv[0] + wk[1] * xv[1] + wk[2] * xv[2];
          }
        }
        v = (cv - mb[k]) * rb[k];
      }
      g[jj][k] = v;
    }
    pf_syncthreads();
    // four k per step: one broadcast ds_read_b128 of g per pixel, the same
    // sequential accumulation order as one k at a time
    for (int k = 0; k < GF_CG; k += 4) {
      float wv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) wv[u] = w2t[(size_t)(t * GF_CG + k + u) * GF_COUT + co];
#pragma unroll
      for (int j = 0; j < HP; ++j) {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(&g[j0 + j][k]);
        acc[j] += wv[0] * gv.x;
        acc[j] += wv[1] * gv.y;
        acc[j] += wv[2] * gv.z;
        acc[j] += wv[3] * gv.w;
      }
    }
  }
  if (!y) {
#pragma unroll
    for (int j = 0; j < HP; ++j) {
      const int r = blockIdx.x * GF_RP + j0 + j;
      if (r < nring) ring[((size_t)b * nring + r) * GF_COUT + co] = acc[j];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < HP; ++j)
    if (pys[j0 + j] >= 0) y[(((size_t)b * H + pys[j0 + j]) * W + pxs[j0 + j]) * ycs + co] = acc[j];
}


// ---- instance-norm statistics of convimg WITHOUT running convimg ------------
// c_k(p) = b1_k + w_k . x(p), x(p) = the 27 zero-padded 3x3 x 3-channel image
// taps around p, so per image mean_k = b1_k + w_k . E[x] and var_k =
// w_k^T (E[x x^T] - E[x] E[x]^T) w_k.  With x extended by a constant 1 (row
// 27) the moments are one Gram matrix G = X^T X of the [HW x 32] im2col
// matrix X: G[27][j] = sum x_j, G[i][j] = sum x_i x_j.  X^T X on fp32 MFMA is
// one v_mfma_f32_32x32x2_f32 per pixel PAIR whose A and B operands are the
// SAME register (lane l: x_{l%32} of pixel 2s + l/32).  gfuse_imgmom_kernel:
// one block per band of 4 rows (staged in LDS), each wave a quarter of the
// band's pixel pairs; the four 32x32 accumulators are summed into an fp64
// band partial.  gfuse_imgstats_kernel sums the band partials in order (fp64)
// and forms mean / rstd for the 64 convimg channels.  Replaces the 3x3 4->64
// conv over the full-resolution image (and its 629 MB output at B = 8,
// 480x640): the only other reader of that output, the border ring,
// recomputes the few values it needs from the image.
constexpr int IM_TAPS = 27, IM_G = 32;  // moments: 27 taps + the constant row
constexpr int IM_ROWS = 4;              // output rows per band

__global__ __launch_bounds__(256) void gfuse_imgmom_kernel(const float* __restrict__ img4, int H,
                                                           int W, double* __restrict__ part) {
  extern __shared__ float tile[];  // [IM_ROWS + 2][W + 2][3], then the fp64 reduction
  const int b = blockIdx.y;
  const int TW = W + 2, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;  // 4 waves
  const float* ib = img4 + (long long)b * H * W * 4;
  const int nband = (H + IM_ROWS - 1) / IM_ROWS;
  // a block walks bands blockIdx.x, + gridDim.x, ...: each band's fp32 MFMA sum
  // is added into per-lane fp64 totals (the per-band rounding of one band /
  // block; few blocks leave the CUs to the main stream's kernels)
  double tot[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) tot[r] = 0.0;
  for (int band = blockIdx.x; band < nband; band += gridDim.x) {
  const int r0 = band * IM_ROWS;
  pf_syncthreads();  // the previous band's tile is consumed
  for (int i = threadIdx.x; i < (IM_ROWS + 2) * TW; i += blockDim.x) {
    const int ty = i / TW, tx = i - ty * TW;
    const int y = r0 - 1 + ty, x = tx - 1;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
      v = *reinterpret_cast<const f32x4*>(ib + ((long long)y * W + x) * 4);
    tile[i * 3] = v.x;
    tile[i * 3 + 1] = v.y;
    tile[i * 3 + 2] = v.z;
  }
  pf_syncthreads();
  // this lane's moment index i = lane % 32: tap (ky, kx), channel c, or 27: 1
  const int i = lane & 31;
  const int ti = i / 3, ci = i - ti * 3;
  const int off = i < IM_TAPS ? ((ti / 3) * TW + ti % 3) * 3 + ci : 0;
  const float cst = i == IM_TAPS ? 1.f : 0.f;
  const bool tap = i < IM_TAPS;
  // wave w owns output row r0 + w; two interleaved accumulator chains so
  // consecutive MFMAs do not wait on each other
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  if (r0 + wave < H) {
    const float* trow = tile + wave * TW * 3 + off + (lane >> 5) * 3;
    int s = 0;
    for (; s + 8 <= W / 2; s += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = tap ? trow[(2 * (s + u)) * 3] : cst;
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u], v[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u + 1], v[u + 1], acc1, 0, 0, 0);
      }
    }
    for (; s < W / 2; ++s) {
      const float v = tap ? trow[(2 * s) * 3] : cst;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v, v, acc0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) tot[r] += (double)acc0[r] + (double)acc1[r];
  }
  pf_syncthreads();  // the tile is dead: reuse LDS for the wave sum
  double* red = reinterpret_cast<double*>(tile);  // [4 waves][32][32]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gi = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), gj = lane & 31;
    red[(wave * IM_G + gi) * IM_G + gj] = tot[r];
  }
  pf_syncthreads();
  for (int e = threadIdx.x; e < IM_G * IM_G; e += blockDim.x)
    part[((long long)b * gridDim.x + blockIdx.x) * IM_G * IM_G + e] =
        (red[e] + red[IM_G * IM_G + e]) + (red[2 * IM_G * IM_G + e] + red[3 * IM_G * IM_G + e]);
}

// one block per image, one thread per Gram entry: sum the band partials
// (fixed order), then per convimg channel k: mean = b1 + w.m,
// var = w^T (S/HW - m m^T) w
__global__ __launch_bounds__(1024) void gfuse_imgstats_kernel(const double* __restrict__ part,
                                                             int nband, int HW,
                                                             const float* __restrict__ w1,
                                                             int k1pad, const float* __restrict__ b1,
                                                             float eps, float* __restrict__ mean,
                                                             float* __restrict__ rstd,
                                                             double* __restrict__ gram) {
  __shared__ double G[IM_G * IM_G];
  const int b = blockIdx.x;
  {
    const int e = threadIdx.x;
    const double* pe = part + (long long)b * nband * IM_G * IM_G + e;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int k = 0;
    for (; k + 4 <= nband; k += 4) {
      s0 += pe[(k + 0) * IM_G * IM_G];
      s1 += pe[(k + 1) * IM_G * IM_G];
      s2 += pe[(k + 2) * IM_G * IM_G];
      s3 += pe[(k + 3) * IM_G * IM_G];
    }
    for (; k < nband; ++k) s0 += pe[k * IM_G * IM_G];
    G[e] = ((s0 + s1) + (s2 + s3)) / HW;  // E[x_i x_j], row 27: E[x_j]
    if (gram) gram[(long long)b * IM_G * IM_G + e] = G[e];  // kept for the training backward
  }
  pf_syncthreads();
  const int k = threadIdx.x;
  if (k >= GF_CG) return;
  double w[IM_TAPS];
  for (int i = 0; i < IM_TAPS; ++i) {
    const int t = i / 3, c = i - t * 3;
    w[i] = (double)w1[(size_t)k * k1pad + t * 4 + c];  // packed (kh, kw, cin4)
  }
  const double* m = G + IM_TAPS * IM_G;
  double mu = 0.0;
  for (int i = 0; i < IM_TAPS; ++i) mu += w[i] * m[i];
  double q = 0.0;
  for (int i = 0; i < IM_TAPS; ++i) {
    double t = 0.0;
    for (int j = 0; j < IM_TAPS; ++j) t += (G[i * IM_G + j] - m[i] * m[j]) * w[j];
    q += w[i] * t;
  }
  if (q < 0.0) q = 0.0;
  mean[b * GF_CG + k] = (float)(mu + (double)b1[k]);
  rstd[b * GF_CG + k] = (float)(1.0 / sqrt(q + (double)eps));
}

// ---- the folded 5x5 conv on fp32 MFMA ---------------------------------------
// y[p][co] = bc_b[co] + sum_{t < 25, c < 4} Wc_b[co][t][c] img4[p + t - (2,2)][c]
// Block = 8 x 32 output pixels of one image; wave w owns rows 2w, 2w+1 (two
// 32-pixel MFMA row blocks) x all 128 couts.  The 12 x 36 x 4 image patch and
// the image's 128 x 26 x 4 weights (tap 25 zero, rows padded to 108 floats:
// conflict-free ds_read_b128) sit in LDS.  K = taps x 4 channels: lane half h
// reads tap 2g + h of group g (16 B = 4 channels), MFMA j contracts channel j
// of taps (2g, 2g+1) -- the same pairing on the weights.
constexpr int G5_TR = 8, G5_TC = 32, G5_PR = G5_TR + 4, G5_PC = G5_TC + 4, G5_WP = 108;

__global__ __launch_bounds__(256) void gfuse_conv5_kernel(const float* __restrict__ img4, int H,
                                                          int W, const float* __restrict__ wc,
                                                          const float* __restrict__ bc,
                                                          float* __restrict__ y, int ycs) {
  __shared__ __attribute__((aligned(16))) float sw[GF_COUT * G5_WP];
  __shared__ __attribute__((aligned(16))) float sp[G5_PR * G5_PC * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int b = blockIdx.y;
  const int ntc = (W + G5_TC - 1) / G5_TC;
  const int ty0 = (blockIdx.x / ntc) * G5_TR, tx0 = (blockIdx.x % ntc) * G5_TC;
  const float* ib = img4 + (long long)b * H * W * 4;
  const float* wb = wc + (long long)b * GF_COUT * GF_KPAD;
  for (int i = tid; i < GF_COUT * 26; i += 256) {  // weights: [co][tap][4] -> padded rows
    const int co = i / 26, t = i - co * 26;
    *reinterpret_cast<f32x4*>(sw + co * G5_WP + t * 4) =
        *reinterpret_cast<const f32x4*>(wb + (long long)co * GF_KPAD + t * 4);
  }
  for (int i = tid; i < G5_PR * G5_PC; i += 256) {  // image patch, zero outside
    const int py = i / G5_PC, px = i - py * G5_PC;
    const int yy = ty0 - 2 + py, xx = tx0 - 2 + px;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
      v = *reinterpret_cast<const f32x4*>(ib + ((long long)yy * W + xx) * 4);
    *reinterpret_cast<f32x4*>(sp + i * 4) = v;
  }
  pf_syncthreads();
  f32x16 acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  const int col = lane & 31;
#pragma unroll
  for (int g = 0; g < 13; ++g) {
    const int t = 2 * g + h;
    const int ta = t < 25 ? t : 24;  // tap 25: zero weights (any finite A)
    const int u = ta / 5, v = ta - u * 5;
    f32x4 a[2], bw[4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
      a[mi] = *reinterpret_cast<const f32x4*>(sp + (((2 * wave + mi + u) * G5_PC) + col + v) * 4);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      bw[ni] = *reinterpret_cast<const f32x4*>(sw + (ni * 32 + col) * G5_WP + t * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi][j], bw[ni][j], acc[mi][ni],
                                                              0, 0, 0);
  }
  // acc[mi][ni][r]: pixel (row 2w + mi, column (r&3) + 8(r>>2) + 4h), cout ni*32 + lane%32
  const float* bcb = bc + (long long)b * GF_COUT;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int yy = ty0 + 2 * wave + mi;
    if (yy >= H) continue;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int co = ni * 32 + col;
      const float bias = bcb[co];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int xx = tx0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (xx < W) y[((long long)(b * H + yy) * W + xx) * ycs + co] = acc[mi][ni][r] + bias;
      }
    }
  }
}

// The same conv with bf16x6 products (conv.hip §bf16x6; the default
// arithmetic): K = 28 taps x 4 channels (taps 25..27 zero) in 7 k16 steps of
// v_mfma_f32_32x32x16_bf16 -- lane half h holds taps 4g + 2h, 4g + 2h + 1 (8
// values) of step g for the pixel and for the weights, both split in
// registers into three bf16 terms, six products per pair.  2.5x fewer
// matrix-core cycles than the fp32 form.  Weight rows padded to 116 floats
// (29 16-B slots, odd: conflict-free ds_read_b128).
constexpr int G6_WP = 116;

__global__ __launch_bounds__(256) void gfuse_conv5_bf6_kernel(const float* __restrict__ img4,
                                                              int H, int W,
                                                              const float* __restrict__ wc,
                                                              const float* __restrict__ bc,
                                                              float* __restrict__ y, int ycs) {
  __shared__ __attribute__((aligned(16))) float sw[GF_COUT * G6_WP];
  __shared__ __attribute__((aligned(16))) float sp[G5_PR * G5_PC * 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int b = blockIdx.y;
  const int ntc = (W + G5_TC - 1) / G5_TC;
  const int ty0 = (blockIdx.x / ntc) * G5_TR, tx0 = (blockIdx.x % ntc) * G5_TC;
  const float* ib = img4 + (long long)b * H * W * 4;
  const float* wb = wc + (long long)b * GF_COUT * GF_KPAD;
  for (int i = tid; i < GF_COUT * 28; i += 256) {  // [co][tap][4], taps 25..27 zero
    const int co = i / 28, t = i - co * 28;
    const f32x4 v = t < 25 ? *reinterpret_cast<const f32x4*>(wb + (long long)co * GF_KPAD + t * 4)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(sw + co * G6_WP + t * 4) = v;
  }
  for (int i = tid; i < G5_PR * G5_PC; i += 256) {
    const int py = i / G5_PC, px = i - py * G5_PC;
    const int yy = ty0 - 2 + py, xx = tx0 - 2 + px;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
      v = *reinterpret_cast<const f32x4*>(ib + ((long long)yy * W + xx) * 4);
    *reinterpret_cast<f32x4*>(sp + i * 4) = v;
  }
  pf_syncthreads();
  f32x16 acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  const int col = lane & 31;
#pragma unroll
  for (int g = 0; g < 7; ++g) {
    const int t0 = 4 * g + 2 * h, t1 = t0 + 1;
    const int a0 = t0 < 25 ? t0 : 24, a1 = t1 < 25 ? t1 : 24;  // zero weights beyond 24
    g6_u32x4 ah[2], am[2], al[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int r = 2 * wave + mi;
      g6_split(*reinterpret_cast<const f32x4*>(sp + (((r + a0 / 5) * G5_PC) + col + a0 % 5) * 4),
               *reinterpret_cast<const f32x4*>(sp + (((r + a1 / 5) * G5_PC) + col + a1 % 5) * 4),
               ah[mi], am[mi], al[mi]);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const float* wr = sw + (ni * 32 + col) * G6_WP + t0 * 4;
      g6_u32x4 bh, bm, bl;
      g6_split(*reinterpret_cast<const f32x4*>(wr), *reinterpret_cast<const f32x4*>(wr + 4), bh,
               bm, bl);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        f32x16 c = acc[mi][ni];
        c = g6_mfma(ah[mi], bh, c);
        c = g6_mfma(ah[mi], bm, c);
        c = g6_mfma(am[mi], bh, c);
        c = g6_mfma(ah[mi], bl, c);
        c = g6_mfma(al[mi], bh, c);
        c = g6_mfma(am[mi], bm, c);
        acc[mi][ni] = c;
      }
    }
  }
  const float* bcb = bc + (long long)b * GF_COUT;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int yy = ty0 + 2 * wave + mi;
    if (yy >= H) continue;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int co = ni * 32 + col;
      const float bias = bcb[co];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int xx = tx0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (xx < W) y[((long long)(b * H + yy) * W + xx) * ycs + co] = acc[mi][ni][r] + bias;
      }
    }
  }
}
// ---- the folded 5x5 conv: pre-split weights, 3-channel K = 80 (default) ----
// k = dy*16 + dx*3 + c (dy, dx < 5, c < 3; k % 16 == 15 has zero weight): one
// k16 step per patch row dy, whose 15 taps x channels are 15 CONSECUTIVE
// floats of a 3-channel-packed patch row (tile pixel x starts at float 3x).
// MFMA A = the image's weights, pre-split once per forward into three bf16
// planes [co][80] (gfuse_wsplit_kernel) and staged in LDS once per block;
// B = the pixels' taps, split in registers (lane half h: floats 3x + 8h .. +7
// of row dy; the 16th is the next pixel's channel 0, against a zero weight).
// 80 instead of the 4-channel form's 112 k per output: 29 % fewer
// matrix-core cycles, and no weight split per wave.  acc rows = couts, so a
// lane holds 4 consecutive couts of one pixel: float4 stores.  Block = 8
// waves on a 16-row x 32-pixel tile (wave = 2 pixel rows x 128 couts),
// persistent over the tiles of one image; the next tile's patch is loaded
// into registers while the current one is multiplied.
constexpr int G8_K = 80, G8_KP = 88;  // K, LDS row pitch (bf16; 176 B: conflict-free b128 per 16 lanes)
constexpr int G8_TR = 16, G8_TC = 32, G8_PR = G8_TR + 4, G8_PC = G8_TC + 4;
constexpr int G8_PW = 112;            // patch row pitch (floats): 36 px x 3 + 4 zero
constexpr int G8_NPX = G8_PR * G8_PC;  // 720 patch pixels, <= 2 per thread

__global__ void gfuse_wsplit_kernel(const float* __restrict__ wc, int n,
                                    unsigned short* __restrict__ wp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * GF_COUT * G8_K) return;
  const int k = i % G8_K, r = i / G8_K, co = r % GF_COUT, b = r / GF_COUT;
  const int dy = k >> 4, q = k & 15, dx = q / 3, c = q - dx * 3;
  const float v = q < 15 ? wc[((long long)b * GF_COUT + co) * GF_KPAD + (dy * 5 + dx) * 4 + c] : 0.f;
  unsigned h, m, l;
  pf_split3_pair(v, 0.f, h, m, l);
  const long long pl = (long long)GF_COUT * G8_K;
  unsigned short* o = wp + (long long)b * 3 * pl + (long long)co * G8_K + k;
  o[0] = (unsigned short)(h & 0xffffu);
  o[pl] = (unsigned short)(m & 0xffffu);
  o[2 * pl] = (unsigned short)(l & 0xffffu);
}

__global__ __launch_bounds__(512) void gfuse_conv5_k80_kernel(const float* __restrict__ img4, int H,
                                                              int W,
                                                              const unsigned short* __restrict__ wp,
                                                              const float* __restrict__ bc,
                                                              float* __restrict__ y, int ycs) {
  __shared__ __attribute__((aligned(16))) unsigned short sw[3 * GF_COUT * G8_KP];
  __shared__ __attribute__((aligned(16))) float sp[G8_PR * G8_PW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, col = lane & 31;
  const int b = blockIdx.y;
  const int ntc = (W + G8_TC - 1) / G8_TC, ntiles = ntc * ((H + G8_TR - 1) / G8_TR);
  const float* ib = img4 + (long long)b * H * W * 4;
  {  // the image's weight planes -> LDS rows of 88 (8-element pieces)
    const unsigned short* wb = wp + (long long)b * 3 * GF_COUT * G8_K;
    for (int i = tid; i < 3 * GF_COUT * (G8_K / 8); i += 512) {
      const int row = i / (G8_K / 8), piece = i - row * (G8_K / 8);
      *reinterpret_cast<uint4*>(sw + row * G8_KP + piece * 8) =
          *reinterpret_cast<const uint4*>(wb + (long long)row * G8_K + piece * 8);
    }
  }
  for (int i = tid; i < G8_PR * 4; i += 512)  // the zero tail of every patch row
    sp[(i >> 2) * G8_PW + 108 + (i & 3)] = 0.f;
  auto load_patch = [&](int t, f32x4 (&v)[2]) {
    const int ty0 = (t / ntc) * G8_TR, tx0 = (t % ntc) * G8_TC;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + j * 512;
      v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i < G8_NPX) {
        const int py = i / G8_PC, px = i - py * G8_PC;
        const int yy = ty0 - 2 + py, xx = tx0 - 2 + px;
        if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
          v[j] = *reinterpret_cast<const f32x4*>(ib + ((long long)yy * W + xx) * 4);
      }
    }
  };
  auto store_patch = [&](const f32x4 (&v)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + j * 512;
      if (i < G8_NPX) {
        const int py = i / G8_PC, px = i - py * G8_PC;
        float* d = sp + py * G8_PW + px * 3;
        d[0] = v[j].x;
        d[1] = v[j].y;
        d[2] = v[j].z;
      }
    }
  };
  const float* bcb = bc + (long long)b * GF_COUT;
  f32x4 pv[2];
  int t = blockIdx.x;
  if (t < ntiles) load_patch(t, pv);
  for (; t < ntiles; t += gridDim.x) {
    pf_syncthreads();  // the previous tile's patch is consumed
    store_patch(pv);
    pf_syncthreads();
    if (t + (int)gridDim.x < ntiles) load_patch(t + gridDim.x, pv);  // in flight during the MFMAs
    f32x16 acc[4][2];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 5; ++dy) {
      g6_u32x4 bh[2], bm[2], bl[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const float* pr = sp + (2 * wave + ni + dy) * G8_PW + 3 * col + 8 * h;
        f32x4 p0, p1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          p0[j] = pr[j];
          p1[j] = pr[4 + j];
        }
        g6_split(p0, p1, bh[ni], bm[ni], bl[ni]);
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const unsigned short* wr = sw + (mi * 32 + col) * G8_KP + dy * 16 + 8 * h;
        const g6_u32x4 ah = *reinterpret_cast<const g6_u32x4*>(wr);
        const g6_u32x4 am = *reinterpret_cast<const g6_u32x4*>(wr + GF_COUT * G8_KP);
        const g6_u32x4 al = *reinterpret_cast<const g6_u32x4*>(wr + 2 * GF_COUT * G8_KP);
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          f32x16 c = acc[mi][ni];
          c = g6_mfma(ah, bh[ni], c);
          c = g6_mfma(ah, bm[ni], c);
          c = g6_mfma(am, bh[ni], c);
          c = g6_mfma(ah, bl[ni], c);
          c = g6_mfma(al, bh[ni], c);
          c = g6_mfma(am, bm[ni], c);
          acc[mi][ni] = c;
        }
      }
    }
    // acc[mi][ni][r]: cout mi*32 + (r&3) + 8(r>>2) + 4h, pixel (row 2*wave + ni, column col)
    const int ty0 = (t / ntc) * G8_TR, tx0 = (t % ntc) * G8_TC;
    const int xx = tx0 + col;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int yy = ty0 + 2 * wave + ni;
      if (yy >= H || xx >= W) continue;
      float* yp = y + ((long long)(b * H + yy) * W + xx) * ycs;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = mi * 32 + 8 * j + 4 * h;
          const f32x4 bv = *reinterpret_cast<const f32x4*>(bcb + co);
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = acc[mi][ni][4 * j + e] + bv[e];
          *reinterpret_cast<f32x4*>(yp + co) = o;
        }
    }
  }
}

bool gfuse_k80_on() {
  static const bool on = [] {
    const char* e = pf_ab_getenv("POSFEAT_GFUSE_K80");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

size_t pf_gfuse_wplanes_bytes(int n) { return (size_t)n * 3 * GF_COUT * G8_K * 2; }

// A/B timing ablation of the image branch (POSFEAT_SIDE_ABL, A/B build only;
// wrong results): bit 1 skips the border-ring kernel, 2 the image-moment
// kernel, 4 the composite-weight kernel
static int side_abl() {
  static const int v = [] {
    const char* e = pf_ab_getenv("POSFEAT_SIDE_ABL");
    return e ? atoi(e) : 0;
  }();
  return v;
}

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
  if (!(side_abl() & 4))
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
                  const float* w2_packed, const float* b2, float* y, int ycs, hipStream_t st,
                  const float* w1_packed, const float* b1, unsigned short* wplanes) {
  if (!c && !(w1_packed && b1)) return POSFEAT_E_INVALID;
  if (ycs % 4 || n <= 0) return POSFEAT_E_INVALID;
  const int ntiles = ((W + G5_TC - 1) / G5_TC) * ((H + G5_TR - 1) / G5_TR);
  if (pf_conv_precision() >= 1 && wplanes && gfuse_k80_on()) {
    const int tot = n * GF_COUT * G8_K;
    hipLaunchKernelGGL(gfuse_wsplit_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, wc, n,
                       wplanes);
    const int nt8 = ((W + G8_TC - 1) / G8_TC) * ((H + G8_TR - 1) / G8_TR);
    // persistent blocks (one image's tiles each): POSFEAT_GFUSE_BLOCKS in
    // total over the batch (default 64, at least one per image); fewer leave
    // CUs to the main stream; tiles are independent, so the count never
    // changes results
    static const int tot_blocks = [] {
      const char* e = pf_ab_getenv("POSFEAT_GFUSE_BLOCKS");
      // r3w sweep (B = 8): 512 820, 96 830, 64 841, 48 841, 32 837 img/s;
      // r6w (B = 32, bf6d main stream, two pairs): 32 977.1, 64 971.4, 128
      // 970.2 -- but at 32 the longer side stream lands on iconv3's GEMM
      // (2.39 ms, the dominant launch; r6x), so the default stays 64
      const int v = e ? atoi(e) : 64;
      return v > 0 ? v : 64;
    }();
    const int per_img = std::max(1, std::min(nt8, (tot_blocks + n - 1) / n));
    hipLaunchKernelGGL(gfuse_conv5_k80_kernel, dim3(per_img, n), dim3(512), 0, st, img4, H, W,
                       wplanes, bc, y, ycs);
  } else if (pf_conv_precision() >= 1)  // bf16x6 products (the default conv arithmetic)
    hipLaunchKernelGGL(gfuse_conv5_bf6_kernel, dim3(ntiles, n), dim3(256), 0, st, img4, H, W, wc,
                       bc, y, ycs);
  else
    hipLaunchKernelGGL(gfuse_conv5_kernel, dim3(ntiles, n), dim3(256), 0, st, img4, H, W, wc, bc,
                       y, ycs);
  PF_CHECK_LAUNCH();
  (void)w2_packed;
  const int k1pad = posfeat_conv_packed_k(3, 3, 3);
  const int nring = 2 * W + 2 * (H - 2);
  hipLaunchKernelGGL(gfuse_ring_kernel, dim3((nring + GF_RP - 1) / GF_RP, n), dim3(2 * GF_COUT), 0, st,
                     c, ccs, img4, w1_packed, k1pad, b1, H, W, mean, rstd,
                     bc + (size_t)n * GF_COUT, b2, y, ycs, nullptr);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// ---- the border ring for the fused head, in two passes ----------------------
// gfuse_ring_kernel recomputes convimg's normalised output G at each ring
// pixel's nine conv2 taps (64 channels x 27 MACs per tap, each value three
// times over, since neighbouring ring pixels share taps) and contracts the
// 576 (tap, channel) terms per output on the VALU: 0.66-0.70 ms per 32-image
// step on the side stream, where it slows the main stream's kernels almost
// one for one (r16d: the step 1.4 % faster without it).  Here:
// (1) gfuse_band_kernel: G once at every position a ring pixel's taps reach
//     inside the image -- the border itself (ring 0, pf_ring_index order)
//     and the ring one pixel in (ring 1, the border of the inner
//     (H-2) x (W-2) image) -- band[b][pos][64];
// (2) gfuse_ring_mfma_kernel: y_ring[r][co] = b2[co] + sum_t sum_k
//     W2[co][192+k][t] G(q_t(r))[k] as a gathered [64 ring pixels x 576] x
//     [576 x 128] product on the fp32 matrix cores (v_mfma_f32_32x32x2_f32:
//     fp32 products, fp32 accumulation -- the VALU form's arithmetic class, in
//     another order), taps outside the image contributing 0 (conv2's zero
//     padding of G).
__host__ __device__ inline int gf_nring(int H, int W) { return 2 * W + 2 * (H - 2); }
__host__ __device__ inline int gf_nband(int H, int W) {
  return gf_nring(H, W) + gf_nring(H - 2, W - 2);
}
// (Y, X) of ring index r of an H x W image (the inverse of pf_ring_index)
__device__ __forceinline__ void gf_ring_pos(int r, int H, int W, int& Y, int& X) {
  if (r < W) {
    Y = 0;
    X = r;
  } else if (r < 2 * W) {
    Y = H - 1;
    X = r - W;
  } else if (r < 2 * W + H - 2) {
    Y = 1 + (r - 2 * W);
    X = 0;
  } else {
    Y = 1 + (r - 2 * W - (H - 2));
    X = W - 1;
  }
}
// band index of position (Y, X): ring 0, then ring 1; -1 outside the image or
// deeper inside (no ring pixel's tap lands there)
__device__ __forceinline__ int gf_band_index(int Y, int X, int H, int W) {
  if ((unsigned)Y >= (unsigned)H || (unsigned)X >= (unsigned)W) return -1;
  if (Y == 0 || Y == H - 1 || X == 0 || X == W - 1) return pf_ring_index(Y, X, H, W);
  if (Y == 1 || Y == H - 2 || X == 1 || X == W - 2)
    return gf_nring(H, W) + pf_ring_index(Y - 1, X - 1, H - 2, W - 2);
  return -1;
}

// band[b][pos][k] = (c(q)[k] - mean[k]) rstd[k], c = convimg's raw output
// (read from c when given, else recomputed from the zero-padded image in the
// ring kernel's tap order).  Block = GB_POS positions x 64 channels (thread
// = channel, one position per wave step); convimg's 64 x 36 weights in LDS
// (a lane per channel would otherwise read 64 different rows per load)
constexpr int GB_POS = 16;  // positions per block
__global__ __launch_bounds__(256) void gfuse_band_kernel(
    const float* __restrict__ c, int ccs, const float* __restrict__ img4,
    const float* __restrict__ w1, int k1pad, const float* __restrict__ b1, int H, int W,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ band) {
  __shared__ float w1s[GF_CG][37];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int nb = gf_nband(H, W), n0 = gf_nring(H, W);
  if (!c)
    for (int i = tid; i < GF_CG * 36; i += 256) {
      const int k = i / 36, j = i - k * 36;
      w1s[k][j] = w1[(size_t)k * k1pad + j];
    }
  pf_syncthreads();
  const int k = tid & 63;
  const float mk = mean[(size_t)b * GF_CG + k], rk = rstd[(size_t)b * GF_CG + k];
  const float bk = c ? 0.f : b1[k];
  for (int j = tid >> 6; j < GB_POS; j += 4) {
    const int pos = blockIdx.x * GB_POS + j;
    if (pos >= nb) break;
    int Y, X;
    if (pos < n0) {
      gf_ring_pos(pos, H, W, Y, X);
    } else {
      gf_ring_pos(pos - n0, H - 2, W - 2, Y, X);
      ++Y;
      ++X;
    }
    float cv;
    if (c) {
      cv = c[(((size_t)b * H + Y) * W + X) * ccs + k];
    } else {
      cv = bk;
      for (int s9 = 0; s9 < 9; ++s9) {
        const int iy = Y + s9 / 3 - 1, ix = X + s9 % 3 - 1;
        float x0 = 0.f, x1 = 0.f, x2 = 0.f;
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
          const float* xp = img4 + (((size_t)b * H + iy) * W + ix) * 4;
          x0 = xp[0];
          x1 = xp[1];
          x2 = xp[2];
        }
        cv += w1s[k][s9 * 4] * x0 + w1s[k][s9 * 4 + 1] * x1 + w1s[k][s9 * 4 + 2] * x2;
      }
    }
    band[((size_t)b * nb + pos) * GF_CG + k] = (cv - mk) * rk;
  }
}

// Block = 64 ring pixels of one image x all 128 outputs, 4 waves: wave w owns
// pixels 32 (w & 1) .. + 32 and outputs 64 (w >> 1) .. + 64 (two 32 x 32
// fp32-MFMA tiles).  The pixels' band indices of all nine conv2 taps are
// tabulated once; a tap no pixel of the block reaches inside the image (the
// outward row or column of a straight ring segment: 3 of 9) is skipped; the
// next tap's gathered G rows and W2 slice are loaded into registers while the
// current tap's 64 MFMAs run, then stored to LDS.
constexpr int GR_P = 64;           // ring pixels per block
constexpr int GR_GS = GF_CG + 1;   // LDS row pitch of the gathered G (banks)
constexpr int GR_WS = GF_COUT + 4;  // LDS row pitch of the W2 slice
__global__ __launch_bounds__(256) void gfuse_ring_mfma_kernel(
    const float* __restrict__ band, int H, int W, const float* __restrict__ w2t,
    const float* __restrict__ b2, float* __restrict__ ring) {
  __shared__ float gs[GR_P][GR_GS];
  __shared__ float ws[GF_CG][GR_WS];
  __shared__ int bidx[9][GR_P];
  __shared__ int tap_live[9];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, ph = wave & 1, chh = wave >> 1;
  const int nr = gf_nring(H, W), nb = gf_nband(H, W);
  const int r0 = blockIdx.x * GR_P;
  if (tid < 9) tap_live[tid] = 0;
  pf_syncthreads();
  for (int i = tid; i < 9 * GR_P; i += 256) {
    const int t = i / GR_P, j = i - t * GR_P;
    int idx = -1;
    if (r0 + j < nr) {
      int Y, X;
      gf_ring_pos(r0 + j, H, W, Y, X);
      idx = gf_band_index(Y + t / 3 - 1, X + t % 3 - 1, H, W);
    }
    bidx[t][j] = idx;
    if (idx >= 0) tap_live[t] = 1;  // benign race: every writer stores 1
  }
  pf_syncthreads();
  const float* bb = band + (size_t)b * nb * GF_CG;
  // per thread: 16 gathered G values (pixel j = i / 64, channel k = i % 64,
  // i = tid + 256 u) and 32 W2 values (k = i / 128, co = i % 128)
  float gv[16], wv[32];
  auto load = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = tid + 256 * u, j = i >> 6, k = i & 63;
      const int idx = bidx[t][j];
      gv[u] = idx >= 0 ? bb[(size_t)idx * GF_CG + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) wv[u] = w2t[(size_t)t * GF_CG * GF_COUT + tid + 256 * u];
  };
  f32x16 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  int t = 0;
  while (t < 9 && !tap_live[t]) ++t;
  if (t < 9) load(t);
  while (t < 9) {
    pf_syncthreads();  // the previous tap's operands are read
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int i = tid + 256 * u;
      gs[i >> 6][i & 63] = gv[u];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int i = tid + 256 * u;
      ws[i >> 7][i & 127] = wv[u];
    }
    pf_syncthreads();
    int tn = t + 1;
    while (tn < 9 && !tap_live[tn]) ++tn;
    if (tn < 9) load(tn);  // in flight during this tap's MFMAs
    const int arow = 32 * ph + (lane & 31), kh = lane >> 5;
#pragma unroll 8
    for (int kk = 0; kk < GF_CG / 2; ++kk) {
      const int k = 2 * kk + kh;
      const float a = gs[arow][k];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float bv = ws[k][64 * chh + 32 * i + (lane & 31)];
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[i], 0, 0, 0);
      }
    }
    t = tn;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int co = 64 * chh + 32 * i + (lane & 31);
    const float bias = b2[co];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int rr = r0 + 32 * ph + m;
      if (rr < nr) ring[((size_t)b * nr + rr) * GF_COUT + co] = acc[i][r] + bias;
    }
  }
}

// the ring buffer of the fused head, then the band scratch of its two passes
size_t pf_gfuse_ring_image_floats(int H, int W) { return (size_t)gf_nring(H, W) * GF_COUT; }

size_t pf_gfuse_ring_floats(int n, int H, int W) {
  return (size_t)n * gf_nring(H, W) * GF_COUT + (size_t)n * gf_nband(H, W) * GF_CG;
}

// Everything of the G part but the interior conv itself, which
// up4tap_gcombine_kernel runs on the fly: the pre-split K = 80 weight planes
// and the exact border-ring values (ring, pf_gfuse_ring_floats).
int pf_gfuse_prep(const float* img4, const float* c, int ccs, int n, int H, int W,
                  const float* wc, const float* bc, const float* mean, const float* rstd,
                  const float* b2, const float* w1_packed, const float* b1,
                  unsigned short* wplanes, float* ring, hipStream_t st) {
  if (!c && !(w1_packed && b1)) return POSFEAT_E_INVALID;
  if (n <= 0 || H < 4 || W < 4 || !wplanes || !ring) return POSFEAT_E_INVALID;
  const int tot = n * GF_COUT * G8_K;
  hipLaunchKernelGGL(gfuse_wsplit_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, wc, n,
                     wplanes);
  const int nring = gf_nring(H, W), nband = gf_nband(H, W);
  float* band = ring + (size_t)n * nring * GF_COUT;
  if (!(side_abl() & 1)) {
    hipLaunchKernelGGL(gfuse_band_kernel, dim3((nband + GB_POS - 1) / GB_POS, n), dim3(256), 0, st,
                       c, ccs, img4, w1_packed, posfeat_conv_packed_k(3, 3, 3), b1, H, W, mean,
                       rstd, band);
    hipLaunchKernelGGL(gfuse_ring_mfma_kernel, dim3((nring + GR_P - 1) / GR_P, n), dim3(256), 0,
                       st, band, H, W, bc + (size_t)n * GF_COUT, b2, ring);
  }
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

size_t pf_gfuse_imgstats_ws_bytes(int n, int H) {
  return pf_align((size_t)n * ((H + IM_ROWS - 1) / IM_ROWS) * IM_G * IM_G * sizeof(double), 256);
}

// convimg's instance-norm mean / rstd [n][64] from the image moments (no conv)
int pf_gfuse_imgstats(const float* img4, int n, int H, int W, const float* w1_packed,
                      const float* b1, float* mean, float* rstd, void* ws, size_t ws_bytes,
                      hipStream_t st, double* gram) {
  if (!ws || ws_bytes < pf_gfuse_imgstats_ws_bytes(n, H)) return POSFEAT_E_WORKSPACE;
  // one block per band of rows (r3x: 8 or 16 band-looping blocks per image
  // were no faster); partials = blocks
  const int nband = (H + IM_ROWS - 1) / IM_ROWS;
  const size_t lds = std::max((size_t)(IM_ROWS + 2) * (W + 2) * 3 * sizeof(float),
                              (size_t)4 * IM_G * IM_G * sizeof(double));
  if (lds > 160 * 1024 || W % 2) return POSFEAT_E_UNSUPPORTED;
  double* part = static_cast<double*>(ws);
  // blocks per image (A/B POSFEAT_IMGMOM_BPI; default one per band): a
  // block walks bands blockIdx.x, + gridDim.x, ...
  static const int bpi = [] {
    const char* e = pf_ab_getenv("POSFEAT_IMGMOM_BPI");
    return e ? atoi(e) : 0;
  }();
  const int nblk = bpi > 0 && bpi < nband ? bpi : nband;
  if (!(side_abl() & 2))
    hipLaunchKernelGGL(gfuse_imgmom_kernel, dim3(nblk, n), dim3(256), lds, st, img4, H, W, part);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(gfuse_imgstats_kernel, dim3(n), dim3(IM_G * IM_G), 0, st, part, nblk, H * W,
                     w1_packed, posfeat_conv_packed_k(3, 3, 3), b1, 1e-5f, mean, rstd, gram);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
