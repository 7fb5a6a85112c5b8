// wino.hip -- Winograd F(4x4, 3x3) / F(2x2, 3x3) for the decoder's 3x3 stride-1 convs
// (upconv3/iconv3/upconv2/iconv2, DescNet.py:41-45: 4 x 45.3 GFLOP per
// 480x640 image, 43 % of the extraction's conv work).
//
//   U = G g G^T   (once per weight update; [16][Cout][Cin])
//   V = B^T d B   per 2x2 output tile, 4x4 input patch   ([16][T][Cin])
//   M_xi = V_xi U_xi^T   16 GEMMs in ONE launch of the conv engine's
//                        conv_glds_kernel (blockIdx.y = xi)   ([16][T][Cout])
//   Y = A^T M A (+ bias, activation) into the NHWC output (channel slice)
//
// F(2x2): 16 instead of 36 MACs per 2x2 tile and channel pair (GEMM 2.25x
// smaller than the direct conv); F(4x4) (used when h, w % 4 == 0): 36 instead
// of 144 per 4x4 tile (4x smaller), 36 transform-domain GEMMs, and 2.25/4 of
// F(2x2)'s transform traffic.  The transforms are two HBM passes.  Transforms are
// exact-weight (+-1, 1/2) so the result differs from the direct conv by fp32
// rounding only (tests/test_gpu_ops.py).
#include <algorithm>

#include "common.h"
#include "fmap.h"
#include "train.h"

namespace {

int grid_for(long long total, int block) {
  long long g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

// U[xi][co][ci] from the engine-packed 3x3 weights [Cout][Kpad], K order
// ((ci/32)*9 + tap)*32 + ci%32 (Cin % 32 == 0)
// Ub != nullptr: U as three bf16 planes (plane stride 16 Cout Cin) for the
// pre-split bf16x6 GEMM tiles, instead of fp32
__global__ void wino_weights_kernel(const float* __restrict__ wpk, int Cout, int Cin, int kpad,
                                    float* __restrict__ U, unsigned short* __restrict__ Ub = nullptr) {
  const long long n = (long long)Cout * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
    const float* w = wpk + (long long)co * kpad + (ci >> 5) * 9 * 32 + (ci & 31);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[t * 32];
    float r[4][3];  // G g
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      r[0][c] = g[0][c];
      r[1][c] = 0.5f * (g[0][c] + g[1][c] + g[2][c]);
      r[2][c] = 0.5f * (g[0][c] - g[1][c] + g[2][c]);
      r[3][c] = g[2][c];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const float u0 = r[a][0], u1 = 0.5f * (r[a][0] + r[a][1] + r[a][2]);
      const float u2 = 0.5f * (r[a][0] - r[a][1] + r[a][2]), u3 = r[a][2];
      const float uu[4] = {u0, u1, u2, u3};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const long long o = ((long long)(a * 4 + b) * Cout + co) * Cin + ci;
        if (Ub) {
          unsigned hh, mm, ll;
          pf_split3_pair(uu[b], 0.f, hh, mm, ll);
          Ub[o] = (unsigned short)hh;
          Ub[o + 16 * n] = (unsigned short)mm;
          Ub[o + 32 * n] = (unsigned short)ll;
        } else {
          U[o] = uu[b];
        }
      }
    }
  }
}

// V[xi][tile][c] = (B^T d B)[xi] for the 4x4 patch at rows 2ty-1.., cols 2tx-1..
__global__ void wino_input_kernel(const float* __restrict__ x, int xcs, int n, int h, int w,
                                  int c4n, float* __restrict__ V) {
  const int th = h / 2, tw = w / 2;
  const long long T = (long long)n * th * tw;
  const long long total = T * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    f32x4 d[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int yy = 2 * ty - 1 + r;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int xx = 2 * tx - 1 + c;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
          v = *reinterpret_cast<const f32x4*>(x + (((long long)b * h + yy) * w + xx) * xcs + q * 4);
        d[r][c] = v;
      }
    }
    f32x4 t[4][4];  // B^T d
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t[0][c] = d[0][c] - d[2][c];
      t[1][c] = d[1][c] + d[2][c];
      t[2][c] = d[2][c] - d[1][c];
      t[3][c] = d[1][c] - d[3][c];
    }
    float* vo = V + tile * C + q * 4;
    const long long xs = T * C;  // xi stride
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      *reinterpret_cast<f32x4*>(vo + (a * 4 + 0) * xs) = t[a][0] - t[a][2];
      *reinterpret_cast<f32x4*>(vo + (a * 4 + 1) * xs) = t[a][1] + t[a][2];
      *reinterpret_cast<f32x4*>(vo + (a * 4 + 2) * xs) = t[a][2] - t[a][1];
      *reinterpret_cast<f32x4*>(vo + (a * 4 + 3) * xs) = t[a][1] - t[a][3];
    }
  }
}

// y[2ty+i][2tx+j] = act((A^T M A)[i][j] + bias)
__global__ void wino_output_kernel(const float* __restrict__ M, int n, int h, int w, int c4n,
                                   const float* __restrict__ bias, int act, float* __restrict__ y,
                                   int ycs) {
  const int th = h / 2, tw = w / 2;
  const long long T = (long long)n * th * tw;
  const long long total = T * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    const float* mi = M + tile * C + q * 4;
    const long long xs = T * C;
    f32x4 m[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) m[a][c] = *reinterpret_cast<const f32x4*>(mi + (a * 4 + c) * xs);
    f32x4 s[2][4];  // A^T M
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s[0][c] = m[0][c] + m[1][c] + m[2][c];
      s[1][c] = m[1][c] - m[2][c] - m[3][c];
    }
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (bias) bv = *reinterpret_cast<const f32x4*>(bias + q * 4);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      f32x4 o[2];
      o[0] = s[a][0] + s[a][1] + s[a][2] + bv;
      o[1] = s[a][1] - s[a][2] - s[a][3] + bv;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = o[c][j];
          v = act == POSFEAT_ACT_RELU ? fmaxf(v, 0.f) : act == POSFEAT_ACT_ELU ? pf_elu(v) : v;
          o[c][j] = v;
        }
        *reinterpret_cast<f32x4*>(
            y + (((long long)b * h + 2 * ty + a) * w + 2 * tx + c) * ycs + q * 4) = o[c];
      }
    }
  }
}

// ---------------------------------------------------------------- F(4x4, 3x3)
// 36 multiplies per 16 outputs (4x fewer MACs than direct; 1.78x fewer than
// F(2x2)), transform matrices of Lavin & Gray (2016):
constexpr float W4_BT[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0},
                                  {0, 4, -4, -1, 1, 0}, {0, -2, -1, 2, 1, 0},
                                  {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
constexpr float W4_G[6][3] = {{0.25f, 0, 0},
                                 {-1.f / 6, -1.f / 6, -1.f / 6},
                                 {-1.f / 6, 1.f / 6, -1.f / 6},
                                 {1.f / 24, 1.f / 12, 1.f / 6},
                                 {1.f / 24, -1.f / 12, 1.f / 6},
                                 {0, 0, 1}};
constexpr float W4_AT[4][6] = {
    {1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};

// Ub != nullptr: U as three bf16 planes (plane stride 36 Cout Cin) for the
// bf16x6 GEMM (gemm6.hip), instead of fp32
__global__ void wino4_weights_kernel(const float* __restrict__ wpk, int Cout, int Cin, int kpad,
                                     float* __restrict__ U, unsigned short* __restrict__ Ub) {
  const long long n = (long long)Cout * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
    const float* w = wpk + (long long)co * kpad + (ci >> 5) * 9 * 32 + (ci & 31);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[t * 32];
    float r[6][3];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        r[a][c] = W4_G[a][0] * g[0][c] + W4_G[a][1] * g[1][c] + W4_G[a][2] * g[2][c];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const float u = r[a][0] * W4_G[b][0] + r[a][1] * W4_G[b][1] + r[a][2] * W4_G[b][2];
        const long long o = ((long long)(a * 6 + b) * Cout + co) * Cin + ci;
        if (Ub) {
          unsigned hh, mm, ll;
          pf_split3_pair(u, 0.f, hh, mm, ll);
          Ub[o] = (unsigned short)hh;
          Ub[o + 36 * n] = (unsigned short)mm;
          Ub[o + 72 * n] = (unsigned short)ll;
        } else {
          U[o] = u;
        }
      }
  }
}

// V[xi][tile][c], 6x6 patch at rows 4ty-1.., cols 4tx-1..; Vb != nullptr: V
// as three bf16 planes (plane stride 36 T C) for the bf16x6 GEMM instead
// up2: x is the h/2 x w/2 map whose x2 align_corners upsample is the conv
// input (upconv, DescNet.py:182-190): its values are interpolated here
// (pf_up2ac_at, the upsample kernel's own arithmetic) instead of read from a
// materialised upsample
__global__ __launch_bounds__(256) PF_NO_PK_FP32 void wino4_input_kernel(const float* __restrict__ x, int xcs,
                                                          int n, int h, int w, int c4n,
                                                          float* __restrict__ V, int clamp = 0,
                                                          unsigned short* __restrict__ Vb = nullptr,
                                                          int up2 = 0) {
  const int th = h / 4, tw = w / 4;
  const int h2 = h / 2, w2 = w / 2;
  const float sh = h > 1 ? (float)(h2 - 1) / (float)(h - 1) : 0.f;
  const float sw = w > 1 ? (float)(w2 - 1) / (float)(w - 1) : 0.f;
  const long long T = (long long)n * th * tw;
  const long long total = T * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    f32x4 t[6][6];  // B^T d, built row by row of d
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c < 6; ++c) t[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      int yy = 4 * ty - 1 + r;
      if (clamp) yy = min(max(yy, 0), h - 1);  // replicate extension (conv_up4's L halo)
      f32x4 d[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        int xx = 4 * tx - 1 + c;
        if (clamp) xx = min(max(xx, 0), w - 1);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
          v = up2 ? pf_up2ac_at(x + (long long)b * h2 * w2 * xcs + q * 4, h2, w2, xcs, sh, sw, yy,
                                xx)
                  : *reinterpret_cast<const f32x4*>(x + (((long long)b * h + yy) * w + xx) * xcs +
                                                    q * 4);
        d[c] = v;
      }
#pragma unroll
      for (int a = 0; a < 6; ++a)
        if (W4_BT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 6; ++c) t[a][c] += W4_BT[a][r] * d[c];
    }
    const long long xs = T * C;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 6; ++c)
          if (W4_BT[bb][c] != 0.f) v += W4_BT[bb][c] * t[a][c];
        const long long o = (a * 6 + bb) * xs + tile * C + q * 4;
        if (Vb) {
          uint2 vh, vm, vl;
          pf_split3x4(v, vh, vm, vl);
          *reinterpret_cast<uint2*>(Vb + o) = vh;
          *reinterpret_cast<uint2*>(Vb + o + 36 * xs) = vm;
          *reinterpret_cast<uint2*>(Vb + o + 72 * xs) = vl;
        } else {
          *reinterpret_cast<f32x4*>(V + o) = v;
        }
      }
  }
}

__global__ __launch_bounds__(256) void wino4_output_kernel(const float* __restrict__ M, int n,
                                                           int h, int w, int c4n,
                                                           const float* __restrict__ bias, int act,
                                                           float* __restrict__ y, int ycs) {
  const int th = h / 4, tw = w / 4;
  const long long T = (long long)n * th * tw;
  const long long total = T * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    const float* mi = M + tile * C + q * 4;
    const long long xs = T * C;
    f32x4 s[4][6];  // A^T M
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 6; ++c) s[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      f32x4 m[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) m[c] = *reinterpret_cast<const f32x4*>(mi + (r * 6 + c) * xs);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        if (W4_AT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 6; ++c) s[a][c] += W4_AT[a][r] * m[c];
    }
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if (bias) bv = *reinterpret_cast<const f32x4*>(bias + q * 4);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        f32x4 o = bv;
#pragma unroll
        for (int c = 0; c < 6; ++c)
          if (W4_AT[bb][c] != 0.f) o += W4_AT[bb][c] * s[a][c];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = o[j];
          o[j] = act == POSFEAT_ACT_RELU ? fmaxf(v, 0.f) : act == POSFEAT_ACT_ELU ? pf_elu(v) : v;
        }
        *reinterpret_cast<f32x4*>(
            y + (((long long)b * h + 4 * ty + a) * w + 4 * tx + bb) * ycs + q * 4) = o;
      }
  }
}

// ---------------------------------------------------------------- F(4x4) weight gradient
// Y = A^T [U (.) V] A with U = G g G^T  =>  dM = A dY A^T (6x6 per 4x4 output
// tile), dU_xi = sum_tiles dM_xi (x) V_xi (36 batched GEMMs over the tiles),
// dg = G^T dU G.  The Winograd identity holds for the gradient exactly as for
// the forward, so this is the same reduction in a 4x smaller MAC count.
__global__ __launch_bounds__(256) void wino4_dy_kernel(const float* __restrict__ dy, int ldy, int n,
                                                       int h, int w, int c4n,
                                                       float* __restrict__ dM) {
  const int th = h / 4, tw = w / 4;
  const long long T = (long long)n * th * tw;
  const long long total = T * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    f32x4 t[6][4];  // A dY
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) t[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      f32x4 g[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        g[j] = *reinterpret_cast<const f32x4*>(
            dy + (((long long)b * h + 4 * ty + ii) * w + 4 * tx + j) * ldy + q * 4);
#pragma unroll
      for (int r = 0; r < 6; ++r)
        if (W4_AT[ii][r] != 0.f)
#pragma unroll
          for (int j = 0; j < 4; ++j) t[r][j] += W4_AT[ii][r] * g[j];
    }
    float* mo = dM + tile * C + q * 4;
    const long long xs = T * C;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (W4_AT[j][c] != 0.f) v += W4_AT[j][c] * t[r][j];
        *reinterpret_cast<f32x4*>(mo + (r * 6 + c) * xs) = v;
      }
  }
}

// dU = sum of the nsplit GEMM partials; dW[co][(ci/32, tap, ci%32)] (+)=
// (G^T dU G)[tap]; db (+)= sum of the bias partials
__global__ void wino4_wgrad_out_kernel(const float* __restrict__ part, int nsplit, int Cout,
                                       int Cin, int kpad, float* __restrict__ dw,
                                       const float* __restrict__ partb, float* __restrict__ db,
                                       int acc) {
  const long long n = (long long)Cout * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
    // split-outer: the 36 loads of one split are in flight together, each
    // u[a][b] still sums its splits in order s = 0, 1, ...
    float u[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b) u[a][b] = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      float v[36];
#pragma unroll
      for (int x = 0; x < 36; ++x) v[x] = part[((long long)x * nsplit + s) * n + i];
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 6; ++b) u[a][b] += v[a * 6 + b];
    }
    float sv[3][6];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        float v = 0.f;
#pragma unroll
        for (int a = 0; a < 6; ++a)
          if (W4_G[a][kh] != 0.f) v += W4_G[a][kh] * u[a][b];
        sv[kh][b] = v;
      }
    float* out = dw + (long long)co * kpad + (ci >> 5) * 9 * 32 + (ci & 31);
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float v = 0.f;
#pragma unroll
        for (int b = 0; b < 6; ++b)
          if (W4_G[b][kw] != 0.f) v += sv[kh][b] * W4_G[b][kw];
        float* o = out + (kh * 3 + kw) * 32;
        *o = acc ? *o + v : v;
      }
    if (db && ci == 0) {
      const float v = pf_ordered_sum(partb + co, Cout, nsplit);
      db[co] = acc ? db[co] + v : v;
    }
  }
}

// ---------------------------------------------------------------- head.conv2 L part
// conv_up4_kernel's per-phase low-res convs (conv.hip: phase (ry, rx) applies
// |E(ry)| x |E(rx)| combined taps, E = {-1,0} / {-1,0,1} / {0,1}, to the
// replicate-extended L) are one 3x3 conv of L with 16 x 128 = 2048 output
// channels whose missing taps are zero.  That conv is a Winograd F(4x4,3x3)
// on the LOW-RES grid: 36 MACs per 16 low-res positions and output channel
// instead of 6.25 per position on average -- 2.78x fewer than the phase
// kernel.  The output transform scatters each (position, phase) to its
// full-res pixel (4 qy + ry, 4 qx + rx) and adds it to y, which already holds
// the G part + bias - the zero-padding border terms (pf_up4_border).
constexpr int UW_CU = 192, UW_COUT = 128, UW_NO = 16 * UW_COUT;
constexpr int UW_KP = (UW_CU / 32) * 9 * 32;  // conv.hip UP4_KP: per-phase packed K

__global__ void up4_wino_weights_kernel(const float* __restrict__ wph, float* __restrict__ U) {
  const long long n = (long long)UW_NO * UW_CU;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(i / UW_CU), ci = (int)(i - (long long)o * UW_CU);
    const int phase = o / UW_COUT, ry = phase >> 2, rx = phase & 3;
    const int ney = (ry == 0 || ry == 3) ? 2 : 3, nex = (rx == 0 || rx == 3) ? 2 : 3;
    const int ey0 = ry == 3 ? 0 : -1, ex0 = rx == 3 ? 0 : -1;
    const int T = ney * nex, slab = ci >> 5;
    const float* w = wph + (long long)o * UW_KP + (ci & 31);
    float g[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    for (int tj = 0; tj < T; ++tj)
      g[ey0 + tj / nex + 1][ex0 + tj % nex + 1] = w[(slab * T + tj) * 32];
    float r[6][3];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        r[a][c] = W4_G[a][0] * g[0][c] + W4_G[a][1] * g[1][c] + W4_G[a][2] * g[2][c];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = 0; b < 6; ++b)
        U[((long long)(a * 6 + b) * UW_NO + o) * UW_CU + ci] =
            r[a][0] * W4_G[b][0] + r[a][1] * W4_G[b][1] + r[a][2] * W4_G[b][2];
  }
}

// y[(b, 4 qy + ry, 4 qx + rx)][co] += (A^T M A)[qy, qx] for o = phase * 128 + co.
// One item per thread, exact grid (T * 512 / 256 blocks): a block is one
// tile x 8 phases x 32 channel quads, so with part != null it also reduces
// the final y values over its 8 phases (fixed order, LDS) into the instance-
// norm partials part[b][(tile in image) * 2 + half][co][2] (sum, sum of squares).
__global__ __launch_bounds__(256) void up4_wino_output_kernel(const float* __restrict__ M, int n,
                                                              int lh, int lw,
                                                              float* __restrict__ y, int ycs,
                                                              double* __restrict__ part) {
  __shared__ double red[8][32][8];
  const int th = lh / 4, tw = lw / 4, H = 4 * lh, W = 4 * lw;
  constexpr int c4n = UW_NO / 4;
  const long long T = (long long)n * th * tw;
  {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    int q, tx, ty;
    const int b = pf_tile_split(i, c4n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    const int phase = (q * 4) / UW_COUT, co = q * 4 - phase * UW_COUT;
    const int ry = phase >> 2, rx = phase & 3;
    const float* mi = M + tile * UW_NO + q * 4;
    const long long xs = T * UW_NO;
    f32x4 s[4][6];  // A^T M
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 6; ++c) s[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      f32x4 m[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) m[c] = *reinterpret_cast<const f32x4*>(mi + (r * 6 + c) * xs);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        if (W4_AT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 6; ++c) s[a][c] += W4_AT[a][r] * m[c];
    }
    double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 6; ++c)
          if (W4_AT[bb][c] != 0.f) o += W4_AT[bb][c] * s[a][c];
        const int Y = 4 * (4 * ty + a) + ry, X = 4 * (4 * tx + bb) + rx;
        f32x4* dst = reinterpret_cast<f32x4*>(y + (((long long)b * H + Y) * W + X) * ycs + co);
        o = *dst + o;
        *dst = o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s1[j] += (double)o[j];
          s2[j] += (double)o[j] * (double)o[j];
        }
      }
    if (part) {
      const int pl = threadIdx.x >> 5, cq = threadIdx.x & 31;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[pl][cq][j] = s1[j];
        red[pl][cq][4 + j] = s2[j];
      }
      pf_syncthreads();
      if (pl == 0) {
        double a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = 0.0;
        for (int r = 0; r < 8; ++r)
#pragma unroll
          for (int k = 0; k < 8; ++k) a[k] += red[r][cq][k];
        const long long tin = tile - (long long)b * th * tw;
        double* o = part + (((long long)b * th * tw + tin) * 2 + (phase >> 3)) * UW_COUT * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[(co + j) * 2] = a[j];
          o[(co + j) * 2 + 1] = a[4 + j];
        }
      }
    }
  }
}

}  // namespace

size_t pf_up4_wino_weights_floats() { return (size_t)36 * UW_NO * UW_CU; }

size_t pf_up4_wino_ws_bytes(int n, int H, int W) {
  const long long T = (long long)n * (H / 16) * (W / 16);
  return pf_align(36 * T * UW_CU * 4, 256) + pf_align(36 * T * UW_NO * 4, 256) +
         pf_align((size_t)T * 2 * UW_COUT * 2 * sizeof(double), 256);
}

int pf_up4_wino_weights(const float* wph, float* U, hipStream_t st) {
  hipLaunchKernelGGL(up4_wino_weights_kernel, dim3(grid_for((long long)UW_NO * UW_CU, 256)),
                     dim3(256), 0, st, wph, U);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// y (n x H x W x 128, pitch ycs) += the 192 upsampled channels' part of
// head.conv2 from L (n x H/4 x W/4 x 192, pitch lcs); H/4, W/4 % 4 == 0
// stages: bit 0 input transform, bit 1 the 36 GEMMs, bit 2 output transform
// (the engine times them separately)
int pf_up4_wino(int n, int H, int W, const float* L, int lcs, const float* U, float* y, int ycs,
                void* ws, size_t ws_bytes, hipStream_t st, int stages, float* mean, float* rstd) {
  const int lh = H / 4, lw = W / 4;
  if (H % 16 || W % 16 || lcs % 4 || ycs % 4) return POSFEAT_E_INVALID;
  if (!ws || ws_bytes < pf_up4_wino_ws_bytes(n, H, W)) return POSFEAT_E_WORKSPACE;
  const long long T = (long long)n * (lh / 4) * (lw / 4);
  float* V = static_cast<float*>(ws);
  float* M = reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(36 * T * UW_CU * 4, 256));
  double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(M) +
                                           pf_align(36 * T * UW_NO * 4, 256));
  if (stages & 1) {
    hipLaunchKernelGGL(wino4_input_kernel, dim3(grid_for(T * (UW_CU / 4), 256)), dim3(256), 0, st,
                       L, lcs, n, lh, lw, UW_CU / 4, V, 1);
    PF_CHECK_LAUNCH();
  }
  if (stages & 2)
    PF_TRY(pf_gemm_batched(V, UW_CU, T * UW_CU, U, (long long)UW_NO * UW_CU, M, UW_NO, T * UW_NO,
                           36, (int)T, UW_NO, UW_CU, st));
  if (stages & 4) {
    // exact grid: the statistics reduce one block = one tile x 8 phases
    hipLaunchKernelGGL(up4_wino_output_kernel, dim3((unsigned)(T * (UW_NO / 4) / 256)), dim3(256),
                       0, st, M, n, lh, lw, y, ycs, mean ? part : nullptr);
    PF_CHECK_LAUNCH();
    if (mean)
      PF_TRY(pf_in_finalize(part, n, (lh / 4) * (lw / 4) * 2, H * W, UW_COUT, mean, rstd, st));
  }
  return POSFEAT_OK;
}

// U as bf16 planes for the pre-split bf16x6 GEMM tiles: Cout a multiple of
// 64 (128-wide tiles, or 64-wide ones for 192 = head.conv1; the tiles clamp
// their rows past Cout, the epilogue never stores them)
static bool wino_planes_ok(int Cout) { return Cout % 64 == 0; }

// ---------------------------------------------------------------- F(6x6, 3x3)
// 64 multiplies per 36 outputs: 1.27x fewer MACs than F(4x4) (2.25 -> 1.78 per
// output and channel pair) and 0.79x its transform-domain bytes.  Points 0,
// +-1, +-2, +-1/2 (Lavin & Gray's construction): B^T and A^T are exact in
// fp32 (quarters and powers of two), G carries ninths; tests/test_gpu_ops.py
// bounds the result against the direct conv.  Tiles are ceil(h/6) x ceil(w/6):
// the last row / column of tiles reads zeros past the map (the conv's own
// padding for the outputs kept) and drops the outputs past it.  One channel
// PAIR per thread: the 8x8 transform of four channels would hold 256 VGPRs.
namespace {
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr float W6_BT[8][8] = {{1, 0, -5.25f, 0, 5.25f, 0, -1, 0},
                               {0, 1, 1, -4.25f, -4.25f, 1, 1, 0},
                               {0, -1, 1, 4.25f, -4.25f, -1, 1, 0},
                               {0, 0.5f, 0.25f, -2.5f, -1.25f, 2, 1, 0},
                               {0, -0.5f, 0.25f, 2.5f, -1.25f, -2, 1, 0},
                               {0, 2, 4, -2.5f, -5, 0.5f, 1, 0},
                               {0, -2, 4, 2.5f, -5, -0.5f, 1, 0},
                               {0, -1, 0, 5.25f, 0, -5.25f, 0, 1}};
constexpr float W6_G[8][3] = {{1, 0, 0},
                              {-2.f / 9, -2.f / 9, -2.f / 9},
                              {-2.f / 9, 2.f / 9, -2.f / 9},
                              {1.f / 90, 1.f / 45, 2.f / 45},
                              {1.f / 90, -1.f / 45, 2.f / 45},
                              {32.f / 45, 16.f / 45, 8.f / 45},
                              {32.f / 45, -16.f / 45, 8.f / 45},
                              {0, 0, 1}};
constexpr float W6_AT[6][8] = {{1, 1, 1, 1, 1, 1, 1, 0},
                               {0, 1, -1, 2, -2, 0.5f, -0.5f, 0},
                               {0, 1, 1, 4, 4, 0.25f, 0.25f, 0},
                               {0, 1, -1, 8, -8, 0.125f, -0.125f, 0},
                               {0, 1, 1, 16, 16, 0.0625f, 0.0625f, 0},
                               {0, 1, -1, 32, -32, 0.03125f, -0.03125f, 1}};

// U[xi][co][ci] (64 matrices), Ub != nullptr: three bf16 planes (stride 64 Cout Cin)
__global__ void wino6_weights_kernel(const float* __restrict__ wpk, int Cout, int Cin, int kpad,
                                     float* __restrict__ U, unsigned short* __restrict__ Ub) {
  const long long n = (long long)Cout * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
    const float* w = wpk + (long long)co * kpad + (ci >> 5) * 9 * 32 + (ci & 31);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[t * 32];
    float r[8][3];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int c = 0; c < 3; ++c)
        r[a][c] = W6_G[a][0] * g[0][c] + W6_G[a][1] * g[1][c] + W6_G[a][2] * g[2][c];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const float u = r[a][0] * W6_G[b][0] + r[a][1] * W6_G[b][1] + r[a][2] * W6_G[b][2];
        const long long o = ((long long)(a * 8 + b) * Cout + co) * Cin + ci;
        if (Ub) {
          unsigned hh, mm, ll;
          pf_split3_pair(u, 0.f, hh, mm, ll);
          Ub[o] = (unsigned short)hh;
          Ub[o + 64 * n] = (unsigned short)mm;
          Ub[o + 128 * n] = (unsigned short)ll;
        } else {
          U[o] = u;
        }
      }
  }
}

template <int VW> struct W6Vec;
template <> struct W6Vec<1> { typedef float t; };
template <> struct W6Vec<2> { typedef f32x2 t; };
// acc + k x as one explicit fma: the transform's arithmetic is then the same
// per channel whether a thread holds one channel or a pair (the fused-upsample
// kernel and the plain one must agree bit for bit, test_gpu_bf6r.py)
__device__ __forceinline__ float w6_fma(float k, float x, float acc) {
  return __builtin_fmaf(k, x, acc);
}
__device__ __forceinline__ f32x2 w6_fma(float k, f32x2 x, f32x2 acc) {
  return __builtin_elementwise_fma(f32x2{k, k}, x, acc);
}

// x-interpolated half-res row sy at the 8 patch columns (pf_up2ac_at's inner
// terms hx v(sy, x0) + lx v(sy, x1), same operations): 0 past the map
template <typename T>
__device__ __forceinline__ void up2_row8(const float* base, int w2, int cs, float sw, int w, int sy,
                                         int xc0, T (&X)[8]) {
#pragma clang fp contract(off)
  const float* row = base + (long long)sy * w2 * cs;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    // branch-free: a column past the map interpolates column w - 1, then 0
    const int xx = xc0 + c;
    const bool in = (unsigned)xx < (unsigned)w;
    const float rx = sw * (in ? xx : w - 1);
    const int x0 = (int)rx;
    const int x1 = x0 + (x0 < w2 - 1 ? 1 : 0);
    const float lx = rx - x0, hx = 1.f - lx;
    const T v0 = *reinterpret_cast<const T*>(row + x0 * cs);
    const T v1 = *reinterpret_cast<const T*>(row + x1 * cs);
    const T v = hx * v0 + lx * v1;
    X[c] = in ? v : T(0.f);
  }
}

// X = rows[k] for a wave-uniform k in [0, 6): uniform branches, no selects
template <typename T>
__device__ __forceinline__ void up2_pick(const T (&rows)[6][8], int k, T (&X)[8]) {
  switch (__builtin_amdgcn_readfirstlane(k)) {
#define UP2_PICK_CASE(j) \
  case j:                \
    for (int c = 0; c < 8; ++c) X[c] = rows[j][c]; \
    break;
    UP2_PICK_CASE(0) UP2_PICK_CASE(1) UP2_PICK_CASE(2) UP2_PICK_CASE(3) UP2_PICK_CASE(4)
    default:
      for (int c = 0; c < 8; ++c) X[c] = rows[5][c];
#undef UP2_PICK_CASE
  }
}

// pf_up2ac_at's outer term hy X(y0) + ly X(y1), same operations
template <typename T>
__device__ __forceinline__ T up2_lerp_y(float hy, T a, float ly, T b) {
#pragma clang fp contract(off)
  return hy * a + ly * b;
}

// V[xi][tile][c] = (B^T d B)[xi], d the 8x8 patch at rows 6ty-1.., cols 6tx-1..
// (zero outside the map), VW channels per thread (the 8x8 accumulator is 64 VW
// VGPRs).  UP2: x is the h/2 x w/2 map whose x2 align_corners upsample is the
// conv input (upconv, DescNet.py:182-190), interpolated here with
// pf_up2ac_at's arithmetic (x then y, no contraction: the upsample kernel's
// bits) -- each half-res row's x interpolation is formed once and kept in a
// two-row window that slides down the patch (the patch's 8 rows read 5-6
// half-res rows), instead of four gathered loads per tap.  A wave is 64
// channel groups of one tile (Cin / VW >= 64 on every caller), so the window's
// branches are wave-uniform.
// UPM (UP2): 0 the half-res rows x-interpolated as the patch rows reach them
// (a two-row window); 1 all six the patch can touch loaded and interpolated
// first (every load in flight at once), the patch rows picked from them
template <bool UP2, int VW, int UPM = 0>
__global__ __launch_bounds__(256) void wino6_input_kernel(const float* __restrict__ x, int xcs,
                                                          int n, int h, int w, int cvn,
                                                          float* __restrict__ V) {
  typedef typename W6Vec<VW>::t T;
  const int th = (h + 5) / 6, tw = (w + 5) / 6;
  const int h2 = h / 2, w2 = w / 2;
  const float sh = h > 1 ? (float)(h2 - 1) / (float)(h - 1) : 0.f;
  const float sw = w > 1 ? (float)(w2 - 1) / (float)(w - 1) : 0.f;
  const long long Tn = (long long)n * th * tw;
  const long long total = Tn * cvn;
  const int C = cvn * VW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, cvn, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    T t[8][8];  // B^T d, built row by row of d
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int c = 0; c < 8; ++c) t[a][c] = T(0.f);
    const float* base = UP2 ? x + (long long)b * h2 * w2 * xcs + q * VW : nullptr;
    T XA[8], XB[8];  // UP2: x-interpolated half-res rows ka, kb
    int ka = -1, kb = -1;
    // UPM 1: the half-res rows ybase .. ybase + 5 (sh < 1/2: the patch's 8
    // rows need at most rows y0 - ybase <= 4 and y1 - ybase <= 5)
    constexpr int NXR = UP2 && UPM >= 1 ? 6 : 1;
    T XR[NXR][8];
    int ybase = 0;
    if constexpr (UP2 && UPM >= 1) {
      ybase = (int)(sh * max(6 * ty - 1, 0));
#pragma unroll
      for (int j = 0; j < 6; ++j) up2_row8(base, w2, xcs, sw, w, min(ybase + j, h2 - 1), 6 * tx - 1, XR[j]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int yy = 6 * ty - 1 + r;
      T d[8];
      if (UP2) {
#pragma unroll
        for (int c = 0; c < 8; ++c) d[c] = T(0.f);
        if ((unsigned)yy < (unsigned)h) {
          const float ry = sh * yy;
          const int y0 = (int)ry;
          const int y1 = y0 + (y0 < h2 - 1 ? 1 : 0);
          const float ly = ry - y0, hy = 1.f - ly;
          if constexpr (UPM >= 1) {
            up2_pick(XR, y0 - ybase, XA);
            up2_pick(XR, y1 - ybase, XB);
          } else {
          if (y0 != ka) {
            if (y0 == kb) {
#pragma unroll
              for (int c = 0; c < 8; ++c) XA[c] = XB[c];
            } else {
              up2_row8(base, w2, xcs, sw, w, y0, 6 * tx - 1, XA);
            }
            ka = y0;
          }
          if (y1 != kb) {
            if (y1 == ka) {
#pragma unroll
              for (int c = 0; c < 8; ++c) XB[c] = XA[c];
            } else {
              up2_row8(base, w2, xcs, sw, w, y1, 6 * tx - 1, XB);
            }
            kb = y1;
          }
          }
#pragma unroll
          for (int c = 0; c < 8; ++c) d[c] = up2_lerp_y(hy, XA[c], ly, XB[c]);
          // (columns past the map: XA = XB = 0 there, so d = 0 as required)
        }
      } else {
        // branch-free taps (clamped address, 0 outside the map)
        const bool rin = (unsigned)yy < (unsigned)h;
        const float* xr = x + ((long long)b * h + min(max(yy, 0), h - 1)) * w * xcs + q * VW;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int xx = 6 * tx - 1 + c;
          const bool in = rin && (unsigned)xx < (unsigned)w;
          const T v = *reinterpret_cast<const T*>(xr + min(max(xx, 0), w - 1) * xcs);
          d[c] = in ? v : T(0.f);
        }
      }
#pragma unroll
      for (int a = 0; a < 8; ++a)
        if (W6_BT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 8; ++c) t[a][c] = w6_fma(W6_BT[a][r], d[c], t[a][c]);
    }
    // one running store pointer: 64 precomputed plane offsets (64-bit,
    // uniform) took 128 SGPRs and spilled
    const long long xs = Tn * C;
    float* vp = V + tile * C + q * VW;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        T v = T(0.f);
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (W6_BT[bb][c] != 0.f) v = w6_fma(W6_BT[bb][c], t[a][c], v);
        *reinterpret_cast<T*>(vp) = v;
        vp += xs;
        asm volatile("" : "+v"(vp));
      }
  }
}

// y = act(A^T M A + bias) for the 6x6 outputs of each tile inside the map
template <int VW>
__global__ __launch_bounds__(256) void wino6_output_kernel(const float* __restrict__ M, int n,
                                                           int h, int w, int cvn,
                                                           const float* __restrict__ bias, int act,
                                                           float* __restrict__ y, int ycs) {
  typedef typename W6Vec<VW>::t TV;
  const int th = (h + 5) / 6, tw = (w + 5) / 6;
  const long long T = (long long)n * th * tw;
  const long long total = T * cvn;
  const int C = cvn * VW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, cvn, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    const float* mi = M + tile * C + q * VW;
    const long long xs = T * C;
    TV s[6][8];  // A^T M
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c < 8; ++c) s[a][c] = TV(0.f);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      TV m[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) m[c] = *reinterpret_cast<const TV*>(mi + (r * 8 + c) * xs);
#pragma unroll
      for (int a = 0; a < 6; ++a)
        if (W6_AT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 8; ++c) s[a][c] += W6_AT[a][r] * m[c];
    }
    TV bv = TV(0.f);
    if (bias) bv = *reinterpret_cast<const TV*>(bias + q * VW);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int oy = 6 * ty + a;
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        const int ox = 6 * tx + bb;
        TV o = bv;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (W6_AT[bb][c] != 0.f) o += W6_AT[bb][c] * s[a][c];
        if constexpr (VW == 1) {
          o = act == POSFEAT_ACT_RELU ? fmaxf(o, 0.f) : act == POSFEAT_ACT_ELU ? pf_elu(o) : o;
        } else {
#pragma unroll
          for (int j = 0; j < VW; ++j) {
            const float v = o[j];
            o[j] = act == POSFEAT_ACT_RELU ? fmaxf(v, 0.f) : act == POSFEAT_ACT_ELU ? pf_elu(v) : v;
          }
        }
        if (oy < h && ox < w)
          *reinterpret_cast<TV*>(y + (((long long)b * h + oy) * w + ox) * ycs + q * VW) = o;
      }
    }
  }
}
// wino6_output_kernel<1> (act none) whose block is 4 consecutive tiles of one
// image x 64 channels, with the instance-norm partial sums of its outputs:
// per thread fp64 sums over the tile's 36 outputs inside the map, the block's
// four tiles summed in tile order (deterministic), written per (image, tile
// group, channel) -- head.conv1's statistics without a pass over its output
__global__ __launch_bounds__(256) void wino6_output_stats_kernel(
    const float* __restrict__ M, int n, int h, int w, int C, const float* __restrict__ bias,
    float* __restrict__ y, int ycs, double* __restrict__ part) {
  const int th = (h + 5) / 6, tw = (w + 5) / 6, tpi = th * tw;
  const int ng = (tpi + 3) / 4, ncq = C / 64;
  const int cq = blockIdx.x % ncq, bg = blockIdx.x / ncq;
  const int b = bg / ng, g = bg - b * ng;
  const int ql = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int q = cq * 64 + ql, ti = g * 4 + tl;  // tile within the image
  const long long T = (long long)n * tpi;
  double s1 = 0.0, s2 = 0.0;
  if (ti < tpi) {
    const int ty = ti / tw, tx = ti - ty * tw;
    const long long tile = (long long)b * tpi + ti;
    const float* mi = M + tile * C + q;
    const long long xs = T * C;
    float sa[6][8];  // A^T M
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = 0; c < 8; ++c) sa[a][c] = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float m[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) m[c] = mi[(r * 8 + c) * xs];
#pragma unroll
      for (int a = 0; a < 6; ++a)
        if (W6_AT[a][r] != 0.f)
#pragma unroll
          for (int c = 0; c < 8; ++c) sa[a][c] += W6_AT[a][r] * m[c];
    }
    const float bv = bias ? bias[q] : 0.f;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int oy = 6 * ty + a;
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        const int ox = 6 * tx + bb;
        float o = bv;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (W6_AT[bb][c] != 0.f) o += W6_AT[bb][c] * sa[a][c];
        if (oy < h && ox < w) {
          y[(((long long)b * h + oy) * w + ox) * ycs + q] = o;
          s1 += (double)o;
          s2 += (double)o * (double)o;
        }
      }
    }
  }
  __shared__ double red[4][64][2];
  red[tl][ql][0] = s1;
  red[tl][ql][1] = s2;
  pf_syncthreads();
  if (tl == 0) {
    double* o = part + (((long long)b * ng + g) * C + q) * 2;
    o[0] = ((red[0][ql][0] + red[1][ql][0]) + red[2][ql][0]) + red[3][ql][0];
    o[1] = ((red[0][ql][1] + red[1][ql][1]) + red[2][ql][1]) + red[3][ql][1];
  }
}
}  // namespace

// ---- F(6x6) weight gradient (the train-mode decoder): dM = A dY A^T per 6x6
// output tile (8x8, dY = 0 past the map), dU_xi = sum_tiles dM_xi (x) V_xi
// (64 batched GEMMs), dg = G^T dU G.  xi = (1, 1) sums dY (column 1 of A is
// all ones): the bias gradient.
namespace {
__global__ __launch_bounds__(256) void wino6_dy_kernel(const float* __restrict__ dy, int ldy, int n,
                                                       int h, int w, int c2n,
                                                       float* __restrict__ dM) {
  const int th = (h + 5) / 6, tw = (w + 5) / 6;
  const long long T = (long long)n * th * tw;
  const long long total = T * c2n;
  const int C = c2n * 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    int q, tx, ty;
    const int b = pf_tile_split(i, c2n, tw, th, q, tx, ty);
    const long long tile = ((long long)b * th + ty) * tw + tx;
    f32x2 t[8][6];  // A dY
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int j = 0; j < 6; ++j) t[r][j] = f32x2{0.f, 0.f};
#pragma unroll
    for (int ii = 0; ii < 6; ++ii) {
      const int yy = 6 * ty + ii;
      const bool rin = yy < h;
      const float* dr = dy + ((long long)b * h + min(yy, h - 1)) * w * ldy + q * 2;
      f32x2 g[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int xx = 6 * tx + j;
        const f32x2 v = *reinterpret_cast<const f32x2*>(dr + min(xx, w - 1) * ldy);
        g[j] = rin && xx < w ? v : f32x2{0.f, 0.f};
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (W6_AT[ii][r] != 0.f)
#pragma unroll
          for (int j = 0; j < 6; ++j) t[r][j] = w6_fma(W6_AT[ii][r], g[j], t[r][j]);
    }
    const long long xs = T * C;
    float* mo = dM + tile * C + q * 2;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        f32x2 v = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (W6_AT[j][c] != 0.f) v = w6_fma(W6_AT[j][c], t[r][j], v);
        *reinterpret_cast<f32x2*>(mo) = v;
        mo += xs;
        asm volatile("" : "+v"(mo));
      }
  }
}

// dU = the nsplit GEMM partials summed in order; dW[co][(ci/32, tap, ci%32)]
// (+)= (G^T dU G)[tap]; db (+)= the bias partials summed in order
__global__ void wino6_wgrad_out_kernel(const float* __restrict__ part, int nsplit, int Cout,
                                       int Cin, int kpad, float* __restrict__ dw,
                                       const float* __restrict__ partb, float* __restrict__ db,
                                       int acc) {
  const long long n = (long long)Cout * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / Cin), ci = (int)(i - (long long)co * Cin);
    float u[64];
#pragma unroll
    for (int x = 0; x < 64; ++x) u[x] = 0.f;
    for (int s = 0; s < nsplit; ++s) {  // the 64 loads of a split in flight together
      float v[64];
#pragma unroll
      for (int x = 0; x < 64; ++x) v[x] = part[((long long)x * nsplit + s) * n + i];
#pragma unroll
      for (int x = 0; x < 64; ++x) u[x] += v[x];
    }
    float sv[3][8];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        float v = 0.f;
#pragma unroll
        for (int a = 0; a < 8; ++a)
          if (W6_G[a][kh] != 0.f) v += W6_G[a][kh] * u[a * 8 + b];
        sv[kh][b] = v;
      }
    float* out = dw + (long long)co * kpad + (ci >> 5) * 9 * 32 + (ci & 31);
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        float v = 0.f;
#pragma unroll
        for (int b = 0; b < 8; ++b)
          if (W6_G[b][kw] != 0.f) v += sv[kh][b] * W6_G[b][kw];
        float* o = out + (kh * 3 + kw) * 32;
        *o = acc ? *o + v : v;
      }
    if (db && ci == 0) {
      const float v = pf_ordered_sum(partb + co, Cout, nsplit);
      db[co] = acc ? db[co] + v : v;
    }
  }
}
}  // namespace

size_t pf_wino6_ws_bytes(int n, int h, int w, int Cin, int Cout) {
  const size_t T = (size_t)n * ((h + 5) / 6) * ((w + 5) / 6);
  return pf_align(64 * T * Cin * 4, 256) + pf_align(64 * T * Cout * 4, 256);
}

size_t pf_wino6_weights_floats(int Cin, int Cout, bool planes) {
  return (size_t)(planes ? 96 : 64) * Cin * Cout;
}

int pf_wino6_weights(const float* wpk, int Cout, int Cin, float* U, hipStream_t st, bool planes) {
  if (Cin % 32 || Cout % 4) return POSFEAT_E_INVALID;
  const int kpad = posfeat_conv_packed_k(Cin, 3, 3);
  planes = planes && wino_planes_ok(Cout);  // the condition pf_wino6_conv checks
  hipLaunchKernelGGL(wino6_weights_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256), 0,
                     st, wpk, Cout, Cin, kpad, U,
                     planes ? reinterpret_cast<unsigned short*>(U) : nullptr);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// The F(6x6) transforms one channel per thread (default, r16m) or channel
// pairs (POSFEAT_W6IN_VW1=0 / POSFEAT_W6OUT_VW1=0, A/B): the pair forms held
// 232 / 176 VGPRs (two waves per SIMD), the single-channel ones 111 / 104
// (four).  Same box, B = 32: output transforms 0.353 -> 0.322 ms
// (upconv2 / iconv2), 0.194 -> 0.163 (iconv3); the plain input transform
// 0.663 -> 0.654, 0.355 -> 0.345; bench 1299.0 -> 1308.1 img/s.  The same
// fma per channel: bit-identical.
static bool w6out_vw1() {
  static const bool v = [] {
    const char* e = pf_ab_getenv("POSFEAT_W6OUT_VW1");
    return !(e && e[0] == '0');
  }();
  return v;
}
// the fused upsample's half-res rows all loaded first (UPM = 1; A/B:
// POSFEAT_W6IN_UPM=0 -- the two-row window).  (Measured and removed, r16zn:
// each row from a six-column window with per-column picks instead of two
// loads per column -- bit-identical, 781 -> 839 us for upconv2's transform:
// the loads it saved hit in cache; and, r16zu, UPM = 1 forced to four waves
// per SIMD: 128 VGPRs with 24 spilled, 0.59 -> 0.82 ms)
static bool w6in_upm() {
  static const bool v = [] {
    const char* e = pf_ab_getenv("POSFEAT_W6IN_UPM");
    return !(e && e[0] == '0');
  }();
  return v;
}
static bool w6in_vw1() {
  static const bool v = [] {
    const char* e = pf_ab_getenv("POSFEAT_W6IN_VW1");
    return !(e && e[0] == '0');
  }();
  return v;
}

// planes 1: U holds the bf16 planes of pf_wino6_weights(.., planes = true)
// (Cout % 64 == 0), the GEMM splits V on the fly; 0: fp32 U.  up2: x is the
// (h/2, w/2) map, h and w even.
int pf_wino6_conv(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                  const float* bias, int Cout, int act, float* y, int ycs, void* ws,
                  size_t ws_bytes, hipStream_t st, int stages, int planes, int up2,
                  float* vkeep, double* stats) {
  if (stats && (act != POSFEAT_ACT_NONE || Cout % 64)) return POSFEAT_E_INVALID;
  if (Cin % 32 || Cout % 4 || xcs % 2 || ycs % 2 || n <= 0 || h <= 0 || w <= 0 || planes > 1)
    return POSFEAT_E_INVALID;
  if (up2 && ((h & 1) || (w & 1))) return POSFEAT_E_INVALID;
  if (ws_bytes < pf_wino6_ws_bytes(n, h, w, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  const long long T = (long long)n * ((h + 5) / 6) * ((w + 5) / 6);
  float* V = vkeep ? vkeep : static_cast<float*>(ws);
  float* M = reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(64 * T * Cin * 4, 256));
  if (stages & 1) {
    // fused upsample: one channel per thread (occupancy); plain: channel pairs
    if (up2 && w6in_upm())
      hipLaunchKernelGGL((wino6_input_kernel<true, 1, 1>), dim3(grid_for(T * Cin, 256)), dim3(256),
                         0, st, x, xcs, n, h, w, Cin, V);
    else if (up2)
      hipLaunchKernelGGL((wino6_input_kernel<true, 1>), dim3(grid_for(T * Cin, 256)), dim3(256), 0,
                         st, x, xcs, n, h, w, Cin, V);
    else if (w6in_vw1())  // A/B: one channel per thread (fewer VGPRs, more waves)
      hipLaunchKernelGGL((wino6_input_kernel<false, 1>), dim3(grid_for(T * Cin, 256)), dim3(256),
                         0, st, x, xcs, n, h, w, Cin, V);
    else
      hipLaunchKernelGGL((wino6_input_kernel<false, 2>), dim3(grid_for(T * (Cin / 2), 256)),
                         dim3(256), 0, st, x, xcs, n, h, w, Cin / 2, V);
    PF_CHECK_LAUNCH();
  }
  const unsigned short* Ub =
      planes == 1 && wino_planes_ok(Cout) ? reinterpret_cast<const unsigned short*>(U) : nullptr;
  if (stages & 2)
    PF_TRY(pf_gemm_batched(V, Cin, T * Cin, U, (long long)Cout * Cin, M, Cout, T * Cout, 64, (int)T,
                           Cout, Cin, st, Ub, 64LL * Cout * Cin));
  if ((stages & 4) && stats) {
    const int ng = pf_wino6_stats_groups(h, w);
    hipLaunchKernelGGL(wino6_output_stats_kernel, dim3((unsigned)(n * ng * (Cout / 64))),
                       dim3(256), 0, st, M, n, h, w, Cout, bias, y, ycs, stats);
    PF_CHECK_LAUNCH();
  } else if (stages & 4) {
    if (w6out_vw1())  // A/B: one channel per thread
      hipLaunchKernelGGL((wino6_output_kernel<1>), dim3(grid_for(T * Cout, 256)), dim3(256), 0, st,
                         M, n, h, w, Cout, bias, act, y, ycs);
    else
      hipLaunchKernelGGL((wino6_output_kernel<2>), dim3(grid_for(T * (Cout / 2), 256)), dim3(256),
                         0, st, M, n, h, w, Cout / 2, bias, act, y, ycs);
    PF_CHECK_LAUNCH();
  }
  return POSFEAT_OK;
}

namespace {

// F(4x4) when both dims are multiples of 4 (all decoder layers at 480x640)
// unless POSFEAT_WINO=1 (F(2x2) only)
bool use_f4(int h, int w) {
  static const bool f2only = [] {
    const char* e = pf_ab_getenv("POSFEAT_WINO");
    return e && e[0] == '1';
  }();
  return !f2only && h % 4 == 0 && w % 4 == 0;
}

}  // namespace

// workspace / weights sized for the larger of the two variants (F(2x2):
// 16 x T2, F(4x4): 36 x T2 / 4), so callers need not know which runs
size_t pf_wino_ws_bytes(int n, int h, int w, int Cin, int Cout) {
  const size_t T = (size_t)n * (h / 2) * (w / 2);
  return pf_align(16 * T * Cin * 4, 256) + pf_align(16 * T * Cout * 4, 256);
}

size_t pf_wino_weights_floats(int Cin, int Cout) { return (size_t)36 * Cin * Cout; }

// U for the variant pf_wino_conv will pick at (h, w); h = w = 0: F(2x2)
size_t pf_wino_weights_floats_bf6p(int Cin, int Cout) { return (size_t)54 * Cin * Cout; }


int pf_wino_weights_hw(const float* wpk, int Cout, int Cin, int h, int w, float* U,
                       hipStream_t st, bool bf6p) {
  if (Cin % 32 || Cout % 4) return POSFEAT_E_INVALID;
  const int kpad = posfeat_conv_packed_k(Cin, 3, 3);
  bf6p = bf6p && wino_planes_ok(Cout);  // the same condition as wino_conv_impl's plane paths
  if (h > 0 && use_f4(h, w))
    hipLaunchKernelGGL(wino4_weights_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256),
                       0, st, wpk, Cout, Cin, kpad, U,
                       bf6p ? reinterpret_cast<unsigned short*>(U) : nullptr);
  else
    hipLaunchKernelGGL(wino_weights_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256),
                       0, st, wpk, Cout, Cin, kpad, U,
                       bf6p && h > 0 ? reinterpret_cast<unsigned short*>(U) : nullptr);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_wino_weights(const float* wpk, int Cout, int Cin, float* U, hipStream_t st) {
  return pf_wino_weights_hw(wpk, Cout, Cin, 0, 0, U, st);
}

static int wino_conv_impl(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                          bool U_is_f4, const float* bias, int Cout, int act, float* y, int ycs,
                          void* ws, size_t ws_bytes, hipStream_t st, int stages = 7,
                          int planes = 0, int up2 = 0) {
  const bool bf6p = planes == 2;
  if (up2 && !(use_f4(h, w) && U_is_f4 && h % 2 == 0 && w % 2 == 0)) return POSFEAT_E_UNSUPPORTED;
  if ((h & 1) || (w & 1) || Cin % 32 || Cout % 4 || xcs % 4 || ycs % 4 || n <= 0)
    return POSFEAT_E_INVALID;
  if (ws_bytes < pf_wino_ws_bytes(n, h, w, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  if (use_f4(h, w) && U_is_f4 && bf6p && wino_planes_ok(Cout)) {
    // bf16x6: V as three bf16 planes (54 T4 Cin bytes <= the F(2x2) V region),
    // M after them; U holds three planes (pf_wino_weights_hw(..., bf6p))
    const long long T4 = (long long)n * (h / 4) * (w / 4);
    unsigned short* Vb = static_cast<unsigned short*>(ws);
    float* M4 =
        reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(36 * T4 * Cin * 6, 256));
    if (stages & 1) {
      hipLaunchKernelGGL(wino4_input_kernel, dim3(grid_for(T4 * (Cin / 4), 256)), dim3(256), 0, st,
                         x, xcs, n, h, w, Cin / 4, nullptr, 0, Vb, up2);
      PF_CHECK_LAUNCH();
    }
    if (stages & 2)
      PF_TRY(pf_gemm_bf6p(Vb, Cin, 36 * T4 * Cin, T4 * Cin,
                          reinterpret_cast<const unsigned short*>(U), Cin, 36LL * Cout * Cin,
                          (long long)Cout * Cin, M4, Cout, T4 * Cout, 36, (int)T4, Cout, Cin, st));
    if (stages & 4) {
      hipLaunchKernelGGL(wino4_output_kernel, dim3(grid_for(T4 * (Cout / 4), 256)), dim3(256), 0,
                         st, M4, n, h, w, Cout / 4, bias, act, y, ycs);
      PF_CHECK_LAUNCH();
    }
    return POSFEAT_OK;
  }
  if (use_f4(h, w) && U_is_f4) {
    const long long T4 = (long long)n * (h / 4) * (w / 4);
    float* V4 = static_cast<float*>(ws);
    float* M4 =
        reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(36 * T4 * Cin * 4, 256));
    if (stages & 1) {
      hipLaunchKernelGGL(wino4_input_kernel, dim3(grid_for(T4 * (Cin / 4), 256)), dim3(256), 0, st,
                         x, xcs, n, h, w, Cin / 4, V4, 0, nullptr, up2);
      PF_CHECK_LAUNCH();
    }
    if (stages & 2)  // planes == 1: U holds its bf16 planes (pre-split bf16x6 tiles)
      PF_TRY(pf_gemm_batched(V4, Cin, T4 * Cin, U, (long long)Cout * Cin, M4, Cout, T4 * Cout, 36,
                             (int)T4, Cout, Cin, st,
                             planes == 1 && wino_planes_ok(Cout)
                                 ? reinterpret_cast<const unsigned short*>(U)
                                 : nullptr,
                             36LL * Cout * Cin));
    if (stages & 4) {
      hipLaunchKernelGGL(wino4_output_kernel, dim3(grid_for(T4 * (Cout / 4), 256)), dim3(256), 0,
                         st, M4, n, h, w, Cout / 4, bias, act, y, ycs);
      PF_CHECK_LAUNCH();
    }
    return POSFEAT_OK;
  }
  const long long T = (long long)n * (h / 2) * (w / 2);
  float* V = static_cast<float*>(ws);
  float* M = reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(16 * T * Cin * 4, 256));
  if (stages & 1) {
    hipLaunchKernelGGL(wino_input_kernel, dim3(grid_for(T * (Cin / 4), 256)), dim3(256), 0, st, x,
                       xcs, n, h, w, Cin / 4, V);
    PF_CHECK_LAUNCH();
  }
  if (stages & 2)  // planes == 1 (and U from pf_wino_weights_hw for this h, w): bf16 planes
    PF_TRY(pf_gemm_batched(V, Cin, T * Cin, U, (long long)Cout * Cin, M, Cout, T * Cout, 16,
                           (int)T, Cout, Cin, st,
                           planes >= 1 && U_is_f4 && wino_planes_ok(Cout)
                               ? reinterpret_cast<const unsigned short*>(U)
                               : nullptr,
                           16LL * Cout * Cin));
  if (stages & 4) {
    hipLaunchKernelGGL(wino_output_kernel, dim3(grid_for(T * (Cout / 4), 256)), dim3(256), 0, st,
                       M, n, h, w, Cout / 4, bias, act, y, ycs);
    PF_CHECK_LAUNCH();
  }
  return POSFEAT_OK;
}

// U from pf_wino_weights_hw(.., h, w, ..): the variant is chosen from (h, w)
int pf_wino_conv(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                 const float* bias, int Cout, int act, float* y, int ycs, void* ws, size_t ws_bytes,
                 hipStream_t st, int stages, int planes, int up2) {
  return wino_conv_impl(x, xcs, n, h, w, Cin, U, true, bias, Cout, act, y, ycs, ws, ws_bytes, st,
                        stages, planes, up2);
}

namespace {
// split the tile reduction so the 36 x (Cout/128) x (Cin/128) GEMM tiles reach >= 2048
// workgroups (1024..8192 measured within 1% of each other)
int wino_wgrad_nsplit(long long T, int Cin, int Cout, int nb = 36) {
  // (Cin, Cout % 128 == 0 for every caller; guarded so no shape divides by 0 --
  // tools/asan_host.py found posfeat_wino_wgrad_workspace(.., cin = 32, ..)
  // raising SIGFPE here)
  const long long tiles = std::max(1LL, (long long)nb * (Cout / 128) * (Cin / 128));
  static const int target = [] {  // A/B knob POSFEAT_WINO_WG_TARGET (unset: 2048)
    const char* e = pf_ab_getenv("POSFEAT_WINO_WG_TARGET");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 2048;
  }();
  long long s = (target + tiles - 1) / tiles;
  const long long chunks = (T + 63) / 64;
  s = std::min(s, std::max(1LL, chunks / 8));  // >= 8 row chunks per split
  return (int)std::max(1LL, std::min(s, 16LL));
}
}  // namespace

// V [36][T][Cin] | dM [36][T][Cout] | GEMM partials [36][nsplit][Cout][Cin] | bias partials
size_t pf_wino_wgrad_ws_bytes(int n, int h, int w, int Cin, int Cout) {
  const long long T = (long long)n * (h / 4) * (w / 4);
  const int ns = wino_wgrad_nsplit(T, Cin, Cout);
  return pf_align(36 * T * Cin * 4, 256) + pf_align(36 * T * Cout * 4, 256) +
         pf_align((size_t)36 * ns * Cout * Cin * 4, 256) + pf_align((size_t)ns * Cout * 4, 256);
}

// Weight gradient of a 3x3 stride-1 pad-1 conv by F(4x4) (h, w % 4 == 0;
// Cin, Cout % 128 == 0): dy compact [n][h][w][Cout] (pitch ldy), x the layer
// input (pitch xcs); dw packed like the engine's weights, db optional; acc adds.
int pf_wino_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int h, int w, int Cin,
                  int Cout, float* dw, float* db, int acc, void* ws, size_t ws_bytes,
                  hipStream_t st) {
  if (h % 4 || w % 4 || Cin % 128 || Cout % 128 || ldy % 4 || xcs % 4) return POSFEAT_E_INVALID;
  if (ws_bytes < pf_wino_wgrad_ws_bytes(n, h, w, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  const long long T = (long long)n * (h / 4) * (w / 4);
  const int ns = wino_wgrad_nsplit(T, Cin, Cout);
  char* p = static_cast<char*>(ws);
  float* V = reinterpret_cast<float*>(p);
  p += pf_align(36 * T * Cin * 4, 256);
  float* dM = reinterpret_cast<float*>(p);
  p += pf_align(36 * T * Cout * 4, 256);
  float* part = reinterpret_cast<float*>(p);
  p += pf_align((size_t)36 * ns * Cout * Cin * 4, 256);
  float* partb = reinterpret_cast<float*>(p);
  hipLaunchKernelGGL(wino4_input_kernel, dim3(grid_for(T * (Cin / 4), 256)), dim3(256), 0, st, x,
                     xcs, n, h, w, Cin / 4, V, 0);
  hipLaunchKernelGGL(wino4_dy_kernel, dim3(grid_for(T * (Cout / 4), 256)), dim3(256), 0, st, dy,
                     ldy, n, h, w, Cout / 4, dM);
  PF_CHECK_LAUNCH();
  // xi = (1, 1): A^T's column 1 is all ones, so sum_tiles dM_7 = sum_pixels dy (the bias)
  PF_TRY(pf_wgrad_gemm_batched(dM, Cout, T * Cout, V, Cin, T * Cin, (int)T, Cin, Cout, 36, ns,
                               part, db ? partb : nullptr, 7, st));
  const int kpad = posfeat_conv_packed_k(Cin, 3, 3);
  hipLaunchKernelGGL(wino4_wgrad_out_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256),
                     0, st, part, ns, Cout, Cin, kpad, dw, partb, db, acc);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// V [64][T][Cin] | dM [64][T][Cout] | GEMM partials [64][nsplit][Cout][Cin] | bias partials
size_t pf_wino6_wgrad_ws_bytes(int n, int h, int w, int Cin, int Cout) {
  const long long T = (long long)n * ((h + 5) / 6) * ((w + 5) / 6);
  const int ns = wino_wgrad_nsplit(T, Cin, Cout, 64);
  return pf_align(64 * T * Cin * 4, 256) + pf_align(64 * T * Cout * 4, 256) +
         pf_align((size_t)64 * ns * Cout * Cin * 4, 256) + pf_align((size_t)ns * Cout * 4, 256);
}

// Weight gradient of a 3x3 stride-1 pad-1 conv by F(6x6) (any h, w; Cin,
// Cout % 128 == 0), arguments as pf_wino_wgrad's
int pf_wino6_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int h, int w, int Cin,
                   int Cout, float* dw, float* db, int acc, void* ws, size_t ws_bytes,
                   hipStream_t st, const float* vpre) {
  if (Cin % 128 || Cout % 128 || ldy % 2 || xcs % 2 || n <= 0 || h <= 0 || w <= 0)
    return POSFEAT_E_INVALID;
  if (ws_bytes < pf_wino6_wgrad_ws_bytes(n, h, w, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  const long long T = (long long)n * ((h + 5) / 6) * ((w + 5) / 6);
  const int ns = wino_wgrad_nsplit(T, Cin, Cout, 64);
  char* p = static_cast<char*>(ws);
  float* V = reinterpret_cast<float*>(p);
  p += pf_align(64 * T * Cin * 4, 256);
  float* dM = reinterpret_cast<float*>(p);
  p += pf_align(64 * T * Cout * 4, 256);
  float* part = reinterpret_cast<float*>(p);
  p += pf_align((size_t)64 * ns * Cout * Cin * 4, 256);
  float* partb = reinterpret_cast<float*>(p);
  if (vpre)  // the forward's V of the same x (pf_wino6_conv's vkeep)
    V = const_cast<float*>(vpre);
  else
    hipLaunchKernelGGL((wino6_input_kernel<false, 2>), dim3(grid_for(T * (Cin / 2), 256)),
                       dim3(256), 0, st, x, xcs, n, h, w, Cin / 2, V);
  hipLaunchKernelGGL(wino6_dy_kernel, dim3(grid_for(T * (Cout / 2), 256)), dim3(256), 0, st, dy,
                     ldy, n, h, w, Cout / 2, dM);
  PF_CHECK_LAUNCH();
  PF_TRY(pf_wgrad_gemm_batched(dM, Cout, T * Cout, V, Cin, T * Cin, (int)T, Cin, Cout, 64, ns,
                               part, db ? partb : nullptr, 9, st));
  const int kpad = posfeat_conv_packed_k(Cin, 3, 3);
  hipLaunchKernelGGL(wino6_wgrad_out_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256),
                     0, st, part, ns, Cout, Cin, kpad, dw, partb, db, acc);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" size_t posfeat_wino_wgrad_workspace(int n, int h, int w, int cin, int cout) {
  // the shapes posfeat_conv3x3_wino_wgrad accepts (pf_wino_wgrad), else 0
  if (n <= 0 || h <= 0 || w <= 0 || (h & 3) || (w & 3) || cin <= 0 || cout <= 0 || cin % 128 ||
      cout % 128)
    return 0;
  return pf_wino_wgrad_ws_bytes(n, h, w, cin, cout);
}

extern "C" int posfeat_conv3x3_wino_wgrad(const float* dy, int dy_cstride, const float* x,
                                          int x_cstride, int n, int h, int w, int cin, int cout,
                                          float* dw, float* db, void* ws, size_t ws_bytes,
                                          void* stream) {
  if (!dy || !x || !dw || !ws || n <= 0) return POSFEAT_E_INVALID;
  return pf_wino_wgrad(dy, dy_cstride, x, x_cstride, n, h, w, cin, cout, dw, db, 0, ws, ws_bytes,
                       pf_stream(stream));
}

extern "C" size_t posfeat_wino_workspace(int n, int h, int w, int cin, int cout) {
  if (n <= 0 || h <= 0 || w <= 0 || (h & 1) || (w & 1)) return 0;
  return pf_wino_ws_bytes(n, h, w, cin, cout);
}

extern "C" int posfeat_wino_weights(const float* w_packed, int cout, int cin, int h, int w,
                                    float* U, void* stream) {
  if (!w_packed || !U) return POSFEAT_E_INVALID;
  return pf_wino_weights_hw(w_packed, cout, cin, h, w, U, pf_stream(stream));
}

extern "C" int posfeat_conv3x3_wino(const float* x, int x_cstride, int n, int h, int w, int cin,
                                    const float* U, const float* bias, int cout, int act, float* y,
                                    int y_cstride, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !U || !y || !ws) return POSFEAT_E_INVALID;
  return pf_wino_conv(x, x_cstride, n, h, w, cin, U, bias, cout, act, y, y_cstride, ws, ws_bytes,
                      pf_stream(stream));
}

extern "C" size_t posfeat_wino6_workspace(int n, int h, int w, int cin, int cout) {
  if (n <= 0 || h <= 0 || w <= 0) return 0;
  return pf_wino6_ws_bytes(n, h, w, cin, cout);
}

extern "C" int posfeat_wino6_weights(const float* w_packed, int cout, int cin, float* U,
                                     void* stream) {
  if (!w_packed || !U) return POSFEAT_E_INVALID;
  return pf_wino6_weights(w_packed, cout, cin, U, pf_stream(stream), false);
}

extern "C" int posfeat_conv3x3_wino6(const float* x, int x_cstride, int n, int h, int w, int cin,
                                     const float* U, const float* bias, int cout, int act, float* y,
                                     int y_cstride, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !U || !y || !ws) return POSFEAT_E_INVALID;
  return pf_wino6_conv(x, x_cstride, n, h, w, cin, U, bias, cout, act, y, y_cstride, ws, ws_bytes,
                       pf_stream(stream), 7, 0, 0);
}

// ---- test surfaces of the engine's F(6x6) paths -----------------------------
// (the extraction engine's bf16 three-plane U, the decoder's fused x2
// upsample, and the training step's F(6x6) weight gradient)
extern "C" size_t posfeat_wino6_weights_floats(int cin, int cout, int planes) {
  if (cin <= 0 || cout <= 0) return 0;
  return pf_wino6_weights_floats(cin, cout, planes != 0 && wino_planes_ok(cout));
}

extern "C" int posfeat_wino6_weights_planes(const float* w_packed, int cout, int cin, int planes,
                                            float* U, void* stream) {
  if (!w_packed || !U || planes < 0 || planes > 1) return POSFEAT_E_INVALID;
  return pf_wino6_weights(w_packed, cout, cin, U, pf_stream(stream), planes != 0);
}

extern "C" int posfeat_conv3x3_wino6_ex(const float* x, int x_cstride, int n, int h, int w,
                                        int cin, const float* U, int planes, int up2,
                                        const float* bias, int cout, int act, float* y,
                                        int y_cstride, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !U || !y || !ws || planes < 0 || planes > 1 || up2 < 0 || up2 > 1)
    return POSFEAT_E_INVALID;
  if (planes && !wino_planes_ok(cout)) return POSFEAT_E_INVALID;
  return pf_wino6_conv(x, x_cstride, n, h, w, cin, U, bias, cout, act, y, y_cstride, ws, ws_bytes,
                       pf_stream(stream), 7, planes, up2);
}

extern "C" size_t posfeat_wino6_wgrad_workspace(int n, int h, int w, int cin, int cout) {
  if (n <= 0 || h <= 0 || w <= 0 || cin % 128 || cout % 128 || cin <= 0 || cout <= 0) return 0;
  return pf_wino6_wgrad_ws_bytes(n, h, w, cin, cout);
}

extern "C" int posfeat_conv3x3_wino6_wgrad(const float* dy, int dy_cstride, const float* x,
                                           int x_cstride, int n, int h, int w, int cin, int cout,
                                           float* dw, float* db, void* ws, size_t ws_bytes,
                                           void* stream) {
  if (!dy || !x || !dw || !ws || n <= 0) return POSFEAT_E_INVALID;
  return pf_wino6_wgrad(dy, dy_cstride, x, x_cstride, n, h, w, cin, cout, dw, db, 0, ws, ws_bytes,
                        pf_stream(stream), nullptr);
}
