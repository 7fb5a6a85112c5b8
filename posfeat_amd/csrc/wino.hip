// wino.hip -- Winograd F(2x2, 3x3) for the decoder's 3x3 stride-1 convs
// (upconv3/iconv3/upconv2/iconv2, DescNet.py:41-45: 4 x 45.3 GFLOP per
// 480x640 image, 43 % of the extraction's conv work).
//
//   U = G g G^T   (once per weight update; [16][Cout][Cin])
//   V = B^T d B   per 2x2 output tile, 4x4 input patch   ([16][T][Cin])
//   M_xi = V_xi U_xi^T   16 GEMMs in ONE launch of the conv engine's
//                        conv_glds_kernel (blockIdx.y = xi)   ([16][T][Cout])
//   Y = A^T M A (+ bias, activation) into the NHWC output (channel slice)
//
// 16 instead of 36 MACs per tile and channel pair: the GEMM is 2.25x smaller
// than the direct conv; the transforms are two HBM passes.  Transforms are
// exact-weight (+-1, 1/2) so the result differs from the direct conv by fp32
// rounding only (tests/test_gpu_ops.py).
#include "common.h"
#include "fmap.h"

namespace {

int grid_for(long long total, int block) {
  long long g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

// U[xi][co][ci] from the engine-packed 3x3 weights [Cout][Kpad], K order
// ((ci/32)*9 + tap)*32 + ci%32 (Cin % 32 == 0)
__global__ void wino_weights_kernel(const float* __restrict__ wpk, int Cout, int Cin, int kpad,
                                    float* __restrict__ U) {
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
      U[((long long)(a * 4 + 0) * Cout + co) * Cin + ci] = u0;
      U[((long long)(a * 4 + 1) * Cout + co) * Cin + ci] = u1;
      U[((long long)(a * 4 + 2) * Cout + co) * Cin + ci] = u2;
      U[((long long)(a * 4 + 3) * Cout + co) * Cin + ci] = u3;
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
    const int q = (int)(i % c4n);
    const long long tile = i / c4n;
    const int tx = (int)(tile % tw);
    const long long r0 = tile / tw;
    const int ty = (int)(r0 % th);
    const int b = (int)(r0 / th);
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
    const int q = (int)(i % c4n);
    const long long tile = i / c4n;
    const int tx = (int)(tile % tw);
    const long long r0 = tile / tw;
    const int ty = (int)(r0 % th);
    const int b = (int)(r0 / th);
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

}  // namespace

size_t pf_wino_ws_bytes(int n, int h, int w, int Cin, int Cout) {
  const size_t T = (size_t)n * (h / 2) * (w / 2);
  return pf_align(16 * T * Cin * 4, 256) + pf_align(16 * T * Cout * 4, 256);
}

size_t pf_wino_weights_floats(int Cin, int Cout) { return (size_t)16 * Cin * Cout; }

int pf_wino_weights(const float* wpk, int Cout, int Cin, float* U, hipStream_t st) {
  if (Cin % 32 || Cout % 4) return POSFEAT_E_INVALID;
  const int kpad = posfeat_conv_packed_k(Cin, 3, 3);
  hipLaunchKernelGGL(wino_weights_kernel, dim3(grid_for((long long)Cout * Cin, 256)), dim3(256), 0,
                     st, wpk, Cout, Cin, kpad, U);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_wino_conv(const float* x, int xcs, int n, int h, int w, int Cin, const float* U,
                 const float* bias, int Cout, int act, float* y, int ycs, void* ws, size_t ws_bytes,
                 hipStream_t st) {
  if ((h & 1) || (w & 1) || Cin % 32 || Cout % 4 || xcs % 4 || ycs % 4 || n <= 0)
    return POSFEAT_E_INVALID;
  if (ws_bytes < pf_wino_ws_bytes(n, h, w, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  const long long T = (long long)n * (h / 2) * (w / 2);
  float* V = static_cast<float*>(ws);
  float* M = reinterpret_cast<float*>(static_cast<char*>(ws) + pf_align(16 * T * Cin * 4, 256));
  hipLaunchKernelGGL(wino_input_kernel, dim3(grid_for(T * (Cin / 4), 256)), dim3(256), 0, st, x,
                     xcs, n, h, w, Cin / 4, V);
  PF_CHECK_LAUNCH();
  PF_TRY(pf_gemm_batched(V, Cin, T * Cin, U, (long long)Cout * Cin, M, Cout, T * Cout, 16, (int)T,
                         Cout, Cin, st));
  hipLaunchKernelGGL(wino_output_kernel, dim3(grid_for(T * (Cout / 4), 256)), dim3(256), 0, st, M,
                     n, h, w, Cout / 4, bias, act, y, ycs);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" size_t posfeat_wino_workspace(int n, int h, int w, int cin, int cout) {
  if (n <= 0 || h <= 0 || w <= 0 || (h & 1) || (w & 1)) return 0;
  return pf_wino_ws_bytes(n, h, w, cin, cout);
}

extern "C" int posfeat_wino_weights(const float* w_packed, int cout, int cin, float* U,
                                    void* stream) {
  if (!w_packed || !U) return POSFEAT_E_INVALID;
  return pf_wino_weights(w_packed, cout, cin, U, pf_stream(stream));
}

extern "C" int posfeat_conv3x3_wino(const float* x, int x_cstride, int n, int h, int w, int cin,
                                    const float* U, const float* bias, int cout, int act, float* y,
                                    int y_cstride, void* ws, size_t ws_bytes, void* stream) {
  if (!x || !U || !y || !ws) return POSFEAT_E_INVALID;
  return pf_wino_conv(x, x_cstride, n, h, w, cin, U, bias, cout, act, y, y_cstride, ws, ws_bytes,
                      pf_stream(stream));
}
