// conv.hip -- fused NHWC convolution as an implicit GEMM on gfx950 FP32 MFMA.
//
// Replaces the ATen conv2d (+ eval BatchNorm + ReLU/ELU + residual add) of
// networks/DescNet.py:167-190, the torchvision Bottleneck convs used at
// DescNet.py:27-35, and the bias-only convs of networks/DeteNet.py:11-21.
//
// GEMM view: M = output pixels (n, oh, ow), N = cout, K = (kh, kw, cin).
//   A[m][k] = x[n][oh*s-p+kh][ow*s-p+kw][cin]  (gathered, zero outside)
//   B[k][n] = w[cout][k]  (packed host-side, BN folded, K padded to 32)
// Tiles: BM x BN per 4-wave workgroup, BK = 32, two LDS stages filled by
// register staging (global loads for chunk c+1 are in flight while chunk c
// is multiplied).  LDS rows are k-contiguous with a 36-float pitch, so the
// MFMA operand reads are conflict-free ds_read_b128 (9 slots per row: odd).
// Each lane half supplies 4 consecutive k per b128 read; MFMA j of a k-group
// of 8 contracts k-pair {j, 4+j} -- the same permutation on A and B, so the
// product is exact f32 fmaf chains in a fixed (deterministic) order.
#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int LDSP = BK + 4;  // LDS row pitch (floats)

struct ConvArgs {
  const float* x;
  const float* w;
  const float* bias;
  const float* res;
  float* y;
  int H, W, Cin, xcs;
  int Cout, KH, KW, stride, pad;
  int OH, OW, M, K, Kpad;
  int ycs, rcs, act;
  int tiles_n, nwg;
};

template <int BM, int BN, int WM, int WN, bool CIN32>
__global__ __launch_bounds__(WM* WN * 64) void conv_mfma_kernel(ConvArgs a) {
  constexpr int THREADS = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int A_LD = BM * (BK / 4) / THREADS;
  constexpr int B_LD = BN * (BK / 4) / THREADS;
  static_assert(A_LD >= 1 && B_LD >= 1, "tile too small for the block");
  static_assert(MI >= 1 && NI >= 1, "wave tile must be >= 32x32");

  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDSP];
  float* As = smem;                    // [2][BM][LDSP]
  float* Bs = smem + 2 * BM * LDSP;    // [2][BN][LDSP]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a
  // contiguous range of tile ids so the N-tiles of one M-tile share its L2.
  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread A rows (fixed across K) --------------------------------
  const float* xrow[A_LD];
  int ih0[A_LD], iw0[A_LD];
  const int kq = tid & 7;
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int row = (tid >> 3) + i * (THREADS / 8);
    const int m = m0 + row;
    if (m < a.M) {
      const int hw = a.OH * a.OW;
      const int n = m / hw;
      const int rem = m - n * hw;
      const int oh = rem / a.OW;
      const int ow = rem - oh * a.OW;
      xrow[i] = a.x + (size_t)n * a.H * a.W * a.xcs;
      ih0[i] = oh * a.stride - a.pad;
      iw0[i] = ow * a.stride - a.pad;
    } else {
      xrow[i] = nullptr;
      ih0[i] = -100000;
      iw0[i] = -100000;
    }
  }
  const float* wrow[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int row = (tid >> 3) + i * (THREADS / 8);
    wrow[i] = (n0 + row < a.Cout) ? a.w + (size_t)(n0 + row) * a.Kpad + kq * 4 : nullptr;
  }

  f32x4 ra[A_LD], rb[B_LD];
  int tap = 0, c0 = 0;  // CIN32 path: k0 = tap*Cin + c0

  auto load_chunk = [&](int k0) {
    if constexpr (CIN32) {
      const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const int ih = ih0[i] + kh, iw = iw0[i] + kw;
        if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) {
          ra[i] = *reinterpret_cast<const f32x4*>(xrow[i] + ((size_t)ih * a.W + iw) * a.xcs +
                                                   c0 + kq * 4);
        } else {
          ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    } else {
      const int k = k0 + kq * 4;
      int kh = 0, kw = 0, c = 0;
      const bool kin = k < a.K;
      if (kin) {
        const int t = k / a.Cin;
        c = k - t * a.Cin;
        kh = t / a.KW;
        kw = t - kh * a.KW;
      }
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        const int ih = ih0[i] + kh, iw = iw0[i] + kw;
        if (kin && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) {
          ra[i] = *reinterpret_cast<const f32x4*>(xrow[i] + ((size_t)ih * a.W + iw) * a.xcs + c);
        } else {
          ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      rb[i] = wrow[i] ? *reinterpret_cast<const f32x4*>(wrow[i] + k0) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (CIN32) {
      c0 += BK;
      if (c0 == a.Cin) {
        c0 = 0;
        ++tap;
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int row = (tid >> 3) + i * (THREADS / 8);
      *reinterpret_cast<f32x4*>(As + (buf * BM + row) * LDSP + kq * 4) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int row = (tid >> 3) + i * (THREADS / 8);
      *reinterpret_cast<f32x4*>(Bs + (buf * BN + row) * LDSP + kq * 4) = rb[i];
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int nch = a.Kpad / BK;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();

  const int arow = wm * TM + (lane & 31);
  const int brow = wn * TN + (lane & 31);
  const int kofs = 4 * (lane >> 5);

  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) load_chunk((c + 1) * BK);
    const float* Ab = As + (cur * BM + arow) * LDSP + kofs;
    const float* Bb = Bs + (cur * BN + brow) * LDSP + kofs;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      f32x4 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const f32x4*>(Ab + mi * 32 * LDSP + kk * 8);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const f32x4*>(Bb + ni * 32 * LDSP + kk * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][j], bv[ni][j], acc[mi][ni],
                                                                0, 0, 0);
    }
    if (c + 1 < nch) store_chunk(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias + residual + activation, NHWC store ----------------
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn * TN + ni * 32 + (lane & 31);
    if (col >= a.Cout) continue;
    const float bsv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= a.M) continue;
        float v = acc[mi][ni][r] + bsv;
        if (a.res) v += a.res[(size_t)m * a.rcs + col];
        if (a.act == POSFEAT_ACT_RELU) v = fmaxf(v, 0.f);
        else if (a.act == POSFEAT_ACT_ELU) v = pf_elu(v);
        a.y[(size_t)m * a.ycs + col] = v;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(ConvArgs& a, bool cin32, hipStream_t st) {
  const int tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.nwg = tiles_m * a.tiles_n;
  dim3 grid(a.nwg), block(WM * WN * 64);
  if (cin32)
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, true>), grid, block, 0, st, a);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, false>), grid, block, 0, st, a);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

}  // namespace

extern "C" int posfeat_conv_packed_k(int cin, int kh, int kw) {
  const int cinp = (cin + 3) / 4 * 4;
  const int k = kh * kw * cinp;
  return (k + BK - 1) / BK * BK;
}

extern "C" int posfeat_conv2d_nhwc(const posfeat_conv_desc* d, const float* x, const float* w,
                                   const float* bias, const float* res, float* y, void* stream) {
  if (!d || !x || !w || !y) return POSFEAT_E_INVALID;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->cin <= 0 || d->cin % 4 || d->cout <= 0)
    return POSFEAT_E_INVALID;
  if (d->x_cstride < d->cin || d->x_cstride % 4 || d->y_cstride < d->cout) return POSFEAT_E_INVALID;
  if (d->kh <= 0 || d->kw <= 0 || d->stride <= 0 || d->pad < 0) return POSFEAT_E_INVALID;
  if (res && d->res_cstride < d->cout) return POSFEAT_E_INVALID;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15))
    return POSFEAT_E_INVALID;
  ConvArgs a;
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.H = d->h;
  a.W = d->w;
  a.Cin = d->cin;
  a.xcs = d->x_cstride;
  a.Cout = d->cout;
  a.KH = d->kh;
  a.KW = d->kw;
  a.stride = d->stride;
  a.pad = d->pad;
  a.OH = (d->h + 2 * d->pad - d->kh) / d->stride + 1;
  a.OW = (d->w + 2 * d->pad - d->kw) / d->stride + 1;
  if (a.OH <= 0 || a.OW <= 0) return POSFEAT_E_INVALID;
  a.M = d->n * a.OH * a.OW;
  a.K = d->kh * d->kw * d->cin;
  a.Kpad = posfeat_conv_packed_k(d->cin, d->kh, d->kw);
  a.ycs = d->y_cstride;
  a.rcs = d->res_cstride;
  a.act = d->act;
  const bool cin32 = (d->cin % BK) == 0;
  hipStream_t st = pf_stream(stream);
  // Tile choice: the largest tile that still gives >= 2 workgroups per CU.
  const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
  const long long t128x64 = (long long)((a.M + 127) / 128) * ((a.Cout + 63) / 64);
  if (a.Cout > 64 && t128 >= 512) return launch_cfg<128, 128, 2, 2>(a, cin32, st);
  if (t128x64 >= 512) return launch_cfg<128, 64, 2, 2>(a, cin32, st);
  return launch_cfg<64, 64, 2, 2>(a, cin32, st);
}
