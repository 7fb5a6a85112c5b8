// conv.hip -- fused NHWC convolution as an implicit GEMM on gfx950 FP32 MFMA.
//
// Replaces the ATen conv2d (+ eval BatchNorm + ReLU/ELU + residual add) of
// networks/DescNet.py:167-190, the torchvision Bottleneck convs used at
// DescNet.py:27-35, and the bias-only convs of networks/DeteNet.py:11-21.
//
// GEMM view: M = output pixels (n, oh, ow), N = cout, K = (kh, kw, cin).
//   A[m][k] = x[n][oh*s-p+kh][ow*s-p+kw][cin]  (gathered, zero outside)
//   B[k][n] = w[cout][k]  (packed host-side, BN folded, K padded to 32)
// K order: when Cin % 32 == 0 the packed K index is (cin/32, kh, kw, cin%32):
// all taps of one 32-channel slab are consumed back to back, so the 3x3 halo
// of that slab (a few tens of KB per tile) is re-read from L1/L2 instead of
// once per tap from the Infinity Cache/HBM.  Otherwise (Cin = 4: the stem and
// convimg) K is (kh, kw, cin4) zero-padded to a multiple of 32.
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
  int ksplit;        // > 1: grid = nwg * ksplit, raw partials to `part`
  float* part;       // [ksplit][M][Cout] fp32 partial sums
  float* stats;      // optional [tiles_m][2 slots][Cout][2] per-tile (sum, sumsq)
  int hw;            // OH*OW (image boundary inside a tile for `stats`)
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
  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
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
  const int ntap = a.KH * a.KW;
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);
  int tap = ch0 % ntap, c0 = (ch0 / ntap) * BK;  // CIN32: chunk = (c0/32)*KH*KW + tap

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
      if (++tap == ntap) {
        tap = 0;
        c0 += BK;
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

  const int nch = ch1 - ch0;
  const int kbase = ch0 * BK;
  load_chunk(kbase);
  store_chunk(0);
  __syncthreads();

  const int arow = wm * TM + (lane & 31);
  const int brow = wn * TN + (lane & 31);
  const int kofs = 4 * (lane >> 5);

  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) load_chunk(kbase + (c + 1) * BK);
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

  // ---- epilogue, staged through LDS so global traffic is 16-B per lane ----
  // acc -> T[BM][BN+4] (conflict-free: a half-wave writes 32 consecutive
  // floats of one row), then each thread owns a fixed 4-column group and walks
  // rows: residual loads are all issued before use, stores are float4.
  constexpr int TP = BN + 4;
  float* T = smem;  // the K loop ended with a barrier: staging LDS is free
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        T[(wm * TM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * TP + wn * TN + ni * 32 +
          (lane & 31)] = acc[mi][ni][r];
  __syncthreads();
  constexpr int C4 = BN / 4;
  constexpr int RPP = THREADS / C4;  // rows per pass
  constexpr int NP = BM / RPP;
  const int q = tid % C4, r0 = tid / C4;
  const int col = n0 + 4 * q;
  const bool colok = col < a.Cout;
  if (a.ksplit > 1) {  // raw partial sums; conv_splitk_reduce finishes
    float* pp = a.part + (size_t)split * a.M * a.Cout;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = r0 + p * RPP;
      const int m = m0 + row;
      if (colok && m < a.M)
        *reinterpret_cast<f32x4*>(pp + (size_t)m * a.Cout + col) =
            *reinterpret_cast<const f32x4*>(T + row * TP + 4 * q);
    }
    return;
  }
  f32x4 rv[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int m = m0 + r0 + p * RPP;
    rv[p] = (a.res && colok && m < a.M)
                ? *reinterpret_cast<const f32x4*>(a.res + (size_t)m * a.rcs + col)
                : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const f32x4 bv = (a.bias && colok) ? *reinterpret_cast<const f32x4*>(a.bias + col)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 s1[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, s2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  const int img0 = m0 / a.hw;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = r0 + p * RPP;
    const int m = m0 + row;
    if (!colok || m >= a.M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(T + row * TP + 4 * q) + bv + rv[p];
    if (a.act == POSFEAT_ACT_RELU) {
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
    } else if (a.act == POSFEAT_ACT_ELU) {
      v.x = pf_elu(v.x);
      v.y = pf_elu(v.y);
      v.z = pf_elu(v.z);
      v.w = pf_elu(v.w);
    }
    *reinterpret_cast<f32x4*>(a.y + (size_t)m * a.ycs + col) = v;
    if (a.stats) {
      const int sl = (m / a.hw) != img0;
      if (sl) {
        s1[1] += v;
        s2[1] += v * v;
      } else {
        s1[0] += v;
        s2[0] += v * v;
      }
    }
  }
  if (a.stats) {  // reduce the RPP row groups of each column in a fixed order
    __syncthreads();
    float* R = smem;  // [RPP][2 slots][BN][2]
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        R[((r0 * 2 + sl) * BN + 4 * q + k) * 2 + 0] = s1[sl][k];
        R[((r0 * 2 + sl) * BN + 4 * q + k) * 2 + 1] = s2[sl][k];
      }
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += THREADS) {
      const int sl = e / BN, c = e - sl * BN;
      if (n0 + c >= a.Cout) continue;
      float t1 = 0.f, t2 = 0.f;
      for (int rr = 0; rr < RPP; ++rr) {
        t1 += R[((rr * 2 + sl) * BN + c) * 2 + 0];
        t2 += R[((rr * 2 + sl) * BN + c) * 2 + 1];
      }
      float* o = a.stats + (((size_t)tm * 2 + sl) * a.Cout + n0 + c) * 2;
      o[0] = t1;
      o[1] = t2;
    }
  }
}

// Instance-norm statistics from the per-tile partials of the conv epilogue.
// Image b covers tiles [b*hw/BM, ((b+1)*hw-1)/BM]; slot 0 of a tile belongs to
// the image of its first row, slot 1 to the next image.  Two deterministic
// levels: (1) block (image, 64-channel group, chunk of STAT_CHUNK tiles), 16
// tile-lanes x 64 channels, fixed-order LDS reduce -> fp64 chunk partials;
// (2) one thread per (image, channel) sums its chunks in order.
constexpr int STAT_CHUNK = 256;

__global__ __launch_bounds__(1024) void conv_stats_chunk(const float* __restrict__ part, int BM,
                                                         int hw, int C, int nchunk,
                                                         double* __restrict__ chunks) {
  const int b = blockIdx.z, cg = blockIdx.y, ch = blockIdx.x;
  const int c = cg * 64 + (threadIdx.x & 63), tl = threadIdx.x >> 6;  // 16 tile lanes
  const long long t0 = (long long)b * hw / BM, t1 = ((long long)(b + 1) * hw - 1) / BM;
  const long long ts = t0 + (long long)ch * STAT_CHUNK;
  const long long te = min(t1 + 1, ts + STAT_CHUNK);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    for (long long t = ts + tl; t < te; t += 16) {
      const int sl = (t * BM) / hw == b ? 0 : 1;
      const float* p = part + ((t * 2 + sl) * C + c) * 2;
      s1 += p[0];
      s2 += p[1];
    }
  }
  __shared__ double r1[16][64], r2[16][64];
  r1[tl][threadIdx.x & 63] = s1;
  r2[tl][threadIdx.x & 63] = s2;
  __syncthreads();
  if (tl == 0 && c < C) {
    double a1 = 0.0, a2 = 0.0;
    for (int k = 0; k < 16; ++k) {
      a1 += r1[k][threadIdx.x];
      a2 += r2[k][threadIdx.x];
    }
    double* o = chunks + (((long long)b * nchunk + ch) * C + c) * 2;
    o[0] = a1;
    o[1] = a2;
  }
}

__global__ void conv_stats_finalize(const double* __restrict__ chunks, int nchunk, int hw, int C,
                                    int nb, float eps, float* __restrict__ mean,
                                    float* __restrict__ rstd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * C) return;
  const int b = i / C, c = i - b * C;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const double* p = chunks + (((long long)b * nchunk + k) * C + c) * 2;
    s1 += p[0];
    s2 += p[1];
  }
  const double mu = s1 / hw;
  double var = s2 / hw - mu * mu;
  if (var < 0) var = 0;
  mean[i] = (float)mu;
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

// y = act(sum_s part[s] + bias + res), fixed split order (deterministic)
__global__ void conv_splitk_reduce(const float* __restrict__ part, int ks, int M, int C,
                                   const float* __restrict__ bias, const float* __restrict__ res,
                                   int rcs, int act, float* __restrict__ y, int ycs) {
  const int c4n = C / 4;
  const long long total = (long long)M * c4n;
  const size_t slab = (size_t)M * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % c4n);
    const long long m = i / c4n;
    f32x4 v = *reinterpret_cast<const f32x4*>(part + m * C + q * 4);
    for (int s = 1; s < ks; ++s) v += *reinterpret_cast<const f32x4*>(part + s * slab + m * C + q * 4);
    if (bias) v += *reinterpret_cast<const f32x4*>(bias + q * 4);
    if (res) {
      const float* rp = res + m * rcs + q * 4;
      v.x += rp[0];
      v.y += rp[1];
      v.z += rp[2];
      v.w += rp[3];
    }
    for (int k = 0; k < 4; ++k) {
      float t = v[k];
      if (act == POSFEAT_ACT_RELU) t = fmaxf(t, 0.f);
      else if (act == POSFEAT_ACT_ELU) t = pf_elu(t);
      y[m * ycs + q * 4 + k] = t;
    }
  }
}

template <int BM, int BN, int WM, int WN>
int launch_cfg(ConvArgs& a, bool cin32, hipStream_t st) {
  const int tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.nwg = tiles_m * a.tiles_n;
  dim3 grid(a.nwg * a.ksplit), block(WM * WN * 64);
  if (cin32)
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, true>), grid, block, 0, st, a);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, false>), grid, block, 0, st, a);
  PF_CHECK_LAUNCH();
  if (a.ksplit > 1) {
    const long long total = (long long)a.M * (a.Cout / 4);
    long long g = (total + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(conv_splitk_reduce, dim3((int)g), dim3(256), 0, st, a.part, a.ksplit, a.M,
                       a.Cout, a.bias, a.res, a.rcs, a.act, a.y, a.ycs);
    PF_CHECK_LAUNCH();
  }
  return POSFEAT_OK;
}

// Split-K factor for the 128x128 tile: only for deep K (>= 32 chunks) where
// the tile count leaves the last wave of workgroups badly underfilled.
int choose_ksplit(long long tiles, int nch) {
  const double slots = 256.0 * 2.0;  // CUs x resident 128x128 blocks
  if (nch < 64) return 1;
  int best = 1;
  double best_eff = 0.0;
  for (int ks = 1; ks <= 4; ++ks) {
    if (nch / ks < 32) break;
    const double r = tiles * ks / slots;
    const double eff = r / ceil(r) * (ks == 1 ? 1.0 : 0.97);  // ~3% for the reduce pass
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = ks;
    }
  }
  return best;
}

}  // namespace

extern "C" int posfeat_conv_packed_k(int cin, int kh, int kw) {
  const int cinp = (cin + 3) / 4 * 4;
  const int k = kh * kw * cinp;
  return (k + BK - 1) / BK * BK;
}

static int conv_prepare(const posfeat_conv_desc* d, const float* x, const float* w,
                        const float* bias, const float* res, float* y, ConvArgs& a) {
  if (!d || !x || !w || !y) return POSFEAT_E_INVALID;
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->cin <= 0 || d->cin % 4 || d->cout <= 0)
    return POSFEAT_E_INVALID;
  if (d->x_cstride < d->cin || d->x_cstride % 4 || d->y_cstride < d->cout) return POSFEAT_E_INVALID;
  if (d->kh <= 0 || d->kw <= 0 || d->stride <= 0 || d->pad < 0) return POSFEAT_E_INVALID;
  if (res && d->res_cstride < d->cout) return POSFEAT_E_INVALID;
  // 16-B vector epilogue: channel counts/strides multiple of 4, aligned bases
  if (d->cout % 4 || d->y_cstride % 4 || (res && d->res_cstride % 4)) return POSFEAT_E_INVALID;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(res) & 15) ||
      (reinterpret_cast<uintptr_t>(bias) & 15))
    return POSFEAT_E_INVALID;
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
  a.ksplit = 1;
  a.part = nullptr;
  a.stats = nullptr;
  a.hw = a.OH * a.OW;
  return POSFEAT_OK;
}

// Tile choice: the largest tile that still gives >= 2 workgroups per CU.
// 0: 128x128, 1: 128x64, 2: 64x64
static int conv_cfg(const ConvArgs& a) {
  const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
  const long long t128x64 = (long long)((a.M + 127) / 128) * ((a.Cout + 63) / 64);
  if (a.Cout > 64 && (t128 >= 512 || a.ksplit > 1)) return 0;
  if (t128x64 >= 512) return 1;
  return 2;
}

static int cfg_bm(int cfg) { return cfg == 2 ? 64 : 128; }

static int conv_launch(ConvArgs& a, hipStream_t st) {
  const bool cin32 = (a.Cin % BK) == 0;
  switch (conv_cfg(a)) {
    case 0: return launch_cfg<128, 128, 2, 2>(a, cin32, st);
    case 1: return launch_cfg<128, 64, 2, 2>(a, cin32, st);
    default: return launch_cfg<64, 64, 2, 2>(a, cin32, st);
  }
}

extern "C" int posfeat_conv2d_nhwc(const posfeat_conv_desc* d, const float* x, const float* w,
                                   const float* bias, const float* res, float* y, void* stream) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, res, y, a));
  return conv_launch(a, pf_stream(stream));
}

extern "C" size_t posfeat_conv2d_workspace(const posfeat_conv_desc* d) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
  if (a.Cout % 4 || a.Cout <= 64) return 0;
  const int ks = choose_ksplit(t128, a.Kpad / BK);
  return ks > 1 ? (size_t)ks * a.M * a.Cout * sizeof(float) : 0;
}

extern "C" int posfeat_conv2d_nhwc_ws(const posfeat_conv_desc* d, const float* x, const float* w,
                                      const float* bias, const float* res, float* y, void* ws,
                                      size_t ws_bytes, void* stream) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, res, y, a));
  const size_t need = posfeat_conv2d_workspace(d);
  if (need > 0 && ws && ws_bytes >= need) {
    const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
    a.ksplit = choose_ksplit(t128, a.Kpad / BK);
    a.part = static_cast<float*>(ws);
  }
  return conv_launch(a, pf_stream(stream));
}

extern "C" size_t posfeat_conv2d_stats_workspace(const posfeat_conv_desc* d) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  const int bm = cfg_bm(conv_cfg(a));
  if (a.hw < bm) return 0;  // a tile may span > 2 images: not supported
  const size_t tiles_m = (a.M + bm - 1) / bm;
  const size_t per_img = (size_t)(a.hw + bm - 1) / bm + 1;
  const size_t nchunk = (per_img + STAT_CHUNK - 1) / STAT_CHUNK;
  return pf_align(tiles_m * 2 * a.Cout * 2 * sizeof(float), 256) +
         (size_t)d->n * nchunk * a.Cout * 2 * sizeof(double);
}

extern "C" int posfeat_conv2d_nhwc_stats(const posfeat_conv_desc* d, const float* x,
                                         const float* w, const float* bias, float* y, void* ws,
                                         size_t ws_bytes, float* mean, float* rstd, float eps,
                                         void* stream) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, nullptr, y, a));
  const size_t need = posfeat_conv2d_stats_workspace(d);
  if (need == 0) return POSFEAT_E_UNSUPPORTED;
  if (!ws || ws_bytes < need || !mean || !rstd) return POSFEAT_E_WORKSPACE;
  a.stats = static_cast<float*>(ws);
  hipStream_t st = pf_stream(stream);
  const int bm = cfg_bm(conv_cfg(a));
  PF_TRY(conv_launch(a, st));
  const int nb = d->n;
  const size_t tiles_m = (a.M + bm - 1) / bm;
  const int per_img = (a.hw + bm - 1) / bm + 1;
  const int nchunk = (per_img + STAT_CHUNK - 1) / STAT_CHUNK;
  double* chunks = reinterpret_cast<double*>(static_cast<char*>(ws) +
                                             pf_align(tiles_m * 2 * a.Cout * 2 * sizeof(float), 256));
  hipLaunchKernelGGL(conv_stats_chunk, dim3(nchunk, (a.Cout + 63) / 64, nb), dim3(1024), 0, st,
                     a.stats, bm, a.hw, a.Cout, nchunk, chunks);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(conv_stats_finalize, dim3((nb * a.Cout + 255) / 256), dim3(256), 0, st,
                     chunks, nchunk, a.hw, a.Cout, nb, eps, mean, rstd);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
