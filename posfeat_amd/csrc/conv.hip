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
#include "fmap.h"

// Product arithmetic of the row-tile convs / GEMMs (posfeat_set_conv_precision):
// 0 fp32 MFMA (v_mfma_f32_32x32x2_f32), 1 bf16x6 on the bf16 matrix cores
// (default), 2 bf16x6 with producer-split operands for the Winograd / tap
// GEMMs (gemm6.hip; measured no faster, A/B only).  POSFEAT_BF6 sets the
// initial value.
static int g_conv_precision = -1;
int pf_conv_precision() {
  if (g_conv_precision < 0) {
    const char* e = pf_ab_getenv("POSFEAT_BF6");
    g_conv_precision = e ? (e[0] == '0' ? 0 : e[0] == '2' ? 2 : 1) : 1;
  }
  return g_conv_precision;
}

extern "C" int posfeat_set_conv_precision(int mode) {
  const int prev = pf_conv_precision();
  if (mode == -1) return prev;  // query
  if (mode < 0 || mode > 2) return -1;
  g_conv_precision = mode;
  return prev;
}

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
  double* bnpart;    // optional [tiles_m][2][Cout] per-tile fp64 (sum, sum of squares) of y
                     // over every image: train-mode BatchNorm statistics (pf_conv_run_tile_bn)
  int hw;            // OH*OW (image boundary inside a tile for `stats`)
  // conv_up4_kernel only: the low-res grid
  int lh, lw;
  // batched 1x1 GEMMs (conv_glds_kernel only): blockIdx.y selects x/w/y + z*stride
  int nbatch;
  long long bx, bw, by;
  // pre-split weights (conv_bf6b_kernel): three bf16 planes of w's layout
  const unsigned short* wb;
  long long wplane, bwb;
  const float* zero;  // a zeroed 16-B device word (pf_conv_zero16), read by masked DMA lanes
  // pre-split A (conv_bf6s_kernel): three bf16 planes of x's [M][xcs] layout,
  // plane stride xplane, batch stride bxb (elements)
  const unsigned short* xb;
  long long xplane, bxb;
  // two-source 1x1 GEMM (conv_bf6x_kernel AM = 3, pf_conv_dual): K chunks
  // [0, k1ch) read x at the output pixel (stride 1), chunks [k1ch, Kpad / BK)
  // read x2 at input pixel (n, oh * s2, ow * s2) of its H2 x W2 map
  const float* x2;
  int x2cs, k1ch, H2, W2, s2;
  // normalised A (conv_bf6x_kernel AM = 4, pf_conv_run_tile_np): each A value
  // of image n, channel c enters as PReLU((x - amean[n][c]) * arstd[n][c])
  // with slope *aslope -- instance norm + PReLU applied on load (in_apply's
  // arithmetic), the normalised map never written
  const float* amean;
  const float* arstd;
  const float* aslope;
  // also write y NCHW here ([n][Cout][OH*OW]; PfNchwSink): conv_epilogue_t
  float* ynchw;
};

// Epilogue shared by both kernels: acc -> LDS T[BM][BN+4] (conflict-free: a
// half-wave writes 32 consecutive floats of one row), then each thread owns a
// fixed 4-column group and walks rows: residual loads are all issued before
// use, stores are float4.  Optional fused instance-norm partials.  Requires
// the caller's K loop to have ended with a barrier (smem is reused).
// `rowm(row)` maps a tile row to its output pixel m (or -1: outside); img0 is
// the image of the tile's first row (stats slot 0).
// `resp(row, m)` returns the residual row (channels n0..) or nullptr.
// SL > 1: the tile is staged in SL row slices of BM / SL rows (the waves of one
// slice write, every thread stores, barrier, next slice), so T needs only
// BM / SL rows of LDS -- the pre-split GEMM tiles use SL = 2 to keep their LDS
// at the B ring's 48 KB (three blocks per CU instead of two).  Same values,
// same stores: bit-identical to SL = 1.
// conv_epilogue_t: the same with the staging of slice s into T (row pitch
// BN + 4, rows s * BM / SL ..) left to `stage(T, s)` -- the accumulator layout
// of the MFMA shape the kernel ran (conv_epilogue below: 32x32 blocks;
// conv_bf6x_kernel: 16x16 blocks).
// BNS: the BatchNorm partial-sum mode is compiled in (off for the bf6x tiles,
// which the train-mode step never runs: pf_conv_run_tile_bn falls back there)
template <int BM, int BN, int THREADS, int SL, bool BNS = true, class RowMap, class ResMap,
          class Stage>
__device__ __forceinline__ void conv_epilogue_t(const ConvArgs& a, float* smem, int tm, int n0,
                                                int split, RowMap rowm, int img0, ResMap resp,
                                                Stage&& stage) {
  constexpr int SR = BM / SL;  // rows per slice
  const int tid = threadIdx.x;
  constexpr int TP = BN + 4;
  float* T = smem;  // the K loop ended with a barrier: staging LDS is free
  constexpr int C4 = BN / 4;
  // rows per pass: THREADS / C4, rounded down to a power of two that divides
  // the slice (BN = 192: 48 quads, 4 rows per pass, threads 192.. idle)
  constexpr int RPP0 = THREADS / C4;
  constexpr int RPP = RPP0 >= 16 ? 16 : RPP0 >= 8 ? 8 : RPP0 >= 4 ? 4 : RPP0 >= 2 ? 2 : 1;
  // (every thread active when the quads divide a power-of-two block; six
  // waves with BN = 128: 12 rows per pass rounded to 8, a third idle)
  static_assert(RPP0 == RPP || THREADS % C4 != 0 || (THREADS & (THREADS - 1)) != 0,
                "every thread active when the quads divide");
  static_assert(SR % RPP == 0, "rows per pass divide the slice");
  constexpr int NP = SR / RPP;       // passes per slice
  const int q = tid % C4, r0 = tid / C4;
  const bool active = r0 < RPP;      // every thread when THREADS % C4 == 0
  const int col = n0 + 4 * q;
  const bool colok = active && col < a.Cout;
  const f32x4 bv = (a.ksplit <= 1 && a.bias && colok)
                       ? *reinterpret_cast<const f32x4*>(a.bias + col)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 s1[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, s2[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  double b1[4] = {0, 0, 0, 0}, b2[4] = {0, 0, 0, 0};  // a.bnpart: this thread's rows, in order
#pragma unroll
  for (int s = 0; s < SL; ++s) {
    if (s > 0) __syncthreads();  // the previous slice's rows are read
    stage(T, s);
    __syncthreads();
    if (a.ksplit > 1) {  // raw partial sums; conv_splitk_reduce finishes
      float* pp = a.part + (size_t)split * a.M * a.Cout;
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int row = r0 + p * RPP;
        const int m = rowm(s * SR + row);
        if (colok && m >= 0)
          *reinterpret_cast<f32x4*>(pp + (size_t)m * a.Cout + col) =
              *reinterpret_cast<const f32x4*>(T + row * TP + 4 * q);
      }
      continue;
    }
    f32x4 rv[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = s * SR + r0 + p * RPP;
      const int m = rowm(row);
      const float* rp = (colok && m >= 0) ? resp(row, m) : nullptr;
      rv[p] = rp ? *reinterpret_cast<const f32x4*>(rp + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int row = r0 + p * RPP;
      const int m = rowm(s * SR + row);
      if (!colok || m < 0) continue;
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
      if (BNS && a.bnpart) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          b1[k] += (double)v[k];
          b2[k] += (double)v[k] * (double)v[k];
        }
      }
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
    if (a.ynchw) {
      // the slice again, column-major: 4 consecutive rows (pixels) of one
      // column per float4 store into [n][Cout][hw]; the same bias + act
      // arithmetic as the NHWC store above (no residual on this path)
      // (lanes walk the pixels of one column: a wave stores 256-B runs)
      constexpr int R4 = SR / 4;           // 4-row groups in the slice
      for (int e = tid; e < R4 * BN; e += THREADS) {
        const int g4 = e % R4, cc = e / R4;
        const int colx = n0 + cc;
        if (colx >= a.Cout) continue;
        const float bcol = (a.ksplit <= 1 && a.bias) ? a.bias[colx] : 0.f;
        float o4[4];
        int mm[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int row = g4 * 4 + k;
          mm[k] = rowm(s * SR + row);
          float v = T[row * TP + cc] + bcol;
          if (a.act == POSFEAT_ACT_RELU) v = fmaxf(v, 0.f);
          else if (a.act == POSFEAT_ACT_ELU) v = pf_elu(v);
          o4[k] = v;
        }
        const int nimg = mm[0] >= 0 ? mm[0] / a.hw : -1, p0 = mm[0] - nimg * a.hw;
        if (nimg >= 0 && mm[3] == mm[0] + 3 && (p0 & 3) == 0 && p0 + 3 < a.hw) {
          *reinterpret_cast<f32x4*>(a.ynchw + ((size_t)nimg * a.Cout + colx) * a.hw + p0) =
              f32x4{o4[0], o4[1], o4[2], o4[3]};
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (mm[k] >= 0) {
              const int ni = mm[k] / a.hw;
              a.ynchw[((size_t)ni * a.Cout + colx) * a.hw + (mm[k] - ni * a.hw)] = o4[k];
            }
        }
      }
    }
  }
  if (a.ksplit > 1) return;
  if (BNS && a.bnpart) {  // the RPP row groups of each column summed in a fixed order (fp64)
    __syncthreads();
    double* R = reinterpret_cast<double*>(smem);  // [RPP][2][BN]: the IN path's 64 B / thread
    if (active) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        R[(r0 * 2 + 0) * BN + 4 * q + k] = b1[k];
        R[(r0 * 2 + 1) * BN + 4 * q + k] = b2[k];
      }
    }
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += THREADS) {
      const int which = e / BN, c = e - which * BN;
      if (n0 + c >= a.Cout) continue;
      double t = 0.0;
      for (int rr = 0; rr < RPP; ++rr) t += R[(rr * 2 + which) * BN + c];
      a.bnpart[((size_t)tm * 2 + which) * a.Cout + n0 + c] = t;
    }
  }
  if (a.stats) {  // reduce the RPP row groups of each column in a fixed order
    __syncthreads();
    float* R = smem;  // [RPP][2 slots][BN][2]
    if (active) {
#pragma unroll
      for (int sl = 0; sl < 2; ++sl)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          R[((r0 * 2 + sl) * BN + 4 * q + k) * 2 + 0] = s1[sl][k];
          R[((r0 * 2 + sl) * BN + 4 * q + k) * 2 + 1] = s2[sl][k];
        }
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

template <int BM, int BN, int WM, int WN, int SL = 1, class RowMap, class ResMap>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a,
                                              f32x16 (&acc)[BM / WM / 32][BN / WN / 32],
                                              float* smem, int tm, int n0, int split,
                                              RowMap rowm, int img0, ResMap resp) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 32, NI = TN / 32;
  static_assert(SL == 1 || (WN == 1 && WM % SL == 0), "row slices need whole waves");
  constexpr int SR = BM / SL, TP = BN + 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  conv_epilogue_t<BM, BN, WM * WN * 64, SL>(
      a, smem, tm, n0, split, rowm, img0, resp, [&](float* T, int s) {
        if (SL == 1 || wm * TM / SR == s) {
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                T[(wm * TM - s * SR + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * TP +
                  wn * TN + ni * 32 + (lane & 31)] = acc[mi][ni][r];
        }
      });
}

// bf16x6 helpers (described with the row tiles below)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// common.h: the compiler-visible conversion (an inline-asm one hid its VGPR
// write from the hazard recognizer: MFMAs read stale operands)
__device__ __forceinline__ unsigned cvt_pk_bf16(float lo, float hi) {
  return pf_cvt_pk_bf16(lo, hi);
}

// 8 fp32 (k order) -> the three bf16 fragments of one MFMA operand
__device__ __forceinline__ void split3(const f32x4& p0, const f32x4& p1, u32x4_t& h, u32x4_t& m,
                                       u32x4_t& l) {
  const float x[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    const unsigned hp = cvt_pk_bf16(a, b);
    const float ra = a - __uint_as_float(hp << 16), rb = b - __uint_as_float(hp & 0xffff0000u);
    const unsigned mp = cvt_pk_bf16(ra, rb);
    const float sa = ra - __uint_as_float(mp << 16), sb = rb - __uint_as_float(mp & 0xffff0000u);
    h[i] = hp;
    m[i] = mp;
    l[i] = cvt_pk_bf16(sa, sb);
  }
}

__device__ __forceinline__ f32x16 mfma_bf16(const u32x4_t& a, const u32x4_t& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16_bf16(const u32x4_t& a, const u32x4_t& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// BF6 (the Cin = 4 stem in bf16x6 mode): the products as six bf16 MFMAs per
// fp32 product (split3 / mfma_bf16 below, fp32-exact); the staging is the same.
template <int BM, int BN, int WM, int WN, bool CIN32, bool BF6 = false>
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
    if constexpr (BF6) {
      // lane (r, h) feeds k = 16 g + 8 h .. +7 of rows r: two 16-B reads per
      // operand row (36-float rows: the 16 rows of a ds_read_b128 lane group
      // start on distinct 4-bank quads, conflict-free)
      const float* Ab6 = As + (cur * BM + arow) * LDSP + 8 * (lane >> 5);
      const float* Bb6 = Bs + (cur * BN + brow) * LDSP + 8 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < BK / 16; ++g) {
        u32x4_t ah[MI], am[MI], al[MI], bh[NI], bm[NI], bl[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          split3(*reinterpret_cast<const f32x4*>(Ab6 + mi * 32 * LDSP + 16 * g),
                 *reinterpret_cast<const f32x4*>(Ab6 + mi * 32 * LDSP + 16 * g + 4), ah[mi],
                 am[mi], al[mi]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          split3(*reinterpret_cast<const f32x4*>(Bb6 + ni * 32 * LDSP + 16 * g),
                 *reinterpret_cast<const f32x4*>(Bb6 + ni * 32 * LDSP + 16 * g + 4), bh[ni],
                 bm[ni], bl[ni]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            f32x16 cc = acc[mi][ni];
            cc = mfma_bf16(ah[mi], bh[ni], cc);
            cc = mfma_bf16(ah[mi], bm[ni], cc);
            cc = mfma_bf16(am[mi], bh[ni], cc);
            cc = mfma_bf16(ah[mi], bl[ni], cc);
            cc = mfma_bf16(al[mi], bh[ni], cc);
            cc = mfma_bf16(am[mi], bm[ni], cc);
            acc[mi][ni] = cc;
          }
      }
      if (c + 1 < nch) store_chunk(cur ^ 1);
      __syncthreads();
      continue;
    }
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

  conv_epilogue<BM, BN, WM, WN>(
      a, acc, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; },
      m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}

// ---------------------------------------------------------------------------
// Direct-to-LDS variant for Cin % 32 == 0 (every deep layer).  The register-
// staged loop above spends ~18% of the head.conv2 time on staging (global
// loads into VGPRs + ds_write_b128, whose VGPR->LDS transfer competes with the
// MFMA issue; ablation in DESIGN.md).  Here each lane issues
// global_load_lds_dwordx4: one wave-instruction fills 8 LDS rows of 128 B
// (one 32-channel chunk of 8 pixels / 8 couts) with no VGPR round trip.
// LDS rows carry no padding (the DMA destination is lane-linear), so bank
// conflicts on the MFMA operand reads are removed by an XOR swizzle: 16-B slot
// s of row r is stored at slot s ^ ((r >> 1) & 7) -- distinct banks for every
// 16-lane group of ds_read_b128.  The swizzle is applied on the per-lane
// global SOURCE address (LDS image stays lane-linear) and undone on the read.
// Zero padding (out-of-image taps, M / Cout tails) loads from a zeroed
// 16-B device word.  Two LDS stages: chunk c+1 is in flight while chunk c is
// multiplied; vmcnt(0) + barrier at the end of each chunk.
// 64 floats (not just the one 16-B word the DMA lanes read): conv_bf6d_kernel's
// masked A rows read 4 DISTINCT 16-B words of it, so the compiler cannot merge
// them into one load plus register copies (which it did, behind a vmcnt(0))
__device__ __attribute__((aligned(16))) float pf_conv_zero16[64];
#define PF_GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define PF_LPTR(p) ((__attribute__((address_space(3))) void*)(p))

// sched_barrier mask: every instruction class except vector memory (0x10 and
// its read / write sub-classes 0x20 / 0x40) may be scheduled across
#define PF_SCHED_NO_VMEM 0x78F
// sched_barrier mask that lets VALU, SALU, DS and transcendental instructions
// cross but pins vector-memory instructions AND MFMAs in program order
// (conv_bf6x_kernel's interleaving)
#define PF_SCHED_PIN_VMEM_MFMA 0x786

// vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 s_waitcnt encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// ... and every LDS access of this wave completed: the K loops' barriers
// then never overtake one of the wave's own fragment reads, whatever the
// relative latency of the LDS and of the DMA that refills the stage after
// the barrier (tools/isa_check.py fails an s_barrier crossed with LDS
// accesses outstanding)
template <int N>
__device__ __forceinline__ void wait_vmcnt_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
}

// ---- fp32-exact products on the bf16 matrix cores ("bf16x6") -------------
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the rate of the fp32-input MFMA
// (32 cycles for 32x32x16 vs 64 for 32x32x2).  Each fp32 operand is split
// exactly into three bf16 terms, x = h + m + l (h = RNE_bf16(x), m =
// RNE_bf16(x - h), l = RNE_bf16(x - h - m); both differences are exact in
// fp32), |x - h - m - l| <= 2^-27 |x|.  The product keeps the six terms of
// order >= 2^-16: a b ~ hh + hm + mh + hl + lh + mm, dropping ml + lm + ll
// (<= 3 * 2^-27 |ab|).  Every partial product of two bf16 values is exact in
// the fp32 accumulator, so the per-product error (~2e-8 relative) is below an
// fp32 fmaf's own rounding (2^-24 = 6e-8): the result is fp32-accurate, not a
// reduced-precision approximation, at 6 x 32 = 192 matrix-core cycles per
// 32x32x16 step instead of 8 x 64 = 512.  The split runs on the VALU beside
// the MFMAs (v_cvt_pk_bf16_f32, RNE).  Accumulation order is fixed (k, then
// the six terms in the order above): deterministic, tile-size independent.

// One step of an LDS-DMA pipeline: the next chunk's DMA into LDS through
// (d0, d1), then the MFMA work reading LDS through (s0, s1).  The four are
// __restrict__ so that, once inlined, the LDS reads carry alias scopes
// disjoint from the DMA's and the waitcnt pass lets the DMA fly under the
// multiply; without them it conservatively waits vmcnt(0) before the first
// read (ISA r5j: DMA and MFMA serialised in every ring kernel here).  Valid
// because the bytes a step's DMA writes (the stage being refilled) are never
// read in that step -- the pointers may share a base, the accessed stages
// are disjoint.
template <class P0, class P1, class Q0, class Q1, class Issue, class Compute>
__device__ __forceinline__ void pf_dma_overlap_step(P0* __restrict__ d0, P1* __restrict__ d1,
                                                    const Q0* __restrict__ s0,
                                                    const Q1* __restrict__ s1, bool issue,
                                                    Issue&& issue_to, Compute&& compute_from) {
  if (issue) issue_to(d0, d1);
  compute_from(s0, s1);
}

// The refilled stage and the multiplied stage of a step whose DMAs are
// interleaved with its LDS reads (conv_bf6x_kernel): both as __restrict__
// parameters of one body, for the same reason as pf_dma_overlap_step.
template <class F>
__device__ __forceinline__ void pf_dma_interleave(unsigned short* __restrict__ d,
                                                  const unsigned short* __restrict__ s, F&& body) {
  body(d, s);
}

// NST = 2: two LDS stages, vmcnt(0) + barrier per chunk (the DMA of chunk c+1
// overlaps chunk c).  NST = 3: a three-stage ring -- chunks c+1 and c+2 are
// in flight while c is multiplied; each chunk waits only for its own DMA
// (counted vmcnt) and one raw s_barrier (no fence, so the younger chunk's
// DMA stays in flight across it).  96 KB of LDS at 128x128: one block per CU.
// BF6: the products on the bf16 matrix cores (split3 / mfma_bf16 above).
template <int BM, int BN, int WM, int WN, int NST = 2, bool BF6 = false>
__global__ __launch_bounds__(WM* WN * 64) void conv_glds_kernel(ConvArgs a) {
  constexpr int THREADS = WM * WN * 64;
  constexpr int NW = THREADS / 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int A_G = BM / 8 / NW;  // DMA wave-instructions per chunk for A
  constexpr int B_G = BN / 8 / NW;
  static_assert(A_G >= 1 && B_G >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile");
  static_assert(MI >= 1 && NI >= 1, "wave tile must be >= 32x32");
  static_assert(NST >= 2 && NST <= 5, "stages");
  constexpr int RING = NST * (BM + BN) * BK;
  constexpr int STAGE = BM * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > STAGE ? RING : STAGE];
  float* As = smem;                  // [NST][BM][BK] swizzled
  float* Bs = smem + NST * BM * BK;  // [NST][BN][BK] swizzled

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR: scalar DMA targets
  const int wm = wave / WN, wn = wave % WN;

  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  if (a.nbatch > 1) {  // batched GEMMs (Winograd): one operand set per blockIdx.y
    const long long zb = blockIdx.y;
    a.x += zb * a.bx;
    a.w += zb * a.bw;
    a.y += zb * a.by;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-lane DMA sources (fixed across K) -------------------------------
  // instruction i of this wave fills rows [(wave*G + i)*8, +8); lane L -> row
  // +(L>>3), LDS slot L&7, which holds source k-slot (L&7) ^ ((row>>1)&7)
  // dense 1x1 convs without padding: rows past M / Cout read the last valid
  // row (never stored) instead of a per-DMA zero select (see conv_bf6b_kernel)
  const bool dense = a.KH == 1 && a.KW == 1 && a.pad == 0;
  const float* zero = a.zero;
  const int lrow = lane >> 3;
  const float* xsrc[A_G];
  unsigned tapok[A_G];  // bit t: tap t of this pixel is inside the image
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int row = (wave * A_G + i) * 8 + lrow;
    const int sslot = (lane & 7) ^ ((row >> 1) & 7);
    const int m = dense ? min(m0 + row, a.M - 1) : m0 + row;
    tapok[i] = 0u;
    xsrc[i] = a.x;
    if (m < a.M) {
      const int n = m / a.hw;
      const int rem = m - n * a.hw;
      const int oh = rem / a.OW;
      const int ow = rem - oh * a.OW;
      const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
            tapok[i] |= 1u << (kh * a.KW + kw);
      // base of tap (0,0); taps add a uniform offset (may point outside the
      // image for masked taps: never dereferenced)
      xsrc[i] = a.x + (long long)n * a.H * a.W * a.xcs + ((long long)ih0 * a.W + iw0) * a.xcs +
                sslot * 4;
    }
  }
  const float* wsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int row = (wave * B_G + i) * 8 + lrow;
    const int sslot = (lane & 7) ^ ((row >> 1) & 7);
    wsrc[i] = a.w + (size_t)min(n0 + row, a.Cout - 1) * a.Kpad + sslot * 4;
  }

  const int ntap = a.KH * a.KW;
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);

  // issue the DMA of the next chunk (chunks go out in order: (slab, tap, kh,
  // kw) advance incrementally, no per-chunk division) into stage `buf`
  int nx_slab = ch0 / ntap, nx_tap = ch0 - nx_slab * ntap;
  int nx_kh = nx_tap / a.KW, nx_kw = nx_tap - nx_kh * a.KW;
  long long nx_b = (long long)ch0 * BK;
  auto issue_chunk = [&](float* Ad, float* Bd, int buf) {
    const long long delta = ((long long)nx_kh * a.W + nx_kw) * a.xcs + nx_slab * BK;
    if (dense) {
#pragma unroll
      for (int i = 0; i < A_G; ++i)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(xsrc[i] + delta),
            (__attribute__((address_space(3))) void*)(Ad + (buf * BM + (wave * A_G + i) * 8) * BK),
            16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < A_G; ++i) {
        const float* src = ((tapok[i] >> nx_tap) & 1u) ? xsrc[i] + delta : zero;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)src,
            (__attribute__((address_space(3))) void*)(Ad + (buf * BM + (wave * A_G + i) * 8) * BK),
            16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(wsrc[i] + nx_b),
          (__attribute__((address_space(3))) void*)(Bd + (buf * BN + (wave * B_G + i) * 8) * BK),
          16, 0, 0);
    nx_b += BK;
    ++nx_tap;
    if (++nx_kw == a.KW) {
      nx_kw = 0;
      if (++nx_kh == a.KH) {
        nx_kh = 0;
        nx_tap = 0;
        ++nx_slab;
      }
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // operand reads: row R = 32-aligned base + (lane & 31), k-slot (lane>>5) + 2kk
  const int sw = ((lane & 31) >> 1) & 7;
  const int arow = wm * TM + (lane & 31);
  const int brow = wn * TN + (lane & 31);
  int kofs[BK / 8];
#pragma unroll
  for (int kk = 0; kk < BK / 8; ++kk) kofs[kk] = (((lane >> 5) + 2 * kk) ^ sw) * 4;

  auto compute = [&](const float* Ar, const float* Br, int slot) {
    const float* Ab = Ar + (slot * BM + arow) * BK;
    const float* Bb = Br + (slot * BN + brow) * BK;
    if constexpr (BF6) {
      // k16 group g: lane half h holds k = 16g + 8h + j, i.e. k-slots 4g+2h, 4g+2h+1
#pragma unroll
      for (int g = 0; g < BK / 16; ++g) {
        const int s0 = ((4 * g + 2 * (lane >> 5)) ^ sw) * 4;
        const int s1 = ((4 * g + 2 * (lane >> 5) + 1) ^ sw) * 4;
        u32x4_t ah[MI], am[MI], al[MI], bh[NI], bm[NI], bl[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          split3(*reinterpret_cast<const f32x4*>(Ab + mi * 32 * BK + s0),
                 *reinterpret_cast<const f32x4*>(Ab + mi * 32 * BK + s1), ah[mi], am[mi], al[mi]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          split3(*reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + s0),
                 *reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + s1), bh[ni], bm[ni], bl[ni]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            f32x16 c = acc[mi][ni];
            c = mfma_bf16(ah[mi], bh[ni], c);
            c = mfma_bf16(ah[mi], bm[ni], c);
            c = mfma_bf16(am[mi], bh[ni], c);
            c = mfma_bf16(ah[mi], bl[ni], c);
            c = mfma_bf16(al[mi], bh[ni], c);
            c = mfma_bf16(am[mi], bm[ni], c);
            acc[mi][ni] = c;
          }
      }
      return;
    }
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      f32x4 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const f32x4*>(Ab + mi * 32 * BK + kofs[kk]);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + kofs[kk]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][j], bv[ni][j], acc[mi][ni],
                                                                0, 0, 0);
    }
  };

  if constexpr (NST == 2) {
    if (ch0 < ch1) issue_chunk(As, Bs, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): the DMA has landed (this wave)
    __syncthreads();
    for (int c = ch0; c < ch1; ++c) {
      const int cur = (c - ch0) & 1;
      pf_dma_overlap_step(
          As + (cur ^ 1) * BM * BK, Bs + (cur ^ 1) * BN * BK, As + cur * BM * BK,
          Bs + cur * BN * BK, c + 1 < ch1,
          [&](float* Ad, float* Bd) { issue_chunk(Ad, Bd, 0); },
          [&](const float* Ar, const float* Br) { compute(Ar, Br, 0); });
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
    }
  } else {
    // NST-stage ring: chunks i+1 .. i+NST-2 are in flight while i is
    // multiplied; each chunk waits only for its own DMA (counted vmcnt) and
    // one raw s_barrier (no fence: the younger chunks' DMAs stay in flight)
    const int nch = ch1 - ch0;
    for (int j = 0; j < NST - 1 && j < nch; ++j) issue_chunk(As, Bs, j);
    int slot = 0;
    for (int i = 0; i < nch; ++i) {
      const int ahead = min(NST - 2, nch - 1 - i);  // younger chunks already issued
      if (ahead >= 3)
        wait_vmcnt<(NST >= 5 ? 3 : 0) * (A_G + B_G)>();
      else if (ahead == 2)
        wait_vmcnt<(NST >= 4 ? 2 : 0) * (A_G + B_G)>();
      else if (ahead == 1)
        wait_vmcnt<A_G + B_G>();
      else
        wait_vmcnt<0>();
      // every wave: chunk i landed, and chunk i-1 (the slot refilled below) consumed
      __builtin_amdgcn_s_barrier();
      const int refill = slot == 0 ? NST - 1 : slot - 1;
      pf_dma_overlap_step(
          As + refill * BM * BK, Bs + refill * BN * BK, As + slot * BM * BK, Bs + slot * BN * BK,
          i + NST - 1 < nch, [&](float* Ad, float* Bd) { issue_chunk(Ad, Bd, 0); },
          [&](const float* Ar, const float* Br) { compute(Ar, Br, 0); });
      slot = slot == NST - 1 ? 0 : slot + 1;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  conv_epilogue<BM, BN, WM, WN>(
      a, acc, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; },
      m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}

// ---------------------------------------------------------------------------
// bf16x6 with PRE-SPLIT weights (the engine's forward path): B = the packed
// weights as three bf16 planes of the same [Cout][Kpad] layout (a.wb, plane
// stride a.wplane; split once per forward), A = the activations split in
// registers.  The split VALU work bounds the both-operands form (split3 of
// every A and B fragment per wave; PMC: matrix pipe ~33 % busy, issue-bound
// with the LDS-DMA pieces).  Here the 4 waves stack along M (wave tile
// 32 x BN): ONE A fragment is split per k16 step against NI = BN/32 B
// fragments read ready-made -- 1/4 of the split work per MFMA of the 2x2
// layout.  LDS stage: A fp32 [BM][32] (swizzled as conv_glds_kernel) + B
// [3 planes][BN][32] bf16 (16-B slot s of row r holding k-slot
// s ^ ((r >> 2) & 3): conflict-free ds_read_b128).  Two stages; at
// BM = BN = 128 that is 80 KB, two blocks per CU.  Products and their order
// are those of the BF6 tiles: results are bit-identical to them.
// amdgpu_waves_per_eu(2): the accumulators move from AGPRs to VGPRs within
// the 256-register budget of two waves per SIMD (same box, r5y: +0.6 %)
template <int BM, int BN, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2)))
void conv_bf6b_kernel(ConvArgs a) {
  constexpr int WM = NWV, WN = 1, NW = NWV;
  constexpr int TM = BM / WM, TN = BN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int A_G = BM / 8 / NW;
  constexpr int B_G = 3 * BN / 16 / NW;  // 16 plane-rows (64 B) per DMA piece
  static_assert(MI == 1 && A_G >= 1 && B_G >= 1 && (3 * BN / 16) % NW == 0, "tile");
  constexpr int ASTAGE = BM * BK;         // floats
  constexpr int BSTAGE = 3 * BN * BK / 2; // floats (u16 pairs)
  constexpr int RING = 2 * (ASTAGE + BSTAGE);
  constexpr int EPI = BM * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > EPI ? RING : EPI];
  float* As = smem;
  unsigned short* Bs = reinterpret_cast<unsigned short*>(smem + 2 * ASTAGE);

  // wave index as an SGPR value: the DMA's LDS targets (M0) stay scalar math
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave;
  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const unsigned short* wb = a.wb;
  if (a.nbatch > 1) {
    const long long zb = blockIdx.y;
    a.x += zb * a.bx;
    a.y += zb * a.by;
    wb += zb * a.bwb;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // dense: a 1x1 conv without padding (every Winograd / tap GEMM, every 1x1
  // layer) has no zero taps; rows past M / Cout read the last valid row
  // instead (the epilogue never stores them), so a chunk's DMA addresses are
  // the lane's fixed pointer + one uniform offset: no per-DMA select
  const bool dense = a.KH == 1 && a.KW == 1 && a.pad == 0;
  const float* zero = a.zero;
  const int lrow = lane >> 3;
  const float* xsrc[A_G];
  unsigned tapok[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int row = (wave * A_G + i) * 8 + lrow;
    const int sslot = (lane & 7) ^ ((row >> 1) & 7);
    const int m = dense ? min(m0 + row, a.M - 1) : m0 + row;
    tapok[i] = 0u;
    xsrc[i] = a.x;
    if (m < a.M) {
      const int n = m / a.hw;
      const int rem = m - n * a.hw;
      const int oh = rem / a.OW;
      const int ow = rem - oh * a.OW;
      const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
            tapok[i] |= 1u << (kh * a.KW + kw);
      xsrc[i] = a.x + (long long)n * a.H * a.W * a.xcs + ((long long)ih0 * a.W + iw0) * a.xcs +
                sslot * 4;
    }
  }
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = wb + plane * a.wplane + (long long)min(n0 + row, a.Cout - 1) * a.Kpad + ks * 8;
  }
  const int ntap = a.KH * a.KW;
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);

  // chunks are issued in order: (slab, tap, kh, kw) of the next one advance
  // incrementally (one division per workgroup, none per chunk)
  int nx_slab = ch0 / ntap, nx_tap = ch0 - nx_slab * ntap;
  int nx_kh = nx_tap / a.KW, nx_kw = nx_tap - nx_kh * a.KW;
  long long nx_b = (long long)ch0 * BK;
  // the next chunk's DMA into stage (dA, dB)
  auto issue_to = [&](float* dA, unsigned short* dB) {
    const long long delta = ((long long)nx_kh * a.W + nx_kw) * a.xcs + nx_slab * BK;
    if (dense) {  // wave-uniform branch
#pragma unroll
      for (int i = 0; i < A_G; ++i)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(xsrc[i] + delta),
            (__attribute__((address_space(3))) void*)(dA + (wave * A_G + i) * 8 * BK), 16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < A_G; ++i) {
        const float* src = ((tapok[i] >> nx_tap) & 1u) ? xsrc[i] + delta : zero;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)src,
            (__attribute__((address_space(3))) void*)(dA + (wave * A_G + i) * 8 * BK), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[i] + nx_b),
          (__attribute__((address_space(3))) void*)(dB + (wave * B_G + i) * 16 * BK), 16, 0, 0);
    nx_b += BK;
    ++nx_tap;
    if (++nx_kw == a.KW) {
      nx_kw = 0;
      if (++nx_kh == a.KH) {
        nx_kh = 0;
        nx_tap = 0;
        ++nx_slab;
      }
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][ni][r] = 0.f;

  const int sw = ((lane & 31) >> 1) & 7, hh = lane >> 5, r32 = lane & 31;
  const int arow = wm * TM + r32;
  auto compute_from = [&](const float* sA, const unsigned short* sB) {
    const float* Ab = sA + arow * BK;
    const unsigned short* Bb = sB;
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      const int s0 = ((4 * g + 2 * hh) ^ sw) * 4, s1 = ((4 * g + 2 * hh + 1) ^ sw) * 4;
      u32x4_t ah, am, al;
      split3(*reinterpret_cast<const f32x4*>(Ab + s0), *reinterpret_cast<const f32x4*>(Ab + s1),
             ah, am, al);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int row = ni * 32 + r32;
        const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
        const unsigned short* bp = Bb + row * BK + slot * 8;
        const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
        const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
        const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
        f32x16 c = acc[0][ni];
        c = mfma_bf16(ah, bh, c);
        c = mfma_bf16(ah, bm, c);
        c = mfma_bf16(am, bh, c);
        c = mfma_bf16(ah, bl, c);
        c = mfma_bf16(al, bh, c);
        c = mfma_bf16(am, bm, c);
        acc[0][ni] = c;
      }
    }
  };

  // Stage s: A at As + s * ASTAGE, B at Bs + 2 * s * BSTAGE.  Each step
  // issues chunk c+1's DMA into one stage and multiplies chunk c out of the
  // other through pf_dma_overlap_step's __restrict__ parameters: the compiler
  // then knows the stage being read is not the one the DMA writes and does
  // not put a vmcnt(0) before the reads (it did -- ISA r5j: DMA and MFMA
  // fully serialised, the "no overlap" of the r3c ablations)
  float* const A0 = As;
  float* const A1 = As + ASTAGE;
  unsigned short* const B0 = Bs;
  unsigned short* const B1 = Bs + 2 * BSTAGE;
  if (ch0 < ch1) issue_to(A0, B0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int c = ch0; c < ch1; ++c) {
    const bool more = c + 1 < ch1;
    if (((c - ch0) & 1) == 0)
      pf_dma_overlap_step(A1, B1, A0, B0, more, issue_to, compute_from);
    else
      pf_dma_overlap_step(A0, B0, A1, B1, more, issue_to, compute_from);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  conv_epilogue<BM, BN, WM, WN>(
      a, acc, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; },
      m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}

// ---------------------------------------------------------------------------
// Pre-split-weight GEMM / conv tiles with a DEEP A prefetch (conv_bf6d_kernel,
// POSFEAT_BF6D = D; any KH x KW / stride / pad with Cin % 32 == 0).  The LDS ring of conv_bf6b_kernel bounds the bytes
// in flight per CU (two 40-KB stages per block, half of them being read): with
// HBM latencies of several thousand cycles under load the next chunk often
// lands after the current one is multiplied.  Here A (the streaming operand,
// V / activations) goes straight to registers D chunks ahead (16 VGPRs per
// chunk per lane), and only the weight planes (L2-resident) use a two-stage
// LDS ring.  Per chunk: wait for B(c) (the A loads issued after it stay in
// flight), barrier, DMA B(c+1), split A(c), load A(c+D) into the freed
// registers, 48 MFMAs.  Same products in the same order as bf6b: bit-identical.
// The default for the pre-split tiles (bf6d_depth below: D = 2).
template <int BM, int BN, int D, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2)))
void conv_bf6d_kernel(ConvArgs a) {
  constexpr int WM = NWV, WN = 1, NW = NWV;
  constexpr int TM = BM / WM, TN = BN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int B_G = 3 * BN / 16 / NW;
  static_assert(MI == 1 && B_G >= 1 && (3 * BN / 16) % NW == 0 && D >= 2 && D <= 4, "tile");
  constexpr int BSTAGE = 3 * BN * BK / 2;  // floats (u16 pairs)
  constexpr int RING = 2 * BSTAGE;
  // the epilogue stages the tile in SL row slices so it fits in the ring's LDS
  constexpr int SL = BM * (BN + 4) <= RING ? 1 : BM / 2 * (BN + 4) <= RING ? 2 : 4;
  static_assert(WM % SL == 0, "epilogue slices");
  constexpr int EPI = BM / SL * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > EPI ? RING : EPI];
  unsigned short* const Bs = reinterpret_cast<unsigned short*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const unsigned short* wb = a.wb;
  if (a.nbatch > 1) {
    const long long zb = blockIdx.y;
    a.x += zb * a.bx;
    a.y += zb * a.by;
    wb += zb * a.bwb;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r32 = lane & 31, hh = lane >> 5;
  // the lane's A row (base of tap (0,0) + its k offset 8h) and the taps that
  // fall inside the image; rows past M read zeros (never stored)
  const float* xrow = a.x;
  unsigned tapok = 0u;
  {
    const int m = m0 + wave * 32 + r32;
    if (m < a.M) {
      const int n = m / a.hw, rem = m - n * a.hw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih0 + kh) < (unsigned)a.H && (unsigned)(iw0 + kw) < (unsigned)a.W)
            tapok |= 1u << (kh * a.KW + kw);
      xrow = a.x + (long long)n * a.H * a.W * a.xcs + ((long long)ih0 * a.W + iw0) * a.xcs + hh * 8;
    }
  }
  const int ntap = a.KH * a.KW;
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = wb + plane * a.wplane + (long long)min(n0 + row, a.Cout - 1) * a.Kpad + ks * 8;
  }
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);
  const int nch = ch1 - ch0;

  auto issue_b = [&](unsigned short* Bd, int c) {
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)c * BK),
          (__attribute__((address_space(3))) void*)(Bd + (wave * B_G + i) * 16 * BK), 16, 0, 0);
  };
  // A chunk = (slab, tap): always four loads per lane, so the per-chunk vmcnt
  // accounting below holds.  A masked lane (tap outside the image, row past
  // M) selects the zero block as its base and reads the same four offsets
  // from it: one per-lane pointer select, four distinct addresses.  (Selecting
  // the one zero word per load let the compiler branch on the mask and merge
  // the masked lanes' identical loads into one load + register copies behind
  // an s_waitcnt vmcnt(0) -- a full drain of the prefetch -- and a wave with
  // every lane masked issued 3 loads, not 4.)  The chunk to load next is
  // tracked incrementally (no per-chunk divisions) and clamped at the last
  // chunk: EVERY step issues one B DMA and four A loads (past the end they
  // re-read the last chunk, an L2 hit, never used), so every path through the
  // loop has the same vector-memory count -- the compiler's own waits for the
  // A registers then stay counted instead of falling back to vmcnt(0) where
  // paths with and without loads met.
  const float* const zero = a.zero;
  int la_c = ch0, la_slab = ch0 / ntap, la_tap = ch0 - (ch0 / ntap) * ntap;
  int la_kh = la_tap / a.KW, la_kw = la_tap - (la_tap / a.KW) * a.KW;
  auto load_a_next = [&](f32x4 (&v)[4]) {
    const bool ok = (tapok >> la_tap) & 1u;
    const float* p = xrow + ((long long)la_kh * a.W + la_kw) * a.xcs + (long long)la_slab * BK;
    const float* base = ok ? p : zero;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = *reinterpret_cast<const f32x4*>(base + (j >> 1) * 16 + (j & 1) * 4);
    if (la_c + 1 < ch1) {  // uniform
      ++la_c;
      ++la_tap;
      if (++la_kw == a.KW) {
        la_kw = 0;
        if (++la_kh == a.KH) {
          la_kh = 0;
          la_tap = 0;
          ++la_slab;
        }
      }
    }
  };

  f32x16 acc[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ni][r] = 0.f;

  // The counted waits below (vmcnt(4) / vmcnt(4 D)) assume every B DMA is
  // issued BEFORE the A loads that follow it in program order: vmcnt retires
  // in issue order, so B(c) is covered only if exactly the A loads issued
  // after it are younger.  The A loads read memory the DMA does not write, so
  // the scheduler could legally hoist them above the DMA; sched barriers pin
  // the order of the vector-memory instructions (mask PF_SCHED_NO_VMEM: ALU,
  // MFMA and LDS instructions may still move across).  tools/isa_check.py
  // checks the built ISA.
  // Prologue: A(0) .. A(D-2), then B(0), then A(D-1): B(0) too has exactly
  // four younger loads, so every step waits vmcnt(4) (one loop body, no
  // first-step special case for the compiler to peel).
  f32x4 va[D][4];
  if (nch > 0) {  // (every plan gives each split >= 1 chunk; no load past the slice)
#pragma unroll
    for (int j = 0; j < D - 1; ++j) load_a_next(va[j]);
    __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
    issue_b(Bs, ch0);
    __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
    load_a_next(va[D - 1]);
  }

  for (int i = 0; i < nch; i += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int ii = i + u;
      // B(ii) landed (and with it every older load, A(ii) included): it was
      // issued right before the 4 A loads of the previous step / the prologue
      __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
      wait_vmcnt_lgkm0<4>();
      __builtin_amdgcn_s_barrier();
      const int s = ii & 1;
      // split this chunk's A (frees va[u] for chunk ii + D)
      u32x4_t ah[2], am[2], al[2];
#pragma unroll
      for (int g = 0; g < 2; ++g) split3(va[u][2 * g], va[u][2 * g + 1], ah[g], am[g], al[g]);
      pf_dma_overlap_step(
          Bs + (s ^ 1) * 2 * BSTAGE, Bs + (s ^ 1) * 2 * BSTAGE + BSTAGE, Bs + s * 2 * BSTAGE,
          Bs + s * 2 * BSTAGE + BSTAGE, true,
          [&](unsigned short* Bd, unsigned short*) {
            issue_b(Bd, min(ch0 + ii + 1, ch1 - 1));
            __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);  // B(ii+1) strictly before A(ii+D)
            load_a_next(va[u]);
          },
          [&](const unsigned short* Bb, const unsigned short*) {
            if (ii >= nch) return;  // the tail of the last D-group: loads only
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
              for (int ni = 0; ni < NI; ++ni) {
                const int row = ni * 32 + r32;
                const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
                const unsigned short* bp = Bb + row * BK + slot * 8;
                const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
                const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
                const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
                f32x16 c = acc[ni];
                c = mfma_bf16(ah[g], bh, c);
                c = mfma_bf16(ah[g], bm, c);
                c = mfma_bf16(am[g], bh, c);
                c = mfma_bf16(ah[g], bl, c);
                c = mfma_bf16(al[g], bh, c);
                c = mfma_bf16(am[g], bm, c);
                acc[ni] = c;
              }
          });
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  f32x16 accm[1][NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) accm[0][ni] = acc[ni];
  conv_epilogue<BM, BN, WM, WN, SL>(
      a, accm, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; },
      m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}

// ---------------------------------------------------------------------------
// conv_bf6d_kernel with A PRE-SPLIT by its producer (conv_bf6s_kernel, conv
// precision mode 2): A arrives as three bf16 planes (h, m, l of split3, the
// Winograd input transform / head.conv1's output writing them), so the MFMA
// loop does no conversion at all -- per lane and chunk six 16-B loads (two
// k16 groups x three planes) that ARE the MFMA operands.  Dense GEMMs only
// (the Winograd transform-domain GEMMs and the tap GEMM: 1x1, no padding;
// rows past M re-read the last row, never stored).  The same h, m, l values
// and the same product order as the in-kernel split: bit-identical to
// conv_bf6d / conv_bf6b.  Same B ring, waits (now vmcnt(6): six A loads per
// chunk) and epilogue as conv_bf6d_kernel.
template <int BM, int BN, int D, int NWV = 4>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2)))
void conv_bf6s_kernel(ConvArgs a) {
  constexpr int WM = NWV, WN = 1, NW = NWV;
  constexpr int TM = BM / WM, TN = BN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int B_G = 3 * BN / 16 / NW;
  static_assert(MI == 1 && B_G >= 1 && (3 * BN / 16) % NW == 0 && D >= 2 && D <= 3, "tile");
  constexpr int BSTAGE = 3 * BN * BK / 2;  // floats (u16 pairs)
  constexpr int RING = 2 * BSTAGE;
  // the epilogue stages the tile in SL row slices so it fits in the ring's LDS
  constexpr int SL = BM * (BN + 4) <= RING ? 1 : BM / 2 * (BN + 4) <= RING ? 2 : 4;
  static_assert(WM % SL == 0, "epilogue slices");
  constexpr int EPI = BM / SL * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > EPI ? RING : EPI];
  unsigned short* const Bs = reinterpret_cast<unsigned short*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const unsigned short* wb = a.wb;
  const unsigned short* xb = a.xb;
  if (a.nbatch > 1) {
    const long long zb = blockIdx.y;
    xb += zb * a.bxb;
    a.y += zb * a.by;
    wb += zb * a.bwb;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r32 = lane & 31, hh = lane >> 5;
  const unsigned short* xrow =
      xb + (long long)min(m0 + wave * 32 + r32, a.M - 1) * a.xcs + hh * 8;
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = wb + plane * a.wplane + (long long)min(n0 + row, a.Cout - 1) * a.Kpad + ks * 8;
  }
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);
  const int nch = ch1 - ch0;

  auto issue_b = [&](unsigned short* Bd, int c) {
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)c * BK),
          (__attribute__((address_space(3))) void*)(Bd + (wave * B_G + i) * 16 * BK), 16, 0, 0);
  };
  // six loads per chunk: k16 group g, plane p (h, m, l); clamped at the last
  // chunk so every step issues the same count (see conv_bf6d_kernel)
  const long long xpl = a.xplane;
  int la_c = ch0;
  auto load_a_next = [&](u32x4_t (&v)[6]) {
    const unsigned short* p = xrow + (long long)la_c * BK;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      v[j] = *reinterpret_cast<const u32x4_t*>(p + (j % 3) * xpl + (j / 3) * 16);
    if (la_c + 1 < ch1) ++la_c;
  };

  f32x16 acc[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ni][r] = 0.f;

  u32x4_t va[D][6];
  if (nch > 0) {
#pragma unroll
    for (int j = 0; j < D - 1; ++j) load_a_next(va[j]);
    __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
    issue_b(Bs, ch0);
    __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
    load_a_next(va[D - 1]);
  }

  for (int i = 0; i < nch; i += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int ii = i + u;
      __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
      wait_vmcnt_lgkm0<6>();  // B(ii) and everything older (A(ii) included) landed
      __builtin_amdgcn_s_barrier();
      const int s = ii & 1;
      const u32x4_t ah0 = va[u][0], am0 = va[u][1], al0 = va[u][2];
      const u32x4_t ah1 = va[u][3], am1 = va[u][4], al1 = va[u][5];
      pf_dma_overlap_step(
          Bs + (s ^ 1) * 2 * BSTAGE, Bs + (s ^ 1) * 2 * BSTAGE + BSTAGE, Bs + s * 2 * BSTAGE,
          Bs + s * 2 * BSTAGE + BSTAGE, true,
          [&](unsigned short* Bd, unsigned short*) {
            issue_b(Bd, min(ch0 + ii + 1, ch1 - 1));
            __builtin_amdgcn_sched_barrier(PF_SCHED_NO_VMEM);
            load_a_next(va[u]);
            // the loads go out before this chunk's MFMAs (left to itself the
            // scheduler put the MFMAs first: a chunk less prefetch lead)
            __builtin_amdgcn_sched_barrier(0);
          },
          [&](const unsigned short* Bb, const unsigned short*) {
            if (ii >= nch) return;
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
              for (int ni = 0; ni < NI; ++ni) {
                const u32x4_t ah = g ? ah1 : ah0, am = g ? am1 : am0, al = g ? al1 : al0;
                const int row = ni * 32 + r32;
                const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
                const unsigned short* bp = Bb + row * BK + slot * 8;
                const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
                const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
                const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
                f32x16 c = acc[ni];
                c = mfma_bf16(ah, bh, c);
                c = mfma_bf16(ah, bm, c);
                c = mfma_bf16(am, bh, c);
                c = mfma_bf16(ah, bl, c);
                c = mfma_bf16(al, bh, c);
                c = mfma_bf16(am, bm, c);
                acc[ni] = c;
              }
          });
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  f32x16 accm[1][NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) accm[0][ni] = acc[ni];
  conv_epilogue<BM, BN, WM, WN, SL>(
      a, accm, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; },
      m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}


// ---------------------------------------------------------------------------
// Dense pre-split-weight GEMM tiles on v_mfma_f32_16x16x32_bf16 with the
// memory instructions interleaved among the MFMAs (conv_bf6x_kernel, the
// default for the dense GEMMs: the Winograd transform-domain GEMMs and the
// 1x1 convs / tap GEMM with no padding).  Measured on the upconv2 / iconv2
// GEMM shape (tools/probe/gemm_probe.hip): the bf6d structure spends its
// memory time and its MFMA time one after the other -- a chunk's six B DMAs
// and four A loads go out in one burst after the barrier, the MFMAs follow --
// so the loop runs at about the sum of a memory-only loop (0.74 ms) and an
// MFMA-only loop (1.4 ms).  Here one memory instruction follows each group of
// twelve MFMAs (pinned by sched barriers), so the DMA / load issue and the
// returns overlap the matrix pipe, and the 16x16x32 shape holds a higher clock
// under load than 32x32x16 (MI355X_MICROARCH.md "DVFS give-back" 7).
// Strided 1x1 convs (the encoder's downsample layers) too: output row m reads
// input pixel (n, s oh, s ow).
// Tile BM = 64 RB x BN (64 or 128), four waves stacked along M, each 16 RB
// rows = RB 16-row blocks x BN / 16 column blocks; one MFMA covers a 32-wide k
// chunk.  RB = 4 (TILE_BF6X_256x128) halves the B traffic per MFMA; per
// output element the MFMA sequence is the same, so RB = 2 and 4 are
// bit-identical (autotune candidates of each other).
// A (fp32 rows, pitch xcs) goes global -> registers one chunk ahead (lane l:
// row l & 15 of its block, k (l >> 4) * 8 .. + 7 -- sixteen 128-B rows per
// load instruction), split in registers (split3); B (three bf16 planes) by
// LDS DMA into a two-stage ring (the bf6d layout and swizzle).  Each step
// waits vmcnt(0): the chunk's loads were issued a whole step earlier, in the
// first part of the previous step's MFMA sequence.  Rows past M re-read the
// last row (never stored).  Products: the same six bf16 terms as bf6d, but
// the 16x16x32 instruction sums 32 products per step where 32x32x16 sums 16,
// so results are NOT bit-identical to the 32x32 tiles (fp32-exact products,
// different fp32 accumulation grouping); the GEMMs that use it use only it.
// 16-B slot swizzle of the B stage rows for the 16x16x32 reads: lane l reads
// row (l & 15) of a 16-row block at logical slot l >> 4; with physical slot =
// logical ^ g((row >> 2) & 3), g = (0, 2, 3, 1), the 16 lanes of each
// ds_read_b128 lane group (MI355X_MICROARCH.md LDS table) hit 16 distinct
// 4-bank groups (the bf6d swizzle g = identity left them 2-way conflicted)
__device__ __forceinline__ int bx_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// AM: the A (pixel-row) operand -- 0 dense rows (1x1 convs, GEMMs), 1 G4:
// 4-channel input taps (the stem), 2 GT: 32-channel slab x tap chunks (3x3 /
// strided convs with Cin % 32 == 0, the packed K order (cin/32, kh, kw, cin%32)),
// 3 DU: dense rows from two maps (a bottleneck's conv3 + its downsample as one
// GEMM, ConvArgs x2)
// NW: waves stacked along M (4; 6 for TILE_BF6X_192x128)
template <int BN, int RB = 2, int AM = 0, int NW = 4>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2)))
void conv_bf6x_kernel(ConvArgs a) {
  constexpr bool G4 = AM == 1, GT = AM == 2, DU = AM == 3, NP = AM == 4;
  constexpr int BM = NW * RB * 16, NB = BN / 16;
  constexpr int NPK = 256;  // NP: K <= NPK (the tap GEMM: 192)
  constexpr int B_G = 3 * BN / 16 / NW;  // B DMA instructions per wave per chunk
  constexpr int NA = 2 * RB;             // A loads per lane per chunk
  constexpr int NOPS = B_G + NA;
  static_assert((3 * BN / 16) % NW == 0 && NOPS <= 3 * NB && (RB == 2 || RB == 4), "tile");
  constexpr int BSTAGE = 3 * BN * BK / 2;  // floats (u16 pairs)
  constexpr int RING = 2 * BSTAGE;
  // epilogue row slices: whole waves per slice, the slice within the B ring
  constexpr int WR = RB * 16;  // rows per wave
  constexpr int SL = BM * (BN + 4) <= RING                                  ? 1
                     : (BM / 2) % WR == 0 && BM / 2 * (BN + 4) <= RING     ? 2
                     : BM % 3 == 0 && (BM / 3) % WR == 0 && BM / 3 * (BN + 4) <= RING ? 3
                                                                            : 4;
  static_assert(BM % SL == 0 && (BM / SL) % WR == 0 && BM / SL * (BN + 4) <= RING, "slices");
  constexpr int EPI = BM / SL * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > EPI ? RING : EPI];
  // NP: mean / rstd of the (at most two) images of the tile's rows, [2][2][NPK]
  __shared__ __attribute__((aligned(16))) float anp[NP ? 4 * NPK : 4];
  unsigned short* const Bs = reinterpret_cast<unsigned short*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const unsigned short* wb = a.wb;
  if (a.nbatch > 1) {
    const long long zb = blockIdx.y;
    a.x += zb * a.bx;
    a.y += zb * a.by;
    wb += zb * a.bwb;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r16 = lane & 15, kq = lane >> 4;
  int npo[NP ? RB : 1];  // NP: this lane's rows' parameter offsets in anp
  float slope = 0.f;
  if (NP) {
    const int img0 = m0 / a.hw, img1 = min(m0 + BM - 1, a.M - 1) / a.hw;
    for (int e = tid; e < 4 * NPK; e += NW * 64) {
      const int im = e / (2 * NPK), which = (e / NPK) & 1, c = e % NPK;
      const float* src = which ? a.arstd : a.amean;
      anp[e] = c < a.Kpad ? src[(long long)(im ? img1 : img0) * a.Kpad + c] : 0.f;
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const int m = min(m0 + wave * RB * 16 + rb * 16 + r16, a.M - 1);
      npo[rb] = (m / a.hw == img0 ? 0 : 2 * NPK) + kq * 8;
    }
    slope = *a.aslope;
  }
  const float* xrow[RB];
  const float* xrow2[DU ? RB : 1];  // DU: the row in x2
  int ih0[RB], iw0[RB];  // G4: the row's top-left input tap
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int m = min(m0 + wave * RB * 16 + rb * 16 + r16, a.M - 1);
    if (DU) {
      const int n = m / a.hw, rem = m - n * a.hw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      xrow2[rb] = a.x2 + (((long long)n * a.H2 + oh * a.s2) * a.W2 + ow * a.s2) * a.x2cs + kq * 8;
    }
    long long pix = m;  // stride 1: output row m is input pixel m
    if (a.stride != 1 || G4 || GT) {
      const int n = m / a.hw, rem = m - n * a.hw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      pix = ((long long)n * a.H + oh * a.stride) * a.W + ow * a.stride;
      if (G4 || GT) {
        ih0[rb] = oh * a.stride - a.pad;
        iw0[rb] = ow * a.stride - a.pad;
        pix = (long long)n * a.H * a.W;  // the image's base
      }
    }
    xrow[rb] = a.x + pix * a.xcs + (G4 ? 0 : kq * 8);
  }
  // G4 (4-channel input, K order (kh, kw, c4)): load jj of a lane is tap
  // t = 8 chunk + 2 kq + jj, tracked as (kh, kw) and advanced by 8 taps per
  // chunk (KW in [5, 8]: one conditional wrap); outside the image or past the
  // last tap the lane reads the zeroed 16-B word
  // GT: chunk = (slab, tap), tracked as (slab, kh, kw) and advanced by one
  // tap per chunk; a tap outside the image reads the zeroed word
  int tkh[2] = {0, 0}, tkw[2] = {0, 0};
  int g_slab = 0, g_kh = 0, g_kw = 0;
  auto a_ptr = [&](int rb, int jj, int chunk) -> const float* {
    if (GT) {
      const int ih = ih0[rb] + g_kh, iw = iw0[rb] + g_kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      return ok ? xrow[rb] + ((long long)ih * a.W + iw) * a.xcs + g_slab * BK + jj * 4 : a.zero;
    }
    if (DU)  // uniform: every lane is at the same chunk
      return chunk < a.k1ch ? xrow[rb] + (long long)chunk * BK + jj * 4
                            : xrow2[rb] + (long long)(chunk - a.k1ch) * BK + jj * 4;
    if (!G4) return xrow[rb] + (long long)chunk * BK + jj * 4;
    const int ih = ih0[rb] + tkh[jj], iw = iw0[rb] + tkw[jj];
    const bool ok = tkh[jj] < a.KH && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    return ok ? xrow[rb] + ((long long)ih * a.W + iw) * 4 : a.zero;
  };
  auto advance_taps = [&]() {
    if (GT) {
      if (++g_kw == a.KW) {
        g_kw = 0;
        if (++g_kh == a.KH) {
          g_kh = 0;
          ++g_slab;
        }
      }
      return;
    }
    if (!G4) return;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      tkw[jj] += 8 - a.KW;
      tkh[jj] += 1;
      if (tkw[jj] >= a.KW) {
        tkw[jj] -= a.KW;
        tkh[jj] += 1;
      }
    }
  };
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ bx_swz(row);
    bsrc[i] = wb + plane * a.wplane + (long long)min(n0 + row, a.Cout - 1) * a.Kpad + ks * 8;
  }
  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);
  const int nch = ch1 - ch0;

  f32x4 acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 va[RB][2];
  int la_c = ch0;  // chunk of the next A loads (clamped at the last: same count every step)
  if (G4) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int t = ch0 * 8 + kq * 2 + jj;
      tkh[jj] = t / a.KW;
      tkw[jj] = t - tkh[jj] * a.KW;
    }
  }
  if (GT) {
    const int ntap = a.KH * a.KW, tap = ch0 % ntap;
    g_slab = ch0 / ntap;
    g_kh = tap / a.KW;
    g_kw = tap - g_kh * a.KW;
  }
  if (nch > 0) {
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)ch0 * BK),
          (__attribute__((address_space(3))) void*)(Bs + (wave * B_G + i) * 16 * BK), 16, 0, 0);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int j = 0; j < 2; ++j) va[rb][j] = *reinterpret_cast<const f32x4*>(a_ptr(rb, j, ch0));
    if (la_c + 1 < ch1) {
      ++la_c;
      advance_taps();
    }
  }
  for (int ii = 0; ii < nch; ++ii) {
    __builtin_amdgcn_s_waitcnt(0);  // (vmcnt 0; lgkm too) B(ii) and A(ii) landed
    __builtin_amdgcn_s_barrier();   // every wave's B(ii) part landed; stage s^1 free
    const int s = ii & 1;
    u32x4_t ah[RB], am[RB], al[RB];
    if (NP) {  // in_apply's arithmetic: (x - mean) * rstd, then PReLU
      const int cb0 = (ch0 + ii) * BK;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const float* pp = anp + npo[rb] + cb0 + jj * 4;
          const f32x4 mu = *reinterpret_cast<const f32x4*>(pp);
          const f32x4 rs = *reinterpret_cast<const f32x4*>(pp + NPK);
          f32x4 v = (va[rb][jj] - mu) * rs;
          v.x = v.x > 0.f ? v.x : slope * v.x;
          v.y = v.y > 0.f ? v.y : slope * v.y;
          v.z = v.z > 0.f ? v.z : slope * v.z;
          v.w = v.w > 0.f ? v.w : slope * v.w;
          va[rb][jj] = v;
        }
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) split3(va[rb][0], va[rb][1], ah[rb], am[rb], al[rb]);
    const int cb = min(ch0 + ii + 1, ch1 - 1);  // next B chunk (the last one re-read at the end)
    pf_dma_interleave(
        Bs + (s ^ 1) * 2 * BSTAGE, Bs + s * 2 * BSTAGE,
        [&](unsigned short* __restrict__ Bd, const unsigned short* __restrict__ Bb) {
          int op = 0;
          auto mem = [&]() {  // the op-th memory instruction of this step, pinned in place
            __builtin_amdgcn_sched_barrier(PF_SCHED_PIN_VMEM_MFMA);
            if (op < B_G) {
              __builtin_amdgcn_global_load_lds(
                  (const __attribute__((address_space(1))) void*)(bsrc[op] + (long long)cb * BK),
                  (__attribute__((address_space(3))) void*)(Bd + (wave * B_G + op) * 16 * BK), 16,
                  0, 0);
            } else if (op < NOPS) {
              const int j = op - B_G, rb = j >> 1, jj = j & 1;
              va[rb][jj] = *reinterpret_cast<const f32x4*>(a_ptr(rb, jj, la_c));
            }
            __builtin_amdgcn_sched_barrier(PF_SCHED_PIN_VMEM_MFMA);
            ++op;
          };
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            const int row = nb * 16 + r16;
            const int slot = kq ^ bx_swz(row);
            const unsigned short* bp = Bb + row * BK + slot * 8;
            const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
            const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
            const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
              f32x4 c = acc[rb][nb];
              c = mfma16_bf16(ah[rb], bh, c);
              c = mfma16_bf16(ah[rb], bm, c);
              c = mfma16_bf16(am[rb], bh, c);
              c = mfma16_bf16(ah[rb], bl, c);
              c = mfma16_bf16(al[rb], bh, c);
              c = mfma16_bf16(am[rb], bm, c);
              acc[rb][nb] = c;
            }
            // memory instructions spread evenly over the NB column blocks
            while (op < (nb + 1) * NOPS / NB) mem();
          }
        });
    if (la_c + 1 < ch1) {
      ++la_c;
      advance_taps();
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  conv_epilogue_t<BM, BN, NW * 64, SL, false>(
      a, smem, tm, n0, split, [&](int row) { return m0 + row < a.M ? m0 + row : -1; }, m0 / a.hw,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; },
      [&](float* T, int sl) {
        constexpr int SR = BM / SL;
        if (SL == 1 || wave * RB * 16 / SR == sl) {
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int nb = 0; nb < NB; ++nb)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                T[(wave * RB * 16 - sl * SR + rb * 16 + kq * 4 + r) * (BN + 4) + nb * 16 + r16] =
                    acc[rb][nb][r];
        }
      });
}

// ---------------------------------------------------------------------------
// Weight-stationary GEMM (head.conv2's tap GEMM [M x 192] x [192 x 1152],
// and the short-K 1x1 convs): in conv_bf6x_kernel every 128-row M tile
// re-reads its 128 x K weight planes (147 KB at K = 192, 6 B per weight) from
// L2 -- 1.5 K / BM of the output bytes, the largest operand stream of a
// short-K GEMM.  Here a persistent block keeps its BN output columns' planes
// resident in LDS (loaded once, in the bf6x stage layout and swizzle) and
// walks M tiles of 32 NW rows (A straight to registers one chunk ahead,
// split3, the same six bf16 MFMA terms per 16x16x32 step and the same k order
// as conv_bf6x_kernel: the same sums); the accumulators are stored straight
// from the registers, through the conv epilogue's order where there is one.
// Block b (after the XCD remap): column tile b % (N / BN), M tiles
// b / (N / BN) + i * per_n.
struct WsArgs {
  const float* x;
  const unsigned short* wb;
  float* y;
  long long wplane;
  int lda, ldc, M, N, per_n;
  int abl;  // A/B build, POSFEAT_TAPWS_ABL: 1 no stores, 2 no A loads (timing ablations, wrong
            // results), 4 the plain block -> tile order
  // epilogue (the 1x1 convs): y = act(acc + bias (+ res)), conv_bf6x_kernel's order
  const float* bias;
  const float* res;
  int rcs, act;
  int kpad;  // the weights' row pitch (<= 32 KC: chunks past it are zero)
  // AM = 1 (G4, the stem): 4-channel NHWC input H x W, output OW wide, ohw
  // pixels per image, stride / pad; taps outside the image read `zero`
  int H, W, OW, ohw, stride, pad;
  const float* zero;
  // batched (grid.y GEMMs): element strides of A, C and the B planes
  long long bx, by, bwb;
};

// PD: A prefetch distance in chunks (PD + 1 register buffers); NW waves (2 or
// 3 per SIMD: the block holds the CU's LDS), 32 rows each; KC k chunks of 32
// (K = 32 KC, the weights' row pitch); NB column blocks of 16 (BN = 16 NB)
// EP: the epilogue -- 0 the accumulators stored as they are (the tap GEMM), 1
// bias + activation, 2 bias + residual + activation
// AM: the A rows -- 0 dense (pitch lda), 1 G4: the 7x7 taps of a 4-channel
// image (K order (kh, kw, c4), conv_bf6x_kernel's G4 gather: a lane's load jj
// of chunk c is tap 8 c + 2 kq + jj)
template <int PD, int NW, int KC, int NB, int EP = 0, int AM = 0>
__global__ __launch_bounds__(NW * 64) void gemm_ws_kernel(WsArgs a) {
  constexpr bool RES = EP == 2, G4 = AM == 1;
  constexpr int G4K = 7;  // the stem's kernel size
  constexpr int NBUF = PD + 1, WS_NW = NW, WS_BM = NW * 32, WS_NCH = KC, WS_K = KC * BK;
  constexpr int WS_BN = 16 * NB;
  static_assert(WS_NCH % NBUF == 0 && PD >= 1 && PD < WS_NCH, "a tile starts at buffer 0");
  static_assert(WS_NCH * 3 * WS_BN * BK * 2 <= 160 * 1024, "resident weight planes");
  __shared__ __attribute__((aligned(16))) unsigned short Bres[WS_NCH * 3 * WS_BN * BK];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = a.N / WS_BN;
  if (gridDim.y > 1) {  // GEMM blockIdx.y of a batch
    a.x += blockIdx.y * a.bx;
    a.y += blockIdx.y * a.by;
    a.wb += blockIdx.y * a.bwb;
  }
  // (j, tn) pairs p = j * ntn + tn in contiguous runs per XCD (block b runs on
  // XCD b % 8): the ntn blocks that walk the same M tiles share an L2 for A
  int p = blockIdx.x;
  if (!(a.abl & 4)) {  // (A/B: POSFEAT_TAPWS_ABL=4 -- p = block index)
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, xcd = p & 7, slot = p >> 3;
    p = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tn = p % ntn, j = p / ntn;
  const int n0 = tn * WS_BN;
  const int ntm = (a.M + WS_BM - 1) / WS_BM;
  if (j >= ntm) return;  // block-uniform, before the only barrier
  // the block's weight planes, resident: [chunk][plane][row][BK], 16-B slot s
  // of row r at s ^ bx_swz(r) (conv_bf6x_kernel's stage layout)
  for (int e = tid; e < WS_NCH * 3 * WS_BN * 4; e += WS_NW * 64) {
    const int sl = e & 3, row = (e >> 2) % WS_BN, cp = (e >> 2) / WS_BN;
    const int c = cp / 3, pl = cp - c * 3;
    const int k = c * BK + sl * 8;
    const u32x4_t v = k < a.kpad ? *reinterpret_cast<const u32x4_t*>(
                                       a.wb + pl * a.wplane + (long long)(n0 + row) * a.kpad + k)
                                 : u32x4_t{0u, 0u, 0u, 0u};
    *reinterpret_cast<u32x4_t*>(Bres + (cp * WS_BN + row) * BK + (sl ^ bx_swz(row)) * 8) = v;
  }
  pf_syncthreads();
  const int r16 = lane & 15, kq = lane >> 4;
  struct Row {
    const float* p;  // dense: the row (+ this lane's k offset); G4: the image
    int ih0, iw0;    // G4: the output pixel's top-left tap
  };
  auto rowp = [&](int mt, int rb) -> Row {
    const int m = min(mt * WS_BM + wave * 32 + rb * 16 + r16, a.M - 1);
    if constexpr (G4) {
      const int n = m / a.ohw, rem = m - n * a.ohw, oh = rem / a.OW, ow = rem - oh * a.OW;
      return Row{a.x + (long long)n * a.H * a.W * 4, oh * a.stride - a.pad, ow * a.stride - a.pad};
    } else {
      return Row{a.x + (long long)m * a.lda + kq * 8, 0, 0};
    }
  };
  // load jj of chunk cc of row r
  auto aptr = [&](const Row& r, int cc, int jj) -> const float* {
    if constexpr (G4) {
      const int t = 8 * cc + 2 * kq + jj, kh = t / G4K, kw = t - kh * G4K;
      const int ih = r.ih0 + kh, iw = r.iw0 + kw;
      const bool ok = kh < G4K && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      return ok ? r.p + ((long long)ih * a.W + iw) * 4 : a.zero;
    } else {
      return r.p + cc * BK + jj * 4;
    }
  };
  int mt = j;
  Row xr[2] = {rowp(mt, 0), rowp(mt, 1)};
  f32x4 va[NBUF][2][2];  // [buffer][rb][jj]: chunk g of the block's walk in buffer g % NBUF
#pragma unroll
  for (int c = 0; c < PD; ++c)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        va[c][rb][jj] = *reinterpret_cast<const f32x4*>(aptr(xr[rb], c, jj));
  for (;;) {
    f32x4 acc[2][NB];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nmt = mt + a.per_n;
    const bool more = nmt < ntm;
    // opaque per tile: with one chunk group (K = 64) the B fragment reads are
    // loop-invariant, and hoisting all of them out of the tile loop spills
    int boff = 0;
    if constexpr (KC == 2) asm volatile("" : "+s"(boff));
    const Row xn[2] = {rowp(more ? nmt : mt, 0), rowp(more ? nmt : mt, 1)};
    // one chunk: split buffer `cur`, load chunk c + PD (this tile's, else the
    // next tile's) into buffer (cur + PD) % NBUF, 6 RB NB MFMAs
    auto step = [&](int c, auto cur_t) __attribute__((always_inline)) {
      constexpr int cur = decltype(cur_t)::value, nxt = (cur + PD) % NBUF;
      u32x4_t ah[2], am[2], al[2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) split3(va[cur][rb][0], va[cur][rb][1], ah[rb], am[rb], al[rb]);
      const int cl = c + PD;
      if (a.abl & 2) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) va[nxt][rb][jj] = va[cur][rb][jj];
      } else if (cl < WS_NCH || more) {
        const int cc = cl < WS_NCH ? cl : cl - WS_NCH;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const Row& src = cl < WS_NCH ? xr[rb] : xn[rb];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            va[nxt][rb][jj] = *reinterpret_cast<const f32x4*>(aptr(src, cc, jj));
        }
      }
      const unsigned short* Bc = Bres + boff + c * 3 * WS_BN * BK;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int row = nb * 16 + r16;
        const unsigned short* bp = Bc + row * BK + (kq ^ bx_swz(row)) * 8;
        const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
        const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + WS_BN * BK);
        const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * WS_BN * BK);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          f32x4 cc = acc[rb][nb];
          cc = mfma16_bf16(ah[rb], bh, cc);
          cc = mfma16_bf16(ah[rb], bm, cc);
          cc = mfma16_bf16(am[rb], bh, cc);
          cc = mfma16_bf16(ah[rb], bl, cc);
          cc = mfma16_bf16(al[rb], bh, cc);
          cc = mfma16_bf16(am[rb], bm, cc);
          acc[rb][nb] = cc;
        }
      }
    };
#pragma unroll 1
    for (int c = 0; c < WS_NCH; c += NBUF) {
      step(c, std::integral_constant<int, 0>{});
      if constexpr (KC == 2) __builtin_amdgcn_sched_barrier(0);
      step(c + 1, std::integral_constant<int, 1 % NBUF>{});
      if constexpr (NBUF > 2) step(c + 2, std::integral_constant<int, 2 % NBUF>{});
    }
    static_assert(NBUF <= 3, "step group");
    float bcol[NB];  // this lane's columns' biases (loaded here: no registers held over the k loop)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bcol[nb] = EP && a.bias ? a.bias[n0 + nb * 16 + r16] : 0.f;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      if (a.abl & 1) break;
      const int mb = mt * WS_BM + wave * 32 + rb * 16 + kq * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (mb + i >= a.M) continue;
        float* yr = a.y + (long long)(mb + i) * a.ldc + n0 + r16;
        // the row's residual loaded together, ahead of its stores (which the
        // compiler may not move loads past): one round trip per row, not NB
        float rv[NB];
        if constexpr (RES) {
          const float* rr = a.res + (long long)(mb + i) * a.rcs + n0 + r16;
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) rv[nb] = __builtin_nontemporal_load(rr + nb * 16);
        }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          float v = acc[rb][nb][i];
          if constexpr (EP > 0) {
            v += bcol[nb];
            if constexpr (RES) v += rv[nb];
            if (a.act == POSFEAT_ACT_RELU) v = fmaxf(v, 0.f);
            else if (a.act == POSFEAT_ACT_ELU) v = pf_elu(v);
          }
          yr[nb * 16] = v;
        }
      }
    }
    if (!more) break;
    mt = nmt;
    xr[0] = xn[0];
    xr[1] = xn[1];
  }
}

// ---------------------------------------------------------------------------
// Spatial-halo variant for stride-1 convs with Cin % 32 == 0 (every 3x3
// decoder/head layer).  The M tile is a PH x 16 patch of output pixels of one
// image; for each 32-channel slab its (PH+KH-1) x (16+KW-1) input halo is
// DMA'd into LDS ONCE and all KH*KW taps read it at shifted rows, so the A
// staging per slab drops from KH*KW*BM pixel rows to the halo (180 vs 1152
// for 8x16, 3x3).  B (weights) is staged per (slab, tap) chunk as above.
// LDS halo row hp = hy*(16+KW-1) + hx holds 128 B (32 channels) with 16-B slot
// s stored at s ^ ((hx >> 1) & 7): the 16 lanes of a ds_read_b128 group cover
// 16 consecutive output columns, i.e. 16 distinct hx mod 16 for every tap
// shift -> conflict-free.  Next slab's halo and next chunk's weights are in
// flight while the current chunk is multiplied (two LDS stages each).
// BF6: the products as bf16x6 (both operands split in registers, see split3)
template <int PH, int BN, int WM, int WN, int KH, int KW, bool BF6 = false>
__global__ __launch_bounds__(WM* WN * 64) __attribute__((amdgpu_waves_per_eu(2)))
void conv_halo_kernel(ConvArgs a) {
  constexpr int PW = 16;
  constexpr int BM = PH * PW;
  constexpr int THREADS = WM * WN * 64;
  constexpr int NW = THREADS / 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int NTAP = KH * KW;
  constexpr int HX = PW + KW - 1, HY = PH + KH - 1, HP = HX * HY;
  constexpr int A_G = (HP + 8 * NW - 1) / (8 * NW);  // halo DMA instructions per wave
  constexpr int HPR = A_G * 8 * NW;                  // LDS halo rows (>= HP)
  constexpr int B_G = BN / 8 / NW;
  static_assert(TM % 32 == 0 && MI >= 1 && NI >= 1 && B_G >= 1 && BN % (8 * NW) == 0, "tile");
  constexpr int RING = 2 * (HPR + BN) * BK;
  constexpr int STAGE = BM * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > STAGE ? RING : STAGE];
  float* As = smem;                 // [2][HPR][BK] halo, swizzled by hx
  float* Bs = smem + 2 * HPR * BK;  // [2][BN][BK] swizzled by row

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  int bid = blockIdx.x % a.nwg;
  const int split = blockIdx.x / a.nwg;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int n0 = tn * BN;
  const int ptx = (a.OW + PW - 1) / PW, ppi = ptx * ((a.OH + PH - 1) / PH);
  const int img = tm / ppi, prem = tm - img * ppi;
  const int oy0 = (prem / ptx) * PH, ox0 = (prem - (prem / ptx) * ptx) * PW;

  // ---- per-lane halo DMA sources (slab 0) ----------------------------------
  const int lrow = lane >> 3;
  const float* hsrc[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int hp = (wave * A_G + i) * 8 + lrow;
    const int hy = hp / HX, hx = hp - (hp / HX) * HX;
    const int ih = oy0 - a.pad + hy, iw = ox0 - a.pad + hx;
    const int sslot = (lane & 7) ^ ((hx >> 1) & 7);
    hsrc[i] = (hp < HP && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                  ? a.x + (((long long)img * a.H + ih) * a.W + iw) * a.xcs + sslot * 4
                  : nullptr;
  }
  const float* wsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int row = (wave * B_G + i) * 8 + lrow;
    const int sslot = (lane & 7) ^ ((row >> 1) & 7);
    wsrc[i] = (n0 + row < a.Cout) ? a.w + (size_t)(n0 + row) * a.Kpad + sslot * 4 : nullptr;
  }
  auto issue_halo = [&](float* Ad, int slab, int buf) {
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const float* src = hsrc[i] ? hsrc[i] + slab * BK : pf_conv_zero16;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(Ad + (buf * HPR + (wave * A_G + i) * 8) * BK),
          16, 0, 0);
    }
  };
  auto issue_w = [&](float* Bd, int c, int buf) {
#pragma unroll
    for (int i = 0; i < B_G; ++i) {
      const float* src = wsrc[i] ? wsrc[i] + (size_t)c * BK : pf_conv_zero16;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(Bd + (buf * BN + (wave * B_G + i) * 8) * BK),
          16, 0, 0);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // operand rows: tile row R = wm*TM + mi*32 + (lane&31) -> patch (R>>4, R&15)
  const int px = lane & 15;
  const int hrow0 = ((wm * TM + (lane & 31)) >> 4) * HX + px;  // tap (0,0), mi = 0
  const int brow = wn * TN + (lane & 31);
  const int bsw = ((lane & 31) >> 1) & 7;

  const int nch_all = a.Kpad / BK;
  const int ch0 = (int)((long long)nch_all * split / a.ksplit);
  const int ch1 = (int)((long long)nch_all * (split + 1) / a.ksplit);
  int slab = ch0 / NTAP, tap = ch0 - slab * NTAP;
  issue_halo(As, slab, 0);
  issue_w(Bs, ch0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  int abuf = 0;
  for (int c = ch0; c < ch1; ++c) {
    const int bcur = (c - ch0) & 1;
    const int kh = tap / KW, kw = tap - (tap / KW) * KW;
    const int hsw = ((px + kw) >> 1) & 7;
    pf_dma_overlap_step(As + (abuf ^ 1) * HPR * BK, Bs + (bcur ^ 1) * BN * BK,
                        As + abuf * HPR * BK, Bs + bcur * BN * BK, c + 1 < ch1,
                        [&](float* Ad, float* Bd) {
                          issue_w(Bd, c + 1, 0);
                          if (tap == NTAP - 1) issue_halo(Ad, slab + 1, 0);
                        },
                        [&](const float* Ar, const float* Br) {
    const float* Ab = Ar + (hrow0 + kh * HX + kw) * BK;
    const float* Bb = Br + brow * BK;
    if constexpr (BF6) {
#pragma unroll
      for (int g = 0; g < BK / 16; ++g) {
        const int k0 = 4 * g + 2 * (lane >> 5);
        u32x4_t ah[MI], am[MI], al[MI], bh[NI], bm[NI], bl[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          split3(*reinterpret_cast<const f32x4*>(Ab + mi * 2 * HX * BK + (k0 ^ hsw) * 4),
                 *reinterpret_cast<const f32x4*>(Ab + mi * 2 * HX * BK + ((k0 + 1) ^ hsw) * 4),
                 ah[mi], am[mi], al[mi]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          split3(*reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + (k0 ^ bsw) * 4),
                 *reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + ((k0 + 1) ^ bsw) * 4),
                 bh[ni], bm[ni], bl[ni]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            f32x16 cc = acc[mi][ni];
            cc = mfma_bf16(ah[mi], bh[ni], cc);
            cc = mfma_bf16(ah[mi], bm[ni], cc);
            cc = mfma_bf16(am[mi], bh[ni], cc);
            cc = mfma_bf16(ah[mi], bl[ni], cc);
            cc = mfma_bf16(al[mi], bh[ni], cc);
            cc = mfma_bf16(am[mi], bm[ni], cc);
            acc[mi][ni] = cc;
          }
      }
    } else
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      const int s = (lane >> 5) + 2 * kk;
      f32x4 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const f32x4*>(Ab + mi * 2 * HX * BK + (s ^ hsw) * 4);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + (s ^ bsw) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][j], bv[ni][j], acc[mi][ni],
                                                                0, 0, 0);
    }
                        });
    if (++tap == NTAP) {
      tap = 0;
      ++slab;
      abuf ^= 1;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  conv_epilogue<BM, BN, WM, WN>(
      a, acc, smem, tm, n0, split,
      [&](int row) {
        const int oy = oy0 + (row >> 4), ox = ox0 + (row & 15);
        return (oy < a.OH && ox < a.OW) ? (img * a.OH + oy) * a.OW + ox : -1;
      },
      img,
      [&](int, int m) { return a.res ? a.res + (size_t)m * a.rcs : (const float*)nullptr; });
}

// ---------------------------------------------------------------------------
// head.conv2 by bilinear phases (networks/DeteNet.py:108-112).  The input is
// cat[up4(L) (192 ch), G (64 ch)] with up4 = F.interpolate(x4, bilinear,
// align_corners=False).  For output row Y = 4q + r every upsampled row the 3x3
// taps touch is a fixed combination (weights k/8) of low-res rows q+e,
// e in E(r) = {-1,0} (r=0), {-1,0,1} (r=1,2), {0,1} (r=3), once the low-res
// map is replicate-extended by one row/col (which is exactly how the
// interpolation clamps).  So at phase (ry, rx) the 192-channel part is a
// |E(ry)| x |E(rx)| conv on the LOW-RES map with combined weights (6.25 taps
// on average instead of 9: -23% MACs for the whole layer) and the x4
// upsampled 256-channel map is never materialised.  The 64 full-res channels
// (G) are an ordinary 3x3 conv done first by conv_halo_kernel into y; this
// kernel adds y as a same-thread residual.  Conv zero padding breaks the
// periodicity only on the outermost rows/cols: up4_border_corr_kernel
// subtracts those taps from y beforehand.  Tile: an 8x16 patch of low-res
// positions of one phase; the L halo (10x18, replicate-clamped) is staged once
// per 32-channel slab like conv_halo_kernel.
constexpr int UP4_CU = 192, UP4_CG = 64, UP4_COUT = 128;
constexpr int UP4_KP = (UP4_CU / 32) * 9 * 32;  // per-phase packed K capacity (<= 9 taps)
constexpr int UP4_GK = (UP4_CG / 32) * 9 * 32;  // K of the G conv (576)

__device__ __forceinline__ int up4_ne(int r) { return (r == 0 || r == 3) ? 2 : 3; }
// index of border pixel (Y, X) in the order of up4_border_pixel, -1 inside
__device__ __forceinline__ int up4_border_index(int Y, int X, int H, int W) {
  if (Y == 0) return X;
  if (Y == H - 1) return W + X;
  if (X == 0) return 2 * W + Y - 1;
  if (X == W - 1) return 2 * W + (H - 2) + Y - 1;
  return -1;
}
__device__ __forceinline__ int up4_e0(int r) { return r == 3 ? 0 : -1; }

template <int PH>
__global__ __launch_bounds__(256) void conv_up4_kernel(ConvArgs a) {
  constexpr int PW = 16, BM = PH * PW, BN = UP4_COUT, WM = 2, WN = 2, NW = 4;
  constexpr int TM = BM / WM, TN = BN / WN, MI = TM / 32, NI = TN / 32;
  constexpr int HX = PW + 2, HY = PH + 2, HP = HX * HY;
  constexpr int A_G = (HP + 8 * NW - 1) / (8 * NW);
  constexpr int HPR = A_G * 8 * NW;
  constexpr int B_G = BN / 8 / NW;
  static_assert(MI >= 1 && NI >= 1, "tile");
  constexpr int RING = 2 * (HPR + BN) * BK;
  constexpr int STAGE = BM * (BN + 4);
  __shared__ __attribute__((aligned(16))) float smem[RING > STAGE ? RING : STAGE];
  float* As = smem;
  float* Bs = smem + 2 * HPR * BK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  // tile = (img * 16 + phase) * ppi + patch: after the XCD remap each XCD
  // sweeps whole phases of an image, so one phase's combined weights stay in
  // its L2 (interleaving all 16 phase weight sets streamed them from HBM for
  // every block)
  const int ptx = (a.lw + PW - 1) / PW, ppi = ptx * ((a.lh + PH - 1) / PH);
  const int t2 = bid / ppi, prem = bid - t2 * ppi;
  const int img = t2 >> 4, phase = t2 & 15;
  const int qy0 = (prem / ptx) * PH, qx0 = (prem - (prem / ptx) * ptx) * PW;
  const int ry = phase >> 2, rx = phase & 3;
  const int nex = up4_ne(rx), ey0 = up4_e0(ry), ex0 = up4_e0(rx);
  const int T = up4_ne(ry) * nex;
  const int nch = (UP4_CU / 32) * T;
  const int H = a.H, W = a.W;

  const int lrow = lane >> 3;
  // L halo sources: low-res (qy0-1+hy, qx0-1+hx), replicate-clamped
  const float* hsrc[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int hp = (wave * A_G + i) * 8 + lrow;
    const int hy = hp / HX, hx = hp - (hp / HX) * HX;
    const int ly = min(max(qy0 - 1 + hy, 0), a.lh - 1), lx = min(max(qx0 - 1 + hx, 0), a.lw - 1);
    const int sslot = (lane & 7) ^ ((hx >> 1) & 7);
    hsrc[i] = hp < HP ? a.x + (((long long)img * a.lh + ly) * a.lw + lx) * a.xcs + sslot * 4
                      : nullptr;
  }
  const float* wsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int row = (wave * B_G + i) * 8 + lrow;
    const int sslot = (lane & 7) ^ ((row >> 1) & 7);
    wsrc[i] = a.w + ((size_t)phase * BN + row) * UP4_KP + sslot * 4;
  }
  auto issue_halo = [&](int slab, int buf) {
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const float* src = hsrc[i] ? hsrc[i] + slab * BK : pf_conv_zero16;
      __builtin_amdgcn_global_load_lds(PF_GPTR(src),
                                       PF_LPTR(As + (buf * HPR + (wave * A_G + i) * 8) * BK), 16,
                                       0, 0);
    }
  };
  auto issue_w = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(PF_GPTR(wsrc[i] + (size_t)c * BK),
                                       PF_LPTR(Bs + (buf * BN + (wave * B_G + i) * 8) * BK), 16,
                                       0, 0);
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int px = lane & 15;
  const int hrow0 = ((wm * TM + (lane & 31)) >> 4) * HX + px;
  const int bsw = ((lane & 31) >> 1) & 7;
  const int brow = wn * TN + (lane & 31);

  issue_halo(0, 0);
  issue_w(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  int abuf = 0, slab = 0, tj = 0;
  for (int c = 0; c < nch; ++c) {
    const int bcur = c & 1;
    const bool last_tap = tj == T - 1;
    if (c + 1 < nch) {
      issue_w(c + 1, bcur ^ 1);
      if (last_tap) issue_halo(slab + 1, abuf ^ 1);
    }
    const int ey = ey0 + tj / nex, ex = ex0 + (tj - (tj / nex) * nex);
    const float* Ab = As + (abuf * HPR + hrow0 + (ey + 1) * HX + ex + 1) * BK;
    const int hsw = ((px + ex + 1) >> 1) & 7;
    const float* Bb = Bs + (bcur * BN + brow) * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 8; ++kk) {
      const int s = (lane >> 5) + 2 * kk;
      f32x4 av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        av[mi] = *reinterpret_cast<const f32x4*>(Ab + mi * 2 * HX * BK + (s ^ hsw) * 4);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bv[ni] = *reinterpret_cast<const f32x4*>(Bb + ni * 32 * BK + (s ^ bsw) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi][j], bv[ni][j], acc[mi][ni],
                                                                0, 0, 0);
    }
    if (last_tap) {
      tj = 0;
      ++slab;
      abuf ^= 1;
    } else {
      ++tj;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // y already holds G-conv + bias (- border corrections): same-thread residual
  conv_epilogue<BM, BN, WM, WN>(
      a, acc, smem, bid, 0, 0,
      [&](int row) {
        const int qy = qy0 + (row >> 4), qx = qx0 + (row & 15);
        return (qy < a.lh && qx < a.lw) ? (img * H + 4 * qy + ry) * W + 4 * qx + rx : -1;
      },
      img, [&](int, int m) { return (const float*)a.y + (size_t)m * a.ycs; });
}

// Phase weights from the packed conv2 weights ([128][2304], K order
// (cin/32, kh, kw, cin%32)): wph[phase][cout][c*32 + ci] in the phase's chunk
// order (per low-res slab its |E(ry)|x|E(rx)| taps), combined in fp64:
// W'(ey,ex) = sum_{dy,dx} cy(dy,ey) cx(dx,ex) W(dy,dx).  Followed by the
// transposed 3x3 taps of the 192 upsampled channels (border correction) and
// the packed 64-channel G conv ([128][576], a contiguous slice of each row).
__device__ double up4_coef(int r, int d, int e) {
  // coefficient of low-res row q+e in upsampled row 4q+r+d (d in -1..1)
  const int t = r + d;                    // -1..4
  const int qo = t < 0 ? -1 : (t > 3 ? 1 : 0);
  const int rr = t - 4 * qo;              // 0..3
  const int lo = rr < 2 ? -1 : 0;         // first low-res neighbour (relative to q+qo)
  const double wl = rr == 0 ? 0.375 : rr == 1 ? 0.125 : rr == 2 ? 0.875 : 0.625;
  if (e == qo + lo) return wl;
  if (e == qo + lo + 1) return 1.0 - wl;
  return 0.0;
}

__global__ void up4_phase_weights_kernel(const float* __restrict__ wpk, float* __restrict__ wph) {
  const int phase = blockIdx.y, o = blockIdx.x, ci = threadIdx.x & 31, cg = threadIdx.x >> 5;
  const int ry = phase >> 2, rx = phase & 3;
  const int nex = up4_ne(rx), ey0 = up4_e0(ry), ex0 = up4_e0(rx), T = up4_ne(ry) * nex;
  const int nch = (UP4_CU / 32) * T;
  const float* w = wpk + (size_t)o * 2304;
  float* dst = wph + ((size_t)phase * UP4_COUT + o) * UP4_KP;
  for (int c = cg; c < UP4_KP / 32; c += blockDim.x / 32) {
    float v = 0.f;
    if (c < nch) {
      const int slab = c / T, tj = c - slab * T;
      const int ey = ey0 + tj / nex, ex = ex0 + tj % nex;
      double acc = 0.0;
      for (int dy = -1; dy <= 1; ++dy) {
        const double cy = up4_coef(ry, dy, ey);
        if (cy == 0.0) continue;
        for (int dx = -1; dx <= 1; ++dx) {
          const double cx = up4_coef(rx, dx, ex);
          if (cx == 0.0) continue;
          acc += cy * cx * (double)w[(slab * 9 + (dy + 1) * 3 + (dx + 1)) * 32 + ci];
        }
      }
      v = (float)acc;
    }
    dst[c * 32 + ci] = v;
  }
  if (phase == 0) {
    float* wct = wph + (size_t)16 * UP4_COUT * UP4_KP;
    for (int e = threadIdx.x; e < 9 * UP4_CU; e += blockDim.x) {
      const int t = e / UP4_CU, ch = e % UP4_CU;
      wct[((size_t)t * UP4_CU + ch) * UP4_COUT + o] = w[((ch >> 5) * 9 + t) * 32 + (ch & 31)];
    }
  } else if (phase == 1) {
    float* wg = wph + (size_t)16 * UP4_COUT * UP4_KP + (size_t)9 * UP4_CU * UP4_COUT;
    for (int e = threadIdx.x; e < UP4_GK; e += blockDim.x)
      wg[(size_t)o * UP4_GK + e] = w[(UP4_CU / 32) * 9 * 32 + e];
  }
}

// Border pixel j of an image (rows 0 and H-1, then cols 0 and W-1 without the
// corners): 2W + 2(H-2) pixels.
__device__ __forceinline__ void up4_border_pixel(int j, int H, int W, int& Y, int& X) {
  if (j < W) { Y = 0; X = j; }
  else if (j < 2 * W) { Y = H - 1; X = j - W; }
  else {
    const int k = j - 2 * W;
    if (k < H - 2) { Y = 1 + k; X = 0; }
    else { Y = 1 + (k - (H - 2)); X = W - 1; }
  }
}

// Border correction.  On the outermost rows/cols the phase formula also sums
// taps that fall into conv2's zero padding, reading the replicate extension of
// the upsampled map there -- which equals the nearest in-image upsampled
// pixel.  y[border pixel][co] -= sum over out-of-image taps (dy,dx) of
// W[co][c][dy][dx] * up4(L)[clamp(Y+dy)][clamp(X+dx)][c]  (c < 192; the G
// conv has exact zero padding), before conv_up4_kernel adds its sum to y.  8 border pixels per block,
// (pixel half, cout) per thread, weights transposed to wct[tap][c][co].
constexpr int UP4_CPB = 16;
__global__ __launch_bounds__(2 * UP4_COUT) void up4_border_corr_kernel(
    const float* __restrict__ L, int lcs, int lh, int lw, int H, int W, int nbp,
    const float* __restrict__ wct, float* __restrict__ y, int ycs) {
  // u[k][c][p]: up4(L) at the clamped position of tap tl[k] for pixel p, or 0
  // where that tap is inside the image for p (k over the union of the block's
  // out-of-image taps: <= 5).  Each weight load then serves all 16 pixels.
  __shared__ float u[5][UP4_CU][UP4_CPB];
  __shared__ int tl[5], nt, bad[UP4_CPB], pyx[UP4_CPB][2];
  // blocks never straddle two border segments (top, bottom, left, right):
  // the union of out-of-image taps then has <= 5 members
  const int img = blockIdx.y, tid = threadIdx.x;
  const int bw = (W + UP4_CPB - 1) / UP4_CPB, bh = (H - 2 + UP4_CPB - 1) / UP4_CPB;
  int seg = blockIdx.x, sb;
  if (seg < 2 * bw) {
    sb = seg % bw;
    seg = seg / bw;
  } else {
    sb = (seg - 2 * bw) % bh;
    seg = 2 + (seg - 2 * bw) / bh;
  }
  const int seglen = seg < 2 ? W : H - 2;
  const int segbase = seg < 2 ? seg * W : 2 * W + (seg - 2) * (H - 2);
  const int j0 = segbase + sb * UP4_CPB;
  const int jend = segbase + seglen;
  const float sh = (float)lh / (float)H, sw = (float)lw / (float)W;
  if (tid < UP4_CPB) {
    int Y = 0, X = 0, mask = 0;
    if (j0 + tid < jend) {
      up4_border_pixel(j0 + tid, H, W, Y, X);
      for (int t = 0; t < 9; ++t) {
        const int yy = Y + t / 3 - 1, xx = X + t % 3 - 1;
        if ((unsigned)yy >= (unsigned)H || (unsigned)xx >= (unsigned)W) mask |= 1 << t;
      }
    }
    bad[tid] = mask;
    pyx[tid][0] = Y;
    pyx[tid][1] = X;
  }
  __syncthreads();
  if (tid == 0) {
    int um = 0;
    for (int p = 0; p < UP4_CPB; ++p) um |= bad[p];
    int k = 0;
    for (int t = 0; t < 9; ++t)
      if ((um >> t) & 1) tl[k++] = t;
    nt = k;
  }
  __syncthreads();
#pragma unroll 4
  for (int e = tid; e < nt * UP4_CU * UP4_CPB; e += 2 * UP4_COUT) {
    const int k = e / (UP4_CU * UP4_CPB), c = (e / UP4_CPB) % UP4_CU, p = e % UP4_CPB;
    const int t = tl[k];
    float v = 0.f;
    if ((bad[p] >> t) & 1) {
      const int yy = min(max(pyx[p][0] + t / 3 - 1, 0), H - 1);
      const int xx = min(max(pyx[p][1] + t % 3 - 1, 0), W - 1);
      // PyTorch upsample_bilinear2d, align_corners=False (as norm_prelu_upsample)
      float fy = sh * (yy + 0.5f) - 0.5f, fx = sw * (xx + 0.5f) - 0.5f;
      fy = fy < 0.f ? 0.f : fy;
      fx = fx < 0.f ? 0.f : fx;
      const int y0 = (int)fy, x0 = (int)fx;
      const int y1 = y0 + (y0 < lh - 1 ? 1 : 0), x1 = x0 + (x0 < lw - 1 ? 1 : 0);
      const float ly = fy - y0, lx = fx - x0, hy = 1.f - ly, hx = 1.f - lx;
      const float* b = L + (size_t)img * lh * lw * lcs + c;
      const float v00 = b[((size_t)y0 * lw + x0) * lcs], v01 = b[((size_t)y0 * lw + x1) * lcs];
      const float v10 = b[((size_t)y1 * lw + x0) * lcs], v11 = b[((size_t)y1 * lw + x1) * lcs];
      v = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
    }
    u[k][c][p] = v;
  }
  __syncthreads();
  // thread = (pixel half, cout); fixed (tap, channel) order -> deterministic
  constexpr int PH2 = UP4_CPB / 2;
  const int co = tid & (UP4_COUT - 1), p0 = (tid >> 7) * PH2;
  float acc[PH2];
#pragma unroll
  for (int p = 0; p < PH2; ++p) acc[p] = 0.f;
  for (int k = 0; k < nt; ++k) {
    const float* w = wct + (size_t)tl[k] * UP4_CU * UP4_COUT + co;
    for (int c = 0; c < UP4_CU; ++c) {
      const float wv = w[(size_t)c * UP4_COUT];
#pragma unroll
      for (int p = 0; p < PH2; ++p) acc[p] = fmaf(wv, u[k][c][p0 + p], acc[p]);
    }
  }
#pragma unroll
  for (int p = 0; p < PH2; ++p)
    if (j0 + p0 + p < jend) {
      int Y, X;
      up4_border_pixel(j0 + p0 + p, H, W, Y, X);
      y[(((size_t)img * H + Y) * W + X) * ycs + co] -= acc[p];
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
                                                         int ppi, int hw, int C, int nchunk,
                                                         double* __restrict__ chunks) {
  const int b = blockIdx.z, cg = blockIdx.y, ch = blockIdx.x;
  const int c = cg * 64 + (threadIdx.x & 63), tl = threadIdx.x >> 6;  // 16 tile lanes
  // image b's tiles: contiguous rows [b*hw/BM, ((b+1)*hw-1)/BM] or patches [b*ppi, (b+1)*ppi)
  const long long t0 = ppi ? (long long)b * ppi : (long long)b * hw / BM;
  const long long t1 = ppi ? (long long)(b + 1) * ppi - 1 : ((long long)(b + 1) * hw - 1) / BM;
  const long long ts = t0 + (long long)ch * STAT_CHUNK;
  const long long te = min(t1 + 1, ts + STAT_CHUNK);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    for (long long t = ts + tl; t < te; t += 16) {
      const int sl = (ppi || (t * BM) / hw == b) ? 0 : 1;
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
                                    float* __restrict__ rstd,
                                    const double* __restrict__ chunks2 = nullptr,
                                    int nchunk2 = 0) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * C) return;
  const int b = i / C, c = i - b * C;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const double* p = chunks + (((long long)b * nchunk + k) * C + c) * 2;
    s1 += p[0];
    s2 += p[1];
  }
  for (int k = 0; k < nchunk2; ++k) {  // second tiling of the same images (disjoint pixels)
    const double* p = chunks2 + (((long long)b * nchunk2 + k) * C + c) * 2;
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
    long long m;
    const int q = pf_quad_split(i, c4n, m);
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

// ---------------------------------------------------------------------------
// Launch planning: one Plan decides kernel, tile and split for a conv so the
// launch, the split-K workspace and the stats reduction agree on the tiling.
enum ConvKern { KERN_STAGED = 0, KERN_GLDS = 1, KERN_HALO = 2 };
enum ConvTile {
  TILE_128x128 = 0, TILE_128x64 = 1, TILE_64x64 = 2, TILE_256x128 = 3,  // contiguous rows
  TILE_H8x128 = 10, TILE_H8x64 = 11, TILE_H16x128 = 12,                 // 8/16 x 16 patches
  TILE_BF6_128x128 = 20, TILE_BF6_128x256 = 21, TILE_BF6_64x128 = 22,   // rows, bf16x6 products
  TILE_BF6_128x64 = 23, TILE_BF6B_128x128 = 24, TILE_BF6B_128x64 = 25,  // + pre-split weights
  TILE_BF6R_128x128 = 26, TILE_BF6R_128x64 = 27,  // + A straight to registers
  TILE_BF6B_256x128 = 28,  // pre-split weights, 8 waves stacked along M (one 135-KB block per CU)
  TILE_BF6X_128x128 = 29, TILE_BF6X_128x64 = 30,  // dense, 16x16x32 MFMAs (conv_bf6x_kernel)
  TILE_BF6X_256x128 = 31,
  TILE_BF6X_128x192 = 32,  // N % 192 == 0 (head.conv1's Winograd GEMMs, the tap GEMM): A read once per 192 columns
  TILE_BF6X_128x256 = 33,  // N % 256 == 0 batched GEMMs (A/B POSFEAT_BF6X_N256: A read once per 256 columns)
  TILE_BF6X_192x128 = 34,  // dense: six waves stacked along M, the B tile's L2 -> CU bytes per output 2/3
  TILE_BF6X_256x64 = 35    // dense / G4 (the stem), 64 columns: RB = 4, half the B bytes per output
};

// POSFEAT_BF6=1: every conv the row-tile DMA kernel serves (1x1, strided, the
// batched Winograd / tap GEMMs) runs its products as bf16x6 (fp32-exact,
// see split3); 3x3 stride-1 convs keep the fp32 halo kernel.  The candidate
// set of a conv is then either all-bf16x6 or all-fp32, so the autotuner's
// choice never changes results.
bool bf6_on() { return pf_conv_precision() >= 1; }
// the 3x3 stride-1 halo kernel in bf16x6 too (POSFEAT_BF6_HALO=0: fp32 MFMA);
// PfHaloFp32Scope keeps the calling thread's launches on fp32 halo tiles (the
// train-mode backbone, whose fp64-pinned gradient fixtures were validated on
// them, bbtrain.hip)
thread_local int tl_halo_fp32 = 0;
thread_local int tl_dense32 = 0;  // PfDense32Scope
thread_local int tl_stem32 = 0;   // PfHaloFp32Scope(false)
bool halo_bf6_on() {
  static const bool off = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6_HALO");
    return e && e[0] == '0';
  }();
  return bf6_on() && !off && tl_halo_fp32 == 0;
}
// Dense pre-split tiles (TILE_BF6B_*) and the register-A candidates
// (TILE_BF6R_*: any conv, masked taps included) run conv_bf6d_kernel with A
// prefetched POSFEAT_BF6D = 2..4 chunks ahead in registers (default 2; 0: the
// LDS-staged conv_bf6b_kernel).  The 8-wave TILE_BF6B_256x128 caps D at 3 (its
// register budget at two waves per SIMD): D = 4 runs D = 3 there.  (Round 2's
// register-A twin with a one-chunk prefetch, conv_bf6r_kernel, and the
// persistent conv_bf6p_kernel lost their A/Bs and are no longer built.)  Same box,
// r6k: 945.6 -> 970 img/s (D = 3), decoder Winograd GEMMs -4..-7 %, tap GEMM
// -9 %; r6q, two pairs each: D = 2 973.1, 3 968.4, 4 966.3 img/s;
// bit-identical (test_gpu_bf6r.py)
int bf6d_depth() {
  static const int d = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6D");
    const int v = e ? atoi(e) : 2;
    return v >= 2 && v <= 4 ? v : 0;
  }();
  return d;
}

// Dense pre-split GEMMs / 1x1 convs (no padding, stride 1) run the 16x16x32
// conv_bf6x_kernel (POSFEAT_BF6X=0: the 32x32x16 bf6d tiles, A/B).  Their
// candidate set is then the two BF6X tiles only, so the autotuner's choice
// never changes results (the 16x16x32 sums are not bit-identical to the
// 32x32x16 tiles').  The train-mode backbone (PfHaloFp32Scope) keeps the
// 32x32x16 tiles: its one-step gradient against fp64 on the 2 x 128 x 160
// fixture case (BatchNorm over 160 pixels in layer3) moved from a worst
// per-tensor error of 0.014 (both 32x32 arithmetics) to 0.117 with the
// 16x16x32 sums (tools/bb_step_err.py), while every conv
// and the extraction model stay within the fp32 bounds (test_gpu_bf6x.py).
bool bf6x_on() {
  static const bool off = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6X");
    return e && e[0] == '0';
  }();
  return bf6_on() && !off && tl_halo_fp32 == 0 && tl_dense32 == 0;
}
// 1x1, no padding, any stride (a strided 1x1 conv is a GEMM over the
// subsampled pixel rows: conv_bf6x_kernel maps each row to its input pixel)
bool dense_gemm(const ConvArgs& a) {
  return a.KH == 1 && a.KW == 1 && a.pad == 0 && a.wb && !a.xb;
}
// Cin % 32 == 0 convs with taps or padding (3x3 stride 1 / 2): the bf6x tile
// gathers each lane's rows per (slab, tap) chunk (conv_bf6x_kernel GT)
bool gt_gemm(const ConvArgs& a) {
  return a.Cin % BK == 0 && !(a.KH == 1 && a.KW == 1 && a.pad == 0) && a.KH * a.KW <= 32 &&
         a.wb && !a.xb;
}
// 4-channel input (NHWC4: the 7x7 stem), K order (kh, kw, c4): the bf6x tile
// gathers each lane's two taps per chunk (conv_bf6x_kernel G4)
bool g4_gemm(const ConvArgs& a) {
  return a.Cin == 4 && a.xcs == 4 && a.KW >= 5 && a.KW <= 8 && a.wb && !a.xb &&
         a.Kpad == (a.KH * a.KW * 4 + BK - 1) / BK * BK;
}

struct Plan {
  int kern, tile, bm, bn, ppi;  // ppi: patches per image (halo), 0 = contiguous rows
  long long tiles_m;
  int ksplit;
};

// Environment switches for A/B timing only (defaults are the tuned choice):
// POSFEAT_CONV_KERNEL=staged|glds|halo caps the kernel family, POSFEAT_CONV_TILE
// forces a tile id where legal.
struct ConvEnv {
  int kmax = KERN_HALO, tile = -1, maxsplit = 4;
  ConvEnv() {
    if (const char* e = pf_ab_getenv("POSFEAT_CONV_MAXSPLIT")) maxsplit = atoi(e);
    if (const char* e = pf_ab_getenv("POSFEAT_CONV_KERNEL")) {
      if (e[0] == 's') kmax = KERN_STAGED;
      else if (e[0] == 'g') kmax = KERN_GLDS;
    }
    if (const char* e = getenv("POSFEAT_CONV_TILE")) tile = atoi(e);
  }
};
const ConvEnv& conv_env() {
  static const ConvEnv e;
  return e;
}

// Split-K factor: only for deep K (>= 64 chunks) where the tile count leaves
// the last round of resident workgroups badly underfilled.
int choose_ksplit(long long tiles, int nch, double slots) {
  // (splitting underfilled grids' shorter K too was measured no faster, r3v)
  if (nch < 64) return 1;
  int best = 1;
  double best_eff = 0.0;
  for (int ks = 1; ks <= conv_env().maxsplit; ++ks) {
    if (nch / ks < 32) break;
    const double r = tiles * ks / slots;
    const double eff = r / ceil(r) * (ks == 1 ? 1.0 : 0.97);  // ~3% for the reduce pass
    // split only for a clear gain (A/B at 480x640: decoder layers gain nothing)
    if (eff > best_eff * 1.08) {
      best_eff = eff;
      best = ks;
    }
  }
  return best;
}

// Geometry of one tile id for this conv (ksplit = 1); kern = -1 if illegal.
Plan plan_for_tile(const ConvArgs& a, int tile) {
  Plan p{};
  p.kern = -1;
  p.tile = tile;
  p.ksplit = 1;
  const bool cin32 = a.Cin % BK == 0;
  const bool halo_ok = cin32 && conv_env().kmax >= KERN_HALO && a.stride == 1 && a.KH == 3 &&
                       a.KW == 3 && a.OW >= 16 && a.OH >= 8 && a.Cout % 64 == 0;
  const bool glds_ok = cin32 && conv_env().kmax >= KERN_GLDS && a.KH * a.KW <= 32;
  // bf16x6 mode: halo-eligible convs keep fp32 halo tiles only, the rest
  // bf16x6 row tiles only
  if (bf6_on() && glds_ok) {
    // pre-split convs on the bf6x tiles (dense GEMMs, slab x tap gathers):
    // the 16x16x32 tiles only, and only they
    const bool x_tile = tile >= TILE_BF6X_128x128 && tile <= TILE_BF6X_256x64;
    if (bf6x_on() && (dense_gemm(a) || gt_gemm(a))) {
      if (!x_tile) return p;
    } else {
      if (x_tile) return p;
      const bool bf6_tile = tile >= TILE_BF6_128x128 && tile <= TILE_BF6B_256x128;
      if (halo_ok ? bf6_tile || tile < TILE_H8x128 : !bf6_tile) return p;
    }
  }
  switch (tile) {
    case TILE_BF6X_128x128:
    case TILE_BF6X_128x64:
    case TILE_BF6X_256x128:
    case TILE_BF6X_128x192:
    case TILE_BF6X_128x256:
    case TILE_BF6X_192x128:
    case TILE_BF6X_256x64:
      if (!bf6x_on() || !((glds_ok && (dense_gemm(a) || gt_gemm(a))) || g4_gemm(a))) return p;
      if (g4_gemm(a) && tile != TILE_BF6X_128x64 && tile != TILE_BF6X_256x64) return p;
      if (tile == TILE_BF6X_128x192 && (!dense_gemm(a) || a.Cout % 192)) return p;
      if (tile == TILE_BF6X_128x256 && (!dense_gemm(a) || a.Cout % 256)) return p;
      if (tile == TILE_BF6X_192x128 && !dense_gemm(a) && !a.x2) return p;
      if (tile == TILE_BF6X_256x64 && !dense_gemm(a) && !g4_gemm(a)) return p;
      p.kern = KERN_GLDS;
      p.bm = tile == TILE_BF6X_256x128 || tile == TILE_BF6X_256x64 ? 256
             : tile == TILE_BF6X_192x128                          ? 192
                                                                  : 128;
      p.bn = tile == TILE_BF6X_128x64 || tile == TILE_BF6X_256x64 ? 64
             : tile == TILE_BF6X_128x192 ? 192
             : tile == TILE_BF6X_128x256 ? 256
                                         : 128;
      p.ppi = 0;
      p.tiles_m = (a.M + p.bm - 1) / p.bm;
      return p;
    case TILE_BF6B_256x128:
      if (!glds_ok || !bf6_on() || !a.wb || a.Cout <= 64) return p;
      p.kern = KERN_GLDS;
      p.bm = 256;
      p.bn = 128;
      p.ppi = 0;
      p.tiles_m = (a.M + p.bm - 1) / p.bm;
      return p;
    case TILE_BF6B_128x128:
    case TILE_BF6B_128x64:
    case TILE_BF6R_128x128:
    case TILE_BF6R_128x64:
      if (!glds_ok || !bf6_on() || !a.wb) return p;
      p.kern = KERN_GLDS;
      p.bm = 128;
      p.bn = tile == TILE_BF6B_128x64 || tile == TILE_BF6R_128x64 ? 64 : 128;
      p.ppi = 0;
      p.tiles_m = (a.M + p.bm - 1) / p.bm;
      return p;
    case TILE_BF6_128x128:
    case TILE_BF6_128x256:
    case TILE_BF6_64x128:
    case TILE_BF6_128x64:
      if (!glds_ok || !bf6_on() || (tile == TILE_BF6_128x256 && a.Cout % 256)) return p;
      p.kern = KERN_GLDS;
      p.bm = tile == TILE_BF6_64x128 ? 64 : 128;
      p.bn = tile == TILE_BF6_128x256 ? 256 : tile == TILE_BF6_128x64 ? 64 : 128;
      p.ppi = 0;
      p.tiles_m = (a.M + p.bm - 1) / p.bm;
      return p;
    case TILE_H8x128:
    case TILE_H16x128:
    case TILE_H8x64: {
      if (!halo_ok || (tile != TILE_H8x64 && a.Cout % 128)) return p;
      const int ph = tile == TILE_H16x128 ? 16 : 8;
      p.kern = KERN_HALO;
      p.bm = ph * 16;
      p.bn = tile == TILE_H8x64 ? 64 : 128;
      p.ppi = ((a.OW + 15) / 16) * ((a.OH + ph - 1) / ph);
      p.tiles_m = (long long)(a.M / a.hw) * p.ppi;
      return p;
    }
    case TILE_256x128:
      if (!cin32 || a.Cout % 128) return p;
      p.bm = 256;
      p.bn = 128;
      break;
    case TILE_128x128: p.bm = 128; p.bn = 128; break;
    case TILE_128x64: p.bm = 128; p.bn = 64; break;
    case TILE_64x64: p.bm = 64; p.bn = 64; break;
    default: return p;
  }
  // the 4-channel-input convs the G4 bf6x tile serves: it is their only
  // candidate (its sums are not bit-identical to the staged tiles')
  if (bf6x_on() && g4_gemm(a)) return p;
  p.kern = !cin32 ? KERN_STAGED
                  : (conv_env().kmax >= KERN_GLDS && a.KH * a.KW <= 32 ? KERN_GLDS : KERN_STAGED);
  if (tile == TILE_256x128 && p.kern != KERN_GLDS) {
    p.kern = -1;
    return p;
  }
  p.ppi = 0;
  p.tiles_m = (a.M + p.bm - 1) / p.bm;
  return p;
}

// Default plan (heuristic), optionally overridden by a legal tile id.  The
// split factor comes from the default choice whatever the tile, and every
// kernel/tile runs the same fmaf sequence per output, so results do not
// depend on the tile (the engine's autotuner relies on this).
Plan conv_plan(const ConvArgs& a, bool allow_split, int forced = -1) {
  const ConvEnv& env = conv_env();
  if (forced < 0 && env.tile >= 0) forced = env.tile;  // POSFEAT_CONV_TILE: any legal tile
  const bool cin32 = a.Cin % BK == 0;
  const int nch = a.Kpad / BK;
  Plan d = plan_for_tile(a, a.Cout % 128 == 0 ? TILE_H8x128 : TILE_H8x64);
  if (d.kern == KERN_HALO) {
    if ((env.tile == TILE_H16x128) && a.Cout % 128 == 0) d = plan_for_tile(a, TILE_H16x128);
    const double slots = d.tile == TILE_H16x128 ? 256.0 : 512.0;
    d.ksplit = allow_split ? choose_ksplit(d.tiles_m * ((a.Cout + d.bn - 1) / d.bn), nch, slots) : 1;
  } else {
    const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
    const long long t256 = (long long)((a.M + 255) / 256) * ((a.Cout + 127) / 128);
    const int ks = (allow_split && a.Cout > 64) ? choose_ksplit(t128, nch, 512.0) : 1;
    int tile;
    if (env.tile == TILE_256x128 && cin32 && a.Cout % 128 == 0 && t256 >= 256 && ks == 1)
      tile = TILE_256x128;
    else if (a.Cout > 64 && (t128 >= 512 || ks > 1))
      tile = TILE_128x128;
    else if (cin32 && (long long)((a.M + 127) / 128) * ((a.Cout + 63) / 64) >= 512)
      tile = TILE_128x64;  // Cin = 4 layers (stem, convimg): 64x64 measured faster
    else
      tile = TILE_64x64;
    d = plan_for_tile(a, tile);
    d.ksplit = tile == TILE_128x128 ? ks : 1;
    if (bf6x_on() && g4_gemm(a)) {  // the stem: the G4 bf6x tile only
      d = plan_for_tile(a, TILE_BF6X_128x64);
      d.ksplit = 1;
    }
    if (bf6_on() && cin32 && a.KH * a.KW <= 32 && env.kmax >= KERN_GLDS) {
      const bool x = bf6x_on() && dense_gemm(a);
      Plan b = plan_for_tile(a, x ? (a.Cout > 64 ? TILE_BF6X_128x128 : TILE_BF6X_128x64)
                                : a.wb ? (a.Cout > 64 ? TILE_BF6B_128x128 : TILE_BF6B_128x64)
                                       : (a.Cout > 64 ? TILE_BF6_128x128 : TILE_BF6_128x64));
      if (b.kern >= 0) {
        b.ksplit = ks;
        d = b;
      }
    }
  }
  // Cin % 32 convs with taps on the pre-split planes: the GT bf6x tile
  if (bf6x_on() && gt_gemm(a) && env.kmax >= KERN_GLDS) {
    Plan b = plan_for_tile(a, a.Cout > 64 ? TILE_BF6X_128x128 : TILE_BF6X_128x64);
    if (b.kern >= 0) {
      const long long t128 = (long long)((a.M + 127) / 128) * ((a.Cout + 127) / 128);
      b.ksplit = allow_split ? choose_ksplit(t128, nch, 768.0) : 1;
      d = b;
    }
  }
  if (forced >= 0) {
    Plan f = plan_for_tile(a, forced);
    if (f.kern >= 0) {
      f.ksplit = d.ksplit;
      return f;
    }
  }
  return d;
}


// The Cin = 4 register-staged convs (the stem) in bf16x6 with the rest of the
// conv family (POSFEAT_BF6_STEM=0: fp32 MFMA); the train-mode backbone keeps
// fp32 there as on its halo tiles (PfHaloFp32Scope).  All staged tiles of a
// conv share the arithmetic, so the autotuner's choice never changes results.
bool stem_bf6_on() {
  static const bool off = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6_STEM");
    return e && e[0] == '0';
  }();
  return bf6_on() && !off && tl_halo_fp32 == 0 && tl_stem32 == 0;
}

template <int BM, int BN, int WM, int WN>
void launch_rows(ConvArgs& a, int kern, hipStream_t st) {
  dim3 grid(a.nwg * a.ksplit, a.nbatch), block(WM * WN * 64);
  if (kern == KERN_GLDS)
    hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WM, WN>), grid, block, 0, st, a);
  else if (a.Cin % BK == 0)
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, true>), grid, block, 0, st, a);
  else if (stem_bf6_on())
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, false, true>), grid, block, 0, st, a);
  else
    hipLaunchKernelGGL((conv_mfma_kernel<BM, BN, WM, WN, false>), grid, block, 0, st, a);
}

// A/B (POSFEAT_BF6X_BM192=1): the dense / two-source 128 x 128 bf6x plans
// run as 192 x 128 tiles
static bool bf6x_bm192() {
  static const bool on = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6X_BM192");
    return e && e[0] == '1';
  }();
  return on;
}

thread_local float* tl_nchw_sink = nullptr;
thread_local bool tl_nchw_done = false;

int conv_run(ConvArgs& a, const Plan& p0, hipStream_t st) {
  if (!a.zero) return POSFEAT_E_HIP;
  Plan p = p0;
  // (the bf6x tiles' epilogue, conv_epilogue_t, carries the NCHW pass;
  // split-K plans write y in the reduce kernel instead)
  const bool xt = p.tile >= TILE_BF6X_128x128 && p.tile <= TILE_BF6X_256x64;
  a.ynchw = (tl_nchw_sink && xt && p.ksplit <= 1 && a.nbatch <= 1 && !a.res && a.hw % 4 == 0)
                ? tl_nchw_sink
                : nullptr;
  tl_nchw_done = a.ynchw != nullptr;
  if (bf6x_bm192() && p.tile == TILE_BF6X_128x128 && p.ksplit == 1 && (dense_gemm(a) || a.x2)) {
    const Plan q = plan_for_tile(a, TILE_BF6X_192x128);
    if (q.kern >= 0) p = q;
  }
  static const bool rb4n64 = [] {  // A/B: the 128 x 64 dense / stem plans on 256 x 64 tiles
    const char* e = pf_ab_getenv("POSFEAT_BF6X_RB4N64");
    return e && e[0] == '1';
  }();
  if (rb4n64 && p.tile == TILE_BF6X_128x64 && p.ksplit == 1 && (dense_gemm(a) || g4_gemm(a)) &&
      !a.x2) {
    const Plan q = plan_for_tile(a, TILE_BF6X_256x64);
    if (q.kern >= 0) p = q;
  }
  a.tiles_n = (a.Cout + p.bn - 1) / p.bn;
  a.nwg = (int)(p.tiles_m * a.tiles_n);
  a.ksplit = p.ksplit;
  const dim3 grid(a.nwg * a.ksplit);
  switch (p.tile) {
    case TILE_H8x128:
      if (halo_bf6_on())
        hipLaunchKernelGGL((conv_halo_kernel<8, 128, 2, 2, 3, 3, true>), grid, dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((conv_halo_kernel<8, 128, 2, 2, 3, 3>), grid, dim3(256), 0, st, a);
      break;
    case TILE_H8x64:
      if (halo_bf6_on())
        hipLaunchKernelGGL((conv_halo_kernel<8, 64, 2, 2, 3, 3, true>), grid, dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((conv_halo_kernel<8, 64, 2, 2, 3, 3>), grid, dim3(256), 0, st, a);
      break;
    case TILE_H16x128:
      hipLaunchKernelGGL((conv_halo_kernel<16, 128, 4, 2, 3, 3>), grid, dim3(512), 0, st, a);
      break;
    case TILE_BF6_128x128:
      hipLaunchKernelGGL((conv_glds_kernel<128, 128, 2, 2, 2, true>),
                         dim3(a.nwg * a.ksplit, a.nbatch), dim3(256), 0, st, a);
      break;
    case TILE_BF6_128x256:
      hipLaunchKernelGGL((conv_glds_kernel<128, 256, 2, 2, 2, true>), dim3(a.nwg * a.ksplit, a.nbatch),
                         dim3(256), 0, st, a);
      break;
    case TILE_BF6_64x128:
      hipLaunchKernelGGL((conv_glds_kernel<64, 128, 2, 2, 2, true>), dim3(a.nwg * a.ksplit, a.nbatch),
                         dim3(256), 0, st, a);
      break;
    case TILE_BF6_128x64:
      hipLaunchKernelGGL((conv_glds_kernel<128, 64, 2, 2, 2, true>),
                         dim3(a.nwg * a.ksplit, a.nbatch), dim3(256), 0, st, a);
      break;
    case TILE_BF6X_128x128:
      if (a.x2)  // pf_conv_dual
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 2, 3>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      else if (a.amean)  // pf_conv_run_tile_np
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 2, 4>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      else if (dense_gemm(a))
        hipLaunchKernelGGL((conv_bf6x_kernel<128>), dim3(a.nwg * a.ksplit, a.nbatch), dim3(256),
                           0, st, a);
      else  // gt_gemm: the slab x tap gather
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 2, 2>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      break;
    case TILE_BF6X_128x64:
      if (a.Cin == 4)  // g4_gemm: the 4-channel tap gather
        hipLaunchKernelGGL((conv_bf6x_kernel<64, 2, 1>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      else if (dense_gemm(a))
        hipLaunchKernelGGL((conv_bf6x_kernel<64>), dim3(a.nwg * a.ksplit, a.nbatch), dim3(256), 0,
                           st, a);
      else
        hipLaunchKernelGGL((conv_bf6x_kernel<64, 2, 2>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      break;
    case TILE_BF6X_128x192:  // dense GEMMs only (plan_for_tile)
      hipLaunchKernelGGL((conv_bf6x_kernel<192>), dim3(a.nwg * a.ksplit, a.nbatch), dim3(256), 0,
                         st, a);
      break;
    case TILE_BF6X_256x64:
      if (a.Cin == 4)
        hipLaunchKernelGGL((conv_bf6x_kernel<64, 4, 1>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((conv_bf6x_kernel<64, 4>), dim3(a.nwg * a.ksplit, a.nbatch), dim3(256),
                           0, st, a);
      break;
    case TILE_BF6X_192x128:  // dense / two-source GEMMs only (plan_for_tile)
      if (a.x2)
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 2, 3, 6>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(384), 0, st, a);
      else
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 2, 0, 6>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(384), 0, st, a);
      break;
    case TILE_BF6X_128x256:  // dense GEMMs only (plan_for_tile)
      hipLaunchKernelGGL((conv_bf6x_kernel<256>), dim3(a.nwg * a.ksplit, a.nbatch), dim3(256), 0,
                         st, a);
      break;
    case TILE_BF6X_256x128:
      if (dense_gemm(a))
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 4>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((conv_bf6x_kernel<128, 4, 2>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      break;
    case TILE_BF6B_128x128:
    case TILE_BF6B_128x64: {
      const bool wide = p.tile == TILE_BF6B_128x128;
      if (a.xb) {  // A pre-split by its producer (pf_gemm_batched_pre)
        const dim3 g(a.nwg * a.ksplit, a.nbatch);
        if (wide)
          hipLaunchKernelGGL((conv_bf6s_kernel<128, 128, 2>), g, dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((conv_bf6s_kernel<128, 64, 2>), g, dim3(256), 0, st, a);
      } else if (bf6d_depth() && a.KH == 1 && a.KW == 1 && a.pad == 0) {
        const dim3 g(a.nwg * a.ksplit, a.nbatch);
        const int dd = bf6d_depth();
        if (wide && dd == 2)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 2>), g, dim3(256), 0, st, a);
        else if (wide && dd == 3)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 3>), g, dim3(256), 0, st, a);
        else if (wide)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 4>), g, dim3(256), 0, st, a);
        else if (dd == 2)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 2>), g, dim3(256), 0, st, a);
        else if (dd == 3)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 3>), g, dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 4>), g, dim3(256), 0, st, a);
      } else if (wide) {
        hipLaunchKernelGGL((conv_bf6b_kernel<128, 128>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL((conv_bf6b_kernel<128, 64>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      }
      break;
    }
    case TILE_BF6B_256x128:
      if (bf6d_depth() == 2)
        hipLaunchKernelGGL((conv_bf6d_kernel<256, 128, 2, 8>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(512), 0, st, a);
      else if (bf6d_depth())
        hipLaunchKernelGGL((conv_bf6d_kernel<256, 128, 3, 8>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((conv_bf6b_kernel<256, 128, 8>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(512), 0, st, a);
      break;
    case TILE_BF6R_128x128:
      if (bf6d_depth()) {  // the register-A tiles: A now prefetched D chunks ahead
        const dim3 g(a.nwg * a.ksplit, a.nbatch);
        if (bf6d_depth() == 2)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 2>), g, dim3(256), 0, st, a);
        else if (bf6d_depth() == 3)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 3>), g, dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 128, 4>), g, dim3(256), 0, st, a);
      } else {  // POSFEAT_BF6D=0: the LDS-staged form
        hipLaunchKernelGGL((conv_bf6b_kernel<128, 128>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      }
      break;
    case TILE_BF6R_128x64:
      if (bf6d_depth()) {
        const dim3 g(a.nwg * a.ksplit, a.nbatch);
        if (bf6d_depth() == 2)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 2>), g, dim3(256), 0, st, a);
        else if (bf6d_depth() == 3)
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 3>), g, dim3(256), 0, st, a);
        else
          hipLaunchKernelGGL((conv_bf6d_kernel<128, 64, 4>), g, dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL((conv_bf6b_kernel<128, 64>), dim3(a.nwg * a.ksplit, a.nbatch),
                           dim3(256), 0, st, a);
      }
      break;
    case TILE_256x128: launch_rows<256, 128, 4, 2>(a, p.kern, st); break;
    case TILE_128x128: launch_rows<128, 128, 2, 2>(a, p.kern, st); break;
    case TILE_128x64: launch_rows<128, 64, 2, 2>(a, p.kern, st); break;
    default: launch_rows<64, 64, 2, 2>(a, p.kern, st); break;
  }
  PF_CHECK_LAUNCH();
  // bf16x6: every BF6* tile, the bf16x6 halo twins and the bf16x6 stem;
  // fp32 MFMA: the fp32 halo / row tiles
  const bool bf6 = p.tile >= TILE_BF6_128x128 ||
                   ((p.tile == TILE_H8x128 || p.tile == TILE_H8x64) && halo_bf6_on()) ||
                   (p.tile < TILE_H8x128 && p.kern == KERN_STAGED && a.Cin % BK != 0 &&
                    stem_bf6_on());
  pf_note_arith(bf6 ? PF_ARITH_BF6 : PF_ARITH_FP32);
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

void launch_up4(const ConvArgs& a, hipStream_t st) {
  pf_note_arith(PF_ARITH_FP32);
  hipLaunchKernelGGL(conv_up4_kernel<8>, dim3(a.nwg), dim3(256), 0, st, a);
}

void launch_up4_weights(const float* w_packed, float* wph, hipStream_t st) {
  hipLaunchKernelGGL(up4_phase_weights_kernel, dim3(UP4_COUT, 16), dim3(256), 0, st, w_packed,
                     wph);
}

}  // namespace

bool pf_bf6x_on() { return bf6x_on(); }
bool pf_halo_bf6_on() { return halo_bf6_on(); }
PfHaloFp32Scope::PfHaloFp32Scope(bool halo_fp32) : halo_(halo_fp32) {
  if (halo_) {
    ++tl_halo_fp32;
  } else {
    ++tl_dense32;
    ++tl_stem32;
  }
}
PfHaloFp32Scope::~PfHaloFp32Scope() {
  if (halo_) {
    --tl_halo_fp32;
  } else {
    --tl_dense32;
    --tl_stem32;
  }
}
PfNchwSink::PfNchwSink(float* dst) {
  tl_nchw_sink = dst;
  tl_nchw_done = false;
}
PfNchwSink::~PfNchwSink() { tl_nchw_sink = nullptr; }
bool PfNchwSink::done() const { return tl_nchw_done; }
PfDense32Scope::PfDense32Scope(bool on) : on_(on) { tl_dense32 += on ? 1 : 0; }
PfDense32Scope::~PfDense32Scope() { tl_dense32 -= on_ ? 1 : 0; }

extern "C" int posfeat_conv_packed_k(int cin, int kh, int kw) {
  const int cinp = (cin + 3) / 4 * 4;
  const int k = kh * kw * cinp;
  return (k + BK - 1) / BK * BK;
}

// device address of pf_conv_zero16 on the current device (cached per thread)
static const float* conv_zero_ptr() {
  thread_local int dev = -1;
  thread_local const float* p = nullptr;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  if (d != dev) {
    void* q = nullptr;
    if (hipGetSymbolAddress(&q, HIP_SYMBOL(pf_conv_zero16)) != hipSuccess) return nullptr;
    p = static_cast<const float*>(q);
    dev = d;
  }
  return p;
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
  a.bnpart = nullptr;
  a.hw = a.OH * a.OW;
  a.nbatch = 1;
  a.bx = a.bw = a.by = 0;
  a.wb = nullptr;
  a.xb = nullptr;
  a.xplane = a.bxb = 0;
  a.wplane = a.bwb = 0;
  a.x2 = nullptr;
  a.x2cs = a.k1ch = a.H2 = a.W2 = a.s2 = 0;
  a.amean = a.arstd = a.aslope = nullptr;
  a.ynchw = nullptr;
  a.zero = conv_zero_ptr();  // checked at launch (planning calls need no device)
  return POSFEAT_OK;
}

extern "C" int posfeat_conv2d_nhwc(const posfeat_conv_desc* d, const float* x, const float* w,
                                   const float* bias, const float* res, float* y, void* stream) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, res, y, a));
  return conv_run(a, conv_plan(a, false), pf_stream(stream));
}

extern "C" size_t posfeat_conv2d_workspace(const posfeat_conv_desc* d) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  const Plan p = conv_plan(a, true);
  return p.ksplit > 1 ? (size_t)p.ksplit * a.M * a.Cout * sizeof(float) : 0;
}

extern "C" int posfeat_conv2d_nhwc_ws(const posfeat_conv_desc* d, const float* x, const float* w,
                                      const float* bias, const float* res, float* y, void* ws,
                                      size_t ws_bytes, void* stream) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, res, y, a));
  const size_t need = posfeat_conv2d_workspace(d);
  const bool split = need > 0 && ws && ws_bytes >= need;
  const Plan p = conv_plan(a, split);
  if (p.ksplit > 1) a.part = static_cast<float*>(ws);
  return conv_run(a, p, pf_stream(stream));
}

extern "C" int posfeat_conv2d_nhwc_planes(const posfeat_conv_desc* d, const float* x,
                                          const float* w, const unsigned short* wb,
                                          long long wplane, const float* bias, const float* res,
                                          float* y, void* ws, size_t ws_bytes, int tile,
                                          void* stream) {
  if (!d || !wb || wplane <= 0) return POSFEAT_E_INVALID;
  // the three planes must not overlap: each holds cout x packed-K bf16 values
  if (wplane < (long long)d->cout * posfeat_conv_packed_k(d->cin, d->kh, d->kw))
    return POSFEAT_E_INVALID;
  return pf_conv_run_tile(d, x, w, bias, res, y, ws, ws_bytes, tile, pf_stream(stream), wb,
                          wplane);
}

// Stats tiling: contiguous-row tiles may straddle two images (slot 1 holds the
// second image's rows); patch tiles belong to one image.
static size_t stats_tiles_per_img(const ConvArgs& a, const Plan& p) {
  return p.ppi > 0 ? (size_t)p.ppi : (size_t)(a.hw + p.bm - 1) / p.bm + 1;
}

extern "C" size_t posfeat_conv2d_stats_workspace(const posfeat_conv_desc* d) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  const Plan p = conv_plan(a, false);
  if (p.ppi == 0 && a.hw < p.bm) return 0;  // a tile may span > 2 images: not supported
  const size_t nchunk = (stats_tiles_per_img(a, p) + STAT_CHUNK - 1) / STAT_CHUNK;
  return pf_align((size_t)p.tiles_m * 2 * a.Cout * 2 * sizeof(float), 256) +
         (size_t)d->n * nchunk * a.Cout * 2 * sizeof(double);
}

extern "C" int posfeat_conv2d_nhwc_stats(const posfeat_conv_desc* d, const float* x,
                                         const float* w, const float* bias, float* y, void* ws,
                                         size_t ws_bytes, float* mean, float* rstd, float eps,
                                         void* stream) {
  return pf_conv_stats_run_tile(d, x, w, bias, y, ws, ws_bytes, mean, rstd, eps, -1,
                                pf_stream(stream));
}

// ---------------------------------------------------------------------------
// Tile-aware entry points for the engine's autotuner (fmap.h).
static const int kAllTiles[] = {TILE_H8x128,      TILE_H8x64,       TILE_128x128,
                                TILE_128x64,      TILE_64x64,       TILE_256x128,
                                TILE_BF6_128x128, TILE_BF6_128x256, TILE_BF6_64x128,
                                TILE_BF6_128x64,  TILE_BF6B_128x128, TILE_BF6B_128x64,
                                TILE_BF6R_128x128, TILE_BF6R_128x64,  TILE_BF6B_256x128,
                                TILE_BF6X_128x128, TILE_BF6X_128x64, TILE_BF6X_128x192};
// (TILE_BF6X_256x128 is legal where forced -- POSFEAT_CONV_TILE, the planes
// ABI's tile argument -- but not an autotune candidate: never faster, and the
// timing noise let it take the tap GEMM at +5 %, r7i)

int pf_conv_candidates(const posfeat_conv_desc* d, int* tiles, int max, bool wplanes) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  if (wplanes) a.wb = reinterpret_cast<const unsigned short*>(dummy);
  int n = 0;
  for (int t : kAllTiles)
    if (plan_for_tile(a, t).kern >= 0 && n < max) tiles[n++] = t;
  return n;
}

int pf_conv_run_tile(const posfeat_conv_desc* d, const float* x, const float* w,
                     const float* bias, const float* res, float* y, void* ws, size_t ws_bytes,
                     int tile, hipStream_t st, const unsigned short* wb, long long wplane) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, res, y, a));
  a.wb = wb;
  a.wplane = wplane;
  const size_t need = posfeat_conv2d_workspace(d);
  const bool split = need > 0 && ws && ws_bytes >= need;
  const Plan p = conv_plan(a, split, tile);
  if (p.ksplit > 1) a.part = static_cast<float*>(ws);
  return conv_run(a, p, st);
}

// y = act(x1 . W1^T + x2(strided) . W2^T + bias): a torchvision bottleneck's
// conv3 and its downsample branch (networks/DescNet.py:29-35, the encoder's
// first block of each stage) as ONE GEMM over K = k1 + k2 -- the downsample
// output never crosses HBM (it was written, then re-read as conv3's residual).
// x1: [n][oh][ow] rows of k1 channels (pitch x1cs); x2: [n][h2][w2] rows of k2
// channels (pitch x2cs) read at (oh * s2, ow * s2); wb: three bf16 planes of
// the [cout][k1 + k2] weights (plane stride wplane); bias: the summed biases.
// k1, k2 % 32 == 0, cout % 128 == 0.
int pf_conv_dual(int n, int oh, int ow, const float* x1, int x1cs, int k1, const float* x2,
                 int x2cs, int h2, int w2, int s2, int k2, int cout,
                 const unsigned short* wb, long long wplane, const float* bias, int act, float* y,
                 int ycs, hipStream_t st) {
  if (k1 <= 0 || k2 <= 0 || k1 % BK || k2 % BK || cout % 128 || !x2 || !wb || s2 < 1 ||
      (oh - 1) * s2 >= h2 || (ow - 1) * s2 >= w2 || x2cs % 4 || (reinterpret_cast<uintptr_t>(x2) & 15))
    return POSFEAT_E_INVALID;
  posfeat_conv_desc d{};
  d.n = n;
  d.h = oh;
  d.w = ow;
  d.cin = k1 + k2;
  d.x_cstride = std::max(x1cs, k1 + k2);  // (conv_prepare's one-source check; x1's pitch below)
  d.cout = cout;
  d.kh = d.kw = 1;
  d.stride = 1;
  d.pad = 0;
  d.y_cstride = ycs;
  d.res_cstride = 0;
  d.act = act;
  ConvArgs a;
  if (x1cs < k1 || x1cs % 4) return POSFEAT_E_INVALID;
  PF_TRY(conv_prepare(&d, x1, bias, bias, nullptr, y, a));
  a.xcs = x1cs;
  a.wb = wb;
  a.wplane = wplane;
  a.x2 = x2;
  a.x2cs = x2cs;
  a.k1ch = k1 / BK;
  a.H2 = h2;
  a.W2 = w2;
  a.s2 = s2;
  Plan p = plan_for_tile(a, TILE_BF6X_128x128);
  if (p.kern < 0) return POSFEAT_E_INVALID;
  return conv_run(a, p, st);
}

// GEMMs on the weight-stationary persistent kernel (gemm_ws_kernel):
// y [M][ldc] = act(x [M][lda] . W^T + bias (+ res)), W as three bf16 planes
// [3][N][K] (plane stride wplane, row pitch K).  Instantiated shapes: head.conv2's
// tap GEMM (K = 192, N % 128 == 0) and the short-K 1x1 convs (pf_ws_gemm_ok);
// POSFEAT_E_UNSUPPORTED for another K / N.
static bool ws_shape(int K, int N, int* kc, int* nb) {
  *kc = K / BK;
  if (K % BK) return false;
  // the resident planes must fit the CU's LDS: 3 x BN x K bf16
  if (K == 192 && N % 128 == 0) { *nb = 8; return true; }
  if ((K == 64 || K == 128) && N % 128 == 0) { *nb = 8; return true; }
  if (K == 256 && N % 64 == 0) { *nb = 4; return true; }
  return false;
}
bool pf_ws_gemm_ok(int K, int N) {
  int kc, nb;
  return ws_shape(K, N, &kc, &nb);
}
int pf_gemm_ws(const float* x, int lda, int M, int K, const unsigned short* wb, long long wplane,
               int N, const float* bias, const float* res, int rcs, int act, float* y, int ldc,
               hipStream_t st) {
  int kc = 0, nbk = 0;
  if (!ws_shape(K, N, &kc, &nbk)) return POSFEAT_E_UNSUPPORTED;
  const int bn = 16 * nbk;
  // (16-B A loads and weight-plane loads: aligned bases)
  if (!x || !wb || !y || M <= 0 || lda < K || ldc < N || lda % 4 || (res && rcs < N) ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wb)) & 15) || wplane % 8)
    return POSFEAT_E_INVALID;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return POSFEAT_E_HIP;
  static const int pd = [] {  // A/B: POSFEAT_TAPWS_PD=2 (three A buffers; the tap GEMM)
    const char* e = pf_ab_getenv("POSFEAT_TAPWS_PD");
    return e && e[0] == '2' ? 2 : 1;
  }();
  static const int nw0 = [] {  // twelve waves: three per SIMD (A/B: POSFEAT_TAPWS_NW=8)
    const char* e = pf_ab_getenv("POSFEAT_TAPWS_NW");
    return e && atoi(e) == 8 ? 8 : 12;
  }();
  const bool tap = kc == 6 && nbk == 8;  // (the tap GEMM: no epilogue)
  if (tap && (bias || res || act != POSFEAT_ACT_NONE)) return POSFEAT_E_UNSUPPORTED;
  const int nw = tap ? nw0 : 12;
  const int bm = nw * 32;
  const int ntn = N / bn, ntm = (M + bm - 1) / bm;
  const int per_n = std::max(1, std::min(ntm, ncu / std::max(1, std::min(ntn, ncu))));
  static const int abl = [] {
    const char* e = pf_ab_getenv("POSFEAT_TAPWS_ABL");
    return e ? atoi(e) : 0;
  }();
  WsArgs a{x, wb, y, wplane, lda, ldc, M, N, per_n, abl, bias, res, rcs, act};
  a.kpad = K;
  const dim3 grid((unsigned)(per_n * ntn));
  if (tap && pd == 2)
    hipLaunchKernelGGL((gemm_ws_kernel<2, 8, 6, 8>), grid, dim3(8 * 64), 0, st, a);
  else if (tap && nw == 8)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 8, 6, 8>), grid, dim3(8 * 64), 0, st, a);
  else if (tap)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 6, 8>), grid, dim3(12 * 64), 0, st, a);
  else if (kc == 2 && res)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 2, 8, 2>), grid, dim3(12 * 64), 0, st, a);
  else if (kc == 2)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 2, 8, 1>), grid, dim3(12 * 64), 0, st, a);
  else if (kc == 4 && res)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 4, 8, 2>), grid, dim3(12 * 64), 0, st, a);
  else if (kc == 4)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 4, 8, 1>), grid, dim3(12 * 64), 0, st, a);
  else if (res)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 8, 4, 2>), grid, dim3(12 * 64), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 8, 4, 1>), grid, dim3(12 * 64), 0, st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(PF_ARITH_BF6);
  return POSFEAT_OK;
}
// the stem (7x7 stride-s conv of a 4-channel NHWC image, weights [N][kpad]
// with kpad = 224: the G4 K order) on the weight-stationary kernel: eight
// chunks resident (the eighth zero), N = 64, bias + activation epilogue
int pf_gemm_ws_stem(const float* x, int n, int H, int W, int OH, int OW, int stride, int pad,
                    const unsigned short* wb, long long wplane, int kpad, int N, const float* bias,
                    int act, float* y, int ldc, hipStream_t st) {
  if (N != 64 || kpad != 224 || !x || !wb || !y || n <= 0 || OH <= 0 || OW <= 0 || ldc < N ||
      (OH - 1) * stride - pad >= H || (OW - 1) * stride - pad >= W || wplane % 8 ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(wb)) & 15))
    return POSFEAT_E_UNSUPPORTED;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return POSFEAT_E_HIP;
  const float* zero = conv_zero_ptr();
  if (!zero) return POSFEAT_E_HIP;
  const int M = n * OH * OW, bm = 12 * 32, ntm = (M + bm - 1) / bm;
  const int per_n = std::max(1, std::min(ntm, ncu));
  WsArgs a{x, wb, y, wplane, 4, ldc, M, N, per_n, 0, bias, nullptr, 0, act};
  a.kpad = kpad;
  a.H = H;
  a.W = W;
  a.OW = OW;
  a.ohw = OH * OW;
  a.stride = stride;
  a.pad = pad;
  a.zero = zero;
  hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 8, 4, 1, 1>), dim3((unsigned)per_n), dim3(12 * 64), 0,
                     st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(PF_ARITH_BF6);
  return POSFEAT_OK;
}

// batched short-K GEMMs on the weight-stationary kernel, one GEMM per grid.y:
// head.conv1's F(6x6) transform-domain GEMMs (K = N = 192: 96-column tiles,
// 110 KB of planes per block), layer2's (K = N = 128: one 128-column
// tile) and layer3's (K = N = 256: 64-column tiles) -- the same sums as the
// bf6x tiles
static int ws_batched_cfg(int K, int N, int* nbk) {
  if (K == 192 && N % 96 == 0 && N <= 192) return *nbk = 6, 6;
  if (K == 128 && N % 128 == 0) return *nbk = 8, 4;
  if (K == 256 && N % 64 == 0) return *nbk = 4, 8;
  return 0;
}
bool pf_gemm_ws_batched_ok(int K, int N) {
  int nbk = 0;
  return ws_batched_cfg(K, N, &nbk) != 0;
}
int pf_gemm_ws_batched(const float* A, int lda, long long sa, const unsigned short* Bb,
                       long long bplane, long long sb, float* C, int ldc, long long sc, int nb,
                       int M, int N, int K, hipStream_t st) {
  if (!pf_gemm_ws_batched_ok(K, N) || !A || !Bb || !C || M <= 0 || nb < 1 || nb > 65535 ||
      lda < K || lda % 4 || ldc < N || sa % 4 || sb % 8 || bplane % 8 ||
      ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(Bb)) & 15))
    return POSFEAT_E_UNSUPPORTED;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return POSFEAT_E_HIP;
  int nbk = 0;
  const int kc = ws_batched_cfg(K, N, &nbk);
  const int bm = 12 * 32, ntn = N / (16 * nbk), ntm = (M + bm - 1) / bm;
  const int per_n = std::max(1, std::min(ntm, ncu / std::max(1, ntn * nb)));
  WsArgs a{A, Bb, C, bplane, lda, ldc, M, N, per_n, 0, nullptr, nullptr, 0, POSFEAT_ACT_NONE};
  a.kpad = K;
  a.bx = sa;
  a.by = sc;
  a.bwb = sb;
  const dim3 grid((unsigned)(per_n * ntn), (unsigned)nb);
  if (kc == 6)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 6, 6>), grid, dim3(12 * 64), 0, st, a);
  else if (kc == 4)
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 4, 8>), grid, dim3(12 * 64), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_ws_kernel<1, 12, 8, 4>), grid, dim3(12 * 64), 0, st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(PF_ARITH_BF6);
  return POSFEAT_OK;
}

int pf_tap_gemm_ws(const float* x, int lda, int M, const unsigned short* wb, long long wplane,
                   int N, float* y, int ldc, hipStream_t st) {
  return pf_gemm_ws(x, lda, M, 192, wb, wplane, N, nullptr, nullptr, 0, POSFEAT_ACT_NONE, y, ldc,
                    st);
}

// pf_conv_run_tile for a dense 1x1 GEMM whose A is normalised on load
// (ConvArgs amean / arstd / aslope: x's per-image channel mean / rstd, the
// PReLU slope): head.conv2's tap GEMM straight from conv1's raw output, the
// normalised L never written.  Only the 128 x 128 bf6x tile carries it
// (POSFEAT_E_UNSUPPORTED otherwise: the caller normalises and runs the plain
// GEMM).  Bit-identical to in_apply + the plain GEMM.
int pf_conv_run_tile_np(const posfeat_conv_desc* d, const float* x, const float* w,
                        float* y, int tile, hipStream_t st, const unsigned short* wb,
                        long long wplane, const float* mean, const float* rstd,
                        const float* slope) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, nullptr, nullptr, y, a));
  if (!wb || !mean || !rstd || !slope || a.Kpad > 256 || d->cin != a.Kpad) return POSFEAT_E_INVALID;
  a.wb = wb;
  a.wplane = wplane;
  const Plan p = conv_plan(a, false, tile);
  if (p.tile != TILE_BF6X_128x128 || p.ksplit != 1 || !dense_gemm(a) || bf6x_bm192())
    return POSFEAT_E_UNSUPPORTED;
  a.amean = mean;
  a.arstd = rstd;
  a.aslope = slope;
  return conv_run(a, p, st);
}

extern "C" int posfeat_conv1x1_dual(int n, int oh, int ow, const float* x1, int x1cs, int k1,
                                    const float* x2, int x2cs, int h2, int w2, int s2, int k2,
                                    int cout, const unsigned short* wb, const float* bias,
                                    int act, float* y, int ycs, void* stream) {
  if (!bias) return POSFEAT_E_INVALID;
  return pf_conv_dual(n, oh, ow, x1, x1cs, k1, x2, x2cs, h2, w2, s2, k2, cout, wb,
                      (long long)cout * (k1 + k2), bias, act, y, ycs, pf_stream(stream));
}

namespace {
__global__ void dual_weights_kernel(const unsigned short* __restrict__ w1, int k1,
                                    const unsigned short* __restrict__ w2, int k2, long long sp,
                                    int cout, const float* __restrict__ b1,
                                    const float* __restrict__ b2, unsigned short* __restrict__ dst,
                                    float* __restrict__ bdst) {
  const int kc = k1 + k2;
  const long long per = (long long)cout * kc, total = 3 * per;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int pl = (int)(i / per);
    const long long r = i - pl * per;
    const int co = (int)(r / kc), k = (int)(r - (long long)co * kc);
    dst[i] = k < k1 ? w1[pl * sp + (long long)co * k1 + k] : w2[pl * sp + (long long)co * k2 + k - k1];
  }
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < cout; c += blockDim.x) bdst[c] = b1[c] + b2[c];
}
}  // namespace

int pf_dual_weights(const unsigned short* w1, int k1, const unsigned short* w2, int k2,
                    long long sp, int cout, const float* b1, const float* b2,
                    unsigned short* dst, float* bdst, hipStream_t st) {
  if (!w1 || !w2 || !dst || !b1 || !b2 || !bdst || k1 <= 0 || k2 <= 0 || cout <= 0)
    return POSFEAT_E_INVALID;
  const long long total = 3LL * cout * (k1 + k2);
  hipLaunchKernelGGL(dual_weights_kernel, dim3((unsigned)std::min<long long>((total + 255) / 256, 4096)),
                     dim3(256), 0, st, w1, k1, w2, k2, sp, cout, b1, b2, dst, bdst);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// pf_conv_run_tile with the train-mode BatchNorm partial sums of y from the
// epilogue (bbtrain.hip layer_fwd): part[tile][2][Cout] fp64 (sum, sum of
// squares over the tile's pixels of every image; the layout of
// bn_partial_kernel<0>'s chunks, which bn_stats_final_kernel / bn_sums_kernel
// reduce), *nparts = the tile count.  A split-K plan (raw partials: the reduce
// writes y) or a part buffer too small for the plan's tiles runs the plain
// conv with *nparts = 0: the caller then takes the statistics pass.
int pf_conv_run_tile_bn(const posfeat_conv_desc* d, const float* x, const float* w,
                        const float* bias, float* y, void* ws, size_t ws_bytes, int tile,
                        hipStream_t st, const unsigned short* wb, long long wplane, double* part,
                        size_t part_bytes, int* nparts) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, nullptr, y, a));
  if (!nparts) return POSFEAT_E_INVALID;
  *nparts = 0;
  a.wb = wb;
  a.wplane = wplane;
  const size_t need = posfeat_conv2d_workspace(d);
  const bool split = need > 0 && ws && ws_bytes >= need;
  const Plan p = conv_plan(a, split, tile);
  if (p.ksplit > 1) {
    a.part = static_cast<float*>(ws);
  } else if (part && p.tiles_m * 2 * (size_t)a.Cout * sizeof(double) <= part_bytes &&
             p.tiles_m <= 0x7fffffff &&
             !(p.tile >= TILE_BF6X_128x128 && p.tile <= TILE_BF6X_256x64)) {
    a.bnpart = part;
    *nparts = (int)p.tiles_m;
  }
  const int rc = conv_run(a, p, st);
  if (rc != POSFEAT_OK) *nparts = 0;
  return rc;
}

static size_t stats_ws_for(const ConvArgs& a, const Plan& p, int n) {
  if (p.ppi == 0 && a.hw < p.bm) return 0;
  const size_t nchunk = (stats_tiles_per_img(a, p) + STAT_CHUNK - 1) / STAT_CHUNK;
  return pf_align((size_t)p.tiles_m * 2 * a.Cout * 2 * sizeof(float), 256) +
         (size_t)n * nchunk * a.Cout * 2 * sizeof(double);
}

size_t pf_conv_stats_ws_max(const posfeat_conv_desc* d) {
  ConvArgs a;
  float dummy[4] __attribute__((aligned(16)));
  if (conv_prepare(d, dummy, dummy, nullptr, nullptr, dummy, a) != POSFEAT_OK) return 0;
  size_t mx = 0;
  for (int t : kAllTiles) {
    const Plan p = plan_for_tile(a, t);
    if (p.kern < 0) continue;
    const size_t s = stats_ws_for(a, p, d->n);
    if (s > mx) mx = s;
  }
  return mx;
}

int pf_conv_stats_run_tile(const posfeat_conv_desc* d, const float* x, const float* w,
                           const float* bias, float* y, void* ws, size_t ws_bytes, float* mean,
                           float* rstd, float eps, int tile, hipStream_t st,
                           const unsigned short* wb, long long wplane) {
  ConvArgs a;
  PF_TRY(conv_prepare(d, x, w, bias, nullptr, y, a));
  a.wb = wb;
  a.wplane = wplane;
  const Plan p = conv_plan(a, false, tile);
  const size_t need = stats_ws_for(a, p, d->n);
  if (need == 0) return POSFEAT_E_UNSUPPORTED;
  if (!ws || ws_bytes < need || !mean || !rstd) return POSFEAT_E_WORKSPACE;
  a.stats = static_cast<float*>(ws);
  PF_TRY(conv_run(a, p, st));
  const int nb = d->n;
  const int nchunk = (int)((stats_tiles_per_img(a, p) + STAT_CHUNK - 1) / STAT_CHUNK);
  double* chunks = reinterpret_cast<double*>(
      static_cast<char*>(ws) + pf_align((size_t)p.tiles_m * 2 * a.Cout * 2 * sizeof(float), 256));
  hipLaunchKernelGGL(conv_stats_chunk, dim3(nchunk, (a.Cout + 63) / 64, nb), dim3(1024), 0, st,
                     a.stats, p.bm, p.ppi, a.hw, a.Cout, nchunk, chunks);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(conv_stats_finalize, dim3((nb * a.Cout + 255) / 256), dim3(256), 0, st,
                     chunks, nchunk, a.hw, a.Cout, nb, eps, mean, rstd, nullptr, 0);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// ---------------------------------------------------------------------------
// head.conv2 by bilinear phases (see conv_up4_kernel).
static int up4_nbp(int H, int W) { return 2 * W + 2 * (H - 2); }
static int up4_ppi(int H, int W) { return ((W / 4 + 15) / 16) * ((H / 4 + 7) / 8); }
static const size_t UP4_WPH_FLOATS = (size_t)16 * UP4_COUT * UP4_KP +
                                     (size_t)9 * UP4_CU * UP4_COUT + (size_t)UP4_COUT * UP4_GK;

struct Up4Ws {
  size_t stats, chunks, total;
  int nch;
};

static Up4Ws up4_layout(int n, int H, int W) {
  Up4Ws L{};
  const int ppi = up4_ppi(H, W);
  L.nch = (16 * ppi + STAT_CHUNK - 1) / STAT_CHUNK;
  size_t cur = 0;
  auto take = [&](size_t bytes) {
    const size_t at = cur;
    cur += pf_align(bytes, 256);
    return at;
  };
  L.stats = take((size_t)n * ppi * 16 * 2 * UP4_COUT * 2 * sizeof(float));
  L.chunks = take((size_t)n * L.nch * UP4_COUT * 2 * sizeof(double));
  L.total = cur;
  return L;
}

extern "C" size_t posfeat_conv2_up4_weights_floats(void) { return UP4_WPH_FLOATS; }

extern "C" size_t posfeat_conv2_up4_workspace(int n, int H, int W) {
  if (n <= 0 || H < 16 || W < 16 || H % 4 || W % 4) return 0;
  return up4_layout(n, H, W).total;
}

extern "C" int posfeat_conv2_up4_weights(const float* w_packed, float* wph, void* stream) {
  if (!w_packed || !wph) return POSFEAT_E_INVALID;
  launch_up4_weights(w_packed, wph, pf_stream(stream));
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// The three steps (also sequenced and timed one by one by engine.hip).
int pf_up4_gconv(int n, int H, int W, const float* G, int gcs, const float* wph,
                 const float* bias, float* y, int ycs, hipStream_t st) {
  const float* wg = wph + (size_t)16 * UP4_COUT * UP4_KP + (size_t)9 * UP4_CU * UP4_COUT;
  posfeat_conv_desc d{};
  d.n = n;
  d.h = H;
  d.w = W;
  d.cin = UP4_CG;
  d.x_cstride = gcs;
  d.cout = UP4_COUT;
  d.kh = 3;
  d.kw = 3;
  d.stride = 1;
  d.pad = 1;
  d.y_cstride = ycs;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  ConvArgs g;
  PF_TRY(conv_prepare(&d, G, wg, bias, nullptr, y, g));
  return conv_run(g, conv_plan(g, false), st);
}

int pf_up4_border(int n, int H, int W, const float* L, int lcs, const float* wph, float* y,
                  int ycs, hipStream_t st) {
  const int ncb = 2 * ((W + UP4_CPB - 1) / UP4_CPB) + 2 * ((H - 2 + UP4_CPB - 1) / UP4_CPB);
  hipLaunchKernelGGL(up4_border_corr_kernel, dim3(ncb, n), dim3(2 * UP4_COUT), 0, st, L, lcs,
                     H / 4, W / 4, H, W, up4_nbp(H, W), wph + (size_t)16 * UP4_COUT * UP4_KP, y,
                     ycs);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_up4_main(int n, int H, int W, const float* L, int lcs, const float* wph, float* y, int ycs,
                void* ws, size_t ws_bytes, float* mean, float* rstd, float eps, hipStream_t st) {
  const Up4Ws lay = up4_layout(n, H, W);
  if (!ws || ws_bytes < lay.total) return POSFEAT_E_WORKSPACE;
  char* base = static_cast<char*>(ws);
  const int ppi = up4_ppi(H, W);
  ConvArgs a{};
  a.x = L;
  a.xcs = lcs;
  a.w = wph;
  a.bias = nullptr;
  a.res = nullptr;
  a.y = y;
  a.ycs = ycs;
  a.H = H;
  a.W = W;
  a.OH = H;
  a.OW = W;
  a.lh = H / 4;
  a.lw = W / 4;
  a.Cin = UP4_CU;
  a.Cout = UP4_COUT;
  a.M = n * H * W;
  a.hw = H * W;
  a.act = POSFEAT_ACT_NONE;
  a.ksplit = 1;
  a.tiles_n = 1;
  a.nwg = n * ppi * 16;
  a.stats = reinterpret_cast<float*>(base + lay.stats);
  launch_up4(a, st);
  PF_CHECK_LAUNCH();
  double* ch = reinterpret_cast<double*>(base + lay.chunks);
  hipLaunchKernelGGL(conv_stats_chunk, dim3(lay.nch, UP4_COUT / 64, n), dim3(1024), 0, st,
                     a.stats, 128, 16 * ppi, a.hw, UP4_COUT, lay.nch, ch);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(conv_stats_finalize, dim3((n * UP4_COUT + 255) / 256), dim3(256), 0, st, ch,
                     lay.nch, H * W, UP4_COUT, n, eps, mean, rstd, nullptr, 0);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_conv2_up4(int n, int H, int W, const float* L, int lcs, const float* G,
                                 int gcs, const float* wph, const float* w_packed,
                                 const float* bias, float* y, int ycs, void* ws, size_t ws_bytes,
                                 float* mean, float* rstd, float eps, void* stream) {
  (void)w_packed;  // folded into wph (phase weights, border taps, G conv)
  if (n <= 0 || H < 16 || W < 16 || H % 4 || W % 4 || !L || !G || !wph || !y || !mean || !rstd)
    return POSFEAT_E_INVALID;
  if (lcs < UP4_CU || lcs % 4 || gcs < UP4_CG || gcs % 4 || ycs < UP4_COUT || ycs % 4)
    return POSFEAT_E_INVALID;
  const uintptr_t al = reinterpret_cast<uintptr_t>(L) | reinterpret_cast<uintptr_t>(G) |
                       reinterpret_cast<uintptr_t>(wph) | reinterpret_cast<uintptr_t>(y) |
                       reinterpret_cast<uintptr_t>(bias);
  if (al & 15) return POSFEAT_E_INVALID;
  hipStream_t st = pf_stream(stream);
  // 1. y = conv3x3(G, W[:, 192:]) + bias  (full-res halo kernel)
  PF_TRY(pf_up4_gconv(n, H, W, G, gcs, wph, bias, y, ycs, st));
  // 2. border lines: remove the taps that fall into conv2's zero padding
  PF_TRY(pf_up4_border(n, H, W, L, lcs, wph, y, ycs, st));
  // 3. the 192 upsampled channels by phases, + y, IN statistics
  return pf_up4_main(n, H, W, L, lcs, wph, y, ycs, ws, ws_bytes, mean, rstd, eps, st);
}

// C[z] [M][N] = A[z] [M][K] (row pitch lda) x B[z]^T, B[z] packed [N][K] (K % 32
// == 0, the 1x1-conv weight layout), z < nb: ONE launch of conv_glds_kernel with
// blockIdx.y = z (Winograd's 16 transform-domain GEMMs, wino.hip).
// The batched GEMMs with BOTH operands pre-split into three bf16 planes
// (conv precision mode 2): A [nb][M][lda] planes at Ab + p * pa, batch
// stride sa; B as pf_gemm_batched's Bb.  conv_bf6s_kernel, 128x128 tiles (or
// 128x64 where N % 128 != 0).  Replaces round 2's LDS-staged gemm6 kernel.
int pf_gemm_batched_pre(const unsigned short* Ab, int lda, long long pa, long long sa,
                        const unsigned short* Bb, long long bplane, long long sb, float* C, int ldc,
                        long long sc, int nb, int M, int N, int K, hipStream_t st) {
  if (K % BK || N % 64 || nb < 1 || lda % 8 || !Ab || !Bb) return POSFEAT_E_INVALID;
  posfeat_conv_desc d;
  d.n = 1;
  d.h = 1;
  d.w = M;
  d.cin = K;
  d.x_cstride = lda;
  d.cout = N;
  d.kh = d.kw = 1;
  d.stride = 1;
  d.pad = 0;
  d.y_cstride = ldc;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  ConvArgs a;
  // x / w are never read (A and B come as planes); any non-null pointers
  PF_TRY(conv_prepare(&d, reinterpret_cast<const float*>(Ab), reinterpret_cast<const float*>(Bb),
                      nullptr, nullptr, C, a));
  a.wb = Bb;
  a.wplane = bplane;
  a.xb = Ab;
  a.xplane = pa;
  const Plan p = conv_plan(a, false, N % 128 == 0 ? TILE_BF6B_128x128 : TILE_BF6B_128x64);
  if (p.tile != TILE_BF6B_128x128 && p.tile != TILE_BF6B_128x64) return POSFEAT_E_UNSUPPORTED;
  a.nbatch = nb;
  a.bxb = sa;
  a.bwb = sb;
  a.by = sc;
  return conv_run(a, p, st);
}

int pf_gemm_batched(const float* A, int lda, long long sa, const float* B, long long sb, float* C,
                    int ldc, long long sc, int nb, int M, int N, int K, hipStream_t st,
                    const unsigned short* Bb, long long bplane) {
  if (K % BK || N % 4 || nb < 1) return POSFEAT_E_INVALID;
  // the short-K batched GEMMs on the weight-stationary kernel: head.conv1's
  // (K = 192), layer2's and layer3's conv2 (K = 128, 256) Winograd GEMMs
  // (r16zz4, B = 32, two runs: 0.628 -> 0.484, 0.087 -> 0.076, 0.078 -> 0.070
  // ms; bit-identical).  A/B POSFEAT_WSB: 0 off, 1 K = 192 only, 2 K <= 192
  static const int wsb = [] {
    const char* e = pf_ab_getenv("POSFEAT_WSB");
    return e ? atoi(e) : 3;
  }();
  if (wsb && Bb && bf6x_on() && pf_gemm_ws_batched_ok(K, N) && lda % 4 == 0 &&
      (K == 192 || (K == 128 && wsb >= 2) || (K == 256 && wsb >= 3))) {
    const int r = pf_gemm_ws_batched(A, lda, sa, Bb, bplane, sb, C, ldc, sc, nb, M, N, K, st);
    if (r != POSFEAT_E_UNSUPPORTED) return r;  // (else: the bf6x tiles below)
  }
  posfeat_conv_desc d;
  d.n = 1;
  d.h = 1;
  d.w = M;
  d.cin = K;
  d.x_cstride = lda;
  d.cout = N;
  d.kh = d.kw = 1;
  d.stride = 1;
  d.pad = 0;
  d.y_cstride = ldc;
  d.res_cstride = 0;
  d.act = POSFEAT_ACT_NONE;
  ConvArgs a;
  PF_TRY(conv_prepare(&d, A, B, nullptr, nullptr, C, a));
  a.wb = Bb;  // B as three bf16 planes (plane stride bplane, batch stride sb)
  a.wplane = bplane;
  // the heuristic sizes tiles for ONE GEMM; with nb of them in the grid the
  // 128x128 tile (2x the operand reuse of 64x64) still fills the chip
  const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128) * nb;
  // N = 192 (head.conv1's Winograd GEMMs) on pre-split planes: three 64-wide
  // column tiles instead of two 128-wide ones, the second of them half empty
  // POSFEAT_GEMM_B256=1 (A/B): the 8-wave 256x128 pre-split tiles
  static const bool b256 = [] {
    const char* e = pf_ab_getenv("POSFEAT_GEMM_B256");
    return e && e[0] == '1';
  }();
  // POSFEAT_TRAIN_WINO_BF6X=1 (A/B, off): the train-mode backbone's batched
  // (Winograd decoder) GEMMs on the 16x16x32 tiles too, its halo scope lifted
  // for them.  The fp64 fixture step's per-tensor errors unchanged to the
  // digits shown; same-box train_desc +0.5..2 % over four pairs, but the
  // four decoder GEMM launches 1704 us (32x32x16, r15e) vs 1718 us (16x16x32,
  // r15j) per set and the per-label breakdown flat: not the
  // default.
  static const bool twx = [] {
    const char* e = pf_ab_getenv("POSFEAT_TRAIN_WINO_BF6X");
    return e && e[0] == '1';
  }();
  struct HaloLift {  // the calling thread's halo scope lifted for this call
    int saved;
    bool on;
    explicit HaloLift(bool o) : saved(tl_halo_fp32), on(o) {
      if (on) tl_halo_fp32 = 0;
    }
    ~HaloLift() {
      if (on) tl_halo_fp32 = saved;
    }
  } const lift(twx && Bb);
  const bool x = Bb && bf6x_on();
  // POSFEAT_BF6X_RB4=1 (A/B): the 256-row 16x16x32 tiles for the batched GEMMs
  static const bool rb4 = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6X_RB4");
    return e && e[0] == '1';
  }();
  // N = 192 (head.conv1): one 192-wide column tile reads A once (three
  // 64-wide tiles read it three times)
  // POSFEAT_BF6X_N256=1 (A/B): one 256-wide column tile for N % 256 == 0
  // (the decoder's Winograd GEMMs: A read once per 256 columns, not twice)
  static const bool n256 = [] {
    const char* e = pf_ab_getenv("POSFEAT_BF6X_N256");
    return e && e[0] == '1';
  }();
  const int want = x ? (n256 && N % 256 == 0 ? TILE_BF6X_128x256
                        : N % 128 == 0 ? (rb4 ? TILE_BF6X_256x128 : TILE_BF6X_128x128)
                        : N % 192 == 0 ? TILE_BF6X_128x192
                                       : TILE_BF6X_128x64)
                   : (Bb && b256 && N % 128 == 0) ? TILE_BF6B_256x128
                   : (N % 128 == 0 && t128 >= 1024) ? TILE_128x128
                   : (Bb && N % 128 != 0 && N % 64 == 0) ? TILE_BF6B_128x64
                                                                 : -1;
  const Plan p = conv_plan(a, false, want);
  if (p.kern != KERN_GLDS) return POSFEAT_E_UNSUPPORTED;
  a.nbatch = nb;
  a.bx = sa;
  a.bw = sb;
  a.bwb = sb;
  a.by = sc;
  return conv_run(a, p, st);
}


int& pf_arith_mask() {
  static thread_local int m = 0;
  return m;
}
