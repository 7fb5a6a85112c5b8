// train.hip -- backward kernels of the keypoint-head training step on gfx950.
//
// Config 5 of BASELINE.json (configs/train_kp.yaml): only `localheader`
// (KeypointDet, networks/DeteNet.py:9-121) is optimised (train_kp.yaml:11-13,
// SGD lr 1e-3); the backbone output is detached (PoSFeat_model.py:97-102) and
// the loss is DiskLoss (losses/kploss.py:132-197).  The reference gets these
// gradients from autograd over ATen (managers/trainer.py:330-331); here each
// adjoint is an explicit gfx950 kernel:
//
//   conv_wgrad_kernel     dW[co][k] = sum_p dy[p][co] * im2col(x)[p][k]  (FP32 MFMA,
//                         K in the engine's packed order so dW lands in the
//                         weight blob's layout; pixel-split partials summed in a
//                         fixed order -> deterministic), + db[co] = sum_p dy
//   dgrad_weights_kernel  W'[ci][(co/32, kh', kw', co%32)] = W[co][flip][ci]: the
//                         input gradient is then an ordinary forward conv
//                         (conv.hip) of dy with W'
//   up4_adj_x/y_kernel    adjoint of F.interpolate(x4, bilinear,
//                         align_corners=False) (DeteNet.py:109), separable gather
//   in_bwd_*              InstanceNorm2d (affine=False, biased var) backward,
//                         optionally through the shared PReLU (DeteNet.py:108,112)
//   tail_bwd_*            Softplus(IN(conv3(PReLU(IN(conv2))))) backward
//                         (DeteNet.py:112-113) down to d(conv2 output)
//   sgd_kernel            torch.optim.SGD step (no momentum / weight decay)
#include <algorithm>

#include "common.h"
#include "fmap.h"
#include "train.h"

namespace {

constexpr int WG_RB = 32;  // pixels per reduction chunk

struct WgradArgs {
  const float* dy;
  int ldy;
  const float* x;
  int xcs;
  int H, W, Cin, KH, KW, pad;  // H, W: dy (output) dims
  int Hin, Win, stride;         // input dims and conv stride (halo kernel: stride 1)
  long long d_row, d_img;       // x offset corrections when a pixel walk wraps a row / image
  int Cout, Kpad, K, M;
  int tiles_n, ntiles, nsplit, nchunks;
  // batched 1x1 use (Winograd weight gradient): blockIdx.y = z selects
  // dy/x/part + z * stride; only batch zb writes the bias partial
  long long bdy, bx, bpart;
  int zb;
  float* part;   // [nsplit][Cout][Kpad]
  float* partb;  // [nsplit][Cout] or nullptr
};

__device__ __attribute__((aligned(16))) float pf_wg_zero16[4];

// One 256-thread workgroup computes a BM x BN tile of dW over one pixel range.
// Per 32-pixel chunk both operands are DMA'd (global_load_lds_dwordx4) into LDS
// rows [pixel][channel]: A = dy rows (couts), B = the im2col rows (packed k).
// The MFMA reduction index is the pixel: lane l feeds A[co = l%32][px = l/32]
// and B[px = l/32][k = l%32] with ds_read_b32 (32 consecutive dwords per lane
// group: conflict-free).  Two LDS stages: chunk c+1 is in flight while chunk c
// is multiplied.
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int WN = 2;
  constexpr int TM = BM / 2, TN = BN / WN;
  constexpr int MI = TM / 32, NI = TN / 32;
  constexpr int A_G = BM / 32, B_G = BN / 32;  // DMA wave-instructions per chunk per wave
  static_assert(MI >= 1 && NI >= 1, "tile");
  __shared__ __attribute__((aligned(16))) float smem[2 * WG_RB * (BM + BN)];
  float* As = smem;                    // [2][32][BM]
  float* Bs = smem + 2 * WG_RB * BM;   // [2][32][BN]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int bid = blockIdx.x;
  {  // XCD-aware bijective remap: consecutive logical ids share an XCD's L2, so
     // the tiles of one pixel range (same dy rows, same input pixels) do too
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int split = bid / a.ntiles, tile = bid - split * a.ntiles;
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  if (gridDim.y > 1) {
    const long long z = blockIdx.y;
    a.dy += z * a.bdy;
    a.x += z * a.bx;
    a.part += z * a.bpart;
    if ((int)z != a.zb) a.partb = nullptr;
  }
  const int c_begin = (int)((long long)a.nchunks * split / a.nsplit);
  const int c_end = (int)((long long)a.nchunks * (split + 1) / a.nsplit);

  // ---- per-lane DMA roles (fixed across chunks) ----------------------------
  // A: instruction i of this wave covers stage bytes [(wave*A_G+i)*1024, +1024)
  int a_row[A_G], a_col[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int e = ((wave * A_G + i) * 1024 + lane * 16) / 4;  // float index in the stage
    a_row[i] = e / BM;
    a_col[i] = e - a_row[i] * BM;
  }
  // B: row (pixel in chunk), k column -> (kh-pad, kw-pad, ci)
  int b_row[B_G], b_dy[B_G], b_dx[B_G], b_ci[B_G];
  bool b_kok[B_G];
  const int ntap = a.KH * a.KW;
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int e = ((wave * B_G + i) * 1024 + lane * 16) / 4;
    b_row[i] = e / BN;
    const int k = n0 + (e - b_row[i] * BN);
    int tap, ci;
    bool ok;
    if ((a.Cin & 31) == 0) {
      const int c = k >> 5, slab = c / ntap;
      tap = c - slab * ntap;
      ci = slab * 32 + (k & 31);
      ok = k < a.Kpad;
    } else {  // Cin == 4: K = (kh, kw, cin4), zero-padded to Kpad
      tap = k >> 2;
      ci = 0;
      ok = k < a.K;
    }
    b_kok[i] = ok;
    b_dy[i] = ok ? tap / a.KW - a.pad : 0;
    b_dx[i] = ok ? tap - (tap / a.KW) * a.KW - a.pad : 0;
    b_ci[i] = ci;
  }
  // Pixel of each B slot tracked incrementally (chunks of one workgroup are
  // consecutive): no integer division in the loop.  bp = element offset of
  // the tap's source pixel (+ channel) from x, valid iff in the image; output
  // pixel (oh, ow) reads input (s*oh + dy, s*ow + dx).
  const int HW = a.H * a.W, s = a.stride;
  int b_oh[B_G], b_ow[B_G];
  long long b_ptr[B_G];
  {
    const long long m0 = (long long)c_begin * WG_RB;
#pragma unroll
    for (int i = 0; i < B_G; ++i) {
      const long long m = m0 + b_row[i];
      const long long img = m / HW, rem = m - img * HW;
      b_oh[i] = (int)(rem / a.W);
      b_ow[i] = (int)(rem - (long long)b_oh[i] * a.W);
      b_ptr[i] = ((img * a.Hin + s * b_oh[i] + b_dy[i]) * a.Win + s * b_ow[i] + b_dx[i]) * a.xcs +
                 b_ci[i];
    }
  }
  const long long a_step = (long long)WG_RB * a.ldy, b_step = (long long)WG_RB * s * a.xcs;
  long long a_ptr[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i)
    a_ptr[i] = ((long long)c_begin * WG_RB + a_row[i]) * a.ldy + co0 + a_col[i];
  auto issue = [&](int chunk, int buf) {
    const int m0 = chunk * WG_RB;
#pragma unroll
    for (int i = 0; i < A_G; ++i) {
      const bool ok = m0 + a_row[i] < a.M && co0 + a_col[i] < a.Cout;
      const float* src = ok ? a.dy + a_ptr[i] : pf_wg_zero16;
      a_ptr[i] += a_step;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(As + buf * WG_RB * BM + (wave * A_G + i) * 256),
          16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_G; ++i) {
      const bool ok = b_kok[i] && m0 + b_row[i] < a.M &&
                      (unsigned)(s * b_oh[i] + b_dy[i]) < (unsigned)a.Hin &&
                      (unsigned)(s * b_ow[i] + b_dx[i]) < (unsigned)a.Win;
      const float* src = ok ? a.x + b_ptr[i] : pf_wg_zero16;
      b_ptr[i] += b_step;
      b_ow[i] += WG_RB;
      while (b_ow[i] >= a.W) {
        b_ow[i] -= a.W;
        b_ptr[i] += a.d_row;
        if (++b_oh[i] == a.H) {
          b_oh[i] = 0;
          b_ptr[i] += a.d_img;
        }
      }
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(Bs + buf * WG_RB * BN + (wave * B_G + i) * 256),
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
  float bsum[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) bsum[mi] = 0.f;
  const bool do_bias = a.partb && tn == 0 && wn == 0;

  if (c_begin < c_end) {
    issue(c_begin, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  const int acol = wm * TM + (lane & 31), bcol = wn * TN + (lane & 31), rsel = lane >> 5;
  for (int c = c_begin; c < c_end; ++c) {
    const int cur = (c - c_begin) & 1;
    if (c + 1 < c_end) issue(c + 1, cur ^ 1);
    const float* Ab = As + cur * WG_RB * BM + rsel * BM + acol;
    const float* Bb = Bs + cur * WG_RB * BN + rsel * BN + bcol;
#pragma unroll
    for (int kk = 0; kk < WG_RB / 2; ++kk) {
      float av[MI], bv[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) av[mi] = Ab[2 * kk * BM + mi * 32];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bv[ni] = Bb[2 * kk * BN + ni * 32];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) bsum[mi] += av[mi];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // ---- raw partials: row (cout) = (r&3) + 8(r>>2) + 4(lane>>5), col = lane&31
  float* pp = a.part + (long long)split * a.Cout * a.Kpad;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int k = n0 + wn * TN + ni * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * TM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (co < a.Cout && k < a.Kpad) pp[(long long)co * a.Kpad + k] = acc[mi][ni][r];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const float s = bsum[mi] + __shfl_xor(bsum[mi], 32, 64);
      const int co = co0 + wm * TM + mi * 32 + (lane & 31);
      if (lane < 32 && co < a.Cout) a.partb[(long long)split * a.Cout + co] = s;
    }
  }
}

// bf16x6 variant of the row-tile weight gradient (Cin % 32 == 0, 128 x 128
// tiles): the same tile / split / partial layout, products on the bf16
// matrix cores (conv.hip split3: six products per fp32 pair, per-product
// error below one fp32 rounding).  The MFMA reduction index is the PIXEL,
// which is the row index of dy and of the im2col rows in memory, so the
// operands cannot be DMA'd as they lie: each thread global-loads 4 pixels x 4
// couts of dy and 4 pixels x 4 k of the im2col (one chunk ahead, in
// registers), splits every value ONCE into three bf16 terms and writes them
// pixel-contiguous into LDS planes [plane][co or k][32 px] (80-B rows:
// conflict-free ds_read_b128 per 16 lanes), from which each lane reads its
// 8 consecutive pixels per k16 group directly.  The split is per element, not
// per wave read: 176 VALU per 48 MFMAs per wave.
constexpr int WB_PP = 40;  // LDS row pitch (bf16): 32 pixels + 8

__global__ __launch_bounds__(256) void conv_wgrad_bf6_kernel(WgradArgs a) {
  constexpr int BM = 128, BN = 128, WN = 2, TM = 64, TN = 64, MI = 2, NI = 2;
  __shared__ __attribute__((aligned(16))) unsigned short As[3 * BM * WB_PP];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[3 * BN * WB_PP];
  __shared__ float red[8 * BM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int split = bid / a.ntiles, tile = bid - split * a.ntiles;
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  if (gridDim.y > 1) {
    const long long z = blockIdx.y;
    a.dy += z * a.bdy;
    a.x += z * a.bx;
    a.part += z * a.bpart;
    if ((int)z != a.zb) a.partb = nullptr;
  }
  const int c_begin = (int)((long long)a.nchunks * split / a.nsplit);
  const int c_end = (int)((long long)a.nchunks * (split + 1) / a.nsplit);
  // staging role: quad q (4 couts of dy / 4 k of the im2col), pixel group pg (4 px).
  // A wave's 64 lanes are 8 quads x the 8 pixel groups, so each 8-byte plane
  // store of a half-wave covers 4 whole 64-byte rows (row pitch 20 dwords =
  // 4 mod 8: consecutive rows alternate bank halves): two cycles, the
  // minimum.  (32 quads x 2 groups per wave put every lane of a store on the
  // same two banks: PMC 18.7 conflict cycles per LDS instruction, a third of
  // the wave cycles waiting on LDS issue.)  Same elements per thread.
  const int q = tid >> 3, pg = tid & 7;
  const bool aok = co0 + 4 * q < a.Cout;
  const int k = n0 + 4 * q;  // 4 consecutive k share one tap (Cin % 32 == 0)
  const int ntap = a.KH * a.KW;
  const int cidx = k >> 5, slab = cidx / ntap, tap = cidx - slab * ntap;
  const bool kok = k < a.Kpad;
  const int kdy = tap / a.KW - a.pad, kdx = tap - (tap / a.KW) * a.KW - a.pad;
  const int kci = slab * 32 + (k & 31);
  const int HW = a.H * a.W, s = a.stride;
  // pixel (img, oh, ow) of this thread's first pixel of the current chunk
  int p_img, p_oh, p_ow;
  {
    const long long m = (long long)c_begin * WG_RB + pg * 4;
    p_img = (int)(m / HW);
    const int rem = (int)(m - (long long)p_img * HW);
    p_oh = rem / a.W;
    p_ow = rem - p_oh * a.W;
  }
  f32x4 ra[4], rb[4];
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.partb && tn == 0;
  auto load = [&](int c) {
    const long long m0 = (long long)c * WG_RB + pg * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int img = p_img, oh = p_oh, ow = p_ow + j;
      if (ow >= a.W) {  // W >= 4: at most one wrap
        ow -= a.W;
        if (++oh == a.H) {
          oh = 0;
          ++img;
        }
      }
      const bool mok = m0 + j < a.M;
      ra[j] = mok && aok ? *reinterpret_cast<const f32x4*>(a.dy + (m0 + j) * a.ldy + co0 + 4 * q)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
      const int iy = s * oh + kdy, ix = s * ow + kdx;
      rb[j] = mok && kok && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win
                  ? *reinterpret_cast<const f32x4*>(
                        a.x + (((long long)img * a.Hin + iy) * a.Win + ix) * a.xcs + kci)
                  : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // advance to the next chunk's first pixel (+32)
    p_ow += WG_RB;
    while (p_ow >= a.W) {
      p_ow -= a.W;
      if (++p_oh == a.H) {
        p_oh = 0;
        ++p_img;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f32x4 va = {ra[0][e], ra[1][e], ra[2][e], ra[3][e]};
      const f32x4 vb = {rb[0][e], rb[1][e], rb[2][e], rb[3][e]};
      uint2 h, m, l;
      pf_split3x4(va, h, m, l);
      unsigned short* pa = As + (4 * q + e) * WB_PP + pg * 4;
      *reinterpret_cast<uint2*>(pa) = h;
      *reinterpret_cast<uint2*>(pa + BM * WB_PP) = m;
      *reinterpret_cast<uint2*>(pa + 2 * BM * WB_PP) = l;
      pf_split3x4(vb, h, m, l);
      unsigned short* pb = Bs + (4 * q + e) * WB_PP + pg * 4;
      *reinterpret_cast<uint2*>(pb) = h;
      *reinterpret_cast<uint2*>(pb + BN * WB_PP) = m;
      *reinterpret_cast<uint2*>(pb + 2 * BN * WB_PP) = l;
      if (do_bias) bsum[e] += (va.x + va.y) + (va.z + va.w);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  typedef __bf16 wb_bf16x8 __attribute__((ext_vector_type(8)));
  typedef unsigned wb_u32x4 __attribute__((ext_vector_type(4)));
  auto mf = [](const wb_u32x4& x, const wb_u32x4& y, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(wb_bf16x8, x),
                                                   __builtin_bit_cast(wb_bf16x8, y), c, 0, 0, 0);
  };
  const int r32 = lane & 31, hh = lane >> 5;
  if (c_begin < c_end) load(c_begin);
  for (int c = c_begin; c < c_end; ++c) {
    __syncthreads();  // the previous chunk's planes are consumed
    store();
    __syncthreads();
    if (c + 1 < c_end) load(c + 1);  // in flight during the MFMAs
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      wb_u32x4 ah[MI], am[MI], al[MI], bh[NI], bm[NI], bl[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const unsigned short* p = As + (wm * TM + mi * 32 + r32) * WB_PP + 16 * g + 8 * hh;
        ah[mi] = *reinterpret_cast<const wb_u32x4*>(p);
        am[mi] = *reinterpret_cast<const wb_u32x4*>(p + BM * WB_PP);
        al[mi] = *reinterpret_cast<const wb_u32x4*>(p + 2 * BM * WB_PP);
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const unsigned short* p = Bs + (wn * TN + ni * 32 + r32) * WB_PP + 16 * g + 8 * hh;
        bh[ni] = *reinterpret_cast<const wb_u32x4*>(p);
        bm[ni] = *reinterpret_cast<const wb_u32x4*>(p + BN * WB_PP);
        bl[ni] = *reinterpret_cast<const wb_u32x4*>(p + 2 * BN * WB_PP);
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          f32x16 cc = acc[mi][ni];
          cc = mf(ah[mi], bh[ni], cc);
          cc = mf(ah[mi], bm[ni], cc);
          cc = mf(am[mi], bh[ni], cc);
          cc = mf(ah[mi], bl[ni], cc);
          cc = mf(al[mi], bh[ni], cc);
          cc = mf(am[mi], bm[ni], cc);
          acc[mi][ni] = cc;
        }
    }
  }
  // raw partials: row (cout) = (r&3) + 8(r>>2) + 4(lane>>5), col = lane&31
  float* pp = a.part + (long long)split * a.Cout * a.Kpad;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int kk = n0 + wn * TN + ni * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * TM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (co < a.Cout && kk < a.Kpad) pp[(long long)co * a.Kpad + kk] = acc[mi][ni][r];
      }
    }
  if (do_bias) {  // sum the 8 pixel groups of each cout in a fixed order
#pragma unroll
    for (int e = 0; e < 4; ++e) red[pg * BM + 4 * q + e] = bsum[e];
    __syncthreads();
    if (tid < BM && co0 + tid < a.Cout) {
      float t = 0.f;
      for (int g2 = 0; g2 < 8; ++g2) t += red[g2 * BM + tid];
      a.partb[(long long)split * a.Cout + co0 + tid] = t;
    }
  }
}

bool wgrad_bf6_on() {
  static const bool off = [] {
    const char* e = pf_ab_getenv("POSFEAT_WGRAD_BF6");
    return e && e[0] == '0';
  }();
  return pf_conv_precision() >= 1 && !off;
}

// Halo variant for 3x3 stride-1 convs with Cin % 32 == 0 (head.conv1/conv2).
// Work item = one 32-pixel row segment (img, y, x0..x0+31) x one 32-channel
// input slab x BM couts.  Per segment the dy rows [32 px][BM] and the input
// halo [3 rows][34 px][32 ch] of the slab are DMA'd into LDS once; the 9 taps
// are 9 shifted reads of the halo, so the block's tile is BM x 288 packed k
// ((slab, tap, ci) = a contiguous range of the packed order) and it stages
// 2.5x fewer bytes per MAC than the row-tile kernel above.  Wave w owns couts
// [w*32, w*32+32) for all 9 taps: per pixel pair 1 A read + 9 B reads feed 9
// MFMAs.
constexpr int WH_HX = 34, WH_HROWS = 3 * WH_HX;  // halo pixels per segment
constexpr int WH_HG = (WH_HROWS + 7) / 8;        // DMA instructions for the halo (8 px each)

template <int NW>
__global__ __launch_bounds__(NW * 64) void conv_wgrad_halo_kernel(WgradArgs a) {
  constexpr int BM = NW * 32;
  constexpr int A_INS = 32 * BM * 4 / 1024;  // dy DMA instructions per segment
  constexpr int ASZ = 32 * BM, XSZ = WH_HG * 8 * 32;
  __shared__ __attribute__((aligned(16))) float smem[2 * (ASZ + XSZ)];
  float* As = smem;             // [2][32 px][BM]
  float* Xs = smem + 2 * ASZ;   // [2][104 halo px][32 ch]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int split = bid / a.ntiles, tile = bid - split * a.ntiles;
  const int nslab = a.Cin / 32;
  const int tm = tile / nslab, slab = tile - tm * nslab;
  const int co0 = tm * BM;
  const int XB = (a.W + 31) / 32;  // segments per image row
  const int c_begin = (int)((long long)a.nchunks * split / a.nsplit);
  const int c_end = (int)((long long)a.nchunks * (split + 1) / a.nsplit);

  // segment c -> (img, y, x0): tracked incrementally (wave-uniform)
  int s_img, s_y, s_xb;
  {
    const int per_img = a.H * XB;
    s_img = c_begin / per_img;
    const int rem = c_begin - s_img * per_img;
    s_y = rem / XB;
    s_xb = rem - s_y * XB;
  }
  const long long HW = (long long)a.H * a.W;
  auto issue = [&](int buf) {
    const int y = s_y, x0 = s_xb * 32;
    const long long rowbase = (long long)s_img * HW + (long long)y * a.W;
    // dy rows: 32 px x BM couts
    for (int i = wave; i < A_INS; i += NW) {
      const int e = (i * 1024 + lane * 16) / 4;
      const int px = e / BM, col = e - px * BM;
      const bool ok = x0 + px < a.W && co0 + col < a.Cout;
      const float* src = ok ? a.dy + (rowbase + x0 + px) * a.ldy + co0 + col : pf_wg_zero16;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(As + buf * ASZ + i * 256), 16, 0, 0);
    }
    // halo: rows y-1..y+1, px x0-1..x0+32, channels slab*32..+31
    for (int i = wave; i < WH_HG; i += NW) {
      const int hp = i * 8 + (lane >> 3), sl = lane & 7;
      const int hy = hp / WH_HX, hx = hp - hy * WH_HX;
      const int iy = y - 1 + hy, ix = x0 - 1 + hx;
      const bool ok = hp < WH_HROWS && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
      const float* src =
          ok ? a.x + ((long long)s_img * HW + (long long)iy * a.W + ix) * a.xcs + slab * 32 + sl * 4
             : pf_wg_zero16;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(Xs + buf * XSZ + i * 256), 16, 0, 0);
    }
    if (++s_xb == XB) {
      s_xb = 0;
      if (++s_y == a.H) {
        s_y = 0;
        ++s_img;
      }
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum = 0.f;
  const bool do_bias = a.partb && slab == 0;

  if (c_begin < c_end) {
    issue(0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  const int rsel = lane >> 5;
  for (int c = c_begin; c < c_end; ++c) {
    const int cur = (c - c_begin) & 1;
    if (c + 1 < c_end) issue(cur ^ 1);
    const float* Ab = As + cur * ASZ + rsel * BM + wave * 32 + (lane & 31);
    const float* Xb = Xs + cur * XSZ + rsel * 32 + (lane & 31);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const float av = Ab[2 * kk * BM];
      float bv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) bv[t] = Xb[((t / 3) * WH_HX + 2 * kk + t % 3) * 32];
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[t], acc[t], 0, 0, 0);
      if (do_bias) bsum += av;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // raw partials, packed k = (slab*9 + t)*32 + ci
  float* pp = a.part + (long long)split * a.Cout * a.Kpad;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int k = (slab * 9 + t) * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (co < a.Cout) pp[(long long)co * a.Kpad + k] = acc[t][r];
    }
  }
  if (do_bias) {
    const float s = bsum + __shfl_xor(bsum, 32, 64);
    const int co = co0 + wave * 32 + (lane & 31);
    if (lane < 32 && co < a.Cout) a.partb[(long long)split * a.Cout + co] = s;
  }
}

// dw[co][k] = sum_s part[s][co][k] (split order: deterministic); db likewise.
// acc: add to the existing gradient (the two image batches of one step)
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, const float* __restrict__ partb,
                                    int nsplit, int Cout, int Kpad, float* __restrict__ dw,
                                    float* __restrict__ db, int acc) {
  const long long n = (long long)Cout * Kpad;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i < n) {
    const float s = pf_ordered_sum(part + i, n, nsplit);
    dw[i] = acc ? dw[i] + s : s;
  }
  if (db && i < Cout) {
    const float s = pf_ordered_sum(partb + i, Cout, nsplit);
    db[i] = acc ? db[i] + s : s;
  }
}

// W'[ci][k'] with k' = ((co/32)*ntap + tap')*32 + co%32, tap' = ntap-1-tap:
// the spatially flipped, channel-transposed kernel (stride 1, same padding)
__global__ void dgrad_weights_kernel(const float* __restrict__ w, int Cout, int Cin, int ntap,
                                     int kpad_f, float* __restrict__ wt, int kpad_t,
                                     unsigned short* __restrict__ planes) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long n = (long long)Cin * kpad_t;
  if (i >= n) return;
  const int ci = (int)(i / kpad_t), kp = (int)(i - (long long)ci * kpad_t);
  const int c = kp >> 5, slab = c / ntap, tapp = c - slab * ntap, co = slab * 32 + (kp & 31);
  float v = 0.f;
  if (co < Cout) {
    const int tap = ntap - 1 - tapp;
    v = w[(long long)co * kpad_f + ((ci >> 5) * ntap + tap) * 32 + (ci & 31)];
  }
  wt[i] = v;
  if (planes) {  // split3 per element: the same bits as pf_split3_rows
    unsigned hh, mm, ll;
    pf_split3_pair(v, 0.f, hh, mm, ll);
    planes[i] = (unsigned short)hh;
    planes[i + n] = (unsigned short)mm;
    planes[i + 2 * n] = (unsigned short)ll;
  }
}

// ---------------------------------------------------------------- x4 upsample adjoint
// forward (fmap.hip norm_prelu_upsample_kernel / ATen upsample_bilinear2d,
// align_corners=False): src = s*(o+0.5)-0.5 clamped at 0, i0 = floor, i1 =
// i0 + (i0 < n-1), weights (1-l, l).  Weight of output o on input q:
__device__ __forceinline__ float up_w(int o, int q, float s, int n) {
  float f = s * (o + 0.5f) - 0.5f;
  f = f < 0.f ? 0.f : f;
  const int i0 = (int)f;
  const int i1 = i0 + (i0 < n - 1 ? 1 : 0);
  const float l = f - i0;
  return (i0 == q ? 1.f - l : 0.f) + (i1 == q ? l : 0.f);
}

// t[b][oy][qx][c] = sum_ox w(ox, qx) g[b][oy][ox][c]   (c < C, quads)
__global__ void up4_adj_x_kernel(const float* __restrict__ g, int gcs, int nb, int OH, int OW,
                                 int w, int c4n, float* __restrict__ t) {
  const float s = (float)w / (float)OW;
  const long long total = (long long)nb * OH * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const int qx = (int)(p % w);
    const long long row = p / w;  // b*OH + oy
    const float* gr = g + row * OW * gcs + q * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int o0 = max(0, 4 * qx - 4), o1 = min(OW - 1, 4 * qx + 5);
    for (int ox = o0; ox <= o1; ++ox) {
      const float wt = up_w(ox, qx, s, w);
      if (wt != 0.f) acc += wt * *reinterpret_cast<const f32x4*>(gr + (long long)ox * gcs);
    }
    *reinterpret_cast<f32x4*>(t + p * (c4n * 4) + q * 4) = acc;
  }
}

// d[b][qy][qx][c] = sum_oy w(oy, qy) t[b][oy][qx][c]
__global__ void up4_adj_y_kernel(const float* __restrict__ t, int nb, int OH, int h, int w,
                                 int c4n, float* __restrict__ d, int dcs) {
  const float s = (float)h / (float)OH;
  const long long total = (long long)nb * h * w * c4n;
  const int C = c4n * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const int qx = (int)(p % w);
    p /= w;
    const int qy = (int)(p % h);
    const int b = (int)(p / h);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int o0 = max(0, 4 * qy - 4), o1 = min(OH - 1, 4 * qy + 5);
    for (int oy = o0; oy <= o1; ++oy) {
      const float wt = up_w(oy, qy, s, h);
      if (wt != 0.f)
        acc += wt * *reinterpret_cast<const f32x4*>(t + (((long long)b * OH + oy) * w + qx) * C + q * 4);
    }
    *reinterpret_cast<f32x4*>(d + (((long long)b * h + qy) * w + qx) * dcs + q * 4) = acc;
  }
}

// ---------------------------------------------------------------- instance-norm backward
// For x^ = (x - mean) * rstd and upstream g = dL/d(act(x^)) with act = PReLU
// (slope a) or identity:  dx^ = act'(x^) g,  dx = rstd (dx^ - E[dx^] - x^ E[dx^ x^]).
// Partials per (image, pixel chunk): sum dx^, sum dx^ x^ per channel (fp64) and,
// for PReLU, sum x^<=0 ? x^ g : 0 (the slope gradient, torch prelu backward).
constexpr int INB_CHUNK = 2048;

template <bool PRELU>
__device__ __forceinline__ void inb_load(const float* xr, const float* gr, f32x4 m, f32x4 r,
                                         float a, f32x4& xh, f32x4& dxh, f32x4& sg) {
  const f32x4 xv = *reinterpret_cast<const f32x4*>(xr);
  const f32x4 gv = *reinterpret_cast<const f32x4*>(gr);
  if (PRELU) {
    xh = (xv - m) * r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool pos = xh[k] > 0.f;
      dxh[k] = pos ? gv[k] : a * gv[k];
      sg[k] = pos ? 0.f : xh[k] * gv[k];
    }
  } else {
    xh = xv;  // already normalised
    dxh = gv;
    sg = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

template <bool PRELU>
__global__ __launch_bounds__(256) void in_bwd_partial_kernel(
    const float* __restrict__ x, int xcs, const float* __restrict__ g, int gcs, int hw, int C,
    const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ slope,
    double* __restrict__ part, double* __restrict__ spart) {
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int c4n = C / 4, tid = threadIdx.x;
  const int rows = blockDim.x / c4n;
  const int q = tid % c4n, pl = tid / c4n;
  const float a = PRELU ? *slope : 0.f;
  f32x4 s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0}, s3 = {0, 0, 0, 0};
  if (pl < rows) {
    f32x4 m = {0, 0, 0, 0}, r = {1, 1, 1, 1};
    if (PRELU) {
      m = *reinterpret_cast<const f32x4*>(mean + b * C + q * 4);
      r = *reinterpret_cast<const f32x4*>(rstd + b * C + q * 4);
    }
    const int p0 = chunk * INB_CHUNK, p1 = min(hw, p0 + INB_CHUNK);
    for (int p = p0 + pl; p < p1; p += rows) {
      const long long pix = (long long)b * hw + p;
      f32x4 xh, dxh, sg;
      inb_load<PRELU>(x + pix * xcs + q * 4, g + pix * gcs + q * 4, m, r, a, xh, dxh, sg);
      s1 += dxh;
      s2 += dxh * xh;
      s3 += sg;
    }
  }
  __shared__ double red[256 * 9];
  for (int k = 0; k < 4; ++k) {
    red[tid * 9 + k] = s1[k];
    red[tid * 9 + 4 + k] = s2[k];
  }
  red[tid * 9 + 8] = (double)s3[0] + s3[1] + s3[2] + s3[3];
  __syncthreads();
  if (tid < c4n) {
    double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int rr = 0; rr < rows; ++rr)
      for (int k = 0; k < 8; ++k) t[k] += red[(rr * c4n + tid) * 9 + k];
    double* o = part + ((long long)b * nchunk + chunk) * C * 2;
    for (int k = 0; k < 4; ++k) {
      o[(tid * 4 + k) * 2] = t[k];
      o[(tid * 4 + k) * 2 + 1] = t[4 + k];
    }
  }
  if (PRELU && tid == 0) {
    double t = 0;
    for (int k = 0; k < rows * c4n; ++k) t += red[k * 9 + 8];
    spart[(long long)b * nchunk + chunk] = t;
  }
}

// E[dx^], E[dx^ x^] per (image, channel)
__global__ void in_bwd_finalize_kernel(const double* __restrict__ part, int nchunk, int nb, int C,
                                       int hw, float* __restrict__ e1, float* __restrict__ e2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * C) return;
  const int b = i / C, c = i - b * C;
  double s1 = 0, s2 = 0;
  const double* p = part + (long long)b * nchunk * C * 2;
  for (int k = 0; k < nchunk; ++k) {
    s1 += p[(k * C + c) * 2];
    s2 += p[(k * C + c) * 2 + 1];
  }
  e1[i] = (float)(s1 / hw);
  e2[i] = (float)(s2 / hw);
}

template <bool PRELU>
__global__ void in_bwd_apply_kernel(const float* __restrict__ x, int xcs, const float* g, int gcs,
                                    int nb, int hw, int c4n, const float* __restrict__ mean,
                                    const float* __restrict__ rstd,
                                    const float* __restrict__ slope, const float* __restrict__ e1,
                                    const float* __restrict__ e2, float* dx, int dxcs) {
  const long long total = (long long)nb * hw * c4n;
  const int C = c4n * 4;
  const float a = PRELU ? *slope : 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long pix;
    const int q = pf_quad_split(i, c4n, pix);
    const int b = (int)(pix / hw);
    // identity mode: x is already normalised (mean is NULL); rstd still scales dx
    const f32x4 m = PRELU ? *reinterpret_cast<const f32x4*>(mean + b * C + q * 4)
                          : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 r = *reinterpret_cast<const f32x4*>(rstd + b * C + q * 4);
    f32x4 xh, dxh, sg;
    inb_load<PRELU>(x + pix * xcs + q * 4, g + pix * gcs + q * 4, m, r, a, xh, dxh, sg);
    const f32x4 m1 = *reinterpret_cast<const f32x4*>(e1 + b * C + q * 4);
    const f32x4 m2 = *reinterpret_cast<const f32x4*>(e2 + b * C + q * 4);
    *reinterpret_cast<f32x4*>(dx + pix * dxcs + q * 4) = r * (dxh - m1 - xh * m2);
  }
}

// ---------------------------------------------------------------- head tail backward
// local_point = softplus(z^), z^ = (y3 - m3) r3, y3 = conv3(a2) + b3, a2 = PReLU(x2^),
// x2^ = (c2 - m2) r2  (DeteNet.py:112-113; Softplus beta 1 threshold 20)
// tail1: per image sums of dz and dz z^ (dz = dLP * softplus'(z^))
__device__ __forceinline__ float softplus_grad(float z) {
  // torch softplus_backward: z > threshold ? 1 : exp(z) / (exp(z) + 1)
  if (z > 20.f) return 1.f;
  const float e = expf(z);
  return e / (e + 1.f);
}

__global__ __launch_bounds__(256) void tail1_partial_kernel(const float* __restrict__ dlp,
                                                            const float* __restrict__ y3, int hw,
                                                            const float* __restrict__ m3,
                                                            const float* __restrict__ r3,
                                                            double* __restrict__ part) {
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const float m = m3[b], r = r3[b];
  float s1 = 0.f, s2 = 0.f;
  const int p0 = chunk * INB_CHUNK, p1 = min(hw, p0 + INB_CHUNK);
  for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const long long i = (long long)b * hw + p;
    const float z = (y3[i] - m) * r;
    const float dz = dlp[i] * softplus_grad(z);
    s1 += dz;
    s2 += dz * z;
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((long long)b * nchunk + chunk) * 2] = r1[0];
    part[((long long)b * nchunk + chunk) * 2 + 1] = r2[0];
  }
}

// tail2: dy3 per pixel (stored), then per channel of conv2's output the partial
// sums sum dx2^, sum dx2^ x2^ (norm2 backward), sum dy3 a2 (dW3), and per block
// sum dy3 (db3) and the PReLU slope term.  Block = 32 channel quads x 8 pixel
// lanes over one chunk of one image.
__global__ __launch_bounds__(256) void tail2_partial_kernel(
    const float* __restrict__ dlp, const float* __restrict__ y3, const float* __restrict__ c2,
    int c2cs, int hw, const float* __restrict__ m3, const float* __restrict__ r3,
    const double* __restrict__ t1part, int t1chunks, const float* __restrict__ m2,
    const float* __restrict__ r2, const float* __restrict__ slope, const float* __restrict__ w3,
    float* __restrict__ dy3, double* __restrict__ part, double* __restrict__ spart) {
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int tid = threadIdx.x, q = tid & 31, pl = tid >> 5;
  __shared__ float sh_e[2];
  if (tid == 0) {
    double s1 = 0, s2 = 0;
    for (int k = 0; k < t1chunks; ++k) {
      s1 += t1part[((long long)b * t1chunks + k) * 2];
      s2 += t1part[((long long)b * t1chunks + k) * 2 + 1];
    }
    sh_e[0] = (float)(s1 / hw);
    sh_e[1] = (float)(s2 / hw);
  }
  __syncthreads();
  const float e1 = sh_e[0], e2 = sh_e[1];
  const float mz = m3[b], rz = r3[b], a = *slope;
  const f32x4 m = *reinterpret_cast<const f32x4*>(m2 + b * 128 + q * 4);
  const f32x4 r = *reinterpret_cast<const f32x4*>(r2 + b * 128 + q * 4);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w3 + q * 4);
  f32x4 s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0}, s3 = {0, 0, 0, 0};
  float sb = 0.f, ss = 0.f;
  const int p0 = chunk * INB_CHUNK, p1 = min(hw, p0 + INB_CHUNK);
  for (int p = p0 + pl; p < p1; p += 8) {
    const long long i = (long long)b * hw + p;
    const float z = (y3[i] - mz) * rz;
    const float dz = dlp[i] * softplus_grad(z);
    const float d3 = rz * (dz - e1 - z * e2);
    if (q == 0) {
      dy3[i] = d3;
      sb += d3;
    }
    const f32x4 xh = (*reinterpret_cast<const f32x4*>(c2 + i * c2cs + q * 4) - m) * r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool pos = xh[k] > 0.f;
      const float a2 = pos ? xh[k] : a * xh[k];
      const float da2 = d3 * wv[k];
      const float dxh = pos ? da2 : a * da2;
      s1[k] += dxh;
      s2[k] += dxh * xh[k];
      s3[k] += d3 * a2;
      ss += pos ? 0.f : xh[k] * da2;
    }
  }
  __shared__ double red[256 * 12];
  for (int k = 0; k < 4; ++k) {
    red[tid * 12 + k] = s1[k];
    red[tid * 12 + 4 + k] = s2[k];
    red[tid * 12 + 8 + k] = s3[k];
  }
  __syncthreads();
  if (tid < 32) {
    double t[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int rr = 0; rr < 8; ++rr)
      for (int k = 0; k < 12; ++k) t[k] += red[(rr * 32 + tid) * 12 + k];
    double* o = part + ((long long)b * nchunk + chunk) * 128 * 3;
    for (int k = 0; k < 4; ++k) {
      o[(tid * 4 + k) * 3] = t[k];
      o[(tid * 4 + k) * 3 + 1] = t[4 + k];
      o[(tid * 4 + k) * 3 + 2] = t[8 + k];
    }
  }
  __syncthreads();
  red[tid * 2] = sb;
  red[tid * 2 + 1] = ss;
  __syncthreads();
  if (tid == 0) {
    double tb = 0, ts = 0;
    for (int k = 0; k < 256; ++k) {
      tb += red[k * 2];
      ts += red[k * 2 + 1];
    }
    spart[((long long)b * nchunk + chunk) * 2] = tb;
    spart[((long long)b * nchunk + chunk) * 2 + 1] = ts;
  }
}

// per (image, channel): E[dx2^], E[dx2^ x2^]; one block per image, thread
// (channel c, lane j of 8) sums the chunks k = j mod 8, the 8 partials are
// added in j order (fixed order, deterministic).  The image's dW3 share goes
// to part[b][0][c][2] (this block has read the whole image's part by then);
// tail2_dw3_kernel sums the images in order.  (One block of 128 threads
// walking nb x nchunk chunks was latency-bound: 0.88 ms at 16 x 150.)
__global__ __launch_bounds__(1024) void tail2_finalize_kernel(double* __restrict__ part,
                                                              int nchunk, int hw,
                                                              float* __restrict__ e1,
                                                              float* __restrict__ e2) {
  const int b = blockIdx.x, c = threadIdx.x & 127, j = threadIdx.x >> 7;
  double* p = part + (long long)b * nchunk * 128 * 3;
  double s1 = 0, s2 = 0, s3 = 0;
  for (int k = j; k < nchunk; k += 8) {
    s1 += p[(k * 128 + c) * 3];
    s2 += p[(k * 128 + c) * 3 + 1];
    s3 += p[(k * 128 + c) * 3 + 2];
  }
  __shared__ double red[8][128][3];
  red[j][c][0] = s1;
  red[j][c][1] = s2;
  red[j][c][2] = s3;
  __syncthreads();
  if (j == 0) {
    double t1 = 0, t2 = 0, t3 = 0;
    for (int q = 0; q < 8; ++q) {
      t1 += red[q][c][0];
      t2 += red[q][c][1];
      t3 += red[q][c][2];
    }
    e1[b * 128 + c] = (float)(t1 / hw);
    e2[b * 128 + c] = (float)(t2 / hw);
    p[c * 3 + 2] = t3;
  }
}

// dW3[c] = sum over images (in order) of the per-image shares
__global__ void tail2_dw3_kernel(const double* __restrict__ part, int nchunk, int nb,
                                 float* __restrict__ dw3) {
  const int c = threadIdx.x;  // 128 threads
  double w = 0;
  for (int b = 0; b < nb; ++b) w += part[(long long)b * nchunk * 128 * 3 + c * 3 + 2];
  dw3[c] = (float)w;
}

// dc2 = r2 (dx2^ - E[dx2^] - x2^ E[dx2^ x2^]), dx2^ recomputed from dy3
__global__ void tail3_kernel(const float* __restrict__ dy3, const float* __restrict__ c2, int c2cs,
                             int nb, int hw, const float* __restrict__ m2,
                             const float* __restrict__ r2, const float* __restrict__ slope,
                             const float* __restrict__ w3, const float* __restrict__ e1,
                             const float* __restrict__ e2, float* __restrict__ dc2, int dcs) {
  const long long total = (long long)nb * hw * 32;
  const float a = *slope;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i & 31);
    const long long pix = i >> 5;
    const int b = (int)(pix / hw);
    const f32x4 m = *reinterpret_cast<const f32x4*>(m2 + b * 128 + q * 4);
    const f32x4 r = *reinterpret_cast<const f32x4*>(r2 + b * 128 + q * 4);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w3 + q * 4);
    const f32x4 xh = (*reinterpret_cast<const f32x4*>(c2 + pix * c2cs + q * 4) - m) * r;
    const float d3 = dy3[pix];
    f32x4 dxh;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float da2 = d3 * wv[k];
      dxh[k] = xh[k] > 0.f ? da2 : a * da2;
    }
    const f32x4 me1 = *reinterpret_cast<const f32x4*>(e1 + b * 128 + q * 4);
    const f32x4 me2 = *reinterpret_cast<const f32x4*>(e2 + b * 128 + q * 4);
    *reinterpret_cast<f32x4*>(dc2 + pix * dcs + q * 4) = r * (dxh - me1 - xh * me2);
  }
}

// small scalars of the head gradient, fixed order:
//   db3 = sum dy3;  dslope = sum(tail slope terms) + sum(conv1-path slope terms)
__global__ __launch_bounds__(1024) void head_scalars_kernel(const double* __restrict__ t2s, int n2,
                                                            const double* __restrict__ c1s, int n1,
                                                            float* __restrict__ db3,
                                                            float* __restrict__ dslope) {
  // thread t sums its contiguous slice of each list in order; the 1024
  // partials then meet in a fixed pairwise tree (deterministic; a single
  // thread walking both lists took 0.37 ms)
  const int t = threadIdx.x;
  const int k2 = (n2 + 1023) / 1024, k1 = (n1 + 1023) / 1024;
  double b = 0, s = 0;
  for (int i = t * k2; i < min(n2, (t + 1) * k2); ++i) {
    b += t2s[2 * i];
    s += t2s[2 * i + 1];
  }
  for (int i = t * k1; i < min(n1, (t + 1) * k1); ++i) s += c1s[i];
  __shared__ double rb[1024], rs[1024];
  rb[t] = b;
  rs[t] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (t < o) {
      rb[t] += rb[t + o];
      rs[t] += rs[t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    *db3 = (float)rb[0];
    *dslope = (float)rs[0];
  }
}

__global__ void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, long long n,
                           float lr) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    w[i] -= lr * g[i];
}

inline int grid_for(long long total, int block) {
  long long g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

// A/B knobs (POSFEAT_WG_TARGET / POSFEAT_WG_MINCH; unset: 1024 workgroups,
// >= 8 chunks per split)
int wg_knob(const char* name, int dflt) {
  const char* e = pf_ab_getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
int wg_target() {
  static const int v = wg_knob("POSFEAT_WG_TARGET", 1024);
  return v;
}
int wg_minch() {
  static const int v = wg_knob("POSFEAT_WG_MINCH", 8);
  return v;
}

struct WgPlan {
  bool halo;
  int BM, BN, tiles_m, tiles_n, nsplit, nchunks, Kpad, K, ntiles;
};

// H, W: output (dy) dims
WgPlan wgrad_plan(int n, int H, int W, int Cin, int Cout, int KH, int KW, int stride) {
  WgPlan p;
  p.Kpad = posfeat_conv_packed_k(Cin, KH, KW);
  p.K = KH * KW * Cin;
  p.halo = Cin % 32 == 0 && KH == 3 && KW == 3 && stride == 1;
  if (p.halo) {
    // tiles = (cout block, input slab); chunks = 32-pixel row segments
    p.BM = (Cout % 192 == 0) ? 192 : (Cout % 128 == 0) ? 128 : 64;
    p.BN = 288;
    p.tiles_m = (Cout + p.BM - 1) / p.BM;
    p.tiles_n = Cin / 32;
    p.nchunks = n * H * ((W + 31) / 32);
  } else {
    p.BM = (Cout % 128 == 0) ? 128 : 64;
    p.BN = (p.Kpad % 128 == 0) ? 128 : 64;
    p.tiles_m = (Cout + p.BM - 1) / p.BM;
    p.tiles_n = (p.Kpad + p.BN - 1) / p.BN;
    const long long M = (long long)n * H * W;
    p.nchunks = (int)((M + WG_RB - 1) / WG_RB);
  }
  p.ntiles = p.tiles_m * p.tiles_n;
  // >= 1024 workgroups (2 rounds of the 2-per-CU residency), >= 8 chunks each,
  // partial slabs capped at 128 per tile
  const int s = (wg_target() + p.ntiles - 1) / p.ntiles;
  const int maxs = std::max(1, p.nchunks / wg_minch());
  p.nsplit = std::max(1, std::min(std::min(s, maxs), 128));
  return p;
}

// POSFEAT_WGRAD_BF6_ALL=1 (A/B, off): conv_wgrad_bf6_kernel for every
// Cin % 32 == 0 conv (3x3 stride 1 too, instead of the fp32 halo tiles):
// 128 x 128 tiles, ragged last cout / k tiles (the kernel guards both).
// Measured r4e: slower where the halo tiles reuse the staged input across
// the 9 taps (keypoint head: image-branch A 3.2 -> 5.1 ms, conv1 2.2 -> 3.0)
bool wgrad_bf6_all() {
  static const bool on = [] {
    const char* e = pf_ab_getenv("POSFEAT_WGRAD_BF6_ALL");
    return e && e[0] == '1';
  }();
  return on;
}
WgPlan wgrad_plan_bf6(int n, int H, int W, int Cin, int Cout, int KH, int KW) {
  WgPlan p;
  p.Kpad = posfeat_conv_packed_k(Cin, KH, KW);
  p.K = KH * KW * Cin;
  p.halo = false;
  p.BM = p.BN = 128;
  p.tiles_m = (Cout + 127) / 128;
  p.tiles_n = (p.Kpad + 127) / 128;
  const long long M = (long long)n * H * W;
  p.nchunks = (int)((M + WG_RB - 1) / WG_RB);
  p.ntiles = p.tiles_m * p.tiles_n;
  const int s = (wg_target() + p.ntiles - 1) / p.ntiles;
  const int maxs = std::max(1, p.nchunks / wg_minch());
  p.nsplit = std::max(1, std::min(std::min(s, maxs), 128));
  return p;
}

}  // namespace

// ------------------------------------------------------------------ launchers
static inline int wg_out(int H, int K, int stride) { return (H + 2 * ((K - 1) / 2) - K) / stride + 1; }

size_t pf_conv_wgrad_ws_bytes(int n, int H, int W, int Cin, int Cout, int KH, int KW, int stride) {
  const int OH = wg_out(H, KH, stride), OW = wg_out(W, KW, stride);
  const WgPlan p = wgrad_plan(n, OH, OW, Cin, Cout, KH, KW, stride);
  const WgPlan q = wgrad_plan_bf6(n, OH, OW, Cin, Cout, KH, KW);
  const int ns = std::max(p.nsplit, q.nsplit);
  return pf_align((size_t)ns * Cout * p.Kpad * 4, 256) + pf_align((size_t)ns * Cout * 4, 256);
}

int pf_conv_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int H, int W, int Cin,
                  int Cout, int KH, int KW, int stride, float* dw, float* db, int acc, void* ws,
                  size_t ws_bytes, hipStream_t st) {
  if ((Cin % 32 != 0 && Cin != 4) || Cout % 32 || ldy % 4 || xcs % 4 || KH != KW || KH % 2 == 0 ||
      stride < 1 || stride > 2)
    return POSFEAT_E_INVALID;
  if (reinterpret_cast<uintptr_t>(dy) % 16 || reinterpret_cast<uintptr_t>(x) % 16)
    return POSFEAT_E_INVALID;
  if (ws_bytes < pf_conv_wgrad_ws_bytes(n, H, W, Cin, Cout, KH, KW, stride))
    return POSFEAT_E_WORKSPACE;
  const int OH = wg_out(H, KH, stride), OW = wg_out(W, KW, stride);
  const bool b6all = Cin % 32 == 0 && wgrad_bf6_on() && wgrad_bf6_all() && OW >= 4;
  const WgPlan p = b6all ? wgrad_plan_bf6(n, OH, OW, Cin, Cout, KH, KW)
                         : wgrad_plan(n, OH, OW, Cin, Cout, KH, KW, stride);
  WgradArgs a;
  a.dy = dy;
  a.ldy = ldy;
  a.x = x;
  a.xcs = xcs;
  a.H = OH;
  a.W = OW;
  a.Hin = H;
  a.Win = W;
  a.stride = stride;
  a.d_row = (long long)(stride * W - stride * OW) * xcs;
  a.d_img = ((long long)H * W - (long long)stride * OH * W) * xcs;
  a.Cin = Cin;
  a.KH = KH;
  a.KW = KW;
  a.pad = (KH - 1) / 2;
  a.Cout = Cout;
  a.Kpad = p.Kpad;
  a.K = p.K;
  a.M = n * OH * OW;
  a.tiles_n = p.tiles_n;
  a.ntiles = p.ntiles;
  a.nsplit = p.nsplit;
  a.nchunks = p.nchunks;
  a.bdy = a.bx = a.bpart = 0;
  a.zb = 0;
  a.part = static_cast<float*>(ws);
  a.partb = db ? reinterpret_cast<float*>(static_cast<char*>(ws) +
                                          pf_align((size_t)p.nsplit * Cout * p.Kpad * 4, 256))
               : nullptr;
  const dim3 grid(a.ntiles * a.nsplit);
  if (b6all) {
    hipLaunchKernelGGL(conv_wgrad_bf6_kernel, grid, dim3(256), 0, st, a);
  } else if (p.halo) {
    if (p.BM == 192)
      hipLaunchKernelGGL(conv_wgrad_halo_kernel<6>, grid, dim3(384), 0, st, a);
    else if (p.BM == 128)
      hipLaunchKernelGGL(conv_wgrad_halo_kernel<4>, grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(conv_wgrad_halo_kernel<2>, grid, dim3(128), 0, st, a);
  } else if (p.BM == 128 && p.BN == 128 && Cin % 32 == 0 && wgrad_bf6_on())
    hipLaunchKernelGGL(conv_wgrad_bf6_kernel, grid, dim3(256), 0, st, a);
  else if (p.BM == 128 && p.BN == 128)
    hipLaunchKernelGGL((conv_wgrad_kernel<128, 128>), grid, dim3(256), 0, st, a);
  else if (p.BM == 128)
    hipLaunchKernelGGL((conv_wgrad_kernel<128, 64>), grid, dim3(256), 0, st, a);
  else if (p.BN == 128)
    hipLaunchKernelGGL((conv_wgrad_kernel<64, 128>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<64, 64>), grid, dim3(256), 0, st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(b6all || (!p.halo && p.BM == 128 && p.BN == 128 && Cin % 32 == 0 && wgrad_bf6_on())
                    ? PF_ARITH_BF6
                    : PF_ARITH_FP32);
  const long long ne = (long long)Cout * p.Kpad;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st,
                     a.part, a.partb, p.nsplit, Cout, p.Kpad, dw, db, acc);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// Per-image weight gradient of a 3x3 stride-1 conv (halo kernel): with
// nsplit = n * k the pixel-range splits never straddle an image (split
// z*k + j covers rows of image z only), so summing splits z*k .. z*k+k-1 in
// order gives image z's gradient alone.  Used by the keypoint-head backward,
// whose image-branch gradients contract per-image statistics.
namespace {
bool per_image_bf6(int H, int W, int Cin) {
  return Cin % 32 == 0 && wgrad_bf6_on() && wgrad_bf6_all() && W >= 4 && (H * W) % WG_RB == 0;
}
int per_image_k(int n, int H, int W, int Cin, int Cout) {
  const WgPlan p = per_image_bf6(H, W, Cin) ? wgrad_plan_bf6(n, H, W, Cin, Cout, 3, 3)
                                             : wgrad_plan(n, H, W, Cin, Cout, 3, 3, 1);
  const int per_img = per_image_bf6(H, W, Cin) ? H * W / WG_RB : H * ((W + 31) / 32);
  const int k = (1024 + n * p.ntiles - 1) / (n * p.ntiles);
  return std::max(1, std::min(std::min(k, per_img / 8), 128));
}
__global__ void wgrad_reduce_images_kernel(const float* __restrict__ part, int k, long long per,
                                           int n, float* __restrict__ dw) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= per * n) return;
  const long long z = i / per, e = i - z * per;
  dw[i] = pf_ordered_sum(part + z * k * per + e, per, k);
}
}  // namespace

size_t pf_conv_wgrad_per_image_ws_bytes(int n, int H, int W, int Cin, int Cout) {
  const int k = per_image_k(n, H, W, Cin, Cout);
  return pf_align((size_t)n * k * Cout * posfeat_conv_packed_k(Cin, 3, 3) * 4, 256);
}

int pf_conv_wgrad_per_image(const float* dy, int ldy, const float* x, int xcs, int n, int H, int W,
                            int Cin, int Cout, float* dw, void* ws, size_t ws_bytes,
                            hipStream_t st) {
  if (Cin % 32 || Cout % 32 || ldy % 4 || xcs % 4 || n <= 0) return POSFEAT_E_INVALID;
  if (reinterpret_cast<uintptr_t>(dy) % 16 || reinterpret_cast<uintptr_t>(x) % 16)
    return POSFEAT_E_INVALID;
  if (ws_bytes < pf_conv_wgrad_per_image_ws_bytes(n, H, W, Cin, Cout)) return POSFEAT_E_WORKSPACE;
  const bool b6 = per_image_bf6(H, W, Cin);
  const WgPlan p = b6 ? wgrad_plan_bf6(n, H, W, Cin, Cout, 3, 3) : wgrad_plan(n, H, W, Cin, Cout, 3, 3, 1);
  const int k = per_image_k(n, H, W, Cin, Cout);
  WgradArgs a;
  a.dy = dy;
  a.ldy = ldy;
  a.x = x;
  a.xcs = xcs;
  a.H = a.Hin = H;
  a.W = a.Win = W;
  a.stride = 1;
  a.d_row = a.d_img = 0;
  a.Cin = Cin;
  a.KH = a.KW = 3;
  a.pad = 1;
  a.Cout = Cout;
  a.Kpad = p.Kpad;
  a.K = p.K;
  a.M = n * H * W;
  a.tiles_n = p.tiles_n;
  a.ntiles = p.ntiles;
  a.nsplit = n * k;
  a.nchunks = p.nchunks;
  a.bdy = a.bx = a.bpart = 0;
  a.zb = 0;
  a.part = static_cast<float*>(ws);
  a.partb = nullptr;
  const dim3 grid(a.ntiles * a.nsplit);
  if (b6)  // image-aligned 32-pixel chunks (H W % 32 == 0): splits z*k.. stay in image z
    hipLaunchKernelGGL(conv_wgrad_bf6_kernel, grid, dim3(256), 0, st, a);
  else if (p.BM == 192)
    hipLaunchKernelGGL(conv_wgrad_halo_kernel<6>, grid, dim3(384), 0, st, a);
  else if (p.BM == 128)
    hipLaunchKernelGGL(conv_wgrad_halo_kernel<4>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(conv_wgrad_halo_kernel<2>, grid, dim3(128), 0, st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(b6 ? PF_ARITH_BF6 : PF_ARITH_FP32);
  const long long per = (long long)Cout * p.Kpad;
  hipLaunchKernelGGL(wgrad_reduce_images_kernel, dim3((unsigned)((per * n + 255) / 256)), dim3(256),
                     0, st, a.part, k, per, n, dw);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// part[z][s] [Cout][Cin] = sum_{m in split s} dy[z][m][co] x[z][m][ci], z < nb,
// in ONE launch (blockIdx.y = z): the Winograd weight gradient's 36
// transform-domain GEMMs (wino.hip), whose output transform sums the nsplit
// partials.  Cin, Cout % 128 == 0; partb (optional) [nsplit][Cout] receives
// the split sums of dy[zb].
int pf_wgrad_gemm_batched(const float* dy, int ldy, long long sdy, const float* x, int xcs,
                          long long sx, int M, int Cin, int Cout, int nb, int nsplit, float* part,
                          float* partb, int zb, hipStream_t st) {
  if (Cin % 128 || Cout % 128 || ldy % 4 || xcs % 4 || nb < 1 || M < 1 || nsplit < 1)
    return POSFEAT_E_INVALID;
  WgradArgs a;
  a.dy = dy;
  a.ldy = ldy;
  a.x = x;
  a.xcs = xcs;
  a.H = 1;
  a.W = M;
  a.Hin = 1;
  a.Win = M;
  a.stride = 1;
  a.d_row = 0;
  a.d_img = 0;
  a.Cin = Cin;
  a.KH = a.KW = 1;
  a.pad = 0;
  a.Cout = Cout;
  a.Kpad = Cin;
  a.K = Cin;
  a.M = M;
  a.tiles_n = Cin / 128;
  a.ntiles = (Cout / 128) * a.tiles_n;
  a.nsplit = nsplit;
  a.nchunks = (M + WG_RB - 1) / WG_RB;
  a.part = part;
  a.partb = partb;
  a.bdy = sdy;
  a.bx = sx;
  a.bpart = (long long)nsplit * Cout * Cin;
  a.zb = zb;
  if (wgrad_bf6_on())
    hipLaunchKernelGGL(conv_wgrad_bf6_kernel, dim3(a.ntiles * nsplit, nb), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<128, 128>), dim3(a.ntiles * nsplit, nb), dim3(256), 0,
                       st, a);
  PF_CHECK_LAUNCH();
  pf_note_arith(wgrad_bf6_on() ? PF_ARITH_BF6 : PF_ARITH_FP32);
  return POSFEAT_OK;
}

int pf_dgrad_weights(const float* w, int Cout, int Cin, int KH, int KW, float* wt,
                     hipStream_t st, unsigned short* planes) {
  if (Cout % 32 || Cin % 32) return POSFEAT_E_INVALID;
  const int kf = posfeat_conv_packed_k(Cin, KH, KW), kt = posfeat_conv_packed_k(Cout, KH, KW);
  const long long n = (long long)Cin * kt;
  hipLaunchKernelGGL(dgrad_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w,
                     Cout, Cin, KH * KW, kf, wt, kt, planes);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_up4_adjoint(const float* g, int gcs, int nb, int OH, int OW, int h, int w, int C, float* t,
                   float* d, int dcs, hipStream_t st) {
  if (C % 4 || gcs % 4 || dcs % 4) return POSFEAT_E_INVALID;
  const int c4n = C / 4;
  hipLaunchKernelGGL(up4_adj_x_kernel, dim3(grid_for((long long)nb * OH * w * c4n, 256)), dim3(256),
                     0, st, g, gcs, nb, OH, OW, w, c4n, t);
  hipLaunchKernelGGL(up4_adj_y_kernel, dim3(grid_for((long long)nb * h * w * c4n, 256)), dim3(256),
                     0, st, t, nb, OH, h, w, c4n, d, dcs);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

size_t pf_in_bwd_ws_bytes(int nb, int hw, int C) {
  const int nchunk = (hw + INB_CHUNK - 1) / INB_CHUNK;
  return pf_align((size_t)nb * nchunk * C * 2 * 8, 256) + pf_align((size_t)nb * nchunk * 8, 256) +
         2 * pf_align((size_t)nb * C * 4, 256);
}

int pf_in_backward(const float* x, int xcs, const float* g, int gcs, int nb, int hw, int C,
                   const float* mean, const float* rstd, const float* slope, float* dx, int dxcs,
                   void* ws, double** slope_part, int* slope_nparts, hipStream_t st) {
  if (C % 4 || C / 4 > 256 || xcs % 4 || gcs % 4 || dxcs % 4) return POSFEAT_E_INVALID;
  const int nchunk = (hw + INB_CHUNK - 1) / INB_CHUNK;
  char* p = static_cast<char*>(ws);
  double* part = reinterpret_cast<double*>(p);
  p += pf_align((size_t)nb * nchunk * C * 2 * 8, 256);
  double* spart = reinterpret_cast<double*>(p);
  p += pf_align((size_t)nb * nchunk * 8, 256);
  float* e1 = reinterpret_cast<float*>(p);
  p += pf_align((size_t)nb * C * 4, 256);
  float* e2 = reinterpret_cast<float*>(p);
  const bool prelu = slope != nullptr;
  if (prelu)
    hipLaunchKernelGGL(in_bwd_partial_kernel<true>, dim3(nchunk, nb), dim3(256), 0, st, x, xcs, g,
                       gcs, hw, C, mean, rstd, slope, part, spart);
  else
    hipLaunchKernelGGL(in_bwd_partial_kernel<false>, dim3(nchunk, nb), dim3(256), 0, st, x, xcs, g,
                       gcs, hw, C, mean, rstd, slope, part, spart);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3((nb * C + 255) / 256), dim3(256), 0, st, part,
                     nchunk, nb, C, hw, e1, e2);
  const long long total = (long long)nb * hw * (C / 4);
  if (prelu)
    hipLaunchKernelGGL(in_bwd_apply_kernel<true>, dim3(grid_for(total, 256)), dim3(256), 0, st, x,
                       xcs, g, gcs, nb, hw, C / 4, mean, rstd, slope, e1, e2, dx, dxcs);
  else
    hipLaunchKernelGGL(in_bwd_apply_kernel<false>, dim3(grid_for(total, 256)), dim3(256), 0, st,
                       x, xcs, g, gcs, nb, hw, C / 4, mean, rstd, slope, e1, e2, dx, dxcs);
  PF_CHECK_LAUNCH();
  if (slope_part) *slope_part = spart;
  if (slope_nparts) *slope_nparts = nb * nchunk;
  return POSFEAT_OK;
}

size_t pf_tail_bwd_ws_bytes(int nb, int hw) {
  const int nchunk = (hw + INB_CHUNK - 1) / INB_CHUNK;
  return pf_align((size_t)nb * nchunk * 2 * 8, 256) + pf_align((size_t)nb * nchunk * 128 * 3 * 8, 256) +
         pf_align((size_t)nb * nchunk * 2 * 8, 256) + 2 * pf_align((size_t)nb * 128 * 4, 256);
}

int pf_tail_backward(const float* dlp, const float* y3, const float* m3, const float* r3,
                     const float* c2, int c2cs, const float* m2, const float* r2,
                     const float* slope, const float* w3, int nb, int hw, float* dy3, float* dc2,
                     int dcs, float* dw3, void* ws, double** t2s, int* t2n, hipStream_t st) {
  const int nchunk = (hw + INB_CHUNK - 1) / INB_CHUNK;
  char* p = static_cast<char*>(ws);
  double* t1 = reinterpret_cast<double*>(p);
  p += pf_align((size_t)nb * nchunk * 2 * 8, 256);
  double* part = reinterpret_cast<double*>(p);
  p += pf_align((size_t)nb * nchunk * 128 * 3 * 8, 256);
  double* spart = reinterpret_cast<double*>(p);
  p += pf_align((size_t)nb * nchunk * 2 * 8, 256);
  float* e1 = reinterpret_cast<float*>(p);
  p += pf_align((size_t)nb * 128 * 4, 256);
  float* e2 = reinterpret_cast<float*>(p);
  hipLaunchKernelGGL(tail1_partial_kernel, dim3(nchunk, nb), dim3(256), 0, st, dlp, y3, hw, m3, r3,
                     t1);
  hipLaunchKernelGGL(tail2_partial_kernel, dim3(nchunk, nb), dim3(256), 0, st, dlp, y3, c2, c2cs,
                     hw, m3, r3, t1, nchunk, m2, r2, slope, w3, dy3, part, spart);
  hipLaunchKernelGGL(tail2_finalize_kernel, dim3(nb), dim3(1024), 0, st, part, nchunk, hw, e1, e2);
  hipLaunchKernelGGL(tail2_dw3_kernel, dim3(1), dim3(128), 0, st, part, nchunk, nb, dw3);
  const long long total = (long long)nb * hw * 32;
  hipLaunchKernelGGL(tail3_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, dy3, c2, c2cs, nb,
                     hw, m2, r2, slope, w3, e1, e2, dc2, dcs);
  PF_CHECK_LAUNCH();
  *t2s = spart;
  *t2n = nb * nchunk;
  return POSFEAT_OK;
}

int pf_head_scalars(const double* t2s, int n2, const double* c1s, int n1, float* db3,
                    float* dslope, hipStream_t st) {
  hipLaunchKernelGGL(head_scalars_kernel, dim3(1), dim3(1024), 0, st, t2s, n2, c1s, n1, db3, dslope);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_sgd(float* w, const float* g, long long n, float lr, void* stream) {
  if (!w || !g || n < 0) return POSFEAT_E_INVALID;
  if (n == 0) return POSFEAT_OK;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, pf_stream(stream), w, g, n,
                     lr);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" size_t posfeat_conv_wgrad_workspace(int n, int h, int w, int cin, int cout, int kh,
                                               int kw) {
  if (n <= 0 || h <= 0 || w <= 0 || cout <= 0 || cin <= 0) return 0;
  return pf_conv_wgrad_ws_bytes(n, h, w, cin, cout, kh, kw, 1);
}

extern "C" int posfeat_conv_wgrad(const float* dy, int dy_cstride, const float* x, int x_cstride,
                                  int n, int h, int w, int cin, int cout, int kh, int kw,
                                  float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  if (!dy || !x || !dw || !ws || n <= 0 || h <= 0 || w <= 0) return POSFEAT_E_INVALID;
  return pf_conv_wgrad(dy, dy_cstride, x, x_cstride, n, h, w, cin, cout, kh, kw, 1, dw, db, 0, ws,
                       ws_bytes, pf_stream(stream));
}
