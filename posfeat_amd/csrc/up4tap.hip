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

// Block = (image, 4 low-res rows = 16 output rows, 8 low-res columns = 32
// output columns, 32-channel group); thread = (output column X, channel quad).
// Phase 1 stages the P tile the block needs -- low-res rows q0-1 .. q0+4,
// columns qx0-1 .. qx0+8, 9 taps, 32 channels (69 KB) -- into LDS with every
// load independent (17 float4 per thread) and, in the same burst, loads the 16
// y values the thread will update: the HBM latency is paid once per block.
// Phase 2 walks the low-res rows with a sliding window of the x-interpolated
// taps R_ky(iy) = sum_kx [X + kx - 1 in image] (wa P_k[iy][ia] + wb P_k[iy][ib])
// (conflict-free ds_read_b128: a wave reads 2 low-res columns x 128 B), and
// y[4q + r][X] += sum_ky [4q + r + ky - 1 in image] (wa R_ky(q+lo) + wb R_ky(q+lo+1)).
constexpr int CB_QX = 8, CB_CG = 32, CB_RY = TQ + 2, CB_CX = CB_QX + 2;
constexpr int CB_SEG = CB_RY * CB_CX * 9;  // 128-B (32-channel) segments per block
constexpr int CB_SEGP = (CB_SEG + 7) / 8 * 8;  // padded to whole DMA wave-instructions

__global__ __launch_bounds__(256) void up4tap_combine_kernel(const float* __restrict__ P, int h,
                                                             int w, float* __restrict__ y, int ycs,
                                                             double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sp[CB_SEGP * CB_CG];
  const int H = 4 * h, W = 4 * w;
  const int tid = threadIdx.x;
  const int c4 = tid & 7, xl = tid >> 3;  // 8 channel quads x 32 output columns
  const int nxb = (w + CB_QX - 1) / CB_QX, nqb = h / TQ, ncg = TAP_CO / CB_CG;
  int id = blockIdx.x;
  const int cg = id % ncg;
  id /= ncg;
  const int xb = id % nxb;
  id /= nxb;
  const int qb = id % nqb, b = id / nqb;
  const int q0 = qb * TQ, qx0 = xb * CB_QX;
  const int X = qx0 * 4 + xl, qx = X >> 2, rx = X & 3;
  const bool xok = X < W;  // the last column block may be ragged (w % 8 != 0)
  // ---- phase 1: P tile -> LDS by DMA (global_load_lds: no VGPR round trip,
  // every request independent), y -> registers -----------------------------
  // wave-instruction j fills segments 8j .. 8j+7 (lane L: segment 8j + L/8,
  // 16-B piece L%8); the LDS image is segment-contiguous, i.e. lane-linear
  const float* Pb = P + (long long)b * h * w * TAP_N + cg * CB_CG;
  {
    const int lane = tid & 63, wv = tid >> 6;
    for (int j = wv; j < CB_SEGP / 8; j += 4) {
      int seg = j * 8 + (lane >> 3);
      seg = min(seg, CB_SEG - 1);  // pad segments of the last instruction re-read a valid one
      const int k = seg % 9, cell = seg / 9;
      const int cx = cell % CB_CX, ry = cell / CB_CX;
      const int iy = min(max(q0 - 1 + ry, 0), h - 1), ix = min(max(qx0 - 1 + cx, 0), w - 1);
      const float* src = Pb + ((long long)iy * w + ix) * TAP_N + k * TAP_CO + (lane & 7) * 4;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(sp + j * 8 * CB_CG),
                                       16, 0, 0);
    }
  }
  float* yb = y + ((long long)b * H * W + min(X, W - 1)) * ycs + cg * CB_CG + c4 * 4;
  const long long yrow = (long long)W * ycs;
  f32x4 o[TQ][4];
#pragma unroll
  for (int i = 0; i < TQ; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      o[i][r] = xok ? *reinterpret_cast<const f32x4*>(yb + (4 * (q0 + i) + r) * yrow)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
  // column taps: LDS columns (tile-relative) and weights, 0 weight for padding
  int cola[3], colb[3];
  float wxa[3], wxb[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    int lo;
    up4_w(rx + kx - 1, lo, wxa[kx], wxb[kx]);
    const int u = X + kx - 1;
    if (u < 0 || u >= W) wxa[kx] = wxb[kx] = 0.f;
    // clamped source column, expressed in tile coordinates (the tile's own
    // clamped columns hold the same data)
    cola[kx] = min(max(min(qx + lo, w - 1), 0) - (qx0 - 1), CB_CX - 1);
    colb[kx] = min(max(min(qx + lo + 1, w - 1), 0) - (qx0 - 1), CB_CX - 1);
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (y too)
  __syncthreads();                 // ... and every other wave's
  // ---- phase 2 --------------------------------------------------------------
  auto rowR = [&](int ry, f32x4 (&R)[3]) {  // ry: tile row (iy = q0 - 1 + ry)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int k = ky * 3 + kx;
        const f32x4 pa = *reinterpret_cast<const f32x4*>(
            sp + ((ry * CB_CX + cola[kx]) * 9 + k) * CB_CG + c4 * 4);
        const f32x4 pb = *reinterpret_cast<const f32x4*>(
            sp + ((ry * CB_CX + colb[kx]) * 9 + k) * CB_CG + c4 * 4);
        s += wxa[kx] * pa + wxb[kx] * pb;
      }
      R[ky] = s;
    }
  };
  f32x4 Rm[3], R0[3], Rp[3];
  rowR(0, Rm);
  rowR(1, R0);
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < TQ; ++i) {
    rowR(i + 2, Rp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int Y = 4 * (q0 + i) + r;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int v = Y + ky - 1;
        int lo;
        float wa, wb;
        up4_w(r + ky - 1, lo, wa, wb);
        if (v < 0 || v >= H) wa = wb = 0.f;  // conv2's zero padding
        if (lo < 0)
          o[i][r] += wa * Rm[ky] + wb * R0[ky];
        else
          o[i][r] += wa * R0[ky] + wb * Rp[ky];
      }
      if (!xok) continue;
      *reinterpret_cast<f32x4*>(yb + Y * yrow) = o[i][r];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
  // ---- statistics: reduce the 32 columns of each channel (fixed order) -------
  __syncthreads();  // LDS reuse
  double* red = reinterpret_cast<double*>(sp);  // [32 columns][32 channels][2]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[(xl * CB_CG + c4 * 4 + j) * 2] = s1[j];
    red[(xl * CB_CG + c4 * 4 + j) * 2 + 1] = s2[j];
  }
  __syncthreads();
  if (tid < 2 * CB_CG) {
    const int c = tid >> 1, which = tid & 1;
    double a = 0.0;
    for (int x = 0; x < 32; ++x) a += red[(x * CB_CG + c) * 2 + which];
    const long long chunk = (long long)qb * nxb + xb;
    const long long nchunk = (long long)nxb * nqb;
    part[(((long long)b * nchunk + chunk) * TAP_CO + cg * CB_CG + c) * 2 + which] = a;
  }
}

// ---- the combine with head.conv2's G part computed in place -----------------
// up4tap_combine_kernel above adds the upsampled part to y = G part + bias,
// which gfuse_conv5_k80_kernel wrote beforehand: y crosses HBM three times
// (write, read, write; 3 x 5 GB at B = 32, 480 x 640).  Here the same block
// (image, 16 output rows, 32 output columns, 32 channels) first computes its G
// part -- the per-image folded 5x5 conv of the image (gfuse.hip), K = 80
// bf16x6 over pre-split weight planes -- while its P tile streams into LDS,
// then adds the tap-summed interpolation and writes y once, with the IN
// statistics.  The MFMA roles are swapped against the k80 kernel (A = pixels,
// B = couts), with the 32 M rows of a tile mapped to 16 rows x 2 columns:
// acc[r] of lane (cout n, half h) is then output row r of column 2p + h, i.e.
// a lane holds one channel of one output column over all 16 rows -- exactly
// the combine's per-thread sliding-window layout (one channel instead of a
// quad), so the accumulators become the combine's running sums with no LDS
// transpose.  Border-ring pixels take their G value from the ring buffer
// (pf_gfuse_prep: conv2 sees G's zero padding there, not the fold).
constexpr int GC_PR = 20, GC_PC = 36;  // image patch rows / pixels (16 x 32 + the 5x5 halo)
constexpr int GC_PP = 38;              // LDS pixel slots per patch row (conflict-free b128 A reads)
constexpr int GC_PDMA = 12;            // patch DMA instructions (64 slots each, >= 20 x 38)
constexpr int GC_K = 80;               // k = dy * 16 + dx * 3 + c, k % 16 == 15: zero weight
constexpr int GC_DMA = CB_SEGP / 8 / 4;  // P-tile DMA instructions per wave
static_assert(CB_SEGP % 32 == 0, "P-tile DMA instructions split evenly over the 4 waves");
static_assert(GC_PDMA % 4 == 0 && GC_PDMA * 64 >= GC_PR * GC_PP, "patch DMA covers the patch");
__device__ float gc_zero4[4];  // the DMA source of patch pixels outside the image

// wait until at most N vector-memory operations of this wave are outstanding
template <int N>
__device__ __forceinline__ void gc_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__global__ __launch_bounds__(256, 2) void up4tap_gcombine_kernel(
    const float* __restrict__ P, int h, int w, const float* __restrict__ img4,
    const unsigned short* __restrict__ wp, const float* __restrict__ bc,
    const float* __restrict__ ring, float* __restrict__ y, int ycs, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sp[CB_SEGP * CB_CG];
  __shared__ __attribute__((aligned(16))) float spat[GC_PDMA * 64 * 4];  // [row][38 slots][4]
  const int H = 4 * h, W = 4 * w;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ln = lane & 31;
  const int nxb = (w + CB_QX - 1) / CB_QX, nqb = h / TQ, ncg = TAP_CO / CB_CG;
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs, so block i
  // takes tile (i % 8) * (n / 8) + i / 8 -- neighbouring tiles, which share P
  // halo columns, run on one XCD's L2
  int id = blockIdx.x;
  if ((gridDim.x & 7) == 0) id = (id & 7) * (gridDim.x >> 3) + (id >> 3);
  const int cg = id % ncg;
  id /= ncg;
  const int xb = id % nxb;
  id /= nxb;
  const int qb = id % nqb, b = id / nqb;
  const int q0 = qb * TQ, qx0 = xb * CB_QX, Y0 = 4 * q0, X0 = 4 * qx0;
  // ---- loads, in this order: the B operands (this channel group's weight
  // planes) into registers, then the image patch and the P tile by DMA.  The
  // MFMA phase waits for all but the P tile's 17 instructions --------------
  const int co = cg * CB_CG + ln;
  const float bias = bc[(long long)b * TAP_CO + co];
  g6_u32x4 wv[5][3];
  {
    const unsigned short* wb = wp + (long long)b * 3 * TAP_CO * GC_K + (long long)co * GC_K + 8 * hl;
#pragma unroll
    for (int dy = 0; dy < 5; ++dy)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        wv[dy][pl] = *reinterpret_cast<const g6_u32x4*>(wb + (long long)pl * TAP_CO * GC_K + dy * 16);
  }
  __builtin_amdgcn_sched_barrier(0);
  const float* ib = img4 + (long long)b * H * W * 4;
#pragma unroll
  for (int jj = 0; jj < GC_PDMA / 4; ++jj) {  // slot s -> patch pixel (s / 38, s % 38)
    const int j = wave + 4 * jj, s = j * 64 + lane;
    const int py = s / GC_PP, px = s - py * GC_PP;
    const int yy = Y0 - 2 + py, xx = X0 - 2 + px;
    const bool ok = py < GC_PR && px < GC_PC && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
    const float* src = ok ? ib + ((long long)yy * W + xx) * 4 : gc_zero4;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(spat + j * 64 * 4),
                                     16, 0, 0);
  }
  const float* Pb = P + (long long)b * h * w * TAP_N + cg * CB_CG;
#pragma unroll
  for (int jj = 0; jj < GC_DMA; ++jj) {  // as up4tap_combine_kernel's phase 1
    const int j = wave + 4 * jj;
    int seg = j * 8 + (lane >> 3);
    seg = min(seg, CB_SEG - 1);
    const int k = seg % 9, cell = seg / 9;
    const int cx = cell % CB_CX, ry = cell / CB_CX;
    const int iy = min(max(q0 - 1 + ry, 0), h - 1), ix = min(max(qx0 - 1 + cx, 0), w - 1);
    const float* src = Pb + ((long long)iy * w + ix) * TAP_N + k * TAP_CO + (lane & 7) * 4;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(sp + j * 8 * CB_CG),
                                     16, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  gc_wait_vmcnt<GC_DMA>();        // weights + this wave's patch DMA have landed
  asm volatile("" ::: "memory");  // no LDS access moves across the barrier
  __builtin_amdgcn_s_barrier();   // ... and every wave's (no fence: it would drain the P tile)
  asm volatile("" ::: "memory");
  // ---- G part: wave = 4 column pairs p = 4 wave + t; A row m = pixel (row
  // (m & 3) + 4 (m >> 3), column 2p + ((m >> 2) & 1)), k half hl: the 8 taps
  // k = 8 hl .. 8 hl + 7 of row dy are channels of the three pixels from
  // column 2p + (m's column) + 2 hl on -- (c0 c1 c2 | c0 c1 c2 | c0 c1) for
  // hl = 0, (c2 | c0 c1 c2 | c0 c1 c2 | 0) for hl = 1 (k = 15: zero weight)
  const int arow = (ln & 3) + 4 * (ln >> 3), acol = (ln >> 2) & 1;
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
  for (int dy = 0; dy < 5; ++dy) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const f32x4* pr = reinterpret_cast<const f32x4*>(spat) + (arow + dy) * GC_PP +
                        2 * (4 * wave + t) + acol + 2 * hl;
      const f32x4 a = pr[0], bq = pr[1], cq = pr[2];
      f32x4 p0, p1;
      p0[0] = hl ? a.z : a.x;
      p0[1] = hl ? bq.x : a.y;
      p0[2] = hl ? bq.y : a.z;
      p0[3] = hl ? bq.z : bq.x;
      p1[0] = hl ? cq.x : bq.y;
      p1[1] = hl ? cq.y : bq.z;
      p1[2] = hl ? cq.z : cq.x;
      p1[3] = hl ? 0.f : cq.y;
      g6_u32x4 ph, pm, plo;
      g6_split(p0, p1, ph, pm, plo);
      // the k80 kernel's six products in its order, operands swapped
      f32x16 c = acc[t];
      c = g6_mfma(ph, wv[dy][0], c);
      c = g6_mfma(pm, wv[dy][0], c);
      c = g6_mfma(ph, wv[dy][1], c);
      c = g6_mfma(plo, wv[dy][0], c);
      c = g6_mfma(ph, wv[dy][2], c);
      c = g6_mfma(pm, wv[dy][1], c);
      acc[t] = c;
    }
  }
  const int nring = 2 * W + 2 * (H - 2);
  const float* rb = ring + (long long)b * nring * TAP_CO + co;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int X = X0 + 2 * (4 * wave + t) + hl;
    const bool edge_x = X == 0 || X == W - 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int Y = Y0 + r;
      acc[t][r] = (edge_x || Y == 0 || Y == H - 1) && X < W
                      ? rb[(long long)pf_ring_index(Y, X, H, W) * TAP_CO]
                      : acc[t][r] + bias;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed
  __syncthreads();                 // ... and every other wave's
  // ---- the upsampled part: per column, the sliding window of
  // up4tap_combine_kernel on one channel ---------------------------------------
  double s1 = 0.0, s2 = 0.0;
  const long long yrow = (long long)W * ycs;
  float* yb = y + (long long)b * H * W * ycs + co;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int X = X0 + 2 * (4 * wave + t) + hl, qx = X >> 2, rx = X & 3;
    const bool xok = X < W;
    int cola[3], colb[3];
    float wxa[3], wxb[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      int lo;
      up4_w(rx + kx - 1, lo, wxa[kx], wxb[kx]);
      const int u = X + kx - 1;
      if (u < 0 || u >= W) wxa[kx] = wxb[kx] = 0.f;
      cola[kx] = min(max(min(qx + lo, w - 1), 0) - (qx0 - 1), CB_CX - 1);
      colb[kx] = min(max(min(qx + lo + 1, w - 1), 0) - (qx0 - 1), CB_CX - 1);
    }
    auto rowR = [&](int ry, float (&R)[3]) {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        float s = 0.f;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int k = ky * 3 + kx;
          const float pa = sp[((ry * CB_CX + cola[kx]) * 9 + k) * CB_CG + ln];
          const float pb = sp[((ry * CB_CX + colb[kx]) * 9 + k) * CB_CG + ln];
          s += wxa[kx] * pa + wxb[kx] * pb;
        }
        R[ky] = s;
      }
    };
    float Rm[3], R0[3], Rp[3];
    rowR(0, Rm);
    rowR(1, R0);
#pragma unroll
    for (int i = 0; i < TQ; ++i) {
      rowR(i + 2, Rp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int Y = Y0 + 4 * i + r;
        float o = acc[t][4 * i + r];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int v = Y + ky - 1;
          int lo;
          float wa, wb;
          up4_w(r + ky - 1, lo, wa, wb);
          if (v < 0 || v >= H) wa = wb = 0.f;
          if (lo < 0)
            o += wa * Rm[ky] + wb * R0[ky];
          else
            o += wa * R0[ky] + wb * Rp[ky];
        }
        if (!xok) continue;
        yb[Y * yrow + (long long)X * ycs] = o;
        s1 += (double)o;
        s2 += (double)o * (double)o;
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        Rm[ky] = R0[ky];
        R0[ky] = Rp[ky];
      }
    }
  }
  if (!part) return;
  // ---- statistics: the block's 32 columns of each channel, fixed order ------
  __syncthreads();  // LDS reuse
  double* red = reinterpret_cast<double*>(sp);  // [wave][half][32 channels][2]
  red[((wave * 2 + hl) * CB_CG + ln) * 2] = s1;
  red[((wave * 2 + hl) * CB_CG + ln) * 2 + 1] = s2;
  __syncthreads();
  if (tid < 2 * CB_CG) {
    const int c = tid >> 1, which = tid & 1;
    double a = 0.0;
    for (int x = 0; x < 8; ++x) a += red[(x * CB_CG + c) * 2 + which];
    const long long chunk = (long long)qb * nxb + xb;
    const long long nchunk = (long long)nxb * nqb;
    part[(((long long)b * nchunk + chunk) * TAP_CO + cg * CB_CG + c) * 2 + which] = a;
  }
}

// ---- adjoint (keypoint-head training, config 5) ------------------------------
// weight with which low-res index i feeds full-res coordinate u of an n -> 4n
// bilinear upsample (align_corners=False): u's two clamped source taps
// (ia, wa), (ib, wb) as in the forward above (a tap clamped onto its partner
// adds its weight to it, as ATen's weight (1, 0) at the border); 0 outside
// [0, 4n): the conv's zero padding
__device__ __forceinline__ float up4_cw(int u, int i, int n) {
  if (u < 0 || u >= 4 * n) return 0.f;
  int lo;
  float wa, wb;
  up4_w(u & 3, lo, wa, wb);
  const int q = u >> 2;
  const int ia = min(max(q + lo, 0), n - 1), ib = min(max(q + lo + 1, 0), n - 1);
  return (ia == i ? wa : 0.f) + (ib == i ? wb : 0.f);
}

// D[b][iy][ix][k * 128 + co] = dL/dP_k = sum over the full-res output pixels
// (Y, X) of cw(v, iy) cw(u, ix) dy[b][Y][X][co], v = Y + ky - 1, u = X + kx - 1:
// the adjoint of the combine's tap-summed interpolation.  Thread = (low-res
// column ix, channel quad); block = 8 columns x 32 quads of one image over TQ
// low-res rows.  Separable: per dy row Y the x-adjoint
// E_kx = sum_u cw(u, ix) dy[Y][u - kx + 1] (10 float4 loads, 24 FMAs), then
// each E_kx goes to the (iy, ky) accumulators whose v = Y + ky - 1 lies in iy's
// support [4 iy - 2, 4 iy + 5] (which pairs those are is fixed at compile time;
// the weight itself clamps at the borders).
template <int TQ>
__global__ __launch_bounds__(256) void up4tap_adjoint_kernel(const float* __restrict__ dy, int dycs,
                                                             int h, int w, float* __restrict__ D) {
  const int H = 4 * h, W = 4 * w;
  const int tid = threadIdx.x, cq = tid & 31, xl = tid >> 5;
  const int nxb = (w + 7) / 8, nqb = (h + TQ - 1) / TQ;
  int id = blockIdx.x;
  const int xb = id % nxb;
  id /= nxb;
  const int qb = id % nqb, b = id / nqb;
  const int ix = xb * 8 + xl, q0 = qb * TQ;
  const bool active = ix < w;
  float wx[8];  // u = 4 ix - 2 + j
#pragma unroll
  for (int j = 0; j < 8; ++j) wx[j] = active ? up4_cw(4 * ix - 2 + j, ix, w) : 0.f;
  f32x4 acc[TQ][9];
#pragma unroll
  for (int t = 0; t < TQ; ++t)
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[t][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* dyb = dy + (long long)b * H * W * dycs + cq * 4;
  const int Y0 = 4 * q0 - 3;
#pragma unroll
  for (int ry = 0; ry < 4 * TQ + 6; ++ry) {
    const int Y = Y0 + ry;
    if (Y < 0 || Y >= H) continue;
    f32x4 d[10];  // X = 4 ix - 3 + j
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int X = 4 * ix - 3 + j;
      d[j] = active && X >= 0 && X < W
                 ? *reinterpret_cast<const f32x4*>(dyb + ((long long)Y * W + X) * dycs)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 E[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 8; ++j) s += wx[j] * d[j + 2 - kx];
      E[kx] = s;
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int rv = ry + ky - 4;  // v - 4 q0
#pragma unroll
      for (int t = 0; t < TQ; ++t) {
        if (rv < 4 * t - 2 || rv > 4 * t + 5) continue;
        const float cy = up4_cw(Y + ky - 1, q0 + t, h);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc[t][ky * 3 + kx] += cy * E[kx];
      }
    }
  }
  if (!active) return;
#pragma unroll
  for (int t = 0; t < TQ; ++t) {
    const int iy = q0 + t;
    if (iy >= h) break;
    float* o = D + (((long long)b * h + iy) * w + ix) * TAP_N + cq * 4;
#pragma unroll
    for (int k = 0; k < 9; ++k) *reinterpret_cast<f32x4*>(o + k * TAP_CO) = acc[t][k];
  }
}

// WtT[ci][k * 128 + co] = W2[co][ci][ky][kx], ci < 192: dL = D . WtT^T
__global__ void up4tap_weights_t_kernel(const float* __restrict__ w2p, float* __restrict__ wt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= TAP_N * TAP_CU) return;
  const int ci = i / TAP_N, o = i - ci * TAP_N;
  const int k = o / TAP_CO, co = o - k * TAP_CO;
  wt[i] = w2p[(long long)co * TAP_KP2 + (ci >> 5) * 288 + k * 32 + (ci & 31)];
}

}  // namespace

size_t pf_up4tap_weights_floats() { return (size_t)TAP_N * TAP_CU; }
size_t pf_up4tap_p_floats(int n, int H, int W) { return (size_t)n * (H / 4) * (W / 4) * TAP_N; }
size_t pf_up4tap_part_bytes(int n, int H, int W) {
  return (size_t)n * ((H / 4) / TQ) * ((W / 4 + CB_QX - 1) / CB_QX) * TAP_CO * 2 * sizeof(double);
}

int pf_up4tap_weights(const float* w2_packed, float* wt, hipStream_t st) {
  hipLaunchKernelGGL(up4tap_weights_kernel, dim3((TAP_N * TAP_CU + 255) / 256), dim3(256), 0, st,
                     w2_packed, wt);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// y (n x H x W x 128, pitch ycs) += the upsampled part of head.conv2 from the
// nine tap maps P (n x H/4 x W/4 x 1152); mean/rstd (optional) = the
// instance-norm statistics of the resulting y.  H, W % 16 == 0.
int pf_up4tap_combine(int n, int H, int W, const float* P, float* y, int ycs, double* part,
                      float* mean, float* rstd, hipStream_t st) {
  const int h = H / 4, w = W / 4;
  if (H % 16 || W % 16 || ycs % 4 || n <= 0) return POSFEAT_E_INVALID;
  if (mean && !part) return POSFEAT_E_INVALID;
  const int nchunk = (h / TQ) * ((w + CB_QX - 1) / CB_QX);
  hipLaunchKernelGGL(up4tap_combine_kernel, dim3(n * nchunk * (TAP_CO / CB_CG)), dim3(256), 0, st,
                     P, h, w, y, ycs, mean ? part : nullptr);
  PF_CHECK_LAUNCH();
  if (mean) PF_TRY(pf_in_finalize(part, n, nchunk, H * W, TAP_CO, mean, rstd, st));
  return POSFEAT_OK;
}

// y (n x H x W x 128, pitch ycs) = head.conv2's full output: the G part from
// the image (img4, pitch 4) with the pre-split weight planes wp and biases bc
// of pf_gfuse_weights / pf_gfuse_prep, the border ring from `ring`, plus the
// upsampled part from P; mean/rstd (optional) its instance-norm statistics.
// The same part layout as pf_up4tap_combine.  H, W % 16 == 0.
int pf_up4tap_gcombine(int n, int H, int W, const float* P, const float* img4,
                       const unsigned short* wp, const float* bc, const float* ring, float* y,
                       int ycs, double* part, float* mean, float* rstd, hipStream_t st) {
  const int h = H / 4, w = W / 4;
  if (H % 16 || W % 16 || ycs % 4 || ycs < TAP_CO || n <= 0) return POSFEAT_E_INVALID;
  if (!P || !img4 || !wp || !bc || !ring || !y || (mean && !part)) return POSFEAT_E_INVALID;
  const int nchunk = (h / TQ) * ((w + CB_QX - 1) / CB_QX);
  hipLaunchKernelGGL(up4tap_gcombine_kernel, dim3(n * nchunk * (TAP_CO / CB_CG)), dim3(256), 0, st,
                     P, h, w, img4, wp, bc, ring, y, ycs, mean ? part : nullptr);
  PF_CHECK_LAUNCH();
  if (mean) PF_TRY(pf_in_finalize(part, n, nchunk, H * W, TAP_CO, mean, rstd, st));
  return POSFEAT_OK;
}

// D (n x H/4 x W/4 x 1152) = the adjoint of pf_up4tap_combine applied to dy
// (n x H x W x 128, pitch dycs): dL/dP.  H, W % 16 == 0.
int pf_up4tap_adjoint(int n, int H, int W, const float* dy, int dycs, float* D, hipStream_t st) {
  const int h = H / 4, w = W / 4;
  constexpr int TQA = 4;
  if (H % 16 || W % 16 || dycs % 4 || n <= 0) return POSFEAT_E_INVALID;
  const long long nb = (long long)n * ((h + TQA - 1) / TQA) * ((w + 7) / 8);
  hipLaunchKernelGGL(up4tap_adjoint_kernel<TQA>, dim3((unsigned)nb), dim3(256), 0, st, dy, dycs, h,
                     w, D);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_up4tap_weights_t(const float* w2_packed, float* wt, hipStream_t st) {
  hipLaunchKernelGGL(up4tap_weights_t_kernel, dim3((TAP_N * TAP_CU + 255) / 256), dim3(256), 0, st,
                     w2_packed, wt);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
