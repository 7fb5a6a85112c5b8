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

__global__ __launch_bounds__(256) PF_NO_PK_FP32 void up4tap_combine_kernel(const float* __restrict__ P, int h,
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
  pf_syncthreads();                 // ... and every other wave's
  // ---- phase 2 --------------------------------------------------------------
  auto rowR = [&](int ry, f32x4 (&R)[3]) __attribute__((always_inline)) {  // ry: tile row (iy = q0 - 1 + ry)
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
  pf_syncthreads();  // LDS reuse
  double* red = reinterpret_cast<double*>(sp);  // [32 columns][32 channels][2]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[(xl * CB_CG + c4 * 4 + j) * 2] = s1[j];
    red[(xl * CB_CG + c4 * 4 + j) * 2 + 1] = s2[j];
  }
  pf_syncthreads();
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
// bf16x6 over pre-split weight planes -- while its P tile streams in, then
// adds the tap-summed interpolation and writes y once, with the IN
// statistics.
//
// Round 4 layout (the round-3 form was VALU-bound: 4486 VALU per 120 MFMA per
// wave, PMC):
// * The image patch (20 x 36 pixels) is split into its three bf16 planes ONCE
//   per block -- each thread splits a pixel pair from registers -- and stored
//   3-channel packed (GC_S dwords per patch row and plane), so an MFMA operand
//   (8 consecutive k = dx * 3 + c of one patch row) is 8 consecutive bf16.
//   The round-3 kernel split every operand in registers (each patch pixel
//   once per column tile and tap row).
// * The 32 MFMA rows of tile t are 16 output rows x the columns (c, c + 4),
//   c = 8 wave + t: an operand's start element 3c + 8h (+ 12) has the parity of
//   t in every lane, so even tiles read whole dwords and odd tiles one extra
//   dword and a v_alignbit each -- no lane-dependent selects -- and an output
//   column's phase X % 4 is t, a compile-time constant of the interpolation.
// * The P tile is staged through registers into an LDS layout that pairs tile
//   rows: [row pair][column][tap][channel][2 rows], so the x interpolation of
//   two rows is one ds_read_b64 and one v_pk_fma_f32 per tap.  Rows 0-3 load
//   before the G phase and land during it; rows 4-5 share LDS with the patch
//   planes and are written after it (68 KB: two blocks per CU).
// * The y interpolation runs on output-row pairs in packed fp32 with
//   compile-time coefficient pairs; y leaves through buffer stores (uniform row
//   offset, no per-store address arithmetic).
// * Blocks away from the image border (every clamp, the conv's zero padding,
//   the border ring and ragged columns need no test there) take a branch-free
//   instantiation.
// The MFMA roles: A = pixels, B = couts; acc[t][r] of lane (cout n, half h) is
// output row r of column 8 wave + t + 4h -- one channel of one column over all
// 16 rows, the combine's sliding-window layout.  Border-ring pixels take their
// G value from the ring buffer (pf_gfuse_prep: conv2 sees G's zero padding
// there, not the fold).
constexpr int GC_PR = 20, GC_PC = 36;       // image patch rows / pixels (16 x 32 + the 5x5 halo)
constexpr int GC_S = 60;                    // dwords per patch row and plane (54 used; banks)
constexpr int GC_PLANE = GC_PR * GC_S;      // dwords per plane
constexpr int GC_PAIRS = GC_PR * GC_PC / 2;  // pixel pairs of the patch (one split each)
constexpr int GC_K = 80;                    // k = dy * 16 + dx * 3 + c, k % 16 == 15: zero weight
constexpr int GC_CELL = 9 * CB_CG * 2;      // floats per (row pair, column): 9 taps x 32 ch x 2 rows
constexpr int GC_RP = CB_CX * GC_CELL;      // floats per row pair
constexpr int GC_NA = 2 * CB_CX * 9 * (CB_CG / 4);  // P items (2 rows x 4 ch) of rows 0-3
constexpr int GC_NB = CB_CX * 9 * (CB_CG / 4);      // ... of rows 4-5
constexpr int GC_UA = (GC_NA + 255) / 256, GC_UB = (GC_NB + 255) / 256;  // per thread
static_assert(3 * GC_PLANE <= GC_NB * 8, "the patch planes fit over P-tile rows 4-5");
static_assert(16 * 32 * CB_CG + 4 * CB_CG * 4 <= (GC_NA + GC_NB) * 8, "y tile + statistics fit");
static_assert(GC_PAIRS <= 512, "two pixel pairs per thread");

// this wave's LDS operations have completed (vector memory untouched)
__device__ __forceinline__ void gc_wait_lgkm0() {
  __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
}
// wait until at most N vector-memory operations of this wave are outstanding
template <int N>
__device__ __forceinline__ void gc_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// workgroup barrier without the fence __syncthreads() adds (a fence drains
// vmcnt: the loads in flight and the y stores)
__device__ __forceinline__ void gc_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// y-interpolation coefficient of R row i + j (j in -1..1) for output row
// 4 i + r and tap row ky: up4_w of d = r + ky - 1
__host__ __device__ constexpr float gc_cy(int r, int ky, int j) {
  const int d = r + ky - 1;
  const int lo = d <= 1 ? -1 : 0;
  const float wa = d == -1 ? 0.625f : d == 0 ? 0.375f : d == 1 ? 0.125f
                 : d == 2 ? 0.875f : d == 3 ? 0.625f : 0.375f;
  return j == lo ? wa : j == lo + 1 ? 1.f - wa : 0.f;
}

typedef float gc_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gc_f2 gc_fma2(gc_f2 a, gc_f2 b, gc_f2 c) {
  return __builtin_elementwise_fma(a, b, c);
}
__device__ __forceinline__ f32x4 gc_bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// the per-launch arguments of the gcombine kernel
struct GcArgs {
  const float* P;
  const float* img4;
  const unsigned short* wp;
  const float* bc;
  const float* ring;
  float* y;
  double* part;
  int h, w, ycs, nqb, nxb;
  int colmajor;  // block order: tile rows fastest (1) or tile columns fastest (0)
  int ystore;    // 0 (A/B ablation POSFEAT_GC_NOSTORE=1): statistics only, y not written
};

// patch pixel pairs of tile (q0, qx0) of image b into registers
template <bool IN>
__device__ __forceinline__ void gc_issue_patch(const GcArgs& A, int b, int q0, int qx0, int tid,
                                               f32x4 (&px)[2][2]) {
  const int H = 4 * A.h, W = 4 * A.w, Y0 = 4 * q0, X0 = 4 * qx0;
  const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A.img4 + (long long)b * H * W * 4), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = min(tid + 256 * u, GC_PAIRS - 1);
    const int py = j / (GC_PC / 2), pc = 2 * (j - py * (GC_PC / 2));
    const int yy = Y0 - 2 + py, xx = X0 - 2 + pc;
    if (IN) {
      const int o = (yy * W + xx) * 16;
      px[u][0] = gc_bload(irs, o);
      px[u][1] = gc_bload(irs, o + 16);
    } else {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const bool ok = (unsigned)yy < (unsigned)H && (unsigned)(xx + e) < (unsigned)W;
        const f32x4 v =
            gc_bload(irs, (min(max(yy, 0), H - 1) * W + min(max(xx + e, 0), W - 1)) * 16);
        px[u][e] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
}

// P items of tile (q0, qx0), image b, channel group cg into registers: item n
// of row pair rp = tile rows (2 rp, 2 rp + 1), column cx, tap k, channel quad,
// m = n within the row pair = (cx * 9 + k) * 8 + quad; rows 0-3 (RP = 0: the
// two pairs, GC_UA items per thread) or rows 4-5 (RP = 2, GC_UB)
template <bool IN, int RP, int U>
__device__ __forceinline__ void gc_issue_p(const GcArgs& A, int b, int q0, int qx0, int cg,
                                           int tid, f32x4 (&pr)[U][2]) {
  const int h = A.h, w = A.w;
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A.P + (long long)b * h * w * TAP_N + cg * CB_CG), (short)0, 0x7fffffff,
      0x00020000);
  constexpr int NI = RP == 0 ? GC_NA : GC_NB;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int n = min(tid + 256 * u, NI - 1);  // the last item repeats: the same data
    const int rp = RP == 0 ? (n >= GC_NA / 2 ? 1 : 0) : 2;
    const int m = n - (RP == 0 ? rp * (GC_NA / 2) : 0);
    int oa, ob;
    if (IN) {
      oa = (((q0 - 1 + 2 * rp) * w + qx0 - 1) * TAP_N + (m >> 3) * TAP_CO + (m & 7) * 4) * 4;
      ob = oa + w * TAP_N * 4;
    } else {
      const int kk = m >> 3, k = kk % 9, cx = kk / 9;
      const int ix = min(max(qx0 - 1 + cx, 0), w - 1);
      const int ia = min(max(q0 - 1 + 2 * rp, 0), h - 1), ib = min(max(q0 + 2 * rp, 0), h - 1);
      const int c = ix * TAP_N + k * TAP_CO + (m & 7) * 4;
      oa = (ia * w * TAP_N + c) * 4;
      ob = (ib * w * TAP_N + c) * 4;
    }
    pr[u][0] = gc_bload(prs, oa);
    pr[u][1] = gc_bload(prs, ob);
  }
}

// One block = one tile (image b, 16 output rows, 32 output columns, channel
// group cg).  Measured and not kept (r10r): two tiles per block with the next
// tile's patch loaded during this one's combine -- 2457 vs 2272 us (the
// prefetch registers push the combine past 256 registers unless the block is
// restructured around them, and the half-size grid tails worse).
template <bool IN>
__device__ __forceinline__ void gc_block(const GcArgs& A, float* spA, float* spB, int b, int qb,
                                         int xb, int cg) {
  const int h = A.h, w = A.w, H = 4 * h, W = 4 * w, nxb = A.nxb;
  const int q0 = qb * TQ, Y0 = 4 * q0;
  unsigned* pl = reinterpret_cast<unsigned*>(spB);
  f32x4 px[2][2], pA[GC_UA][2], pB[GC_UB][2];
  {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ln = lane & 31;
    const int qx0 = xb * CB_QX, X0 = 4 * qx0;
    const int co = cg * CB_CG + ln;
    const float bias = A.bc[(long long)b * TAP_CO + co];
    const unsigned short* wbase =
        A.wp + (long long)b * 3 * TAP_CO * GC_K + (long long)co * GC_K + 8 * hl;
    gc_issue_patch<IN>(A, b, q0, qx0, tid, px);
    // ---- P rows 0-3 (needed after the G phase, which hides their latency) -----
    gc_issue_p<IN, 0>(A, b, q0, qx0, cg, tid, pA);
    // ---- B operands: this channel group's weight planes ----------------------
    g6_u32x4 wv[5][3];
#pragma unroll
    for (int dy = 0; dy < 5; ++dy)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        wv[dy][p] = *reinterpret_cast<const g6_u32x4*>(wbase + (long long)p * TAP_CO * GC_K + dy * 16);
    // ---- the patch's bf16 planes over P-tile rows 4-5 ------------------------
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = tid + 256 * u;
      if (u == 1 && j >= GC_PAIRS) break;
      const int py = j / (GC_PC / 2);
      const int d = py * GC_S + 3 * (j - py * (GC_PC / 2));
      unsigned hh[3], mm[3], ll[3];
      pf_split3_pair(px[u][0].x, px[u][0].y, hh[0], mm[0], ll[0]);
      pf_split3_pair(px[u][0].z, px[u][1].x, hh[1], mm[1], ll[1]);
      pf_split3_pair(px[u][1].y, px[u][1].z, hh[2], mm[2], ll[2]);
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        pl[d + e] = hh[e];
        pl[GC_PLANE + d + e] = mm[e];
        pl[2 * GC_PLANE + d + e] = ll[e];
      }
    }
    // dword 54 of a row is read (times a zero weight: k = 15) by the last tile
    if (tid < 3 * GC_PR) pl[tid * GC_S + 3 * GC_PC / 2] = 0u;
    // P-tile rows 4-5 into registers (their LDS is the planes' until after G)
    gc_issue_p<IN, 2>(A, b, q0, qx0, cg, tid, pB);
    gc_wait_lgkm0();
    gc_barrier();
    // ---- G part: tile t = output columns (c, c + 4), c = 8 wave + t; A row m =
    // pixel (row (m & 3) + 4 (m >> 3), column c + 4 ((m >> 2) & 1)), k half hl:
    // the 8 bf16 from element 3 (column) + 8 hl of patch row (row + dy), i.e.
    // dword d0 = 12 wave + 6 colsel + 4 hl + (3 t) / 2 (+ a 16-bit shift for odd t)
    const int arow = (ln & 3) + 4 * (ln >> 3), colsel = (ln >> 2) & 1;
    const int pbase = arow * GC_S + 6 * colsel + 4 * hl + 12 * wave;  // even
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 5; ++dy) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        g6_u32x4 f[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const int d = pbase + p * GC_PLANE + dy * GC_S;  // even
          const uint2* q2 = reinterpret_cast<const uint2*>(pl) + (d >> 1);
          if (t == 0) {  // dwords d .. d+3
            const uint2 a = q2[0], c = q2[1];
            f[p] = g6_u32x4{a.x, a.y, c.x, c.y};
          } else if (t == 1) {  // elements from d+1 (odd): dwords d+1 .. d+5, shifted
            const unsigned s0 = pl[d + 1];
            const uint2 a = q2[1], c = q2[2];
            f[p] = g6_u32x4{__builtin_amdgcn_alignbit(a.x, s0, 16),
                            __builtin_amdgcn_alignbit(a.y, a.x, 16),
                            __builtin_amdgcn_alignbit(c.x, a.y, 16),
                            __builtin_amdgcn_alignbit(c.y, c.x, 16)};
          } else if (t == 2) {  // dwords d+3 .. d+6
            const uint2 a = q2[2];
            f[p] = g6_u32x4{pl[d + 3], a.x, a.y, pl[d + 6]};
          } else {  // elements from d+4 (odd): dwords d+4 .. d+8, shifted
            const uint2 a = q2[2], c = q2[3];
            const unsigned s4 = pl[d + 8];
            f[p] = g6_u32x4{__builtin_amdgcn_alignbit(a.y, a.x, 16),
                            __builtin_amdgcn_alignbit(c.x, a.y, 16),
                            __builtin_amdgcn_alignbit(c.y, c.x, 16),
                            __builtin_amdgcn_alignbit(s4, c.y, 16)};
          }
        }
        // the k80 kernel's six products in its order, operands swapped
        f32x16 c = acc[t];
        c = g6_mfma(f[0], wv[dy][0], c);
        c = g6_mfma(f[1], wv[dy][0], c);
        c = g6_mfma(f[0], wv[dy][1], c);
        c = g6_mfma(f[2], wv[dy][0], c);
        c = g6_mfma(f[0], wv[dy][2], c);
        c = g6_mfma(f[1], wv[dy][1], c);
        acc[t] = c;
      }
    }
    // ---- P tile -> LDS: [row pair][column][tap][channel][2 rows] --------------
    auto pstore = [&](float* base, int n, const f32x4& a, const f32x4& c) {
      f32x4* d = reinterpret_cast<f32x4*>(base + 8 * n);
      d[0] = f32x4{a.x, c.x, a.y, c.y};
      d[1] = f32x4{a.z, c.z, a.w, c.w};
    };
#pragma unroll
    for (int u = 0; u < GC_UA; ++u) pstore(spA, min(tid + 256 * u, GC_NA - 1), pA[u][0], pA[u][1]);
    gc_wait_lgkm0();  // every plane read of this wave has completed ...
    gc_barrier();     // ... in every wave: rows 4-5 may overwrite the planes
#pragma unroll
    for (int u = 0; u < GC_UB; ++u) pstore(spB, min(tid + 256 * u, GC_NB - 1), pB[u][0], pB[u][1]);
    // ---- bias; border-ring pixels take the ring value -----------------------
    if (IN) {
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] += bias;
    } else {
      const int nring = 2 * W + 2 * (H - 2);
      const float* rb = A.ring + (long long)b * nring * TAP_CO + co;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int X = X0 + 8 * wave + t + 4 * hl;
        const bool edge_x = X == 0 || X == W - 1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int Y = Y0 + r;
          acc[t][r] = (edge_x || Y == 0 || Y == H - 1) && X < W
                          ? rb[(long long)pf_ring_index(Y, X, H, W) * TAP_CO]
                          : acc[t][r] + bias;
        }
      }
    }
    gc_wait_lgkm0();
    gc_barrier();
    // ---- the upsampled part --------------------------------------------------
    const float ztop = q0 == 0 ? 0.f : 1.f, zbot = q0 + TQ == h ? 0.f : 1.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int X = X0 + 8 * wave + t + 4 * hl;  // X % 4 == t
      // x interpolation: R[rp][ky] = sum_kx wa P[rows][ca][k] + wb P[rows][cb][k]
      // for the tile-row pair rp (k = 3 ky + kx), two rows per v_pk_fma_f32
      int oa[3], ob[3];
      float wa[3], wb[3];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        int lo;
        up4_w(t + kx - 1, lo, wa[kx], wb[kx]);
        int ca, cb;
        if (IN) {
          ca = 1 + 2 * wave + hl + lo;  // tile column of X >> 2, plus lo
          cb = ca + 1;
        } else {
          const int u = X + kx - 1;
          if (u < 0 || u >= W) wa[kx] = wb[kx] = 0.f;
          const int qx = X >> 2;
          ca = min(max(min(qx + lo, w - 1), 0) - (qx0 - 1), CB_CX - 1);
          cb = min(max(min(qx + lo + 1, w - 1), 0) - (qx0 - 1), CB_CX - 1);
        }
        oa[kx] = ca * GC_CELL + kx * 2 * CB_CG + 2 * ln;
        ob[kx] = cb * GC_CELL + kx * 2 * CB_CG + 2 * ln;
      }
      gc_f2 R[3][3];
#pragma unroll
      for (int rp = 0; rp < 3; ++rp) {
        const float* base = rp < 2 ? spA + rp * GC_RP : spB;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          gc_f2 s = {0.f, 0.f};
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const gc_f2 pa = *reinterpret_cast<const gc_f2*>(base + oa[kx] + ky * 6 * CB_CG);
            const gc_f2 pb = *reinterpret_cast<const gc_f2*>(base + ob[kx] + ky * 6 * CB_CG);
            s = gc_fma2(gc_f2{wa[kx], wa[kx]}, pa, s);
            s = gc_fma2(gc_f2{wb[kx], wb[kx]}, pb, s);
          }
          R[rp][ky] = s;
        }
      }
      // y interpolation of output rows 4 i + r from R rows i + j, j in -1..1.
      // Scalar FMAs: the packed form (pairs of output rows, the R value
      // broadcast by op_sel) compiled to v_pk_fma_f32 whose low result reads
      // the high dword of its own destination pair, and gave run-to-run
      // different row-14 values in lanes 48-63 (isa_check
      // fails a build holding that form)
#pragma unroll
      for (int i = 0; i < TQ; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = acc[t][4 * i + r];
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
            for (int j = -1; j <= 1; ++j) {
              float c = gc_cy(r, ky, j);
              if (c == 0.f) continue;
              if (!IN && i == 0 && r == 0 && ky == 0) c *= ztop;  // conv2's zero padding
              if (!IN && i == TQ - 1 && r == 3 && ky == 2) c *= zbot;
              const int ry = i + 1 + j;  // tile row
              o = __builtin_fmaf(c, R[ry >> 1][ky][ry & 1], o);
            }
          }
          acc[t][4 * i + r] = o;
        }
      }
    }
    // ---- the instance-norm statistics (this lane's channel, its 4 columns) ---
    // per column: pairwise fp32 sums of the 16 rows (depth 4; a sequential fp64
    // chain of 64 dependent adds per lane was the tile's longest dependency),
    // then fp64 across the columns and the block
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int X = X0 + 8 * wave + t + 4 * hl;
      if (!IN && X >= W) continue;
      float a[16], q[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        a[r] = acc[t][r];
        q[r] = acc[t][r] * acc[t][r];
      }
#pragma unroll
      for (int st = 8; st >= 1; st >>= 1)
#pragma unroll
        for (int r = 0; r < st; ++r) {
          a[r] += a[r + st];
          q[r] += q[r + st];
        }
      s1 += (double)a[0];
      s2 += (double)q[0];
    }
    s1 += __shfl_xor(s1, 32, 64);  // lanes l and l ^ 32 hold the same channel
    s2 += __shfl_xor(s2, 32, 64);
    // ---- y through LDS: [row][column][channel], then 16-B stores of 4
    // channels (a lane's 16 rows x 1 channel would be 64 dword stores: the
    // store tail was issue-bound) ------------------------------------------------
    // every wave is done reading the P tile: the y tile overwrites it.  (The
    // ISA had no LDS access in flight here already -- the R values were all
    // consumed above -- the wait states it in the source; tools/isa_check.py
    // reports any s_barrier crossed with LDS accesses outstanding.)
    gc_wait_lgkm0();
    gc_barrier();
    if (A.ystore) {
      float* so = spA + (8 * wave + 4 * hl) * CB_CG + ln;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) so[(r * 32 + t) * CB_CG] = acc[t][r];
    }
    double* red = reinterpret_cast<double*>(spA + 16 * 32 * CB_CG);  // [wave][32 channels][2]
    if (A.part && hl == 0) {
      red[(wave * CB_CG + ln) * 2] = s1;
      red[(wave * CB_CG + ln) * 2 + 1] = s2;
    }
    gc_wait_lgkm0();
    gc_barrier();
    if (A.ystore) {
      const int col = tid >> 3, quad = tid & 7, X = X0 + col;
      const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
          A.y + ((long long)b * H + Y0) * W * A.ycs, (short)0, 0x7fffffff, 0x00020000);
      const int yrow = W * A.ycs * 4, xo = (X * A.ycs + cg * CB_CG + quad * 4) * 4;
      const f32x4* si = reinterpret_cast<const f32x4*>(spA) + tid;
      if (IN || X < W) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(g6_u32x4, si[r * 256]), yrs,
                                                 xo, r * yrow, 0);
      }
    }
    // ---- statistics: the block's 32 columns of each channel, fixed order ----
    if (A.part && tid < 2 * CB_CG) {
      const int c = tid >> 1, which = tid & 1;
      double a = 0.0;
      for (int x = 0; x < 4; ++x) a += red[(x * CB_CG + c) * 2 + which];
      const long long chunk = (long long)qb * nxb + xb;
      const long long nchunk = (long long)nxb * A.nqb;
      A.part[(((long long)b * nchunk + chunk) * TAP_CO + cg * CB_CG + c) * 2 + which] = a;
    }
  }
}

// the gcombine block order: tile rows fastest, so a tile's vertical
// neighbours (which share its P halo rows) run 4 blocks later on the same
// XCD while those rows are still in its L2 (gcombine 2.39 -> 2.35 ms, r15b;
// strips of 2 / 4 tile columns measured no better, r15c).  A/B:
// POSFEAT_GC_ORDER=0 -- tile columns fastest
int gc_colmajor() {
  static const int v = [] {
    const char* e = pf_ab_getenv("POSFEAT_GC_ORDER");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

__global__ __launch_bounds__(256, 2) void up4tap_gcombine_kernel(GcArgs A) {
  // P-tile rows 0-3 (spA), the patch planes then rows 4-5 (spB); at the end of
  // each tile the y tile (64 KB) and the statistics
  __shared__ __attribute__((aligned(16))) float smem[(GC_NA + GC_NB) * 8];
  float* spA = smem;
  float* spB = smem + GC_NA * 8;
  const int ncg = TAP_CO / CB_CG;
  // XCD-aware order: blocks are dealt round-robin over the 8 XCDs, so block i
  // takes tile (i % 8) * (n / 8) + i / 8 -- neighbouring tiles, which share P
  // halo columns, run on one XCD's L2
  int id = blockIdx.x;
  if ((gridDim.x & 7) == 0) id = (id & 7) * (gridDim.x >> 3) + (id >> 3);
  const int cg = id % ncg;
  id /= ncg;
  int xb, qb, b;
  if (A.colmajor) {  // tile rows fastest: a tile's vertical neighbours run 4 blocks apart
    qb = id % A.nqb;
    id /= A.nqb;
    xb = id % A.nxb;
    b = id / A.nxb;
  } else {
    xb = id % A.nxb;
    id /= A.nxb;
    qb = id % A.nqb;
    b = id / A.nqb;
  }
  // away from the image border: the branch-free form
  const bool interior = qb > 0 && qb < A.nqb - 1 && xb > 0 && xb * CB_QX + CB_QX < A.w;
  if (interior)
    gc_block<true>(A, spA, spB, b, qb, xb, cg);
  else
    gc_block<false>(A, spA, spB, b, qb, xb, cg);
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
__global__ __launch_bounds__(256) PF_NO_PK_FP32 void up4tap_adjoint_kernel(const float* __restrict__ dy, int dycs,
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
  GcArgs A;
  A.P = P;
  A.img4 = img4;
  A.wp = wp;
  A.bc = bc;
  A.ring = ring;
  A.y = y;
  A.part = mean ? part : nullptr;
  A.h = h;
  A.w = w;
  A.ycs = ycs;
  A.nqb = h / TQ;
  A.nxb = (w + CB_QX - 1) / CB_QX;
  A.colmajor = gc_colmajor();
  {
    static const bool nostore = [] {
      const char* e = pf_ab_getenv("POSFEAT_GC_NOSTORE");
      return e && e[0] == '1';
    }();
    A.ystore = nostore ? 0 : 1;
  }
  const int nblk = n * A.nqb * A.nxb * (TAP_CO / CB_CG);
  hipLaunchKernelGGL(up4tap_gcombine_kernel, dim3(nblk), dim3(256), 0, st, A);
  PF_CHECK_LAUNCH();
  if (mean) PF_TRY(pf_in_finalize(part, n, nchunk, H * W, TAP_CO, mean, rstd, st));
  return POSFEAT_OK;
}

// D (n x H/4 x W/4 x 1152) = the adjoint of pf_up4tap_combine applied to dy
// (n x H x W x 128, pitch dycs): dL/dP.  H, W % 16 == 0.
int pf_up4tap_adjoint(int n, int H, int W, const float* dy, int dycs, float* D, hipStream_t st) {
  const int h = H / 4, w = W / 4;
  if (H % 16 || W % 16 || dycs % 4 || n <= 0) return POSFEAT_E_INVALID;
  // low-res rows per block (A/B POSFEAT_ADJ_TQ=2: 2 -- fewer accumulators,
  // more waves per SIMD, more dy rows re-read; default 4)
  static const int tq = [] {
    const char* e = pf_ab_getenv("POSFEAT_ADJ_TQ");
    return e && e[0] == '2' ? 2 : 4;
  }();
  const long long nb = (long long)n * ((h + tq - 1) / tq) * ((w + 7) / 8);
  if (tq == 2)
    hipLaunchKernelGGL(up4tap_adjoint_kernel<2>, dim3((unsigned)nb), dim3(256), 0, st, dy, dycs, h,
                       w, D);
  else
    hipLaunchKernelGGL(up4tap_adjoint_kernel<4>, dim3((unsigned)nb), dim3(256), 0, st, dy, dycs, h,
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
