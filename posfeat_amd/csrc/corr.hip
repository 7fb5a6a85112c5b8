// corr.hip -- training-side dense descriptor correlation on gfx950.
//
// Replaces (forward) Preprocess_Line2Window.forward (losses/preprocess.py:27-121)
// with its helpers generate_kpts_regular_grid_random (preprocess_utils.py:598-659),
// epipolar_line_search (661-694), get_endpoints (696-719),
// get_expected_correspondence_within_window (721-758), and
// EpipolarLoss_full.forward (losses/epipolarloss.py:38-101).
//
// Pipeline per call (B pairs, n = (H/g)*(W/g) grid points per image):
//   grid_points      sel (Categorical draw per g x g cell) -> normalised+pixel coords
//   sample_desc      L2-normalised descriptors at the grid points (sample.hip)
//   l2norm_scale     fm = T * normalize(xf) per pixel (NHWC)
//   cos-sim          S = f1 f2^T  (conv_mfma 1x1 implicit GEMM, FP32 MFMA)
//   row/col stats    softmax(T S) along n and along m with the coordinate
//                    expectations and stds (online softmax, fp32)
//   line_window      one wave per query point: epipolar endpoints, 100
//                    border-padded bilinear samples of fm along the line,
//                    dot/softmax/arg-max (+ loc_rand jitter), then the
//                    12x16 window of zero-padded samples around it,
//                    softmax expectation + std
//   epipolar_loss    one workgroup: costs, masks, std weights, means
// Random draws (grid sel, jitter) are inputs: the caller owns the RNG.
#include <algorithm>

#include "common.h"

int pf_sample_desc(const float* fmap, int b, int c, int h, int w, int cs, const float* coord,
                   int npts, const int32_t* n_valid, int normalize, float* out, hipStream_t st);

namespace {

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += pf_shfl_xor(v, o, 64);
  return v;
}

// torch.linspace(lo, hi, n)[i] in float32 (ATen's two-sided formula)
__device__ __forceinline__ float linspace_f(float lo, float hi, int n, int i) {
  if (n == 1) return lo;
  const float step = __fdiv_rn(__fsub_rn(hi, lo), (float)(n - 1));
  return i < n / 2 ? __fadd_rn(lo, __fmul_rn(step, (float)i))
                   : __fsub_rn(hi, __fmul_rn(step, (float)(n - 1 - i)));
}

__global__ void grid_points_kernel(const int32_t* __restrict__ sel, int nb, int H, int W, int g,
                                   float* __restrict__ cn, float* __restrict__ cp) {
  const int hc = H / g, wc = W / g, n = hc * wc;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * n) return;
  const int k = i % n;
  const int cy = k / wc, cx = k - cy * wc;
  const int s = sel[i];
  const int iy = cy * g + s / g, ix = cx * g + s % g;
  const float xn = linspace_f(-1.f, 1.f, W, ix), yn = linspace_f(-1.f, 1.f, H, iy);
  cn[2 * i] = xn;
  cn[2 * i + 1] = yn;
  // denormalize_coords: n * c + c, c = ((W-1)/2, (H-1)/2)
  const float c0 = (float)((W - 1) / 2.0), c1 = (float)((H - 1) / 2.0);
  cp[2 * i] = __fadd_rn(__fmul_rn(xn, c0), c0);
  cp[2 * i + 1] = __fadd_rn(__fmul_rn(yn, c1), c1);
}

// y[p][c] = scale * x[p][c] / max(||x[p]||, 1e-12), C == 128, one wave per pixel
__global__ void l2norm_scale_kernel(const float* __restrict__ x, long long npix, int cs,
                                    float scale, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= npix) return;
  const float a = x[wid * cs + lane], b = x[wid * cs + lane + 64];
  const float inv = 1.f / fmaxf(sqrtf(pf_wave_sum(a * a + b * b)), 1e-12f);
  y[wid * 128 + lane] = scale * (a * inv);
  y[wid * 128 + lane + 64] = scale * (b * inv);
}

// softmax_n(T*S[m][:]) expectations; one wave per row m.
//   g  = sum_n p c2px[n]       (pixels)
//   sd = sum_d sqrt(max(sum_n p c2n[n]_d^2 - normalize(g)_d^2, 1e-6))
__global__ void corr_row_kernel(const float* __restrict__ S, int nb, int n1, int n2, float T,
                                const float* __restrict__ c2px, const float* __restrict__ c2n,
                                int H2, int W2, float* __restrict__ g, float* __restrict__ sd) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n1) return;
  const int b = (int)(wid / n1);
  const float* row = S + wid * n2;
  const float* cp = c2px + (long long)b * n2 * 2;
  const float* cn = c2n + (long long)b * n2 * 2;
  float mx = -INFINITY;
  for (int k = lane; k < n2; k += 64) mx = fmaxf(mx, T * row[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, pf_shfl_xor(mx, o, 64));
  // fp64 accumulation of the softmax moments: var = E[n^2] - E[n]^2 cancels
  // catastrophically in fp32 when the softmax is peaked (small std); the
  // weights e and the coordinates stay the fp32 values the reference uses
  double se = 0.0, gx = 0.0, gy = 0.0, qx = 0.0, qy = 0.0;
  for (int k = lane; k < n2; k += 64) {
    const double e = (double)expf(T * row[k] - mx);
    const double nx = cn[2 * k], ny = cn[2 * k + 1];
    se += e;
    gx += e * (double)cp[2 * k];
    gy += e * (double)cp[2 * k + 1];
    qx += e * nx * nx;
    qy += e * ny * ny;
  }
  se = wave_sum_d(se);
  gx = wave_sum_d(gx) / se;
  gy = wave_sum_d(gy) / se;
  qx = wave_sum_d(qx) / se;
  qy = wave_sum_d(qy) / se;
  if (lane == 0) {
    g[wid * 2] = (float)gx;
    g[wid * 2 + 1] = (float)gy;
    const double c0 = (W2 - 1) / 2.0, c1 = (H2 - 1) / 2.0;
    const double nx = (gx - c0) / c0, ny = (gy - c1) / c1;
    sd[wid] = (float)(sqrt(fmax(qx - nx * nx, 1e-6)) + sqrt(fmax(qy - ny * ny, 1e-6)));
  }
}

// softmax_m(T*S[:][n]) expectations, two levels: block = 64 columns x one of
// COL_CH row chunks with 4 row lanes per column (coalesced 256-B row reads),
// online max-rescaled accumulation of (sum e, e*px, e*py, e*nx^2, e*ny^2);
// then the chunk partials are merged in order (deterministic).
constexpr int COL_CH = 8;
struct ColAcc {  // running max (fp32, the logits' type) + fp64 moments
  float mx;
  double se, gx, gy, qx, qy;
};

__global__ __launch_bounds__(256) void corr_col_partial_kernel(
    const float* __restrict__ S, int n1, int n2, float T, const float* __restrict__ c1px,
    const float* __restrict__ c1n, ColAcc* __restrict__ part) {
  const int b = blockIdx.z, ch = blockIdx.y, rg = threadIdx.x >> 6, cl = threadIdx.x & 63;
  const int col = blockIdx.x * 64 + cl;
  const int m0 = (int)((long long)n1 * ch / COL_CH), m1 = (int)((long long)n1 * (ch + 1) / COL_CH);
  const float* Sb = S + (long long)b * n1 * n2;
  const float* cp = c1px + (long long)b * n1 * 2;
  const float* cn = c1n + (long long)b * n1 * 2;
  ColAcc a{-INFINITY, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (col < n2) {
    for (int m = m0 + rg; m < m1; m += 4) {
      const float v = T * Sb[(long long)m * n2 + col];
      const double px = cp[2 * m], py = cp[2 * m + 1], nx = cn[2 * m], ny = cn[2 * m + 1];
      double e;
      if (v > a.mx) {
        const double f = (double)expf(a.mx - v);
        a.se *= f;
        a.gx *= f;
        a.gy *= f;
        a.qx *= f;
        a.qy *= f;
        a.mx = v;
        e = 1.0;
      } else {
        e = (double)expf(v - a.mx);
      }
      a.se += e;
      a.gx += e * px;
      a.gy += e * py;
      a.qx += e * nx * nx;
      a.qy += e * ny * ny;
    }
  }
  __shared__ ColAcc sh[4][64];
  sh[rg][cl] = a;
  pf_syncthreads();
  if (rg == 0 && col < n2) {
    float M = sh[0][cl].mx;
    for (int r = 1; r < 4; ++r) M = fmaxf(M, sh[r][cl].mx);
    ColAcc o{M, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int r = 0; r < 4; ++r) {
      const ColAcc& q = sh[r][cl];
      const double f = (double)expf(q.mx - M);
      o.se += q.se * f;
      o.gx += q.gx * f;
      o.gy += q.gy * f;
      o.qx += q.qx * f;
      o.qy += q.qy * f;
    }
    part[((long long)b * COL_CH + ch) * n2 + col] = o;
  }
}

__global__ void corr_col_final_kernel(const ColAcc* __restrict__ part, int nb, int n2, int H1,
                                      int W1, float* __restrict__ g, float* __restrict__ sd) {
  const long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (o >= (long long)nb * n2) return;
  const int b = (int)(o / n2), col = (int)(o - (long long)b * n2);
  const ColAcc* p = part + (long long)b * COL_CH * n2 + col;
  float M = -INFINITY;
  for (int ch = 0; ch < COL_CH; ++ch) M = fmaxf(M, p[(long long)ch * n2].mx);
  double se = 0.0, gx = 0.0, gy = 0.0, qx = 0.0, qy = 0.0;
  for (int ch = 0; ch < COL_CH; ++ch) {
    const ColAcc& q = p[(long long)ch * n2];
    const double f = (double)expf(q.mx - M);
    se += q.se * f;
    gx += q.gx * f;
    gy += q.gy * f;
    qx += q.qx * f;
    qy += q.qy * f;
  }
  gx /= se;
  gy /= se;
  qx /= se;
  qy /= se;
  g[o * 2] = (float)gx;
  g[o * 2 + 1] = (float)gy;
  const double c0 = (W1 - 1) / 2.0, c1 = (H1 - 1) / 2.0;
  const double nx = (gx - c0) / c0, ny = (gy - c1) / c1;
  sd[o] = (float)(sqrt(fmax(qx - nx * nx, 1e-6)) + sqrt(fmax(qy - ny * ny, 1e-6)));
}

// bilinear sample of a 128-channel NHWC map at normalised (x, y), align_corners
// False; border: clamp the source index (padding_mode='border'), else zeros.
// Returns this lane's two channels (lane, lane+64).
template <bool BORDER>
__device__ __forceinline__ float2 bilinear128(const float* __restrict__ fm, int h, int w, float gx,
                                              float gy, int lane) {
  float ix = ((gx + 1.f) * w - 1.f) / 2.f;
  float iy = ((gy + 1.f) * h - 1.f) / 2.f;
  if (BORDER) {
    ix = fminf(fmaxf(ix, 0.f), (float)(w - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(h - 1));
  }
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  const float wx1 = ix - fx, wx0 = 1.f - wx1;  // (x1 - ix), (ix - x0)
  const float wy1 = iy - fy, wy0 = 1.f - wy1;
  // branch-free: every corner is loaded (index clamped into the map) and a
  // corner outside it weighs 0, so a loop over samples can keep several
  // samples' loads in flight; the sums keep their order (x + 0 p = x)
  const bool bx0 = (unsigned)x0 < (unsigned)w, bx1 = (unsigned)x1 < (unsigned)w;
  const bool by0 = (unsigned)y0 < (unsigned)h, by1 = (unsigned)y1 < (unsigned)h;
  const int cx0 = min(max(x0, 0), w - 1), cx1 = min(max(x1, 0), w - 1);
  const int cy0 = min(max(y0, 0), h - 1), cy1 = min(max(y1, 0), h - 1);
  const float* p00 = fm + ((long long)cy0 * w + cx0) * 128 + lane;
  const float* p01 = fm + ((long long)cy0 * w + cx1) * 128 + lane;
  const float* p10 = fm + ((long long)cy1 * w + cx0) * 128 + lane;
  const float* p11 = fm + ((long long)cy1 * w + cx1) * 128 + lane;
  const float a00 = p00[0], b00 = p00[64], a01 = p01[0], b01 = p01[64];
  const float a10 = p10[0], b10 = p10[64], a11 = p11[0], b11 = p11[64];
  const float w00 = (by0 && bx0) ? ((float)x1 - ix) * ((float)y1 - iy) : 0.f;
  const float w01 = (by0 && bx1) ? (ix - (float)x0) * ((float)y1 - iy) : 0.f;
  const float w10 = (by1 && bx0) ? ((float)x1 - ix) * (iy - (float)y0) : 0.f;
  const float w11 = (by1 && bx1) ? (ix - (float)x0) * (iy - (float)y0) : 0.f;
  float2 r = {0.f, 0.f};
  r.x += a00 * w00;
  r.y += b00 * w00;
  r.x += a01 * w01;
  r.y += b01 * w01;
  r.x += a10 * w10;
  r.y += b10 * w10;
  r.x += a11 * w11;
  r.y += b11 * w11;
  (void)wx0;
  (void)wx1;
  (void)wy0;
  (void)wy1;
  return r;
}

// bilinear128's sample (same corner weights and per-channel sums), for this
// lane's 8 channels cl*8 .. cl*8+7 (16 lanes per sample, 16-B loads), dotted
// with the query's same 8 channels: the 16-lane group then sums the partials
template <bool BORDER>
__device__ __forceinline__ float bilinear_dot8(const float* __restrict__ fm, int h, int w, float gx,
                                               float gy, int cl, const f32x4& qa, const f32x4& qb) {
  float ix = ((gx + 1.f) * w - 1.f) / 2.f;
  float iy = ((gy + 1.f) * h - 1.f) / 2.f;
  if (BORDER) {
    ix = fminf(fmaxf(ix, 0.f), (float)(w - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(h - 1));
  }
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  const bool bx0 = (unsigned)x0 < (unsigned)w, bx1 = (unsigned)x1 < (unsigned)w;
  const bool by0 = (unsigned)y0 < (unsigned)h, by1 = (unsigned)y1 < (unsigned)h;
  const int cx0 = min(max(x0, 0), w - 1), cx1 = min(max(x1, 0), w - 1);
  const int cy0 = min(max(y0, 0), h - 1), cy1 = min(max(y1, 0), h - 1);
  const float* p00 = fm + ((long long)cy0 * w + cx0) * 128 + cl * 8;
  const float* p01 = fm + ((long long)cy0 * w + cx1) * 128 + cl * 8;
  const float* p10 = fm + ((long long)cy1 * w + cx0) * 128 + cl * 8;
  const float* p11 = fm + ((long long)cy1 * w + cx1) * 128 + cl * 8;
  const f32x4 a00 = *reinterpret_cast<const f32x4*>(p00), b00 = *reinterpret_cast<const f32x4*>(p00 + 4);
  const f32x4 a01 = *reinterpret_cast<const f32x4*>(p01), b01 = *reinterpret_cast<const f32x4*>(p01 + 4);
  const f32x4 a10 = *reinterpret_cast<const f32x4*>(p10), b10 = *reinterpret_cast<const f32x4*>(p10 + 4);
  const f32x4 a11 = *reinterpret_cast<const f32x4*>(p11), b11 = *reinterpret_cast<const f32x4*>(p11 + 4);
  const float w00 = (by0 && bx0) ? ((float)x1 - ix) * ((float)y1 - iy) : 0.f;
  const float w01 = (by0 && bx1) ? (ix - (float)x0) * ((float)y1 - iy) : 0.f;
  const float w10 = (by1 && bx0) ? ((float)x1 - ix) * (iy - (float)y0) : 0.f;
  const float w11 = (by1 && bx1) ? (ix - (float)x0) * (iy - (float)y0) : 0.f;
  f32x4 ra = a00 * w00, rb = b00 * w00;
  ra += a01 * w01;
  rb += b01 * w01;
  ra += a10 * w10;
  rb += b10 * w10;
  ra += a11 * w11;
  rb += b11 * w11;
  return qa.x * ra.x + qa.y * ra.y + qa.z * ra.z + qa.w * ra.w + qb.x * rb.x + qb.y * rb.y +
         qb.z * rb.z + qb.w * rb.w;
}

constexpr int MAX_LINE = 128;   // line_step <= 128 (2 logits per lane)
constexpr int MAX_WIN = 512;    // window taps <= 512 (8 logits per lane)

constexpr int WB_PATCH = 1024, WB_TAPS = MAX_WIN, WB_AXES = 256;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// bilinear weight of pixel coordinate p for sample position f (0 unless p is
// one of f's two neighbours): the 1-D factors of bilinear128's corner weights
__device__ __forceinline__ float lin_w(float f, int p) {
  const float fl = floorf(f);
  const int p0 = (int)fl;
  return p == p0 ? (float)(p0 + 1) - f : (p == p0 + 1 ? f - fl : 0.f);
}

// Window logits over the patch (shared by the forward and the backward):
// fills ax (fx per ix, fy per iy), pc (q . fm per patch pixel, 0 outside the
// map) and the tap logits wl[r] of taps lane + 64 r (-inf past nw).
constexpr int WP_K = 8;  // patch pixels per 16-lane group per pass (round 3: 4)

struct WinPatch {
  int px0, py0, PW, PH;
};

// the window's tap axes (fx per ix, fy per iy) into ax and its pixel patch
__device__ __forceinline__ WinPatch window_patch_geom(int h2, int w2, float jx, float jy, int win_h,
                                                      int win_w, float window_size, float* ax) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < win_w; i += 64)
    ax[i] = ((jx + linspace_f(-window_size, window_size, win_w, i) + 1.f) * w2 - 1.f) / 2.f;
  for (int i = lane; i < win_h; i += 64)
    ax[win_w + i] = ((jy + linspace_f(-window_size, window_size, win_h, i) + 1.f) * h2 - 1.f) / 2.f;
  wave_lds_sync();
  WinPatch P;
  P.px0 = (int)floorf(ax[0]);
  P.py0 = (int)floorf(ax[win_w]);
  P.PW = (int)floorf(ax[win_w - 1]) + 2 - P.px0;
  P.PH = (int)floorf(ax[win_w + win_h - 1]) + 2 - P.py0;
  return P;
}

__device__ __forceinline__ WinPatch window_patch_logits(const float* __restrict__ fmb, int h2,
                                                        int w2, const float* __restrict__ qp,
                                                        float jx, float jy, int win_h, int win_w,
                                                        float window_size, float* pc, float* ax,
                                                        float (&wl)[MAX_WIN / 64]) {
  const int lane = threadIdx.x & 63, grp = lane >> 4, cl = lane & 15;
  const WinPatch P = window_patch_geom(h2, w2, jx, jy, win_h, win_w, window_size, ax);
  const int np = P.PW * P.PH;
  const f32x4 qa = *reinterpret_cast<const f32x4*>(qp + cl * 8);
  const f32x4 qb = *reinterpret_cast<const f32x4*>(qp + cl * 8 + 4);
  // WP_K * 4 pixels per pass, branch-free (a pixel outside the map or past
  // the patch reads a clamped address and yields 0), so their loads overlap
  for (int base = 0; base < np; base += 4 * WP_K) {
    float v[WP_K];
#pragma unroll
    for (int k = 0; k < WP_K; ++k) {
      const int pp = base + 4 * k + grp;
      const int py = P.py0 + pp / P.PW, px = P.px0 + pp % P.PW;
      const bool in = pp < np && (unsigned)py < (unsigned)h2 && (unsigned)px < (unsigned)w2;
      const float* src = fmb + ((long long)min(max(py, 0), h2 - 1) * w2 + min(max(px, 0), w2 - 1)) *
                                   128 + cl * 8;
      const f32x4 a = *reinterpret_cast<const f32x4*>(src);
      const f32x4 c = *reinterpret_cast<const f32x4*>(src + 4);
      const float d = qa.x * a.x + qa.y * a.y + qa.z * a.z + qa.w * a.w + qb.x * c.x + qb.y * c.y +
                      qb.z * c.z + qb.w * c.w;
      v[k] = in ? d : 0.f;
    }
#pragma unroll
    for (int k = 0; k < WP_K; ++k) {
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v[k] += pf_shfl_xor(v[k], o, 64);
      const int pp = base + 4 * k + grp;
      if (cl == 0 && pp < np) pc[pp] = v[k];
    }
  }
  wave_lds_sync();
  const int nw = win_h * win_w;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    wl[r] = -INFINITY;
    if (s < nw) {
      const int iy = s / win_w, ix = s - iy * win_w;
      const float fx = ax[ix], fy = ax[win_w + iy];
      const float flx = floorf(fx), fly = floorf(fy);
      const float* r0 = pc + ((int)fly - P.py0) * P.PW + ((int)flx - P.px0);
      const float ax1 = fx - flx, ay1 = fy - fly, ax0 = 1.f - ax1, ay0 = 1.f - ay1;
      wl[r] = ay0 * (ax0 * r0[0] + ax1 * r0[1]) + ay1 * (ax0 * r0[P.PW] + ax1 * r0[P.PW + 1]);
    }
  }
  return P;
}

// One wave per query point: epipolar line search + window expectation.
__global__ PF_NO_PK_FP32 void line_window_kernel(const float* __restrict__ cpx,   // [b][n][2] query pixels
                                   const float* __restrict__ Fm,    // [b][3][3]
                                   const float* __restrict__ f1,    // [b][n][128] L2-normed
                                   const float* __restrict__ fm2,   // [b][h2][w2][128] T*norm
                                   const float* __restrict__ rnd,   // [b][n][2] U(0,1)
                                   int nb, int n, int h2, int w2, int H2, int W2, int line_step,
                                   int win_h, int win_w, float window_size,
                                   float* __restrict__ l_exp_n, float* __restrict__ l_org_n,
                                   uint8_t* __restrict__ valid, float* __restrict__ w_px,
                                   float* __restrict__ w_std, int use_patch,
                                   float* __restrict__ wlog) {
  __shared__ float s_pc[4][WB_PATCH];
  __shared__ float s_ax[4][WB_AXES];
  __shared__ float s_lg[4][MAX_LINE];
  const int lane = threadIdx.x & 63;
  // one image's points on one XCD: a line sweeps its whole map (4 corners x
  // 512 B per sample, ~200 KB per point), so the L2 working set is one map,
  // not all b (the kernel streams ~2 GB of corner reads per launch)
  const long long wid = pf_xcd_block(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n) return;
  const int b = (int)(wid / n);
  const float* F = Fm + b * 9;
  const float* fmb = fm2 + (long long)b * h2 * w2 * 128;
  const float q0 = f1[wid * 128 + lane], q1 = f1[wid * 128 + lane + 64];
  const float x = cpx[wid * 2], y = cpx[wid * 2 + 1];
  // ---- get_endpoints (preprocess_utils.py:696-719), image size H2 x W2
  const float la = fmaf(F[2], 1.f, fmaf(F[1], y, F[0] * x));
  const float lb = fmaf(F[5], 1.f, fmaf(F[4], y, F[3] * x));
  const float lc = fmaf(F[8], 1.f, fmaf(F[7], y, F[6] * x));
  const float Wm = (float)(W2 - 1), Hm = (float)(H2 - 1);
  float px[4], py[4];
  px[0] = 0.f;
  py[0] = -lc / lb;
  px[1] = Wm;
  py[1] = -(la * Wm + lc) / lb;
  px[2] = -(lb * Hm + lc) / la;
  py[2] = Hm;
  px[3] = -lc / la;
  py[3] = 0.f;
  int cnt = 0, first = -1, second = -1;
  for (int k = 0; k < 4; ++k) {
    const bool in = px[k] >= 0.f && px[k] <= Wm && py[k] >= 0.f && py[k] <= Hm;
    if (in) {
      if (first < 0) first = k;
      else if (second < 0) second = k;
      ++cnt;
    }
  }
  bool ok = cnt == 2;
  if (!ok) {
    first = 0;
    second = 1;
  }
  const float c0 = (float)((W2 - 1) / 2.0), c1 = (float)((H2 - 1) / 2.0);
  const float e1x = (px[first] - c0) / c0, e1y = (py[first] - c1) / c1;
  const float e2x = (px[second] - c0) / c0, e2y = (py[second] - c1) / c1;
  const float dx = e2x - e1x, dy = e2y - e1y;
  // ---- line samples: logits (lane s holds logit s and s+64).  16 lanes per
  // sample (8 channels each, 16-B corner loads), 4 samples per wave and LU per
  // group in one pass, so 4 * LU samples' corner loads are in flight together;
  // the logits go through LDS to their lanes.  (Round 3: 64 lanes per sample,
  // 4-B loads, 4 samples per pass.)
  constexpr int LU = 2;
  const int grp = lane >> 4, cl = lane & 15;
  const f32x4 qa = *reinterpret_cast<const f32x4*>(f1 + wid * 128 + cl * 8);
  const f32x4 qb = *reinterpret_cast<const f32x4*>(f1 + wid * 128 + cl * 8 + 4);
  float* slg = s_lg[threadIdx.x >> 6];
  for (int s0 = 0; s0 < line_step; s0 += 4 * LU) {
    float d[LU];
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      const int s = min(s0 + grp + 4 * u, line_step - 1);
      const float t = linspace_f(0.f, 1.f, line_step, s);
      const float gx = __fadd_rn(__fmul_rn(dx, t), e1x), gy = __fadd_rn(__fmul_rn(dy, t), e1y);
      d[u] = bilinear_dot8<true>(fmb, h2, w2, gx, gy, cl, qa, qb);
    }
#pragma unroll
    for (int u = 0; u < LU; ++u) {
      float v = d[u];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += pf_shfl_xor(v, o, 64);
      const int s = s0 + grp + 4 * u;
      if (cl == 0 && s < line_step) slg[s] = v;
    }
  }
  wave_lds_sync();
  float lg[2];
  lg[0] = lane < line_step ? slg[lane] : -INFINITY;
  lg[1] = lane + 64 < line_step ? slg[lane + 64] : -INFINITY;
  float mx = fmaxf(lg[0], lg[1]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, pf_shfl_xor(mx, o, 64));
  // use_nn: sum of the grid points whose prob equals the max
  float ox = 0.f, oy = 0.f;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int s = lane + 64 * r;
    if (s < line_step && lg[r] == mx) {
      const float t = linspace_f(0.f, 1.f, line_step, s);
      ox += __fadd_rn(__fmul_rn(dx, t), e1x);
      oy += __fadd_rn(__fmul_rn(dy, t), e1y);
    }
  }
  ox = pf_wave_sum(ox);
  oy = pf_wave_sum(oy);
  const float jx = ox + 0.707f * window_size * (2.f * rnd[wid * 2] - 1.f);
  const float jy = oy + 0.707f * window_size * (2.f * rnd[wid * 2 + 1] - 1.f);
  ok = ok && jx >= -1.f && jx <= 1.f && jy >= -1.f && jy <= 1.f;
  // ---- window around the jittered line expectation
  const int nw = win_h * win_w;
  float wl[MAX_WIN / 64];
  if (use_patch) {  // logits through the window's pixel patch (see window_patch_logits)
    const int wv = threadIdx.x >> 6;
    window_patch_logits(fmb, h2, w2, f1 + wid * 128, jx, jy, win_h, win_w, window_size, s_pc[wv],
                        s_ax[wv], wl);
  } else {
#pragma unroll
    for (int r = 0; r < MAX_WIN / 64; ++r) wl[r] = -INFINITY;
    for (int s = 0; s < nw; ++s) {
      const int iy = s / win_w, ix = s - iy * win_w;
      const float gx = jx + linspace_f(-window_size, window_size, win_w, ix);
      const float gy = jy + linspace_f(-window_size, window_size, win_h, iy);
      const float2 v = bilinear128<false>(fmb, h2, w2, gx, gy, lane);
      const float d = pf_wave_sum(q0 * v.x + q1 * v.y);
#pragma unroll
      for (int r = 0; r < MAX_WIN / 64; ++r)
        if (s == lane + 64 * r) wl[r] = d;
    }
  }
  if (wlog)  // kept for the backward (window_bwd_patch_kernel): it skips the patch pass
#pragma unroll
    for (int r = 0; r < MAX_WIN / 64; ++r)
      if (lane + 64 * r < nw) wlog[wid * MAX_WIN + lane + 64 * r] = wl[r];
  float wm = -INFINITY;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) wm = fmaxf(wm, wl[r]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wm = fmaxf(wm, pf_shfl_xor(wm, o, 64));
  // softmax moments over the window in fp64 (get_expected_correspondence_
  // within_window, preprocess_utils.py:745-750): the fp32 E[g^2] - E[g]^2 of
  // the reference loses most of its digits when the window softmax is peaked;
  // the tap coordinates g stay the fp32 values coord2_n_grid holds
  double se = 0.0, ex = 0.0, ey = 0.0, vx = 0.0, vy = 0.0;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    if (s < nw) {
      const int iy = s / win_w, ix = s - iy * win_w;
      const double gx = jx + linspace_f(-window_size, window_size, win_w, ix);
      const double gy = jy + linspace_f(-window_size, window_size, win_h, iy);
      const double e = (double)expf(wl[r] - wm);
      se += e;
      ex += e * gx;
      ey += e * gy;
      vx += e * gx * gx;
      vy += e * gy * gy;
    }
  }
  se = wave_sum_d(se);
  ex = wave_sum_d(ex) / se;
  ey = wave_sum_d(ey) / se;
  vx = wave_sum_d(vx) / se - ex * ex;
  vy = wave_sum_d(vy) / se - ey * ey;
  if (lane == 0) {
    l_exp_n[wid * 2] = jx;
    l_exp_n[wid * 2 + 1] = jy;
    l_org_n[wid * 2] = ox;
    l_org_n[wid * 2 + 1] = oy;
    valid[wid] = ok ? 1 : 0;
    w_px[wid * 2] = (float)ex * c0 + c0;
    w_px[wid * 2 + 1] = (float)ey * c1 + c1;
    w_std[wid] = (float)(sqrt(fmax(vx, 1e-10)) + sqrt(fmax(vy, 1e-10)));
  }
}

// |x2^T l| with l = F x1 / ||l[:2]|| (epipolarloss.py:16-22)
__device__ __forceinline__ float epi_cost(const float* F, float x1, float y1, float x2, float y2) {
  const float a = F[0] * x1 + F[1] * y1 + F[2];
  const float b = F[3] * x1 + F[4] * y1 + F[5];
  const float c = F[6] * x1 + F[7] * y1 + F[8];
  const float nrm = fmaxf(sqrtf(a * a + b * b), 1e-8f);
  return fabsf(x2 * (a / nrm) + y2 * (b / nrm) + (c / nrm));
}

// EpipolarLoss_full.forward: one workgroup.  out[0] = loss, out[1..6] =
// loss_g1, loss_w1, loss_g2, loss_w2, percent_g, percent_w.
__global__ __launch_bounds__(1024) PF_NO_PK_FP32 void epipolar_loss_kernel(
    int nb, int n, const float* __restrict__ F1, const float* __restrict__ F2,
    const float* __restrict__ c1, const float* __restrict__ c2, const float* __restrict__ g1,
    const float* __restrict__ g2, const float* __restrict__ w1, const float* __restrict__ w2,
    const float* __restrict__ sg1, const float* __restrict__ sg2, const float* __restrict__ sw1,
    const float* __restrict__ sw2, const uint8_t* __restrict__ v1, const uint8_t* __restrict__ v2,
    float short_edge, float gthr, float wthr, float wg, float ww, float* __restrict__ out) {
  const int tid = threadIdx.x;
  const int total = nb * n;
  // one pass per set: with inv_i = 1 / std_i and m_i the mask, the weights
  // w_i = m_i inv_i / mean(inv) give sum w = S / mean(inv) and sum w cost =
  // C / mean(inv), S = sum m_i inv_i, C = sum m_i inv_i cost_i -- the same
  // sums as set_weight's two passes, factored (fp64 throughout)
  __shared__ double red[16][16];
  double acc[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double a1 = 0.0, a2 = 0.0, sm = 0.0, cm = 0.0;
    for (int i = tid; i < total; i += blockDim.x) {
      const int b = i / n;
      const float* F = (k < 2 ? F1 : F2) + b * 9;
      const float* p = (k < 2 ? c1 : c2) + 2 * i;
      const float* q = (k == 0 ? g1 : k == 1 ? w1 : k == 2 ? g2 : w2) + 2 * i;
      const float sd = (k == 0 ? sg1 : k == 1 ? sw1 : k == 2 ? sg2 : sw2)[i];
      const float cost = epi_cost(F, p[0], p[1], q[0], q[1]);
      // branch-free (the flag loaded whatever the cost; a masked point adds
      // 0.0): one workgroup walks every point, so iterations must overlap
      const bool vf = (k < 2 ? v1 : v2)[i] != 0;
      const bool m = (cost < short_edge * ((k & 1) ? wthr : gthr)) & vf;
      const double inv = 1.0 / fmaxf(sd, 1e-10f);
      a1 += inv;
      a2 += m ? 1.0 : 0.0;
      sm += m ? inv : 0.0;
      cm += m ? inv * cost : 0.0;
    }
    acc[k][0] = a1;
    acc[k][1] = a2;
    acc[k][2] = sm;
    acc[k][3] = cm;
  }
  // block reduce (fixed order)
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double r = acc[k][j];
      for (int o = 32; o > 0; o >>= 1) r += pf_shfl_xor(r, o, 64);
      if ((tid & 63) == 0) red[tid >> 6][k * 4 + j] = r;
    }
  pf_syncthreads();
  double lsum[4], msum[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double a1 = 0.0, cnt = 0.0, sm = 0.0, cm = 0.0;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) {
      a1 += red[wv][k * 4];
      cnt += red[wv][k * 4 + 1];
      sm += red[wv][k * 4 + 2];
      cm += red[wv][k * 4 + 3];
    }
    const double inv_mean = a1 / total;
    const double wmean = sm / inv_mean / total + 1e-8;
    lsum[k] = cm / inv_mean / wmean / total;
    msum[k] = cnt / total;
  }
  if (tid == 0) {
    out[1] = (float)lsum[0];
    out[2] = (float)lsum[1];
    out[3] = (float)lsum[2];
    out[4] = (float)lsum[3];
    out[0] = (float)(wg * (lsum[0] + lsum[2]) + ww * (lsum[1] + lsum[3]));
    out[5] = (float)((msum[0] + msum[2]) / 2);
    out[6] = (float)((msum[1] + msum[3]) / 2);
  }
}

// ---------------------------------------------------------------- backward
// Descriptor training (configs/train_desc.yaml: weight_grid 0, weight_window 1,
// use_std_as_weight): the weights are detached (epipolarloss.py:25-36), the
// line search runs under no_grad (preprocess_utils.py:661), so dL/d local_map
// flows only through the window expectation (721-758): its softmax over the
// window taps, the zero-padded bilinear samples of T*normalize(xf) (scatter to
// the map) and the query descriptor (normalize(grid_sample(xf)) at the grid
// point).  Scatters accumulate in 64-bit fixed point (2^-40): integer adds
// commute, so the result does not depend on the order the atomics land in.
constexpr double FX_SCALE = 1099511627776.0;  // 2^40

__device__ __forceinline__ void fx_add(unsigned long long* p, float v) {
  const long long q = llrint((double)v * FX_SCALE);
  if (q != 0) atomicAdd(p, (unsigned long long)q);
}

// dL/d(window expectation, normalised) per point for one direction (k = 1: w1
// with F1, coords1, image-2 size; k = 3: w2): one workgroup, the forward's
// fixed-order reductions recomputed.  d loss/d cost_i = ww * wt_i / total,
// d cost/d x2 = sign(x2^T l) l[:2] (l normalised), x2 = E * c + c.
__global__ __launch_bounds__(1024) PF_NO_PK_FP32 void epi_loss_bwd_kernel(
    int nb, int n, const float* __restrict__ Fm, const float* __restrict__ cq,
    const float* __restrict__ wpx, const float* __restrict__ wsd, const uint8_t* __restrict__ v,
    float short_edge, float wthr, float ww, float c0, float c1, float* __restrict__ gE) {
  const int tid = threadIdx.x;
  const int total = nb * n;
  __shared__ double red[16][2];
  // sum inv and sum m inv in one pass (the forward's factored set_weight sums)
  double a1 = 0.0, b1 = 0.0;
  for (int i = tid; i < total; i += blockDim.x) {
    const double inv = 1.0 / fmaxf(wsd[i], 1e-10f);
    const float* F = Fm + (i / n) * 9;
    const float cost = epi_cost(F, cq[2 * i], cq[2 * i + 1], wpx[2 * i], wpx[2 * i + 1]);
    a1 += inv;
    const bool vf = v[i] != 0;
    b1 += ((cost < short_edge * wthr) & vf) ? inv : 0.0;  // branch-free (as the forward)
  }
  for (int o = 32; o > 0; o >>= 1) {
    a1 += pf_shfl_xor(a1, o, 64);
    b1 += pf_shfl_xor(b1, o, 64);
  }
  if ((tid & 63) == 0) {
    red[tid >> 6][0] = a1;
    red[tid >> 6][1] = b1;
  }
  pf_syncthreads();
  double sa = 0.0, sb = 0.0;
  for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) {
    sa += red[wv][0];
    sb += red[wv][1];
  }
  const double inv_mean = sa / total;
  const double sw = sb / inv_mean;
  const double wmean = sw / total + 1e-8;
  for (int i = tid; i < total; i += blockDim.x) {
    const float* F = Fm + (i / n) * 9;
    const float x1 = cq[2 * i], y1 = cq[2 * i + 1], x2 = wpx[2 * i], y2 = wpx[2 * i + 1];
    const float a = F[0] * x1 + F[1] * y1 + F[2];
    const float b = F[3] * x1 + F[4] * y1 + F[5];
    const float c = F[6] * x1 + F[7] * y1 + F[8];
    const float nrm = fmaxf(sqrtf(a * a + b * b), 1e-8f);
    const float sv = x2 * (a / nrm) + y2 * (b / nrm) + (c / nrm);
    const bool vf = v[i] != 0;
    const bool m = (fabsf(sv) < short_edge * wthr) & vf;
    float gx = 0.f, gy = 0.f;
    if (m) {
      const double wt = (1.0 / fmaxf(wsd[i], 1e-10f)) / inv_mean / wmean;
      const float coef = (float)(ww * wt / total) * (sv > 0.f ? 1.f : (sv < 0.f ? -1.f : 0.f));
      gx = coef * (a / nrm) * c0;
      gy = coef * (b / nrm) * c1;
    }
    gE[2 * i] = gx;
    gE[2 * i + 1] = gy;
  }
}

// Window-expectation backward, one wave per query point (mirrors the window
// part of line_window_kernel): recompute the logits and softmax, then
//   dp_s = gE . g_s,  dsim_s = p_s (dp_s - sum p dp),
//   dq   = sum_s dsim_s v_s            (query descriptor, written to dq)
//   d fm[corner] += bilinear_w * dsim_s * q   (fixed-point scatter)
__global__ PF_NO_PK_FP32 void window_bwd_kernel(const float* __restrict__ f1, const float* __restrict__ fm2,
                                  const float* __restrict__ center, const float* __restrict__ gE,
                                  int nb, int n, int h2, int w2, int win_h, int win_w,
                                  float window_size, float* __restrict__ dq,
                                  unsigned long long* __restrict__ acc) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n) return;
  const int b = (int)(wid / n);
  const float gx0 = gE[wid * 2], gy0 = gE[wid * 2 + 1];
  if (gx0 == 0.f && gy0 == 0.f) {  // masked point: no gradient
    dq[wid * 128 + lane] = 0.f;
    dq[wid * 128 + lane + 64] = 0.f;
    return;
  }
  const float* fmb = fm2 + (long long)b * h2 * w2 * 128;
  unsigned long long* accb = acc + (long long)b * h2 * w2 * 128;
  const float q0 = f1[wid * 128 + lane], q1 = f1[wid * 128 + lane + 64];
  const float jx = center[wid * 2], jy = center[wid * 2 + 1];
  const int nw = win_h * win_w;
  float wl[MAX_WIN / 64];
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) wl[r] = -INFINITY;
  for (int s = 0; s < nw; ++s) {
    const int iy = s / win_w, ix = s - iy * win_w;
    const float gx = jx + linspace_f(-window_size, window_size, win_w, ix);
    const float gy = jy + linspace_f(-window_size, window_size, win_h, iy);
    const float2 vv = bilinear128<false>(fmb, h2, w2, gx, gy, lane);
    const float d = pf_wave_sum(q0 * vv.x + q1 * vv.y);
#pragma unroll
    for (int r = 0; r < MAX_WIN / 64; ++r)
      if (s == lane + 64 * r) wl[r] = d;
  }
  float wm = -INFINITY;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) wm = fmaxf(wm, wl[r]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wm = fmaxf(wm, pf_shfl_xor(wm, o, 64));
  float se = 0.f;
  float pr[MAX_WIN / 64], dp[MAX_WIN / 64];
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    pr[r] = s < nw ? expf(wl[r] - wm) : 0.f;
    se += pr[r];
  }
  se = pf_wave_sum(se);
  float sdp = 0.f;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    pr[r] /= se;
    dp[r] = 0.f;
    if (s < nw) {
      const int iy = s / win_w, ix = s - iy * win_w;
      const float gx = jx + linspace_f(-window_size, window_size, win_w, ix);
      const float gy = jy + linspace_f(-window_size, window_size, win_h, iy);
      dp[r] = gx0 * gx + gy0 * gy;
      sdp += pr[r] * dp[r];
    }
  }
  sdp = pf_wave_sum(sdp);
  float ds[MAX_WIN / 64];
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) ds[r] = pr[r] * (dp[r] - sdp);
  float dq0 = 0.f, dq1 = 0.f;
  for (int s = 0; s < nw; ++s) {
    float dsv = 0.f;
#pragma unroll
    for (int r = 0; r < MAX_WIN / 64; ++r)
      if ((s >> 6) == r) dsv = pf_shfl(ds[r], s & 63, 64);
    const int iy = s / win_w, ix = s - iy * win_w;
    const float gx = jx + linspace_f(-window_size, window_size, win_w, ix);
    const float gy = jy + linspace_f(-window_size, window_size, win_h, iy);
    const float2 vv = bilinear128<false>(fmb, h2, w2, gx, gy, lane);
    dq0 += dsv * vv.x;
    dq1 += dsv * vv.y;
    // scatter dsv * q over the 4 zero-padded corners (same weights as bilinear128)
    const float fx = ((gx + 1.f) * w2 - 1.f) / 2.f, fy = ((gy + 1.f) * h2 - 1.f) / 2.f;
    const float flx = floorf(fx), fly = floorf(fy);
    const int x0 = (int)flx, y0 = (int)fly, x1 = x0 + 1, y1 = y0 + 1;
    const float t0 = dsv * q0, t1 = dsv * q1;
    const bool bx0 = (unsigned)x0 < (unsigned)w2, bx1 = (unsigned)x1 < (unsigned)w2;
    const bool by0 = (unsigned)y0 < (unsigned)h2, by1 = (unsigned)y1 < (unsigned)h2;
    if (by0 && bx0) {
      const float wt = ((float)x1 - fx) * ((float)y1 - fy);
      unsigned long long* p = accb + ((long long)y0 * w2 + x0) * 128;
      fx_add(p + lane, wt * t0);
      fx_add(p + lane + 64, wt * t1);
    }
    if (by0 && bx1) {
      const float wt = (fx - (float)x0) * ((float)y1 - fy);
      unsigned long long* p = accb + ((long long)y0 * w2 + x1) * 128;
      fx_add(p + lane, wt * t0);
      fx_add(p + lane + 64, wt * t1);
    }
    if (by1 && bx0) {
      const float wt = ((float)x1 - fx) * (fy - (float)y0);
      unsigned long long* p = accb + ((long long)y1 * w2 + x0) * 128;
      fx_add(p + lane, wt * t0);
      fx_add(p + lane + 64, wt * t1);
    }
    if (by1 && bx1) {
      const float wt = (fx - (float)x0) * (fy - (float)y0);
      unsigned long long* p = accb + ((long long)y1 * w2 + x1) * 128;
      fx_add(p + lane, wt * t0);
      fx_add(p + lane + 64, wt * t1);
    }
  }
  dq[wid * 128 + lane] = dq0;
  dq[wid * 128 + lane + 64] = dq1;
}

// The same backward over the window's pixel patch instead of its taps.  Every
// tap's 4 bilinear corners land in a patch of at most (win_w+4) x (win_h+4)
// pixels, and both the logits and the map gradient factor through it:
//   logit_s = q . v_s = sum_corners w_c (q . fm[c])     (qd: one dot per pixel)
//   d fm[p] = (sum_s w(s, p) dsim_s) q = c_p q           (c: separable adjoint)
//   dq      = sum_p c_p fm[p]
// so the map is read twice per patch pixel (not 2 x 4 per tap) and each patch
// pixel takes one 128-wide fixed-point scatter (not up to 4 per tap).  One
// wave per query point, wave-private LDS; the 16-lane groups of a wave own 4
// patch pixels at a time (8 channels per lane).
__global__ __launch_bounds__(256) void window_bwd_patch_kernel(
    const float* __restrict__ f1, const float* __restrict__ fm2, const float* __restrict__ center,
    const float* __restrict__ gE, int nb, int n, int h2, int w2, int win_h, int win_w,
    float window_size, float* __restrict__ dq, int rec_stride, float* __restrict__ crec,
    int4* __restrict__ prec, const float* __restrict__ wlog) {
  __shared__ float s_pc[4][WB_PATCH];  // q . fm per patch pixel, then c
  __shared__ float s_t[4][WB_PATCH];   // separable adjoint, first stage [iy][px]
  __shared__ float s_ds[4][WB_TAPS];   // dsim per tap
  __shared__ float s_ax[4][WB_AXES];   // fx per ix, then fy per iy
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, cl = lane & 15;
  const long long wid = pf_xcd_block(blockIdx.x, gridDim.x) * 4LL + wv;  // see line_window_kernel
  if (wid >= (long long)nb * n) return;
  const float gx0 = gE[wid * 2], gy0 = gE[wid * 2 + 1];
  if (gx0 == 0.f && gy0 == 0.f) {  // masked point: no gradient
    dq[wid * 128 + lane] = 0.f;
    dq[wid * 128 + lane + 64] = 0.f;
    if (lane == 0) prec[wid] = make_int4(0, 0, 0, 0);
    return;
  }
  const int b = (int)(wid / n);
  const float* fmb = fm2 + (long long)b * h2 * w2 * 128;
  float* pc = s_pc[wv];
  float* tt = s_t[wv];
  float* dsv = s_ds[wv];
  float* ax = s_ax[wv];
  const float jx = center[wid * 2], jy = center[wid * 2 + 1];
  const float* qp = f1 + wid * 128;
  float wl[MAX_WIN / 64];
  const int nw = win_h * win_w;
  WinPatch P;
  if (wlog) {  // the forward's logits (line_window_kernel): no pass over the patch
    P = window_patch_geom(h2, w2, jx, jy, win_h, win_w, window_size, ax);
#pragma unroll
    for (int r = 0; r < MAX_WIN / 64; ++r)
      wl[r] = lane + 64 * r < nw ? wlog[wid * MAX_WIN + lane + 64 * r] : -INFINITY;
  } else {
    P = window_patch_logits(fmb, h2, w2, qp, jx, jy, win_h, win_w, window_size, pc, ax, wl);
  }
  const int px0 = P.px0, py0 = P.py0, PW = P.PW, np = P.PW * P.PH;
  float wm = -INFINITY;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) wm = fmaxf(wm, wl[r]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wm = fmaxf(wm, pf_shfl_xor(wm, o, 64));
  float pr[MAX_WIN / 64], dp[MAX_WIN / 64];
  float se = 0.f;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    pr[r] = s < nw ? expf(wl[r] - wm) : 0.f;
    se += pr[r];
  }
  se = pf_wave_sum(se);
  float sdp = 0.f;
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    pr[r] /= se;
    dp[r] = 0.f;
    if (s < nw) {
      const int iy = s / win_w, ix = s - iy * win_w;
      const float gx = jx + linspace_f(-window_size, window_size, win_w, ix);
      const float gy = jy + linspace_f(-window_size, window_size, win_h, iy);
      dp[r] = gx0 * gx + gy0 * gy;
      sdp += pr[r] * dp[r];
    }
  }
  sdp = pf_wave_sum(sdp);
#pragma unroll
  for (int r = 0; r < MAX_WIN / 64; ++r) {
    const int s = lane + 64 * r;
    if (s < nw) dsv[s] = pr[r] * (dp[r] - sdp);
  }
  wave_lds_sync();
  // c = Wy^T dsim Wx, separably: t[iy][px] = sum_ix wx(ix, px) dsim[iy][ix]
  for (int e = lane; e < win_h * PW; e += 64) {
    const int iy = e / PW, px = px0 + e % PW;
    float v = 0.f;
    for (int ix = 0; ix < win_w; ++ix) {
      const float wx = lin_w(ax[ix], px);
      if (wx != 0.f) v += wx * dsv[iy * win_w + ix];
    }
    tt[e] = v;
  }
  wave_lds_sync();
  for (int e = lane; e < np; e += 64) {
    const int py = py0 + e / PW, pxl = e % PW;
    float v = 0.f;
    for (int iy = 0; iy < win_h; ++iy) {
      const float wy = lin_w(ax[win_w + iy], py);
      if (wy != 0.f) v += wy * tt[iy * PW + pxl];
    }
    pc[e] = v;
  }
  wave_lds_sync();
  // the patch's c values and geometry for window_gather_kernel, which forms
  // d fm[p] = sum_points c_p q per pixel tile (a gather: no atomics)
  for (int e = lane; e < np && e < rec_stride; e += 64) crec[wid * rec_stride + e] = pc[e];
  if (lane == 0) prec[wid] = make_int4(px0, py0, PW, P.PH);
  // pass 2: dq = sum_p c_p fm[p]
  f32x4 da = {0.f, 0.f, 0.f, 0.f}, db = {0.f, 0.f, 0.f, 0.f};
  for (int base = 0; base < np; base += 16) {
    // 16 pixels per pass, branch-free (clamped address, skipped pixels add
    // nothing: the sums keep their order and values), so their loads overlap
    f32x4 va[4], vb[4];
    float c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pp = base + 4 * k + grp;
      const int py = py0 + pp / PW, px = px0 + pp % PW;
      const bool in = pp < np && (unsigned)py < (unsigned)h2 && (unsigned)px < (unsigned)w2;
      c[k] = in ? pc[min(pp, np - 1)] : 0.f;
      const float* src = fmb + ((long long)min(max(py, 0), h2 - 1) * w2 + min(max(px, 0), w2 - 1)) *
                                   128 + cl * 8;
      va[k] = *reinterpret_cast<const f32x4*>(src);
      vb[k] = *reinterpret_cast<const f32x4*>(src + 4);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      da += c[k] * va[k];  // c = 0: adds +-0 (the map is finite)
      db += c[k] * vb[k];
    }
  }
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    da.x += pf_shfl_xor(da.x, o, 64);
    da.y += pf_shfl_xor(da.y, o, 64);
    da.z += pf_shfl_xor(da.z, o, 64);
    da.w += pf_shfl_xor(da.w, o, 64);
    db.x += pf_shfl_xor(db.x, o, 64);
    db.y += pf_shfl_xor(db.y, o, 64);
    db.z += pf_shfl_xor(db.z, o, 64);
    db.w += pf_shfl_xor(db.w, o, 64);
  }
  if (grp == 0) {
    *reinterpret_cast<f32x4*>(dq + wid * 128 + cl * 8) = da;
    *reinterpret_cast<f32x4*>(dq + wid * 128 + cl * 8 + 4) = db;
  }
}

// d fm[p] = sum_i c_i(p) q_i for every pixel p of one 8 x 8 tile of image b,
// over the query points i whose window patch (window_bwd_patch_kernel's
// record) overlaps the tile, in increasing i: deterministic, no atomics.  The
// list is built by a block-wide ordered compaction; c and q of 16 points at a
// time are staged in LDS; thread = (tile row, channel quad), 8 pixels x 4
// channels of accumulators.
constexpr int WG_T = 8, WG_CH = 16, WG_MAXN = 4096;
__global__ __launch_bounds__(256) void window_gather_kernel(
    const float* __restrict__ q, const float* __restrict__ crec, const int4* __restrict__ prec,
    int rec_stride, int n, int h2, int w2, float* __restrict__ dfm) {
  __shared__ int s_list[WG_MAXN];
  __shared__ int s_cnt[256];
  __shared__ __attribute__((aligned(16))) float s_q[WG_CH][128];
  __shared__ float s_c[WG_CH][WG_T * WG_T];
  const int t = threadIdx.x, b = blockIdx.y;
  const int ntx = (w2 + WG_T - 1) / WG_T;
  const int tx0 = (blockIdx.x % ntx) * WG_T, ty0 = (blockIdx.x / ntx) * WG_T;
  const int4* pb = prec + (long long)b * n;
  // ordered list of the overlapping points
  int total = 0;
  for (int base = 0; base < n; base += 256) {
    const int i = base + t;
    int f = 0;
    if (i < n) {
      const int4 r = pb[i];
      f = r.z > 0 && r.x < tx0 + WG_T && r.x + r.z > tx0 && r.y < ty0 + WG_T && r.y + r.w > ty0;
    }
    s_cnt[t] = f;
    pf_syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      const int v = t >= d ? s_cnt[t - d] : 0;
      pf_syncthreads();
      s_cnt[t] += v;
      pf_syncthreads();
    }
    if (f) s_list[total + s_cnt[t] - 1] = i;
    total += s_cnt[255];
    pf_syncthreads();
  }
  const int row = t >> 5, cq = t & 31;
  f32x4 acc[WG_T];
#pragma unroll
  for (int j = 0; j < WG_T; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* qb = q + (long long)b * n * 128;
  const float* cb = crec + (long long)b * n * rec_stride;
  for (int c0 = 0; c0 < total; c0 += WG_CH) {
    const int m = min(WG_CH, total - c0);
    for (int e = t; e < m * 32; e += 256) {  // q rows, float4 each
      const int k = e >> 5, qq = e & 31;
      *reinterpret_cast<f32x4*>(&s_q[k][qq * 4]) =
          *reinterpret_cast<const f32x4*>(qb + (long long)s_list[c0 + k] * 128 + qq * 4);
    }
    for (int e = t; e < m * WG_T * WG_T; e += 256) {  // c of the tile pixels
      const int k = e / (WG_T * WG_T), pp = e - k * (WG_T * WG_T);
      const int i = s_list[c0 + k];
      const int4 r = pb[i];
      const int px = tx0 + (pp % WG_T) - r.x, py = ty0 + (pp / WG_T) - r.y;
      s_c[k][pp] = ((unsigned)px < (unsigned)r.z && (unsigned)py < (unsigned)r.w)
                       ? cb[(long long)i * rec_stride + py * r.z + px]
                       : 0.f;
    }
    pf_syncthreads();
    for (int k = 0; k < m; ++k) {
      const f32x4 qv = *reinterpret_cast<const f32x4*>(&s_q[k][cq * 4]);
#pragma unroll
      for (int j = 0; j < WG_T; ++j) acc[j] += s_c[k][row * WG_T + j] * qv;
    }
    pf_syncthreads();
  }
  const int py = ty0 + row;
  if (py >= h2) return;
#pragma unroll
  for (int j = 0; j < WG_T; ++j) {
    const int px = tx0 + j;
    if (px < w2)
      *reinterpret_cast<f32x4*>(dfm + (((long long)b * h2 + py) * w2 + px) * 128 + cq * 4) = acc[j];
  }
}

// the patch kernel's LDS bounds (patch <= (win + 4)^2, see above)
// POSFEAT_WINPATCH=0: the per-tap kernels (A/B runs)
bool window_patch_on() {
  const char* e = pf_ab_getenv("POSFEAT_WINPATCH");
  return !(e && e[0] == '0');
}

bool window_patch_fits(int win_h, int win_w) {
  return (win_w + 4) * (win_h + 4) <= WB_PATCH && win_w + win_h <= WB_AXES &&
         win_h * win_w <= WB_TAPS;
}

// Query-descriptor backward: f = normalize(s), s = grid_sample(xf, c) (zeros,
// align_corners=False): ds = (dq - f (f.dq)) / max(|s|, 1e-12) scattered over
// the 4 corners of c into acc (raw-map gradient, fixed point).  One wave/point.
// Query-descriptor backward, per point: g = d(sample)/d(loss) from dq through
// the L2 normalisation (f = s / |s|), written over dq ([b][n][128]); the
// bilinear spread of g into the map's 4 corner pixels is gathered per pixel by
// l2norm_bwd_kernel (no zeroed fixed-point accumulator, no atomics).
__global__ PF_NO_PK_FP32 void query_bwd_kernel(const float* __restrict__ xf, int cs, const float* __restrict__ cn,
                                 const float* __restrict__ f, float* __restrict__ dq, int nb, int n,
                                 int h, int w) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n) return;
  const int b = (int)(wid / n);
  const float d0 = dq[wid * 128 + lane], d1 = dq[wid * 128 + lane + 64];
  if (pf_wave_sum(fabsf(d0) + fabsf(d1)) == 0.f) return;  // g = 0 = dq already
  const float* xb = xf + (long long)b * h * w * cs;
  const float gx = cn[wid * 2], gy = cn[wid * 2 + 1];
  const float fx = ((gx + 1.f) * w - 1.f) / 2.f, fy = ((gy + 1.f) * h - 1.f) / 2.f;
  const float flx = floorf(fx), fly = floorf(fy);
  const int x0 = (int)flx, y0 = (int)fly, x1 = x0 + 1, y1 = y0 + 1;
  const bool bx0 = (unsigned)x0 < (unsigned)w, bx1 = (unsigned)x1 < (unsigned)w;
  const bool by0 = (unsigned)y0 < (unsigned)h, by1 = (unsigned)y1 < (unsigned)h;
  const float w00 = ((float)x1 - fx) * ((float)y1 - fy), w01 = (fx - (float)x0) * ((float)y1 - fy);
  const float w10 = ((float)x1 - fx) * (fy - (float)y0), w11 = (fx - (float)x0) * (fy - (float)y0);
  float s0 = 0.f, s1 = 0.f;  // the raw sample (for |s|), same order as sample.hip
  if (by0 && bx0) {
    const float* p = xb + ((long long)y0 * w + x0) * cs;
    s0 += p[lane] * w00;
    s1 += p[lane + 64] * w00;
  }
  if (by0 && bx1) {
    const float* p = xb + ((long long)y0 * w + x1) * cs;
    s0 += p[lane] * w01;
    s1 += p[lane + 64] * w01;
  }
  if (by1 && bx0) {
    const float* p = xb + ((long long)y1 * w + x0) * cs;
    s0 += p[lane] * w10;
    s1 += p[lane + 64] * w10;
  }
  if (by1 && bx1) {
    const float* p = xb + ((long long)y1 * w + x1) * cs;
    s0 += p[lane] * w11;
    s1 += p[lane + 64] * w11;
  }
  const float nrm = sqrtf(pf_wave_sum(s0 * s0 + s1 * s1));
  const float f0 = f[wid * 128 + lane], f1v = f[wid * 128 + lane + 64];
  const float fd = pf_wave_sum(f0 * d0 + f1v * d1);
  const float inv = 1.f / fmaxf(nrm, 1e-12f);
  dq[wid * 128 + lane] = nrm > 1e-12f ? (d0 - f0 * fd) * inv : d0 * inv;
  dq[wid * 128 + lane + 64] = nrm > 1e-12f ? (d1 - f1v * fd) * inv : d1 * inv;
}

// dxf = normalize_bwd(T * acc_fm) + acc_x, one wave per pixel:
// y = x / max(|x|, 1e-12); dx = (dy - y (y.dy)) / |x| (|x| > eps), dy / eps otherwise
// afm: the window-backward map gradient, fixed point (per-tap scatter path) or
// fp32 (dfm, from window_gather_kernel) when dfm != null
// dx[p] = the window term through the T * normalize(xf) map + the query term:
// sum over the grid points whose bilinear sample has p as a corner of
// corner weight x g (query_bwd_kernel), over the cells that can hold such a
// sample (a sample sits in its cell) in a fixed order
__global__ PF_NO_PK_FP32 void l2norm_bwd_kernel(const float* __restrict__ x, int cs,
                                  const unsigned long long* __restrict__ afm,
                                  const float* __restrict__ dfm, const float* __restrict__ cn,
                                  const float* __restrict__ gq, int h, int w, int grid,
                                  int ncx, int ncy, long long npix, float T,
                                  float* __restrict__ dx, int dcs) {
  const int lane = threadIdx.x & 63;
  const long long pix = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (pix >= npix) return;
  const int b = (int)(pix / ((long long)h * w));
  const int rem = (int)(pix - (long long)b * h * w), py = rem / w, px = rem - py * w;
  // the pixel's own loads first, all independent of the cell search below
  const float x0 = x[pix * cs + lane], x1 = x[pix * cs + lane + 64];
  const float gl0 = dfm ? dfm[pix * 128 + lane]
                        : (float)((double)(long long)afm[pix * 128 + lane] / FX_SCALE);
  const float gl1 = dfm ? dfm[pix * 128 + lane + 64]
                        : (float)((double)(long long)afm[pix * 128 + lane + 64] / FX_SCALE);
  float q0 = 0.f, q1 = 0.f;
  {
    // cells (grid image pixels wide) holding image pixels 4 (p - 2) .. 4 (p + 3):
    // every sample whose bilinear corners can include map pixel p -- at most
    // 3 x 3 for grid >= 10 (the caller's grid 16); their sample coordinates
    // are loaded together (clamped cell, masked), then visited in the same
    // row-major order (the same sums as one dependent load per cell)
    const int cx0 = max(4 * (px - 2), 0) / grid, cx1 = min((4 * (px + 3) - 1) / grid, ncx - 1);
    const int cy0 = max(4 * (py - 2), 0) / grid, cy1 = min((4 * (py + 3) - 1) / grid, ncy - 1);
    const int n = ncx * ncy;
    if (cx1 - cx0 < 3 && cy1 - cy0 < 3) {
      float cxv[9], cyv[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int cy = min(cy0 + k / 3, cy1), cxx = min(cx0 + k % 3, cx1);
        const long long i = (long long)b * n + cy * ncx + cxx;
        cxv[k] = cn[i * 2];
        cyv[k] = cn[i * 2 + 1];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int cy = cy0 + k / 3, cxx = cx0 + k % 3;
        if (cy > cy1 || cxx > cx1) continue;
        const long long i = (long long)b * n + cy * ncx + cxx;
        const float fx = ((cxv[k] + 1.f) * w - 1.f) / 2.f;
        const float fy = ((cyv[k] + 1.f) * h - 1.f) / 2.f;
        const float flx = floorf(fx), fly = floorf(fy);
        const int ix0 = (int)flx, iy0 = (int)fly;
        if (px != ix0 && px != ix0 + 1) continue;  // (uniform across the wave)
        if (py != iy0 && py != iy0 + 1) continue;
        const float wx = px == ix0 ? (float)(ix0 + 1) - fx : fx - (float)ix0;
        const float wy = py == iy0 ? (float)(iy0 + 1) - fy : fy - (float)iy0;
        const float wt = wx * wy;
        q0 += wt * gq[i * 128 + lane];
        q1 += wt * gq[i * 128 + lane + 64];
      }
    } else {
      for (int cy = cy0; cy <= cy1; ++cy)
        for (int cxx = cx0; cxx <= cx1; ++cxx) {
          const long long i = (long long)b * n + cy * ncx + cxx;
          const float fx = ((cn[i * 2] + 1.f) * w - 1.f) / 2.f;
          const float fy = ((cn[i * 2 + 1] + 1.f) * h - 1.f) / 2.f;
          const float flx = floorf(fx), fly = floorf(fy);
          const int ix0 = (int)flx, iy0 = (int)fly;
          if (px != ix0 && px != ix0 + 1) continue;
          if (py != iy0 && py != iy0 + 1) continue;
          const float wx = px == ix0 ? (float)(ix0 + 1) - fx : fx - (float)ix0;
          const float wy = py == iy0 ? (float)(iy0 + 1) - fy : fy - (float)iy0;
          const float wt = wx * wy;
          q0 += wt * gq[i * 128 + lane];
          q1 += wt * gq[i * 128 + lane + 64];
        }
    }
  }
  const float nrm = sqrtf(pf_wave_sum(x0 * x0 + x1 * x1));
  const float inv = 1.f / fmaxf(nrm, 1e-12f);
  const float y0 = x0 * inv, y1 = x1 * inv;
  const float g0 = T * gl0, g1 = T * gl1;
  const float yg = pf_wave_sum(y0 * g0 + y1 * g1);
  float r0 = nrm > 1e-12f ? (g0 - y0 * yg) * inv : g0 * inv;
  float r1 = nrm > 1e-12f ? (g1 - y1 * yg) * inv : g1 * inv;
  r0 += q0;
  r1 += q1;
  dx[pix * dcs + lane] = r0;
  dx[pix * dcs + lane + 64] = r1;
}

}  // namespace

// Forward workspace layout (shared with posfeat_line2window_backward, which
// reads the grid points, descriptors and T*normalize maps the forward left).
struct L2WLayout {
  size_t c1n, c1p, c2n, c2p, f1, f2, S, fm1, fm2, colp, wl1, wl2, total;
};

static L2WLayout l2w_layout(int b, int H1, int W1, int H2, int W2, int grid) {
  L2WLayout L{};
  const size_t n1 = (size_t)(H1 / grid) * (W1 / grid), n2 = (size_t)(H2 / grid) * (W2 / grid);
  size_t cur = 0;
  auto take = [&](size_t bytes) {
    const size_t at = cur;
    cur += pf_align(bytes, 256);
    return at;
  };
  L.c1n = take(b * n1 * 8);
  L.c1p = take(b * n1 * 8);
  L.c2n = take(b * n2 * 8);
  L.c2p = take(b * n2 * 8);
  L.f1 = take(b * n1 * 512);
  L.f2 = take(b * n2 * 512);
  L.S = take(b * n1 * n2 * 4);
  L.fm1 = take((size_t)b * (H1 / 4) * (W1 / 4) * 512);
  L.fm2 = take((size_t)b * (H2 / 4) * (W2 / 4) * 512);
  L.colp = take((size_t)b * COL_CH * n2 * sizeof(ColAcc));
  // the window logits of both directions (MAX_WIN per point), read by the backward
  L.wl1 = take((size_t)b * n1 * MAX_WIN * 4);
  L.wl2 = take((size_t)b * n2 * MAX_WIN * 4);
  L.total = cur;
  return L;
}

extern "C" size_t posfeat_line2window_workspace(int b, int H1, int W1, int H2, int W2, int grid) {
  if (b <= 0 || grid <= 0) return 0;
  return l2w_layout(b, H1, W1, H2, W2, grid).total;
}

extern "C" int posfeat_line2window(const float* xf1, int cs1, const float* xf2, int cs2, int b,
                                   int H1, int W1, int H2, int W2, const float* F1,
                                   const float* F2, const int32_t* sel1, const int32_t* sel2,
                                   const float* rand1, const float* rand2, float temperature,
                                   int grid, float window_size, int line_step,
                                   posfeat_l2w_out* out, void* ws, size_t ws_bytes,
                                   void* stream) {
  if (!xf1 || !xf2 || !F1 || !F2 || !sel1 || !sel2 || !rand1 || !rand2 || !out || !ws)
    return POSFEAT_E_INVALID;
  if (b <= 0 || grid <= 0 || H1 % 4 || W1 % 4 || H2 % 4 || W2 % 4 || cs1 < 128 || cs2 < 128 ||
      line_step <= 1 || line_step > MAX_LINE)
    return POSFEAT_E_INVALID;
  const int h1 = H1 / 4, w1 = W1 / 4, h2 = H2 / 4, w2 = W2 / 4;
  const int win_h2 = (int)(window_size * h2), win_w2 = (int)(window_size * w2);
  const int win_h1 = (int)(window_size * h1), win_w1 = (int)(window_size * w1);
  if (win_h2 * win_w2 > MAX_WIN || win_h1 * win_w1 > MAX_WIN || win_h1 < 1 || win_w1 < 1 ||
      win_h2 < 1 || win_w2 < 1)
    return POSFEAT_E_UNSUPPORTED;
  if (ws_bytes < posfeat_line2window_workspace(b, H1, W1, H2, W2, grid)) return POSFEAT_E_WORKSPACE;
  const int n1 = (H1 / grid) * (W1 / grid), n2 = (H2 / grid) * (W2 / grid);
  hipStream_t st = pf_stream(stream);
  const L2WLayout lay = l2w_layout(b, H1, W1, H2, W2, grid);
  char* wb = static_cast<char*>(ws);
  float* c1n = reinterpret_cast<float*>(wb + lay.c1n);
  float* c1p = reinterpret_cast<float*>(wb + lay.c1p);
  float* c2n = reinterpret_cast<float*>(wb + lay.c2n);
  float* c2p = reinterpret_cast<float*>(wb + lay.c2p);
  float* f1 = reinterpret_cast<float*>(wb + lay.f1);
  float* f2 = reinterpret_cast<float*>(wb + lay.f2);
  float* S = reinterpret_cast<float*>(wb + lay.S);
  float* fm1 = reinterpret_cast<float*>(wb + lay.fm1);
  float* fm2 = reinterpret_cast<float*>(wb + lay.fm2);
  ColAcc* colp = reinterpret_cast<ColAcc*>(wb + lay.colp);
  // grid points
  hipLaunchKernelGGL(grid_points_kernel, dim3((b * n1 + 255) / 256), dim3(256), 0, st, sel1, b,
                     H1, W1, grid, c1n, c1p);
  hipLaunchKernelGGL(grid_points_kernel, dim3((b * n2 + 255) / 256), dim3(256), 0, st, sel2, b,
                     H2, W2, grid, c2n, c2p);
  PF_CHECK_LAUNCH();
  if (out->coord1 &&
      hipMemcpyAsync(out->coord1, c1p, (size_t)b * n1 * 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return POSFEAT_E_HIP;
  if (out->coord2 &&
      hipMemcpyAsync(out->coord2, c2p, (size_t)b * n2 * 8, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return POSFEAT_E_HIP;
  // descriptors at the grid points (sample_feat_by_coord, norm=True)
  PF_TRY(pf_sample_desc(xf1, b, 128, h1, w1, cs1, c1n, n1, nullptr, 1, f1, st));
  PF_TRY(pf_sample_desc(xf2, b, 128, h2, w2, cs2, c2n, n2, nullptr, 1, f2, st));
  // T * normalize(xf) maps
  hipLaunchKernelGGL(l2norm_scale_kernel, dim3((unsigned)(((long long)b * h1 * w1 + 3) / 4)),
                     dim3(256), 0, st, xf1, (long long)b * h1 * w1, cs1, temperature, fm1);
  hipLaunchKernelGGL(l2norm_scale_kernel, dim3((unsigned)(((long long)b * h2 * w2 + 3) / 4)),
                     dim3(256), 0, st, xf2, (long long)b * h2 * w2, cs2, temperature, fm2);
  PF_CHECK_LAUNCH();
  // S = f1 f2^T per pair on the MFMA conv engine (1x1 conv, weights = f2)
  if (n2 % 4 == 0) {
    for (int i = 0; i < b; ++i) {
      posfeat_conv_desc d;
      d.n = 1;
      d.h = 1;
      d.w = n1;
      d.cin = 128;
      d.x_cstride = 128;
      d.cout = n2;
      d.kh = d.kw = d.stride = 1;
      d.pad = 0;
      d.y_cstride = n2;
      d.res_cstride = 0;
      d.act = POSFEAT_ACT_NONE;
      PF_TRY(posfeat_conv2d_nhwc(&d, f1 + (size_t)i * n1 * 128, f2 + (size_t)i * n2 * 128, nullptr,
                                 nullptr, S + (size_t)i * n1 * n2, st));
    }
  } else {
    return POSFEAT_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL(corr_row_kernel, dim3((b * n1 + 3) / 4), dim3(256), 0, st, S, b, n1, n2,
                     temperature, c2p, c2n, H2, W2, out->g1, out->g1_std);
  hipLaunchKernelGGL(corr_col_partial_kernel, dim3((n2 + 63) / 64, COL_CH, b), dim3(256), 0, st,
                     S, n1, n2, temperature, c1p, c1n, colp);
  hipLaunchKernelGGL(corr_col_final_kernel, dim3((b * n2 + 255) / 256), dim3(256), 0, st, colp, b,
                     n2, H1, W1, out->g2, out->g2_std);
  PF_CHECK_LAUNCH();
  // line search + window, both directions
  hipLaunchKernelGGL(line_window_kernel, dim3((b * n1 + 3) / 4), dim3(256), 0, st, c1p, F1, f1,
                     fm2, rand1, b, n1, h2, w2, H2, W2, line_step, win_h2, win_w2, window_size,
                     out->l1_exp_n, out->l1_org_n, out->valid1, out->w1, out->w1_std,
                     (int)(window_patch_on() && window_patch_fits(win_h2, win_w2)),
                     reinterpret_cast<float*>(wb + lay.wl1));
  hipLaunchKernelGGL(line_window_kernel, dim3((b * n2 + 3) / 4), dim3(256), 0, st, c2p, F2, f2,
                     fm1, rand2, b, n2, h1, w1, H1, W1, line_step, win_h1, win_w1, window_size,
                     out->l2_exp_n, out->l2_org_n, out->valid2, out->w2, out->w2_std,
                     (int)(window_patch_on() && window_patch_fits(win_h1, win_w1)),
                     reinterpret_cast<float*>(wb + lay.wl2));
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_epipolar_loss(int b, int n, const float* F1, const float* F2,
                                     const float* c1, const float* c2, const float* g1,
                                     const float* g2, const float* w1, const float* w2,
                                     const float* sg1, const float* sg2, const float* sw1,
                                     const float* sw2, const uint8_t* v1, const uint8_t* v2,
                                     float short_edge, float grid_thr, float win_thr,
                                     float weight_grid, float weight_window, float* out,
                                     void* stream) {
  if (b <= 0 || n <= 0 || !out) return POSFEAT_E_INVALID;
  hipLaunchKernelGGL(epipolar_loss_kernel, dim3(1), dim3(1024), 0, pf_stream(stream), b, n, F1,
                     F2, c1, c2, g1, g2, w1, w2, sg1, sg2, sw1, sw2, v1, v2, short_edge, grid_thr,
                     win_thr, weight_grid, weight_window, out);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// per-point window patch record (window_bwd_patch_kernel -> window_gather_kernel):
// sized for the largest patch the patch kernel accepts on an h x w map at the
// configs' window_size 0.1 ... 0.125 -- (0.125 w + 4) x (0.125 h + 4), at most WB_PATCH
static size_t wb_rec_stride(int h, int w) {
  const size_t s = (size_t)((int)(0.125f * w) + 4) * (size_t)((int)(0.125f * h) + 4);
  return std::min(s, (size_t)WB_PATCH);
}

extern "C" size_t posfeat_line2window_backward_workspace(int b, int H1, int W1, int H2, int W2,
                                                        int grid) {
  if (b <= 0 || grid <= 0) return 0;
  const size_t n1 = (size_t)(H1 / grid) * (W1 / grid), n2 = (size_t)(H2 / grid) * (W2 / grid);
  const size_t p1 = (size_t)b * (H1 / 4) * (W1 / 4) * 128, p2 = (size_t)b * (H2 / 4) * (W2 / 4) * 128;
  const size_t r1 = wb_rec_stride(H2 / 4, W2 / 4), r2 = wb_rec_stride(H1 / 4, W1 / 4);
  return pf_align(b * n1 * 8, 256) + pf_align(b * n2 * 8, 256) + pf_align(b * n1 * 512, 256) +
         pf_align(b * n2 * 512, 256) + pf_align(p1 * 8, 256) + pf_align(p2 * 8, 256) +
         pf_align(b * n1 * r1 * 4, 256) + pf_align(b * n2 * r2 * 4, 256) +
         pf_align(b * n1 * 16, 256) + pf_align(b * n2 * 16, 256);
}

extern "C" int posfeat_line2window_backward(
    const float* xf1, int cs1, const float* xf2, int cs2, int b, int H1, int W1, int H2, int W2,
    const float* F1, const float* F2, const posfeat_l2w_out* fwd, const void* fwd_ws,
    float temperature, int grid, float window_size, float short_edge, float grid_thr,
    float win_thr, float weight_grid, float weight_window, float* dxf1, int dcs1, float* dxf2,
    int dcs2, void* ws, size_t ws_bytes, void* stream) {
  (void)grid_thr;
  if (!xf1 || !xf2 || !F1 || !F2 || !fwd || !fwd_ws || !dxf1 || !dxf2 || !ws)
    return POSFEAT_E_INVALID;
  if (!fwd->coord1 || !fwd->coord2 || !fwd->l1_exp_n || !fwd->l2_exp_n || !fwd->w1 || !fwd->w2 ||
      !fwd->w1_std || !fwd->w2_std || !fwd->valid1 || !fwd->valid2)
    return POSFEAT_E_INVALID;
  if (weight_grid != 0.f) return POSFEAT_E_UNSUPPORTED;  // train_desc.yaml: weight_grid 0
  if (b <= 0 || grid <= 0 || H1 % 4 || W1 % 4 || H2 % 4 || W2 % 4 || cs1 < 128 || cs2 < 128 ||
      dcs1 < 128 || dcs2 < 128)
    return POSFEAT_E_INVALID;
  if (ws_bytes < posfeat_line2window_backward_workspace(b, H1, W1, H2, W2, grid))
    return POSFEAT_E_WORKSPACE;
  const int h1 = H1 / 4, w1 = W1 / 4, h2 = H2 / 4, w2 = W2 / 4;
  const int win_h2 = (int)(window_size * h2), win_w2 = (int)(window_size * w2);
  const int win_h1 = (int)(window_size * h1), win_w1 = (int)(window_size * w1);
  if (win_h2 * win_w2 > MAX_WIN || win_h1 * win_w1 > MAX_WIN) return POSFEAT_E_UNSUPPORTED;
  const int n1 = (H1 / grid) * (W1 / grid), n2 = (H2 / grid) * (W2 / grid);
  hipStream_t st = pf_stream(stream);
  const L2WLayout lay = l2w_layout(b, H1, W1, H2, W2, grid);
  const char* fb = static_cast<const char*>(fwd_ws);
  const float* c1n = reinterpret_cast<const float*>(fb + lay.c1n);
  const float* c2n = reinterpret_cast<const float*>(fb + lay.c2n);
  const float* f1 = reinterpret_cast<const float*>(fb + lay.f1);
  const float* f2 = reinterpret_cast<const float*>(fb + lay.f2);
  const float* fm1 = reinterpret_cast<const float*>(fb + lay.fm1);
  const float* fm2 = reinterpret_cast<const float*>(fb + lay.fm2);
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += pf_align(bytes, 256);
    return r;
  };
  float* gE1 = reinterpret_cast<float*>(take((size_t)b * n1 * 8));
  float* gE2 = reinterpret_cast<float*>(take((size_t)b * n2 * 8));
  float* dq1 = reinterpret_cast<float*>(take((size_t)b * n1 * 512));
  float* dq2 = reinterpret_cast<float*>(take((size_t)b * n2 * 512));
  const size_t p1 = (size_t)b * h1 * w1 * 128, p2 = (size_t)b * h2 * w2 * 128;
  char* accs = p;
  unsigned long long* afm1 = reinterpret_cast<unsigned long long*>(take(p1 * 8));
  unsigned long long* afm2 = reinterpret_cast<unsigned long long*>(take(p2 * 8));
  const size_t rs1 = wb_rec_stride(h2, w2), rs2 = wb_rec_stride(h1, w1);
  float* crec1 = reinterpret_cast<float*>(take((size_t)b * n1 * rs1 * 4));
  float* crec2 = reinterpret_cast<float*>(take((size_t)b * n2 * rs2 * 4));
  int4* prec1 = reinterpret_cast<int4*>(take((size_t)b * n1 * 16));
  int4* prec2 = reinterpret_cast<int4*>(take((size_t)b * n2 * 16));
  // patch path (default): the window gradient w.r.t. fm is gathered per pixel
  // tile into fp32 buffers that reuse the afm storage (no fixed-point scatter)
  const bool gather1 = window_patch_on() && window_patch_fits(win_h2, win_w2) &&
                       (size_t)(win_w2 + 4) * (win_h2 + 4) <= rs1 && n1 <= WG_MAXN;
  const bool gather2 = window_patch_on() && window_patch_fits(win_h1, win_w1) &&
                       (size_t)(win_w1 + 4) * (win_h1 + 4) <= rs2 && n2 <= WG_MAXN;
  // zero the fixed-point accumulators; a gathered window gradient (window_gather_kernel
  // writes every pixel of its map) needs no zeroed afm
  (void)accs;
  if ((!gather2 && hipMemsetAsync(afm1, 0, p1 * 8, st) != hipSuccess) ||
      (!gather1 && hipMemsetAsync(afm2, 0, p2 * 8, st) != hipSuccess))
    return POSFEAT_E_HIP;
  // d loss / d window expectations (w1 lives in image 2, w2 in image 1)
  hipLaunchKernelGGL(epi_loss_bwd_kernel, dim3(1), dim3(1024), 0, st, b, n1, F1, fwd->coord1,
                     fwd->w1, fwd->w1_std, fwd->valid1, short_edge, win_thr, weight_window,
                     (float)((W2 - 1) / 2.0), (float)((H2 - 1) / 2.0), gE1);
  hipLaunchKernelGGL(epi_loss_bwd_kernel, dim3(1), dim3(1024), 0, st, b, n2, F2, fwd->coord2,
                     fwd->w2, fwd->w2_std, fwd->valid2, short_edge, win_thr, weight_window,
                     (float)((W1 - 1) / 2.0), (float)((H1 - 1) / 2.0), gE2);
  PF_CHECK_LAUNCH();
  // window softmax backward: direction 1 scatters into image 2's map, and back
  float* dfm2 = gather1 ? reinterpret_cast<float*>(afm2) : nullptr;
  float* dfm1 = gather2 ? reinterpret_cast<float*>(afm1) : nullptr;
  if (gather1) {
    hipLaunchKernelGGL(window_bwd_patch_kernel, dim3((b * n1 + 3) / 4), dim3(256), 0, st, f1, fm2,
                       fwd->l1_exp_n, gE1, b, n1, h2, w2, win_h2, win_w2, window_size, dq1,
                       (int)rs1, crec1, prec1, reinterpret_cast<const float*>(fb + lay.wl1));
    hipLaunchKernelGGL(window_gather_kernel,
                       dim3(((w2 + WG_T - 1) / WG_T) * ((h2 + WG_T - 1) / WG_T), b), dim3(256), 0,
                       st, f1, crec1, prec1, (int)rs1, n1, h2, w2, dfm2);
  } else {
    hipLaunchKernelGGL(window_bwd_kernel, dim3((b * n1 + 3) / 4), dim3(256), 0, st, f1, fm2,
                       fwd->l1_exp_n, gE1, b, n1, h2, w2, win_h2, win_w2, window_size, dq1, afm2);
  }
  if (gather2) {
    hipLaunchKernelGGL(window_bwd_patch_kernel, dim3((b * n2 + 3) / 4), dim3(256), 0, st, f2, fm1,
                       fwd->l2_exp_n, gE2, b, n2, h1, w1, win_h1, win_w1, window_size, dq2,
                       (int)rs2, crec2, prec2, reinterpret_cast<const float*>(fb + lay.wl2));
    hipLaunchKernelGGL(window_gather_kernel,
                       dim3(((w1 + WG_T - 1) / WG_T) * ((h1 + WG_T - 1) / WG_T), b), dim3(256), 0,
                       st, f2, crec2, prec2, (int)rs2, n2, h1, w1, dfm1);
  } else {
    hipLaunchKernelGGL(window_bwd_kernel, dim3((b * n2 + 3) / 4), dim3(256), 0, st, f2, fm1,
                       fwd->l2_exp_n, gE2, b, n2, h1, w1, win_h1, win_w1, window_size, dq2, afm1);
  }
  // query descriptors: the normalisation's backward per point (over dq), the
  // grid_sample backward gathered per pixel below
  hipLaunchKernelGGL(query_bwd_kernel, dim3((b * n1 + 3) / 4), dim3(256), 0, st, xf1, cs1, c1n, f1,
                     dq1, b, n1, h1, w1);
  hipLaunchKernelGGL(query_bwd_kernel, dim3((b * n2 + 3) / 4), dim3(256), 0, st, xf2, cs2, c2n, f2,
                     dq2, b, n2, h2, w2);
  PF_CHECK_LAUNCH();
  const long long np1 = (long long)b * h1 * w1, np2 = (long long)b * h2 * w2;
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((unsigned)((np1 + 3) / 4)), dim3(256), 0, st, xf1, cs1,
                     afm1, dfm1, c1n, dq1, h1, w1, grid, W1 / grid, H1 / grid, np1, temperature,
                     dxf1, dcs1);
  hipLaunchKernelGGL(l2norm_bwd_kernel, dim3((unsigned)((np2 + 3) / 4)), dim3(256), 0, st, xf2, cs2,
                     afm2, dfm2, c2n, dq2, h2, w2, grid, W2 / grid, H2 / grid, np2, temperature,
                     dxf2, dcs2);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
