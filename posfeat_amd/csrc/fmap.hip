// fmap.hip -- memory-bound feature-map kernels of the extraction path (gfx950).
//
//   layout      NCHW <-> NHWC (API boundary; torch tensors are NCHW)
//   maxpool     ResNet stem max_pool2d(3, 2, 1)             (DescNet.py:66 via torchvision)
//   upsample2x  bilinear x2, align_corners=True            (DescNet.py:189)
//   instance norm stats / apply (+PReLU)                   (DeteNet.py:12-22, 108-113)
//   norm_prelu_upsample  IN+PReLU then bilinear to image size, align_corners=False
//                                                          (DeteNet.py:108-109)
//   head tail   conv3 1x1 on PReLU(IN(conv2)) + IN + Softplus (DeteNet.py:112-113)
//   global_feat F.normalize(global_map).mean([2,3])        (PoSFeat_model.py:115-117)
//
// All are HBM/L2-bound; feature maps are NHWC with a pixel stride so a
// producer can write straight into a channel slice of a concat buffer.
#include <algorithm>

#include "common.h"
#include "fmap.h"

namespace {

// ---------------------------------------------------------------- layout
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int n, int c, int hw, int cso,
                                    float* __restrict__ y) {
  const long long total = (long long)n * hw * cso;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % cso);
    const long long p = i / cso;
    const int b = (int)(p / hw);
    const int pix = (int)(p - (long long)b * hw);
    y[i] = ch < c ? x[((long long)b * c + ch) * hw + pix] : 0.f;
  }
}

// c <= 4 into a 4-float pixel (the image into the stem's NHWC4 layout): one
// thread per pixel, one coalesced load per channel plane, one 16-B store
__global__ void nchw_to_nhwc4_kernel(const float* __restrict__ x, int n, int c, int hw,
                                     float* __restrict__ y) {
  const long long total = (long long)n * hw;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(p / hw);
    const int pix = (int)(p - (long long)b * hw);
    const float* xb = x + (long long)b * c * hw + pix;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (c > 0) v.x = xb[0];
    if (c > 1) v.y = xb[hw];
    if (c > 2) v.z = xb[2 * (long long)hw];
    if (c > 3) v.w = xb[3 * (long long)hw];
    *reinterpret_cast<f32x4*>(y + p * 4) = v;
  }
}

// datasets' to_input on the device: uint8 HWC RGB -> ImageNet-normalised
// float NCHW, ((u / 255) - mean[c]) / std[c] with IEEE round-to-nearest fp32
// division and subtraction -- the same three roundings as numpy's
// (im.astype(float32) / float32(255) - MEAN) / STD, so the result is
// bit-identical to the host path (transforms.ToTensor + Normalize,
// datasets/hpatches.py:14-17).  One thread per pixel: 3 bytes in, 3 floats out.
__global__ void normalize_rgb8_kernel(const unsigned char* __restrict__ src, int hw, int src_pitch,
                                      int w, float* __restrict__ dst) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= hw) return;
  const int y = p / w, x = p - y * w;
  const unsigned char* s = src + (long long)b * (hw / w) * src_pitch + (long long)y * src_pitch + x * 3;
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
  float* d = dst + (long long)b * 3 * hw + p;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    d[(long long)c * hw] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)s[c], 255.f), mean[c]), stdv[c]);
}

// 64 pixels x 64 channels tile through LDS.
__global__ void nhwc_to_nchw_kernel(const float* __restrict__ x, int c, int hw, int csi,
                                    float* __restrict__ y) {
  __shared__ float t[64][65];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: ty 0..3
  for (int r = ty; r < 64; r += 4) {
    const int p = p0 + r, ch = c0 + tx;
    t[r][tx] = (p < hw && ch < c) ? x[((long long)b * hw + p) * csi + ch] : 0.f;
  }
  pf_syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int ch = c0 + r, p = p0 + tx;
    if (ch < c && p < hw) y[((long long)b * c + ch) * hw + p] = t[tx][r];
  }
}

// the same for whole 64 x 64 tiles with 16-B global accesses (c % 64 == 0,
// hw % 64 == 0, csi % 4 == 0, 16-B aligned): a thread loads 4 channels of a
// pixel and stores 4 pixels of a channel; the LDS tile is padded by one float
// per row (the column reads stay conflict-free)
__global__ void nhwc_to_nchw64_kernel(const float* __restrict__ x, int c, int hw, int csi,
                                      float* __restrict__ y) {
  __shared__ float t[64][65];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {  // 64 pixels x 16 channel quads
    const int e = it * 256 + tid, r = e >> 4, q = e & 15;
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + ((long long)b * hw + p0 + r) * csi + c0 + 4 * q);
    t[r][4 * q + 0] = v.x;
    t[r][4 * q + 1] = v.y;
    t[r][4 * q + 2] = v.z;
    t[r][4 * q + 3] = v.w;
  }
  pf_syncthreads();
#pragma unroll
  for (int it = 0; it < 4; ++it) {  // 64 channels x 16 pixel quads
    const int e = it * 256 + tid, ch = e >> 4, q = e & 15;
    const f32x4 o = {t[4 * q + 0][ch], t[4 * q + 1][ch], t[4 * q + 2][ch], t[4 * q + 3][ch]};
    *reinterpret_cast<f32x4*>(y + ((long long)b * c + c0 + ch) * hw + p0 + 4 * q) = o;
  }
}

// ---------------------------------------------------------------- maxpool 3x3 s2 p1
__global__ void maxpool3s2_kernel(const float* __restrict__ x, int n, int h, int w, int c4,
                                  int csi, int oh, int ow, int cso, float* __restrict__ y) {
  const long long total = (long long)n * oh * ow * c4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % c4);
    long long p = i / c4;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    // branch-free: the nine taps' loads go out together (a tap in the padding
    // loads a clamped address and counts as -inf, as if skipped)
    f32x4 v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * oy + t / 3 - 1, ix = 2 * ox + t % 3 - 1;
      ok[t] = (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      const int cy = min(max(iy, 0), h - 1), cx = min(max(ix, 0), w - 1);
      v[t] = *reinterpret_cast<const f32x4*>(x + (((long long)b * h + cy) * w + cx) * csi + q * 4);
    }
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      m.x = fmaxf(m.x, v[t].x);
      m.y = fmaxf(m.y, v[t].y);
      m.z = fmaxf(m.z, v[t].z);
      m.w = fmaxf(m.w, v[t].w);
    }
    *reinterpret_cast<f32x4*>(y + (((long long)b * oh + oy) * ow + ox) * cso + q * 4) = m;
  }
}

// ---------------------------------------------------------------- bilinear x2, align_corners=True
__global__ void upsample2x_ac_kernel(const float* __restrict__ x, int n, int h, int w, int c4,
                                     int csi, float* __restrict__ y, int cso) {
  const int oh = 2 * h, ow = 2 * w;
  const float sh = oh > 1 ? (float)(h - 1) / (float)(oh - 1) : 0.f;
  const float sw = ow > 1 ? (float)(w - 1) / (float)(ow - 1) : 0.f;
  const long long total = (long long)n * oh * ow * c4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(i % c4);
    long long p = i / c4;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    const f32x4 o =
        pf_up2ac_at(x + (long long)b * h * w * csi + q * 4, h, w, csi, sh, sw, oy, ox);
    *reinterpret_cast<f32x4*>(y + (((long long)b * oh + oy) * ow + ox) * cso + q * 4) = o;
  }
}

// ---------------------------------------------------------------- instance norm statistics
// Partial shifted sums: block (chunk, b) covers `chunk_px` pixels of image b for
// all C channels (C % 4 == 0).  shift = value at pixel 0 (keeps sum-of-squares
// well conditioned).  part[b][chunk][c] = {sum(x-s), sum((x-s)^2)} as double.
__global__ void in_partial_kernel(const float* __restrict__ x, int hw, int C, int cs,
                                  int chunk_px, double* __restrict__ part) {
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int c4n = C / 4;
  const int tid = threadIdx.x;
  const int rows = blockDim.x / c4n;  // pixel lanes
  const int q = tid % c4n, pl = tid / c4n;
  const float* xb = x + (long long)b * hw * cs;
  f32x4 s1 = {0, 0, 0, 0}, s2 = {0, 0, 0, 0};
  f32x4 sh = {0, 0, 0, 0};
  if (pl < rows) {
    sh = *reinterpret_cast<const f32x4*>(xb + q * 4);
    const int p0 = chunk * chunk_px, p1 = min(hw, p0 + chunk_px);
    for (int p = p0 + pl; p < p1; p += rows) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xb + (long long)p * cs + q * 4) - sh;
      s1 += v;
      s2 += v * v;
    }
  }
  // reduce over pixel lanes in a fixed order through LDS (deterministic)
  extern __shared__ __attribute__((aligned(16))) double red[];  // [blockDim][8]
  red[tid * 8 + 0] = s1.x;
  red[tid * 8 + 1] = s1.y;
  red[tid * 8 + 2] = s1.z;
  red[tid * 8 + 3] = s1.w;
  red[tid * 8 + 4] = s2.x;
  red[tid * 8 + 5] = s2.y;
  red[tid * 8 + 6] = s2.z;
  red[tid * 8 + 7] = s2.w;
  pf_syncthreads();
  if (tid < c4n) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < rows; ++r)
      for (int k = 0; k < 8; ++k) a[k] += red[(r * c4n + tid) * 8 + k];
    double* o = part + ((long long)b * nchunk + chunk) * C * 2;
    for (int k = 0; k < 4; ++k) {
      o[(tid * 4 + k) * 2 + 0] = a[k];
      o[(tid * 4 + k) * 2 + 1] = a[4 + k];
    }
  }
}

// Chunk partials -> mean / rstd: block = (4 channels x 64 chunk lanes, image);
// fixed-order strided sums + LDS tree (deterministic, no serial per-channel
// chain of nchunk dependent loads)
__global__ __launch_bounds__(256) void in_finalize_kernel(
    const float* __restrict__ x, int hw, int C, int cs, int nchunk,
    const double* __restrict__ part, float eps, float* __restrict__ mean,
    float* __restrict__ rstd, int nb) {
  __shared__ double red[2][64][4];
  const int cl = threadIdx.x & 3, kl = threadIdx.x >> 2;
  const int b = blockIdx.y, c = blockIdx.x * 4 + cl;
  double s1 = 0, s2 = 0;
  const double* p = part + (long long)b * nchunk * C * 2;
  if (c < C)
    for (int k = kl; k < nchunk; k += 64) {
      s1 += p[((long long)k * C + c) * 2];
      s2 += p[((long long)k * C + c) * 2 + 1];
    }
  red[0][kl][cl] = s1;
  red[1][kl][cl] = s2;
  pf_syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (kl < o) {
      red[0][kl][cl] += red[0][kl + o][cl];
      red[1][kl][cl] += red[1][kl + o][cl];
    }
    pf_syncthreads();
  }
  if (kl != 0 || c >= C) return;
  s1 = red[0][0][cl];
  s2 = red[1][0][cl];
  const int i = b * C + c;
  const double sh = x ? x[(long long)b * hw * cs + c] : 0.0;  // x null: unshifted partials
  const double m1 = s1 / hw;
  double var = s2 / hw - m1 * m1;
  if (var < 0) var = 0;
  mean[i] = (float)(sh + m1);
  rstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

// single-channel map (norm3 over the 1-channel score): block partial sums
__global__ void in1_partial_kernel(const float* __restrict__ x, int hw, int chunk_px,
                                   double* __restrict__ part) {
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const float* xb = x + (long long)b * hw;
  const float sh = xb[0];
  float s1 = 0.f, s2 = 0.f;
  const int p0 = chunk * chunk_px, p1 = min(hw, p0 + chunk_px);
  for (int p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const float v = xb[p] - sh;
    s1 += v;
    s2 += v * v;
  }
  __shared__ double r1[256], r2[256];
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  pf_syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    pf_syncthreads();
  }
  if (threadIdx.x == 0) {
    part[((long long)b * nchunk + chunk) * 2] = r1[0];
    part[((long long)b * nchunk + chunk) * 2 + 1] = r2[0];
  }
}

// ---------------------------------------------------------------- apply
__global__ void in_apply_kernel(float* __restrict__ x, int n, int hw, int c4n, int cs,
                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                int prelu, const float* __restrict__ slope) {
  const long long total = (long long)n * hw * c4n;
  const int C = c4n * 4;
  const float a = prelu ? *slope : 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const int b = (int)(p / hw);
    float* ptr = x + p * cs + q * 4;
    f32x4 v = *reinterpret_cast<f32x4*>(ptr);
    const f32x4 m = *reinterpret_cast<const f32x4*>(mean + b * C + q * 4);
    const f32x4 r = *reinterpret_cast<const f32x4*>(rstd + b * C + q * 4);
    v = (v - m) * r;
    if (prelu) {
      v.x = v.x > 0.f ? v.x : a * v.x;
      v.y = v.y > 0.f ? v.y : a * v.y;
      v.z = v.z > 0.f ? v.z : a * v.z;
      v.w = v.w > 0.f ? v.w : a * v.w;
    }
    *reinterpret_cast<f32x4*>(ptr) = v;
  }
}

__device__ __forceinline__ f32x4 norm_prelu4(f32x4 v, f32x4 m, f32x4 r, float a) {
  v = (v - m) * r;
  v.x = v.x > 0.f ? v.x : a * v.x;
  v.y = v.y > 0.f ? v.y : a * v.y;
  v.z = v.z > 0.f ? v.z : a * v.z;
  v.w = v.w > 0.f ? v.w : a * v.w;
  return v;
}

// PReLU(IN(x)) at low resolution, then bilinear resize (align_corners=False)
// to (OH, OW), written into a channel slice of the output.
__global__ void norm_prelu_upsample_kernel(const float* __restrict__ x, int n, int h, int w,
                                           int c4n, int csi, const float* __restrict__ mean,
                                           const float* __restrict__ rstd,
                                           const float* __restrict__ slope, int OH, int OW,
                                           float* __restrict__ y, int cso) {
  const float a = *slope;
  const int C = c4n * 4;
  const float sh = (float)h / (float)OH, sw = (float)w / (float)OW;
  const long long total = (long long)n * OH * OW * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const int ox = (int)(p % OW);
    p /= OW;
    const int oy = (int)(p % OH);
    const int b = (int)(p / OH);
    float ry = sh * (oy + 0.5f) - 0.5f;
    float rx = sw * (ox + 0.5f) - 0.5f;
    ry = ry < 0.f ? 0.f : ry;
    rx = rx < 0.f ? 0.f : rx;
    const int y0 = (int)ry, x0 = (int)rx;
    const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
    const float ly = ry - y0, lx = rx - x0, hy = 1.f - ly, hx = 1.f - lx;
    const float* base = x + (long long)b * h * w * csi + q * 4;
    const f32x4 m = *reinterpret_cast<const f32x4*>(mean + b * C + q * 4);
    const f32x4 r = *reinterpret_cast<const f32x4*>(rstd + b * C + q * 4);
    const f32x4 v00 =
        norm_prelu4(*reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x0) * csi), m, r, a);
    const f32x4 v01 =
        norm_prelu4(*reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x1) * csi), m, r, a);
    const f32x4 v10 =
        norm_prelu4(*reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x0) * csi), m, r, a);
    const f32x4 v11 =
        norm_prelu4(*reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x1) * csi), m, r, a);
    const f32x4 o = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
    *reinterpret_cast<f32x4*>(y + (((long long)b * OH + oy) * OW + ox) * cso + q * 4) = o;
  }
}

// y[b][p] = bias + sum_c w[c] * PReLU((x[b][p][c]-mean)*rstd), C == 128.
// One wave handles two pixels per step (32 lanes x float4 each), over a
// contiguous range of pixel pairs (its image's mean / rstd reloaded only when
// the range crosses an image), HT_U steps per pass with all their loads issued
// before the first reduction.  Same per-pixel arithmetic and order.
// IL: the waves interleaved over the pixels (each step's HT_U pairs of all
// waves one contiguous stream) instead of a contiguous range per wave
template <int HT_U, bool NT, bool IL = false>
__global__ void head_tail_conv3_kernel(const float* __restrict__ x, int n, int hw, int cs,
                                       const float* __restrict__ mean,
                                       const float* __restrict__ rstd,
                                       const float* __restrict__ slope,
                                       const float* __restrict__ w3,
                                       const float* __restrict__ b3, float* __restrict__ y) {
  const float a = *slope;
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w3 + l32 * 4);
  const float bias = *b3;
  const long long total = (long long)n * hw;
  const long long pairs = (total + 1) / 2;
  const long long per = (pairs + waves - 1) / waves;
  const long long q0 = IL ? wid * HT_U : wid * per, q1 = IL ? pairs : min(pairs, q0 + per);
  const long long qstep = IL ? waves * HT_U : HT_U;
  // this lane's image and its pixel range [lo, hi): a 64-bit division only
  // where the lane's pixels cross into the next image (one per pixel was the
  // loop's largest VALU cost)
  long long lo = 0, hi = -1;
  f32x4 m = {0.f, 0.f, 0.f, 0.f}, r = {0.f, 0.f, 0.f, 0.f};
  for (long long q = q0; q < q1; q += qstep) {
    f32x4 xv[HT_U];
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
      const long long p = min(2 * min(q + u, q1 - 1) + half, total - 1);  // clamped: in bounds
      const f32x4* src = reinterpret_cast<const f32x4*>(x + p * cs + l32 * 4);
      xv[u] = NT ? __builtin_nontemporal_load(src) : *src;
    }
    float s[HT_U];
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
      const long long p = min(2 * min(q + u, q1 - 1) + half, total - 1);
      if (p < lo || p >= hi) {  // wave-uniform except where a pair straddles two images
        const int b = (int)(p / hw);
        m = *reinterpret_cast<const f32x4*>(mean + b * 128 + l32 * 4);
        r = *reinterpret_cast<const f32x4*>(rstd + b * 128 + l32 * 4);
        lo = (long long)b * hw;
        hi = lo + hw;
      }
      const f32x4 v = norm_prelu4(xv[u], m, r, a);
      s[u] = v.x * wv.x + v.y * wv.y + v.z * wv.z + v.w * wv.w;
    }
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s[u] += pf_shfl_xor(s[u], o, 64);
      const long long p = 2 * (q + u) + half;
      if (l32 == 0 && q + u < q1 && p < total) y[p] = s[u] + bias;
    }
  }
}

// head_tail_conv3_kernel<HT_U, false, true> with 32-bit pixel and element
// indices (n hw cs < 2^31: the 64-bit index math held a third of its
// registers) -- the same loads, arithmetic and order
template <int HT_U>
__global__ __launch_bounds__(256) void head_tail_il32_kernel(
    const float* __restrict__ x, int n, int hw, int cs, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ slope,
    const float* __restrict__ w3, const float* __restrict__ b3, float* __restrict__ y) {
  const float a = *slope;
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5, l32 = lane & 31;
  const int waves = gridDim.x * (blockDim.x >> 6);
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w3 + l32 * 4);
  const float bias = *b3;
  const int total = n * hw, pairs = (total + 1) / 2;
  int lo = 0, hi = -1;
  f32x4 m = {0.f, 0.f, 0.f, 0.f}, r = {0.f, 0.f, 0.f, 0.f};
  for (int q = wid * HT_U; q < pairs; q += waves * HT_U) {
    f32x4 xv[HT_U];
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
      const int p = min(2 * min(q + u, pairs - 1) + half, total - 1);
      xv[u] = *reinterpret_cast<const f32x4*>(x + (unsigned)(p * cs + l32 * 4));
    }
    float s[HT_U];
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
      const int p = min(2 * min(q + u, pairs - 1) + half, total - 1);
      if (p < lo || p >= hi) {
        const int b = p / hw;
        m = *reinterpret_cast<const f32x4*>(mean + b * 128 + l32 * 4);
        r = *reinterpret_cast<const f32x4*>(rstd + b * 128 + l32 * 4);
        lo = b * hw;
        hi = lo + hw;
      }
      const f32x4 v = norm_prelu4(xv[u], m, r, a);
      s[u] = v.x * wv.x + v.y * wv.y + v.z * wv.z + v.w * wv.w;
    }
#pragma unroll
    for (int u = 0; u < HT_U; ++u) {
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s[u] += pf_shfl_xor(s[u], o, 64);
      const int p = 2 * (q + u) + half;
      if (l32 == 0 && q + u < pairs && p < total) y[p] = s[u] + bias;
    }
  }
}

__global__ PF_NO_PK_FP32 void softplus_norm_kernel(const float* __restrict__ x, int n, int hw,
                                     const float* __restrict__ mean,
                                     const float* __restrict__ rstd, float* __restrict__ y) {
  const long long total = (long long)n * hw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / hw);
    y[i] = pf_softplus((x[i] - mean[b]) * rstd[b]);
  }
}

// the same, four pixels (16 B) per thread (hw % 4 == 0: one image per quad)
__global__ PF_NO_PK_FP32 void softplus_norm4_kernel(const float* __restrict__ x, int n, int hw,
                                      const float* __restrict__ mean,
                                      const float* __restrict__ rstd, float* __restrict__ y) {
  const long long total4 = (long long)n * hw / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(4 * i / hw);
    const float m = mean[b], r = rstd[b];
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + 4 * i);
    f32x4 o;
    o.x = pf_softplus((v.x - m) * r);
    o.y = pf_softplus((v.y - m) * r);
    o.z = pf_softplus((v.z - m) * r);
    o.w = pf_softplus((v.w - m) * r);
    *reinterpret_cast<f32x4*>(y + 4 * i) = o;
  }
}

// global_feat[b][c] = mean_p normalize(gmap[b][p][:])[c], C == 128, one block per image
__global__ void global_feat_kernel(const float* __restrict__ g, int hw, int cs,
                                   float* __restrict__ out) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  float a0 = 0.f, a1 = 0.f;
  // four of this wave's pixels per pass, loads issued together (the wave
  // sums serialised one pixel's load latency after another); the sums add in
  // the same pixel order
  constexpr int GU = 4;
  for (int p = wv; p < hw; p += GU * nw) {
    float x0[GU], x1[GU], inv[GU];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const float* v = g + ((long long)b * hw + min(p + u * nw, hw - 1)) * cs;
      x0[u] = v[lane];
      x1[u] = v[lane + 64];
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const float ss = pf_wave_sum(x0[u] * x0[u] + x1[u] * x1[u]);
      inv[u] = 1.f / fmaxf(sqrtf(ss), 1e-12f);
    }
#pragma unroll
    for (int u = 0; u < GU; ++u)
      if (p + u * nw < hw) {
        a0 += x0[u] * inv[u];
        a1 += x1[u] * inv[u];
      }
  }
  __shared__ float red[16][128];
  red[wv][lane] = a0;
  red[wv][lane + 64] = a1;
  pf_syncthreads();
  if (threadIdx.x < 128) {
    float s = 0.f;
    for (int k = 0; k < nw; ++k) s += red[k][threadIdx.x];
    out[b * 128 + threadIdx.x] = s / (float)hw;
  }
}

inline int grid_for(long long total, int block) {
  long long g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// ------------------------------------------------------------------ launchers
int pf_nchw_to_nhwc(const float* x, int n, int c, int h, int w, int cso, float* y, hipStream_t st) {
  if (cso == 4 && c <= 4 && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
    hipLaunchKernelGGL(nchw_to_nhwc4_kernel, dim3(grid_for((long long)n * h * w, 256)), dim3(256),
                       0, st, x, n, c, h * w, y);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  }
  const long long total = (long long)n * h * w * cso;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, n, c,
                     h * w, cso, y);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_nhwc_to_nchw(const float* x, int n, int c, int h, int w, int csi, float* y, hipStream_t st) {
  dim3 grid((h * w + 63) / 64, (c + 63) / 64, n);
  if (c % 64 == 0 && (h * w) % 64 == 0 && csi % 4 == 0 &&
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0)
    hipLaunchKernelGGL(nhwc_to_nchw64_kernel, grid, dim3(256), 0, st, x, c, h * w, csi, y);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel, grid, dim3(256), 0, st, x, c, h * w, csi, y);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_maxpool3s2(const float* x, int n, int h, int w, int c, int csi, float* y, int cso,
                  hipStream_t st) {
  const int oh = (h + 2 - 3) / 2 + 1, ow = (w + 2 - 3) / 2 + 1;
  const long long total = (long long)n * oh * ow * (c / 4);
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, n, h, w,
                     c / 4, csi, oh, ow, cso, y);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_upsample2x_ac(const float* x, int n, int h, int w, int c, int csi, float* y, int cso,
                     hipStream_t st) {
  const long long total = (long long)n * 4 * h * w * (c / 4);
  hipLaunchKernelGGL(upsample2x_ac_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, n, h,
                     w, c / 4, csi, y, cso);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// pixels per partial-sum block: ~512 blocks over the batch, >= 64 pixels each
// ~4096 blocks over the batch (16 per CU): at 512 the 472 MB of head.conv1's
// output streamed through 2 blocks per CU at 3.2 TB/s (150 us, r12l)
static int in_chunk(int n, int hw) {
  const int want = std::max(1, (4096 + n - 1) / n);
  const int chunk = std::max(64, (hw + want - 1) / want);
  return chunk;
}

size_t pf_in_stats_ws_bytes(int n, int hw, int C) {
  const int chunk = in_chunk(n, hw);
  const int nchunk = (hw + chunk - 1) / chunk;
  return (size_t)n * nchunk * (C < 1 ? 1 : C) * 2 * sizeof(double);
}

int pf_in_stats(const float* x, int n, int hw, int C, int cs, float* mean, float* rstd,
                double* part, hipStream_t st) {
  const int chunk = in_chunk(n, hw);
  const int nchunk = (hw + chunk - 1) / chunk;
  if (C == 1 && cs == 1) {
    hipLaunchKernelGGL(in1_partial_kernel, dim3(nchunk, n), dim3(256), 0, st, x, hw, chunk, part);
  } else {
    if (C % 4 || C / 4 > 256) return POSFEAT_E_INVALID;
    const int threads = 256;
    hipLaunchKernelGGL(in_partial_kernel, dim3(nchunk, n), dim3(threads),
                       threads * 8 * sizeof(double), st, x, hw, C, cs, chunk, part);
  }
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(in_finalize_kernel, dim3((C + 3) / 4, n), dim3(256), 0, st, x, hw, C, cs,
                     nchunk, part, 1e-5f, mean, rstd, n);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// mean / rstd from unshifted partials part[b][nchunk][C][2] (sum, sum of squares)
// produced by a fused producer (e.g. wino.hip's head.conv2 output transform)
int pf_in_finalize(const double* part, int n, int nchunk, int hw, int C, float* mean, float* rstd,
                   hipStream_t st) {
  hipLaunchKernelGGL(in_finalize_kernel, dim3((C + 3) / 4, n), dim3(256), 0, st, nullptr, hw, C, 0,
                     nchunk, part, 1e-5f, mean, rstd, n);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_in_apply(float* x, int n, int hw, int C, int cs, const float* mean, const float* rstd,
                const float* prelu_slope, hipStream_t st) {
  const long long total = (long long)n * hw * (C / 4);
  hipLaunchKernelGGL(in_apply_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, n, hw,
                     C / 4, cs, mean, rstd, prelu_slope ? 1 : 0, prelu_slope);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_norm_prelu_upsample(const float* x, int n, int h, int w, int C, int csi, const float* mean,
                           const float* rstd, const float* slope, int OH, int OW, float* y,
                           int cso, hipStream_t st) {
  const long long total = (long long)n * OH * OW * (C / 4);
  hipLaunchKernelGGL(norm_prelu_upsample_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x,
                     n, h, w, C / 4, csi, mean, rstd, slope, OH, OW, y, cso);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_head_tail(const float* x, int n, int hw, int cs, const float* mean, const float* rstd,
                 const float* slope, const float* w3, const float* b3, float* yraw, float* out,
                 float* mean1, float* rstd1, double* part, hipStream_t st) {
  const long long total = (long long)n * hw;
  // A/B (POSFEAT_TAIL=<u><n>, A/B build): u pixel pairs per wave step in
  // flight, n = 1: nontemporal loads (y is read once), n = 2 / 3: the waves
  // interleaved over the pixels, nontemporal / plain loads.  Default 43
  // (r16zm, same box, B = 32, two runs each: 41 1.035 / 1.041, 42 1.020 /
  // 1.020, 43 1.007 / 1.005 ms for the tail; earlier, r16i: 40 1.091, 41
  // 1.031, 80 1.493, 81 1.338; 8192 / 16384 / 32768 blocks at 40: 1.091 /
  // 1.073 / 1.053, 2048 at 42: 1.07)
  static const int ab = [] {
    const char* e = pf_ab_getenv("POSFEAT_TAIL");
    return e ? atoi(e) : 43;
  }();
  static const int tmax = [] {
    const char* e = pf_ab_getenv("POSFEAT_TAIL_BLOCKS");
    return e ? atoi(e) : 8192;
  }();
  int blocks = (int)((total / 2 + 3) / 4);
  if (blocks > tmax) blocks = tmax;
  if (blocks < 1) blocks = 1;
  const bool i32 = (long long)total * cs + 128 < (1LL << 31);
  if (ab == 46 && i32)  // (A/B: 32-bit indices, 4 / 8 pairs per step)
    hipLaunchKernelGGL((head_tail_il32_kernel<4>), dim3(blocks), dim3(256), 0, st, x, n, hw, cs,
                       mean, rstd, slope, w3, b3, yraw);
  else if (ab == 47 && i32)
    hipLaunchKernelGGL((head_tail_il32_kernel<8>), dim3(blocks), dim3(256), 0, st, x, n, hw, cs,
                       mean, rstd, slope, w3, b3, yraw);
  else if (ab == 42)  // (A/B: interleaved waves)
    hipLaunchKernelGGL((head_tail_conv3_kernel<4, true, true>), dim3(blocks), dim3(256), 0, st, x, n,
                       hw, cs, mean, rstd, slope, w3, b3, yraw);
  else if (ab == 43)
    hipLaunchKernelGGL((head_tail_conv3_kernel<4, false, true>), dim3(blocks), dim3(256), 0, st, x,
                       n, hw, cs, mean, rstd, slope, w3, b3, yraw);
  else if (ab == 80)
    hipLaunchKernelGGL((head_tail_conv3_kernel<8, false>), dim3(blocks), dim3(256), 0, st, x, n, hw,
                       cs, mean, rstd, slope, w3, b3, yraw);
  else if (ab == 81)
    hipLaunchKernelGGL((head_tail_conv3_kernel<8, true>), dim3(blocks), dim3(256), 0, st, x, n, hw,
                       cs, mean, rstd, slope, w3, b3, yraw);
  else if (ab == 41)
    hipLaunchKernelGGL((head_tail_conv3_kernel<4, true>), dim3(blocks), dim3(256), 0, st, x, n, hw,
                       cs, mean, rstd, slope, w3, b3, yraw);
  else
    hipLaunchKernelGGL((head_tail_conv3_kernel<4, false>), dim3(blocks), dim3(256), 0, st, x, n, hw,
                       cs, mean, rstd, slope, w3, b3, yraw);
  PF_CHECK_LAUNCH();
  PF_TRY(pf_in_stats(yraw, n, hw, 1, 1, mean1, rstd1, part, st));
  if (hw % 4 == 0 && ((reinterpret_cast<uintptr_t>(yraw) | reinterpret_cast<uintptr_t>(out)) & 15) == 0)
    hipLaunchKernelGGL(softplus_norm4_kernel, dim3(grid_for(total / 4, 256)), dim3(256), 0, st,
                       yraw, n, hw, mean1, rstd1, out);
  else
    hipLaunchKernelGGL(softplus_norm_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, yraw,
                       n, hw, mean1, rstd1, out);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_global_feat(const float* g, int n, int hw, int cs, float* out, hipStream_t st) {
  hipLaunchKernelGGL(global_feat_kernel, dim3(n), dim3(1024), 0, st, g, hw, cs, out);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_nchw_to_nhwc(const float* x, int n, int c, int h, int w, int cstride_out,
                                    float* y, void* stream) {
  if (!x || !y || n <= 0 || c <= 0 || h <= 0 || w <= 0 || cstride_out < c) return POSFEAT_E_INVALID;
  return pf_nchw_to_nhwc(x, n, c, h, w, cstride_out, y, pf_stream(stream));
}

extern "C" int posfeat_normalize_rgb8(const unsigned char* src, int b, int h, int w,
                                      int src_pitch, float* dst, void* stream) {
  if (!src || !dst || b <= 0 || h <= 0 || w <= 0 || src_pitch < 3 * w) return POSFEAT_E_INVALID;
  hipLaunchKernelGGL(normalize_rgb8_kernel, dim3((h * w + 255) / 256, b), dim3(256), 0,
                     pf_stream(stream), src, h * w, src_pitch, w, dst);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_nhwc_to_nchw(const float* x, int n, int c, int h, int w, int cstride_in,
                                    float* y, void* stream) {
  if (!x || !y || n <= 0 || c <= 0 || h <= 0 || w <= 0 || cstride_in < c) return POSFEAT_E_INVALID;
  return pf_nhwc_to_nchw(x, n, c, h, w, cstride_in, y, pf_stream(stream));
}
