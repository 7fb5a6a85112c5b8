// sample.hip -- bilinear descriptor sampling at keypoints + L2 norm (gfx950).
//
// Replaces losses/preprocess_utils.py:40-53 sample_feat_by_coord:
//   F.grid_sample(x, coord_n[:, :, None], mode='bilinear', padding_mode='zeros',
//                 align_corners=False) -> F.normalize(p=2, dim=1, eps=1e-12)
// One wave per keypoint.  The map is NHWC, so each of the 4 bilinear taps is a
// contiguous C-float row (512 B at C=128): lane l reads channels l, l+64, ...
// -> fully coalesced; the sum of squares is a wave shuffle reduction.
#include "common.h"

namespace {

template <int CPL>  // channels per lane (C <= 64*CPL)
__global__ void sample_desc_kernel(const float* __restrict__ fmap, int nb, int C, int h, int w,
                                   int cs, const float* __restrict__ coord, int npts,
                                   const int32_t* __restrict__ n_valid, int each,
                                   int normalize, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long total = (long long)nb * npts;
  if (wid >= total) return;
  const int b = (int)(wid / npts);
  const int k = (int)(wid - (long long)b * npts);
  float* o = out + wid * C;
  const int nv = n_valid ? n_valid[each ? b : 0] : npts;
  if (k >= nv) {
    for (int c = lane; c < C; c += 64) o[c] = 0.f;
    return;
  }
  const float gx = coord[wid * 2 + 0], gy = coord[wid * 2 + 1];
  // grid_sampler_compute_source_index, align_corners=False
  const float ix = ((gx + 1.f) * w - 1.f) / 2.f;
  const float iy = ((gy + 1.f) * h - 1.f) / 2.f;
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  const float wnw = (x1 - ix) * (y1 - iy);
  const float wne = (ix - x0) * (y1 - iy);
  const float wsw = (x1 - ix) * (iy - y0);
  const float wse = (ix - x0) * (iy - y0);
  const bool bx0 = (unsigned)x0 < (unsigned)w, bx1 = (unsigned)x1 < (unsigned)w;
  const bool by0 = (unsigned)y0 < (unsigned)h, by1 = (unsigned)y1 < (unsigned)h;
  const float* base = fmap + (long long)b * h * w * cs;
  float v[CPL];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    float acc = 0.f;
    if (c < C) {
      if (by0 && bx0) acc += base[((long long)y0 * w + x0) * cs + c] * wnw;
      if (by0 && bx1) acc += base[((long long)y0 * w + x1) * cs + c] * wne;
      if (by1 && bx0) acc += base[((long long)y1 * w + x0) * cs + c] * wsw;
      if (by1 && bx1) acc += base[((long long)y1 * w + x1) * cs + c] * wse;
    }
    v[q] = acc;
    ss += acc * acc;
  }
  float inv = 1.f;
  if (normalize) {
    ss = pf_wave_sum(ss);
    inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  }
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    if (c < C) o[c] = normalize ? v[q] * inv : v[q];
  }
}

// C == 128: a half-wave per keypoint, 4 channels (16-B loads) per lane --
// two keypoints per wave and half the load instructions of the one-wave form;
// each channel's bilinear sum in the same order (the norm's sum of squares is
// grouped differently: per-lane quads, then a 32-lane tree)
__global__ PF_NO_PK_FP32 void sample_desc128_kernel(const float* __restrict__ fmap, int nb, int h, int w, int cs,
                                      const float* __restrict__ coord, int npts,
                                      const int32_t* __restrict__ n_valid, int each,
                                      int normalize, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const long long kid =
      (blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + half;
  const long long total = (long long)nb * npts;
  if (kid >= total) return;  // (total is even per wave unless npts * nb is odd: the pair's
                             // other half still runs its own shuffles below)
  const int b = (int)(kid / npts);
  const int k = (int)(kid - (long long)b * npts);
  float* o = out + kid * 128 + 4 * l32;
  const int nv = n_valid ? n_valid[each ? b : 0] : npts;
  const bool valid = k < nv;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (valid) {
    const float gx = coord[kid * 2 + 0], gy = coord[kid * 2 + 1];
    const float ix = ((gx + 1.f) * w - 1.f) / 2.f;
    const float iy = ((gy + 1.f) * h - 1.f) / 2.f;
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = (x1 - ix) * (y1 - iy);
    const float wne = (ix - x0) * (y1 - iy);
    const float wsw = (x1 - ix) * (iy - y0);
    const float wse = (ix - x0) * (iy - y0);
    const bool bx0 = (unsigned)x0 < (unsigned)w, bx1 = (unsigned)x1 < (unsigned)w;
    const bool by0 = (unsigned)y0 < (unsigned)h, by1 = (unsigned)y1 < (unsigned)h;
    const float* base = fmap + (long long)b * h * w * cs + 4 * l32;
    if (by0 && bx0) acc += *reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x0) * cs) * wnw;
    if (by0 && bx1) acc += *reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x1) * cs) * wne;
    if (by1 && bx0) acc += *reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x0) * cs) * wsw;
    if (by1 && bx1) acc += *reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x1) * cs) * wse;
  }
  float inv = 1.f;
  if (normalize) {
    float ss = acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) ss += pf_shfl_xor(ss, off, 64);
    inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  }
  *reinterpret_cast<f32x4*>(o) = valid ? (normalize ? acc * inv : acc) : f32x4{0.f, 0.f, 0.f, 0.f};
}

}  // namespace

namespace {

int sample_impl(const float* fmap, int b, int c, int h, int w, int cs, const float* coord,
                int npts, const int32_t* n_valid, int each, int normalize, float* out,
                hipStream_t st) {
  const long long waves = (long long)b * npts;
  if (waves == 0) return POSFEAT_OK;
  const int wpb = 4;
  if (c == 128 && cs % 4 == 0 && (reinterpret_cast<uintptr_t>(fmap) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const long long w2 = (waves + 1) / 2;  // two keypoints per wave
    hipLaunchKernelGGL(sample_desc128_kernel, dim3((unsigned)((w2 + wpb - 1) / wpb)),
                       dim3(64 * wpb), 0, st, fmap, b, h, w, cs, coord, npts, n_valid, each,
                       normalize, out);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  }
  const dim3 grid((unsigned)((waves + wpb - 1) / wpb)), block(64 * wpb);
  if (c <= 64)
    hipLaunchKernelGGL(sample_desc_kernel<1>, grid, block, 0, st, fmap, b, c, h, w, cs, coord,
                       npts, n_valid, each, normalize, out);
  else if (c <= 128)
    hipLaunchKernelGGL(sample_desc_kernel<2>, grid, block, 0, st, fmap, b, c, h, w, cs, coord,
                       npts, n_valid, each, normalize, out);
  else if (c <= 256)
    hipLaunchKernelGGL(sample_desc_kernel<4>, grid, block, 0, st, fmap, b, c, h, w, cs, coord,
                       npts, n_valid, each, normalize, out);
  else if (c <= 1024)
    hipLaunchKernelGGL(sample_desc_kernel<16>, grid, block, 0, st, fmap, b, c, h, w, cs, coord,
                       npts, n_valid, each, normalize, out);
  else
    return POSFEAT_E_UNSUPPORTED;
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

}  // namespace

int pf_sample_desc(const float* fmap, int b, int c, int h, int w, int cs, const float* coord,
                   int npts, const int32_t* n_valid, int normalize, float* out, hipStream_t st) {
  return sample_impl(fmap, b, c, h, w, cs, coord, npts, n_valid, 0, normalize, out, st);
}

extern "C" int posfeat_sample_desc(const float* fmap, int b, int c, int h, int w, int cstride,
                                   const float* coord, int npts, const int32_t* n_valid,
                                   int normalize, float* out, void* stream) {
  if (!fmap || !coord || !out || b <= 0 || c <= 0 || h <= 0 || w <= 0 || npts < 0 || cstride < c)
    return POSFEAT_E_INVALID;
  return pf_sample_desc(fmap, b, c, h, w, cstride, coord, npts, n_valid, normalize, out,
                        pf_stream(stream));
}

extern "C" int posfeat_sample_desc_each(const float* fmap, int b, int c, int h, int w,
                                        int cstride, const float* coord, int npts,
                                        const int32_t* n_valid, int normalize, float* out,
                                        void* stream) {
  if (!fmap || !coord || !n_valid || !out || b <= 0 || c <= 0 || h <= 0 || w <= 0 || npts < 0 ||
      cstride < c)
    return POSFEAT_E_INVALID;
  return sample_impl(fmap, b, c, h, w, cstride, coord, npts, n_valid, 1, normalize, out,
                     pf_stream(stream));
}
