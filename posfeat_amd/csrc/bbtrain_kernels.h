// bbtrain_kernels.h -- device kernels of the train-mode ResUNet (bbtrain.hip):
// BatchNorm statistics / apply / backward, stride-2 zero insertion, max-pool
// and x2-upsample adjoints, Adam.  Included by bbtrain.hip only.
#pragma once
#include "common.h"

namespace bbt {

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2 };
constexpr float BN_EPS = 1e-5f;
// doubles per SyncBatchNorm exchange slot: [sum | sum of squares | count] of up
// to 1024 channels (2 C + 1), padded
constexpr int BN_SUM_SLOT = 2 * 1024 + 8;

__device__ __forceinline__ float act_grad(int act, float a) {
  return act == ACT_RELU ? (a > 0.f ? 1.f : 0.f) : act == ACT_ELU ? (a > 0.f ? 1.f : a + 1.f) : 1.f;
}

// BatchNorm partial sums: block = (pixel chunk, group of <= 64 channel quads);
// lanes own one quad each, the R = 256/qpb rows of the block stride over the
// chunk's pixels; fp64 accumulation, LDS sum over rows, part[chunk][2][C].
// MODE 0 (forward statistics): sums of y and y^2.
// MODE 1 (backward): g = da act'(a); sums of g and g x^, x^ = (y - mean) rstd.
// the BN output before the residual add, and the activation, exactly as
// bn_apply_kernel evaluates them (the backward recomputes a = act(z) from y
// for non-residual layers instead of re-reading the stored activation)
__device__ __forceinline__ float bn_z(float g, float v, float mu, float rs, float b) {
  return g * (v - mu) * rs + b;
}
__device__ __forceinline__ float act_fwd(int act, float z) {
  return act == ACT_RELU ? fmaxf(z, 0.f) : act == ACT_ELU ? pf_elu(z) : z;
}

// (batch, row, column) of pixel p of an [n][h][w] map, 32-bit when p fits
__device__ __forceinline__ int pix_split(long long p, int w, int h, int& x, int& y) {
  if ((unsigned long long)p <= 0xffffffffULL) {
    const unsigned pu = (unsigned)p, r = pu / (unsigned)w, b = r / (unsigned)h;
    x = (int)(pu - r * (unsigned)w);
    y = (int)(r - b * (unsigned)h);
    return (int)b;
  }
  x = (int)(p % w);
  const long long r = p / w;
  y = (int)(r % h);
  return (int)(r / h);
}

template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(
    const float* __restrict__ y, long long P, int C, int chunk, const float* __restrict__ a, int acs,
    const float* __restrict__ da, int dacs, int act, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gam, const float* __restrict__ bet,
    double* __restrict__ part) {
  __shared__ double red[256][8];
  const int c4n = C / 4, qpb = c4n < 64 ? c4n : 64, R = 256 / qpb;
  const int tid = threadIdx.x, ql = tid % qpb, r = tid / qpb;
  const int q = blockIdx.y * qpb + ql;
  const long long p0 = (long long)blockIdx.x * chunk;
  const long long p1 = p0 + chunk < P ? p0 + chunk : P;
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  f32x4 mu = {0, 0, 0, 0}, rs = {0, 0, 0, 0}, gm = {0, 0, 0, 0}, bt = {0, 0, 0, 0};
  if (MODE == 1) {
    mu = *reinterpret_cast<const f32x4*>(mean + q * 4);
    rs = *reinterpret_cast<const f32x4*>(rstd + q * 4);
    if (!a && act != ACT_NONE) {
      gm = *reinterpret_cast<const f32x4*>(gam + q * 4);
      bt = *reinterpret_cast<const f32x4*>(bet + q * 4);
    }
  }
  // U rows per trip with every load issued before the first add (one 16-byte
  // load per lane in flight left the pass at ~2.5 TB/s); the adds keep the
  // row order p, p + R, ... so the sums are the same bits as one row per trip
  constexpr int U = MODE == 0 ? 4 : 2;
  const float* ap = (MODE == 1 && act != ACT_NONE) ? a : nullptr;
  long long p = p0 + r;
  for (; p + (U - 1) * R < p1; p += U * R) {
    f32x4 v[U], gd[U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long pu = p + u * R;
      v[u] = *reinterpret_cast<const f32x4*>(y + pu * C + q * 4);
      if (MODE == 1) {
        gd[u] = *reinterpret_cast<const f32x4*>(da + pu * dacs + q * 4);
        if (ap) av[u] = *reinterpret_cast<const f32x4*>(ap + pu * acs + q * 4);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          s0[j] += (double)v[u][j];
          s1[j] += (double)v[u][j] * (double)v[u][j];
        }
      } else {
        if (act == ACT_NONE) {
          av[u] = f32x4{0, 0, 0, 0};
        } else if (!ap) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            av[u][j] = act_fwd(act, bn_z(gm[j], v[u][j], mu[j], rs[j], bt[j]));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g = gd[u][j] * act_grad(act, av[u][j]);
          const float xh = (v[u][j] - mu[j]) * rs[j];
          s0[j] += (double)g;
          s1[j] += (double)g * (double)xh;
        }
      }
    }
  }
  for (; p < p1; p += R) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + p * C + q * 4);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0[j] += (double)v[j];
        s1[j] += (double)v[j] * (double)v[j];
      }
    } else {
      const f32x4 gd = *reinterpret_cast<const f32x4*>(da + p * dacs + q * 4);
      f32x4 av = {0, 0, 0, 0};
      if (act != ACT_NONE) {
        if (a) {
          av = *reinterpret_cast<const f32x4*>(a + p * acs + q * 4);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) av[j] = act_fwd(act, bn_z(gm[j], v[j], mu[j], rs[j], bt[j]));
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g = gd[j] * act_grad(act, av[j]);
        const float xh = (v[j] - mu[j]) * rs[j];
        s0[j] += (double)g;
        s1[j] += (double)g * (double)xh;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[tid][j] = s0[j];
    red[tid][4 + j] = s1[j];
  }
  __syncthreads();
  if (r == 0) {
    for (int rr = 1; rr < R; ++rr)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[tid][j] += red[rr * qpb + ql][j];
    double* o = part + (long long)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[q * 4 + j] = red[tid][j];
      o[C + q * 4 + j] = red[tid][4 + j];
    }
  }
}

// Chunk partials -> per-channel totals: block = 4 channels x 64 chunk lanes,
// fixed-order strided sums + LDS tree (deterministic, no serial 1000-deep
// dependent-load chain per channel).
__device__ __forceinline__ void bn_chunk_sum(const double* __restrict__ part, int nchunk, int C,
                                             double (*red)[64][4], double& s0, double& s1) {
  const int cl = threadIdx.x & 3, kl = threadIdx.x >> 2;
  const int c = blockIdx.x * 4 + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    // four chunks' loads in flight per trip, added in chunk order
    int k = kl;
    for (; k + 3 * 64 < nchunk; k += 4 * 64) {
      double va[4], vb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        va[u] = part[(long long)(k + u * 64) * 2 * C + c];
        vb[u] = part[(long long)(k + u * 64) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a += va[u];
        b += vb[u];
      }
    }
    for (; k < nchunk; k += 64) {
      a += part[(long long)k * 2 * C + c];
      b += part[(long long)k * 2 * C + C + c];
    }
  }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (kl < o) {
      red[0][kl][cl] += red[0][kl + o][cl];
      red[1][kl][cl] += red[1][kl + o][cl];
    }
    __syncthreads();
  }
  s0 = red[0][0][cl];
  s1 = red[1][0][cl];
}

// batch mean / rstd (biased variance) and the running-stat update
// (torch: running = (1 - m) running + m batch, with the unbiased variance)
__global__ __launch_bounds__(256) void bn_stats_final_kernel(
    const double* __restrict__ part, int nchunk, int C, long long P, float mom,
    float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rm,
    float* __restrict__ rv) {
  __shared__ double red[2][64][4];
  double s, ss;
  bn_chunk_sum(part, nchunk, C, red, s, ss);
  const int c = blockIdx.x * 4 + (threadIdx.x & 3);
  if ((threadIdx.x >> 2) != 0 || c >= C) return;
  const double mu = s / (double)P;
  double var = ss / (double)P - mu * mu;
  var = var > 0.0 ? var : 0.0;
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + (double)BN_EPS));
  if (rm) {
    const float vu = (float)(P > 1 ? var * (double)P / (double)(P - 1) : var);
    rm[c] = (1.f - mom) * rm[c] + mom * (float)mu;
    rv[c] = (1.f - mom) * rv[c] + mom * vu;
  }
}

// SyncBatchNorm split of the two final kernels: chunk partials -> per-channel
// sums [2][C] (fp64), then (after the cross-rank sum) the statistics from the
// group totals over Ptot = the group's pixel count.
// SyncBatchNorm: this rank's [sum | sum of squares | pixel count] (2 C + 1
// doubles) for the group all-reduce; the count travels with the sums so the
// group normalises by the total count even when ranks hold different batches
// (torch.nn.SyncBatchNorm gathers the per-rank counts the same way)
__global__ __launch_bounds__(256) void bn_sums_kernel(const double* __restrict__ part, int nchunk,
                                                      int C, double count,
                                                      double* __restrict__ sums,
                                                      double* __restrict__ sums_copy) {
  __shared__ double red[2][64][4];
  double s, ss;
  bn_chunk_sum(part, nchunk, C, red, s, ss);
  const int c = blockIdx.x * 4 + (threadIdx.x & 3);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    sums[2 * C] = count;
    if (sums_copy) sums_copy[2 * C] = count;
  }
  if ((threadIdx.x >> 2) != 0 || c >= C) return;
  sums[c] = s;
  sums[C + c] = ss;
  if (sums_copy) {
    sums_copy[c] = s;
    sums_copy[C + c] = ss;
  }
}

__global__ void bn_stats_from_sums_kernel(const double* __restrict__ sums, int C, float mom,
                                          float* __restrict__ mean, float* __restrict__ rstd,
                                          float* __restrict__ rm, float* __restrict__ rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double Ptot = sums[2 * C];  // the group's pixel count
  const double mu = sums[c] / Ptot;
  double var = sums[C + c] / Ptot - mu * mu;
  var = var > 0.0 ? var : 0.0;
  mean[c] = (float)mu;
  rstd[c] = (float)(1.0 / sqrt(var + (double)BN_EPS));
  if (rm) {
    const float vu = (float)(Ptot > 1.0 ? var * Ptot / (Ptot - 1.0) : var);
    rm[c] = (1.f - mom) * rm[c] + mom * (float)mu;
    rv[c] = (1.f - mom) * rv[c] + mom * vu;
  }
}

// dgamma / dbeta from this rank's sums, the apply coefficients from the group's
__global__ void bn_bwd_from_sums_kernel(const double* __restrict__ local,
                                        const double* __restrict__ group, int C,
                                        const float* __restrict__ gam,
                                        const float* __restrict__ rstd, float* __restrict__ dgam,
                                        float* __restrict__ dbet, int acc,
                                        float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double Ptot = group[2 * C];  // the group's pixel count
  const double sg = local[c], sgx = local[C + c];
  dgam[c] = acc ? dgam[c] + (float)sgx : (float)sgx;
  dbet[c] = acc ? dbet[c] + (float)sg : (float)sg;
  coef[c] = gam[c] * rstd[c];
  coef[C + c] = (float)(group[c] / Ptot);
  coef[2 * C + c] = (float)(group[C + c] / Ptot);
}

// out = act(gamma (y - mean) rstd + beta [+ res])
__global__ void bn_apply_kernel(const float* __restrict__ y, long long P, int c4n,
                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                const float* __restrict__ gam, const float* __restrict__ bet,
                                const float* __restrict__ res, int rcs, int act,
                                float* __restrict__ out, int ocs) {
  const long long total = P * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + i * 4);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + q * 4);
    const f32x4 rs = *reinterpret_cast<const f32x4*>(rstd + q * 4);
    const f32x4 g = *reinterpret_cast<const f32x4*>(gam + q * 4);
    const f32x4 b = *reinterpret_cast<const f32x4*>(bet + q * 4);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = bn_z(g[j], v[j], mu[j], rs[j], b[j]);
    if (res) o += *reinterpret_cast<const f32x4*>(res + p * rcs + q * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = act_fwd(act, o[j]);
    *reinterpret_cast<f32x4*>(out + p * ocs + q * 4) = o;
  }
}

// dgamma / dbeta (accumulated over the step's batches) and the apply coefficients
__global__ __launch_bounds__(256) void bn_bwd_final_kernel(
    const double* __restrict__ part, int nchunk, int C, long long P, const float* __restrict__ gam,
    const float* __restrict__ rstd, float* __restrict__ dgam, float* __restrict__ dbet, int acc,
    float* __restrict__ coef) {
  __shared__ double red[2][64][4];
  double sg, sgx;
  bn_chunk_sum(part, nchunk, C, red, sg, sgx);
  const int c = blockIdx.x * 4 + (threadIdx.x & 3);
  if ((threadIdx.x >> 2) != 0 || c >= C) return;
  dgam[c] = acc ? dgam[c] + (float)sgx : (float)sgx;
  dbet[c] = acc ? dbet[c] + (float)sg : (float)sg;
  coef[c] = gam[c] * rstd[c];
  coef[C + c] = (float)(sg / (double)P);
  coef[2 * C + c] = (float)(sgx / (double)P);
}

// dy = gamma rstd (g - E[g] - x^ E[g x^]) (compact); gout = g (optional)
__global__ void bn_bwd_apply_kernel(const float* __restrict__ y, long long P, int c4n,
                                    const float* __restrict__ a, int acs,
                                    const float* __restrict__ da, int dacs, int act,
                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                    const float* __restrict__ gam, const float* __restrict__ bet,
                                    const float* __restrict__ coef, float* __restrict__ dy,
                                    float* __restrict__ gout) {
  const int C = c4n * 4;
  const long long total = P * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const f32x4 v = *reinterpret_cast<const f32x4*>(y + i * 4);
    const f32x4 gd = *reinterpret_cast<const f32x4*>(da + p * dacs + q * 4);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(mean + q * 4);
    const f32x4 rs = *reinterpret_cast<const f32x4*>(rstd + q * 4);
    f32x4 av = {0, 0, 0, 0};
    if (act != ACT_NONE) {
      if (a) {
        av = *reinterpret_cast<const f32x4*>(a + p * acs + q * 4);
      } else {
        const f32x4 gm = *reinterpret_cast<const f32x4*>(gam + q * 4);
        const f32x4 bt = *reinterpret_cast<const f32x4*>(bet + q * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) av[j] = act_fwd(act, bn_z(gm[j], v[j], mu[j], rs[j], bt[j]));
      }
    }
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(coef + q * 4);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(coef + C + q * 4);
    const f32x4 c2 = *reinterpret_cast<const f32x4*>(coef + 2 * C + q * 4);
    f32x4 g, o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[j] = gd[j] * act_grad(act, av[j]);
      const float xh = (v[j] - mu[j]) * rs[j];
      o[j] = c0[j] * (g[j] - c1[j] - xh * c2[j]);
    }
    *reinterpret_cast<f32x4*>(dy + i * 4) = o;
    if (gout) *reinterpret_cast<f32x4*>(gout + i * 4) = g;
  }
}

// Input gradient of a 3x3 stride-2 pad-1 conv by output phases.  dx row iy
// reads dy rows oy with 2 oy - 1 + ky = iy, so the dx row pair (2t-1, 2t)
// depends on dy rows {t-1, t} only: one 2x2 pad-1 conv over dy with 4·Cin
// output channels (phase pe_y·2 + pe_x, pe = 1 for the even row/column of the
// pair) computes all four phases with 16/9 of the exact MACs (zero insertion:
// 4x).  Tap (r, c) of phase (pe_y, pe_x) is the forward tap (kmap(pe_y, r),
// kmap(pe_x, c)), kmap = {(0,0): 2, (0,1): 0, (1,0): none, (1,1): 1}.
// wp [4 Cin][((c/32)*4 + tap)*32 + c%32] from the forward's packed
// w [C][((ci/32)*9 + tap)*32 + ci%32]; Cin, C % 32 == 0.
__device__ __forceinline__ int s2_kmap(int pe, int r) { return pe ? (r ? 1 : -1) : (r ? 0 : 2); }

// planes (optional): wp also as three bf16 planes (pf_split3_rows' layout)
__global__ void s2_phase_weights_kernel(const float* __restrict__ w, int C, int Cin,
                                        float* __restrict__ wp, unsigned short* __restrict__ planes) {
  const int kp4 = C * 4, kp9 = C * 9;
  const long long total = 4LL * Cin * kp4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(i / kp4), k = (int)(i - (long long)o * kp4);
    const int ph = o / Cin, ci = o - ph * Cin;
    const int tap = (k >> 5) & 3, c = (k >> 7) * 32 + (k & 31);
    const int ky = s2_kmap(ph >> 1, tap >> 1), kx = s2_kmap(ph & 1, tap & 1);
    const float v = (ky >= 0 && kx >= 0)
                        ? w[(long long)c * kp9 + ((ci >> 5) * 9 + ky * 3 + kx) * 32 + (ci & 31)]
                        : 0.f;
    wp[i] = v;
    if (planes) {
      unsigned hh, mm, ll;
      pf_split3_pair(v, 0.f, hh, mm, ll);
      planes[i] = (unsigned short)hh;
      planes[i + total] = (unsigned short)mm;
      planes[i + 2 * total] = (unsigned short)ll;
    }
  }
}

// dx [n][h][w] (pitch dxcs) = the stride-2 input gradient from
//   mode 1: the phase conv's output src [n][h/2+1][w/2+1][4 Cin]
//   mode 0: a 1x1 conv's compact output src [n][h/2][w/2][Cin] (even pixels; 0 elsewhere)
// plus add (pitch addcs) when given
__global__ void s2_scatter_kernel(const float* __restrict__ src, int mode, int n, int h, int w,
                                  int c4n, const float* __restrict__ add, int addcs,
                                  float* __restrict__ dx, int dxcs) {
  const int Cin = c4n * 4, oh = h / 2, ow = w / 2;
  const long long total = (long long)n * h * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    int ix, iy;
    const int b = pix_split(p, w, h, ix, iy);
    f32x4 v = {0, 0, 0, 0};
    if (mode == 1) {
      const int t = (iy + 1) >> 1, s = (ix + 1) >> 1;
      const int ph = (1 - (iy & 1)) * 2 + (1 - (ix & 1));
      v = *reinterpret_cast<const f32x4*>(
          src + (((long long)b * (oh + 1) + t) * (ow + 1) + s) * 4 * Cin + ph * Cin + q * 4);
    } else if (!(iy & 1) && !(ix & 1)) {
      v = *reinterpret_cast<const f32x4*>(
          src + (((long long)b * oh + (iy >> 1)) * ow + (ix >> 1)) * Cin + q * 4);
    }
    if (add) v += *reinterpret_cast<const f32x4*>(add + p * addcs + q * 4);
    *reinterpret_cast<f32x4*>(dx + p * dxcs + q * 4) = v;
  }
}

// dst [n][h][w][C] = src [n][h/2][w/2][C] at even (y, x), 0 elsewhere: the
// input grid of a stride-2 conv (its output pixel i reads input 2i - pad + k)
__global__ void zero_insert_kernel(const float* __restrict__ src, int n, int h, int w, int c4n,
                                   float* __restrict__ dst) {
  const int oh = (h + 1) / 2, ow = (w + 1) / 2;
  const long long total = (long long)n * h * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    int x, yy;
    const int b = pix_split(p, w, h, x, yy);
    f32x4 v = {0, 0, 0, 0};
    if (!(x & 1) && !(yy & 1))
      v = *reinterpret_cast<const f32x4*>(
          src + ((((long long)b * oh + (yy >> 1)) * ow + (x >> 1)) * c4n + q) * 4);
    *reinterpret_cast<f32x4*>(dst + i * 4) = v;
  }
}

// max_pool2d(3, 2, 1) forward that also records each output's arg-max tap
// t = 3 (iy - 2 oy + 1) + (ix - 2 ox + 1) per channel (one byte, idx
// [n][oh][ow][C]), chosen by the adjoint's rule (scan order, replace on '>'
// or NaN, start at the window's first valid pixel); y = the value there
// (= fmaxf over the window for finite input, as maxpool3s2_kernel)
__global__ void maxpool3s2_idx_kernel(const float* __restrict__ x, int xcs, int n, int h, int w,
                                      int c4n, int oh, int ow, float* __restrict__ y, int ycs,
                                      unsigned* __restrict__ idx) {
  const long long total = (long long)n * oh * ow * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    int ox, oy;
    const int b = pix_split(p, ow, oh, ox, oy);
    f32x4 v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = 2 * oy + t / 3 - 1, ix = 2 * ox + t % 3 - 1;
      ok[t] = (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      const int cy = min(max(iy, 0), h - 1), cx = min(max(ix, 0), w - 1);
      v[t] = *reinterpret_cast<const f32x4*>(x + (((long long)b * h + cy) * w + cx) * xcs + q * 4);
    }
    f32x4 mv = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int mt[4] = {-1, -1, -1, -1};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (mt[j] < 0 || v[t][j] > mv[j] || isnan(v[t][j])) {
          mv[j] = v[t][j];
          mt[j] = t;
        }
    }
    *reinterpret_cast<f32x4*>(y + p * ycs + q * 4) = mv;
    idx[i] = (unsigned)mt[0] | ((unsigned)mt[1] << 8) | ((unsigned)mt[2] << 16) |
             ((unsigned)mt[3] << 24);
  }
}

// max_pool2d(3, 2, 1) adjoint as a gather from the recorded arg-max taps:
// input pixel (iy, ix) sums the gradient of every window whose tap points at
// it, windows in row-major order (the sums of the round-4 form, which re-read
// and re-ranked the nine inputs of each window: 4 + 16 bytes per window now)
__global__ void maxpool_adjoint_idx_kernel(const unsigned* __restrict__ idx, int n, int h, int w,
                                           int c4n, const float* __restrict__ g, int gcs, int oh,
                                           int ow, float* __restrict__ dx, int dxcs) {
  const long long total = (long long)n * h * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    int ix, iy;
    const int b = pix_split(p, w, h, ix, iy);
    f32x4 acc = {0, 0, 0, 0};
    const int oy0 = iy / 2, oy1 = min(oh - 1, (iy + 1) / 2);
    const int ox0 = ix / 2, ox1 = min(ow - 1, (ix + 1) / 2);
    for (int oy = oy0; oy <= oy1; ++oy) {
      for (int ox = ox0; ox <= ox1; ++ox) {
        const long long o = ((long long)b * oh + oy) * ow + ox;
        const unsigned tw = idx[o * c4n + q];
        const f32x4 gv = *reinterpret_cast<const f32x4*>(g + o * gcs + q * 4);
        const int ty = iy - 2 * oy + 1, tx = ix - 2 * ox + 1;
        const unsigned me = (unsigned)(3 * ty + tx);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (((tw >> (8 * j)) & 255u) == me) acc[j] += gv[j];
      }
    }
    *reinterpret_cast<f32x4*>(dx + p * dxcs + q * 4) = acc;
  }
}

// bilinear x2, align_corners=True (fmap.hip upsample2x_ac_kernel): weight of
// output o on input q, with the forward's own float arithmetic
__device__ __forceinline__ float ac_w(int o, int q, float sc, int nin) {
  const float r = sc * o;
  const int i0 = (int)r;
  const int i1 = i0 + (i0 < nin - 1 ? 1 : 0);
  const float l = r - i0;
  return (i0 == q ? 1.f - l : 0.f) + (i1 == q ? l : 0.f);
}

// t[b][oy][qx][c] = sum_ox w(ox, qx) g[b][oy][ox][c]
__global__ void up2_adj_x_kernel(const float* __restrict__ g, int gcs, int nb, int OH, int OW, int w,
                                 int c4n, float* __restrict__ t) {
  const float sc = OW > 1 ? (float)(w - 1) / (float)(OW - 1) : 0.f;
  const long long total = (long long)nb * OH * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    const int qx = (int)(p % w);
    const long long row = p / w;
    const float* gr = g + row * OW * gcs + q * 4;
    f32x4 acc = {0, 0, 0, 0};
    const int o0 = max(0, 2 * qx - 2), o1 = min(OW - 1, 2 * qx + 4);
    for (int ox = o0; ox <= o1; ++ox) {
      const float wt = ac_w(ox, qx, sc, w);
      if (wt != 0.f) acc += wt * *reinterpret_cast<const f32x4*>(gr + (long long)ox * gcs);
    }
    *reinterpret_cast<f32x4*>(t + p * (c4n * 4) + q * 4) = acc;
  }
}

// d[b][qy][qx][c] = sum_oy w(oy, qy) t[b][oy][qx][c]
__global__ void up2_adj_y_kernel(const float* __restrict__ t, int nb, int OH, int h, int w, int c4n,
                                 float* __restrict__ d, int dcs) {
  const float sc = OH > 1 ? (float)(h - 1) / (float)(OH - 1) : 0.f;
  const int C = c4n * 4;
  const long long total = (long long)nb * h * w * c4n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long p;
    const int q = pf_quad_split(i, c4n, p);
    int qx, qy;
    const int b = pix_split(p, w, h, qx, qy);
    f32x4 acc = {0, 0, 0, 0};
    const int o0 = max(0, 2 * qy - 2), o1 = min(OH - 1, 2 * qy + 4);
    for (int oy = o0; oy <= o1; ++oy) {
      const float wt = ac_w(oy, qy, sc, h);
      if (wt != 0.f)
        acc += wt * *reinterpret_cast<const f32x4*>(t + (((long long)b * OH + oy) * w + qx) * C + q * 4);
    }
    *reinterpret_cast<f32x4*>(d + (((long long)b * h + qy) * w + qx) * dcs + q * 4) = acc;
  }
}

// torch.optim.Adam (no amsgrad): m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p += (-lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)   (torch/optim/adam.py)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float neg_step, float b1, float b2,
                            float eps, float bc2_sqrt, float gscale, float wd) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    if (wd != 0.f) gi += wd * p[i];
    const float w1 = 1.f - b1;
    float mi = m[i];
    mi = w1 < 0.5f ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float den = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + neg_step * (mi / den);
  }
}

}  // namespace bbt
