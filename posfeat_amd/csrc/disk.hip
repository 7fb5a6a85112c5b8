// disk.hip -- DiskLoss forward on gfx950 (keypoint-head REINFORCE loss).
//
// Replaces losses/kploss.py:132-197 DiskLoss.forward with point_distribution
// (20-35), point_sample (37-48) and constant_reward (50-89), configuration of
// configs/train_kp.yaml:56-73 (grid 8, T 60, reward_thr 2, +1 / -0.25,
// kp_penalty -0.001, cor_detach).
//
//   disk_point       one wave per 8x8 cell (64 lanes = 64 logits): log-softmax,
//                    Categorical proposal (given, or Gumbel-max from uniforms),
//                    Bernoulli acceptance (given, or u < sigmoid(l)), logp, pixel
//                    and normalised coordinates
//   sample_desc      L2-normalised descriptors at the proposals (sample.hip)
//   S = f1 f2^T      conv_mfma 1x1 implicit GEMM (FP32 MFMA), [n1][n2] per pair
//   row/col lse      logsumexp of aff = -T(1 - S) along n and along m
//   epi lines        normalised epipolar lines l1 = F1 x1/|..|, l2 = F2 x2/|..|
//   reinforce        sum over accepted pairs of reward * p * (logp_dense + logp1 +
//                    logp2), p = softmax_row * softmax_col, fixed-order block
//                    partials (fp64) + one final workgroup -> deterministic
// The dense B x n x n probability matrices of the reference are never
// materialised.  Default (flash) path: S is not materialised either --
// disk_flash_kernel recomputes S = f1 f2^T tiles with fp32 MFMA in four
// passes and folds them on the fly:
//   LSE  (A, B) = (f1, f2) -> column logsumexp lse_c;  (f2, f1) -> lse_r
//   SUM  (A, B) = (f1 acc, f2 acc) -> per accepted column n: sum_m reward p
//        (= -dL/dlogp2[n] - penalty) and sum_m reward p (logp_dense + logp1 + logp2)
//        (the reinforce partial);  (f2 acc, f1 acc) -> sum_n reward p per m
// Each pass keeps, per column lane, a running state over the A rows (B's
// columns stay in VGPRs as MFMA fragments; A streams through LDS by DMA), so
// every reduction is a per-lane sequential sum in increasing row order plus
// fixed-order merges: deterministic, no atomics.  The SUM passes run only over
// the accepted points (stable compaction first).  POSFEAT_DISK_FLASH=0 keeps
// the S-materialising path (92 MB per pair at 480x640) for A/B.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "fmap.h"

int pf_sample_desc(const float* fmap, int b, int c, int h, int w, int cs, const float* coord,
                   int npts, const int32_t* n_valid, int normalize, float* out, hipStream_t st);

namespace {

// torch binary_cross_entropy_with_logits(x, y) -> logp = -loss
__device__ __forceinline__ float bern_logp(float x, bool y) {
  const float t = log1pf(expf(-fabsf(x)));
  return y ? -(fmaxf(-x, 0.f) + t) : -(fmaxf(x, 0.f) + t);
}

__global__ PF_NO_PK_FP32 void disk_point_kernel(const float* __restrict__ kp, int nb, int H, int W,
                                  const int32_t* __restrict__ prop_in,
                                  const uint8_t* __restrict__ acc_in,
                                  const float* __restrict__ uni,  // [b][n][65] if sampling
                                  int32_t* __restrict__ prop_out, uint8_t* __restrict__ acc_out,
                                  float* __restrict__ cpx, float* __restrict__ cn,
                                  float* __restrict__ logp) {
  constexpr int G = 8;
  const int lane = threadIdx.x & 63;
  const int hc = H / G, wc = W / G, n = hc * wc;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n) return;
  const int b = (int)(wid / n), k = (int)(wid - (long long)b * n);
  const int cy = k / wc, cx = k - cy * wc;
  const float v = kp[((long long)b * H + cy * G + lane / G) * W + cx * G + lane % G];
  float mx = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, pf_shfl_xor(mx, o, 64));
  const float lse = mx + logf(pf_wave_sum(expf(v - mx)));
  int p;
  bool a;
  if (uni) {  // Gumbel-max == Categorical(logits) sample; accept ~ Bernoulli(sigmoid)
    const float u = fminf(fmaxf(uni[wid * 65 + lane], 1e-20f), 1.f - 1e-7f);
    float key = v - logf(-logf(u));
    int arg = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ok = pf_shfl_xor(key, o, 64);
      const int oa = pf_shfl_xor(arg, o, 64);
      if (ok > key || (ok == key && oa < arg)) {
        key = ok;
        arg = oa;
      }
    }
    p = arg;
    const float lp = pf_shfl(v, p, 64);
    a = uni[wid * 65 + 64] < 1.f / (1.f + expf(-lp));
  } else {
    p = prop_in[wid];
    a = acc_in[wid] != 0;
  }
  const float lv = pf_shfl(v, p, 64);
  if (lane == 0) {
    prop_out[wid] = p;
    acc_out[wid] = a ? 1 : 0;
    logp[wid] = (lv - lse) + bern_logp(lv, a);
    const float x = (float)(cx * G + p % G), y = (float)(cy * G + p / G);
    cpx[wid * 2] = x;
    cpx[wid * 2 + 1] = y;
    const float c0 = (float)((W - 1) / 2.0), c1 = (float)((H - 1) / 2.0);
    cn[wid * 2] = (x - c0) / c0;
    cn[wid * 2 + 1] = (y - c1) / c1;
  }
}

// lse_r[m] = logsumexp_n(T*S[m][n] - T); one wave per row
__global__ void row_lse_kernel(const float* __restrict__ S, long long rows, int n2, float T,
                               float* __restrict__ lse) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= rows) return;
  const float* r = S + wid * n2;
  float mx = -INFINITY;
  for (int k = lane; k < n2; k += 64) mx = fmaxf(mx, T * r[k] - T);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, pf_shfl_xor(mx, o, 64));
  float s = 0.f;
  for (int k = lane; k < n2; k += 64) s += expf((T * r[k] - T) - mx);
  s = pf_wave_sum(s);
  if (lane == 0) lse[wid] = mx + logf(s);
}

// lse_c[n] = logsumexp_m(T*S[m][n] - T), two levels: block = 64 columns x
// one of COL_CH row chunks, 4 row lanes per column (each wave reads 256
// contiguous bytes of a row), online max-rescaled sums; then the chunk
// partials of each column are merged in chunk order (deterministic).
constexpr int COL_CH = 8;
__global__ __launch_bounds__(256) void col_lse_partial_kernel(const float* __restrict__ S, int n1,
                                                              int n2, float T,
                                                              float2* __restrict__ part) {
  const int b = blockIdx.z, ch = blockIdx.y, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int m0 = (int)((long long)n1 * ch / COL_CH), m1 = (int)((long long)n1 * (ch + 1) / COL_CH);
  const float* Sb = S + (long long)b * n1 * n2;
  float mx = -INFINITY, sm = 0.f;
  if (col < n2) {
    for (int m = m0 + rg; m < m1; m += 4) {
      const float v = T * Sb[(long long)m * n2 + col] - T;
      if (v > mx) {
        sm = sm * expf(mx - v) + 1.f;
        mx = v;
      } else {
        sm += expf(v - mx);
      }
    }
  }
  __shared__ float smx[4][64], ssm[4][64];
  smx[rg][threadIdx.x & 63] = mx;
  ssm[rg][threadIdx.x & 63] = sm;
  pf_syncthreads();
  if (rg == 0 && col < n2) {
    float M = smx[0][threadIdx.x];
    for (int r = 1; r < 4; ++r) M = fmaxf(M, smx[r][threadIdx.x]);
    float t = 0.f;
    for (int r = 0; r < 4; ++r) t += ssm[r][threadIdx.x] * expf(smx[r][threadIdx.x] - M);
    part[((long long)b * COL_CH + ch) * n2 + col] = make_float2(M, t);
  }
}

__global__ void col_lse_final_kernel(const float2* __restrict__ part, int nb, int n2,
                                     float* __restrict__ lse) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nb * n2) return;
  const int b = (int)(i / n2), col = (int)(i - (long long)b * n2);
  float M = -INFINITY;
  for (int ch = 0; ch < COL_CH; ++ch) M = fmaxf(M, part[((long long)b * COL_CH + ch) * n2 + col].x);
  float t = 0.f;
  for (int ch = 0; ch < COL_CH; ++ch) {
    const float2 q = part[((long long)b * COL_CH + ch) * n2 + col];
    t += q.y * expf(q.x - M);
  }
  lse[i] = M + logf(t);
}

// normalised epipolar line of each point: l = F x / max(|l[:2]|, 1e-8)
__global__ void epi_line_kernel(const float* __restrict__ Fm, const float* __restrict__ cpx,
                                int nb, int n, float* __restrict__ line) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * n) return;
  const float* F = Fm + (i / n) * 9;
  const float x = cpx[2 * i], y = cpx[2 * i + 1];
  const float a = F[0] * x + F[1] * y + F[2];
  const float b = F[3] * x + F[4] * y + F[5];
  const float c = F[6] * x + F[7] * y + F[8];
  const float nr = fmaxf(sqrtf(a * a + b * b), 1e-8f);
  line[3 * i] = a / nr;
  line[3 * i + 1] = b / nr;
  line[3 * i + 2] = c / nr;
}

constexpr int RB = 256;  // threads per reinforce block

// per-block partial of sum_{acc1[m] & acc2[n]} reward * p * (logp_dense + logp1 + logp2)
// block = (row tile of 4 rows, pair); threads sweep the columns
__global__ __launch_bounds__(RB) void reinforce_kernel(
    const float* __restrict__ S, int n1, int n2, float T, const float* __restrict__ lse_r,
    const float* __restrict__ lse_c, const uint8_t* __restrict__ acc1,
    const uint8_t* __restrict__ acc2, const float* __restrict__ logp1,
    const float* __restrict__ logp2, const float* __restrict__ line1,
    const float* __restrict__ line2, const float* __restrict__ c1px, const float* __restrict__ c2px,
    float thr, float good, float bad, double* __restrict__ part) {
  const int b = blockIdx.y;
  const int m0 = blockIdx.x * 4;
  const float* Sb = S + (long long)b * n1 * n2;
  double acc = 0.0;
  for (int mm = 0; mm < 4; ++mm) {
    const int m = m0 + mm;
    if (m >= n1) break;
    const long long gm = (long long)b * n1 + m;
    if (!acc1[gm]) continue;  // uniform per block
    const float lr = lse_r[gm], lp1 = logp1[gm];
    const float a1 = line1[3 * gm], b1 = line1[3 * gm + 1], k1 = line1[3 * gm + 2];
    const float x1 = c1px[2 * gm], y1 = c1px[2 * gm + 1];
    float rowsum = 0.f;
    for (int nn = threadIdx.x; nn < n2; nn += RB) {
      const long long gn = (long long)b * n2 + nn;
      if (!acc2[gn]) continue;
      const float aff = T * Sb[(long long)m * n2 + nn] - T;
      const float lpr = aff - lr, lpc = aff - lse_c[gn];
      const float p = expf(lpr) * expf(lpc);
      const float x2 = c2px[2 * gn], y2 = c2px[2 * gn + 1];
      const float d1 = fabsf(a1 * x2 + b1 * y2 + k1);
      const float d2 = fabsf(line2[3 * gn] * x1 + line2[3 * gn + 1] * y1 + line2[3 * gn + 2]);
      const float rw = (d1 < thr && d2 < thr) ? good : bad;
      rowsum += rw * (p * ((lpr + lpc) + (lp1 + logp2[gn])));
    }
    acc += rowsum;
  }
  // fixed-order block reduction
  __shared__ double red[RB];
  red[threadIdx.x] = acc;
  pf_syncthreads();
  for (int o = RB / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    pf_syncthreads();
  }
  if (threadIdx.x == 0) part[(long long)b * gridDim.x + blockIdx.x] = red[0];
}

// ---------------------------------------------------------------- backward
// With cor_detach (sample_p detached) and match_grad False the loss depends on
// the score maps only through kps_logp (kploss.py:175-182):
//   dL/dlogp1[m] = acc1[m] * (-sum_{n: acc2} reward p - kp_penalty), likewise for 2
// and logp = log_softmax(cell)[prop] + log sigmoid(+/- logit[prop]) (20-35).
struct PairCtx {
  const float* S;
  int n1, n2;
  float T, thr, good, bad;
  const float *lse_r, *lse_c, *line1, *line2, *c1px, *c2px;
};

// reward * p for accepted pair (m, n) of pair b: the same float expression as
// reinforce_kernel
__device__ __forceinline__ float pair_rp(const PairCtx& c, int b, int m, int nn) {
  const long long gm = (long long)b * c.n1 + m, gn = (long long)b * c.n2 + nn;
  const float aff = c.T * c.S[((long long)b * c.n1 + m) * c.n2 + nn] - c.T;
  const float p = expf(aff - c.lse_r[gm]) * expf(aff - c.lse_c[gn]);
  const float x1 = c.c1px[2 * gm], y1 = c.c1px[2 * gm + 1];
  const float x2 = c.c2px[2 * gn], y2 = c.c2px[2 * gn + 1];
  const float d1 = fabsf(c.line1[3 * gm] * x2 + c.line1[3 * gm + 1] * y2 + c.line1[3 * gm + 2]);
  const float d2 = fabsf(c.line2[3 * gn] * x1 + c.line2[3 * gn + 1] * y1 + c.line2[3 * gn + 2]);
  return ((d1 < c.thr && d2 < c.thr) ? c.good : c.bad) * p;
}

// g1[m] = dL/dlogp1[m]; one wave per row
__global__ void grad_row_kernel(PairCtx c, int nb, const uint8_t* __restrict__ acc1,
                                const uint8_t* __restrict__ acc2, float kp_penalty,
                                float* __restrict__ g1) {
  const int lane = threadIdx.x & 63;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * c.n1) return;
  const int b = (int)(wid / c.n1), m = (int)(wid - (long long)b * c.n1);
  if (!acc1[wid]) {
    if (lane == 0) g1[wid] = 0.f;
    return;
  }
  float s = 0.f;
  for (int nn = lane; nn < c.n2; nn += 64)
    if (acc2[(long long)b * c.n2 + nn]) s += pair_rp(c, b, m, nn);
  s = pf_wave_sum(s);
  if (lane == 0) g1[wid] = -s - kp_penalty;
}

// g2[n] = dL/dlogp2[n]: column sums in COL_CH row chunks (4 row lanes per
// column), merged in chunk order
__global__ __launch_bounds__(256) void grad_col_partial_kernel(PairCtx c,
                                                               const uint8_t* __restrict__ acc1,
                                                               const uint8_t* __restrict__ acc2,
                                                               float* __restrict__ part) {
  const int b = blockIdx.z, ch = blockIdx.y, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int m0 = (int)((long long)c.n1 * ch / COL_CH), m1 = (int)((long long)c.n1 * (ch + 1) / COL_CH);
  float s = 0.f;
  if (col < c.n2 && acc2[(long long)b * c.n2 + col])
    for (int m = m0 + rg; m < m1; m += 4)
      if (acc1[(long long)b * c.n1 + m]) s += pair_rp(c, b, m, col);
  __shared__ float ss[4][64];
  ss[rg][threadIdx.x & 63] = s;
  pf_syncthreads();
  if (rg == 0 && col < c.n2)
    part[((long long)b * COL_CH + ch) * c.n2 + col] =
        ((ss[0][threadIdx.x] + ss[1][threadIdx.x]) + ss[2][threadIdx.x]) + ss[3][threadIdx.x];
}

__global__ void grad_col_final_kernel(const float* __restrict__ part, int nb, int n2,
                                      const uint8_t* __restrict__ acc2, float kp_penalty,
                                      float* __restrict__ g2) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nb * n2) return;
  const int b = (int)(i / n2), col = (int)(i - (long long)b * n2);
  float t = 0.f;
  for (int ch = 0; ch < COL_CH; ++ch) t += part[((long long)b * COL_CH + ch) * n2 + col];
  g2[i] = acc2[i] ? -t - kp_penalty : 0.f;
}

// dkp over one 8x8 cell (one wave): g * ([j == prop] (1 + d alogp/dl) - softmax_j),
// d alogp/dl = accepted ? 1 - sigmoid(l) : -sigmoid(l)
__global__ void disk_point_grad_kernel(const float* __restrict__ kp, int nb, int H, int W,
                                       const int32_t* __restrict__ prop,
                                       const uint8_t* __restrict__ acc,
                                       const float* __restrict__ g, float* __restrict__ dkp) {
  constexpr int G = 8;
  const int lane = threadIdx.x & 63;
  const int hc = H / G, wc = W / G, n = hc * wc;
  const long long wid = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long long)nb * n) return;
  const int b = (int)(wid / n), k = (int)(wid - (long long)b * n);
  const int cy = k / wc, cx = k - cy * wc;
  const long long pix = ((long long)b * H + cy * G + lane / G) * W + cx * G + lane % G;
  const float v = kp[pix];
  float mx = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, pf_shfl_xor(mx, o, 64));
  const float e = expf(v - mx);
  const float sm = e / pf_wave_sum(e);
  const int p = prop[wid];
  const float lv = pf_shfl(v, p, 64);
  const float sg = 1.f / (1.f + expf(-lv));
  const float dacc = acc[wid] ? 1.f - sg : -sg;
  const float gg = g[wid];
  dkp[pix] = gg * ((lane == p ? 1.f + dacc : 0.f) - sm);
}

// out[0] = loss, out[1] = reinforce, out[2] = kp_penalty, out[3] = n_kps
__global__ __launch_bounds__(1024) void disk_final_kernel(const double* __restrict__ part,
                                                          int nparts, const uint8_t* acc1,
                                                          const uint8_t* acc2, const float* logp1,
                                                          const float* logp2, int nb, int n1,
                                                          int n2, float kp_penalty,
                                                          float* __restrict__ out) {
  __shared__ double r1[1024], r2[1024], r3[1024];
  double s = 0.0, lp = 0.0, nk = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += part[i];
  // branch-free (logp loaded whatever the flag, a rejected point adds 0.0):
  // one workgroup walks every point, so the loads of consecutive iterations
  // must not wait on each other's flags
  for (int i = threadIdx.x; i < nb * n1; i += blockDim.x) {
    const bool a = acc1[i] != 0;
    const double v = logp1[i];
    lp += a ? v : 0.0;
    nk += a ? 1.0 : 0.0;
  }
  for (int i = threadIdx.x; i < nb * n2; i += blockDim.x) {
    const bool a = acc2[i] != 0;
    const double v = logp2[i];
    lp += a ? v : 0.0;
    nk += a ? 1.0 : 0.0;
  }
  r1[threadIdx.x] = s;
  r2[threadIdx.x] = lp;
  r3[threadIdx.x] = nk;
  pf_syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
      r3[threadIdx.x] += r3[threadIdx.x + o];
    }
    pf_syncthreads();
  }
  if (threadIdx.x == 0) {
    const double reinforce = r1[0], pen = (double)kp_penalty * r2[0];
    out[0] = (float)(-reinforce - pen);
    out[1] = (float)reinforce;
    out[2] = (float)pen;
    out[3] = (float)(r3[0] / nb);
  }
}

// ---------------------------------------------------------------- flash path
constexpr int FD = 128;     // descriptor dimension
constexpr int FCOLS = 128;  // columns (B points) per block: 4 waves x 32
constexpr int FSTEP = 64;   // A rows per LDS step

struct FlashSide {          // per-point data of one side (1: image 1, 2: image 2)
  const float* f;           // [b][n][128] L2-normalised descriptors
  const int32_t* idx;       // SUM: [b][n] compacted accepted point ids, else null
  const int32_t* cnt;       // SUM: [b] accepted count
  const float* lse;         // SUM: [b][n] lse of this side (lse_r for 1, lse_c for 2)
  const float* line;        // SUM: [b][n][3] normalised epipolar line of each point
  const float* cpx;         // SUM: [b][n][2] pixel coordinates
  const float* logp;        // SUM: [b][n] point log-probability
  const unsigned short* pl = nullptr;  // BF6: [b][3][n][128] bf16 planes of f (flash_split_kernel)
  const float* meta = nullptr;         // BF6 SUM: [b][n][8] lse, line(3), cpx(2), logp, 0
};

struct FlashArgs {
  FlashSide A, B;
  int n, rows_per_split;
  float T, thr, good, bad;
  float2* lse_part;         // LSE: [b][split][n] (max, sum)
  float* g_part;            // SUM: [b][split][n] sum reward p
  double* r_part;           // SUM (want_r): [b][split][n] sum reward p (logp terms)
};

template <bool SUM>
__global__ __launch_bounds__(256) void disk_flash_kernel(FlashArgs a, int want_r) {
  __shared__ __attribute__((aligned(16))) float As[2 * FSTEP * FD];  // 2 x 32 KB
  __shared__ float meta[2][FSTEP][8];  // SUM: lse, line(3), cpx(2), logp per A row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int b = blockIdx.z, split = blockIdx.y;
  const int ncolB = SUM ? a.B.cnt[b] : a.n;
  const int nrowA = SUM ? a.A.cnt[b] : a.n;
  const int cbase = blockIdx.x * FCOLS;
  const int r0 = split * a.rows_per_split;
  const int r1 = min(nrowA, r0 + a.rows_per_split);
  const long long pb = (long long)b * a.n;
  if (cbase >= ncolB) return;  // block-uniform: nothing to do (accepted subsets)
  const int cl = cbase + wave * 32 + (lane & 31);
  const bool cok = cl < ncolB;
  const int cpt = SUM ? a.B.idx[pb + min(cl, ncolB - 1)] : min(cl, ncolB - 1);  // point id
  f32x4 breg[FD / 8];
  {
    const float* brow = a.B.f + (pb + cpt) * FD;
#pragma unroll
    for (int g = 0; g < FD / 8; ++g) breg[g] = *reinterpret_cast<const f32x4*>(brow + 8 * g + 4 * h);
  }
  float bl = 0.f, bl0 = 0.f, bl1 = 0.f, bl2 = 0.f, bx = 0.f, by = 0.f, blp = 0.f;
  if (SUM) {
    bl = a.B.lse[pb + cpt];
    bl0 = a.B.line[(pb + cpt) * 3];
    bl1 = a.B.line[(pb + cpt) * 3 + 1];
    bl2 = a.B.line[(pb + cpt) * 3 + 2];
    bx = a.B.cpx[(pb + cpt) * 2];
    by = a.B.cpx[(pb + cpt) * 2 + 1];
    blp = a.B.logp[pb + cpt];
  }
  const int nsteps = r1 > r0 ? (r1 - r0 + FSTEP - 1) / FSTEP : 0;
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int t = 0; t < FSTEP / 8; ++t) {
      const int lr = (wave * (FSTEP / 8) + t) * 2 + h;
      const int row = min(r0 + s * FSTEP + lr, r1 - 1);
      const int pt = SUM ? a.A.idx[pb + row] : row;
      const int slot = (lane & 31) ^ (lr & 15);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(a.A.f + (pb + pt) * FD + slot * 4),
          (__attribute__((address_space(3))) void*)(As + buf * FSTEP * FD +
                                                     (wave * (FSTEP / 8) + t) * 2 * FD),
          16, 0, 0);
    }
    if (SUM && tid < FSTEP) {  // row metadata (plain loads; consumed after the barrier)
      const int row = min(r0 + s * FSTEP + tid, r1 - 1);
      const long long q = pb + a.A.idx[pb + row];
      float* mm = meta[buf][tid];
      mm[0] = a.A.lse[q];
      mm[1] = a.A.line[q * 3];
      mm[2] = a.A.line[q * 3 + 1];
      mm[3] = a.A.line[q * 3 + 2];
      mm[4] = a.A.cpx[q * 2];
      mm[5] = a.A.cpx[q * 2 + 1];
      mm[6] = a.A.logp[q];
    }
  };
  float run_m = -INFINITY, run_s = 0.f;  // LSE: running max / sum of exp
  float gs = 0.f;                        // SUM: sum reward p
  double rs = 0.0;                       // SUM: sum reward p (logp terms)
  if (nsteps > 0) issue(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  pf_syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) issue(s + 1, cur ^ 1);
    const float* Ab = As + cur * FSTEP * FD;
    // both 32-row blocks at once: two independent accumulation chains per B
    // fragment (the MFMA pipe never waits on one chain's ds_read)
    f32x16 accs[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) accs[0][r] = accs[1][r] = 0.f;
    {
      const int la = lane & 31;  // rows la and 32 + la share the swizzle (la & 15)
      const float* arow0 = Ab + la * FD;
      const float* arow1 = Ab + (32 + la) * FD;
#pragma unroll
      for (int g = 0; g < FD / 8; ++g) {
        const int off = ((2 * g + h) ^ (la & 15)) * 4;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(arow0 + off);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(arow1 + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          accs[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[j], breg[g][j], accs[0], 0, 0, 0);
          accs[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[j], breg[g][j], accs[1], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const f32x16& acc = accs[mi];
      // acc[r] = S(A row, B column cl) for A row r0 + s*64 + mi*32 + (r&3) + 8(r>>2) + 4h
      const int rb = s * FSTEP + mi * 32 + 4 * h;
      if (!SUM) {
        float smax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (r0 + rb + (r & 3) + 8 * (r >> 2) < r1) smax = fmaxf(smax, a.T * acc[r] - a.T);
        if (smax > -INFINITY) {
          const float nm = fmaxf(run_m, smax);
          float add = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (r0 + rb + (r & 3) + 8 * (r >> 2) < r1) add += expf((a.T * acc[r] - a.T) - nm);
          run_s = run_s * expf(run_m - nm) + add;
          run_m = nm;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int lr = rb - s * FSTEP + (r & 3) + 8 * (r >> 2);  // row within the step
          if (r0 + s * FSTEP + lr >= r1) continue;
          const float* mm = meta[cur][lr];
          const float aff = a.T * acc[r] - a.T;
          const float lpa = aff - mm[0], lpb = aff - bl;
          const float p = expf(lpa) * expf(lpb);
          const float dA = fabsf(mm[1] * bx + mm[2] * by + mm[3]);  // A's line at B's point
          const float dB = fabsf(bl0 * mm[4] + bl1 * mm[5] + bl2);  // B's line at A's point
          const float rp = ((dA < a.thr && dB < a.thr) ? a.good : a.bad) * p;
          gs += rp;
          if (want_r) rs += (double)(rp * ((lpa + lpb) + (mm[6] + blp)));
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    pf_syncthreads();
  }
  // merge the two lane halves (interleaved row sets) in a fixed order
  const long long o = ((long long)b * gridDim.y + split) * a.n + cl;
  if (!SUM) {
    const float om = pf_shfl_xor(run_m, 32, 64), os = pf_shfl_xor(run_s, 32, 64);
    if (h == 0 && cok) {
      const float M = fmaxf(run_m, om);
      const float t = (M == -INFINITY) ? 0.f : run_s * expf(run_m - M) + os * expf(om - M);
      a.lse_part[o] = make_float2(M, t);
    }
  } else {
    const float og = pf_shfl_xor(gs, 32, 64);
    const double orr = pf_shfl_xor(rs, 32, 64);
    if (h == 0 && cok) {
      a.g_part[o] = gs + og;
      if (want_r) a.r_part[o] = rs + orr;
    }
  }
}

// the refilled ring slot and the multiplied one as __restrict__ parameters of
// one body, so the waitcnt pass does not order the stage's LDS reads behind
// the younger DMA (conv.hip pf_dma_overlap_step)
template <class F>
__device__ __forceinline__ void flash6_step(unsigned short* __restrict__ d,
                                            const unsigned short* __restrict__ s,
                                            const unsigned short* __restrict__ sp, F&& body) {
  body(d, s, sp);
}

// vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 s_waitcnt encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// The flash passes with the similarity products in bf16x6 on
// v_mfma_f32_32x32x16_bf16 (six bf16 products per fp32 product, fp32-exact
// per product: common.h split3).  Both sides arrive as three bf16 planes,
// split once per loss (flash_split_kernel); the SUM passes' sides arrive
// compacted to their accepted points in order, planes and per-point metadata
// (flash_gather_kernel), so every A row of a step is a contiguous DMA and
// nothing in the loop waits on an index load.  B's column (this lane's 128 k)
// sits in registers; A's rows stream in 32-row stages (3 planes x 8 KB, plus
// 1 KB of metadata for SUM) through a three-slot LDS ring: stages i+1 and
// i+2 are in flight while stage i is multiplied.  LSE is software-pipelined:
// step i multiplies stage i into one accumulator while the VALU epilogue of
// stage i-1 (online logsumexp) is threaded through its dependent MFMA chain
// (mma_lse), so the matrix pipe and the VALU overlap inside each wave.  Only a split's
// last stage can hold rows past its end: its epilogue, after the loop, is the
// one with per-row checks.  75 KB of LDS: two workgroups per CU.  Row /
// column semantics as disk_flash_kernel; WR: the SUM pass also sums the
// reinforce terms (fp64).
constexpr int F6STEP = 32;  // A rows per stage
constexpr int F6NST = 3;    // LDS slots

template <bool SUM, bool WR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void disk_flash6_kernel(FlashArgs a) {
  // a stage: 3 planes x 32 rows x 256 B, then (SUM) 32 rows x 32 B of metadata --
  // one array, so the DMAs into a slot and the reads of others go through the
  // same pair of __restrict__ pointers (flash6_step)
  constexpr int PLANES = 3 * F6STEP * FD;                  // bf16 per stage's planes (24 KB)
  constexpr int PSTAGE = PLANES + (SUM ? F6STEP * 16 : 0);  // + metadata (1 KB as bf16 units)
  __shared__ __attribute__((aligned(16))) unsigned short Ps[F6NST * PSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, la = lane & 31;
  const int b = blockIdx.z, split = blockIdx.y;
  const int ncolB = SUM ? a.B.cnt[b] : a.n;
  const int nrowA = SUM ? a.A.cnt[b] : a.n;
  const int cbase = blockIdx.x * FCOLS;
  const int r0 = split * a.rows_per_split;
  const int r1 = min(nrowA, r0 + a.rows_per_split);
  const long long pb = (long long)b * a.n;
  if (cbase >= ncolB) return;  // block-uniform
  const int cl = cbase + wave * 32 + la;
  const bool cok = cl < ncolB;
  const int cpt = min(cl, ncolB - 1);  // SUM: compacted column
  g6_u32x4 bpl[FD / 16][3];            // per k16 group the h, m, l operands of column cpt
  f32x4 bm0 = {0.f, 0.f, 0.f, 0.f}, bm1 = {0.f, 0.f, 0.f, 0.f};  // SUM: column metadata
  const int nsteps = r1 > r0 ? (r1 - r0 + F6STEP - 1) / F6STEP : 0;
  const int rlast = max(r1 - 1, 0);  // rows clamp here
  // stage s into slot d: 24 wave DMAs of 4 plane rows (6 per wave); LDS row lr
  // holds its 16-B chunk c at slot c ^ (lr & 15).  SUM: each wave also moves 8
  // rows of metadata (64 lanes x 4 B).
  auto issue = [&](int s, unsigned short* d) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const int q = wave * 6 + t, pln = q >> 3, lr = (q & 7) * 4 + (lane >> 4);
      const int row = min(r0 + s * F6STEP + lr, rlast);
      const int slot = (lane & 15) ^ (lr & 15);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(a.A.pl + (3 * pb + (long long)pln * a.n +
                                                                    row) * FD + slot * 8),
          (__attribute__((address_space(3))) void*)(d + (pln * F6STEP + (q & 7) * 4) * FD), 16, 0,
          0);
    }
    if (SUM) {  // no divergent branch around the DMA
      const int row = min(r0 + s * F6STEP + wave * 8 + (lane >> 3), rlast);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(a.A.meta + (pb + row) * 8 + (lane & 7)),
          (__attribute__((address_space(3))) void*)(d + PLANES + wave * 8 * 16), 4, 0, 0);
    }
  };
  const float c2 = a.T * 1.4426950408889634f;  // T log2(e)
  float t2 = 0.f, k2 = 0.f;  // SUM: 2 T log2(e), (-2 T - lse_B) log2(e) (set with B's metadata)
  // the two rewards held in VGPRs once (as kernel arguments they were moved
  // from SGPRs into VGPRs for every element's select)
  float vgood = a.good, vbad = a.bad;
  asm volatile("" : "+v"(vgood), "+v"(vbad));
  float run_m = -INFINITY, run_s = 0.f;  // LSE: running max (base 2) / sum of exp
  float gs = 0.f;                        // SUM: sum reward p
  double rs = 0.0;                       // SUM (WR): sum reward p (logp terms)
  // stage s's 32x32 similarity tile from slot L: k16 group g, lane (row la,
  // half h) supplies k = 16 g + 8 h .. + 7 = chunk 2 g + h of its row per plane
  auto mma = [&](const unsigned short* L, f32x16& acc) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int g = 0; g < FD / 16; ++g) {
      const int off = la * FD + (((2 * g + h) ^ (la & 15)) * 8);
      const g6_u32x4 ah = *reinterpret_cast<const g6_u32x4*>(L + off);
      const g6_u32x4 am = *reinterpret_cast<const g6_u32x4*>(L + F6STEP * FD + off);
      const g6_u32x4 al = *reinterpret_cast<const g6_u32x4*>(L + 2 * F6STEP * FD + off);
      acc = g6_mfma(ah, bpl[g][0], acc);
      acc = g6_mfma(ah, bpl[g][1], acc);
      acc = g6_mfma(am, bpl[g][0], acc);
      acc = g6_mfma(ah, bpl[g][2], acc);
      acc = g6_mfma(al, bpl[g][0], acc);
      acc = g6_mfma(am, bpl[g][1], acc);
    }
  };
  // LSE: the same tile with the previous stage's online-logsumexp epilogue
  // (prev, FULL) threaded through the dependent MFMA chain by hand: fill(j)
  // after the j-th MFMA, each slice at most an fma, a v_exp_f32 and an add
  // (within the ~24 cycles an MFMA gap hides), a sched_barrier after each so
  // the scheduler cannot cluster them again; the next k16 group's operands are
  // read one group ahead
  auto mma_lse = [&](const unsigned short* L, f32x16& acc, const f32x16& prev)
      __attribute__((always_inline)) {
    float sm = -INFINITY, nm = 0.f, nmc = 0.f, off = 0.f, scale = 0.f;
    float ad[4] = {0.f, 0.f, 0.f, 0.f};
    auto fill = [&](int j) __attribute__((always_inline)) {
      if (j < 8) {
        sm = fmaxf(sm, fmaxf(prev[2 * j], prev[2 * j + 1]));
      } else if (j == 8) {
        nm = fmaxf(run_m, c2 * sm - c2);
        nmc = nm == -INFINITY ? 0.f : nm;
        off = -c2 - nmc;
      } else if (j == 9) {
        scale = __builtin_amdgcn_exp2f(run_m - nmc);
      } else if (j < 26) {
        const int r = j - 10;
        ad[r & 3] += __builtin_amdgcn_exp2f(fmaf(c2, prev[r], off));
      } else if (j == 26) {
        run_s = run_s * scale + ((ad[0] + ad[1]) + (ad[2] + ad[3]));
        run_m = nm;
      }
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    g6_u32x4 op[2][3];
    auto ld = [&](int g, g6_u32x4* d) __attribute__((always_inline)) {
      const int o = la * FD + (((2 * g + h) ^ (la & 15)) * 8);
      d[0] = *reinterpret_cast<const g6_u32x4*>(L + o);
      d[1] = *reinterpret_cast<const g6_u32x4*>(L + F6STEP * FD + o);
      d[2] = *reinterpret_cast<const g6_u32x4*>(L + 2 * F6STEP * FD + o);
    };
    ld(0, op[0]);
#pragma unroll
    for (int g = 0; g < FD / 16; ++g) {
      if (g + 1 < FD / 16) ld(g + 1, op[(g + 1) & 1]);
      const g6_u32x4* A = op[g & 1];
      const int pa[6] = {0, 0, 1, 0, 2, 1}, pb[6] = {0, 1, 0, 2, 0, 1};  // hh hm mh hl lh mm
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        acc = g6_mfma(A[pa[k]], bpl[g][pb[k]], acc);
        fill(6 * g + k);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // acc[r] = S(A row r0 + s*32 + (r&3) + 8(r>>2) + 4h, B column cl); M: the
  // stage's metadata (SUM).  FULL: every row of the stage exists.
  auto epilogue = [&](auto full_t, int s, const f32x16& acc, const float* M)
      __attribute__((always_inline)) {
    constexpr bool FULL = decltype(full_t)::value;
    const int rb = r0 + s * F6STEP + 4 * h;
    auto valid = [&](int r) { return FULL || rb + (r & 3) + 8 * (r >> 2) < r1; };
    if (!SUM) {
      // base-2 online logsumexp of x = T (s - 1): x log2(e) = c2 s - c2; the
      // max over the raw similarities (c2 > 0); one fma + v_exp_f32 per
      // element, four partial sums.  Branch-free: a stage with no valid row
      // (sm = -inf) adds exp2(-inf) = 0 and rescales by exp2(-inf - 0) = 0.
      float sm = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (valid(r)) sm = fmaxf(sm, acc[r]);
      const float nm = fmaxf(run_m, c2 * sm - c2);
      const float nmc = nm == -INFINITY ? 0.f : nm;
      const float off = -c2 - nmc;
      float ad[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (valid(r)) ad[r & 3] += __builtin_amdgcn_exp2f(fmaf(c2, acc[r], off));
      run_s = run_s * __builtin_amdgcn_exp2f(run_m - nmc) + ((ad[0] + ad[1]) + (ad[2] + ad[3]));
      run_m = nm;
    } else {
      // log2 p = 2 T log2(e) s + (-2 T - lse_A - lse_B) log2(e): one sub (the
      // column's part is a lane constant, the row's is metadata [7]), one fma,
      // one v_exp_f32 -- the round-4 form took 2 subs, an add, an fma and a mul;
      // the two line tests as one max of their magnitudes (the SUM passes
      // were VALU-bound, 8.8-13 k VALU per 1.1 k MFMA per wave)
      float gp[2] = {0.f, 0.f};
      // WR: the stage's 16 reinforce terms summed in fp32 (two interleaved
      // partials), then added to the fp64 total once per stage (a cvt and an
      // fp64 add per element made the WR pass the slowest, r14a: 302 vs 252 us)
      float rp2[2] = {0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (!valid(r)) continue;
        const int lr = 4 * h + (r & 3) + 8 * (r >> 2);  // row within the stage
        const f32x4 m0 = *reinterpret_cast<const f32x4*>(M + lr * 8);
        const f32x4 m1 = *reinterpret_cast<const f32x4*>(M + lr * 8 + 4);
        const float lp2 = fmaf(t2, acc[r], k2 - m1[3]);  // log2 p
        const float p = __builtin_amdgcn_exp2f(lp2);
        const float dA = fmaf(m0[1], bm1[0], fmaf(m0[2], bm1[1], m0[3]));    // A's line at B's pt
        const float dB = fmaf(bm0[1], m1[0], fmaf(bm0[2], m1[1], bm0[3]));  // B's line at A's pt
        const float rp = (fmaxf(fabsf(dA), fabsf(dB)) < a.thr ? vgood : vbad) * p;
        gp[r & 1] += rp;
        if (WR) rp2[r & 1] = fmaf(rp, lp2 * 0.6931471805599453f + (m1[2] + bm1[2]), rp2[r & 1]);
      }
      gs += gp[0] + gp[1];
      if (WR) rs += (double)rp2[0] + (double)rp2[1];
    }
  };
  // prologue: stage 0, then B's column (waited for explicitly: the waitcnt
  // pass could not prove the counted waits retire it and put a vmcnt(0) in
  // front of every step's first MFMA)
  if (nsteps > 0) issue(0, Ps);
  {
    const unsigned short* bp = a.B.pl + (3 * pb + cpt) * FD;
#pragma unroll
    for (int g = 0; g < FD / 16; ++g)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bpl[g][q] = *reinterpret_cast<const g6_u32x4*>(bp + (long long)q * a.n * FD + 16 * g + 8 * h);
  }
  if (SUM) {
    bm0 = *reinterpret_cast<const f32x4*>(a.B.meta + (pb + cpt) * 8);
    bm1 = *reinterpret_cast<const f32x4*>(a.B.meta + (pb + cpt) * 8 + 4);
    t2 = 2.f * c2;
    k2 = -t2 - bm1[3];
  }
  // LSE: stage i's MFMAs and stage i-1's epilogue in one block (no branch
  // between them), free to interleave.  SUM: each stage's epilogue right after
  // its MFMAs (pipelined, its sixteen rows of metadata pushed the registers
  // past two waves per SIMD).
  // (two accumulators, named statically: the loop below is unrolled by two)
  f32x16 acc0, acc1;
  auto work = [&](int i, const unsigned short* L, f32x16& cur, const f32x16& prev)
      __attribute__((always_inline)) {
    if constexpr (SUM) {
      mma(L, cur);
      const float* M = reinterpret_cast<const float*>(L + PLANES);
      if (!WR && i + 1 < nsteps)  // WR: the checked form (its fp64 sums need the registers)
        epilogue(std::true_type{}, i, cur, M);
      else
        epilogue(std::false_type{}, i, cur, M);
    } else {
      mma_lse(L, cur, prev);  // + stage i-1's epilogue (i >= 1 here)
    }
  };
  wait_vmcnt<0>();  // B's column and stage 0
  if (nsteps > 1) issue(1, Ps + PSTAGE);
  __builtin_amdgcn_s_barrier();
  // step i: stages i+1 (issued a step earlier) and i+2 (issued now, into the
  // slot of stage i-1, whose reads all finished before this step's barrier)
  // stay in flight while stage i is multiplied
  if (nsteps > 0)  // step 0 (LSE: no epilogue yet)
    flash6_step(Ps + 2 * PSTAGE, Ps, Ps + PSTAGE,
                [&](unsigned short* d, const unsigned short* L, const unsigned short*) {
                  if (nsteps > 2) issue(2, d);
                  if constexpr (SUM)
                    work(0, L, acc0, acc1);
                  else
                    mma(L, acc0);
                });
  int slot = 1;  // stage i's slot; i-1's (= i+2's) is slot - 1 (mod 3)
  auto step = [&](int i, f32x16& cur, const f32x16& prev) __attribute__((always_inline)) {
    if (i + 1 < nsteps)
      wait_vmcnt<SUM ? 7 : 6>();  // stage i landed, stage i+1 may stay in flight
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's part of stage i; stage i-1's slot free
    const int nxt = slot == F6NST - 1 ? 0 : slot + 1, prv = slot == 0 ? F6NST - 1 : slot - 1;
    flash6_step(Ps + prv * PSTAGE, Ps + slot * PSTAGE, Ps + nxt * PSTAGE,
                [&](unsigned short* d, const unsigned short* L, const unsigned short*) {
                  if (i + 2 < nsteps) issue(i + 2, d);
                  work(i, L, cur, prev);
                });
    slot = nxt;
  };
  for (int i = 1; i < nsteps; i += 2) {  // odd steps into acc1, even into acc0
    step(i, acc1, acc0);
    if (i + 1 < nsteps) step(i + 1, acc0, acc1);
  }
  if (!SUM && nsteps > 0)
    epilogue(std::false_type{}, nsteps - 1, (nsteps - 1) & 1 ? acc1 : acc0, nullptr);
  // merge the two lane halves (interleaved row sets) in a fixed order; the
  // partial's max back in natural units
  const long long o = ((long long)b * gridDim.y + split) * a.n + cl;
  if (!SUM) {
    const float om = pf_shfl_xor(run_m, 32, 64), os = pf_shfl_xor(run_s, 32, 64);
    if (h == 0 && cok) {
      const float M = fmaxf(run_m, om);
      const float t = (M == -INFINITY) ? 0.f
                                       : run_s * __builtin_amdgcn_exp2f(run_m - M) +
                                             os * __builtin_amdgcn_exp2f(om - M);
      a.lse_part[o] = make_float2(M * 0.6931471805599453f, t);
    }
  } else {
    const float og = pf_shfl_xor(gs, 32, 64);
    const double orr = pf_shfl_xor(rs, 32, 64);
    if (h == 0 && cok) {
      a.g_part[o] = gs + og;
      if (WR) a.r_part[o] = rs + orr;
    }
  }
}

// SUM passes' side data in accepted order (flash_compact_kernel's ids): row i
// < cnt[b] of cpl / cmeta = planes / metadata of point idx[b][i]
__global__ void flash_gather_kernel(const unsigned short* __restrict__ pl, FlashSide s, int nb,
                                    int n, unsigned short* __restrict__ cpl,
                                    float* __restrict__ cmeta) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;  // (b, i, chunk)
  if (t >= (long long)nb * n * (FD / 8)) return;
  const long long r = t / (FD / 8);
  const int c = (int)(t - r * (FD / 8));
  const int bb = (int)(r / n), i = (int)(r - (long long)bb * n);
  if (i >= s.cnt[bb]) return;
  const long long pb = (long long)bb * n, src = s.idx[pb + i];
#pragma unroll
  for (int q = 0; q < 3; ++q)
    *reinterpret_cast<g6_u32x4*>(cpl + (3 * pb + (long long)q * n + i) * FD + c * 8) =
        *reinterpret_cast<const g6_u32x4*>(pl + (3 * pb + (long long)q * n + src) * FD + c * 8);
  if (c == 0) {
    const long long p = pb + src;
    float* m = cmeta + (pb + i) * 8;
    *reinterpret_cast<f32x4*>(m) = f32x4{s.lse[p], s.line[p * 3], s.line[p * 3 + 1], s.line[p * 3 + 2]};
    // [7]: lse in base 2, the SUM epilogue's per-row term (disk_flash6_kernel)
    *reinterpret_cast<f32x4*>(m + 4) =
        f32x4{s.cpx[p * 2], s.cpx[p * 2 + 1], s.logp[p], s.lse[p] * 1.4426950408889634f};
  }
}

// the three bf16 planes of L2-normalised descriptors for the BF6 flash passes:
// pl[b][q][n][128] = plane q (h, m, l of common.h g6_split) of f[b][n][128];
// one thread per 8 values
__global__ void flash_split_kernel(const float* __restrict__ f, long long rows, int n,
                                   unsigned short* __restrict__ pl) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= rows * (FD / 8)) return;
  const long long r = i / (FD / 8), bb = r / n, pr = r - bb * n;
  const int c = (int)(i - r * (FD / 8));
  g6_u32x4 hp, mp, lp;
  g6_split(*reinterpret_cast<const f32x4*>(f + r * FD + c * 8),
           *reinterpret_cast<const f32x4*>(f + r * FD + c * 8 + 4), hp, mp, lp);
  unsigned short* o = pl + (3 * bb * n + pr) * FD + c * 8;
  *reinterpret_cast<g6_u32x4*>(o) = hp;
  *reinterpret_cast<g6_u32x4*>(o + (long long)n * FD) = mp;
  *reinterpret_cast<g6_u32x4*>(o + 2LL * n * FD) = lp;
}

// lse[b][p] = merge of the split (max, sum) partials in split order
__global__ void flash_lse_final_kernel(const float2* __restrict__ part, int nb, int ns, int n,
                                       float* __restrict__ lse) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nb * n) return;
  const int b = (int)(i / n), c = (int)(i - (long long)b * n);
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, part[((long long)b * ns + s) * n + c].x);
  float t = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float2 q = part[((long long)b * ns + s) * n + c];
    if (q.y > 0.f) t += q.y * expf(q.x - M);
  }
  lse[i] = M + logf(t);
}

// stable compaction of the accepted points of each image (one block per image)
__global__ __launch_bounds__(1024) void flash_compact_kernel(const uint8_t* __restrict__ acc,
                                                             int n, int32_t* __restrict__ idx,
                                                             int32_t* __restrict__ cnt) {
  __shared__ int off[1024];
  const int b = blockIdx.x, t = threadIdx.x, per = (n + 1023) / 1024;
  const uint8_t* ab = acc + (long long)b * n;
  const int i0 = min(n, t * per), i1 = min(n, i0 + per);
  int c = 0;
  for (int i = i0; i < i1; ++i) c += ab[i] ? 1 : 0;
  off[t] = c;
  pf_syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int v = t >= d ? off[t - d] : 0;
    pf_syncthreads();
    off[t] += v;
    pf_syncthreads();
  }
  int o = off[t] - c;
  for (int i = i0; i < i1; ++i)
    if (ab[i]) idx[(long long)b * n + o++] = i;
  if (t == 1023) cnt[b] = off[1023];
}

// per point of one side: dL/dlogp (accepted: -sum_s g_part - penalty; else 0)
// and, for the side whose SUM pass ran with want_r, the reinforce partial of
// each accepted column (sum over splits in order) -> rcol
__global__ void flash_sum_final_kernel(const float* __restrict__ gpart,
                                       const double* __restrict__ rpart, int nb, int ns, int n,
                                       const int32_t* __restrict__ idx,
                                       const int32_t* __restrict__ cnt, float kp_penalty,
                                       float* __restrict__ g, double* __restrict__ rcol) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)nb * n) return;
  const int b = (int)(i / n), c = (int)(i - (long long)b * n);
  if (rcol) rcol[i] = 0.0;
  if (c >= cnt[b]) return;
  float t = 0.f;
  double r = 0.0;
  for (int s = 0; s < ns; ++s) {
    t += gpart[((long long)b * ns + s) * n + c];
    if (rpart) r += rpart[((long long)b * ns + s) * n + c];
  }
  const long long pt = (long long)b * n + idx[(long long)b * n + c];
  if (g) g[pt] = -t - kp_penalty;
  if (rcol) rcol[i] = r;
}

// zero dL/dlogp of the rejected points (the accepted ones are written above)
__global__ void flash_grad_init_kernel(const uint8_t* __restrict__ acc, long long total,
                                       float* __restrict__ g) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i < total && !acc[i]) g[i] = 0.f;
}

// A-row split: fill whole rounds of the 512 resident workgroups (2 per CU)
// -- the fraction of the last round left idle is the tail loss -- with at
// least two 64-row steps per split
int flash_nsplit(int n, int nb) {
  const int ncb = (n + FCOLS - 1) / FCOLS;
  const int smax = std::max(1, std::min(32, n / (2 * FSTEP)));
  int best = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= smax; ++s) {
    const double r = (double)ncb * nb * s / 512.0;
    const double eff = r / std::ceil(r) * (r < 1.0 ? r : 1.0);
    if (eff >= 0.94) return s;  // the fewest splits that keep the tail small
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

// read per call (a few getenv per loss) so tests can A/B both paths in-process
// the flash passes' product arithmetic follows the conv precision mode
// (posfeat_set_conv_precision: >= 1 bf16x6, the default; 0 fp32 MFMA)
bool flash_bf6() { return pf_conv_precision() >= 1; }

// planes of f [b][n][128] into pl (flash_bf6() only; pl has b * n * 768 bytes)
void flash_split(const float* f, int b, int n, unsigned short* pl, hipStream_t st) {
  const long long t = (long long)b * n * (FD / 8);
  hipLaunchKernelGGL(flash_split_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, f,
                     (long long)b * n, n, pl);
}

template <bool SUM>
void launch_flash(dim3 grid, hipStream_t st, const FlashArgs& fa, int want_r) {
  if (!flash_bf6())
    hipLaunchKernelGGL(disk_flash_kernel<SUM>, grid, dim3(256), 0, st, fa, want_r);
  else if (SUM && want_r)
    hipLaunchKernelGGL((disk_flash6_kernel<true, true>), grid, dim3(256), 0, st, fa);
  else
    hipLaunchKernelGGL((disk_flash6_kernel<SUM, false>), grid, dim3(256), 0, st, fa);
}

bool use_flash() {
  const char* e = pf_ab_getenv("POSFEAT_DISK_FLASH");
  return !(e && e[0] == '0');
}

}  // namespace

static size_t disk_common_bytes(size_t b, size_t n) {
  size_t s = 0;
  s += 2 * pf_align(b * n * 2 * 4, 256);          // cpx1/2
  s += 2 * pf_align(b * n * 2 * 4, 256);          // cn1/2
  s += 2 * pf_align(b * n * 4, 256);              // logp1/2
  s += 2 * pf_align(b * n * 4, 256);              // prop1/2
  s += 2 * pf_align(b * n, 256);                  // acc1/2
  s += 2 * pf_align(b * n * 128 * 4, 256);        // f1/f2
  s += 2 * pf_align(b * n * 4, 256);              // lse_r, lse_c
  s += 2 * pf_align(b * n * 3 * 4, 256);          // lines
  return s;
}

static size_t disk_flash_bytes(size_t b, size_t n) {  // flash path scratch after the common part
  const size_t ns = (size_t)flash_nsplit((int)n, (int)b);
  return pf_align(b * ns * n * 8, 256) +            // LSE partials (max, sum)
         pf_align(b * ns * n * 4, 256) +            // reward p partials
         pf_align(b * ns * n * 8, 256) +            // reinforce partials (fp64)
         2 * pf_align(b * n * 4, 256) +             // compacted ids
         pf_align(2 * b * 4, 256) +                 // counts
         pf_align(b * n * 8, 256) +                 // reinforce per column (fp64)
         4 * pf_align(b * n * FD * 6, 256) +        // bf16x6 planes of f1 / f2, compacted
         2 * pf_align(b * n * 32, 256);             // compacted per-point metadata
}

static size_t disk_dense_bytes(size_t b, size_t n) {  // S-materialising path
  return pf_align(b * n * n * 4, 256) + pf_align(b * ((n + 3) / 4) * 8, 256) +
         pf_align(b * COL_CH * n * 8, 256);
}

extern "C" size_t posfeat_disk_loss_workspace(int b, int H, int W) {
  if (b <= 0 || H % 8 || W % 8) return 0;
  const size_t n = (size_t)(H / 8) * (W / 8);
  return disk_common_bytes(b, n) + (use_flash() ? disk_flash_bytes(b, n) : disk_dense_bytes(b, n));
}

extern "C" size_t posfeat_disk_loss_grad_workspace(int b, int H, int W) {
  if (b <= 0 || H % 8 || W % 8) return 0;
  const size_t n = (size_t)(H / 8) * (W / 8);
  return posfeat_disk_loss_workspace(b, H, W) + 2 * pf_align(b * n * 4, 256) +
         (use_flash() ? 0 : pf_align(b * COL_CH * n * 4, 256));
}

static int disk_loss_impl(const float* kp1, const float* kp2, const float* xf1, int cs1,
                          const float* xf2, int cs2, int b, int H, int W, const float* F1,
                          const float* F2, const int32_t* prop1, const int32_t* prop2,
                          const uint8_t* acc1, const uint8_t* acc2, const float* uni1,
                          const float* uni2, float temperature, float reward_thr,
                          float good_reward, float bad_reward, float kp_penalty, float* out,
                          float* dkp1, float* dkp2, void* ws, size_t ws_bytes, void* stream) {
  if (!kp1 || !kp2 || !xf1 || !xf2 || !F1 || !F2 || !out || !ws) return POSFEAT_E_INVALID;
  if (b <= 0 || H % 8 || W % 8 || H % 4 || cs1 < 128 || cs2 < 128) return POSFEAT_E_INVALID;
  const bool sampled = uni1 && uni2;
  const bool grad = dkp1 && dkp2;
  if (!sampled && !(prop1 && prop2 && acc1 && acc2)) return POSFEAT_E_INVALID;
  if (ws_bytes < (grad ? posfeat_disk_loss_grad_workspace(b, H, W)
                       : posfeat_disk_loss_workspace(b, H, W)))
    return POSFEAT_E_WORKSPACE;
  const int n = (H / 8) * (W / 8);
  if (n % 4) return POSFEAT_E_UNSUPPORTED;
  hipStream_t st = pf_stream(stream);
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += pf_align(bytes, 256);
    return static_cast<void*>(r);
  };
  float* cpx1 = static_cast<float*>(take((size_t)b * n * 8));
  float* cpx2 = static_cast<float*>(take((size_t)b * n * 8));
  float* cn1 = static_cast<float*>(take((size_t)b * n * 8));
  float* cn2 = static_cast<float*>(take((size_t)b * n * 8));
  float* lp1 = static_cast<float*>(take((size_t)b * n * 4));
  float* lp2 = static_cast<float*>(take((size_t)b * n * 4));
  int32_t* pr1 = static_cast<int32_t*>(take((size_t)b * n * 4));
  int32_t* pr2 = static_cast<int32_t*>(take((size_t)b * n * 4));
  uint8_t* ac1 = static_cast<uint8_t*>(take((size_t)b * n));
  uint8_t* ac2 = static_cast<uint8_t*>(take((size_t)b * n));
  float* f1 = static_cast<float*>(take((size_t)b * n * 512));
  float* f2 = static_cast<float*>(take((size_t)b * n * 512));
  float* lr = static_cast<float*>(take((size_t)b * n * 4));
  float* lc = static_cast<float*>(take((size_t)b * n * 4));
  float* ln1 = static_cast<float*>(take((size_t)b * n * 12));
  float* ln2 = static_cast<float*>(take((size_t)b * n * 12));
  const unsigned pts_blocks = (unsigned)(((long long)b * n + 3) / 4);
  hipLaunchKernelGGL(disk_point_kernel, dim3(pts_blocks), dim3(256), 0, st, kp1, b, H, W, prop1,
                     acc1, sampled ? uni1 : nullptr, pr1, ac1, cpx1, cn1, lp1);
  hipLaunchKernelGGL(disk_point_kernel, dim3(pts_blocks), dim3(256), 0, st, kp2, b, H, W, prop2,
                     acc2, sampled ? uni2 : nullptr, pr2, ac2, cpx2, cn2, lp2);
  PF_CHECK_LAUNCH();
  PF_TRY(pf_sample_desc(xf1, b, 128, H / 4, W / 4, cs1, cn1, n, nullptr, 1, f1, st));
  PF_TRY(pf_sample_desc(xf2, b, 128, H / 4, W / 4, cs2, cn2, n, nullptr, 1, f2, st));
  hipLaunchKernelGGL(epi_line_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, F1, cpx1, b, n,
                     ln1);
  hipLaunchKernelGGL(epi_line_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, F2, cpx2, b, n,
                     ln2);
  PF_CHECK_LAUNCH();
  if (use_flash()) {
    const int ns = flash_nsplit(n, b);
    float2* lsep = static_cast<float2*>(take((size_t)b * ns * n * 8));
    float* gp = static_cast<float*>(take((size_t)b * ns * n * 4));
    double* rp = static_cast<double*>(take((size_t)b * ns * n * 8));
    int32_t* id1 = static_cast<int32_t*>(take((size_t)b * n * 4));
    int32_t* id2 = static_cast<int32_t*>(take((size_t)b * n * 4));
    int32_t* cnt = static_cast<int32_t*>(take((size_t)2 * b * 4));
    double* rcol = static_cast<double*>(take((size_t)b * n * 8));
    unsigned short* pl1 = static_cast<unsigned short*>(take((size_t)b * n * FD * 6));
    unsigned short* pl2 = static_cast<unsigned short*>(take((size_t)b * n * FD * 6));
    unsigned short* cpl1 = static_cast<unsigned short*>(take((size_t)b * n * FD * 6));
    unsigned short* cpl2 = static_cast<unsigned short*>(take((size_t)b * n * FD * 6));
    float* cm1 = static_cast<float*>(take((size_t)b * n * 32));
    float* cm2 = static_cast<float*>(take((size_t)b * n * 32));
    const bool bf6 = flash_bf6();
    if (bf6) {
      flash_split(f1, b, n, pl1, st);
      flash_split(f2, b, n, pl2, st);
    }
    const int rps = ((n + ns - 1) / ns + FSTEP - 1) / FSTEP * FSTEP;
    const dim3 fgrid((n + FCOLS - 1) / FCOLS, ns, b);
    FlashArgs fa{};
    fa.n = n;
    fa.rows_per_split = rps;
    fa.T = temperature;
    fa.thr = reward_thr;
    fa.good = good_reward;
    fa.bad = bad_reward;
    fa.lse_part = lsep;
    fa.g_part = gp;
    fa.r_part = rp;
    const FlashSide s1{f1, id1, cnt, lr, ln1, cpx1, lp1, cpl1, cm1},
        s2{f2, id2, cnt + b, lc, ln2, cpx2, lp2, cpl2, cm2};
    const FlashSide a1{f1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, pl1},
        a2{f2, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, pl2};
    // column LSE (over image-1 points) and row LSE (over image-2 points), all points
    fa.A = a1;
    fa.B = a2;
    launch_flash<false>(fgrid, st, fa, 0);
    hipLaunchKernelGGL(flash_lse_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, lsep,
                       b, ns, n, lc);
    fa.A = a2;
    fa.B = a1;
    launch_flash<false>(fgrid, st, fa, 0);
    hipLaunchKernelGGL(flash_lse_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, lsep,
                       b, ns, n, lr);
    hipLaunchKernelGGL(flash_compact_kernel, dim3(b), dim3(1024), 0, st, ac1, n, id1, cnt);
    hipLaunchKernelGGL(flash_compact_kernel, dim3(b), dim3(1024), 0, st, ac2, n, id2, cnt + b);
    if (bf6) {  // the accepted points of each side, in order, for the SUM passes
      const unsigned gb = (unsigned)(((long long)b * n * (FD / 8) + 255) / 256);
      hipLaunchKernelGGL(flash_gather_kernel, dim3(gb), dim3(256), 0, st, pl1, s1, b, n, cpl1, cm1);
      hipLaunchKernelGGL(flash_gather_kernel, dim3(gb), dim3(256), 0, st, pl2, s2, b, n, cpl2, cm2);
    }
    PF_CHECK_LAUNCH();
    // accepted pairs, columns = image-2 points: sum_m reward p and the reinforce
    float* g1 = grad ? static_cast<float*>(take((size_t)b * n * 4)) : nullptr;
    float* g2 = grad ? static_cast<float*>(take((size_t)b * n * 4)) : nullptr;
    if (grad) {
      hipLaunchKernelGGL(flash_grad_init_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, ac1,
                         (long long)b * n, g1);
      hipLaunchKernelGGL(flash_grad_init_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, ac2,
                         (long long)b * n, g2);
    }
    fa.A = s1;
    fa.B = s2;
    launch_flash<true>(fgrid, st, fa, 1);
    hipLaunchKernelGGL(flash_sum_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, gp, rp,
                       b, ns, n, id2, cnt + b, kp_penalty, g2, rcol);
    PF_CHECK_LAUNCH();
    hipLaunchKernelGGL(disk_final_kernel, dim3(1), dim3(1024), 0, st, rcol, b * n, ac1, ac2, lp1,
                       lp2, b, n, n, kp_penalty, out);
    PF_CHECK_LAUNCH();
    if (!grad) return POSFEAT_OK;
    // columns = image-1 points: sum_n reward p
    fa.A = s2;
    fa.B = s1;
    launch_flash<true>(fgrid, st, fa, 0);
    hipLaunchKernelGGL(flash_sum_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, gp,
                       (const double*)nullptr, b, ns, n, id1, cnt, kp_penalty, g1,
                       (double*)nullptr);
    hipLaunchKernelGGL(disk_point_grad_kernel, dim3(pts_blocks), dim3(256), 0, st, kp1, b, H, W,
                       pr1, ac1, g1, dkp1);
    hipLaunchKernelGGL(disk_point_grad_kernel, dim3(pts_blocks), dim3(256), 0, st, kp2, b, H, W,
                       pr2, ac2, g2, dkp2);
    PF_CHECK_LAUNCH();
    return POSFEAT_OK;
  }
  float* S = static_cast<float*>(take((size_t)b * n * n * 4));
  double* part = static_cast<double*>(take((size_t)b * ((n + 3) / 4) * 8));
  float2* colp = static_cast<float2*>(take((size_t)b * COL_CH * n * 8));
  for (int i = 0; i < b; ++i) {
    posfeat_conv_desc d;
    d.n = 1;
    d.h = 1;
    d.w = n;
    d.cin = 128;
    d.x_cstride = 128;
    d.cout = n;
    d.kh = d.kw = d.stride = 1;
    d.pad = 0;
    d.y_cstride = n;
    d.res_cstride = 0;
    d.act = POSFEAT_ACT_NONE;
    PF_TRY(posfeat_conv2d_nhwc(&d, f1 + (size_t)i * n * 128, f2 + (size_t)i * n * 128, nullptr,
                               nullptr, S + (size_t)i * n * n, st));
  }
  hipLaunchKernelGGL(row_lse_kernel, dim3(pts_blocks), dim3(256), 0, st, S, (long long)b * n, n,
                     temperature, lr);
  hipLaunchKernelGGL(col_lse_partial_kernel, dim3((n + 63) / 64, COL_CH, b), dim3(256), 0, st, S,
                     n, n, temperature, colp);
  hipLaunchKernelGGL(col_lse_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, colp, b,
                     n, lc);
  PF_CHECK_LAUNCH();
  const int mblocks = (n + 3) / 4;
  hipLaunchKernelGGL(reinforce_kernel, dim3(mblocks, b), dim3(RB), 0, st, S, n, n, temperature,
                     lr, lc, ac1, ac2, lp1, lp2, ln1, ln2, cpx1, cpx2, reward_thr, good_reward,
                     bad_reward, part);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(disk_final_kernel, dim3(1), dim3(1024), 0, st, part, b * mblocks, ac1, ac2,
                     lp1, lp2, b, n, n, kp_penalty, out);
  PF_CHECK_LAUNCH();
  if (!grad) return POSFEAT_OK;
  float* g1 = static_cast<float*>(take((size_t)b * n * 4));
  float* g2 = static_cast<float*>(take((size_t)b * n * 4));
  float* gcp = static_cast<float*>(take((size_t)b * COL_CH * n * 4));
  PairCtx pc{S, n, n, temperature, reward_thr, good_reward, bad_reward, lr, lc, ln1, ln2, cpx1, cpx2};
  hipLaunchKernelGGL(grad_row_kernel, dim3(pts_blocks), dim3(256), 0, st, pc, b, ac1, ac2,
                     kp_penalty, g1);
  hipLaunchKernelGGL(grad_col_partial_kernel, dim3((n + 63) / 64, COL_CH, b), dim3(256), 0, st, pc,
                     ac1, ac2, gcp);
  hipLaunchKernelGGL(grad_col_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st, gcp, b, n,
                     ac2, kp_penalty, g2);
  hipLaunchKernelGGL(disk_point_grad_kernel, dim3(pts_blocks), dim3(256), 0, st, kp1, b, H, W, pr1,
                     ac1, g1, dkp1);
  hipLaunchKernelGGL(disk_point_grad_kernel, dim3(pts_blocks), dim3(256), 0, st, kp2, b, H, W, pr2,
                     ac2, g2, dkp2);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

// The flash LSE pass on its own (the softmax normaliser of DiskLoss,
// kploss.py:160-166): lse[b][j] = logsumexp_i(T <fa_i, fb_j> - T) over the n
// rows of fa, for each of the n rows of fb; fa, fb [b][n][128] L2-normalised.
extern "C" size_t posfeat_disk_flash_lse_workspace(int b, int n) {
  if (b <= 0 || n <= 0) return 0;
  return pf_align((size_t)b * flash_nsplit(n, b) * n * 8, 256) +
         2 * pf_align((size_t)b * n * FD * 6, 256);  // bf16x6 planes of fa / fb
}

extern "C" int posfeat_disk_flash_lse(const float* fa, const float* fb, int b, int n, float T,
                                      float* lse, void* ws, size_t ws_bytes, void* stream) {
  if (!fa || !fb || !lse || !ws || b <= 0 || n <= 0) return POSFEAT_E_INVALID;
  if (ws_bytes < posfeat_disk_flash_lse_workspace(b, n)) return POSFEAT_E_WORKSPACE;
  hipStream_t st = pf_stream(stream);
  const int ns = flash_nsplit(n, b);
  FlashArgs fa_{};
  char* pw = static_cast<char*>(ws) + pf_align((size_t)b * ns * n * 8, 256);
  unsigned short* pla = reinterpret_cast<unsigned short*>(pw);
  unsigned short* plb = reinterpret_cast<unsigned short*>(pw + pf_align((size_t)b * n * FD * 6, 256));
  if (flash_bf6()) {
    flash_split(fa, b, n, pla, st);
    flash_split(fb, b, n, plb, st);
  }
  fa_.A = FlashSide{fa, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, pla};
  fa_.B = FlashSide{fb, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, plb};
  fa_.n = n;
  fa_.rows_per_split = ((n + ns - 1) / ns + FSTEP - 1) / FSTEP * FSTEP;
  fa_.T = T;
  fa_.lse_part = static_cast<float2*>(ws);
  launch_flash<false>(dim3((n + FCOLS - 1) / FCOLS, ns, b), st, fa_, 0);
  hipLaunchKernelGGL(flash_lse_final_kernel, dim3((b * n + 255) / 256), dim3(256), 0, st,
                     fa_.lse_part, b, ns, n, lse);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

extern "C" int posfeat_disk_loss(const float* kp1, const float* kp2, const float* xf1, int cs1,
                                 const float* xf2, int cs2, int b, int H, int W, const float* F1,
                                 const float* F2, const int32_t* prop1, const int32_t* prop2,
                                 const uint8_t* acc1, const uint8_t* acc2, const float* uni1,
                                 const float* uni2, float temperature, float reward_thr,
                                 float good_reward, float bad_reward, float kp_penalty,
                                 float* out, void* ws, size_t ws_bytes, void* stream) {
  return disk_loss_impl(kp1, kp2, xf1, cs1, xf2, cs2, b, H, W, F1, F2, prop1, prop2, acc1, acc2,
                        uni1, uni2, temperature, reward_thr, good_reward, bad_reward, kp_penalty,
                        out, nullptr, nullptr, ws, ws_bytes, stream);
}

extern "C" int posfeat_disk_loss_grad(const float* kp1, const float* kp2, const float* xf1,
                                      int cs1, const float* xf2, int cs2, int b, int H, int W,
                                      const float* F1, const float* F2, const int32_t* prop1,
                                      const int32_t* prop2, const uint8_t* acc1,
                                      const uint8_t* acc2, const float* uni1, const float* uni2,
                                      float temperature, float reward_thr, float good_reward,
                                      float bad_reward, float kp_penalty, float* out, float* dkp1,
                                      float* dkp2, void* ws, size_t ws_bytes, void* stream) {
  if (!dkp1 || !dkp2) return POSFEAT_E_INVALID;
  return disk_loss_impl(kp1, kp2, xf1, cs1, xf2, cs2, b, H, W, F1, F2, prop1, prop2, acc1, acc2,
                        uni1, uni2, temperature, reward_thr, good_reward, bad_reward, kp_penalty,
                        out, dkp1, dkp2, ws, ws_bytes, stream);
}
