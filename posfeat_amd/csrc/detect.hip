// detect.hip -- keypoint selection on the score map (gfx950).
//
// Replaces losses/preprocess_utils.py:215-278 generate_kpts_single (stable
// branch) incl. nms (449-464).  Three launches per call:
//   K0 (thr 'max'/'mean' only) per-image threshold statistic
//   K1 det_mask    : reflect-padded NMS with the first-occurrence tie rule,
//                    threshold, order-preserving uint32 key of the masked
//                    score; survivors compacted (wave ballot + one atomic per
//                    block, four pixels per thread) into a per-image
//                    candidate list, whose length is the survivor count
//   K2 det_select  : one workgroup per image -- n = clamp(min count), 4-pass
//                    8-bit radix select of the n-th largest key over the
//                    candidates only (masked-out cells are counted, not
//                    read; 16 loads in flight per thread, the digit from a
//                    parallel suffix scan); keys == T resolved by smallest
//                    index
//   K3 det_rank    : rank each selected cell by (key desc, index asc) with an
//                    LDS-tiled counting sort (n^2 compares, exact, eight
//                    entries per step; the selected list may be in any
//                    order), compute the 3x3
//                    soft-argmax refine and 3x3 max score and scatter to the
//                    output row = rank
// Everything is integer/compare work, so the result is bit-exact and
// deterministic (the candidate order depends on atomics; the output does not).
#include "common.h"

namespace {

__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}

// torch.linspace(-1, 1, n)[i] in float32 (ATen's two-sided formula)
__device__ __forceinline__ float lin_m11(int i, int n) {
  const float step = __fdiv_rn(2.0f, (float)(n - 1));
  return i < n / 2 ? __fadd_rn(-1.0f, __fmul_rn(step, (float)i))
                   : __fsub_rn(1.0f, __fmul_rn(step, (float)(n - 1 - i)));
}

__global__ void det_thr_kernel(const float* __restrict__ kp, int h, int w, int mode, float thr,
                               float* __restrict__ tout) {
  const int b = blockIdx.x;
  const int Hi = h - 2, Wi = w - 2, P = Hi * Wi;
  const float* m = kp + (long long)b * h * w;
  double s = 0.0;
  float mx = -INFINITY;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const int i = p / Wi, j = p - (p / Wi) * Wi;
    const float v = m[(i + 1) * w + j + 1];
    s += v;
    mx = fmaxf(mx, v);
  }
  __shared__ double rs[256];
  __shared__ float rm[256];
  rs[threadIdx.x] = s;
  rm[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      rs[threadIdx.x] += rs[threadIdx.x + o];
      rm[threadIdx.x] = fmaxf(rm[threadIdx.x], rm[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float stat = mode == 2 ? rm[0] : (float)(rs[0] / (double)P);
    tout[b] = __fmul_rn(thr, stat);
  }
}

// r = 1 (the configs' nms_radius): the eight neighbours loaded together and
// compared branch-free (the early-exit loop below waited out one load latency
// per neighbour); the same decision
__device__ __forceinline__ bool nms_keep1(const float* __restrict__ m, int w, int Hi, int Wi,
                                          int off, int i, int j, float S) {
  const int y0 = reflect_idx(i - 1, Hi) + off, y1 = i + off, y2 = reflect_idx(i + 1, Hi) + off;
  const int x0 = reflect_idx(j - 1, Wi) + off, x1 = j + off, x2 = reflect_idx(j + 1, Wi) + off;
  const float v0 = m[y0 * w + x0], v1 = m[y0 * w + x1], v2 = m[y0 * w + x2], v3 = m[y1 * w + x0];
  const float v5 = m[y1 * w + x2], v6 = m[y2 * w + x0], v7 = m[y2 * w + x1], v8 = m[y2 * w + x2];
  // earlier window positions (0-3) must be < S, later ones (5-8) <= S
  return (v0 < S) & (v1 < S) & (v2 < S) & (v3 < S) & (v5 <= S) & (v6 <= S) & (v7 <= S) & (v8 <= S);
}

// NMS decision for pixel (i, j) of an Hi x Wi map stored with row pitch `w`
// at offset (off, off): reflect padding, first-occurrence tie rule.
__device__ __forceinline__ bool nms_keep(const float* __restrict__ m, int w, int Hi, int Wi, int off,
                                         int i, int j, int r, float S) {
  if (r == 1) return nms_keep1(m, w, Hi, Wi, off, i, j, S);
  const int ws = 2 * r + 1, center = r * ws + r;
  int pos = 0;
  for (int dy = -r; dy <= r; ++dy) {
    const int yy = reflect_idx(i + dy, Hi) + off;
    for (int dx = -r; dx <= r; ++dx, ++pos) {
      if (pos == center) continue;
      const float v = m[yy * w + reflect_idx(j + dx, Wi) + off];
      if (pos < center ? !(v < S) : !(v <= S)) return false;
    }
  }
  return true;
}

__global__ void nms_mask_kernel(const float* __restrict__ score, int h, int w, int r,
                                uint8_t* __restrict__ mask) {
  const int b = blockIdx.y;
  const float* m = score + (long long)b * h * w;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < h * w; p += gridDim.x * blockDim.x) {
    const int i = p / w, j = p - (p / w) * w;
    mask[(long long)b * h * w + p] = nms_keep(m, w, h, w, 0, i, j, r, m[p]) ? 1 : 0;
  }
}

// PX pixels per thread (p = base + k * 1024 + tid): the PX decisions' loads
// are independent and go out together, one LDS atomic per wave and one
// global atomic per block cover all PX * 1024 pixels.  With one pixel per
// thread (PX = 1, A/B: POSFEAT_DET_PX=1) each 1024-pixel block paid a chain
// of load -> compare -> LDS atomic -> barrier -> global atomic -> barrier
// latencies for its 1024 pixels (112 us for 32 x 478 x 638 cells, r16n).
template <int PX>
__global__ __launch_bounds__(1024) void det_mask_kernel(const float* __restrict__ kp, int h, int w,
                                                        int r, int use_nms, int use_thr,
                                                        const float* __restrict__ thr_t,
                                                        uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ cand_key,
                                                        int32_t* __restrict__ cand_idx,
                                                        int32_t* __restrict__ counts) {
  const int b = blockIdx.y;  // one image per grid row: block-uniform counter
  const int Hi = h - 2, Wi = w - 2, P = Hi * Wi;
  const float* m = kp + (long long)b * h * w;
  const float t = use_thr ? thr_t[b] : 0.f;
  __shared__ uint32_t s_key[PX * 1024];
  __shared__ int32_t s_idx[PX * 1024];
  __shared__ int s_cnt, s_base;
  const int lane = threadIdx.x & 63;
  constexpr int CH = PX * 1024;
  const int stride = gridDim.x * CH;
  for (int base = blockIdx.x * CH; base < P; base += stride) {
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    bool keep[PX];
    uint32_t key[PX];
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      const int p = base + k * 1024 + threadIdx.x;
      keep[k] = false;
      key[k] = 0x80000000u;
      if (p < P) {
        const int i = p / Wi, j = p - (p / Wi) * Wi;
        const float S = m[(i + 1) * w + j + 1];
        bool kk = use_thr ? (S > t) : true;
        if (kk && use_nms) kk = nms_keep(m, w, Hi, Wi, 1, i, j, r, S);
        keep[k] = kk;
        key[k] = pf_fkey(kk ? S : 0.0f);
        keys[(long long)b * P + p] = key[k];
      }
    }
    // wave-aggregated LDS compaction of the survivors: one atomic per wave
    unsigned long long bal[PX];
    int tot = 0;
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      bal[k] = __ballot(keep[k]);
      tot += __popcll(bal[k]);
    }
    int wbase = 0;
    if (lane == 0 && tot) wbase = atomicAdd(&s_cnt, tot);
    wbase = __shfl(wbase, 0, 64);
#pragma unroll
    for (int k = 0; k < PX; ++k) {
      if (keep[k]) {
        const int o = wbase + __popcll(bal[k] & ((1ull << lane) - 1ull));
        s_key[o] = key[k];
        s_idx[o] = base + k * 1024 + threadIdx.x;
      }
      wbase += __popcll(bal[k]);
    }
    __syncthreads();
    const int cnt = s_cnt;
    if (threadIdx.x == 0 && cnt) s_base = atomicAdd(&counts[b], cnt);
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
      cand_key[(long long)b * P + s_base + k] = s_key[k];
      cand_idx[(long long)b * P + s_base + k] = s_idx[k];
    }
    __syncthreads();
  }
}

// block-wide exclusive scan of per-thread 0/1 flags in ascending thread order.
// Returns the exclusive prefix, sets *total.
__device__ __forceinline__ int block_scan_flag(bool f, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(f);
  const int pre = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[wv] = __popcll(bal);
  __syncthreads();
  int off = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) {
    const int v = wsum[k];
    off += (k < wv) ? v : 0;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + pre;
}

// One workgroup per image.  Selects the n cells ranking first by (key desc,
// index asc) among all P inner cells: the survivors live in the candidate
// list, every other cell has the masked-out key ZKEY.
//   1. n = clamp(min count); 8-bit radix select of the n-th key over the
//      candidates + (P - count) virtual ZKEY entries
//   2. take every key > T (all candidates when T >= ZKEY); of the keys == T
//      take the need_eq with the smallest index (candidates sorted in LDS, or
//      an ascending scan of the full key array when T == ZKEY)
//   3. rare T < ZKEY (negative kept scores, n close to P): ascending scan of
//      the full key array, as in the single-pass formulation
__global__ __launch_bounds__(1024) void det_select_kernel(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ cand_key,
    const int32_t* __restrict__ cand_idx, int nb, int P, const int32_t* __restrict__ counts,
    int num_pts, int cap, int32_t* __restrict__ sel, uint32_t* __restrict__ selkey,
    int32_t* __restrict__ n_sel, int each) {
  const int b = blockIdx.x;
  const uint32_t ZKEY = 0x80000000u;
  const uint32_t* kb = keys + (long long)b * P;
  const uint32_t* ck = cand_key + (long long)b * P;
  const int32_t* ci = cand_idx + (long long)b * P;
  int32_t* so = sel + (long long)b * cap;
  uint32_t* sko = selkey + (long long)b * cap;
  __shared__ int hist[256];
  __shared__ int wsum[16];
  __shared__ uint32_t s_prefix;
  __shared__ int s_krem, s_n, s_taken, s_dig, s_above;
  __shared__ int s_eqidx[1024];
  __shared__ int s_eqn;
  const int tid = threadIdx.x;
  const int count = counts[b];
  const int nzero = P - count;  // masked-out cells, key ZKEY
  if (tid == 0) {
    int minc = counts[each ? b : 0];
    if (!each)
      for (int k = 1; k < nb; ++k) minc = min(minc, counts[k]);
    int n = num_pts > 0 ? min(num_pts, minc) : minc;
    if (n < 128) n = 128;
    n = min(n, P);
    n = min(n, cap);
    s_n = n;
    s_krem = n;
    s_prefix = 0u;
    s_taken = 0;
    s_eqn = 0;
    if (each) n_sel[b] = n;
    else if (b == 0) *n_sel = n;
  }
  __syncthreads();
  const int n = s_n;
  uint32_t pmask = 0u;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int k = tid; k < 256; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    if (tid == 0 && nzero > 0 && (ZKEY & pmask) == prefix)
      atomicAdd(&hist[(ZKEY >> shift) & 0xFF], nzero);
    // DU candidates per thread per round trip, loads first (a histogram: the
    // counts do not depend on the order; round 5 loaded four, and each pass
    // was a chain of count / 4096 dependent global-load latencies)
    constexpr int DU = 16;
    const int bd = blockDim.x;
    for (int k = tid; k < count; k += DU * bd) {
      uint32_t kk[DU];
#pragma unroll
      for (int u = 0; u < DU; ++u) kk[u] = k + u * bd < count ? ck[k + u * bd] : ~pmask;
#pragma unroll
      for (int u = 0; u < DU; ++u)
        if (k + u * bd < count && (kk[u] & pmask) == prefix)
          atomicAdd(&hist[(kk[u] >> shift) & 0xFF], 1);
    }
    __syncthreads();
    // the digit: the largest d with S(d) = sum_{d' >= d} hist[d'] >= krem (d = 0
    // if none), found by threads 0-255 from a suffix scan (the round-5 form
    // walked the 256 bins serially in one thread: 256 dependent LDS reads per
    // pass)
    int hd = 0, sfx = 0;
    if (tid < 256) {  // waves 0-3: the within-wave suffix sums
      const int lane = tid & 63;
      hd = hist[tid];
      sfx = hd;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_down(sfx, o, 64);
        if (lane + o < 64) sfx += v;
      }
      if (lane == 0) wsum[tid >> 6] = sfx;  // the wave's total
    }
    __syncthreads();
    if (tid < 256) {
      for (int k = (tid >> 6) + 1; k < 4; ++k) sfx += wsum[k];
      const int krem = s_krem;
      const int above = sfx - hd;  // S(d + 1)
      if ((sfx >= krem || tid == 0) && above < krem) {
        s_dig = tid;
        s_above = above;
      }
    }
    __syncthreads();
    if (tid == 0) {
      s_krem -= s_above;
      s_prefix = prefix | ((uint32_t)s_dig << shift);
    }
    pmask |= 0xFFu << shift;
    __syncthreads();
  }
  const uint32_t T = s_prefix;
  const int need_eq = s_krem;  // how many keys == T are taken (>= 1)
  if (T > ZKEY) {
    // (a) every candidate key > T; collect the == T ones (keys loaded DU at
    // a time: the index is read only for the ~n taken ones)
    constexpr int DU = 8;
    for (int k0 = tid; k0 < count; k0 += DU * (int)blockDim.x) {
      uint32_t kk[DU];
#pragma unroll
      for (int u = 0; u < DU; ++u) kk[u] = k0 + u * (int)blockDim.x < count ? ck[k0 + u * blockDim.x] : 0u;
#pragma unroll
      for (int u = 0; u < DU; ++u) {
        const int k = k0 + u * blockDim.x;
        if (kk[u] > T) {  // (0 < T for the padding lanes)
          const int pos = atomicAdd(&s_taken, 1);
          so[pos] = ci[k];
          sko[pos] = kk[u];
        } else if (kk[u] == T) {
          const int e = atomicAdd(&s_eqn, 1);
          if (e < 1024) s_eqidx[e] = ci[k];
        }
      }
    }
    __syncthreads();
    const int neq = s_eqn;
    if (neq <= 1024) {
      const int base = s_taken;
      // (b) the need_eq smallest indices among the equal keys (rank by index)
      for (int e = tid; e < neq; e += blockDim.x) {
        const int my = s_eqidx[e];
        int rk = 0;
        for (int f = 0; f < neq; ++f) rk += s_eqidx[f] < my;
        if (rk < need_eq) {
          so[base + rk] = my;
          sko[base + rk] = T;
        }
      }
      return;
    }
    // > 1024 exact ties at the cut: fall through to the ordered scan (rewrites)
  }
  else if (T == ZKEY) {
    // all positive candidates, then the need_eq lowest-index cells with key ZKEY
    constexpr int DU = 8;
    for (int k0 = tid; k0 < count; k0 += DU * (int)blockDim.x) {
      uint32_t kk[DU];
#pragma unroll
      for (int u = 0; u < DU; ++u) kk[u] = k0 + u * (int)blockDim.x < count ? ck[k0 + u * blockDim.x] : 0u;
#pragma unroll
      for (int u = 0; u < DU; ++u)
        if (kk[u] > ZKEY) {
          const int pos = atomicAdd(&s_taken, 1);
          so[pos] = ci[k0 + u * blockDim.x];
          sko[pos] = kk[u];
        }
    }
    __syncthreads();
    int taken = s_taken, eq_seen = 0;
    for (int base = 0; base < P && eq_seen < need_eq; base += blockDim.x) {
      const int p = base + tid;
      const bool eq = p < P && kb[p] == ZKEY;
      int tot;
      const int pre = block_scan_flag(eq, wsum, &tot);
      if (eq && eq_seen + pre < need_eq) {
        so[taken + pre] = p;
        sko[taken + pre] = ZKEY;
      }
      const int add = min(tot, need_eq - eq_seen);
      eq_seen += add;
      taken += add;
    }
    return;
  }
  // T < ZKEY: ordered compaction over the full key array
  int eq_seen = 0, taken = 0;
  for (int base = 0; base < P; base += blockDim.x) {
    const int p = base + tid;
    const uint32_t k = p < P ? kb[p] : 0u;
    const bool gt = p < P && k > T;
    const bool eq = p < P && k == T;
    int eq_tot;
    const int eq_pre = block_scan_flag(eq, wsum, &eq_tot);
    const bool take = gt || (eq && (eq_seen + eq_pre) < need_eq);
    int tk_tot;
    const int tk_pre = block_scan_flag(take, wsum, &tk_tot);
    if (take) {
      so[taken + tk_pre] = p;
      sko[taken + tk_pre] = k;
    }
    eq_seen += eq_tot;
    taken += tk_tot;
    if (taken >= n) break;  // uniform across the block
  }
}

__global__ void det_rank_kernel(const float* __restrict__ kp, int h, int w, int cap,
                                const int32_t* __restrict__ sel, const uint32_t* __restrict__ selkey,
                                const int32_t* __restrict__ n_sel, int each,
                                int32_t* __restrict__ idx_out, float* __restrict__ coord,
                                float* __restrict__ score) {
  const int b = blockIdx.y;
  const int n = n_sel[each ? b : 0];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= n) return;  // block-uniform
  const bool active = t < n;
  const uint32_t* kb = selkey + (long long)b * cap;
  const int32_t* ib = sel + (long long)b * cap;
  const uint32_t myk = active ? kb[t] : 0u;
  const int myi = active ? ib[t] : 0;
  // (key desc, index asc) as one 64-bit composite, (key << 32) | ~index:
  // "o ranks before me" is one unsigned 64-bit compare (the && / || form
  // compiled to a branch per entry); two composites per 16-B LDS read, eight
  // entries per step with four partial counts (round 5: one dependent LDS
  // read per entry, 59 us at n = 2048, B = 32)
  typedef unsigned long long u64;
  const u64 myc = ((u64)myk << 32) | (u64)(0xFFFFFFFFu - (uint32_t)myi);
  __shared__ __attribute__((aligned(16))) u64 tile[1024];
  int rank = 0;
  for (int base = 0; base < n; base += 1024) {
    for (int k = threadIdx.x; k < 1024; k += blockDim.x)
      tile[k] = base + k < n ? ((u64)kb[base + k] << 32) | (u64)(0xFFFFFFFFu - (uint32_t)ib[base + k])
                             : 0ull;
    __syncthreads();
    const int lim = min(1024, n - base);
    if (active) {
      int r4[4] = {0, 0, 0, 0};
      const int full = lim & ~7;
      for (int k = 0; k < full; k += 8) {
        ulonglong2 o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) o[u] = *reinterpret_cast<const ulonglong2*>(tile + k + 2 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) r4[u] += (int)(o[u].x > myc) + (int)(o[u].y > myc);
      }
      for (int k = full; k < lim; ++k) r4[0] += (int)(tile[k] > myc);
      rank += (r4[0] + r4[1]) + (r4[2] + r4[3]);
    }
    __syncthreads();
  }
  if (!active) return;
  const int Wi = w - 2;
  const int p = sel[(long long)b * cap + t];
  const int i = p / Wi, j = p - (p / Wi) * Wi;
  const float* m = kp + (long long)b * h * w;
  float sx = 0.f, sy = 0.f, sw = 0.f, mx = -INFINITY;
  for (int dy = 0; dy < 3; ++dy) {
    const float gy = lin_m11(i + dy, h);
    for (int dx = 0; dx < 3; ++dx) {
      const float v = m[(i + dy) * w + j + dx];
      const float gx = lin_m11(j + dx, w);
      sx = __fadd_rn(sx, __fmul_rn(v, gx));
      sy = __fadd_rn(sy, __fmul_rn(v, gy));
      sw = __fadd_rn(sw, v);
      mx = fmaxf(mx, v);
    }
  }
  const float aw = __fdiv_rn(sw, 9.0f);
  const long long o = (long long)b * cap + rank;
  idx_out[o] = p;
  coord[o * 2 + 0] = __fdiv_rn(__fdiv_rn(sx, 9.0f), aw);
  coord[o * 2 + 1] = __fdiv_rn(__fdiv_rn(sy, 9.0f), aw);
  score[o] = mx;
}

}  // namespace

extern "C" int posfeat_detect_workspace(int b, int h, int w, int cap, size_t* bytes) {
  if (b <= 0 || h < 3 || w < 3 || cap <= 0 || !bytes) return POSFEAT_E_INVALID;
  const size_t P = (size_t)(h - 2) * (w - 2);
  size_t s = pf_align((size_t)b * P * sizeof(uint32_t), 256);    // keys
  s += pf_align((size_t)b * P * sizeof(uint32_t), 256);          // cand_key
  s += pf_align((size_t)b * P * sizeof(int32_t), 256);           // cand_idx
  s += pf_align((size_t)b * cap * sizeof(int32_t), 256);         // sel
  s += pf_align((size_t)b * cap * sizeof(uint32_t), 256);        // selkey
  s += pf_align((size_t)b * sizeof(float), 256);                 // thr
  *bytes = s;
  return POSFEAT_OK;
}

namespace {

// each = 0: one n for the batch (posfeat_detect); 1: n per image (posfeat_detect_each)
int detect_impl(const float* kp_map, int b, int h, int w, int nms_radius, int use_nms,
                int thr_mode, float thr, int num_pts, int cap, int32_t* idx, float* coord,
                float* score, int32_t* n_sel, int32_t* counts, void* ws, size_t ws_bytes,
                void* stream, int each) {
  if (!kp_map || !idx || !coord || !score || !n_sel || !counts || !ws) return POSFEAT_E_INVALID;
  if (b <= 0 || h < 3 || w < 3 || nms_radius < 0 || thr_mode < 0 || thr_mode > 3)
    return POSFEAT_E_INVALID;
  const int Hi = h - 2, Wi = w - 2, P = Hi * Wi;
  if (use_nms && (nms_radius >= Hi || nms_radius >= Wi)) return POSFEAT_E_INVALID;  // reflect pad limit
  const int need = num_pts > 0 ? (num_pts < 128 ? 128 : num_pts) : P;
  if (cap < (need < P ? need : P)) return POSFEAT_E_INVALID;
  size_t need_ws = 0;
  posfeat_detect_workspace(b, h, w, cap, &need_ws);
  if (ws_bytes < need_ws) return POSFEAT_E_WORKSPACE;
  hipStream_t st = pf_stream(stream);
  char* base = static_cast<char*>(ws);
  uint32_t* keys = reinterpret_cast<uint32_t*>(base);
  base += pf_align((size_t)b * P * sizeof(uint32_t), 256);
  uint32_t* cand_key = reinterpret_cast<uint32_t*>(base);
  base += pf_align((size_t)b * P * sizeof(uint32_t), 256);
  int32_t* cand_idx = reinterpret_cast<int32_t*>(base);
  base += pf_align((size_t)b * P * sizeof(int32_t), 256);
  int32_t* sel = reinterpret_cast<int32_t*>(base);
  base += pf_align((size_t)b * cap * sizeof(int32_t), 256);
  uint32_t* selkey = reinterpret_cast<uint32_t*>(base);
  base += pf_align((size_t)b * cap * sizeof(uint32_t), 256);
  float* thr_t = reinterpret_cast<float*>(base);

  if (hipMemsetAsync(counts, 0, sizeof(int32_t) * b, st) != hipSuccess) return POSFEAT_E_HIP;
  const int use_thr = thr_mode != 0;
  if (thr_mode == 1) {
    // 'abs': thr * tensor(1.)  (preprocess_utils.py:237-239)
    float t[64];
    if (b > 64) return POSFEAT_E_INVALID;
    for (int k = 0; k < b; ++k) t[k] = thr * 1.0f;
    if (hipMemcpyAsync(thr_t, t, sizeof(float) * b, hipMemcpyHostToDevice, st) != hipSuccess)
      return POSFEAT_E_HIP;
  } else if (thr_mode >= 2) {
    hipLaunchKernelGGL(det_thr_kernel, dim3(b), dim3(256), 0, st, kp_map, h, w, thr_mode, thr,
                       thr_t);
    PF_CHECK_LAUNCH();
  }
  {
    static const int px = [] {  // A/B: POSFEAT_DET_PX=1 / 8
      const char* e = pf_ab_getenv("POSFEAT_DET_PX");
      const int v = e ? atoi(e) : 4;
      return v == 1 || v == 8 ? v : 4;
    }();
    int g = (P + px * 1024 - 1) / (px * 1024);
    if (g > 1024) g = 1024;
    if (px == 1)
      hipLaunchKernelGGL(det_mask_kernel<1>, dim3(g, b), dim3(1024), 0, st, kp_map, h, w,
                         nms_radius, use_nms, use_thr, thr_t, keys, cand_key, cand_idx, counts);
    else if (px == 8)
      hipLaunchKernelGGL(det_mask_kernel<8>, dim3(g, b), dim3(1024), 0, st, kp_map, h, w,
                         nms_radius, use_nms, use_thr, thr_t, keys, cand_key, cand_idx, counts);
    else
      hipLaunchKernelGGL(det_mask_kernel<4>, dim3(g, b), dim3(1024), 0, st, kp_map, h, w,
                         nms_radius, use_nms, use_thr, thr_t, keys, cand_key, cand_idx, counts);
    PF_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(det_select_kernel, dim3(b), dim3(1024), 0, st, keys, cand_key, cand_idx, b,
                     P, counts, num_pts, cap, sel, selkey, n_sel, each);
  PF_CHECK_LAUNCH();
  const int maxn = cap < P ? cap : P;
  hipLaunchKernelGGL(det_rank_kernel, dim3((maxn + 255) / 256, b), dim3(256), 0, st, kp_map, h, w,
                     cap, sel, selkey, n_sel, each, idx, coord, score);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

}  // namespace

extern "C" int posfeat_detect(const float* kp_map, int b, int h, int w, int nms_radius,
                              int use_nms, int thr_mode, float thr, int num_pts, int cap,
                              int32_t* idx, float* coord, float* score, int32_t* n_sel,
                              int32_t* counts, void* ws, size_t ws_bytes, void* stream) {
  return detect_impl(kp_map, b, h, w, nms_radius, use_nms, thr_mode, thr, num_pts, cap, idx, coord,
                     score, n_sel, counts, ws, ws_bytes, stream, 0);
}

extern "C" int posfeat_detect_each(const float* kp_map, int b, int h, int w, int nms_radius,
                                   int use_nms, int thr_mode, float thr, int num_pts, int cap,
                                   int32_t* idx, float* coord, float* score, int32_t* n_sel,
                                   int32_t* counts, void* ws, size_t ws_bytes, void* stream) {
  return detect_impl(kp_map, b, h, w, nms_radius, use_nms, thr_mode, thr, num_pts, cap, idx, coord,
                     score, n_sel, counts, ws, ws_bytes, stream, 1);
}

extern "C" int posfeat_nms_mask(const float* score, int b, int h, int w, int radius,
                                uint8_t* mask, void* stream) {
  if (!score || !mask || b <= 0 || h <= 0 || w <= 0 || radius < 0) return POSFEAT_E_INVALID;
  if (radius >= h || radius >= w) return POSFEAT_E_INVALID;  // reflect pad limit (as torch)
  int g = (h * w + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(nms_mask_kernel, dim3(g, b), dim3(256), 0, pf_stream(stream), score, h, w,
                     radius, mask);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
