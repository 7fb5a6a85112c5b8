// match.hip -- the evaluation matchers on gfx950.
//
// Replaces, for L2-normalised 128-d descriptors:
//   mnn_matcher              losses/preprocess_utils.py:795-803
//                            (= evaluations/hpatches/evaluation.py:28-38)
//   mutual_nn_matcher        evaluations/aachen/matchers.py:5-14
//                            (= evaluations/ETH_local_feature/custom_matcher.py:5-14)
//   ratio_matcher            evaluations/aachen/matchers.py:17-44
//   mutual_nn_ratio_matcher  evaluations/aachen/matchers.py:47-75
//
// All four need, per row of sim = d1 d2^T and per column, the arg-max and the
// top-2 similarities.  sim is never written: match_top2_kernel computes one
// side's statistics (for every row j of B: top-2 over the rows i of A of
// <A_i, B_j>) with fp32 MFMA and keeps them in registers; it runs twice, with
// (A, B) = (d1, d2) for the columns and (d2, d1) for the rows.  The k order of
// the fmaf chain is the same in both runs, so both read identical sim bits.
//
// Layout: each wave holds 32 B rows (its columns) as MFMA B fragments in 64
// VGPRs for the whole launch; A is streamed in 64-row steps through LDS by
// DMA (global_load_lds, XOR-swizzled 16-B slots: conflict-free ds_read_b128),
// two stages.  Per step each wave runs 2 x 64 v_mfma_f32_32x32x2_f32 and folds
// the 32 x 32 accumulators into a running (best value, best index, second
// value) per column lane -- in increasing row order with strict '>' updates,
// so the FIRST index wins an arg-max tie (the stated tie rule; the second
// value is the 2nd largest with multiplicity, as torch.topk(2) returns it).
// A rows are split over blockIdx.y so launches reach >= 512 workgroups; the
// split partials are merged in split order (deterministic).  The match
// kernel applies the reference's mask (mutual, ratio via sqrt(2 - 2 s) in
// fp32, or both) and compacts the matches in ascending first index.
#include <algorithm>
#include <cmath>

#include "common.h"

namespace {

constexpr int MD = 128;       // descriptor dimension
constexpr int MCOLS = 128;    // B rows (columns of sim) per block: 4 waves x 32
constexpr int MSTEP = 64;     // A rows per LDS step (2 x 32-row MFMA blocks)

struct Top2 {
  float v1;
  int i1;
  float v2;
};

// merge two partial top-2 sets (value descending, index ascending)
__device__ __forceinline__ Top2 top2_merge(const Top2& a, const Top2& b) {
  const bool a_first = a.v1 > b.v1 || (a.v1 == b.v1 && a.i1 < b.i1);
  const Top2& f = a_first ? a : b;
  const Top2& s = a_first ? b : a;
  return Top2{f.v1, f.i1, fmaxf(f.v2, s.v1)};
}

__global__ __launch_bounds__(256) void match_top2_kernel(const float* __restrict__ A, int na,
                                                         const float* __restrict__ B, int nb,
                                                         int rows_per_split,
                                                         float* __restrict__ pv1,
                                                         int* __restrict__ pi1,
                                                         float* __restrict__ pv2) {
  __shared__ __attribute__((aligned(16))) float As[2 * MSTEP * MD];  // 2 x 32 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int col = blockIdx.x * MCOLS + wave * 32 + (lane & 31);
  const int split = blockIdx.y;
  // this wave's B fragments: lane half h supplies k = 8g + 4h + j for MFMA j
  f32x4 breg[MD / 8];
  {
    const float* brow = B + (long long)min(col, nb - 1) * MD;
#pragma unroll
    for (int g = 0; g < MD / 8; ++g) breg[g] = *reinterpret_cast<const f32x4*>(brow + 8 * g + 4 * h);
  }
  const int r0 = split * rows_per_split;
  const int r1 = min(na, r0 + rows_per_split);
  const int nsteps = (r1 - r0 + MSTEP - 1) / MSTEP;
  // DMA of step s into stage `buf`: wave-instruction t covers rows 2t, 2t+1
  // of the step (lane L: row 2t + L/32, physical slot L%32 holding logical
  // slot (L%32) ^ (row & 15)); rows past r1 re-read row r1 - 1 (masked later)
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int t = 0; t < MSTEP / 2 / 4; ++t) {
      const int lr = (wave * (MSTEP / 8) + t) * 2 + h;
      const int row = min(r0 + s * MSTEP + lr, r1 - 1);
      const int slot = (lane & 31) ^ (lr & 15);
      const float* src = A + (long long)row * MD + slot * 4;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)src,
          (__attribute__((address_space(3))) void*)(As + buf * MSTEP * MD +
                                                     (wave * (MSTEP / 8) + t) * 2 * MD),
          16, 0, 0);
    }
  };
  Top2 best{-INFINITY, 0x7fffffff, -INFINITY};
  if (nsteps > 0) issue(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) issue(s + 1, cur ^ 1);
    const float* Ab = As + cur * MSTEP * MD;
    // both 32-row blocks at once: two independent accumulation chains
    f32x16 accs[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) accs[0][r] = accs[1][r] = 0.f;
    {
      const int la = lane & 31;  // rows la and 32 + la share the swizzle (la & 15)
      const float* arow0 = Ab + la * MD;
      const float* arow1 = Ab + (32 + la) * MD;
#pragma unroll
      for (int g = 0; g < MD / 8; ++g) {
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
      // acc[r] = sim(A row i, B row col), i = step base + mi*32 + (r&3) + 8(r>>2) + 4h:
      // increasing in r, so strict '>' keeps the first index on ties
      const int ib = r0 + s * MSTEP + mi * 32 + 4 * h;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = ib + (r & 3) + 8 * (r >> 2);
        const float v = i < r1 ? acc[r] : -INFINITY;
        if (v > best.v1) {
          best.v2 = best.v1;
          best.v1 = v;
          best.i1 = i;
        } else if (v > best.v2) {
          best.v2 = v;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  // the two lane halves of a column hold interleaved row sets: merge
  Top2 o;
  o.v1 = __shfl_xor(best.v1, 32, 64);
  o.i1 = __shfl_xor(best.i1, 32, 64);
  o.v2 = __shfl_xor(best.v2, 32, 64);
  best = h == 0 ? top2_merge(best, o) : top2_merge(o, best);
  if (h == 0 && col < nb) {
    const long long p = (long long)split * nb + col;
    pv1[p] = best.v1;
    pi1[p] = best.i1;
    pv2[p] = best.v2;
  }
}

// merge the split partials of each column in split order
__global__ void match_merge_kernel(const float* __restrict__ pv1, const int* __restrict__ pi1,
                                   const float* __restrict__ pv2, int nsplit, int nb,
                                   int* __restrict__ nn, float* __restrict__ v1,
                                   float* __restrict__ v2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nb) return;
  Top2 t{pv1[c], pi1[c], pv2[c]};
  for (int s = 1; s < nsplit; ++s) {
    const long long p = (long long)s * nb + c;
    t = top2_merge(t, Top2{pv1[p], pi1[p], pv2[p]});
  }
  nn[c] = t.i1;
  v1[c] = t.v1;
  v2[c] = t.v2;
}

// torch: sqrt(2 - 2 s) in fp32; ratio = d1 / (d2 + 1e-8)
__device__ __forceinline__ float lowe_ratio(float s1, float s2) {
  const float d1 = __fsqrt_rn(__fsub_rn(2.f, __fmul_rn(2.f, s1)));
  const float d2 = __fsqrt_rn(__fsub_rn(2.f, __fmul_rn(2.f, s2)));
  return __fdiv_rn(d1, __fadd_rn(d2, 1e-8f));
}

// mode: 0 mutual NN, 1 symmetric ratio, 2 mutual NN + symmetric ratio.
// One workgroup: each thread owns a contiguous range of rows i, counts its
// matches, an exclusive scan in LDS gives its output offset (matches come
// out in ascending i, as the reference's boolean-mask indexing orders them).
__global__ __launch_bounds__(1024) void match_select_kernel(
    const int* __restrict__ nn12, const float* __restrict__ r1a, const float* __restrict__ r1b,
    const int* __restrict__ nn21, const float* __restrict__ r2a, const float* __restrict__ r2b,
    int n1, int mode, float ratio, int* __restrict__ matches, int* __restrict__ count) {
  __shared__ int off[1024];
  const int t = threadIdx.x, per = (n1 + 1023) / 1024;
  const int i0 = min(n1, t * per), i1 = min(n1, i0 + per);
  auto keep = [&](int i) {
    const int j = nn12[i];
    bool k = true;
    if (mode != 1) k = nn21[j] == i;
    if (mode != 0) {
      const float q12 = lowe_ratio(r1a[i], r1b[i]);
      const float q21 = lowe_ratio(r2a[j], r2b[j]);
      k = k && (q12 <= ratio) && (q21 <= ratio);  // NaN compares false, as in torch
    }
    return k;
  };
  int c = 0;
  for (int i = i0; i < i1; ++i) c += keep(i) ? 1 : 0;
  off[t] = c;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
    const int v = t >= d ? off[t - d] : 0;
    __syncthreads();
    off[t] += v;
    __syncthreads();
  }
  int o = off[t] - c;
  for (int i = i0; i < i1; ++i)
    if (keep(i)) {
      matches[2 * o] = i;
      matches[2 * o + 1] = nn12[i];
      ++o;
    }
  if (t == 1023) *count = off[1023];
}

// A-row split filling whole rounds of the 512 resident workgroups (2 per CU)
int nsplit_for(int na, int nb) {
  const int ncb = (nb + MCOLS - 1) / MCOLS;
  const int smax = std::max(1, std::min(32, (na + MSTEP - 1) / MSTEP));
  int best = 1;
  double best_eff = 0.0;
  for (int s = 1; s <= smax; ++s) {
    const double r = (double)ncb * s / 512.0;
    const double eff = r / std::ceil(r) * (r < 1.0 ? r : 1.0);
    if (eff >= 0.94) return s;  // the fewest splits that keep the tail small
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = s;
    }
  }
  return best;
}

size_t side_ws(int na, int nb) {  // partials (3 per column per split) + merged (3 per column)
  return pf_align((size_t)nsplit_for(na, nb) * nb * 12, 256) + pf_align((size_t)nb * 12, 256);
}

// per row j of B: (arg-max_i, top value, 2nd value) over the rows i of A
int top2_side(const float* A, int na, const float* B, int nb, char* ws, int* nn, float* v1,
              float* v2, hipStream_t st) {
  const int ns = nsplit_for(na, nb);
  const int rps = ((na + ns - 1) / ns + MSTEP - 1) / MSTEP * MSTEP;
  const int ns_eff = (na + rps - 1) / rps;
  float* pv1 = reinterpret_cast<float*>(ws);
  int* pi1 = reinterpret_cast<int*>(ws + (size_t)ns * nb * 4);
  float* pv2 = reinterpret_cast<float*>(ws + (size_t)ns * nb * 8);
  hipLaunchKernelGGL(match_top2_kernel, dim3((nb + MCOLS - 1) / MCOLS, ns_eff), dim3(256), 0, st,
                     A, na, B, nb, rps, pv1, pi1, pv2);
  PF_CHECK_LAUNCH();
  hipLaunchKernelGGL(match_merge_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, pv1, pi1, pv2,
                     ns_eff, nb, nn, v1, v2);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

}  // namespace

extern "C" size_t posfeat_match_workspace(int n1, int n2) {
  if (n1 <= 0 || n2 <= 0) return 0;
  return side_ws(n2, n1) + side_ws(n1, n2) + 256;
}

extern "C" int posfeat_match(const float* d1, int n1, const float* d2, int n2, int dim, int mode,
                             float ratio, int32_t* matches, int32_t* count, void* ws,
                             size_t ws_bytes, void* stream) {
  if (!d1 || !d2 || !matches || !count || !ws || n1 <= 0 || n2 <= 0) return POSFEAT_E_INVALID;
  if (dim != MD || mode < 0 || mode > 2) return POSFEAT_E_UNSUPPORTED;
  if ((reinterpret_cast<uintptr_t>(d1) & 15) || (reinterpret_cast<uintptr_t>(d2) & 15) ||
      (reinterpret_cast<uintptr_t>(ws) & 255))
    return POSFEAT_E_INVALID;
  if (ws_bytes < posfeat_match_workspace(n1, n2)) return POSFEAT_E_WORKSPACE;
  hipStream_t st = pf_stream(stream);
  char* w = static_cast<char*>(ws);
  // rows of sim: for each d1 row i, top-2 over d2 rows (A = d2, B = d1)
  char* rws = w;
  char* rout = rws + pf_align((size_t)nsplit_for(n2, n1) * n1 * 12, 256);
  int* nn12 = reinterpret_cast<int*>(rout);
  float* r1a = reinterpret_cast<float*>(rout + (size_t)n1 * 4);
  float* r1b = reinterpret_cast<float*>(rout + (size_t)n1 * 8);
  PF_TRY(top2_side(d2, n2, d1, n1, rws, nn12, r1a, r1b, st));
  // columns: for each d2 row j, top-2 over d1 rows (A = d1, B = d2)
  char* cws = w + side_ws(n2, n1);
  char* cout_ = cws + pf_align((size_t)nsplit_for(n1, n2) * n2 * 12, 256);
  int* nn21 = reinterpret_cast<int*>(cout_);
  float* r2a = reinterpret_cast<float*>(cout_ + (size_t)n2 * 4);
  float* r2b = reinterpret_cast<float*>(cout_ + (size_t)n2 * 8);
  PF_TRY(top2_side(d1, n1, d2, n2, cws, nn21, r2a, r2b, st));
  hipLaunchKernelGGL(match_select_kernel, dim3(1), dim3(1024), 0, st, nn12, r1a, r1b, nn21, r2a,
                     r2b, n1, mode, ratio, matches, count);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
