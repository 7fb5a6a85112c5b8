// gemm6.hip -- fp32-exact GEMMs on the bf16 matrix cores with PRE-SPLIT
// operands ("bf16x6", see conv.hip split3 for the arithmetic).
//
// The in-kernel split of conv.hip's BF6 row tiles costs ~11 VALU
// instructions per operand pair per MFMA k-step, which is what bounds it
// (PMC: the matrix pipe ~33 % busy, VALU-issue and DMA waits the rest).  The
// GEMMs whose operands are produced by our own kernels -- the Winograd
// transform-domain GEMMs (V from the input transform, U from the weight
// transform) and head.conv2's low-res tap GEMM (L, the tap weights) -- get
// their operands already split by the producer, as three bf16 planes
// (h, m, l) of the fp32 array's shape.  The GEMM then only stages bf16 by
// LDS-DMA and issues MFMAs: per 32x32x16 step 6 MFMAs and 6 ds_read_b128 of
// operand fragments per wave, no conversion work.
//
// C[z] [M][N] (row pitch ldc, fp32) = sum over the six term products of
// A[z] [M][K] x B[z] [N][K]^T; plane p of A at A + p * pa (elements), row pitch
// lda; likewise B.  K % 32 == 0, N % BN == 0, 16-B aligned rows.
#include "common.h"
#include "fmap.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_bf16(const u32x4_t& a, const u32x4_t& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

constexpr int GK = 32;  // k per LDS stage (64 B per plane row)
__device__ __attribute__((aligned(16))) unsigned short g6_zero[8];  // masked rows read zeros

// 4 waves (2 x 2), wave tile (BM/2) x (BN/2); LDS stage = [3 planes][BM + BN
// rows][4 slots of 16 B], slot s of row r holding k-slot s ^ ((r >> 2) & 3)
// (conflict-free ds_read_b128: 16 consecutive rows x one k-slot hit 16
// distinct 16-B bank groups).  Two stages; the DMA of chunk c+1 is in flight
// while chunk c is multiplied.
template <int BM, int BN>
__global__ __launch_bounds__(256) void gemm_bf6p_kernel(
    const unsigned short* __restrict__ A, int lda, long long pa, long long sa,
    const unsigned short* __restrict__ B, int ldb, long long pb, long long sb,
    float* __restrict__ C, int ldc, long long sc, int M, int N, int K, int tiles_n, int nwg) {
  constexpr int ROWS = BM + BN;
  constexpr int STAGE = 3 * ROWS * 32;  // u16 per stage
  constexpr int TM = BM / 2, TN = BN / 2, MI = TM / 32, NI = TN / 32;
  constexpr int EPI = BM * (BN + 4) * 4;
  constexpr int RING = 2 * STAGE * 2;
  __shared__ __attribute__((aligned(16))) char smem[RING > EPI ? RING : EPI];
  unsigned short* S = reinterpret_cast<unsigned short*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  int bid = blockIdx.x;
  {
    const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const long long z = blockIdx.y;
  A += z * sa;
  B += z * sb;
  C += z * sc;
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // DMA: one wave-instruction = 64 lanes x 16 B = 16 plane-rows of 64 B;
  // lane L -> plane-row (L >> 2) of the group, LDS slot L & 3
  constexpr int NG = 3 * ROWS / 16;  // instructions per stage
  static_assert(NG % 4 == 0, "groups per wave");
  constexpr int GPW = NG / 4;
  const unsigned short* src[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int pr = (wave * GPW + i) * 16 + (lane >> 2);  // plane-row index
    const int plane = pr / ROWS, row = pr - plane * ROWS;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    const unsigned short* s = nullptr;
    if (row < BM) {
      if (m0 + row < M) s = A + plane * pa + (long long)(m0 + row) * lda + ks * 8;
    } else {
      s = B + plane * pb + (long long)(n0 + row - BM) * ldb + ks * 8;
    }
    src[i] = s;
  }
  auto issue = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const unsigned short* s = src[i] ? src[i] + (long long)c * GK : (const unsigned short*)g6_zero;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)s,
          (__attribute__((address_space(3))) void*)(S + buf * STAGE + (wave * GPW + i) * 16 * 32),
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

  const int r32 = lane & 31, hh = lane >> 5;
  auto frag = [&](int buf, int plane, int row, int g) {
    const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
    return *reinterpret_cast<const u32x4_t*>(S + buf * STAGE + (plane * ROWS + row) * 32 + slot * 8);
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int g = 0; g < GK / 16; ++g) {
      u32x4_t a[3][MI], b[3][NI];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) a[p][mi] = frag(buf, p, wm * TM + mi * 32 + r32, g);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) b[p][ni] = frag(buf, p, BM + wn * TN + ni * 32 + r32, g);
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          f32x16 c = acc[mi][ni];
          c = mfma_bf16(a[0][mi], b[0][ni], c);
          c = mfma_bf16(a[0][mi], b[1][ni], c);
          c = mfma_bf16(a[1][mi], b[0][ni], c);
          c = mfma_bf16(a[0][mi], b[2][ni], c);
          c = mfma_bf16(a[2][mi], b[0][ni], c);
          c = mfma_bf16(a[1][mi], b[1][ni], c);
          acc[mi][ni] = c;
        }
    }
  };

  const int nch = K / GK;
  issue(0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) issue(c + 1, cur ^ 1);
    compute(cur);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }

  // epilogue: acc -> LDS [BM][BN+4] -> coalesced f32x4 rows
  float* T = reinterpret_cast<float*>(smem);
  constexpr int TP = BN + 4;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        T[(wm * TM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh) * TP + wn * TN + ni * 32 + r32] =
            acc[mi][ni][r];
  __syncthreads();
  constexpr int C4 = BN / 4, RPP = 256 / C4;
  const int q = tid % C4, r0 = tid / C4;
  for (int row = r0; row < BM; row += RPP) {
    const int m = m0 + row;
    if (m < M)
      *reinterpret_cast<f32x4*>(C + (long long)m * ldc + n0 + 4 * q) =
          *reinterpret_cast<const f32x4*>(T + row * TP + 4 * q);
  }
}

// x (rows x cols, pitch ldx, fp32) -> three bf16 planes (pitch cols, plane
// stride rows * cols elements); 4 elements per thread
__global__ void split3_rows_kernel(const float* __restrict__ x, long long rows, int cols, int ldx,
                                   unsigned short* __restrict__ out) {
  const int c4 = cols / 4;
  const long long total = rows * c4, plane = rows * cols;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c4;
    const int q = (int)(i - r * c4);
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + r * ldx + q * 4);
    uint2 h, m, l;
    pf_split3x4(v, h, m, l);
    uint2* o = reinterpret_cast<uint2*>(out + r * cols + q * 4);
    o[0] = h;
    o[plane / 4] = m;
    o[plane / 2] = l;
  }
}

}  // namespace

bool pf_bf6p_on() { return pf_conv_precision() == 2; }

int pf_split3_rows(const float* x, long long rows, int cols, int ldx, unsigned short* out,
                   hipStream_t st) {
  if (cols % 4 || ldx % 4 || ((rows * cols) % 4)) return POSFEAT_E_INVALID;
  const long long total = rows * (cols / 4);
  long long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(split3_rows_kernel, dim3((int)g), dim3(256), 0, st, x, rows, cols, ldx, out);
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}

int pf_gemm_bf6p(const unsigned short* A, int lda, long long pa, long long sa,
                 const unsigned short* B, int ldb, long long pb, long long sb, float* C, int ldc,
                 long long sc, int nb, int M, int N, int K, hipStream_t st) {
  if (K % GK || nb < 1 || M < 1 || lda % 8 || ldb % 8 || ldc % 4) return POSFEAT_E_INVALID;
  const bool wide = N % 256 == 0 && (long long)((M + 127) / 128) * (N / 256) * nb >= 512;
  if (N % 128) return POSFEAT_E_UNSUPPORTED;
  if (wide) {
    const int tn = N / 256, nwg = ((M + 127) / 128) * tn;
    hipLaunchKernelGGL((gemm_bf6p_kernel<128, 256>), dim3(nwg, nb), dim3(256), 0, st, A, lda, pa,
                       sa, B, ldb, pb, sb, C, ldc, sc, M, N, K, tn, nwg);
  } else {
    const int tn = N / 128, nwg = ((M + 127) / 128) * tn;
    hipLaunchKernelGGL((gemm_bf6p_kernel<128, 128>), dim3(nwg, nb), dim3(256), 0, st, A, lda, pa,
                       sa, B, ldb, pb, sb, C, ldc, sc, M, N, K, tn, nwg);
  }
  PF_CHECK_LAUNCH();
  return POSFEAT_OK;
}
