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
// (h, m, l) of the fp32 array's shape (conv precision mode 2).  The GEMM is
// conv.hip's conv_bf6s_kernel (register-prefetched A planes, no conversion
// work in the MFMA loop); this file keeps the plane producer for arrays that
// are not written by a transform kernel and the mode switch.
#include "common.h"
#include "fmap.h"

namespace {

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
  // the conv family's register-prefetch tiles with A pre-split
  // (conv_bf6s_kernel); B rows are the tiles' [N][K] pre-split weight rows
  if (ldb != K || ldc % 4) return POSFEAT_E_INVALID;
  return pf_gemm_batched_pre(A, lda, pa, sa, B, pb, sb, C, ldc, sc, nb, M, N, K, st);
}
