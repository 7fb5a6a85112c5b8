// mfma_numerics.hip -- how v_mfma_f32_16x16x32_bf16 and v_mfma_f32_32x32x16_bf16
// add their (exact) bf16 products to the fp32 accumulator: internal precision
// of the product sum and the rounding of the final add, on crafted operands.
// Every lane supplies the same 8 bf16 of A and of B, so each output element is
// C + sum over K of a_k b_k with the per-lane k pattern below.  Not part of
// the library.  Build: tools/probe/build.sh; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// a, b: 32 values each (the k index of the 16x16x32 / two 32x32x16 steps)
__global__ void k16(const float* a, const float* b, float c0, float* out) {
  const int lane = threadIdx.x, kq = lane >> 4;
  bf16x8_t av, bv;
  for (int j = 0; j < 8; ++j) {
    av[j] = (__bf16)a[kq * 8 + j];
    bv[j] = (__bf16)b[kq * 8 + j];
  }
  f32x4 c = {c0, c0, c0, c0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  if (lane == 0) out[0] = c[0];
}
__global__ void k32(const float* a, const float* b, float c0, float* out) {
  const int lane = threadIdx.x, hh = lane >> 5;
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = c0;
  for (int s = 0; s < 2; ++s) {  // k 0..15, then 16..31
    bf16x8_t av, bv;
    for (int j = 0; j < 8; ++j) {
      av[j] = (__bf16)a[s * 16 + hh * 8 + j];
      bv[j] = (__bf16)b[s * 16 + hh * 8 + j];
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
  }
  if (lane == 0) out[0] = c[0];
}

struct Case {
  const char* name;
  float c0;
  float a[32], b[32];
};

int main() {
  float *da, *db, *dout;
  hipMalloc(&da, 128);
  hipMalloc(&db, 128);
  hipMalloc(&dout, 16);
  auto run = [&](const char* name, float c0, const float* a, const float* b) {
    hipMemcpy(da, a, 128, hipMemcpyHostToDevice);
    hipMemcpy(db, b, 128, hipMemcpyHostToDevice);
    float r16, r32;
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
    hipMemcpy(&r16, dout, 4, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, da, db, c0, dout);
    hipMemcpy(&r32, dout, 4, hipMemcpyDeviceToHost);
    long double exact = c0;
    for (int k = 0; k < 32; ++k) exact += (long double)a[k] * b[k];
    const float rn = (float)exact;  // the correctly rounded (RNE) fp32 result
    const float ulp = std::nextafter(std::fabs(rn), INFINITY) - std::fabs(rn);
    printf("%-44s exact %.10Lg  RNE %.9g  16x16x32 %.9g (%+.2f ulp)  32x32x16 %.9g (%+.2f ulp)\n",
           name, exact, rn, r16, (r16 - rn) / ulp, r32, (r32 - rn) / ulp);
  };
  float a[32], b[32];
  auto zero = [&]() { memset(a, 0, sizeof a); memset(b, 0, sizeof b); };
  // 1. 32 products of 2^-25 on 1.0: exact 1 + 2^-20; an fp32 chain gives 1.0
  zero();
  for (int k = 0; k < 32; ++k) a[k] = ldexpf(1, -13), b[k] = ldexpf(1, -12);
  run("32 x 2^-25 on 1.0", 1.0f, a, b);
  // 2. one product 0.75 ulp(1) on 1.0: RNE -> 1 + ulp, truncation -> 1
  zero();
  a[0] = 1.5f * ldexpf(1, -12); b[0] = ldexpf(1, -12);  // 1.5 * 2^-24 = 0.75 ulp(1)
  run("0.75 ulp on 1.0", 1.0f, a, b);
  run("0.75 ulp on -1.0 (opposite sign)", -1.0f, a, b);
  // 3. 0.75 ulp made of 3 products of 0.25 ulp each
  zero();
  for (int k = 0; k < 3; ++k) a[k] = ldexpf(1, -13), b[k] = ldexpf(1, -12);
  run("3 x 0.25 ulp on 1.0", 1.0f, a, b);
  // 4. cancellation: big +x and -x products plus a small one
  zero();
  a[0] = 1.0f; b[0] = 3.0f; a[1] = -1.0f; b[1] = 3.0f; a[2] = ldexpf(1, -20); b[2] = 1.0f;
  run("3 - 3 + 2^-20 on 0", 0.0f, a, b);
  // 5. a small product next to a large one (alignment loss inside the sum?)
  zero();
  a[0] = 1.0f; b[0] = 1.0f; a[1] = ldexpf(1, -30); b[1] = 1.0f;
  run("1 + 2^-30 on 0", 0.0f, a, b);
  zero();
  a[0] = 1.0f; b[0] = 1.0f; a[1] = 1.5f * ldexpf(1, -24); b[1] = 1.0f;
  run("1 + 0.75 ulp (in the sum) on 0", 0.0f, a, b);
  // 6. random-ish: mixed magnitudes, many rounding steps
  zero();
  unsigned s = 12345;
  for (int k = 0; k < 32; ++k) {
    s = s * 1664525u + 1013904223u;
    a[k] = (float)(__bf16)(((int)(s >> 8) % 2001 - 1000) / 997.0f);
    s = s * 1664525u + 1013904223u;
    b[k] = (float)(__bf16)(((int)(s >> 8) % 2001 - 1000) / 991.0f);
  }
  run("random bf16 on 0.3", 0.3f, a, b);
  return 0;
}
