// gemm_y.hip -- timing probe for an 8-wave bf16x6 GEMM tile with BOTH operands
// staged by LDS DMA (the dense pre-split-weight GEMM of conv.hip, on the
// upconv2 / iconv2 Winograd GEMM shape: M = 38400, N = 256, K = 512, 36
// batches).  Not part of the library.  Build: tools/probe/build.sh.
//
// Why: conv_bf6x_kernel keeps the fp32 A operand (the
// Winograd V, streamed from HBM) in registers one 32-k chunk ahead; per CU that
// is ~48 KB of A in flight at most, about what Little's law allows at ~2 us of
// loaded HBM latency for the ~12 GB/s per CU the GEMM draws at 0.48 of the
// ceiling.  Here one 512-thread block per CU computes a 128 x 256 tile (A is
// read once per M tile instead of once per 128-column half), A arrives by LDS
// DMA into a ring of AST stages (AST - 1 chunks ahead: 32 KB in flight per CU
// at AST = 3), B's three bf16 planes into a two-stage ring, and one counted
// vmcnt + barrier per chunk.
//
// Wave w: rows 32 (w & 3) .. + 31 (two 16-row blocks), columns 128 (w >> 2) ..
// + 127 (eight 16-column blocks); 96 v_mfma_f32_16x16x32_bf16 per chunk.
// FL bits: 1 no A DMA in the loop, 2 no B DMA in the loop, 16 no MFMAs.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int BK = 32;
#define NO_VMEM 0x78F
#define PIN 0x786

__device__ __forceinline__ unsigned cvt_pk(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ void split3(const f32x4& p0, const f32x4& p1, u32x4_t& h, u32x4_t& m,
                                       u32x4_t& l) {
  const float x[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = x[2 * i], b = x[2 * i + 1];
    const unsigned hp = cvt_pk(a, b);
    const float ra = a - __uint_as_float(hp << 16), rb = b - __uint_as_float(hp & 0xffff0000u);
    const unsigned mp = cvt_pk(ra, rb);
    const float sa = ra - __uint_as_float(mp << 16), sb = rb - __uint_as_float(mp & 0xffff0000u);
    h[i] = hp;
    m[i] = mp;
    l[i] = cvt_pk(sa, sb);
  }
}
__device__ __forceinline__ f32x4 mfma16(const u32x4_t& a, const u32x4_t& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
// A stage: [128 rows][8 slots of 16 B] fp32, slot s of row r at s ^ aswz(r):
// the 16 lanes of every ds_read_b128 lane group hit 16 distinct 4-bank groups
__device__ __forceinline__ int aswz(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 2); }
// B stage: per plane [256 rows][4 slots of 16 B] bf16 (conv.hip bx_swz)
__device__ __forceinline__ int bswz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {  // vmcnt(N), lgkmcnt(0)
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
}

struct Args {
  const float* A;            // [nb][M][K]
  const unsigned short* Bp;  // [nb][3][N][K]
  float* C;                  // [nb][M][N]
  int M, N, K, tiles_n, nwg;
};

template <class F>
__device__ __forceinline__ void stages(unsigned short* __restrict__ bd, float* __restrict__ ad,
                                       const unsigned short* __restrict__ bs,
                                       const float* __restrict__ as, F&& f) {
  f(bd, ad, bs, as);
}

template <int AST, int FL>
__global__ __launch_bounds__(512) void ky(Args a) {
  constexpr int BM = 128, BN = 256, RB = 2, NB = 8;
  constexpr int ASTAGE = BM * BK;          // floats
  constexpr int BSTAGE = 3 * BN * BK;      // u16
  constexpr int A_G = ASTAGE / 256 / 8;    // A DMA instructions per wave per chunk (2)
  constexpr int B_G = BSTAGE / 512 / 8;    // B DMA instructions per wave per chunk (6)
  constexpr int NOPS = A_G + B_G;
  __shared__ __attribute__((aligned(16))) float As[AST * ASTAGE];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2 * BSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const long long z = blockIdx.y;
  const float* A = a.A + z * a.M * a.K;
  const unsigned short* Bp = a.Bp + z * 3LL * a.N * a.K;
  float* C = a.C + z * a.M * a.N;
  const int m0 = bid * BM;
  const int r16 = lane & 15, kq = lane >> 4;
  // DMA sources: A instruction i of this wave fills stage rows (wave A_G + i) 8 + lane / 8
  const float* asrc[A_G];
#pragma unroll
  for (int i = 0; i < A_G; ++i) {
    const int row = (wave * A_G + i) * 8 + (lane >> 3);
    const int ls = (lane & 7) ^ aswz(row & 15);
    asrc[i] = A + (long long)min(m0 + row, a.M - 1) * a.K + ls * 4;
  }
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ bswz(row);
    bsrc[i] = Bp + (long long)plane * a.N * a.K + (long long)row * a.K + ks * 8;
  }
  const int nch = a.K / BK;
  auto dma_a = [&](float* st, int c, int i) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(asrc[i] + (long long)min(c, nch - 1) * BK),
        (__attribute__((address_space(3))) void*)(st + (wave * A_G + i) * 256), 16, 0, 0);
  };
  auto dma_b = [&](unsigned short* st, int c, int i) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)min(c, nch - 1) * BK),
        (__attribute__((address_space(3))) void*)(st + (wave * B_G + i) * 512), 16, 0, 0);
  };
  f32x4 acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // prologue: A(0 .. AST-3), then step 0 = [B(0), A(AST-2)]; step k's ops are
  // issued in chunk k-1: [B(k), A(k + AST - 2)], so at the top of chunk c all
  // but the A(c + AST - 2) DMAs (A_G, the youngest) must have landed
#pragma unroll
  for (int c = 0; c < AST - 2; ++c)
#pragma unroll
    for (int i = 0; i < A_G; ++i) dma_a(As + c * ASTAGE, c, i);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
#pragma unroll
  for (int i = 0; i < B_G; ++i) dma_b(Bs, 0, i);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
#pragma unroll
  for (int i = 0; i < A_G; ++i) dma_a(As + (AST - 2) * ASTAGE, AST - 2, i);
  int sa = 0;  // A stage of chunk c
  for (int c = 0; c < nch; ++c) {
    __builtin_amdgcn_sched_barrier(NO_VMEM);
    wait_vm_lgkm0<(AST >= 3 ? A_G : 0)>();  // AST = 2: A(c) is among the youngest
    __builtin_amdgcn_s_barrier();
    const int sb = c & 1;
    const int swa = sa == 0 ? AST - 1 : sa - 1;  // A stage refilled: chunk c + AST - 1
    stages(Bs + (sb ^ 1) * BSTAGE, As + swa * ASTAGE, Bs + sb * BSTAGE, As + sa * ASTAGE,
           [&](unsigned short* __restrict__ Bd, float* __restrict__ Ad,
               const unsigned short* __restrict__ Bb, const float* __restrict__ Ab) {
             // this wave's A fragments: rows 32 wm + 16 rb + r16, k 8 kq .. + 7
             u32x4_t ah[RB], am[RB], al[RB];
#pragma unroll
             for (int rb = 0; rb < RB; ++rb) {
               const int row = wm * 32 + rb * 16 + r16;
               const float* ap = Ab + row * BK;
               const f32x4 v0 = *reinterpret_cast<const f32x4*>(ap + ((2 * kq) ^ aswz(r16)) * 4);
               const f32x4 v1 =
                   *reinterpret_cast<const f32x4*>(ap + ((2 * kq + 1) ^ aswz(r16)) * 4);
               split3(v0, v1, ah[rb], am[rb], al[rb]);
             }
             int op = 0;
             auto mem = [&]() {
               __builtin_amdgcn_sched_barrier(PIN);
               if (op < B_G) {
                 if (!(FL & 2)) dma_b(Bd, c + 1, op);
               } else if (op < NOPS) {
                 if (!(FL & 1)) dma_a(Ad, c + AST - 1, op - B_G);
               }
               __builtin_amdgcn_sched_barrier(PIN);
               ++op;
             };
#pragma unroll
             for (int nb = 0; nb < NB; ++nb) {
               const int row = wn * 128 + nb * 16 + r16;
               const int slot = kq ^ bswz(row);
               const unsigned short* bp = Bb + row * BK + slot * 8;
               const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
               const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
               const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
#pragma unroll
               for (int rb = 0; rb < RB; ++rb) {
                 f32x4 cc = acc[rb][nb];
                 if (FL & 16) {
                   cc[0] += __uint_as_float(ah[rb][0] ^ bh[0] ^ bm[1] ^ bl[2] ^ am[rb][1] ^ al[rb][2]);
                 } else {
                   cc = mfma16(ah[rb], bh, cc);
                   cc = mfma16(ah[rb], bm, cc);
                   cc = mfma16(am[rb], bh, cc);
                   cc = mfma16(ah[rb], bl, cc);
                   cc = mfma16(al[rb], bh, cc);
                   cc = mfma16(am[rb], bm, cc);
                 }
                 acc[rb][nb] = cc;
               }
               while (op < (nb + 1) * NOPS / NB) mem();
             }
             while (op < NOPS) mem();
           });
    sa = sa + 1 == AST ? 0 : sa + 1;
  }
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + rb * 16 + kq * 4 + r;
        if (row < a.M) C[(long long)row * a.N + wn * 128 + nb * 16 + r16] = acc[rb][nb][r];
      }
}

// reference for the check: C = A * (Bh + Bm + Bl)^T products as the six
// bf16 terms, fp32 accumulate, on the host (one batch, a few rows)
static unsigned short rne(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
static float bf(unsigned short u) {
  unsigned v = (unsigned)u << 16;
  float f;
  memcpy(&f, &v, 4);
  return f;
}

template <class K>
float run(K kern, Args a, int nb, int reps, int threads) {
  a.tiles_n = 1;
  a.nwg = (a.M + 127) / 128;
  dim3 g(a.nwg, nb);
  hipLaunchKernelGGL(kern, g, dim3(threads), 0, 0, a);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, g, dim3(threads), 0, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int M = 38400, N = 256, K = 512, nb = 36, reps = argc > 1 ? atoi(argv[1]) : 10;
  Args a;
  a.M = M;
  a.N = N;
  a.K = K;
  float *A, *C;
  unsigned short* Bp;
  CK(hipMalloc(&A, (size_t)nb * M * K * 4));
  CK(hipMalloc(&C, (size_t)nb * M * N * 4));
  CK(hipMalloc(&Bp, (size_t)nb * 3 * N * K * 2));
  std::vector<float> h((size_t)M * K);
  std::vector<unsigned short> hb((size_t)nb * 3 * N * K);
  {
    unsigned s = 1;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = (int)(s >> 9) * (1.0f / 4194304.0f) - 1.0f;
    }
    for (int z = 0; z < nb; ++z)
      CK(hipMemcpy(A + (size_t)z * M * K, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    for (auto& v : hb) {
      s = s * 1664525u + 1013904223u;
      v = 0x3c00 + ((s >> 16) & 0xff);
    }
    CK(hipMemcpy(Bp, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  }
  a.A = A;
  a.Bp = Bp;
  a.C = C;
  const double fl = 2.0 * nb * M * N * K;
  auto rep = [&](const char* name, float ms) {
    printf("%-30s %8.3f ms  %7.1f TF/s fp32-eq  %.3f of 416.7\n", name, ms, fl / ms / 1e9,
           fl / ms / 1e9 / 416.7);
    fflush(stdout);
  };
  // correctness of the AST = 3 kernel against a host sum of the same six
  // bf16 products (fp64 accumulation; the GPU's fp32 sums agree to ~1e-6 rel)
  run(ky<3, 0>, a, nb, 1, 512);
  {
    std::vector<float> hc((size_t)M * N);
    CK(hipMemcpy(hc.data(), C + (size_t)5 * M * N, hc.size() * 4, hipMemcpyDeviceToHost));
    const unsigned short* B5 = hb.data() + (size_t)5 * 3 * N * K;
    double maxrel = 0;
    for (int m : {0, 1, 17, 127, 128, 20000, M - 1})
      for (int n : {0, 5, 127, 128, 200, N - 1}) {
        double s = 0, sa = 0;
        for (int k = 0; k < K; ++k) {
          const float x = h[(size_t)m * K + k];
          const float xh = bf(rne(x)), xm = bf(rne(x - xh)), xl = bf(rne(x - xh - xm));
          const double bh = bf(B5[(size_t)n * K + k]), bm = bf(B5[(size_t)N * K + (size_t)n * K + k]),
                       bl = bf(B5[2 * (size_t)N * K + (size_t)n * K + k]);
          const double t = (double)xh * bh + (double)xh * bm + (double)xm * bh + (double)xh * bl +
                           (double)xl * bh + (double)xm * bm;
          s += t;
          sa += fabs(t);
        }
        const double g = hc[(size_t)m * N + n];
        maxrel = fmax(maxrel, fabs(g - s) / fmax(sa, 1e-30));
      }
    printf("check: max |C - ref| / sum|terms| = %.3e (%s)\n", maxrel, maxrel < 1e-5 ? "ok" : "BAD");
  }
  rep("ky AST3", run(ky<3, 0>, a, nb, reps, 512));
  rep("ky AST2", run(ky<2, 0>, a, nb, reps, 512));
  rep("ky AST3 no-A-dma", run(ky<3, 1>, a, nb, reps, 512));
  rep("ky AST3 no-B-dma", run(ky<3, 2>, a, nb, reps, 512));
  rep("ky AST3 no-dma", run(ky<3, 3>, a, nb, reps, 512));
  rep("ky AST3 no-mfma", run(ky<3, 16>, a, nb, reps, 512));
  rep("ky AST3 again", run(ky<3, 0>, a, nb, reps, 512));
  return 0;
}
