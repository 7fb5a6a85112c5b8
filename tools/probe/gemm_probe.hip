// gemm_probe.hip -- standalone timing probe for the bf16x6 pre-split-weight
// GEMM tile (the structure of conv.hip's conv_bf6d_kernel on a dense batched
// GEMM: the Winograd transform-domain GEMMs of upconv2 / iconv2, M = 38400,
// N = 256, K = 512, 36 batches), with compile-time ablations and tile
// variants, so the bound of the production tile can be read from differences.
// Not part of the library.  Build: tools/probe/build.sh; run on the GPU box.
//
// FL bits: 1 no A loads in the loop, 2 no B DMA in the loop, 4 no A split
// (raw bits as operands), 8 no s_barrier, 16 no MFMAs.
// MI: 32-row MFMA blocks per wave (BM = 128 * MI with 4 waves).
// S16: v_mfma_f32_16x16x32_bf16 instead of 32x32x16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int BK = 32;
#define NO_VMEM 0x78F

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
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
__device__ __forceinline__ f32x16 mfma32(const u32x4_t& a, const u32x4_t& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// the refilled and the multiplied LDS stage as distinct __restrict__ pointers
// (conv.hip pf_dma_overlap_step: otherwise the waitcnt pass puts vmcnt(0)
// before the stage reads)
template <class I, class C>
__device__ __forceinline__ void overlap(unsigned short* __restrict__ d,
                                        const unsigned short* __restrict__ s, I&& issue, C&& comp) {
  issue(d);
  comp(s);
}

template <class F>
__device__ __forceinline__ void overlap2(unsigned short* __restrict__ d,
                                         const unsigned short* __restrict__ s, F&& f) {
  f(d, s);
}
// sched_barrier mask: VALU, SALU, DS and transcendental may cross; VMEM and MFMA may not
#define PIN 0x786

struct Args {
  const float* A;            // [nb][M][K]
  const unsigned short* Bp;  // [nb][3][N][K]
  float* C;                  // [nb][M][N]
  int M, N, K, tiles_n, nwg;
};

// 32x32x16 tile: 4 waves stacked along M, each MI x 32 rows, BN = 128
template <int MI, int D, int FL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k32(Args a) {
  constexpr int BN = 128, NI = BN / 32, NW = 4, BM = NW * MI * 32;
  constexpr int B_G = 3 * BN / 16 / NW;
  constexpr int BSTAGE = 3 * BN * BK;  // u16
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2 * BSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const long long z = blockIdx.y;
  const float* A = a.A + z * a.M * a.K;
  const unsigned short* Bp = a.Bp + z * 3LL * a.N * a.K;
  float* C = a.C + z * a.M * a.N;
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r32 = lane & 31, hh = lane >> 5;
  const float* xrow[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
    xrow[mi] = A + (long long)min(m0 + (wave * MI + mi) * 32 + r32, a.M - 1) * a.K + hh * 8;
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = Bp + (long long)plane * a.N * a.K + (long long)(n0 + row) * a.K + ks * 8;
  }
  const int nch = a.K / BK;
  auto issue_b = [&](unsigned short* Bd, int c) {
#pragma unroll
    for (int i = 0; i < B_G; ++i)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)c * BK),
          (__attribute__((address_space(3))) void*)(Bd + (wave * B_G + i) * 16 * BK), 16, 0, 0);
  };
  int la_c = 0;
  auto load_a = [&](f32x4 (&v)[MI][4]) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[mi][j] = *reinterpret_cast<const f32x4*>(xrow[mi] + (long long)la_c * BK + (j >> 1) * 16 +
                                                   (j & 1) * 4);
    if (la_c + 1 < nch) ++la_c;
  };
  constexpr int NA = 4 * MI;  // A loads per chunk
  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
  f32x4 va[D][MI][4];
#pragma unroll
  for (int j = 0; j < D - 1; ++j) load_a(va[j]);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
  issue_b(Bs, 0);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
  load_a(va[D - 1]);
  for (int i = 0; i < nch; i += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int ii = i + u;
      __builtin_amdgcn_sched_barrier(NO_VMEM);
      if ((FL & 3) || D == 1)
        __builtin_amdgcn_s_waitcnt(0);
      else
        wait_vmcnt<NA>();
      if (!(FL & 8)) __builtin_amdgcn_s_barrier();
      const int s = ii & 1;
      u32x4_t ah[MI][2], am[MI][2], al[MI][2];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          if (FL & 64) {
          } else if (FL & 4) {
            ah[mi][g] = __builtin_bit_cast(u32x4_t, va[u][mi][2 * g]);
            am[mi][g] = __builtin_bit_cast(u32x4_t, va[u][mi][2 * g + 1]);
            al[mi][g] = ah[mi][g] ^ am[mi][g];
          } else {
            split3(va[u][mi][2 * g], va[u][mi][2 * g + 1], ah[mi][g], am[mi][g], al[mi][g]);
          }
        }
      if (FL & 32) {  // memory ops interleaved among the MFMAs
        overlap2(Bs + (s ^ 1) * BSTAGE, Bs + s * BSTAGE,
                 [&](unsigned short* __restrict__ Bn, const unsigned short* __restrict__ Bb) {
          int op = 0;
          auto mem = [&]() {  // the op-th memory instruction of this step
            __builtin_amdgcn_sched_barrier(PIN);
            if (op < B_G) {
              __builtin_amdgcn_global_load_lds(
                  (const __attribute__((address_space(1))) void*)(bsrc[op] +
                                                                  (long long)min(ii + 1, nch - 1) * BK),
                  (__attribute__((address_space(3))) void*)(Bn + (wave * B_G + op) * 16 * BK), 16, 0, 0);
            } else if (op < B_G + NA) {
              const int j = op - B_G, mi = j >> 2, jj = j & 3;
              va[u][mi][jj] = *reinterpret_cast<const f32x4*>(xrow[mi] + (long long)la_c * BK +
                                                              (jj >> 1) * 16 + (jj & 1) * 4);
              if (j == NA - 1 && la_c + 1 < nch) ++la_c;
            }
            __builtin_amdgcn_sched_barrier(PIN);
            ++op;
          };
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) {
              if ((FL & 64) && ni == 0) {
#pragma unroll
                for (int mi = 0; mi < MI; ++mi)
                  split3(va[u][mi][2 * g], va[u][mi][2 * g + 1], ah[mi][g], am[mi][g], al[mi][g]);
              }
              const int row = ni * 32 + r32;
              const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
              const unsigned short* bp = Bb + row * BK + slot * 8;
              const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
              const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
              const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
#pragma unroll
              for (int mi = 0; mi < MI; ++mi) {
                f32x16 c = acc[mi][ni];
                c = mfma32(ah[mi][g], bh, c);
                c = mfma32(ah[mi][g], bm, c);
                c = mfma32(am[mi][g], bh, c);
                if (mi == 0) mem();
                c = mfma32(ah[mi][g], bl, c);
                c = mfma32(al[mi][g], bh, c);
                c = mfma32(am[mi][g], bm, c);
                if (mi == 0) mem();
                acc[mi][ni] = c;
              }
            }
          while (op < B_G + NA) mem();
        });
        continue;
      }
      overlap(Bs + (s ^ 1) * BSTAGE, Bs + s * BSTAGE, [&](unsigned short* Bn) {
      if (!(FL & 2)) issue_b(Bn, min(ii + 1, nch - 1));
      __builtin_amdgcn_sched_barrier(NO_VMEM);
      if (!(FL & 1)) load_a(va[u]);
      __builtin_amdgcn_sched_barrier(0);
      }, [&](const unsigned short* Bb) {
      if (ii < nch && !(FL & 16)) {
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            const int row = ni * 32 + r32;
            const int slot = (2 * g + hh) ^ ((row >> 2) & 3);
            const unsigned short* bp = Bb + row * BK + slot * 8;
            const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
            const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
            const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) {
              f32x16 c = acc[mi][ni];
              c = mfma32(ah[mi][g], bh, c);
              c = mfma32(ah[mi][g], bm, c);
              c = mfma32(am[mi][g], bh, c);
              c = mfma32(ah[mi][g], bl, c);
              c = mfma32(al[mi][g], bh, c);
              c = mfma32(am[mi][g], bm, c);
              acc[mi][ni] = c;
            }
          }
      }
      });
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  // direct register stores (the probe's epilogue; production stages via LDS)
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + (wave * MI + mi) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (row < a.M) C[(long long)row * a.N + n0 + ni * 32 + r32] = acc[mi][ni][r];
      }
}

__device__ __forceinline__ f32x4 mfma16(const u32x4_t& a, const u32x4_t& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// 16x16x32 tile: 4 waves stacked along M, each 32 rows (two 16-row blocks) x
// 128 columns (eight 16-column blocks); one MFMA covers the chunk's K = 32.
// Lane l: A row (l & 15), k (l >> 4) * 8 .. + 7; B column (l & 15), same k.
template <int D, int FL, int RB = 2, int NW = 4>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void k16(Args a) {
  constexpr int BN = 128, NB = BN / 16, BM = NW * RB * 16;
  constexpr int B_G = 3 * BN / 16 / NW;
  constexpr int BSTAGE = 3 * BN * BK;  // u16
  constexpr int NA = 2 * RB;           // A loads per chunk (two f32x4 per row block)
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2 * BSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const long long z = blockIdx.y;
  const float* A = a.A + z * a.M * a.K;
  const unsigned short* Bp = a.Bp + z * 3LL * a.N * a.K;
  float* C = a.C + z * a.M * a.N;
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r16 = lane & 15, kq = lane >> 4;
  const float* xrow[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
    // FL & 8: A loads 64 contiguous bytes per row per instruction (k = 16 jj + 4 kq
    // .. + 3: timing only -- the k pairing with B is not the MFMA's)
    xrow[rb] = A + (long long)min(m0 + wave * RB * 16 + rb * 16 + r16, a.M - 1) * a.K +
               ((FL & 8) ? kq * 4 : kq * 8);
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = Bp + (long long)plane * a.N * a.K + (long long)(n0 + row) * a.K + ks * 8;
  }
  const int nch = a.K / BK;
  int la_c = 0;
  f32x4 acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 va[D][RB][2];
  auto load_a = [&](f32x4 (&v)[RB][2]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        v[rb][j] = *reinterpret_cast<const f32x4*>(xrow[rb] + (long long)la_c * BK +
                                                   j * ((FL & 8) ? 16 : 4));
    if (la_c + 1 < nch) ++la_c;
  };
#pragma unroll
  for (int j = 0; j < D - 1; ++j) load_a(va[j]);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
#pragma unroll
  for (int i = 0; i < B_G; ++i)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)bsrc[i],
                                     (__attribute__((address_space(3))) void*)(Bs + (wave * B_G + i) * 16 * BK),
                                     16, 0, 0);
  __builtin_amdgcn_sched_barrier(NO_VMEM);
  load_a(va[D - 1]);
  for (int i = 0; i < nch; i += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int ii = i + u;
      __builtin_amdgcn_sched_barrier(NO_VMEM);
      if (D == 1)
        __builtin_amdgcn_s_waitcnt(0);
      else
        wait_vmcnt<NA>();
      __builtin_amdgcn_s_barrier();
      const int s = ii & 1;
      overlap2(Bs + (s ^ 1) * BSTAGE, Bs + s * BSTAGE,
               [&](unsigned short* __restrict__ Bn, const unsigned short* __restrict__ Bb) {
        int op = 0;
        auto mem = [&]() {
          __builtin_amdgcn_sched_barrier(PIN);
          if (op < B_G) {
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(bsrc[op] +
                                                                (long long)min(ii + 1, nch - 1) * BK),
                (__attribute__((address_space(3))) void*)(Bn + (wave * B_G + op) * 16 * BK), 16, 0, 0);
          } else if (op < B_G + NA) {
            const int j = op - B_G, rb = j >> 1, jj = j & 1;
            va[u][rb][jj] = *reinterpret_cast<const f32x4*>(xrow[rb] + (long long)la_c * BK +
                                                            jj * ((FL & 8) ? 16 : 4));
            if (j == NA - 1 && la_c + 1 < nch) ++la_c;
          }
          __builtin_amdgcn_sched_barrier(PIN);
          ++op;
        };
        u32x4_t ah[RB], am[RB], al[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) split3(va[u][rb][0], va[u][rb][1], ah[rb], am[rb], al[rb]);
        u32x4_t bf[2][3];
        auto readb = [&](int nb, u32x4_t (&o)[3]) {
          const int row = nb * 16 + r16;
          const int slot = kq ^ ((row >> 2) & 3);
          const unsigned short* bp = Bb + row * BK + slot * 8;
          o[0] = *reinterpret_cast<const u32x4_t*>(bp);
          o[1] = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
          o[2] = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
        };
        if (FL & 1) readb(0, bf[0]);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          u32x4_t cur[3];
          if (FL & 1) {
            if (nb + 1 < NB) readb(nb + 1, bf[(nb + 1) & 1]);
#pragma unroll
            for (int p = 0; p < 3; ++p) cur[p] = bf[nb & 1][p];
          } else {
            readb(nb, cur);
          }
          const u32x4_t bh = cur[0], bm = cur[1], bl = cur[2];
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            f32x4 c = acc[rb][nb];
            c = mfma16(ah[rb], bh, c);
            c = mfma16(ah[rb], bm, c);
            c = mfma16(am[rb], bh, c);
            c = mfma16(ah[rb], bl, c);
            c = mfma16(al[rb], bh, c);
            c = mfma16(am[rb], bm, c);
            acc[rb][nb] = c;
          }
          if (FL & 4) {
            if (nb < NB / 2) { mem(); mem(); if (nb == NB / 2 - 1) while (op < B_G + NA) mem(); }
          } else {
            mem();
            if (nb >= NB - (B_G + NA - NB)) mem();
          }
        }
        while (op < B_G + NA) mem();
      });
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wave * RB * 16 + rb * 16 + kq * 4 + r;
        if (row < a.M) C[(long long)row * a.N + n0 + nb * 16 + r16] = acc[rb][nb][r];
      }
}


// k16r: three-stage B ring, B DMA two chunks ahead, A in registers D chunks
// ahead (D buffers), one counted wait (vmcnt = the ops of the previous chunk)
// + barrier per chunk; 72 KB LDS: two blocks per CU.
template <int D, int FL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k16r(Args a) {
  constexpr int RB = 2, NW = 4, BN = 128, NB = BN / 16, BM = NW * RB * 16;
  constexpr int B_G = 3 * BN / 16 / NW;
  constexpr int BSTAGE = 3 * BN * BK;  // u16
  constexpr int NA = 2 * RB;
  constexpr int NOPS = B_G + NA;
  __shared__ __attribute__((aligned(16))) unsigned short Bs[3 * BSTAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  {
    const int nwg = a.nwg, q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const long long z = blockIdx.y;
  const float* A = a.A + z * a.M * a.K;
  const unsigned short* Bp = a.Bp + z * 3LL * a.N * a.K;
  float* C = a.C + z * a.M * a.N;
  const int tm = bid / a.tiles_n, tn = bid - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int r16 = lane & 15, kq = lane >> 4;
  const float* xrow[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
    xrow[rb] = A + (long long)min(m0 + wave * RB * 16 + rb * 16 + r16, a.M - 1) * a.K +
               ((FL & 8) ? kq * 4 : kq * 8);
  const unsigned short* bsrc[B_G];
#pragma unroll
  for (int i = 0; i < B_G; ++i) {
    const int pr = (wave * B_G + i) * 16 + (lane >> 2);
    const int plane = pr / BN, row = pr - plane * BN;
    const int ks = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[i] = Bp + (long long)plane * a.N * a.K + (long long)(n0 + row) * a.K + ks * 8;
  }
  const int nch = a.K / BK;
  f32x4 acc[RB][NB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 va[D][RB][2];
  auto aload = [&](int c, int rb, int jj) -> f32x4 {
    return *reinterpret_cast<const f32x4*>(xrow[rb] + (long long)min(c, nch - 1) * BK +
                                           jj * ((FL & 8) ? 16 : 4));
  };
  auto bdma = [&](int c, int i, unsigned short* st) {
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(bsrc[i] + (long long)min(c, nch - 1) * BK),
        (__attribute__((address_space(3))) void*)(st + (wave * B_G + i) * 16 * BK), 16, 0, 0);
  };
  // prologue: B chunks 0, 1 and A chunks 0 .. D-1, in the per-chunk op order
#pragma unroll
  for (int c = 0; c < (D > 2 ? D : 2); ++c) {
    __builtin_amdgcn_sched_barrier(NO_VMEM);
    if (c < 2)
#pragma unroll
      for (int i = 0; i < B_G; ++i) bdma(c, i, Bs + c * BSTAGE);
    if (c < D)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int j = 0; j < 2; ++j) va[c][rb][j] = aload(c, rb, j);
  }
  __builtin_amdgcn_sched_barrier(NO_VMEM);
  for (int i = 0; i < nch; i += 3 * D) {
#pragma unroll
    for (int u = 0; u < 3 * D; ++u) {
      const int ii = i + u;
      if (ii >= nch) break;
      __builtin_amdgcn_sched_barrier(NO_VMEM);
      // chunk ii's B (issued two chunks back) and A (D back) landed: everything
      // but the previous chunk's ops; LDS reads of this wave done too
      __builtin_amdgcn_s_waitcnt((NOPS & 15) | (7 << 4) | (0 << 8) | ((NOPS >> 4) << 14));
      __builtin_amdgcn_s_barrier();
      const int sr = u % 3, sw = (u + 2) % 3;
      overlap2(Bs + sw * BSTAGE, Bs + sr * BSTAGE,
               [&](unsigned short* __restrict__ Bn, const unsigned short* __restrict__ Bb) {
        u32x4_t ah[RB], am[RB], al[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) split3(va[u % D][rb][0], va[u % D][rb][1], ah[rb], am[rb], al[rb]);
        int op = 0;
        auto mem = [&]() {
          __builtin_amdgcn_sched_barrier(PIN);
          if (op < B_G) {
            bdma(ii + 2, op, Bn);
          } else if (op < NOPS) {
            const int j = op - B_G, rb = j >> 1, jj = j & 1;
            va[u % D][rb][jj] = aload(ii + D, rb, jj);
          }
          __builtin_amdgcn_sched_barrier(PIN);
          ++op;
        };
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const int row = nb * 16 + r16;
          const int slot = kq ^ ((row >> 2) & 3);
          const unsigned short* bp = Bb + row * BK + slot * 8;
          const u32x4_t bh = *reinterpret_cast<const u32x4_t*>(bp);
          const u32x4_t bm = *reinterpret_cast<const u32x4_t*>(bp + BN * BK);
          const u32x4_t bl = *reinterpret_cast<const u32x4_t*>(bp + 2 * BN * BK);
#pragma unroll
          for (int rb = 0; rb < RB; ++rb) {
            f32x4 c = acc[rb][nb];
            c = mfma16(ah[rb], bh, c);
            c = mfma16(ah[rb], bm, c);
            c = mfma16(am[rb], bh, c);
            c = mfma16(ah[rb], bl, c);
            c = mfma16(al[rb], bh, c);
            c = mfma16(am[rb], bm, c);
            acc[rb][nb] = c;
          }
          while (op < (nb + 1) * NOPS / NB) mem();
        }
        while (op < NOPS) mem();
      });
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wave * RB * 16 + rb * 16 + kq * 4 + r;
        if (row < a.M) C[(long long)row * a.N + n0 + nb * 16 + r16] = acc[rb][nb][r];
      }
}

template <class K>
float run(K kern, Args a, int bm, int nb, int reps, int threads = 256) {
  a.tiles_n = a.N / 128;
  a.nwg = (a.M + bm - 1) / bm * a.tiles_n;
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
  {
    std::vector<float> h((size_t)M * K);
    unsigned s = 1;
    for (auto& v : h) {
      s = s * 1664525u + 1013904223u;
      v = (int)(s >> 9) * (1.0f / 4194304.0f) - 1.0f;
    }
    for (int z = 0; z < nb; ++z) CK(hipMemcpy(A + (size_t)z * M * K, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<unsigned short> hb((size_t)nb * 3 * N * K);
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
    printf("%-28s %8.3f ms  %7.1f TF/s fp32-eq  %.3f of 416.7\n", name, ms, fl / ms / 1e9,
           fl / ms / 1e9 / 416.7);
  };
  rep("16x16x32 D1", run(k16<1, 0>, a, 128, nb, reps));
  rep("ring3 D2", run(k16r<2, 0>, a, 128, nb, reps));
  rep("ring3 D2 contiguous-A", run(k16r<2, 8>, a, 128, nb, reps));
  rep("ring3 D3", run(k16r<3, 0>, a, 128, nb, reps));
  rep("16x16x32 D1 contiguous-A", run(k16<1, 8>, a, 128, nb, reps));
  rep("16x16x32 D1 again", run(k16<1, 0>, a, 128, nb, reps));
  rep("ring3 D2 again", run(k16r<2, 0>, a, 128, nb, reps));
  return 0;
}
