// common.h -- shared helpers for the gfx950 kernels of libposfeat_hip.so
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/posfeat_hip.h"

#define PF_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define PF_CHECK_LAUNCH()                                  \
  do {                                                     \
    hipError_t _e = hipGetLastError();                     \
    if (_e != hipSuccess) return POSFEAT_E_HIP;            \
  } while (0)

#define PF_TRY(expr)                  \
  do {                                \
    int _r = (expr);                  \
    if (_r != POSFEAT_OK) return _r;  \
  } while (0)

// The arithmetic of the MFMA launches a timing label covers (bench.py prices
// each roofline against the ceiling of the arithmetic its kernel runs): the
// conv / weight-gradient launchers OR their mode into the calling thread's
// mask; the timed() helpers clear it before a label's launches and read it
// after (posfeat_*_timing_event_arith).
enum { PF_ARITH_FP32 = 1, PF_ARITH_BF6 = 2 };
int &pf_arith_mask();
static inline void pf_note_arith(int a) { pf_arith_mask() |= a; }

// Kernels built without packed-fp32 VALU ops (v_pk_fma/mul/add_f32,
// v_pk_mov_b32 on fp32 pairs).  The compiler forms them from scalar code and
// sometimes lets a packed op read, cross-half, a register pair it also writes
// (the low result from the high dword of its own destination): the form that
// gave run-to-run different results in lanes 48-63 on gfx950 (DESIGN.md
// 4.1r).  tools/isa_check.py fails every such op in the shipped library;
// kernels whose compiled code held one carry this attribute (device side
// only: the host compile ignores it, hence the diagnostic off).
#pragma clang diagnostic ignored "-Wignored-attributes"
#define PF_NO_PK_FP32 __attribute__((target("no-packed-fp32-ops")))

static inline hipStream_t pf_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

static inline size_t pf_align(size_t x, size_t a) { return (x + a - 1) / a * a; }

// __syncthreads / __shfl / __shfl_xor (width 64) as always-inline code: the
// HIP runtime's versions are plain inline functions, which a kernel built
// without packed-fp32 ops (PF_NO_PK_FP32) does not inline -- they became
// device-function calls there (tools/isa_check.py fails any s_swappc).  Same
// instructions as the runtime's: fence + s_barrier + fence; ds_bpermute.
__device__ __forceinline__ void pf_syncthreads() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ int pf_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
template <class T>
__device__ __forceinline__ T pf_bperm(T v, int addr) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte lanes");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, v)));
  } else {
    typedef int i2 __attribute__((ext_vector_type(2)));
    i2 w = __builtin_bit_cast(i2, v);
    w.x = __builtin_amdgcn_ds_bpermute(addr, w.x);
    w.y = __builtin_amdgcn_ds_bpermute(addr, w.y);
    return __builtin_bit_cast(T, w);
  }
}
template <class T>
__device__ __forceinline__ T pf_shfl_xor(T v, int mask, int width = 64) {
  (void)width;  // whole waves only (every caller passes 64)
  return pf_bperm(v, (pf_lane() ^ mask) << 2);
}
template <class T>
__device__ __forceinline__ T pf_shfl(T v, int src, int width = 64) {
  (void)width;
  return pf_bperm(v, (src & 63) << 2);
}

__device__ __forceinline__ float pf_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += pf_shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float pf_elu(float x) { return x > 0.f ? x : expm1f(x); }

// torch softplus(beta=1, threshold=20)
__device__ __forceinline__ float pf_softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// order-preserving uint32 key of a float (+0 == -0)
__device__ __forceinline__ uint32_t pf_fkey(float v) {
  uint32_t u = __float_as_uint(v + 0.0f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ---- bf16x6 operand split (conv.hip BF6 tiles, gemm6.hip) -----------------
// x = h + m + l exactly up to 2^-27 |x|: h = RNE_bf16(x), m = RNE_bf16(x - h),
// l = RNE_bf16(x - h - m) (both differences exact in fp32).
// Two RNE conversions packed into one dword: hipcc emits ONE v_cvt_pk_bf16_f32
// for this.  Never an inline-asm v_cvt_pk_bf16_f32: the compiler's hazard
// recognizer does not see an asm's VGPR write as a VALU write, so it put no
// wait states between it and an MFMA reading the result as SrcA / SrcB --
// the MFMA then read the register's previous value whenever the schedule
// placed it right behind the conversion (timing-dependent, nondeterministic
// results: conv_glds_kernel<128,64,..,BF6> once its loop was rescheduled, and
// round 2's bf16x6 stem variant; tools/tile_sweep.py).
typedef __bf16 pf_bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pf_cvt_pk_bf16(float lo, float hi) {
  const pf_bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ void pf_split3_pair(float a, float b, unsigned& h, unsigned& m,
                                               unsigned& l) {
  h = pf_cvt_pk_bf16(a, b);
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  m = pf_cvt_pk_bf16(ra, rb);
  const float sa = ra - __uint_as_float(m << 16), sb = rb - __uint_as_float(m & 0xffff0000u);
  l = pf_cvt_pk_bf16(sa, sb);
}
// 4 floats -> 4 bf16 of each plane (uint2 = elements 0..3 in order)
__device__ __forceinline__ void pf_split3x4(const f32x4& v, uint2& h, uint2& m, uint2& l) {
  pf_split3_pair(v.x, v.y, h.x, m.x, l.x);
  pf_split3_pair(v.z, v.w, h.y, m.y, l.y);
}

// one v_mfma_f32_32x32x16_bf16 on 8 bf16 per lane of each operand, given as
// packed dwords (gfuse.hip, up4tap.hip): g6_split turns 8 fp32 into the three
// planes' operands
typedef __bf16 g6_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned g6_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void g6_split(const f32x4& p0, const f32x4& p1, g6_u32x4& h,
                                         g6_u32x4& m, g6_u32x4& l) {
  uint2 h0, m0, l0, h1, m1, l1;
  pf_split3x4(p0, h0, m0, l0);
  pf_split3x4(p1, h1, m1, l1);
  h = g6_u32x4{h0.x, h0.y, h1.x, h1.y};
  m = g6_u32x4{m0.x, m0.y, m1.x, m1.y};
  l = g6_u32x4{l0.x, l0.y, l1.x, l1.y};
}
__device__ __forceinline__ f32x16 g6_mfma(const g6_u32x4& a, const g6_u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(g6_bf16x8, a),
                                                 __builtin_bit_cast(g6_bf16x8, b), c, 0, 0, 0);
}

// value of the x2 bilinear upsample (align_corners=True, F.interpolate as
// DescNet.py:187 calls it) of an h x w NHWC map at output pixel (oy, ox), 4
// channels from `base` (= map + image offset + channel offset); sh, sw =
// (h-1)/(2h-1), (w-1)/(2w-1).  Shared by the upsample kernel and the Winograd
// input transform that reads the low-res map directly: the same arithmetic.
// A/B switches.  The paths that lost their A/B (bf6d / bf6b dense tiles for
// extraction, precision mode 2, the unfused head, the Winograd / phase forms
// of head.conv2, the dense DiskLoss, ...) are selected by POSFEAT_* variables
// that only the A/B build reads (`make ab` -> libposfeat_hip_ab.so, built with
// -DPOSFEAT_AB=1); the shipped library ignores them and always runs the
// default paths.  Operational variables (POSFEAT_AUTOTUNE, _AUTOTUNE_LOG,
// _CONV_TILE: a legal tile forced for the tile tests) use getenv directly.
#ifndef POSFEAT_AB
#define POSFEAT_AB 0
#endif
inline const char* pf_ab_getenv(const char* name) {
#if POSFEAT_AB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// XCD-aware bijective block remap: the hardware deals consecutive
// workgroups round-robin over the 8 XCDs (XCD = bid & 7); XCD x gets the
// contiguous logical range [x q + min(x, r), ...) of the nwg blocks, so
// blocks that read the same data (e.g. one image's points) share one XCD's L2
// sum_{k < n} p[k stride] in k order (the same bits as the plain loop), with
// 8 loads in flight per trip: a loop that adds each load before issuing the
// next waits one memory latency per term (the split-K reductions were
// latency-bound that way)
__device__ __forceinline__ float pf_ordered_sum(const float* __restrict__ p, long long stride,
                                                int n) {
  float s = 0.f;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(long long)(k + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < n; ++k) s += p[(long long)k * stride];
  return s;
}

// (pixel, channel quad) of flat quad index i: 32-bit division whenever i fits
// (every map here does); a 64-bit divide is a ~50-instruction sequence per
// element, enough to leave an elementwise pass VALU-bound
__device__ __forceinline__ int pf_quad_split(long long i, int c4n, long long& p) {
  if ((unsigned long long)i <= 0xffffffffULL) {
    const unsigned iu = (unsigned)i, pu = iu / (unsigned)c4n;
    p = pu;
    return (int)(iu - pu * (unsigned)c4n);
  }
  p = i / c4n;
  return (int)(i - p * c4n);
}

// (b, ty, tx, q) of flat index i over [n][th][tw][c4n]: 32-bit divisions
// whenever i fits (a 64-bit divide is a ~50-instruction sequence per thread)
__device__ __forceinline__ int pf_tile_split(long long i, int c4n, int tw, int th, int& q, int& tx,
                                             int& ty) {
  if ((unsigned long long)i <= 0xffffffffULL) {
    const unsigned iu = (unsigned)i, t = iu / (unsigned)c4n, r = t / (unsigned)tw,
                   b = r / (unsigned)th;
    q = (int)(iu - t * (unsigned)c4n);
    tx = (int)(t - r * (unsigned)tw);
    ty = (int)(r - b * (unsigned)th);
    return (int)b;
  }
  const long long t = i / c4n, r = t / tw;
  q = (int)(i - t * c4n);
  tx = (int)(t - r * tw);
  ty = (int)(r % th);
  return (int)(r / th);
}

__device__ __forceinline__ long long pf_xcd_block(long long bid, long long nwg) {
  const long long q = nwg >> 3, r = nwg & 7, xcd = bid & 7, slot = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

__device__ __forceinline__ f32x4 pf_up2ac_at(const float* base, int h, int w, int cs, float sh,
                                             float sw, int oy, int ox) {
#pragma clang fp contract(off)  // one fixed mul/add sequence wherever it is inlined
  const float ry = sh * oy, rx = sw * ox;
  const int y0 = (int)ry, x0 = (int)rx;
  const int y1 = y0 + (y0 < h - 1 ? 1 : 0), x1 = x0 + (x0 < w - 1 ? 1 : 0);
  const float ly = ry - y0, lx = rx - x0, hy = 1.f - ly, hx = 1.f - lx;
  const f32x4 v00 = *reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x0) * cs);
  const f32x4 v01 = *reinterpret_cast<const f32x4*>(base + ((long long)y0 * w + x1) * cs);
  const f32x4 v10 = *reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x0) * cs);
  const f32x4 v11 = *reinterpret_cast<const f32x4*>(base + ((long long)y1 * w + x1) * cs);
  return hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
}
