// pk_hazard.hip -- does a packed-fp32 VOP3P instruction whose destination pair
// is also a source pair, read cross-half by op_sel / op_sel_hi, compute what the
// ISA says on gfx950?  (up4tap_gcombine_kernel's y interpolation gave
// run-to-run different low results in lanes 48-63 on
//   v_pk_fma_f32 v[68:69], v[68:69], s[10:11], v[84:85] op_sel:[1,0,0]
// DESIGN.md 4.1q.)  Each case runs the instruction by inline asm on every lane
// of many waves, with a dependent VALU producer right before it, and counts
// lanes whose result differs from the host formula.  Not part of the library.
// Build: tools/probe/build.sh; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

// case 0: dst == src0, op_sel:[1,0,0]   lo = x.hi*c.lo + a.lo, hi = x.hi*c.hi + a.hi
// case 1: dst == src0, op_sel_hi:[0,1,1] lo = x.lo*c.lo + a.lo, hi = x.lo*c.hi + a.hi
// case 2: dst == src1, op_sel_hi:[1,0,1] lo = a.lo*x.lo + b.lo, hi = a.hi*x.lo + b.hi
// case 3: dst != srcs, op_sel:[1,0,0] (control)
// case 4: v_pk_mul_f32 dst == src1, op_sel_hi:[1,0]: lo = a.lo*x.lo, hi = a.hi*x.lo
// case 5: v_pk_add_f32 dst == src0, op_sel:[1,0]: lo = x.hi + a.lo, hi = x.hi + a.hi
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
// MF: 0 no MFMA; 1 the same wave keeps MFMAs in flight between the packed ops;
// 2 the partner waves on the same SIMDs (waves 4-7 of the 512-thread block)
// run MFMA chains while waves 0-3 run the packed ops
template <int CASE, int MF>
__global__ __launch_bounds__(512) void kern(const float* in, float* out, int reps, float* sink) {
  const int wave = threadIdx.x >> 6;
  if (MF == 2 && wave >= 4) {
    bf8v a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.001f * (threadIdx.x + j)); b[j] = (__bf16)0.5f; }
    f16v c = {};
    for (int r = 0; r < reps * 8; ++r) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    if (c[0] == 12345.f) sink[0] = c[1];
    return;
  }
  const int i = (MF == 2 ? blockIdx.x * 256 : blockIdx.x * blockDim.x) + (threadIdx.x & (MF == 2 ? 255 : 511));
  bf8v ma, mb;
  f16v mc = {};
  if (MF == 1)
    for (int j = 0; j < 8; ++j) { ma[j] = (__bf16)(0.001f * (threadIdx.x + j)); mb[j] = (__bf16)0.5f; }
  f2 x = {in[4 * i], in[4 * i + 1]};
  f2 a = {in[4 * i + 2], in[4 * i + 3]};
  float acc0 = 0.f, acc1 = 0.f;
  for (int r = 0; r < reps; ++r) {
    if (MF == 1) mc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ma, mb, mc, 0, 0, 0);
    f2 y = x * 1.0f + (float)r;  // dependent producer right before
    f2 z;
    if (CASE == 0) {
      z = y;
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel:[1,0,0]" : "+v"(z) : "v"(f2{0.5f, 0.25f}), "v"(a));
    } else if (CASE == 1) {
      z = y;
      asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[0,1,1]" : "+v"(z) : "v"(f2{0.5f, 0.25f}), "v"(a));
    } else if (CASE == 2) {
      z = y;
      asm volatile("v_pk_fma_f32 %0, %1, %0, %2 op_sel_hi:[1,0,1]" : "+v"(z) : "v"(a), "v"(f2{0.5f, 0.25f}));
    } else if (CASE == 3) {
      asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0]" : "=v"(z) : "v"(y), "v"(f2{0.5f, 0.25f}), "v"(a));
    } else if (CASE == 4) {
      z = y;
      asm volatile("v_pk_mul_f32 %0, %1, %0 op_sel_hi:[1,0]" : "+v"(z) : "v"(a));
    } else if (CASE == 5) {
      z = y;
      asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[1,0]" : "+v"(z) : "v"(a));
    } else if (CASE == 6) {  // SGPR pair src1, high half rewritten by SALU right before
      z = y;
      asm volatile(
          "s_mov_b32 s40, 0x3f000000\n s_mov_b32 s41, 0x3e800000\n"
          "v_pk_fma_f32 %0, %0, s[40:41], %1 op_sel:[1,0,0]"
          : "+v"(z) : "v"(a) : "s40", "s41");
    } else if (CASE == 7) {  // SGPR pair: read (hi unused), SALU rewrites hi, read hi
      z = y;
      f2 w = y;
      asm volatile(
          "s_mov_b32 s40, 0x3f000000\n s_mov_b32 s41, 0x40400000\n"
          "v_pk_fma_f32 %1, %1, s[40:41], %2 op_sel_hi:[1,0,1]\n"
          "s_mov_b32 s41, 0x3e800000\n"
          "v_pk_fma_f32 %0, %0, s[40:41], %2 op_sel:[1,0,0]"
          : "+v"(z), "+v"(w) : "v"(a) : "s40", "s41");
      z += w * 0.f;
    } else if (CASE == 8) {  // the gcombine sequence: dst == src0 after two reads of it
      z = y;
      f2 o = a, p = a;
      asm volatile(
          "s_mov_b32 s40, 0x3f000000\n s_mov_b32 s41, 0x3e800000\n"
          "v_pk_fma_f32 %1, %0, s[40:41], %1 op_sel_hi:[0,0,1]\n"
          "v_pk_fma_f32 %2, %0, s[40:41], %2 op_sel_hi:[0,1,1]\n"
          "v_pk_fma_f32 %0, %0, s[40:41], %1 op_sel:[1,0,0]"
          : "+v"(z), "+v"(o), "+v"(p) : : "s40", "s41");
      z += p * 0.f;
    } else {  // control for 8 with a fresh destination
      f2 o = a, p = a;
      asm volatile(
          "s_mov_b32 s40, 0x3f000000\n s_mov_b32 s41, 0x3e800000\n"
          "v_pk_fma_f32 %1, %3, s[40:41], %1 op_sel_hi:[0,0,1]\n"
          "v_pk_fma_f32 %2, %3, s[40:41], %2 op_sel_hi:[0,1,1]\n"
          "v_pk_fma_f32 %0, %3, s[40:41], %1 op_sel:[1,0,0]"
          : "=&v"(z), "+v"(o), "+v"(p) : "v"(y) : "s40", "s41");
      z += p * 0.f;
    }
    acc0 += z.x;
    acc1 += z.y;
    x.x = x.x * 1.0000001f;
  }
  out[2 * i] = acc0;
  out[2 * i + 1] = acc1;
  if (MF == 1 && mc[0] == 12345.f) sink[0] = mc[1];
}

template <int CASE>
void host_ref(const std::vector<float>& in, std::vector<float>& out, int n, int reps) {
  for (int i = 0; i < n; ++i) {
    float xl = in[4 * i], xh = in[4 * i + 1], al = in[4 * i + 2], ah = in[4 * i + 3];
    float acc0 = 0.f, acc1 = 0.f;
    for (int r = 0; r < reps; ++r) {
      float yl = xl * 1.0f + (float)r, yh = xh * 1.0f + (float)r, zl, zh;
      if (CASE == 0) { zl = __builtin_fmaf(yh, 0.5f, al); zh = __builtin_fmaf(yh, 0.25f, ah); }
      else if (CASE == 1) { zl = __builtin_fmaf(yl, 0.5f, al); zh = __builtin_fmaf(yl, 0.25f, ah); }
      else if (CASE == 2) { zl = __builtin_fmaf(al, yl, 0.5f); zh = __builtin_fmaf(ah, yl, 0.25f); }
      else if (CASE == 3) { zl = __builtin_fmaf(yh, 0.5f, al); zh = __builtin_fmaf(yh, 0.25f, ah); }
      else if (CASE == 4) { zl = al * yl; zh = ah * yl; }
      else if (CASE == 5) { zl = yh + al; zh = yh + ah; }
      else if (CASE == 6 || CASE == 7) { zl = __builtin_fmaf(yh, 0.5f, al); zh = __builtin_fmaf(yh, 0.25f, ah); }
      else {  // 8, 9: o = a + y.lo * (0.5, 0.5); z = y.hi * (0.5, 0.25) + o
        float ol = __builtin_fmaf(yl, 0.5f, al), oh = __builtin_fmaf(yl, 0.5f, ah);
        zl = __builtin_fmaf(yh, 0.5f, ol); zh = __builtin_fmaf(yh, 0.25f, oh);
      }
      acc0 += zl;
      acc1 += zh;
      xl = xl * 1.0000001f;
    }
    out[2 * i] = acc0;
    out[2 * i + 1] = acc1;
  }
}

template <int CASE, int MF>
void run(const char* name, int n, int reps, const float* din, float* dout, const std::vector<float>& in,
         float* sink) {
  std::vector<float> ref(2 * n), got(2 * n);
  host_ref<CASE>(in, ref, n, reps);
  int bad_runs = 0, bad_lo = 0, bad_hi = 0, lane_hist[4] = {0, 0, 0, 0};
  for (int it = 0; it < 5; ++it) {
    if (MF == 2)
      hipLaunchKernelGGL((kern<CASE, MF>), dim3(n / 256), dim3(512), 0, 0, din, dout, reps, sink);
    else
      hipLaunchKernelGGL((kern<CASE, MF>), dim3(n / 512), dim3(512), 0, 0, din, dout, reps, sink);
    hipDeviceSynchronize();
    hipMemcpy(got.data(), dout, 8 * n, hipMemcpyDeviceToHost);
    int b = 0;
    for (int i = 0; i < n; ++i)
      for (int h = 0; h < 2; ++h)
        if (memcmp(&got[2 * i + h], &ref[2 * i + h], 4)) {
          ++b;
          (h ? bad_hi : bad_lo)++;
          lane_hist[(i & 63) >> 4]++;
        }
    bad_runs += b != 0;
  }
  printf("MF%d %-44s runs with mismatches %d/5  lo %d hi %d  by lane quarter %d %d %d %d\n", MF, name, bad_runs,
         bad_lo, bad_hi, lane_hist[0], lane_hist[1], lane_hist[2], lane_hist[3]);
}

int main() {
  const int n = 256 * 2048, reps = 64;
  std::vector<float> in(4 * n);
  unsigned s = 12345;
  for (auto& v : in) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xffff) / 4096.f - 8.f; }
  float *din, *dout, *sink;
  (void)hipMalloc(&sink, 64);
  hipMalloc(&din, 16 * n);
  hipMalloc(&dout, 8 * n);
  hipMemcpy(din, in.data(), 16 * n, hipMemcpyHostToDevice);
  run<0, 0>("fma dst==src0 op_sel:[1,0,0]", n, reps, din, dout, in, sink);
  run<1, 0>("fma dst==src0 op_sel_hi:[0,1,1]", n, reps, din, dout, in, sink);
  run<2, 0>("fma dst==src1 op_sel_hi:[1,0,1]", n, reps, din, dout, in, sink);
  run<3, 0>("fma dst!=src op_sel:[1,0,0] (control)", n, reps, din, dout, in, sink);
  run<4, 0>("mul dst==src1 op_sel_hi:[1,0]", n, reps, din, dout, in, sink);
  run<5, 0>("add dst==src0 op_sel:[1,0]", n, reps, din, dout, in, sink);
  run<0, 1>("fma dst==src0 op_sel:[1,0,0]", n, reps, din, dout, in, sink);
  run<1, 1>("fma dst==src0 op_sel_hi:[0,1,1]", n, reps, din, dout, in, sink);
  run<2, 1>("fma dst==src1 op_sel_hi:[1,0,1]", n, reps, din, dout, in, sink);
  run<3, 1>("fma dst!=src op_sel:[1,0,0] (control)", n, reps, din, dout, in, sink);
  run<4, 1>("mul dst==src1 op_sel_hi:[1,0]", n, reps, din, dout, in, sink);
  run<5, 1>("add dst==src0 op_sel:[1,0]", n, reps, din, dout, in, sink);
  run<0, 2>("fma dst==src0 op_sel:[1,0,0]", n, reps, din, dout, in, sink);
  run<1, 2>("fma dst==src0 op_sel_hi:[0,1,1]", n, reps, din, dout, in, sink);
  run<2, 2>("fma dst==src1 op_sel_hi:[1,0,1]", n, reps, din, dout, in, sink);
  run<3, 2>("fma dst!=src op_sel:[1,0,0] (control)", n, reps, din, dout, in, sink);
  run<4, 2>("mul dst==src1 op_sel_hi:[1,0]", n, reps, din, dout, in, sink);
  run<5, 2>("add dst==src0 op_sel:[1,0]", n, reps, din, dout, in, sink);
  run<6, 0>("fma sgpr src1 written just before", n, reps, din, dout, in, sink);
  run<7, 0>("fma sgpr hi rewritten between reads", n, reps, din, dout, in, sink);
  run<8, 0>("gcombine seq dst==src0", n, reps, din, dout, in, sink);
  run<9, 0>("gcombine seq control", n, reps, din, dout, in, sink);
  run<6, 1>("fma sgpr src1 written just before", n, reps, din, dout, in, sink);
  run<7, 1>("fma sgpr hi rewritten between reads", n, reps, din, dout, in, sink);
  run<8, 1>("gcombine seq dst==src0", n, reps, din, dout, in, sink);
  run<9, 1>("gcombine seq control", n, reps, din, dout, in, sink);
  run<6, 2>("fma sgpr src1 written just before", n, reps, din, dout, in, sink);
  run<7, 2>("fma sgpr hi rewritten between reads", n, reps, din, dout, in, sink);
  run<8, 2>("gcombine seq dst==src0", n, reps, din, dout, in, sink);
  run<9, 2>("gcombine seq control", n, reps, din, dout, in, sink);
  return 0;
}
