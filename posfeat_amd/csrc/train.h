// train.h -- internal (non-ABI) launchers of the keypoint-head backward (train.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../../include/posfeat_hip.h"

// dW [Cout][Kpad] (engine-packed K order) and db [Cout] of a conv with
// padding (K-1)/2 and stride 1 or 2 over an H x W input (dy at the output
// size): dw = sum_p dy[p] (x) im2col(x)[p].  Cin % 32 == 0 or Cin == 4.
// acc != 0 adds to dw / db instead of overwriting them.
size_t pf_conv_wgrad_ws_bytes(int n, int H, int W, int Cin, int Cout, int KH, int KW, int stride);
int pf_conv_wgrad(const float* dy, int ldy, const float* x, int xcs, int n, int H, int W, int Cin,
                  int Cout, int KH, int KW, int stride, float* dw, float* db, int acc, void* ws,
                  size_t ws_bytes, hipStream_t st);
// packed weights of the input-gradient conv (flipped taps, cin <-> cout)
// planes (optional): wt also as three bf16 planes (pf_split3_rows' layout:
// pitch = wt's row length, plane stride = its element count)
int pf_dgrad_weights(const float* w, int Cout, int Cin, int KH, int KW, float* wt, hipStream_t st,
                     unsigned short* planes = nullptr);
// adjoint of the bilinear (align_corners=False) resize h x w -> OH x OW over C
// channels: g [nb][OH][OW] (pitch gcs) -> d [nb][h][w] (pitch dcs); t: nb*OH*w*C floats
int pf_up4_adjoint(const float* g, int gcs, int nb, int OH, int OW, int h, int w, int C, float* t,
                   float* d, int dcs, hipStream_t st);
// InstanceNorm (+ optional PReLU) backward: x is the raw conv output (PReLU
// mode, with mean/rstd) or the normalised map (identity mode, slope == NULL,
// mean unused); rstd is always required (dx = rstd (dx^ - E - x^ E'))
size_t pf_in_bwd_ws_bytes(int nb, int hw, int C);
int pf_in_backward(const float* x, int xcs, const float* g, int gcs, int nb, int hw, int C,
                   const float* mean, const float* rstd, const float* slope, float* dx, int dxcs,
                   void* ws, double** slope_part, int* slope_nparts, hipStream_t st);
// Softplus(IN(conv3(PReLU(IN(conv2))))) backward to d(conv2 output)
size_t pf_tail_bwd_ws_bytes(int nb, int hw);
int pf_tail_backward(const float* dlp, const float* y3, const float* m3, const float* r3,
                     const float* c2, int c2cs, const float* m2, const float* r2,
                     const float* slope, const float* w3, int nb, int hw, float* dy3, float* dc2,
                     int dcs, float* dw3, void* ws, double** t2s, int* t2n, hipStream_t st);
int pf_head_scalars(const double* t2s, int n2, const double* c1s, int n1, float* db3,
                    float* dslope, hipStream_t st);
// batched 1x1 weight-gradient GEMMs without split-K (Winograd weight gradient)
int pf_wgrad_gemm_batched(const float* dy, int ldy, long long sdy, const float* x, int xcs,
                          long long sx, int M, int Cin, int Cout, int nb, int nsplit, float* part,
                          float* partb, int zb, hipStream_t st);
