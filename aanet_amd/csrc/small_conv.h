// small_conv.h -- internal interface of the direct few-channel convolution (small_conv.hip),
// dispatched from aanet_conv2d_fused_f32 (mdcn.hip) for the shapes it takes.
#pragma once

#include "common.h"

struct DirectArgs {
  const float *x;       // [N][C][H][W] (in_nhwc: [N][H][W][C])
  const float *w;       // [Co][C][k][k], or packed [k][k][Co][C] (packed != 0)
  const float *bias, *post_scale, *post_shift, *residual;  // residual: out's shape
  float *out;           // [N][Co][Ho][Wo]
  int act, packed, in_nhwc;
  int N, C, H, W, Co, Ho, Wo, pad;
};

// refine_stem_kernel (aanet_refine_stem_f32)
struct StemArgs {
  const float *warped, *left, *disp;   // [N][3][H][W], [N][3][H][W], [N][1][H][W]
  const float *w1, *b1, *w2, *b2;      // [16][6][3][3], [16], [16][1][3][3], [16] (BN folded)
  float *out;                          // [N][H][W][32]
  int act, N, H, W;
};

// AANET_OK, AANET_EUNSUPPORTED (no instance for the shape: the caller runs the engine), or a
// positive hipError_t.  y = act(post_scale*(conv + bias) + post_shift + residual).
int conv_direct_launch(const DirectArgs &a, int k, int stride, int dil, hipStream_t st);
