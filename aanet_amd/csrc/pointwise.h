// pointwise.h -- internal interface of the streaming 1x1 convolution (pointwise.hip).  Not part
// of the C ABI: mdcn.hip's conv engine launcher (aanet_conv2d_fused_f32) dispatches here when the
// conv is 1x1 / stride 1 / no padding / one group, with split-bf16 weight fragments, C in {32, 64}
// and Co <= 64 ("1x1 convolutions").
#pragma once

#include "common.h"

struct PwArgs {
  const float *x;          // [N][C][P] (in_nhwc: [N][P][C])
  const void *wsplit;      // split-bf16 A fragments (aanet_conv_weight_pack_split_f32), 1x1
  const float *bias, *post_scale, *post_shift, *residual;  // residual: out's layout
  int act;
  float *out;              // [N][Co][P] (out_nhwc: [N][P][Co])
  int N, C, P, Co, in_nhwc, out_nhwc;
};

// 1 when pw_conv_launch takes the shape (np = N*P pixels, p = P pixels per image).
int pw_conv_supported(int c, int co, int kh, int kw, int stride, int pad, int groups, long np,
                      int out_nhwc, int p);
int pw_conv_launch(const PwArgs &a, hipStream_t stream);
