// dcn_small.h -- internal interface of the few-channel deformable conv (dcn_small.hip).
// Not part of the C ABI: mdcn.hip's aanet_mdcn_pw_f32 / aanet_mdcn_fwd_fused_f32 launchers
// dispatch here when the shape fits.
#pragma once

#include "common.h"

struct DcnSmallArgs {
  const float *x;        // NCHW [N][16][H][W]
  const float *offset;   // offset planes (NCHW), group g, tap k at 2(gK+k) (h) and 2(gK+k)+1 (w)
  long off_bs;
  const float *mask;     // mask logits (or values), plane gK + k
  long mask_bs;
  int mask_logits;
  float mask_scale;
  const float *w;        // DCN weight, packed fp32 [k][co][c] (aanet_conv_weight_pack_f32) or raw
  int packed;            // [co][c][kh][kw] (packed = 0; op-level form only)
  const float *bias;     // DCN bias or NULL
  const float *post_scale, *post_shift;  // BN2 (folded) or NULL
  int act;
  const float *tail_w;   // conv3 1x1 weight, packed [co2][c] (BN3 folded), or NULL: op-level DCN
  const float *tail_b;
  int tail_act;
  const float *residual; // block input (NCHW, Co2 channels) or NULL
  float *out;            // NCHW [N][16][H][W]
  int N, C, H, W, Co, Co2, pad, dil, dg;
};

// AANET_OK, AANET_EUNSUPPORTED (not C = Co (= Co2) = 16, two deformable groups, 3x3, stride 1,
// pad = dil: the caller runs the generic engine), or a positive hipError_t.
int dcn_small_launch(const DcnSmallArgs &a, hipStream_t stream);
int dcn_small_supported(int c, int co, int co2, int kh, int kw, int stride, int pad, int dil,
                        int dg, int groups);
