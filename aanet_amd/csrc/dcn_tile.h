// dcn_tile.h -- internal interface of the LDS-window deformable bottleneck tail (dcn_tile.hip).
// Not part of the C ABI: mdcn.hip's aanet_mdcn_pw_f32 launcher dispatches here when the shape
// fits ("DCN tail, window form").
#pragma once

#include "common.h"

struct DcnTileArgs {
  const float *x;        // conv1 output, channels-last [N][H][W][C] (or NCHW: x_nchw)
  const float *offset;   // offset_conv output planes (NCHW), offsets of group g, tap k at 2(gK+k)
  long off_bs;
  const float *mask;     // mask logits (or values) plane g*K + k
  long mask_bs;
  int mask_logits;
  float mask_scale;
  const void *wsplit;    // DCN weight, pre-split bf16 fragments (aanet_conv_weight_pack_split_f32)
  const float *bias;     // DCN bias or NULL
  const float *post_scale, *post_shift;  // BN2 (folded) or NULL
  int act;
  const void *tail_wsplit;  // conv3 weight fragments
  const float *tail_b;
  int tail_act;
  const float *residual;    // block input (NCHW, Co2 channels) or NULL
  float *out;               // NCHW [N][Co2][H][W]
  float *csa_out;           // cross-scale sum output or NULL
  const float *up[2];
  int up_h[2], up_w[2], up_r[2], num_up, csa_act;
  // optional post stage on the block's branch output v (csa_out's values when csa_out is set,
  // else out's): the next pointwise conv of the path, so its input never makes a second HBM trip
  //   t = post_w . v + post_b   (post_w: pre-split fragments of a [64][64] 1x1 weight, BN folded)
  //   post_out (channels-last [N][H][W][64]) = post_act(t)          -- the next module's conv1
  //   post_disp ([N][H][W]) = sum_d d softmax_d(t)                  -- final_conv + regression
  // (either output may be NULL; needs Co2 == 64)
  const void *post_wsplit;
  const float *post_b;
  int post_act;
  float *post_out;
  float *post_disp;
  int post_skip;  // the post stage's outputs only (out / csa_out not stored)
  int N, C, H, W, Co, Co2, dil, dg;
  int x_nchw;  // x is NCHW [N][C][H][W] (plain form only)
  int plain;   // op-level DCN: out = act(post_scale*(DCN + bias) + post_shift), NCHW; no tail
  int dbg;  // AANET_DCN_DBG timing-attribution switches (wrong results; tools/dcn_tile_bench.py)
};

// AANET_OK, AANET_EUNSUPPORTED (shape outside the window kernel: caller uses the generic engine),
// or a positive hipError_t.
int dcn_tile_launch(const DcnTileArgs &a, hipStream_t stream);
// 1 when the window kernel takes this shape (3x3, stride 1, pad = dil = 2, C = Co = Co2 = 64 or
// 32, two deformable groups, W % 4 == 0).
int dcn_tile_supported(int c, int co, int co2, int kh, int kw, int stride, int pad, int dil,
                       int dg, int groups, int w);
