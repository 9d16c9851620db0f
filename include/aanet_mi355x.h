/*
 * aanet_mi355x.h -- C ABI of the MI355X (gfx950) AANet cost-volume hot path.
 *
 * Every entry point:
 *   - takes plain device pointers (fp32, NCHW / NCDHW contiguous unless a stride is given),
 *     sizes as int, and an explicit HIP stream (hipStream_t, passed as aanet_stream_t);
 *   - allocates nothing and never synchronises (graph-capturable); the caller owns buffers;
 *   - returns 0 on success, a negative AANET_E* code for an invalid argument, or a positive
 *     hipError_t for a launch failure.  Nothing is swallowed or only printed.
 *
 * Each function names the reference interface (wuzhongwulidong/aanet, file:line) it replaces.
 */
#ifndef AANET_MI355X_H
#define AANET_MI355X_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *aanet_stream_t; /* identical to hipStream_t */

/* ABI version (aanet_version()).  4: every descriptor struct starts with `struct_size`
 * (round 4; version 1 had none, and aanet_csa_epilogue_t grew a `post` member in round 3 without
 * a way for the library to tell the two layouts apart). */
#define AANET_ABI_VERSION 4

enum {
  AANET_OK = 0,
  AANET_EINVAL = -1,      /* bad size / null pointer / inconsistent shape */
  AANET_EUNSUPPORTED = -2, /* valid for the reference but outside what this build implements */
  AANET_EABI = -3         /* a descriptor's struct_size is not this library's sizeof: the caller
                             was built against another version of this header */
};

/* Activation layouts of the conv engine (the `layout` argument of the fused entry points).
 * NHWC ("channels-last") intermediates let a 32-channel chunk at one position be read as one
 * 128-byte line (8 lanes x 16 B); the bottleneck keeps its conv1 output in NHWC.  NHWC needs
 * packed weights and 32-channel groups (c/groups % 32 == 0, and c/dg % 32 == 0 for the DCN). */
enum {
  AANET_LAYOUT_NCHW = 0,
  AANET_LAYOUT_IN_NHWC = 1,  /* x is [n][h][w][c] */
  AANET_LAYOUT_OUT_NHWC = 2, /* out (and residual) are [n][ho][wo][co] */
  /* Contraction arithmetic flag, OR-ed into `layout`.  Clear (default): where the engine has the
   * configuration (packed weights, 32-channel chunks, >= 32 output channels per group) the
   * 3x3/1x1/deformable contraction runs on the bf16 matrix cores with every fp32 operand split
   * into three bf16 pieces and fp32 accumulation (six piece products; the dropped ones are below
   * 2^-23 of each product), fp32-accurate: against an fp64 reference its error is no larger than
   * the exact f32 MFMA chain's (mdcn.hip, split3).  Set: exact f32 MFMA (v_mfma_f32_16x16x4_f32,
   * bitwise an fp32 fma chain) everywhere. */
  AANET_CONV_EXACT_F32 = 8,
  /* The weight buffers (weight_packed, and pw_weight_packed of the tail kernels) come from
   * aanet_conv_weight_pack_split_f32: the f32 packed weights followed by their bf16 piece
   * fragments.  Without it the engine runs the exact f32 contraction. */
  AANET_CONV_WEIGHTS_SPLIT = 16,
  /* aanet_mdcn_pw_f32 only: run the generic implicit-GEMM engine even where the LDS-window
   * deformable tail (3x3, stride 1, pad = dil = 2, 64 channels in two 32-channel deformable
   * groups, NHWC input, split weights) would take the shape.  Same results to
   * fp32 rounding; for A/B measurements and parity tests. */
  AANET_CONV_GENERIC_DCN = 32
};

int aanet_version(void); /* AANET_ABI_VERSION of the library */
const char *aanet_status_string(int status);

/* ------------------------------------------------------------------ cost volumes ------- */

/* nets/cost.py:40-48 (CostVolume, feature_similarity='correlation').
 * left, right [n, c, h, w] -> out [n, max_disp, h, w];
 * out[b,d,y,x] = (1/c) * sum_c left[b,c,y,x] * right[b,c,y,x-d] for x >= d, else 0. */
int aanet_corr_volume_f32(const float *left, const float *right, float *out, int n, int c, int h,
                          int w, int max_disp, aanet_stream_t stream);

/* Autograd of nets/cost.py:40-48: grad_left / grad_right [n,c,h,w] are OVERWRITTEN. */
int aanet_corr_volume_bwd_f32(const float *left, const float *right, const float *grad_out,
                              float *grad_left, float *grad_right, int n, int c, int h, int w,
                              int max_disp, aanet_stream_t stream);

/* nets/cost.py:31-38 (concat): out [n, 2c, max_disp, h, w]. */
int aanet_concat_volume_f32(const float *left, const float *right, float *out, int n, int c, int h,
                            int w, int max_disp, aanet_stream_t stream);

/* nets/cost.py:22-29 (difference): out [n, c, max_disp, h, w]. */
int aanet_diff_volume_f32(const float *left, const float *right, float *out, int n, int c, int h,
                          int w, int max_disp, aanet_stream_t stream);

/* Autograd of concat / difference: grad_left / grad_right [n,c,h,w] OVERWRITTEN. */
int aanet_concat_volume_bwd_f32(const float *grad_out, float *grad_left, float *grad_right, int n,
                                int c, int h, int w, int max_disp, aanet_stream_t stream);
int aanet_diff_volume_bwd_f32(const float *grad_out, float *grad_left, float *grad_right, int n,
                              int c, int h, int w, int max_disp, aanet_stream_t stream);

/* nets/cost.py:58-76 (CostVolumePyramid, correlation): scale s uses max_disp >> s.
 * Arrays of num_scales device pointers / sizes (host arrays); all scales are enqueued by one
 * call. */
int aanet_corr_pyramid_f32(int num_scales, const float *const *left, const float *const *right,
                           float *const *out, const int *c, const int *h, const int *w, int n,
                           int max_disp, aanet_stream_t stream);

/* ------------------------------------------------------------ disparity regression ----- */

/* nets/estimation.py:13-30 (DisparityEstimation): cost [n, d, h, w] -> disp [n, h, w];
 * disp = sum_i i * softmax_i(negate ? -cost : cost).  d = cost.size(1). */
int aanet_disp_regress_f32(const float *cost, float *disp, int n, int d, int h, int w, int negate,
                           aanet_stream_t stream);

/* Autograd of the above: grad_cost [n, d, h, w] OVERWRITTEN. */
int aanet_disp_regress_bwd_f32(const float *cost, const float *grad_disp, float *grad_cost, int n,
                               int d, int h, int w, int negate, aanet_stream_t stream);

/* ------------------------------------------------------------ disparity warp ----------- */

/* nets/warp.py:41-64 (disp_warp, padding 'border'): img [n, c, h, w], disp [n, 1, h, w] ->
 * warped [n, c, h, w] = img sampled at (x - disp, y) (grid_sample, bilinear, align_corners=True,
 * border padding); valid_mask [n, c, h, w] (or NULL) = 1 where grid_sample of ones with zeros
 * padding is >= 0.9999, else 0.  Both OVERWRITTEN.  h, w >= 2.  The reference's
 * `assert disp.min() >= 0` (warp.py:52) is the caller's: the kernel warps any disparity. */
int aanet_disp_warp_f32(const float *img, const float *disp, float *warped, float *valid_mask,
                        int n, int c, int h, int w, aanet_stream_t stream);

/* Autograd of the warped image: grad_disp [n, 1, h, w] OVERWRITTEN; grad_img [n, c, h, w]
 * (or NULL) ACCUMULATED (caller zeroes; float atomics). */
int aanet_disp_warp_bwd_f32(const float *img, const float *disp, const float *grad_warped,
                            float *grad_disp, float *grad_img, int n, int c, int h, int w,
                            aanet_stream_t stream);

/* ------------------------------------------------------ modulated deformable conv ------ */

/* deform_conv_cuda.cpp:490-569 (modulated_deform_conv_cuda_forward) + kernel.cu:570-633.
 * x [n,c,h,w]; offset [n, dg*2*kh*kw, ho, wo]; mask [n, dg*kh*kw, ho, wo];
 * weight [co, c/groups, kh, kw]; bias [co] or NULL; out [n, co, ho, wo] OVERWRITTEN.
 * ho = (h + 2*pad - (dil*(kh-1)+1)) / stride + 1 (deform_conv.py:174-183). */
int aanet_mdcn_fwd_f32(const float *x, const float *offset, const float *mask, const float *weight,
                       const float *bias, float *out, int n, int c, int h, int w, int co, int kh,
                       int kw, int stride, int pad, int dil, int groups, int dg,
                       aanet_stream_t stream);

/* Eval-mode fused form used by DeformSimpleBottleneck (nets/deform.py:78-97, 216-226):
 *   - offset and mask may be channel slices of one tensor: per-image strides in elements;
 *   - mask_logits != 0: the mask pointer holds pre-sigmoid logits, m = mask_scale*sigmoid(l)
 *     (deform.py:86-89 with double_mask => mask_scale = 2);
 *   - epilogue: y = act(post_scale[co] * (conv + bias[co]) + post_shift[co]); act 0 none,
 *     1 ReLU, 2 LeakyReLU(0.2).  post_scale / post_shift may be NULL (identity);
 *   - weight_packed != 0: weight is in the [kh][kw][co][c/groups] layout produced by
 *     aanet_conv_weight_pack_f32 (coalesced K-chunk loads); 0: reference [co][c/groups][kh][kw];
 *   - layout: AANET_LAYOUT_NCHW or AANET_LAYOUT_IN_NHWC, plus AANET_CONV_WEIGHTS_SPLIT when the
 *     weight is an aanet_conv_weight_pack_split_f32 buffer (split-bf16 contraction).  With split
 *     weights the shapes of aanet_mdcn_window_fwd_supported run the LDS-window kernel (NCHW or
 *     channels-last x, NCHW out); AANET_CONV_GENERIC_DCN forces the generic engine.
 * This is also the op-level forward of the aggregation's DCNs (mask_logits = 0, separate
 * offset / mask tensors): aanet_amd.ops.mdcn_forward packs the weight and calls it. */
int aanet_mdcn_fwd_fused_f32(const float *x, const float *offset, long offset_batch_stride,
                             const float *mask, long mask_batch_stride, int mask_logits,
                             float mask_scale, const float *weight, int weight_packed,
                             const float *bias,
                             const float *post_scale, const float *post_shift, int act, float *out,
                             int n, int c, int h, int w, int co, int kh, int kw, int stride,
                             int pad, int dil, int groups, int dg, int layout,
                             aanet_stream_t stream);

/* 1 when aanet_mdcn_fwd_fused_f32 with split weights runs the LDS-window DCN kernel for this
 * shape (output size = input size): 3x3, stride 1, pad = dil = 2, groups 1, dg 2, c = co = 64 or
 * 32, w % 4 == 0 -- the aggregation's deformable convs (nets/deform.py:216-226). */
int aanet_mdcn_window_fwd_supported(int c, int co, int kh, int kw, int stride, int pad, int dil,
                                    int groups, int dg, int w);

/* Plain convolution on the same implicit-GEMM engine, for the eval fast path of every other
 * conv in the ISA/CSA blocks (nets/deform.py:6-14 conv1x1/conv3x3, nets/deform.py:70-72
 * offset_conv, nets/aggregation.py:354-370 fuse layers, :447 final_conv), which the reference
 * runs through cuDNN.  BN is folded by the caller into weight/bias (or passed as post_scale /
 * post_shift).  y = act(post_scale*(conv(x) + bias) + post_shift + residual); act 0 none,
 * 1 ReLU, 2 LeakyReLU(0.2).  bias / post_* / residual may be NULL; residual has out's shape. */
int aanet_conv2d_fused_f32(const float *x, const float *weight, const float *bias,
                           const float *post_scale, const float *post_shift, const float *residual,
                           int act, int weight_packed, float *out, int n, int c, int h, int w,
                           int co, int kh, int kw, int stride, int pad, int dil, int groups,
                           int layout, aanet_stream_t stream);

/* Cross-scale-aggregation epilogue of a tail kernel (nets/aggregation.py:387-400 for the output
 * branch at the tail's resolution): besides `out`, write
 *   out_csa = act(out + up(up[0]) + ... + up(up[num_up-1]))
 * where up() is F.interpolate(bilinear, align_corners=False) by an exact factor 2 or 4
 * (up_h * r == ho and up_w * r == wo); each up[j] is [n][co2][up_h][up_w].  Needs wo % 4 == 0
 * and num_up <= 2 in this build (AANET_EUNSUPPORTED otherwise; 3 scales give at most 2 terms).
 * act: 0 none, 1 ReLU, 2 LeakyReLU(0.2). */
/* Post stage of the CSA epilogue (round 3): the next pointwise conv of the path applied to the
 * CSA output in the same kernel, so the branch output is not read back from HBM:
 *   t = weight . csa_out + bias                (1x1, 64 -> 64 channels, BN folded by the caller)
 *   out_nhwc[n][y][x][:] = act(t)              -- the next AAModule's bottleneck conv1 + BN1 + ReLU
 *                                                 (nets/deform.py:207-209), channels-last
 *   disp[n][y][x] = sum_d d * softmax_d(t)     -- final_conv (nets/aggregation.py:443-447) +
 *                                                 DisparityEstimation (nets/estimation.py:13-30)
 * weight: an aanet_conv_weight_pack_split_f32 buffer of the [64][64][1][1] weight.  Either output
 * may be NULL.  Tail kernels that cannot run it return AANET_EUNSUPPORTED (the caller then runs
 * the stage as separate kernels). */
typedef struct {
  size_t struct_size; /* sizeof(aanet_post_stage_t); AANET_EABI otherwise */
  const void *weight;
  const float *bias;
  int act;
  float *out_nhwc;
  float *disp;
  int skip_outputs; /* 1: the tail's out / csa out are not stored (only the post stage's are;
                       the last module with disp: nothing else reads them) */
} aanet_post_stage_t;

typedef struct {
  size_t struct_size; /* sizeof(aanet_csa_epilogue_t); AANET_EABI otherwise */
  float *out;
  int num_up;
  const float *up[3];
  int up_h[3], up_w[3];
  int act;
  const aanet_post_stage_t *post; /* optional post stage on out (NULL: none) */
} aanet_csa_epilogue_t;

/* Bottleneck tail fusion (nets/deform.py:171-184 / 223-236 in eval): the pointwise conv3
 * (+ folded BN3) runs in the epilogue of conv2, so the conv2 activation never goes to HBM:
 *   t   = act(post_scale*(conv(x) + bias) + post_shift)                  [co channels]
 *   out = pw_act(pw_weight . t + pw_bias + residual)                     [co2 channels]
 * weight_packed / pw_weight_packed in the aanet_conv_weight_pack_f32 layout ([co2][co] for the
 * pointwise one).  Requires groups == 1, co <= 64, co2 <= 64.  The _mdcn_ form takes the
 * deformable sampler arguments of aanet_mdcn_fwd_fused_f32.  layout: AANET_LAYOUT_NCHW or
 * AANET_LAYOUT_IN_NHWC (the output is NCHW).  csa: optional CSA epilogue (NULL = none). */
int aanet_conv2d_pw_f32(const float *x, const float *weight_packed, const float *bias,
                        const float *post_scale, const float *post_shift, int act,
                        const float *pw_weight_packed, const float *pw_bias,
                        const float *residual, int pw_act, int co2, float *out, int n, int c,
                        int h, int w, int co, int kh, int kw, int stride, int pad, int dil,
                        const aanet_csa_epilogue_t *csa, int layout, aanet_stream_t stream);
int aanet_mdcn_pw_f32(const float *x, const float *offset, long offset_batch_stride,
                      const float *mask, long mask_batch_stride, int mask_logits,
                      float mask_scale, const float *weight_packed, const float *bias,
                      const float *post_scale, const float *post_shift, int act,
                      const float *pw_weight_packed, const float *pw_bias, const float *residual,
                      int pw_act, int co2, float *out, int n, int c, int h, int w, int co,
                      int kh, int kw, int stride, int pad, int dil, int dg,
                      const aanet_csa_epilogue_t *csa, int layout, aanet_stream_t stream);

/* Weight repack for the conv engine: [co][cg][kh][kw] -> [kh][kw][co][cg].  Done once per
 * weight version by the caller (the eval path caches it with the folded BN). */
int aanet_conv_weight_pack_f32(const float *weight, float *weight_packed, int co, int cg, int kh,
                               int kw, aanet_stream_t stream);

/* The data gradient of a conv as a forward conv (train.EngineConv2dFunction): weight [co][cg][kh][kw]
 * of a conv with `groups` -> the aanet_conv_weight_pack_f32 layout of its per-group transposed,
 * spatially flipped weight ([groups*cg][co/groups][kh][kw], i.e. [kh][kw][groups*cg][co/groups])
 * in one launch.  cuDNN's backward-data (the reference's training) has no such caller-side step. */
int aanet_conv_weight_pack_dgrad_f32(const float *weight, float *weight_packed, int co, int cg,
                                     int kh, int kw, int groups, aanet_stream_t stream);

/* Weight buffer for the split-bf16 contraction (AANET_CONV_WEIGHTS_SPLIT): the
 * aanet_conv_weight_pack_f32 layout, then (at a 256-byte aligned offset) every weight split into
 * three bf16 pieces and laid out as MFMA operand fragments (mdcn.hip, split_frag_offset).
 * weight is the reference layout [co][cg][kh][kw] of a conv with `groups` groups; needs
 * cg % 32 == 0.  _bytes returns the buffer size, 0 when unsupported. */
long aanet_conv_weight_pack_split_bytes(int co, int cg, int kh, int kw, int groups);
int aanet_conv_weight_pack_split_f32(const float *weight, void *out, int co, int cg, int kh, int kw,
                                     int groups, aanet_stream_t stream);

/* Cross-scale fusion sum (nets/aggregation.py:387-400): out[n,c,h,w] =
 * act(sum_j resize(inputs[j])), j in input order; inputs whose (in_h, in_w) differ from
 * (h, w) are resized bilinearly with align_corners=False (aggregation.py:395-396).
 * Up to 4 inputs, each [n, c, in_h[j], in_w[j]]. */
int aanet_csa_sum_f32(float *out, int n, int c, int h, int w, int num_inputs,
                      const float *const *inputs, const int *in_h, const int *in_w, int act,
                      aanet_stream_t stream);

/* The CSA down exchange convs (nets/aggregation.py:362-371 in eval: 3x3, stride 2, pad 1, BN
 * folded into weight/bias), several of which may share one input: the output channels
 * [0, co_a) go to out_a ([n][co_a][ho][wo], activation act_a) and [co_a, co) to out_b
 * ([n][co - co_a][ho][wo], act_b), ho = (h + 1) / 2, wo = (w + 1) / 2.  At C2 scale 0 the
 * branch-1 conv (64 -> 32) and the first conv of the branch-2 chain (64 -> 64, LeakyReLU) run
 * as one co = 96 launch that reads the scale-0 block output once.  x is NCHW, c % 32 == 0,
 * co % 16 == 0, co <= 96 (AANET_EUNSUPPORTED otherwise); wsplit: aanet_conv3x3s2_pack_f32 of the
 * [co][c][3][3] weight into aanet_conv3x3s2_pack_bytes(co, c) device bytes.  Split-bf16
 * contraction (fp32-accurate, see AANET_EXACT_F32 above for the arithmetic).  act: 0 none,
 * 1 ReLU, 2 LeakyReLU(0.2). */
size_t aanet_conv3x3s2_pack_bytes(int co, int c);
int aanet_conv3x3s2_pack_f32(const float *w, int co, int c, void *wsplit, aanet_stream_t stream);
int aanet_conv3x3s2_f32(const float *x, const void *wsplit, const float *bias, int n, int c, int h,
                        int w, int co, int co_a, float *out_a, int act_a, float *out_b, int act_b,
                        aanet_stream_t stream);

/* The deformable bottleneck's offset_conv in eval (nets/deform.py:58-60, 76-79: nn.Conv2d(c, co,
 * 3, padding=dil, dilation=dil, groups=groups, bias=True); the reference runs it through
 * cuDNN, deform.py:81 / aggregation.py:418-432): out = conv(x) + bias, x channels-last
 * ([n][h][w][c], the conv1 output the DCN tail reads next), out NCHW [n][co][h][w] (read in
 * place as the offset / mask planes).  c / groups % 32 == 0, co % groups == 0,
 * ceil(co / groups / 16) <= 2 (AANET_EUNSUPPORTED otherwise); the AANet instances are
 * 64 -> 54 with two groups (scale 0) and 32k -> 27 / 54 with one.  wsplit:
 * aanet_conv3x3_grouped_pack_f32 of the [co][c / groups][3][3] weight into
 * aanet_conv3x3_grouped_pack_bytes(co, c, groups) device bytes.  Split-bf16 contraction
 * (fp32-accurate, see AANET_EXACT_F32 above for the arithmetic). */
size_t aanet_conv3x3_grouped_pack_bytes(int co, int c, int groups);
int aanet_conv3x3_grouped_pack_f32(const float *w, int co, int c, int groups, void *wsplit,
                                   aanet_stream_t stream);
int aanet_conv3x3_grouped_nhwc_f32(const float *x, const void *wsplit, const float *bias, int n,
                                   int c, int h, int w, int co, int groups, int dil, float *out,
                                   aanet_stream_t stream);

/* aanet_conv3x3s2_f32 with the CSA sum of output a in its epilogue (aggregation.py:388-400 for an
 * output branch whose finer-scale term is this conv):
 *   out_a = act_a(conv + bias [+ identity] [+ resize(up)])
 * in that order, resize = F.interpolate(up, (ho, wo), mode='bilinear', align_corners=False).
 * x2 (optional, c2 % 32 == 0 channels, same n/h/w as x): a second input whose channels follow
 * x's in the contraction (wsplit packs the [co][c + c2][3][3] weight), so two down terms that
 * land on the same branch are one launch whose output is their sum (C2 branch 2: the 64->16
 * conv of the scale-0 chain and the 32->16 conv from scale 1).  identity: [n][co_a][ho][wo];
 * up: [n][co_a][up_h][up_w].  terms may be NULL (= aanet_conv3x3s2_f32). */
typedef struct aanet_s2_terms {
  size_t struct_size; /* sizeof(aanet_s2_terms_t); AANET_EABI otherwise */
  const float *x2;
  int c2;
  const float *identity;
  const float *up;
  int up_h, up_w;
} aanet_s2_terms_t;
int aanet_conv3x3s2_terms_f32(const float *x, const void *wsplit, const float *bias, int n, int c,
                              int h, int w, int co, int co_a, float *out_a, int act_a,
                              float *out_b, int act_b, const aanet_s2_terms_t *terms,
                              aanet_stream_t stream);

/* ConvTranspose2d(k = 4, stride 2, padding 1) assembly (nets/feature.py:342-376 Conv2x(deconv=True),
 * used by GANetFeature and HourglassRefinement, refinement.py:109-197): the transposed conv runs as
 * one 2x2, pad-1 conv with 4*co phase outputs (ph [n][4co][h+1][w+1], channel 4c + 2a + b; the
 * Python layer's ops.deconv2x); this writes out [n][co + cr][2h][2w] with
 * out[c][2y+a][2x+b] = ph[4c+2a+b][y+a][x+b] for c < co and the skip tensor rem [n][cr][2h][2w]
 * as channels co .. co+cr-1 (the torch.cat of Conv2x.forward; cr = 0: no skip, rem may be NULL). */
int aanet_deconv2x_assemble_f32(const float *ph, const float *rem, float *out, int n, int co, int cr,
                                int h, int w, aanet_stream_t stream);
/* The same assembly written channels-last: out [n][2h][2w][co + cr] (NHWC), for a consumer conv
 * that stages NHWC input (Conv2x's conv2 on the halo tile).  EUNSUPPORTED when co + cr > 496. */
int aanet_deconv2x_assemble_nhwc_f32(const float *ph, const float *rem, float *out, int n, int co,
                                     int cr, int h, int w, aanet_stream_t stream);
/* torch.cat((a, b), 1) of two NCHW tensors [n][ca][h][w], [n][cb][h][w] written channels-last
 * (out [n][h][w][ca + cb]): the concat of a non-transposed Conv2x (nets/feature.py:342-376) for
 * its conv2 on the halo tile.  EUNSUPPORTED for odd h or w or ca + cb > 496 (callers fall back to
 * torch.cat). */
int aanet_concat_nhwc_f32(const float *a, const float *b, float *out, int n, int ca, int cb, int h,
                          int w, aanet_stream_t stream);

/* The warp-error stem of StereoDRNet / Hourglass refinement (nets/refinement.py:92-99, 148-155):
 *   out_nhwc[n][y][x][0:16]  = act(conv3x3([warped - left, left]; w1) + b1)   (conv1, 6 -> 16)
 *   out_nhwc[n][y][x][16:32] = act(conv3x3(disp; w2) + b2)                    (conv2, 1 -> 16)
 * i.e. torch.cat((conv1(cat(warped - left, left)), conv2(disp)), 1) written channels-last.
 * warped, left: [n][3][h][w]; disp: [n][1][h][w]; w1: [16][6][3][3], w2: [16][1][3][3] with the
 * BatchNorms folded by the caller; pad 1, stride 1. */
int aanet_refine_stem_f32(const float *warped, const float *left, const float *disp,
                          const float *w1, const float *b1, const float *w2, const float *b2,
                          int act, float *out_nhwc, int n, int h, int w, aanet_stream_t stream);

/* F.interpolate(x, size=(out_h, out_w), mode='bilinear', align_corners=False) on [planes, in_h,
 * in_w] -> y [planes, out_h, out_w] (aggregation.py:395-396 in training; the loss's upsampling,
 * model.py:115-117): one thread per output element, the reference kernel's stencil and order. */
int aanet_resize_bilinear_f32(const float *x, float *y, long planes, int in_h, int in_w, int out_h,
                              int out_w, aanet_stream_t stream);

/* Backward of F.interpolate(x, size=(out_h, out_w), mode='bilinear', align_corners=False)
 * (aggregation.py:395-396 in training; the loss's upsampling, model.py:115-117):
 * grad_in [planes, in_h, in_w] is OVERWRITTEN with the gather-form sum over grad_out
 * [planes, out_h, out_w] -- fixed summation order, no atomics (bit-reproducible). */
int aanet_resize_bilinear_bwd_f32(const float *grad_out, float *grad_in, long planes, int in_h,
                                  int in_w, int out_h, int out_w, aanet_stream_t stream);

/* deform_conv_cuda.cpp:571-685 (modulated_deform_conv_cuda_backward) + kernel.cu:635-767.
 * grad_x, grad_offset, grad_mask are OVERWRITTEN; grad_weight and grad_bias (may be NULL)
 * ACCUMULATE, as in the reference (cpp:660-671). */
int aanet_mdcn_bwd_f32(const float *x, const float *offset, const float *mask, const float *weight,
                       const float *grad_out, float *grad_x, float *grad_offset, float *grad_mask,
                       float *grad_weight, float *grad_bias, int n, int c, int h, int w, int co,
                       int kh, int kw, int stride, int pad, int dil, int groups, int dg,
                       aanet_stream_t stream);

/* Faster form of aanet_mdcn_bwd_f32 (same contract, float atomics): grad_x is scattered into a
 * caller-owned NHWC workspace (coalesced 128-byte atomic lines) and then transposed into grad_x.
 * `workspace` (device) must hold aanet_mdcn_bwd_ws_workspace_size(...) = n*c*h*w*4 bytes. */
size_t aanet_mdcn_bwd_ws_workspace_size(int n, int c, int h, int w, int co, int kh, int kw,
                                        int stride, int pad, int dil, int groups, int dg);
int aanet_mdcn_bwd_ws_f32(const float *x, const float *offset, const float *mask,
                          const float *weight, const float *grad_out, float *grad_x,
                          float *grad_offset, float *grad_mask, float *grad_weight,
                          float *grad_bias, int n, int c, int h, int w, int co, int kh, int kw,
                          int stride, int pad, int dil, int groups, int dg, void *workspace,
                          size_t workspace_bytes, aanet_stream_t stream);

/* Deterministic form of aanet_mdcn_bwd_f32 (same contract, bit-reproducible run to run):
 *   - grad_x: 64-bit fixed-point atomics. Integer adds are associative, so the sum does not
 *     depend on atomic ordering. The fixed-point scale is a power of two chosen on the device from
 *     max_{c,k} sum_co |W| * max|grad_out| * max|mask|, so there is no host synchronisation.
 *   - grad_weight: partial sums reduced in a fixed order -- per split of the weight kernel, or,
 *     when the window form applies (stride 1 or 2, <= 128 channels per deformable group, <= 9
 *     taps, <= 128 output channels in multiples of 16, C and C/dg multiples of 4), int64
 *     fixed-point sums of every 8x8 output tile's weight-gradient block (order-free).
 * `workspace` (device, caller-owned) must hold aanet_mdcn_bwd_det_workspace_size(...) bytes; with
 * the window form that includes tiles * co * c * kh * kw floats of tile partials
 * (tiles = n * ceil(ho / 8) * ceil(wo / 8)).
 * The atomic col2im of the reference (kernel.cu:688) has no such guarantee. */
size_t aanet_mdcn_bwd_det_workspace_size(int n, int c, int h, int w, int co, int kh, int kw,
                                         int stride, int pad, int dil, int groups, int dg);
int aanet_mdcn_bwd_det_f32(const float *x, const float *offset, const float *mask,
                           const float *weight, const float *grad_out, float *grad_x,
                           float *grad_offset, float *grad_mask, float *grad_weight,
                           float *grad_bias, int n, int c, int h, int w, int co, int kh, int kw,
                           int stride, int pad, int dil, int groups, int dg, void *workspace,
                           size_t workspace_bytes, aanet_stream_t stream);

/* The same backward with the grad_x algorithm chosen explicitly (the _ws / _det entry points use
 * AANET_DCN_BWD_AUTO).  deterministic: 0 = float atomics (workspace of
 * aanet_mdcn_bwd_ws_workspace_size bytes), 1 = fixed point (aanet_mdcn_bwd_det_workspace_size). */
enum {
  AANET_DCN_BWD_AUTO = 0,   /* the window form where it measured faster (stride 1, <= 32
                               channels per deformable group, Co <= 64: the aggregation's DCNs),
                               else global (both modes) */
  AANET_DCN_BWD_GLOBAL = 1, /* one global atomic per (pixel, tap, corner, channel) contribution,
                               the reference's col2im pattern (kernel.cu:635-693), into an NHWC
                               accumulator */
  AANET_DCN_BWD_WINDOW = 2  /* stride 1 or 2, <= 128 channels per deformable group, C and C/dg
                               divisible by 4, <= 9 taps, Co <= 128 and a multiple of 16, and the
                               window's LDS
                               (grows with the dilation) within the CU's 160 KiB: each
                               (8x8 output tile, 16-channel slice) sums its
                               contributions in an int64 fixed-point LDS window and adds the
                               window once -- float atomics (deterministic = 0) or int64 ones
                               (AANET_EUNSUPPORTED for other shapes) */
};
int aanet_mdcn_bwd_algo_f32(const float *x, const float *offset, const float *mask,
                            const float *weight, const float *grad_out, float *grad_x,
                            float *grad_offset, float *grad_mask, float *grad_weight,
                            float *grad_bias, int n, int c, int h, int w, int co, int kh, int kw,
                            int stride, int pad, int dil, int groups, int dg, int deterministic,
                            int algo, void *workspace, size_t workspace_bytes,
                            aanet_stream_t stream);

/* Weight (and bias) gradient of an ordinary convolution -- the wgrad of every nn.Conv2d of the
 * ISA/CSA blocks in training (nets/deform.py:6-14, 70-72; nets/aggregation.py:354-370, 447),
 * which the reference leaves to cuDNN.  x [n, c, h, w]; grad_out [n, co, ho, wo] (NCHW);
 * grad_weight [co, c/groups, kh, kw] and grad_bias [co] (may be NULL) ACCUMULATE.
 * deterministic != 0: per-split partial sums reduced in a fixed order (bit-reproducible), with
 * `workspace` (device) of aanet_conv2d_wgrad_workspace_size(...) bytes; 0: float atomics, no
 * workspace; 2: the fixed-order form that STORES grad_weight / grad_bias instead of adding to
 * them (no zero fill needed).  The fixed-order form is also the faster one (round 5: 18 + 6 us against 36 us per
 * launch in the training step; the atomics of every pixel split hit the same weight elements),
 * and the Python layer calls it by default.  The data gradient is a forward conv on aanet_conv2d_fused_f32 (flipped,
 * transposed weight; zero-inserted grad_out for stride 2) -- aanet_amd/train.py. */
size_t aanet_conv2d_wgrad_workspace_size(int n, int c, int h, int w, int co, int kh, int kw,
                                         int stride, int pad, int dil, int groups);
int aanet_conv2d_wgrad_f32(const float *x, const float *grad_out, float *grad_weight,
                           float *grad_bias, int n, int c, int h, int w, int co, int kh, int kw,
                           int stride, int pad, int dil, int groups, int deterministic,
                           void *workspace, size_t workspace_bytes, aanet_stream_t stream);

/* Debug exports for bit-exact checks (SURVEY.md §8c pin 6):
 * im2col of ONE image, kernel.cu:570-633: col [c*kh*kw, ho*wo]. */
int aanet_mdcn_im2col_f32(const float *x, const float *offset, const float *mask, float *col,
                          int c, int h, int w, int kh, int kw, int stride, int pad, int dil,
                          int dg, aanet_stream_t stream);
/* sampling indices (floor of the fp32 coordinates) and the kernel.cu:618 validity flag,
 * [n, dg, kh*kw, ho*wo] int32 each. */
int aanet_mdcn_sample_index(const float *offset, int *h_low, int *w_low, int *valid, int n, int h,
                            int w, int kh, int kw, int stride, int pad, int dil, int dg,
                            aanet_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* AANET_MI355X_H */
