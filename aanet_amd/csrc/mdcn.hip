// mdcn.hip -- modulated deformable convolution (DCNv2) for gfx950.
// Replaces nets/deform_conv/src/deform_conv_cuda.cpp:490-685 and
// deform_conv_cuda_kernel.cu:467-866 (modulated kernels only; AANet never uses DCNv1).
//
// Forward = implicit GEMM.  A workgroup owns 64 output pixels of one image and up to 64
// output channels.  The K dimension (C_in * kh * kw) is walked in chunks of one tap k and
// <= 32 channels of one deformable group, so the sampling coordinates / bilinear weights of a
// (pixel, k, group) are computed ONCE in registers and reused for every channel of the chunk.
// The chunk's im2col tile is built in LDS (never written to HBM, unlike the reference's
// 122.7 MB-per-image `columns` buffer) and contracted with the weights by
// v_mfma_f32_16x16x4_f32 (exact fp32).
//
// Bit-exactness: the coordinate h = float(int) + offset is one fp32 add (kernel.cu:615-616);
// floor / bilinear follow kernel.cu:467-497 with fp contraction disabled, so im2col values
// and sampling indices equal the CPU oracle's bit for bit (tests/test_gpu_mdcn.py).
#include "common.h"
#include "dcn_small.h"
#include "dcn_tile.h"
#include "pointwise.h"
#include "small_conv.h"

#include <cstdio>
#include <stdlib.h>

namespace {

constexpr int NT = 256;
constexpr int PT = 64;     // pixels per workgroup tile
constexpr int KC = 32;     // max channels per K chunk
constexpr int CP = PT + 16;  // sCol pitch (floats): rows r, r+1 land 16 banks apart

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

struct MdcnArgs {
  const float *x;
  const float *offset;
  long off_bs;
  const float *mask;
  long mask_bs;
  int mask_logits;
  float mask_scale;
  const float *weight;
  const float *bias;
  const float *post_scale;
  const float *post_shift;
  const float *residual;  // added before the (last) activation, same shape as out, or NULL
  int act;
  // pointwise tail (bottleneck conv3 fused into this conv's epilogue); tail_w == NULL: none.
  // out = tail_act(tail_w . act(post_scale*(conv + bias) + post_shift) + tail_b + residual)
  const float *tail_w;  // packed [Co2][Co]
  const float *tail_b;
  int tail_act, Co2;
  float *out;
  int N, C, H, W, Co, kh, kw, stride, pad, dil, groups, dg, Ho, Wo;
  int layout;  // AANET_LAYOUT_* bits (conv engine only)
  int split;   // conv engine: split-bf16 contraction (AANET_CONV_EXACT_F32 clear, weights carry pieces)
  int halo;    // conv engine: 3x3 stride-1 halo-tile form (conv_fwd_kernel HALO)
  const bf16x8_t *wsplit, *tail_wsplit;  // bf16 piece fragments of weight / tail_w (split_frag_offset)
  int dbg_noatom;  // AANET_DCN_BWD_DBG=1: the backward data kernels skip the grad_x scatter (timing)
  // CSA epilogue (tail kernels): csa_out = csa_act(out + sum_j up_r[j](up[j])), r = 2 or 4
  float *csa_out;
  const float *up[3];
  int up_h[3], up_w[3], up_r[3], num_up, csa_act;
  const aanet_post_stage_t *post;  // HOST pointer (launch checks only): the post stage on csa_out
  // its fields for the device (HALO 1 tail, POST instantiation)
  const char *post_w;     // split fragments of the [64][64] 1x1 weight
  const float *post_b;
  int post_act;
  float *post_out;        // NHWC [N][Ho][Wo][64]
};

// the backward's timing switch: a kernel argument in the debug build, a compile-time 0 otherwise
// (so the product kernels carry no branch for it)
__device__ __forceinline__ int bwd_dbg(const MdcnArgs &a) {
#ifdef AANET_DEBUG_SWITCHES
  return a.dbg_noatom;
#else
  (void)a;
  return 0;
#endif
}

// Bilinear sampling state of one (pixel, tap, deformable group).  Invalid corners get
// weight 0 and a clamped (valid) address, which reproduces the reference's `v = 0` branch
// exactly: w*0 adds a zero term, as 0-valued v does in kernel.cu:478-493.
struct Samp {
  int i1, i2, i3, i4;
  float w1, w2, w3, w4;
  float m;
  float lh, lw;   // fractional parts (backward)
  int hl, wl;     // floor of the sampling position (backward window form)
  int valid;
  int ok;         // corner validity bits (backward)
};

__device__ __forceinline__ void make_samp(Samp &s, float h, float w, int H, int W, float m) {
#pragma clang fp contract(off)
  const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - (float)hl, lw = w - (float)wl;
  const float hh = 1.f - lh, hw = 1.f - lw;
  const bool ok1 = valid && hl >= 0 && wl >= 0;
  const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
  const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
  const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
  s.w1 = ok1 ? hh * hw : 0.f;
  s.w2 = ok2 ? hh * lw : 0.f;
  s.w3 = ok3 ? lh * hw : 0.f;
  s.w4 = ok4 ? lh * lw : 0.f;
  s.i1 = ok1 ? hl * W + wl : 0;
  s.i2 = ok2 ? hl * W + wl + 1 : 0;
  s.i3 = ok3 ? (hl + 1) * W + wl : 0;
  s.i4 = ok4 ? (hl + 1) * W + wl + 1 : 0;
  s.m = m;
  s.lh = lh;
  s.lw = lw;
  s.hl = hl;
  s.wl = wl;
  s.valid = valid;
  s.ok = (ok1 ? 1 : 0) | (ok2 ? 2 : 0) | (ok3 ? 4 : 0) | (ok4 ? 8 : 0);
}

// kernel.cu:494-496 then `val * mask` (kernel.cu:627): ((w1 v1 + w2 v2) + w3 v3) + w4 v4.
__device__ __forceinline__ float samp_val(const float *__restrict__ im, const Samp &s) {
#pragma clang fp contract(off)
  const float v = s.w1 * im[s.i1] + s.w2 * im[s.i2] + s.w3 * im[s.i3] + s.w4 * im[s.i4];
  return v * s.m;
}

// Forward form of the sampler: the two horizontal corners of a row are read with ONE 8-byte
// load (dword aligned) at a column base clamped into [0, W-2]; invalid corners carry weight 0
// so the clamped read never changes the value.  Same products and sum order as samp_val.
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
struct Samp2 {
  int itop, ibot;   // element offsets of the 2-wide column pair in rows hl and hl+1
  int swap;         // 1 when the pair base is wl+1 (wl == -1) -> corners swapped
  float w1, w2, w3, w4, m;
};

__device__ __forceinline__ void make_samp2(Samp2 &s, float h, float w, int H, int W, float m) {
#pragma clang fp contract(off)
  const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - (float)hl, lw = w - (float)wl;
  const float hh = 1.f - lh, hw = 1.f - lw;
  const bool ok1 = valid && hl >= 0 && wl >= 0;
  const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
  const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
  const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
  s.w1 = ok1 ? hh * hw : 0.f;
  s.w2 = ok2 ? hh * lw : 0.f;
  s.w3 = ok3 ? lh * hw : 0.f;
  s.w4 = ok4 ? lh * lw : 0.f;
  const int pb = valid ? min(max(wl, 0), W - 2) : 0;
  const int rt = valid ? min(max(hl, 0), H - 1) : 0;
  const int rb = valid ? min(max(hl + 1, 0), H - 1) : 0;
  s.itop = rt * W + pb;
  s.ibot = rb * W + pb;
  s.swap = (valid && pb != wl) ? 1 : 0;
  s.m = m;
}

__device__ __forceinline__ float samp_val2(const float *__restrict__ im, const Samp2 &s) {
#pragma clang fp contract(off)
  const f2u t = *reinterpret_cast<const f2u *>(im + s.itop);
  const f2u b = *reinterpret_cast<const f2u *>(im + s.ibot);
  const float v1 = s.swap ? t.y : t.x, v2 = s.swap ? t.x : t.y;
  const float v3 = s.swap ? b.y : b.x, v4 = s.swap ? b.x : b.y;
  const float v = s.w1 * v1 + s.w2 * v2 + s.w3 * v3 + s.w4 * v4;
  return v * s.m;
}

__device__ __forceinline__ float load_mask(const MdcnArgs &a, int n, int g, int k, int K, long P,
                                           long p) {
  const float v = a.mask[(long)n * a.mask_bs + ((long)g * K + k) * P + p];
  if (!a.mask_logits) return v;
  return a.mask_scale * (1.f / (1.f + expf(-v)));  // deform.py:86-89
}

// Sampling state for output pixel p of image n, tap k (= i*kw + j), deformable group g.
__device__ __forceinline__ void pixel_samp(Samp &s, const MdcnArgs &a, int n, int g, int k, long p,
                                           int ho, int wo) {
#pragma clang fp contract(off)
  const int K = a.kh * a.kw;
  const long P = (long)a.Ho * a.Wo;
  const int i = k / a.kw, j = k % a.kw;
  const float *off = a.offset + (long)n * a.off_bs + (long)g * 2 * K * P;
  const float oh = off[(long)(2 * k) * P + p], ow = off[(long)(2 * k + 1) * P + p];
  const float m = load_mask(a, n, g, k, K, P, p);
  const float h = (float)(ho * a.stride - a.pad + i * a.dil) + oh;
  const float w = (float)(wo * a.stride - a.pad + j * a.dil) + ow;
  make_samp(s, h, w, a.H, a.W, m);
}

__device__ __forceinline__ void pixel_samp2(Samp2 &s, const MdcnArgs &a, int n, int g, int k,
                                            long p, int ho, int wo) {
#pragma clang fp contract(off)
  const int K = a.kh * a.kw;
  const long P = (long)a.Ho * a.Wo;
  const int i = k / a.kw, j = k % a.kw;
  const float *off = a.offset + (long)n * a.off_bs + (long)g * 2 * K * P;
  const float oh = off[(long)(2 * k) * P + p], ow = off[(long)(2 * k + 1) * P + p];
  const float m = load_mask(a, n, g, k, K, P, p);
  const float h = (float)(ho * a.stride - a.pad + i * a.dil) + oh;
  const float w = (float)(wo * a.stride - a.pad + j * a.dil) + ow;
  make_samp2(s, h, w, a.H, a.W, m);
}

// Plain convolution tap: one in-bounds element or zero.
struct SampP {
  int idx;
  int ok;
};

__device__ __forceinline__ float apply_act(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);  // selects, no scalar branches
  return v > 0.f ? v : neg;
}

// ------------------------------------------------------------------------ forward -------
// Implicit-GEMM convolution engine.  MODE 1: modulated deformable (bilinear sampler, the DCN);
// MODE 0: plain convolution (one tap per input element; every other conv of the ISA/CSA
// blocks: 1x1, 3x3, dilated, grouped, strided).
//
// Workgroup = 256 threads, output tile CO_T channels x PTT pixels of one image.  The K
// dimension is walked in chunks of (<= 32 input channels of one deformable group, tap k),
// taps innermost so a chunk's 32 channel planes stay L2-resident across its 9 taps:
//   stage   : each thread builds PTT*32/256 im2col values of the chunk for ONE pixel -> LDS
//             [pixel][channel]; the sampling state of a (pixel, tap, group) is computed once.
//             Gathers are buffer loads: per-lane 32-bit offset (the tap position) + wave-uniform
//             SGPR offset (the channel plane), so a gather costs no address VALU; the plain
//             conv's zero padding comes from the buffer range check (offset past the image).
//             The weight slice -> LDS [co][channel].
//   contract: wave w owns CO_T x (PTT/4) outputs; per 16 channels one ds_read_b128 per 16-row
//             operand block, then 4 k-steps of v_mfma_f32_16x16x4_f32 -- the reduction index
//             is permuted (lane group kr takes channels 4kr..4kr+3) identically for both operands.
// Software pipeline: LDS double buffer; while the MFMAs of chunk c run, the global loads of
// chunk c+1 are in flight in registers and the offsets/mask of chunk c+2 are being fetched;
// one barrier per chunk.  Blocks are remapped so each XCD gets a contiguous range of tiles
// (neighbouring tiles share input rows -> same L2).
// Epilogue: the tile is transposed through LDS and written as 16-byte row segments:
// y = act(post_scale*(acc + bias) + post_shift + residual).
// grid: x = N * ceil(P/PTT), y = groups * ceil(Cog/CO_T).
constexpr int FNT = 512;  // forward conv engine: 8 waves = 2 (output channels) x 4 (pixels)
constexpr int SP = 40;  // LDS row pitch (floats) of both staging tiles: conflict-free b128 reads

typedef int i2v __attribute__((ext_vector_type(2)));

// K chunk = (tap k, channels [c0, c1)); chunks of ck channels, cut at deformable-group
// boundaries when `cut` (a chunk that spans groups carries one sampling state per group).
template <int CK>
struct ChunkIt {
  int k, c0, c1;
  __device__ __forceinline__ static int next_end(int c0, int cend, int cpg, int cut) {
    int e = min(c0 + CK, cend);
    if (cut) e = min(e, (c0 / cpg + 1) * cpg);
    return e;
  }
  __device__ __forceinline__ void first(int cbeg, int cend, int cpg, int cut) {
    k = 0;
    c0 = cbeg;
    c1 = next_end(cbeg, cend, cpg, cut);
  }
  __device__ __forceinline__ void advance(int K, int cend, int cpg, int cut) {
    if (++k == K) {
      k = 0;
      c0 = c1;
      c1 = next_end(c0, cend, cpg, cut);
    }
  }
};

// Pair-gather sampling state with the corner selection and the modulation mask folded into the
// weights: val = (wa_t*t.x + wa_b*b.x) + (wb_t*t.y + wb_b*b.y), evaluated with two packed-fp32
// ops and one add (kernel.cu:494-496 computes the same sum in another order: the values agree
// to rounding; the sampling positions and corner indices are bit-exact).  f32 MFMA and VALU
// never co-issue on gfx950, so every VALU op here is taken from the matrix pipe.
typedef float f2v __attribute__((ext_vector_type(2)));
struct SampW {
  int ot, ob;  // byte offsets of the 2-wide pairs in rows hl, hl+1
  f2v wt, wb;  // (wa_t, wb_t) * m, (wa_b, wb_b) * m
};

__device__ __forceinline__ void make_sampw(SampW &s, float h, float w, int H, int W, float m) {
#pragma clang fp contract(off)
  const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - (float)hl, lw = w - (float)wl;
  const float hh = 1.f - lh, hw = 1.f - lw;
  const bool ok1 = valid && hl >= 0 && wl >= 0;
  const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
  const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
  const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
  const float w1 = ok1 ? hh * hw : 0.f, w2 = ok2 ? hh * lw : 0.f;
  const float w3 = ok3 ? lh * hw : 0.f, w4 = ok4 ? lh * lw : 0.f;
  const int pb = valid ? min(max(wl, 0), W - 2) : 0;
  const int rt = valid ? min(max(hl, 0), H - 1) : 0;
  const int rb = valid ? min(max(hl + 1, 0), H - 1) : 0;
  s.ot = (rt * W + pb) * 4;
  s.ob = (rb * W + pb) * 4;
  const bool swap = valid && pb != wl;  // wl == -1: pair = (wl+1, wl+2); wl == W-1: (wl-1, wl)
  const bool left = wl < pb;             // wl == -1
  const float wat = swap ? (left ? w2 : 0.f) : w1;
  const float wbt = swap ? (left ? 0.f : w1) : w2;
  const float wab = swap ? (left ? w4 : 0.f) : w3;
  const float wbb = swap ? (left ? 0.f : w3) : w4;
  s.wt = f2v{wat, wbt} * m;
  s.wb = f2v{wab, wbb} * m;
}

// NHWC sampling state: byte offsets of the 4 corners (`oob` for an invalid corner: the buffer
// range check reads it as 0) and their weights with the mask folded in.  Same validity rules
// and corner indices as make_samp (kernel.cu:467-497).
__device__ __forceinline__ void make_samp4(int o[4], f32x4 &wv, float h, float w, int H, int W,
                                           int rowb, int oob, float m) {
#pragma clang fp contract(off)
  const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - (float)hl, lw = w - (float)wl;
  const float hh = 1.f - lh, hw = 1.f - lw;
  const bool ok1 = valid && hl >= 0 && wl >= 0;
  const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
  const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
  const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
  wv = f32x4{ok1 ? hh * hw : 0.f, ok2 ? hh * lw : 0.f, ok3 ? lh * hw : 0.f, ok4 ? lh * lw : 0.f} * m;
  o[0] = ok1 ? (hl * W + wl) * rowb : oob;
  o[1] = ok2 ? (hl * W + wl + 1) * rowb : oob;
  o[2] = ok3 ? ((hl + 1) * W + wl) * rowb : oob;
  o[3] = ok4 ? ((hl + 1) * W + wl + 1) * rowb : oob;
}

// ---- split-bf16 contraction (conv engine PREC 1) --------------------------------------------
// x = h + m + l exactly, three bf16 pieces carrying x's 24 significand bits (weights: round to
// nearest even, h = bf16(x), m = bf16(x - h), l = x - h - m; activations: truncation, split3).  A product
// a*b = sum_{i,j} a_i b_j; the six terms down to 2^-16 relative (mm, hl, lh, hm, mh, hh -- small
// first) run as v_mfma_f32_16x16x32_bf16 with fp32 accumulation.  Every bf16 x bf16 product is
// exact in fp32 and the three dropped terms (ml, lm, ll) are below 2^-23 |a b|, i.e. under one
// fp32 rounding of the product: the contraction is fp32-accurate, not a reduced-precision one.
// Measured on the C2 scale-0 3x3 conv against an fp64 reference (tools/split_lab.hip): max error
// 8.7e-6 (split) vs 1.0e-5 (exact f32 MFMA fma chain), mean 3.9e-7 vs 4.8e-7; keeping all nine
// terms changed no output.  bf16 MFMA runs at 16x the f32-MFMA rate, so the six products take
// 6/16 of the matrix-pipe time of the f32 contraction.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef bf16x8_t bf16x8;

// Weights for PREC 1 are split once (aanet_conv_weight_pack_split_f32) into MFMA A-operand
// fragments, streamed from L2 straight into registers: frag(g, t, k, cc, blk, pc, lane) = the 8
// bf16 of piece pc of rows co = g*Cog + 64t + 16blk + (lane & 15), channels 32cc + 8(lane >> 4)
// + 0..7 of tap k (zero past the group's Cog).  They follow the f32 packed weights in the same
// buffer, at a 256-byte aligned offset, so the f32 engine reads the buffer unchanged.
__host__ __device__ inline long split_frag_offset(int co, int cg, int kk) {
  return ((long)co * cg * kk * 4 + 255) / 256 * 256;
}
__host__ __device__ inline long split_frag_count(int co, int cg, int kk, int groups) {
  const int cog = co / groups;
  return (long)groups * ((cog + 63) / 64) * kk * ((cg + 31) / 32) * 4 * 3 * 64;
}

// Activations are split two values at a time by common.h split_pair (x = h + m + l exactly).
__device__ __forceinline__ void split3(f32x4 v, bf16x4 &h, bf16x4 &m, bf16x4 &l) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 hh, mm, ll;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    unsigned a, b, c;
    split_pair(v[2 * i], v[2 * i + 1], a, b, c);
    hh[i] = a;
    mm[i] = b;
    ll[i] = c;
  }
  h = __builtin_bit_cast(bf16x4, hh);
  m = __builtin_bit_cast(bf16x4, mm);
  l = __builtin_bit_cast(bf16x4, ll);
}

// Element offset of (row, 16-byte quad q8) in a [rows][32] bf16 piece plane.  Four 64-byte rows
// fill the 256-byte bank row; quads are XOR-swizzled by bit 2 of the row (q8 ^ 2 on rows 4-7 of
// every 8).  An MFMA operand read (ds_read_b128, lane (kr, jj) = quad kr of row base + jj) is
// serviced in the lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32):
// MI355X_MICROARCH.md §LDS), and with this swizzle every group hits 16 distinct 16-byte bank
// quads for ANY base row (the halo taps' shifts included); the previous row>>2 & 3 swizzle was
// conflict-free for 16 lanes at one quad, which is not how the hardware groups them (2-way
// conflicts on most reads: SQ_LDS_BANK_CONFLICT 31-41 % of the LDS cycles of the halo kernels).
__device__ __forceinline__ int swz(int row, int q8) { return row * 32 + ((q8 ^ (((row >> 2) & 1) << 1)) << 3); }

// channels 4*q4 .. 4*q4+3 of one row, as its three pieces (planes `pe` elements apart)
// The tail kernels' B staging (PAIRED: lanes write whole 16-byte quads, ds_write_b128 in lane
// groups of 8 consecutive lanes = 8 consecutive rows at one quad): quads XOR-swizzled by bits 1-2
// of the row, so those 8 lanes hit 8 distinct 16-byte bank slots, and the MFMA operand reads
// (lane groups as in swz) still hit 16 distinct ones (checked for every base row % 16 == 0).
__device__ __forceinline__ int swz_tail(int row, int q8) { return row * 32 + ((q8 ^ ((row >> 1) & 3)) << 3); }
// 8 values -> three bf16x8 pieces, the element-wise split of split3
__device__ __forceinline__ void split8_t(const float (&v)[8], bf16x8_t (&p)[3]) {
  bf16x4 h0, m0, l0, h1, m1, l1;
  split3(f32x4{v[0], v[1], v[2], v[3]}, h0, m0, l0);
  split3(f32x4{v[4], v[5], v[6], v[7]}, h1, m1, l1);
  p[0] = bf16x8_t{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
  p[1] = bf16x8_t{m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
  p[2] = bf16x8_t{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
}

__device__ __forceinline__ void put_split(__bf16 *plane, int pe, int row, int q4, f32x4 v) {
  bf16x4 h, m, l;
  split3(v, h, m, l);
  const int o = swz(row, q4 >> 1) + ((q4 & 1) << 2);
  *reinterpret_cast<bf16x4 *>(plane + o) = h;
  *reinterpret_cast<bf16x4 *>(plane + pe + o) = m;
  *reinterpret_cast<bf16x4 *>(plane + 2 * pe + o) = l;
}

__device__ __forceinline__ f32x4 mfma_split6(const bf16x8 (&A)[3], const bf16x8 (&B)[3], f32x4 t) {
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], t, 0, 0, 0);
}

// FULL: every chunk holds KC channels (Cg % KC == 0, and cpg % KC == 0 for the DCN), so the
// staging code has no per-row guards.  Those guards are wave-uniform, and the compiler turns
// them into scalar branches, which split the loop body and defeat the MFMA/staging interleave.
// LAYOUT bit 0: input NHWC (channels-last; each staging item is one 16-byte load of 4 channels
// at one position, so a DCN corner or a conv tap of 32 channels is 8 lanes x 16 B = one 128-B
// line; needs FULL).  Bit 1: output NHWC.
// CFG: chunk shape.  0: 32 channels of one deformable group; 1: 16 channels (16-channel conv
// groups: the second MFMA half of a chunk is skipped); 2: 32 channels spanning two 16-channel
// deformable groups (one sampling state per (pixel, group)).
// HALO (plain 3x3, stride 1, pad = dil <= 2, NHWC input, PREC 1): the tile is 8 rows x 16
// columns of outputs; per 32-channel chunk its (8+2d) x (16+2d) input halo is loaded, split and
// stored to LDS ONCE, and all nine taps read their B operand from it at shifted positions (the
// im2col form stages, splits and synchronises once per tap).  The next chunk's halo is in flight
// in registers during the nine taps; A fragments are double-buffered across taps.
// POST (HALO 1/2 tails with the CSA epilogue, CO_T = Co2 = 64): the post stage of
// aanet_post_stage_t on the CSA output, NHWC out only (the next module's conv1).
template <int MODE, int CO_T, int PTT, int PACKED, int TAIL, int SCHED, int FULL, int LAYOUT,
          int CFG = 0, int PREC = 0, int HALO = 0, int POST = 0>
__global__ __launch_bounds__(FNT, 4) void conv_fwd_kernel(MdcnArgs a) {
  constexpr int CK = CFG == 1 ? 16 : 32;   // channels per K chunk
  constexpr int GPC = CFG == 2 ? 2 : 1;    // deformable groups per chunk
  constexpr int WC = CO_T >= 32 ? 2 : 1;   // waves along the output channels
  constexpr int WP = FNT / 64 / WC;        // waves along the pixels
  constexpr int NCB = CO_T / 16 / WC;      // 16-row output-channel blocks per wave
  constexpr int NPB = PTT / 16 / WP;       // 16-col pixel blocks per wave
  constexpr int CPT = CK * PTT / FNT;      // im2col values staged per thread per chunk
  constexpr int WPT = CK * CO_T / FNT;     // weights staged per thread per chunk
  static_assert(NCB >= 1 && NPB >= 1 && WPT >= 1 && CPT % 4 == 0, "tile shape");
  static_assert(CFG == 0 || FULL, "chunk configurations 1/2 need full chunks");
  constexpr bool INH = (LAYOUT & 1) != 0, ONH = (LAYOUT & 2) != 0;
  constexpr int NIT = INH ? PTT * (CK / 4) / FNT : 1;  // NHWC staging items per thread
  static_assert(!INH || (FULL && NIT >= 1 && FNT % (CK / 4) == 0), "NHWC staging needs full chunks");
  static_assert(!(ONH && TAIL), "NHWC output with a pointwise tail is not instantiated");
  // PREC 1 (split-bf16 contraction, see split4 / SplitLds): both operand tiles as three bf16
  // piece planes of 32-channel rows, 64 B per row (XOR-swizzled 16-byte quads, no padding)
  constexpr bool SPL = PREC == 1;
  // (partial chunks: plain NCHW convs whose group width is a multiple of 16 but not 32 -- the
  // zero-padded split pack, rows past the group staged as zeros)
  static_assert(!SPL || (CK == 32 && (FULL || (MODE == 0 && !INH && !TAIL)) && PACKED && CO_T >= 32),
                "split-bf16 configuration");
  constexpr int BUF = SPL ? PTT * 48 : (PTT + CO_T) * SP; // floats per LDS buffer
  constexpr int OP = PTT + 4;            // epilogue tile pitch
  static_assert(CO_T * OP <= 2 * BUF, "epilogue tile must fit the staging buffers");
  // DCN: the sampling state of a (pixel, tap, deformable group) is computed once, by the threads
  // tid < GPC*PTT (group gi = tid / PTT of the chunk), and published through a double-buffered
  // LDS slot to the threads that stage channels of that pixel and group (the VALU it saves is
  // matrix-pipe time).
  constexpr int PSLOT = GPC * PTT * 8;
  __shared__ __attribute__((aligned(16))) float smem[2 * BUF + (MODE ? 2 * PSLOT : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool pwave = __builtin_amdgcn_readfirstlane(wave) < GPC * PTT / 64;  // tid < GPC*PTT
  const int pgi = MODE ? __builtin_amdgcn_readfirstlane(wave / (PTT / 64)) : 0;  // param group
  const int wc0 = __builtin_amdgcn_readfirstlane((wave / WP) * NCB);  // first co block of the wave
  const int wp0 = __builtin_amdgcn_readfirstlane((wave % WP) * NPB);  // first px block of the wave
  const long P = (long)a.Ho * a.Wo;
  static_assert(!HALO || (MODE == 0 && PREC == 1 && (HALO <= 2 || HALO == 4) && PTT == 128 && (LAYOUT & 1)),
                "halo configuration");
  // HALO 4: the phase-strided halo tile.  A 3x3 conv of dilation D (= pad, stride 1) is D x D
  // independent dilation-1 convs, one per phase (pixels y % D = pa, x % D = pb): the tile is
  // 8 x 16 outputs of one phase, its halo the (8+2) x (16+2) phase positions around them, so
  // dilations 4 / 8 (nets/refinement.py:60-106) stage 1.4 positions per output instead of the
  // (8+2D)(16+2D)/128 of a plain halo or the nine of im2col.  NHWC in and out only.
  constexpr bool PH = HALO == 4;
  static_assert(!PH || (LAYOUT == 3 && !TAIL && !POST), "phase-strided halo: NHWC in/out, no tail");
  constexpr int TRH = 8;  // output rows of a halo tile (16 columns)
  const int pd = PH ? a.dil : 1;                       // phase stride
  const int hWo = PH ? (a.Wo + pd - 1) / pd : a.Wo;    // (largest) phase image size
  const int hHo = PH ? (a.Ho + pd - 1) / pd : a.Ho;
  const int htx = HALO ? (hWo + 15) / 16 : 1;
  const int hty = HALO ? (hHo + TRH - 1) / TRH : 1;
  const int ntiles = HALO ? pd * pd * htx * hty : (int)((P + PTT - 1) / PTT);
  // XCD-aware remap of the pixel-tile index (bijective for any grid size)
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile0 = bid % ntiles;
  const int ph = PH ? tile0 / (htx * hty) : 0, tile = PH ? tile0 - ph * (htx * hty) : tile0;
  const int pa = PH ? ph / pd : 0, pb = PH ? ph - pa * pd : 0;  // the tile's phase
  // HALO tile origin (phase coordinates for HALO 4: image row pa + pd * y)
  const int hy0 = HALO ? (tile / htx) * TRH : 0, hx0 = HALO ? (tile % htx) * 16 : 0;
  const int Cg = a.C / a.groups, Cog = a.Co / a.groups, K = a.kh * a.kw, cpg = a.C / a.dg;
  const int ncot = (Cog + CO_T - 1) / CO_T;
  const int gc = blockIdx.y / ncot, cot = blockIdx.y % ncot;
  const int co0 = gc * Cog + cot * CO_T, co_end = min(co0 + CO_T, (gc + 1) * Cog);
  const int cbeg = gc * Cg, cend = (gc + 1) * Cg;
  const long HW = (long)a.H * a.W;
  const int img_bytes = (int)(a.C * HW * 4);
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void *)(a.x + (long)n * a.C * HW), (short)0,
                                                     img_bytes, 0x00020000);
  const int plane_bytes = (int)(HW * 4);

  // staging role: one pixel, CPT consecutive channels of the chunk (wave-uniform base)
  const int spx = tid % PTT;
  const int scb = __builtin_amdgcn_readfirstlane((tid / PTT) * CPT);
  const long p = (long)tile * PTT + spx;
  const bool pvalid = p < P;
  const int ho = pvalid ? (int)(p / a.Wo) : 0, wo = pvalid ? (int)(p % a.Wo) : 0;
  const long psafe = pvalid ? p : 0;
  // NHWC staging roles: lane quad nq = channels 4nq..4nq+3, pixels npx[i]
  const int nq = tid & (CK / 4 - 1);
  int npx[NIT], nho[NIT], nwo[NIT];
  bool nval[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    npx[i] = tid / (CK / 4) + (FNT / (CK / 4)) * i;
    const long pp = (long)tile * PTT + npx[i];
    nval[i] = pp < P;
    nho[i] = nval[i] ? (int)(pp / a.Wo) : 0;
    nwo[i] = nval[i] ? (int)(pp % a.Wo) : 0;
  }
  f32x4 nv[INH && MODE == 0 ? NIT : 1];        // conv tap values (NHWC)
  f32x4 nc[INH && MODE ? NIT : 1][4];          // DCN corner values (NHWC)
  int noff[INH && MODE ? NIT : 1][4];          // DCN corner byte offsets (NHWC)
  f32x4 nw[INH && MODE ? NIT : 1];             // DCN corner weights (mask folded)

  float wreg[WPT];
  float vraw[MODE ? 1 : CPT];
  i2v traw[MODE ? CPT : 1], braw[MODE ? CPT : 1];
  SampW snext;                                 // sampling state of the chunk being loaded
  float off_h = 0.f, off_w = 0.f, mlog = 0.f;  // raw offsets/mask of the chunk after it

  // offsets / mask / weights through buffer descriptors too: per-lane part fixed for the whole
  // kernel, chunk-dependent part in an SGPR.
  const auto offr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(MODE ? a.offset + (long)n * a.off_bs : a.x), (short)0, 0x7ffffff0, 0x00020000);
  const auto mskr = __builtin_amdgcn_make_buffer_rsrc(
      (void *)(MODE ? a.mask + (long)n * a.mask_bs : a.x), (short)0, 0x7ffffff0, 0x00020000);
  const int w_bytes = (int)((long)a.Co * Cg * K * 4);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc((void *)a.weight, (short)0, w_bytes, 0x00020000);
  int wlane[WPT];  // per-lane weight byte offsets (chunk-invariant)
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int e = tid + FNT * i, co = e / CK, cl = e % CK;
    // rows past the chunk read a neighbouring channel (multiplied by a zero im2col value);
    // reads past the tensor are out of range -> 0; co past co_end is never stored
    wlane[i] = PACKED ? (co * Cg + cl) * 4 : (co * Cg * K + cl * K) * 4;
  }
  const int pl4 = (int)psafe * 4;
  // PREC 1: the wave's A fragments (its NCB 16-row blocks x 3 pieces) come from the pre-split
  // weight fragments in global memory (L2-resident), loaded one chunk ahead of their MFMAs
  bf16x8 fa[SPL ? NCB : 1][3];
  const int sT = (Cog + 63) / 64, sNCC = (Cg + 31) / 32;
  const int st64 = (cot * CO_T) / 64, sbb = ((cot * CO_T) % 64) / 16 + wc0;
  auto load_a = [&](const bf16x8 *frag, long tile_base) {
#pragma unroll
    for (int m = 0; m < NCB; ++m)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) fa[m][pc] = frag[((tile_base + sbb + m) * 3 + pc) * 64 + lane];
  };
  auto load_a_chunk = [&](const ChunkIt<CK> &c) {
    load_a(a.wsplit, ((((long)gc * sT + st64) * K + c.k) * sNCC + ((c.c0 - cbeg) >> 5)) * 4);
  };

  auto load_params_raw = [&](const ChunkIt<CK> &c) {
    const int g = c.c0 / cpg + pgi;
    const int ob = __builtin_amdgcn_readfirstlane((int)(((long)g * 2 * K + 2 * c.k) * P * 4));
    const int mb = __builtin_amdgcn_readfirstlane((int)(((long)g * K + c.k) * P * 4));
    off_h = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, pl4, ob, 0));
    off_w = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, pl4, ob + (int)(P * 4), 0));
    mlog = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mskr, pl4, mb, 0));
  };
  auto finish_params = [&](const ChunkIt<CK> &c, int slot) {
#pragma clang fp contract(off)
    const int i = c.k / a.kw, j = c.k % a.kw;
    float m = a.mask_logits ? a.mask_scale * __builtin_amdgcn_rcpf(1.f + __expf(-mlog)) : mlog;
    if (!pvalid) m = 0.f;
    const float h = (float)(ho * a.stride - a.pad + i * a.dil) + off_h;
    const float w = (float)(wo * a.stride - a.pad + j * a.dil) + off_w;
    float *d = smem + 2 * BUF + slot * PSLOT + (pgi * PTT + spx) * 8;
    if constexpr (INH) {
      int o[4];
      f32x4 wv;
      make_samp4(o, wv, h, w, a.H, a.W, a.C * 4, img_bytes, m);
      *reinterpret_cast<f32x4 *>(d) = f32x4{__builtin_bit_cast(float, o[0]), __builtin_bit_cast(float, o[1]),
                                            __builtin_bit_cast(float, o[2]), __builtin_bit_cast(float, o[3])};
      *reinterpret_cast<f32x4 *>(d + 4) = wv;
    } else {
      SampW sw;
      make_sampw(sw, h, w, a.H, a.W, m);
      *reinterpret_cast<f32x4 *>(d) = f32x4{__builtin_bit_cast(float, sw.ot),
                                            __builtin_bit_cast(float, sw.ob), sw.wt.x, sw.wt.y};
      *reinterpret_cast<f2v *>(d + 4) = sw.wb;
    }
  };
  auto get_params = [&](int slot) {
    if constexpr (INH) {
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int gi = GPC == 2 ? nq >> 2 : 0;  // 16-channel group of this lane's quad
        const float *d = smem + 2 * BUF + slot * PSLOT + (gi * PTT + npx[i]) * 8;
        const f32x4 q = *reinterpret_cast<const f32x4 *>(d);
        const float q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];  // see below
        noff[i][0] = __builtin_bit_cast(int, q0);
        noff[i][1] = __builtin_bit_cast(int, q1);
        noff[i][2] = __builtin_bit_cast(int, q2);
        noff[i][3] = __builtin_bit_cast(int, q3);
        nw[i] = *reinterpret_cast<const f32x4 *>(d + 4);
      }
      return;
    }
    const int gi = GPC == 2 ? scb >> 4 : 0;  // scb: multiple of CPT (8) -> one group per thread
    const float *d = smem + 2 * BUF + slot * PSLOT + (gi * PTT + spx) * 8;
    const f32x4 q = *reinterpret_cast<const f32x4 *>(d);
    // copy the elements to scalars first: __builtin_bit_cast of an ext-vector element lvalue
    // (q[1]) reads element 0 with this clang
    const float q0 = q[0], q1 = q[1];
    snext.ot = __builtin_bit_cast(int, q0);
    snext.ob = __builtin_bit_cast(int, q1);
    snext.wt = f2v{q[2], q[3]};
    snext.wb = *reinterpret_cast<const f2v *>(d + 4);
  };
  auto issue_loads = [&](const ChunkIt<CK> &c) {
    const int rows = c.c1 - c.c0;
    const int wbase = PACKED ? (((c.k * a.Co + co0) * Cg + (c.c0 - cbeg)) * 4)
                             : (((co0 * Cg + (c.c0 - cbeg)) * K + c.k) * 4);
    if constexpr (!SPL) {
#pragma unroll
      for (int i = 0; i < WPT; ++i)
        wreg[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, wlane[i], wbase, 0));
    }
    if constexpr (INH) {
      const int soff = __builtin_amdgcn_readfirstlane(c.c0 * 4);
      if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
          const int hi = nho[i] * a.stride - a.pad + (c.k / a.kw) * a.dil;
          const int wi = nwo[i] * a.stride - a.pad + (c.k % a.kw) * a.dil;
          const bool ok = nval[i] && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
          const int voff = ok ? (hi * a.W + wi) * (a.C * 4) + nq * 16 : img_bytes;
          nv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, voff, soff, 0));
        }
      } else {
#pragma unroll
        for (int i = 0; i < NIT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            nc[i][j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, noff[i][j] + nq * 16, soff, 0));
      }
      return;
    }
    const int cbase = __builtin_amdgcn_readfirstlane((c.c0 + scb) * plane_bytes);
    if (MODE == 0) {
      const int hi = ho * a.stride - a.pad + (c.k / a.kw) * a.dil;
      const int wi = wo * a.stride - a.pad + (c.k % a.kw) * a.dil;
      const bool ok = pvalid && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      const int voff = ok ? (hi * a.W + wi) * 4 : img_bytes;  // past the end -> reads 0
#pragma unroll
      for (int e = 0; e < CPT; ++e) {
        const int soff = cbase + e * plane_bytes;
        vraw[e] = (FULL || scb + e < rows)
                      ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, voff, soff, 0))
                      : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < CPT; ++e) {
        const int soff = cbase + (FULL ? e : min(e, rows - 1 - scb)) * plane_bytes;
        traw[e] = __builtin_amdgcn_raw_buffer_load_b64(xr, snext.ot, soff, 0);
        braw[e] = __builtin_amdgcn_raw_buffer_load_b64(xr, snext.ob, soff, 0);
      }
    }
  };
  auto store_stage = [&](const ChunkIt<CK> &c, int buf) {
    float *sC = smem + buf * BUF, *sW = sC + PTT * SP;
    __bf16 *sB = reinterpret_cast<__bf16 *>(smem + buf * BUF);
    const int rows = c.c1 - c.c0;
    if constexpr (!SPL) {
#pragma unroll
      for (int i = 0; i < WPT; ++i) {
        const int e = tid + FNT * i;
        sW[(e / CK) * SP + e % CK] = wreg[i];
      }
    }
    if constexpr (INH) {
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        f32x4 v;
        if (MODE == 0) {
          v = nv[i];
        } else {
          // Bilinear blend of the 4 corner quads: ((c0 w0 + c1 w1) + c2 w2) + c3 w3 per channel,
          // as scalar v_mul/v_fma_f32 in asm.  The packed form the compiler picks for this
          // (v_pk_fma_f32 with a broadcast weight) gave non-reproducible results in the split
          // DCN tail kernel: pixels staged by lanes 48-63 read a stale broadcast weight register
          // written by the VALU instruction just before (tools/diag_race3.py).
          const float w0 = nw[i][0], w1 = nw[i][1], w2 = nw[i][2], w3 = nw[i][3];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float t;
            asm("v_mul_f32 %0, %1, %2" : "=v"(t) : "v"(nc[i][0][u]), "v"(w0));
            asm("v_fma_f32 %0, %1, %2, %0" : "+v"(t) : "v"(nc[i][1][u]), "v"(w1));
            asm("v_fma_f32 %0, %1, %2, %0" : "+v"(t) : "v"(nc[i][2][u]), "v"(w2));
            asm("v_fma_f32 %0, %1, %2, %0" : "+v"(t) : "v"(nc[i][3][u]), "v"(w3));
            v[u] = t;
          }
        }
        if constexpr (SPL)
          put_split(sB, PTT * 32, npx[i], nq, v);
        else
          *reinterpret_cast<f32x4 *>(sC + npx[i] * SP + 4 * nq) = v;
      }
      return;
    }
    float v[CPT];
#pragma unroll
    for (int e = 0; e < CPT; ++e) {
      if (MODE == 0) {
        v[e] = vraw[e];
      } else {
        const f2v p = __builtin_elementwise_fma(snext.wb, __builtin_bit_cast(f2v, braw[e]),
                                                snext.wt * __builtin_bit_cast(f2v, traw[e]));
        float r;  // scalar add of the two halves (keeps the vectorizer from re-pairing them)
        asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(p.x), "v"(p.y));
        v[e] = (FULL || scb + e < rows) ? r : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < CPT / 4; ++q) {
      const f32x4 vq = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
      if constexpr (SPL)
        put_split(sB, PTT * 32, spx, scb / 4 + q, vq);
      else
        *reinterpret_cast<f32x4 *>(sC + spx * SP + scb + 4 * q) = vq;
    }
  };

  f32x4 acc[NCB][NPB];
#pragma unroll
  for (int m = 0; m < NCB; ++m)
#pragma unroll
    for (int b = 0; b < NPB; ++b) acc[m][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kr = lane >> 4, jj = lane & 15;
  constexpr int CUT = MODE && GPC == 1;  // chunks stop at deformable-group boundaries
  ChunkIt<CK> cur, nxt, nn;
  bool has_next = false;
  int slot = 1;  // parameter slot of `nxt`
  if constexpr (!HALO) {
  cur.first(cbeg, cend, cpg, CUT);
  if (MODE) {
    if (pwave) {
      load_params_raw(cur);
      finish_params(cur, 0);
    }
    __syncthreads();
    get_params(0);
  }
  issue_loads(cur);
  if constexpr (SPL) load_a_chunk(cur);
  store_stage(cur, 0);
  nxt = cur;
  nxt.advance(K, cend, cpg, CUT);
  has_next = nxt.c0 < cend;
  if (MODE && has_next && pwave) {
    load_params_raw(nxt);
    finish_params(nxt, 1);
  }
  __syncthreads();
  }

  struct Frag {
    f32x4 A[NCB], B[NPB];
  };
  auto read_frag = [&](int buf, int h, Frag &f) {
    const float *sC = smem + buf * BUF, *sW = sC + PTT * SP;
#pragma unroll
    for (int m = 0; m < NCB; ++m)
      f.A[m] = *reinterpret_cast<const f32x4 *>(sW + (16 * (wc0 + m) + jj) * SP + 16 * h + 4 * kr);
#pragma unroll
    for (int b = 0; b < NPB; ++b)
      f.B[b] = *reinterpret_cast<const f32x4 *>(sC + (16 * (wp0 + b) + jj) * SP + 16 * h + 4 * kr);
  };
  auto mma = [&](const Frag &f) {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int m = 0; m < NCB; ++m)
#pragma unroll
        for (int b = 0; b < NPB; ++b) {
          acc[m][b] = mfma16x16x4(f.A[m][s4], f.B[b][s4], acc[m][b]);
        }
  };
  auto mfma_half = [&](int buf, int h) {
    Frag f;
    read_frag(buf, h, f);
    mma(f);
  };
  // PREC 1: the whole 32-channel chunk is one K step of v_mfma_f32_16x16x32_bf16 per piece pair.
  // A: the fragments in fa; B: read one 16-pixel block at a time (12 VGPRs live, not 24).
  auto mma_s = [&](int buf) {
    const __bf16 *sB = reinterpret_cast<const __bf16 *>(smem + buf * BUF);
#pragma unroll
    for (int b = 0; b < NPB; ++b) {
      bf16x8 fb[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        fb[pc] = *reinterpret_cast<const bf16x8 *>(sB + pc * PTT * 32 + swz(16 * (wp0 + b) + jj, kr));
#pragma unroll
      for (int m = 0; m < NCB; ++m) acc[m][b] = mfma_split6(fa[m], fb, acc[m][b]);
    }
  };
  auto mfma_chunk = [&](int buf) {
    if constexpr (SPL) {
      mma_s(buf);
    } else {
      mfma_half(buf, 0);
      mfma_half(buf, 1);
    }
  };

  if constexpr (!HALO) for (int buf = 0;; buf ^= 1) {
    nn = nxt;
    nn.advance(K, cend, cpg, CUT);
    const bool has_nn = has_next && nn.c0 < cend;
    if (has_next) {
      if (MODE) get_params(slot);
      issue_loads(nxt);
    }
    if (MODE && has_nn && pwave) load_params_raw(nn);
    if (SPL && SCHED && MODE == 0) {
      // all B fragments of chunk c first; then chunk c+1's staging (split, LDS writes) is
      // interleaved with chunk c's bf16 MFMAs.  (The DCN variants keep the sequential order: the
      // extra 12 live VGPRs of this form spill them past the 128-VGPR cap.)
      const __bf16 *sB = reinterpret_cast<const __bf16 *>(smem + buf * BUF);
      bf16x8 fb[NPB][3];
#pragma unroll
      for (int b = 0; b < NPB; ++b)
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          fb[b][pc] = *reinterpret_cast<const bf16x8 *>(sB + pc * PTT * 32 + swz(16 * (wp0 + b) + jj, kr));
      if (has_next) store_stage(nxt, buf ^ 1);
#pragma unroll
      for (int b = 0; b < NPB; ++b)
#pragma unroll
        for (int m = 0; m < NCB; ++m) acc[m][b] = mfma_split6(fa[m], fb[b], acc[m][b]);
      if (has_next) {
#pragma unroll
        for (int i = 0; i < 6 * NCB * NPB; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
          if (i % 3 == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS_WRITE
        }
      }
      if (!has_next) break;
      load_a_chunk(nxt);
    } else if (SPL) {
      mma_s(buf);
      if (!has_next) break;
      load_a_chunk(nxt);
      store_stage(nxt, buf ^ 1);
    } else if (SCHED) {
      // chunk c+1's staging math + LDS writes are interleaved with the second half of chunk c's
      // MFMAs (different LDS buffers), so each wave keeps its matrix pipe busy by itself.
      // The half-1 operands are read before the staging writes: LDS reads and writes of the two
      // buffers cannot be proven disjoint, so reads issued after the writes would hold every
      // MFMA of half 1 behind the whole staging store.
      Frag f1;
      if (CK == 32) {
        mfma_half(buf, 0);
        read_frag(buf, 1, f1);
      } else {  // 16-channel chunks: one half, which carries the staging interleave
        read_frag(buf, 0, f1);
      }
      if (!has_next) {
        mma(f1);
        break;
      }
      store_stage(nxt, buf ^ 1);
      mma(f1);
#pragma unroll
      for (int i = 0; i < 4 * NCB * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // VALU
        if (i % 2 == 0) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS_WRITE
      }
    } else {
      mfma_half(buf, 0);
      if (CK == 32) mfma_half(buf, 1);
      if (!has_next) break;
      store_stage(nxt, buf ^ 1);
    }
    if (MODE && has_nn && pwave) finish_params(nn, slot ^ 1);
    __syncthreads();
    slot ^= 1;
    nxt = nn;
    has_next = has_nn;
  }

  if constexpr (HALO) {
    // stride 1, dilation = padding = d (the round-3 stride-2 NCHW form, HALO 3, was removed in
    // round 4: faster alone, slower in the two-stream step)
    constexpr int d = PH ? 1 : HALO;  // tap spacing in the halo
    constexpr int hw = 16 + 2 * d, npos = (8 + 2 * d) * hw;
    const int hy = hy0 - d, hx = hx0 - d;
    constexpr int HIT = (npos * 8 + FNT - 1) / FNT;  // halo quads per thread (NHWC)
    f32x4 hv[HIT];
    // 64-channel tiles recompute the halo quad offsets per chunk (a few VALU) rather than hold
    // them across the chunk loop: held, they were spilled to scratch and re-read every chunk
    // (76 B/lane at the 128-VGPR cap).  32-channel tiles have the registers to hold them.
    auto load_halo = [&](int c0) {
      const int soff = __builtin_amdgcn_readfirstlane(c0 * 4);
      int t = tid;
      if constexpr (CO_T >= 64) asm volatile("" : "+v"(t));  // keep the arithmetic in the loop
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = t + FNT * i, pos = e >> 3;
        const int yy = hy + pos / hw, xx = hx + pos % hw;
        const int iy = PH ? pa + pd * yy : yy, ix = PH ? pb + pd * xx : xx;  // image position
        const bool ok = pos < npos && yy >= 0 && iy < a.H && xx >= 0 && ix < a.W;
        const int off = ok ? ((iy * a.W + ix) * a.C + 4 * (e & 7)) * 4 : img_bytes;  // zero padding: OOB
        hv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, soff, 0));
      }
    };
    bf16x8 ha0[NCB][3], ha1[NCB][3];  // A fragments of two taps (double buffer)
    // A fragments by buffer loads: per-lane offset lane*16 (one VGPR), everything else in the
    // wave-uniform SGPR offset, so no per-tap address lives in VGPRs
    const auto war = __builtin_amdgcn_make_buffer_rsrc((void *)a.wsplit, (short)0, 0x7ffffff0, 0x00020000);
    auto load_ha = [&](bf16x8 (&ha)[NCB][3], int c0, int k) {
      const int base = ((((gc * sT + st64) * K + k) * sNCC + ((c0 - cbeg) >> 5)) * 4 + sbb) * 3;
#pragma unroll
      for (int m = 0; m < NCB; ++m)
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          ha[m][pc] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
              war, lane * 16, __builtin_amdgcn_readfirstlane((base + 3 * m + pc) * 1024), 0));
    };
    // B fragment LDS address of (tile row r, column jj) at halo row/column shift (si, sj)
    const int jjd = jj;
    // tap k of the chunk at c0: prefetch the next tap's A (the next chunk's tap 0 after tap 8),
    // then the B fragments at the tap's shifted halo positions and the MFMAs
    auto tap = [&](bf16x8 (&cur)[NCB][3], bf16x8 (&nxt)[NCB][3], int k, int c0, bool more) {
      // keep the scheduler from hoisting later taps' work (SSA values, no WAR on the buffers)
      // above this tap: 9 taps of fragments and addresses would not fit the 128-VGPR budget
      __builtin_amdgcn_sched_barrier(0);
      if (k < 8)
        load_ha(nxt, c0, k + 1);
      else if (more)
        load_ha(nxt, c0 + 32, 0);
      const int ti = k / 3, tj = k % 3;
      int col = jjd;
      asm volatile("" : "+v"(col));  // recomputed per tap (not hoisted as 18 live addresses)
#pragma unroll
      for (int b = 0; b < NPB; ++b) {
        const int pos = (wp0 + b + ti * d) * hw + col + tj * d;
        const __bf16 *sH = reinterpret_cast<const __bf16 *>(smem) + swz(pos, kr);
        bf16x8 fb[3];
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) fb[pc] = *reinterpret_cast<const bf16x8 *>(sH + pc * npos * 32);
#pragma unroll
        for (int m = 0; m < NCB; ++m) acc[m][b] = mfma_split6(cur[m], fb, acc[m][b]);
      }
    };
    auto stage = [&](int c0) {
      __syncthreads();  // every wave is done with the previous chunk's halo
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int pos = (tid + FNT * i) >> 3;
        if (pos < npos) put_split(reinterpret_cast<__bf16 *>(smem), npos * 32, pos, tid & 7, hv[i]);
      }
      __syncthreads();
      const bool more = c0 + 32 < cend;
      if (more) load_halo(c0 + 32);
      return more;
    };
    load_halo(cbeg);
    load_ha(ha0, cbeg, 0);
    // nine taps per chunk: the A buffers alternate, so consecutive chunks start on opposite ones
    for (int c0 = cbeg; c0 < cend; c0 += 64) {
      bool more = stage(c0);
      tap(ha0, ha1, 0, c0, more); tap(ha1, ha0, 1, c0, more); tap(ha0, ha1, 2, c0, more);
      tap(ha1, ha0, 3, c0, more); tap(ha0, ha1, 4, c0, more); tap(ha1, ha0, 5, c0, more);
      tap(ha0, ha1, 6, c0, more); tap(ha1, ha0, 7, c0, more); tap(ha0, ha1, 8, c0, more);
      if (!more) break;
      more = stage(c0 + 32);
      tap(ha1, ha0, 0, c0 + 32, more); tap(ha0, ha1, 1, c0 + 32, more); tap(ha1, ha0, 2, c0 + 32, more);
      tap(ha0, ha1, 3, c0 + 32, more); tap(ha1, ha0, 4, c0 + 32, more); tap(ha0, ha1, 5, c0 + 32, more);
      tap(ha1, ha0, 6, c0 + 32, more); tap(ha0, ha1, 7, c0 + 32, more); tap(ha1, ha0, 8, c0 + 32, more);
    }
  }

  if (TAIL) {
    // act(post_scale*(acc+bias)+post_shift) -> LDS as the B operand [px][c] of a second GEMM with
    // the pointwise weights [co2][c] (channels 32h..32h+31 in buffer h), then re-contract.
    // The per-channel parameters of the wave's accumulator rows (and, PREC 1, every A fragment
    // of the pointwise weights) are loaded as one batch ahead of the barrier: element-wise
    // guarded loads would each wait out an L2 round trip.
    constexpr int NH = (CO_T + 31) / 32;  // channel chunks of the pointwise GEMM
    float pb[NCB][4], ps[NCB][4], ph[NCB][4];
#pragma unroll
    for (int m = 0; m < NCB; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cc = min(co0 + 16 * (wc0 + m) + 4 * kr + r, co_end - 1);
        pb[m][r] = a.bias ? a.bias[cc] : 0.f;
        ps[m][r] = a.post_scale ? a.post_scale[cc] : 1.f;
        ph[m][r] = a.post_scale ? a.post_shift[cc] : 0.f;
      }
    bf16x8 ta[SPL ? NH : 1][SPL ? NCB : 1][3];
    if constexpr (SPL) {
#pragma unroll
      for (int h2 = 0; h2 < NH; ++h2)
#pragma unroll
        for (int m = 0; m < NCB; ++m)
#pragma unroll
          for (int pc = 0; pc < 3; ++pc)
            ta[h2][m][pc] = a.tail_wsplit[((h2 * 4 + sbb + m) * 3 + pc) * 64 + lane];
    }
    __syncthreads();
    // SPL with two co blocks per wave (the 64-channel tails): the wave's blocks are the lower and
    // upper 16 channels of one 32-channel chunk, and lane (kr, jj) holds 4 channels of each: half
    // of a 16-byte piece quad.  Lanes kr and kr ^ 1 (16 apart, same pixel) swap one half so that
    // each holds a whole quad -- the even lane quad kr / 2 of the lower block, the odd lane quad
    // 2 + kr / 2 of the upper -- and the pieces go to LDS as ds_write_b128 under swz_tail.  The
    // round-3 form wrote each half with ds_write_b64 (16 rows at one quad per lane group: 4-way
    // bank conflicts, 144 conflict cycles per wave; MI355X_MICROARCH.md §LDS lane groups).
#ifndef AANET_TAIL_PAIRED  // A/B build switch (tools/build_variant.sh): 0 = the round-3 b64 staging
#define AANET_TAIL_PAIRED 1
#endif
    constexpr bool PAIRED = AANET_TAIL_PAIRED && SPL && NCB == 2;
    if constexpr (PAIRED) {
      float *sC = smem + (wc0 >> 1) * BUF;
      const bool odd = (kr & 1) != 0;
      const int unit = odd ? 2 + (kr >> 1) : (kr >> 1);
#pragma unroll
      for (int b = 0; b < NPB; ++b) {
        f32x4 v[2];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int co = co0 + 16 * (wc0 + m) + 4 * kr + r;
            const float t = apply_act((acc[m][b][r] + pb[m][r]) * ps[m][r] + ph[m][r], a.act);
            v[m][r] = co < co_end ? t : 0.f;
          }
        float f8[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float recv = __shfl_xor(odd ? v[0][r] : v[1][r], 16);
          f8[r] = odd ? recv : v[0][r];
          f8[4 + r] = odd ? v[1][r] : recv;
        }
        bf16x8_t pcs[3];
        split8_t(f8, pcs);
        __bf16 *plane = reinterpret_cast<__bf16 *>(sC);
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          *reinterpret_cast<bf16x8_t *>(plane + pc * PTT * 32 + swz_tail(16 * (wp0 + b) + jj, unit)) = pcs[pc];
        acc[0][b] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[1][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int m = 0; m < NCB && !PAIRED; ++m) {
      const int mg = wc0 + m;
      float *sC = smem + (mg >> 1) * BUF;
#pragma unroll
      for (int b = 0; b < NPB; ++b) {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + 16 * mg + 4 * kr + r;
          const float t = apply_act((acc[m][b][r] + pb[m][r]) * ps[m][r] + ph[m][r], a.act);
          v[r] = co < co_end ? t : 0.f;
        }
        if constexpr (SPL)
          put_split(reinterpret_cast<__bf16 *>(sC), PTT * 32, 16 * (wp0 + b) + jj, 4 * (mg & 1) + kr, v);
        else
          *reinterpret_cast<f32x4 *>(sC + (16 * (wp0 + b) + jj) * SP + 16 * (mg & 1) + 4 * kr) = v;
        acc[m][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int h2 = 0; h2 < NH; ++h2) {
      if constexpr (SPL) continue;  // tail weights: pre-split fragments (tail_wsplit)
      float *sW = smem + h2 * BUF + PTT * SP;
      for (int e = tid; e < KC * CO_T; e += FNT) {
        const int co2 = e / KC, cl = e % KC, c = 32 * h2 + cl;
        sW[co2 * SP + cl] = (co2 < a.Co2 && c < a.Co) ? a.tail_w[(long)co2 * a.Co + c] : 0.f;
      }
      if (CO_T == 16) {  // channels 16..31 of the single chunk were never written
        float *sC = smem;
        for (int e = tid; e < PTT * 16; e += FNT) sC[(e / 16) * SP + 16 + e % 16] = 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int h2 = 0; h2 < NH; ++h2) {
      if constexpr (SPL) {
        const __bf16 *sB = reinterpret_cast<const __bf16 *>(smem + h2 * BUF);
#pragma unroll
        for (int b = 0; b < NPB; ++b) {
          bf16x8 fb[3];
#pragma unroll
          for (int pc = 0; pc < 3; ++pc)
            fb[pc] = *reinterpret_cast<const bf16x8 *>(
                sB + pc * PTT * 32 + (PAIRED ? swz_tail(16 * (wp0 + b) + jj, kr) : swz(16 * (wp0 + b) + jj, kr)));
#pragma unroll
          for (int m = 0; m < NCB; ++m) acc[m][b] = mfma_split6(ta[h2][m], fb, acc[m][b]);
        }
      } else {
        mfma_chunk(h2);
      }
    }
  }

  // Epilogue: accumulators -> LDS [co][px] -> 16-byte row segments (+ residual) -> HBM.
  constexpr int QPR = PTT / 4;  // float4 per tile row
  constexpr int CQ = CO_T / 4;  // channel quads (NHWC output rows)
  constexpr int NE = ONH ? PTT * CQ : CO_T * QPR;
  constexpr int EPT = (NE + FNT - 1) / FNT;
  const int cout = TAIL ? a.Co2 : a.Co;
  const int cend_o = TAIL ? a.Co2 : co_end;
  const float *ebias = TAIL ? a.tail_b : a.bias;
  const float *esc = TAIL ? nullptr : a.post_scale;
  const float *esh = TAIL ? nullptr : a.post_shift;
  const int eact = TAIL ? a.tail_act : a.act;
  __syncthreads();
  float *sO = smem;
#pragma unroll
  for (int m = 0; m < NCB; ++m)
#pragma unroll
    for (int b = 0; b < NPB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sO[(16 * (wc0 + m) + 4 * kr + r) * OP + 16 * (wp0 + b) + jj] = acc[m][b][r];
  static_assert(!ONH || FNT % CQ == 0, "NHWC epilogue: one channel quad per thread");
  // NHWC output: the 4 channels of the thread's quad (the NCHW form loads per item: holding its
  // parameters here costs the DCN tail kernel spills)
  float eb[4] = {0.f, 0.f, 0.f, 0.f}, es[4] = {1.f, 1.f, 1.f, 1.f}, eh[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (ONH) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cc = min(co0 + 4 * (tid % CQ) + i, cend_o - 1);
      eb[i] = ebias ? ebias[cc] : 0.f;
      es[i] = esc ? esc[cc] : 1.f;
      eh[i] = esc ? esh[cc] : 0.f;
    }
  }
  __syncthreads();
  const long p0 = (long)tile * PTT;
  // output pixel of tile-local index px (flattened, -1 outside the image); quad q = px 4q..4q+3
  auto pix = [&](int px) -> long {
    if constexpr (HALO) {
      int y = hy0 + (px >> 4), x = hx0 + (px & 15);
      if constexpr (PH) y = pa + pd * y, x = pb + pd * x;
      return (y < a.Ho && x < a.Wo) ? (long)y * a.Wo + x : -1;
    } else {
      return p0 + px < P ? p0 + px : -1;
    }
  };
  const bool vec = HALO ? (a.Wo & 3) == 0 : (P & 3) == 0;
  auto quad_ok = [&](int q) -> bool {  // the quad is inside the image and 16-byte aligned
    if constexpr (HALO)
      return vec && hy0 + (q >> 2) < a.Ho && hx0 + 4 * (q & 3) + 3 < a.Wo;
    else
      return vec && p0 + 4 * q + 3 < P;
  };
  if constexpr (ONH) {  // [px][co] rows of 16-byte channel quads
    for (int e = tid; e < PTT * CQ; e += FNT) {
      const int px = e / CQ, cq = e % CQ, co = co0 + 4 * cq;
      const long pe = pix(px);
      if (co >= co_end || pe < 0) continue;
      f32x4 v;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = sO[(4 * cq + u) * OP + px] + eb[u];
        if (a.post_scale) t = t * es[u] + eh[u];
        v[u] = t;
      }
      const long o = ((long)n * P + pe) * a.Co + co;
      if (a.residual) v += *reinterpret_cast<const f32x4 *>(a.residual + o);
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = apply_act(v[u], a.act);
      *reinterpret_cast<f32x4 *>(a.out + o) = v;
    }
    return;
  }
  // Items (4 pixels x 1 channel) are processed two at a time with every global load of the pair
  // (residual, CSA source segments) issued before any use: a per-item load->use chain would
  // expose the HBM / L2 latency once per item.
  constexpr int EB = EPT >= 2 ? 2 : 1;
  const bool csa = TAIL && a.csa_out;
  // Every item of a thread has the same quad q = tid % QPR (FNT is a multiple of QPR): its pixel,
  // and for the CSA terms the source rows, segment start and row weights, are computed once per
  // thread here (round 5: they were recomputed per item in both passes -- an integer division and
  // 64-bit address math per item and term); per item only the channel plane changes.
  static_assert(FNT % QPR == 0, "items of a thread share their quad");
  const int qt = tid % QPR;
  const long pet = pix(4 * qt);
  const bool qokt = quad_ok(qt);
  // buffer resources over image n's planes (SGPRs) and 32-bit byte offsets per item: the output,
  // CSA output and residual at (co P + pixel) * 4, the CSA sources at (co ih iw + row + column) * 4
  // (round 5: per item a 64-bit plane product and pointer per access)
  const long img = (long)n * cout * P;
  const brsrc_t ro = buf_rsrc(a.out + img, (long)cout * P * 4);
  const brsrc_t rcs = buf_rsrc(csa ? a.csa_out + img : a.out + img, (long)cout * P * 4);
  const brsrc_t rre = buf_rsrc(a.residual ? a.residual + img : a.out + img, (long)cout * P * 4);
  const unsigned pq = qokt ? 4u * (unsigned)pet : 0u;
  brsrc_t ru[2] = {ro, ro};
  unsigned urow0[2] = {0u, 0u}, urow1[2] = {0u, 0u}, uhw[2] = {0u, 0u};
  int us0[2] = {0, 0}, uiw[2] = {4, 4};
  float uh0[2] = {1.f, 1.f}, uh1[2] = {0.f, 0.f};
  bool sfast = true;
  if (csa) {
    // (the halo tile knows its row and column; the flat form divides in 32 bits: a 64-bit
    // division here was ~150 instructions of the epilogue)
    int y, qq;
    if constexpr (HALO) {
      y = hy0 + ((4 * qt) >> 4);
      qq = (hx0 + 4 * (qt & 3)) >> 2;
    } else {
      y = qokt ? (int)pet / a.Wo : 0;
      qq = qokt ? ((int)pet % a.Wo) >> 2 : 0;  // Wo % 4 == 0 (launcher)
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j >= a.num_up) break;
      const int ih = a.up_h[j], iw = a.up_w[j], r = a.up_r[j];
      ru[j] = buf_rsrc(a.up[j] + (long)n * cout * ih * iw, (long)cout * ih * iw * 4);
      uhw[j] = 4u * (unsigned)(ih * iw);
      uiw[j] = iw;
      // PyTorch's area_pixel_compute_scale (ih / Ho) and source row, align_corners=False
      float hr = ((float)ih / (float)a.Ho) * ((float)y + 0.5f) - 0.5f;
      hr = hr < 0.f ? 0.f : hr;
      const int h1 = (int)hr, h1p = h1 < ih - 1 ? 1 : 0;
      urow0[j] = 4u * (unsigned)(h1 * iw);
      urow1[j] = 4u * (unsigned)((h1 + h1p) * iw);
      us0[j] = r == 2 ? 2 * qq - 1 : qq - 1;
      sfast = sfast && us0[j] >= 0 && us0[j] + 3 <= iw - 1;
      uh1[j] = hr - (float)h1;
      uh0[j] = 1.f - uh1[j];
    }
  }
  // the image-edge quads read clamped columns: a wave with one takes the per-column loads
  const bool wfast = __all(sfast || !qokt);
#pragma unroll
  for (int i0 = 0; i0 < EPT; i0 += EB) {
    f32x4 ev[EB], er[EB], eu[EB][2][2];
    float pbi[EB], psc[EB], psh[EB];
    bool eok[EB];
#pragma unroll
    for (int b = 0; b < EB; ++b) {
      const int e = tid + (i0 + b) * FNT;
      const int col = e / QPR, co = co0 + col;
      eok[b] = (NE % FNT == 0 || e < NE) && co < cend_o && qokt;
      if (!eok[b]) continue;
      // the channel's parameters in this load pass too: loaded in the use pass, each item
      // waited for its own
      pbi[b] = ebias ? ebias[co] : 0.f;
      psc[b] = esc ? esc[co] : 1.f;
      psh[b] = esc ? esh[co] : 0.f;
      ev[b] = *reinterpret_cast<const f32x4 *>(sO + col * OP + 4 * qt);
      if (a.residual) er[b] = buf_ld4(rre, 4u * (unsigned)(co * (int)P) + pq);
      if (csa) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= a.num_up) break;
          const unsigned pl = (unsigned)co * uhw[j];
          eu[b][j][0] = buf_seg(ru[j], pl + urow0[j], us0[j], uiw[j], wfast);
          eu[b][j][1] = buf_seg(ru[j], pl + urow1[j], us0[j], uiw[j], wfast);
        }
      }
    }
#pragma unroll
    for (int b = 0; b < EB; ++b) {
      if (!eok[b]) continue;
      const int e = tid + (i0 + b) * FNT;
      const int col = e / QPR, co = co0 + col;
      const unsigned po = 4u * (unsigned)(co * (int)P) + pq;
      const float bias = pbi[b], sc = psc[b], sh = psh[b];
      f32x4 v = ev[b];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = v[u] + bias;
        if (esc) t = t * sc + sh;
        if (a.residual) t += er[b][u];
        v[u] = apply_act(t, eact);
      }
      buf_st4(ro, po, v);
      if (csa) {
        // cross-scale sum of this output branch (nets/aggregation.py:387-400): the block output
        // (the identity term) + exact 2x/4x upsamplings of the coarser exchange terms, LeakyReLU
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= a.num_up) break;
          v += uh0[j] * hlerp(eu[b][j][0], a.up_r[j]) + uh1[j] * hlerp(eu[b][j][1], a.up_r[j]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = apply_act(v[u], a.csa_act);
        buf_st4(rcs, po, v);
        // post stage: the CSA output back into the item's own slot (its B operand)
        if constexpr (POST) *reinterpret_cast<f32x4 *>(sO + col * OP + 4 * qt) = v;
      }
    }
  }
  // pixels the quad path does not cover (P % 4 != 0, ragged last tile): one element at a time
  if (!quad_ok(QPR - 1) || !quad_ok(0)) {
    for (int e = tid; e < NE; e += FNT) {
      const int col = e / QPR, q = e % QPR, co = co0 + col;
      if (co >= cend_o || quad_ok(q)) continue;
      const float bias = ebias ? ebias[co] : 0.f;
      const float sc = esc ? esc[co] : 1.f;
      const float sh = esc ? esh[co] : 0.f;
      const f32x4 v = *reinterpret_cast<const f32x4 *>(sO + col * OP + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long pe = pix(4 * q + u);
        if (pe < 0) continue;
        const long o = ((long)n * cout + co) * P + pe;
        float t = v[u] + bias;
        if (esc) t = t * sc + sh;
        if (a.residual) t += a.residual[o];
        a.out[o] = apply_act(t, eact);
      }
    }
  }
  if constexpr (POST && TAIL && HALO && CO_T == 64 && PTT == 128 && SPL) {
    // ---- post stage (aanet_post_stage_t, NHWC out): t = W . csa + b, act, channels-last ------
    // The wave keeps its (co blocks wc0.., px blocks wp0..) layout.  B of lane (kr, jj): channels
    // {32h2 + 4kr + r, 32h2 + 16 + 4kr + r} of the pixel (rows 4kr apart in sO: 4 OP = 16 mod 32
    // banks); A: the same permutation read from the standard fragments in global memory.
    __syncthreads();  // every item's CSA value is in sO
    bf16x8 pb3[NPB][2][3];
#pragma unroll
    for (int b = 0; b < NPB; ++b)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        f32x4 lo4, hi4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          lo4[r] = sO[(32 * h2 + 4 * kr + r) * OP + 16 * (wp0 + b) + jj];
          hi4[r] = sO[(32 * h2 + 16 + 4 * kr + r) * OP + 16 * (wp0 + b) + jj];
        }
        bf16x4 h0, m0, l0, h1, m1, l1;
        split3(lo4, h0, m0, l0);
        split3(hi4, h1, m1, l1);
        pb3[b][h2][0] = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
        pb3[b][h2][1] = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
        pb3[b][h2][2] = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    const char *pw = a.post_w + ((((kr >> 1) << 4) | jj) * 16 + 8 * (kr & 1));
    typedef unsigned pu32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned pu32x4 __attribute__((ext_vector_type(4)));
    f32x4 pacc[NCB][NPB];
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
#pragma unroll
      for (int b = 0; b < NPB; ++b) pacc[m][b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        bf16x8 A[3];
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
          const char *f = pw + ((h2 * 4 + wc0 + m) * 3 + pc) * 1024;
          const pu32x2 lo = *reinterpret_cast<const pu32x2 *>(f);
          const pu32x2 hi = *reinterpret_cast<const pu32x2 *>(f + 512);
          A[pc] = __builtin_bit_cast(bf16x8, pu32x4{lo.x, lo.y, hi.x, hi.y});
        }
#pragma unroll
        for (int b = 0; b < NPB; ++b) pacc[m][b] = mfma_split6(A, pb3[b][h2], pacc[m][b]);
      }
    }
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
      const int co = 16 * (wc0 + m) + 4 * kr;
      const f32x4 bb = a.post_b ? *reinterpret_cast<const f32x4 *>(a.post_b + co)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < NPB; ++b) {
        const long pe = pix(16 * (wp0 + b) + jj);
        if (pe < 0) continue;
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(pacc[m][b][r] + bb[r], a.post_act);
        *reinterpret_cast<f32x4 *>(a.post_out + ((long)n * P + pe) * 64 + co) = v;
      }
    }
  }
}

// --------------------------------------------------------------- debug: im2col / index --
__global__ void mdcn_im2col_kernel(MdcnArgs a, float *__restrict__ col) {
  const long P = (long)a.Ho * a.Wo;
  const int K = a.kh * a.kw, cpg = a.C / a.dg;
  const long total = (long)a.C * K * P;
  const long HW = (long)a.H * a.W;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const long p = e % P;
    const int ck = (int)(e / P), c = ck / K, k = ck % K;
    Samp2 s;
    pixel_samp2(s, a, 0, c / cpg, k, p, (int)(p / a.Wo), (int)(p % a.Wo));
    col[e] = samp_val2(a.x + (long)c * HW, s);
  }
}

__global__ void mdcn_sample_index_kernel(MdcnArgs a, int *__restrict__ hl, int *__restrict__ wl,
                                         int *__restrict__ vd) {
#pragma clang fp contract(off)
  const long P = (long)a.Ho * a.Wo;
  const int K = a.kh * a.kw;
  const long total = (long)a.N * a.dg * K * P;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const long p = e % P;
    long t = e / P;
    const int k = (int)(t % K);
    t /= K;
    const int g = (int)(t % a.dg), n = (int)(t / a.dg);
    const int i = k / a.kw, j = k % a.kw, ho = (int)(p / a.Wo), wo = (int)(p % a.Wo);
    const float *off = a.offset + (long)n * a.off_bs + (long)g * 2 * K * P;
    const float h = (float)(ho * a.stride - a.pad + i * a.dil) + off[(long)(2 * k) * P + p];
    const float w = (float)(wo * a.stride - a.pad + j * a.dil) + off[(long)(2 * k + 1) * P + p];
    hl[e] = (int)floorf(h);
    wl[e] = (int)floorf(w);
    vd[e] = (h > -1.f && w > -1.f && h < (float)a.H && w < (float)a.W) ? 1 : 0;
  }
}

// ---------------------------------------------------------------------- backward --------
// (1) data/coordinate gradients.  Workgroup = (image n, 64-pixel tile, deformable group g);
// groups == 1.  gOut tile [Co][64] is staged in LDS once; per (tap k, <=32-channel chunk)
// colg = W^T gOut is formed by MFMA into LDS (the reference's `columns` never touches HBM),
// then each thread (pixel, channel subset) accumulates grad_mask / grad_offset partials
// (kernel.cu:695-767) and scatters grad_x to the 4 bilinear corners (kernel.cu:635-693,
// float atomics like the reference).
// DET: grad_x is accumulated in 64-bit fixed point (value * scale, scale a power of two chosen
// on the device from a bound on any single contribution, det_bound_kernel).  Integer adds are
// associative, so the sum -- and the fp32 grad_x converted from it -- does not depend on the
// order in which the atomics land: the deterministic backward of torch's
// use_deterministic_algorithms (the reference's col2im atomics, kernel.cu:688, are not).
// NHS (float atomics only): grad_x is scattered into an NHWC workspace [N][H*W][C] with the lanes
// of a wave on 32 consecutive channels of a corner -- each atomic instruction covers two fully used
// 128-byte lines, where the NCHW form (lanes = pixels with data-dependent corners) spreads one
// instruction over a dozen partly used lines; nhwc_to_nchw_kernel then writes grad_x.
template <int DET, int NHS = 0>
__global__ __launch_bounds__(NT) void mdcn_bwd_data_kernel(MdcnArgs a, const float *__restrict__ gout,
                                                           float *__restrict__ gx,
                                                           float *__restrict__ goff,
                                                           float *__restrict__ gmask, int GP,
                                                           int WTP, long long *__restrict__ gxi,
                                                           const double *__restrict__ det_scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Co = a.Co;
  float *sG = sm;                       // [Co][GP]      gOut tile
  float *sWt = sG + Co * GP;            // [KC][WTP]     W^T chunk
  float *sCg = sWt + KC * WTP;          // [KC][CP]      colg chunk
  float *sRed = sCg + KC * CP;          // [3][4][64]    cross-wave reduction
  float *sS = sRed + 3 * 4 * 64;        // [PT][12]      NHS: per-pixel corners, weights, mask

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long P = (long)a.Ho * a.Wo;
  const int ntiles = (int)((P + PT - 1) / PT);
  const int n = blockIdx.x / ntiles, tile = blockIdx.x % ntiles, g = blockIdx.y;
  const int K = a.kh * a.kw, cpg = a.C / a.dg, C = a.C;
  const long p = (long)tile * PT + lane;
  const bool pvalid = p < P;
  const int ho = pvalid ? (int)(p / a.Wo) : 0, wo = pvalid ? (int)(p % a.Wo) : 0;
  const long HW = (long)a.H * a.W;
  const float *xn = a.x + (long)n * C * HW;
  float *gxn = gx + (long)n * C * HW;
  long long *gxin = DET ? gxi + (long)n * C * HW : nullptr;
  const double scale = DET ? *det_scale : 1.0;
  auto scatter = [&](long idx, float v) {
    if (DET)
      atomicAdd(reinterpret_cast<unsigned long long *>(gxin + idx),
                (unsigned long long)__double2ll_rn((double)v * scale));
    else
      atomicAdd(gxn + idx, v);
  };

  for (int e = tid; e < Co * PT; e += NT) {
    const int co = e / PT, pl = e % PT;
    const long pp = (long)tile * PT + pl;
    sG[co * GP + pl] = pp < P ? gout[((long)n * Co + co) * P + pp] : 0.f;
  }

  const int kr = lane >> 4, jj = lane & 15;
  for (int k = 0; k < K; ++k) {
    Samp s;
    pixel_samp(s, a, n, g, k, pvalid ? p : 0, ho, wo);
    float gm = 0.f, goh = 0.f, gow = 0.f;
    if (NHS && wave == 0) {  // published for the chunk loop (its first barrier orders it)
#pragma clang fp contract(off)
      const bool on = pvalid && s.valid;
      const float hh = 1.f - s.lh, hw = 1.f - s.lw;
      float *q = sS + lane * 12;
      q[0] = __builtin_bit_cast(float, on && (s.ok & 1) ? s.i1 : -1);
      q[1] = __builtin_bit_cast(float, on && (s.ok & 2) ? s.i2 : -1);
      q[2] = __builtin_bit_cast(float, on && (s.ok & 4) ? s.i3 : -1);
      q[3] = __builtin_bit_cast(float, on && (s.ok & 8) ? s.i4 : -1);
      q[4] = hh * hw, q[5] = hh * s.lw, q[6] = s.lh * hw, q[7] = s.lh * s.lw;
      q[8] = s.m;
    }
    for (int c0 = g * cpg; c0 < (g + 1) * cpg; c0 += KC) {
      const int rows = min(KC, (g + 1) * cpg - c0);
      __syncthreads();  // previous chunk's sCg / sWt readers are done
      for (int e = tid; e < KC * Co; e += NT) {
        const int cl = e % KC, co = e / KC;
        sWt[cl * WTP + co] = cl < rows ? a.weight[((long)co * C + c0 + cl) * K + k] : 0.f;
      }
      __syncthreads();
      // colg[c][px] = sum_co W[co][c][k] gOut[co][px]: 2 channel blocks x this wave's 16 px.
      f32x4 cacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      for (int ks = 0; ks < Co / 4; ++ks) {
        const float bv = sG[(4 * ks + kr) * GP + 16 * wave + jj];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float av = sWt[(16 * cb + jj) * WTP + 4 * ks + kr];
          cacc[cb] = mfma16x16x4(av, bv, cacc[cb]);
        }
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) sCg[(16 * cb + 4 * kr + r) * CP + 16 * wave + jj] = cacc[cb][r];
      __syncthreads();
      if (pvalid && s.valid) {
#pragma unroll 2
        for (int ii = 0; ii < KC / 4; ++ii) {
          const int cl = wave + 4 * ii;
          if (cl >= rows) break;
          const int c = c0 + cl;
          const float cg = sCg[cl * CP + lane];
          const float *im = xn + (long)c * HW;
          const float v1 = (s.ok & 1) ? im[s.i1] : 0.f, v2 = (s.ok & 2) ? im[s.i2] : 0.f;
          const float v3 = (s.ok & 4) ? im[s.i3] : 0.f, v4 = (s.ok & 8) ? im[s.i4] : 0.f;
          const float hh = 1.f - s.lh, hw = 1.f - s.lw;
          const float val = hh * hw * v1 + hh * s.lw * v2 + s.lh * hw * v3 + s.lh * s.lw * v4;
          gm += cg * val;
          const float wh = -hw * v1 - s.lw * v2 + hw * v3 + s.lw * v4;
          const float ww = -hh * v1 + hh * v2 - s.lh * v3 + s.lh * v4;
          const float top = cg * s.m;
          goh += wh * top;
          gow += ww * top;
          if (NHS) continue;
          const long cb = (long)c * HW;
          if (s.ok & 1) scatter(cb + s.i1, hh * hw * top);
          if (s.ok & 2) scatter(cb + s.i2, hh * s.lw * top);
          if (s.ok & 4) scatter(cb + s.i3, s.lh * hw * top);
          if (s.ok & 8) scatter(cb + s.i4, s.lh * s.lw * top);
        }
      }
      if (NHS) {
        // lanes 0-31: channel cl of pixel 16w + 2t, lanes 32-63: of pixel 16w + 2t + 1
        const int cl = lane & 31;
        if (cl < rows) {
          const long cbase = (long)n * HW * C + c0 + cl;
          auto nadd = [&](int i, float v) {
            if (DET)
              atomicAdd(reinterpret_cast<unsigned long long *>(gxi + cbase + (long)i * C),
                        (unsigned long long)__double2ll_rn((double)v * scale));
            else
              atomicAdd(gx + cbase + (long)i * C, v);
          };
#pragma unroll 2
          for (int t = 0; t < 8; ++t) {
#pragma clang fp contract(off)
            const int px = 16 * wave + 2 * t + (lane >> 5);
            const float *q = sS + px * 12;
            const f32x4 qi = *reinterpret_cast<const f32x4 *>(q);
            const f32x4 qw = *reinterpret_cast<const f32x4 *>(q + 4);
            const float top = sCg[cl * CP + px] * q[8];
            const float qi0 = qi[0], qi1 = qi[1], qi2 = qi[2], qi3 = qi[3];  // (bit_cast of an
            const int i1 = __builtin_bit_cast(int, qi0), i2 = __builtin_bit_cast(int, qi1);  // element
            const int i3 = __builtin_bit_cast(int, qi2), i4 = __builtin_bit_cast(int, qi3);  // lvalue)
            if (i1 >= 0) nadd(i1, qw[0] * top);
            if (i2 >= 0) nadd(i2, qw[1] * top);
            if (i3 >= 0) nadd(i3, qw[2] * top);
            if (i4 >= 0) nadd(i4, qw[3] * top);
          }
        }
      }
    }
    // reduce the 4 waves' channel partials for each pixel
    sRed[(0 * 4 + wave) * 64 + lane] = gm;
    sRed[(1 * 4 + wave) * 64 + lane] = goh;
    sRed[(2 * 4 + wave) * 64 + lane] = gow;
    __syncthreads();
    if (wave == 0 && pvalid) {
      float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        t0 += sRed[(0 * 4 + q) * 64 + lane];
        t1 += sRed[(1 * 4 + q) * 64 + lane];
        t2 += sRed[(2 * 4 + q) * 64 + lane];
      }
      const long ob = (long)n * a.dg * 2 * K * P + (long)g * 2 * K * P;
      goff[ob + (long)(2 * k) * P + p] = t1;
      goff[ob + (long)(2 * k + 1) * P + p] = t2;
      gmask[(long)n * a.dg * K * P + ((long)g * K + k) * P + p] = t0;
    }
  }
}

// (1b) the same data/coordinate gradients from channels-last copies: x as [N][H*W][C] and the
// weight as wT[k][c][co] (both made by the launcher into the workspace), for C % 4 == 0 and
// C/dg % 4 == 0.  Workgroup = (image n, 64-pixel tile, deformable group g).  Per (tap, chunk):
//  - the W^T chunk is staged with coalesced rows of wT, colg = W^T gOut by MFMA into LDS;
//  - offset/mask partials: thread = (pixel, channel quad), each corner one 16-byte load of 4
//    channels (8 lanes = one 128-B line of a corner), reduced over the 8 quads by shuffles;
//  - grad_x: lanes on 32 consecutive channels of a corner, atomics into the NHWC accumulator.
template <int DET>
__global__ __launch_bounds__(NT) void mdcn_bwd_data_nhwc_kernel(MdcnArgs a, const float *__restrict__ xh,
                                                                const float *__restrict__ wT,
                                                                const float *__restrict__ gout,
                                                                float *__restrict__ gx,
                                                                float *__restrict__ goff,
                                                                float *__restrict__ gmask, int GP,
                                                                int WTP, long long *__restrict__ gxi,
                                                                const double *__restrict__ det_scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Co = a.Co;
  float *sG = sm;                       // [Co][GP]      gOut tile
  float *sWt = sG + Co * GP;            // [KC][WTP]     W^T chunk
  float *sCg = sWt + KC * WTP;          // [KC][CP]      colg chunk
  float *sS = sCg + KC * CP;            // [PT][12]      per-pixel corners, weights, mask, fractions
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long P = (long)a.Ho * a.Wo;
  const int ntiles = (int)((P + PT - 1) / PT);
  const int n = blockIdx.x / ntiles, tile = blockIdx.x % ntiles, g = blockIdx.y;
  const int K = a.kh * a.kw, cpg = a.C / a.dg, C = a.C;
  const long HW = (long)a.H * a.W;
  const double scale = DET ? *det_scale : 1.0;
  const float *xn = xh + (long)n * HW * C;

  for (int e = tid; e < Co * PT; e += NT) {
    const int co = e / PT, pl = e % PT;
    const long pp = (long)tile * PT + pl;
    sG[co * GP + pl] = pp < P ? gout[((long)n * Co + co) * P + pp] : 0.f;
  }
  const int kr = lane >> 4, jj = lane & 15;
  const int q = tid & 7;  // channel quad of the gradient role; pixels (tid >> 3) + 32 it
  for (int k = 0; k < K; ++k) {
    if (k) __syncthreads();  // every wave is done scattering tap k-1 (it reads sS)
    if (wave == 0) {  // published for the chunk loop (its first barrier orders it)
#pragma clang fp contract(off)
      const long p = (long)tile * PT + lane;
      const bool pvalid = p < P;
      Samp s;
      pixel_samp(s, a, n, g, k, pvalid ? p : 0, pvalid ? (int)(p / a.Wo) : 0, pvalid ? (int)(p % a.Wo) : 0);
      const bool on = pvalid && s.valid;
      const float hh = 1.f - s.lh, hw = 1.f - s.lw;
      float *qq = sS + lane * 12;
      qq[0] = __builtin_bit_cast(float, on && (s.ok & 1) ? s.i1 : -1);
      qq[1] = __builtin_bit_cast(float, on && (s.ok & 2) ? s.i2 : -1);
      qq[2] = __builtin_bit_cast(float, on && (s.ok & 4) ? s.i3 : -1);
      qq[3] = __builtin_bit_cast(float, on && (s.ok & 8) ? s.i4 : -1);
      qq[4] = hh * hw, qq[5] = hh * s.lw, qq[6] = s.lh * hw, qq[7] = s.lh * s.lw;
      qq[8] = s.m, qq[9] = s.lh, qq[10] = s.lw, qq[11] = on ? 1.f : 0.f;
    }
    float gm[2] = {0.f, 0.f}, goh[2] = {0.f, 0.f}, gow[2] = {0.f, 0.f};
    for (int c0 = g * cpg; c0 < (g + 1) * cpg; c0 += KC) {
      const int rows = min(KC, (g + 1) * cpg - c0);
      __syncthreads();  // previous chunk's sCg / sWt readers are done
      for (int e = tid; e < KC * Co; e += NT) {
        const int co = e % Co, cl = e / Co;
        sWt[cl * WTP + co] = cl < rows ? wT[((long)k * C + c0 + cl) * Co + co] : 0.f;
      }
      __syncthreads();
      f32x4 cacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      for (int ks = 0; ks < Co / 4; ++ks) {
        const float bv = sG[(4 * ks + kr) * GP + 16 * wave + jj];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float av = sWt[(16 * cb + jj) * WTP + 4 * ks + kr];
          cacc[cb] = mfma16x16x4(av, bv, cacc[cb]);
        }
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int r = 0; r < 4; ++r) sCg[(16 * cb + 4 * kr + r) * CP + 16 * wave + jj] = cacc[cb][r];
      __syncthreads();
      // offset / mask partials: (pixel, channel quad)
      if (4 * q < rows) {
#pragma unroll
        for (int it = 0; it < 2; ++it) {
#pragma clang fp contract(off)
          const int px = (tid >> 3) + 32 * it;
          const float *qq = sS + px * 12;
          const f32x4 qi = *reinterpret_cast<const f32x4 *>(qq);
          const float qi0 = qi[0], qi1 = qi[1], qi2 = qi[2], qi3 = qi[3];
          const int i1 = __builtin_bit_cast(int, qi0), i2 = __builtin_bit_cast(int, qi1);
          const int i3 = __builtin_bit_cast(int, qi2), i4 = __builtin_bit_cast(int, qi3);
          const float m = qq[8], lh = qq[9], lw = qq[10];
          const float hh = 1.f - lh, hw = 1.f - lw;
          const int cq = c0 + 4 * q;
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          const f32x4 v1 = i1 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i1 * C + cq) : z;
          const f32x4 v2 = i2 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i2 * C + cq) : z;
          const f32x4 v3 = i3 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i3 * C + cq) : z;
          const f32x4 v4 = i4 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i4 * C + cq) : z;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float cg = sCg[(4 * q + u) * CP + px];
            const float val = hh * hw * v1[u] + hh * lw * v2[u] + lh * hw * v3[u] + lh * lw * v4[u];
            gm[it] += cg * val;
            const float wh = -hw * v1[u] - lw * v2[u] + hw * v3[u] + lw * v4[u];
            const float ww = -hh * v1[u] + hh * v2[u] - lh * v3[u] + lh * v4[u];
            const float top = cg * m;
            goh[it] += wh * top;
            gow[it] += ww * top;
          }
        }
      }
      // grad_x: lanes 0-31 channel cl of pixel 16w + 2t, lanes 32-63 of pixel 16w + 2t + 1
      const int cl = lane & 31;
      if (cl < rows && !bwd_dbg(a)) {
        const long cbase = (long)n * HW * C + c0 + cl;
        auto nadd = [&](int i, float v) {
          if (DET)
            atomicAdd(reinterpret_cast<unsigned long long *>(gxi + cbase + (long)i * C),
                      (unsigned long long)__double2ll_rn((double)v * scale));
          else
            atomicAdd(gx + cbase + (long)i * C, v);
        };
#pragma unroll 2
        for (int t = 0; t < 8; ++t) {
#pragma clang fp contract(off)
          const int px = 16 * wave + 2 * t + (lane >> 5);
          const float *qq = sS + px * 12;
          const f32x4 qi = *reinterpret_cast<const f32x4 *>(qq);
          const f32x4 qw = *reinterpret_cast<const f32x4 *>(qq + 4);
          const float top = sCg[cl * CP + px] * qq[8];
          const float qi0 = qi[0], qi1 = qi[1], qi2 = qi[2], qi3 = qi[3];
          const int i1 = __builtin_bit_cast(int, qi0), i2 = __builtin_bit_cast(int, qi1);
          const int i3 = __builtin_bit_cast(int, qi2), i4 = __builtin_bit_cast(int, qi3);
          if (i1 >= 0) nadd(i1, qw[0] * top);
          if (i2 >= 0) nadd(i2, qw[1] * top);
          if (i3 >= 0) nadd(i3, qw[2] * top);
          if (i4 >= 0) nadd(i4, qw[3] * top);
        }
      }
    }
    // reduce the 8 channel quads of each pixel (lanes 8j .. 8j+7), fixed order
#pragma unroll
    for (int it = 0; it < 2; ++it) {
#pragma unroll
      for (int msk = 1; msk < 8; msk <<= 1) {
        gm[it] += __shfl_xor(gm[it], msk);
        goh[it] += __shfl_xor(goh[it], msk);
        gow[it] += __shfl_xor(gow[it], msk);
      }
      const long p = (long)tile * PT + (tid >> 3) + 32 * it;
      if (q == 0 && p < P) {
        const long ob = (long)n * a.dg * 2 * K * P + (long)g * 2 * K * P;
        goff[ob + (long)(2 * k) * P + p] = goh[it];
        goff[ob + (long)(2 * k + 1) * P + p] = gow[it];
        gmask[(long)n * a.dg * K * P + ((long)g * K + k) * P + p] = gm[it];
      }
    }
  }
}

// Window form of mdcn_bwd_data_nhwc_kernel (stride 1 or 2, <= 128 channels per deformable group,
// K <= 9 taps, <= 128 output channels; round 6 added the feature extractor's stride-2, 64-channel
// group, Co = 128 shapes).  The workgroup owns an 8 x 8 output tile and one deformable group, and walks the
// group's channels in 16-channel slices: per slice it sums the grad_x corner contributions in an
// LDS copy of the tile's input window (rows/cols [origin, origin + WR/WC): the corners of every
// offset in [-R, R)), then adds the window to the global accumulator once -- one global add per
// window element instead of one per (pixel, tap, corner, channel).  Corners outside the window
// take a global atomic directly.
// The window is INT64 FIXED POINT in both modes (scale 2^(38 - ceil(log2 bound)), computed on
// the device by det_scale_kernel): an LDS ds_add_u64 costs ~26 cycles per wave-instruction per CU
// against ~196 for ds_add_f32 (tools/lds_rmw_lab.hip, profiles/r04_lds_scatter_probe.txt), and
// the integer sums do not depend on the order.  The 16-channel slice keeps the window at 32 KB
// (two workgroups per CU).  DET: the window and the out-of-window corners go to the int64 global
// accumulator (bit-reproducible); otherwise the window is converted once to float and added with
// float atomics (its per-tile sums are exact to 2^-38 of the bound before that one rounding).
// grad_offset / grad_mask: the first slice's per-(tap, pixel) channel sums wait in LDS (sP) and
// the last slice adds its own and stores the result -- no atomics, fixed order.
// Taps are software-pipelined: the raw offsets / mask of the next tap (wave 0, lane = pixel) and
// this thread's elements of the next tap's W^T slice are loaded into registers one tap ahead.
// Round 4 also tried an atomic-free "owner computes" form (per-tap tables of the pixels whose
// corner block starts at each window position): bit-reproducible, but slower -- agg_s0 backward
// 7.84 ms float / 8.20 ms fixed point: the owner loop is a chain of dependent LDS reads per window
// position and tap.  It is in the git history (round 4).
// FUSEW (float mode): the weight gradient of the tile rides along -- the sampled column values
// (the forward's (w1 v1 + w2 v2 + w3 v3 + w4 v4) * mask, from the corner quads the offset / mask
// partials load anyway) go to LDS, one 16x16x4 f32 MFMA run per (tap, slice) forms the tile's
// [64 co][16 c] product with the staged gOut tile, and it is added with float atomics into a
// [K][Co][C] accumulator (64-byte segments; transposed into grad_weight afterwards).  DET: the
// same products go to an int64 fixed-point [K][Co][C] accumulator (scale det_scale[1]), so the sum
// does not depend on the order of the tiles and the workspace holds one copy of the weight
// gradient (round 4 stored a float partial per tile and reduced them in a fixed order: ~0.08 ms
// faster at agg_s0, but ~0.9 GB of workspace at B = 8).  This replaces mdcn_bwd_weight_kernel,
// whose 18 chunks each re-read gOut and re-gathered the corners.
// dynamic LDS: sG [Co][GP], sWt [16][WTP], sCg [16][CP], sS [PT][16], sP [3][9][PT],
// [FUSEW: sCol [16][CP]], window [WR*WC][16] int64
constexpr int WHC = 16;  // channels per window slice
// row pitch of the colg / column tiles of the window kernel: 66 (= 2 mod 32) makes the partials'
// (rows 4q+u, lanes q), the scatter's and the fused weight gradient's (rows = lane % 16) reads
// conflict-free; the engine's CP = 80 left them 4- to 8-way conflicted
constexpr int WCP = PT + 2;
constexpr int WKMAX = 9; // taps the sP partial buffer holds
constexpr int WCOMAX = 128;  // output channels (the W^T slice is prefetched in registers)
constexpr int GW_COPIES = 8; // copies of the fused weight-gradient accumulator, summed afterwards
template <int DET, int FUSEW = 0>
__global__ __launch_bounds__(NT, 2) void mdcn_bwd_data_win_kernel(MdcnArgs a, const float *__restrict__ xh,
                                                               const float *__restrict__ wT,
                                                               const float *__restrict__ gout,
                                                               float *__restrict__ gx,
                                                               float *__restrict__ goff,
                                                               float *__restrict__ gmask, int GP,
                                                               int WTP, long long *__restrict__ gxi,
                                                               const double *__restrict__ det_scale,
                                                               int WR, int WCc, int R,
                                                               float *__restrict__ gwT = nullptr,
                                                               long long *__restrict__ gwi = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int Co = a.Co;
  float *sG = sm;                       // [Co][GP]      gOut tile
  float *sWt = sG + Co * GP;            // [16][WTP]     W^T slice
  float *sCg = sWt + WHC * WTP;         // [16][WCP]      colg slice
  float *sS = sCg + WHC * WCP;           // [PT][16]      per-pixel corners, weights, mask, window pos
  float *sP = sS + PT * 16;             // [3][WKMAX][PT] first slice's grad_offset / mask sums
  float *sCol = sP + 3 * WKMAX * PT;    // [16][WCP]      sampled columns (FUSEW)
  long long *sAcc = reinterpret_cast<long long *>(sCol + (FUSEW ? WHC * WCP : 0));  // [WR*WC][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long P = (long)a.Ho * a.Wo;
  const int ttx = (a.Wo + 7) / 8, tpi = ttx * ((a.Ho + 7) / 8);
  const int K = a.kh * a.kw, cpg = a.C / a.dg, C = a.C;
  const int NH = (cpg + WHC - 1) / WHC;
  const int n = blockIdx.x / tpi, tile = blockIdx.x % tpi, g = blockIdx.y;
  const int ty0 = (tile / ttx) * 8, tx0 = (tile % ttx) * 8;
  const long HW = (long)a.H * a.W;
  const double scale = *det_scale;
  const double inv = 1.0 / scale;
  const double wscale = DET && FUSEW ? det_scale[1] : 1.0;  // the weight gradient's fixed point
  // the weight-gradient accumulator copy of this workgroup (consecutive workgroups run on
  // different XCDs: one copy per XCD keeps the atomics on one element from crossing them)
  const long gwc = (long)(blockIdx.x & (GW_COPIES - 1)) * K * Co * C;
  const float *xn = xh + (long)n * HW * C;
  // window origin: the tile's first input row / column (stride s: 8 output pixels span 7s + 1)
  const int wy0 = ty0 * a.stride - a.pad - R, wx0 = tx0 * a.stride - a.pad - R;
  const int nwin = WR * WCc * WHC;
  auto pix = [&](int pl) -> long {  // linear output pixel of tile pixel pl, or -1
    const int y = ty0 + (pl >> 3), x = tx0 + (pl & 7);
    return (y < a.Ho && x < a.Wo) ? (long)y * a.Wo + x : -1;
  };
  for (int e = tid; e < Co * PT; e += NT) {
    const int co = e / PT, pl = e % PT;
    const long pp = pix(pl);
    sG[co * GP + pl] = pp >= 0 ? gout[((long)n * Co + co) * P + pp] : 0.f;
  }
  const int kr = lane >> 4, jj = lane & 15;
  const int q = tid & 3, qpx = tid >> 2;  // gradient role: channel quad q of pixel qpx
  const long sp = pix(lane);
  const int sy = sp >= 0 ? (int)(sp / a.Wo) : 0, sx = sp >= 0 ? (int)(sp % a.Wo) : 0;
  const float *offg = a.offset + (long)n * a.off_bs + (long)g * 2 * K * P + (sp >= 0 ? sp : 0);
  constexpr int WPT = WHC * WCOMAX / NT;  // W^T slice elements per thread
  float roh = 0.f, row = 0.f, rm = 0.f, rw[WPT];
  auto prefetch = [&](int kk, int c0) {  // tap kk's offsets / mask and W^T rows c0 .. c0+15
    if (wave == 0) {
      roh = offg[(long)(2 * kk) * P];
      row = offg[(long)(2 * kk + 1) * P];
      rm = a.mask[(long)n * a.mask_bs + ((long)g * K + kk) * P + (sp >= 0 ? sp : 0)];
    }
    const int nr = min(WHC, (g + 1) * cpg - c0);
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
      const int e = tid + NT * j, co = e % Co, cl = e / Co;
      rw[j] = (e < WHC * Co && cl < nr) ? wT[((long)kk * C + c0 + cl) * Co + co] : 0.f;
    }
  };
  prefetch(0, g * cpg);
  for (int sl = 0; sl < NH; ++sl) {
    const int cb0 = g * cpg + sl * WHC, rows = min(WHC, (g + 1) * cpg - cb0);
    const bool last = sl == NH - 1;
    for (int e = tid; e < nwin; e += NT) sAcc[e] = 0;  // ordered by the first tap's barrier
    for (int k = 0; k < K; ++k) {
      __syncthreads();  // every wave is done with tap k-1 (sS, sWt, sCg) and the last flush
      if (wave == 0) {
#pragma clang fp contract(off)
        const bool pvalid = sp >= 0;
        const int i = k / a.kw, j = k % a.kw;
        const float m = a.mask_logits ? a.mask_scale * (1.f / (1.f + expf(-rm))) : rm;  // deform.py:86-89
        Samp s;
        make_samp(s, (float)(sy * a.stride - a.pad + i * a.dil) + roh,
                  (float)(sx * a.stride - a.pad + j * a.dil) + row, a.H, a.W, m);
        const bool on = pvalid && s.valid;
        const float hh = 1.f - s.lh, hw = 1.f - s.lw;
        float *qq = sS + lane * 16;
        qq[0] = __builtin_bit_cast(float, on && (s.ok & 1) ? s.i1 : -1);
        qq[1] = __builtin_bit_cast(float, on && (s.ok & 2) ? s.i2 : -1);
        qq[2] = __builtin_bit_cast(float, on && (s.ok & 4) ? s.i3 : -1);
        qq[3] = __builtin_bit_cast(float, on && (s.ok & 8) ? s.i4 : -1);
        qq[4] = hh * hw, qq[5] = hh * s.lw, qq[6] = s.lh * hw, qq[7] = s.lh * s.lw;
        qq[8] = s.m, qq[9] = s.lh, qq[10] = s.lw, qq[11] = on ? 1.f : 0.f;
        // window position of the 2x2 corner block (top-left), or -1: global atomics
        int wpos = -1;
        if (on) {
          const int rh = s.hl - wy0, rw_ = s.wl - wx0;
          if ((unsigned)rh <= (unsigned)(WR - 2) && (unsigned)rw_ <= (unsigned)(WCc - 2)) wpos = rh * WCc + rw_;
        }
        qq[12] = __builtin_bit_cast(float, wpos);
      }
#pragma unroll
      for (int j = 0; j < WPT; ++j) {
        const int e = tid + NT * j, co = e % Co, cl = e / Co;
        if (e < WHC * Co) sWt[cl * WTP + co] = rw[j];
      }
      if (k + 1 < K)
        prefetch(k + 1, cb0);
      else if (!last)
        prefetch(0, cb0 + WHC);
      __syncthreads();
      // corner quads of the offset / mask partials (pixel qpx, channel quad q), issued before the
      // colg MFMAs so their latency overlaps them
      const float *qq = sS + qpx * 16;
      const f32x4 qi = *reinterpret_cast<const f32x4 *>(qq);
      const float qi0 = qi[0], qi1 = qi[1], qi2 = qi[2], qi3 = qi[3];
      const int i1 = __builtin_bit_cast(int, qi0), i2 = __builtin_bit_cast(int, qi1);
      const int i3 = __builtin_bit_cast(int, qi2), i4 = __builtin_bit_cast(int, qi3);
      const bool qon = 4 * q < rows;
      const int cq = cb0 + 4 * q;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 v1 = qon && i1 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i1 * C + cq) : z;
      const f32x4 v2 = qon && i2 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i2 * C + cq) : z;
      const f32x4 v3 = qon && i3 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i3 * C + cq) : z;
      const f32x4 v4 = qon && i4 >= 0 ? *reinterpret_cast<const f32x4 *>(xn + (long)i4 * C + cq) : z;
      f32x4 cacc = {0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < Co / 4; ++ks) {
        const float bv = sG[(4 * ks + kr) * GP + 16 * wave + jj];
        const float av = sWt[jj * WTP + 4 * ks + kr];
        cacc = mfma16x16x4(av, bv, cacc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sCg[(4 * kr + r) * WCP + 16 * wave + jj] = cacc[r];
      if constexpr (FUSEW) {
#pragma clang fp contract(off)
        // the forward's sampled value (samp_val order) times the mask; zeros past the slice
        const f32x4 wq = *reinterpret_cast<const f32x4 *>(qq + 4);
        const float mq = qq[8];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          sCol[(4 * q + u) * WCP + qpx] = (wq[0] * v1[u] + wq[1] * v2[u] + wq[2] * v3[u] + wq[3] * v4[u]) * mq;
      }
      __syncthreads();
      if constexpr (FUSEW) {
        // this tile's weight-gradient block: wave w = output channels cbk + 16w .. + 15 for each
        // 64-channel block cbk (Co <= 128, Co % 16 == 0: whole blocks), the slice's 16 channels,
        // K = the tile's 64 pixels; one float atomic per element into gwT[k][co][c]
        for (int cbk = 0; cbk < Co; cbk += 64) {
          const int cw = cbk + 16 * wave;  // wave-uniform
          if (cw >= Co) break;
          f32x4 wacc = {0.f, 0.f, 0.f, 0.f};
          for (int ks = 0; ks < PT / 4; ++ks) {
            const float av = sG[(cw + jj) * GP + 4 * ks + kr];
            const float bv = sCol[jj * WCP + 4 * ks + kr];
            wacc = mfma16x16x4(av, bv, wacc);
          }
          if (jj < rows) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int co = cw + 4 * kr + r;
              if (DET)  // int64 fixed point: the sum does not depend on the order of the tiles
                atomicAdd(reinterpret_cast<unsigned long long *>(gwi) + gwc + ((long)k * Co + co) * C + cb0 + jj,
                          (unsigned long long)__double2ll_rn((double)wacc[r] * wscale));
              else
                atomicAdd(gwT + gwc + ((long)k * Co + co) * C + cb0 + jj, wacc[r]);
            }
          }
        }
      }
      float gm = 0.f, goh = 0.f, gow = 0.f;
      if (qon) {
#pragma clang fp contract(off)
        const float m = qq[8], lh = qq[9], lw = qq[10];
        const float hh = 1.f - lh, hw = 1.f - lw;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float cg = sCg[(4 * q + u) * WCP + qpx];
          const float val = hh * hw * v1[u] + hh * lw * v2[u] + lh * hw * v3[u] + lh * lw * v4[u];
          gm += cg * val;
          const float wh = -hw * v1[u] - lw * v2[u] + hw * v3[u] + lw * v4[u];
          const float ww = -hh * v1[u] + hh * v2[u] - lh * v3[u] + lh * v4[u];
          const float top = cg * m;
          goh += wh * top;
          gow += ww * top;
        }
      }
      // grad_x: lane (pixel 16 w + 4 t + lane / 16, channel lane % 16)
      const int cl = lane & 15;
      if (cl < rows && bwd_dbg(a) != 1) {
        const long cbase = (long)n * HW * C + cb0 + cl;
#pragma unroll 2
        for (int t = 0; t < 4; ++t) {
#pragma clang fp contract(off)
          const int px = 16 * wave + 4 * t + (lane >> 4);
          const float *qp = sS + px * 16;
          const f32x4 pi = *reinterpret_cast<const f32x4 *>(qp);
          const f32x4 qw = *reinterpret_cast<const f32x4 *>(qp + 4);
          const float top = sCg[cl * WCP + px] * qp[8];
          const float pi0 = pi[0], pi1 = pi[1], pi2 = pi[2], pi3 = pi[3], q12 = qp[12];
          const int j1 = __builtin_bit_cast(int, pi0), j2 = __builtin_bit_cast(int, pi1);
          const int j3 = __builtin_bit_cast(int, pi2), j4 = __builtin_bit_cast(int, pi3);
          const int wp = __builtin_bit_cast(int, q12);
          if (wp >= 0) {  // corners outside the image have index -1 (skipped), as below
            unsigned long long *w0 = reinterpret_cast<unsigned long long *>(sAcc) + (long)wp * WHC + cl;
            if (j1 >= 0) atomicAdd(w0, (unsigned long long)__double2ll_rn((double)(qw[0] * top) * scale));
            if (j2 >= 0) atomicAdd(w0 + WHC, (unsigned long long)__double2ll_rn((double)(qw[1] * top) * scale));
            if (j3 >= 0) atomicAdd(w0 + WCc * WHC, (unsigned long long)__double2ll_rn((double)(qw[2] * top) * scale));
            if (j4 >= 0) atomicAdd(w0 + (WCc + 1) * WHC, (unsigned long long)__double2ll_rn((double)(qw[3] * top) * scale));
          } else {
            auto gadd = [&](int i, float v) {
              if (DET)
                atomicAdd(reinterpret_cast<unsigned long long *>(gxi + cbase + (long)i * C),
                          (unsigned long long)__double2ll_rn((double)v * scale));
              else
                atomicAdd(gx + cbase + (long)i * C, v);
            };
            if (j1 >= 0) gadd(j1, qw[0] * top);
            if (j2 >= 0) gadd(j2, qw[1] * top);
            if (j3 >= 0) gadd(j3, qw[2] * top);
            if (j4 >= 0) gadd(j4, qw[3] * top);
          }
        }
      }
      // reduce the 4 channel quads of each pixel (lanes 4j .. 4j+3), fixed order; the first
      // slice parks its sums in sP, the last adds them (slice order) and stores
#pragma unroll
      for (int msk = 1; msk < 4; msk <<= 1) {
        gm += __shfl_xor(gm, msk);
        goh += __shfl_xor(goh, msk);
        gow += __shfl_xor(gow, msk);
      }
      if (q == 0) {
        float *pp = sP + k * PT + qpx;
        if (sl > 0) {
          goh = pp[0] + goh;
          gow = pp[WKMAX * PT] + gow;
          gm = pp[2 * WKMAX * PT] + gm;
        }
        if (!last) {
          pp[0] = goh, pp[WKMAX * PT] = gow, pp[2 * WKMAX * PT] = gm;
        } else {
          const long p = pix(qpx);
          if (p >= 0) {
            const long ob = (long)n * a.dg * 2 * K * P + (long)g * 2 * K * P;
            goff[ob + (long)(2 * k) * P + p] = goh;
            goff[ob + (long)(2 * k + 1) * P + p] = gow;
            gmask[(long)n * a.dg * K * P + ((long)g * K + k) * P + p] = gm;
          }
        }
      }
    }
    __syncthreads();  // the slice's window is complete
    if (bwd_dbg(a)) continue;
    // add the window to the global accumulator: consecutive threads take consecutive channels of a
    // position (16 lanes = one 64-byte (float) / 128-byte (int64) segment); zero elements skipped
    for (int e = tid; e < nwin; e += NT) {
      const int pos = e / WHC, wc = e - pos * WHC;
      const int gy = wy0 + pos / WCc, gxp = wx0 + pos % WCc;
      if (wc >= rows || gy < 0 || gy >= a.H || gxp < 0 || gxp >= a.W) continue;
      const long o = ((long)n * HW + (long)gy * a.W + gxp) * C + cb0 + wc;
      const long long v = sAcc[e];
      // a non-finite bound (scale = NaN) converts every contribution to 0: add the NaN read-back
      // anyway (float mode), so grad_x is poisoned like the reference's float col2im
      if (!v && (DET || inv == inv)) continue;
      if (DET)
        atomicAdd(reinterpret_cast<unsigned long long *>(gxi + o), (unsigned long long)v);
      else
        atomicAdd(gx + o, (float)((double)v * inv));
    }
  }
}

// grad_weight [Co][C][K] += gwi [K][Co][C] / scale (the deterministic window form's int64
// fixed-point weight-gradient accumulator; NaN scale -> NaN, as det_scale_kernel says)
__global__ __launch_bounds__(256) void det_gw_final_kernel(const long long *__restrict__ gwi,
                                                           float *__restrict__ gw, int Co, int C, int K,
                                                           const double *__restrict__ wscale) {
  const long nw = (long)Co * C * K;
  const double inv = 1.0 / *wscale;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nw; e += (long)gridDim.x * 256) {
    const int k = (int)(e % K), c = (int)((e / K) % C), co = (int)(e / ((long)K * C));
    long long v = 0;
#pragma unroll
    for (int j = 0; j < GW_COPIES; ++j) v += gwi[j * nw + ((long)k * Co + co) * C + c];
    gw[e] += (float)((double)v * inv);
  }
}

// grad_weight [Co][C][K] += gwT [K][Co][C] (the fused window form's accumulator)
__global__ __launch_bounds__(256) void gw_kcoc_add_kernel(const float *__restrict__ gwT,
                                                          float *__restrict__ gw, int Co, int C, int K) {
  const long nw = (long)Co * C * K;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nw; e += (long)gridDim.x * 256) {
    const int k = (int)(e % K), c = (int)((e / K) % C), co = (int)(e / ((long)K * C));
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < GW_COPIES; ++j) v += gwT[j * nw + ((long)k * Co + co) * C + c];
    gw[e] += v;
  }
}

// x [N][C][HW] -> [N][HW][C] and w [Co][C][K] -> wT [K][C][Co] (inputs of mdcn_bwd_data_nhwc_kernel)
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float *__restrict__ src,
                                                           float *__restrict__ dst, int C, long HW) {
  __shared__ float t[32][33];
  const int n = blockIdx.z;
  const long s0 = (long)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float *sn = src + (long)n * C * HW;
  float *dn = dst + (long)n * HW * C;
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r;
    t[r][tx] = (c < C && s0 + tx < HW) ? sn[(long)c * HW + s0 + tx] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const long sp = s0 + r;
    if (sp < HW && c0 + tx < C) dn[sp * C + c0 + tx] = t[tx][r];
  }
}

__global__ __launch_bounds__(256) void weight_kcco_kernel(const float *__restrict__ w,
                                                          float *__restrict__ wT, int Co, int C, int K) {
  const long n = (long)Co * C * K;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int co = (int)(e % Co), c = (int)((e / Co) % C), k = (int)(e / ((long)Co * C));
    wT[e] = w[((long)co * C + c) * K + k];
  }
}

// (2) weight gradient: gW[co][c][k] += sum_{n,p} gOut[n][co][p] * col[c*K+k][n,p].
// Workgroup = one K chunk (tap k, <=32 channels of group g) x one range of pixels (all
// images flattened) x one 64-wide output-channel tile.  The col chunk is re-sampled into LDS
// per 64-pixel sub-tile, the [co][c] tile accumulates in MFMA registers across the whole
// pixel range, then one float atomic per element (grad accumulates, cpp:660-669).
// DET: each pixel-range split writes its partial sums to part[split][co][c][k] (no atomics);
// det_weight_reduce_kernel adds them to grad_weight in split order.
// NR: the col chunk is sampled from the channels-last copy xh [N][H*W][C] (C, C/dg % 4 == 0):
// thread = (pixel, channel quad), one 16-byte load per corner (8 lanes = one 128-B line); the
// sub-tile loop is software-pipelined (see the NR branch).
// PLAIN: the weight gradient of an ordinary (grouped) convolution (aanet_conv2d_wgrad_f32): the
// col chunk is the tap's shifted window of x (zero outside), a.dg carries the conv's groups,
// grad_weight is [Co][C/groups][K] and output-channel tiles stay inside the chunk's group.
template <int DET, int NR = 0, int PLAIN = 0>
__global__ __launch_bounds__(NT) void mdcn_bwd_weight_kernel(MdcnArgs a, const float *__restrict__ gout,
                                                             float *__restrict__ gw, int npieces,
                                                             long range, float *__restrict__ part,
                                                             const float *__restrict__ xh = nullptr) {
  constexpr int GP2 = PT + 2;  // A/B reads (16 rows x 4 cols per 16 lanes) conflict-free
  __shared__ __attribute__((aligned(16))) float sG[64 * GP2];
  __shared__ __attribute__((aligned(16))) float sC[KC * GP2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long P = (long)a.Ho * a.Wo, T = (long)a.N * P;
  const int K = a.kh * a.kw, cpg = a.C / a.dg, C = a.C, Co = a.Co;
  const int chunk = blockIdx.x;
  const int k = chunk / (a.dg * npieces), rem = chunk % (a.dg * npieces);
  const int g = rem / npieces, piece = rem % npieces;
  const int c0 = g * cpg + piece * KC, rows = min(KC, (g + 1) * cpg - c0);
  const int cog = PLAIN ? Co / a.dg : Co;  // output channels of the chunk's group
  const int co0 = (PLAIN ? g * cog : 0) + blockIdx.z * 64, coE = PLAIN ? (g + 1) * cog : Co;
  const int Cw = PLAIN ? cpg : C, cw0 = PLAIN ? c0 - g * cpg : c0;  // grad_weight's [co][c] view
  const long r0 = (long)blockIdx.y * range, r1 = min(r0 + range, T);
  const long HW = (long)a.H * a.W;
  const int kr = lane >> 4, jj = lane & 15;
  // wave w: output-channel block w (16 co), both 16-channel blocks of the chunk
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if constexpr (PLAIN) {
    // software-pipelined: the next sub-tile's column values and grad_out tile are loaded into
    // registers while the MFMAs of the current one run from LDS
    float rc[KC / 4], rg[64 * PT / NT];
    const int ki = (k / a.kw) * a.dil - a.pad, kj = (k % a.kw) * a.dil - a.pad;
    auto load = [&](long t0) {
      const long t = t0 + lane;
      const int n = t < r1 ? (int)(t / P) : 0;
      const long p = t < r1 ? t % P : 0;
      const int hi = (int)(p / a.Wo) * a.stride + ki, wi = (int)(p % a.Wo) * a.stride + kj;
      const bool ok = t < r1 && hi >= 0 && hi < a.H && wi >= 0 && wi < a.W;
      const float *xn = a.x + (long)n * C * HW + (long)hi * a.W + wi;
#pragma unroll
      for (int ii = 0; ii < KC / 4; ++ii) {
        const int cl = wave + 4 * ii;
        rc[ii] = (cl < rows && ok) ? xn[(long)(c0 + cl) * HW] : 0.f;
      }
      const float *gp = gout + (long)n * Co * P + p;  // thread = pixel lane, rows wave + 4i
#pragma unroll
      for (int i = 0; i < 64 * PT / NT; ++i) {
        const int co = co0 + wave + 4 * i;
        rg[i] = (t < r1 && co < coE) ? gp[(long)co * P] : 0.f;
      }
    };
    auto store = [&]() {
#pragma unroll
      for (int ii = 0; ii < KC / 4; ++ii) sC[(wave + 4 * ii) * GP2 + lane] = rc[ii];
#pragma unroll
      for (int i = 0; i < 64 * PT / NT; ++i) sG[(wave + 4 * i) * GP2 + lane] = rg[i];
    };
    load(r0);
    store();
    __syncthreads();
    for (long t0 = r0; t0 < r1; t0 += PT) {
      const bool more = t0 + PT < r1;
      if (more) load(t0 + PT);
#pragma unroll 4
      for (int ks = 0; ks < PT / 4; ++ks) {
        const float av = sG[(16 * wave + jj) * GP2 + 4 * ks + kr];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float bv = sC[(16 * cb + jj) * GP2 + 4 * ks + kr];
          acc[cb] = mfma16x16x4(av, bv, acc[cb]);
        }
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }
  if constexpr (NR && !PLAIN) {
    // Three-stage pipeline over the 64-pixel sub-tiles: the offsets / mask of sub-tile t+2 and
    // the corner quads + grad_out tile of t+1 are loaded while the MFMAs of t run from LDS
    // (sampling positions depend on the offsets: two dependent load levels per sub-tile).
    const int q = tid & 7;
    const int K2 = 2 * K;
    float oh[2][2], ow[2][2], om[2][2];  // [stage slot][it]
    f32x4 rc[2][4];                       // corner quads of the next sub-tile, per it
    float rwt[2][5];                      // w1..w4, mask
    float rg[64 * PT / NT];
    auto off_load = [&](long t0, int sl) {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const long t = t0 + (tid >> 3) + 32 * it;
        const bool tv = t < r1;
        const int n = tv ? (int)(t / P) : 0;
        const long p = tv ? t % P : 0;
        const float *off = a.offset + (long)n * a.off_bs + (long)g * K2 * P;
        oh[sl][it] = tv ? off[(long)(2 * k) * P + p] : 0.f;
        ow[sl][it] = tv ? off[(long)(2 * k + 1) * P + p] : 0.f;
        om[sl][it] = tv ? load_mask(a, n, g, k, K, P, p) : 0.f;
      }
    };
    auto corner_load = [&](long t0, int sl) {
#pragma clang fp contract(off)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const long t = t0 + (tid >> 3) + 32 * it;
        const bool tv = t < r1;
        const int n = tv ? (int)(t / P) : 0;
        const long p = tv ? t % P : 0;
        const int ho = (int)(p / a.Wo), wo = (int)(p % a.Wo);
        const float h = (float)(ho * a.stride - a.pad + (k / a.kw) * a.dil) + oh[sl][it];
        const float w = (float)(wo * a.stride - a.pad + (k % a.kw) * a.dil) + ow[sl][it];
        Samp sp;
        make_samp(sp, h, w, a.H, a.W, om[sl][it]);
        const bool ok = tv && 4 * q < rows;
        const float *xq = xh + (long)n * HW * C + c0 + 4 * q;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        rc[it][0] = ok ? *reinterpret_cast<const f32x4 *>(xq + (long)sp.i1 * C) : z;
        rc[it][1] = ok ? *reinterpret_cast<const f32x4 *>(xq + (long)sp.i2 * C) : z;
        rc[it][2] = ok ? *reinterpret_cast<const f32x4 *>(xq + (long)sp.i3 * C) : z;
        rc[it][3] = ok ? *reinterpret_cast<const f32x4 *>(xq + (long)sp.i4 * C) : z;
        rwt[it][0] = sp.w1;
        rwt[it][1] = sp.w2;
        rwt[it][2] = sp.w3;
        rwt[it][3] = sp.w4;
        rwt[it][4] = ok ? sp.m : 0.f;  // 0 * (finite corners) = 0: masked-out rows stage zeros
      }
      const long t = t0 + lane;
      const int n = t < r1 ? (int)(t / P) : 0;
      const long p = t < r1 ? t % P : 0;
      const float *gp = gout + (long)n * Co * P + p;
#pragma unroll
      for (int i = 0; i < 64 * PT / NT; ++i) {
        const int co = co0 + wave + 4 * i;
        rg[i] = (t < r1 && co < coE) ? gp[(long)co * P] : 0.f;
      }
    };
    auto store = [&]() {
#pragma clang fp contract(off)
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int pl = (tid >> 3) + 32 * it;
#pragma unroll
        for (int u = 0; u < 4; ++u)  // samp_val per channel (same products and order)
          sC[(4 * q + u) * GP2 + pl] = (rwt[it][0] * rc[it][0][u] + rwt[it][1] * rc[it][1][u] +
                                        rwt[it][2] * rc[it][2][u] + rwt[it][3] * rc[it][3][u]) * rwt[it][4];
      }
#pragma unroll
      for (int i = 0; i < 64 * PT / NT; ++i) sG[(wave + 4 * i) * GP2 + lane] = rg[i];
    };
    off_load(r0, 0);
    corner_load(r0, 0);
    if (r0 + PT < r1) off_load(r0 + PT, 1);
    store();
    __syncthreads();
    int sl = 1;  // offset slot of sub-tile t0 + PT
    for (long t0 = r0; t0 < r1; t0 += PT) {
      const bool more = t0 + PT < r1;
      if (more) {
        corner_load(t0 + PT, sl);
        if (t0 + 2 * PT < r1) off_load(t0 + 2 * PT, sl ^ 1);
      }
#pragma unroll 4
      for (int ks = 0; ks < PT / 4; ++ks) {
        const float av = sG[(16 * wave + jj) * GP2 + 4 * ks + kr];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          const float bv = sC[(16 * cb + jj) * GP2 + 4 * ks + kr];
          acc[cb] = mfma16x16x4(av, bv, acc[cb]);
        }
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
      sl ^= 1;
    }
  }
  // NCHW x (neither PLAIN nor NR): the sampled col chunk and the grad_out tile per sub-tile
  for (long t0 = r0; t0 < r1 && !PLAIN && !NR; t0 += PT) {
    const long t = t0 + lane;
    const bool tv = t < r1;
    const int n = tv ? (int)(t / P) : 0;
    const long p = tv ? t % P : 0;
    Samp s;
    pixel_samp(s, a, n, g, k, p, (int)(p / a.Wo), (int)(p % a.Wo));
    const float *xn = a.x + (long)n * C * HW;
#pragma unroll
    for (int ii = 0; ii < KC / 4; ++ii) {
      const int cl = wave + 4 * ii;
      float v = 0.f;
      if (cl < rows && tv) v = samp_val(xn + (long)(c0 + cl) * HW, s);
      sC[cl * GP2 + lane] = v;
    }
    for (int e = tid; e < 64 * PT; e += NT) {
      const int col = e / PT, pl = e % PT;
      const long tt = t0 + pl;
      const int co = co0 + col;
      float v = 0.f;
      if (tt < r1 && co < coE) v = gout[((long)(tt / P) * Co + co) * P + tt % P];
      sG[col * GP2 + pl] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int ks = 0; ks < PT / 4; ++ks) {
      const float av = sG[(16 * wave + jj) * GP2 + 4 * ks + kr];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const float bv = sC[(16 * cb + jj) * GP2 + 4 * ks + kr];
        acc[cb] = mfma16x16x4(av, bv, acc[cb]);
      }
    }
    __syncthreads();
  }
  // D[i = co (4kr + r)][jj = channel]
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * wave + 4 * kr + r, cl = 16 * cb + jj;
      if (co < coE && cl < rows) {
        const long e = ((long)co * Cw + cw0 + cl) * K + k;
        if (DET)
          part[(long)blockIdx.y * Co * Cw * K + e] = acc[cb][r];
        else
          atomicAdd(gw + e, acc[cb][r]);
      }
    }
}

// gb[co] += sum over n, p of gout[n][co][p]: one 1024-thread workgroup per channel, 16-byte
// loads when P % 4 == 0, fixed-order tree reduction (bit-reproducible).
__global__ __launch_bounds__(1024) void bias_grad_kernel(const float *__restrict__ gout,
                                                         float *__restrict__ gb, int N, int Co,
                                                         long P, int overwrite = 0) {
  const int co = blockIdx.x;
  float s = 0.f;
  if ((P & 3) == 0 && (reinterpret_cast<uintptr_t>(gout) & 15) == 0) {
    for (int n = 0; n < N; ++n) {
      const f32x4 *g4 = reinterpret_cast<const f32x4 *>(gout + ((long)n * Co + co) * P);
      for (long q = threadIdx.x; q < (P >> 2); q += 1024) {
        const f32x4 v = g4[q];
        s += (v[0] + v[1]) + (v[2] + v[3]);
      }
    }
  } else {
    for (int n = 0; n < N; ++n)
      for (long p = threadIdx.x; p < P; p += 1024) s += gout[((long)n * Co + co) * P + p];
  }
  __shared__ float red[1024];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) gb[co] = overwrite ? red[0] : gb[co] + red[0];
}

// grad_x NHWC workspace [N][HW][C] -> NCHW: 32 x 32 tiles through LDS (both sides coalesced).
// T = long long: the deterministic fixed-point accumulator (value * scale), converted to fp32 here.
template <typename T>
__global__ __launch_bounds__(256) void nhwc_to_nchw_kernel(const T *__restrict__ src,
                                                           float *__restrict__ dst, int C, long HW,
                                                           const double *__restrict__ det_scale) {
  __shared__ float t[32][33];
  const double inv = det_scale ? 1.0 / *det_scale : 1.0;
  const int n = blockIdx.z;
  const long s0 = (long)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const T *sn = src + (long)n * HW * C;
  float *dn = dst + (long)n * C * HW;
  for (int r = ty; r < 32; r += 8) {
    const long sp = s0 + r;
    float v = 0.f;
    if (sp < HW && c0 + tx < C) {
      if constexpr (sizeof(T) == 8)
        v = (float)((double)sn[sp * C + c0 + tx] * inv);
      else
        v = sn[sp * C + c0 + tx];
    }
    t[r][tx] = v;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r;
    if (c < C && s0 + tx < HW) dn[(long)c * HW + s0 + tx] = t[tx][r];
  }
}

int check_shapes(const MdcnArgs &a) {
  if (a.N <= 0 || a.C <= 0 || a.H <= 0 || a.W <= 0 || a.Co <= 0 || a.kh <= 0 || a.kw <= 0 ||
      a.stride <= 0 || a.pad < 0 || a.dil <= 0 || a.groups <= 0 || a.dg <= 0)
    return AANET_EINVAL;
  if (a.C % a.groups || a.Co % a.groups || a.C % a.dg) return AANET_EINVAL;
  if (a.Ho <= 0 || a.Wo <= 0) return AANET_EINVAL;
  // one image's planes are addressed by 32-bit buffer offsets (the epilogues)
  if ((long)a.C * a.H * a.W * 4 >= (1L << 31) || (long)a.Co * a.Ho * a.Wo * 4 >= (1L << 31))
    return AANET_EUNSUPPORTED;
  return AANET_OK;
}

MdcnArgs make_args(const float *x, const float *offset, long off_bs, const float *mask,
                   long mask_bs, int mask_logits, float mask_scale, const float *weight,
                   const float *bias, const float *ps, const float *psh, int act, float *out,
                   int n, int c, int h, int w, int co, int kh, int kw, int stride, int pad,
                   int dil, int groups, int dg) {
  MdcnArgs a;
  a.x = x;
  a.offset = offset;
  a.mask = mask;
  a.mask_logits = mask_logits;
  a.mask_scale = mask_scale;
  a.weight = weight;
  a.bias = bias;
  a.post_scale = ps;
  a.post_shift = psh;
  a.residual = nullptr;
  a.tail_w = nullptr;
  a.tail_b = nullptr;
  a.tail_act = 0;
  a.Co2 = co;
  a.act = act;
  a.out = out;
  a.N = n;
  a.C = c;
  a.H = h;
  a.W = w;
  a.Co = co;
  a.kh = kh;
  a.kw = kw;
  a.stride = stride;
  a.pad = pad;
  a.dil = dil;
  a.groups = groups;
  a.dg = dg;
  a.layout = 0;
  a.split = 0;
  a.halo = 0;
  a.dbg_noatom = 0;
  a.csa_out = nullptr;
  a.num_up = 0;
  a.csa_act = 0;
  a.post = nullptr;
  a.post_w = nullptr;
  a.post_b = nullptr;
  a.post_act = 0;
  a.post_out = nullptr;
  for (int j = 0; j < 3; ++j) {
    a.up[j] = nullptr;
    a.up_h[j] = a.up_w[j] = a.up_r[j] = 1;
  }
  a.Ho = conv_out_size(h, kh, stride, pad, dil);
  a.Wo = conv_out_size(w, kw, stride, pad, dil);
  const long P = (long)a.Ho * a.Wo, K = (long)kh * kw;
  a.off_bs = off_bs >= 0 ? off_bs : (long)dg * 2 * K * P;
  a.mask_bs = mask_bs >= 0 ? mask_bs : (long)dg * K * P;
  return a;
}

// DcnSmallArgs of the op-level form (no tail) from the engine's arguments
DcnSmallArgs small_args(const MdcnArgs &a, const float *weight, int packed) {
  DcnSmallArgs t{};
  t.x = a.x;
  t.offset = a.offset;
  t.off_bs = a.off_bs;
  t.mask = a.mask;
  t.mask_bs = a.mask_bs;
  t.mask_logits = a.mask_logits;
  t.mask_scale = a.mask_scale;
  t.w = weight;
  t.packed = packed;
  t.bias = a.bias;
  t.post_scale = a.post_scale;
  t.post_shift = a.post_shift;
  t.act = a.act;
  t.out = a.out;
  t.N = a.N;
  t.C = a.C;
  t.H = a.H;
  t.W = a.W;
  t.Co = a.Co;
  t.Co2 = a.Co;
  t.pad = a.pad;
  t.dil = a.dil;
  t.dg = a.dg;
  return t;
}

template <int MODE, int CO_T, int PTT, int FULL, int CFG>
void launch_fwd_f(const MdcnArgs &a, int packed, dim3 grid, hipStream_t st) {
  const dim3 blk(FNT);
  if constexpr (!FULL && MODE == 0 && CFG == 0 && CO_T >= 32) {
    // plain NCHW conv, group width 16 (mod 32): split-bf16 over zero-padded 32-channel chunks
    if (a.split && packed && !a.tail_w && a.layout == 0) {
      hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, PTT, 1, 0, 1, 0, 0, 0, 1>), grid, blk, 0, st, a);
      return;
    }
  }
  if constexpr (FULL && CFG == 0 && CO_T >= 32) {  // split-bf16 contraction (PREC 1)
    if constexpr (MODE == 0 && PTT == 128) {
      if (a.split && packed && a.halo == 4) {  // phase-strided halo tile (dilation > 2)
        if (a.layout == 3)
          hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 0, 1, 1, 3, CFG, 1, 4>), grid, blk, 0, st, a);
        return;
      }
      if (a.split && packed && a.halo == 1) {  // 3x3 stride-1 halo-tile form (NHWC input), HALO = dil
        if (a.dil == 1) {
          if (a.tail_w && a.post && CO_T == 64)
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 1, 1, 1, 1, CFG, 1, 1, 1>), grid, blk, 0, st, a);
          else if (a.tail_w)
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 1, 1, 1, 1, CFG, 1, 1>), grid, blk, 0, st, a);
          else if (a.layout == 3)
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 0, 1, 1, 3, CFG, 1, 1>), grid, blk, 0, st, a);
          else
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 0, 1, 1, 1, CFG, 1, 1>), grid, blk, 0, st, a);
        } else {
          if (a.tail_w)
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 1, 1, 1, 1, CFG, 1, 2>), grid, blk, 0, st, a);
          else if (a.layout == 3)
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 0, 1, 1, 3, CFG, 1, 2>), grid, blk, 0, st, a);
          else
            hipLaunchKernelGGL((conv_fwd_kernel<0, CO_T, 128, 1, 0, 1, 1, 1, CFG, 1, 2>), grid, blk, 0, st, a);
        }
        return;
      }
    }
    if (a.split && packed) {
      if (a.tail_w) {
        if (a.layout == 1)
          hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 1, 1, 1, 1, CFG, 1>), grid, blk, 0, st, a);
        else
          hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 1, 1, 1, 0, CFG, 1>), grid, blk, 0, st, a);
        return;
      }
      switch (a.layout) {
        case 1: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, 1, 1, CFG, 1>), grid, blk, 0, st, a); break;
        case 2: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, 1, 2, CFG, 1>), grid, blk, 0, st, a); break;
        case 3: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, 1, 3, CFG, 1>), grid, blk, 0, st, a); break;
        default: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, 1, 0, CFG, 1>), grid, blk, 0, st, a); break;
      }
      return;
    }
  }
  if (a.tail_w) {
    if (FULL && a.layout == 1)
      hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 1, 1, FULL, FULL ? 1 : 0, CFG>), grid, blk, 0, st, a);
    else
      hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 1, 1, FULL, 0, CFG>), grid, blk, 0, st, a);
  } else if (packed) {
    switch (FULL ? a.layout : 0) {
      case 1: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, FULL, FULL ? 1 : 0, CFG>), grid, blk, 0, st, a); break;
      case 2: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, FULL, 2, CFG>), grid, blk, 0, st, a); break;
      case 3: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, FULL, FULL ? 3 : 2, CFG>), grid, blk, 0, st, a); break;
      default: hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 1, 0, 1, FULL, 0, CFG>), grid, blk, 0, st, a); break;
    }
  } else {
    hipLaunchKernelGGL((conv_fwd_kernel<MODE, CO_T, PTT, 0, 0, 0, FULL, 0, CFG>), grid, blk, 0, st, a);
  }
}

// Chunk configuration (conv_fwd_kernel CFG) for which every chunk is full, or -1.
int full_cfg(const MdcnArgs &a, int mode, int co_t) {
  const int Cg = a.C / a.groups, cpg = a.C / a.dg;
  if (Cg % KC == 0 && (!mode || cpg % KC == 0)) return 0;
  if (mode && Cg % KC == 0 && cpg == 16) return 2;
  if (co_t >= 32 && Cg % 16 == 0 && (!mode || cpg % 16 == 0)) return 1;
  return -1;
}

template <int MODE, int CO_T, int PTT>
void launch_fwd_t(const MdcnArgs &a, int packed, dim3 grid, hipStream_t st) {
  const int cfg = full_cfg(a, MODE, CO_T);
  if (MODE == 0 && CO_T >= 32 && a.split && packed && !a.tail_w && a.layout == 0 && (a.C / a.groups) % 32) {
    launch_fwd_f<MODE, CO_T, PTT, 0, 0>(a, packed, grid, st);  // zero-padded split chunks
    return;
  }
  constexpr bool C1 = CO_T >= 32 && PTT == 128;  // 16-channel chunks: 4 staged values per thread
  if (cfg == 0)
    launch_fwd_f<MODE, CO_T, PTT, 1, 0>(a, packed, grid, st);
  else if (cfg == 1 && C1)
    launch_fwd_f<MODE, CO_T, PTT, 1, C1 ? 1 : 0>(a, packed, grid, st);
  else if (cfg == 2 && MODE)
    launch_fwd_f<MODE, CO_T, PTT, 1, MODE ? 2 : 0>(a, packed, grid, st);
  else
    launch_fwd_f<MODE, CO_T, PTT, 0, 0>(a, packed, grid, st);
}

template <int MODE>
int launch_fwd(const MdcnArgs &a_in, int packed, hipStream_t st) {
  MdcnArgs a = a_in;
  const int rc = check_shapes(a);
  if (rc) return rc;
  if (!a.x || !a.weight || !a.out) return AANET_EINVAL;
  if (MODE && (!a.offset || !a.mask)) return AANET_EINVAL;
  if (MODE && a.W < 2) return AANET_EUNSUPPORTED;  // pair-gather sampler needs 2 columns
  if (a.post_scale && !a.post_shift) return AANET_EINVAL;
  const long P = (long)a.Ho * a.Wo;
  const int Cog = a.Co / a.groups;
  if (a.layout < 0 || a.layout > 3) return AANET_EINVAL;
  if (a.csa_out) {  // CSA epilogue: tail kernels, quad-aligned rows, exact 2x / 4x terms
    if (!a.tail_w || a.Wo % 4 || a.num_up < 0 || a.num_up > 2) return AANET_EUNSUPPORTED;
    for (int j = 0; j < a.num_up; ++j) {
      const int r = a.up_r[j];
      if (!a.up[j] || (r != 2 && r != 4) || a.up_h[j] * r != a.Ho || a.up_w[j] * r != a.Wo)
        return AANET_EUNSUPPORTED;
    }
  }
  int co_t = Cog <= 16 ? 16 : (Cog <= 32 ? 32 : 64);
  if (a.tail_w) {  // the whole conv output column of a pixel must sit in one workgroup
    if (a.groups != 1 || a.Co > 64 || a.Co2 <= 0 || a.Co2 > 64 || !packed) return AANET_EUNSUPPORTED;
    co_t = max(a.Co, a.Co2) <= 16 ? 16 : (max(a.Co, a.Co2) <= 32 ? 32 : 64);
  }
  if (a.layout) {  // NHWC paths: packed weights, full chunks (full_cfg), 4-channel quads
    if (!packed || a.C % 4 || full_cfg(a, MODE, co_t) < 0) return AANET_EUNSUPPORTED;
    if ((a.layout & 2) && (a.tail_w || Cog % 4)) return AANET_EUNSUPPORTED;
  }
  const int ncot = host_div_up(Cog, co_t);
  // 128-pixel tiles when they still give >= 2 workgroups per CU (the scale-1 convs of the C2
  // pyramid, 832 tiles: stride-2 64->64 exchange conv 93 -> 86 us), else 64
  int ptt = co_t == 16 || (long)a.N * host_div_up(P, 128) * a.groups * ncot >= 512 ? 128 : 64;
  if (full_cfg(a, MODE, co_t) == 1) ptt = 128;  // 16-channel chunks are staged 4 per thread
  a.halo = MODE == 0 && a.split && packed && (a.layout & 1) && a.kh == 3 && a.kw == 3 &&
           a.stride == 1 && a.pad == a.dil && a.dil <= 2 && co_t >= 32 && full_cfg(a, 0, co_t) == 0;
  // dilations > 2 (the refinement's dilated blocks): the phase-strided halo tile (HALO 4),
  // NHWC in and out, no tail
  if (!a.halo && MODE == 0 && a.split && packed && a.layout == 3 && a.kh == 3 && a.kw == 3 &&
      a.stride == 1 && a.pad == a.dil && a.dil > 2 && co_t >= 32 && !a.tail_w && !a.csa_out &&
      !a.post && full_cfg(a, 0, co_t) == 0)
    a.halo = 4;
  if (a.halo) ptt = 128;
  // post stage (aanet_post_stage_t): the HALO 1 tail with the CSA epilogue, 64 -> 64 channels,
  // NHWC output only; anything else is left to the caller before any launch
  if (a.post && (MODE != 0 || !a.csa_out || !a.halo || a.dil != 1 || co_t != 64 || a.Co2 != 64 ||
                 a.post->disp || !a.post->out_nhwc || a.post->skip_outputs || !a.split || !packed))
    return AANET_EUNSUPPORTED;
  const int hd = a.halo == 4 ? a.dil : 1;  // phase stride (HALO 4)
  dim3 grid((unsigned)(a.halo ? (long)a.N * hd * hd * host_div_up(host_div_up(a.Wo, hd), 16) *
                                    host_div_up(host_div_up(a.Ho, hd), 8)
                              : a.N * host_div_up(P, ptt)),
            (unsigned)(a.groups * ncot));
  if (ptt == 128) {
    switch (co_t) {
      case 16: launch_fwd_t<MODE, 16, 128>(a, packed, grid, st); break;
      case 32: launch_fwd_t<MODE, 32, 128>(a, packed, grid, st); break;
      default: launch_fwd_t<MODE, 64, 128>(a, packed, grid, st); break;
    }
  } else {
    switch (co_t) {
      case 16: break;  // unreachable: 16-channel tiles always take 128-pixel tiles
      case 32: launch_fwd_t<MODE, 32, 64>(a, packed, grid, st); break;
      default: launch_fwd_t<MODE, 64, 64>(a, packed, grid, st); break;
    }
  }
  return aanet_launch_status();
}

// ---- deterministic-backward helpers ---------------------------------------------------------
// bounds[0] = max_{c,k} sum_co |W[co][c][k]|, bounds[1] = max|gOut|, bounds[2] = max|mask|, as
// float bits (non-negative floats order like their bit patterns).  Every grad_x contribution is
// colg * w_corner * m with |colg| <= bounds[0]*bounds[1] and |w_corner| <= 1.
__global__ __launch_bounds__(256) void det_wbound_kernel(const float *__restrict__ w, int Co, int CK,
                                                         unsigned *__restrict__ bounds) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < CK; e += gridDim.x * 256) {
    float s = 0.f;
    for (int co = 0; co < Co; ++co) s += fabsf(w[(long)co * CK + e]);
    atomicMax(bounds, __float_as_uint(s) & 0x7fffffffu);  // NaN bits order above +inf
  }
}

// max |v| into *slot (as the uint bits of a non-negative float): 16-byte loads when v is
// 16-byte aligned, one atomic per workgroup (a few hundred workgroups: per-wave atomics on one
// address serialise at the L2 and dominated this kernel).  The max is taken over the bit
// patterns of |v|, which order like the values and put NaN (0x7fc...) above +inf: a NaN or an
// inf anywhere reaches the bound (fmaxf would drop a NaN), and det_scale_kernel then poisons.
__device__ __forceinline__ unsigned abs_bits(float x) { return __float_as_uint(x) & 0x7fffffffu; }
__global__ __launch_bounds__(256) void det_absmax_kernel(const float *__restrict__ v, long n,
                                                         unsigned *__restrict__ slot) {
  __shared__ unsigned red[4];
  unsigned m = 0u;
  const long stride = (long)gridDim.x * 256, t0 = (long)blockIdx.x * 256 + threadIdx.x;
  long tail = 0;
  if ((reinterpret_cast<uintptr_t>(v) & 15) == 0) {
    const long n4 = n >> 2;
    for (long q = t0; q < n4; q += stride) {
      const f32x4 x = reinterpret_cast<const f32x4 *>(v)[q];
      m = max(m, max(max(abs_bits(x[0]), abs_bits(x[1])), max(abs_bits(x[2]), abs_bits(x[3]))));
    }
    tail = n4 << 2;
  }
  for (long e = tail + t0; e < n; e += stride) m = max(m, abs_bits(v[e]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(slot, max(max(red[0], red[1]), max(red[2], red[3])));
}

// scale[0] = 2^(38 - ceil(log2 bound)): a single contribution stays below 2^38, so up to 2^25 of
// them can meet in one element before the int64 sum could overflow; the fixed-point step
// (2^-38 of the largest possible contribution) is far below fp32 rounding of typical sums.
// A non-finite bound (an inf or NaN in the weights, grad_out or mask) gives scale = NaN: the
// fixed-point sums are then read back through 1/scale = NaN, so grad_x comes out NaN instead
// of finite garbage from __double2ll_rn(inf/NaN) (the reference's float col2im would propagate
// the non-finite value).
// scale[1]: the deterministic window form's weight-gradient accumulator.  Every element is a sum
// over the npix output pixels of gOut * column, |column| <= max|x| * max|mask| (bilinear weights
// sum to <= 1), so the whole sum is bounded by bw = npix * bounds[1] * bounds[3] * bounds[2] and
// 2^(62 - ceil(log2 bw)) keeps it (plus half a step per tile of rounding) inside int64.
__global__ void det_scale_kernel(const unsigned *__restrict__ bounds, double *__restrict__ scale, long npix) {
  const double b = (double)__uint_as_float(bounds[0]) * (double)__uint_as_float(bounds[1]) *
                   (double)__uint_as_float(bounds[2]);
  scale[0] = !isfinite(b) ? __builtin_nan("") : (b > 0.0 ? ldexp(1.0, 38 - (int)ceil(log2(b))) : 1.0);
  const double bw = (double)npix * (double)__uint_as_float(bounds[1]) * (double)__uint_as_float(bounds[2]) *
                    (double)__uint_as_float(bounds[3]);
  scale[1] = !isfinite(bw) ? __builtin_nan("") : (bw > 0.0 ? ldexp(1.0, 62 - (int)ceil(log2(bw))) : 1.0);
}

// gw[e] += sum over the splits of part[split][e], in a fixed order: workgroup = 64 consecutive
// elements x 4 split lanes (lane l sums splits l, l+4, ... in order, 4 loads in flight), then the
// 4 lane sums are added in lane order -- bit-reproducible for a given nsplit.
__global__ __launch_bounds__(256) void det_weight_reduce_kernel(const float *__restrict__ part,
                                                                float *__restrict__ gw, long n,
                                                                int nsplit, int overwrite = 0) {
  __shared__ float red[4][64];
  const int ex = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + ex;
  float s = 0.f;
  if (e < n) {
    int y = sl;
    for (; y + 12 < nsplit; y += 16) {
      const float v0 = part[(long)y * n + e], v1 = part[(long)(y + 4) * n + e];
      const float v2 = part[(long)(y + 8) * n + e], v3 = part[(long)(y + 12) * n + e];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; y < nsplit; y += 4) s += part[(long)y * n + e];
  }
  red[sl][ex] = s;
  __syncthreads();
  if (sl == 0 && e < n) {
    const float v = ((red[0][ex] + red[1][ex]) + red[2][ex]) + red[3][ex];
    gw[e] = overwrite ? v : gw[e] + v;
  }
}

__global__ void pack_weight_kernel(const float *__restrict__ w, float *__restrict__ wp, int Co,
                                   int Cg, int K) {
  const long total = (long)Co * Cg * K;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int k = (int)(e % K);
    const long t = e / K;
    const int c = (int)(t % Cg), co = (int)(t / Cg);
    wp[((long)k * Co + co) * Cg + c] = w[e];
  }
}

// PREC 1 needs weight buffers from aanet_conv_weight_pack_split_f32 (AANET_CONV_WEIGHTS_SPLIT)
// and the split arithmetic selected (AANET_CONV_EXACT_F32 clear); a tail kernel's pointwise
// weights then carry their fragments too.
void set_split(MdcnArgs &a, int flags, int packed) {
  a.split = packed && (flags & AANET_CONV_WEIGHTS_SPLIT) && !(flags & AANET_CONV_EXACT_F32);
  if (!a.split) return;
  const int cg = a.C / a.groups, kk = a.kh * a.kw;
  a.wsplit = reinterpret_cast<const bf16x8_t *>(reinterpret_cast<const char *>(a.weight) +
                                                split_frag_offset(a.Co, cg, kk));
  if (a.tail_w)
    a.tail_wsplit = reinterpret_cast<const bf16x8_t *>(reinterpret_cast<const char *>(a.tail_w) +
                                                       split_frag_offset(a.Co2, a.Co, 1));
}

// one thread per (g, t, k, cc, blk, lane): 8 weights -> their three bf16 pieces
__global__ void pack_split_kernel(const float *__restrict__ w, bf16x8_t *__restrict__ frag, int Co,
                                  int Cg, int K, int groups) {
  const int Cog = Co / groups, T = (Cog + 63) / 64, NCC = (Cg + 31) / 32;  // zero-padded chunks
  const long total = (long)groups * T * K * NCC * 4 * 64;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int lane = (int)(e & 63);
    long r = e >> 6;
    const int blk = (int)(r & 3);
    r >>= 2;
    const int cc = (int)(r % NCC);
    r /= NCC;
    const int k = (int)(r % K);
    r /= K;
    const int t = (int)(r % T), g = (int)(r / T);
    const int row = 64 * t + 16 * blk + (lane & 15);
    const int co = g * Cog + row;
    bf16x8_t ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 32 * cc + 8 * (lane >> 4) + j;
      const float v = row < Cog && c < Cg ? w[((long)co * Cg + c) * K + k] : 0.f;
      const __bf16 h = (__bf16)v;
      const float r1 = v - (float)h;
      const __bf16 m = (__bf16)r1;
      ph[j] = h;
      pm[j] = m;
      pl[j] = (__bf16)(r1 - (float)m);
    }
    const long o = (((((long)g * T + t) * K + k) * NCC + cc) * 4 + blk) * 3 * 64 + lane;
    frag[o] = ph;
    frag[o + 64] = pm;
    frag[o + 128] = pl;
  }
}

int set_csa(MdcnArgs &a, const aanet_csa_epilogue_t *csa) {
  if (!csa) return AANET_OK;
  if (csa->struct_size != sizeof(aanet_csa_epilogue_t)) return AANET_EABI;
  a.post = csa->post;
  if (a.post && a.post->struct_size != sizeof(aanet_post_stage_t)) return AANET_EABI;
  if (a.post && ((!a.post->out_nhwc && !a.post->disp) || !a.post->weight || a.post->act < 0 ||
                 a.post->act > 2))
    return AANET_EINVAL;
  if (a.post) {  // copied by value: the kernel never dereferences the host descriptor
    a.post_w = reinterpret_cast<const char *>(a.post->weight) + split_frag_offset(64, 64, 1);
    a.post_b = a.post->bias;
    a.post_act = a.post->act;
    a.post_out = a.post->out_nhwc;
  }
  if (!csa->out || csa->num_up < 0 || csa->num_up > 3 || csa->act < 0 || csa->act > 2)
    return AANET_EINVAL;
  a.csa_out = csa->out;
  a.num_up = csa->num_up;
  a.csa_act = csa->act;
  for (int j = 0; j < csa->num_up; ++j) {
    if (!csa->up[j] || csa->up_h[j] <= 0 || csa->up_w[j] <= 0) return AANET_EINVAL;
    a.up[j] = csa->up[j];
    a.up_h[j] = csa->up_h[j];
    a.up_w[j] = csa->up_w[j];
    a.up_r[j] = csa->up_h[j] > 0 ? a.Ho / csa->up_h[j] : 0;
  }
  return AANET_OK;
}

int round_pitch(int v, int mod32) {  // smallest p >= v with p % 32 == mod32
  int p = v;
  while (p % 32 != mod32) ++p;
  return p;
}

}  // namespace

extern "C" int aanet_mdcn_fwd_f32(const float *x, const float *offset, const float *mask,
                                  const float *weight, const float *bias, float *out, int n, int c,
                                  int h, int w, int co, int kh, int kw, int stride, int pad,
                                  int dil, int groups, int dg, aanet_stream_t stream) {
  MdcnArgs a = make_args(x, offset, -1, mask, -1, 0, 1.f, weight, bias, nullptr, nullptr, 0, out,
                         n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg);
  // 16 channels in two 8-channel groups (the aggregation's coarsest scale): direct fp32 form
  if (!check_shapes(a) && groups == 1 && a.Ho == h && a.Wo == w &&
      dcn_small_supported(c, co, 0, kh, kw, stride, pad, dil, dg, groups)) {
    const int rc = dcn_small_launch(small_args(a, weight, 0), as_hip(stream));
    if (rc != AANET_EUNSUPPORTED) return rc;
  }
  return launch_fwd<1>(a, 0, as_hip(stream));
}

extern "C" int aanet_conv2d_fused_f32(const float *x, const float *weight, const float *bias,
                                      const float *post_scale, const float *post_shift,
                                      const float *residual, int act, int weight_packed,
                                      float *out, int n, int c, int h, int w, int co, int kh,
                                      int kw, int stride, int pad, int dil, int groups, int layout,
                                      aanet_stream_t stream) {
  if (act < 0 || act > 2) return AANET_EINVAL;
  // the argument checks of launch_fwd, before any of the specialised kernels below is chosen
  if (!x || !weight || !out || (post_scale && !post_shift)) return AANET_EINVAL;
  MdcnArgs a = make_args(x, nullptr, 0, nullptr, 0, 0, 1.f, weight, bias, post_scale, post_shift,
                         act, out, n, c, h, w, co, kh, kw, stride, pad, dil, groups, 1);
  a.residual = residual;
  set_split(a, layout, weight_packed);
  a.layout = layout & ~(AANET_CONV_EXACT_F32 | AANET_CONV_WEIGHTS_SPLIT);
  // few-channel convs (Cin <= 6 or Co == 1): the direct VALU kernel (small_conv.hip)
  if ((a.layout == 0 || a.layout == 1) && groups == 1 && kh == kw && !check_shapes(a)) {
    DirectArgs d;
    d.x = x;
    d.w = weight;
    d.bias = bias;
    d.post_scale = post_scale;
    d.post_shift = post_shift;
    d.residual = residual;
    d.out = out;
    d.act = act;
    d.packed = weight_packed != 0;
    d.in_nhwc = a.layout & 1;
    d.N = n;
    d.C = c;
    d.H = h;
    d.W = w;
    d.Co = co;
    d.Ho = a.Ho;
    d.Wo = a.Wo;
    d.pad = pad;
    const int rc = conv_direct_launch(d, kh, stride, dil, as_hip(stream));
    if (rc != AANET_EUNSUPPORTED) return rc;
  }
  if (a.split && a.layout >= 0 && a.layout <= 3 && !check_shapes(a) &&
      pw_conv_supported(c, co, kh, kw, stride, pad, groups, (long)n * h * w, a.layout >> 1, h * w)) {
    PwArgs p;  // 1x1: the streaming kernel (pointwise.hip)
    p.x = x;
    p.wsplit = a.wsplit;
    p.bias = bias;
    p.post_scale = post_scale;
    p.post_shift = post_shift;
    p.residual = residual;
    p.act = act;
    p.out = out;
    p.N = n;
    p.C = c;
    p.P = h * w;
    p.Co = co;
    p.in_nhwc = a.layout & 1;
    p.out_nhwc = a.layout >> 1;
    const int rc = pw_conv_launch(p, as_hip(stream));
    if (rc != AANET_EUNSUPPORTED) return rc;
  }
  return launch_fwd<0>(a, weight_packed, as_hip(stream));
}

extern "C" int aanet_conv2d_pw_f32(const float *x, const float *weight_packed, const float *bias,
                                   const float *post_scale, const float *post_shift, int act,
                                   const float *pw_weight_packed, const float *pw_bias,
                                   const float *residual, int pw_act, int co2, float *out, int n,
                                   int c, int h, int w, int co, int kh, int kw, int stride,
                                   int pad, int dil, const aanet_csa_epilogue_t *csa, int layout,
                                   aanet_stream_t stream) {
  if (act < 0 || act > 2 || pw_act < 0 || pw_act > 2 || !pw_weight_packed) return AANET_EINVAL;
  const int flags = layout;
  layout &= ~(AANET_CONV_EXACT_F32 | AANET_CONV_WEIGHTS_SPLIT);
  if (layout != 0 && layout != 1) return AANET_EINVAL;
  MdcnArgs a = make_args(x, nullptr, 0, nullptr, 0, 0, 1.f, weight_packed, bias, post_scale,
                         post_shift, act, out, n, c, h, w, co, kh, kw, stride, pad, dil, 1, 1);
  a.layout = layout;
  const int rc = set_csa(a, csa);
  if (rc) return rc;
  a.tail_w = pw_weight_packed;
  a.tail_b = pw_bias;
  a.tail_act = pw_act;
  a.Co2 = co2;
  a.residual = residual;
  set_split(a, flags, 1);
  return launch_fwd<0>(a, 1, as_hip(stream));
}

extern "C" int aanet_mdcn_pw_f32(const float *x, const float *offset, long offset_batch_stride,
                                 const float *mask, long mask_batch_stride, int mask_logits,
                                 float mask_scale, const float *weight_packed, const float *bias,
                                 const float *post_scale, const float *post_shift, int act,
                                 const float *pw_weight_packed, const float *pw_bias,
                                 const float *residual, int pw_act, int co2, float *out, int n,
                                 int c, int h, int w, int co, int kh, int kw, int stride, int pad,
                                 int dil, int dg, const aanet_csa_epilogue_t *csa, int layout,
                                 aanet_stream_t stream) {
  if (act < 0 || act > 2 || pw_act < 0 || pw_act > 2 || !pw_weight_packed) return AANET_EINVAL;
  const int flags = layout;
  const bool generic = (layout & AANET_CONV_GENERIC_DCN) != 0;
  layout &= ~(AANET_CONV_EXACT_F32 | AANET_CONV_WEIGHTS_SPLIT | AANET_CONV_GENERIC_DCN);
  if (layout != 0 && layout != 1) return AANET_EINVAL;
  MdcnArgs a = make_args(x, offset, offset_batch_stride, mask, mask_batch_stride, mask_logits,
                         mask_scale, weight_packed, bias, post_scale, post_shift, act, out, n, c,
                         h, w, co, kh, kw, stride, pad, dil, 1, dg);
  a.layout = layout;
  const int rc = set_csa(a, csa);
  if (rc) return rc;
  a.tail_w = pw_weight_packed;
  a.tail_b = pw_bias;
  a.tail_act = pw_act;
  a.Co2 = co2;
  a.residual = residual;
  set_split(a, flags, 1);
  // the deformable bottleneck tail of the aggregation: LDS-window form (dcn_tile.hip)
  if (!generic && a.split && layout == 1 && a.Ho == h && a.Wo == w &&
      dcn_tile_supported(c, co, co2, kh, kw, stride, pad, dil, dg, 1, w)) {
    DcnTileArgs t{};
    t.x = x;
    t.offset = a.offset;
    t.off_bs = a.off_bs;
    t.mask = a.mask;
    t.mask_bs = a.mask_bs;
    t.mask_logits = mask_logits;
    t.mask_scale = mask_scale;
    t.wsplit = a.wsplit;
    t.bias = bias;
    t.post_scale = post_scale;
    t.post_shift = post_shift;
    t.act = act;
    t.tail_wsplit = a.tail_wsplit;
    t.tail_b = pw_bias;
    t.tail_act = pw_act;
    t.residual = residual;
    t.out = out;
    t.csa_out = a.csa_out;
    t.num_up = a.csa_out ? a.num_up : 0;
    t.csa_act = a.csa_act;
    for (int j = 0; j < 2; ++j) {
      t.up[j] = a.up[j];
      t.up_h[j] = a.up_h[j];
      t.up_w[j] = a.up_w[j];
      t.up_r[j] = a.up_r[j];
    }
    t.N = n;
    t.C = c;
    t.H = h;
    t.W = w;
    t.Co = co;
    t.Co2 = co2;
    t.dil = dil;
    t.dg = dg;
    t.dbg = 0;
    t.post_wsplit = nullptr;
    t.post_b = nullptr;
    t.post_act = 0;
    t.post_out = t.post_disp = nullptr;
    t.post_skip = 0;
    if (a.post) {
      if (co2 != 64) return AANET_EUNSUPPORTED;
      t.post_wsplit = reinterpret_cast<const char *>(a.post->weight) + split_frag_offset(64, 64, 1);
      t.post_b = a.post->bias;
      t.post_act = a.post->act;
      t.post_out = a.post->out_nhwc;
      t.post_disp = a.post->disp;
      t.post_skip = a.post->skip_outputs != 0;
    }
    const int rc2 = (a.csa_out && a.num_up > 2) ? AANET_EUNSUPPORTED : dcn_tile_launch(t, as_hip(stream));
    if (rc2 != AANET_EUNSUPPORTED) return rc2;
  }
  if (a.post) return AANET_EUNSUPPORTED;  // the generic engine has no post stage
  // the coarsest scale's 16-channel block (two 8-channel groups): direct fp32 form (dcn_small.hip)
  if (!generic && layout == 0 && !a.csa_out && a.Ho == h && a.Wo == w &&
      dcn_small_supported(c, co, co2, kh, kw, stride, pad, dil, dg, 1)) {
    DcnSmallArgs t = small_args(a, weight_packed, 1);
    t.tail_w = pw_weight_packed;
    t.tail_b = pw_bias;
    t.tail_act = pw_act;
    t.residual = residual;
    t.Co2 = co2;
    const int rc2 = dcn_small_launch(t, as_hip(stream));
    if (rc2 != AANET_EUNSUPPORTED) return rc2;
  }
  return launch_fwd<1>(a, 1, as_hip(stream));
}

extern "C" int aanet_mdcn_fwd_fused_f32(const float *x, const float *offset,
                                        long offset_batch_stride, const float *mask,
                                        long mask_batch_stride, int mask_logits, float mask_scale,
                                        const float *weight, int weight_packed, const float *bias,
                                        const float *post_scale, const float *post_shift, int act,
                                        float *out, int n, int c, int h, int w, int co, int kh,
                                        int kw, int stride, int pad, int dil, int groups, int dg,
                                        int layout, aanet_stream_t stream) {
  if (act < 0 || act > 2) return AANET_EINVAL;
  MdcnArgs a = make_args(x, offset, offset_batch_stride, mask, mask_batch_stride, mask_logits,
                         mask_scale, weight, bias, post_scale, post_shift, act, out, n, c, h, w,
                         co, kh, kw, stride, pad, dil, groups, dg);
  set_split(a, layout, weight_packed);
  const bool generic = (layout & AANET_CONV_GENERIC_DCN) != 0;
  a.layout = layout & ~(AANET_CONV_EXACT_F32 | AANET_CONV_WEIGHTS_SPLIT | AANET_CONV_GENERIC_DCN);
  // the aggregation's deformable convs (3x3, dil 2, two groups of 16 / 32 channels): LDS-window
  // form with the plain epilogue (dcn_tile.hip), NCHW or channels-last x, NCHW out
  if (!generic && a.split && (a.layout == 0 || a.layout == 1) && groups == 1 && a.Ho == h &&
      a.Wo == w && dcn_tile_supported(c, co, co, kh, kw, stride, pad, dil, dg, 1, w)) {
    DcnTileArgs t{};
    t.x = x;
    t.offset = a.offset;
    t.off_bs = a.off_bs;
    t.mask = a.mask;
    t.mask_bs = a.mask_bs;
    t.mask_logits = mask_logits;
    t.mask_scale = mask_scale;
    t.wsplit = a.wsplit;
    t.bias = bias;
    t.post_scale = post_scale;
    t.post_shift = post_shift;
    t.act = act;
    t.out = out;
    t.N = n;
    t.C = c;
    t.H = h;
    t.W = w;
    t.Co = co;
    t.Co2 = co;
    t.dil = dil;
    t.dg = dg;
    t.x_nchw = a.layout == 0;
    t.plain = 1;
    const int rc = dcn_tile_launch(t, as_hip(stream));
    if (rc != AANET_EUNSUPPORTED) return rc;
  }
  if (!generic && a.layout == 0 && groups == 1 && a.Ho == h && a.Wo == w &&
      dcn_small_supported(c, co, 0, kh, kw, stride, pad, dil, dg, groups)) {
    const int rc = dcn_small_launch(small_args(a, weight, weight_packed), as_hip(stream));
    if (rc != AANET_EUNSUPPORTED) return rc;
  }
  return launch_fwd<1>(a, weight_packed, as_hip(stream));
}

extern "C" int aanet_mdcn_window_fwd_supported(int c, int co, int kh, int kw, int stride, int pad,
                                               int dil, int groups, int dg, int w) {
  return groups == 1 && dcn_tile_supported(c, co, co, kh, kw, stride, pad, dil, dg, 1, w);
}

// The data gradient's weight straight into the engine layout: wt[g*cg + i][j][k] =
// w[g*(co/groups) + j][i][K-1-k] (per-group transpose, spatial flip), stored [k][co'][cg'] with
// co' = groups*cg, cg' = co/groups -- what pack_weight_kernel makes of the transposed, flipped
// copy, in one pass over w.
__global__ void pack_weight_dgrad_kernel(const float *__restrict__ w, float *__restrict__ wp, int Co,
                                         int Cg, int K, int groups) {
  const int Cot = groups * Cg, Cgt = Co / groups;
  const long total = (long)Cot * Cgt * K;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long)gridDim.x * blockDim.x) {
    const int c = (int)(e % Cgt);  // wt's input channel j (output order: [k][co'][cg'])
    const long t = e / Cgt;
    const int cot = (int)(t % Cot), k = (int)(t / Cot);
    const int g = cot / Cg, i = cot - g * Cg;
    wp[e] = w[((long)(g * Cgt + c) * Cg + i) * K + (K - 1 - k)];
  }
}

extern "C" int aanet_conv_weight_pack_dgrad_f32(const float *weight, float *weight_packed, int co,
                                                int cg, int kh, int kw, int groups,
                                                aanet_stream_t stream) {
  AANET_HOST_CHECK(weight && weight_packed && co > 0 && cg > 0 && kh > 0 && kw > 0 && groups > 0 &&
                   co % groups == 0);
  const long total = (long)co * cg * kh * kw;
  hipLaunchKernelGGL(pack_weight_dgrad_kernel,
                     dim3(host_div_up(total, 256) > 4096 ? 4096 : host_div_up(total, 256)), dim3(256),
                     0, as_hip(stream), weight, weight_packed, co, cg, kh * kw, groups);
  return aanet_launch_status();
}

extern "C" int aanet_conv_weight_pack_f32(const float *weight, float *weight_packed, int co,
                                          int cg, int kh, int kw, aanet_stream_t stream) {
  AANET_HOST_CHECK(weight && weight_packed && co > 0 && cg > 0 && kh > 0 && kw > 0);
  const long total = (long)co * cg * kh * kw;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(host_div_up(total, 256) > 4096 ? 4096 : host_div_up(total, 256)),
                     dim3(256), 0, as_hip(stream), weight, weight_packed, co, cg, kh * kw);
  return aanet_launch_status();
}

extern "C" long aanet_conv_weight_pack_split_bytes(int co, int cg, int kh, int kw, int groups) {
  // cg a multiple of 32, or of 16 past 32 (48, 80, ...: the last chunk zero-padded; plain NCHW
  // convs only take the split form then)
  if (co <= 0 || cg <= 0 || kh <= 0 || kw <= 0 || groups <= 0 || co % groups) return 0;
  if (cg % 32 && (cg % 16 || cg < 48)) return 0;
  return split_frag_offset(co, cg, kh * kw) + split_frag_count(co, cg, kh * kw, groups) * 16;
}

extern "C" int aanet_conv_weight_pack_split_f32(const float *weight, void *out, int co, int cg,
                                                int kh, int kw, int groups,
                                                aanet_stream_t stream) {
  AANET_HOST_CHECK(weight && out);
  if (aanet_conv_weight_pack_split_bytes(co, cg, kh, kw, groups) == 0) return AANET_EUNSUPPORTED;
  const int rc = aanet_conv_weight_pack_f32(weight, static_cast<float *>(out), co, cg, kh, kw, stream);
  if (rc) return rc;
  const int kk = kh * kw;
  const long n = split_frag_count(co, cg, kk, groups) / 3;
  hipLaunchKernelGGL(pack_split_kernel, dim3(host_div_up(n, 256) > 4096 ? 4096 : host_div_up(n, 256)),
                     dim3(256), 0, as_hip(stream), weight,
                     reinterpret_cast<bf16x8_t *>(static_cast<char *>(out) + split_frag_offset(co, cg, kk)),
                     co, cg, kk, groups);
  return aanet_launch_status();
}

extern "C" int aanet_mdcn_im2col_f32(const float *x, const float *offset, const float *mask,
                                     float *col, int c, int h, int w, int kh, int kw, int stride,
                                     int pad, int dil, int dg, aanet_stream_t stream) {
  MdcnArgs a = make_args(x, offset, -1, mask, -1, 0, 1.f, nullptr, nullptr, nullptr, nullptr, 0,
                         nullptr, 1, c, h, w, 1, kh, kw, stride, pad, dil, 1, dg);
  const int rc = check_shapes(a);
  if (rc) return rc;
  if (!x || !offset || !mask || !col) return AANET_EINVAL;
  if (w < 2) return AANET_EUNSUPPORTED;
  const long total = (long)c * kh * kw * a.Ho * a.Wo;
  hipLaunchKernelGGL(mdcn_im2col_kernel, dim3(host_div_up(total, 256) > 8192 ? 8192 : host_div_up(total, 256)),
                     dim3(256), 0, as_hip(stream), a, col);
  return aanet_launch_status();
}

extern "C" int aanet_mdcn_sample_index(const float *offset, int *h_low, int *w_low, int *valid,
                                       int n, int h, int w, int kh, int kw, int stride, int pad,
                                       int dil, int dg, aanet_stream_t stream) {
  MdcnArgs a = make_args(nullptr, offset, -1, nullptr, -1, 0, 1.f, nullptr, nullptr, nullptr,
                         nullptr, 0, nullptr, n, dg, h, w, 1, kh, kw, stride, pad, dil, 1, dg);
  const int rc = check_shapes(a);
  if (rc) return rc;
  if (!offset || !h_low || !w_low || !valid) return AANET_EINVAL;
  const long total = (long)n * dg * kh * kw * a.Ho * a.Wo;
  hipLaunchKernelGGL(mdcn_sample_index_kernel,
                     dim3(host_div_up(total, 256) > 8192 ? 8192 : host_div_up(total, 256)), dim3(256),
                     0, as_hip(stream), a, h_low, w_low, valid);
  return aanet_launch_status();
}

namespace {

struct BwdPlan {
  int npieces, nchunks, nsplit;
  long range;
};

BwdPlan bwd_plan(const MdcnArgs &a, long target = 2048) {
  BwdPlan pl;
  const long P = (long)a.Ho * a.Wo, T = (long)a.N * P;
  const int K = a.kh * a.kw, cpg = a.C / a.dg;
  pl.npieces = host_div_up(cpg, KC);
  pl.nchunks = K * a.dg * pl.npieces;
  // ~target workgroups in total; each covers `range` flattened pixels
  long nsplit = target / pl.nchunks;
  if (nsplit < 1) nsplit = 1;
  long range = (T + nsplit - 1) / nsplit;
  range = ((range + PT - 1) / PT) * PT;
  pl.nsplit = (int)((T + range - 1) / range);
  pl.range = range;
  return pl;
}

// Deterministic-backward workspace, per chunk of images (det_chunk): [grad_x as int64]
// [weight-gradient partials (global form) | int64 [K][Co][C] accumulator (window form)]
// [bounds, scales][x channels-last][W^T]
struct DetLayout {
  size_t gxi, part, bounds, scale, xh, wt, gw, total;
};

bool bwd_nhwc_reads(const MdcnArgs &a);
// the window form's LDS (mdcn_bwd_impl), fused weight gradient, and whether a shape takes it
// the window of an 8 x 8 output tile: 7 * stride + 1 input rows / columns under the taps' reach,
// plus the R = 2 margin on both sides (offsets in [-2, 2) stay inside)
int win_rows(int kh, int dil, int stride) { return 7 * stride + 1 + (kh - 1) * dil + 4; }
size_t win_smem(const MdcnArgs &a) {
  const int GPW = round_pitch(PT, 2), WTP = round_pitch(a.Co, 2);
  const int WR = win_rows(a.kh, a.dil, a.stride), WCw = win_rows(a.kw, a.dil, a.stride);
  return sizeof(float) * ((size_t)a.Co * GPW + (size_t)WHC * WTP + (size_t)WHC * WCP + (size_t)PT * 16 +
                          (size_t)3 * WKMAX * PT + (size_t)WHC * WCP) +
         (size_t)WR * WCw * WHC * 8;
}
// round 6: stride 2, up to 128 channels per deformable group (the 16-channel slices' offset /
// mask partials accumulate in sP in slice order) and up to 128 output channels (the fused weight
// gradient loops over 64-channel blocks): the feature extractor's DCNs (nets/resnet.py:133-134)
bool win_shape_ok(const MdcnArgs &a) {
  return bwd_nhwc_reads(a) && (a.stride == 1 || a.stride == 2) && a.C / a.dg <= 8 * WHC &&
         a.kh * a.kw <= WKMAX && a.Co <= WCOMAX && a.Co % 16 == 0 && win_smem(a) <= 160 * 1024;
}

// The deterministic backward runs over the batch in chunks of images whose int64 grad_x
// accumulator + channels-last x (12 bytes per input element) fit DET_CHUNK_BYTES: the workspace
// no longer grows with the batch (agg_s0 at B = 8: 377 MB unchunked).  Chunks are a fixed
// function of the shape, so the result stays bit-reproducible.
constexpr size_t DET_CHUNK_BYTES = (size_t)96 << 20;
int det_chunk(const MdcnArgs &a) {
  const size_t per = (size_t)12 * a.C * a.H * a.W;
  size_t nc = per ? DET_CHUNK_BYTES / per : (size_t)a.N;
  if (nc < 1) nc = 1;
  return nc < (size_t)a.N ? (int)nc : a.N;
}

DetLayout det_layout(const MdcnArgs &a0, const BwdPlan &) {
  auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
  MdcnArgs a = a0;
  a.N = det_chunk(a0);
  const BwdPlan pl = bwd_plan(a);
  DetLayout L{};
  const size_t nx = (size_t)a.N * a.C * a.H * a.W;
  const size_t nw = (size_t)a.Co * a.C * a.kh * a.kw;
  const size_t part = (size_t)pl.nsplit * nw * 4;
  L.gxi = 0;
  L.part = up(L.gxi + nx * 8);
  L.gw = L.part;  // the window form's accumulator shares the region with the global form's partials
  L.bounds = up(L.part + (part > GW_COPIES * nw * 8 ? part : GW_COPIES * nw * 8));
  L.scale = L.bounds + 16;
  L.xh = up(L.scale + 16);  // channels-last x and wT[k][c][co] (mdcn_bwd_data_nhwc_kernel)
  L.wt = up(L.xh + nx * 4);
  L.total = up(L.wt + nw * 4);
  return L;
}

// Float-atomic workspace (aanet_mdcn_bwd_ws_f32): [grad_x NHWC accumulator][x NHWC][wT]
// [bounds, scale] (the window form's fixed-point scale)
DetLayout ws_layout(const MdcnArgs &a) {
  auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
  DetLayout L{};
  const size_t nx = (size_t)a.N * a.C * a.H * a.W;
  const size_t nw = (size_t)a.Co * a.C * a.kh * a.kw;
  L.gxi = 0;
  L.xh = up(nx * 4);
  L.wt = up(L.xh + nx * 4);
  L.bounds = up(L.wt + nw * 4);
  L.scale = L.bounds + 16;
  L.gw = up(L.scale + 16);  // [GW_COPIES][K][Co][C] weight-gradient accumulator of the fused window form
  L.total = up(L.gw + GW_COPIES * nw * 4);
  return L;
}

bool bwd_nhwc_reads(const MdcnArgs &a) { return a.C % 4 == 0 && (a.C / a.dg) % 4 == 0; }

int mdcn_bwd_core(const float *x, const float *offset, const float *mask, const float *weight,
                  const float *grad_out, float *grad_x, float *grad_offset, float *grad_mask,
                  float *grad_weight, float *grad_bias, int n, int c, int h, int w, int co,
                  int kh, int kw, int stride, int pad, int dil, int groups, int dg, int det,
                  int algo, void *ws, size_t ws_bytes, hipStream_t st) {
  if (algo < AANET_DCN_BWD_AUTO || algo > AANET_DCN_BWD_WINDOW) return AANET_EINVAL;
  MdcnArgs a = make_args(x, offset, -1, mask, -1, 0, 1.f, weight, nullptr, nullptr, nullptr, 0,
                         nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg);
  int rc = check_shapes(a);
  if (rc) return rc;
  if (!x || !offset || !mask || !weight || !grad_out || !grad_x || !grad_offset || !grad_mask ||
      !grad_weight)
    return AANET_EINVAL;
  if (groups != 1) return AANET_EUNSUPPORTED;  // AANet uses groups=1 (nets/deform.py:25)
  if (co % 4 || co > 256) return AANET_EUNSUPPORTED;
  const long P = (long)a.Ho * a.Wo;
  const int K = kh * kw;
  const BwdPlan pl = bwd_plan(a);
  DetLayout L{};
  char *wb = static_cast<char *>(ws);
  // det: 0 float atomics into grad_x (NCHW); 1 deterministic (fixed point, workspace);
  // 2 float atomics into an NHWC workspace of n*h*w*c floats, then transposed into grad_x
  // (the deterministic form always scatters into its fixed-point accumulator in NHWC order)
  const int nhs = det != 0;
  det = det == 1;
  if (det || nhs) {
    L = det ? det_layout(a, pl) : ws_layout(a);
    if (!ws || ws_bytes < L.total) return AANET_EINVAL;
  }
  const bool nr = nhs && bwd_nhwc_reads(a);  // channels-last reads too
  const int GP = round_pitch(PT, 16), WTP = round_pitch(co, 2);
  // window form of grad_x (stride 1 / 2, <= 128 channels per deformable group, channels-last reads,
  // <= 9 taps, <= 64 output channels): 8x8 tile per workgroup in 16-channel slices, int64
  // fixed-point LDS window.
  // AUTO takes it in both modes; GLOBAL / WINDOW force one form (tests, A/B).
  const int R = 2;
  const int WR = win_rows(kh, dil, stride), WCw = win_rows(kw, dil, stride);
  const bool fusew = true;  // the weight gradient rides in the window kernel (both modes)
  // gOut tile pitch of the window kernel: 80 (= 16 mod 32) keeps the colg reads (rows kr,
  // columns jj) conflict-free; the fused weight gradient also reads it transposed (rows jj), which
  // that pitch makes 8-way conflicted, so the fused form uses 66 (2-way for both)
  const int GPW = fusew ? round_pitch(PT, 2) : GP;
  const size_t smem3 = sizeof(float) * ((size_t)co * GPW + (size_t)WHC * WTP + (size_t)WHC * WCP + (size_t)PT * 16 +
                                       (size_t)3 * WKMAX * PT + (fusew ? (size_t)WHC * WCP : 0)) +
                       (size_t)WR * WCw * WHC * 8;
  const bool win_ok = nr && win_shape_ok(a) && smem3 <= 160 * 1024;
  if (algo == AANET_DCN_BWD_WINDOW && !win_ok) return AANET_EUNSUPPORTED;
  // AUTO takes the window form where it measured faster: the aggregation's shapes (stride 1,
  // <= 32 channels per group, Co <= 64).  At the feature extractor's shapes (64-channel groups,
  // Co = 128, one workgroup per CU for its LDS) it measured slower in float mode (C4 feat_s1 /
  // feat_s2 990 / 1089 us vs 853 / 856 us global) and mixed in fixed point (983 vs 1046 us at
  // stride 1, 1177 vs 1073 at stride 2; CHANGELOG.md round 6): WINDOW selects it there.
  const bool win_auto = a.stride == 1 && a.C / a.dg <= 2 * WHC && a.Co <= 64;
  const bool use_win = win_ok && (algo == AANET_DCN_BWD_WINDOW || (algo == AANET_DCN_BWD_AUTO && win_auto));
  float *xh = nhs ? reinterpret_cast<float *>(wb + L.xh) : nullptr;
  float *wt = nhs ? reinterpret_cast<float *>(wb + L.wt) : nullptr;
  long long *gxi = det ? reinterpret_cast<long long *>(wb + L.gxi) : nullptr;
  float *part = det ? reinterpret_cast<float *>(wb + L.part) : nullptr;
  const bool fixed = det || use_win;  // a fixed-point scale is needed
  unsigned *bounds = fixed ? reinterpret_cast<unsigned *>(wb + L.bounds) : nullptr;
  double *scale = fixed ? reinterpret_cast<double *>(wb + L.scale) : nullptr;
  const size_t nx = (size_t)n * c * h * w;
  hipError_t e;
  if (det)
    e = hipMemsetAsync(gxi, 0, nx * 8, st);
  else
    e = hipMemsetAsync(nhs ? ws : grad_x, 0, sizeof(float) * nx, st);  // float atomics
  if (e != hipSuccess) return (int)e;
  if (fixed) {
    e = hipMemsetAsync(bounds, 0, 16, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(det_wbound_kernel, dim3(host_div_up((long)c * K, 256)), dim3(256), 0, st,
                       weight, co, c * K, bounds);
    const long ng = (long)n * co * P, nm = (long)n * dg * K * P;
    hipLaunchKernelGGL(det_absmax_kernel, dim3(host_div_up(ng, 1024) > 512 ? 512 : host_div_up(ng, 1024)),
                       dim3(256), 0, st, grad_out, ng, bounds + 1);
    hipLaunchKernelGGL(det_absmax_kernel, dim3(host_div_up(nm, 1024) > 512 ? 512 : host_div_up(nm, 1024)),
                       dim3(256), 0, st, mask, nm, bounds + 2);
    if (det && use_win) {  // max|x|: the window form's weight-gradient bound (det_scale_kernel)
      const long nxl = (long)nx;
      hipLaunchKernelGGL(det_absmax_kernel, dim3(host_div_up(nxl, 1024) > 512 ? 512 : host_div_up(nxl, 1024)),
                         dim3(256), 0, st, x, nxl, bounds + 3);
    }
    hipLaunchKernelGGL(det_scale_kernel, dim3(1), dim3(1), 0, st, bounds, scale, (long)n * P);
  }
  const size_t smem = sizeof(float) * ((size_t)co * GP + (size_t)KC * WTP + (size_t)KC * CP + 3 * 4 * 64 +
                                      (size_t)PT * 12);
  // sG grows with Co (Co = 128 in the feature extractor's DCNs: ~69 KB); a gfx950 workgroup may
  // use the CU's whole 160 KiB of LDS
  if (smem > 160 * 1024) return AANET_EUNSUPPORTED;
  static const bool lds_attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_kernel<0>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_kernel<1, 1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_kernel<0, 1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_nhwc_kernel<0>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_nhwc_kernel<1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_win_kernel<1, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mdcn_bwd_data_win_kernel<0, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)lds_attr;
  const dim3 gdata((unsigned)(n * host_div_up(P, PT)), (unsigned)dg);
  if (nr) {
    const long HW = (long)h * w;
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((unsigned)host_div_up(HW, 32), (unsigned)host_div_up(c, 32), (unsigned)n),
                       dim3(256), 0, st, x, xh, c, HW);
    const long nw = (long)co * c * K;
    hipLaunchKernelGGL(weight_kcco_kernel, dim3(host_div_up(nw, 256) > 1024 ? 1024 : host_div_up(nw, 256)),
                       dim3(256), 0, st, weight, wt, co, c, K);
    const size_t smem2 = sizeof(float) * ((size_t)co * GP + (size_t)KC * WTP + (size_t)KC * CP + (size_t)PT * 12);
#ifdef AANET_DEBUG_SWITCHES  // timing build only (skips the grad_x scatter: WRONG gradients)
    const char *dbg_env = getenv("AANET_DCN_BWD_DBG");
    a.dbg_noatom = dbg_env ? atoi(dbg_env) : 0;
    if (a.dbg_noatom) fprintf(stderr, "aanet: AANET_DCN_BWD_DBG -- timing build, gradients INVALID\n");
#else
    a.dbg_noatom = 0;
#endif
    if (use_win) {
      const dim3 gwin((unsigned)(n * host_div_up(a.Wo, 8) * host_div_up(a.Ho, 8)), (unsigned)dg);
      if (det) {
        long long *gwi = reinterpret_cast<long long *>(wb + L.gw);
        const long nw = (long)co * c * K;
        e = hipMemsetAsync(gwi, 0, sizeof(long long) * GW_COPIES * (size_t)nw, st);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL((mdcn_bwd_data_win_kernel<1, 1>), gwin, dim3(NT), smem3, st, a, xh, wt, grad_out,
                           grad_x, grad_offset, grad_mask, GPW, WTP, gxi, scale, WR, WCw, R, nullptr, gwi);
        hipLaunchKernelGGL(det_gw_final_kernel, dim3(host_div_up(nw, 256) > 1024 ? 1024 : host_div_up(nw, 256)),
                           dim3(256), 0, st, gwi, grad_weight, co, c, K, scale + 1);
      } else {
        float *gwT = reinterpret_cast<float *>(wb + L.gw);
        const long nw = (long)co * c * K;
        e = hipMemsetAsync(gwT, 0, sizeof(float) * GW_COPIES * (size_t)nw, st);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL((mdcn_bwd_data_win_kernel<0, 1>), gwin, dim3(NT), smem3, st, a, xh, wt, grad_out,
                           reinterpret_cast<float *>(wb + L.gxi), grad_offset, grad_mask, GPW, WTP,
                           nullptr, scale, WR, WCw, R, gwT);
        hipLaunchKernelGGL(gw_kcoc_add_kernel, dim3(host_div_up(nw, 256) > 1024 ? 1024 : host_div_up(nw, 256)),
                           dim3(256), 0, st, gwT, grad_weight, co, c, K);
      }
    } else if (det)
      hipLaunchKernelGGL(mdcn_bwd_data_nhwc_kernel<1>, gdata, dim3(NT), smem2, st, a, xh, wt, grad_out,
                         grad_x, grad_offset, grad_mask, GP, WTP, gxi, scale);
    else
      hipLaunchKernelGGL(mdcn_bwd_data_nhwc_kernel<0>, gdata, dim3(NT), smem2, st, a, xh, wt, grad_out,
                         reinterpret_cast<float *>(wb + L.gxi), grad_offset, grad_mask, GP, WTP,
                         nullptr, nullptr);
  } else if (det)
    hipLaunchKernelGGL((mdcn_bwd_data_kernel<1, 1>), gdata, dim3(NT), smem, st, a, grad_out, grad_x,
                       grad_offset, grad_mask, GP, WTP, gxi, scale);
  else if (nhs)
    hipLaunchKernelGGL((mdcn_bwd_data_kernel<0, 1>), gdata, dim3(NT), smem, st, a, grad_out,
                       reinterpret_cast<float *>(wb + L.gxi), grad_offset, grad_mask, GP, WTP, nullptr, nullptr);
  else
    hipLaunchKernelGGL(mdcn_bwd_data_kernel<0>, gdata, dim3(NT), smem, st, a, grad_out, grad_x,
                       grad_offset, grad_mask, GP, WTP, nullptr, nullptr);
  rc = aanet_launch_status();
  if (rc) return rc;
  {
    const long HW = (long)h * w;
    const dim3 gt((unsigned)host_div_up(HW, 32), (unsigned)host_div_up(c, 32), (unsigned)n);
    if (det)
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<long long>, gt, dim3(256), 0, st, gxi, grad_x, c, HW, scale);
    else if (nhs)
      hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, gt, dim3(256), 0, st,
                         reinterpret_cast<const float *>(wb + L.gxi), grad_x, c, HW, nullptr);
    rc = aanet_launch_status();
    if (rc) return rc;
  }
  const dim3 gw3(pl.nchunks, (unsigned)pl.nsplit, host_div_up(co, 64));
  if (use_win && fusew)
    ;  // the window kernel added the weight gradient
  else if (nr && det)
    hipLaunchKernelGGL((mdcn_bwd_weight_kernel<1, 1>), gw3, dim3(NT), 0, st, a, grad_out, grad_weight,
                       pl.npieces, pl.range, part, xh);
  else if (nr)
    hipLaunchKernelGGL((mdcn_bwd_weight_kernel<0, 1>), gw3, dim3(NT), 0, st, a, grad_out, grad_weight,
                       pl.npieces, pl.range, nullptr, xh);
  else if (det)
    hipLaunchKernelGGL(mdcn_bwd_weight_kernel<1>, gw3, dim3(NT), 0, st, a, grad_out, grad_weight,
                       pl.npieces, pl.range, part);
  else
    hipLaunchKernelGGL(mdcn_bwd_weight_kernel<0>, gw3, dim3(NT), 0, st, a, grad_out, grad_weight,
                       pl.npieces, pl.range, nullptr);
  rc = aanet_launch_status();
  if (rc) return rc;
  if (det && !(use_win && fusew)) {
    const long nw = (long)co * c * K;
    hipLaunchKernelGGL(det_weight_reduce_kernel, dim3(host_div_up(nw, 64)), dim3(256), 0, st,
                       part, grad_weight, nw, pl.nsplit);
    rc = aanet_launch_status();
    if (rc) return rc;
  }
  if (grad_bias) {
    hipLaunchKernelGGL(bias_grad_kernel, dim3(co), dim3(1024), 0, st, grad_out, grad_bias, n, co, P);
    rc = aanet_launch_status();
  }
  return rc;
}

// The backward entry: the deterministic mode (det == 1) runs mdcn_bwd_core over chunks of images
// (det_chunk) that share one workspace -- grad_x / grad_offset / grad_mask are per image, the
// weight gradient is added per chunk in chunk order -- and the bias gradient once over the batch.
int mdcn_bwd_impl(const float *x, const float *offset, const float *mask, const float *weight,
                  const float *grad_out, float *grad_x, float *grad_offset, float *grad_mask,
                  float *grad_weight, float *grad_bias, int n, int c, int h, int w, int co,
                  int kh, int kw, int stride, int pad, int dil, int groups, int dg, int det,
                  int algo, void *ws, size_t ws_bytes, hipStream_t st) {
  MdcnArgs a = make_args(x, offset, -1, mask, -1, 0, 1.f, weight, nullptr, nullptr, nullptr, 0,
                         nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg);
  if (det != 1 || check_shapes(a) || !x || !offset || !mask || !grad_out || !grad_x || !grad_offset ||
      !grad_mask)
    return mdcn_bwd_core(x, offset, mask, weight, grad_out, grad_x, grad_offset, grad_mask, grad_weight,
                         grad_bias, n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg, det, algo, ws,
                         ws_bytes, st);
  const int nc = det_chunk(a);
  if (ws_bytes < det_layout(a, BwdPlan{}).total) return AANET_EINVAL;
  const long P = (long)a.Ho * a.Wo, K = (long)kh * kw;
  const long sx = (long)c * h * w, soff = 2L * dg * K * P, sm = (long)dg * K * P, sg = (long)co * P;
  for (int i0 = 0; i0 < n; i0 += nc) {
    const int m = n - i0 < nc ? n - i0 : nc;
    const int rc = mdcn_bwd_core(x + i0 * sx, offset + i0 * soff, mask + i0 * sm, weight, grad_out + i0 * sg,
                                 grad_x + i0 * sx, grad_offset + i0 * soff, grad_mask + i0 * sm, grad_weight,
                                 nullptr, m, c, h, w, co, kh, kw, stride, pad, dil, groups, dg, det, algo, ws,
                                 ws_bytes, st);
    if (rc) return rc;
  }
  if (grad_bias) {
    hipLaunchKernelGGL(bias_grad_kernel, dim3(co), dim3(1024), 0, st, grad_out, grad_bias, n, co, P);
    return aanet_launch_status();
  }
  return 0;
}

// Workgroups per conv weight-gradient launch (pixel splits x chunks x co tiles, before rounding):
// fewer splits mean longer MFMA accumulation per workgroup and less partial-sum traffic for the
// reduction.  Training step (bench.py --train, same-call A/B): 14.44 ms at 1024, 14.59 at 2048,
// 14.42 at 768, 14.53 at 512, 14.87 at 4096.
#ifndef AANET_WGRAD_WGS
#define AANET_WGRAD_WGS 1024
#endif
// aanet_conv2d_wgrad_f32: the weight kernel in PLAIN form (a.dg = groups), then for det the
// fixed-order reduction of the per-split partials; the bias gradient is a per-channel sum in a
// fixed order either way.  det == 2: the same, but the reduction and the bias sum STORE their
// results (grad_weight / grad_bias need no zero fill beforehand).
int conv_wgrad_impl(const float *x, const float *grad_out, float *grad_weight, float *grad_bias,
                    int n, int c, int h, int w, int co, int kh, int kw, int stride, int pad,
                    int dil, int groups, int det, void *ws, size_t ws_bytes, hipStream_t st) {
  MdcnArgs a = make_args(x, nullptr, -1, nullptr, -1, 0, 1.f, nullptr, nullptr, nullptr, nullptr,
                         0, nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups, groups);
  int rc = check_shapes(a);
  if (rc) return rc;
  if (!x || !grad_out || !grad_weight || det < 0 || det > 2) return AANET_EINVAL;
  const BwdPlan pl = bwd_plan(a, AANET_WGRAD_WGS);
  const long nw = (long)co * (c / groups) * kh * kw;
  float *part = nullptr;
  if (det) {
    if (!ws || ws_bytes < (size_t)pl.nsplit * nw * 4) return AANET_EINVAL;
    part = static_cast<float *>(ws);
  }
  const dim3 gw3(pl.nchunks, (unsigned)pl.nsplit, host_div_up(co / groups, 64));
  if (det)
    hipLaunchKernelGGL((mdcn_bwd_weight_kernel<1, 0, 1>), gw3, dim3(NT), 0, st, a, grad_out,
                       grad_weight, pl.npieces, pl.range, part, nullptr);
  else
    hipLaunchKernelGGL((mdcn_bwd_weight_kernel<0, 0, 1>), gw3, dim3(NT), 0, st, a, grad_out,
                       grad_weight, pl.npieces, pl.range, nullptr, nullptr);
  rc = aanet_launch_status();
  if (rc) return rc;
  if (det) {
    hipLaunchKernelGGL(det_weight_reduce_kernel, dim3(host_div_up(nw, 64)), dim3(256), 0, st,
                       part, grad_weight, nw, pl.nsplit, (int)(det == 2));
    rc = aanet_launch_status();
    if (rc) return rc;
  }
  if (grad_bias) {
    hipLaunchKernelGGL(bias_grad_kernel, dim3(co), dim3(1024), 0, st, grad_out, grad_bias, n, co,
                       (long)a.Ho * a.Wo, (int)(det == 2));
    rc = aanet_launch_status();
  }
  return rc;
}

}  // namespace

extern "C" size_t aanet_conv2d_wgrad_workspace_size(int n, int c, int h, int w, int co, int kh,
                                                    int kw, int stride, int pad, int dil,
                                                    int groups) {
  MdcnArgs a = make_args(nullptr, nullptr, -1, nullptr, -1, 0, 1.f, nullptr, nullptr, nullptr,
                         nullptr, 0, nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups,
                         groups);
  if (check_shapes(a)) return 0;
  return (size_t)bwd_plan(a, AANET_WGRAD_WGS).nsplit * co * (c / groups) * kh * kw * 4;
}

extern "C" int aanet_conv2d_wgrad_f32(const float *x, const float *grad_out, float *grad_weight,
                                      float *grad_bias, int n, int c, int h, int w, int co, int kh,
                                      int kw, int stride, int pad, int dil, int groups,
                                      int deterministic, void *workspace, size_t workspace_bytes,
                                      aanet_stream_t stream) {
  return conv_wgrad_impl(x, grad_out, grad_weight, grad_bias, n, c, h, w, co, kh, kw, stride, pad,
                         dil, groups, deterministic, workspace, workspace_bytes, as_hip(stream));
}

extern "C" int aanet_mdcn_bwd_f32(const float *x, const float *offset, const float *mask,
                                  const float *weight, const float *grad_out, float *grad_x,
                                  float *grad_offset, float *grad_mask, float *grad_weight,
                                  float *grad_bias, int n, int c, int h, int w, int co, int kh,
                                  int kw, int stride, int pad, int dil, int groups, int dg,
                                  aanet_stream_t stream) {
  return mdcn_bwd_impl(x, offset, mask, weight, grad_out, grad_x, grad_offset, grad_mask,
                       grad_weight, grad_bias, n, c, h, w, co, kh, kw, stride, pad, dil, groups,
                       dg, 0, AANET_DCN_BWD_GLOBAL, nullptr, 0, as_hip(stream));
}

extern "C" size_t aanet_mdcn_bwd_ws_workspace_size(int n, int c, int h, int w, int co, int kh,
                                                   int kw, int stride, int pad, int dil,
                                                   int groups, int dg) {
  MdcnArgs a = make_args(nullptr, nullptr, -1, nullptr, -1, 0, 1.f, nullptr, nullptr, nullptr,
                         nullptr, 0, nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg);
  if (check_shapes(a)) return 0;
  return ws_layout(a).total;
}

extern "C" int aanet_mdcn_bwd_ws_f32(const float *x, const float *offset, const float *mask,
                                     const float *weight, const float *grad_out, float *grad_x,
                                     float *grad_offset, float *grad_mask, float *grad_weight,
                                     float *grad_bias, int n, int c, int h, int w, int co, int kh,
                                     int kw, int stride, int pad, int dil, int groups, int dg,
                                     void *workspace, size_t workspace_bytes,
                                     aanet_stream_t stream) {
  return mdcn_bwd_impl(x, offset, mask, weight, grad_out, grad_x, grad_offset, grad_mask,
                       grad_weight, grad_bias, n, c, h, w, co, kh, kw, stride, pad, dil, groups,
                       dg, 2, AANET_DCN_BWD_AUTO, workspace, workspace_bytes, as_hip(stream));
}

extern "C" size_t aanet_mdcn_bwd_det_workspace_size(int n, int c, int h, int w, int co, int kh,
                                                    int kw, int stride, int pad, int dil,
                                                    int groups, int dg) {
  MdcnArgs a = make_args(nullptr, nullptr, -1, nullptr, -1, 0, 1.f, nullptr, nullptr, nullptr,
                         nullptr, 0, nullptr, n, c, h, w, co, kh, kw, stride, pad, dil, groups, dg);
  if (check_shapes(a)) return 0;
  return det_layout(a, bwd_plan(a)).total;
}

extern "C" int aanet_mdcn_bwd_det_f32(const float *x, const float *offset, const float *mask,
                                      const float *weight, const float *grad_out, float *grad_x,
                                      float *grad_offset, float *grad_mask, float *grad_weight,
                                      float *grad_bias, int n, int c, int h, int w, int co,
                                      int kh, int kw, int stride, int pad, int dil, int groups,
                                      int dg, void *workspace, size_t workspace_bytes,
                                      aanet_stream_t stream) {
  return mdcn_bwd_impl(x, offset, mask, weight, grad_out, grad_x, grad_offset, grad_mask,
                       grad_weight, grad_bias, n, c, h, w, co, kh, kw, stride, pad, dil, groups,
                       dg, 1, AANET_DCN_BWD_AUTO, workspace, workspace_bytes, as_hip(stream));
}

extern "C" int aanet_mdcn_bwd_algo_f32(const float *x, const float *offset, const float *mask,
                                       const float *weight, const float *grad_out, float *grad_x,
                                       float *grad_offset, float *grad_mask, float *grad_weight,
                                       float *grad_bias, int n, int c, int h, int w, int co,
                                       int kh, int kw, int stride, int pad, int dil, int groups,
                                       int dg, int deterministic, int algo, void *workspace,
                                       size_t workspace_bytes, aanet_stream_t stream) {
  if (deterministic != 0 && deterministic != 1) return AANET_EINVAL;
  return mdcn_bwd_impl(x, offset, mask, weight, grad_out, grad_x, grad_offset, grad_mask,
                       grad_weight, grad_bias, n, c, h, w, co, kh, kw, stride, pad, dil, groups,
                       dg, deterministic ? 1 : 2, algo, workspace, workspace_bytes, as_hip(stream));
}
