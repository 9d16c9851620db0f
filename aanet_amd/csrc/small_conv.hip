// small_conv.hip -- direct (VALU) convolution for the few-channel convs around the hot path,
// behind aanet_conv2d_fused_f32: the first conv of the AANet feature extractor (3 -> 32, 7x7,
// stride 3; nets/resnet.py), GA-Net's conv_start (3 -> 32, 3x3; nets/feature.py), the refinement
// stems (6 -> 16 and 1 -> 16, 3x3; nets/refinement.py:92-99) and the refinement's final_conv
// (32 -> 1, 3x3, channels-last input; nets/refinement.py:100-106).
//
// On the implicit-GEMM engine these shapes waste most of the matrix work: a K chunk is 32
// channels of ONE tap, so Cin = 3 pads every tap to 32 (the 7x7 stride-3 conv ran 10.7x its
// MACs, 457 us for 4 GFLOP at B=8), and Co = 1 fills one row of a 16-row MFMA tile (370 us for a
// 61 us memory-bound conv).  Here a thread computes one output pixel and all CO_T output channels
// with f32 FMAs (exact fp32, the reference's arithmetic): the input tile (with its halo) and the
// weights, transposed to [ci][ky][kx][co], are staged in LDS once per workgroup; each tap reads
// one input value (consecutive lanes, consecutive or stride-S words: conflict-free) and the
// CO_T weights as broadcast ds_read_b128 (all lanes one address).  Bound: the VALU FMA rate
// (CIN*KS*KS*CO_T FMAs per pixel) or, for Co = 1, the LDS read rate.
#include "small_conv.h"

namespace {

constexpr int NT = 256;
constexpr int TY = 8, TX = 32;  // output tile: 8 rows x 32 columns, one pixel per thread

__device__ __forceinline__ float act_f(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);
  return v > 0.f ? v : neg;
}

template <int CIN, int KS, int S, int CO_T, bool NHWC_IN>
__global__ __launch_bounds__(NT) void conv_direct_kernel(DirectArgs a) {
  constexpr int IR = (TY - 1) * S + KS, IC = (TX - 1) * S + KS;  // input tile (dilation 1)
  constexpr int NK = CIN * KS * KS;
  __shared__ __attribute__((aligned(16))) float sIn[CIN * IR * IC];
  __shared__ __attribute__((aligned(16))) float sW[NK * CO_T];
  const int tid = threadIdx.x;
  const int tx_n = (a.Wo + TX - 1) / TX, ty_n = (a.Ho + TY - 1) / TY;
  const int n = blockIdx.x / (tx_n * ty_n), t = blockIdx.x % (tx_n * ty_n);
  const int oy0 = (t / tx_n) * TY, ox0 = (t % tx_n) * TX;
  const int iy0 = oy0 * S - a.pad, ix0 = ox0 * S - a.pad;
  const long HW = (long)a.H * a.W;
  // weights -> sW[(ci*KS*KS + k) * CO_T + co] (zero past Co); raw [co][ci][ky][kx] or packed
  // [ky][kx][co][ci] (aanet_conv_weight_pack_f32)
  for (int e = tid; e < NK * CO_T; e += NT) {
    const int co = e % CO_T, ik = e / CO_T, ci = ik / (KS * KS), k = ik % (KS * KS);
    float v = 0.f;
    if (co < a.Co) v = a.packed ? a.w[((long)k * a.Co + co) * CIN + ci] : a.w[((long)co * CIN + ci) * KS * KS + k];
    sW[e] = v;
  }
  // input tile with its halo, zero outside the image: [ci][row][col]
  if constexpr (NHWC_IN) {
    static_assert(CIN % 4 == 0, "channels-last staging reads channel quads");
    const float *xn = a.x + (long)n * HW * CIN;
    for (int e = tid; e < IR * IC * (CIN / 4); e += NT) {
      const int q = e % (CIN / 4), pos = e / (CIN / 4), r = pos / IC, c = pos % IC;
      const int gy = iy0 + r, gx = ix0 + c;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W)
        v = *reinterpret_cast<const f32x4 *>(xn + ((long)gy * a.W + gx) * CIN + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) sIn[((4 * q + u) * IR + r) * IC + c] = v[u];
    }
  } else {
    const float *xn = a.x + (long)n * CIN * HW;
    for (int e = tid; e < CIN * IR * IC; e += NT) {
      const int c = e % IC, r = (e / IC) % IR, ci = e / (IC * IR);
      const int gy = iy0 + r, gx = ix0 + c;
      sIn[e] = (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) ? xn[(long)ci * HW + (long)gy * a.W + gx] : 0.f;
    }
  }
  __syncthreads();
  const int ty = tid / TX, tx = tid % TX;
  float acc[CO_T];
#pragma unroll
  for (int co = 0; co < CO_T; ++co) acc[co] = 0.f;
  // one kernel row (KS taps) of one input channel
  auto row = [&](int ci, int ky) {
      const float *ip = sIn + (ci * IR + ty * S + ky) * IC + tx * S;
      const float *wp = sW + ((ci * KS + ky) * KS) * CO_T;
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float v = ip[kx];
        if constexpr (CO_T % 4 == 0) {
#pragma unroll
          for (int q = 0; q < CO_T / 4; ++q) {
            const f32x4 w4 = *reinterpret_cast<const f32x4 *>(wp + kx * CO_T + 4 * q);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[4 * q + u] = __builtin_fmaf(w4[u], v, acc[4 * q + u]);
          }
        } else {
#pragma unroll
          for (int co = 0; co < CO_T; ++co) acc[co] = __builtin_fmaf(wp[kx * CO_T + co], v, acc[co]);
        }
      }
  };
  auto channel = [&](int ci) {
    if constexpr (KS > 3) {  // 7x7: the rows as a loop (the unrolled body would be ~6k instructions)
#pragma unroll 1
      for (int ky = 0; ky < KS; ++ky) row(ci, ky);
    } else {
#pragma unroll
      for (int ky = 0; ky < KS; ++ky) row(ci, ky);
    }
  };
  if constexpr (CIN >= 16) {
    // many-channel inputs (final_conv, 32 channels): a loop over channels, or the unrolled reads
    // of all 288 taps are hoisted into registers (256 VGPRs + scratch)
#pragma unroll 4
    for (int ci = 0; ci < CIN; ++ci) channel(ci);
  } else {
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) channel(ci);
  }
  const int oy = oy0 + ty, ox = ox0 + tx;
  if (oy >= a.Ho || ox >= a.Wo) return;
  const long P = (long)a.Ho * a.Wo, p = (long)oy * a.Wo + ox;
#pragma unroll
  for (int co = 0; co < CO_T; ++co) {
    if (co >= a.Co) break;
    float v = acc[co] + (a.bias ? a.bias[co] : 0.f);
    if (a.post_scale) v = v * a.post_scale[co] + a.post_shift[co];
    const long o = ((long)n * a.Co + co) * P + p;
    if (a.residual) v += a.residual[o];
    a.out[o] = act_f(v, a.act);
  }
}

template <int CIN, int KS, int S, int CO_T, bool NHWC_IN>
int launch(const DirectArgs &a, hipStream_t st) {
  const long tiles = (long)host_div_up(a.Wo, TX) * host_div_up(a.Ho, TY);
  hipLaunchKernelGGL((conv_direct_kernel<CIN, KS, S, CO_T, NHWC_IN>), dim3((unsigned)(a.N * tiles)),
                     dim3(NT), 0, st, a);
  return aanet_launch_status();
}

// The warp-error stem of the StereoDRNet / Hourglass refinement (nets/refinement.py:92-99,
// 148-155) in one launch: conv1 (3x3, [warped - left, left] -> 16, BN folded, LeakyReLU) and conv2
// (3x3, disparity -> 16, same) written side by side as the 32 channels of ONE channels-last
// tensor -- what torch.cat((conv1, conv2), 1) followed by the dilated stack's NCHW -> NHWC copy
// produced (6 launches: subtraction, two concats, two convs, the copy; 0.9 ms at 384x1248, B=8).
// Per output channel the arithmetic is conv_direct_kernel's (<6,3,1,16> / <1,3,1,16>): the same
// staged tile, the same tap and channel order, so the values are identical.
__global__ __launch_bounds__(NT) void refine_stem_kernel(StemArgs a) {
  constexpr int IR = TY + 2, IC = TX + 2, CA = 6;  // input tile (3x3, pad 1); conv1's channels
  __shared__ __attribute__((aligned(16))) float sIn[(CA + 1) * IR * IC];
  __shared__ __attribute__((aligned(16))) float sW1[CA * 9 * 16];
  __shared__ __attribute__((aligned(16))) float sW2[9 * 16];
  const int tid = threadIdx.x;
  const int tx_n = (a.W + TX - 1) / TX, ty_n = (a.H + TY - 1) / TY;
  const int n = blockIdx.x / (tx_n * ty_n), t = blockIdx.x % (tx_n * ty_n);
  const int oy0 = (t / tx_n) * TY, ox0 = (t % tx_n) * TX;
  const long HW = (long)a.H * a.W;
  // weights, raw [co][ci][ky][kx] -> [(ci*9 + k) * 16 + co]
  for (int e = tid; e < CA * 9 * 16; e += NT) {
    const int co = e % 16, ik = e / 16, ci = ik / 9, k = ik % 9;
    sW1[e] = a.w1[(co * CA + ci) * 9 + k];
  }
  for (int e = tid; e < 9 * 16; e += NT) sW2[e] = a.w2[(e % 16) * 9 + e / 16];
  // [warped - left (3), left (3), disparity] with the halo, zero outside the image
  const float *wn = a.warped + (long)n * 3 * HW, *ln = a.left + (long)n * 3 * HW, *dn = a.disp + (long)n * HW;
  for (int e = tid; e < (CA + 1) * IR * IC; e += NT) {
    const int c = e % IC, r = (e / IC) % IR, ci = e / (IC * IR);
    const int gy = oy0 - 1 + r, gx = ox0 - 1 + c;
    float v = 0.f;
    if (gy >= 0 && gy < a.H && gx >= 0 && gx < a.W) {
      const long o = (long)gy * a.W + gx;
      v = ci < 3 ? wn[ci * HW + o] - ln[ci * HW + o] : (ci < CA ? ln[(ci - 3) * HW + o] : dn[o]);
    }
    sIn[e] = v;
  }
  __syncthreads();
  const int ty = tid / TX, tx = tid % TX;
  float acc[32];
#pragma unroll
  for (int co = 0; co < 32; ++co) acc[co] = 0.f;
  auto tap_row = [&](int ci, int ky, const float *wrow, int c0) {
    const float *ip = sIn + (ci * IR + ty + ky) * IC + tx;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const float v = ip[kx];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 w4 = *reinterpret_cast<const f32x4 *>(wrow + kx * 16 + 4 * q);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[c0 + 4 * q + u] = __builtin_fmaf(w4[u], v, acc[c0 + 4 * q + u]);
      }
    }
  };
#pragma unroll
  for (int ci = 0; ci < CA; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) tap_row(ci, ky, sW1 + (ci * 3 + ky) * 3 * 16, 0);
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) tap_row(CA, ky, sW2 + ky * 3 * 16, 16);
  const int oy = oy0 + ty, ox = ox0 + tx;
  if (oy >= a.H || ox >= a.W) return;
  float *dst = a.out + ((long)n * HW + (long)oy * a.W + ox) * 32;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    f32x4 v;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int co = 4 * q + u;
      v[u] = act_f(acc[co] + (co < 16 ? a.b1[co] : a.b2[co - 16]), a.act);
    }
    *reinterpret_cast<f32x4 *>(dst + 4 * q) = v;
  }
}

}  // namespace

extern "C" int aanet_refine_stem_f32(const float *warped, const float *left, const float *disp,
                                     const float *w1, const float *b1, const float *w2,
                                     const float *b2, int act, float *out_nhwc, int n, int h,
                                     int w, aanet_stream_t stream) {
  if (!warped || !left || !disp || !w1 || !b1 || !w2 || !b2 || !out_nhwc || act < 0 || act > 2 ||
      n < 0 || h < 0 || w < 0)
    return AANET_EINVAL;
  const long tiles = (long)host_div_up(w, TX) * host_div_up(h, TY);
  if ((long)n * tiles == 0) return AANET_OK;
  if ((long)n * tiles >= (1L << 31)) return AANET_EUNSUPPORTED;
  StemArgs a{warped, left, disp, w1, b1, w2, b2, out_nhwc, act, n, h, w};
  hipLaunchKernelGGL(refine_stem_kernel, dim3((unsigned)(n * tiles)), dim3(NT), 0, as_hip(stream), a);
  return aanet_launch_status();
}

int conv_direct_launch(const DirectArgs &a, int k, int stride, int dil, hipStream_t st) {
  if (dil != 1 || a.N <= 0 || (long)a.N * host_div_up(a.Wo, TX) * host_div_up(a.Ho, TY) >= (1L << 31))
    return AANET_EUNSUPPORTED;
  const int C = a.C, Co = a.Co;
  if (!a.in_nhwc) {
    if (C == 3 && k == 7 && stride == 3 && Co <= 32) return launch<3, 7, 3, 32, false>(a, st);
    if (C == 3 && k == 3 && stride == 1 && Co <= 32) return launch<3, 3, 1, 32, false>(a, st);
    if (C == 6 && k == 3 && stride == 1 && Co <= 16) return launch<6, 3, 1, 16, false>(a, st);
    if (C == 1 && k == 3 && stride == 1 && Co <= 16) return launch<1, 3, 1, 16, false>(a, st);
    if (C == 32 && k == 3 && stride == 1 && Co == 1) return launch<32, 3, 1, 1, false>(a, st);
  } else {
    if (C == 32 && k == 3 && stride == 1 && Co == 1) return launch<32, 3, 1, 1, true>(a, st);
  }
  return AANET_EUNSUPPORTED;
}
