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

}  // namespace

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
