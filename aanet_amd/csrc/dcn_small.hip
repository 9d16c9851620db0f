// dcn_small.hip -- the deformable conv of the aggregation's coarsest scale (nets/deform.py:216-236
// at scale 2 of the C2 config: 16 channels in two deformable groups of 8, Co = 16, 3x3, dil 2), as
// the bottleneck tail (DCN + BN2 + ReLU -> conv3 1x1 + BN3 + identity + ReLU) or the op-level DCN
// (ModulatedDeformConvFunction: act(post_scale * (DCN + bias) + post_shift)).
//
// Why a third DCN kernel.  The implicit-GEMM engine (mdcn.hip conv_fwd_kernel, MODE 1) pads each
// K chunk to 32 channels of one deformable group, so 8-channel groups run 4x their MACs through
// the matrix pipe, and its 16-channel output tiles give 208 workgroups for the whole batch: 35 us
// for 0.12 GFLOP (C4 agg_s2).  The work is tiny (26.6 k pixels x 144 x 16 MACs) and latency-bound,
// so here it is plain fp32 VALU, one output pixel per lane: a workgroup is six waves over the same
// 64 pixels, wave w taking deformable group w % 2 and taps 3(w / 2) .. 3(w / 2) + 2 (8 channels x
// 3 taps = 24 sampled values per pixel), so that a wave's whole input is two dependent memory
// rounds.  The weights are wave-uniform (group, tap), read as broadcast LDS operands.  The six
// partial sums meet in LDS, and four waves finish 4 of the 16 output channels each.
//
// Numerics: the sampling state follows kernel.cu:467-497 (dcn_tile.hip tap_state) bit for bit
// (fp contraction off), the blend is ((c0 w0 + c1 w1) + c2 w2) + c3 w3 with the mask folded into
// the weights, and the contraction is exact fp32 products with fp32 sums (the reference's im2col +
// fp32 GEMM arithmetic; only the summation order differs).
#include "dcn_small.h"

namespace {

constexpr int TS = 3;          // tap thirds: wave w takes group w % 2, taps 3(w / 2) .. +2
constexpr int NW = 2 * TS;     // waves per workgroup, all on the same 64 pixels
constexpr int NT = 64 * NW;
constexpr int K = 9;           // 3x3 taps
constexpr int KT = K / TS;     // taps per wave
constexpr int CG = 8;          // channels per deformable group
constexpr int CT = 16;         // channels = Co (= Co2)
constexpr int EW = 4;          // epilogue waves (CT / EW output channels each)

__device__ __forceinline__ float act_f(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);
  return v > 0.f ? v : neg;
}

struct Samp {
  unsigned o[4];  // corner byte offsets within a channel plane (out of range: corner invalid)
  float w[4];     // corner weights, mask folded
};

template <bool TAIL, bool PACKED>
__global__ __launch_bounds__(NT) void dcn_small_kernel(DcnSmallArgs a) {
  __shared__ float sP[NW][CT][64];  // per-wave partial sums [wave][co][pixel]
  // weights [group][tap][co][c] (broadcast ds_read_b128 operands: wave-uniform addresses) and
  // conv3 [co2][c].  (As scalar loads, 1152 SGPR operands per wave spilled through VGPR lanes.)
  __shared__ __attribute__((aligned(16))) float sW[2][K][CT][CG];
  __shared__ __attribute__((aligned(16))) float sT[CT][CT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave & 1, t0 = (wave >> 1) * KT;
  const int n = blockIdx.y;
  const int H = a.H, W = a.W, P = H * W, dil = a.dil;
  const int p = blockIdx.x * 64 + lane;
  const bool pv = p < P;
  const int py = pv ? p / W : 0, px = pv ? p - (p / W) * W : 0;
  const unsigned plane = 4u * (unsigned)P;
  const unsigned oob = plane * CT;  // past the image: the buffer load returns 0

  const brsrc_t xr = buf_rsrc(a.x + (long)n * CT * P, (long)CT * P * 4);
  const brsrc_t offr = buf_rsrc(a.offset + (long)n * a.off_bs, (long)2 * 2 * K * P * 4);
  const brsrc_t mskr = buf_rsrc(a.mask + (long)n * a.mask_bs, (long)2 * K * P * 4);
  const unsigned p4 = 4u * (unsigned)(pv ? p : 0);

  // The whole wave's input in two dependent rounds: its taps' offsets / mask, then every corner
  // of its 3 taps x 8 channels (96 dword gathers in flight).  The 6 waves of a workgroup (and
  // the 2-3 workgroups per CU) overlap each other's rounds.  (Two waves of 9 taps each, pipelined
  // one tap ahead, waited on each tap's gathers: 19.4 us for C4 agg_s2.)
  float oh[KT], ow[KT], ml[KT];
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    const int k = t0 + u;
    oh[u] = buf_ld1(offr, p4 + (unsigned)(g * 2 * K + 2 * k) * plane);
    ow[u] = buf_ld1(offr, p4 + (unsigned)(g * 2 * K + 2 * k + 1) * plane);
    ml[u] = buf_ld1(mskr, p4 + (unsigned)(g * K + k) * plane);
  }
  // weights -> LDS (packed [k][co][c] or raw [co][c][k]), while the offsets are in flight
  for (int e = tid; e < CT * CT * K; e += NT) {
    int k, co, c;
    if (PACKED) {
      c = e % CT, co = (e / CT) % CT, k = e / (CT * CT);
    } else {
      k = e % K, c = (e / K) % CT, co = e / (K * CT);
    }
    sW[c / CG][k][co][c % CG] = a.w[e];
  }
  if (TAIL)
    for (int e = tid; e < CT * CT; e += NT) sT[e / CT][e % CT] = a.tail_w[e];
  Samp st[KT];
#pragma unroll
  for (int u = 0; u < KT; ++u) {
#pragma clang fp contract(off)
    const int k = t0 + u, i = k / 3, j = k - 3 * (k / 3);
    float m = a.mask_logits ? a.mask_scale * __builtin_amdgcn_rcpf(1.f + __expf(-ml[u])) : ml[u];
    if (!pv) m = 0.f;
    const float h = (float)(py - a.pad + i * dil) + oh[u];
    const float w = (float)(px - a.pad + j * dil) + ow[u];
    const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
    const int hl = (int)floorf(h), wl = (int)floorf(w);
    const float lh = h - (float)hl, lw = w - (float)wl;
    const float hh = 1.f - lh, hw = 1.f - lw;
    const bool ok1 = valid && hl >= 0 && wl >= 0;
    const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
    const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
    const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
    st[u].w[0] = (ok1 ? hh * hw : 0.f) * m;
    st[u].w[1] = (ok2 ? hh * lw : 0.f) * m;
    st[u].w[2] = (ok3 ? lh * hw : 0.f) * m;
    st[u].w[3] = (ok4 ? lh * lw : 0.f) * m;
    const unsigned b = 4u * (unsigned)(hl * W + wl);
    st[u].o[0] = ok1 ? b : oob;
    st[u].o[1] = ok2 ? b + 4u : oob;
    st[u].o[2] = ok3 ? b + 4u * (unsigned)W : oob;
    st[u].o[3] = ok4 ? b + 4u * (unsigned)(W + 1) : oob;
  }
  // the group's 8 channel planes: plane offset in the SGPR soffset, corner offset per lane
  float v[KT][CG][4];
#pragma unroll
  for (int u = 0; u < KT; ++u)
#pragma unroll
    for (int c = 0; c < CG; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[u][c][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   xr, (int)st[u].o[q], (int)((g * CG + c) * plane), 0));
  __syncthreads();  // weights staged
  // blend the corners, then acc[co] += w[k][co][c] * value[c] (weights: broadcast LDS reads)
  float acc[CT];
#pragma unroll
  for (int co = 0; co < CT; ++co) acc[co] = 0.f;
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    float b[CG];
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      float t = v[u][c][0] * st[u].w[0];
      t = __builtin_fmaf(v[u][c][1], st[u].w[1], t);
      t = __builtin_fmaf(v[u][c][2], st[u].w[2], t);
      b[c] = __builtin_fmaf(v[u][c][3], st[u].w[3], t);
    }
#pragma unroll
    for (int co = 0; co < CT; ++co) {
      const f32x4 w0 = *reinterpret_cast<const f32x4 *>(&sW[g][t0 + u][co][0]);
      const f32x4 w1 = *reinterpret_cast<const f32x4 *>(&sW[g][t0 + u][co][4]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[co] = __builtin_fmaf(w0[c], b[c], acc[co]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[co] = __builtin_fmaf(w1[c], b[4 + c], acc[co]);
    }
  }
#pragma unroll
  for (int co = 0; co < CT; ++co) sP[wave][co][lane] = acc[co];
  __syncthreads();
  if (wave >= EW) return;  // (no barrier follows)

  // epilogue: wave e finishes output channels 4e .. 4e+3
  const int c0 = wave * (CT / EW);
  const long ob = (long)n * CT * P;
  float res[CT / EW];
  const bool hres = TAIL && a.residual;
  if (hres) {
    const brsrc_t rr = buf_rsrc(a.residual + ob, (long)CT * P * 4);
#pragma unroll
    for (int c = 0; c < CT / EW; ++c) res[c] = buf_ld1(rr, p4 + (unsigned)(c0 + c) * plane);
  }
  // DCN output: group 0's taps then group 1's, in tap order (the same sum in every wave) -> bias,
  // BN2, act
  auto dcn_out = [&](int co) {
    float s = 0.f;
#pragma unroll
    for (int gg = 0; gg < 2; ++gg)
#pragma unroll
      for (int h = 0; h < TS; ++h) s += sP[2 * h + gg][co][lane];
    const float bs = a.bias ? a.bias[co] : 0.f;
    const float sc = a.post_scale ? a.post_scale[co] : 1.f;
    const float sh = a.post_scale ? a.post_shift[co] : 0.f;
    return act_f((s + bs) * sc + sh, a.act);
  };
  const brsrc_t outr = buf_rsrc(a.out + ob, (long)CT * P * 4);
  if constexpr (!TAIL) {
#pragma unroll
    for (int c = 0; c < CT / EW; ++c) {
      const float y = dcn_out(c0 + c);
      if (pv) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), outr,
                                                    (int)(p4 + (unsigned)(c0 + c) * plane), 0, 0);
    }
    return;
  }
  float y[CT];
#pragma unroll
  for (int co = 0; co < CT; ++co) y[co] = dcn_out(co);
  // conv3 (1x1, BN3 folded; packed [co2][c]) + bias + identity + act
#pragma unroll
  for (int c = 0; c < CT / EW; ++c) {
    const int co2 = c0 + c;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < CT / 4; ++q) {
      const f32x4 tw = *reinterpret_cast<const f32x4 *>(&sT[co2][4 * q]);
#pragma unroll
      for (int u = 0; u < 4; ++u) t = __builtin_fmaf(tw[u], y[4 * q + u], t);
    }
    t += a.tail_b ? a.tail_b[co2] : 0.f;
    if (hres) t += res[c];
    t = act_f(t, a.tail_act);
    if (pv) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, t), outr,
                                                  (int)(p4 + (unsigned)co2 * plane), 0, 0);
  }
}

}  // namespace

int dcn_small_supported(int c, int co, int co2, int kh, int kw, int stride, int pad, int dil,
                        int dg, int groups) {
  return c == CT && co == CT && (co2 == 0 || co2 == CT) && kh == 3 && kw == 3 && stride == 1 &&
         pad == dil && dil >= 1 && dg == 2 && groups == 1;
}

int dcn_small_launch(const DcnSmallArgs &a, hipStream_t stream) {
  const bool tail = a.tail_w != nullptr;
  if (!dcn_small_supported(a.C, a.Co, tail ? a.Co2 : 0, 3, 3, 1, a.pad, a.dil, a.dg, 1))
    return AANET_EUNSUPPORTED;
  if (!a.x || !a.offset || !a.mask || !a.w || !a.out) return AANET_EINVAL;
  if (a.post_scale && !a.post_shift) return AANET_EINVAL;
  if (!tail && (a.residual || a.tail_b)) return AANET_EINVAL;
  const long P = (long)a.H * a.W;
  if (a.N <= 0 || P <= 0) return AANET_OK;
  // 32-bit buffer offsets over one image's planes (x / out 16 planes, offsets 36, mask 18)
  if ((long)2 * 2 * K * P * 4 >= (1L << 31) || a.N > 65535) return AANET_EUNSUPPORTED;
  const dim3 grid((unsigned)host_div_up(P, 64), (unsigned)a.N);
  if (tail && !a.packed) return AANET_EINVAL;
  if (tail)
    hipLaunchKernelGGL((dcn_small_kernel<true, true>), grid, dim3(NT), 0, stream, a);
  else if (a.packed)
    hipLaunchKernelGGL((dcn_small_kernel<false, true>), grid, dim3(NT), 0, stream, a);
  else
    hipLaunchKernelGGL((dcn_small_kernel<false, false>), grid, dim3(NT), 0, stream, a);
  return aanet_launch_status();
}
