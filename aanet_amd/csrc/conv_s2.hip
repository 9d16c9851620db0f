// conv_s2.hip -- the down exchange terms of the cross-scale aggregation (nets/aggregation.py:
// 362-371: 3x3 stride-2 pad-1 convs + BN [+ LeakyReLU] from a finer scale to a coarser one) for
// gfx950, with the first conv of EVERY down chain that starts at the same input fused into one
// launch: at C2 scale 0 the 64->32 (branch 1) and 64->64 (first half of branch 2) convs of the
// scale-0 block output become one 64->96 contraction that reads the 109 MB input once.
//
// Why not the conv engine.  The engine's stride-2 forms (im2col, or the opt-in 9x33 halo tile)
// stage the NCHW input through LDS once per output-channel tile and run one 64-pixel tile per
// workgroup: 84 + 67 us for the two convs alone (0.22 of the split-bf16 ceiling), 155 us when
// they run side by side, and the step spent 0.7 ms in them.  This kernel: 82 us
// for the merged 64 -> 96 launch (0.34); the narrow 64/32 -> 16 convs run as fast as on the
// engine (20 / 12 us).  A barrier-free variant for the narrow convs (per-wave A loads, three
// steps in flight) measured the same, alone and in the step, and was dropped.
//
// Work split.  A workgroup owns an 8 x 16 tile of OUTPUT pixels and every output channel (up to
// 96): wave w = tile row w, lane (kr = lane / 16, jj = lane % 16) = output pixel jj, channels
// 8kr..8kr+7 of the 32-channel chunk.  That is exactly the lane's B fragment of
// v_mfma_f32_16x16x32_bf16, so the im2col is loaded straight into registers: per (chunk, tap),
// eight dword loads at input (2y+ti-1, 2x+tj-1) of channels 8kr..8kr+7 (16 lanes of a channel
// cover 128 contiguous bytes, half of them this tap's; the other taps of the row hit the same
// lines in L1/L2), split into three bf16 pieces and contracted against the pre-split weights.
// The weights of one (chunk, tap) -- NCB blocks x 3 pieces x 1 KB -- arrive by LDS-DMA one step
// ahead into two separate __shared__ buffers (see dcn_tile.hip for why two objects), together
// with the next step's input loads, so each step waits only on loads issued one step earlier.
// The epilogue adds the folded-BN bias, applies each output's activation and stores 64-byte row
// segments straight from the accumulators (channel 16m + 4kr + r, pixel jj).
//
// Numerics: the split-bf16 contraction of the conv engine (split.h: truncation split, six piece
// products, fp32 accumulation), taps and chunks in ascending order.
#include <hip/hip_runtime.h>

#include "common.h"
#include "split.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int NT = 512;         // 8 waves, one output row each
constexpr int TR = 8, TC = 16;  // output tile

struct S2Args {
  const float *x;      // [N][C][H][W]
  const char *wsplit;  // [C/32][9][NCB][3][64 lanes][16 B]
  const float *bias;   // [Co] or NULL
  float *out[2];
  int co_a, act[2];
  int N, C, H, W, Ho, Wo, Co;
};

__device__ __forceinline__ float s2_act(float v, int act) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : 0.2f * v;
  return v;
}

template <int NCB>
__global__ __launch_bounds__(NT, 4) void conv3x3s2_kernel(S2Args a) {
  constexpr int AB = NCB * 3 * 1024;  // A fragments of one (chunk, tap) step
  __shared__ __attribute__((aligned(16))) char sA0[AB];
  __shared__ __attribute__((aligned(16))) char sA1[AB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kr = lane >> 4, jj = lane & 15;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int tx = (Wo + TC - 1) / TC, ntiles = tx * ((Ho + TR - 1) / TR);
  // XCD-aware bijective remap: each XCD walks a contiguous range of tiles (shared input rows)
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile = bid % ntiles;
  const int y = (tile / tx) * TR + wave, x = (tile % tx) * TC + jj;
  const bool pv = y < Ho && x < Wo;
  const int HW = H * W;
  const int img_bytes = a.C * HW * 4;  // < 2^31 (launcher)
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void *)(a.x + (long)n * a.C * HW), (short)0,
                                                     img_bytes, 0x00020000);
  // lane base: channel 8kr of the chunk, input row 2y-1, column 2x-1 (tap (ti, tj) adds ti*W+tj)
  const int yy0 = 2 * y - 1, xx0 = 2 * x - 1;
  const int lbase = (8 * kr * HW + yy0 * W + xx0) * 4;
  bool rok[3], cok[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    rok[t] = pv && (unsigned)(yy0 + t) < (unsigned)H;
    cok[t] = (unsigned)(xx0 + t) < (unsigned)W;
  }
  const int nsteps = (a.C / 32) * 9;

  // the eight channel values of this lane's B fragment at step s = (chunk s/9, tap s%9);
  // out of the image: the out-of-range offset, whose buffer load returns 0 (zero padding)
  auto load_b = [&](int s, float (&v)[8]) {
    const int cc = s / 9, k = s - 9 * (s / 9), ti = k / 3, tj = k - 3 * (k / 3);
    const bool ok = rok[ti] && cok[tj];
    const int off = ok ? lbase + (ti * W + tj) * 4 : img_bytes;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
          xr, off, __builtin_amdgcn_readfirstlane((32 * cc + u) * HW * 4), 0));
  };
  auto issue_a = [&](int s, char *dst) {
    const char *src = a.wsplit + (long)s * AB + lane * 16;
    for (int pc = wave; pc < 3 * NCB; pc += 8)
      __builtin_amdgcn_global_load_lds((const void *)(src + pc * 1024), (lds_void *)(dst + pc * 1024), 16, 0, 0);
  };

  f32x4 acc[NCB];
#pragma unroll
  for (int m = 0; m < NCB; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto step = [&](int s, const char *cur, char *nxt, const float (&vc)[8], float (&vn)[8]) {
    if (s + 1 < nsteps) {  // next step's weights and input, behind this step's MFMAs
      issue_a(s + 1, nxt);
      load_b(s + 1, vn);
    }
    bf16x8 B[3];
    split8(vc, B);
    const char *ab = cur + lane * 16;
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
      bf16x8 A[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) A[pc] = *reinterpret_cast<const bf16x8 *>(ab + (m * 3 + pc) * 1024);
      acc[m] = mfma_split6(A, B, acc[m]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's loads of step s+1 landed ...
    __syncthreads();                                   // ... and every other wave's DMA
  };

  float v0[8], v1[8];
  issue_a(0, sA0);
  load_b(0, v0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll 1
  for (int s = 0; s < nsteps; s += 2) {
    step(s, sA0, sA1, v0, v1);
    if (s + 1 < nsteps) step(s + 1, sA1, sA0, v1, v0);
  }

  // epilogue: channel co = 16m + 4kr + r of pixel (y, x); rows of 16 pixels = 64-byte segments
  if (!pv) return;
  const long P = (long)Ho * Wo, pix = (long)y * Wo + x;
  const int cb = a.Co - a.co_a;
#pragma unroll
  for (int m = 0; m < NCB; ++m) {
    const int c4 = 16 * m + 4 * kr;
    const f32x4 bs = a.bias ? *reinterpret_cast<const f32x4 *>(a.bias + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = c4 + r;
      const float v = acc[m][r] + bs[r];
      if (co < a.co_a)
        a.out[0][((long)n * a.co_a + co) * P + pix] = s2_act(v, a.act[0]);
      else
        a.out[1][((long)n * cb + co - a.co_a) * P + pix] = s2_act(v, a.act[1]);
    }
  }
}

// w [Co][C][3][3] fp32 -> [C/32][9][Co/16][3][64 lanes][8 bf16]: lane l of block m holds row
// co = 16m + l%16, channels 32cc + 8(l/16) + 0..7 (the A fragment of v_mfma_f32_16x16x32_bf16),
// as three exact bf16 pieces (split8)
__global__ void conv3x3s2_pack_kernel(const float *__restrict__ w, bf16x8 *__restrict__ out, int Co,
                                      int C) {
  const int ncb = Co / 16, total = (C / 32) * 9 * ncb * 64;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int l = e % 64, m = (e / 64) % ncb, k = (e / 64 / ncb) % 9, cc = e / 64 / ncb / 9;
    const int co = 16 * m + (l & 15), c0 = 32 * cc + 8 * (l >> 4);
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = w[((long)co * C + c0 + u) * 9 + k];
    bf16x8 b[3];
    split8(v, b);
    const long base = (((long)(cc * 9 + k) * ncb + m) * 3) * 64 + l;
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) out[base + pc * 64] = b[pc];
  }
}

}  // namespace

extern "C" {

size_t aanet_conv3x3s2_pack_bytes(int co, int c) {
  if (co <= 0 || co % 16 || c <= 0 || c % 32) return 0;
  return (size_t)(c / 32) * 9 * (co / 16) * 3 * 1024;
}

int aanet_conv3x3s2_pack_f32(const float *w, int co, int c, void *wsplit, aanet_stream_t stream) {
  if (!w || !wsplit || !aanet_conv3x3s2_pack_bytes(co, c)) return AANET_EINVAL;
  const int total = (c / 32) * 9 * (co / 16) * 64;
  hipLaunchKernelGGL(conv3x3s2_pack_kernel, dim3(host_div_up(total, 256)), dim3(256), 0, as_hip(stream),
                     w, reinterpret_cast<bf16x8 *>(wsplit), co, c);
  return aanet_launch_status();
}

int aanet_conv3x3s2_f32(const float *x, const void *wsplit, const float *bias, int n, int c, int h,
                        int w, int co, int co_a, float *out_a, int act_a, float *out_b, int act_b,
                        aanet_stream_t stream) {
  if (!x || !wsplit || n < 0 || h < 0 || w < 0 || co_a < 0 || co_a > co) return AANET_EINVAL;
  if (co <= 0 || co % 16 || c <= 0 || c % 32) return AANET_EUNSUPPORTED;
  if ((co_a > 0 && !out_a) || (co_a < co && !out_b)) return AANET_EINVAL;
  if ((long)c * h * w * 4 >= (1L << 31)) return AANET_EUNSUPPORTED;
  if (n == 0 || h == 0 || w == 0) return AANET_OK;
  S2Args a;
  a.x = x;
  a.wsplit = reinterpret_cast<const char *>(wsplit);
  a.bias = bias;
  a.out[0] = out_a;
  a.out[1] = out_b;
  a.co_a = co_a;
  a.act[0] = act_a;
  a.act[1] = act_b;
  a.N = n, a.C = c, a.H = h, a.W = w, a.Co = co;
  a.Ho = (h + 1) / 2;
  a.Wo = (w + 1) / 2;
  const long tiles = (long)host_div_up(a.Wo, TC) * host_div_up(a.Ho, TR) * n;
  if (tiles > 0x7fffffffL) return AANET_EUNSUPPORTED;
  const dim3 grid((unsigned)tiles), blk(NT);
  hipStream_t st = as_hip(stream);
  switch (co / 16) {
    case 1: hipLaunchKernelGGL(conv3x3s2_kernel<1>, grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL(conv3x3s2_kernel<2>, grid, blk, 0, st, a); break;
    case 3: hipLaunchKernelGGL(conv3x3s2_kernel<3>, grid, blk, 0, st, a); break;
    case 4: hipLaunchKernelGGL(conv3x3s2_kernel<4>, grid, blk, 0, st, a); break;
    case 5: hipLaunchKernelGGL(conv3x3s2_kernel<5>, grid, blk, 0, st, a); break;
    case 6: hipLaunchKernelGGL(conv3x3s2_kernel<6>, grid, blk, 0, st, a); break;
    default: return AANET_EUNSUPPORTED;
  }
  return aanet_launch_status();
}

}  // extern "C"
