// pointwise.hip -- the 1x1 convolutions of the ISA/CSA blocks (nets/deform.py:6-14 conv1x1 +
// BN folded, nets/aggregation.py:354-360 exchange terms, :447 final_conv) as a streaming
// split-bf16 GEMM for gfx950: out[px][co] = act(post_scale*(sum_c W[co][c] x[c][px] + bias)
// + post_shift + residual).
//
// The generic engine (mdcn.hip conv_fwd_kernel) stages a 128-pixel tile through LDS, one K chunk
// at a time, and has a single chunk of loads in flight: a 1x1 conv has only C/32 chunks, so each
// workgroup's life is load latency -> LDS -> MFMA -> epilogue, and the C2 scale-0 conv1 ran at
// 0.43 of HBM.  Here there is no LDS and no barrier:
//   - a wave streams 16-pixel blocks; lane (jj, kr) loads channels 8kr..8kr+7 of pixel jj of
//     every 32-channel chunk, which is exactly its B fragment of v_mfma_f32_16x16x32_bf16
//     (channels-last input: two 16-byte loads per chunk, 4 lanes = one 128-byte line);
//   - the next block's loads are issued before the current block's MFMAs (ping-pong registers);
//   - the weight fragments (pre-split, L2-resident) stay in registers for the whole kernel;
//   - D holds channels 4kr..4kr+3 of pixel jj: one 16-byte store per lane for channels-last
//     output, 64-byte row segments for NCHW.
// Waves pair up when Co > 32 (each owns 32 output channels of the same pixel block).
#include "pointwise.h"

#include <stdlib.h>

#include "split.h"

#ifndef AANET_PW_GCAP
#define AANET_PW_GCAP 1024  // workgroups per co tile of the Co > 64 streaming form
#endif

namespace {

__device__ __forceinline__ float pw_act(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);  // selects, no scalar branches
  return v > 0.f ? v : neg;
}

// Epilogue of one 16-pixel column block: lane holds channels c0..c0+3 (c0 = 16 blk + 4kr) of
// flattened pixel t.
// (n, p): image and pixel of t for the NCHW output (callers derive them without a division).
template <int NB, int ONH>
__device__ __forceinline__ void pw_store(const PwArgs &a, const f32x4 (&acc)[NB],
                                         const float (&eb)[NB][4], int t, int half, int kr, int n,
                                         int p, int co_base = 0, bool pre = false,
                                         f32x4 rpre = f32x4{0.f, 0.f, 0.f, 0.f}) {
  const int T = a.N * a.P, P = a.P, Co = a.Co;
  if (t >= T) return;
#pragma unroll
  for (int m = 0; m < NB; ++m) {
    const int c0 = co_base + 16 * (NB * half + m) + 4 * kr;
    if (c0 >= Co) continue;
    f32x4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = acc[m][r] + eb[m][r];
      if (a.post_scale) {
        const int co = min(c0 + r, Co - 1);
        s = s * a.post_scale[co] + a.post_shift[co];
      }
      y[r] = s;
    }
    if constexpr (ONH) {  // Co % 4 == 0 (pw_conv_supported)
      const long o = (long)t * Co + c0;
      if (a.residual) y += *reinterpret_cast<const f32x4 *>(a.residual + o);
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = pw_act(y[r], a.act);
      *reinterpret_cast<f32x4 *>(a.out + o) = y;
    } else {
      // every residual load before the first store: out may alias residual for the compiler, so
      // a load issued after a store waited for it -- one memory round trip per channel (the
      // bottleneck conv3 with its identity ran 3.4x the time of the plain conv)
      float rv[4] = {0.f, 0.f, 0.f, 0.f};
      if (pre) {  // NB == 1: the caller's prefetched identity values
#pragma unroll
        for (int r = 0; r < 4; ++r) rv[r] = rpre[r];
      } else if (a.residual) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c0 + r < Co) rv[r] = a.residual[((long)n * Co + c0 + r) * P + p];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (c0 + r >= Co) break;
        const long o = ((long)n * Co + c0 + r) * P + p;
        a.out[o] = pw_act(a.residual ? y[r] + rv[r] : y[r], a.act);
      }
    }
  }
}

// Channels-last input.  CI input channels (32 or 64); NB 16-channel output blocks per wave;
// NCOH waves per pixel block.
template <int CI, int NB, int NCOH, int ONH>
__global__ __launch_bounds__(256) void pw_conv_kernel(PwArgs a) {
  constexpr int NCC = CI / 32;
  constexpr int GPW = 4 / NCOH;  // pixel-block streams per workgroup
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int jj = lane & 15, kr = lane >> 4;
  const int half = wave % NCOH;
  const int T = a.N * a.P, Co = a.Co;
  const int nblk = (T + 15) >> 4;
  const int G = gridDim.x * GPW, gid = blockIdx.x * GPW + wave / NCOH;
  const int per = (nblk + G - 1) / G;
  const int b0 = gid * per, b1 = min(nblk, b0 + per);
  if (b0 >= b1) return;  // wave-uniform: the kernel has no barrier

  const bf16x8 *fr = static_cast<const bf16x8 *>(a.wsplit);
  bf16x8 A[NCC][NB][3];
#pragma unroll
  for (int cc = 0; cc < NCC; ++cc)
#pragma unroll
    for (int m = 0; m < NB; ++m)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) A[cc][m][pc] = fr[((cc * 4 + NB * half + m) * 3 + pc) * 64 + lane];
  float eb[NB][4];
#pragma unroll
  for (int m = 0; m < NB; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = 16 * (NB * half + m) + 4 * kr + r;
      eb[m][r] = (a.bias && co < Co) ? a.bias[co] : 0.f;
    }

  auto load = [&](int b, float (&v)[NCC][8]) {
    const int t = b * 16 + jj;
    const bool ok = t < T;
    const float *src = a.x + (long)(ok ? t : 0) * CI + 8 * kr;
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) {
      const f32x4 lo = ok ? *reinterpret_cast<const f32x4 *>(src + 32 * cc) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 hi = ok ? *reinterpret_cast<const f32x4 *>(src + 32 * cc + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[cc][u] = lo[u];
        v[cc][4 + u] = hi[u];
      }
    }
  };

  auto compute_store = [&](int b, const float (&v)[NCC][8]) {
    f32x4 acc[NB];
#pragma unroll
    for (int m = 0; m < NB; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < NCC; ++cc) {
      bf16x8 B[3];
      split8(v[cc], B);
#pragma unroll
      for (int m = 0; m < NB; ++m) acc[m] = mfma_split6(A[cc][m], B, acc[m]);
    }
    const int t = b * 16 + jj, n = ONH ? 0 : t / a.P;
    pw_store<NB, ONH>(a, acc, eb, t, half, kr, n, t - n * a.P);
  };

  float va[NCC][8], vb[NCC][8];
  load(b0, va);
  for (int b = b0; b < b1; b += 2) {
    if (b + 1 < b1) load(b + 1, vb);
    compute_store(b, va);
    if (b + 1 >= b1) break;
    if (b + 2 < b1) load(b + 2, va);
    compute_store(b + 1, vb);
  }
}

// NCHW input: a lane's B fragment would be 8 loads 4*P bytes apart, each wave instruction
// moving 64-byte row pieces.  Instead the workgroup loads a block of SW*SUB pixels as whole
// 128-byte channel rows (16-byte loads), stages it in LDS as [ch][px] (double-buffered, one
// barrier per block), and each wave reads its B fragments from there: wave w computes output
// channel block w % CB (16 channels) of pixel sub-block w / CB (SW pixels), CB * SUB = 4.  The
// next block's row loads are in flight during the current block's MFMAs.
template <int CI, int CB, int ONH>
__global__ __launch_bounds__(256) void pw_conv_nchw_kernel(PwArgs a) {
  constexpr int NCC = CI / 32;
  constexpr int SUB = 4 / CB;               // pixel sub-blocks per workgroup block
  constexpr int SW = CB == 4 ? 64 : 32;     // pixels per sub-block (16-pixel MFMA column groups)
  constexpr int BP = SW * SUB;              // pixels per block
  // LDS row pitch (floats): 8 * PXP = 16 (mod 32), so the two lane groups kr, kr+1 of a 32-lane
  // half read banks 16 apart (conflict-free fragment reads); rows are 8-byte aligned
  constexpr int PXP = BP + 2;
  constexpr int QPR = BP / 4;               // 16-byte pieces per channel row
  constexpr int LV = CI * QPR / 256;        // pieces per thread per block
  static_assert(LV >= 1 && 256 % QPR == 0, "block shape");
  __shared__ __attribute__((aligned(16))) float sX[2][CI * PXP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jj = lane & 15, kr = lane >> 4;
  const int cb = wave % CB, sub = wave / CB;
  const int T = a.N * a.P, P = a.P, Co = a.Co;
  const int nblk = (T + BP - 1) / BP;
  const int per = (nblk + gridDim.x - 1) / gridDim.x;
  const int b0 = blockIdx.x * per, b1 = min(nblk, b0 + per);
  if (b0 >= b1) return;  // workgroup-uniform

  const bf16x8 *fr = static_cast<const bf16x8 *>(a.wsplit);
  bf16x8 A[NCC][3];
#pragma unroll
  for (int cc = 0; cc < NCC; ++cc)
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) A[cc][pc] = fr[((cc * 4 + cb) * 3 + pc) * 64 + lane];
  float eb[1][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = 16 * cb + 4 * kr + r;
    eb[0][r] = (a.bias && co < Co) ? a.bias[co] : 0.f;
  }

  const int lrow = tid / QPR, lq = tid % QPR;  // piece i: channel lrow + i*(256/QPR), px 4lq..
  constexpr int RSTEP = 256 / QPR;
  f32x4 rv[LV];
  auto load = [&](int b) {
    const int t0 = b * BP, n = t0 / P, p0 = t0 - n * P;
    if ((P & 3) == 0 && p0 + BP <= P) {  // workgroup-uniform: the block lies in one image
      const float *src = a.x + ((long)n * CI + lrow) * P + p0 + 4 * lq;
#pragma unroll
      for (int i = 0; i < LV; ++i) rv[i] = *reinterpret_cast<const f32x4 *>(src + (long)(RSTEP * i) * P);
    } else {
#pragma unroll
      for (int i = 0; i < LV; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int t = t0 + 4 * lq + u;
          const int nn = t < T ? t / P : 0, pp = t < T ? t - nn * P : 0;
          rv[i][u] = t < T ? a.x[((long)nn * CI + RSTEP * i + lrow) * P + pp] : 0.f;
        }
    }
  };
  auto stage = [&](int buf) {
    typedef float f32x2_t __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < LV; ++i) {
      float *d = &sX[buf][(RSTEP * i + lrow) * PXP + 4 * lq];
      *reinterpret_cast<f32x2_t *>(d) = f32x2_t{rv[i][0], rv[i][1]};
      *reinterpret_cast<f32x2_t *>(d + 2) = f32x2_t{rv[i][2], rv[i][3]};
    }
  };

  load(b0);
  stage(0);
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const int buf = (b - b0) & 1;
    if (b + 1 < b1) load(b + 1);
    const float *xs = sX[buf];
    const int n0b = __builtin_amdgcn_readfirstlane((b * BP) / P), p0b = b * BP - n0b * P;
#pragma unroll
    for (int g = 0; g < SW / 16; ++g) {
      f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = xs[(32 * cc + 8 * kr + u) * PXP + SW * sub + 16 * g + jj];
        bf16x8 B[3];
        split8(v, B);
        acc[0] = mfma_split6(A[cc], B, acc[0]);
      }
      // the block's first pixel is (n0, p0) (one scalar division per block); a block spans at
      // most 1 + BP / P images, so the carry below runs at most once when P >= BP
      const int off = SW * sub + 16 * g + jj;
      int nn = n0b, pp = p0b + off;
      while (pp >= P) {
        pp -= P;
        ++nn;
      }
      pw_store<1, ONH>(a, acc, eb, b * BP + off, cb, kr, nn, pp);
    }
    if (b + 1 < b1) {
      stage(buf ^ 1);
      __syncthreads();
    }
  }
}

// NCHW input, split once (CB = 2 or 4: 64-pixel blocks).  pw_conv_nchw_kernel splits every
// staged value in each of the CB * SUB = 4 waves that read it (3,494 VALU per wave at C2 conv1,
// 4x the needed split work).  Here the staging thread splits its values once and stores the three
// bf16 pieces as [piece][pixel][channel] planes (CI * 2-byte pixel rows) with the 16-byte chunks
// XOR-swizzled per pixel (swz below): the staging writes (8 lanes = 8 pixels of one chunk) and
// the fragment reads (16 lanes = 16 pixels, lane groups kr and kr + 1) are both conflict-free.  A lane's B fragment is then three ds_read_b128.  Staging: thread = (pixel
// t % 64, 8-channel groups (t / 64) + 4i), eight dword loads per group (lanes = consecutive
// pixels: 256-byte wave loads), next block's loads in flight during the current block's MFMAs.
// Measured at C2 scale 0 (64 -> 64, same call): 43.8-44.2 vs 40.3-41.3 us alone (48 KB of LDS:
// three workgroups per CU instead of four, 4x the load instructions), but the bench step
// 3.369-3.387 vs 3.385-3.407 ms -- its VALU no longer competes with the concurrent kernels.
template <int CI, int CB, int ONH>
__global__ __launch_bounds__(256) void pw_conv_nchw_s_kernel(PwArgs a) {
  constexpr int NCC = CI / 32;
  constexpr int BP = 64;                    // pixels per block
  constexpr int SUB = 4 / CB, SW = BP / SUB;  // pixel sub-blocks per block, pixels per sub-block
  constexpr int NQ = CI / 8;                // 16-byte chunks (8 channels) per pixel row
  constexpr int GPT = NQ / 4;               // 8-channel groups per staging thread
  constexpr int PL = BP * CI;               // bf16 per piece plane
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][3 * PL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int jj = lane & 15, kr = lane >> 4;
  const int cb = wave % CB, sub = wave / CB;
  const int T = a.N * a.P, P = a.P, Co = a.Co;
  const int nblk = (T + BP - 1) / BP;
  const int per = (nblk + gridDim.x - 1) / gridDim.x;
  const int b0 = blockIdx.x * per, b1 = min(nblk, b0 + per);
  if (b0 >= b1) return;  // workgroup-uniform

  // output channels [64 t, 64 t + 64) (Co > 64: one co tile per grid row, the input re-staged
  // per tile); the split weight fragments of tile t follow tile t - 1's
  const int cot = blockIdx.y, co_base = 64 * cot;
  const bf16x8 *fr = static_cast<const bf16x8 *>(a.wsplit) + (long)cot * NCC * 4 * 3 * 64;
  bf16x8 A[NCC][3];
#pragma unroll
  for (int cc = 0; cc < NCC; ++cc)
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) A[cc][pc] = fr[((cc * 4 + cb) * 3 + pc) * 64 + lane];
  float eb[1][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co_base + 16 * cb + 4 * kr + r;
    eb[0][r] = (a.bias && co < Co) ? a.bias[co] : 0.f;
  }

  const int spx = tid & 63, sg = tid >> 6;  // staging: pixel, first 8-channel group
  float rv[GPT][8];
  auto load = [&](int b) {
    const int t = b * BP + spx;
    const bool ok = t < T;
    const int n = ok ? t / P : 0, p = ok ? t - n * P : 0;
    const float *src = a.x + (long)n * CI * P + p;
#pragma unroll
    for (int i = 0; i < GPT; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u) rv[i][u] = ok ? src[(long)(8 * (sg + 4 * i) + u) * P] : 0.f;
  };
  // CI = 64: chunk q ^ (px & 7); CI = 32 (64-byte rows): q ^ ((px + (px >> 1)) & 3) -- both
  // conflict-free for the staging writes and the fragment reads (checked per lane group)
  auto swz = [](int px, int q) {
    const int x = CI == 64 ? (px & 7) : (((px & 3) + ((px >> 1) & 3)) & 3);
    return px * CI + ((q ^ x) << 3);
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      bf16x8 pcs[3];
      split8(rv[i], pcs);
      const int o = swz(spx, sg + 4 * i);
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) *reinterpret_cast<bf16x8 *>(&sB[buf][pc * PL + o]) = pcs[pc];
    }
  };

  load(b0);
  stage(0);
  __syncthreads();
  for (int b = b0; b < b1; ++b) {
    const int buf = (b - b0) & 1;
    if (b + 1 < b1) load(b + 1);
    const __bf16 *xs = sB[buf];
    const int n0b = __builtin_amdgcn_readfirstlane((b * BP) / P), p0b = b * BP - n0b * P;
    // the block's identity values (NCHW out) load before its MFMAs: issued per 16-pixel group at
    // its store, each group waited a full memory round trip (32 -> 128 with identity 138 us vs
    // 58 without)
    f32x4 rpf[SW / 16];
    if (!ONH && a.residual) {
#pragma unroll
      for (int g = 0; g < SW / 16; ++g) {
        const int off = SW * sub + 16 * g + jj, t = b * BP + off;
        int nn = n0b, pp = p0b + off;
        while (pp >= P) {
          pp -= P;
          ++nn;
        }
        const int c0 = co_base + 16 * cb + 4 * kr;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rpf[g][r] = (t < T && c0 + r < Co) ? a.residual[((long)nn * Co + c0 + r) * P + pp] : 0.f;
      }
    }
#pragma unroll
    for (int g = 0; g < SW / 16; ++g) {
      const int px = SW * sub + 16 * g + jj;
      f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int cc = 0; cc < NCC; ++cc) {
        bf16x8 B[3];
        const int o = swz(px, 4 * cc + kr);
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) B[pc] = *reinterpret_cast<const bf16x8 *>(&xs[pc * PL + o]);
        acc[0] = mfma_split6(A[cc], B, acc[0]);
      }
      const int off = SW * sub + 16 * g + jj;
      int nn = n0b, pp = p0b + off;
      while (pp >= P) {
        pp -= P;
        ++nn;
      }
      pw_store<1, ONH>(a, acc, eb, b * BP + off, cb, kr, nn, pp, co_base, !ONH && a.residual,
                       (!ONH && a.residual) ? rpf[g] : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    if (b + 1 < b1) {
      stage(buf ^ 1);
      __syncthreads();
    }
  }
}

template <int CI, int NB, int NCOH>
void launch_nb(const PwArgs &a, dim3 grid, hipStream_t st) {
  const dim3 blk(256);
  if (a.in_nhwc) {
    if (a.out_nhwc)
      hipLaunchKernelGGL((pw_conv_kernel<CI, NB, NCOH, 1>), grid, blk, 0, st, a);
    else
      hipLaunchKernelGGL((pw_conv_kernel<CI, NB, NCOH, 0>), grid, blk, 0, st, a);
  } else {
    constexpr int CB = NB * NCOH;  // 16-channel output blocks: 1, 2 or 4
    const long bp = CB == 4 ? 64 : 128 / CB;  // pixels per block (pw_conv_nchw_kernel BP)
    const long nblk = ((long)a.N * a.P + bp - 1) / bp;
    long g = (nblk + 3) / 4;  // about 4 blocks per workgroup at least
    if (g > 1024) g = 1024;
    if (CB >= 2) {
      if (a.out_nhwc)
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<CI, CB, 1>), dim3((unsigned)g), blk, 0, st, a);
      else
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<CI, CB, 0>), dim3((unsigned)g), blk, 0, st, a);
    } else if (a.out_nhwc)
      hipLaunchKernelGGL((pw_conv_nchw_kernel<CI, CB, 1>), dim3((unsigned)g), blk, 0, st, a);
    else
      hipLaunchKernelGGL((pw_conv_nchw_kernel<CI, CB, 0>), dim3((unsigned)g), blk, 0, st, a);
  }
}

template <int CI>
void launch_ci(const PwArgs &a, hipStream_t st) {
  const long T = (long)a.N * a.P, nblk = (T + 15) / 16;
  const int ncoh = a.Co > 32 ? 2 : 1, gpw = 4 / ncoh;
  // about 4 blocks per stream at least, and one resident round of workgroups at most (the
  // 64-channel, two-block form holds ~150 VGPRs: 3 waves per SIMD)
  long grid = (nblk + 4 * gpw - 1) / (4 * gpw);
  const long cap = CI == 64 && a.Co > 16 ? 768 : 1024;
  if (grid > cap) grid = cap;
  const dim3 g((unsigned)grid);
  if (a.Co <= 16)
    launch_nb<CI, 1, 1>(a, g, st);
  else if (a.Co <= 32)
    launch_nb<CI, 2, 1>(a, g, st);
  else
    launch_nb<CI, 2, 2>(a, g, st);
}

}  // namespace

int pw_conv_supported(int c, int co, int kh, int kw, int stride, int pad, int groups, long np,
                      int out_nhwc, int p) {
  return kh == 1 && kw == 1 && stride == 1 && pad == 0 && groups == 1 && (c == 32 || c == 64) &&
         co >= 1 && (co <= 64 || (co <= 512 && co % 64 == 0)) && np + 16 < 0x7fffffffL &&
         (!out_nhwc || co % 4 == 0) && p >= 1;
}

int pw_conv_launch(const PwArgs &a, hipStream_t st) {
  if (!a.x || !a.wsplit || !a.out || (a.post_scale && !a.post_shift)) return AANET_EINVAL;
  if (!pw_conv_supported(a.C, a.Co, 1, 1, 1, 0, 1, (long)a.N * a.P, a.out_nhwc, a.P))
    return AANET_EUNSUPPORTED;
  if (a.Co > 64) {
    // Co = 128 .. 512 (the feature extractors' expansions): 64-channel tiles over grid rows, NCHW
    // input only (the channels-last kernel keeps its weights for all of Co in registers)
    if (a.in_nhwc) return AANET_EUNSUPPORTED;
    const long nblk = ((long)a.N * a.P + 63) / 64;
    long g = (nblk + 3) / 4;
    if (g > AANET_PW_GCAP) g = AANET_PW_GCAP;
    const dim3 grid((unsigned)g, (unsigned)(a.Co / 64)), blk(256);
    if (a.C == 32) {
      if (a.out_nhwc)
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<32, 4, 1>), grid, blk, 0, st, a);
      else
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<32, 4, 0>), grid, blk, 0, st, a);
    } else {
      if (a.out_nhwc)
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<64, 4, 1>), grid, blk, 0, st, a);
      else
        hipLaunchKernelGGL((pw_conv_nchw_s_kernel<64, 4, 0>), grid, blk, 0, st, a);
    }
    return aanet_launch_status();
  }
  if (a.C == 32)
    launch_ci<32>(a, st);
  else
    launch_ci<64>(a, st);
  return aanet_launch_status();
}
