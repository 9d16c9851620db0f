// dcn_win.hip -- the LDS-window deformable tail (DcnTileArgs, dcn_tile.h) in a software-pipelined
// form: nets/deform.py:207-236 (DeformConv2d + BN2 + ReLU -> conv3 1x1 + BN3 + identity + ReLU)
// with the scale-0 cross-scale sum of nets/aggregation.py:387-400, or the plain op-level DCN
// (deform_conv_cuda.cpp:490-569).
//
// dcn_tile.hip runs one tile row per wave, eight waves per workgroup and four waves per SIMD at
// 128 VGPRs.  Each chunk (one tap of a 32-channel deformable group) is one dependent chain per
// wave -- sampling-state hand-off, window corner reads, bilinear blend, bf16 split, 24 MFMAs --
// closed by a barrier, so a wave's vector work and its matrix work never overlap; only the other
// waves of the SIMD can fill the matrix pipe, and the two waves of one workgroup on a SIMD run in
// lockstep (steady chunk ~3.9k cycles against ~1.5k of matrix work per SIMD).
//
// Here a workgroup is four waves (one per SIMD) over the same 8 x 16 tile, each wave owning two
// tile rows, and two workgroups share a CU (72 KB of LDS each), so every SIMD holds two waves of
// DIFFERENT workgroups (no barrier couples them) with up to 256 VGPRs each.  The chunk loop is
// software-pipelined inside each wave: while the MFMAs of chunk c run on B(c), the wave reads the
// window corners of chunk c+1 and blends and splits them into B(c+1), in the same basic block, so
// the vector work issues in the MFMA gaps.  One A fragment read from LDS now feeds two rows.
// The window, the A-fragment LDS-DMA one tap ahead, the sampling state (4 taps per pass, handed
// over by ds_bpermute) and the numerics are those of dcn_tile.hip.
#include "dcn_tile.h"
#include "split.h"

#include <type_traits>
#include <utility>

namespace {

// f(std::integral_constant<int, I>) for I = 0 .. N-1, expanded in the AST (not a loop)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NT = 256;          // 4 waves, two tile rows each
constexpr int TR = 8, TC = 16;   // tile: 8 rows x 16 columns of output pixels
constexpr int RW = 2;            // window margin beyond the taps: offsets in [-RW, RW) stay inside
constexpr int K = 9;             // 3x3 taps
constexpr int DIL = 2;
constexpr int OP = TR * TC + 4;  // epilogue tile pitch (floats)

__device__ __forceinline__ float act_f(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);
  return v > 0.f ? v : neg;
}

struct TapState {
  int pos;
  float w0, w1, w2, w3;
};

// Sampling state of one (pixel, tap, deformable group): window position of the top-left corner
// (-1: a corner lies outside the window -> global gather) and the four mask-folded corner weights.
// Same float steps as dcn_tile.hip tap_state / mdcn.hip make_samp4 (kernel.cu:467-497).
template <int WR, int WC>
__device__ __forceinline__ TapState tap_state(float oh, float ow, float ml, int yy, int xx, bool pv,
                                              int t, int H, int W, int wy0, int wx0,
                                              int mask_logits, float mask_scale) {
#pragma clang fp contract(off)
  const int i = t / 3, j = t - 3 * (t / 3);
  float m = mask_logits ? mask_scale * __builtin_amdgcn_rcpf(1.f + __expf(-ml)) : ml;
  if (!pv) m = 0.f;
  const float h = (float)(yy - DIL + i * DIL) + oh;
  const float w = (float)(xx - DIL + j * DIL) + ow;
  const bool valid = h > -1.f && w > -1.f && h < (float)H && w < (float)W;
  const int hl = (int)floorf(h), wl = (int)floorf(w);
  const float lh = h - (float)hl, lw = w - (float)wl;
  const float hh = 1.f - lh, hw = 1.f - lw;
  TapState s;
  const bool ok1 = valid && hl >= 0 && wl >= 0;
  const bool ok2 = valid && hl >= 0 && wl + 1 <= W - 1;
  const bool ok3 = valid && hl + 1 <= H - 1 && wl >= 0;
  const bool ok4 = valid && hl + 1 <= H - 1 && wl + 1 <= W - 1;
  s.w0 = (ok1 ? hh * hw : 0.f) * m;
  s.w1 = (ok2 ? hh * lw : 0.f) * m;
  s.w2 = (ok3 ? lh * hw : 0.f) * m;
  s.w3 = (ok4 ? lh * lw : 0.f) * m;
  const int rh = hl - wy0, rw = wl - wx0;
  const bool inwin = (unsigned)rh <= (unsigned)(WR - 2) && (unsigned)rw <= (unsigned)(WC - 2);
  s.pos = !valid ? 0 : (inwin ? rh * WC + rw : -1);
  return s;
}

// CG = channels per deformable group (two groups): 32 (C = 64) or 16 (C = 32: both groups in one
// 32-channel K slice, lane groups kr = 0, 1 carry group 0's channels and kr = 2, 3 group 1's).
// XN: x is NCHW instead of channels-last.  PLAIN: out = act(post_scale * (DCN + bias) +
// post_shift), NCHW, no bottleneck tail.
template <int CG, bool XN, bool PLAIN>
__global__ __launch_bounds__(NT, 2) void dcn_win_kernel(DcnTileArgs a) {
  constexpr int CT = 2 * CG;             // channels = Co (= Co2)
  constexpr int NPH = CT / 32;           // 32-channel K slices ("phases")
  constexpr int NCH = NPH * K;           // chunks
  constexpr int NCO = CT / 16;           // 16-row co blocks
  constexpr int ABUF = NCO * 3 * 1024;   // one chunk's A fragments
  constexpr int TPP = CG == 32 ? 4 : 2;  // taps per sampling pass
  constexpr int MG = DIL + RW;
  constexpr int WR = TR + 2 * MG, WC = TC + 2 * MG;
  constexpr int NPOS = (WR * WC + 63) / 64 * 64;
  constexpr int WIN = 8 * NPOS * 16;     // [8 channel quads][NPOS][16 B]
  constexpr int NWI = 8 * NPOS / NT;     // 16-byte window pieces per thread
  static_assert(8 * NPOS % NT == 0 && NWI * NT * 16 == WIN, "window staging");
  static_assert(!XN || (WC % 4 == 0 && 32 * WR * (WC / 4) == NT * NWI), "NCHW window staging");
  static_assert(WIN >= CT * OP * 4, "epilogue tile must fit the window");
  // three LDS objects: a ds_read is ordered after an outstanding LDS-DMA only when they may alias
  __shared__ __attribute__((aligned(16))) char sWin[WIN];
  __shared__ __attribute__((aligned(16))) char sA0[ABUF];
  __shared__ __attribute__((aligned(16))) char sA1[ABUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kr = lane >> 4, jj = lane & 15;
  const int H = a.H, W = a.W, C = a.C;
  const int tx = (W + TC - 1) / TC, ntiles = tx * ((H + TR - 1) / TR);
  // XCD-aware bijective remap: each XCD walks a contiguous range of tiles (shared window rows)
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile = bid % ntiles;
  const int y0 = (tile / tx) * TR, x0 = (tile % tx) * TC;
  const int wy0 = y0 - MG, wx0 = x0 - MG;
  const int px = x0 + jj;
  const int P = H * W;
  int py[2], p4[2];
  bool pv[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    py[r] = y0 + 2 * wave + r;
    pv[r] = py[r] < H && px < W;
    p4[r] = (pv[r] ? py[r] * W + px : 0) * 4;
  }
  const int img_bytes = C * P * 4;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void *)(a.x + (long)n * C * P), (short)0, img_bytes, 0x00020000);
  const auto offr = __builtin_amdgcn_make_buffer_rsrc((void *)(a.offset + (long)n * a.off_bs), (short)0, 0x7ffffff0, 0x00020000);
  const auto mskr = __builtin_amdgcn_make_buffer_rsrc((void *)(a.mask + (long)n * a.mask_bs), (short)0, 0x7ffffff0, 0x00020000);

  // ---- window staging (as dcn_tile.hip): channels-last -- 8 consecutive lanes take one quad of
  // 8 consecutive positions; NCHW -- one 16-byte segment (4 columns) of one window row of one
  // channel per element, scattered to the 4 positions' slots.  Outside the image: zeros.
  f32x4 wv[NWI];
  auto load_window = [&](int g) {
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int e = tid + NT * i;
      if constexpr (XN) {
        const int seg = e % (WC / 4), rest = e / (WC / 4), row = rest % WR, ch = rest / WR;
        const int wy = wy0 + row, wx = wx0 + 4 * seg;
        const bool ok = wy >= 0 && wy < H && wx >= 0 && wx < W;
        const int off = ok ? (((g * 32 + ch) * H + wy) * W + wx) * 4 : img_bytes;
        wv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      } else {
        const int q = (e >> 3) & 7, pos = (e & 7) | ((e >> 6) << 3);
        const int wy = wy0 + pos / WC, wx = wx0 + pos % WC;
        const bool ok = pos < WR * WC && wy >= 0 && wy < H && wx >= 0 && wx < W;
        const int off = ok ? ((wy * W + wx) * C + 4 * q) * 4 : img_bytes;
        wv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, g * 128, 0));
      }
    }
  };
  auto store_window = [&]() {
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int e = tid + NT * i;
      if constexpr (XN) {
        const int seg = e % (WC / 4), rest = e / (WC / 4), row = rest % WR, ch = rest / WR;
        float *dst = reinterpret_cast<float *>(sWin + ((ch >> 2) * NPOS + row * WC + 4 * seg) * 16) + (ch & 3);
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[4 * u] = wv[i][u];
      } else {
        const int q = (e >> 3) & 7, pos = (e & 7) | ((e >> 6) << 3);
        *reinterpret_cast<f32x4 *>(sWin + (q * NPOS + pos) * 16) = wv[i];
      }
    }
  };

  // ---- A fragments of chunk c = (phase g, tap k): lane-linear, by LDS-DMA one tap ahead
  const char *wsp = reinterpret_cast<const char *>(a.wsplit);
  const int ncc = C / 32;
  auto issue_a = [&](int c, char *dst) {
    const int g = c / K, k = c - K * (c / K);
    // the packed buffer holds 64 rows (4 blocks x 3 pieces = 12 KB) per (tap, K chunk) whatever
    // Co is (split_frag_count pads Co to a 64-row tile); the first 3 NCO pieces are this Co's
    const char *src = wsp + (long)((k * ncc + g) * 12) * 1024 + lane * 16;
#pragma unroll
    for (int pc = wave; pc < 3 * NCO; pc += 4)
      __builtin_amdgcn_global_load_lds((const void *)(src + pc * 1024), (lds_void *)(dst + pc * 1024), 16, 0, 0);
  };

  // ---- sampling passes: lane group kr computes (tap, group) pt(kr) of its pixel in both rows
  const int pt = CG == 32 ? kr : (kr & 1);
  const int lgrp = CG == 32 ? 0 : (kr >> 1);
  float poh[2], pow_[2], pml[2];
  auto load_pass = [&](int g, int t0) {
    const int t = min(t0 + pt, K - 1), gr = CG == 32 ? g : (kr >> 1);
    const unsigned P4 = (unsigned)P * 4u;
    const int o_h = (int)__umul24((unsigned)(gr * 2 * K + 2 * t), P4);
    const int o_m = (int)__umul24((unsigned)(gr * K + t), P4);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      poh[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, o_h + p4[r], 0, 0));
      pow_[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, o_h + (int)P4 + p4[r], 0, 0));
      pml[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mskr, o_m + p4[r], 0, 0));
    }
  };
  TapState ps[2];
  // the pass of chunk cn when it starts one (tap kn == t0n), then the next pass's offsets
  auto pass_for = [&](int cn) {
    const int gn = cn / K, kn = cn - K * gn, t0n = kn - kn % TPP;
    if (kn != t0n) return;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      ps[r] = tap_state<WR, WC>(poh[r], pow_[r], pml[r], py[r], px, pv[r], min(t0n + pt, K - 1), H, W,
                                wy0, wx0, a.mask_logits, a.mask_scale);
    if (t0n + TPP < K)
      load_pass(gn, t0n + TPP);
    else if (gn + 1 < NPH)
      load_pass(gn + 1, 0);
  };
  auto get_state = [&](int r, int cn) -> TapState {
    const int gn = cn / K, kn = cn - K * gn, t0n = kn - kn % TPP;
    const int src = (((kn - t0n + 2 * lgrp) << 4) | jj) << 2;
    TapState s;
    s.pos = __builtin_amdgcn_ds_bpermute(src, ps[r].pos);
    s.w0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, ps[r].w0)));
    s.w1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, ps[r].w1)));
    s.w2 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, ps[r].w2)));
    s.w3 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, ps[r].w3)));
    return s;
  };

  // bilinear blend of this lane's 8 channels from the window ((c0 w0 + c1 w1) + c2 w2) + c3 w3
  auto blend_win = [&](const TapState &s, float (&v)[8]) {
    const char *base = sWin + (max(s.pos, 0) + kr * 2 * NPOS) * 16;
    f32x4 cq[4][2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      cq[0][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16);
      cq[1][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + 16);
      cq[2][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + WC * 16);
      cq[3][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + (WC + 1) * 16);
    }
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = cq[0][h2][u] * s.w0;
        t = __builtin_fmaf(cq[1][h2][u], s.w1, t);
        t = __builtin_fmaf(cq[2][h2][u], s.w2, t);
        t = __builtin_fmaf(cq[3][h2][u], s.w3, t);
        v[4 * h2 + u] = t;
      }
  };
  // the same from global memory, for a sample outside the window (any offset is handled)
  auto blend_global = [&](const TapState &s, int r, int cn, float (&v)[8]) {
#pragma clang fp contract(off)
    const int g = cn / K, k = cn - K * g;
    const int oplane = ((CG == 32 ? g : lgrp) * 2 * K + 2 * k) * P * 4;
    const float oh = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, p4[r] + oplane, 0, 0));
    const float ow = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(offr, p4[r] + oplane + P * 4, 0, 0));
    const int i = k / 3, j = k - 3 * (k / 3);
    const float h = (float)(py[r] - DIL + i * DIL) + oh;
    const float w = (float)(px - DIL + j * DIL) + ow;
    const int hl = (int)floorf(h), wl = (int)floorf(w);
    const int rb = XN ? 4 : C * 4, qo = XN ? (g * 32 + 8 * kr) * P * 4 : (g * 8 + 2 * kr) * 16;
    int o[4];
    o[0] = (hl >= 0 && wl >= 0) ? (hl * W + wl) * rb + qo : img_bytes;
    o[1] = (hl >= 0 && wl + 1 <= W - 1) ? (hl * W + wl + 1) * rb + qo : img_bytes;
    o[2] = (hl + 1 <= H - 1 && wl >= 0) ? ((hl + 1) * W + wl) * rb + qo : img_bytes;
    o[3] = (hl + 1 <= H - 1 && wl + 1 <= W - 1) ? ((hl + 1) * W + wl + 1) * rb + qo : img_bytes;
    f32x4 gq[4][2];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        if constexpr (XN) {
          const int pl = o[cc] == img_bytes ? 0 : P * 4;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            gq[cc][h2][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o[cc] + (4 * h2 + u) * pl, 0, 0));
        } else {
          gq[cc][h2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o[cc], h2 * 16, 0));
        }
      }
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = gq[0][h2][u] * s.w0;
        t = __builtin_fmaf(gq[1][h2][u], s.w1, t);
        t = __builtin_fmaf(gq[2][h2][u], s.w2, t);
        t = __builtin_fmaf(gq[3][h2][u], s.w3, t);
        v[4 * h2 + u] = t;
      }
  };
  // B(cn) of both rows with the out-of-window fallback (prologue and the slow path)
  auto build_any = [&](const TapState (&s)[2], int cn, u32x4 (&B)[2][3]) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float v[8];
      blend_win(s[r], v);
      if (__builtin_amdgcn_ballot_w64(s[r].pos < 0)) {
        if (s[r].pos < 0) blend_global(s[r], r, cn, v);
      }
      bf16x8 t[3];
      split8(v, t);
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) B[r][pc] = __builtin_bit_cast(u32x4, t[pc]);
    }
  };

  f32x4 acc[2][NCO];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int m = 0; m < NCO; ++m) acc[r][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma_chunk = [&](const char *sAc, const u32x4 (&Bc)[2][3]) {
    const char *ab = sAc + lane * 16;
#pragma unroll
    for (int m = 0; m < NCO; ++m) {
      bf16x8 A[3], B0[3], B1[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) {
        A[pc] = *reinterpret_cast<const bf16x8 *>(ab + (m * 3 + pc) * 1024);
        B0[pc] = __builtin_bit_cast(bf16x8, Bc[0][pc]);
        B1[pc] = __builtin_bit_cast(bf16x8, Bc[1][pc]);
      }
      acc[0][m] = mfma_split6(A, B0, acc[0][m]);
      acc[1][m] = mfma_split6(A, B1, acc[1][m]);
    }
  };

  // ---- the pipelined block: the 12 NCO MFMAs of chunk c (one product of one row each) issued in
  // a fixed order, with the vector work of chunk c+1 placed between them in "units" (the blend of
  // one channel of one row: 4 ops; the split of one channel pair: 7 ops), fenced by sched_barrier
  // so the compiler keeps the placement.  The first units wait a few MFMAs for the corner reads.
  // Each accumulator still sums its six products in mfma_split6's order: results are identical.
  auto mfma1 = [&](const u32x4 (&Au)[3], const u32x4 (&Bu)[3], f32x4 &t, int p) {
    bf16x8 A[3], B[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      A[i] = __builtin_bit_cast(bf16x8, Au[i]);
      B[i] = __builtin_bit_cast(bf16x8, Bu[i]);
    }
    switch (p) {
      case 0: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], t, 0, 0, 0); break;
      case 1: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], t, 0, 0, 0); break;
      case 2: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], t, 0, 0, 0); break;
      case 3: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], t, 0, 0, 0); break;
      case 4: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], t, 0, 0, 0); break;
      default: t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], t, 0, 0, 0); break;
    }
  };
  auto pipelined = [&](const char *sAc, const u32x4 (&Bc)[2][3], u32x4 (&Bn)[2][3], const TapState (&s)[2]) {
    constexpr int NSLOT = 12 * NCO, NUNIT = 24, FIRST = 4;
    const char *ab = sAc + lane * 16;
    u32x4 Ab[2][3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) Ab[0][pc] = *reinterpret_cast<const u32x4 *>(ab + pc * 1024);
    // window corners of row r (8 reads); row 0's are read up front, row 1's at slot ROW1, under
    // the first MFMAs
    constexpr int ROW1 = 10;
    f32x4 cq[2][4][2];
    auto read_corners = [&](int r) {
      const char *base = sWin + (max(s[r].pos, 0) + kr * 2 * NPOS) * 16;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        cq[r][0][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16);
        cq[r][1][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + 16);
        cq[r][2][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + WC * 16);
        cq[r][3][h2] = *reinterpret_cast<const f32x4 *>(base + h2 * NPOS * 16 + (WC + 1) * 16);
      }
    };
    read_corners(0);
    float v[2][8];
    u32x4 pcs[2][3];
    // unit u: rows in turn, each row's 8 blends then its 4 splits
    auto unit = [&](int u) {
      const int r = u / 12, k = u % 12;
      if (k < 8) {
        const int h2 = k >> 2, e = k & 3;
        float t = cq[r][0][h2][e] * s[r].w0;
        t = __builtin_fmaf(cq[r][1][h2][e], s[r].w1, t);
        t = __builtin_fmaf(cq[r][2][h2][e], s[r].w2, t);
        t = __builtin_fmaf(cq[r][3][h2][e], s[r].w3, t);
        v[r][k] = t;
      } else {
        const int q = k - 8;
        unsigned h, m, l;
        split_pair(v[r][2 * q], v[r][2 * q + 1], h, m, l);
        pcs[r][0][q] = h;
        pcs[r][1][q] = m;
        pcs[r][2][q] = l;
      }
    };
    __builtin_amdgcn_sched_barrier(0);
    static_for<NSLOT>([&](auto S) {
      constexpr int slot = decltype(S)::value;
      constexpr int m = slot / 12, q = slot % 12, r = q & 1, pr = q >> 1;
      if constexpr (q == 0 && m + 1 < NCO) {
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
          Ab[(m + 1) & 1][pc] = *reinterpret_cast<const u32x4 *>(ab + ((m + 1) * 3 + pc) * 1024);
      }
      if constexpr (slot == ROW1) read_corners(1);
      mfma1(Ab[m & 1], Bc[r], acc[r][m], pr);
      // units spread evenly over slots FIRST .. NSLOT-1
      static_for<NUNIT>([&](auto U) {
        constexpr int u = decltype(U)::value;
        if constexpr (FIRST + (u * (NSLOT - FIRST)) / NUNIT == slot) unit(u);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) Bn[r][pc] = pcs[r][pc];
  };

  auto next_state = [&](int cn, TapState (&s)[2]) {
    pass_for(cn);
    s[0] = get_state(0, cn);
    s[1] = get_state(1, cn);
  };

  // ---- one pipelined step c: the MFMAs of chunk c on B(c) || the corners, blend and split of
  // chunk c+1 (sampling state Sc, handed over in the step before); then the state of chunk c+2
  // (Sn), so no step waits on its own ds_bpermute hand-off
  float pf_res = 0.f;
  auto step = [&](int c, const u32x4 (&Bc)[2][3], u32x4 (&Bn)[2][3], const char *sAc, char *sAn,
                  const TapState (&Sc)[2], TapState (&Sn)[2]) {
    if (c + 1 < NCH) issue_a(c + 1, sAn);
    if (NPH == 2 && c == K - 1) {
      // phase switch: phase 1's window is loaded under chunk c's MFMAs and stored once every wave
      // is past them (each built its last phase-0 chunk before the previous barrier); B(c+1) is
      // then built outside the pipeline (once per workgroup)
      load_window(1);
      mfma_chunk(sAc, Bc);
      store_window();
      __syncthreads();
      build_any(Sc, c + 1, Bn);
      next_state(c + 2, Sn);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      return;
    }
    if (!PLAIN && c == NCH - 4 && a.residual) {  // L2 warm-up of the epilogue's identity rows
      const int yy = min(y0 + (tid & 7), H - 1), co2 = min(tid >> 3, a.Co2 - 1);
      pf_res = a.residual[((long)(n * a.Co2 + co2) * H + yy) * W + x0];
    }
    if (c + 1 < NCH) {
      // Sc is a step old: this wave-uniform test waits on nothing
      if (!__builtin_amdgcn_ballot_w64(Sc[0].pos < 0 || Sc[1].pos < 0)) {
        pipelined(sAc, Bc, Bn, Sc);
      } else {
        mfma_chunk(sAc, Bc);
        build_any(Sc, c + 1, Bn);
      }
      if (c + 2 < NCH) next_state(c + 2, Sn);
    } else {
      mfma_chunk(sAc, Bc);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of A(c+1) landed ...
    __syncthreads();                                   // ... and every other wave's
  };

  // ---- prologue: window of phase 0, pass 0, A(0), B(0), the state of chunk 1
  load_window(0);
  load_pass(0, 0);
  issue_a(0, sA0);
  store_window();
  __syncthreads();
  u32x4 B0[2][3], B1[2][3];
  TapState S0[2], S1[2];
  next_state(0, S0);
  build_any(S0, 0, B0);
  next_state(1, S1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < NCH - 1; c += 2) {
    step(c, B0, B1, sA0, sA1, S1, S0);
    step(c + 1, B1, B0, sA1, sA0, S0, S1);
  }
  if constexpr (NCH % 2) step(NCH - 1, B0, B1, sA0, sA1, S1, S0);
  asm volatile("" ::"v"(pf_res));

  if constexpr (PLAIN) {
    // ---- op-level DCN: act(post_scale * (acc + bias) + post_shift) -> LDS [co][px] -> NCHW rows
    float *sO = reinterpret_cast<float *>(sWin);
#pragma unroll
    for (int m = 0; m < NCO; ++m) {
      const int co = 16 * m + 4 * kr;
      const f32x4 bs = a.bias ? *reinterpret_cast<const f32x4 *>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 sc = a.post_scale ? *reinterpret_cast<const f32x4 *>(a.post_scale + co) : f32x4{1.f, 1.f, 1.f, 1.f};
      const f32x4 sh = a.post_scale ? *reinterpret_cast<const f32x4 *>(a.post_shift + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          sO[(co + i) * OP + (2 * wave + r) * 16 + jj] = act_f((acc[r][m][i] + bs[i]) * sc[i] + sh[i], a.act);
    }
    __syncthreads();
    constexpr int EPP = CT * TR * (TC / 4) / NT;
#pragma unroll
    for (int i = 0; i < EPP; ++i) {
      const int e = tid + NT * i, co = e >> 5, qi = e & 31, yy = y0 + (qi >> 2), xx = x0 + 4 * (qi & 3);
      if (yy < H && xx < W)
        *reinterpret_cast<f32x4 *>(a.out + ((long)(n * CT + co) * H + yy) * W + xx) =
            *reinterpret_cast<const f32x4 *>(sO + co * OP + (qi >> 2) * 16 + 4 * (qi & 3));
    }
    return;
  }

  // ---- epilogue items (4 pixels x 1 channel): identity loads issued before the conv3 tail
  constexpr int EPT = CT * TR * (TC / 4) / NT;  // items per thread
  const int Co2 = a.Co2;
  const bool res = a.residual != nullptr, csa = a.csa_out != nullptr;
  f32x4 er[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + NT * i, co2 = e >> 5, qi = e & 31, yy = y0 + (qi >> 2), xx = x0 + 4 * (qi & 3);
    if (res && co2 < Co2 && yy < H && xx < W)
      er[i] = *reinterpret_cast<const f32x4 *>(a.residual + ((long)(n * Co2 + co2) * H + yy) * W + xx);
  }

  // ---- tail: BN2 + act -> conv3 (pointwise, split-bf16); conv3's A fragments (NPH K chunks x
  // NCO blocks x 3 pieces, standard fragment order) by LDS-DMA into the two A slots
  {
    const char *src = reinterpret_cast<const char *>(a.tail_wsplit) + lane * 16;
#pragma unroll
    for (int pc = wave; pc < 3 * NCO * NPH; pc += 4) {
      char *dst = pc < 3 * NCO ? sA0 + pc * 1024 : sA1 + (pc - 3 * NCO) * 1024;
      __builtin_amdgcn_global_load_lds((const void *)(src + pc * 1024), (lds_void *)dst, 16, 0, 0);
    }
  }
  // accumulator of co block m holds channels 16m + 4kr + i of pixel jj: for the conv3 K chunk h2
  // lane group kr supplies {32h2 + 4kr + i, 32h2 + 16 + 4kr + i} (a permutation of the K index
  // that the A fragments below are read in)
  bf16x8 B2[2][NPH][3];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int h2 = 0; h2 < NPH; ++h2) {
      float v[8];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int m = 2 * h2 + half, co = 16 * m + 4 * kr;
        const f32x4 bs = a.bias ? *reinterpret_cast<const f32x4 *>(a.bias + co) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 sc = a.post_scale ? *reinterpret_cast<const f32x4 *>(a.post_scale + co) : f32x4{1.f, 1.f, 1.f, 1.f};
        const f32x4 sh = a.post_scale ? *reinterpret_cast<const f32x4 *>(a.post_shift + co) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) v[4 * half + i] = act_f((acc[r][m][i] + bs[i]) * sc[i] + sh[i], a.act);
      }
      split8(v, B2[r][h2]);
    }
  f32x4 acc2[2][NCO];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int m = 0; m < NCO; ++m) acc2[r][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed ...
  __syncthreads();                                   // ... and every other wave's
  {
    // standard fragment (cc = h2, blk = m2, piece pc): lane l holds row 16 m2 + (l & 15), channels
    // 32 h2 + 8 (l >> 4) + 0..7.  Channels 32h2 + 4kr + 0..3 are lane (kr/2)*16 + jj, bytes
    // 8 (kr & 1); channels 32h2 + 16 + 4kr + 0..3 the same 32 lanes further.
    const int tl = (((kr >> 1) << 4) | jj) * 16 + 8 * (kr & 1);
#pragma unroll
    for (int m2 = 0; m2 < NCO; ++m2)
#pragma unroll
      for (int h2 = 0; h2 < NPH; ++h2) {
        bf16x8 A[3];
#pragma unroll
        for (int pc = 0; pc < 3; ++pc) {
          const char *f = (h2 ? sA1 : sA0) + tl + (m2 * 3 + pc) * 1024;
          const u32x2 lo = *reinterpret_cast<const u32x2 *>(f);
          const u32x2 hi = *reinterpret_cast<const u32x2 *>(f + 512);
          A[pc] = __builtin_bit_cast(bf16x8, u32x4{lo.x, lo.y, hi.x, hi.y});
        }
        acc2[0][m2] = mfma_split6(A, B2[0][h2], acc2[0][m2]);
        acc2[1][m2] = mfma_split6(A, B2[1][h2], acc2[1][m2]);
      }
  }
  // ---- epilogue: tile -> LDS [co2][px] -> 16-byte row quads (+ bias, identity, act, CSA) ------
  float *sO = reinterpret_cast<float *>(sWin);
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int m2 = 0; m2 < NCO; ++m2)
#pragma unroll
      for (int i = 0; i < 4; ++i) sO[(16 * m2 + 4 * kr + i) * OP + (2 * wave + r) * 16 + jj] = acc2[r][m2][i];
  __syncthreads();
  float rsc[2] = {1.f, 1.f};
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (csa && j < a.num_up) rsc[j] = (float)a.up_h[j] / (float)H;
  // two batches of items: every global load of a batch (the CSA terms' source segments) issued
  // before its first use
  constexpr int EB = EPT >= 4 ? EPT / 2 : EPT;
#pragma unroll
  for (int i0 = 0; i0 < EPT; i0 += EB) {
    f32x4 ev[EB], eu[EB][2][2];
#pragma unroll
    for (int ii = 0; ii < EB; ++ii) {
      const int i = i0 + ii;
      const int e = tid + NT * i, co2 = e >> 5, qi = e & 31, yy = y0 + (qi >> 2), xx = x0 + 4 * (qi & 3);
      ev[ii] = *reinterpret_cast<const f32x4 *>(sO + co2 * OP + (qi >> 2) * 16 + 4 * (qi & 3));
      if (!(co2 < Co2 && yy < H && xx < W) || !csa) continue;
      const long plane = (long)n * Co2 + co2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (j >= a.num_up) break;
        const int ih = a.up_h[j], iw = a.up_w[j], rr = a.up_r[j];
        float hr = rsc[j] * ((float)yy + 0.5f) - 0.5f;
        hr = hr < 0.f ? 0.f : hr;
        const int h1 = (int)hr, h1p = h1 < ih - 1 ? 1 : 0;
        const float *im = a.up[j] + plane * ih * iw;
        const int s0 = rr == 2 ? 2 * (xx >> 2) - 1 : (xx >> 2) - 1;
        eu[ii][j][0] = load_seg(im + (long)h1 * iw, iw, s0);
        eu[ii][j][1] = load_seg(im + (long)(h1 + h1p) * iw, iw, s0);
      }
    }
#pragma unroll
    for (int ii = 0; ii < EB; ++ii) {
      const int i = i0 + ii;
      const int e = tid + NT * i, co2 = e >> 5, qi = e & 31, yy = y0 + (qi >> 2), xx = x0 + 4 * (qi & 3);
      if (!(co2 < Co2 && yy < H && xx < W)) continue;
      const long eo = ((long)(n * Co2 + co2) * H + yy) * W + xx;
      const float eb = a.tail_b ? a.tail_b[co2] : 0.f;
      f32x4 v = ev[ii];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float t = v[u] + eb;
        if (res) t += er[i][u];
        v[u] = act_f(t, a.tail_act);
      }
      *reinterpret_cast<f32x4 *>(a.out + eo) = v;
      if (csa) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (j >= a.num_up) break;
          float hr = rsc[j] * ((float)yy + 0.5f) - 0.5f;
          hr = hr < 0.f ? 0.f : hr;
          const float h1l = hr - (float)(int)hr, h0l = 1.f - h1l;
          v += h0l * hlerp(eu[ii][j][0], a.up_r[j]) + h1l * hlerp(eu[ii][j][1], a.up_r[j]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = act_f(v[u], a.csa_act);
        *reinterpret_cast<f32x4 *>(a.csa_out + eo) = v;
      }
    }
  }
}

}  // namespace

// The pipelined form takes the tail without the post stage and the plain form, at C = 64 or 32
// (dcn_tile_supported's shapes); AANET_EUNSUPPORTED otherwise (dcn_tile.hip's kernel then runs).
int dcn_win_launch(const DcnTileArgs &a, hipStream_t stream) {
  if (a.post_wsplit || a.dbg) return AANET_EUNSUPPORTED;
  const long tiles = (long)host_div_up(a.W, TC) * host_div_up(a.H, TR);
  const dim3 grid((unsigned)(a.N * tiles)), block(NT);
  if (a.plain) {
    if (a.C == 64 && a.x_nchw)
      hipLaunchKernelGGL((dcn_win_kernel<32, true, true>), grid, block, 0, stream, a);
    else if (a.C == 64)
      hipLaunchKernelGGL((dcn_win_kernel<32, false, true>), grid, block, 0, stream, a);
    else if (a.x_nchw)
      hipLaunchKernelGGL((dcn_win_kernel<16, true, true>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((dcn_win_kernel<16, false, true>), grid, block, 0, stream, a);
  } else {
    if (a.x_nchw) return AANET_EUNSUPPORTED;
    if (a.C == 64)
      hipLaunchKernelGGL((dcn_win_kernel<32, false, false>), grid, block, 0, stream, a);
    else
      hipLaunchKernelGGL((dcn_win_kernel<16, false, false>), grid, block, 0, stream, a);
  }
  return aanet_launch_status();
}
