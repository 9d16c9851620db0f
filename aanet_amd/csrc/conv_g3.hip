// conv_g3.hip -- the deformable bottleneck's offset_conv (nets/deform.py:58-60, 76-79: 3x3,
// dilation d, padding d, groups = deformable_groups, bias, no BN / activation) for gfx950, read
// straight from the channels-last conv1 output that the DCN tail reads next.
//
// Why not the conv engine.  The engine's halo tile holds ONE 32-channel group per workgroup
// (grid.y = groups): at C2 scale 0 (64 -> 54, two groups of 32 -> 27, dilation 2) every
// workgroup stages, splits and contracts a single K chunk, so its prologue and epilogue latency
// are never hidden (≈115 us alone, 0.28 of the split ceiling, 208-222 us inside the step where
// it shares the CUs with the coarse-scale work).  Here a workgroup owns an 8 x 16 output tile
// and EVERY group and output channel, and walks (group, chunk, tap) steps like the stride-2
// row kernel (conv_s2.hip): wave w = tile row w, lane (kr = lane / 16, jj = lane % 16) = pixel
// jj and channels 8kr..8kr+7 of the chunk -- exactly its B fragment of v_mfma_f32_16x16x32_bf16,
// read from NHWC as two 16-byte loads (no im2col, no LDS staging of the input) -- and the
// step's pre-split A fragments (the group's ceil(Cog / 16) co blocks x 3 pieces) arrive by
// LDS-DMA two steps ahead into a ring of three slots.  Every wave issues exactly one DMA piece
// per step (waves past the step's piece count copy into a dummy slot), so the counted
// s_waitcnt of every wave names exactly the loads it needs.
//
// Numerics: the split-bf16 contraction of the conv engine (split.h), taps ascending within a
// chunk and chunks ascending within a group; output NCHW + bias.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"
#include "split.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;         // 8 waves, one output row each
constexpr int TR = 8, TC = 16;  // output tile
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ u32x4 make_rsrc(const void *base, int bytes) {
  const unsigned long p = reinterpret_cast<unsigned long>(base);
  return u32x4{(unsigned)__builtin_amdgcn_readfirstlane((int)p),
               (unsigned)__builtin_amdgcn_readfirstlane((int)((p >> 32) & 0xffffu)),
               (unsigned)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}

template <typename F, int... S>
__device__ __forceinline__ void for_steps(F &&f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}

struct G3Args {
  const float *x;      // [N][H][W][C] (channels-last)
  const char *wsplit;  // [G][Cg/32][9][NCB][3][64 lanes][16 B]
  const float *bias;   // [Co] or NULL
  float *out;          // [N][Co][H][W]
  int N, C, H, W, Co, dil;
};

// G groups of NCC 32-channel chunks, NCB 16-row co blocks per group (Cog <= 16 NCB)
template <int G, int NCC, int NCB>
__global__ __launch_bounds__(NT, 4) void conv3x3_g3_kernel(G3Args a) {
  constexpr int NPC = 3 * NCB;             // 1-KB DMA pieces per step (<= 8)
  constexpr int AB = NPC * 1024;
  constexpr int NS = G * NCC * 9;          // steps
  static_assert(NPC <= 8, "one DMA piece per wave and step");
  __shared__ __attribute__((aligned(16))) char sA0[AB];
  __shared__ __attribute__((aligned(16))) char sA1[AB];
  __shared__ __attribute__((aligned(16))) char sA2[AB];
  __shared__ __attribute__((aligned(16))) char sDummy[NPC < 8 ? 1024 : 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kr = lane >> 4, jj = lane & 15;
  const int H = a.H, W = a.W, C = a.C, d = a.dil;
  const int tx = (W + TC - 1) / TC, ntiles = tx * ((H + TR - 1) / TR);
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile = bid % ntiles;
  const int y = (tile / tx) * TR + wave, x = (tile % tx) * TC + jj;
  const bool pv = y < H && x < W;
  const long HW = (long)H * W;
  const u32x4 xr = make_rsrc(a.x + n * HW * C, (int)(HW * C * 4));
  // lane base: pixel (y - d, x - d), channel 8kr (tap (ti, tj) adds (ti W + tj) d pixels)
  const int lbase = (((y - d) * W + (x - d)) * C + 8 * kr) * 4;
  unsigned okmask = 0;  // bit k: tap k's input pixel lies inside the image
#pragma unroll
  for (int k = 0; k < 9; ++k)
    okmask |= (pv && (unsigned)(y + (k / 3 - 1) * d) < (unsigned)H &&
               (unsigned)(x + (k % 3 - 1) * d) < (unsigned)W) ? 1u << k : 0u;

  // step s = (group s / (9 NCC), chunk, tap s % 9): the lane's eight channels of its tap pixel
  auto load_b = [&](int s, f32x4 (&v)[2]) {
    const int g = s / (9 * NCC), cc = (s / 9) % NCC, k = s % 9, ti = k / 3, tj = k % 3;
    const unsigned keep = 0u - ((okmask >> k) & 1u);
    const unsigned off = ((unsigned)(lbase + (ti * W + tj) * d * C * 4) & keep) | (OOB & ~keep);
    const int so = __builtin_amdgcn_readfirstlane((g * NCC + cc) * 32 * 4);
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v[0]) : "v"(off), "s"(xr), "s"(so) : "memory");
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:16" : "=v"(v[1]) : "v"(off), "s"(xr), "s"(so) : "memory");
  };
  // one piece per wave: pieces 0..NPC-1 of the step's A fragments, waves past them a dummy copy
  auto issue_a = [&](int s, char *dst) {
    const int pc = wave < NPC ? wave : 0;
    const char *src = a.wsplit + (long)s * AB + pc * 1024 + lane * 16;
    char *dp = wave < NPC ? dst + pc * 1024 : sDummy;
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void *)dp);
    asm volatile("global_load_lds_dwordx4 %0, off" :: "v"(src), "{m0}"(m0) : "memory");
  };
  // wait until at most CNT of this wave's vector-memory ops are in flight, then the workgroup
  // barrier, in ONE asm statement; the B values about to be used pass through as operands
  auto wait_bar = [&](auto cnt_c, f32x4 (&v)[2]) {
    constexpr int CNT = decltype(cnt_c)::value;
    asm volatile("s_waitcnt vmcnt(%2)\n\ts_barrier" : "+v"(v[0]), "+v"(v[1]) : "n"(CNT) : "memory");
  };
  auto slot = [&](int i) -> char * { return i == 0 ? sA0 : (i == 1 ? sA1 : sA2); };

  f32x4 acc[G][NCB];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int m = 0; m < NCB; ++m) acc[g][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 bv[3][2];
  // steps s+1 and s+2 are in flight while step s computes: each step issues [A(s+2), B(s+2)]
  // (3 ops) and then waits for everything but those three -- i.e. for step s+1's
  issue_a(0, sA0);
  load_b(0, bv[0]);
  issue_a(1, sA1);
  load_b(1, bv[1]);
  wait_bar(std::integral_constant<int, 3>{}, bv[0]);
  for_steps([&](auto s_c) {
    constexpr int S = decltype(s_c)::value;
    constexpr int GS = S / (9 * NCC);
    if constexpr (S + 2 < NS) {
      issue_a(S + 2, slot((S + 2) % 3));
      load_b(S + 2, bv[(S + 2) % 3]);
    }
    float v8[8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v8[u] = bv[S % 3][0][u];
      v8[4 + u] = bv[S % 3][1][u];
    }
    bf16x8 B[3];
    split8(v8, B);
    const char *ab = slot(S % 3) + lane * 16;
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
      bf16x8 A[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) A[pc] = *reinterpret_cast<const bf16x8 *>(ab + (m * 3 + pc) * 1024);
      acc[GS][m] = mfma_split6(A, B, acc[GS][m]);
    }
    if constexpr (S + 1 < NS) {
      constexpr int CNT = S + 2 < NS ? 3 : 0;
      wait_bar(std::integral_constant<int, CNT>{}, bv[(S + 1) % 3]);
    }
  }, std::make_integer_sequence<int, NS>{});

  // epilogue: channel g Cog + 16m + 4kr + r of pixel (y, x), NCHW (16 lanes = 64-byte segments)
  if (!pv) return;
  const int Cog = a.Co / G;
  const long pix = (long)y * W + x;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int m = 0; m < NCB; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * m + 4 * kr + r;
        if (cl < Cog) {
          const int co = g * Cog + cl;
          a.out[((long)n * a.Co + co) * HW + pix] = acc[g][m][r] + (a.bias ? a.bias[co] : 0.f);
        }
      }
}

// w [Co][Cg][3][3] fp32 (groups G, Cog = Co / G) -> [G][Cg/32][9][NCB][3][64 lanes][8 bf16]: lane
// l of co block m holds row g Cog + 16m + l%16 (zero past Cog), channels 32cc + 8(l/16) + 0..7
// of the group, as three exact bf16 pieces
__global__ void conv3x3_g3_pack_kernel(const float *__restrict__ w, bf16x8 *__restrict__ out, int Co,
                                       int Cg, int G, int ncb) {
  const int Cog = Co / G, ncc = Cg / 32, total = G * ncc * 9 * ncb * 64;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int l = e % 64, m = (e / 64) % ncb, k = (e / 64 / ncb) % 9, cc = (e / 64 / ncb / 9) % ncc,
              g = e / 64 / ncb / 9 / ncc;
    const int cl = 16 * m + (l & 15), c0 = 32 * cc + 8 * (l >> 4);
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = cl < Cog ? w[((long)(g * Cog + cl) * Cg + c0 + u) * 9 + k] : 0.f;
    bf16x8 b[3];
    split8(v, b);
    const long base = (((long)((g * ncc + cc) * 9 + k) * ncb + m) * 3) * 64 + l;
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) out[base + pc * 64] = b[pc];
  }
}

int g3_ncb(int co, int groups) { return (co / groups + 15) / 16; }

}  // namespace

extern "C" {

size_t aanet_conv3x3_grouped_pack_bytes(int co, int c, int groups) {
  if (co <= 0 || c <= 0 || groups <= 0 || co % groups || c % groups || (c / groups) % 32) return 0;
  const int ncb = g3_ncb(co, groups);
  if (ncb > 2) return 0;
  return (size_t)groups * (c / groups / 32) * 9 * ncb * 3 * 1024;
}

int aanet_conv3x3_grouped_pack_f32(const float *w, int co, int c, int groups, void *wsplit,
                                   aanet_stream_t stream) {
  if (!w || !wsplit || !aanet_conv3x3_grouped_pack_bytes(co, c, groups)) return AANET_EINVAL;
  const int ncb = g3_ncb(co, groups), cg = c / groups;
  const int total = groups * (cg / 32) * 9 * ncb * 64;
  hipLaunchKernelGGL(conv3x3_g3_pack_kernel, dim3(host_div_up(total, 256)), dim3(256), 0, as_hip(stream),
                     w, reinterpret_cast<bf16x8 *>(wsplit), co, cg, groups, ncb);
  return aanet_launch_status();
}

int aanet_conv3x3_grouped_nhwc_f32(const float *x, const void *wsplit, const float *bias, int n,
                                   int c, int h, int w, int co, int groups, int dil, float *out,
                                   aanet_stream_t stream) {
  if (!x || !wsplit || !out || n < 0 || h < 0 || w < 0 || dil < 1) return AANET_EINVAL;
  if (!aanet_conv3x3_grouped_pack_bytes(co, c, groups)) return AANET_EUNSUPPORTED;
  if ((long)h * w * c * 4 >= (1L << 31)) return AANET_EUNSUPPORTED;
  if (n == 0 || h == 0 || w == 0) return AANET_OK;
  const int ncb = g3_ncb(co, groups), ncc = c / groups / 32;
  G3Args a;
  a.x = x;
  a.wsplit = reinterpret_cast<const char *>(wsplit);
  a.bias = bias;
  a.out = out;
  a.N = n, a.C = c, a.H = h, a.W = w, a.Co = co, a.dil = dil;
  const long tiles = (long)host_div_up(w, TC) * host_div_up(h, TR) * n;
  if (tiles > 0x7fffffffL) return AANET_EUNSUPPORTED;
  const dim3 grid((unsigned)tiles), blk(NT);
  hipStream_t st = as_hip(stream);
  // the AANet offset convs: two 32-channel groups (scale 0) or one (single group)
  if (groups == 2 && ncc == 1 && ncb == 2)
    hipLaunchKernelGGL((conv3x3_g3_kernel<2, 1, 2>), grid, blk, 0, st, a);
  else if (groups == 2 && ncc == 1 && ncb == 1)
    hipLaunchKernelGGL((conv3x3_g3_kernel<2, 1, 1>), grid, blk, 0, st, a);
  else if (groups == 1 && ncc == 1 && ncb == 2)
    hipLaunchKernelGGL((conv3x3_g3_kernel<1, 1, 2>), grid, blk, 0, st, a);
  else if (groups == 1 && ncc == 2 && ncb == 2)
    hipLaunchKernelGGL((conv3x3_g3_kernel<1, 2, 2>), grid, blk, 0, st, a);
  else
    return AANET_EUNSUPPORTED;
  return aanet_launch_status();
}

}  // extern "C"
