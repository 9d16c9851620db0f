// conv_g3.hip -- the deformable bottleneck's offset_conv (nets/deform.py:58-60, 76-79: 3x3,
// dilation d, padding d, groups = deformable_groups, bias, no BN / activation) for gfx950, read
// from the channels-last conv1 output that the DCN tail reads next.
//
// Why not the conv engine.  The engine's halo tile holds ONE 32-channel group per workgroup
// (grid.y = groups): at C2 scale 0 (64 -> 54, two groups of 32 -> 27, dilation 2) every
// workgroup stages, splits and contracts a single K chunk, so its prologue and epilogue latency
// are never hidden (95-111 us alone, 0.33 of the split ceiling, 208-222 us inside the step where
// it shares the CUs with the coarse-scale work).  Here a workgroup owns an 8 x 16 output tile
// and EVERY group and output channel, and walks its K chunks (group, 32-channel chunk) in turn.
//
// Per chunk the tile's (8 + 2d) x (16 + 2d) input halo is loaded once, split into three bf16
// pieces once and stored in LDS (the engine's XOR-swizzled 64-byte rows: conflict-free
// ds_read_b128 for any tap shift); the next chunk's halo loads are in flight in registers during
// this chunk's taps.  Wave w = tile row w, lane (kr = lane / 16, jj = lane % 16) = pixel jj and
// channels 8kr..8kr+7: tap (ti, tj) reads its B fragment (3 pieces) at halo position
// (w + ti d, jj + tj d).  A step = one tap of one chunk; its pre-split A fragments (the group's
// ceil(Cog / 16) co blocks x 3 pieces) arrive by LDS-DMA two steps ahead into a ring of three
// slots, every wave issuing exactly one piece per step (waves past the step's piece count copy
// into a dummy slot), so the counted s_waitcnt of every wave names exactly the loads it needs.
// (The round-3 form of this kernel read and split the B values per tap -- 9x the split VALU --
// and ran at 160 us.)
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

// put 4 channels (quad q4 of a 32-channel row) of halo position pos into the three piece planes
// (plane stride pe bf16), at the engine's swizzled offset (mdcn.hip swz / put_split)
__device__ __forceinline__ int g3_swz(int row, int q8) { return row * 32 + ((q8 ^ (((row >> 2) & 1) << 1)) << 3); }
__device__ __forceinline__ void g3_put(__bf16 *plane, int pe, int pos, int q4, f32x4 v) {
  float a[8] = {v[0], v[1], v[2], v[3], 0.f, 0.f, 0.f, 0.f};
  bf16x8 b[3];
  split8(a, b);
  const int o = g3_swz(pos, q4 >> 1) + ((q4 & 1) << 2);
#pragma unroll
  for (int pc = 0; pc < 3; ++pc) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x4 w = __builtin_bit_cast(u32x4, b[pc]);
    *reinterpret_cast<u32x2 *>(plane + pc * pe + o) = u32x2{w[0], w[1]};
  }
}

// G groups of NCC 32-channel chunks, NCB 16-row co blocks per group (Cog <= 16 NCB), dilation D
template <int G, int NCC, int NCB, int D>
__global__ __launch_bounds__(NT, 2) void conv3x3_g3_kernel(G3Args a) {
  constexpr int NPC = 3 * NCB;             // 1-KB DMA pieces per step (<= 8)
  constexpr int AB = NPC * 1024;
  constexpr int NCH = G * NCC;             // K chunks
  constexpr int NS = NCH * 9;              // steps
  constexpr int HWW = TC + 2 * D, HR = TR + 2 * D, NPOS = HR * HWW;  // halo
  constexpr int HIT = (NPOS * 8 + NT - 1) / NT;  // halo quads per thread
  constexpr int PE = NPOS * 32;            // bf16 per piece plane
  static_assert(NPC <= 8, "one DMA piece per wave and step");
  __shared__ __attribute__((aligned(16))) __bf16 sH[3 * PE];
  __shared__ __attribute__((aligned(16))) char sA0[AB];
  __shared__ __attribute__((aligned(16))) char sA1[AB];
  __shared__ __attribute__((aligned(16))) char sA2[AB];
  __shared__ __attribute__((aligned(16))) char sDummy[NPC < 8 ? 1024 : 16];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kr = lane >> 4, jj = lane & 15;
  const int H = a.H, W = a.W, C = a.C;
  const int tx = (W + TC - 1) / TC, ntiles = tx * ((H + TR - 1) / TR);
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile = bid % ntiles;
  const int y0 = (tile / tx) * TR, x0 = (tile % tx) * TC;
  const int y = y0 + wave, x = x0 + jj;
  const bool pv = y < H && x < W;
  const long HW = (long)H * W;
  const u32x4 xr = make_rsrc(a.x + n * HW * C, (int)(HW * C * 4));
  const int Cg = C / G;

  // halo item i of this thread: position e >> 3, channel quad e & 7 (8 lanes = one 128-B line);
  // the byte offset of its quad in chunk 0 (chunk ch adds the SGPR offset), OOB outside the image
  int hoff[HIT];
#pragma unroll
  for (int i = 0; i < HIT; ++i) {
    const int e = tid + NT * i, pos = e >> 3;
    const int yy = y0 - D + pos / HWW, xx = x0 - D + pos % HWW;
    const bool ok = pos < NPOS && yy >= 0 && yy < H && xx >= 0 && xx < W;
    hoff[i] = ok ? ((yy * W + xx) * C + 4 * (e & 7)) * 4 : (int)OOB;
  }
  auto load_halo = [&](int ch, f32x4 (&hv)[HIT]) {
    const int g = ch / NCC, cc = ch % NCC;
    const int so = __builtin_amdgcn_readfirstlane((g * Cg + 32 * cc) * 4);
#pragma unroll
    for (int i = 0; i < HIT; ++i)
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(hv[i]) : "v"(hoff[i]), "s"(xr), "s"(so) : "memory");
  };
  auto store_halo = [&](const f32x4 (&hv)[HIT]) {
#pragma unroll
    for (int i = 0; i < HIT; ++i) {
      const int e = tid + NT * i, pos = e >> 3;
      if (pos < NPOS) g3_put(sH, PE, pos, e & 7, hv[i]);
    }
  };
  // one piece per wave: pieces 0..NPC-1 of the step's A fragments, waves past them a dummy copy
  // (the step's base address in an SGPR pair, the lane's offset in one VGPR for the whole
  // kernel: a per-step 64-bit VALU address was ~40 of the kernel's VALU instructions)
  const int pcw = wave < NPC ? wave : 0;
  const unsigned avo = pcw * 1024 + lane * 16;
  auto issue_a = [&](int s, char *dst) {
    const char *sb = a.wsplit + (long)s * AB;
    char *dp = wave < NPC ? dst + pcw * 1024 : sDummy;
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void *)dp);
    asm volatile("global_load_lds_dwordx4 %0, %1" :: "v"(avo), "s"(sb), "{m0}"(m0) : "memory");
  };
  // wait until at most CNT of this wave's vector-memory ops are in flight AND its LDS reads have
  // completed, then the workgroup barrier, in ONE asm statement (the halo values in flight pass
  // through as operands, so no use is scheduled ahead of the wait).  lgkmcnt(0): a wave could
  // reach the barrier with its reads of a weight slot still queued at the LDS, and the DMA
  // another wave issues into that slot right after the barrier enters the LDS by the memory
  // return path, unordered with them -- a stale-slot race that showed as run-to-run differences
  // of the offset (1-3 runs in 30 beside other work, tools/race_probe.py; round 5)
  auto wait_bar = [&](auto cnt_c, f32x4 (&hv)[HIT]) {
    constexpr int CNT = decltype(cnt_c)::value;
    if constexpr (HIT == 4)
      asm volatile("s_waitcnt vmcnt(%4) lgkmcnt(0)\n\ts_barrier" : "+v"(hv[0]), "+v"(hv[1]), "+v"(hv[2]), "+v"(hv[3]) : "n"(CNT) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%3) lgkmcnt(0)\n\ts_barrier" : "+v"(hv[0]), "+v"(hv[1]), "+v"(hv[2]) : "n"(CNT) : "memory");
  };
  auto slot = [&](int i) -> char * { return i == 0 ? sA0 : (i == 1 ? sA1 : sA2); };

  f32x4 acc[G][NCB];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int m = 0; m < NCB; ++m) acc[g][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  // prologue: chunk 0's halo, A(0), A(1); everything landed, halo into LDS
  f32x4 hv[HIT];
  load_halo(0, hv);
  issue_a(0, sA0);
  issue_a(1, sA1);
  wait_bar(std::integral_constant<int, 0>{}, hv);
  store_halo(hv);
  __syncthreads();
  // step s = (chunk s / 9, tap s % 9): issue A(s + 2) [and, at tap 0 of a chunk with a successor,
  // the next chunk's halo after it], contract, then wait for A(s + 1) and barrier.  vmcnt counts
  // in issue order, so A(s + 1) has landed when at most the ops issued after it remain: A(s + 2)
  // (1) plus this step's halo loads (HIT) at tap 0 -- and at tap 1 the halo, now older than
  // A(s + 2), must land too (two steps of cover).  At tap 8 the halo goes into LDS.
  for_steps([&](auto s_c) {
    constexpr int S = decltype(s_c)::value;
    constexpr int CH = S / 9, K = S % 9, TI = K / 3, TJ = K % 3;
    constexpr int GS = CH / NCC;
    constexpr bool HALO_NEXT = K == 0 && CH + 1 < NCH;
    if constexpr (S + 2 < NS) issue_a(S + 2, slot((S + 2) % 3));
    if constexpr (HALO_NEXT) load_halo(CH + 1, hv);
    const __bf16 *bp = sH + g3_swz((wave + TI * D) * HWW + jj + TJ * D, kr);
    bf16x8 B[3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) B[pc] = *reinterpret_cast<const bf16x8 *>(bp + pc * PE);
    const char *ab = slot(S % 3) + lane * 16;
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
      bf16x8 A[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) A[pc] = *reinterpret_cast<const bf16x8 *>(ab + (m * 3 + pc) * 1024);
      acc[GS][m] = mfma_split6(A, B, acc[GS][m]);
    }
    if constexpr (S + 1 < NS) {
      constexpr int CNT = (S + 2 < NS ? 1 : 0) + (HALO_NEXT ? HIT : 0);
      wait_bar(std::integral_constant<int, CNT>{}, hv);
      if constexpr (K == 8) {  // next chunk: every wave is done with this halo (the barrier)
        store_halo(hv);
        __syncthreads();
      }
    }
  }, std::make_integer_sequence<int, NS>{});

  // epilogue: channel g Cog + 16m + 4kr + r of pixel (y, x), NCHW (16 lanes = 64-byte segments)
  if (!pv) return;
  const int Cog = a.Co / G;
  // the biases first, as one batch under one wave-uniform test (rows past Cog are never stored):
  // loaded per value under the lane-varying cl < Cog, each load was followed by its own full wait
  // (buffer loads: channel offset in the SGPR operand, rows past Co read 0 by the range check)
  float bv[G][NCB][4] = {};
  if (a.bias) {
    const u32x4 br = make_rsrc(a.bias, a.Co * 4);
    const unsigned bvo = 16u * kr;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int m = 0; m < NCB; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int so = __builtin_amdgcn_readfirstlane((g * Cog + 16 * m + r) * 4);
          asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(bv[g][m][r]) : "v"(bvo), "s"(br), "s"(so) : "memory");
        }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // buffer stores over this image's output: the thread's byte offset (channel 4kr, its pixel) in
  // one VGPR, the channel offset (g Cog + 16m + r) * HW * 4 in the SGPR operand, and channels past
  // Cog pushed out of the buffer's range (dropped by the range check) instead of branched around:
  // no per-store 64-bit address or exec-mask branch
  const u32x4 orr = make_rsrc(a.out + (long)n * a.Co * HW, (int)((long)a.Co * HW * 4));
  const int hw4 = (int)HW * 4;
  const unsigned vo = (unsigned)((4 * kr) * hw4 + (y * W + x) * 4);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int m = 0; m < NCB; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cl = 16 * m + 4 * kr + r;
        const unsigned v = cl < Cog ? vo : OOB;
        const int so = __builtin_amdgcn_readfirstlane((g * Cog + 16 * m + r) * hw4);
        const float val = acc[g][m][r] + bv[g][m][r];
        asm volatile("buffer_store_dword %0, %1, %2, %3 offen" :: "v"(val), "v"(v), "s"(orr), "s"(so) : "memory");
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
  if ((long)h * w * c * 4 >= (1L << 31) || (long)h * w * co * 4 >= (1L << 31)) return AANET_EUNSUPPORTED;
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
  // the AANet offset convs: two 32-channel groups (scale 0) or one (single group); dilation 1/2
  auto launch = [&](auto g_c, auto ncc_c, auto ncb_c) -> bool {
    constexpr int G = decltype(g_c)::value, NCC = decltype(ncc_c)::value, NCB = decltype(ncb_c)::value;
    if (dil == 2)
      hipLaunchKernelGGL((conv3x3_g3_kernel<G, NCC, NCB, 2>), grid, blk, 0, st, a);
    else if (dil == 1)
      hipLaunchKernelGGL((conv3x3_g3_kernel<G, NCC, NCB, 1>), grid, blk, 0, st, a);
    else
      return false;
    return true;
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  bool ok = false;
  if (groups == 2 && ncc == 1 && ncb == 2)
    ok = launch(I2{}, I1{}, I2{});
  else if (groups == 2 && ncc == 1 && ncb == 1)
    ok = launch(I2{}, I1{}, I1{});
  else if (groups == 1 && ncc == 1 && ncb == 2)
    ok = launch(I1{}, I1{}, I2{});
  else if (groups == 1 && ncc == 2 && ncb == 2)
    ok = launch(I1{}, I2{}, I2{});
  if (!ok) return AANET_EUNSUPPORTED;
  return aanet_launch_status();
}

}  // extern "C"
