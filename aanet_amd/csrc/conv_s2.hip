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

#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "split.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int NT = 512;         // 8 waves, one output row each
constexpr int TR = 8, TC = 16;  // output tile
constexpr unsigned OOB = 0x80000000u;  // buffer offset past any num_records: loads return 0

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// raw buffer resource (stride 0): base, num_records bytes, the flags of make_buffer_rsrc above
__device__ __forceinline__ u32x4 make_rsrc(const float *base, int bytes) {
  const unsigned long p = reinterpret_cast<unsigned long>(base);
  // wave-uniform by construction; readfirstlane keeps the "s" asm operand in SGPRs
  return u32x4{(unsigned)__builtin_amdgcn_readfirstlane((int)p),
               (unsigned)__builtin_amdgcn_readfirstlane((int)((p >> 32) & 0xffffu)),
               (unsigned)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}

struct S2Args {
  const float *x;      // [N][C1][H][W]
  const float *x2;     // [N][C - C1][H][W] (channels appended after x's), or NULL
  const char *wsplit;  // [C/32][9][NCB][3][64 lanes][16 B]
  const float *bias;   // [Co] or NULL
  float *out[2];
  int co_a, act[2];
  // CSA terms of output a, added before act[0] (aggregation.py:388-400 order): the same-size
  // identity, then the bilinearly resized coarser term
  const float *id;     // [N][co_a][Ho][Wo] or NULL
  const float *up;     // [N][co_a][up_h][up_w] or NULL
  int up_h, up_w;
  float up_sh, up_sw;  // up_h / Ho, up_w / Wo
  int N, C, C1, H, W, Ho, Wo, Co;
  int ncbt;            // Co / 16: co blocks per weight step (a workgroup takes NCB of them)
};

__device__ __forceinline__ float s2_act(float v, int act) {
  const float neg = act == 2 ? 0.2f * v : (act == 1 ? 0.f : v);  // selects, no scalar branches
  return v > 0.f ? v : neg;
}

// compile-time step loop: f(integral_constant<int, S>) for S = 0 .. N-1 (straight-line code)
template <typename F, int... S>
__device__ __forceinline__ void for_steps(F &&f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}

// epilogue: channel co = co_base + 16m + 4kr + r of pixel (y, x).  Every global access is a
// buffer op on a per-image resource: a 32-bit lane offset (channel 4kr's plane + the pixel, or the
// resize corner) formed once, and a wave-uniform plane offset per (m, r) in an SGPR, so no access
// pays 64-bit address arithmetic (round 6: the 64-bit form was 1,963 of the kernel's 3,238 static
// VALU at the C2 heads shape).  co_a is a multiple of 16, so a 16-channel block lies wholly in
// output a (where the CSA terms apply) or wholly in output b: one wave-uniform branch per block.
// The term loads of a block are all issued before its first use.  The arithmetic is the
// reference order: bias, identity, resized term, act.
template <int NCB>
__device__ __forceinline__ void s2_epilogue(const S2Args &a, const f32x4 (&acc)[NCB], int n, int y, int x,
                                            int kr, int co_base, bool pv) {
  const int Ho = a.Ho, Wo = a.Wo;
  if (!pv) return;
  const int P = Ho * Wo, pix = y * Wo + x;
  const int co_a = a.co_a, cb = a.Co - co_a;
  const bool hid = a.id != nullptr, hup = a.up != nullptr;
  const int upa = a.up_h * a.up_w;
  // per-image resources (num_records: that image's planes; the host checks the 2^31 bound)
  const auto r_id = __builtin_amdgcn_make_buffer_rsrc((void *)(hid ? a.id + (long)n * co_a * P : a.x),
                                                      (short)0, hid ? co_a * P * 4 : 0, 0x00020000);
  const auto r_up = __builtin_amdgcn_make_buffer_rsrc((void *)(hup ? a.up + (long)n * co_a * upa : a.x),
                                                      (short)0, hup ? co_a * upa * 4 : 0, 0x00020000);
  const auto r_oa = __builtin_amdgcn_make_buffer_rsrc((void *)(co_a ? a.out[0] + (long)n * co_a * P : a.x),
                                                      (short)0, co_a * P * 4, 0x00020000);
  const auto r_ob = __builtin_amdgcn_make_buffer_rsrc((void *)(cb ? a.out[1] + (long)n * cb * P : a.x),
                                                      (short)0, cb * P * 4, 0x00020000);
  const int lo = (4 * kr * P + pix) * 4;  // channel 4kr's plane + this pixel
  // the resize stencil of this pixel (PyTorch upsample_bilinear2d, align_corners=False, as in
  // csa.hip's bilinear_resize): the same four offsets and weights for every channel plane
  int lu[4] = {0, 0, 0, 0};
  float h0l = 0.f, h1l = 0.f, w0l = 0.f, w1l = 0.f;
  if (hup) {
    float hr = a.up_sh * ((float)y + 0.5f) - 0.5f;
    hr = hr < 0.f ? 0.f : hr;
    float wr = a.up_sw * ((float)x + 0.5f) - 0.5f;
    wr = wr < 0.f ? 0.f : wr;
    const int h1 = (int)hr, w1 = (int)wr;
    const int h1p = h1 < a.up_h - 1 ? 1 : 0, w1p = w1 < a.up_w - 1 ? 1 : 0;
    h1l = hr - (float)h1, h0l = 1.f - h1l;
    w1l = wr - (float)w1, w0l = 1.f - w1l;
    const int o00 = h1 * a.up_w + w1, o10 = (h1 + h1p) * a.up_w + w1;
    const int lb = 4 * kr * upa;
    lu[0] = (lb + o00) * 4;
    lu[1] = (lb + o00 + w1p) * 4;
    lu[2] = (lb + o10) * 4;
    lu[3] = (lb + o10 + w1p) * 4;
  }
#pragma unroll
  for (int m = 0; m < NCB; ++m) {
    const int cm = co_base + 16 * m;  // wave-uniform
    const int c4 = cm + 4 * kr;
    const f32x4 bs = a.bias ? *reinterpret_cast<const f32x4 *>(a.bias + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (cm < co_a) {
      float tid[4] = {}, tq[4][4] = {};
      if (hid) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          tid[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r_id, lo, (cm + r) * P * 4, 0));
      }
      if (hup) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            tq[r][q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r_up, lu[q], (cm + r) * upa * 4, 0));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[m][r] + bs[r];
        if (hid) v = v + tid[r];
        if (hup) v = v + (h0l * (w0l * tq[r][0] + w1l * tq[r][1]) + h1l * (w0l * tq[r][2] + w1l * tq[r][3]));
        v = s2_act(v, a.act[0]);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r_oa, lo, (cm + r) * P * 4, 0);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s2_act(acc[m][r] + bs[r], a.act[1]);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r_ob, lo, (cm - co_a + r) * P * 4, 0);
      }
    }
  }
}

// ---- row form for the wide tiles (round 3) ------------------------------------------------
// A counter pass of the round-3 straight-line form (one dword gather per (channel, tap); removed
// in round 4) at the C2 heads shape (tools/s2_pmc.sh): the matrix pipe busy 37 % of the kernel,
// the texture unit 47 %, and the L1 sending 8.4x the input's bytes to L2: every (channel, tap)
// was its own dword gather, so a lane's three taps of one input row are
// three instructions that touch the same lines three steps apart, and with 16 waves per CU
// streaming through a 32 KB L1 the lines are gone by the second touch.  (A rolled 64-VGPR
// variant with twice the waves per SIMD was SLOWER, 102 vs 91 us: more waves, more misses.)
// Here a lane loads the three columns 2x-1 .. 2x+1 of one (channel, input row) with ONE
// buffer_load_dwordx3 (dword-aligned; gfx9 buffer loads need no more), i.e. one instruction per
// (channel, row) instead of three, each touching its lines once.  Steps stay per tap (the A
// slot of a step is one tap's weights, two steps ahead in a ring of three slots: 2 x 54 KB per CU
// at NCB = 6, still two workgroups per CU); row r+1 is issued at the first tap of row r, so it
// has the row's three steps to land.
// Left border: the x = 0 lane loads columns 0..2 and shifts them (column -1 is padding); right
// border (odd W): column 2x+1 = W is zeroed.  Same numerics as the straight-line form (taps and
// chunks in ascending order, the same split and piece products): bit-identical outputs.
typedef float f32x3 __attribute__((ext_vector_type(3)));

template <int NCB, int NCH>
__global__ __launch_bounds__(NT, 4) void conv3x3s2_rows_kernel(S2Args a) {
  constexpr int AB = NCB * 3 * 1024;
  constexpr int NPC = 3 * NCB, ND_LO = NPC / 8, ND_HI = (NPC + 7) / 8;
  constexpr int NS = 9 * NCH, NR = 3 * NCH;  // steps (taps), rows
  __shared__ __attribute__((aligned(16))) char sA0[AB];
  __shared__ __attribute__((aligned(16))) char sA1[AB];
  __shared__ __attribute__((aligned(16))) char sA2[AB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kr = lane >> 4, jj = lane & 15;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int tx = (Wo + TC - 1) / TC, ntiles = tx * ((Ho + TR - 1) / TR);
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int n = bid / ntiles, tile = bid % ntiles;
  const int cot = blockIdx.y, co_base = 16 * NCB * cot;
  const bool nd_hi = wave < NPC % 8;
  const int txi = __builtin_amdgcn_readfirstlane(tile % tx);  // x tile (wave-uniform)
  const int y = (tile / tx) * TR + wave, x = txi * TC + jj;
  const bool pv = y < Ho && x < Wo;
  const int HW = H * W;
  const int C1 = a.C1, C2 = a.C - a.C1, nc1 = C1 / 32;
  const float *xb2 = a.x2 ? a.x2 + (long)n * C2 * HW : a.x;
  const u32x4 xr = make_rsrc(a.x + (long)n * C1 * HW, C1 * HW * 4);
  const u32x4 xr2 = make_rsrc(xb2, a.x2 ? C2 * HW * 4 : 0);
  // lane base: channel 8kr of the chunk, input row 2y-1, first loaded column 2x-1 (x = 0: 0)
  const int yy0 = 2 * y - 1, xl = x > 0 ? 2 * x - 1 : 0;
  const int lbase = (8 * kr * HW + yy0 * W + xl) * 4;
  // bit ti: input row 2y-1+ti lies inside the image (and the pixel is valid)
  unsigned rowok = 0;
#pragma unroll
  for (int ti = 0; ti < 3; ++ti) rowok |= (pv && (unsigned)(yy0 + ti) < (unsigned)H) ? 1u << ti : 0u;
  const bool fix_left = txi == 0;                                 // wave-uniform
  const bool fix_right = (W & 1) && txi == tx - 1;                // wave-uniform
  const bool rz = 2 * x + 1 >= W;                                 // this lane's column 2x+1 is padding

  // the three columns of this lane's eight channels of row r = (chunk r / 3, input row r % 3)
  auto load_row = [&](int r, f32x3 (&v)[8]) {
    const int cc = r / 3, ti = r - 3 * (r / 3);
    const unsigned keep = 0u - ((rowok >> ti) & 1u);
    const unsigned off = ((unsigned)(lbase + ti * W * 4) & keep) | (OOB & ~keep);
    const bool second = cc >= nc1;
    const int c0 = second ? cc - nc1 : cc;
    u32x4 rs = second ? xr2 : xr;
#pragma unroll
    for (int q = 0; q < 4; ++q) rs[q] = (unsigned)__builtin_amdgcn_readfirstlane((int)rs[q]);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int so = __builtin_amdgcn_readfirstlane((32 * c0 + u) * HW * 4);
      asm volatile("buffer_load_dwordx3 %0, %1, %2, %3 offen" : "=v"(v[u]) : "v"(off), "s"(rs), "s"(so) : "memory");
    }
  };
  // wait until this wave has at most CNT vector-memory ops in flight, then the workgroup barrier,
  // in ONE asm statement: the bare s_barrier intrinsic does not order memory for the compiler (an
  // A read hoisted between wait and barrier would race with the other waves' DMAs), and
  // __syncthreads' fence would wait for every load in flight.  A branch between two such
  // statements would make the compiler copy the pending registers before them.  The row values
  // about to be used pass through as operands so that no use is scheduled ahead of the wait.
  // lgkmcnt(0): this wave's reads of the weight slot must have completed before another wave's
  // LDS-DMA into it, issued after the barrier, can land (conv_g3.hip wait_bar; round 5)
  auto wait_bar = [&](auto cnt_c, f32x3 (&v)[8]) {
    constexpr int CNT = decltype(cnt_c)::value;
    asm volatile("s_waitcnt vmcnt(%8) lgkmcnt(0)\n\ts_barrier"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "n"(CNT) : "memory");
  };
  auto issue_a = [&](int s, char *dst) {
    const char *src = a.wsplit + ((long)s * a.ncbt + NCB * cot) * 3072 + lane * 16;
#pragma unroll
    for (int r = 0; r < ND_HI; ++r) {
      const int pc = wave + 8 * r;
      if (r == ND_LO && !nd_hi) break;  // wave-uniform
      const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void *)(dst + pc * 1024));
      asm volatile("global_load_lds_dwordx4 %0, off" :: "v"(src + pc * 1024), "{m0}"(m0) : "memory");
    }
  };
  auto slot = [&](int i) -> char * { return i == 0 ? sA0 : (i == 1 ? sA1 : sA2); };
  // border fix-ups of a landed row (wave-uniform branches, taken by the border tiles only)
  auto fix_row = [&](f32x3 (&v)[8]) {
    if (fix_left) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (x == 0) v[u] = f32x3{0.f, v[u][0], v[u][1]};
    }
    if (fix_right) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (rz) v[u][2] = 0.f;
    }
  };

  f32x4 acc[NCB];
#pragma unroll
  for (int m = 0; m < NCB; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x3 rv[2][8];
  // Weights two steps ahead in a ring of three slots: step s issues A(s+2) into slot (s+2) % 3,
  // the slot step s-1 read (every wave passed the barrier after it).  The first step of row r
  // also issues row r+1's values, AFTER A(s+2).  vmcnt counts in issue order, so each wait names
  // exactly the ops younger than the one it needs (a wave that issued ND_HI pieces waits for
  // one piece more than necessary):
  //   end of tap 0: A(s+1) landed; A(s+2) and row r+1 may stay in flight
  //   end of tap 1: A(s+1) landed (issued before row r+1); row r+1 and A(s+2) may stay in flight
  //   end of tap 2: A(s+1) landed, hence row r+1 too (older); A(s+2) may stay in flight
  issue_a(0, sA0);
  issue_a(1, sA1);
  load_row(0, rv[0]);
  wait_bar(std::integral_constant<int, 0>{}, rv[0]);
  for_steps([&](auto s_c) {
    constexpr int S = decltype(s_c)::value;
    constexpr int R = S / 3, TJ = S % 3;
    constexpr bool A2 = S + 2 < NS;                // A(S+2) issued by this step
    constexpr bool ROWN = TJ == 0 && R + 1 < NR;   // row R+1 issued by this step
    constexpr bool ROWP = TJ == 1 && R + 1 < NR;   // row R+1 issued by the previous step
    if constexpr (TJ == 0) fix_row(rv[R % 2]);
    if constexpr (A2) issue_a(S + 2, slot((S + 2) % 3));
    if constexpr (ROWN) load_row(R + 1, rv[(R + 1) % 2]);
    float v8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v8[u] = rv[R % 2][u][TJ];
    bf16x8 B[3];
    split8(v8, B);
    const char *ab = slot(S % 3) + lane * 16;
#pragma unroll
    for (int m = 0; m < NCB; ++m) {
      bf16x8 A[3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) A[pc] = *reinterpret_cast<const bf16x8 *>(ab + (m * 3 + pc) * 1024);
      acc[m] = mfma_split6(A, B, acc[m]);
    }
    if constexpr (S + 1 < NS) {
      constexpr int CNT = (A2 ? ND_LO : 0) + ((ROWN || ROWP) ? 8 : 0);
      wait_bar(std::integral_constant<int, CNT>{}, rv[(TJ == 2 ? R + 1 : R) % 2]);
    }
  }, std::make_integer_sequence<int, NS>{});

  s2_epilogue<NCB>(a, acc, n, y, x, kr, co_base, pv);
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

template <int NCB>
void launch_s2(int nch, dim3 grid, dim3 blk, hipStream_t st, const S2Args &a) {
  switch (nch) {  // the AANet pyramid: 32 / 64 / 96 input channels
    case 1: hipLaunchKernelGGL((conv3x3s2_rows_kernel<NCB, 1>), grid, blk, 0, st, a); return;
    case 2: hipLaunchKernelGGL((conv3x3s2_rows_kernel<NCB, 2>), grid, blk, 0, st, a); return;
    case 3: hipLaunchKernelGGL((conv3x3s2_rows_kernel<NCB, 3>), grid, blk, 0, st, a); return;
    default: hipLaunchKernelGGL((conv3x3s2_rows_kernel<NCB, 4>), grid, blk, 0, st, a); return;
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

int aanet_conv3x3s2_terms_f32(const float *x, const void *wsplit, const float *bias, int n,
                              int c, int h, int w, int co, int co_a, float *out_a, int act_a,
                              float *out_b, int act_b, const aanet_s2_terms_t *terms,
                              aanet_stream_t stream) {
  if (terms && terms->struct_size != sizeof(aanet_s2_terms_t)) return AANET_EABI;
  if (!x || !wsplit || n < 0 || h < 0 || w < 0 || co_a < 0 || co_a > co) return AANET_EINVAL;
  const int c2 = terms && terms->x2 ? terms->c2 : 0;
  if (c2 < 0 || (terms && terms->x2 == nullptr && terms->c2 != 0)) return AANET_EINVAL;
  if (co <= 0 || co % 16 || c <= 0 || c % 32 || c2 % 32 || c + c2 > 128) return AANET_EUNSUPPORTED;
  if ((co_a > 0 && !out_a) || (co_a < co && !out_b)) return AANET_EINVAL;
  if ((long)c * h * w * 4 >= (1L << 31) || (long)c2 * h * w * 4 >= (1L << 31)) return AANET_EUNSUPPORTED;
  const int ho = (h + 1) / 2, wo = (w + 1) / 2;
  // the epilogue's block-uniform output choice and 32-bit buffer offsets
  if (co_a % 16 || (long)co * ho * wo * 4 >= (1L << 31)) return AANET_EUNSUPPORTED;
  const bool has_terms = terms && (terms->identity || terms->up);
  if (has_terms && co_a == 0) return AANET_EINVAL;
  if (terms && terms->up && (terms->up_h <= 0 || terms->up_w <= 0)) return AANET_EINVAL;
  if (n == 0 || h == 0 || w == 0) return AANET_OK;
  S2Args a;
  a.x = x;
  a.x2 = c2 ? terms->x2 : nullptr;
  a.wsplit = reinterpret_cast<const char *>(wsplit);
  a.bias = bias;
  a.out[0] = out_a;
  a.out[1] = out_b;
  a.co_a = co_a;
  a.act[0] = act_a;
  a.act[1] = act_b;
  a.id = terms ? terms->identity : nullptr;
  a.up = terms ? terms->up : nullptr;
  a.up_h = a.up ? terms->up_h : 1;
  a.up_w = a.up ? terms->up_w : 1;
  a.up_sh = (float)a.up_h / (float)ho;
  a.up_sw = (float)a.up_w / (float)wo;
  a.N = n, a.C = c + c2, a.C1 = c, a.H = h, a.W = w, a.Co = co;
  a.Ho = ho;
  a.Wo = wo;
  const long tiles = (long)host_div_up(a.Wo, TC) * host_div_up(a.Ho, TR) * n;
  if (tiles > 0x7fffffffL) return AANET_EUNSUPPORTED;
  a.ncbt = co / 16;
  // one workgroup takes every output channel (co tiles of 48 sharing the input through L2
  // measured 114 vs 93 us for the C2 heads launch)
  const int ncb = a.ncbt;
  const dim3 grid((unsigned)tiles), blk(NT);
  hipStream_t st = as_hip(stream);
  const int nch = a.C / 32;
  switch (ncb) {
    case 1: launch_s2<1>(nch, grid, blk, st, a); break;
    case 2: launch_s2<2>(nch, grid, blk, st, a); break;
    case 3: launch_s2<3>(nch, grid, blk, st, a); break;
    case 4: launch_s2<4>(nch, grid, blk, st, a); break;
    case 5: launch_s2<5>(nch, grid, blk, st, a); break;
    case 6: launch_s2<6>(nch, grid, blk, st, a); break;
    default: return AANET_EUNSUPPORTED;
  }
  return aanet_launch_status();
}

int aanet_conv3x3s2_f32(const float *x, const void *wsplit, const float *bias, int n, int c, int h,
                        int w, int co, int co_a, float *out_a, int act_a, float *out_b, int act_b,
                        aanet_stream_t stream) {
  return aanet_conv3x3s2_terms_f32(x, wsplit, bias, n, c, h, w, co, co_a, out_a, act_a, out_b,
                                   act_b, nullptr, stream);
}

}  // extern "C"
