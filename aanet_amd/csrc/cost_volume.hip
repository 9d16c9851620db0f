// cost_volume.hip -- cost-volume construction for gfx950 (replaces nets/cost.py:19-76).
//
// Correlation (cost.py:40-48) is a banded contraction over channels:
//   P[x][x'] = sum_c L[c][x] * R[c][x'],  out[d][x] = P[x][x-d] / C  for 0 <= d < D.
// One workgroup owns a 64-wide x tile of one (b, y) row and a chunk of <=64 disparities.
// Channels stream through LDS in 16-channel stages (double-buffered LDS, two stages of loads in
// flight in a register ring; for C in {32, 64, 128} the branch-free, fully unrolled ring tile
// corr_reg_tile, otherwise the general corr_tile).  Each of the 4 waves owns 16 x
// and computes the 16 x (16*NJ) band of P with v_mfma_f32_16x16x4_f32 (exact fp32), so
// every L / R element is read from HBM once and the FMAs run on the matrix pipe.  The band
// is transposed through LDS to [d][x] and stored as full 256-B rows.  x' < 0 reads are
// zero, which produces the x < d zero fill of cost.py:41 for free.
#include "common.h"

#include <type_traits>

namespace {

constexpr int TX = 64;      // x positions per workgroup
constexpr int CC = 16;      // channels per LDS stage
constexpr int NTHREADS = 256;

template <int NJ>
struct CorrSmem {
  static constexpr int RW = TX + 16 * (NJ - 1);       // right-feature window width
  static constexpr int DC = 16 * (NJ - 1) + 1 > 64 ? 64 : 16 * (NJ - 1) + 1;
  // LDS row pitches = 16 (mod 32) dwords: an MFMA operand read (ds_read_b32, two 32-lane groups,
  // bank = dword mod 32) has lanes kr = 0,1 one row apart -> 16 banks apart, conflict-free
  static constexpr int LP = TX + 16;
  static constexpr int RP = RW + 16;
  static constexpr int STAGE = CC * LP + CC * RP;      // floats per stage
  // [d][x] band tile pitch: odd (lanes jj distinct) with 4*(OUTP+1) = 16 (mod 32) (kr groups
  // disjoint) -> conflict-free band writes
  static constexpr int OUTP = TX + 3;
  // band rows dl = 16j + i - jj span [-15, 16*NJ): rows outside [0, dchunk) are scratch, so the
  // band is written without per-element predicates (immediate LDS offsets from one base)
  static constexpr int OROWS = 16 * NJ + 15;
  static constexpr int BYTES_STAGE = 2 * STAGE * 4;
  static constexpr int BYTES_OUT = OROWS * OUTP * 4;
  static constexpr int BYTES = BYTES_STAGE > BYTES_OUT ? BYTES_STAGE : BYTES_OUT;
};

// grid: 1-D, ntx * nchunks * H * N blocks.  Block ids are remapped so that every XCD owns a
// contiguous range of (x tile fastest, then d chunk, row, image): the right-feature windows of
// neighbouring x tiles overlap by half, and the overlap is then served by the same L2.
// Loads are 16-byte buffer loads whose range check supplies the zero padding (x < 0, x >= W,
// c >= C); requires W % 4 == 0 (the launcher falls back to the scalar kernel otherwise).
// Staging is a two-slot register ring: stage s+2's loads are issued before stage s's MFMAs, so
// two stages (24 KB per workgroup) are in flight.  L is read once: non-temporal loads; the
// volume is written once: non-temporal stores (tools/corr_lab.hip: -6 % vs default policy).
// R keeps the default policy, because the neighbouring tile re-reads half of its window from L2.
__device__ __forceinline__ int xcd_remap(int nwg, int b0) {  // bijective for any grid size
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
}

// One workgroup of the correlation: work item `id` of one volume (x tile fastest, then d chunk,
// row, image).  smem: CorrSmem<NJ>::BYTES.
template <int NJ, int VEC>
__device__ __forceinline__ void corr_tile(const float *__restrict__ L, const float *__restrict__ R,
                                          float *__restrict__ out, int C, int H, int W, int D,
                                          int dchunk, int ntx, int nchunks, int id, float *smem) {
  using S = CorrSmem<NJ>;
  constexpr int RW = S::RW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tx = id % ntx;
  id /= ntx;
  const int chunk = id % nchunks;
  id /= nchunks;
  const int y = id % H, b = id / H;
  const int x0 = tx * TX, d0 = chunk * dchunk;
  const int xr0 = x0 - d0 - 16 * (NJ - 1);  // first x' of the right window
  const long HW = (long)H * W;
  const int img_bytes = (int)(C * HW * 4);
  const auto Lr = __builtin_amdgcn_make_buffer_rsrc((void *)(L + (long)b * C * HW), (short)0,
                                                     img_bytes, 0x00020000);
  const auto Rr = __builtin_amdgcn_make_buffer_rsrc((void *)(R + (long)b * C * HW), (short)0,
                                                     img_bytes, 0x00020000);
  const float *Lrow = L + (long)b * C * HW + (long)y * W;
  const float *Rrow = R + (long)b * C * HW + (long)y * W;

  constexpr int LQ = CC * TX / 4;            // float4 per stage of L (256: one per thread)
  constexpr int RQ = CC * RW / 4;            // float4 per stage of R
  constexpr int RPT4 = (RQ + NTHREADS - 1) / NTHREADS;
  constexpr int LPT = CC * TX / NTHREADS;    // scalar fallback
  constexpr int RPT = (CC * RW + NTHREADS - 1) / NTHREADS;
  f32x4 lq[2][1], rq[2][VEC ? RPT4 : 1];
  float lreg[2][VEC ? 1 : LPT], rreg[2][VEC ? 1 : RPT];
  const int HW4 = (int)(HW * 4);  // VEC requires C*H*W*4 < 2^31 (launcher)
  const int lrow = tid / (TX / 4), lcol = x0 + 4 * (tid % (TX / 4));
  const bool lok = lcol < W;
  const int lbase = (lrow * (int)HW + y * W + lcol) * 4;
  int rrow[RPT4], rbase[RPT4];
  bool rok[RPT4];
#pragma unroll
  for (int i = 0; i < RPT4; ++i) {
    const int e = tid + i * NTHREADS;
    const int x = xr0 + 4 * (e % (RW / 4));
    rrow[i] = e / (RW / 4);
    rok[i] = e < RQ && x >= 0 && x < W;
    rbase[i] = (rrow[i] * (int)HW + y * W + x) * 4;
  }

  auto load_stage = [&](int c0, int slot) {
    if (VEC) {
      // per-thread int32 byte offsets (lbase / rbase, hoisted) + the stage's channel offset
      // (scalar); out-of-range elements take the OOB offset, whose load returns 0
      const int coff = c0 * HW4;
      lq[slot][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
          Lr, (c0 + lrow < C && lok && tid < LQ) ? lbase + coff : img_bytes, 0, 2 /* nt */));
#pragma unroll
      for (int i = 0; i < RPT4; ++i)
        rq[slot][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
            Rr, (c0 + rrow[i] < C && rok[i]) ? rbase[i] + coff : img_bytes, 0, 0));
    } else {
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int e = tid + i * NTHREADS, row = e / TX, col = e % TX;
        const int c = c0 + row, x = x0 + col;
        lreg[slot][i] = (c < C && x < W) ? Lrow[(long)c * HW + x] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int e = tid + i * NTHREADS, row = e / RW, col = e % RW;
        const int c = c0 + row, x = xr0 + col;
        rreg[slot][i] = (e < CC * RW && c < C && x >= 0 && x < W) ? Rrow[(long)c * HW + x] : 0.f;
      }
    }
  };
  auto store_stage = [&](int slot, int buf) {
    float *sL = smem + buf * S::STAGE, *sR = sL + CC * S::LP;
    if (VEC) {
      if (tid < LQ)
        *reinterpret_cast<f32x4 *>(sL + lrow * S::LP + 4 * (tid % (TX / 4))) = lq[slot][0];
#pragma unroll
      for (int i = 0; i < RPT4; ++i) {
        const int e = tid + i * NTHREADS;
        if (e < RQ)
          *reinterpret_cast<f32x4 *>(sR + rrow[i] * S::RP + 4 * (e % (RW / 4))) = rq[slot][i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < LPT; ++i) {
        const int e = tid + i * NTHREADS;
        sL[(e / TX) * S::LP + e % TX] = lreg[slot][i];
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int e = tid + i * NTHREADS;
        if (e < CC * RW) sR[(e / RW) * S::RP + e % RW] = rreg[slot][i];
      }
    }
  };

  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // a wave whose 16 x all lie past W (the last tile of a row whose W is not a multiple of 64)
  // skips its MFMAs; it still stages and meets every barrier
  const bool active = x0 + 16 * wave < W;
  const int kr = lane >> 4, jj = lane & 15;
  // one stage: issue stage s+2's loads into the ring slot stage s vacated, run stage s's MFMAs
  // from LDS buffer P (all operands read before the MFMA run), then stage s+1 into buffer 1-P
  const int nstages = (C + CC - 1) / CC;
  auto step = [&](auto P_, int s) {
    constexpr int P = decltype(P_)::value;
    if (s + 2 < nstages) load_stage((s + 2) * CC, P);
    if (active) {
      const float *sL = smem + P * S::STAGE, *sR = sL + CC * S::LP;
      float a[CC / 4], bv[CC / 4][NJ];
#pragma unroll
      for (int ks = 0; ks < CC / 4; ++ks) {
        const int row = 4 * ks + kr;
        a[ks] = sL[row * S::LP + 16 * wave + jj];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[ks][j] = sR[row * S::RP + 16 * wave + jj + 16 * (NJ - 1 - j)];
      }
#pragma unroll
      for (int ks = 0; ks < CC / 4; ++ks)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x16x4(a[ks], bv[ks][j], acc[j]);
    }
    if (s + 1 < nstages) store_stage(1 - P, 1 - P);
    __syncthreads();
  };
  load_stage(0, 0);
  if (nstages > 1) load_stage(CC, 1);
  store_stage(0, 0);
  __syncthreads();
  for (int s = 0; s < nstages; s += 2) {
    step(std::integral_constant<int, 0>(), s);
    if (s + 1 < nstages) step(std::integral_constant<int, 1>(), s + 1);
  }

  // Band -> [d][x] tile in LDS.  Lane holds x' column jj, rows i = 4*kr + r (x).
  // Row dl = 16j + 4kr + r - jj, column 16*wave + 4kr + r: one base per lane, the (j, r) part
  // is an immediate offset.  Rows outside [0, dmax) land in the scratch rows and are not stored.
  float *sO = smem + 15 * S::OUTP;
  const float invC = 1.f / (float)C;  // exact for power-of-two C (AANet: 128, 32)
  const int dmax = min(dchunk, D - d0);
  float *sOl = sO + (4 * kr - jj) * S::OUTP + 16 * wave + 4 * kr;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) sOl[(16 * j + r) * S::OUTP + r] = acc[j][r] * invC;
  __syncthreads();
  if (VEC) {
    for (int e = tid; e < dmax * (TX / 4); e += NTHREADS) {
      const int dl = e / (TX / 4), xq = e % (TX / 4);
      if (x0 + 4 * xq < W) {
        const float *src = sO + dl * S::OUTP + 4 * xq;
        __builtin_nontemporal_store(
            f32x4{src[0], src[1], src[2], src[3]},
            reinterpret_cast<f32x4 *>(out + (((long)b * D + d0 + dl) * H + y) * W + x0 + 4 * xq));
      }
    }
  } else {
    for (int e = tid; e < dmax * TX; e += NTHREADS) {
      const int dl = e / TX, xl = e % TX;
      if (x0 + xl < W)
        __builtin_nontemporal_store(sO[dl * S::OUTP + xl],
                                    out + (((long)b * D + d0 + dl) * H + y) * W + x0 + xl);
    }
  }
}

template <int NJ, int VEC>
__global__ __launch_bounds__(NTHREADS) void corr_volume_kernel(
    const float *__restrict__ L, const float *__restrict__ R, float *__restrict__ out, int C,
    int H, int W, int D, int dchunk, int ntx, int nchunks) {
  __shared__ __attribute__((aligned(16))) float smem[CorrSmem<NJ>::BYTES / 4];
  corr_tile<NJ, VEC>(L, R, out, C, H, W, D, dchunk, ntx, nchunks, xcd_remap(gridDim.x, blockIdx.x),
                     smem);
}

// The whole pyramid (nets/cost.py:58-76) in ONE launch: a scale-major work list (scale 0's
// tiles first); a workgroup runs the tile code instantiated for its scale's band width, so the
// coarse scales fill the chip while scale 0's last tiles drain instead of running as separate,
// under-filled launches.  XCD placement is balanced PER SCALE: each scale's items are padded to a
// multiple of 8 and block b (dealt to XCD b % 8) takes item (b % 8) * per + j of its scale, so
// every XCD owns a contiguous eighth of every scale (neighbouring x tiles share the R window in
// that XCD's L2).  A remap contiguous over the whole list gave the last XCDs only the cheap
// coarse tiles and the first ones only scale-0 tiles: the launch ran at the pace of the busiest.
constexpr int MAXS = 4;
struct CorrPyramid {
  const float *L[MAXS], *R[MAXS];
  float *out[MAXS];
  int C[MAXS], H[MAXS], W[MAXS], D[MAXS], dchunk[MAXS], ntx[MAXS], nchunks[MAXS], nj[MAXS];
  int cnt[MAXS];         // work items of scale s
  int per[MAXS];         // items of scale s per XCD: ceil(cnt / 8)
  int mstart[MAXS + 1];  // prefix sums of per[]: grid = 8 * mstart[ns]
  int ns;
};

__global__ __launch_bounds__(NTHREADS) void corr_pyramid_kernel(CorrPyramid p) {
  __shared__ __attribute__((aligned(16))) float smem[CorrSmem<5>::BYTES / 4];
  const int xcd = blockIdx.x & 7, i = blockIdx.x >> 3;
  int s = 0;
  while (s + 1 < p.ns && i >= p.mstart[s + 1]) ++s;
  const int local = xcd * p.per[s] + (i - p.mstart[s]);
  if (local >= p.cnt[s]) return;  // padding of scale s to a multiple of 8 (whole workgroup)
#define AANET_CORR_CASE(J) \
  case J: corr_tile<J, 1>(p.L[s], p.R[s], p.out[s], p.C[s], p.H[s], p.W[s], p.D[s], p.dchunk[s], \
                          p.ntx[s], p.nchunks[s], local, smem); break;
  switch (p.nj[s]) {
    AANET_CORR_CASE(1)
    AANET_CORR_CASE(2)
    AANET_CORR_CASE(3)
    AANET_CORR_CASE(4)
    default: corr_tile<5, 1>(p.L[s], p.R[s], p.out[s], p.C[s], p.H[s], p.W[s], p.D[s], p.dchunk[s],
                             p.ntx[s], p.nchunks[s], local, smem);
  }
#undef AANET_CORR_CASE
}

// ------------------------------------------ register-ring correlation tile (round 3) ------
// (An LDS-DMA form of this tile -- buffer_load ... lds into a ring of three stage buffers, no VGPR
// staging -- was bit-identical but 15 % slower: the LDS ring caps the bytes in flight per CU at
// about a third of what five register-staged workgroups keep in flight)
// The round-2 tile's register ring, rebuilt so that nothing serialises it: in the round-2 form
// the staging stores sat behind per-lane guards (exec-masked branches), and on the path around
// a guard the compiler's wait tracking kept the ring registers "pending", so before issuing the
// next stage it waited for nearly all of the previous one (vmcnt(1)) -- one stage in flight.
//   * Every load and every staging store is unconditional: the R window is always 128 wide (its
//     first 16 (5 - NJ) columns read zero through the range check), so each thread owns exactly
//     one L and two R float4 per stage.
//   * The channel offset lives in the buffer resource (base advanced c0 planes, num_records =
//     (C - c0) planes): a lane's byte offsets are fixed for the whole tile, zero VALU per stage.
//   * The stage loop is fully unrolled (NS = C / 16 compile-time): ring slots and LDS buffers are
//     constants and the compiler's vmcnt waits are exact; RING stages are in flight during each
//     stage's MFMAs (RING = 3: 36 KB per workgroup, in VGPRs).
constexpr unsigned OOB = 0x80000000u;  // byte offset past any range: the buffer load returns 0

template <int NJ, int NS, int RING>
__device__ __forceinline__ void corr_reg_tile(const float *__restrict__ L, const float *__restrict__ R,
                                              float *__restrict__ out, int C, int H, int W, int D,
                                              int dchunk, int ntx, int nchunks, int id, float *smem) {
  constexpr int RW = 128, LP = TX + 16, RP = RW + 16;  // pitches = 16 mod 32: conflict-free
  constexpr int STAGE = CC * LP + CC * RP;
  constexpr int OUTP = TX + 3, OROWS = 16 * NJ + 15;
  static_assert(2 * STAGE >= OROWS * OUTP, "band tile fits the stage buffers");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tx = id % ntx;
  id /= ntx;
  const int chunk = id % nchunks;
  id /= nchunks;
  const int y = id % H, b = id / H;
  const int x0 = tx * TX, d0 = chunk * dchunk;
  const int xr0 = x0 - d0 - 64;  // the 128-wide window's first x' (NJ = 5 band reach)
  const int HW = H * W;          // C*H*W*4 < 2^31 (launcher)
  // thread -> (row, quad) of the L tile (one float4) and of the R window (two float4)
  const int lrow = tid >> 4, lq = tid & 15;
  unsigned lofs, rofs[2];
  {
    const int x = x0 + 4 * lq;
    lofs = x < W ? (unsigned)((lrow * HW + y * W + x) * 4) : OOB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i, row = e >> 5, q = e & 31;
      const int xr = xr0 + 4 * q;
      // columns left of the NJ band's reach are never read: keep them zero, no traffic
      const bool need = q >= 4 * (5 - NJ);
      rofs[i] = (need && xr >= 0 && xr < W) ? (unsigned)((row * HW + y * W + xr) * 4) : OOB;
    }
  }
  const float *Lb = L + (long)b * C * HW, *Rb = R + (long)b * C * HW;
  f32x4 lv[RING], rv[RING][2];
  auto load = [&](int slot, int s) {
    const int c0 = s * CC, nrec = (C - c0) * HW * 4;
    const auto rl = __builtin_amdgcn_make_buffer_rsrc((void *)(Lb + (long)c0 * HW), (short)0, nrec,
                                                      0x00020000);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc((void *)(Rb + (long)c0 * HW), (short)0, nrec,
                                                      0x00020000);
    lv[slot] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rl, lofs, 0, 2));
#pragma unroll
    for (int i = 0; i < 2; ++i)
      rv[slot][i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, rofs[i], 0, 0));
  };
  auto store = [&](int slot, int buf) {
    float *sL = smem + buf * STAGE, *sR = sL + CC * LP;
    *reinterpret_cast<f32x4 *>(sL + lrow * LP + 4 * lq) = lv[slot];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      *reinterpret_cast<f32x4 *>(sR + (e >> 5) * RP + 4 * (e & 31)) = rv[slot][i];
    }
  };
  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kr = lane >> 4, jj = lane & 15;
  const bool active = x0 + 16 * wave < W;  // wave-uniform (scalar) branch around the MFMAs only
  auto compute = [&](int buf) {
    const float *sL = smem + buf * STAGE, *sR = sL + CC * LP;
    float a[CC / 4], bv[CC / 4][NJ];
#pragma unroll
    for (int ks = 0; ks < CC / 4; ++ks) {
      const int row = 4 * ks + kr;
      a[ks] = sL[row * LP + 16 * wave + jj];
#pragma unroll
      for (int j = 0; j < NJ; ++j) bv[ks][j] = sR[row * RP + 16 * wave + jj + 16 * (4 - j)];
    }
#pragma unroll
    for (int ks = 0; ks < CC / 4; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[j] = mfma16x16x4(a[ks], bv[ks][j], acc[j]);
  };
#pragma unroll
  for (int k = 0; k < RING; ++k)
    if (k < NS) load(k, k);
  store(0, 0);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s + RING < NS) load(s % RING, s + RING);  // slot of stage s: stored last iteration
    if (active) compute(s & 1);
    if (s + 1 < NS) store((s + 1) % RING, (s + 1) & 1);
    __syncthreads();
  }

  // band -> [d][x] tile in LDS (rows outside [0, dchunk) are scratch), then 256-B row stores
  float *sO = smem + 15 * OUTP;
  const float invC = 1.f / (float)C;
  const int dmax = min(dchunk, D - d0);
  float *sOl = sO + (4 * kr - jj) * OUTP + 16 * wave + 4 * kr;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) sOl[(16 * j + r) * OUTP + r] = acc[j][r] * invC;
  __syncthreads();
  for (int e = tid; e < dmax * (TX / 4); e += NTHREADS) {
    const int dl = e / (TX / 4), xq = e % (TX / 4);
    if (x0 + 4 * xq < W) {
      const float *src = sO + dl * OUTP + 4 * xq;
      __builtin_nontemporal_store(
          f32x4{src[0], src[1], src[2], src[3]},
          reinterpret_cast<f32x4 *>(out + (((long)b * D + d0 + dl) * H + y) * W + x0 + 4 * xq));
    }
  }
}

constexpr int REG_SMEM = 2 * (CC * (TX + 16) + CC * (128 + 16));

template <int NJ, int NS, int RG>
__global__ __launch_bounds__(NTHREADS) void corr_reg_kernel(const float *__restrict__ L,
                                                            const float *__restrict__ R,
                                                            float *__restrict__ out, int C, int H,
                                                            int W, int D, int dchunk, int ntx,
                                                            int nchunks) {
  __shared__ __attribute__((aligned(16))) float smem[REG_SMEM];
  corr_reg_tile<NJ, NS, RG>(L, R, out, C, H, W, D, dchunk, ntx, nchunks,
                            xcd_remap(gridDim.x, blockIdx.x), smem);
}

// The whole pyramid in one launch on the ring tile (the work list of corr_pyramid_kernel); every
// scale has C in {32, 64, 128} (NS = C / 16 in {2, 4, 8}).  The body is compiled in the device
// pass only: the host pass rejects the tile's instantiations in this switch with a bare
// "substitution failure" (clang, ROCm 7.2), and the host never runs a kernel body.
template <int RING>
__global__ __launch_bounds__(NTHREADS) void corr_pyramid_reg_kernel(CorrPyramid p) {
  __shared__ __attribute__((aligned(16))) float smem[REG_SMEM];
#if __HIP_DEVICE_COMPILE__
  const int xcd = blockIdx.x & 7, i = blockIdx.x >> 3;
  int s = 0;
  while (s + 1 < p.ns && i >= p.mstart[s + 1]) ++s;
  const int local = xcd * p.per[s] + (i - p.mstart[s]);
  if (local >= p.cnt[s]) return;
  const int ns = p.C[s] >> 4;
#define AANET_CORR_REG(J, NSV)                                                                    \
  corr_reg_tile<J, NSV, RING>(p.L[s], p.R[s], p.out[s], p.C[s], p.H[s], p.W[s], p.D[s],          \
                              p.dchunk[s], p.ntx[s], p.nchunks[s], local, smem)
#define AANET_CORR_REG_NS(J)                 \
  case J:                                    \
    if (ns == 8) AANET_CORR_REG(J, 8);       \
    else if (ns == 4) AANET_CORR_REG(J, 4);  \
    else AANET_CORR_REG(J, 2);               \
    break;
  switch (p.nj[s]) {
    AANET_CORR_REG_NS(1)
    AANET_CORR_REG_NS(2)
    AANET_CORR_REG_NS(3)
    AANET_CORR_REG_NS(4)
    default:
      if (ns == 8) AANET_CORR_REG(5, 8);
      else if (ns == 4) AANET_CORR_REG(5, 4);
      else AANET_CORR_REG(5, 2);
  }
#undef AANET_CORR_REG_NS
#undef AANET_CORR_REG
#else
  (void)smem;
  (void)p;
#endif
}

constexpr int RING = 2;  // register-ring depth on the product path (3 measured equal)

bool corr_ring_ok(int c, int h, int w) {
  return (c == 32 || c == 64 || c == 128) && w % 4 == 0 && (long)c * h * w * 4 < 0x7fffffffL;
}

int corr_nj(int max_disp) {
  const int dneed = max_disp < 64 ? max_disp : 64;
  return dneed <= 1 ? 1 : 1 + (dneed - 1 + 15) / 16;
}

int corr_dchunk(int nj) {
  switch (nj) {
    case 1: return CorrSmem<1>::DC;
    case 2: return CorrSmem<2>::DC;
    case 3: return CorrSmem<3>::DC;
    case 4: return CorrSmem<4>::DC;
    default: return CorrSmem<5>::DC;
  }
}

template <int NJ>
int launch_corr(const float *L, const float *R, float *out, int n, int c, int h, int w, int D,
                hipStream_t st) {
  const int dchunk = CorrSmem<NJ>::DC;
  const int nchunks = host_div_up(D, dchunk);
  if (corr_ring_ok(c, h, w)) {
    const int ntx = host_div_up(w, TX);
    const long nb = (long)ntx * nchunks * h * n;
    if (nb > 0x7fffffffL) return AANET_EUNSUPPORTED;
    const dim3 grid((unsigned)nb), blk(NTHREADS);
    if (c == 128)
      hipLaunchKernelGGL((corr_reg_kernel<NJ, 8, RING>), grid, blk, 0, st, L, R, out, c, h, w, D,
                         dchunk, ntx, nchunks);
    else if (c == 64)
      hipLaunchKernelGGL((corr_reg_kernel<NJ, 4, RING>), grid, blk, 0, st, L, R, out, c, h, w, D,
                         dchunk, ntx, nchunks);
    else
      hipLaunchKernelGGL((corr_reg_kernel<NJ, 2, RING>), grid, blk, 0, st, L, R, out, c, h, w, D,
                         dchunk, ntx, nchunks);
    return aanet_launch_status();
  }
  const int ntx = host_div_up(w, TX);
  const long nblk = (long)ntx * nchunks * h * n;
  if (nblk > 0x7fffffffL) return AANET_EUNSUPPORTED;
  const bool vec = (w % 4) == 0 && (long)c * h * w * 4 < 0x7fffffffL;
  if (vec)
    hipLaunchKernelGGL((corr_volume_kernel<NJ, 1>), dim3((unsigned)nblk), dim3(NTHREADS), 0, st,
                       L, R, out, c, h, w, D, dchunk, ntx, nchunks);
  else
    hipLaunchKernelGGL((corr_volume_kernel<NJ, 0>), dim3((unsigned)nblk), dim3(NTHREADS), 0, st,
                       L, R, out, c, h, w, D, dchunk, ntx, nchunks);
  return aanet_launch_status();
}

// --------------------------------------------------------------- correlation backward ----
// grad_L[c][x]  = (1/C) sum_d gO[d][x]   * R[c][x-d]   (x-d >= 0)
// grad_R[c][x'] = (1/C) sum_d gO[d][x'+d] * L[c][x'+d] (x'+d < W)
// One workgroup = one (b, y) row x 64-wide x tile; gO band staged in LDS once, channels
// looped.  VALU kernel (training path, not the timed inference path).
constexpr int BTX = 64;
__global__ __launch_bounds__(256) void corr_volume_bwd_kernel(
    const float *__restrict__ L, const float *__restrict__ R, const float *__restrict__ gO,
    float *__restrict__ gL, float *__restrict__ gR, int C, int H, int W, int D, int ntx) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x;
  const int tx = blockIdx.x % ntx, y = blockIdx.y, b = blockIdx.z;
  const int x0 = tx * BTX;
  const int G0 = x0 - (D - 1);         // window start (for R at x-d and gO at x'+d)
  const int GW = BTX + 2 * (D - 1);    // window width
  const long HW = (long)H * W;
  float *sG = sm;                      // [D][GW] grad_out rows at x in window
  float *sLw = sG + (long)D * GW;      // [4][GW]
  float *sRw = sLw + 4 * GW;           // [4][GW]
  for (int e = tid; e < D * GW; e += 256) {
    const int d = e / GW, xx = G0 + e % GW;
    sG[e] = (xx >= 0 && xx < W) ? gO[(((long)b * D + d) * H + y) * W + xx] : 0.f;
  }
  const int xl = tid & 63, cq = tid >> 6;
  const int x = x0 + xl;
  const float invC = 1.f / (float)C;
  for (int c0 = 0; c0 < C; c0 += 4) {
    __syncthreads();
    for (int e = tid; e < 4 * GW; e += 256) {
      const int cc = c0 + e / GW, xx = G0 + e % GW;
      const bool ok = cc < C && xx >= 0 && xx < W;
      sLw[e] = ok ? L[((long)b * C + cc) * HW + (long)y * W + xx] : 0.f;
      sRw[e] = ok ? R[((long)b * C + cc) * HW + (long)y * W + xx] : 0.f;
    }
    __syncthreads();
    const int c = c0 + cq;
    if (c < C && x < W) {
      float gl = 0.f, gr = 0.f;
      const int xi = x - G0;  // index of x in the window
      for (int d = 0; d < D; ++d) {
        gl += sG[d * GW + xi] * sRw[cq * GW + xi - d];          // zero when x-d < 0
        gr += sG[d * GW + xi + d] * sLw[cq * GW + xi + d];      // zero when x+d >= W
      }
      gL[((long)b * C + c) * HW + (long)y * W + x] = gl * invC;
      gR[((long)b * C + c) * HW + (long)y * W + x] = gr * invC;
    }
  }
}

// ----------------------------------------------------------------- concat / difference ---
// Output-indexed, write-bound: out[b][oc][d][y][x]; 4 consecutive x per thread.  Index math is
// 32-bit when the volume has < 2^31 quads (IDX = int; C5 at B=8 is 1.5e8 quads), and the volume
// is written with non-temporal stores (written once, read once by the 3-D aggregation).
template <bool CONCAT, typename IDX>
__global__ __launch_bounds__(256) void shift_volume_kernel(const float *__restrict__ L,
                                                           const float *__restrict__ R,
                                                           float *__restrict__ out, int C, int H,
                                                           int W, int D, long total4_, int W4) {
  const int OC = CONCAT ? 2 * C : C;
  const IDX total4 = (IDX)total4_;
  for (IDX e = (IDX)blockIdx.x * 256 + threadIdx.x; e < total4; e += (IDX)gridDim.x * 256) {
    const int xq = (int)(e % W4);
    IDX t = e / W4;
    const int y = (int)(t % H);
    t /= H;
    const int d = (int)(t % D);
    t /= D;
    const int oc = (int)(t % OC);
    const int b = (int)(t / OC);
    const int x = 4 * xq;
    const long HW = (long)H * W;
    float v[4];
    if (CONCAT && oc < C) {
      const float *src = L + ((long)b * C + oc) * HW + (long)y * W;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (x + u < W && x + u >= d) ? src[x + u] : 0.f;
    } else {
      const int c = CONCAT ? oc - C : oc;
      const float *rs = R + ((long)b * C + c) * HW + (long)y * W - d;
      const float *ls = L + ((long)b * C + c) * HW + (long)y * W;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int xx = x + u;
        float r = 0.f;
        if (xx < W && xx >= d) r = CONCAT ? rs[xx] : ls[xx] - rs[xx];
        v[u] = r;
      }
    }
    float *o = out + ((((long)b * OC + oc) * D + d) * H + y) * W + x;
    if ((W & 3) == 0) {
      __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4 *>(o));
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (x + u < W) o[u] = v[u];
    }
  }
}

// Band form (W % 4 == 0): one workgroup per band of YB consecutive source rows y of one (b, c).
// The band's left and right rows are read once into LDS, then the workgroup writes all D shifted
// copies: concat oc = c (left, x >= d) and oc = C + c (right at x - d); difference oc = c.  Each
// (oc, d) plane receives YB*W contiguous floats (16-byte stores): long contiguous write streams
// run at 5.2 TB/s where one-row (1.2 KB) segments ran at 3.5 TB/s (tools/shift_lab.hip, C5
// [4,32,96,312], D=48).  HBM reads are exactly the two feature maps.
// LDS layout (round 4): each row is stored as 4 residue planes, element x at (x & 3) * W/4 + x/4.
// A thread writes output columns 4k..4k+3 and reads source element 4k + u - d: in the row-major
// layout the 32 lanes of a ds_read_b32 hit words 4 apart (8 banks: a 4-way conflict on every
// read, 5.3k conflict cycles per wave at C5); here consecutive lanes read consecutive words of one
// residue plane ((u - d) & 3 is the same for the lanes of a d), conflict-free.
template <bool CONCAT>
__global__ __launch_bounds__(256) void shift_volume_band_kernel(const float *__restrict__ L,
                                                                const float *__restrict__ R,
                                                                float *__restrict__ out, int C,
                                                                int H, int W, int D, int YB) {
  extern __shared__ __attribute__((aligned(16))) float srow[];
  const int tid = threadIdx.x;
  const int nyb = (H + YB - 1) / YB;
  const int yb = blockIdx.x % nyb, bc = blockIdx.x / nyb, c = bc % C, b = bc / C;
  const int y0 = yb * YB, rows = min(YB, H - y0);
  const int W4 = W >> 2, S4 = rows * W4;
  float *sL = srow, *sR = srow + YB * W;
  const f32x4 *gl = reinterpret_cast<const f32x4 *>(L + ((long)bc * H + y0) * W);
  const f32x4 *gr = reinterpret_cast<const f32x4 *>(R + ((long)bc * H + y0) * W);
  for (int q = tid; q < S4; q += 256) {
    const f32x4 vl = __builtin_nontemporal_load(gl + q), vr = __builtin_nontemporal_load(gr + q);
    const int yy = q / W4, k = q - yy * W4;
    float *dl = sL + yy * W + k, *dr = sR + yy * W + k;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dl[u * W4] = vl[u];
      dr[u * W4] = vr[u];
    }
  }
  __syncthreads();
  const int OC = CONCAT ? 2 * C : C;
  const long HW = (long)H * W;
  float *o0 = out + (((long)b * OC + c) * D * H + y0) * W;               // oc = c
  float *o1 = CONCAT ? o0 + (long)C * D * HW : nullptr;                  // oc = C + c
  // Thread slots r = tid + 256 i (i < MAXSLOT: S4 <= 2048, band_rows): the row / column of a slot
  // and its left values are fixed for the whole d loop; per (d, slot) the right values sit at
  // residue-plane offsets that are the same for every lane ((u - d) & 3 and (u - d) >> 2), so the
  // loop body is 4 LDS reads, 8 selects and 2 stores (the d-major order keeps each plane's 8-row
  // segment a contiguous write stream).  Plain stores: a pure 1 MB-per-workgroup store stream ran
  // at 5.65-5.73 TB/s plain vs 5.27-5.36 TB/s non-temporal (tools/write_ceiling.hip), and this
  // kernel at 277-280 vs 288-289 us (C5).
  constexpr int MAXSLOT = 8;
  int rb[MAXSLOT], x4[MAXSLOT];
  f32x4 lv[MAXSLOT];
#pragma unroll
  for (int i = 0; i < MAXSLOT; ++i) {
    const int r = tid + 256 * i, rr = r < S4 ? r : 0;
    const int yy = rr / W4, k = rr - yy * W4;
    rb[i] = yy * W + k;
    x4[i] = r < S4 ? 4 * k : -0x40000000;  // slots past the band never store
#pragma unroll
    for (int u = 0; u < 4; ++u) lv[i][u] = sL[yy * W + u * W4 + k];
  }
  for (int d = 0; d < D; ++d) {
    int ro[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ro[u] = __builtin_amdgcn_readfirstlane(((u - d) & 3) * W4 + ((u - d) >> 2));
    float *p0 = o0 + (long)d * HW;
    float *p1 = CONCAT ? o1 + (long)d * HW : nullptr;
#pragma unroll
    for (int i = 0; i < MAXSLOT; ++i) {
      if (256 * i >= S4) break;  // uniform
      if (x4[i] < -0x20000000) continue;
      f32x4 vl, vr;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = x4[i] + u >= d;
        vl[u] = ok ? lv[i][u] : 0.f;
        vr[u] = ok ? sR[rb[i] + ro[u]] : 0.f;
      }
      const long off = 4L * (tid + 256 * i);
      if (CONCAT) {
        *reinterpret_cast<f32x4 *>(p0 + off) = vl;
        *reinterpret_cast<f32x4 *>(p1 + off) = vr;
      } else {
        *reinterpret_cast<f32x4 *>(p0 + off) = vl - vr;
      }
    }
  }
}

// rows per band: 16 (round 5: C5 concat 283-285 -> 278-279 us against 8 rows, difference
// unchanged; 24 rows: no better), fewer when the band's two LDS rows would exceed 64 KB (so
// S4 = rows * W / 4 <= 2048: the band kernel's 8 thread slots)
#ifndef AANET_BAND_ROWS
#define AANET_BAND_ROWS 16
#endif
int band_rows(int w) {
  int yb = AANET_BAND_ROWS;
  while (yb > 1 && 2L * yb * w * 4 > 64 * 1024) yb >>= 1;
  return yb;
}

template <bool CONCAT>
__global__ __launch_bounds__(256) void shift_volume_bwd_kernel(const float *__restrict__ gO,
                                                               float *__restrict__ gL,
                                                               float *__restrict__ gR, int C,
                                                               int H, int W, int D, long total) {
  const int OC = CONCAT ? 2 * C : C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int x = (int)(e % W);
    long t = e / W;
    const int y = (int)(t % H);
    t /= H;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    const long plane = (long)H * W, base = (long)y * W;
    float gl = 0.f, gr = 0.f;
    const int ocr = CONCAT ? C + c : c;
    for (int d = 0; d < D; ++d) {
      if (x >= d) gl += gO[(((long)b * OC + c) * D + d) * plane + base + x];
      if (x + d < W) gr += gO[(((long)b * OC + ocr) * D + d) * plane + base + x + d];
    }
    gL[((long)b * C + c) * plane + base + x] = gl;
    gR[((long)b * C + c) * plane + base + x] = CONCAT ? gr : -gr;
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int aanet_corr_volume_f32(const float *left, const float *right, float *out, int n,
                                     int c, int h, int w, int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(left && right && out && n > 0 && c > 0 && h > 0 && w > 0 && max_disp > 0);
  hipStream_t st = as_hip(stream);
  const int dneed = max_disp < 64 ? max_disp : 64;
  const int nj = dneed <= 1 ? 1 : 1 + (dneed - 1 + 15) / 16;
  switch (nj) {
    case 1: return launch_corr<1>(left, right, out, n, c, h, w, max_disp, st);
    case 2: return launch_corr<2>(left, right, out, n, c, h, w, max_disp, st);
    case 3: return launch_corr<3>(left, right, out, n, c, h, w, max_disp, st);
    case 4: return launch_corr<4>(left, right, out, n, c, h, w, max_disp, st);
    default: return launch_corr<5>(left, right, out, n, c, h, w, max_disp, st);
  }
}

extern "C" int aanet_corr_pyramid_f32(int num_scales, const float *const *left,
                                      const float *const *right, float *const *out, const int *c,
                                      const int *h, const int *w, int n, int max_disp,
                                      aanet_stream_t stream) {
  AANET_HOST_CHECK(num_scales > 0 && left && right && out && c && h && w && n > 0);
  // one launch when every scale takes the vector tile path (w % 4 == 0, 32-bit offsets)
  bool one = num_scales <= MAXS;
  bool ring = one;  // every scale on the register-ring tile
  for (int s = 0; ring && s < num_scales; ++s)
    ring = c[s] > 0 && h[s] > 0 && corr_ring_ok(c[s], h[s], w[s]);
  CorrPyramid p;
  p.ns = num_scales;
  long total = 0;
  for (int s = 0; one && s < num_scales; ++s) {
    const int d = max_disp >> s;
    AANET_HOST_CHECK(left[s] && right[s] && out[s] && c[s] > 0 && h[s] > 0 && w[s] > 0 && d > 0);
    if (w[s] % 4 || (long)c[s] * h[s] * w[s] * 4 >= 0x7fffffffL) {
      one = false;
      break;
    }
    p.L[s] = left[s];
    p.R[s] = right[s];
    p.out[s] = out[s];
    p.C[s] = c[s];
    p.H[s] = h[s];
    p.W[s] = w[s];
    p.D[s] = d;
    p.nj[s] = corr_nj(d);
    p.dchunk[s] = corr_dchunk(p.nj[s]);
    p.nchunks[s] = host_div_up(d, p.dchunk[s]);
    p.ntx[s] = host_div_up(w[s], TX);
    const long cnt = (long)p.ntx[s] * p.nchunks[s] * h[s] * n;
    if (cnt > 0x7fffffffL - 8) {
      one = false;
      break;
    }
    p.cnt[s] = (int)cnt;
    p.per[s] = (int)((cnt + 7) / 8);
    p.mstart[s] = (int)(total / 8);
    total += 8L * p.per[s];
    if (total > 0x7fffffffL) one = false;
  }
  if (one) {
    p.mstart[num_scales] = (int)(total / 8);
    if (ring)
      hipLaunchKernelGGL(corr_pyramid_reg_kernel<RING>, dim3((unsigned)total), dim3(NTHREADS), 0,
                         as_hip(stream), p);
    else
      hipLaunchKernelGGL(corr_pyramid_kernel, dim3((unsigned)total), dim3(NTHREADS), 0,
                         as_hip(stream), p);
    return aanet_launch_status();
  }
  for (int s = 0; s < num_scales; ++s) {
    const int d = max_disp >> s;
    const int rc = aanet_corr_volume_f32(left[s], right[s], out[s], n, c[s], h[s], w[s], d, stream);
    if (rc != AANET_OK) return rc;
  }
  return AANET_OK;
}

extern "C" int aanet_corr_volume_bwd_f32(const float *left, const float *right,
                                         const float *grad_out, float *grad_left,
                                         float *grad_right, int n, int c, int h, int w,
                                         int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(left && right && grad_out && grad_left && grad_right && n > 0 && c > 0 &&
                   h > 0 && w > 0 && max_disp > 0);
  const int GW = BTX + 2 * (max_disp - 1);
  const size_t smem = sizeof(float) * ((size_t)max_disp * GW + 8 * GW);
  if (smem > 160 * 1024) return AANET_EUNSUPPORTED;
  const int ntx = host_div_up(w, BTX);
  hipLaunchKernelGGL(corr_volume_bwd_kernel, dim3(ntx, h, n), dim3(256), smem, as_hip(stream),
                     left, right, grad_out, grad_left, grad_right, c, h, w, max_disp, ntx);
  return aanet_launch_status();
}

extern "C" int aanet_concat_volume_f32(const float *left, const float *right, float *out, int n,
                                       int c, int h, int w, int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(left && right && out && n > 0 && c > 0 && h > 0 && w > 0 && max_disp > 0);
  const int W4 = (w + 3) / 4;
  const long total4 = (long)n * 2 * c * max_disp * h * W4;
  if (w % 4 == 0 && 2L * w * 4 <= 64 * 1024 && (long)n * c * h < 0x7fffffffL) {
    const int yb = band_rows(w);
    hipLaunchKernelGGL(shift_volume_band_kernel<true>, dim3((unsigned)(n * c * host_div_up(h, yb))),
                       dim3(256), 2 * yb * w * sizeof(float), as_hip(stream), left, right, out, c,
                       h, w, max_disp, yb);
  } else if (total4 < 0x7fffffffL - 8192L * 256)
    hipLaunchKernelGGL((shift_volume_kernel<true, int>), dim3(grid_for(total4)), dim3(256), 0,
                       as_hip(stream), left, right, out, c, h, w, max_disp, total4, W4);
  else
    hipLaunchKernelGGL((shift_volume_kernel<true, long>), dim3(grid_for(total4)), dim3(256), 0,
                       as_hip(stream), left, right, out, c, h, w, max_disp, total4, W4);
  return aanet_launch_status();
}

extern "C" int aanet_diff_volume_f32(const float *left, const float *right, float *out, int n,
                                     int c, int h, int w, int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(left && right && out && n > 0 && c > 0 && h > 0 && w > 0 && max_disp > 0);
  const int W4 = (w + 3) / 4;
  const long total4 = (long)n * c * max_disp * h * W4;
  if (w % 4 == 0 && 2L * w * 4 <= 64 * 1024 && (long)n * c * h < 0x7fffffffL) {
    const int yb = band_rows(w);
    hipLaunchKernelGGL(shift_volume_band_kernel<false>, dim3((unsigned)(n * c * host_div_up(h, yb))),
                       dim3(256), 2 * yb * w * sizeof(float), as_hip(stream), left, right, out, c,
                       h, w, max_disp, yb);
  } else if (total4 < 0x7fffffffL - 8192L * 256)
    hipLaunchKernelGGL((shift_volume_kernel<false, int>), dim3(grid_for(total4)), dim3(256), 0,
                       as_hip(stream), left, right, out, c, h, w, max_disp, total4, W4);
  else
    hipLaunchKernelGGL((shift_volume_kernel<false, long>), dim3(grid_for(total4)), dim3(256), 0,
                       as_hip(stream), left, right, out, c, h, w, max_disp, total4, W4);
  return aanet_launch_status();
}

extern "C" int aanet_concat_volume_bwd_f32(const float *grad_out, float *grad_left,
                                           float *grad_right, int n, int c, int h, int w,
                                           int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(grad_out && grad_left && grad_right && n > 0 && c > 0 && h > 0 && w > 0 &&
                   max_disp > 0);
  const long total = (long)n * c * h * w;
  hipLaunchKernelGGL(shift_volume_bwd_kernel<true>, dim3(grid_for(total)), dim3(256), 0,
                     as_hip(stream), grad_out, grad_left, grad_right, c, h, w, max_disp, total);
  return aanet_launch_status();
}

extern "C" int aanet_diff_volume_bwd_f32(const float *grad_out, float *grad_left,
                                         float *grad_right, int n, int c, int h, int w,
                                         int max_disp, aanet_stream_t stream) {
  AANET_HOST_CHECK(grad_out && grad_left && grad_right && n > 0 && c > 0 && h > 0 && w > 0 &&
                   max_disp > 0);
  const long total = (long)n * c * h * w;
  hipLaunchKernelGGL(shift_volume_bwd_kernel<false>, dim3(grid_for(total)), dim3(256), 0,
                     as_hip(stream), grad_out, grad_left, grad_right, c, h, w, max_disp, total);
  return aanet_launch_status();
}
