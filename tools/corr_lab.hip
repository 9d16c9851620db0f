// corr_lab.hip -- same-process A/B of correlation-volume kernel variants (a probe, not product
// code).  Includes the product kernel (aanet_amd/csrc/cost_volume.hip) as the baseline and the
// bit-exactness reference, and times candidate variants against it on the C2 scale-0 shape.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/corr_lab.hip -o tools/corr_lab.bin
#include "../aanet_amd/csrc/cost_volume.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t err_ = (x);                                                           \
    if (err_ != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__);            \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

namespace lab {

constexpr int TX = 64, NT = 256;

// Variant: compile-time channel count (CC x NST), register prefetch ring of depth PD, all MFMA
// operands of a stage read before the MFMA run, waves whose 16 x lie past W skip their MFMAs.
template <int NJ, int CC, int NST, int PD, int POL = 0>
__global__ __launch_bounds__(NT) void corr_v2(const float *__restrict__ L, const float *__restrict__ R,
                                              float *__restrict__ out, int H, int W, int D, int dchunk,
                                              int ntx, int nchunks) {
  constexpr int C = CC * NST;
  constexpr int RW = TX + 16 * (NJ - 1);
  constexpr int LP = TX + 16, RP = RW + 16;
  constexpr int STAGE = CC * LP + CC * RP;
  constexpr int OUTP = TX + 3, OROWS = 16 * NJ + 15;
  constexpr int BYTES = (2 * STAGE > OROWS * OUTP ? 2 * STAGE : OROWS * OUTP) * 4;
  __shared__ __attribute__((aligned(16))) float smem[BYTES / 4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int tx = id % ntx;
  id /= ntx;
  const int chunk = id % nchunks;
  id /= nchunks;
  const int y = id % H, b = id / H;
  const int x0 = tx * TX, d0 = chunk * dchunk;
  const int xr0 = x0 - d0 - 16 * (NJ - 1);
  const int HW = H * W;
  const int img_bytes = C * HW * 4;
  const auto Lr = __builtin_amdgcn_make_buffer_rsrc((void *)(L + (long)b * C * HW), (short)0, img_bytes,
                                                    0x00020000);
  const auto Rr = __builtin_amdgcn_make_buffer_rsrc((void *)(R + (long)b * C * HW), (short)0, img_bytes,
                                                    0x00020000);
  constexpr int LQ = CC * TX / 4;
  constexpr int LPT = (LQ + NT - 1) / NT;
  constexpr int RQ = CC * RW / 4;
  constexpr int RPT = (RQ + NT - 1) / NT;
  const int HW4 = HW * 4;
  int loff[LPT], roff[RPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int e = tid + i * NT, row = e / (TX / 4), col = x0 + 4 * (e % (TX / 4));
    loff[i] = (e < LQ && col < W) ? (row * HW + y * W + col) * 4 : -1;
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int e = tid + i * NT, row = e / (RW / 4), x = xr0 + 4 * (e % (RW / 4));
    roff[i] = (e < RQ && x >= 0 && x < W) ? (row * HW + y * W + x) * 4 : -1;
  }
  f32x4 lq[PD][LPT], rq[PD][RPT];
  auto load = [&](int s, int slot) {
    const int coff = s * CC * HW4;
#pragma unroll
    for (int i = 0; i < LPT; ++i)
      lq[slot][i] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(Lr, loff[i] >= 0 ? loff[i] + coff : img_bytes, 0, (POL & 1) ? 2 : 0));
#pragma unroll
    for (int i = 0; i < RPT; ++i)
      rq[slot][i] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(Rr, roff[i] >= 0 ? roff[i] + coff : img_bytes, 0, (POL & 4) ? 2 : 0));
  };
  auto store = [&](int slot, int buf) {
    float *sL = smem + buf * STAGE, *sR = sL + CC * LP;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int e = tid + i * NT;
      if (e < LQ) *reinterpret_cast<f32x4 *>(sL + (e / (TX / 4)) * LP + 4 * (e % (TX / 4))) = lq[slot][i];
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int e = tid + i * NT;
      if (e < RQ) *reinterpret_cast<f32x4 *>(sR + (e / (RW / 4)) * RP + 4 * (e % (RW / 4))) = rq[slot][i];
    }
  };

  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool active = x0 + 16 * wave < W;
  const int kr = lane >> 4, jj = lane & 15;

#pragma unroll
  for (int p = 0; p < PD && p < NST; ++p) load(p, p);
  store(0, 0);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NST; ++s) {
    if (s + PD < NST) load(s + PD, s % PD);
    if (active) {
      const float *sL = smem + (s & 1) * STAGE, *sR = sL + CC * LP;
      float a[CC / 4], bv[CC / 4][NJ];
#pragma unroll
      for (int ks = 0; ks < CC / 4; ++ks) {
        const int row = 4 * ks + kr;
        a[ks] = sL[row * LP + 16 * wave + jj];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[ks][j] = sR[row * RP + 16 * wave + jj + 16 * (NJ - 1 - j)];
      }
#pragma unroll
      for (int ks = 0; ks < CC / 4; ++ks)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x16x4(a[ks], bv[ks][j], acc[j]);
    }
    if (s + 1 < NST) store((s + 1) % PD, (s + 1) & 1);
    __syncthreads();
  }

  float *sO = smem + 15 * OUTP;
  const float invC = 1.f / (float)C;
  const int dmax = min(dchunk, D - d0);
  float *sOl = sO + (4 * kr - jj) * OUTP + 16 * wave + 4 * kr;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) sOl[(16 * j + r) * OUTP + r] = acc[j][r] * invC;
  __syncthreads();
  for (int e = tid; e < dmax * (TX / 4); e += NT) {
    const int dl = e / (TX / 4), xq = e % (TX / 4);
    if (x0 + 4 * xq < W) {
      const float *src = sO + dl * OUTP + 4 * xq;
      f32x4 v = f32x4{src[0], src[1], src[2], src[3]};
      f32x4 *dst = reinterpret_cast<f32x4 *>(out + (((long)b * D + d0 + dl) * H + y) * W + x0 + 4 * xq);
      if (POL & 2) __builtin_nontemporal_store(v, dst); else *dst = v;
    }
  }
}

template <int NJ, int CC, int NST, int PD, int POL = 0>
void launch_v2(const float *L, const float *R, float *out, int n, int h, int w, int D) {
  const int dchunk = 16 * (NJ - 1) + 1 > 64 ? 64 : 16 * (NJ - 1) + 1;
  const int nchunks = (D + dchunk - 1) / dchunk, ntx = (w + TX - 1) / TX;
  const int nblk = ntx * nchunks * h * n;
  hipLaunchKernelGGL((corr_v2<NJ, CC, NST, PD, POL>), dim3(nblk), dim3(NT), 0, 0, L, R, out, h, w, D, dchunk,
                     ntx, nchunks);
}

__global__ void fill(float *p, long n, unsigned seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((float)(x & 0xffffff) / 16777216.f - 0.5f) * 3.f;
  }
}

}  // namespace lab

int main(int argc, char **argv) {
  const int B = 8, C = 128, H = 128, W = 416, D = 64;
  const long nin = (long)B * C * H * W, nout = (long)B * D * H * W;
  float *L, *R, *o_ref, *o;
  CHECK(hipMalloc(&L, nin * 4));
  CHECK(hipMalloc(&R, nin * 4));
  CHECK(hipMalloc(&o_ref, nout * 4));
  CHECK(hipMalloc(&o, nout * 4));
  hipLaunchKernelGGL(lab::fill, dim3(4096), dim3(256), 0, 0, L, nin, 1u);
  hipLaunchKernelGGL(lab::fill, dim3(4096), dim3(256), 0, 0, R, nin, 2u);
  if (aanet_corr_volume_f32(L, R, o_ref, B, C, H, W, D, 0)) { printf("product launch failed\n"); return 1; }
  CHECK(hipDeviceSynchronize());
  std::vector<float> h_ref(nout), h(nout);
  CHECK(hipMemcpy(h_ref.data(), o_ref, nout * 4, hipMemcpyDeviceToHost));

  struct V { const char *name; void (*fn)(const float *, const float *, float *); };
  std::vector<V> vs = {
      {"product", [](const float *l, const float *r, float *out) { aanet_corr_volume_f32(l, r, out, 8, 128, 128, 416, 64, 0); }},
      {"v2 pd2", [](const float *l, const float *r, float *out) { lab::launch_v2<5, 16, 8, 2>(l, r, out, 8, 128, 416, 64); }},
      {"v2 pd2 ntLS", [](const float *l, const float *r, float *out) { lab::launch_v2<5, 16, 8, 2, 3>(l, r, out, 8, 128, 416, 64); }},
  };
  const double bytes = 4.0 * (2.0 * nin + nout);
  for (auto &v : vs) {
    CHECK(hipMemset(o, 0xff, nout * 4));
    v.fn(L, R, o);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), o, nout * 4, hipMemcpyDeviceToHost));
    double md = 0;
    for (long i = 0; i < nout; ++i) md = std::max(md, (double)std::fabs(h[i] - h_ref[i]));
    printf("%-14s maxdiff %.3g\n", v.name, md);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = argc > 1 ? atoi(argv[1]) : 30;
  for (int round = 0; round < 3; ++round)
    for (auto &v : vs) {
      v.fn(L, R, o);
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) v.fn(L, R, o);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / iters;
      printf("round %d %-14s %8.1f us  %6.0f GB/s\n", round, v.name, us, bytes / us / 1e3);
    }
  return 0;
}
