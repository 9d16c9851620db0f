// split_lab.hip -- probe (not product code): can an fp32 3x3 convolution run faster on the bf16
// matrix cores with operands split into bf16 pieces (x = h + m + l, fp32 accumulation), at fp32
// accuracy?  NPROD = 6 keeps the products down to 2^-16 (hh, hm, mh, hl, lh, mm); NPROD = 9 keeps
// all of them (every product exact, only the fp32 accumulation order differs from a fma chain).
// Compared against the product engine (exact f32 MFMA) and an fp64 reference, C2 scale-0 shape:
// x NHWC [8][128][416][64], w [64][64][3][3], pad 1 -> out NCHW [8][64][128][416].
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/split_lab.hip -Laanet_amd -laanet_mi355x
//        -Wl,-rpath,'$ORIGIN/../aanet_amd' -o tools/split_lab.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/aanet_mi355x.h"

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace lab {
constexpr int N = 8, C = 64, H = 128, W = 416, CO = 64, P = H * W;
constexpr int PTT = 128, NT = 512, CK = 32, NCH = 18;  // 9 taps x 2 channel halves
constexpr int BP = 40;                                 // bf16 pitch of a pixel row (80 B)
constexpr int PIECE = PTT * BP;                        // bf16 per piece plane
constexpr int BUF = 3 * PIECE;

__device__ inline void split3(f32x4 v, bf16x4 &h, bf16x4 &m, bf16x4 &l) {
  h = __builtin_convertvector(v, bf16x4);
  const f32x4 r = v - __builtin_convertvector(h, f32x4);
  m = __builtin_convertvector(r, bf16x4);
  const f32x4 r2 = r - __builtin_convertvector(m, f32x4);
  l = __builtin_convertvector(r2, bf16x4);
}

// weights [co][c][3][3] fp32 -> fragments Wf[chunk][piece][blk][lane][8] (chunk = tap*2 + half)
__global__ void prep_w(const float *__restrict__ w, bf16x8 *__restrict__ wf) {
  const int t = blockIdx.x * 256 + threadIdx.x;  // (chunk, blk, lane)
  if (t >= NCH * 4 * 64) return;
  const int lane = t & 63, blk = (t >> 6) & 3, chunk = t >> 8;
  const int tap = chunk >> 1, half = chunk & 1;
  const int co = 16 * blk + (lane & 15);
  bf16x8 hp, mp, lp;
  for (int j = 0; j < 8; ++j) {
    const int c = 32 * half + 8 * (lane >> 4) + j;
    const float v = w[(co * C + c) * 9 + tap];
    const __bf16 h = (__bf16)v;
    const float r = v - (float)h;
    const __bf16 m = (__bf16)r;
    const __bf16 l = (__bf16)(r - (float)m);
    hp[j] = h; mp[j] = m; lp[j] = l;
  }
  wf[((chunk * 3 + 0) * 4 + blk) * 64 + lane] = hp;
  wf[((chunk * 3 + 1) * 4 + blk) * 64 + lane] = mp;
  wf[((chunk * 3 + 2) * 4 + blk) * 64 + lane] = lp;
}

template <int NPROD>
__global__ __launch_bounds__(NT, 2) void conv_split(const float *__restrict__ x, const bf16x8 *__restrict__ wf,
                                                    float *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  constexpr int ntiles = P / PTT;
  const int n = bid / ntiles, tile = bid % ntiles;
  const int wc = wave >> 2, wp = wave & 3;  // 2 (co) x 4 (px) waves; wave tile 32 co x 32 px
  const int kr = lane >> 4, jj = lane & 15;
  // staging: item i -> pixel tid/8 + 64 i, quad nq = tid & 7 (channels 4nq..4nq+3 of the chunk)
  const int nq = tid & 7;
  int ho[2], wo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = tile * PTT + (tid >> 3) + 64 * i;
    ho[i] = p / W;
    wo[i] = p % W;
  }
  const int img_bytes = H * W * C * 4;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void *)(x + (long)n * H * W * C), (short)0, img_bytes, 0x00020000);
  f32x4 braw[2];
  bf16x8 afr[2][2][3];  // [set][m][piece]
  auto load_b = [&](int chunk) {
    const int tap = chunk >> 1, half = chunk & 1;
    const int di = tap / 3 - 1, dj = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int hi = ho[i] + di, wi = wo[i] + dj;
      const bool ok = hi >= 0 && hi < H && wi >= 0 && wi < W;
      const int off = ok ? ((hi * W + wi) * C + 32 * half + 4 * nq) * 4 : img_bytes;
      braw[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto load_a = [&](int chunk, int set) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc) afr[set][m][pc] = wf[((chunk * 3 + pc) * 4 + 2 * wc + m) * 64 + lane];
  };
  auto store_b = [&](int buf) {
    __bf16 *s = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x4 h, m, l;
      split3(braw[i], h, m, l);
      const int px = (tid >> 3) + 64 * i;
      *reinterpret_cast<bf16x4 *>(s + 0 * PIECE + px * BP + 4 * nq) = h;
      *reinterpret_cast<bf16x4 *>(s + 1 * PIECE + px * BP + 4 * nq) = m;
      *reinterpret_cast<bf16x4 *>(s + 2 * PIECE + px * BP + 4 * nq) = l;
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[m][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf, int set) {
    const __bf16 *s = smem + buf * BUF;
    bf16x8 bfr[2][3];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
        bfr[b][pc] = *reinterpret_cast<const bf16x8 *>(s + pc * PIECE + (32 * wp + 16 * b + jj) * BP + 8 * kr);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const bf16x8 *A = afr[set][m], *B = bfr[b];
        f32x4 t = acc[m][b];
        if (NPROD == 9) {
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[1], t, 0, 0, 0);
        }
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], t, 0, 0, 0);
        acc[m][b] = t;
      }
  };
  load_a(0, 0);
  load_b(0);
  store_b(0);
  __syncthreads();
  for (int c = 0; c < NCH; c += 2) {
    // even chunk: A set 0, LDS buffer 0
    load_a(c + 1, 1);
    load_b(c + 1);
    compute(0, 0);
    store_b(1);
    __syncthreads();
    // odd chunk: A set 1, LDS buffer 1
    if (c + 2 < NCH) {
      load_a(c + 2, 0);
      load_b(c + 2);
    }
    compute(1, 1);
    if (c + 2 < NCH) store_b(0);
    __syncthreads();
  }
  // epilogue: D col = px (lane & 15), rows co 4kr + r
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = 32 * wc + 16 * m + 4 * kr + r;
        const int p = tile * PTT + 32 * wp + 16 * b + jj;
        out[((long)n * CO + co) * P + p] = acc[m][b][r];
      }
}

// fp64 reference + the scale sum |x||w| per output
__global__ void ref64(const float *__restrict__ x, const float *__restrict__ w, double *__restrict__ out,
                      double *__restrict__ scale) {
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= (long)N * CO * P) return;
  const int p = t % P, co = (t / P) % CO, n = t / ((long)P * CO);
  const int ho = p / W, wo = p % W;
  double s = 0, a = 0;
  for (int tap = 0; tap < 9; ++tap) {
    const int hi = ho + tap / 3 - 1, wi = wo + tap % 3 - 1;
    if (hi < 0 || hi >= H || wi < 0 || wi >= W) continue;
    const float *xp = x + (((long)n * H + hi) * W + wi) * C;
    for (int c = 0; c < C; ++c) {
      const double v = (double)xp[c] * (double)w[(co * C + c) * 9 + tap];
      s += v;
      a += fabs(v);
    }
  }
  out[t] = s;
  scale[t] = a;
}

__global__ void fill(float *p, long n, unsigned seed, float amp) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned v = (unsigned)i * 2654435761u ^ seed;
    v ^= v >> 13; v *= 0x5bd1e995u; v ^= v >> 15;
    p[i] = ((float)(v & 0xffffff) / 16777216.f - 0.5f) * amp;
  }
}
}  // namespace lab

int main() {
  using namespace lab;
  const long nx = (long)N * H * W * C, nw = (long)CO * C * 9, no = (long)N * CO * P;
  float *x, *w, *wp, *o;
  bf16x8 *wf;
  double *r64, *sc;
  CHECK(hipMalloc(&x, nx * 4));
  CHECK(hipMalloc(&w, nw * 4));
  CHECK(hipMalloc(&wp, nw * 4));
  CHECK(hipMalloc(&wf, NCH * 3 * 4 * 64 * 16));
  CHECK(hipMalloc(&o, no * 4));
  CHECK(hipMalloc(&r64, no * 8));
  CHECK(hipMalloc(&sc, no * 8));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, x, nx, 1u, 4.f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, w, nw, 2u, 0.2f);
  hipLaunchKernelGGL(ref64, dim3((no + 255) / 256), dim3(256), 0, 0, x, w, r64, sc);
  hipLaunchKernelGGL(prep_w, dim3((NCH * 256 + 255) / 256), dim3(256), 0, 0, w, wf);
  if (aanet_conv_weight_pack_f32(w, wp, CO, C, 3, 3, 0)) return 1;
  CHECK(hipDeviceSynchronize());
  std::vector<double> hr(no), hs(no);
  std::vector<float> ho(no);
  CHECK(hipMemcpy(hr.data(), r64, no * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hs.data(), sc, no * 8, hipMemcpyDeviceToHost));
  struct V { const char *name; void (*fn)(const float *, const float *, const bf16x8 *, float *); };
  std::vector<V> vs = {
      {"f32 engine", [](const float *x, const float *wp, const bf16x8 *, float *o) {
         aanet_conv2d_fused_f32(x, wp, nullptr, nullptr, nullptr, nullptr, 0, 1, o, N, C, H, W, CO, 3, 3, 1, 1, 1, 1,
                                AANET_LAYOUT_IN_NHWC, 0); }},
      {"bf16x6", [](const float *x, const float *, const bf16x8 *wf, float *o) {
         hipLaunchKernelGGL(conv_split<6>, dim3(N * P / PTT), dim3(NT), 0, 0, x, wf, o); }},
      {"bf16x9", [](const float *x, const float *, const bf16x8 *wf, float *o) {
         hipLaunchKernelGGL(conv_split<9>, dim3(N * P / PTT), dim3(NT), 0, 0, x, wf, o); }},
  };
  for (auto &v : vs) {
    CHECK(hipMemset(o, 0, no * 4));
    v.fn(x, wp, wf, o);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(ho.data(), o, no * 4, hipMemcpyDeviceToHost));
    double maxe = 0, maxrel = 0, sume = 0;
    for (long i = 0; i < no; ++i) {
      const double e = fabs((double)ho[i] - hr[i]);
      maxe = std::max(maxe, e);
      maxrel = std::max(maxrel, e / (hs[i] + 1e-30));
      sume += e;
    }
    printf("%-11s max|err| %.3e  mean|err| %.3e  max err/sum|xw| %.3e\n", v.name, maxe, sume / no, maxrel);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double flops = 2.0 * N * P * CO * C * 9;
  for (int round = 0; round < 3; ++round)
    for (auto &v : vs) {
      v.fn(x, wp, wf, o);
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) v.fn(x, wp, wf, o);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / 20;
      printf("round %d %-11s %7.1f us  %6.1f TF/s (fp32-equivalent)\n", round, v.name, us, flops / us / 1e6);
    }
  return 0;
}
