// regress_lab.hip -- same-process A/B of soft-argmin regression variants (a probe, not product
// code).  Includes the product kernel as the baseline; C2 scale-0 shape [8,64,128,416].
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/regress_lab.hip -o tools/regress_lab.bin
#include "../aanet_amd/csrc/regression.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t err_ = (x);                                                    \
    if (err_ != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__);     \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

namespace lab {
// all DT values of a pixel loaded up front (DT loads in flight per lane), then max / exp-sum
template <int DT, int NT_LOAD>
__global__ __launch_bounds__(256) void reg_fixed(const float *__restrict__ cost, float *__restrict__ disp,
                                                 int HW, int total, float sign) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int b = e / HW, p = e - b * HW;
  const float *c = cost + (long)b * DT * HW + p;
  float s[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) s[d] = NT_LOAD ? __builtin_nontemporal_load(c + (long)d * HW) : c[(long)d * HW];
  float m = sign * s[0];
#pragma unroll
  for (int d = 1; d < DT; ++d) m = fmaxf(m, sign * s[d]);
  float z = 0.f, acc = 0.f;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const float ev = __expf(sign * s[d] - m);
    z += ev;
    acc += ev * (float)d;
  }
  disp[e] = acc / z;
}

__global__ void fill(float *p, long n, unsigned seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = ((float)(x & 0xffffff) / 16777216.f - 0.5f) * 6.f;
  }
}
}  // namespace lab

int main(int argc, char **argv) {
  const int B = 8, D = 64, H = 128, W = 416, HW = H * W, total = B * HW;
  const long nin = (long)B * D * HW;
  float *cost, *big, *o_ref, *o;
  CHECK(hipMalloc(&cost, nin * 4));
  CHECK(hipMalloc(&big, 512l << 20));  // evicts the Infinity Cache between launches ("cold")
  CHECK(hipMalloc(&o_ref, total * 4));
  CHECK(hipMalloc(&o, total * 4));
  hipLaunchKernelGGL(lab::fill, dim3(4096), dim3(256), 0, 0, cost, nin, 1u);
  if (aanet_disp_regress_f32(cost, o_ref, B, D, H, W, 0, 0)) return 1;
  CHECK(hipDeviceSynchronize());
  std::vector<float> h_ref(total), h(total);
  CHECK(hipMemcpy(h_ref.data(), o_ref, total * 4, hipMemcpyDeviceToHost));
  struct V { const char *name; void (*fn)(const float *, float *); };
  std::vector<V> vs = {
      {"product", [](const float *c, float *out) { aanet_disp_regress_f32(c, out, 8, 64, 128, 416, 0, 0); }},
      {"fixed64", [](const float *c, float *out) { hipLaunchKernelGGL((lab::reg_fixed<64, 0>), dim3(8 * 128 * 416 / 256), dim3(256), 0, 0, c, out, 128 * 416, 8 * 128 * 416, 1.f); }},
      {"fixed64 nt", [](const float *c, float *out) { hipLaunchKernelGGL((lab::reg_fixed<64, 1>), dim3(8 * 128 * 416 / 256), dim3(256), 0, 0, c, out, 128 * 416, 8 * 128 * 416, 1.f); }},
  };
  for (auto &v : vs) {
    v.fn(cost, o);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h.data(), o, total * 4, hipMemcpyDeviceToHost));
    double md = 0;
    for (int i = 0; i < total; ++i) md = std::max(md, (double)std::fabs(h[i] - h_ref[i]));
    printf("%-12s maxdiff %.3g\n", v.name, md);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 4.0 * (nin + total);
  for (int cold = 0; cold < 2; ++cold)
    for (int round = 0; round < 3; ++round)
      for (auto &v : vs) {
        float tot = 0;
        const int iters = 20;
        for (int i = 0; i < iters; ++i) {
          if (cold) CHECK(hipMemsetAsync(big, i, 512l << 20, 0));
          CHECK(hipEventRecord(e0, 0));
          v.fn(cost, o);
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          float ms;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          tot += ms;
        }
        const double us = 1e3 * tot / iters;
        printf("%s round %d %-12s %7.1f us  %6.0f GB/s\n", cold ? "cold" : "warm", round, v.name, us, bytes / us / 1e3);
      }
  return 0;
}
