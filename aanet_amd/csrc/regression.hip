// regression.hip -- fused soft-argmin disparity regression (replaces nets/estimation.py:13-30).
//
// disp[b,y,x] = sum_d d * softmax_d(s),  s = negate ? -cost : cost.
// The reference makes ~5 passes over [D,H,W] (softmax, arange, mul, sum).  Here one thread
// owns one pixel and streams its D values once (coalesced across the wave along x): HBM
// traffic = read D*H*W + write H*W.
#include "common.h"

namespace {

constexpr int RB = 256;

// D known at compile time (AANet's pyramid: 64 / 32 / 16): all D loads of a pixel are issued up
// front (D loads in flight per lane), then max, then one exp-sum pass.  The volume is read once:
// non-temporal loads (tools/regress_lab.hip: 26.2 -> 20.2 us at [8,64,128,416], and 47 -> 23 us
// when the volume is not resident in the Infinity Cache).
template <int DT>
__global__ __launch_bounds__(RB) void disp_regress_fixed_kernel(const float *__restrict__ cost,
                                                                float *__restrict__ disp, int HW,
                                                                int total, float sign) {
  const int e = blockIdx.x * RB + threadIdx.x;
  if (e >= total) return;
  const int b = e / HW, p = e - b * HW;
  const float *c = cost + (long)b * DT * HW + p;
  float s[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) s[d] = sign * __builtin_nontemporal_load(c + (long)d * HW);
  float m = s[0];
#pragma unroll
  for (int d = 1; d < DT; ++d) m = fmaxf(m, s[d]);
  float z = 0.f, acc = 0.f;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const float ev = __expf(s[d] - m);
    z += ev;
    acc += ev * (float)d;
  }
  disp[e] = acc / z;
}

// Any D: chunks of CH disparities, the next chunk's loads issued before the current chunk is
// reduced; online max / normaliser / weighted sum across chunks.
constexpr int CH = 16;
__global__ __launch_bounds__(RB) void disp_regress_kernel(const float *__restrict__ cost,
                                                          float *__restrict__ disp, int D,
                                                          long HW, long total, float sign) {
  const long e = (long)blockIdx.x * RB + threadIdx.x;
  if (e >= total) return;
  const long b = e / HW, p = e % HW;
  const float *c = cost + b * D * HW + p;
  auto load = [&](float (&v)[CH], int d0) {
#pragma unroll
    for (int u = 0; u < CH; ++u)
      v[u] = (d0 + u < D) ? sign * __builtin_nontemporal_load(c + (long)(d0 + u) * HW) : -INFINITY;
  };
  float cur[CH], nxt[CH];
  load(cur, 0);
  float m = -INFINITY, z = 0.f, acc = 0.f;
  for (int d0 = 0; d0 < D; d0 += CH) {
    if (d0 + CH < D) load(nxt, d0 + CH);
    float cm = cur[0];
#pragma unroll
    for (int u = 1; u < CH; ++u) cm = fmaxf(cm, cur[u]);
    if (cm > m) {
      const float sc = __expf(m - cm);  // 0 on the first chunk (m = -inf)
      z *= sc;
      acc *= sc;
      m = cm;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const float ev = __expf(cur[u] - m);  // 0 for padded lanes (s = -inf)
      z += ev;
      acc += ev * (float)(d0 + u);
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) cur[u] = nxt[u];
  }
  disp[e] = acc / z;
}

__global__ __launch_bounds__(RB) void disp_regress_bwd_kernel(const float *__restrict__ cost,
                                                              const float *__restrict__ gdisp,
                                                              float *__restrict__ gcost, int D,
                                                              long HW, long total, float sign) {
  const long e = (long)blockIdx.x * RB + threadIdx.x;
  if (e >= total) return;
  const long b = e / HW, p = e % HW;
  const float *c = cost + b * D * HW + p;
  float m = -INFINITY;
  for (int d = 0; d < D; ++d) m = fmaxf(m, sign * c[(long)d * HW]);
  float z = 0.f, acc = 0.f;
  for (int d = 0; d < D; ++d) {
    const float ev = expf(sign * c[(long)d * HW] - m);
    z += ev;
    acc += ev * (float)d;
  }
  const float inv = 1.f / z, mu = acc * inv, g = gdisp[e];
  float *gc = gcost + b * D * HW + p;
  for (int d = 0; d < D; ++d) {
    const float pr = expf(sign * c[(long)d * HW] - m) * inv;
    gc[(long)d * HW] = sign * g * pr * ((float)d - mu);
  }
}

}  // namespace

extern "C" int aanet_disp_regress_f32(const float *cost, float *disp, int n, int d, int h, int w,
                                      int negate, aanet_stream_t stream) {
  AANET_HOST_CHECK(cost && disp && n > 0 && d > 0 && h > 0 && w > 0);
  const long HW = (long)h * w, total = (long)n * HW;
  const float sign = negate ? -1.f : 1.f;
  const dim3 grid(host_div_up(total, RB));
  hipStream_t st = as_hip(stream);
  if (total * d < 0x7fffffffL && (d == 64 || d == 32 || d == 16)) {
    if (d == 64)
      hipLaunchKernelGGL(disp_regress_fixed_kernel<64>, grid, dim3(RB), 0, st, cost, disp, (int)HW, (int)total, sign);
    else if (d == 32)
      hipLaunchKernelGGL(disp_regress_fixed_kernel<32>, grid, dim3(RB), 0, st, cost, disp, (int)HW, (int)total, sign);
    else
      hipLaunchKernelGGL(disp_regress_fixed_kernel<16>, grid, dim3(RB), 0, st, cost, disp, (int)HW, (int)total, sign);
  } else {
    hipLaunchKernelGGL(disp_regress_kernel, grid, dim3(RB), 0, st, cost, disp, d, HW, total, sign);
  }
  return aanet_launch_status();
}

extern "C" int aanet_disp_regress_bwd_f32(const float *cost, const float *grad_disp,
                                          float *grad_cost, int n, int d, int h, int w,
                                          int negate, aanet_stream_t stream) {
  AANET_HOST_CHECK(cost && grad_disp && grad_cost && n > 0 && d > 0 && h > 0 && w > 0);
  const long HW = (long)h * w, total = (long)n * HW;
  hipLaunchKernelGGL(disp_regress_bwd_kernel, dim3(host_div_up(total, RB)), dim3(RB), 0,
                     as_hip(stream), cost, grad_disp, grad_cost, d, HW, total,
                     negate ? -1.f : 1.f);
  return aanet_launch_status();
}
