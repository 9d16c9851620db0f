// regression.hip -- fused soft-argmin disparity regression (replaces nets/estimation.py:13-30).
//
// disp[b,y,x] = sum_d d * softmax_d(s),  s = negate ? -cost : cost.
// The reference makes ~5 passes over [D,H,W] (softmax, arange, mul, sum).  Here one thread
// owns one pixel and streams its D values once (coalesced across the wave along x), keeping
// an online max / normaliser / weighted sum: HBM traffic = read D*H*W + write H*W.
#include "common.h"

namespace {

constexpr int RB = 256;
constexpr int UNR = 8;

__global__ __launch_bounds__(RB) void disp_regress_kernel(const float *__restrict__ cost,
                                                          float *__restrict__ disp, int D,
                                                          long HW, long total, float sign) {
  const long e = (long)blockIdx.x * RB + threadIdx.x;
  if (e >= total) return;
  const long b = e / HW, p = e % HW;
  const float *c = cost + b * D * HW + p;
  float m = -INFINITY, z = 0.f, acc = 0.f;
  for (int d0 = 0; d0 < D; d0 += UNR) {
    float s[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) s[u] = (d0 + u < D) ? sign * c[(long)(d0 + u) * HW] : -INFINITY;
    float cm = s[0];
#pragma unroll
    for (int u = 1; u < UNR; ++u) cm = fmaxf(cm, s[u]);
    if (cm > m) {
      const float sc = __expf(m - cm);  // 0 on the first chunk (m = -inf)
      z *= sc;
      acc *= sc;
      m = cm;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const float ev = __expf(s[u] - m);  // 0 for padded lanes (s = -inf)
      z += ev;
      acc += ev * (float)(d0 + u);
    }
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
  hipLaunchKernelGGL(disp_regress_kernel, dim3(host_div_up(total, RB)), dim3(RB), 0,
                     as_hip(stream), cost, disp, d, HW, total, negate ? -1.f : 1.f);
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
