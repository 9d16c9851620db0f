// Which fp-contraction pattern reproduces torch's upsample_bilinear2d_out_frame bits?
// Variants of the resize forward, launched through ctypes by tools/resize_lab.py.
#include <hip/hip_runtime.h>
template <int V>
__global__ void rz(const float *x, float *y, long planes, int ih, int iw, int oh, int ow, float sh, float sw) {
  const long total = planes * oh * ow;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % ow);
    const long t = e / ow;
    const int oy = (int)(t % oh);
    const long plane = t / oh;
    float ry, rx;
    if constexpr (V & 1) {
      ry = __builtin_fmaf(sh, (float)oy + 0.5f, -0.5f);
      rx = __builtin_fmaf(sw, (float)ox + 0.5f, -0.5f);
    } else {
#pragma clang fp contract(off)
      ry = sh * ((float)oy + 0.5f) - 0.5f;
      rx = sw * ((float)ox + 0.5f) - 0.5f;
    }
    ry = ry < 0.f ? 0.f : ry;
    rx = rx < 0.f ? 0.f : rx;
    const int y1 = (int)ry, x1 = (int)rx;
    const int y1p = y1 < ih - 1 ? iw : 0, x1p = x1 < iw - 1 ? 1 : 0;
    const float ly1 = ry - (float)y1, ly0 = 1.f - ly1, lx1 = rx - (float)x1, lx0 = 1.f - lx1;
    const float *p = x + plane * ih * iw + (long)y1 * iw + x1;
    const float a = p[0], b = p[x1p], c = p[y1p], d = p[y1p + x1p];
    float v;
    if constexpr ((V >> 1) == 0) {  // no contraction
#pragma clang fp contract(off)
      v = ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * c + lx1 * d);
    } else if constexpr ((V >> 1) == 1) {  // left products fused
      v = __builtin_fmaf(ly0, __builtin_fmaf(lx0, a, lx1 * b), ly1 * __builtin_fmaf(lx0, c, lx1 * d));
    } else if constexpr ((V >> 1) == 2) {  // right products fused
      v = __builtin_fmaf(ly1, __builtin_fmaf(lx1, d, lx0 * c), ly0 * __builtin_fmaf(lx1, b, lx0 * a));
    } else if constexpr ((V >> 1) == 3) {  // inner left, outer right
      v = __builtin_fmaf(ly1, __builtin_fmaf(lx0, c, lx1 * d), ly0 * __builtin_fmaf(lx0, a, lx1 * b));
    } else {  // inner right, outer left
      v = __builtin_fmaf(ly0, __builtin_fmaf(lx1, b, lx0 * a), ly1 * __builtin_fmaf(lx1, d, lx0 * c));
    }
    y[e] = v;
  }
}
extern "C" int lab(int V, const float *x, float *y, long planes, int ih, int iw, int oh, int ow) {
  const float sh = (float)ih / (float)oh, sw = (float)iw / (float)ow;
  const dim3 g(1024), b(256);
  switch (V) {
#define C(v) case v: hipLaunchKernelGGL(rz<v>, g, b, 0, 0, x, y, planes, ih, iw, oh, ow, sh, sw); break;
    C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9)
  }
  return (int)hipDeviceSynchronize();
}
