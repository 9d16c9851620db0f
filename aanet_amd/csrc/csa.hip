// csa.hip -- cross-scale aggregation sum for gfx950 (replaces nets/aggregation.py:387-400 in the
// eval path): out = act(e_0 + up(e_1) + ... ), where every e_j whose spatial size differs from
// the output is bilinearly resized with PyTorch's align_corners=False rule
// (F.interpolate(..., mode='bilinear', align_corners=False), aggregation.py:395-396).
// One pass: each output element reads its same-size term once and 4 taps of each resized term,
// instead of the reference's separate interpolate / add / add / LeakyReLU kernels.
#include "common.h"

namespace {

constexpr int MAXIN = 4;

struct CsaArgs {
  const float *in[MAXIN];
  int ih[MAXIN], iw[MAXIN];
  float sh[MAXIN], sw[MAXIN];  // input/output size ratios (area_pixel_compute_scale)
  int num;
  float *out;
  int N, C, H, W, act;
};

// PyTorch upsample_bilinear2d, align_corners=False: src = scale*(dst+0.5)-0.5, clamped at 0;
// i1 = (int)src; i1p = i1 < in-1; lambda = src - i1.
__device__ __forceinline__ float bilinear_resize(const float *__restrict__ im, int ih, int iw,
                                                 float sh, float sw, int y, int x) {
  float hr = sh * ((float)y + 0.5f) - 0.5f;
  hr = hr < 0.f ? 0.f : hr;
  float wr = sw * ((float)x + 0.5f) - 0.5f;
  wr = wr < 0.f ? 0.f : wr;
  const int h1 = (int)hr, w1 = (int)wr;
  const int h1p = h1 < ih - 1 ? 1 : 0, w1p = w1 < iw - 1 ? 1 : 0;
  const float h1l = hr - (float)h1, h0l = 1.f - h1l;
  const float w1l = wr - (float)w1, w0l = 1.f - w1l;
  const float *r0 = im + (long)h1 * iw, *r1 = im + (long)(h1 + h1p) * iw;
  return h0l * (w0l * r0[w1] + w1l * r0[w1 + w1p]) + h1l * (w0l * r1[w1] + w1l * r1[w1 + w1p]);
}

// One thread = 4 consecutive output columns: the same-size term is read and the result written
// as float4; resized terms (1/2, 1/4 resolution, L2-resident) are gathered per element.
__global__ __launch_bounds__(256) void csa_sum_kernel(CsaArgs a) {
  const int W4 = a.W >> 2;
  const int HW = a.H * a.W;
  const long total = (long)a.N * a.C * a.H * W4;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int xq = (int)(e % W4);
    const long rowid = e / W4;             // (plane, y)
    const int y = (int)(rowid % a.H);
    const long plane = rowid / a.H;
    const long base = plane * HW + (long)y * a.W + 4 * xq;
    f32x4 acc;
#pragma unroll
    for (int j = 0; j < MAXIN; ++j) {
      if (j >= a.num) break;
      f32x4 v;
      if (a.ih[j] == a.H && a.iw[j] == a.W) {
        v = *reinterpret_cast<const f32x4 *>(a.in[j] + base);
      } else {
        const float *im = a.in[j] + plane * a.ih[j] * a.iw[j];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          v[u] = bilinear_resize(im, a.ih[j], a.iw[j], a.sh[j], a.sw[j], y, 4 * xq + u);
      }
      acc = j == 0 ? v : acc + v;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (a.act == 1) acc[u] = acc[u] > 0.f ? acc[u] : 0.f;
      if (a.act == 2) acc[u] = acc[u] > 0.f ? acc[u] : 0.2f * acc[u];
    }
    *reinterpret_cast<f32x4 *>(a.out + base) = acc;
  }
}

// Exact 2x / 4x upsampling (the AANet pyramid: 1/3 -> 1/6 -> 1/12): upsample_quad (common.h)
// reads one 16-byte source segment per row instead of four gathered dwords per output element.
__global__ __launch_bounds__(256) void csa_sum_int_kernel(CsaArgs a, int r0, int r1, int r2, int r3) {
  const int rr[MAXIN] = {r0, r1, r2, r3};
  const unsigned W4 = a.W >> 2, H = a.H;
  const unsigned total = (unsigned)a.N * a.C * a.H * W4;  // < 2^31 (checked by the launcher)
  for (unsigned e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    // 32-bit index math: 64-bit division is a long software sequence on the GPU
    const unsigned rowid = e / W4, q = e - rowid * W4;
    const unsigned plane = rowid / H, y = rowid - plane * H;
    const long base = (long)rowid * a.W + 4 * q;
    f32x4 acc;
#pragma unroll
    for (int j = 0; j < MAXIN; ++j) {
      if (j >= a.num) break;
      f32x4 v;
      const int r = rr[j];
      if (r == 1) {
        v = *reinterpret_cast<const f32x4 *>(a.in[j] + base);
      } else {
        const int ih = a.ih[j], iw = a.iw[j];
        v = upsample_quad(a.in[j] + (long)plane * ih * iw, ih, iw, a.sh[j], r, (int)y, (int)q);
      }
      acc = j == 0 ? v : acc + v;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (a.act == 1) acc[u] = acc[u] > 0.f ? acc[u] : 0.f;
      if (a.act == 2) acc[u] = acc[u] > 0.f ? acc[u] : 0.2f * acc[u];
    }
    *reinterpret_cast<f32x4 *>(a.out + base) = acc;
  }
}

__global__ __launch_bounds__(256) void csa_sum_scalar_kernel(CsaArgs a) {
  const long HW = (long)a.H * a.W;
  const long total = (long)a.N * a.C * HW;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long plane = e / HW;
    const int q = (int)(e % HW), y = q / a.W, x = q % a.W;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < MAXIN; ++j) {
      if (j >= a.num) break;
      float v;
      if (a.ih[j] == a.H && a.iw[j] == a.W) {
        v = a.in[j][e];
      } else {
        v = bilinear_resize(a.in[j] + plane * a.ih[j] * a.iw[j], a.ih[j], a.iw[j], a.sh[j],
                            a.sw[j], y, x);
      }
      acc = j == 0 ? v : acc + v;
    }
    if (a.act == 1) acc = acc > 0.f ? acc : 0.f;
    if (a.act == 2) acc = acc > 0.f ? acc : 0.2f * acc;
    a.out[e] = acc;
  }
}

// Weight of input index i in output index o along one axis (the align_corners=False rule of
// bilinear_resize): lambda0 if i is o's lower tap, lambda1 if its upper one (both at the edge).
__device__ __forceinline__ float bilinear_axis_weight(int o, int i, float s, int in) {
  float r = s * ((float)o + 0.5f) - 0.5f;
  r = r < 0.f ? 0.f : r;
  const int i1 = (int)r, i1p = i1 < in - 1 ? 1 : 0;
  const float l1 = r - (float)i1, l0 = 1.f - l1;
  return (i1 == i ? l0 : 0.f) + (i1 + i1p == i ? l1 : 0.f);
}

// Backward of the resize as a gather: each input element sums, in a fixed order, the output
// gradients of the outputs whose 2x2 stencil covers it (source coordinate in (i-1, i+1)).
// torch's CUDA backward scatters with atomics (and under deterministic algorithms falls back to a
// sort-based index_put); this form is bit-reproducible and atomic-free.
__global__ __launch_bounds__(256) void resize_bilinear_bwd_kernel(const float *__restrict__ go,
                                                                  float *__restrict__ gi,
                                                                  long planes, int ih, int iw,
                                                                  int oh, int ow, float sh,
                                                                  float sw) {
  const long total = planes * ih * iw;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int x = (int)(e % iw);
    const long t = e / iw;
    const int y = (int)(t % ih);
    const long plane = t / ih;
    const int ylo = max(0, (int)floorf(((float)y - 0.5f) / sh - 0.5f) - 1);
    const int yhi = min(oh - 1, (int)ceilf(((float)y + 1.5f) / sh - 0.5f) + 1);
    const int xlo = max(0, (int)floorf(((float)x - 0.5f) / sw - 0.5f) - 1);
    const int xhi = min(ow - 1, (int)ceilf(((float)x + 1.5f) / sw - 0.5f) + 1);
    const float *gp = go + plane * oh * ow;
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      const float wy = bilinear_axis_weight(oy, y, sh, ih);
      if (wy == 0.f) continue;
      float rs = 0.f;
      for (int ox = xlo; ox <= xhi; ++ox)
        rs += bilinear_axis_weight(ox, x, sw, iw) * gp[(long)oy * ow + ox];
      acc += wy * rs;
    }
    gi[e] = acc;
  }
}

// Forward of the resize (F.interpolate(mode='bilinear', align_corners=False) to a given size):
// one thread per output element, the 2x2 stencil of bilinear_axis_weight's rule, combined in the
// reference kernel's order (rows of the stencil first), bit-identical to torch's kernel.  torch's NCHW kernel gives one thread an
// output POSITION and loops over all N*C planes inside it: a 96x192 -> 288x576 resize of 4
// planes ran at 59 us, a few percent of HBM.
__global__ __launch_bounds__(256) void resize_bilinear_fwd_kernel(const float *__restrict__ x,
                                                                  float *__restrict__ y, long planes,
                                                                  int ih, int iw, int oh, int ow,
                                                                  float sh, float sw) {
  const long total = planes * oh * ow;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % ow);
    const long t = e / ow;
    const int oy = (int)(t % oh);
    const long plane = t / oh;
    // explicit FMAs: the contraction torch's kernel gets (tools/resize_lab.hip: bit-identical
    // for this form only; plain or differently fused expressions differ in 2-40% of the outputs)
    float ry = __builtin_fmaf(sh, (float)oy + 0.5f, -0.5f), rx = __builtin_fmaf(sw, (float)ox + 0.5f, -0.5f);
    ry = ry < 0.f ? 0.f : ry;
    rx = rx < 0.f ? 0.f : rx;
    const int y1 = (int)ry, x1 = (int)rx;
    const int y1p = y1 < ih - 1 ? iw : 0, x1p = x1 < iw - 1 ? 1 : 0;
    const float ly1 = ry - (float)y1, ly0 = 1.f - ly1, lx1 = rx - (float)x1, lx0 = 1.f - lx1;
    const float *p = x + plane * ih * iw + (long)y1 * iw + x1;
    y[e] = __builtin_fmaf(ly0, __builtin_fmaf(lx0, p[0], lx1 * p[x1p]),
                          ly1 * __builtin_fmaf(lx0, p[y1p], lx1 * p[y1p + x1p]));
  }
}

}  // namespace

extern "C" int aanet_resize_bilinear_bwd_f32(const float *grad_out, float *grad_in, long planes,
                                             int in_h, int in_w, int out_h, int out_w,
                                             aanet_stream_t stream) {
  AANET_HOST_CHECK(grad_out && grad_in && planes > 0 && in_h > 0 && in_w > 0 && out_h > 0 &&
                   out_w > 0);
  const long total = planes * in_h * in_w;
  long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(resize_bilinear_bwd_kernel, dim3((unsigned)g), dim3(256), 0, as_hip(stream),
                     grad_out, grad_in, planes, in_h, in_w, out_h, out_w,
                     (float)in_h / (float)out_h, (float)in_w / (float)out_w);
  return aanet_launch_status();
}

extern "C" int aanet_resize_bilinear_f32(const float *x, float *y, long planes, int in_h, int in_w,
                                         int out_h, int out_w, aanet_stream_t stream) {
  AANET_HOST_CHECK(x && y && planes > 0 && in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0);
  const long total = planes * out_h * out_w;
  long g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(resize_bilinear_fwd_kernel, dim3((unsigned)g), dim3(256), 0, as_hip(stream), x, y,
                     planes, in_h, in_w, out_h, out_w, (float)in_h / (float)out_h,
                     (float)in_w / (float)out_w);
  return aanet_launch_status();
}

extern "C" int aanet_csa_sum_f32(float *out, int n, int c, int h, int w, int num_inputs,
                                 const float *const *inputs, const int *in_h, const int *in_w,
                                 int act, aanet_stream_t stream) {
  AANET_HOST_CHECK(out && inputs && in_h && in_w && n > 0 && c > 0 && h > 0 && w > 0);
  AANET_HOST_CHECK(num_inputs >= 1 && num_inputs <= MAXIN && act >= 0 && act <= 2);
  CsaArgs a;
  for (int j = 0; j < MAXIN; ++j) {
    a.in[j] = j < num_inputs ? inputs[j] : nullptr;
    a.ih[j] = j < num_inputs ? in_h[j] : 1;
    a.iw[j] = j < num_inputs ? in_w[j] : 1;
    if (j < num_inputs && (!inputs[j] || in_h[j] <= 0 || in_w[j] <= 0)) return AANET_EINVAL;
    a.sh[j] = (float)a.ih[j] / (float)h;
    a.sw[j] = (float)a.iw[j] / (float)w;
  }
  a.num = num_inputs;
  a.out = out;
  a.N = n;
  a.C = c;
  a.H = h;
  a.W = w;
  a.act = act;
  bool vec = (w & 3) == 0;
  for (int j = 0; j < num_inputs; ++j)
    if (in_h[j] == h && in_w[j] == w && (reinterpret_cast<uintptr_t>(inputs[j]) & 15)) vec = false;
  if (reinterpret_cast<uintptr_t>(out) & 15) vec = false;
  const long total = (long)n * c * h * w / (vec ? 4 : 1);
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  // integer-ratio fast path: every resized input is exactly 2x or 4x smaller in both dims
  int rr[MAXIN] = {1, 1, 1, 1};
  bool integer = vec && (long)n * c * h * w < 0x7fffffffL;
  for (int j = 0; j < num_inputs && integer; ++j) {
    if (in_h[j] == h && in_w[j] == w) continue;
    const int r = h / in_h[j];
    integer = (r == 2 || r == 4) && in_h[j] * r == h && in_w[j] * r == w;
    rr[j] = r;
  }
  if (integer)
    hipLaunchKernelGGL(csa_sum_int_kernel, dim3((unsigned)g), dim3(256), 0, as_hip(stream), a,
                       rr[0], rr[1], rr[2], rr[3]);
  else if (vec)
    hipLaunchKernelGGL(csa_sum_kernel, dim3((unsigned)g), dim3(256), 0, as_hip(stream), a);
  else
    hipLaunchKernelGGL(csa_sum_scalar_kernel, dim3((unsigned)g), dim3(256), 0, as_hip(stream), a);
  return aanet_launch_status();
}
