// warp.hip -- disparity warp of the refinement path (replaces nets/warp.py:41-64, disp_warp).
//
// warped[b,c,y,x] = bilinear sample of img[b,c] at (x - disp[b,y,x], y), as the reference
// computes it: a pixel grid minus the disparity, normalised to [-1,1] (warp.py:5-16), then
// F.grid_sample(align_corners=True, padding 'border') -- which unnormalises straight back --
// plus a validity mask from grid_sample of ones with 'zeros' padding thresholded at 0.9999.
// The kernel keeps the same float steps (normalise, unnormalise, clip, floor, 4 corner weights
// in nw/ne/sw/se order) so the sample positions, and the rows the floor() picks, are the
// reference's.  One thread owns one output pixel: the coordinate work is done once and the
// C channels (3 for images) are streamed; rows are coalesced along x.
#include "common.h"

namespace {

constexpr int WB = 256;

struct WarpCoord {
  float ix, iy;   // source position (after the padding rule)
  int x0, y0;     // floor
  float wnw, wne, wsw, wse;
};

__device__ __forceinline__ float normalise(float g, int size) {
  return 2.f * (g / (float)(size - 1)) - 1.f;  // warp.py:12-13
}

__device__ __forceinline__ float unnormalise(float g, int size) {
  return ((g + 1.f) / 2.f) * (float)(size - 1);  // grid_sample, align_corners=True
}

__device__ __forceinline__ WarpCoord make_coord(float ix, float iy) {
  WarpCoord c;
  c.ix = ix;
  c.iy = iy;
  const float fx = floorf(ix), fy = floorf(iy);
  c.x0 = (int)fx;
  c.y0 = (int)fy;
  const float x1 = fx + 1.f, y1 = fy + 1.f;
  c.wnw = (x1 - ix) * (y1 - iy);
  c.wne = (ix - fx) * (y1 - iy);
  c.wsw = (x1 - ix) * (iy - fy);
  c.wse = (ix - fx) * (iy - fy);
  return c;
}

__device__ __forceinline__ bool inb(int y, int x, int H, int W) {
  return y >= 0 && y < H && x >= 0 && x < W;
}

__device__ __forceinline__ float sample(const float *__restrict__ im, const WarpCoord &c, int H,
                                        int W) {
  float acc = 0.f;
  if (inb(c.y0, c.x0, H, W)) acc += im[(long)c.y0 * W + c.x0] * c.wnw;
  if (inb(c.y0, c.x0 + 1, H, W)) acc += im[(long)c.y0 * W + c.x0 + 1] * c.wne;
  if (inb(c.y0 + 1, c.x0, H, W)) acc += im[(long)(c.y0 + 1) * W + c.x0] * c.wsw;
  if (inb(c.y0 + 1, c.x0 + 1, H, W)) acc += im[(long)(c.y0 + 1) * W + c.x0 + 1] * c.wse;
  return acc;
}

// border clip of grid_sample: min(size-1, max(v, 0)); the gradient passes only strictly inside
__device__ __forceinline__ float clip_border(float v, int size, float *dclip) {
  if (v <= 0.f) {
    *dclip = 0.f;
    return 0.f;
  }
  const float hi = (float)(size - 1);
  if (v >= hi) {
    *dclip = 0.f;
    return hi;
  }
  *dclip = 1.f;
  return v;
}

__global__ __launch_bounds__(WB) void disp_warp_kernel(const float *__restrict__ img,
                                                       const float *__restrict__ disp,
                                                       float *__restrict__ out,
                                                       float *__restrict__ valid, int C, int H,
                                                       int W, long total) {
  const long e = (long)blockIdx.x * WB + threadIdx.x;
  if (e >= total) return;
  const long HW = (long)H * W;
  const long b = e / HW, p = e % HW;
  const int y = (int)(p / W), x = (int)(p % W);
  const float gx = unnormalise(normalise((float)x - disp[e], W), W);
  const float gy = unnormalise(normalise((float)y, H), H);
  float dc;
  const WarpCoord cb = make_coord(clip_border(gx, W, &dc), clip_border(gy, H, &dc));
  const float *im = img + b * C * HW;
  float *o = out + b * C * HW + p;
  for (int c = 0; c < C; ++c) o[(long)c * HW] = sample(im + (long)c * HW, cb, H, W);
  if (valid) {
    // grid_sample(ones, padding 'zeros'): sum of the in-bounds corner weights (warp.py:60-63)
    const WarpCoord cz = make_coord(gx, gy);
    float m = 0.f;
    if (inb(cz.y0, cz.x0, H, W)) m += cz.wnw;
    if (inb(cz.y0, cz.x0 + 1, H, W)) m += cz.wne;
    if (inb(cz.y0 + 1, cz.x0, H, W)) m += cz.wsw;
    if (inb(cz.y0 + 1, cz.x0 + 1, H, W)) m += cz.wse;
    const float v = (m < 0.9999f) ? 0.f : (m > 0.f ? 1.f : m);
    float *vo = valid + b * C * HW + p;
    for (int c = 0; c < C; ++c) vo[(long)c * HW] = v;
  }
}

// Backward of the warped image w.r.t. the disparity (a gather: every pixel owns its own
// disparity) and, optionally, w.r.t. the image (scatter to the 4 corners, float atomics).
// d(ix)/d(disp) = -(W-1)/2 * 2/(W-1) * dclip: the reference's normalise/unnormalise chain.
__global__ __launch_bounds__(WB) void disp_warp_bwd_kernel(const float *__restrict__ img,
                                                           const float *__restrict__ disp,
                                                           const float *__restrict__ gout,
                                                           float *__restrict__ gdisp,
                                                           float *__restrict__ gimg, int C, int H,
                                                           int W, long total) {
  const long e = (long)blockIdx.x * WB + threadIdx.x;
  if (e >= total) return;
  const long HW = (long)H * W;
  const long b = e / HW, p = e % HW;
  const int y = (int)(p / W), x = (int)(p % W);
  const float gx = unnormalise(normalise((float)x - disp[e], W), W);
  const float gy = unnormalise(normalise((float)y, H), H);
  float dcx, dcy;
  const WarpCoord c = make_coord(clip_border(gx, W, &dcx), clip_border(gy, H, &dcy));
  const float *im = img + b * C * HW;
  const float *go = gout + b * C * HW + p;
  const float fy = (float)c.y0, fy1 = fy + 1.f;
  float gix = 0.f;
  for (int ch = 0; ch < C; ++ch) {
    const float g = go[(long)ch * HW];
    const float *imc = im + (long)ch * HW;
    const bool bnw = inb(c.y0, c.x0, H, W), bne = inb(c.y0, c.x0 + 1, H, W);
    const bool bsw = inb(c.y0 + 1, c.x0, H, W), bse = inb(c.y0 + 1, c.x0 + 1, H, W);
    const float vnw = bnw ? imc[(long)c.y0 * W + c.x0] : 0.f;
    const float vne = bne ? imc[(long)c.y0 * W + c.x0 + 1] : 0.f;
    const float vsw = bsw ? imc[(long)(c.y0 + 1) * W + c.x0] : 0.f;
    const float vse = bse ? imc[(long)(c.y0 + 1) * W + c.x0 + 1] : 0.f;
    gix -= vnw * (fy1 - c.iy) * g;
    gix += vne * (fy1 - c.iy) * g;
    gix -= vsw * (c.iy - fy) * g;
    gix += vse * (c.iy - fy) * g;
    if (gimg) {
      float *gi = gimg + b * C * HW + (long)ch * HW;
      if (bnw) atomicAdd(gi + (long)c.y0 * W + c.x0, c.wnw * g);
      if (bne) atomicAdd(gi + (long)c.y0 * W + c.x0 + 1, c.wne * g);
      if (bsw) atomicAdd(gi + (long)(c.y0 + 1) * W + c.x0, c.wsw * g);
      if (bse) atomicAdd(gi + (long)(c.y0 + 1) * W + c.x0 + 1, c.wse * g);
    }
  }
  const float half = (float)(W - 1) / 2.f, dn = 2.f / (float)(W - 1);
  gdisp[e] = -((gix * dcx) * half) * dn;
}

}  // namespace

extern "C" int aanet_disp_warp_f32(const float *img, const float *disp, float *warped,
                                   float *valid_mask, int n, int c, int h, int w,
                                   aanet_stream_t stream) {
  AANET_HOST_CHECK(img && disp && warped && n > 0 && c > 0 && h > 1 && w > 1);
  const long total = (long)n * h * w;
  hipLaunchKernelGGL(disp_warp_kernel, dim3(host_div_up(total, WB)), dim3(WB), 0, as_hip(stream),
                     img, disp, warped, valid_mask, c, h, w, total);
  return aanet_launch_status();
}

extern "C" int aanet_disp_warp_bwd_f32(const float *img, const float *disp,
                                       const float *grad_warped, float *grad_disp,
                                       float *grad_img, int n, int c, int h, int w,
                                       aanet_stream_t stream) {
  AANET_HOST_CHECK(img && disp && grad_warped && grad_disp && n > 0 && c > 0 && h > 1 && w > 1);
  const long total = (long)n * h * w;
  hipLaunchKernelGGL(disp_warp_bwd_kernel, dim3(host_div_up(total, WB)), dim3(WB), 0,
                     as_hip(stream), img, disp, grad_warped, grad_disp, grad_img, c, h, w, total);
  return aanet_launch_status();
}
