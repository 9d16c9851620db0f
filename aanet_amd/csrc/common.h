// common.h -- shared helpers for the gfx950 kernels behind include/aanet_mi355x.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aanet_mi355x.h"

#define AANET_HOST_CHECK(cond)       \
  do {                               \
    if (!(cond)) return AANET_EINVAL; \
  } while (0)

// Status after a launch: positive hipError_t, never swallowed.
static inline int aanet_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? AANET_OK : (int)e;
}

static inline hipStream_t as_hip(aanet_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// v_mfma_f32_16x16x4_f32: D[16x16] += A[16x4] * B[4x16], exact fp32 fma chain.
// Lane l holds A[l&15][l>>4], B[l>>4][l&15]; D: col = l&15, row = 4*(l>>4) + reg.
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int div_up(int a, int b) { return (a + b - 1) / b; }

// ---- split-bf16 activations: two fp32 values -> their three exact bf16 pieces each, x = h + m + l,
// by truncation: h = the upper 16 bits of x, r = x - h (exact, <= 16 significant bits), m = the
// upper 16 bits of r, l = r - m (exact, <= 8 significant bits, so its upper half IS its bf16
// value); v_perm_b32 packs two upper halves into one bf16x2 register: 11 VALU per two values.
// (A 7-op form -- h = v_cvt_pk_bf16_f32, residuals by v_dot2c_f32_bf16 against (-1, 0) -- is NOT
// exact on gfx950: tools/split_rne_lab.hip found h + m + l != x for about half of random fp32
// values, i.e. v_dot2c does not return x - h exactly)
__device__ __forceinline__ void split_pair(float a, float b, unsigned &h, unsigned &m, unsigned &l) {
  auto hi2 = [](float x, float y) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, y), __builtin_bit_cast(unsigned, x), 0x07060302u);
  };
  auto t16 = [](float x) { return __builtin_bit_cast(float, __builtin_bit_cast(unsigned, x) & 0xffff0000u); };
  h = hi2(a, b);
  const float r0 = a - t16(a), r1 = b - t16(b);
  m = hi2(r0, r1);
  l = hi2(r0 - t16(r0), r1 - t16(r1));
}

static inline int host_div_up(long a, long b) { return (int)((a + b - 1) / b); }

static inline int conv_out_size(int in, int k, int s, int p, int d) {
  return (in + 2 * p - (d * (k - 1) + 1)) / s + 1;
}

// ---- exact 2x / 4x bilinear upsampling of a 4-column output quad (PyTorch align_corners=False,
// F.interpolate as in nets/aggregation.py:395-396).  With scale 1/r the source coordinate of
// output column 4q+u is 4q/r + (u+0.5)/r - 0.5, so the quad reads one 4-wide source segment
// (s0 = 2q-1 for r = 2, q-1 for r = 4; indices clamped into the row exactly as PyTorch's
// max(src, 0) / x1 = x0 + (x0 < in-1) do) with constant lambdas:
//   r = 2: (0.25, 0.75) pairs; r = 4: lambdas 0.625, 0.875, 0.125, 0.375.
__device__ __forceinline__ f32x4 load_seg(const float *__restrict__ row, int iw, int s0) {
  if (s0 >= 0 && s0 + 3 <= iw - 1) {
    // dword-aligned 16-byte load (unaligned vector access is enabled on gfx9 Linux)
    typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
    const f4u v = *reinterpret_cast<const f4u *>(row + s0);
    return f32x4{v.x, v.y, v.z, v.w};
  }
  f32x4 v;
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = row[min(max(s0 + u, 0), iw - 1)];
  return v;
}

// ---- buffer-resource access for the epilogues: one SGPR resource per image plane set, 32-bit
// byte offsets per lane (no per-access 64-bit address math); range-checked (bytes < 2^31)
typedef __amdgpu_buffer_rsrc_t brsrc_t;
__device__ __forceinline__ brsrc_t buf_rsrc(const void *p, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 buf_ld4(brsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ float buf_ld1(brsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void buf_st4(brsrc_t r, unsigned off, f32x4 v) {
  typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_, v), r, (int)off, 0, 0);
}
// the 4-column source segment starting at column s0 of a row at byte offset `row` (load_seg's
// clamping), wave-uniform choice: `fast` (every lane's segment inside its row) = one 16-byte load
__device__ __forceinline__ f32x4 buf_seg(brsrc_t r, unsigned row, int s0, int iw, bool fast) {
  if (fast) return buf_ld4(r, row + 4u * (unsigned)s0);
  f32x4 v;
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = buf_ld1(r, row + 4u * (unsigned)min(max(s0 + u, 0), iw - 1));
  return v;
}

__device__ __forceinline__ f32x4 hlerp(const f32x4 v, int r) {
  if (r == 2)
    return f32x4{0.25f * v[0] + 0.75f * v[1], 0.75f * v[1] + 0.25f * v[2],
                 0.25f * v[1] + 0.75f * v[2], 0.75f * v[2] + 0.25f * v[3]};
  return f32x4{0.375f * v[0] + 0.625f * v[1], 0.125f * v[0] + 0.875f * v[1],
               0.875f * v[1] + 0.125f * v[2], 0.625f * v[1] + 0.375f * v[2]};
}

// Output quad (row y, columns 4q..4q+3) of an r-times upsampled plane im [ih][iw];
// sh = ih / H (the PyTorch area_pixel_compute_scale for align_corners=False).
__device__ __forceinline__ f32x4 upsample_quad(const float *__restrict__ im, int ih, int iw,
                                               float sh, int r, int y, int q) {
  float hr = sh * ((float)y + 0.5f) - 0.5f;
  hr = hr < 0.f ? 0.f : hr;
  const int h1 = (int)hr, h1p = h1 < ih - 1 ? 1 : 0;
  const float h1l = hr - (float)h1, h0l = 1.f - h1l;
  const int s0 = r == 2 ? 2 * q - 1 : q - 1;
  const f32x4 t = hlerp(load_seg(im + (long)h1 * iw, iw, s0), r);
  const f32x4 b = hlerp(load_seg(im + (long)(h1 + h1p) * iw, iw, s0), r);
  return h0l * t + h1l * b;
}
