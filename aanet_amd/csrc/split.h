// split.h -- the split-bf16 contraction shared by the conv engine kernels (mdcn.hip,
// dcn_tile.hip, pointwise.hip): an fp32 value is carried as three exact bf16 pieces
// (x = h + m + l), a product as the six piece products down to 2^-16 relative, run as
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation (fp32-accurate; see mdcn.hip "split-bf16").
#pragma once

#include "common.h"

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// (bf16 hi(a), bf16 hi(b)) packed into one register
__device__ __forceinline__ unsigned hi_pair(float a, float b) {
  return __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, b), __builtin_bit_cast(unsigned, a), 0x07060302u);
}
__device__ __forceinline__ float trunc16(float a) {
  return __builtin_bit_cast(float, __builtin_bit_cast(unsigned, a) & 0xffff0000u);
}
// 8 values -> their three exact bf16 pieces (activations: truncation split)
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&b)[3]) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t hh, mm, ll;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = v[2 * i], x1 = v[2 * i + 1];
    hh[i] = hi_pair(x0, x1);
    const float r0 = x0 - trunc16(x0), r1 = x1 - trunc16(x1);
    mm[i] = hi_pair(r0, r1);
    ll[i] = hi_pair(r0 - trunc16(r0), r1 - trunc16(r1));
  }
  b[0] = __builtin_bit_cast(bf16x8, hh);
  b[1] = __builtin_bit_cast(bf16x8, mm);
  b[2] = __builtin_bit_cast(bf16x8, ll);
}
// sum of the six piece products, smallest first
__device__ __forceinline__ f32x4 mfma_split6(const bf16x8 (&A)[3], const bf16x8 (&B)[3], f32x4 t) {
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2], B[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1], B[0], t, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0], B[0], t, 0, 0, 0);
}
