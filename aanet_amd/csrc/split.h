// split.h -- the split-bf16 contraction shared by the conv engine kernels (mdcn.hip,
// dcn_tile.hip, pointwise.hip): an fp32 value is carried as three exact bf16 pieces
// (x = h + m + l), a product as the six piece products down to 2^-16 relative, run as
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation (fp32-accurate; see mdcn.hip "split-bf16").
#pragma once

#include "common.h"

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 8 values -> their three exact bf16 pieces (activations: common.h split_pair)
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&b)[3]) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t hh, mm, ll;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned h, m, l;
    split_pair(v[2 * i], v[2 * i + 1], h, m, l);
    hh[i] = h;
    mm[i] = m;
    ll[i] = l;
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
