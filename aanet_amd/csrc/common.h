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

static inline int host_div_up(long a, long b) { return (int)((a + b - 1) / b); }

static inline int conv_out_size(int in, int k, int s, int p, int d) {
  return (in + 2 * p - (d * (k - 1) + 1)) / s + 1;
}
