// split_rne_lab.hip -- probe (not product code): is common.h split_pair exact on gfx950?  For
// 2^27 fp32 values (random bits over every finite exponent, plus +-0 and the subnormals) it checks
// h + m + l == x in double (for |x| >= 2^-100; below, the pieces are subnormal and flushed, a loss
// under 2^-126 absolute) and reports the largest |m|/|x| and |l|/|x|.  Round 5: a 7-op form
// (h = v_cvt_pk_bf16_f32, residuals by v_dot2c_f32_bf16 against (-1, 0)) failed here on about
// half of the values (71,305,007 of 134,217,728 inexact); the truncation form is the product.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/split_rne_lab.hip -o tools/split_rne_lab
#include <cmath>
#include <cstdio>
#include <cstring>

#include "../aanet_amd/csrc/common.h"

__device__ float bf2f(unsigned v, int hi) { return __uint_as_float(hi ? (v & 0xffff0000u) : (v << 16)); }

__global__ void probe(unsigned long long *bad, unsigned long long *tiny, unsigned *mrel, unsigned *lrel,
                      unsigned long long *first) {
  const unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
  unsigned s = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 13) * 0x9E3779B9u;
  s ^= s >> 15; s *= 0x2c1b3c6du; s ^= s >> 12;
  unsigned b0 = s, b1 = s * 0x297a2d39u + 0x6b43a9b5u;
  if ((b0 & 0x7f800000u) == 0x7f800000u) b0 &= 0xbfffffffu;  // keep finite
  if ((b1 & 0x7f800000u) == 0x7f800000u) b1 &= 0xbfffffffu;
  if (i < 256) b0 = (unsigned)i;                             // subnormals and zero
  const float a = __uint_as_float(b0), b = __uint_as_float(b1);
  unsigned h, m, l;
  split_pair(a, b, h, m, l);
  const float x[2] = {a, b};
  for (int k = 0; k < 2; ++k) {
    const double hh = bf2f(h, k), mm = bf2f(m, k), ll = bf2f(l, k);
    if (hh + mm + ll != (double)x[k]) {
      // below 2^-100 the pieces m, l fall into the fp32 subnormals (flushed): a loss < 2^-126
      if (fabs((double)x[k]) < 0x1p-100) atomicAdd(tiny, 1ull);
      else if (atomicAdd(bad, 1ull) == 0) *first = (unsigned long long)__float_as_uint(x[k]);
    }
    if (x[k] != 0.f && fabs((double)x[k]) > 1e-30) {
      atomicMax(mrel, __float_as_uint((float)fabs(mm / x[k])));
      atomicMax(lrel, __float_as_uint((float)fabs(ll / x[k])));
    }
  }
}

int main() {
  unsigned long long *bad, *first, *tiny;
  unsigned *mrel, *lrel;
  if (hipMallocManaged(&bad, 8) || hipMallocManaged(&tiny, 8) || hipMallocManaged(&first, 8) || hipMallocManaged(&mrel, 4) || hipMallocManaged(&lrel, 4)) return 2;
  *bad = 0; *first = 0; *tiny = 0; *mrel = 0; *lrel = 0;
  hipLaunchKernelGGL(probe, dim3(1 << 18), dim3(256), 0, 0, bad, tiny, mrel, lrel, first);
  if (hipDeviceSynchronize()) return 2;
  unsigned mr = *mrel, lr = *lrel;
  float mf, lf;
  memcpy(&mf, &mr, 4); memcpy(&lf, &lr, 4);
  printf("split_pair: %llu inexact of %d values with |x| >= 2^-100 (first bits 0x%llx), %llu below "
         "(flushed subnormal pieces); max |m/x| = 2^%.2f, max |l/x| = 2^%.2f\n",
         *bad, 2 << 26, *first, *tiny, log2(mf), log2(lf));
  return *bad ? 1 : 0;
}
