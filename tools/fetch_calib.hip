// FETCH_SIZE calibration probe (gfx950): how many bytes rocprofv3's FETCH_SIZE reports for read
// shapes the hot-path kernels use, against the bytes actually read.  MI355X_MICROARCH.md §HBM
// calibrates only the wide coalesced read (reported at 1/2).  Shapes here:
//   wide      16 B per lane, 1 KiB contiguous per wave
//   dword     4 B per lane, 256 B contiguous per wave (the regression / offset-plane reads)
//   half      64-B segments: 16 lanes read the first half of a 128-B line, the other half is
//             never read (bytes read = N/2, lines touched = N/128)
//   halves    64-B segments, both halves of every line read, the second half by workgroups
//             dispatched in the second half of the grid (long after the first half was read)
//   seg64x4   16 B per lane, 4 lanes per 64-B segment (the DCN tail's identity-row reads)
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_wide(const float4 *__restrict__ x, long n4, float *sink) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 v = x[i];
  if (v.x + v.y + v.z + v.w == 1234.5f) sink[0] = 1.f;
}

__global__ void k_dword(const float *__restrict__ x, long n, float *sink) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (x[i] == 1234.5f) sink[0] = 1.f;
}

// thread t: line t / 16, dword t % 16 of the line's first half (hf = 0) or second half (hf = 1)
__global__ void k_half(const float *__restrict__ x, long lines, int both, float *sink) {
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long per = lines * 16;
  long u = t;
  int hf = 0;
  if (both && t >= per) u = t - per, hf = 1;
  if (u >= per) return;
  const long line = u >> 4;
  if (x[line * 32 + hf * 16 + (u & 15)] == 1234.5f) sink[0] = 1.f;
}

// 16 B per lane, 4 lanes per 64-B segment, segment s at byte 64 s of the first half of line s
// (lanes 4j..4j+3 read line (wave*16 + j)): 1/2 of the bytes read, every line touched
__global__ void k_seg64(const float4 *__restrict__ x, long lines, float *sink) {
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long line = t >> 2;
  if (line >= lines) return;
  const float4 v = x[line * 8 + (t & 3)];
  if (v.x + v.y + v.z + v.w == 1234.5f) sink[0] = 1.f;
}

int main() {
  const long N = 512L << 20;  // bytes
  float *x, *sink;
  CK(hipMalloc(&x, N));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(x, 0, N));
  const int B = 256;
  const long n = N / 4, n4 = N / 16, lines = N / 128;
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_wide, dim3((n4 + B - 1) / B), dim3(B), 0, 0, (const float4 *)x, n4, sink);
    hipLaunchKernelGGL(k_dword, dim3((n + B - 1) / B), dim3(B), 0, 0, x, n, sink);
    hipLaunchKernelGGL(k_half, dim3((lines * 16 + B - 1) / B), dim3(B), 0, 0, x, lines, 0, sink);
    hipLaunchKernelGGL(k_half, dim3((lines * 32 + B - 1) / B), dim3(B), 0, 0, x, lines, 1, sink);
    hipLaunchKernelGGL(k_seg64, dim3((lines * 4 + B - 1) / B), dim3(B), 0, 0, (const float4 *)x, lines, sink);
  }
  CK(hipDeviceSynchronize());
  printf("bytes: wide %ld dword %ld half %ld halves %ld seg64 %ld (FETCH_SIZE is in KB)\n", N, N, N / 2, N, N / 2);
  CK(hipFree(x));
  CK(hipFree(sink));
  return 0;
}
