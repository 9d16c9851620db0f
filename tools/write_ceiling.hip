// Write-bandwidth ceiling probe (gfx950): the rate of a pure 16-byte-per-lane store stream over
// 1.5 GB (the C5 concat volume's size), plain vs non-temporal stores, grid-stride vs one
// contiguous segment per workgroup, and hipMemsetAsync; plus a float4 copy for reference.
// Build: hipcc -O3 --offload-arch=gfx950 tools/write_ceiling.hip -o tools/write_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_stride(f4 *__restrict__ o, long n4) {
  const f4 v = {1.f, 2.f, 3.f, 4.f};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    if (NT)
      __builtin_nontemporal_store(v, o + i);
    else
      o[i] = v;
  }
}

// workgroup b writes the contiguous segment [b * seg, (b + 1) * seg)
template <bool NT>
__global__ __launch_bounds__(256) void k_seg(f4 *__restrict__ o, long seg4) {
  const f4 v = {1.f, 2.f, 3.f, 4.f};
  f4 *p = o + blockIdx.x * seg4;
  for (long i = threadIdx.x; i < seg4; i += 256) {
    if (NT)
      __builtin_nontemporal_store(v, p + i);
    else
      p[i] = v;
  }
}

// the same segment, 4 independent stores per thread per iteration (more stores in flight)
__global__ __launch_bounds__(256) void k_seg4(f4 *__restrict__ o, long seg4) {
  const f4 v = {1.f, 2.f, 3.f, 4.f};
  f4 *p = o + blockIdx.x * seg4;
  long i = threadIdx.x;
  for (; i + 768 < seg4; i += 1024) {
    p[i] = v;
    p[i + 256] = v;
    p[i + 512] = v;
    p[i + 768] = v;
  }
  for (; i < seg4; i += 256) p[i] = v;
}

// 512-thread workgroups, 8 segments of 128 KB per workgroup-wave pair
__global__ __launch_bounds__(512) void k_seg512(f4 *__restrict__ o, long seg4) {
  const f4 v = {1.f, 2.f, 3.f, 4.f};
  f4 *p = o + blockIdx.x * seg4;
  for (long i = threadIdx.x; i < seg4; i += 512) p[i] = v;
}

__global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ a, f4 *__restrict__ o, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) o[i] = a[i];
}

int main() {
  const long N = 1536L << 20, n4 = N / 16;
  f4 *o, *a;
  if (hipMalloc(&o, N) != hipSuccess || hipMalloc(&a, N) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, auto f, double bytes) {
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.1f us  %6.2f TB/s\n", name, ms * 1e3 / 5, bytes / (ms * 1e-3 / 5) / 1e12);
  };
  const int g = 256 * 8;
  run("grid-stride plain store", [&] { hipLaunchKernelGGL(k_stride<false>, dim3(g), dim3(256), 0, 0, o, n4); }, N);
  run("grid-stride nontemporal store", [&] { hipLaunchKernelGGL(k_stride<true>, dim3(g), dim3(256), 0, 0, o, n4); }, N);
  const long segs = 1536, seg4 = n4 / segs;  // ~1 MB per workgroup, as the concat band kernel
  run("1 MB segment per WG, plain", [&] { hipLaunchKernelGGL(k_seg<false>, dim3(segs), dim3(256), 0, 0, o, seg4); }, N);
  run("1 MB segment per WG, nontemporal", [&] { hipLaunchKernelGGL(k_seg<true>, dim3(segs), dim3(256), 0, 0, o, seg4); }, N);
  run("1 MB segment per WG, plain x4", [&] { hipLaunchKernelGGL(k_seg4, dim3(segs), dim3(256), 0, 0, o, seg4); }, N);
  run("1 MB segment, 512 threads", [&] { hipLaunchKernelGGL(k_seg512, dim3(segs), dim3(512), 0, 0, o, seg4); }, N);
  run("256 KB segment per WG, plain", [&] { hipLaunchKernelGGL(k_seg<false>, dim3(segs * 4), dim3(256), 0, 0, o, seg4 / 4); }, N);
  run("hipMemsetAsync", [&] { (void)hipMemsetAsync(o, 0, N, 0); }, N);
  run("float4 copy (read + write bytes)", [&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, a, o, n4); }, 2.0 * N);
  hipFree(o);
  hipFree(a);
  return 0;
}
