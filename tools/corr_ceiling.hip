// corr_ceiling.hip -- memory ceilings for the correlation kernel's access pattern (a probe,
// not product code).  Build: hipcc -O3 --offload-arch=gfx950 tools/corr_ceiling.hip -o /tmp/cc
//   (1) float4 copy of the same byte volume (read 2 feature maps, write 1 volume-sized buffer)
//   (2) the correlation kernel's exact load pattern (L tile 16x64, R window 16x128 per stage,
//       8 stages, 16-B buffer loads, XCD remap) + its output stores (64 d x 64 x, float4),
//       with no MFMA: an add of the staged values keeps the loads live.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void copy4(const f32x4 *__restrict__ a, f32x4 *__restrict__ b, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) b[i] = a[i];
}

__global__ __launch_bounds__(256) void read_write(const f32x4 *__restrict__ a, const f32x4 *__restrict__ a2,
                                                  f32x4 *__restrict__ b, long nr, long nw) {
  f32x4 s = {0, 0, 0, 0};
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nr; i += (long)gridDim.x * 256) s += a[i] + a2[i];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nw; i += (long)gridDim.x * 256) b[i] = s;
}

template <int MODE>  // 0: loads + stores; 1: loads only; 2: stores only
__global__ __launch_bounds__(256) void corr_pattern(const float *__restrict__ L, const float *__restrict__ R,
                                                    float *__restrict__ out, int C, int H, int W, int D,
                                                    int ntx) {
  constexpr int TX = 64, CC = 16, RW = 128;
  __shared__ __attribute__((aligned(16))) float smem[2 * (CC * TX + CC * RW)];
  const int tid = threadIdx.x;
  const int nwg = gridDim.x, b0 = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b0 & 7;
  int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b0 >> 3);
  const int tx = id % ntx;
  id /= ntx;
  const int y = id % H, b = id / H;
  const int x0 = tx * TX, xr0 = x0 - 64;
  const long HW = (long)H * W;
  const int img_bytes = (int)(C * HW * 4);
  const auto Lr = __builtin_amdgcn_make_buffer_rsrc((void *)(L + (long)b * C * HW), (short)0, img_bytes, 0x00020000);
  const auto Rr = __builtin_amdgcn_make_buffer_rsrc((void *)(R + (long)b * C * HW), (short)0, img_bytes, 0x00020000);
  f32x4 acc = {0, 0, 0, 0};
  if (MODE != 2) {
    for (int c0 = 0; c0 < C; c0 += CC) {
      const int row = tid / 16, col4 = tid % 16;
      int c = c0 + row, x = x0 + 4 * col4;
      int off = (c < C && x < W) ? (int)((((long)c * H + y) * W + x) * 4) : img_bytes;
      f32x4 l = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(Lr, off, 0, 0));
      f32x4 r[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256;
        const int rrow = e / 32, rc4 = e % 32;
        c = c0 + rrow;
        x = xr0 + 4 * rc4;
        off = (c < C && x >= 0 && x < W) ? (int)((((long)c * H + y) * W + x) * 4) : img_bytes;
        r[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(Rr, off, 0, 0));
      }
      acc += l + r[0] + r[1];
    }
    reinterpret_cast<f32x4 *>(smem)[tid] = acc;
    __syncthreads();
  }
  if (MODE != 1) {
    for (int e = tid; e < D * (TX / 4); e += 256) {
      const int dl = e / (TX / 4), xq = e % (TX / 4);
      if (x0 + 4 * xq < W) {
        f32x4 v = MODE == 2 ? f32x4{1.f, 2.f, 3.f, (float)e} : reinterpret_cast<f32x4 *>(smem)[e & 255];
        *reinterpret_cast<f32x4 *>(out + (((long)b * D + dl) * H + y) * W + x0 + 4 * xq) = v;
      }
    }
  } else if (acc[0] == 123.456f) {
    out[tid] = acc[1];
  }
}

int main() {
  const int B = 8, C = 128, H = 128, W = 416, D = 64;
  const long nf = (long)B * C * H * W, nv = (long)B * D * H * W;
  float *L, *R, *O;
  CHECK(hipMalloc(&L, nf * 4));
  CHECK(hipMalloc(&R, nf * 4));
  CHECK(hipMalloc(&O, nv * 4));
  std::vector<float> h(nf, 1.f);
  CHECK(hipMemcpy(L, h.data(), nf * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(R, h.data(), nf * 4, hipMemcpyHostToDevice));
  hipEvent_t s, e;
  CHECK(hipEventCreate(&s));
  CHECK(hipEventCreate(&e));
  const double bytes = 4.0 * (2 * nf + nv);
  auto timeit = [&](auto fn, const char *name, double nbytes) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(s);
    const int it = 50;
    for (int i = 0; i < it; ++i) fn();
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    ms /= it;
    printf("%-34s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, nbytes / ms / 1e6);
  };
  const int ntx = (W + 63) / 64;
  const unsigned grid = (unsigned)(ntx * H * B);
  timeit([&] { hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const f32x4 *)L, (f32x4 *)O, nv / 4); },
         "copy4 (volume-sized)", 8.0 * nv);
  timeit([&] { hipLaunchKernelGGL(read_write, dim3(8192), dim3(256), 0, 0, (const f32x4 *)L, (const f32x4 *)R,
                                  (f32x4 *)O, nf / 4, nv / 4); },
         "read 2 maps + write volume (flat)", bytes);
  timeit([&] { hipLaunchKernelGGL(corr_pattern<0>, dim3(grid), dim3(256), 0, 0, L, R, O, C, H, W, D, ntx); },
         "corr pattern loads+stores", bytes);
  timeit([&] { hipLaunchKernelGGL(corr_pattern<1>, dim3(grid), dim3(256), 0, 0, L, R, O, C, H, W, D, ntx); },
         "corr pattern loads only", 4.0 * 2 * nf);
  timeit([&] { hipLaunchKernelGGL(corr_pattern<2>, dim3(grid), dim3(256), 0, 0, L, R, O, C, H, W, D, ntx); },
         "corr pattern stores only", 4.0 * nv);
  printf("algorithmic bytes per launch: %.1f MB\n", bytes / 1e6);
  return 0;
}
