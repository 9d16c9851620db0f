// LDS scatter-add probe (gfx950): the cost of adding 64 values per wave-instruction into an LDS
// window at data-dependent positions, lanes = 2 positions x 32 channels (the DCN backward's grad_x
// corner shape).  Forms: ds_add_f32 (float LDS atomic, no return), ds_add_u32, ds_add_u64, and a
// plain read-add-write into a wave-private window (no atomic; legal when no two lanes of one
// instruction share an address and no other wave writes the region).
// Build: hipcc -O3 --offload-arch=gfx950 tools/lds_rmw_lab.hip -o tools/lds_rmw_lab
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NT = 256, NPOS = 160, CH = 32, UPD = 512;

// per-wave region: NPOS positions x CH channels (20 KB of floats)
template <int MODE>
__global__ __launch_bounds__(NT) void scatter_kernel(const int *__restrict__ pos, float *__restrict__ out) {
  __shared__ float win[4 * NPOS * CH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 4 * NPOS * CH; i += NT) win[i] = 0.f;
  __syncthreads();
  const int ch = lane & 31, half = lane >> 5;
  float *mine = win + (MODE == 3 ? wave * NPOS * CH : 0);
  const int *pp = pos + (blockIdx.x & 63) * UPD * 2;
  float v = 1.0f + lane * 1e-3f;
  for (int u = 0; u < UPD; ++u) {
    // two distinct positions per instruction (pixel's two corners of one row)
    const int p = pp[2 * u + half];
    const int a = (MODE == 3 ? p : (p + wave * 37) % (4 * NPOS)) * CH + ch;
    if (MODE == 0) {
      atomicAdd(&mine[a], v);
    } else if (MODE == 1) {
      atomicAdd(reinterpret_cast<unsigned *>(&mine[a]), 3u);
    } else if (MODE == 2) {
      atomicAdd(reinterpret_cast<unsigned long long *>(&mine[a & ~1]), 3ull);
    } else {
      mine[a] += v;
    }
    v += 1e-4f;
  }
  __syncthreads();
  float s = 0.f;
  for (int i = tid; i < 4 * NPOS * CH; i += NT) s += win[i];
  if (s == 1234.5f) out[blockIdx.x] = s;
}

int main() {
  const int nblk = 256 * 8;
  int *pos;
  float *out;
  hipMalloc(&pos, 64 * UPD * 2 * sizeof(int));
  hipMalloc(&out, nblk * sizeof(float));
  int *h = new int[64 * UPD * 2];
  unsigned s = 12345;
  for (int i = 0; i < 64 * UPD; ++i) {
    s = s * 1664525u + 1013904223u;
    const int p = (s >> 8) % (NPOS - 1);
    h[2 * i] = p, h[2 * i + 1] = p + 1;  // the two corners of a row: never equal
  }
  hipMemcpy(pos, h, 64 * UPD * 2 * sizeof(int), hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[4] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "plain_rmw_private"};
  for (int m = 0; m < 4; ++m) {
    for (int r = 0; r < 2; ++r) {
      hipEventRecord(e0);
      switch (m) {
        case 0: hipLaunchKernelGGL(scatter_kernel<0>, dim3(nblk), dim3(NT), 0, 0, pos, out); break;
        case 1: hipLaunchKernelGGL(scatter_kernel<1>, dim3(nblk), dim3(NT), 0, 0, pos, out); break;
        case 2: hipLaunchKernelGGL(scatter_kernel<2>, dim3(nblk), dim3(NT), 0, 0, pos, out); break;
        default: hipLaunchKernelGGL(scatter_kernel<3>, dim3(nblk), dim3(NT), 0, 0, pos, out); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // wave-instructions of the scatter per CU (256 CUs), cycles at 2.4 GHz
      const double winstr = (double)nblk * 4 * UPD / 256;
      if (r) printf("%-18s %8.3f ms  %7.1f cycles per wave-instruction per CU\n", names[m], ms, ms * 1e-3 * 2.4e9 / winstr);
    }
  }
  hipDeviceSynchronize();
  return 0;
}
