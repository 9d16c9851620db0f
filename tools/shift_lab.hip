// shift_lab.hip -- A/B of concat-volume store-loop variants (a probe, not product code).
// C5 shape: features [4,32,96,312], D=48 -> volume [4,64,48,96,312].
#include "../aanet_amd/csrc/cost_volume.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

namespace lab {
// V: 0 = nt stores, flat (d, q) loop; 1 = default stores; 2 = one plane after the other;
//    3 = wave-per-row (d = wave, wave + NW, ...; lanes over quads, no division)
template <int V>
__global__ __launch_bounds__(256) void concat_rows(const float *__restrict__ L, const float *__restrict__ R,
                                                   float *__restrict__ out, int C, int H, int W, int D) {
  extern __shared__ __attribute__((aligned(16))) float srow[];
  float *sL = srow, *sR = srow + W;
  const int tid = threadIdx.x;
  const int row = blockIdx.x, y = row % H, bc = row / H, c = bc % C, b = bc / C;
  const int W4 = W >> 2;
  const f32x4 *gl = reinterpret_cast<const f32x4 *>(L + (long)row * W);
  const f32x4 *gr = reinterpret_cast<const f32x4 *>(R + (long)row * W);
  for (int q = tid; q < W4; q += 256) {
    reinterpret_cast<f32x4 *>(sL)[q] = __builtin_nontemporal_load(gl + q);
    reinterpret_cast<f32x4 *>(sR)[q] = __builtin_nontemporal_load(gr + q);
  }
  __syncthreads();
  const long HW = (long)H * W;
  float *o0 = out + (((long)b * 2 * C + c) * D * H + y) * W;
  float *o1 = o0 + (long)C * D * HW;
  auto put = [&](f32x4 v, float *p) {
    if (V == 1) *reinterpret_cast<f32x4 *>(p) = v;
    else __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(p));
  };
  if (V <= 1) {
    for (int e = tid; e < D * W4; e += 256) {
      const int d = e / W4, x = 4 * (e - d * W4);
      f32x4 vl, vr;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = x + u >= d;
        vl[u] = ok ? sL[x + u] : 0.f;
        vr[u] = ok ? sR[x + u - d] : 0.f;
      }
      put(vl, o0 + (long)d * HW + x);
      put(vr, o1 + (long)d * HW + x);
    }
  } else if (V == 2) {
    for (int h = 0; h < 2; ++h) {
      const float *s = h ? sR : sL;
      float *o = h ? o1 : o0;
      for (int e = tid; e < D * W4; e += 256) {
        const int d = e / W4, x = 4 * (e - d * W4);
        f32x4 v;
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = x + u >= d ? s[x + u - (h ? d : 0)] : 0.f;
        put(v, o + (long)d * HW + x);
      }
    }
  } else {
    const int wave = tid >> 6, lane = tid & 63;
    for (int d = wave; d < D; d += 4) {
      for (int q = lane; q < W4; q += 64) {
        const int x = 4 * q;
        f32x4 vl, vr;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool ok = x + u >= d;
          vl[u] = ok ? sL[x + u] : 0.f;
          vr[u] = ok ? sR[x + u - d] : 0.f;
        }
        put(vl, o0 + (long)d * HW + x);
        put(vr, o1 + (long)d * HW + x);
      }
    }
  }
}
// YB consecutive rows y of one (b, c) per block: each d plane gets YB*W contiguous floats
template <int YB>
__global__ __launch_bounds__(256) void concat_band(const float *__restrict__ L, const float *__restrict__ R,
                                                   float *__restrict__ out, int C, int H, int W, int D) {
  extern __shared__ __attribute__((aligned(16))) float srow[];
  const int tid = threadIdx.x;
  const int nyb = H / YB;
  const int yb = blockIdx.x % nyb, bc = blockIdx.x / nyb, c = bc % C, b = bc / C;
  const int W4 = W >> 2, S4 = YB * W4;
  float *sL = srow, *sR = srow + YB * W;
  const f32x4 *gl = reinterpret_cast<const f32x4 *>(L + ((long)bc * H + yb * YB) * W);
  const f32x4 *gr = reinterpret_cast<const f32x4 *>(R + ((long)bc * H + yb * YB) * W);
  for (int q = tid; q < S4; q += 256) {
    reinterpret_cast<f32x4 *>(sL)[q] = __builtin_nontemporal_load(gl + q);
    reinterpret_cast<f32x4 *>(sR)[q] = __builtin_nontemporal_load(gr + q);
  }
  __syncthreads();
  const long HW = (long)H * W;
  float *o0 = out + (((long)b * 2 * C + c) * D * H + yb * YB) * W;
  float *o1 = o0 + (long)C * D * HW;
  for (int e = tid; e < D * S4; e += 256) {
    const int d = e / S4, r = e - d * S4, yy = r / W4, x = 4 * (r - yy * W4);
    const float *l = sL + yy * W, *rr = sR + yy * W;
    f32x4 vl, vr;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = x + u >= d;
      vl[u] = ok ? l[x + u] : 0.f;
      vr[u] = ok ? rr[x + u - d] : 0.f;
    }
    __builtin_nontemporal_store(vl, reinterpret_cast<f32x4 *>(o0 + (long)d * HW + 4 * r));
    __builtin_nontemporal_store(vr, reinterpret_cast<f32x4 *>(o1 + (long)d * HW + 4 * r));
  }
}
__global__ void fill(float *p, long n, unsigned seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (float)(x & 0xffff);
  }
}
}  // namespace lab

int main() {
  const int B = 4, C = 32, H = 96, W = 312, D = 48;
  const long nin = (long)B * C * H * W, nout = (long)B * 2 * C * D * H * W;
  float *L, *R, *o;
  CHECK(hipMalloc(&L, nin * 4));
  CHECK(hipMalloc(&R, nin * 4));
  CHECK(hipMalloc(&o, nout * 4));
  hipLaunchKernelGGL(lab::fill, dim3(2048), dim3(256), 0, 0, L, nin, 1u);
  hipLaunchKernelGGL(lab::fill, dim3(2048), dim3(256), 0, 0, R, nin, 2u);
  std::vector<float> ref(nout), h(nout);
  if (aanet_concat_volume_f32(L, R, o, B, C, H, W, D, 0)) return 1;
  CHECK(hipMemcpy(ref.data(), o, nout * 4, hipMemcpyDeviceToHost));
  struct Var { const char *name; void (*fn)(const float *, const float *, float *); };
  std::vector<Var> vs = {
      {"product", [](const float *l, const float *r, float *out) { aanet_concat_volume_f32(l, r, out, 4, 32, 96, 312, 48, 0); }},
      {"nt flat", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_rows<0>, dim3(4 * 32 * 96), dim3(256), 2 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"default flat", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_rows<1>, dim3(4 * 32 * 96), dim3(256), 2 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"nt planes", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_rows<2>, dim3(4 * 32 * 96), dim3(256), 2 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"nt wave-row", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_rows<3>, dim3(4 * 32 * 96), dim3(256), 2 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"band4", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_band<4>, dim3(4 * 32 * 24), dim3(256), 2 * 4 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"band8", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_band<8>, dim3(4 * 32 * 12), dim3(256), 2 * 8 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
      {"band16", [](const float *l, const float *r, float *out) { hipLaunchKernelGGL(lab::concat_band<16>, dim3(4 * 32 * 6), dim3(256), 2 * 16 * 312 * 4, 0, l, r, out, 32, 96, 312, 48); }},
  };
  for (auto &v : vs) {
    CHECK(hipMemset(o, 0xff, nout * 4));
    v.fn(L, R, o);
    CHECK(hipMemcpy(h.data(), o, nout * 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (long i = 0; i < nout; ++i) bad += h[i] != ref[i];
    printf("%-14s mismatches %ld\n", v.name, bad);
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double bytes = 4.0 * (2 * nin + nout);
  for (int round = 0; round < 3; ++round)
    for (auto &v : vs) {
      v.fn(L, R, o);
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < 10; ++i) v.fn(L, R, o);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      printf("round %d %-14s %7.1f us  %6.0f GB/s\n", round, v.name, 100 * ms, bytes / (100 * ms) / 1e3);
    }
  return 0;
}
