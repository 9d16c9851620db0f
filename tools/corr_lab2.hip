// corr_lab2.hip -- same-process A/B of the round-2 correlation pyramid (corr_pyramid_kernel)
// against the round-3 register-ring tile (corr_pyramid_reg_kernel<2/3>), plus a flat
// read-2/write-1 stream of the scale-0 byte volume (a probe, not product).  Checks the ring
// outputs bit-for-bit against the round-2 kernel on the C2 and C3 (AANet+) pyramids and ragged
// shapes, then times them in alternating rounds.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/corr_lab2.hip -o tools/corr_lab2.bin
#include "../aanet_amd/csrc/cost_volume.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t err_ = (x);                                                       \
    if (err_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__);        \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ __launch_bounds__(256) void rw_flat(const f32x4 *__restrict__ a, const f32x4 *__restrict__ a2,
                                               f32x4 *__restrict__ o, long nr, long nw) {
  // read two maps and write a third array, 4 independent 16-B loads in flight per lane
  const long stride = (long)gridDim.x * 256;
  f32x4 s = {0, 0, 0, 0};
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < nr; i += 2 * stride) {
    f32x4 x0 = __builtin_nontemporal_load(a + i), x1 = __builtin_nontemporal_load(a2 + i);
    f32x4 x2 = __builtin_nontemporal_load(a + i + stride), x3 = __builtin_nontemporal_load(a2 + i + stride);
    s += x0 + x1 + x2 + x3;
  }
  for (; i < nr; i += stride) s += a[i] + a2[i];
  for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < nw; j += stride)
    __builtin_nontemporal_store(s, o + j);
}

struct Pyr {
  int ns, n, maxd;
  int c[3], h[3], w[3];
  float *L[3], *R[3], *o_old[3], *o_new[3];
  size_t fe[3], ve[3];
};

static CorrPyramid make_params(const Pyr &q, float *const *outs, int txw, long *total_out) {
  CorrPyramid p;
  p.ns = q.ns;
  long total = 0;
  for (int s = 0; s < q.ns; ++s) {
    const int d = q.maxd >> s;
    p.L[s] = q.L[s];
    p.R[s] = q.R[s];
    p.out[s] = outs[s];
    p.C[s] = q.c[s];
    p.H[s] = q.h[s];
    p.W[s] = q.w[s];
    p.D[s] = d;
    p.nj[s] = corr_nj(d);
    p.dchunk[s] = corr_dchunk(p.nj[s]);
    p.nchunks[s] = host_div_up(d, p.dchunk[s]);
    p.ntx[s] = host_div_up(q.w[s], txw);
    const long cnt = (long)p.ntx[s] * p.nchunks[s] * q.h[s] * q.n;
    p.cnt[s] = (int)cnt;
    p.per[s] = (int)((cnt + 7) / 8);
    p.mstart[s] = (int)(total / 8);
    total += 8L * p.per[s];
  }
  p.mstart[q.ns] = (int)(total / 8);
  *total_out = total;
  return p;
}

static Pyr alloc_pyr(int n, int maxd, int ns, const int *c, const int *h, const int *w, unsigned seed) {
  Pyr q;
  q.ns = ns;
  q.n = n;
  q.maxd = maxd;
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (int s = 0; s < ns; ++s) {
    q.c[s] = c[s];
    q.h[s] = h[s];
    q.w[s] = w[s];
    q.fe[s] = (size_t)n * c[s] * h[s] * w[s];
    q.ve[s] = (size_t)n * (maxd >> s) * h[s] * w[s];
    std::vector<float> hb(q.fe[s]);
    CHECK(hipMalloc(&q.L[s], q.fe[s] * 4));
    CHECK(hipMalloc(&q.R[s], q.fe[s] * 4));
    CHECK(hipMalloc(&q.o_old[s], q.ve[s] * 4));
    CHECK(hipMalloc(&q.o_new[s], q.ve[s] * 4));
    for (auto &v : hb) v = nd(rng);
    CHECK(hipMemcpy(q.L[s], hb.data(), q.fe[s] * 4, hipMemcpyHostToDevice));
    for (auto &v : hb) v = nd(rng);
    CHECK(hipMemcpy(q.R[s], hb.data(), q.fe[s] * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(q.o_old[s], 0x7f, q.ve[s] * 4));
    CHECK(hipMemset(q.o_new[s], 0x3f, q.ve[s] * 4));
  }
  return q;
}

static double pyr_bytes(const Pyr &q) {
  double b = 0;
  for (int s = 0; s < q.ns; ++s) b += 4.0 * (2.0 * q.fe[s] + q.ve[s]);
  return b;
}

static void launch_old(const Pyr &q, float *const *outs) {
  long total;
  CorrPyramid p = make_params(q, outs, 64, &total);
  hipLaunchKernelGGL(corr_pyramid_kernel, dim3((unsigned)total), dim3(NTHREADS), 0, 0, p);
}

template <int RING>
static void launch_reg(const Pyr &q, float *const *outs) {
  long total;
  CorrPyramid p = make_params(q, outs, 64, &total);
  hipLaunchKernelGGL(corr_pyramid_reg_kernel<RING>, dim3((unsigned)total), dim3(NTHREADS), 0, 0, p);
}

static bool compare(const Pyr &q, const char *what) {
  CHECK(hipDeviceSynchronize());
  bool ok = true;
  for (int s = 0; s < q.ns; ++s) {
    std::vector<float> a(q.ve[s]), b(q.ve[s]);
    CHECK(hipMemcpy(a.data(), q.o_old[s], q.ve[s] * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(b.data(), q.o_new[s], q.ve[s] * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < a.size(); ++i)
      if (memcmp(&a[i], &b[i], 4) != 0) ++bad;
    printf("  %-28s scale %d: %zu of %zu elements differ\n", what, s, bad, a.size());
    ok = ok && bad == 0;
  }
  return ok;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 4;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto fn, int it) {
    fn();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < it; ++i) fn();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / it;
  };

  // ---- correctness: ragged + C3 + C2 ----
  bool all = true;
  {
    const int c[3] = {32, 64, 128}, h[3] = {5, 3, 2}, w[3] = {100, 52, 28};
    Pyr q = alloc_pyr(2, 64, 3, c, h, w, 7);
    launch_old(q, q.o_old);
    launch_reg<2>(q, q.o_new);
    all &= compare(q, "ragged reg2");
    launch_reg<3>(q, q.o_new);
    all &= compare(q, "ragged reg3");
  }
  {
    const int c[3] = {128, 128, 128}, h[3] = {7, 4, 2}, w[3] = {20, 12, 4};
    Pyr q = alloc_pyr(3, 24, 3, c, h, w, 8);  // D=24/12/6 (C1-like), W < D
    launch_old(q, q.o_old);
    launch_reg<3>(q, q.o_new);
    all &= compare(q, "C1-like W<D reg3");
  }
  {
    const int c[3] = {32, 64, 128}, h[3] = {192, 96, 48}, w[3] = {320, 160, 80};
    Pyr q = alloc_pyr(8, 64, 3, c, h, w, 9);
    launch_old(q, q.o_old);
    launch_reg<3>(q, q.o_new);
    all &= compare(q, "C3 AANet+ reg3");
    const double by = pyr_bytes(q);
    for (int r = 0; r < 2; ++r) {
      const double t0 = timeit([&] { launch_old(q, q.o_old); }, 30);
      const double t2 = timeit([&] { launch_reg<3>(q, q.o_new); }, 30);
      printf("C3 round %d: old %7.1f us (%5.0f GB/s)  reg3 %7.1f us (%5.0f GB/s)\n", r, t0,
             by / t0 / 1e3, t2, by / t2 / 1e3);
    }
  }
  const int c[3] = {128, 128, 128}, h[3] = {128, 64, 32}, w[3] = {416, 208, 104};
  Pyr q = alloc_pyr(8, 64, 3, c, h, w, 10);
  launch_old(q, q.o_old);
  launch_reg<2>(q, q.o_new);
  all &= compare(q, "C2 reg2");
  launch_reg<3>(q, q.o_new);
  all &= compare(q, "C2 reg3");
  printf("bit-exact: %s\n", all ? "yes" : "NO");

  // ---- timing (C2 pyramid, B=8) ----
  const double by = pyr_bytes(q);
  Pyr q0 = q;
  q0.ns = 1;  // scale 0 alone
  const double by0 = pyr_bytes(q0);
  float *flat;
  const long nr = (long)(q.fe[0] / 4), nw = (long)(q.ve[0] / 4);
  CHECK(hipMalloc(&flat, q.ve[0] * 4));
  for (int r = 0; r < rounds; ++r) {
    const double t_old = timeit([&] { launch_old(q, q.o_old); }, 50);
    const double s_old = timeit([&] { launch_old(q0, q0.o_old); }, 50);
    const double t_r2 = timeit([&] { launch_reg<2>(q, q.o_new); }, 50);
    const double t_r3 = timeit([&] { launch_reg<3>(q, q.o_new); }, 50);
    const double s_r2 = timeit([&] { launch_reg<2>(q0, q0.o_new); }, 50);
    const double s_r3 = timeit([&] { launch_reg<3>(q0, q0.o_new); }, 50);
    const double t_flat = timeit([&] {
      hipLaunchKernelGGL(rw_flat, dim3(4096), dim3(256), 0, 0, (const f32x4 *)q.L[0],
                         (const f32x4 *)q.R[0], (f32x4 *)flat, nr, nw);
    }, 50);
    printf("round %d: pyramid old %6.1f us (%4.0f GB/s, %.3f)   scale0 old %6.1f us (%4.0f GB/s)  flat r2w1 %6.1f us (%4.0f GB/s)\n",
           r, t_old, by / t_old / 1e3, by / t_old / 8e6, s_old, by0 / s_old / 1e3, t_flat, by0 / t_flat / 1e3);
    printf("         pyramid reg2 %6.1f us (%.3f)  reg3 %6.1f us (%.3f)   scale0 reg2 %6.1f us (%4.0f GB/s)  reg3 %6.1f us (%4.0f GB/s)\n",
           t_r2, by / t_r2 / 8e6, t_r3, by / t_r3 / 8e6, s_r2, by0 / s_r2 / 1e3, s_r3, by0 / s_r3 / 1e3);
  }
  printf("algorithmic bytes: pyramid %.1f MB, scale 0 %.1f MB\n", by / 1e6, by0 / 1e6);
  return all ? 0 : 2;
}
