// deconv.hip -- output assembly of the 2-D transposed convs of the hourglasses (GANetFeature and
// HourglassRefinement: Conv2x(deconv=True) = ConvTranspose2d(k = 4, stride 2, padding 1) + BN +
// ReLU, then torch.cat with the skip; nets/feature.py:342-376, nets/refinement.py:109-197).
//
// A stride-2 transposed conv is four ordinary convs, one per output phase (a, b) = (Y % 2, X % 2):
// out[c][2y+a][2x+b] = sum_ci sum_{ty,tx in 0,1} in[ci][y+a-1+ty][x+b-1+tx] W[ci][c][3-a-2ty][3-b-2tx].
// The host (ops.deconv2x) runs them as ONE 2x2, pad-1 conv on the implicit-GEMM engine with 4*co
// outputs (phase channel 4c + 2a + b; BN folded, ReLU in its epilogue), whose output element
// [4c+2a+b][y+a][x+b] is out[c][2y+a][2x+b].  This kernel scatters those phase planes into the
// 2x resolution output and appends the skip tensor's channels after them (the concat), so the
// transposed conv costs one engine launch and one memory-bound pass -- instead of MIOpen's
// transposed-conv solvers (backward-data GEMM + col2im + layout transposes) and a torch.cat.
#include "common.h"

namespace {

// one thread per 4 output columns (a quad) of one output row of one channel
__global__ __launch_bounds__(256) void deconv2x_assemble_kernel(const float *__restrict__ ph,
                                                                const float *__restrict__ rem,
                                                                float *__restrict__ out, int n,
                                                                int co, int cr, int h, int w) {
  const int W2 = 2 * w, H2 = 2 * h, qpr = (W2 + 3) / 4, ct = co + cr;
  const long total = (long)n * ct * H2 * qpr;
  const long ph_plane = (long)(h + 1) * (w + 1), o_plane = (long)H2 * W2;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int q = (int)(e % qpr);
    long r = e / qpr;
    const int Y = (int)(r % H2);
    r /= H2;
    const int c = (int)(r % ct), img = (int)(r / ct);
    const int X0 = 4 * q;
    float *dst = out + ((long)img * ct + c) * o_plane + (long)Y * W2;
    float v[4];
    if (c < co) {
      // columns X0 + u: phase b = u & 1, input column x = (X0 + u) >> 1, conv column x + b
      const int a = Y & 1, y = Y >> 1;
      const float *p0 = ph + ((long)img * 4 * co + 4 * c + 2 * a) * ph_plane + (long)(y + a) * (w + 1);
      const float *p1 = p0 + ph_plane;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int X = X0 + u, x = X >> 1;
        v[u] = X < W2 ? ((u & 1) ? p1[x + 1] : p0[x]) : 0.f;
      }
    } else {
      const float *src = rem + ((long)img * cr + (c - co)) * o_plane + (long)Y * W2;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = X0 + u < W2 ? src[X0 + u] : 0.f;
    }
    if ((W2 & 3) == 0) {
      *reinterpret_cast<f32x4 *>(dst + X0) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (X0 + u < W2) dst[X0 + u] = v[u];
    }
  }
}

// Channels-last form: the assembled [n][2h][2w][co + cr] tensor, for a consumer conv that stages
// NHWC input (the Conv2x conv2 3x3 on the engine's halo tile).  A workgroup takes 64 output
// columns (32 past 248 channels) of one output row and every channel: the phase / skip rows are read along x (two or
// one contiguous segments per channel) into LDS [channel][column], then each column's channel
// vector is written as contiguous 16-byte quads (the 32 columns' vectors are one contiguous run).
// PHASE false: the first source is a plain NCHW tensor of the output size (the torch.cat of a
// non-transposed Conv2x, aanet_concat_nhwc_f32).
template <bool PHASE, int AC>  // AC: output columns per workgroup (64, or 32 past 248 channels)
__global__ __launch_bounds__(256) void deconv2x_assemble_nhwc_kernel(const float *__restrict__ ph,
                                                                     const float *__restrict__ rem,
                                                                     float *__restrict__ out, int co,
                                                                     int cr, int h, int w) {
  extern __shared__ float s[];  // [ct][AC + 1]
  const int W2 = 2 * w, H2 = 2 * h, ct = co + cr;
  const int X0 = blockIdx.x * AC, Y = blockIdx.y, img = blockIdx.z;
  const int a = Y & 1, y = Y >> 1;
  const long ph_plane = (long)(h + 1) * (w + 1), o_plane = (long)H2 * W2;
  const int ncol = min(AC, W2 - X0);
  // element e = (channel c, lane-column l) with l fastest: one wave instruction reads a whole
  // channel row -- for a phase channel, columns of parity b = l / (AC/2) at phase index
  // j = l % (AC/2) (two contiguous runs, of phases (a, 0) and (a, 1)); for the skip / plain
  // source, AC contiguous columns.  Four loads in flight per thread before their LDS stores.
  constexpr int HALF = AC / 2;
  const int total = ct * AC;
  for (int e0 = threadIdx.x; e0 < total; e0 += 4 * 256) {
    float v[4];
    int so[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = e0 + 256 * i, c = e / AC, l = e % AC;
      int u = l;
      float t = 0.f;
      if (c < co && PHASE) {
        const int b = l / HALF, jx = l % HALF;
        u = 2 * jx + b;
        if (e < total && u < ncol)
          t = ph[((long)img * 4 * co + 4 * c + 2 * a + b) * ph_plane + (long)(y + a) * (w + 1) +
                 X0 / 2 + jx + b];
      } else if (e < total && u < ncol) {
        t = c < co ? ph[((long)img * co + c) * o_plane + (long)Y * W2 + X0 + u]
                   : rem[((long)img * cr + (c - co)) * o_plane + (long)Y * W2 + X0 + u];
      }
      v[i] = t;
      so[i] = e < total ? c * (AC + 1) + u : -1;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (so[i] >= 0) s[so[i]] = v[i];
  }
  __syncthreads();
  float *dst = out + (((long)img * H2 + Y) * W2 + X0) * ct;
  if ((ct & 3) == 0) {
    const int cq = ct / 4;
    for (int e = threadIdx.x; e < ncol * cq; e += 256) {
      const int u = e / cq, c = 4 * (e % cq);
      *reinterpret_cast<f32x4 *>(dst + (long)u * ct + c) =
          f32x4{s[c * (AC + 1) + u], s[(c + 1) * (AC + 1) + u], s[(c + 2) * (AC + 1) + u],
                s[(c + 3) * (AC + 1) + u]};
    }
  } else {
    for (int e = threadIdx.x; e < ncol * ct; e += 256) {
      const int u = e / ct, c = e % ct;
      dst[(long)u * ct + c] = s[c * (AC + 1) + u];
    }
  }
}

template <bool PHASE>
int launch_nhwc(const float *src, const float *rem, float *out, int n, int co, int cr, int h,
                int w, hipStream_t st) {
  const int ct = co + cr;
  if ((long)ct * 65 * 4 <= 64 * 1024)
    hipLaunchKernelGGL((deconv2x_assemble_nhwc_kernel<PHASE, 64>), dim3((unsigned)host_div_up(2 * w, 64), 2 * h, n),
                       dim3(256), (unsigned)(ct * 65 * 4), st, src, rem, out, co, cr, h, w);
  else if ((long)ct * 33 * 4 <= 64 * 1024)
    hipLaunchKernelGGL((deconv2x_assemble_nhwc_kernel<PHASE, 32>), dim3((unsigned)host_div_up(2 * w, 32), 2 * h, n),
                       dim3(256), (unsigned)(ct * 33 * 4), st, src, rem, out, co, cr, h, w);
  else
    return AANET_EUNSUPPORTED;
  return aanet_launch_status();
}

}  // namespace

extern "C" int aanet_deconv2x_assemble_nhwc_f32(const float *ph, const float *rem, float *out,
                                                int n, int co, int cr, int h, int w,
                                                aanet_stream_t stream) {
  if (n < 0 || co < 0 || cr < 0 || h < 0 || w < 0) return AANET_EINVAL;
  if ((long)n * (co + cr) * h * w == 0) return AANET_OK;
  if (!out || (co && !ph) || (cr && !rem)) return AANET_EINVAL;
  if (2L * h > 65535 || n > 65535) return AANET_EUNSUPPORTED;
  return launch_nhwc<true>(ph, rem, out, n, co, cr, h, w, as_hip(stream));
}

extern "C" int aanet_concat_nhwc_f32(const float *a, const float *b, float *out, int n, int ca,
                                     int cb, int h, int w, aanet_stream_t stream) {
  if (n < 0 || ca < 0 || cb < 0 || h < 0 || w < 0) return AANET_EINVAL;
  if ((long)n * (ca + cb) * h * w == 0) return AANET_OK;
  if (!out || (ca && !a) || (cb && !b)) return AANET_EINVAL;
  if (h > 65535 || n > 65535 || (h & 1) || (w & 1)) return AANET_EUNSUPPORTED;
  // the kernel works in output (2h', 2w') units: h' = h / 2, w' = w / 2
  return launch_nhwc<false>(a, b, out, n, ca, cb, h / 2, w / 2, as_hip(stream));
}

extern "C" int aanet_deconv2x_assemble_f32(const float *ph, const float *rem, float *out, int n,
                                           int co, int cr, int h, int w, aanet_stream_t stream) {
  if (n < 0 || co < 0 || cr < 0 || h < 0 || w < 0) return AANET_EINVAL;
  const long total = (long)n * (co + cr) * 2 * h * ((2 * w + 3) / 4);
  if (total == 0) return AANET_OK;
  if (!out || (co && !ph) || (cr && !rem)) return AANET_EINVAL;
  const long blocks = host_div_up(total, 256);
  hipLaunchKernelGGL(deconv2x_assemble_kernel, dim3((unsigned)(blocks > 65536 ? 65536 : blocks)),
                     dim3(256), 0, as_hip(stream), ph, rem, out, n, co, cr, h, w);
  return aanet_launch_status();
}
