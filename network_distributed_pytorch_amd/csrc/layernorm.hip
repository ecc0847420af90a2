// Fused residual add + LayerNorm over the last dimension (DistilBERT: 8192 rows x 768).
//
// DistilBERT's blocks are y = LayerNorm(sublayer(x) + x).  PyTorch-ROCm runs the add, the
// LayerNorm forward, and in backward layer_norm_grad_input + cuComputePartGradGammaBeta +
// cuComputeGradGammaBeta: ~0.9 ms of a 22.7 ms DistilBERT step over 13 LayerNorms
// (profiles/r2/distilbert_psgd_r8_graph_kernels.md).  Here:
//   fwd: one wave per row, the row in registers (D / 64 floats per lane, float4 loads):
//        s = a (+ b), mean and centred variance by wave butterflies (every lane ends with
//        the same value), y = (s - mean) * rstd * gamma + beta; s, mean, rstd are saved.
//   bwd: one wave per row again: xhat = (s - mean) * rstd, g = dy * gamma,
//        dx = rstd * (g - mean(g) - xhat * mean(g * xhat)); each wave also accumulates
//        dy * xhat and dy for its columns over its rows, the 4 waves of a workgroup add
//        theirs in fixed order, and the per-workgroup [dgamma | dbeta] partials are summed
//        by conv.hip's slab sum (fixed order): deterministic, no atomics.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ndp_kernels.h"

namespace ndp {

typedef float f4ln __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float ln_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// V = float4 slots per lane (D = 256 * V)
template <int V>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ y, float* __restrict__ s_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t R, float eps) {
  constexpr int D = 256 * V;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const f4ln* ar = reinterpret_cast<const f4ln*>(a + r * D);
  const f4ln* br = b ? reinterpret_cast<const f4ln*>(b + r * D) : nullptr;
  f4ln v[V];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = ar[lane + 64 * i];
    if (br) v[i] += br[lane + 64 * i];
    sum += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = ln_wave_sum(sum) * (1.f / D);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const f4ln c = v[i] - mean;
    sq += (c.x * c.x + c.y * c.y) + (c.z * c.z + c.w * c.w);
  }
  const float rstd = rsqrtf(ln_wave_sum(sq) * (1.f / D) + eps);
  const f4ln* g4 = reinterpret_cast<const f4ln*>(gamma);
  const f4ln* b4 = reinterpret_cast<const f4ln*>(beta);
  f4ln* yr = reinterpret_cast<f4ln*>(y + r * D);
  f4ln* sr = reinterpret_cast<f4ln*>(s_out + r * D);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int j = lane + 64 * i;
    sr[j] = v[i];
    yr[j] = (v[i] - mean) * rstd * g4[j] + b4[j];
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

template <int V>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ s,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, float* __restrict__ dx,
                                                     float* __restrict__ part, int64_t R, int rows_per_wave) {
  constexpr int D = 256 * V;
  __shared__ f4ln red[2][4][64 * V];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f4ln* g4 = reinterpret_cast<const f4ln*>(gamma);
  f4ln gam[V], accg[V], accb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    gam[i] = g4[lane + 64 * i];
    accg[i] = f4ln{0.f, 0.f, 0.f, 0.f};
    accb[i] = f4ln{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * rows_per_wave;
  for (int k = 0; k < rows_per_wave; ++k) {
    const int64_t r = r0 + k;
    if (r >= R) break;
    const f4ln* dyr = reinterpret_cast<const f4ln*>(dy + r * D);
    const f4ln* sr = reinterpret_cast<const f4ln*>(s + r * D);
    const float mean = mean_in[r], rstd = rstd_in[r];
    f4ln xh[V], gg[V];
    float c1 = 0.f, c2 = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const f4ln d = dyr[lane + 64 * i];
      xh[i] = (sr[lane + 64 * i] - mean) * rstd;
      gg[i] = d * gam[i];
      accg[i] += d * xh[i];
      accb[i] += d;
      c1 += (gg[i].x + gg[i].y) + (gg[i].z + gg[i].w);
      const f4ln p = gg[i] * xh[i];
      c2 += (p.x + p.y) + (p.z + p.w);
    }
    c1 = ln_wave_sum(c1) * (1.f / D);
    c2 = ln_wave_sum(c2) * (1.f / D);
    f4ln* dxr = reinterpret_cast<f4ln*>(dx + r * D);
#pragma unroll
    for (int i = 0; i < V; ++i) dxr[lane + 64 * i] = (gg[i] - c1 - xh[i] * c2) * rstd;
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    red[0][wave][lane + 64 * i] = accg[i];
    red[1][wave][lane + 64 * i] = accb[i];
  }
  __syncthreads();
  // workgroup partial [dgamma | dbeta] (2 * D floats), the 4 waves added in order
  f4ln* out = reinterpret_cast<f4ln*>(part + (int64_t)blockIdx.x * 2 * D);
  for (int j = threadIdx.x; j < 2 * 64 * V; j += 256) {
    const int h = j / (64 * V), c = j - h * 64 * V;
    out[j] = ((red[h][0][c] + red[h][1][c]) + red[h][2][c]) + red[h][3][c];
  }
}

bool ln_supported(int D) { return D == 256 || D == 512 || D == 768 || D == 1024; }

void launch_ln_fwd(const float* a, const float* b, const float* gamma, const float* beta, float* y, float* s,
                   float* mean, float* rstd, int64_t R, int D, float eps, hipStream_t st) {
  const dim3 grid((unsigned)((R + 3) / 4));
  switch (D) {
    case 256: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, dim3(256), 0, st, a, b, gamma, beta, y, s, mean, rstd, R, eps); break;
    case 512: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, dim3(256), 0, st, a, b, gamma, beta, y, s, mean, rstd, R, eps); break;
    case 768: hipLaunchKernelGGL(ln_fwd_kernel<3>, grid, dim3(256), 0, st, a, b, gamma, beta, y, s, mean, rstd, R, eps); break;
    default: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, dim3(256), 0, st, a, b, gamma, beta, y, s, mean, rstd, R, eps); break;
  }
}

// workgroups of the backward (= slabs of its [dgamma | dbeta] partial): <= 512, 4 waves each
int ln_bwd_wgs(int64_t R) {
  int64_t wgs = (R + 3) / 4;  // at least one row per wave
  if (wgs > 512) wgs = 512;
  return (int)(wgs < 1 ? 1 : wgs);
}

void launch_ln_bwd(const float* dy, const float* s, const float* mean, const float* rstd, const float* gamma,
                   float* dx, float* part, float* dgb, int64_t R, int D, hipStream_t st) {
  const int wgs = ln_bwd_wgs(R);
  const int rpw = (int)((R + 4LL * wgs - 1) / (4LL * wgs));
  switch (D) {
    case 256: hipLaunchKernelGGL(ln_bwd_kernel<1>, dim3(wgs), dim3(256), 0, st, dy, s, mean, rstd, gamma, dx, part, R, rpw); break;
    case 512: hipLaunchKernelGGL(ln_bwd_kernel<2>, dim3(wgs), dim3(256), 0, st, dy, s, mean, rstd, gamma, dx, part, R, rpw); break;
    case 768: hipLaunchKernelGGL(ln_bwd_kernel<3>, dim3(wgs), dim3(256), 0, st, dy, s, mean, rstd, gamma, dx, part, R, rpw); break;
    default: hipLaunchKernelGGL(ln_bwd_kernel<4>, dim3(wgs), dim3(256), 0, st, dy, s, mean, rstd, gamma, dx, part, R, rpw); break;
  }
  launch_slab_sum(part, dgb, 2LL * D, wgs, st);
}

}  // namespace ndp
