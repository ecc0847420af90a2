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
//   dropout (HF DistilBERT's hidden dropouts, fused instead of ATen's fused_dropout + mask
//   tensor + masked_scale backward): keep(row, col) = hash(seed, row, col) >= p * 2^32, a
//   stateless counter hash, so backward regenerates the forward mask; the seed is a device
//   int32 (graph-replay safe).
//     DM 1 (FFN):        s = drop(a) + b   -> bwd writes dx (residual) and da = drop'(dx)
//     DM 2 (embeddings): y = drop(LN(a + b)) -> bwd reads dy * keep * scale
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

// keep-mask hash of element (row, col); tools-side twin: ops/layernorm.py ln_keep_mask
__device__ __forceinline__ uint32_t ln_hash(uint32_t seed, uint32_t row, uint32_t col) {
  uint32_t h = (seed * 0x9E3779B1u) ^ ((row + 0x7F4A7C15u) * 0x85EBCA77u);
  h = (h ^ (h >> 15)) * 0x2C1B3C6Du;
  h ^= (col + 0x165667B1u) * 0xC2B2AE3Du;
  h = (h ^ (h >> 13)) * 0x297A2D39u;
  return h ^ (h >> 16);
}

// v * (keep ? scale : 0) for the 4 columns c0..c0+3 of row r
__device__ __forceinline__ f4ln ln_drop4(f4ln v, uint32_t seed, uint32_t r, uint32_t c0, uint32_t thr,
                                         float scale) {
  f4ln o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = ln_hash(seed, r, c0 + j) >= thr ? v[j] * scale : 0.f;
  return o;
}

// V = float4 slots per lane (D = 256 * V); DM = dropout mode (header)
template <int V, int DM>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float* __restrict__ y, float* __restrict__ s_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int64_t R, float eps, LnDrop dp) {
  constexpr int D = 256 * V;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const uint32_t seed = DM ? (uint32_t)*dp.seed : 0u;
  const f4ln* ar = reinterpret_cast<const f4ln*>(a + r * D);
  const f4ln* br = b ? reinterpret_cast<const f4ln*>(b + r * D) : nullptr;
  f4ln v[V];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    v[i] = ar[lane + 64 * i];
    if (DM == 1) v[i] = ln_drop4(v[i], seed, (uint32_t)r, 4u * (lane + 64 * i), dp.thr, dp.scale);
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
    const f4ln o = (v[i] - mean) * rstd * g4[j] + b4[j];
    yr[j] = DM == 2 ? ln_drop4(o, seed, (uint32_t)r, 4u * j, dp.thr, dp.scale) : o;
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

template <int V, int DM>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ s,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, float* __restrict__ dx,
                                                     float* __restrict__ part, int64_t R, int rows_per_wave,
                                                     LnDrop dp) {
  constexpr int D = 256 * V;
  const uint32_t seed = DM ? (uint32_t)*dp.seed : 0u;
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
      f4ln d = dyr[lane + 64 * i];
      if (DM == 2) d = ln_drop4(d, seed, (uint32_t)r, 4u * (lane + 64 * i), dp.thr, dp.scale);
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
    for (int i = 0; i < V; ++i) {
      const f4ln g = (gg[i] - c1 - xh[i] * c2) * rstd;
      dxr[lane + 64 * i] = g;
      if (DM == 1)
        reinterpret_cast<f4ln*>(dp.da + r * D)[lane + 64 * i] =
            ln_drop4(g, seed, (uint32_t)r, 4u * (lane + 64 * i), dp.thr, dp.scale);
    }
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

#define LN_SWITCH(D, DM, K, ...)                                               \
  switch ((D) / 256 * 4 + (DM)) {                                               \
    case 4: K<1, 0>__VA_ARGS__; break;  case 5: K<1, 1>__VA_ARGS__; break;     \
    case 6: K<1, 2>__VA_ARGS__; break;  case 8: K<2, 0>__VA_ARGS__; break;     \
    case 9: K<2, 1>__VA_ARGS__; break;  case 10: K<2, 2>__VA_ARGS__; break;    \
    case 12: K<3, 0>__VA_ARGS__; break; case 13: K<3, 1>__VA_ARGS__; break;    \
    case 14: K<3, 2>__VA_ARGS__; break; case 16: K<4, 0>__VA_ARGS__; break;    \
    case 17: K<4, 1>__VA_ARGS__; break; default: K<4, 2>__VA_ARGS__; break;    \
  }

template <int V, int DM>
static void ln_fwd_go(dim3 grid, hipStream_t st, const float* a, const float* b, const float* gamma, const float* beta,
                      float* y, float* s, float* mean, float* rstd, int64_t R, float eps, const LnDrop& dp) {
  hipLaunchKernelGGL((ln_fwd_kernel<V, DM>), grid, dim3(256), 0, st, a, b, gamma, beta, y, s, mean, rstd, R, eps, dp);
}

template <int V, int DM>
static void ln_bwd_go(dim3 grid, hipStream_t st, const float* dy, const float* s, const float* mean, const float* rstd,
                      const float* gamma, float* dx, float* part, int64_t R, int rpw, const LnDrop& dp) {
  hipLaunchKernelGGL((ln_bwd_kernel<V, DM>), grid, dim3(256), 0, st, dy, s, mean, rstd, gamma, dx, part, R, rpw, dp);
}

void launch_ln_fwd(const float* a, const float* b, const float* gamma, const float* beta, float* y, float* s,
                   float* mean, float* rstd, int64_t R, int D, float eps, hipStream_t st, const LnDrop& dp) {
  const dim3 grid((unsigned)((R + 3) / 4));
  LN_SWITCH(D, dp.mode, ln_fwd_go, (grid, st, a, b, gamma, beta, y, s, mean, rstd, R, eps, dp))
}

// workgroups of the backward (= slabs of its [dgamma | dbeta] partial): <= 512, 4 waves each
int ln_bwd_wgs(int64_t R) {
  int64_t wgs = (R + 3) / 4;  // at least one row per wave
  if (wgs > 512) wgs = 512;
  return (int)(wgs < 1 ? 1 : wgs);
}

void launch_ln_bwd(const float* dy, const float* s, const float* mean, const float* rstd, const float* gamma,
                   float* dx, float* part, float* dgb, int64_t R, int D, hipStream_t st, const LnDrop& dp) {
  const int wgs = ln_bwd_wgs(R);
  const int rpw = (int)((R + 4LL * wgs - 1) / (4LL * wgs));
  LN_SWITCH(D, dp.mode, ln_bwd_go, (dim3(wgs), st, dy, s, mean, rstd, gamma, dx, part, R, rpw, dp))
  if (dgb != nullptr) launch_slab_sum(part, dgb, 2LL * D, wgs, st);  // else: the caller sums (deferred)
}

}  // namespace ndp
