// Linear-layer bias gradient: db[n] = sum_m g[m, n] — deterministic and hipGraph-safe.
//
// PyTorch-ROCm computes it with at::native::reduce_kernel; for the DistilBERT shapes
// (8192 x 768 / 3072 rows x columns) that reduction is multi-block with a global staging
// buffer and, replayed inside a captured hipGraph, returned garbage for some layers
// (k_lin / lin1 bias grads off by 5e-2 while eager was exact — tools/
// diag_bert_graph_vs_eager.py), besides costing 18 µs a call.  Here:
//   pass 1: workgroup (column strip of 256 columns, row chunk) — 64 lanes own 4 columns
//           each (float4 loads, whole rows coalesced), 4 lane groups stride the chunk's
//           rows; the 4 group sums are added in LDS in fixed order -> part[chunk][n];
//   pass 2: db[n] = sum over chunks (conv.hip's split-K slab sum: 16 chunk groups per float4
//           column, group sums added in fixed order — a serial per-column loop here took 18 µs
//           per DistilBERT Linear, profiles/r2/distilbert_psgd_r8_graph_kernels.md).
// Fixed summation order everywhere: bitwise reproducible, no atomics, no semaphores.
#include <hip/hip_runtime.h>
#include "ndp_kernels.h"

namespace ndp {

typedef float f4l __attribute__((ext_vector_type(4)));

// rows of a lane group in flight together (4 independent float4 loads per lane per step)
constexpr int kColUnroll = 4;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ g, int64_t M, int N,
                                                             int rows_per_chunk, float* __restrict__ part) {
  __shared__ f4l red[4][64];
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63);  // float4 column index
  const int grp = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(M, r0 + rows_per_chunk);
  f4l acc = {0.f, 0.f, 0.f, 0.f};
  if (4 * c4 < N) {
    const f4l* src = reinterpret_cast<const f4l*>(g) + c4;
    const int64_t n4 = N / 4;
    int64_t r = r0 + grp;
    for (; r + 4 * (kColUnroll - 1) < r1; r += 4 * kColUnroll) {
      f4l v[kColUnroll];
#pragma unroll
      for (int u = 0; u < kColUnroll; ++u) v[u] = src[(r + 4 * u) * n4];
#pragma unroll
      for (int u = 0; u < kColUnroll; ++u) acc += v[u];
    }
    for (; r < r1; r += 4) acc += src[r * n4];
  }
  red[grp][threadIdx.x & 63] = acc;
  __syncthreads();
  if (grp == 0 && 4 * c4 < N) {
    const int l = threadIdx.x;
    const f4l s = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
    reinterpret_cast<f4l*>(part + (int64_t)blockIdx.y * N)[c4] = s;
  }
}

// FFN first layer (DistilBERT lin1 + exact GELU): dh = g * gelu'(h) with PyTorch's formula
// (GeluBackwardCUDAKernelImpl, approximate='none'), written out AND summed per column chunk in
// the same pass (pass 1 of the bias gradient) — the separate GELU-backward launch and the
// bias-sum re-read of dh (100 MB per DistilBERT layer) disappear.
__device__ __forceinline__ float gelu_grad(float dy, float x) {
  constexpr float kBeta = 0.3989422804014327f;  // M_2_SQRTPI * M_SQRT1_2 * 0.5
  constexpr float kAlpha = 0.7071067811865476f;  // M_SQRT1_2
  const float cdf = 0.5f * (1.f + erff(x * kAlpha));
  const float pdf = expf(-0.5f * x * x) * kBeta;
  return dy * (cdf + x * pdf);
}

__global__ __launch_bounds__(256) void gelu_bwd_colsum_partial_kernel(const float* __restrict__ g,
                                                                      const float* __restrict__ h,
                                                                      float* __restrict__ dh, int64_t M, int N,
                                                                      int rows_per_chunk, float* __restrict__ part) {
  __shared__ f4l red[4][64];
  const int c4 = blockIdx.x * 64 + (threadIdx.x & 63);
  const int grp = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(M, r0 + rows_per_chunk);
  f4l acc = {0.f, 0.f, 0.f, 0.f};
  if (4 * c4 < N) {
    const int64_t n4 = N / 4;
    const f4l* gs = reinterpret_cast<const f4l*>(g) + c4;
    const f4l* hs = reinterpret_cast<const f4l*>(h) + c4;
    f4l* ds = reinterpret_cast<f4l*>(dh) + c4;
    int64_t r = r0 + grp;
    for (; r + 4 * (kColUnroll - 1) < r1; r += 4 * kColUnroll) {
      f4l gv[kColUnroll], hv[kColUnroll];
#pragma unroll
      for (int u = 0; u < kColUnroll; ++u) {
        gv[u] = gs[(r + 4 * u) * n4];
        hv[u] = hs[(r + 4 * u) * n4];
      }
#pragma unroll
      for (int u = 0; u < kColUnroll; ++u) {
        f4l d;
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = gelu_grad(gv[u][j], hv[u][j]);
        ds[(r + 4 * u) * n4] = d;
        acc += d;
      }
    }
    for (; r < r1; r += 4) {
      const f4l gv = gs[r * n4], hv = hs[r * n4];
      f4l d;
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = gelu_grad(gv[j], hv[j]);
      ds[r * n4] = d;
      acc += d;
    }
  }
  red[grp][threadIdx.x & 63] = acc;
  __syncthreads();
  if (grp == 0 && 4 * c4 < N) {
    const int l = threadIdx.x;
    const f4l s = ((red[0][l] + red[1][l]) + red[2][l]) + red[3][l];
    reinterpret_cast<f4l*>(part + (int64_t)blockIdx.y * N)[c4] = s;
  }
}

void launch_gelu_bwd_colsum(const float* g, const float* h, float* dh, int64_t M, int N, float* part, float* out,
                            hipStream_t s) {
  const int chunks = colsum_chunks(M, N);
  const int rpc = (int)((M + chunks - 1) / chunks);
  const int strips = (N / 4 + 63) / 64;
  hipLaunchKernelGGL(gelu_bwd_colsum_partial_kernel, dim3(strips, chunks), dim3(256), 0, s, g, h, dh, M, N, rpc, part);
  if (out != nullptr) launch_slab_sum(part, out, N, chunks, s);  // else: the caller sums (deferred)
}

int colsum_chunks(int64_t M, int N) {
  const int strips = (N / 4 + 63) / 64;
  int chunks = (1024 + strips - 1) / strips;         // ~1024 workgroups (4 per CU) in pass 1
  const int64_t max_chunks = (M + 31) / 32;          // >= 32 rows per chunk
  if (chunks > max_chunks) chunks = (int)max_chunks;
  return chunks < 1 ? 1 : chunks;
}

void launch_colsum(const float* g, int64_t M, int N, float* part, float* out, hipStream_t s) {
  const int chunks = colsum_chunks(M, N);
  const int rpc = (int)((M + chunks - 1) / chunks);
  const int strips = (N / 4 + 63) / 64;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(strips, chunks), dim3(256), 0, s, g, M, N, rpc, part);
  if (out != nullptr) launch_slab_sum(part, out, N, chunks, s);  // else: the caller sums (deferred)
}

}  // namespace ndp
