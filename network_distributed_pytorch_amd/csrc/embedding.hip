// Deterministic, graph-replayable embedding backward (gfx950).
//
// grad_W[v, :] = sum over tokens t with ids[t] == v (in increasing t) of grad_out[t, :],
// rows never referenced (and the padding row) are zero.
//
// Why native: PyTorch-ROCm's embedding_dense_backward sorts the ids with rocPRIM when a
// batch has > 3072 of them (DistilBERT: 16 x 512 = 8192); replaying that inside a hipGraph
// faulted the GPU (rocprim partition_kernel, MEMORY_APERTURE_VIOLATION, 2nd replay —
// tools/diag_graph.py).  This version needs no sort, no atomics and no temporary allocation:
//
//  1. emb_rank_kernel — every token t computes, against ALL ids streamed through LDS in
//     8192-id tiles, below = #{t' : id[t'] < id[t]}, same_before = #{t' < t : id[t'] ==
//     id[t]} and same = #{t' : id[t'] == id[t]} (padding / out-of-range ids excluded).
//     slot = below + same_before is a permutation of the valid tokens sorted by
//     (id, position): perm[slot] = t.  The first occurrence (same_before == 0) also records
//     the row's [start, count).  Sixteen lanes share a token (each scans 1/16 of the ids
//     with int4 LDS reads, then a 16-lane xor-shuffle sum): 8192 tokens = 512 workgroups.
//  2. emb_gather_kernel — one 64-lane slice per row: zeros for unreferenced rows,
//     otherwise the fixed-order sum of its tokens' grad rows (float4), then re-arms the
//     row's count to 0 for the next call (counts start zeroed at allocation).
// Cost at DistilBERT's shape: one dense write of grad_W (94 MB) + one read of grad_out.
#include <hip/hip_runtime.h>
#include "ndp_kernels.h"

namespace ndp {

constexpr int kEmbTile = 8192;  // ids per LDS tile (32 KiB)

constexpr int kEmbLanes = 16;  // lanes per token: each scans 1/16 of every tile, int4 at a time

__global__ __launch_bounds__(256) void emb_rank_kernel(const int64_t* __restrict__ ids, int T, int V, int pad,
                                                       int* __restrict__ perm, int* __restrict__ row_start,
                                                       int* __restrict__ row_cnt) {
  typedef int i4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) int tile[kEmbTile];
  const int gt = blockIdx.x * 256 + threadIdx.x;
  const int t = gt / kEmbLanes, part = gt % kEmbLanes;
  int v = -1;
  if (t < T) {
    const int64_t raw = ids[t];
    v = (raw >= 0 && raw < V && raw != pad) ? (int)raw : -1;
  }
  int below = 0, before = 0, same = 0;
  for (int base = 0; base < T; base += kEmbTile) {
    const int n = min(kEmbTile, T - base);
    const int n64 = (n + 63) & ~63;  // whole int4 steps of all 16 lanes; the tail is -1
    __syncthreads();
    for (int i = threadIdx.x; i < n64; i += 256) {
      const int64_t raw = i < n ? ids[base + i] : -1;
      tile[i] = (raw >= 0 && raw < V && raw != pad) ? (int)raw : -1;
    }
    __syncthreads();
    if (v >= 0) {
      // lane `part` reads int4 number part, part + 16, ...: the 16 lanes of a token cover 64
      // consecutive ids per step (the other tokens of the wave read the same addresses:
      // broadcast, no bank conflict)
#pragma unroll 4
      for (int i = 4 * part; i < n64; i += 4 * kEmbLanes) {
        const i4 u = *reinterpret_cast<const i4*>(tile + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int uj = u[j];
          const int valid = uj >= 0;
          below += valid & (uj < v);
          const int eq = uj == v;
          same += eq;
          before += eq & (base + i + j < t);
        }
      }
    }
  }
#pragma unroll
  for (int o = 1; o < kEmbLanes; o <<= 1) {
    below += __shfl_xor(below, o, 64);
    before += __shfl_xor(before, o, 64);
    same += __shfl_xor(same, o, 64);
  }
  if (v >= 0 && part == 0) {
    perm[below + before] = t;
    if (before == 0) {
      row_start[v] = below;
      row_cnt[v] = same;
    }
  }
}

// 64 lanes per row, 4 rows per 256-thread workgroup; D % 4 == 0
__global__ __launch_bounds__(256) void emb_gather_kernel(const float* __restrict__ gout, const int* __restrict__ perm,
                                                         const int* __restrict__ row_start, int* __restrict__ row_cnt,
                                                         float* __restrict__ gw, int V, int D) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (v >= V) return;
  const int cnt = row_cnt[v];
  const int D4 = D >> 2;
  f4* out = reinterpret_cast<f4*>(gw + (int64_t)v * D);
  if (cnt == 0) {
    for (int j = lane; j < D4; j += 64) out[j] = f4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const int start = row_start[v];
  for (int j = lane; j < D4; j += 64) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < cnt; ++k) {
      const int t = perm[start + k];
      acc += reinterpret_cast<const f4*>(gout + (int64_t)t * D)[j];
    }
    out[j] = acc;
  }
  if (lane == 0) row_cnt[v] = 0;  // re-arm: the next call's rank pass only writes referenced rows
}

void launch_embedding_backward(const int64_t* ids, int T, const float* gout, int V, int D, int pad, int* perm,
                               int* row_start, int* row_cnt, float* gw, hipStream_t s) {
  if (T > 0)
    hipLaunchKernelGGL(emb_rank_kernel, dim3((unsigned)(((int64_t)kEmbLanes * T + 255) / 256)), dim3(256), 0, s, ids, T, V,
                       pad, perm,
                       row_start, row_cnt);
  hipLaunchKernelGGL(emb_gather_kernel, dim3((unsigned)((V + 3) / 4)), dim3(256), 0, s, gout, perm, row_start, row_cnt,
                     gw, V, D);
}

}  // namespace ndp
