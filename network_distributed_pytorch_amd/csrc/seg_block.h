// One workgroup (256 threads) of the segmented reduce-copy (multitensor.hip seg_reduce_kernel):
// block `blk` of the entry table.  Shared with the PowerSGD P pass (powersgd.hip), whose extra
// blocks pack the rank-1 group into the comm buffer in the same launch.
#pragma once
#include <hip/hip_runtime.h>
#include "ndp_kernels.h"

namespace ndp {

typedef float seg_f32x4 __attribute__((ext_vector_type(4)));
#define NDP_SEG_GLOBAL __attribute__((address_space(1)))
__device__ __forceinline__ seg_f32x4 seg_ld4(const float NDP_SEG_GLOBAL* p) {
  return *reinterpret_cast<const seg_f32x4 NDP_SEG_GLOBAL*>(p);
}
__device__ __forceinline__ void seg_st4(float NDP_SEG_GLOBAL* p, seg_f32x4 v) {
  *reinterpret_cast<seg_f32x4 NDP_SEG_GLOBAL*>(p) = v;
}

__device__ __forceinline__ void seg_reduce_block(const SegEntry* __restrict__ ents,
                                                 const int64_t* __restrict__ prefix, int n_ent, int64_t blk) {
  int lo = 0, hi = n_ent - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  const SegEntry E = ents[lo];
  const float NDP_SEG_GLOBAL* const src = (const float NDP_SEG_GLOBAL*)E.src;
  float NDP_SEG_GLOBAL* const dst = (float NDP_SEG_GLOBAL*)E.dst;
  const int64_t base = (blk - prefix[lo]) * kSegBlockElems;
  const bool scale = E.div != 1.0f;
  if (E.vec) {
    // Split-K P / Q slabs (up to ~20 chunks): the chunk loads are issued kSegBatch at a time
    // for both float4 of the thread before any add, so a block costs ~chunks / 8 memory
    // round trips instead of one per chunk (the adds keep chunk order: bitwise unchanged).
    constexpr int QN = kSegBlockElems / 1024;
    constexpr int kSegBatch = 8;
    int64_t kq[QN];
    bool full[QN];
    seg_f32x4 acc[QN];
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      kq[q] = base + (int64_t)(q * 256 + threadIdx.x) * 4;
      full[q] = kq[q] + 3 < E.numel;
      acc[q] = full[q] ? seg_ld4(src + kq[q]) : seg_f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int c = 1;
    for (; c + kSegBatch <= E.chunks; c += kSegBatch) {
      seg_f32x4 t[QN][kSegBatch];
#pragma unroll
      for (int j = 0; j < kSegBatch; ++j)
#pragma unroll
        for (int q = 0; q < QN; ++q)
          t[q][j] = full[q] ? seg_ld4(src + (int64_t)(c + j) * E.stride + kq[q]) : seg_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < QN; ++q)
#pragma unroll
        for (int j = 0; j < kSegBatch; ++j) acc[q] += t[q][j];
    }
    for (; c < E.chunks; ++c)
#pragma unroll
      for (int q = 0; q < QN; ++q)
        if (full[q]) acc[q] += seg_ld4(src + (int64_t)c * E.stride + kq[q]);
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int64_t k = kq[q];
      if (full[q]) {
        if (scale) acc[q] = acc[q] / E.div;
        seg_st4(dst + k, acc[q]);
      } else if (k < E.numel) {
        for (int j = 0; j < 4; ++j) {
          if (k + j >= E.numel) break;
          float t = src[k + j];
          for (int z = 1; z < E.chunks; ++z) t += src[(int64_t)z * E.stride + k + j];
          if (scale) t = t / E.div;
          dst[k + j] = t;
        }
      }
    }
  } else {
    for (int q = 0; q < kSegBlockElems / 256; ++q) {
      const int64_t k = base + q * 256 + threadIdx.x;
      if (k >= E.numel) break;
      float acc = src[k];
      for (int c = 1; c < E.chunks; ++c) acc += src[(int64_t)c * E.stride + k];
      if (scale) acc = acc / E.div;
      dst[k] = acc;
    }
  }
}

}  // namespace ndp
