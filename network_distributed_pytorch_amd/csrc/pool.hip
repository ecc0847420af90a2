// Max-pool 2-D (NCHW fp32) forward / backward for gfx950, deterministic.
//
// ResNet's stem `MaxPool2d(3, stride=2, padding=1)` (torchvision resnet, used by the
// reference at ddp_powersgd_guide_cifar10/ddp_init.py:111) runs in PyTorch-ROCm as
// `max_pool_forward_nchw` (writes int64 argmax indices: 2x the output bytes again) and
// `max_pool_backward_nchw`, which scatters with float atomics into a zero-filled grad
// (an extra fill launch, and a summation order that changes run to run where windows
// overlap).  Here:
//   fwd: one thread per output, the winning tap is stored as a uint8 window offset
//        (kh*KW + kw), first maximum in scan order with NaN propagation (same pick as
//        ATen);
//   bwd: one thread per INPUT element gathers the output gradients of every window that
//        chose it, in a fixed (oh, ow) order: no atomics, no zero-fill, bitwise
//        reproducible.
// One flat 1-D grid over all planes (the stem's 8x8 output planes are too small to give a
// workgroup each).  Index math is 32-bit with multiply-shift division by the run-time
// extents (the first version spent most of its time in integer division), and the
// ResNet window (3, 2, 1) is a compile-time instantiation; other windows use K = 0.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ndp_kernels.h"

namespace ndp {

namespace {

constexpr int kPoolThreads = 256;

// n / d for 32-bit n via one mul-hi and a shift (Granlund-Montgomery; exact for all n < 2^32)
struct FastDiv {
  uint32_t d, m, l;
};

FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.l = 0;
  while ((1ull << f.l) < d) ++f.l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << f.l) - d)) / d) + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint32_t t = __umulhi(f.m, n);
  return (uint32_t)(((uint64_t)t + n) >> f.l);
}

struct PoolArgs {
  PoolGeom g;
  FastDiv in_plane, out_plane, w, ow;
  uint32_t total;
};

template <int K, int S, int P>
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_kernel(const float* __restrict__ x,
                                                                   float* __restrict__ y,
                                                                   uint8_t* __restrict__ idx, PoolArgs a) {
  const uint32_t e = blockIdx.x * kPoolThreads + threadIdx.x;
  if (e >= a.total) return;
  const int KH = K ? K : a.g.KH, KW = K ? K : a.g.KW, st = S ? S : a.g.stride, pd = K ? P : a.g.pad;
  const uint32_t plane = fdiv(e, a.out_plane);
  const uint32_t o = e - plane * a.out_plane.d;
  const float* xp = x + (size_t)plane * a.in_plane.d;
  const int oh = (int)fdiv(o, a.ow), ow = (int)(o - (uint32_t)oh * a.ow.d);
  const int h0 = oh * st - pd, w0 = ow * st - pd;
  const int H = a.g.H, W = a.g.W;
  // ATen's pick: start at the first in-bounds tap with -inf, take v > best or NaN
  const int kh0 = h0 < 0 ? -h0 : 0, kw0 = w0 < 0 ? -w0 : 0;
  float best = -INFINITY;
  int arg = kh0 * KW + kw0;
#pragma unroll
  for (int kh = 0; kh < (K ? K : 16); ++kh) {
    if (!K && kh >= KH) break;
    const int h = h0 + kh;
    if (kh < kh0 || h >= H) continue;
#pragma unroll
    for (int kw = 0; kw < (K ? K : 16); ++kw) {
      if (!K && kw >= KW) break;
      const int w = w0 + kw;
      if (kw < kw0 || w >= W) continue;
      const float v = xp[h * W + w];
      if (v > best || isnan(v)) {
        best = v;
        arg = kh * KW + kw;
      }
    }
  }
  y[e] = best;
  idx[e] = (uint8_t)arg;
}

template <int K, int S, int P>
__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_kernel(const float* __restrict__ dy,
                                                                   const uint8_t* __restrict__ idx,
                                                                   float* __restrict__ dx, PoolArgs a) {
  const uint32_t e = blockIdx.x * kPoolThreads + threadIdx.x;
  if (e >= a.total) return;
  const int KH = K ? K : a.g.KH, KW = K ? K : a.g.KW, st = S ? S : a.g.stride, pd = K ? P : a.g.pad;
  const uint32_t plane = fdiv(e, a.in_plane);
  const uint32_t i = e - plane * a.in_plane.d;
  const float* dyp = dy + (size_t)plane * a.out_plane.d;
  const uint8_t* ip = idx + (size_t)plane * a.out_plane.d;
  const int h = (int)fdiv(i, a.w), w = (int)(i - (uint32_t)h * a.w.d);
  // windows containing (h, w): oh*st - pd <= h <= oh*st - pd + KH - 1
  const int hp = h + pd, wp = w + pd;
  const int oh_lo = hp >= KH ? (hp - KH) / st + 1 : 0;
  const int oh_hi = min(hp / st, a.g.OH - 1);
  const int ow_lo = wp >= KW ? (wp - KW) / st + 1 : 0;
  const int ow_hi = min(wp / st, a.g.OW - 1);
  float acc = 0.f;
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int kh = hp - oh * st;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int kw = wp - ow * st;
      const int o = oh * a.g.OW + ow;
      if (ip[o] == kh * KW + kw) acc += dyp[o];
    }
  }
  dx[e] = acc;
}

PoolArgs pool_args(const PoolGeom& g, int64_t total) {
  PoolArgs a;
  a.g = g;
  a.in_plane = make_fastdiv((uint32_t)(g.H * g.W));
  a.out_plane = make_fastdiv((uint32_t)(g.OH * g.OW));
  a.w = make_fastdiv((uint32_t)g.W);
  a.ow = make_fastdiv((uint32_t)g.OW);
  a.total = (uint32_t)total;
  return a;
}

bool resnet_window(const PoolGeom& g) { return g.KH == 3 && g.KW == 3 && g.stride == 2 && g.pad == 1; }

}  // namespace

void launch_maxpool_fwd(const float* x, float* y, uint8_t* idx, int planes, const PoolGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)planes * g.OH * g.OW;
  if (total <= 0) return;
  const PoolArgs a = pool_args(g, total);
  const dim3 grid((unsigned)((total + kPoolThreads - 1) / kPoolThreads));
  if (resnet_window(g))
    hipLaunchKernelGGL((maxpool_fwd_kernel<3, 2, 1>), grid, dim3(kPoolThreads), 0, s, x, y, idx, a);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<0, 0, 0>), grid, dim3(kPoolThreads), 0, s, x, y, idx, a);
}

void launch_maxpool_bwd(const float* dy, const uint8_t* idx, float* dx, int planes, const PoolGeom& g,
                        hipStream_t s) {
  const int64_t total = (int64_t)planes * g.H * g.W;
  if (total <= 0) return;
  const PoolArgs a = pool_args(g, total);
  const dim3 grid((unsigned)((total + kPoolThreads - 1) / kPoolThreads));
  if (resnet_window(g))
    hipLaunchKernelGGL((maxpool_bwd_kernel<3, 2, 1>), grid, dim3(kPoolThreads), 0, s, dy, idx, dx, a);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<0, 0, 0>), grid, dim3(kPoolThreads), 0, s, dy, idx, dx, a);
}

}  // namespace ndp
