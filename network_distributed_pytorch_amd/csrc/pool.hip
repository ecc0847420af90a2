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
#include "pool_route.h"

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

// ---- ResNet stem window (3, 2, 1) on even maps with W % 4 == 0: vectorised fast paths ----
// fwd: one thread per PAIR of outputs (oh, 2j), (oh, 2j + 1): the three input rows'
//      columns 4j .. 4j+3 come as one float4 each, column 4j - 1 from the left lane (the
//      W/4 lanes of a row are adjacent in the wave, W/4 | 64), 2 outputs + 2 index bytes
//      stored together.  Same scan order / NaN rule as the generic kernel.
// bwd: one thread per output position (i, j) writes the 2x2 input block it owns,
//      [2i, 2i+1] x [2j, 2j+1], gathering the (<= 4) windows that can pick each pixel in
//      the generic kernel's (oh, ow) order: float2 stores, no zero-fill, no atomics.
__global__ __launch_bounds__(kPoolThreads) void maxpool_fwd_s2_kernel(const float* __restrict__ x,
                                                                      float* __restrict__ y,
                                                                      uint8_t* __restrict__ idx, PoolArgs a) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const uint32_t e = blockIdx.x * kPoolThreads + threadIdx.x;  // pair index
  const int H = a.g.H, W = a.g.W, OW = a.g.OW, W4 = W >> 2;
  const uint32_t pairs_per_plane = (uint32_t)(a.g.OH * W4);
  const bool live = e < a.total;
  const uint32_t plane = live ? e / pairs_per_plane : 0;
  const uint32_t r = live ? e - plane * pairs_per_plane : 0;
  const int oh = (int)(r / (uint32_t)W4), j = (int)(r - (uint32_t)oh * W4);
  const float* xp = x + (size_t)plane * a.in_plane.d;
  float v[3][5];  // rows 2oh-1 .. 2oh+1, columns 4j-1 .. 4j+3
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int h = 2 * oh - 1 + kh;
    f4 q = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (live && h >= 0 && h < H) q = *reinterpret_cast<const f4*>(xp + h * W + 4 * j);
    const float left = __shfl_up(q.w, 1, 64);
    v[kh][0] = (j > 0) ? left : -INFINITY;
    v[kh][1] = q.x; v[kh][2] = q.y; v[kh][3] = q.z; v[kh][4] = q.w;
  }
  if (!live) return;
  float out[2];
  uint8_t arg[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {  // output column ow = 2j + t: taps at columns 4j - 1 + 2t + kw
    const int ow = 2 * j + t;
    const int kh0 = oh == 0 ? 1 : 0, kw0 = ow == 0 ? 1 : 0;
    float best = -INFINITY;
    int a0 = kh0 * 3 + kw0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      if (kh < kh0 || 2 * oh - 1 + kh >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        if (kw < kw0 || 2 * ow - 1 + kw >= W) continue;
        const float val = v[kh][2 * t + kw];
        if (val > best || isnan(val)) {
          best = val;
          a0 = kh * 3 + kw;
        }
      }
    }
    out[t] = best;
    arg[t] = (uint8_t)a0;
  }
  const size_t o = (size_t)plane * a.out_plane.d + (size_t)oh * OW + 2 * j;
  *reinterpret_cast<float2*>(y + o) = make_float2(out[0], out[1]);
  idx[o] = arg[0];
  idx[o + 1] = arg[1];
}

__global__ __launch_bounds__(kPoolThreads) void maxpool_bwd_s2_kernel(const float* __restrict__ dy,
                                                                      const uint8_t* __restrict__ idx,
                                                                      float* __restrict__ dx, PoolArgs a,
                                                                      PoolBnStats bs) {
  const uint32_t e = blockIdx.x * kPoolThreads + threadIdx.x;  // output position
  if (e >= a.total) return;
  const int OH = a.g.OH, OW = a.g.OW, W = a.g.W;
  const uint32_t plane = fdiv(e, a.out_plane);
  const uint32_t o = e - plane * a.out_plane.d;
  const int i = (int)fdiv(o, a.ow), j = (int)(o - (uint32_t)i * a.ow.d);
  const float* dyp = dy + (size_t)plane * a.out_plane.d;
  const uint8_t* ip = idx + (size_t)plane * a.out_plane.d;
  float d00, d01, d10, d11;
  if (OH == 8 && OW == 8)  // the stem's 8x8 planes: one wave per plane, neighbours by shuffle
    pool_s2_route_wave(dyp[o], ip[o], i, j, d00, d01, d10, d11);
  else
    pool_s2_route(dyp, ip, i, j, OH, OW, d00, d01, d10, d11);
  if (dx != nullptr) {  // (null: statistics only — the fused stem BN backward re-routes the gradient)
    float* dxp = dx + (size_t)plane * a.in_plane.d + (size_t)(2 * i) * W + 2 * j;
    *reinterpret_cast<float2*>(dxp) = make_float2(d00, d01);
    *reinterpret_cast<float2*>(dxp + W) = make_float2(d10, d11);
  }
  if (bs.stats != nullptr) {
    // the BN backward's statistics of this plane (64 outputs = this wave, launcher-checked):
    // dz = d * mask with the ReLU mask recomputed from the BN input x exactly as the fused
    // forward computed its output (bn_relu_maxpool), xhat = (x - mean) * invstd
    const int ch = (int)(plane % (uint32_t)bs.C), n = (int)(plane / (uint32_t)bs.C);
    const float mean = bs.mean[ch], invstd = bs.invstd[ch];
    const float gam = bs.gamma ? bs.gamma[ch] : 1.f, bet = bs.beta ? bs.beta[ch] : 0.f;
    const float sc = __fmul_rn(gam, invstd), sh = __fsub_rn(bet, __fmul_rn(mean, sc));
    const float* xp = bs.x + (size_t)plane * a.in_plane.d + (size_t)(2 * i) * W + 2 * j;
    const float2 x0 = *reinterpret_cast<const float2*>(xp), x1 = *reinterpret_cast<const float2*>(xp + W);
    const float xs[4] = {x0.x, x0.y, x1.x, x1.y}, ds[4] = {d00, d01, d10, d11};
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float dz = fmaf(xs[k], sc, sh) > 0.f ? ds[k] : 0.f;
      sa += dz;
      sb += dz * ((xs[k] - mean) * invstd);
    }
    double da = (double)sa, db = (double)sb;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      da += __shfl_xor(da, off, 64);
      db += __shfl_xor(db, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      double* st = bs.stats + ((int64_t)ch * bs.N + n) * 2;
      st[0] = da;
      st[1] = db;
    }
  }
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

// the vectorised paths: even maps, whole float4 rows, W/4 lanes per row inside one wave
bool s2_fast(const PoolGeom& g) {
  return resnet_window(g) && g.H == 2 * g.OH && g.W == 2 * g.OW && g.W % 4 == 0 && 64 % (g.W / 4) == 0;
}

}  // namespace

void launch_maxpool_fwd(const float* x, float* y, uint8_t* idx, int planes, const PoolGeom& g, hipStream_t s) {
  const int64_t total = (int64_t)planes * g.OH * g.OW;
  if (total <= 0) return;
  if (s2_fast(g)) {
    const int64_t pairs = (int64_t)planes * g.OH * (g.W / 4);
    const PoolArgs a = pool_args(g, pairs);
    hipLaunchKernelGGL(maxpool_fwd_s2_kernel, dim3((unsigned)((pairs + kPoolThreads - 1) / kPoolThreads)),
                       dim3(kPoolThreads), 0, s, x, y, idx, a);
    return;
  }
  const PoolArgs a = pool_args(g, total);
  const dim3 grid((unsigned)((total + kPoolThreads - 1) / kPoolThreads));
  if (resnet_window(g))
    hipLaunchKernelGGL((maxpool_fwd_kernel<3, 2, 1>), grid, dim3(kPoolThreads), 0, s, x, y, idx, a);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<0, 0, 0>), grid, dim3(kPoolThreads), 0, s, x, y, idx, a);
}

bool maxpool_bwd_bnstats_ok(const PoolGeom& g) { return s2_fast(g) && g.OH * g.OW == 64; }

void launch_maxpool_bwd(const float* dy, const uint8_t* idx, float* dx, int planes, const PoolGeom& g,
                        hipStream_t s, const PoolBnStats& bs) {
  const int64_t total = (int64_t)planes * g.H * g.W;
  if (total <= 0) return;
  if (s2_fast(g)) {
    const int64_t outs = (int64_t)planes * g.OH * g.OW;
    const PoolArgs a = pool_args(g, outs);
    hipLaunchKernelGGL(maxpool_bwd_s2_kernel, dim3((unsigned)((outs + kPoolThreads - 1) / kPoolThreads)),
                       dim3(kPoolThreads), 0, s, dy, idx, dx, a, bs);
    return;
  }
  const PoolArgs a = pool_args(g, total);
  const dim3 grid((unsigned)((total + kPoolThreads - 1) / kPoolThreads));
  if (resnet_window(g))
    hipLaunchKernelGGL((maxpool_bwd_kernel<3, 2, 1>), grid, dim3(kPoolThreads), 0, s, dy, idx, dx, a);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<0, 0, 0>), grid, dim3(kPoolThreads), 0, s, dy, idx, dx, a);
}

}  // namespace ndp
