// Fused training BatchNorm2d (+ residual add) (+ ReLU) for NCHW fp32 on gfx950.
//
// ResNet's conv -> BN -> (+identity) -> ReLU tail costs, in PyTorch-ROCm, a MIOpen BN
// kernel, an ATen ReLU, an ATen add and an ATen `num_batches_tracked += 1` per layer in
// forward and the mirror image in backward: ~100 latency-bound launches per ResNet-18
// step (profiles/resnet18_powersgd_r4_graph_kernels.md).  Here each direction is two
// kernels over a (slice, channel) grid:
//   fwd:  stats  -> per-(channel, slice) fp64 sum / sum of squares
//         apply  -> every workgroup folds its channel's slices in a fixed order (same
//                   value everywhere), y = relu(x*scale + shift [+ res]); slice 0 also
//                   writes save_mean/invstd, the running stats and num_batches_tracked
//   bwd:  stats  -> per-slice sums of dz = dy*(y>0) and dz*xhat
//         apply  -> dx = gamma*invstd/M * (M dz - sum dz - xhat * sum dz*xhat),
//                   dres = dz (residual branch), slice 0 writes dgamma / dbeta
// Statistics are accumulated in fp64 and combined in a fixed order: bitwise
// reproducible, and at least as accurate as the reference's cuDNN/MIOpen BN.
// Semantics follow torch.nn.BatchNorm2d (training): biased variance for normalisation,
// unbiased variance in running_var, running = (1-momentum)*running + momentum*batch.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <string>

#include "ndp_kernels.h"
#include "pool_route.h"

namespace ndp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of two doubles (fixed order); result valid in every thread
__device__ __forceinline__ void block_sum2(double& a, double& b, double* red /*[2][8]*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if (lane == 0) {
    red[wave] = a;
    red[8 + wave] = b;
  }
  __syncthreads();
  a = 0.0;
  b = 0.0;
  for (int w = 0; w < nw; ++w) {
    a += red[w];
    b += red[8 + w];
  }
  __syncthreads();
}

struct BnSlice {
  int64_t n0, n1;
};

// Visit every access of one (channel, slice): W = floats per access (4 or 1).  When a row's
// HW/W accesses divide the 256 threads, each thread owns a fixed column q and strides
// over rows with 32-bit math (no per-element 64-bit division).
template <int W, typename F>
__device__ __forceinline__ void for_slice(int64_t n0, int64_t n1, int C, int c, int HW, F f) {
  const int per = HW / W;
  if (per <= 256 && (256 % per) == 0) {
    const int q = (int)threadIdx.x % per, r = (int)threadIdx.x / per, step = 256 / per;
    for (int64_t n = n0 + r; n < n1; n += step) f((n * C + c) * HW + W * q);
  } else {
    for (int64_t n = n0; n < n1; ++n)
      for (int q = threadIdx.x; q < per; q += 256) f((n * C + c) * HW + W * q);
  }
}

__device__ __forceinline__ BnSlice slice_of(int N, int S, int s) {
  const int64_t base = N / S, rem = N % S;
  const int64_t n0 = s * base + (s < rem ? s : rem);
  return {n0, n0 + base + (s < rem ? 1 : 0)};
}

// for_slice<4> with the thread's FIRST access loaded (ld) before pre() runs — the per-channel
// statistics reduction of an apply kernel — so its HBM latency overlaps that reduction instead
// of following it; then f(o, loaded) for every access in for_slice order.  At the ResNet apply
// shapes a thread's first access is usually its only one.
template <typename T, typename L, typename P, typename F>
__device__ __forceinline__ void for_slice4_pf(int64_t n0, int64_t n1, int C, int c, int HW, L ld, P pre, F f) {
  const int per = HW / 4;
  if (per <= 256 && (256 % per) == 0) {
    const int q = (int)threadIdx.x % per, r = (int)threadIdx.x / per, step = 256 / per;
    int64_t n = n0 + r;
    const bool has = n < n1;
    const int64_t o0 = (n * C + c) * HW + 4 * q;
    T first{};
    if (has) first = ld(o0);
    pre();
    if (has) f(o0, first);
    for (n += step; n < n1; n += step) {
      const int64_t o = (n * C + c) * HW + 4 * q;
      f(o, ld(o));
    }
  } else {
    pre();
    for_slice<4>(n0, n1, C, c, HW, [&](int64_t o) { f(o, ld(o)); });
  }
}

// sums of the S slice partials [c][s][2] of channel c: 8 loads in flight, adds in slice order
__device__ __forceinline__ void slice_sums(const double* __restrict__ part, int c, int S, double& a, double& b) {
  a = 0.0;
  b = 0.0;
  const double* p = part + (int64_t)c * S * 2;
  int k = 0;
  for (; k + 8 <= S; k += 8) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[2 * k + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a += v[2 * u];
      b += v[2 * u + 1];
    }
  }
  for (; k < S; ++k) {
    a += p[2 * k];
    b += p[2 * k + 1];
  }
}

// the same sums over many partials (the S = batch-tile partials a conv epilogue emits,
// conv_fwd_kernel `stats`): strided over the block, then the fixed-order block reduction;
// the result is identical in every workgroup of the channel
__device__ __forceinline__ void slice_sums_block(const double* __restrict__ part, int c, int S, double& a, double& b,
                                                 double* red) {
  a = 0.0;
  b = 0.0;
  const double* p = part + (int64_t)c * S * 2;
  for (int k = threadIdx.x; k < S; k += blockDim.x) {
    a += p[2 * k];
    b += p[2 * k + 1];
  }
  block_sum2(a, b, red);
}

// ---- forward statistics -------------------------------------------------------------
// src (nullable, VEC only): x is the sum of nslab split-K conv slabs (slab order, bitwise equal
// to conv_slab_sum); the kernel adds them, writes x and takes its statistics in one pass.
template <bool VEC>
__global__ __launch_bounds__(256) void bn_fwd_stats_kernel(const float* __restrict__ x, double* __restrict__ part,
                                                           int N, int C, int HW, int S,
                                                           const float* __restrict__ src = nullptr, int nslab = 0) {
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y;
  const BnSlice sl = slice_of(N, S, s);
  double sum = 0.0, sq = 0.0;
  if (VEC) {
    const int64_t slab = (int64_t)N * C * HW;
    for_slice<4>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      f32x4 v;
      if (src != nullptr) {
        v = *reinterpret_cast<const f32x4*>(src + o);
        for (int z = 1; z < nslab; ++z) v += *reinterpret_cast<const f32x4*>(src + z * slab + o);
        *reinterpret_cast<f32x4*>(const_cast<float*>(x) + o) = v;
      } else {
        v = *reinterpret_cast<const f32x4*>(x + o);
      }
      // fp32 pair sums first (exact enough), fp64 across the slice
      const float s4 = (v[0] + v[1]) + (v[2] + v[3]);
      const float q4 = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
      sum += (double)s4;
      sq += (double)q4;
    });
  } else {
    for_slice<1>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      const double v = (double)x[o];
      sum += v;
      sq += v * v;
    });
  }
  block_sum2(sum, sq, red);
  if (threadIdx.x == 0) {
    part[((int64_t)c * S + s) * 2] = sum;
    part[((int64_t)c * S + s) * 2 + 1] = sq;
  }
}

// ---- forward apply --------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256) void bn_fwd_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ res, float* __restrict__ y,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ rmean,
    float* __restrict__ rvar, int64_t* __restrict__ nbt, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, const double* __restrict__ part, int N, int C, int HW, int S,
    float eps, float momentum, int relu, int training, int Sp = 0) {
  // Sp > 0: `part` holds Sp partials per channel from the producing conv's epilogue (folded by
  // the whole block) instead of this launch's S slice partials
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y;
  // per-channel operands first: in flight with the slice partials, not a round trip after them
  const float gam = gamma ? gamma[c] : 1.f, bet = beta ? beta[c] : 0.f;
  const bool writer = training && s == 0 && threadIdx.x == 0 && rmean != nullptr;
  const float rm = writer ? rmean[c] : 0.f, rv = writer ? rvar[c] : 0.f;
  float scale = 0.f, shift = 0.f;
  auto coefficients = [&]() {
    float mean, invstd;
    if (training) {
      double sum, sq;
      if (Sp > 0) slice_sums_block(part, c, Sp, sum, sq, red);
      else slice_sums(part, c, S, sum, sq);
      const double M = (double)N * HW;
      const double mu = sum / M;
      double var = sq / M - mu * mu;
      if (var < 0.0) var = 0.0;
      mean = (float)mu;
      invstd = (float)(1.0 / sqrt(var + (double)eps));
      if (s == 0 && threadIdx.x == 0) {
        save_mean[c] = mean;
        save_invstd[c] = invstd;
        if (rmean != nullptr) {
          const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
          rmean[c] = (float)((1.0 - momentum) * (double)rm + momentum * mu);
          rvar[c] = (float)((1.0 - momentum) * (double)rv + momentum * unb);
        }
        if (nbt != nullptr && c == 0) nbt[0] += 1;
      }
    } else {
      mean = rmean[c];
      invstd = 1.0f / sqrtf(rvar[c] + eps);
    }
    scale = gam * invstd;
    shift = bet - mean * scale;
  };
  const BnSlice sl = slice_of(N, S, s);
  if (VEC) {
    struct XR { f32x4 v, r; };
    for_slice4_pf<XR>(
        sl.n0, sl.n1, C, c, HW,
        [&](int64_t o) {
          XR t;
          t.v = *reinterpret_cast<const f32x4*>(x + o);
          t.r = res ? *reinterpret_cast<const f32x4*>(res + o) : f32x4{0.f, 0.f, 0.f, 0.f};
          return t;
        },
        coefficients,
        [&](int64_t o, XR t) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float z = fmaf(t.v[j], scale, shift) + t.r[j];
            t.v[j] = relu ? fmaxf(z, 0.f) : z;
          }
          *reinterpret_cast<f32x4*>(y + o) = t.v;
        });
  } else {
    coefficients();
    for_slice<1>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      const float z = fmaf(x[o], scale, shift) + (res ? res[o] : 0.f);
      y[o] = relu ? fmaxf(z, 0.f) : z;
    });
  }
}

// ---- backward statistics ----------------------------------------------------------------
// src (nullable, VEC only): dy is the sum of nslab split-K grad-x slabs; written back to dy
// for the apply kernel.
template <bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                           const float* __restrict__ x,
                                                           const float* __restrict__ save_mean,
                                                           const float* __restrict__ save_invstd,
                                                           double* __restrict__ part, int N, int C, int HW,
                                                           int S, int relu, const float* __restrict__ src = nullptr,
                                                           int nslab = 0, const float* __restrict__ sadd = nullptr,
                                                           const float* __restrict__ mgam = nullptr,
                                                           const float* __restrict__ mbet = nullptr) {
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y;
  const BnSlice sl = slice_of(N, S, s);
  const float mean = save_mean[c], invstd = save_invstd[c];
  // mbet != nullptr: the forward output was never stored (bn_relu_maxpool): its ReLU mask is
  // recomputed from x with the forward's own float ops, fmaf(x, scale, shift) > 0
  const float msc = mbet ? __fmul_rn(mgam ? mgam[c] : 1.f, invstd) : 0.f;
  const float msh = mbet ? __fsub_rn(mbet[c], __fmul_rn(mean, msc)) : 0.f;
  double sdz = 0.0, sdzx = 0.0;
  if (VEC) {
    const int64_t slab = (int64_t)N * C * HW;
    for_slice<4>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      f32x4 g;
      if (src != nullptr) {
        g = *reinterpret_cast<const f32x4*>(src + o);
        for (int z = 1; z < nslab; ++z) g += *reinterpret_cast<const f32x4*>(src + z * slab + o);
        if (sadd != nullptr) g += *reinterpret_cast<const f32x4*>(sadd + o);  // deferred addend, last
        *reinterpret_cast<f32x4*>(const_cast<float*>(dy) + o) = g;
      } else {
        g = *reinterpret_cast<const f32x4*>(dy + o);
      }
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + o);
      f32x4 yv = {1.f, 1.f, 1.f, 1.f};
      if (mbet) {
#pragma unroll
        for (int j = 0; j < 4; ++j) yv[j] = fmaf(xv[j], msc, msh);
      } else if (relu) {
        yv = *reinterpret_cast<const f32x4*>(y + o);
      }
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float dz = (yv[j] > 0.f) ? g[j] : 0.f;
        a += dz;
        b += dz * ((xv[j] - mean) * invstd);
      }
      sdz += (double)a;
      sdzx += (double)b;
    });
  } else {
    for_slice<1>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      const float dz = (!relu || y[o] > 0.f) ? dy[o] : 0.f;
      sdz += (double)dz;
      sdzx += (double)dz * (double)((x[o] - mean) * invstd);
    });
  }
  block_sum2(sdz, sdzx, red);
  if (threadIdx.x == 0) {
    part[((int64_t)c * S + s) * 2] = sdz;
    part[((int64_t)c * S + s) * 2 + 1] = sdzx;
  }
}

// ---- backward apply ----------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ x,
    const float* __restrict__ gamma, const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    float* __restrict__ dx, float* __restrict__ dres, float* __restrict__ dgamma, float* __restrict__ dbeta,
    const double* __restrict__ part, int N, int C, int HW, int S, int relu, const float* __restrict__ mbet = nullptr,
    int Sp = 0) {
  // Sp > 0: `part` holds Sp partials per channel from the grad-x epilogue of the conv that
  // produced dy (conv_fwd_kernel backward-mode statistics), folded by the whole block
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y;
  // per-channel operands first: in flight with the slice partials
  const float mean = save_mean[c], invstd = save_invstd[c];
  const float g = gamma ? gamma[c] : 1.f;
  // mbet: ReLU mask recomputed from x (bn_bwd_stats_kernel)
  const float msc = mbet ? __fmul_rn(g, invstd) : 0.f;
  const float msh = mbet ? __fsub_rn(mbet[c], __fmul_rn(mean, msc)) : 0.f;
  float k1 = 0.f, mdz = 0.f, mdzx = 0.f;  // dx = k1 * (dz - mdz - xhat * mdzx)
  auto coefficients = [&]() {
    double sdz, sdzx;
    if (Sp > 0) slice_sums_block(part, c, Sp, sdz, sdzx, red);
    else slice_sums(part, c, S, sdz, sdzx);
    if (s == 0 && threadIdx.x == 0) {
      if (dgamma) dgamma[c] = (float)sdzx;
      if (dbeta) dbeta[c] = (float)sdz;
    }
    const double M = (double)N * HW;
    k1 = g * invstd;
    mdz = (float)(sdz / M);
    mdzx = (float)(sdzx / M);
  };
  const BnSlice sl = slice_of(N, S, s);
  if (VEC) {
    struct GXY { f32x4 gy, xv, yv; };
    for_slice4_pf<GXY>(
        sl.n0, sl.n1, C, c, HW,
        [&](int64_t o) {
          GXY t;
          t.gy = *reinterpret_cast<const f32x4*>(dy + o);
          t.xv = *reinterpret_cast<const f32x4*>(x + o);
          t.yv = (!mbet && relu) ? *reinterpret_cast<const f32x4*>(y + o) : f32x4{1.f, 1.f, 1.f, 1.f};
          return t;
        },
        coefficients,
        [&](int64_t o, GXY t) {
          if (mbet) {
#pragma unroll
            for (int j = 0; j < 4; ++j) t.yv[j] = fmaf(t.xv[j], msc, msh);
          }
          f32x4 dz, out;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            dz[j] = (t.yv[j] > 0.f) ? t.gy[j] : 0.f;
            const float xh = (t.xv[j] - mean) * invstd;
            out[j] = k1 * (dz[j] - mdz - xh * mdzx);
          }
          *reinterpret_cast<f32x4*>(dx + o) = out;
          if (dres) *reinterpret_cast<f32x4*>(dres + o) = dz;
        });
  } else {
    coefficients();
    for_slice<1>(sl.n0, sl.n1, C, c, HW, [&](int64_t o) {
      const float dz = (!relu || y[o] > 0.f) ? dy[o] : 0.f;
      const float xh = (x[o] - mean) * invstd;
      dx[o] = k1 * (dz - mdz - xh * mdzx);
      if (dres) dres[o] = dz;
    });
  }
}

// ---- stem tail backward: max-pool routing + ReLU mask + BN backward apply in one pass ---------
// The pool backward (pool.hip, statistics only) has folded sum dz / sum dz * xhat per (channel,
// image) with dz = routed gradient * ReLU mask; this pass re-routes the pooled gradient (the 8x8
// dY and its uint8 argmax: 1/4 of the 16x16 plane's bytes, plus x) and writes the BN input
// gradient directly — the routed 16x16 gradient is never stored and never re-read (2 x 33 MB at
// batch 512).  Per element the same operations in the same order as maxpool_bwd_s2_kernel +
// bn_bwd_apply_kernel (mbet mask, Sp = N statistics): bitwise equal.  Grid (S, C); 64 threads
// per 8x8 pooled plane, 4 planes per pass.
__global__ __launch_bounds__(256) void stem_pool_bwd_apply_kernel(
    const float* __restrict__ dy, const uint8_t* __restrict__ idx, const float* __restrict__ x,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ save_mean,
    const float* __restrict__ save_invstd, const double* __restrict__ stats, float* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int N, int C, int H, int W) {
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y, S = gridDim.x;
  const float mean = save_mean[c], invstd = save_invstd[c];
  const float g = gamma ? gamma[c] : 1.f;
  const float msc = __fmul_rn(g, invstd);
  const float msh = __fsub_rn(beta ? beta[c] : 0.f, __fmul_rn(mean, msc));
  double sdz, sdzx;
  slice_sums_block(stats, c, N, sdz, sdzx, red);
  if (s == 0 && threadIdx.x == 0) {
    if (dgamma) dgamma[c] = (float)sdzx;
    if (dbeta) dbeta[c] = (float)sdz;
  }
  const double M = (double)N * H * W;
  const float k1 = g * invstd;
  const float mdz = (float)(sdz / M);
  const float mdzx = (float)(sdzx / M);
  const int OH = H / 2, OW = W / 2;  // 64 outputs per plane (launcher-checked)
  const BnSlice sl = slice_of(N, S, s);
  const int o = threadIdx.x & 63, i = o / OW, j = o - i * OW;
  for (int64_t n = sl.n0 + (threadIdx.x >> 6); n < sl.n1; n += 4) {
    const int64_t plane = n * C + c;
    float d[4];
    pool_s2_route_wave(dy[plane * 64 + o], idx[plane * 64 + o], i, j, d[0], d[1], d[2], d[3]);
    const int64_t off = plane * H * W + (int64_t)(2 * i) * W + 2 * j;
    const float2 x0 = *reinterpret_cast<const float2*>(x + off), x1 = *reinterpret_cast<const float2*>(x + off + W);
    const float xs[4] = {x0.x, x0.y, x1.x, x1.y};
    float out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float dz = (fmaf(xs[k], msc, msh) > 0.f) ? d[k] : 0.f;
      const float xh = (xs[k] - mean) * invstd;
      out[k] = k1 * (dz - mdz - xh * mdzx);
    }
    *reinterpret_cast<float2*>(dx + off) = make_float2(out[0], out[1]);
    *reinterpret_cast<float2*>(dx + off + W) = make_float2(out[2], out[3]);
  }
}

void launch_stem_pool_bwd_apply(const float* dy, const uint8_t* idx, const float* x, const float* gamma,
                                const float* beta, const float* save_mean, const float* save_invstd,
                                const double* stats, float* dx, float* dgamma, float* dbeta, int N, int C, int H,
                                int W, hipStream_t s) {
  // slices: 4 images per workgroup at small batches, at most 16 slices (each workgroup folds the
  // channel's N statistics partials)
  const int S = N / 4 < 1 ? 1 : (N / 4 > 16 ? 16 : N / 4);
  hipLaunchKernelGGL(stem_pool_bwd_apply_kernel, dim3((unsigned)S, (unsigned)C), dim3(256), 0, s, dy, idx, x, gamma,
                     beta, save_mean, save_invstd, stats, dx, dgamma, dbeta, N, C, H, W);
}

// ---- stem tail: BN (training) -> ReLU -> MaxPool(3, 2, 1) in one pass ----------------------
// ResNet's stem writes the BN output (the largest activation of the network, 16x16 maps)
// only for the max-pool to read it back.  Here the apply folds the statistics (the conv
// epilogue's partials, Sp > 0, or this BN's statistics pass) and every thread computes
// pooled outputs straight from x: relu(fmaf(x, scale, shift)) per window tap, the winning
// tap stored as the pool's uint8 window offset (the same first-maximum scan as
// pool.hip).  The BN output is never stored: the backward recomputes its ReLU mask from x
// (bn_bwd_*_kernel `mbet`).  Grid (S, C) like bn_fwd_apply: a slice owns whole planes.
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(
    const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ idx, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, const double* __restrict__ part, int N, int C,
    int H, int W, int S, float eps, float momentum, int Sp) {
  __shared__ double red[16];
  const int s = blockIdx.x, c = blockIdx.y;
  const float gam = gamma ? gamma[c] : 1.f, bet = beta ? beta[c] : 0.f;
  const bool writer = s == 0 && threadIdx.x == 0 && rmean != nullptr;
  const float rm = writer ? rmean[c] : 0.f, rv = writer ? rvar[c] : 0.f;
  const int HW = H * W;
  double sum, sq;
  if (Sp > 0) slice_sums_block(part, c, Sp, sum, sq, red);
  else slice_sums(part, c, S, sum, sq);
  const double M = (double)N * HW;
  const double mu = sum / M;
  double var = sq / M - mu * mu;
  if (var < 0.0) var = 0.0;
  const float mean = (float)mu;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  if (s == 0 && threadIdx.x == 0) {
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    if (rmean != nullptr) {
      const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
      rmean[c] = (float)((1.0 - momentum) * (double)rm + momentum * mu);
      rvar[c] = (float)((1.0 - momentum) * (double)rv + momentum * unb);
    }
    if (nbt != nullptr && c == 0) nbt[0] += 1;
  }
  // unfused roundings (no contraction): the backward recomputes these exact values for its mask
  const float scale = __fmul_rn(gam, invstd);
  const float shift = __fsub_rn(bet, __fmul_rn(mean, scale));
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, PQ = OH * OW;
  const BnSlice sl = slice_of(N, S, s);
  if ((W & 3) == 0 && 64 % (W >> 2) == 0 && (H & 1) == 0 && (W & 1) == 0) {
    // pool.hip's vectorised pair scheme: one thread per output pair (oh, 2j), (oh, 2j + 1), the
    // three input rows' columns 4j .. 4j+3 as one float4 each (normalised + ReLU in registers),
    // column 4j - 1 from the left lane (the W/4 lanes of a row are adjacent in the wave)
    const int W4 = W >> 2, pairs = OH * W4;
    const int total = (int)(sl.n1 - sl.n0) * pairs;
    // two items per thread per trip: both items' three input rows are loaded before either is
    // normalised / pooled / stored (one HBM round trip per two items)
    constexpr int U = 2;
    for (int base = 0; base < total; base += 256 * U) {  // uniform trip count: every lane shuffles
      f32x4 q[U][3];
      int tt[U], jj[U], oo[U];
      int64_t pl[U];
      bool lv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int t = base + 256 * k + (int)threadIdx.x;
        lv[k] = t < total;
        const int ni = lv[k] ? t / pairs : 0, r = lv[k] ? t - ni * pairs : 0;
        oo[k] = r / W4;
        jj[k] = r - oo[k] * W4;
        tt[k] = t;
        pl[k] = (sl.n0 + ni) * C + c;
        const float* xp = x + pl[k] * HW;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int hh = 2 * oo[k] - 1 + kh;
          q[k][kh] = (lv[k] && hh >= 0 && hh < H) ? *reinterpret_cast<const f32x4*>(xp + hh * W + 4 * jj[k])
                                                   : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int oh = oo[k], j = jj[k];
        float v[3][5];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int hh = 2 * oh - 1 + kh;
          f32x4 qq = q[k][kh];
          if (lv[k] && hh >= 0 && hh < H) {
#pragma unroll
            for (int u = 0; u < 4; ++u) qq[u] = fmaxf(fmaf(qq[u], scale, shift) + 0.f, 0.f);
          }
          const float left = __shfl_up(qq[3], 1, 64);
          v[kh][0] = (j > 0) ? left : -INFINITY;
          v[kh][1] = qq[0]; v[kh][2] = qq[1]; v[kh][3] = qq[2]; v[kh][4] = qq[3];
        }
        if (!lv[k]) continue;
        float out[2];
        uint8_t arg[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {  // output column ow = 2j + u: taps at columns 4j - 1 + 2u + kw
          const int ow = 2 * j + u;
          const int kh0 = oh == 0 ? 1 : 0, kw0 = ow == 0 ? 1 : 0;
          float best = -INFINITY;
          int a0 = kh0 * 3 + kw0;
#pragma unroll
          for (int kh = 0; kh < 3; ++kh) {
            if (kh < kh0 || 2 * oh - 1 + kh >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              if (kw < kw0 || 2 * ow - 1 + kw >= W) continue;
              const float val = v[kh][2 * u + kw];
              if (val > best || isnan(val)) {
                best = val;
                a0 = kh * 3 + kw;
              }
            }
          }
          out[u] = best;
          arg[u] = (uint8_t)a0;
        }
        const int64_t o = pl[k] * PQ + oh * OW + 2 * j;
        *reinterpret_cast<float2*>(y + o) = make_float2(out[0], out[1]);
        *reinterpret_cast<uint16_t*>(idx + o) = (uint16_t)(arg[0] | (arg[1] << 8));  // o even: 2-B aligned
      }
      (void)tt;
    }
    return;
  }
  const int total = (int)(sl.n1 - sl.n0) * PQ;
  for (int t = threadIdx.x; t < total; t += 256) {
    const int ni = t / PQ, o = t - ni * PQ;
    const int oh = o / OW, ow = o - oh * OW;
    const int64_t plane = (sl.n0 + ni) * C + c;
    const float* xp = x + plane * HW;
    const int h0 = 2 * oh - 1, w0 = 2 * ow - 1;
    const int kh0 = h0 < 0 ? 1 : 0, kw0 = w0 < 0 ? 1 : 0;
    float best = -INFINITY;
    int arg = kh0 * 3 + kw0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hh = h0 + kh;
      if (kh < kh0 || hh >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = w0 + kw;
        if (kw < kw0 || ww >= W) continue;
        const float v = fmaxf(fmaf(xp[hh * W + ww], scale, shift) + 0.f, 0.f);
        if (v > best || isnan(v)) {
          best = v;
          arg = kh * 3 + kw;
        }
      }
    }
    y[plane * PQ + o] = best;
    idx[plane * PQ + o] = (uint8_t)arg;
  }
}

// ---- small feature maps (HW <= 16: ResNet layer3/layer4 on 32x32 inputs) -----------------
// In NCHW a channel's pixels are HW contiguous floats, so the per-(channel, slice) kernels
// above read 4-64 B per cache line there.  These kernels treat x as [N][C*HW] instead: a
// thread owns one column j = c*HW + hw and walks its slice of n (every load instruction is
// 256 consecutive floats), the HW lanes of a channel are combined with shuffles, and a tiny
// per-channel finalize kernel folds the slice partials in a fixed order (deterministic).
// part layout: [c][s][2] partial sums, then 3*C doubles of per-channel coefficients.
constexpr int kSmallNPer = 4;  // images per stats slice: 4 independent loads in flight per thread
int bn_small_slices(int N, int C, int HW) { return (N + kSmallNPer - 1) / kSmallNPer; }

template <int HW>
__global__ __launch_bounds__(256) void bn_small_stats_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ save_mean,
                                                             const float* __restrict__ save_invstd,
                                                             double* __restrict__ part, int N, int C, int S, int bwd,
                                                             int relu) {
  const int CHW = C * HW;
  const int j = blockIdx.y * 256 + threadIdx.x;
  const int s = blockIdx.x;
  const int n0 = s * kSmallNPer;
  double a = 0.0, b = 0.0;
  if (j < CHW) {
    float v[kSmallNPer], d[kSmallNPer], m[kSmallNPer];
#pragma unroll
    for (int k = 0; k < kSmallNPer; ++k) {  // issue every load first
      const bool ok = n0 + k < N;
      const int64_t o = (int64_t)(n0 + k) * CHW + j;
      v[k] = ok ? x[o] : 0.f;
      d[k] = (bwd && ok) ? dy[o] : 0.f;
      m[k] = (bwd && relu && ok) ? y[o] : 1.f;
    }
    if (!bwd) {
#pragma unroll
      for (int k = 0; k < kSmallNPer; ++k) {
        a += (double)v[k];
        b += (double)v[k] * (double)v[k];
      }
    } else {
      const int c = j / HW;
      const float mean = save_mean[c], invstd = save_invstd[c];
#pragma unroll
      for (int k = 0; k < kSmallNPer; ++k) {
        if (n0 + k < N) {
          const float dz = (m[k] > 0.f) ? d[k] : 0.f;
          a += (double)dz;
          b += (double)dz * (double)((v[k] - mean) * invstd);
        }
      }
    }
  }
#pragma unroll
  for (int o = HW / 2; o > 0; o >>= 1) {  // the HW lanes of one channel are adjacent
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (j < CHW && (j % HW) == 0) {
    const int c = j / HW;
    part[((int64_t)c * S + s) * 2] = a;
    part[((int64_t)c * S + s) * 2 + 1] = b;
  }
}

// one wave per channel: lane l adds slices l, l+64, ... then a fixed xor butterfly
// forward: coef[c] = scale, coef[C + c] = shift (+ save_mean / invstd / running stats / nbt)
// backward: coef = (k1, mdz, mdzx) and dgamma / dbeta
__global__ __launch_bounds__(256) void bn_small_finalize_kernel(
    const double* __restrict__ part, double* __restrict__ coef, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int N, int C, int HW, int S, float eps, float momentum, int bwd) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;  // whole waves exit together
  double a = 0.0, b = 0.0;
  for (int k = lane; k < S; k += 64) {
    a += part[((int64_t)c * S + k) * 2];
    b += part[((int64_t)c * S + k) * 2 + 1];
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  if (lane != 0) return;
  const double M = (double)N * HW;
  if (!bwd) {
    const double mu = a / M;
    double var = b / M - mu * mu;
    if (var < 0.0) var = 0.0;
    const float mean = (float)mu, invstd = (float)(1.0 / sqrt(var + (double)eps));
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    if (rmean != nullptr) {
      const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
      rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mu);
      rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
    }
    if (nbt != nullptr && c == 0) nbt[0] += 1;
    const float scale = (gamma ? gamma[c] : 1.f) * invstd;
    coef[c] = scale;
    coef[C + c] = (beta ? beta[c] : 0.f) - mean * scale;
  } else {
    if (dgamma) dgamma[c] = (float)b;
    if (dbeta) dbeta[c] = (float)a;
    coef[c] = (gamma ? gamma[c] : 1.f) * save_invstd[c];  // k1
    coef[C + c] = (float)(a / M);                         // mean dz
    coef[2 * C + c] = (float)(b / M);                     // mean dz * xhat
  }
}

// elementwise over the whole tensor, 4 consecutive elements (one float4) per thread
__global__ __launch_bounds__(256) void bn_small_apply_kernel(
    const float* __restrict__ x, const float* __restrict__ res, const float* __restrict__ dy,
    const float* __restrict__ yin, const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    const double* __restrict__ coef, float* __restrict__ out, float* __restrict__ dres, int total, int C, int HW,
    int relu, int bwd) {
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= total) return;
  const bool full = i0 + 3 < total;  // total % 4 == 0 in practice: one float4 per thread
  f32x4 xv, r = {0.f, 0.f, 0.f, 0.f}, g = {0.f, 0.f, 0.f, 0.f}, yv = {1.f, 1.f, 1.f, 1.f}, o, dz;
  if (full) {
    xv = *reinterpret_cast<const f32x4*>(x + i0);
    if (!bwd && res) r = *reinterpret_cast<const f32x4*>(res + i0);
    if (bwd) g = *reinterpret_cast<const f32x4*>(dy + i0);
    if (bwd && relu) yv = *reinterpret_cast<const f32x4*>(yin + i0);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = i0 + k < total;
      xv[k] = ok ? x[i0 + k] : 0.f;
      if (!bwd && res) r[k] = ok ? res[i0 + k] : 0.f;
      if (bwd) g[k] = ok ? dy[i0 + k] : 0.f;
      if (bwd && relu) yv[k] = ok ? yin[i0 + k] : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = ((i0 + k) / HW) % C;
    if (!bwd) {
      const float z = fmaf(xv[k], (float)coef[c], (float)coef[C + c]) + r[k];
      o[k] = relu ? fmaxf(z, 0.f) : z;
    } else {
      dz[k] = (yv[k] > 0.f) ? g[k] : 0.f;
      const float xh = (xv[k] - save_mean[c]) * save_invstd[c];
      o[k] = (float)coef[c] * (dz[k] - (float)coef[C + c] - xh * (float)coef[2 * C + c]);
    }
  }
  if (full) {
    *reinterpret_cast<f32x4*>(out + i0) = o;
    if (bwd && dres) *reinterpret_cast<f32x4*>(dres + i0) = dz;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < total) {
        out[i0 + k] = o[k];
        if (bwd && dres) dres[i0 + k] = dz[k];
      }
    }
  }
}

// ---- single-launch small-map BN (column block x every image, register resident) ---------
// The three small-map kernels above are each only a few µs of work on 1-2 MB tensors, so
// a ResNet-18 step spends most of their ~300 µs in launch gaps.  This kernel does a whole
// BN direction in ONE launch with no cross-workgroup traffic: a workgroup owns CW
// consecutive columns of the [N][C*HW] view (whole channels, since HW | CW) for EVERY
// image.  Its 512 threads are CW columns x RG = 512 / CW row groups; thread (g, col) keeps
// rows g, g + RG, ... (<= 512 / RG of them) in registers, so the tensor is read once and
// written once.  Per-channel sums (deterministic, every thread ends with the bitwise-same
// value): fp64 per thread -> xor butterfly over the HW lanes of a channel and the row
// groups inside the wave (commutative pairings: identical on every lane) -> fixed-order
// fold of the 8 per-wave partials through LDS.  CW trades grid size (C*HW / CW workgroups;
// 256 CUs to fill) against row-segment width per load (CW * 4 bytes): bn_colw_for picks
// it by measurement.  Used when N <= 512 (ResNet's per-GPU batch).
// NDP_FUSION_OFF=bn_vec4 (knobs.py): the scalar single-launch kernel, for A/B arms; tests flip
// it through bn_set_vec4
static int g_bn_vec4 = -1;
static bool vec_off() {
  if (g_bn_vec4 < 0) {
    const char* e = getenv("NDP_FUSION_OFF");
    const std::string s = std::string(",") + (e ? e : "") + ",";
    g_bn_vec4 = (s.find(",bn_vec4,") != std::string::npos || s.find(",all,") != std::string::npos) ? 0 : 1;
  }
  return g_bn_vec4 == 0;
}
void bn_set_vec4(bool on) { g_bn_vec4 = on ? 1 : 0; }

constexpr int kFusedThreads = 512;
constexpr int kFusedMaxN = 512;

//
// src (nullable): the kernel's main input — x in forward, dy in backward — is the sum of
// `nslab` split-K slabs (slab stride = numel) of the producing convolution (a deferred
// conv_slab_sum, ops/slablink.py), added in slab order exactly like conv_slab_sum_kernel
// (bitwise-equal values); the forward also stores the sum to x (BN's saved input).
// MAXN: largest batch the register arrays hold (512 for HW <= 16; 128 for the 8x8 maps of
// layer1 at the strong-scaling per-GPU batches 64 / 128, CW = HW = 64).
// Workgroups are dealt to the 8 XCDs round-robin (XCD = blockIdx % 8), each XCD with its own L2.
// Column blocks narrower than a 128-B line (CW = 4 / 8 floats) share lines with their neighbours:
// remap so that consecutive column blocks run on the same XCD (one L2 fetches the line once).
__device__ __forceinline__ int xcd_block(int bid, int nblk) {
  const int xcd = bid & 7, idx = bid >> 3, per = nblk >> 3, rem = nblk & 7;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

// PAIR = 1: the downsample block's two BatchNorms in one launch (BnPair: the second BN, over x2 =
// the 1x1 downsample conv's output, same shape).  Forward: out = relu(bn(x) + bn2(x2)), the
// downsample branch's BN output is never stored.  Backward: both BNs see the same
// dz = dy * (out > 0), so one pass forms sum dz, sum dz * xhat, sum dz * xhat2 and writes both
// input gradients (out, p2.out2).  One launch and one tensor round trip fewer per direction and
// downsample block than two single launches.
struct BnPair {
  const float* x2;
  const float* gamma2;
  const float* beta2;
  float* rmean2;
  float* rvar2;
  int64_t* nbt2;
  float* save_mean2;
  float* save_invstd2;
  float* dgamma2;
  float* dbeta2;
  float* out2;
  const float* src2;  // forward: x2 as nslab2 unsummed split-K slabs (summed here, stored to x2), or null
  int nslab2;
};

template <int HW, int BWD, int CW, int MAXN = kFusedMaxN, int PAIR = 0>
__global__ __launch_bounds__(kFusedThreads) void bn_small_fused_kernel(
    const float* __restrict__ x, const float* __restrict__ res, const float* __restrict__ dy,
    const float* __restrict__ yin, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ out,
    float* __restrict__ dres, int N, int C, float eps, float momentum, int relu, const float* __restrict__ src,
    int nslab, BnPair p2) {
  constexpr int RG = kFusedThreads / CW;
  constexpr int NP = MAXN / RG;  // rows per thread
  constexpr int NW = kFusedThreads / 64;
  static_assert(CW % HW == 0 && 64 % CW == 0, "bad column block");
  static_assert(NP >= 1, "bad row count");
  __shared__ double red[PAIR ? 4 : 2][NW][CW];
  const int CHW = C * HW;
  const int col = threadIdx.x % CW, g = threadIdx.x / CW;
  const int cb = xcd_block((int)blockIdx.x, (int)gridDim.x);
  const int j = cb * CW + col;
  const bool ok_col = j < CHW;
  const int c = ok_col ? j / HW : 0;
  float v[NP], d[NP], m[NP], v2[PAIR ? NP : 1];
  // every per-channel operand is loaded up front, alongside the tensor stream: read after the
  // reduction they were a second dependent memory round trip (~2 µs of a ~6 µs launch)
  float mean_s = 0.f, invstd_s = 0.f, gam = 1.f, bet = 0.f, rm = 0.f, rv = 0.f;
  float mean2 = 0.f, invstd2 = 0.f, gam2 = 1.f, bet2 = 0.f, rm2 = 0.f, rv2 = 0.f;
  if (ok_col) {
    if (BWD) {
      mean_s = save_mean[c];
      invstd_s = save_invstd[c];
    }
    if (gamma) gam = gamma[c];
    if (!BWD && beta) bet = beta[c];
    if (!BWD && rmean != nullptr && g == 0 && (j % HW) == 0) {
      rm = rmean[c];
      rv = rvar[c];
    }
    if constexpr (PAIR) {
      if (BWD) {
        mean2 = p2.save_mean2[c];
        invstd2 = p2.save_invstd2[c];
      }
      if (p2.gamma2) gam2 = p2.gamma2[c];
      if (!BWD && p2.beta2) bet2 = p2.beta2[c];
      if (!BWD && p2.rmean2 != nullptr && g == 0 && (j % HW) == 0) {
        rm2 = p2.rmean2[c];
        rv2 = p2.rvar2[c];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {  // every load in flight before any use
    const int n = g + k * RG;
    const bool ok = ok_col && n < N;
    const int64_t o = (int64_t)n * CHW + j;
    float sum = 0.f;
    if (src != nullptr && ok) {  // deferred split-K sum, slab order
      const int64_t slab = (int64_t)N * CHW;
      sum = src[o];
      for (int z = 1; z < nslab; ++z) sum += src[z * slab + o];
      if (BWD && res != nullptr) sum += res[o];  // backward: `res` carries the deferred grad-x addend
    }
    if (!BWD) {
      v[k] = ok ? (src ? sum : x[o]) : 0.f;
      if constexpr (PAIR) {  // the downsample conv output (or its split-K slabs, slab order)
        float t = 0.f;
        if (ok && p2.src2 != nullptr) {
          t = p2.src2[o];
          for (int z = 1; z < p2.nslab2; ++z) t += p2.src2[z * (int64_t)N * CHW + o];
        } else if (ok) {
          t = p2.x2[o];
        }
        d[k] = t;
      } else {
        d[k] = (ok && res) ? res[o] : 0.f;
      }
    } else {
      v[k] = ok ? x[o] : 0.f;
      d[k] = ok ? (src ? sum : dy[o]) : 0.f;
      m[k] = (ok && relu) ? yin[o] : 1.f;
      if constexpr (PAIR) v2[k] = ok ? p2.x2[o] : 0.f;
    }
  }
  if (!BWD && src != nullptr) {  // BN's saved input = the conv output
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = g + k * RG;
      if (ok_col && n < N) const_cast<float*>(x)[(int64_t)n * CHW + j] = v[k];
    }
  }
  if constexpr (PAIR) {
    if (!BWD && p2.src2 != nullptr) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int n = g + k * RG;
        if (ok_col && n < N) const_cast<float*>(p2.x2)[(int64_t)n * CHW + j] = d[k];
      }
    }
  }
  double a = 0.0, b = 0.0, a2 = 0.0, b2 = 0.0;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    if (ok_col && g + k * RG < N) {
      if (!BWD) {
        a += (double)v[k];
        b += (double)v[k] * (double)v[k];
        if constexpr (PAIR) {
          a2 += (double)d[k];
          b2 += (double)d[k] * (double)d[k];
        }
      } else {
        const float dz = (m[k] > 0.f) ? d[k] : 0.f;
        a += (double)dz;
        b += (double)dz * (double)((v[k] - mean_s) * invstd_s);
        if constexpr (PAIR) b2 += (double)dz * (double)((v2[k] - mean2) * invstd2);
      }
    }
  }
#pragma unroll
  for (int o = HW / 2; o > 0; o >>= 1) {  // the HW columns of a channel are adjacent lanes
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    if constexpr (PAIR) {
      a2 += __shfl_xor(a2, o, 64);
      b2 += __shfl_xor(b2, o, 64);
    }
  }
#pragma unroll
  for (int o = CW; o < 64; o <<= 1) {  // row groups inside the wave
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    if constexpr (PAIR) {
      a2 += __shfl_xor(a2, o, 64);
      b2 += __shfl_xor(b2, o, 64);
    }
  }
  const int wave = threadIdx.x / 64;
  if ((threadIdx.x % 64) < CW) {
    red[0][wave][col] = a;
    red[1][wave][col] = b;
    if constexpr (PAIR) {
      red[PAIR ? 2 : 0][wave][col] = a2;
      red[PAIR ? 3 : 0][wave][col] = b2;
    }
  }
  __syncthreads();
  double A = 0.0, B = 0.0, A2 = 0.0, B2 = 0.0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    A += red[0][k][col];
    B += red[1][k][col];
    if constexpr (PAIR) {
      A2 += red[PAIR ? 2 : 0][k][col];
      B2 += red[PAIR ? 3 : 0][k][col];
    }
  }
  if (!ok_col) return;
  const double M = (double)N * HW;
  const bool writer = g == 0 && (j % HW) == 0;
  if (!BWD) {
    const double mu = A / M;
    double var = B / M - mu * mu;
    if (var < 0.0) var = 0.0;
    const float mean = (float)mu, invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float scale = gam * invstd;
    const float shift = bet - mean * scale;
    float scale2 = 0.f, shift2 = 0.f;
    if constexpr (PAIR) {
      const double mu2 = A2 / M;
      double var2 = B2 / M - mu2 * mu2;
      if (var2 < 0.0) var2 = 0.0;
      const float mean2f = (float)mu2, invstd2f = (float)(1.0 / sqrt(var2 + (double)eps));
      scale2 = gam2 * invstd2f;
      shift2 = bet2 - mean2f * scale2;
      if (writer) {
        p2.save_mean2[c] = mean2f;
        p2.save_invstd2[c] = invstd2f;
        if (p2.rmean2 != nullptr) {
          const double unb2 = M > 1.0 ? var2 * M / (M - 1.0) : var2;
          p2.rmean2[c] = (float)((1.0 - momentum) * (double)rm2 + momentum * mu2);
          p2.rvar2[c] = (float)((1.0 - momentum) * (double)rv2 + momentum * unb2);
        }
        if (p2.nbt2 != nullptr && c == 0) p2.nbt2[0] += 1;
      }
    }
    if (writer) {
      save_mean[c] = mean;
      save_invstd[c] = invstd;
      if (rmean != nullptr) {
        const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
        rmean[c] = (float)((1.0 - momentum) * (double)rm + momentum * mu);
        rvar[c] = (float)((1.0 - momentum) * (double)rv + momentum * unb);
      }
      if (nbt != nullptr && c == 0) nbt[0] += 1;
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = g + k * RG;
      if (n < N) {
        const float z = PAIR ? fmaf(v[k], scale, shift) + fmaf(d[k], scale2, shift2) : fmaf(v[k], scale, shift) + d[k];
        out[(int64_t)n * CHW + j] = relu ? fmaxf(z, 0.f) : z;
      }
    }
  } else {
    if (writer) {
      if (dgamma) dgamma[c] = (float)B;
      if (dbeta) dbeta[c] = (float)A;
      if constexpr (PAIR) {
        if (p2.dgamma2) p2.dgamma2[c] = (float)B2;
        if (p2.dbeta2) p2.dbeta2[c] = (float)A;
      }
    }
    const float k1 = gam * invstd_s;
    const float mdz = (float)(A / M), mdzx = (float)(B / M);
    const float k12 = gam2 * invstd2, mdzx2 = (float)(B2 / M);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = g + k * RG;
      if (n < N) {
        const float dz = (m[k] > 0.f) ? d[k] : 0.f;
        const float xh = (v[k] - mean_s) * invstd_s;
        const int64_t o = (int64_t)n * CHW + j;
        out[o] = k1 * (dz - mdz - xh * mdzx);
        if constexpr (PAIR) {
          const float xh2 = (v2[k] - mean2) * invstd2;
          p2.out2[o] = k12 * (dz - mdz - xh2 * mdzx2);
        } else if (dres) {
          dres[o] = dz;
        }
      }
    }
  }
}

// The same single-launch BN with one float4 (4 consecutive columns) per thread instead of one
// float.  The scalar kernel's loads are 64-lane dword accesses: at batch 512 its 128 workgroups
// were bound by the texture-address rate of half the CUs (16 B/clk/CU, ~2 TB/s effective: the
// layer2 backward took 16.5 µs for 21 MB, profiles/r4/kernels_b512_head.md).  dwordx4 moves 4x
// the bytes per address cycle.  A float4 holds whole channels' pixel runs: one channel (HW >= 4,
// its HW/4 float4s on adjacent lanes) or 4 / HW channels (HW = 1, 2: separate sums per
// channel).  Same fp64 sums, same fixed-order fold: deterministic run to run.
// SPLIT > 1 (the 8x8 maps at per-GPU batch <= 128, one channel per column block): the rows of a
// column block are split over SPLIT workgroups that exchange their fp64 partial sums through the
// sc1 form of cdna_hip_programming.md §6 Guideline 16 (write-through partial stores + vmcnt drain +
// a relaxed monotonic arrival counter; every workgroup polls it relaxed, bounded, then reads the
// SPLIT partials with sc1 loads in split order: the same totals, bitwise, in all of them).  One
// workgroup per channel left 3/4 of the CUs idle and every thread held 4 rows.
struct BnSplitCtx {
  double* part;                 // [column block][SPLIT][4] partial sums
  unsigned long long* ctr;      // [column block] arrival counters (monotonic, zeroed once)
  unsigned max_spins;
};

template <int HW, int BWD, int CW, int MAXN = kFusedMaxN, int PAIR = 0, int SPLIT = 1>
__global__ __launch_bounds__(kFusedThreads) void bn_small_fused_v4_kernel(
    const float* __restrict__ x, const float* __restrict__ res, const float* __restrict__ dy,
    const float* __restrict__ yin, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ out,
    float* __restrict__ dres, int N, int C, float eps, float momentum, int relu, const float* __restrict__ src,
    int nslab, BnPair p2, BnSplitCtx sx = BnSplitCtx{}) {
  static_assert(SPLIT == 1 || (PAIR == 0 && HW >= 4 && CW == HW), "row splits: one channel per column block");
  constexpr int CT = CW / 4;                   // threads per row
  constexpr int RG = kFusedThreads / CT;       // row groups
  constexpr int NP = (MAXN / SPLIT + RG - 1) / RG;  // rows per thread
  constexpr int NW = kFusedThreads / 64;
  constexpr int NCH = HW >= 4 ? 1 : 4 / HW;    // channels per float4
  constexpr int CPC = HW >= 4 ? 4 : HW;        // components per channel inside a float4
  constexpr int LPC = HW >= 4 ? HW / 4 : 1;    // lanes per channel
  constexpr int CPW = CW / HW;                 // channels per workgroup
  static_assert(CW % 4 == 0 && CW % HW == 0 && CT <= 64 && 64 % CT == 0, "bad column block");
  __shared__ double red[PAIR ? 4 : 2][NW][CPW];
  const int CHW = C * HW;
  const int ct = threadIdx.x % CT, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the split's rows: row(k) = row0 + g + k RG for g + k RG < rps (SPLIT = 1: all N rows)
  const int split = SPLIT > 1 ? (int)blockIdx.x % SPLIT : 0;
  const int cb = SPLIT > 1 ? (int)blockIdx.x / SPLIT : xcd_block((int)blockIdx.x, (int)gridDim.x);
  const int rps = SPLIT > 1 ? (N + SPLIT - 1) / SPLIT : N;
  const int row0 = split * rps;
  const int g = threadIdx.x / CT;
  const int j0 = cb * CW + 4 * ct;
  const bool ok_col = j0 < CHW;
  const int c0 = ok_col ? j0 / HW : 0;  // first channel of this float4
  auto row_ok = [&](int k) { return g + k * RG < rps && row0 + g + k * RG < N; };
  float mean_s[NCH], invstd_s[NCH], gam[NCH], bet[NCH], rm[NCH], rv[NCH];
  float mean2[NCH], invstd2[NCH], gam2[NCH], bet2[NCH], rm2[NCH], rv2[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = c0 + i;
    mean_s[i] = 0.f; invstd_s[i] = 0.f; gam[i] = 1.f; bet[i] = 0.f; rm[i] = 0.f; rv[i] = 0.f;
    mean2[i] = 0.f; invstd2[i] = 0.f; gam2[i] = 1.f; bet2[i] = 0.f; rm2[i] = 0.f; rv2[i] = 0.f;
    if (ok_col) {
      if (BWD) {
        mean_s[i] = save_mean[c];
        invstd_s[i] = save_invstd[c];
      }
      if (gamma) gam[i] = gamma[c];
      if (!BWD && beta) bet[i] = beta[c];
      if (!BWD && rmean != nullptr && g == 0) {
        rm[i] = rmean[c];
        rv[i] = rvar[c];
      }
      if constexpr (PAIR) {
        if (BWD) {
          mean2[i] = p2.save_mean2[c];
          invstd2[i] = p2.save_invstd2[c];
        }
        if (p2.gamma2) gam2[i] = p2.gamma2[c];
        if (!BWD && p2.beta2) bet2[i] = p2.beta2[c];
        if (!BWD && p2.rmean2 != nullptr && g == 0) {
          rm2[i] = p2.rmean2[c];
          rv2[i] = p2.rvar2[c];
        }
      }
    }
  }
  f32x4 v[NP], d[NP], m[NP], v2[PAIR ? NP : 1];
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f}, one = {1.f, 1.f, 1.f, 1.f};
  const int64_t slab = (int64_t)N * CHW;
#pragma unroll
  for (int k = 0; k < NP; ++k) {  // every load in flight before any use
    const int n = row0 + g + k * RG;
    const bool ok = ok_col && row_ok(k);
    const int64_t o = (int64_t)n * CHW + j0;
    f32x4 sum = zero;
    if (src != nullptr && ok) {  // deferred split-K sum, slab order (bitwise = conv_slab_sum)
      sum = *reinterpret_cast<const f32x4*>(src + o);
      for (int z = 1; z < nslab; ++z) sum += *reinterpret_cast<const f32x4*>(src + z * slab + o);
      if (BWD && res != nullptr) sum += *reinterpret_cast<const f32x4*>(res + o);
    }
    if (!BWD) {
      v[k] = ok ? (src ? sum : *reinterpret_cast<const f32x4*>(x + o)) : zero;
      if constexpr (PAIR) {  // the downsample conv output (or its split-K slabs, slab order)
        f32x4 t = zero;
        if (ok && p2.src2 != nullptr) {
          t = *reinterpret_cast<const f32x4*>(p2.src2 + o);
          for (int z = 1; z < p2.nslab2; ++z) t += *reinterpret_cast<const f32x4*>(p2.src2 + z * slab + o);
        } else if (ok) {
          t = *reinterpret_cast<const f32x4*>(p2.x2 + o);
        }
        d[k] = t;
      } else {
        d[k] = (ok && res) ? *reinterpret_cast<const f32x4*>(res + o) : zero;
      }
    } else {
      v[k] = ok ? *reinterpret_cast<const f32x4*>(x + o) : zero;
      d[k] = ok ? (src ? sum : *reinterpret_cast<const f32x4*>(dy + o)) : zero;
      m[k] = (ok && relu) ? *reinterpret_cast<const f32x4*>(yin + o) : one;
      if constexpr (PAIR) v2[k] = ok ? *reinterpret_cast<const f32x4*>(p2.x2 + o) : zero;
    }
  }
  if (!BWD && src != nullptr) {  // BN's saved input = the conv output
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = row0 + g + k * RG;
      if (ok_col && row_ok(k)) *reinterpret_cast<f32x4*>(const_cast<float*>(x) + (int64_t)n * CHW + j0) = v[k];
    }
  }
  if constexpr (PAIR) {
    if (!BWD && p2.src2 != nullptr) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int n = g + k * RG;
        if (ok_col && n < N) *reinterpret_cast<f32x4*>(const_cast<float*>(p2.x2) + (int64_t)n * CHW + j0) = d[k];
      }
    }
  }
  constexpr int NR = PAIR ? 4 : 2;  // reduced sums per channel: a, b (+ a2, b2)
  double r[NR][NCH];
#pragma unroll
  for (int q = 0; q < NR; ++q)
#pragma unroll
    for (int i = 0; i < NCH; ++i) r[q][i] = 0.0;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    if (ok_col && row_ok(k)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = e / CPC;
        if (!BWD) {
          r[0][i] += (double)v[k][e];
          r[1][i] += (double)v[k][e] * (double)v[k][e];
          if constexpr (PAIR) {
            r[NR - 2][i] += (double)d[k][e];
            r[NR - 1][i] += (double)d[k][e] * (double)d[k][e];
          }
        } else {
          const float dz = (m[k][e] > 0.f) ? d[k][e] : 0.f;
          r[0][i] += (double)dz;
          r[1][i] += (double)dz * (double)((v[k][e] - mean_s[i]) * invstd_s[i]);
          if constexpr (PAIR) r[NR - 1][i] += (double)dz * (double)((v2[k][e] - mean2[i]) * invstd2[i]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    if (BWD && PAIR && q == 2) continue;  // backward: sum dz is shared by both BNs
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
#pragma unroll
      for (int o = LPC / 2; o > 0; o >>= 1)  // the float4s of a channel are adjacent lanes
        r[q][i] += __shfl_xor(r[q][i], o, 64);
#pragma unroll
      for (int o = CT; o < 64; o <<= 1)  // row groups inside the wave
        r[q][i] += __shfl_xor(r[q][i], o, 64);
    }
  }
  // channel slot of this thread's first channel inside the workgroup
  const int slot = (4 * ct) / HW;
  const bool lead = HW >= 4 ? ((4 * ct) % HW) == 0 : true;  // one writer lane per channel
  if (lane < CT && lead) {
#pragma unroll
    for (int q = 0; q < NR; ++q)
#pragma unroll
      for (int i = 0; i < NCH; ++i) red[q][wave][slot + i] = r[q][i];
  }
  __syncthreads();
  double R[NR][NCH];
#pragma unroll
  for (int q = 0; q < NR; ++q)
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      R[q][i] = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) R[q][i] += red[q][w][slot + i];
    }
  if constexpr (SPLIT > 1) {  // the column block's SPLIT partials (NCH = 1, slot = 0 here)
    double* mine = sx.part + ((int64_t)cb * SPLIT + split) * 4;
    if (threadIdx.x < NR) {
#pragma unroll
      for (int q = 0; q < NR; ++q)
        if ((int)threadIdx.x == q) __hip_atomic_store(mine + q, R[q][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave drains
    __syncthreads();  // every wave has read red[] before it is reused as the flag below
    if (threadIdx.x == 0) {
      unsigned long long* ctr = sx.ctr + cb;
      const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long target = (old / SPLIT + 1) * SPLIT;
      unsigned spins = 0;
      int bad = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > sx.max_spins) { bad = 1; break; }  // never hang the GPU: poison (below)
      }
      red[0][0][0] = bad ? __builtin_nan("") : 0.0;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: sc1 loads follow
    const double poison = red[0][0][0];
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(sx.part + (int64_t)cb * SPLIT * 4, (short)0, SPLIT * 4 * 8,
                                                      0x00020000);
    double t[SPLIT][NR];
#pragma unroll
    for (int u = 0; u < SPLIT; ++u)
#pragma unroll
      for (int q = 0; q < NR; ++q)
        t[u][q] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (u * 4 + q) * 8, 0, 16));
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      double acc = t[0][q];
#pragma unroll
      for (int u = 1; u < SPLIT; ++u) acc += t[u][q];
      R[q][0] = acc + poison;
    }
  }
  const double* A = R[0];
  const double* B = R[1];
  if (!ok_col) return;
  const double M = (double)N * HW;
  const bool writer = g == 0 && lead && split == 0;
  if (!BWD) {
    f32x4 sc, sh, sc2 = zero, sh2 = zero;
    if constexpr (PAIR) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const double mu = R[NR - 2][i] / M;
        double var = R[NR - 1][i] / M - mu * mu;
        if (var < 0.0) var = 0.0;
        const float mean = (float)mu, invstd = (float)(1.0 / sqrt(var + (double)eps));
        const float scale = gam2[i] * invstd;
        const float shift = bet2[i] - mean * scale;
#pragma unroll
        for (int e = 0; e < CPC; ++e) {
          sc2[i * CPC + e] = scale;
          sh2[i * CPC + e] = shift;
        }
        if (writer) {
          const int c = c0 + i;
          p2.save_mean2[c] = mean;
          p2.save_invstd2[c] = invstd;
          if (p2.rmean2 != nullptr) {
            const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
            p2.rmean2[c] = (float)((1.0 - momentum) * (double)rm2[i] + momentum * mu);
            p2.rvar2[c] = (float)((1.0 - momentum) * (double)rv2[i] + momentum * unb);
          }
          if (p2.nbt2 != nullptr && c == 0) p2.nbt2[0] += 1;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const double mu = A[i] / M;
      double var = B[i] / M - mu * mu;
      if (var < 0.0) var = 0.0;
      const float mean = (float)mu, invstd = (float)(1.0 / sqrt(var + (double)eps));
      const float scale = gam[i] * invstd;
      const float shift = bet[i] - mean * scale;
#pragma unroll
      for (int e = 0; e < CPC; ++e) {
        sc[i * CPC + e] = scale;
        sh[i * CPC + e] = shift;
      }
      if (writer) {
        const int c = c0 + i;
        save_mean[c] = mean;
        save_invstd[c] = invstd;
        if (rmean != nullptr) {
          const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
          rmean[c] = (float)((1.0 - momentum) * (double)rm[i] + momentum * mu);
          rvar[c] = (float)((1.0 - momentum) * (double)rv[i] + momentum * unb);
        }
        if (nbt != nullptr && c == 0) nbt[0] += 1;
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = row0 + g + k * RG;
      if (row_ok(k)) {
        f32x4 z;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = PAIR ? fmaf(v[k][e], sc[e], sh[e]) + fmaf(d[k][e], sc2[e], sh2[e])
                               : fmaf(v[k][e], sc[e], sh[e]) + d[k][e];
          z[e] = relu ? fmaxf(t, 0.f) : t;
        }
        *reinterpret_cast<f32x4*>(out + (int64_t)n * CHW + j0) = z;
      }
    }
  } else {
    f32x4 k1, mdz, mdzx, mu, is, k12, mdzx2, mu2, is2;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (writer) {
        if (dgamma) dgamma[c0 + i] = (float)B[i];
        if (dbeta) dbeta[c0 + i] = (float)A[i];
        if constexpr (PAIR) {
          if (p2.dgamma2) p2.dgamma2[c0 + i] = (float)R[NR - 1][i];
          if (p2.dbeta2) p2.dbeta2[c0 + i] = (float)A[i];
        }
      }
#pragma unroll
      for (int e = 0; e < CPC; ++e) {
        k1[i * CPC + e] = gam[i] * invstd_s[i];
        mdz[i * CPC + e] = (float)(A[i] / M);
        mdzx[i * CPC + e] = (float)(B[i] / M);
        mu[i * CPC + e] = mean_s[i];
        is[i * CPC + e] = invstd_s[i];
        k12[i * CPC + e] = gam2[i] * invstd2[i];
        mdzx2[i * CPC + e] = (float)(R[NR - 1][i] / M);
        mu2[i * CPC + e] = mean2[i];
        is2[i * CPC + e] = invstd2[i];
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int n = row0 + g + k * RG;
      if (row_ok(k)) {
        f32x4 o4, z4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dz = (m[k][e] > 0.f) ? d[k][e] : 0.f;
          const float xh = (v[k][e] - mu[e]) * is[e];
          o4[e] = k1[e] * (dz - mdz[e] - xh * mdzx[e]);
          if constexpr (PAIR) z4[e] = k12[e] * (dz - mdz[e] - (v2[k][e] - mu2[e]) * is2[e] * mdzx2[e]);
          else z4[e] = dz;
        }
        const int64_t o = (int64_t)n * CHW + j0;
        *reinterpret_cast<f32x4*>(out + o) = o4;
        if constexpr (PAIR) *reinterpret_cast<f32x4*>(p2.out2 + o) = z4;
        else if (dres) *reinterpret_cast<f32x4*>(dres + o) = z4;
      }
    }
  }
}

// Single-launch small-map path: HW in {1, 2, 4, 8, 16} (ResNet-18 step on 1x MI355X: HW <= 4 ->
// 2.165 ms, <= 16 (layer2 too) -> 2.150 ms), N <= kFusedMaxN.  The 8x8 maps of layer1 (64
// workgroups, one per channel) measured slower than the two-kernel path at batch 64 / 128
// (1.0797 vs 1.0772 / 1.2322 vs 1.2122 ms) and so did row splits over a cross-workgroup barrier
// (batch 512 1.908 -> 1.960 / 1.966 ms; round 4, removed in round 5).
// The 8x8 maps (layer1) take it too at per-GPU batch <= 128 (the float4 kernel, one channel per
// workgroup, <= 128 rows): the split-K convs there emit no epilogue statistics, so the two-kernel
// path ran a statistics pass and an apply pass per direction.
constexpr int kFusedMaxN64 = 128;
static bool bn_fused_ok(int N, int C, int HW) {
  return (((HW == 1 || HW == 2 || HW == 4 || HW == 8 || HW == 16) && N <= kFusedMaxN) ||
          (HW == 64 && N <= kFusedMaxN64 && !vec_off())) &&
         N >= 1 && (int64_t)N * C * HW < (1LL << 30);
}

// column-block width for one launch: the widest block that still gives >= 256 workgroups (one per
// CU), else the narrowest allowed one (4 columns, 16-B row segments: grid size matters more than
// segment width).  Measured in round 3 with 4 columns at batch <= 128 only (profiles/r3/bn_colw.md)
// against a fixed 8: ResNet-18 r=4 batch 512 1.945 -> 1.943 ms, batch 64 1.012 -> 1.000 ms,
// ResNet-152 r=4 15.19 -> 14.78 ms, ResNet-50 dense 6.246 -> 6.178 ms.
// Round 5 (float4 kernel): 4-column blocks at every batch, not only <= 128 — ResNet-18 r=4 batch
// 512 1.4994 / 1.4922 -> 1.4864 / 1.4862 ms, batch 256 1.1095 -> 1.1033 (layer3 / layer4 BNs get
// 2x the workgroups; profiles/r5/bench_bn_colw.jsonl).
static int bn_colw_for(int HW, int C, int N) {
  (void)N;
  const int lo = 4;
  const int64_t cols = (int64_t)C * HW;
  for (int cw = 16; cw >= lo; cw >>= 1)
    if (cw >= HW && cols / cw >= 256) return cw;
  return HW > lo ? HW : lo;
}

template <int BWD, int CW>
static void launch_small_fused_cw(int HW, const float* x, const float* res, const float* dy, const float* yin,
                                  const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
                                  float* sm, float* si, float* dgamma, float* dbeta, float* out, float* dres, int N,
                                  int C, float eps, float momentum, int relu, hipStream_t s, const float* src,
                                  int nslab, const BnPair* pr) {
  const int nblk = (int)(((int64_t)C * HW + CW - 1) / CW);
  const BnPair pp = pr ? *pr : BnPair{};
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  // float4 kernel: rows of whole float4s, 16-B aligned operands.  Not for small maps at small
  // batches: with HW <= 4 and N <= 128 the scalar kernel's 4-column blocks keep 4x more threads
  // busy per row and its reduction is shorter — ResNet-18 at batch 64: HW = 1 4.8 vs 6.7 µs, HW = 4
  // 4.8 vs 5.0 µs per launch (v4 wins everywhere at batch 512 and for HW = 16: 8.0 -> 5.3 µs at 64)
  const bool v4 = ((int64_t)C * HW) % 4 == 0 && a16(x) && a16(res) && a16(dy) && a16(yin) && a16(out) &&
                  a16(dres) && a16(src) && (pr == nullptr || (a16(pr->x2) && a16(pr->out2) && a16(pr->src2) && HW >= 4)) &&
                  !vec_off() && (HW >= 8 || N > 128);  // (pair at HW < 4: 4 channels' operands per float4 spill)
#define NDP_BN_FUSED_P(HWV, P)                                                                                     \
  if (v4) {                                                                                                        \
    if constexpr (P == 0 || HWV >= 4)                                                                              \
      hipLaunchKernelGGL((bn_small_fused_v4_kernel<HWV, BWD, CW, kFusedMaxN, P>), dim3((unsigned)nblk),            \
                         dim3(kFusedThreads), 0, s, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma,  \
                         dbeta, out, dres, N, C, eps, momentum, relu, src, nslab, pp);                               \
  } else                                                                                                           \
    hipLaunchKernelGGL((bn_small_fused_kernel<HWV, BWD, CW, kFusedMaxN, P>), dim3((unsigned)nblk),                 \
                       dim3(kFusedThreads), 0, s, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma,    \
                       dbeta, out, dres, N, C, eps, momentum, relu, src, nslab, pp);
#define NDP_BN_FUSED(HWV)                                                                                          \
  if constexpr (CW % HWV == 0) {                                                                                   \
    if (pr) {                                                                                                      \
      NDP_BN_FUSED_P(HWV, 1)                                                                                       \
    } else {                                                                                                       \
      NDP_BN_FUSED_P(HWV, 0)                                                                                       \
    }                                                                                                              \
  }
  switch (HW) {  // the caller picks CW >= HW
    case 1: NDP_BN_FUSED(1); break;
    case 2: NDP_BN_FUSED(2); break;
    case 4: NDP_BN_FUSED(4); break;
    case 8: NDP_BN_FUSED(8); break;
    default: NDP_BN_FUSED(16); break;
  }
#undef NDP_BN_FUSED
#undef NDP_BN_FUSED_P
}

// Row splits of the 8x8-map single-launch BN (bn_small_fused_v4_kernel SPLIT): workgroups per
// channel.  NDP_BN_SPLIT = 1 / 2 / 4 (A/B); the exchange scratch is allocated once per device, on
// the first (eager, never captured) call, and its counters are zeroed then.
// Measured (ResNet-18 r=4, 1x MI355X, round 6): batch 64 split 1 / 2 / 4 = 0.7683 / 0.7607 /
// 0.7671 ms, batch 128 split 1 / 4 = 0.8654 / 0.8547 ms — the launch stays latency-bound (~6 µs
// for 1 MB), so the gain is small; default 2 below 128 rows, 4 from 128.
static int bn_row_split(int N, int C) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("NDP_BN_SPLIT");
    v = e ? atoi(e) : 0;
    if (v != 0 && v != 1 && v != 2 && v != 4) v = 0;
  }
  const int sp = v ? v : (N >= 128 ? 4 : 2);
  if (C > 1024 || N < 8 * sp) return 1;
  return sp;
}

static BnSplitCtx bn_split_ctx(int C, int split) {
  constexpr int kCols = 1024;  // column blocks (channels) covered
  struct Buf { double* part = nullptr; unsigned long long* ctr = nullptr; };
  static Buf bufs[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  Buf& b = bufs[dev & 63];
  if (b.part == nullptr) {
    (void)hipMalloc(&b.part, sizeof(double) * kCols * 4 * 4);
    (void)hipMalloc(&b.ctr, sizeof(unsigned long long) * kCols * 3);
    (void)hipMemset(b.ctr, 0, sizeof(unsigned long long) * kCols * 3);
    (void)hipDeviceSynchronize();
  }
  (void)C;
  // one counter range per split factor: a counter only ever moves in steps of its own SPLIT
  return BnSplitCtx{b.part, b.ctr + (split == 2 ? 0 : kCols), 1u << 22};
}

template <int BWD>
static void launch_small_fused(int HW, const float* x, const float* res, const float* dy, const float* yin,
                               const float* gamma, const float* beta, float* rmean, float* rvar, int64_t* nbt,
                               float* sm, float* si, float* dgamma, float* dbeta, float* out, float* dres, int N,
                               int C, float eps, float momentum, int relu, hipStream_t s, const float* src,
                               int nslab, const BnPair* pr = nullptr) {
  if (HW == 64) {  // one channel per workgroup (bn_fused_ok); float4 unless an operand is unaligned
    auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (pr != nullptr) return;  // (bn_pair_ok: no pair on the 8x8 maps)
    const int split = bn_row_split(N, C);
    if (a16(x) && a16(res) && a16(dy) && a16(yin) && a16(out) && a16(dres) && a16(src) && split > 1) {
      const BnSplitCtx sx = bn_split_ctx(C, split);
#define NDP_BN_SPLIT_LAUNCH(SP)                                                                                  \
  hipLaunchKernelGGL((bn_small_fused_v4_kernel<64, BWD, 64, kFusedMaxN64, 0, SP>), dim3((unsigned)(C * SP)),     \
                     dim3(kFusedThreads), 0, s, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma,  \
                     dbeta, out, dres, N, C, eps, momentum, relu, src, nslab, BnPair{}, sx)
      if (split == 2) NDP_BN_SPLIT_LAUNCH(2);
      else NDP_BN_SPLIT_LAUNCH(4);
#undef NDP_BN_SPLIT_LAUNCH
    } else if (a16(x) && a16(res) && a16(dy) && a16(yin) && a16(out) && a16(dres) && a16(src))
      hipLaunchKernelGGL((bn_small_fused_v4_kernel<64, BWD, 64, kFusedMaxN64>), dim3((unsigned)C),
                         dim3(kFusedThreads), 0, s, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma,
                         dbeta, out, dres, N, C, eps, momentum, relu, src, nslab, BnPair{});
    else
      hipLaunchKernelGGL((bn_small_fused_kernel<64, BWD, 64, kFusedMaxN64>), dim3((unsigned)C), dim3(kFusedThreads),
                         0, s, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma, dbeta, out, dres, N, C,
                         eps, momentum, relu, src, nslab, BnPair{});
    return;
  }
  switch (bn_colw_for(HW, C, N)) {
    case 16:
      launch_small_fused_cw<BWD, 16>(HW, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma, dbeta, out,
                                     dres, N, C, eps, momentum, relu, s, src, nslab, pr);
      break;
    case 4:
      launch_small_fused_cw<BWD, 4>(HW, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma, dbeta, out,
                                    dres, N, C, eps, momentum, relu, s, src, nslab, pr);
      break;
    default:
      launch_small_fused_cw<BWD, 8>(HW, x, res, dy, yin, gamma, beta, rmean, rvar, nbt, sm, si, dgamma, dbeta, out,
                                    dres, N, C, eps, momentum, relu, s, src, nslab, pr);
  }
}


template <int HW>
static void small_stats(const float* x, const float* dy, const float* y, const float* sm, const float* si,
                        double* part, int N, int C, int S, int bwd, int relu, hipStream_t s) {
  const dim3 grid(S, (C * HW + 255) / 256);
  hipLaunchKernelGGL(bn_small_stats_kernel<HW>, grid, dim3(256), 0, s, x, dy, y, sm, si, part, N, C, S, bwd, relu);
}

static void small_stats_any(int HW, const float* x, const float* dy, const float* y, const float* sm, const float* si,
                            double* part, int N, int C, int S, int bwd, int relu, hipStream_t s) {
  switch (HW) {
    case 1: small_stats<1>(x, dy, y, sm, si, part, N, C, S, bwd, relu, s); break;
    case 2: small_stats<2>(x, dy, y, sm, si, part, N, C, S, bwd, relu, s); break;
    case 4: small_stats<4>(x, dy, y, sm, si, part, N, C, S, bwd, relu, s); break;
    case 8: small_stats<8>(x, dy, y, sm, si, part, N, C, S, bwd, relu, s); break;
    default: small_stats<16>(x, dy, y, sm, si, part, N, C, S, bwd, relu, s); break;
  }
}

// the three-kernel small-map path (statistics, finalize, apply) for HW <= 4 where the
// single-launch kernel does not apply (batch > 512); HW = 16 measured faster on the
// per-channel kernels
bool bn_small_path(int N, int C, int HW) {
  return (HW == 1 || HW == 2 || HW == 4) && (int64_t)N * C * HW < (1LL << 30);
}

// scratch: the per-launch slice partials and coefficients (fp64)
int64_t bn_part_numel(int N, int C, int HW) {
  const int64_t big = (int64_t)C * bn_slices(N, C, HW) * 2;
  const int64_t small = (int64_t)C * bn_small_slices(N, C, HW) * 2 + 3 * (int64_t)C;
  return big > small ? big : small;
}

// ----------------------------------- launchers -------------------------------------------
// Deferred conv slabs are summed inside the single-launch BN kernel only up to this many:
// ResNet-18 step on 1x MI355X, layer2 (HW 16) at per-GPU batch 256 (2 slabs) 1.4968 ->
// 1.4688 ms, batch 128 (4) 1.2158 -> 1.2176 (even), batch 64 (8 slabs) 1.0689 -> 1.0746 (the
// BN's 128 workgroups read 8 slabs slower than the 256-CU sum kernel plus a launch).
constexpr int kMaxFusedSlabs = 4;
// Two-kernel path (8x8 maps of layer1): the statistics pass adds the deferred slabs and writes
// the summed tensor, no separate sum launch.  ResNet-18 step on 1x MI355X: batch 128 1.196 /
// 1.198 -> 1.164 / 1.165 ms, batch 64 1.061 / 1.058 -> 1.046 / 1.053.
int bn_slices(int N, int C, int HW) {
  // ~4 workgroups per CU over the whole launch, >= ~2K elements per workgroup
  int64_t s = (1024 + C - 1) / C;
  const int64_t by_work = ((int64_t)N * HW) / 2048;
  if (s > by_work) s = by_work;
  if (s > N) s = N;
  if (s < 1) s = 1;
  return (int)s;
}

// apply-pass slices when the statistics come from a conv epilogue: every apply workgroup folds
// ALL the conv's per-image partials of its channel (fewer, larger workgroups measured slower:
// ResNet-18 r=4 batch 512, S / 1 / 2 / 4 / 8 = 1.862-1.874 / 1.864 / 1.884 / 1.926 ms, round 4)
static int ext_apply_slices(int S) { return S < 1 ? 1 : S; }

void launch_bn_fwd(const float* x, const float* res, float* y, const float* gamma, const float* beta,
                   float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                   double* part, int N, int C, int HW, int S, float eps, float momentum, int relu,
                   int training, int single, hipStream_t s, const float* xpart, int nslab, const double* xstats,
                   int xS) {
  if (!training || xpart != nullptr) xstats = nullptr;
  if (xpart != nullptr && nslab < 2) xpart = nullptr;
  if (xpart != nullptr && nslab > kMaxFusedSlabs) {  // many slabs: the wide sum kernel first
    launch_slab_sum(xpart, const_cast<float*>(x), (int64_t)N * C * HW, nslab, s);
    xpart = nullptr;
  }
  if (training && single && bn_fused_ok(N, C, HW)) {
    launch_small_fused<0>(HW, x, res, nullptr, nullptr, gamma, beta, rmean, rvar, nbt, save_mean, save_invstd,
                          nullptr, nullptr, y, nullptr, N, C, eps, momentum, relu, s, xpart, nslab);
    return;
  }
  const bool vec_ok = (HW % 4) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                      (res == nullptr || ((uintptr_t)res & 15) == 0) && ((uintptr_t)xpart & 15) == 0;
  if (xpart != nullptr && !(training && vec_ok && !bn_small_path(N, C, HW))) {
    // no fused consumer for this shape: finish the conv's split-K sum here
    launch_slab_sum(xpart, const_cast<float*>(x), (int64_t)N * C * HW, nslab, s);
    xpart = nullptr;
  }
  if (training && bn_small_path(N, C, HW)) {
    const int Ss = bn_small_slices(N, C, HW);
    double* coef = part + (int64_t)C * Ss * 2;
    small_stats_any(HW, x, nullptr, nullptr, nullptr, nullptr, part, N, C, Ss, 0, 0, s);
    hipLaunchKernelGGL(bn_small_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, s, part, coef, gamma, beta, rmean,
                       rvar, nbt, save_mean, save_invstd, nullptr, nullptr, N, C, HW, Ss, eps, momentum, 0);
    const int total = N * C * HW;
    hipLaunchKernelGGL(bn_small_apply_kernel, dim3((unsigned)((total / 4 + 255) / 256 + 1)), dim3(256), 0, s, x, res,
                       nullptr, nullptr, nullptr, nullptr, coef, y, nullptr, total, C, HW, relu, 0);
    return;
  }
  const bool vec = (HW % 4) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                   (res == nullptr || ((uintptr_t)res & 15) == 0);
  const dim3 grid(S, C);
  // statistics from the conv epilogue (xstats): no statistics pass, the apply folds xS partials
  const double* ap = xstats != nullptr ? xstats : part;
  const int Sp = xstats != nullptr ? xS : 0;
  if (training && xstats == nullptr) {  // the statistics pass also adds deferred conv slabs (xpart), writes x
    if (vec) hipLaunchKernelGGL(bn_fwd_stats_kernel<true>, grid, dim3(256), 0, s, x, part, N, C, HW, S, xpart, nslab);
    else hipLaunchKernelGGL(bn_fwd_stats_kernel<false>, grid, dim3(256), 0, s, x, part, N, C, HW, S, nullptr, 0);
  }
  const int Sa = Sp > 0 ? ext_apply_slices(S) : S;
  const dim3 agrid(Sa, C);
  if (vec)
    hipLaunchKernelGGL(bn_fwd_apply_kernel<true>, agrid, dim3(256), 0, s, x, res, y, gamma, beta, rmean, rvar, nbt,
                       save_mean, save_invstd, ap, N, C, HW, Sa, eps, momentum, relu, training, Sp);
  else
    hipLaunchKernelGGL(bn_fwd_apply_kernel<false>, agrid, dim3(256), 0, s, x, res, y, gamma, beta, rmean, rvar, nbt,
                       save_mean, save_invstd, ap, N, C, HW, Sa, eps, momentum, relu, training, Sp);
}

// training-mode stem tail (bn_relu_maxpool_kernel); xstats as in launch_bn_fwd (nullable)
void launch_bn_relu_maxpool(const float* x, float* y, uint8_t* idx, const float* gamma, const float* beta,
                            float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                            double* part, int N, int C, int H, int W, float eps, float momentum, hipStream_t s,
                            const double* xstats, int xS) {
  const int HW = H * W;
  const int S = bn_slices(N, C, HW);
  const dim3 grid(S, C);
  if (xstats == nullptr) {
    const bool vec = (HW % 4) == 0 && ((uintptr_t)x & 15) == 0;
    if (vec) hipLaunchKernelGGL(bn_fwd_stats_kernel<true>, grid, dim3(256), 0, s, x, part, N, C, HW, S, nullptr, 0);
    else hipLaunchKernelGGL(bn_fwd_stats_kernel<false>, grid, dim3(256), 0, s, x, part, N, C, HW, S, nullptr, 0);
  }
  const int Sa = xstats != nullptr ? ext_apply_slices(S) : S;
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(Sa, C), dim3(256), 0, s, x, y, idx, gamma, beta, rmean, rvar, nbt,
                     save_mean, save_invstd, xstats != nullptr ? xstats : part, N, C, H, W, Sa, eps, momentum,
                     xstats != nullptr ? xS : 0);
}

// The downsample block's two BatchNorms in one launch (BnPair): the small-map single-launch
// kernels, i.e. layers 2-4 of the ResNet-18 step at per-GPU batch <= 512 (not the 8x8 maps).
bool bn_pair_ok(int N, int C, int HW) { return HW != 64 && bn_fused_ok(N, C, HW); }

void launch_bn_pair_fwd(const float* x, const float* x2, float* y, const float* gamma, const float* beta,
                        float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                        const float* gamma2, const float* beta2, float* rmean2, float* rvar2, int64_t* nbt2,
                        float* save_mean2, float* save_invstd2, int N, int C, int HW, float eps, float momentum,
                        hipStream_t s, const float* xpart, int nslab, const float* x2part, int nslab2) {
  if (xpart != nullptr && nslab < 2) xpart = nullptr;
  if (xpart != nullptr && nslab > kMaxFusedSlabs) {
    launch_slab_sum(xpart, const_cast<float*>(x), (int64_t)N * C * HW, nslab, s);
    xpart = nullptr;
  }
  if (x2part != nullptr && nslab2 < 2) x2part = nullptr;
  if (x2part != nullptr && nslab2 > kMaxFusedSlabs) {
    launch_slab_sum(x2part, const_cast<float*>(x2), (int64_t)N * C * HW, nslab2, s);
    x2part = nullptr;
  }
  const BnPair pr{x2, gamma2, beta2, rmean2, rvar2, nbt2, save_mean2, save_invstd2, nullptr, nullptr, nullptr,
                  x2part, x2part ? nslab2 : 0};
  launch_small_fused<0>(HW, x, nullptr, nullptr, nullptr, gamma, beta, rmean, rvar, nbt, save_mean, save_invstd,
                        nullptr, nullptr, y, nullptr, N, C, eps, momentum, 1, s, xpart, nslab, &pr);
}

void launch_bn_pair_bwd(const float* dy, const float* y, const float* x, const float* x2, const float* gamma,
                        const float* save_mean, const float* save_invstd, const float* gamma2,
                        const float* save_mean2, const float* save_invstd2, float* dx, float* dx2, float* dgamma,
                        float* dbeta, float* dgamma2, float* dbeta2, int N, int C, int HW, hipStream_t s,
                        const float* dypart, int nslab, const float* dyadd) {
  if (dypart != nullptr && nslab < 2) dypart = nullptr;
  if (dypart == nullptr) dyadd = nullptr;
  if (dypart != nullptr && nslab > kMaxFusedSlabs) {
    launch_slab_sum(dypart, const_cast<float*>(dy), (int64_t)N * C * HW, nslab, s, dyadd);
    dypart = nullptr;
    dyadd = nullptr;
  }
  const BnPair pr{x2, gamma2, nullptr, nullptr, nullptr, nullptr, const_cast<float*>(save_mean2),
                  const_cast<float*>(save_invstd2), dgamma2, dbeta2, dx2, nullptr, 0};
  launch_small_fused<1>(HW, x, dyadd, dy, y, gamma, nullptr, nullptr, nullptr, nullptr, const_cast<float*>(save_mean),
                        const_cast<float*>(save_invstd), dgamma, dbeta, dx, nullptr, N, C, 0.f, 0.f, 1, s, dypart,
                        nslab, &pr);
}

bool bn_two_kernel_path(int N, int C, int HW, int single) {
  return !(single && bn_fused_ok(N, C, HW)) && !bn_small_path(N, C, HW);
}

void launch_bn_bwd(const float* dy, const float* y, const float* x, const float* gamma, const float* save_mean,
                   const float* save_invstd, float* dx, float* dres, float* dgamma, float* dbeta, double* part,
                   int N, int C, int HW, int S, int relu, int single, hipStream_t s, const float* dypart,
                   int nslab, const float* dyadd, const float* mbeta, const double* dstats, int dS) {
  if (dypart != nullptr && nslab < 2) dypart = nullptr;
  if (dypart == nullptr) dyadd = nullptr;
  if (dypart != nullptr && nslab > kMaxFusedSlabs) {
    launch_slab_sum(dypart, const_cast<float*>(dy), (int64_t)N * C * HW, nslab, s, dyadd);
    dypart = nullptr;
    dyadd = nullptr;
  }
  if (single && bn_fused_ok(N, C, HW)) {  // (the backward kernel's `res` slot: the slab addend)
    launch_small_fused<1>(HW, x, dyadd, dy, y, gamma, nullptr, nullptr, nullptr, nullptr,
                          const_cast<float*>(save_mean), const_cast<float*>(save_invstd), dgamma, dbeta, dx, dres, N, C,
                          0.f, 0.f, relu, s, dypart, nslab);
    return;
  }
  const bool vec_ok = (HW % 4) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 &&
                      ((uintptr_t)dx & 15) == 0 && (!relu || ((uintptr_t)y & 15) == 0) &&
                      (dres == nullptr || ((uintptr_t)dres & 15) == 0) && ((uintptr_t)dypart & 15) == 0;
  if (dypart != nullptr && !(vec_ok && !bn_small_path(N, C, HW) &&
                             (dyadd == nullptr || ((uintptr_t)dyadd & 15) == 0))) {
    // no fused consumer: finish the conv's split-K grad-x sum into dy
    launch_slab_sum(dypart, const_cast<float*>(dy), (int64_t)N * C * HW, nslab, s, dyadd);
    dypart = nullptr;
    dyadd = nullptr;
  }
  if (bn_small_path(N, C, HW)) {
    const int Ss = bn_small_slices(N, C, HW);
    double* coef = part + (int64_t)C * Ss * 2;
    small_stats_any(HW, x, dy, y, save_mean, save_invstd, part, N, C, Ss, 1, relu, s);
    hipLaunchKernelGGL(bn_small_finalize_kernel, dim3((C + 3) / 4), dim3(256), 0, s, part, coef, gamma, nullptr,
                       nullptr, nullptr, nullptr, nullptr, const_cast<float*>(save_invstd), dgamma, dbeta, N, C, HW, Ss,
                       0.f, 0.f, 1);
    const int total = N * C * HW;
    hipLaunchKernelGGL(bn_small_apply_kernel, dim3((unsigned)((total / 4 + 255) / 256 + 1)), dim3(256), 0, s, x,
                       nullptr, dy, y, save_mean, save_invstd, coef, dx, dres, total, C, HW, relu, 1);
    return;
  }
  const bool vec = (HW % 4) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 &&
                   ((uintptr_t)dx & 15) == 0 && (!relu || ((uintptr_t)y & 15) == 0) &&
                   (dres == nullptr || ((uintptr_t)dres & 15) == 0);
  const dim3 grid(S, C);
  if (vec) {  // the statistics pass also adds deferred grad-x slabs (dypart) and writes dy
    // (dstats: the statistics came from the producing conv's grad-x epilogue, no pass)
    if (dstats == nullptr || dypart != nullptr)
      hipLaunchKernelGGL(bn_bwd_stats_kernel<true>, grid, dim3(256), 0, s, dy, y, x, save_mean, save_invstd, part, N,
                         C, HW, S, relu, dypart, nslab, dyadd, gamma, mbeta);
    const bool ext_st = dstats != nullptr && dypart == nullptr;
    const int Sa = ext_st ? ext_apply_slices(S) : S;
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(Sa, C), dim3(256), 0, s, dy, y, x, gamma, save_mean,
                       save_invstd, dx, dres, dgamma, dbeta, ext_st ? dstats : part, N, C, HW, Sa, relu, mbeta,
                       ext_st ? dS : 0);
  } else {
    hipLaunchKernelGGL(bn_bwd_stats_kernel<false>, grid, dim3(256), 0, s, dy, y, x, save_mean, save_invstd, part, N,
                       C, HW, S, relu);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, grid, dim3(256), 0, s, dy, y, x, gamma, save_mean, save_invstd, dx,
                       dres, dgamma, dbeta, part, N, C, HW, S, relu);
  }
}

}  // namespace ndp
