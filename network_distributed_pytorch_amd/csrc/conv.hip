// Convolution kernels for ResNet on CIFAR-shape inputs (NCHW fp32, gfx950).
//
// ResNet-18 on 32x32 images runs layer3/layer4 at 4x4 -> 2x2 -> 1x1 feature maps, where a
// 3x3 convolution is really a small dense matrix product ("Toeplitz" form, see
// models/conv_gemm.py):  out.view(B, Co*OH*OW) = x.view(B, C*H*W) @ W_big with
//   W_big[(ci,ih,iw), (co,oh,ow)] = W[co, ci, ih - oh*s + p, iw - ow*s + p]   (0 outside).
// The GEMMs run on hipBLASLt; these two kernels build W_big from W and fold grad-W_big back
// into grad-W with index arithmetic (no index tensors, no torch.cat / fill / gather /
// scatter chains: profiles/ showed ~0.6 ms per ResNet-18 step in those ATen launches).
// The fold sums the <= OH*OW taps of each weight in a fixed order: deterministic.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ndp_kernels.h"
#include "wino_dpp.h"

namespace ndp {

typedef float f32x4e __attribute__((ext_vector_type(4)));

// Device orientation: Wt_big = W_big^T, [N = Co*OH*OW rows][K = C*H*W cols], so that both
// kernels walk contiguous memory on both sides (a row of Wt_big reads one filter W[co]).
// grid: (ceil(K/256), N); one thread per Wt_big element
__global__ __launch_bounds__(256) void toeplitz_expand_kernel(const float* __restrict__ w, float* __restrict__ wt,
                                                              ConvGeom g) {
  const int K = g.C * g.H * g.W;
  const int kcol = blockIdx.x * 256 + threadIdx.x;
  if (kcol >= K) return;
  const int n = blockIdx.y;
  const int OHW = g.OH * g.OW;
  const int co = n / OHW, ohw = n - co * OHW;
  const int oh = ohw / g.OW, ow = ohw - oh * g.OW;
  const int HW = g.H * g.W;
  const int ci = kcol / HW, ihw = kcol - ci * HW;
  const int ih = ihw / g.W, iw = ihw - ih * g.W;
  const int kh = ih - oh * g.stride + g.pad, kw = iw - ow * g.stride + g.pad;
  float v = 0.f;
  if (kh >= 0 && kh < g.KH && kw >= 0 && kw < g.KW) v = w[((co * g.C + ci) * g.KH + kh) * g.KW + kw];
  wt[(int64_t)n * K + kcol] = v;
}

// Every Toeplitz layer of a model in ONE launch (forward start, ToeplitzBank in
// models/conv_gemm.py).  One workgroup per W_big^T row n = (co, oh, ow) of one layer (the
// layer is found by scanning the <= kMaxExpand row prefix sums in the kernel arguments — no
// table upload); thread t owns input channels ci = t, t + 256, ... and writes their H*W
// contiguous columns (one float4 per 4 columns for the 2x2 / 4x4 maps): all index math is
// per row or per channel, none per element.
template <int H, int W>
__device__ __forceinline__ void expand_row(const float* __restrict__ w, float* __restrict__ row, const ConvGeom& g,
                                           int co, int oh, int ow) {
  const int h0 = oh * g.stride - g.pad, w0 = ow * g.stride - g.pad;
  for (int ci = threadIdx.x; ci < g.C; ci += 256) {
    const float* wc = w + ((int64_t)co * g.C + ci) * g.KH * g.KW;
    float v[H * W];
#pragma unroll
    for (int ih = 0; ih < H; ++ih)
#pragma unroll
      for (int iw = 0; iw < W; ++iw) {
        const int kh = ih - h0, kw = iw - w0;
        v[ih * W + iw] = (kh >= 0 && kh < g.KH && kw >= 0 && kw < g.KW) ? wc[kh * g.KW + kw] : 0.f;
      }
    float* d = row + (int64_t)ci * (H * W);
    if constexpr ((H * W) % 4 == 0) {
#pragma unroll
      for (int j = 0; j < H * W; j += 4)
        *reinterpret_cast<f32x4e*>(d + j) = f32x4e{v[j], v[j + 1], v[j + 2], v[j + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < H * W; ++j) d[j] = v[j];
    }
  }
}

__global__ __launch_bounds__(256) void toeplitz_expand_many_kernel(ExpandBatch b) {
  const int64_t r = blockIdx.x;
  int e = 0;
  while (e + 1 < b.n && r >= b.end[e]) ++e;
  const ConvGeom& g = b.g[e];
  const int n = (int)(r - (e ? b.end[e - 1] : 0));
  const int OHW = g.OH * g.OW;
  const int co = n / OHW, ohw = n - co * OHW;
  const int oh = ohw / g.OW, ow = ohw - oh * g.OW;
  float* row = b.wt[e] + (int64_t)n * g.C * g.H * g.W;
  if (g.H == 1 && g.W == 1) expand_row<1, 1>(b.w[e], row, g, co, oh, ow);
  else if (g.H == 2 && g.W == 2) expand_row<2, 2>(b.w[e], row, g, co, oh, ow);
  else if (g.H == 4 && g.W == 4) expand_row<4, 4>(b.w[e], row, g, co, oh, ow);
  else {
    const int K = g.C * g.H * g.W, HW = g.H * g.W;
    for (int kcol = threadIdx.x; kcol < K; kcol += 256) {
      const int ci = kcol / HW, ihw = kcol - ci * HW;
      const int ih = ihw / g.W, iw = ihw - ih * g.W;
      const int kh = ih - oh * g.stride + g.pad, kw = iw - ow * g.stride + g.pad;
      float v = 0.f;
      if (kh >= 0 && kh < g.KH && kw >= 0 && kw < g.KW) v = b.w[e][((co * g.C + ci) * g.KH + kh) * g.KW + kw];
      row[kcol] = v;
    }
  }
}

// kExpandRows consecutive W_big^T rows of one layer per workgroup, the 256 threads over the
// rows' (row, ci) pairs: a one-row workgroup left half its threads idle at C = 128 and spent
// its time on the layer scan and index setup for 2-8 KB of stores (21.6 µs per ResNet-18
// forward for ~35 MB, 1.6 TB/s; profiles/r4).  Consecutive threads write consecutive H*W-float
// segments of a row: coalesced.  What remains (~19 µs at batch 64): PMC shows 42 MB READ for
// 37 MB written — layer4's 1x1-map layers use only the centre tap, but every cache line of
// their [co][ci][3][3] weights is fetched to extract it; issuing 2-4 pairs' loads per thread
// before their stores changed nothing (measured).
constexpr int kExpandRows = 8;
template <int H, int W>
__device__ __forceinline__ void expand_rows(const float* __restrict__ w, float* __restrict__ wt, const ConvGeom& g,
                                            int n0) {
  const int C = g.C, OHW = g.OH * g.OW;
  const int64_t K = (int64_t)C * H * W;
  for (int idx = threadIdx.x; idx < kExpandRows * C; idx += 256) {
    const int rr = idx / C, ci = idx - rr * C;
    const int n = n0 + rr;
    const int co = n / OHW, ohw = n - co * OHW;
    const int oh = ohw / g.OW, ow = ohw - oh * g.OW;
    const int h0 = oh * g.stride - g.pad, w0 = ow * g.stride - g.pad;
    const float* wc = w + ((int64_t)co * C + ci) * g.KH * g.KW;
    float v[H * W];
#pragma unroll
    for (int ih = 0; ih < H; ++ih)
#pragma unroll
      for (int iw = 0; iw < W; ++iw) {
        const int kh = ih - h0, kw = iw - w0;
        v[ih * W + iw] = (kh >= 0 && kh < g.KH && kw >= 0 && kw < g.KW) ? wc[kh * g.KW + kw] : 0.f;
      }
    float* d = wt + (int64_t)n * K + (int64_t)ci * (H * W);
    if constexpr ((H * W) % 4 == 0) {
#pragma unroll
      for (int j = 0; j < H * W; j += 4)
        *reinterpret_cast<f32x4e*>(d + j) = f32x4e{v[j], v[j + 1], v[j + 2], v[j + 3]};
    } else {
#pragma unroll
      for (int j = 0; j < H * W; ++j) d[j] = v[j];
    }
  }
}

__global__ __launch_bounds__(256) void toeplitz_expand_rows_kernel(ExpandBatch b) {
  const int64_t r0 = (int64_t)blockIdx.x * kExpandRows;
  int e = 0;
  while (e + 1 < b.n && r0 >= b.end[e]) ++e;
  const ConvGeom& g = b.g[e];
  const int n0 = (int)(r0 - (e ? b.end[e - 1] : 0));
  if (g.H == 1 && g.W == 1) expand_rows<1, 1>(b.w[e], b.wt[e], g, n0);
  else if (g.H == 2 && g.W == 2) expand_rows<2, 2>(b.w[e], b.wt[e], g, n0);
  else expand_rows<4, 4>(b.w[e], b.wt[e], g, n0);
}

void launch_toeplitz_expand_many(const ExpandBatch& b, hipStream_t s) {
  if (b.n <= 0) return;
  bool rows_ok = true;  // every layer's rows split into whole groups of the covered map sizes
  for (int e = 0; e < b.n; ++e) {
    const ConvGeom& g = b.g[e];
    const int64_t rows = b.end[e] - (e ? b.end[e - 1] : 0);
    rows_ok = rows_ok && rows % kExpandRows == 0 && g.H == g.W && (g.H == 1 || g.H == 2 || g.H == 4);
  }
  if (rows_ok)
    hipLaunchKernelGGL(toeplitz_expand_rows_kernel, dim3((unsigned)(b.end[b.n - 1] / kExpandRows)), dim3(256), 0, s,
                       b);
  else
    hipLaunchKernelGGL(toeplitz_expand_many_kernel, dim3((unsigned)b.end[b.n - 1]), dim3(256), 0, s, b);
}

// One thread per (co, ci) weight PAIR: it reads, for every output position (oh, ow), the
// H*W contiguous dWt_big columns of input channel ci (row n = (co, oh, ow)) — lanes with
// consecutive ci read consecutive segments, fully coalesced — and accumulates them into
// its KH*KW taps in registers (the same (oh, ow)-ascending order per tap as the one-thread-
// per-weight fold, so results are bitwise identical); then writes its KH*KW contiguous
// weights.  Toeplitz layers have KH, KW <= 3 and H*W <= 16.
constexpr int kFoldMaxTaps = 9;
__device__ __forceinline__ void fold_pair(const float* __restrict__ dwt, const ConvGeom& g, int pair,
                                          float (&acc)[kFoldMaxTaps]) {
  const int co = pair / g.C, ci = pair - co * g.C;
  const int K = g.C * g.H * g.W, HW = g.H * g.W;
#pragma unroll
  for (int t = 0; t < kFoldMaxTaps; ++t) acc[t] = 0.f;
  for (int oh = 0; oh < g.OH; ++oh)
    for (int ow = 0; ow < g.OW; ++ow) {
      const float* row = dwt + (int64_t)((co * g.OH + oh) * g.OW + ow) * K + ci * HW;
      for (int ih = 0; ih < g.H; ++ih) {
        const int kh = ih - oh * g.stride + g.pad;
        if (kh < 0 || kh >= g.KH) continue;
        for (int iw = 0; iw < g.W; ++iw) {
          const int kw = iw - ow * g.stride + g.pad;
          if (kw < 0 || kw >= g.KW) continue;
          const float v = row[ih * g.W + iw];
#pragma unroll
          for (int t = 0; t < kFoldMaxTaps; ++t)
            if (t == kh * g.KW + kw) acc[t] += v;
        }
      }
    }
}

// The same fold with the geometry at compile time (ResNet-18/34 layer3 / layer4 Toeplitz
// shapes): every tap test resolves statically and the <= OH*OW*H*W loads of a pair issue
// together instead of behind a runtime-bounded loop (the generic fold ran at 1.4 TB/s).
// Same (oh, ow, ih, iw) accumulation order per tap: bitwise equal to fold_pair.
template <int H, int W, int OH, int OW, int ST, int PD, int KH, int KW>
__device__ __forceinline__ void fold_pair_t(const float* __restrict__ dwt, int C, int pair,
                                            float (&acc)[kFoldMaxTaps]) {
  const int co = pair / C, ci = pair - co * C;
  const int64_t K = (int64_t)C * H * W;
#pragma unroll
  for (int t = 0; t < kFoldMaxTaps; ++t) acc[t] = 0.f;
  float v[OH * OW][H * W];
#pragma unroll
  for (int oh = 0; oh < OH; ++oh)
#pragma unroll
    for (int ow = 0; ow < OW; ++ow) {
      const float* row = dwt + (int64_t)((co * OH + oh) * OW + ow) * K + (int64_t)ci * (H * W);
#pragma unroll
      for (int ih = 0; ih < H; ++ih)
#pragma unroll
        for (int iw = 0; iw < W; ++iw) {
          const int kh = ih - oh * ST + PD, kw = iw - ow * ST + PD;
          v[oh * OW + ow][ih * W + iw] = (kh >= 0 && kh < KH && kw >= 0 && kw < KW) ? row[ih * W + iw] : 0.f;
        }
    }
#pragma unroll
  for (int oh = 0; oh < OH; ++oh)
#pragma unroll
    for (int ow = 0; ow < OW; ++ow)
#pragma unroll
      for (int ih = 0; ih < H; ++ih)
#pragma unroll
        for (int iw = 0; iw < W; ++iw) {
          const int kh = ih - oh * ST + PD, kw = iw - ow * ST + PD;
          if (kh >= 0 && kh < KH && kw >= 0 && kw < KW) acc[kh * KW + kw] += v[oh * OW + ow][ih * W + iw];
        }
}

__device__ __forceinline__ void fold_any(const float* __restrict__ dwt, const ConvGeom& g, int pair,
                                         float (&acc)[kFoldMaxTaps]) {
  const bool k3 = g.KH == 3 && g.KW == 3 && g.pad == 1, k1 = g.KH == 1 && g.KW == 1 && g.pad == 0;
  if (k3 && g.H == 2 && g.W == 2 && g.stride == 1) fold_pair_t<2, 2, 2, 2, 1, 1, 3, 3>(dwt, g.C, pair, acc);
  else if (k3 && g.H == 4 && g.W == 4 && g.stride == 2) fold_pair_t<4, 4, 2, 2, 2, 1, 3, 3>(dwt, g.C, pair, acc);
  else if (k1 && g.H == 4 && g.W == 4 && g.stride == 2) fold_pair_t<4, 4, 2, 2, 2, 0, 1, 1>(dwt, g.C, pair, acc);
  else if (k3 && g.H == 2 && g.W == 2 && g.stride == 2) fold_pair_t<2, 2, 1, 1, 2, 1, 3, 3>(dwt, g.C, pair, acc);
  else if (k1 && g.H == 2 && g.W == 2 && g.stride == 2) fold_pair_t<2, 2, 1, 1, 2, 0, 1, 1>(dwt, g.C, pair, acc);
  else if (k3 && g.H == 1 && g.W == 1 && g.stride == 1) fold_pair_t<1, 1, 1, 1, 1, 1, 3, 3>(dwt, g.C, pair, acc);
  else fold_pair(dwt, g, pair, acc);
}

// Every deferred grad-W fold of a backward pass in ONE launch (ops/gradfinish.py): flat
// grid over all layers' (co, ci) pairs, the layer found from the <= kMaxExpand prefix sums
// in the kernel arguments.  A workgroup's 256 pairs own one contiguous run of 256 * KH*KW
// weights, so the taps go through LDS and leave as coalesced float stores (a lane writing
// its own 9 weights would stride the wave's stores by 36 B).
__device__ __forceinline__ void fold_many_block(const FoldBatch& b, int64_t blk, float* __restrict__ stage) {
  const int64_t base = blk * 256;
  const int64_t i = base + threadIdx.x;
  const int64_t total = b.end[b.n - 1];
  int e = 0;
  while (e + 1 < b.n && base >= b.end[e]) ++e;  // the workgroup's first entry
  const int64_t e_lo = e ? b.end[e - 1] : 0;
  const bool one_entry = base + 256 <= b.end[e];  // whole workgroup inside entry e
  if (one_entry) {
    const ConvGeom& g = b.g[e];
    const int T = g.KH * g.KW;
    float acc[kFoldMaxTaps];
    fold_any(b.dwt[e], g, (int)(i - e_lo), acc);
#pragma unroll
    for (int t = 0; t < kFoldMaxTaps; ++t)
      if (t < T) stage[threadIdx.x * T + t] = acc[t];
    __syncthreads();
    float* out = b.dw[e] + (base - e_lo) * T;
    for (int k = threadIdx.x; k < 256 * T; k += 256) out[k] = stage[k];
    return;
  }
  if (i >= total) return;  // straddling workgroup: direct per-lane writes
  while (e + 1 < b.n && i >= b.end[e]) ++e;
  const ConvGeom& g = b.g[e];
  const int T = g.KH * g.KW;
  const int pair = (int)(i - (e ? b.end[e - 1] : 0));
  float acc[kFoldMaxTaps];
  fold_any(b.dwt[e], g, pair, acc);
  float* out = b.dw[e] + (int64_t)pair * T;
#pragma unroll
  for (int t = 0; t < kFoldMaxTaps; ++t)
    if (t < T) out[t] = acc[t];
}

__global__ __launch_bounds__(256) void toeplitz_fold_many_kernel(FoldBatch b) {
  __shared__ float stage[256 * kFoldMaxTaps];
  fold_many_block(b, blockIdx.x, stage);
}

void launch_toeplitz_fold_many(const FoldBatch& b, hipStream_t s) {
  if (b.n <= 0) return;
  const int64_t total = b.end[b.n - 1];  // (co, ci) pairs
  hipLaunchKernelGGL(toeplitz_fold_many_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, b);
}

void launch_toeplitz_expand(const float* w, float* wb, const ConvGeom& g, hipStream_t s) {
  const int N = g.Co * g.OH * g.OW, K = g.C * g.H * g.W;
  hipLaunchKernelGGL(toeplitz_expand_kernel, dim3((K + 255) / 256, N), dim3(256), 0, s, w, wb, g);
}

void launch_toeplitz_fold(const float* dwb, float* dw, const ConvGeom& g, hipStream_t s) {
  FoldBatch b{};
  b.dwt[0] = dwb;
  b.dw[0] = dw;
  b.g[0] = g;
  b.end[0] = (int64_t)g.Co * g.C;
  b.n = 1;
  launch_toeplitz_fold_many(b, s);
}


// =====================================================================================
// Direct (implicit-GEMM) convolutions on v_mfma_f32_32x32x2_f32 — exact f32, NCHW.
//
// ResNet-18 on 32x32 images runs its stem at 16x16 and layer1/layer2 at 8x8 / 4x4 maps
// with 64-128 channels.  MIOpen's fp32 paths for these shapes are Winograd (fwd / grad-x)
// and NHWC implicit-GEMM (grad-W) kernels that need NCHW<->NHWC transposes and zero-fill
// passes around every call (profiles/: ~1.1 ms of a 2.7 ms step).  Here each direction is
// one launch on the matrix cores, reading and writing NCHW directly:
//
// forward  Y[k, (b,p,q)] = sum_{c,r,s} W[k,c,r,s] * Xpad[b, c, p*st + r, q*st + s]
//   GEMM  M = out channels (tile BM), N = output pixels of IMGS whole images, K = C*R*S
//   chunked by CK input channels.  Per chunk the workgroup stages
//     A: W[m0:m0+BM, c0:c0+CK, :, :] transposed to [kk][m] (row stride BM+1: conflict-free
//        transposing writes and conflict-free MFMA reads),
//     B: the raw input planes x[b, c0:c0+CK] into a zero-bordered [img][c][Hp][Wp] image,
//        so the im2col operand is ONE ds_read_b32 at (per-lane pixel base + compile-time
//        tap offset): no bounds checks, no im2col buffer.
//   The two k-values of each MFMA (lane halves) are channels c and c + CK/2 at the same
//   tap, so both halves' addresses differ by a constant and every tap offset is an
//   immediate.  Global loads of chunk i+1 are issued before the MFMAs of chunk i and
//   written to the other LDS buffer after them (one barrier per chunk).
// grad-x (stride 1) is the same kernel on dY with the weight transposed and flipped
//   (TRANSW):  dX[c, (b,h,w)] = sum_{k,r,s} W[k, c, R-1-r, S-1-s] * dYpad[b, k, h + r, w + s]
//   with pad' = R-1-pad.
// grad-W   dW[k, (c,r,s)] = sum_{b,p,q} dY[b,k,p,q] * Xpad[b, c, p*st + r, q*st + s]
//   M = out channels (BM), N = (c,r,s) flattened (CB channels x R*S taps, 32-wide blocks;
//   each lane carries its (c,r,s) as an LDS base offset), K = pixels, two pixels per MFMA:
//   rows p and p + P/2.  The batch is split into slices; every slice writes its partial
//   dW tile to a slab and conv_slab_sum adds the slabs in slice order (deterministic).
// =====================================================================================

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4c __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  // D(32x32) += A(32x2) * B(2x32); lane l supplies A[l&31][l>>5] and B[l>>5][l&31];
  // D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5)
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// PSPLIT (one image per tile only): the tile covers P / PSPLIT output rows of its image
// (blockIdx.x = image * PSPLIT + row block); the whole image is still staged in LDS.  The stem at
// small per-GPU batches: one 16x16-output image per workgroup left 3/4 of the CUs idle at batch 64.
template <int R, int S, int ST, int PD, int H, int W, int CK, int BM, int IMGS, int WM, int NBUF, int KB, bool TRANSW,
          int PSPLIT = 1>
struct ConvFwdCfg {
  static constexpr int P = (H + 2 * PD - R) / ST + 1, Q = (W + 2 * PD - S) / ST + 1, PQ = P * Q;
  static_assert(PSPLIT == 1 || (IMGS == 1 && P % PSPLIT == 0), "row blocks of one image");
  // Bank-conflict-free LDS image (ds_read_b32: bank = dword % 32, one 32-lane half-wave per
  // LDS cycle; the B read of a half-wave is 32 output pixels at pixel_base + tap):
  //  * 8x8 stride 1, one image per tile: lanes cover 8 rows x 4 columns (MAP 1) of a
  //    12-wide row stride -> row offsets 12p mod 32 = {0,12,24,4,16,28,8,20}: 32 banks;
  //  * 4x4 stride 1, 2 images per half-wave: row stride 8 (4 rows x 4 columns = banks
  //    {0-3, 8-11, 16-19, 24-27}) and an image stride = 4 (mod 32) for the second image;
  //  * 8x8 stride 2, 2 images per half-wave: row stride 12 (rows 24p = {0,24,16,8} mod 32,
  //    even columns -> the 16 even banks) and an image stride = 1 (mod 32): odd banks.
  // (Measured before: 34-54 % of LDS cycles were conflict cycles, profiles/r2/pmc_counters.md.)
  //  * 32x32 stride 2 (the 7x7 stem): the even and odd columns of each padded row are stored
  //    apart (DEINT: position (col & 1) * HALF + col / 2, row stride 2 * HALF = 40), so the 16
  //    lanes of an output row read 16 CONSECUTIVE words instead of every other one, and the
  //    next output row (2 input rows = 80 words = 16 mod 32) lands on the other 16 banks
  //    (interleaved: 2-way on every B read, 47 % of LDS cycles in conflict, PMC round 4).
  static constexpr int LAYOUT = (ST == 1 && H == 8 && W == 8 && PD == 1 && IMGS == 1) ? 1
                                : (ST == 1 && H == 4 && W == 4 && IMGS % 2 == 0)      ? 2
                                : (ST == 2 && H == 8 && W == 8 && IMGS % 2 == 0)      ? 3
                                : (ST == 2 && H == 32 && W == 32 && R == 7 && IMGS == 1) ? 4
                                                                                       : 0;
  static constexpr bool DEINT = LAYOUT == 4;
  static constexpr int HALF = (W + 2 * PD + 2) / 2;  // >= every padded column's half position
  static constexpr int Hp = H + 2 * PD;
  static constexpr int Wp = LAYOUT == 1 ? 12 : LAYOUT == 2 ? 8 : LAYOUT == 3 ? 12 : DEINT ? 2 * HALF : W + 2 * PD;
  // LDS column of padded input column `col` within a row
  __device__ static __forceinline__ constexpr int cpos(int col) {
    return DEINT ? (col & 1) * HALF + (col >> 1) : col;
  }
  // channel stride odd: the B staging stores (float4 per lane -> 4 scalar ds_write_b32, a
  // 32-lane group spanning 2-8 channels) land on disjoint bank sets per channel (<= 2-way,
  // which a b32 store absorbs); the reads of a half-wave stay inside one channel
  static constexpr int HWp = (Hp * Wp) | 1, HW = H * W;
  static constexpr int IPAD0 = LAYOUT == 2 ? 4 : LAYOUT == 3 ? 1 : 0;  // target image stride mod 32
  static constexpr int IMGSTR = LAYOUT >= 2 ? (CK * HWp + 31) / 32 * 32 + IPAD0 : CK * HWp;
  static_assert(Wp >= W + 2 * PD && (!DEINT || (ST == 2 && HALF * 2 == Wp && (ST * Wp) % 32 == 16)),
                "row stride holds the zero border");
  // output pixel n of the tile -> (image, row, column)
  __device__ static __forceinline__ void pix(int n, int& img, int& p, int& q) {
    if constexpr (LAYOUT == 1) {
      img = 0;
      p = (n & 31) >> 2;
      q = (n & 3) + 4 * (n >> 5);
    } else {
      img = n / PQ;
      const int pq = n - img * PQ;
      p = pq / Q;
      q = pq - p * Q;
    }
  }
  static constexpr int RS = R * S, KK = CK * RS;
  // PAIRK (the 3-channel 7x7 stem): the two k values of an MFMA step (lane halves h = 0 / 1)
  // were channels c and c + 2 of CK = 4 (98 steps, a quarter of them on the zero 4th channel).
  // Now: steps 0-48 pair channel 0 with channel 1 at the same tap (B offset + 1 plane), steps
  // 49-55 channel 2's kernel row 3 with the zero plane (+ 1 plane), steps 56-76 channel 2's rows
  // 0-2 with its rows 4-6 (+ 4 rows): 77 steps, each half's B offset still a compile-time
  // immediate on one of two per-lane bases.  The A image is staged in the same step order.
  static constexpr bool PAIRK = DEINT && R == 7 && S == 7;
  static constexpr int NSTEP = PAIRK ? 77 : (CK / 2) * RS, NBLK = NSTEP / KB;
  static_assert(!PAIRK || (CK == 4 && 2 * NSTEP <= KK), "stem k pairing");
  // PAIRK: the (c, r, s) tap of lane half 0 at step t
  __device__ static __forceinline__ constexpr int pk_c(int t) { return t < 49 ? 0 : 2; }
  __device__ static __forceinline__ constexpr int pk_r(int t) { return t < 49 ? t / 7 : t < 56 ? 3 : (t - 56) / 7; }
  __device__ static __forceinline__ constexpr int pk_s(int t) { return t < 49 ? t % 7 : t < 56 ? t - 49 : (t - 56) % 7; }
  // PAIRK: A-image row (h * NSTEP + t) of flattened weight index kk = c * 49 + r * 7 + s, or -1
  // (kk < 147: the three real channels; branch-free, every weight of the tile is staged through it)
  __device__ static __forceinline__ int pk_row(int kk) {
    const int c = kk / 49, rem = kk - 49 * c, r = rem / 7, sc = rem - 7 * r;
    const int v2 = r == 3 ? 49 + sc : (r < 3 ? 56 + rem : NSTEP + 28 + rem);
    return c == 0 ? rem : (c == 1 ? NSTEP + rem : v2);
  }
  static constexpr int BN = IMGS * PQ / PSPLIT;
  static constexpr int WN = 4 / WM;
  static constexpr int TM = BM / 32 / WM, TN = BN / 32 / WN;
  // [kk][m] A image.  Reads (32 consecutive m) are conflict-free for any stride; the stride is
  // picked for the transposing scalar stores: forward (m fastest over 4 lanes, then kk in
  // float4 steps) LDA = 1 mod 32 -> <= 2-way; grad-x (TRANSW: 4 consecutive (m, tap) of a
  // weight row per lane) LDA = 2 mod 32 -> <= 2-way (1 mod 32 was 5-way; PMC round 3)
  static constexpr int LDA = TRANSW ? BM + 2 : BM + 1;
  // AV: [m][kk] A image instead (kk contiguous, row stride LDAM with LDAM / 4 odd: the 16 rows
  // of a ds_read_b128 phase start in disjoint 4-bank groups).  Lane half h consumes kk =
  // h * NSTEP + t at MFMA step t, so KB consecutive steps are KB / 4 ds_read_b128 per tile
  // instead of KB ds_read_b32 (each of which the MFMA chain waited on), and the forward's
  // float4 weight loads land as one ds_write_b128.  Needs KB % 4 == 0 and NSTEP % 4 == 0
  // (every 8x8 / 4x4 layer config; the 7x7 stem keeps [kk][m]).
  static constexpr bool AV = KB % 4 == 0 && ((CK / 2) * RS) % 4 == 0;
  static constexpr int LDAM = KK + (((KK / 4) % 2 == 0) ? 4 : 8);
  static constexpr int A_SZ = AV ? BM * LDAM : KK * LDA;
  static constexpr int B_SZ = IMGS * IMGSTR;
  // A staging: float4 rows when every chunk is whole channels and rows are 16-B aligned
  static constexpr int B4 = IMGS * CK * HW / 4, B_PER_T = (B4 + 255) / 256;
  static constexpr size_t LDS_BYTES = (size_t)NBUF * (A_SZ + B_SZ) * sizeof(float);
  static_assert(CK % 2 == 0 && BM % (32 * WM) == 0 && BN % (32 * WN) == 0 && TM >= 1 && TN >= 1, "tile");
  static_assert(NSTEP % KB == 0, "operand prefetch blocks");
  static_assert((W % 4 == 0 || (PD == 0 && H * W == 4)) && BM % 4 == 0, "float4 staging");
  // BatchNorm statistics epilogue (conv_fwd_kernel `stats`): the [BM][BN + 4] output tile
  // fits in the LDS the main loop used, 256 / BM threads per channel, float4 reads
  static constexpr int STATS_LDO = BN + 4, STATS_TPC = 256 / BM;
  static constexpr bool STATS_OK = 256 % BM == 0 && BN % (4 * STATS_TPC) == 0 &&
                                   (size_t)BM * STATS_LDO <= (size_t)NBUF * (A_SZ + B_SZ);
  // backward mode keeps two such tiles (dz and dz * xhat)
  static constexpr bool STATS2_OK = STATS_OK && (size_t)2 * BM * STATS_LDO <= (size_t)NBUF * (A_SZ + B_SZ);
};

// A (weights) is read straight from W: forward rows W[m][c0:c0+CK][:] (CK*RS contiguous
// floats), grad-x rows W[c][m0:m0+BM][:] (BM*RS contiguous) with the taps flipped; both are
// written transposed into the [kk][m] LDS image.  VEC=1 needs Cin % CK == 0 (float4 over
// whole channels); the stem (Cin = 3 < CK) stages scalars.
// SCH (instruction scheduling of the MFMA block, benchmarking variants): 0 = compiler default,
// 1 = __builtin_amdgcn_iglp_opt(0), 2 = pinned interleave of one MFMA and one LDS read (the
// default schedule waits on each operand read right before its MFMA: exposed LDS latency
// at 1-2 waves per SIMD)
// IUPS = 2 (grad-x of the 3x3 stride-2 conv): the input is a (H/2) x (W/2) map staged onto
// the even pixels of the H x W LDS image (the odd ones keep the zero fill), i.e. the stride-1
// correlation of the zero-inserted dY with the flipped weights:
//   dX[c, h, w] = sum_{k,r,s} W[k, c, 2-r, 2-s] * Z[k, h-1+r, w-1+s],  Z[k, 2p, 2q] = dY[k, p, q]

// (a device function of the workgroup's grid coordinates: the downsample-conv backward pairs run it
// on one part of a combined grid, launch_conv_dgrad)
template <int R, int S, int ST, int PD, int H, int W, int CK, int BM, int IMGS, int WM, int NBUF, int KB, bool TRANSW,
          bool VEC, int UPS = 1, int SCH = 0, int IUPS = 1, int PSPLIT = 1>
__device__ __forceinline__ void conv_fwd_body(const float* __restrict__ x, const float* __restrict__ w,
                                              float* __restrict__ y, float* __restrict__ part, int Cin, int Kout,
                                              int cps, int64_t slab, const float* __restrict__ addend,
                                              const ConvBnStats& st, const uint3 bid, const uint3 gdim,
                                              float* __restrict__ smem) {
  using G = ConvFwdCfg<R, S, ST, PD, H, W, CK, BM, IMGS, WM, NBUF, KB, TRANSW, PSPLIT>;
  constexpr int AE = (BM * G::KK + 3) / 4;  // float4 slots (scalar path: 4 scalars per slot)
  constexpr int A_PER_T = (AE + 255) / 256;
  float* As = smem;
  float* Bs = smem + NBUF * G::A_SZ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int h = lane >> 5, l32 = lane & 31;
  const int m0 = bid.y * BM;
  const int b0 = (PSPLIT == 1 ? bid.x : bid.x / PSPLIT) * IMGS;
  const int prow0 = PSPLIT == 1 ? 0 : (bid.x % PSPLIT) * (G::P / PSPLIT);  // first output row
  // split-K: workgroup z reduces channel chunks [ch0, ch0 + nchunks) into output slab z
  const int ch0 = bid.z * cps;
  const int nchunks = min((Cin + CK - 1) / CK - ch0, cps);

  for (int i = tid; i < NBUF * G::B_SZ; i += 256) Bs[i] = 0.f;  // zero borders (never rewritten)

  int a_base[G::TM], b_base[G::TN], b_base2[G::PAIRK ? G::TN : 1];
#pragma unroll
  for (int tm = 0; tm < G::TM; ++tm)
    a_base[tm] = G::AV ? ((wm * G::TM + tm) * 32 + l32) * G::LDAM + h * G::NSTEP
                       : h * G::NSTEP * G::LDA + (wm * G::TM + tm) * 32 + l32;
#pragma unroll
  for (int tn = 0; tn < G::TN; ++tn) {
    const int n = (wn * G::TN + tn) * 32 + l32;
    int img, p, q;
    G::pix(n, img, p, q);
    p += prow0;
    b_base[tn] = img * G::IMGSTR + (G::PAIRK ? h : h * (CK / 2)) * G::HWp + p * ST * G::Wp + (G::DEINT ? q : q * ST);
    if constexpr (G::PAIRK) b_base2[tn] = b_base[tn] - h * G::HWp + h * 4 * G::Wp;
  }

  // B staging: float4 of the (possibly half-size, IUPS) input planes
  constexpr int IW = W / IUPS, IHW = (H / IUPS) * IW;
  constexpr int B4I = IMGS * CK * IHW / 4, BPT = (B4I + 255) / 256;
  // a 2x2 unpadded plane is one float4 stored whole (row stride Wp = W = 2)
  static_assert((IW % 4 == 0 || (PD == 0 && IUPS == 1 && IHW == 4)) && (IUPS == 1 || (ST == 1 && UPS == 1)),
                "input staging");
  // PAIRK stem: the BM x 147 weights of the tile are one contiguous run (Cin = 3): float4 loads
  // of the flat run, scattered to the paired-step rows at the LDS store (the generic scalar path
  // computed and held a 64-bit address and a branch per weight: 400+ registers, 1 wave / SIMD)
  constexpr int PKE = G::PAIRK ? BM * 3 * G::RS / 4 : 1, PK_PER_T = (PKE + 255) / 256;
  static_assert(!G::PAIRK || (BM * 3 * G::RS) % 4 == 0, "stem weight run in float4");
  f32x4c ra[A_PER_T > PK_PER_T ? A_PER_T : PK_PER_T];
  f32x4c rb[BPT];
  auto load = [&](int ch) {
    const int c0 = (ch0 + ch) * CK;
    if constexpr (G::PAIRK) {
      // (staged straight from global in store(): no register copy of the weights)
    } else
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int e = tid + 256 * i;
      f32x4c v = {0.f, 0.f, 0.f, 0.f};
      if (e < AE) {
        if (VEC) {
          if (!TRANSW) {  // lanes: 4 rows (m) fastest, then float4 k4 along the row
            const int r = e >> 2, k4 = r % (G::KK / 4), m = 4 * (r / (G::KK / 4)) + (e & 3);
            v = *reinterpret_cast<const f32x4c*>(w + ((int64_t)(m0 + m) * Cin + c0) * G::RS + 4 * k4);
          } else {
            const int c = e / (BM * G::RS / 4), r4 = e - c * (BM * G::RS / 4);
            v = *reinterpret_cast<const f32x4c*>(w + ((int64_t)(c0 + c) * Kout + m0) * G::RS + 4 * r4);
          }
        } else {  // forward only (stem): 4 scalars, zero past Cin
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int f = 4 * e + j, m = f / G::KK, kk = f - m * G::KK;
            if (f < BM * G::KK && c0 + kk / G::RS < Cin) v[j] = w[((int64_t)(m0 + m) * Cin + c0) * G::RS + kk];
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = tid + 256 * i;  // float4 index within the IMGS x CK x (input plane) block
      f32x4c v = {0.f, 0.f, 0.f, 0.f};
      if (e < B4I) {
        const int img = e / (CK * IHW / 4), rem4 = e - img * (CK * IHW / 4);
        const int c = (4 * rem4) / IHW;
        if (c0 + c < Cin)
          v = *reinterpret_cast<const f32x4c*>(x + ((int64_t)(b0 + img) * Cin + c0) * IHW + 4 * rem4);
      }
      rb[i] = v;
    }
  };
  auto store = [&](int buf) {
    float* A = As + buf * G::A_SZ;
    float* B = Bs + buf * G::B_SZ;
    if constexpr (G::PAIRK) {
      const f32x4c* w4 = reinterpret_cast<const f32x4c*>(w + (int64_t)m0 * 3 * G::RS);
      for (int e = tid; e < PKE; e += 256) {
        const f32x4c v = w4[e];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int f = 4 * e + j, m = f / (3 * G::RS), kk = f - m * (3 * G::RS);
          A[G::pk_row(kk) * G::LDA + m] = v[j];
        }
      }
      for (int idx = tid; idx < 7 * BM; idx += 256)  // the zero partners of channel 2's row 3
        A[(G::NSTEP + 49 + idx / BM) * G::LDA + idx % BM] = 0.f;
    } else
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int e = tid + 256 * i;
      if (e < AE) {
        if (VEC) {
          if (!TRANSW) {
            const int r = e >> 2, k4 = r % (G::KK / 4), m = 4 * (r / (G::KK / 4)) + (e & 3);
            if constexpr (G::AV) {
              *reinterpret_cast<f32x4c*>(A + m * G::LDAM + 4 * k4) = ra[i];
            } else {
              float* d = A + 4 * k4 * G::LDA + m;
              d[0] = ra[i].x; d[G::LDA] = ra[i].y; d[2 * G::LDA] = ra[i].z; d[3 * G::LDA] = ra[i].w;
            }
          } else {
            const int c = e / (BM * G::RS / 4), f = 4 * (e - c * (BM * G::RS / 4));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int m = (f + j) / G::RS, rs = (f + j) - m * G::RS;
              const int kk = c * G::RS + (G::RS - 1 - rs);  // flip the taps
              if constexpr (G::AV) A[m * G::LDAM + kk] = ra[i][j];
              else A[kk * G::LDA + m] = ra[i][j];
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int f = 4 * e + j, m = f / G::KK, kk = f - m * G::KK;
            if (f < BM * G::KK) {
              if constexpr (G::PAIRK) {
                const int row = G::pk_row(kk);
                if (row >= 0) A[row * G::LDA + m] = ra[i][j];
              } else if constexpr (G::AV) {
                A[m * G::LDAM + kk] = ra[i][j];
              } else {
                A[kk * G::LDA + m] = ra[i][j];
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int e = tid + 256 * i;
      if (e < B4I) {
        const int img = e / (CK * IHW / 4), rem = 4 * (e - img * (CK * IHW / 4));
        const int c = rem / IHW, hw = rem - c * IHW;
        const int hh = hw / IW, ww = hw - hh * IW;
        if constexpr (G::DEINT) {
          float* d = B + img * G::IMGSTR + c * G::HWp + (hh + PD) * G::Wp;
#pragma unroll
          for (int j = 0; j < 4; ++j) d[G::cpos(ww + PD + j)] = rb[i][j];
        } else {
          float* d = B + img * G::IMGSTR + c * G::HWp + (IUPS * hh + PD) * G::Wp + IUPS * ww + PD;
          d[0] = rb[i].x; d[IUPS] = rb[i].y; d[2 * IUPS] = rb[i].z; d[3 * IUPS] = rb[i].w;
        }
      }
    }
  };

  f32x16 acc[G::TM][G::TN];
#pragma unroll
  for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  load(0);
  __syncthreads();  // zero fill before interior writes
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const int cur = (NBUF == 2) ? (ch & 1) : 0;
    if (NBUF == 2 && ch + 1 < nchunks) load(ch + 1);
    const float* A = As + cur * G::A_SZ;
    const float* B = Bs + cur * G::B_SZ;
    // operands of block k+1 are read from LDS while the MFMAs of block k issue
    float av[2][KB][G::TM], bv[2][KB][G::TN];
    auto fetch = [&](int blk, int slot) {
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int t = blk * KB + i;
        int c = t / G::RS, rs = t - c * G::RS, r = rs / S, s = rs - r * S;
        if constexpr (G::PAIRK) {
          c = G::pk_c(t);
          r = G::pk_r(t);
          s = G::pk_s(t);
        }
        const int offb = c * G::HWp + r * G::Wp + (G::DEINT ? (s & 1) * G::HALF + (s >> 1) : s);
        if constexpr (!G::AV) {
#pragma unroll
          for (int tm = 0; tm < G::TM; ++tm) av[slot][i][tm] = A[a_base[tm] + t * G::LDA];
        }
#pragma unroll
        for (int tn = 0; tn < G::TN; ++tn) {
          if constexpr (G::PAIRK) bv[slot][i][tn] = B[(t < 56 ? b_base[tn] : b_base2[tn]) + offb];
          else bv[slot][i][tn] = B[b_base[tn] + offb];
        }
      }
      if constexpr (G::AV) {
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
          for (int q = 0; q < KB / 4; ++q) {
            const f32x4c v = *reinterpret_cast<const f32x4c*>(A + a_base[tm] + blk * KB + 4 * q);
#pragma unroll
            for (int j = 0; j < 4; ++j) av[slot][4 * q + j][tm] = v[j];
          }
      }
    };
    if constexpr (SCH == 1) __builtin_amdgcn_iglp_opt(0);
    fetch(0, 0);
#pragma unroll
    for (int blk = 0; blk < G::NBLK; ++blk) {
      if (blk + 1 < G::NBLK) fetch(blk + 1, (blk + 1) & 1);
#pragma unroll
      for (int i = 0; i < KB; ++i)
#pragma unroll
        for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < G::TN; ++tn)
            acc[tm][tn] = mfma32(av[blk & 1][i][tm], bv[blk & 1][i][tn], acc[tm][tn]);
    }
    if constexpr (SCH == 2) {
#pragma unroll
      for (int i = 0; i < G::NSTEP * G::TM * G::TN; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
      }
    }
    if (ch + 1 < nchunks) {
      if (NBUF == 2) {
        store(cur ^ 1);
      } else {
        __syncthreads();  // everyone done reading the single buffer
        load(ch + 1);
        store(0);
      }
    }
    __syncthreads();
  }

  // split-K (gridDim.z > 1): every workgroup stores its partial tile to its slab of `part`
  // (compact [B][Kout][PQ] layout); conv_slab_sum(_ups) adds the slabs in z order
  // (deterministic).  A last-arrival fixup inside this kernel was measured 4x slower: the
  // agent-scope release fence writes the XCD's L2 back and the fixing workgroup re-reads
  // the other XCDs' slabs from HBM on a serial dependency chain.
  if (gdim.z > 1) {
    float* pz = part + (int64_t)bid.z * slab;
#pragma unroll
    for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < G::TN; ++tn) {
        const int n = (wn * G::TN + tn) * 32 + l32;
        int img, p, q;
        G::pix(n, img, p, q);
        p += prow0;
        float* pb = pz + (int64_t)(b0 + img) * Kout * G::PQ + p * G::Q + q;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * G::TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          pb[(int64_t)m * G::PQ] = acc[tm][tn][r];
        }
      }
    return;
  }

  // UPS = 2 (grad-x of a 1x1 stride-2 conv): the result lands on the even pixels of a
  // (2P) x (2Q) plane and the three odd neighbours of each are written as zeros
  constexpr int OPQ = G::PQ * UPS * UPS;
  // BatchNorm partial sums (st.out, see ConvBnStats): unsplit, statistics-capable tiles only.
  // The two per-element quantities go through the LDS the main loop no longer reads (its last
  // iteration ended on a barrier) as [BM][BN + 4] tiles: row writes of 32 consecutive pixels
  // per half-wave, float4 row reads in the reduction below.
  constexpr bool kStats = G::STATS_OK && UPS == 1;
  const bool stats = kStats && st.out != nullptr;
  const bool bstats = G::STATS2_OK && stats && st.bx != nullptr;
  float* L = smem;
  float* L2 = smem + BM * G::STATS_LDO;
#pragma unroll
  for (int tm = 0; tm < G::TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < G::TN; ++tn) {
      const int n = (wn * G::TN + tn) * 32 + l32;
      int img, pp, qq;
      G::pix(n, img, pp, qq);
      pp += prow0;
      const int opix = UPS == 1 ? pp * G::Q + qq : pp * UPS * (UPS * G::Q) + qq * UPS;
      const int64_t yoff = (int64_t)(b0 + img) * Kout * OPQ + opix;
      float* yb = y + yoff;
      // addend (UPS == 1 only): y += addend, e.g. the identity-branch gradient of a residual
      // block added into conv1's grad-x (no separate add launch).  All 16 addends are loaded
      // under ONE uniform branch before any store: a per-element `addend ? acc + addend[o]`
      // compiled to 16 serial load + s_waitcnt vmcnt(0) round trips.
      // UPS == 2: the three odd neighbours of each written pixel carry the addend alone
      float ad[16], ad1[UPS == 2 ? 16 : 1], ad2[UPS == 2 ? 16 : 1], ad3[UPS == 2 ? 16 : 1];
      if (addend != nullptr) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * G::TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float* ap = addend + yoff + (int64_t)m * OPQ;
          ad[r] = ap[0];
          if constexpr (UPS == 2) {
            ad1[r] = ap[1];
            ad2[r] = ap[2 * G::Q];
            ad3[r] = ap[2 * G::Q + 1];
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          ad[r] = 0.f;
          if constexpr (UPS == 2) ad1[r] = ad2[r] = ad3[r] = 0.f;
        }
      }
      float bxv[16], byv[16], bmu[16], bis[16];  // backward statistics operands, same rule
      if (kStats && bstats) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * G::TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          bxv[r] = st.bx[yoff + (int64_t)m * OPQ];
          byv[r] = st.by[yoff + (int64_t)m * OPQ];
          bmu[r] = st.mean[m];
          bis[r] = st.invstd[m];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mloc = (wm * G::TM + tm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int m = m0 + mloc;
        float* d = yb + (int64_t)m * OPQ;
        const float v = acc[tm][tn][r] + ad[r];
        d[0] = v;
        if constexpr (UPS == 2) {
          d[1] = ad1[r];
          d[2 * G::Q] = ad2[r];
          d[2 * G::Q + 1] = ad3[r];
        }
        if constexpr (kStats) {
          if (bstats) {
            const float dz = byv[r] > 0.f ? v : 0.f;
            L[mloc * G::STATS_LDO + n] = dz;
            L2[mloc * G::STATS_LDO + n] = dz * ((bxv[r] - bmu[r]) * bis[r]);
          } else if (stats) {
            L[mloc * G::STATS_LDO + n] = v;
          }
        }
      }
    }

  // Per output channel, fp32 over 4 values then fp64, stored to st.out[(c * S + s) * 2 + {0, 1}]
  // with s = blockIdx.x of S = gridDim.x: the [c][s][2] slice-partial layout the BN kernels fold
  // in a fixed order, so the BN runs no statistics pass (one launch and one full read fewer).
  if constexpr (kStats) {
    if (stats) {
      __syncthreads();
      constexpr int TPC = G::STATS_TPC, NPT = G::BN / TPC;
      const int c = tid / TPC, j = tid - c * TPC;
      const float* src = L + c * G::STATS_LDO + j * NPT;
      const float* src2 = L2 + c * G::STATS_LDO + j * NPT;
      double sum = 0.0, sq = 0.0;
#pragma unroll 4
      for (int i = 0; i < NPT; i += 4) {
        const f32x4c v = *reinterpret_cast<const f32x4c*>(src + i);
        sum += (double)((v.x + v.y) + (v.z + v.w));
        if (bstats) {
          const f32x4c u = *reinterpret_cast<const f32x4c*>(src2 + i);
          sq += (double)((u.x + u.y) + (u.z + u.w));
        } else {
          sq += (double)((v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w));
        }
      }
#pragma unroll
      for (int o = 1; o < TPC; o <<= 1) {
        sum += __shfl_xor(sum, o, 64);
        sq += __shfl_xor(sq, o, 64);
      }
      if (j == 0) {
        double* d = st.out + ((int64_t)(m0 + c) * gdim.x + bid.x) * 2;
        d[0] = sum;
        d[1] = sq;
      }
    }
  }
}

template <int R, int S, int ST, int PD, int H, int W, int CK, int BM, int IMGS, int WM, int NBUF, int KB, bool TRANSW,
          bool VEC, int UPS = 1, int SCH = 0, int IUPS = 1, int PSPLIT = 1>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       float* __restrict__ y, float* __restrict__ part, int Cin,
                                                       int Kout, int cps, int64_t slab,
                                                       const float* __restrict__ addend, ConvBnStats st) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  conv_fwd_body<R, S, ST, PD, H, W, CK, BM, IMGS, WM, NBUF, KB, TRANSW, VEC, UPS, SCH, IUPS, PSPLIT>(
      x, w, y, part, Cin, Kout, cps, slab, addend, st, make_uint3(blockIdx.x, blockIdx.y, blockIdx.z),
      make_uint3(gridDim.x, gridDim.y, gridDim.z), smem);
}

// ---- grad-W -----------------------------------------------------------------------------
template <int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
struct ConvWgCfg {
  static constexpr int P = (H + 2 * PD - R) / ST + 1, Q = (W + 2 * PD - S) / ST + 1, PQ = P * Q;
  // odd channel stride + tap-major columns (TAPMAJ: column j = rs * CB + c, so the 32 lanes of
  // a B read are 32 channels at one tap): conflict-free B reads.  Channel-major (c * RS + rs)
  // put 3-4 channels' 3x3 windows in one half-wave: 2-3-way conflicts (PMC round 3), and the
  // even 8x8 1x1 stride was 32-way.
  static constexpr int Hp = H + 2 * PD, Wp = W + 2 * PD, HWp = (Hp * Wp) | 1, HW = H * W;
  static constexpr int RS = R * S, J = CB * RS, JB = (J + 31) / 32, MB = BM / 32;
  static constexpr bool TAPMAJ = CB % 32 == 0;
  __device__ static __forceinline__ void col(int j, int& c, int& rs) {
    if constexpr (TAPMAJ) {
      rs = j / CB;
      c = j - rs * CB;
    } else {
      c = j / RS;
      rs = j - c * RS;
    }
  }
  static constexpr int NSTEP = PQ / 2, NBLK = NSTEP / KB;
  // AVW: the dY row of a lane is read KB pixels at a time (ds_read_b128) — LDY / 4 odd, so
  // the 16 rows of a b128 phase start in disjoint 4-bank groups; else LDY odd for b32 reads
  static constexpr bool AVW = KB % 4 == 0 && (PQ / 2) % 4 == 0;
  static constexpr int LDY = AVW ? PQ + (((PQ / 4) % 2 == 0) ? 4 : 8) : PQ + 1;
  static constexpr int A_SZ = BM * LDY;  // dY tile of one image: [m][pixel]
  static constexpr int B_SZ = CB * HWp;  // zero-bordered x planes of one image
  static constexpr int NT = 64 * NW;
  static constexpr int A4 = BM * PQ / 4, B4 = CB * HW / 4;
  static constexpr int A_PER_T = (A4 + NT - 1) / NT, B_PER_T = (B4 + NT - 1) / NT;
  // TAPMAJ epilogue: the dW tile goes through LDS back to channel-major rows ([BM][J], row
  // stride LDJ, 16-B aligned) so the slab stores stay contiguous float4 (a lane-per-channel
  // store at stride RS scattered every row over RS x 128 B and doubled the write bytes)
  static constexpr int LDJ = J + 4;
  static constexpr size_t MAIN_BYTES = 2 * (size_t)(A_SZ + B_SZ) * sizeof(float);
  static constexpr size_t EPI_BYTES = TAPMAJ ? (size_t)BM * LDJ * sizeof(float) : 0;
  static constexpr size_t LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  static_assert(MB * JB == NW * NBPW, "every wave owns NBPW 32x32 blocks");
  static_assert(P % 2 == 0 && PQ % 4 == 0 && HW % 4 == 0 && NSTEP % KB == 0, "pixel pairing / float4 loads");
};

// (a device function of the workgroup's grid coordinates: the layer2 backward pairs run it on
// one part of a combined grid, launch_conv_dgrad)
template <int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
__device__ __forceinline__ void conv_wgrad_body(const float* __restrict__ x, const float* __restrict__ dy,
                                                float* __restrict__ part, int Cin, int Kout, int imgs_per_slice,
                                                const uint3 bid, float* __restrict__ smem) {
  using G = ConvWgCfg<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  float* As = smem;                 // [2][A_SZ]
  float* Bs = smem + 2 * G::A_SZ;   // [2][B_SZ]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int slice = bid.x, m0 = bid.y * BM, c0 = bid.z * CB;
  const int bb = slice * imgs_per_slice;

  for (int i = tid; i < 2 * G::B_SZ; i += G::NT) Bs[i] = 0.f;

  int a_base[NBPW], b_base[NBPW];
#pragma unroll
  for (int t = 0; t < NBPW; ++t) {
    const int blk = wave * NBPW + t;
    const int mb = blk / G::JB, jb = blk - mb * G::JB;
    const int j = jb * 32 + l32;
    a_base[t] = (mb * 32 + l32) * G::LDY + h * (G::PQ / 2);
    int c, rs;
    G::col(j, c, rs);
    const int r = rs / S, s = rs - r * S;
    b_base[t] = (j < G::J) ? c * G::HWp + r * G::Wp + s + h * (G::P / 2) * ST * G::Wp : 0;
  }

  f32x4c ra[G::A_PER_T], rb[G::B_PER_T];
  auto load = [&](int b) {
#pragma unroll
    for (int i = 0; i < G::A_PER_T; ++i) {
      const int e = tid + G::NT * i;
      f32x4c v = {0.f, 0.f, 0.f, 0.f};
      if (e < G::A4) v = *reinterpret_cast<const f32x4c*>(dy + ((int64_t)b * Kout + m0) * G::PQ + 4 * e);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < G::B_PER_T; ++i) {
      const int e = tid + G::NT * i;
      f32x4c v = {0.f, 0.f, 0.f, 0.f};
      if (e < G::B4 && c0 + (4 * e) / G::HW < Cin)
        v = *reinterpret_cast<const f32x4c*>(x + ((int64_t)b * Cin + c0) * G::HW + 4 * e);
      rb[i] = v;
    }
  };
  auto store = [&](int buf) {
    float* A = As + buf * G::A_SZ;
    float* B = Bs + buf * G::B_SZ;
#pragma unroll
    for (int i = 0; i < G::A_PER_T; ++i) {
      const int e = tid + G::NT * i;
      if (e < G::A4) {
        const int m = (4 * e) / G::PQ, pq = 4 * e - m * G::PQ;
        float* d = A + m * G::LDY + pq;
        if constexpr (G::AVW) {
          *reinterpret_cast<f32x4c*>(d) = ra[i];
        } else {
          d[0] = ra[i].x; d[1] = ra[i].y; d[2] = ra[i].z; d[3] = ra[i].w;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < G::B_PER_T; ++i) {
      const int e = tid + G::NT * i;
      if (e < G::B4) {
        const int c = (4 * e) / G::HW, hw = 4 * e - c * G::HW;
        const int hh = hw / W, ww = hw - hh * W;
        float* d = B + c * G::HWp + (hh + PD) * G::Wp + ww + PD;
        d[0] = rb[i].x; d[1] = rb[i].y; d[2] = rb[i].z; d[3] = rb[i].w;
      }
    }
  };

  f32x16 acc[NBPW];
#pragma unroll
  for (int t = 0; t < NBPW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  load(bb);
  __syncthreads();
  store(0);
  __syncthreads();
  for (int i = 0; i < imgs_per_slice; ++i) {
    const int cur = i & 1;
    if (i + 1 < imgs_per_slice) load(bb + i + 1);
    const float* A = As + cur * G::A_SZ;
    const float* B = Bs + cur * G::B_SZ;
    float av[2][KB][NBPW], bv[2][KB][NBPW];
    auto fetch = [&](int blk, int slot) {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const int t = blk * KB + k;
        const int p = t / G::Q, q = t - p * G::Q;
#pragma unroll
        for (int u = 0; u < NBPW; ++u) {
          if constexpr (!G::AVW) av[slot][k][u] = A[a_base[u] + t];
          bv[slot][k][u] = B[b_base[u] + p * ST * G::Wp + q * ST];
        }
      }
      if constexpr (G::AVW) {
#pragma unroll
        for (int u = 0; u < NBPW; ++u)
#pragma unroll
          for (int q4 = 0; q4 < KB / 4; ++q4) {
            const f32x4c v = *reinterpret_cast<const f32x4c*>(A + a_base[u] + blk * KB + 4 * q4);
#pragma unroll
            for (int j = 0; j < 4; ++j) av[slot][4 * q4 + j][u] = v[j];
          }
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int blk = 0; blk < G::NBLK; ++blk) {
      if (blk + 1 < G::NBLK) fetch(blk + 1, (blk + 1) & 1);
#pragma unroll
      for (int k = 0; k < KB; ++k)
#pragma unroll
        for (int u = 0; u < NBPW; ++u) acc[u] = mfma32(av[blk & 1][k][u], bv[blk & 1][k][u], acc[u]);
    }
    if (i + 1 < imgs_per_slice) store(cur ^ 1);
    __syncthreads();
  }

  float* out = part + (int64_t)slice * Kout * Cin * G::RS;
  if constexpr (G::TAPMAJ && G::RS > 1) {
    // the loop's last barrier retired every LDS read: reuse the buffers as the staging tile
    float* st = smem;
#pragma unroll
    for (int t = 0; t < NBPW; ++t) {
      const int blk = wave * NBPW + t;
      const int mb = blk / G::JB, jb = blk - mb * G::JB;
      const int j = jb * 32 + l32;
      int c, rs;
      G::col(j, c, rs);
      if (j < G::J) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          st[(mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * G::LDJ + c * G::RS + rs] = acc[t][r];
      }
    }
    __syncthreads();
    const int lim = min(CB, Cin - c0) * G::RS;  // valid columns of a row (partial channel block)
    constexpr int J4 = G::J / 4;
    static_assert(G::J % 4 == 0, "float4 rows");
    for (int i = tid; i < BM * J4; i += G::NT) {
      const int mr = i / J4, q = 4 * (i - mr * J4);
      const f32x4c v = *reinterpret_cast<const f32x4c*>(st + mr * G::LDJ + q);
      float* o = out + ((int64_t)(m0 + mr) * Cin + c0) * G::RS + q;
      if (q + 3 < lim) {
        *reinterpret_cast<f32x4c*>(o) = v;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (q + k < lim) o[k] = v[k];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NBPW; ++t) {
    const int blk = wave * NBPW + t;
    const int mb = blk / G::JB, jb = blk - mb * G::JB;
    const int j = jb * 32 + l32;
    int c, rs;
    G::col(j, c, rs);
    if (j < G::J && c0 + c < Cin) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        out[((int64_t)m * Cin + c0 + c) * G::RS + rs] = acc[t][r];
      }
    }
  }
}

template <int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
__global__ __launch_bounds__(64 * NW) void conv_wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                             float* __restrict__ part, int Cin, int Kout,
                                                             int imgs_per_slice) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  conv_wgrad_body<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>(x, dy, part, Cin, Kout, imgs_per_slice,
                                                           make_uint3(blockIdx.x, blockIdx.y, blockIdx.z), smem);
}

// A layer2 backward pair in ONE launch: workgroups [0, n_dgrad) run the Winograd grad-x
// (wino_dpp.h; 4x4 maps, or the 3x3/2 conv's zero-inserted 8x8 dY), the rest the direct grad-W of
// the same conv (64 NW threads: the surplus wave leaves before any barrier, which then waits for
// the live waves only).  Both read only dY / x / the weights and write disjoint outputs.
template <int WH, int IUPS, int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
__global__ __launch_bounds__(256, 2) void wino_direct_pair_kernel(WinoConvArgs A, uint3 ga, const float* __restrict__ x,
                                                                  const float* __restrict__ dy, float* __restrict__ part,
                                                                  int Cin, int Kout, int imgs, uint3 gw) {
  static_assert(NW <= 4, "grad-W workgroup within the pair's 256 threads");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const unsigned na = ga.x * ga.y * ga.z;
  unsigned b = blockIdx.x;
  if (b < na) {
    wino_dpp_body<WH, IUPS>(A, make_uint3(b % ga.x, (b / ga.x) % ga.y, b / (ga.x * ga.y)), ga, smem);
  } else {
    if (threadIdx.x >= 64 * NW) return;
    b -= na;
    conv_wgrad_body<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>(
        x, dy, part, Cin, Kout, imgs, make_uint3(b % gw.x, (b / gw.x) % gw.y, b / (gw.x * gw.y)), smem);
  }
}

// dw[i] = sum_{s < n_slices} part[s * n + i], n % 4 == 0.  A workgroup owns 16 float4
// columns x 16 slice groups: thread (g, col) sums slices g, g+16, ... of its column, then
// group 0 adds the 16 group sums in order — a fixed summation tree (deterministic) with
// 16x the memory-level parallelism of a one-thread-per-column sum.
__global__ __launch_bounds__(256) void conv_slab_sum_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                            int64_t n, int n_slices,
                                                            const float* __restrict__ addend = nullptr) {
  __shared__ f32x4c red[16][16];
  const int col = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t i4 = ((int64_t)blockIdx.x * 16 + col) * 4;
  f32x4c acc = {0.f, 0.f, 0.f, 0.f};
  if (i4 < n) {
#pragma unroll 4
    for (int s = g; s < n_slices; s += 16) acc += *reinterpret_cast<const f32x4c*>(part + (int64_t)s * n + i4);
  }
  red[g][col] = acc;
  __syncthreads();
  if (g == 0 && i4 < n) {
    f32x4c t = red[0][col];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][col];
    if (addend) t += *reinterpret_cast<const f32x4c*>(addend + i4);  // fused residual-branch gradient
    *reinterpret_cast<f32x4c*>(dw + i4) = t;
  }
}

// Every deferred grad-W slab sum of a backward pass in ONE launch (ops/gradfinish.py):
// entry e owns blocks [end[e-1], end[e]); inside an entry the same 16-group fixed-order
// tree as conv_slab_sum_kernel (bitwise identical results).
__device__ __forceinline__ void slab_sum_many_block(const SlabBatch& b, int64_t blk, f32x4c (*red)[16]) {
  int e = 0;
  while (e + 1 < b.n && blk >= b.end[e]) ++e;
  const int64_t lb = blk - (e ? b.end[e - 1] : 0);
  const float* part = b.part[e];
  const int64_t n = b.numel[e];
  const int n_slices = b.slices[e];
  const int col = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int64_t i4 = (lb * 16 + col) * 4;
  f32x4c acc = {0.f, 0.f, 0.f, 0.f};
  if (i4 < n) {
#pragma unroll 4
    for (int sl = g; sl < n_slices; sl += 16) {
      if (b.nt) acc += __builtin_nontemporal_load(reinterpret_cast<const f32x4c*>(part + (int64_t)sl * n + i4));
      else acc += *reinterpret_cast<const f32x4c*>(part + (int64_t)sl * n + i4);
    }
  }
  red[g][col] = acc;
  __syncthreads();
  if (g == 0 && i4 < n) {
    f32x4c t = red[0][col];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][col];
    *reinterpret_cast<f32x4c*>(b.dw[e] + i4) = t;
  }
}

__global__ __launch_bounds__(256) void conv_slab_sum_many_kernel(SlabBatch b) {
  __shared__ f32x4c red[16][16];
  slab_sum_many_block(b, blockIdx.x, red);
}

// The end-of-backward grad-W finish in ONE launch: blocks [0, slab blocks) run the slab sums,
// the rest the Toeplitz folds (the two lists touch disjoint gradients).  Same per-block
// bodies as the two kernels above, so the results are bitwise identical to them.
__global__ __launch_bounds__(256) void gradw_finish_kernel(SlabBatch sb, FoldBatch fb) {
  constexpr int kFloats = 256 * kFoldMaxTaps > 16 * 16 * 4 ? 256 * kFoldMaxTaps : 16 * 16 * 4;
  __shared__ __attribute__((aligned(16))) float smem[kFloats];
  const int64_t n_slab = sb.n > 0 ? sb.end[sb.n - 1] : 0;
  const int64_t blk = blockIdx.x;
  if (blk < n_slab) slab_sum_many_block(sb, blk, reinterpret_cast<f32x4c (*)[16]>(smem));
  else fold_many_block(fb, blk - n_slab, smem);
}

void launch_gradw_finish(const SlabBatch& sb, const FoldBatch& fb, hipStream_t s) {
  if (sb.n <= 0) return launch_toeplitz_fold_many(fb, s);
  if (fb.n <= 0) return launch_slab_sum_many(sb, s);
  const_cast<SlabBatch&>(sb).nt = 1;
  const int64_t blocks = sb.end[sb.n - 1] + (fb.end[fb.n - 1] + 255) / 256;
  hipLaunchKernelGGL(gradw_finish_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sb, fb);
}

void launch_slab_sum_many(const SlabBatch& b, hipStream_t s) {
  const_cast<SlabBatch&>(b).nt = 1;  // slabs are read once: non-temporal loads (with the Q pass's, b64 -2.5 %)
  if (b.n <= 0) return;
  hipLaunchKernelGGL(conv_slab_sum_many_kernel, dim3((unsigned)b.end[b.n - 1]), dim3(256), 0, s, b);
}

// split-K sum for the stride-2 1x1 grad-x: dx[b, c, 2p + i, 2q + j] = (i == j == 0) ?
// sum_z part[z][b][c][p][q] : 0 (+ addend[b, c, 2p + i, 2q + j]); one thread per float4 of dx
// (a (2P) x (2Q) plane, 2Q / 4 float4 per row; compact P x Q pixels per partial plane)
template <int P, int Q>
__global__ __launch_bounds__(256) void conv_slab_sum_ups_kernel(const float* __restrict__ part, float* __restrict__ dx,
                                                                int64_t slab, int n_slices,
                                                                const float* __restrict__ addend) {
  constexpr int F4R = (2 * Q) / 4, F4P = 2 * P * F4R;
  static_assert((2 * Q) % 4 == 0, "float4 rows");
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index into dx
  if (i4 * 4 >= slab * 4) return;                              // dx has 4x the compact elements
  const int64_t plane = i4 / F4P;
  const int r4 = (int)(i4 - plane * F4P);
  const int row = r4 / F4R, half = r4 - row * F4R;
  f32x4c v = {0.f, 0.f, 0.f, 0.f};
  if (addend != nullptr) v = *reinterpret_cast<const f32x4c*>(addend + i4 * 4);
  if ((row & 1) == 0) {
    const int p = row >> 1, q0 = half * 2;                    // this float4 covers q = q0, q0 + 1
    const float* src = part + plane * (P * Q) + p * Q + q0;
    float a = 0.f, b = 0.f;
    for (int z = 0; z < n_slices; ++z) {
      a += src[z * slab];
      b += src[z * slab + 1];
    }
    v.x += a;
    v.z += b;
  }
  *reinterpret_cast<f32x4c*>(dx + i4 * 4) = v;
}

// ---- dispatch -----------------------------------------------------------------------------
template <typename KernelT>
static void set_lds(KernelT k, size_t bytes) {
  hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// A downsample conv's backward pair (the 1x1 stride-2 classes) in ONE launch: workgroups
// [0, n_dgrad) run the direct grad-x (conv_fwd_body on the transposed weights, UPS = 2 epilogue),
// the rest the direct grad-W (64 NW threads; the surplus waves leave before any barrier).
struct DirectDgradArgs {
  const float* dy;
  const float* w;
  float* dx;
  float* part;
  int Cin, Kout, cps;
  int64_t slab;
  const float* addend;
};
template <int DH, int DW, int DBM, int DIMGS, int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW,
          int NBPW, int KB>
__global__ __launch_bounds__(256) void direct_pair_kernel(DirectDgradArgs A, uint3 ga, const float* __restrict__ x,
                                                          const float* __restrict__ dy, float* __restrict__ part,
                                                          int Cin, int Kout, int imgs, uint3 gw) {
  static_assert(NW <= 4, "grad-W workgroup within the pair's 256 threads");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const unsigned na = ga.x * ga.y * ga.z;
  unsigned b = blockIdx.x;
  if (b < na) {
    conv_fwd_body<1, 1, 1, 0, DH, DW, 8, DBM, DIMGS, 2, 2, 4, true, true, 2>(
        A.dy, A.w, A.dx, A.part, A.Cin, A.Kout, A.cps, A.slab, A.addend, ConvBnStats{},
        make_uint3(b % ga.x, (b / ga.x) % ga.y, b / (ga.x * ga.y)), ga, smem);
  } else {
    if (threadIdx.x >= 64 * NW) return;
    b -= na;
    conv_wgrad_body<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>(
        x, dy, part, Cin, Kout, imgs, make_uint3(b % gw.x, (b / gw.x) % gw.y, b / (gw.x * gw.y)), smem);
  }
}

// ksplit > 1: the ksplit workgroups of an output tile each reduce 1/ksplit of the input
// channels into their own slab of `part`; conv_slab_sum(_ups) adds the slabs in split order
// (deterministic).  Used where B / IMGS * Kout / BM alone cannot fill the 256 CUs
// (small per-GPU batches: the strong-scaling shapes 512 / N).
template <int R, int S, int ST, int PD, int H, int W, int CK, int BM, int IMGS, int WM, int NBUF, int KB, bool TRANSW,
          bool VEC, int UPS = 1, int SCH = 0, int IUPS = 1, int PSPLIT = 1>
static int run_fwd(const float* x, const float* w, float* y, int B, int Cin, int Kout, int ksplit, float* part,
                   hipStream_t s, const float* addend = nullptr, bool defer = false,
                   ConvBnStats stats = ConvBnStats{nullptr, nullptr, nullptr, nullptr, nullptr}) {
  using G = ConvFwdCfg<R, S, ST, PD, H, W, CK, BM, IMGS, WM, NBUF, KB, TRANSW, PSPLIT>;
  auto k = conv_fwd_kernel<R, S, ST, PD, H, W, CK, BM, IMGS, WM, NBUF, KB, TRANSW, VEC, UPS, SCH, IUPS, PSPLIT>;
  static bool attr = false;  // once per instantiation (> 64 KiB of LDS needs the opt-in)
  if (!attr) { set_lds(k, G::LDS_BYTES); attr = true; }
  const int nchunks = (Cin + CK - 1) / CK;
  if (ksplit < 1 || part == nullptr) ksplit = 1;
  const int cps = (nchunks + ksplit - 1) / ksplit;
  ksplit = (nchunks + cps - 1) / cps;
  const int64_t slab = (int64_t)B * Kout * G::PQ;  // compact partial tile layout
  // stats: only unsplit launches of statistics-capable tiles (conv_fwd_stats_slices says which)
  if (!(G::STATS_OK && UPS == 1) || ksplit > 1 || (stats.bx != nullptr && !G::STATS2_OK)) stats.out = nullptr;
  hipLaunchKernelGGL(k, dim3(B / IMGS * PSPLIT, Kout / BM, ksplit), dim3(256), G::LDS_BYTES, s, x, w, y, part, Cin, Kout, cps,
                     slab, ksplit > 1 ? nullptr : addend, stats);
  // defer: leave the ksplit slabs for the consumer (the fused BN kernel sums them while it
  // reads its input, ops/slablink.py) — one launch fewer per conv
  // (an addend then goes to the consumer too: it adds it after the slabs, launch_bn_bwd dyadd)
  if (ksplit > 1 && defer && UPS == 1) return ksplit;
  if (ksplit > 1) {
    if constexpr (UPS == 1)
      hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((slab / 4 + 15) / 16)), dim3(256), 0, s, part, y, slab,
                         ksplit, addend);
    else
      hipLaunchKernelGGL((conv_slab_sum_ups_kernel<G::P, G::Q>), dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, s,
                         part, y, slab, ksplit, addend);
  }
  return 1;
}

// ---- the downsample block's two forward convs in ONE launch --------------------------------
// conv1 (3x3 stride 2, class 2) and the 1x1 stride-2 downsample (class 4) read the same block
// input; the downsample's launch is held back (launch_conv_fwd pair = true) and conv1's launch
// runs both bodies on one grid: conv1's workgroups first (its output feeds bn1 right after).
struct FwdPart {
  const float* x;
  const float* w;
  float* y;
  float* part;
  int Cin, Kout, cps;
  int64_t slab;
};
__global__ __launch_bounds__(256) void ds_fwd_pair_kernel(FwdPart a, uint3 ga, FwdPart b, uint3 gb) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const unsigned na = ga.x * ga.y * ga.z;
  unsigned k = blockIdx.x;
  if (k < na) {
    conv_fwd_body<3, 3, 2, 1, 8, 8, 8, 64, 4, 2, 2, 4, false, true>(
        a.x, a.w, a.y, a.part, a.Cin, a.Kout, a.cps, a.slab, nullptr, ConvBnStats{},
        make_uint3(k % ga.x, (k / ga.x) % ga.y, k / (ga.x * ga.y)), ga, smem);
  } else {
    k -= na;
    conv_fwd_body<1, 1, 2, 0, 8, 8, 8, 64, 4, 2, 2, 4, false, true>(
        b.x, b.w, b.y, b.part, b.Cin, b.Kout, b.cps, b.slab, nullptr, ConvBnStats{},
        make_uint3(k % gb.x, (k / gb.x) % gb.y, k / (gb.x * gb.y)), gb, smem);
  }
}

// the split of a class-2 / class-4 forward as run_fwd normalises it
template <typename G>
static FwdPart fwd_part(const float* x, const float* w, float* y, float* part, int B, int Cin, int Kout, int& ksplit) {
  const int nchunks = (Cin + 8 - 1) / 8;
  if (ksplit < 1 || part == nullptr) ksplit = 1;
  const int cps = (nchunks + ksplit - 1) / ksplit;
  ksplit = (nchunks + cps - 1) / cps;
  return FwdPart{x, w, y, part, Cin, Kout, cps, (int64_t)B * Kout * G::PQ};
}

void launch_slab_sum(const float* part, float* out, int64_t n, int nslab, hipStream_t s, const float* addend) {
  hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((n / 4 + 15) / 16)), dim3(256), 0, s, part, out, n, nslab,
                     addend);
}

template <int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
static void run_wgrad(const float* x, const float* dy, float* part, float* dw, int B, int Cin, int Kout,
                      int imgs, hipStream_t s) {
  using G = ConvWgCfg<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  auto k = conv_wgrad_kernel<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  static bool attr = false;
  if (!attr) { set_lds(k, G::LDS_BYTES); attr = true; }
  const int slices = B / imgs;
  hipLaunchKernelGGL(k, dim3(slices, Kout / BM, (Cin + CB - 1) / CB), dim3(G::NT), G::LDS_BYTES, s, x, dy, part, Cin,
                     Kout, imgs);
  if (dw == nullptr) return;  // partials only: the caller sums the slabs (batched, ops/gradfinish.py)
  const int64_t n = (int64_t)Kout * Cin * G::RS;  // multiple of 4 for every class
  hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((n / 4 + 15) / 16)), dim3(256), 0, s, part, dw, n, slices);
}

// Shape classes with a direct kernel (everything else stays on MIOpen / the Toeplitz path)
//   id 0: 3x3 s1 p1 on 8x8   (ResNet layer1)           C, K % 64 == 0
//   id 1: 3x3 s1 p1 on 4x4   (ResNet layer2)           C, K % 64 == 0
//   id 2: 3x3 s2 p1 8x8->4x4 (layer2 first conv)       C, K % 64 == 0; grad-x = the id-0 kernel on
//         the zero-inserted dY (IUPS = 2 staging)
//   id 3: 7x7 s2 p3 32x32->16x16, C = 3 (stem)         K % 64 == 0
//   id 4: 1x1 s2 p0 8x8->4x4 (layer2 downsample)        C % 32 == 0, K % 64 == 0;
//         grad-x = the 1x1 transposed product on the 4x4 map, written to the even pixels
//         of the 8x8 plane (UPS = 2 epilogue, odd pixels zero)
//   id 5: 1x1 s2 p0 4x4->2x2 (layer3 downsample)        the id-4 scheme one map size down: 16
//         images per tile; the Toeplitz GEMM it replaces multiplied 15 zero rows of W_big per
//         useful one (profiles/r5/toeplitz_layers_b512.md: 72.8 us fwd + bwd at batch 512)
int conv_direct_class(const ConvGeom& g) {
  if (g.KH == 3 && g.KW == 3 && g.pad == 1 && g.stride == 1 && g.H == 8 && g.W == 8 && g.C % 64 == 0 && g.Co % 64 == 0)
    return 0;
  if (g.KH == 3 && g.KW == 3 && g.pad == 1 && g.stride == 1 && g.H == 4 && g.W == 4 && g.C % 64 == 0 && g.Co % 64 == 0)
    return 1;
  if (g.KH == 3 && g.KW == 3 && g.pad == 1 && g.stride == 2 && g.H == 8 && g.W == 8 && g.C % 64 == 0 && g.Co % 64 == 0)
    return 2;
  if (g.KH == 7 && g.KW == 7 && g.pad == 3 && g.stride == 2 && g.H == 32 && g.W == 32 && g.C == 3 && g.Co % 64 == 0)
    return 3;
  if (g.KH == 1 && g.KW == 1 && g.pad == 0 && g.stride == 2 && g.H == 8 && g.W == 8 && g.C % 64 == 0 && g.Co % 64 == 0)
    return 4;
  if (g.KH == 1 && g.KW == 1 && g.pad == 0 && g.stride == 2 && g.H == 4 && g.W == 4 && g.C % 64 == 0 && g.Co % 64 == 0)
    return 5;
  return -1;
}

// images per workgroup of the forward / grad-x kernels, images per grad-W slice
int conv_fwd_imgs(int cls) { return (cls == 0 || cls == 3) ? 1 : cls == 5 ? 16 : 4; }

static constexpr int kFillWgs = 256;  // one workgroup per CU: below this, split the reduction

static int pow2_floor(int v) {
  int p = 1;
  while (p * 2 <= v) p *= 2;
  return p;
}

// images per grad-W slice: the class default, lowered (power of two dividing B) until the
// grid has >= kFillWgs workgroups.  Workgroups per slice = (Kout / 32) * ceil(Cin / CB).
// (Larger slices = fewer slabs to sum measured slower in round 3: batch 512 x2 1.9937, x4
// 1.9969 vs 1.9904 / 1.9927 ms; batch 256 1.4473 / 1.4444 vs 1.441.)
// Round 5 (Winograd grad-W, deferred batched slab sums): doubling the layer1 (Winograd), 3x3/2 and
// stem slices halves their slabs — ResNet-18 r=4 batch 512 1.5118 / 1.5129 -> 1.4977 / 1.4957 ms;
// doubling layer2's (class 1) was slower, 1.5043 -> 1.5165 (profiles/r5/bench_wgrad_slices.jsonl).
int conv_wgrad_imgs(int cls, const ConvGeom& g, int B) {
  // (the geometry test only, not the runtime Winograd switch: the slicing stays fixed for a shape,
  // so scratch sized from a cached plan fits whichever grad-W kernel runs)
  if (cls == 0 && g.H == 8 && g.C % 16 == 0 && g.Co % 16 == 0 && B <= 128 && B % 4 == 0) {
    // Winograd grad-W with the 4-wave reduction (winograd.hip wino_wgrad_kernel RED = 4) at the
    // small per-GPU batches: a workgroup per 16 x 16 block and slice, >= one image per wave.
    // ResNet-18 r=4 batch 64 0.843 -> 0.830 ms (4x fewer slabs: grad-W 31.7 -> 29.9 µs, slab sum
    // 16.0 -> 13.3); at batch 256 / 512 the 4 waves of a workgroup reading different images lost
    // (512: grad-W + slab sum 120.9 -> 124.0 µs; 256: 1.102 -> 1.120 ms at 4 images per slice)
    const int per_slice = (g.Co / 16) * (g.C / 16);
    int d = 32;
    while (d > 4 && (B % d != 0 || (B / d) * per_slice < kFillWgs)) d /= 2;
    if (B % d == 0 && wino_wgrad_red(B, d)) return d;
  }
  if (cls == 0 && g.H == 8 && g.C % 16 == 0 && g.Co % 16 == 0 && B >= 256 && B % 16 == 0 && wino_wgrad_red(B, 16)) {
    // from batch 256: 16-image slices over the 4-wave reduction (4 images per wave) — half the
    // slabs of 8-image slices, two workgroups per CU at 512.  ResNet-18 r=4, ms/step: batch 512
    // 1.3866 / 1.3908 vs 1.4043 / 1.4021 (8-image, 2-wave), batch 256 0.9942 / 0.9993 vs 1.0035 /
    // 1.0046 (8-image, 1-wave); 32-image slices 1.4103 (profiles/r6/bench_l1_wgrad_slices.jsonl)
    return 16;
  }
  // layer2 (class 1) from batch 512: 32-image slices, half the slabs.  Its grad-W now runs in one
  // launch with its grad-x (wino_direct_pair_kernel), which fills the CUs: ResNet-18 r=4 batch 512
  // 1.3711 / 1.3692 vs 1.3775 / 1.3804 ms (16-image), and 1.3806 / 1.3819 vs 1.3877 / 1.3886 on a
  // second box; batch 256 unchanged (0.9927 vs 0.9920 / 0.9914) (profiles/r6/bench_l2_wgrad_slices.jsonl)
  int def = cls == 0 ? 8 : cls == 1 ? (B >= 512 ? 32 : 16) : cls == 2 ? 16 : cls == 4 ? 8 : cls == 5 ? 16 : 4;
  const int cb = cls == 3 ? 3 : 32;
  const int per_slice = (g.Co / 32) * ((g.C + cb - 1) / cb);
  while (def > 1 && B % def != 0) def /= 2;  // a batch that is not a multiple of the default
  while (def > 1 && (B / def) * per_slice < kFillWgs && B % (def / 2) == 0) def /= 2;
  return def;
}

// split-K cap: 4 keeps layer2's slabs summable inside the fused BN kernel (batchnorm.hip
// kMaxFusedSlabs) — ResNet-18 step on 1x MI355X, batch 128 1.216 / 1.197 -> 1.191 / 1.188 ms,
// batch 64 1.050 / 1.050 -> 1.049 / 1.046 (uncapped: 8 slabs at batch 64).  The 1x1 stride-2
// grad-x takes the same cap (a cap of 1 measured 0.960 -> 0.967 ms at batch 64).
static constexpr int kConvMaxSplit = 4;

// split-K factor of the forward (dgrad = false) / grad-x (dgrad = true) kernels: a power of
// two <= the channel chunks, so that (B / IMGS) * (outC / 64) * ksplit >= kFillWgs
int conv_ksplit(int cls, const ConvGeom& g, int B, bool dgrad) {
  if (cls < 0 || cls == 3) return 1;
  // the 1x1/2 grad-x runs in one launch with its grad-W (direct_pair_kernel), whose workgroups fill
  // the CUs: unsplit from batch 512 (no slab-sum launch; 1.4306 / 1.4308 -> 1.4192 / 1.4229 ms, at
  // 256 even: 1.0053 vs 1.0076)
  if (dgrad && (cls == 4 || cls == 5) && B >= 512) return 1;
  const int inC = dgrad ? g.Co : g.C, outC = dgrad ? g.C : g.Co;
  const int imgs = (dgrad && cls == 2) ? 1 : conv_fwd_imgs(cls);  // class-2 grad-x: 8x8 tiles, 1 image
  const int base = (B / imgs) * (outC / 64);
  const int nchunks = inC / 8;
  int ks = 1;
  while (ks * 2 <= nchunks && base * ks < kFillWgs && ks * 2 <= kConvMaxSplit) ks *= 2;
  return pow2_floor(ks);
}
// BatchNorm statistics from the forward epilogue: the layer1 3x3 and stem 7x7 classes (their
// BatchNorms take the two-kernel large-map path; layer2's single-launch BN computes its own),
// unsplit launches only.  Returns the partial count S (= workgroups along the batch), 0 = none.
// split-K Winograd slabs: left to the consumer (defer: it sums them, and an addend after them) or
// summed here in slab order (+ addend), like run_fwd
static int wino_slabs(const float* part, float* out, int64_t n, int ks, bool defer, const float* addend,
                      hipStream_t s) {
  if (defer) return ks;
  hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((n / 4 + 15) / 16)), dim3(256), 0, s, part, out, n, ks,
                     addend);
  return 1;
}

// Winograd F(2x2, 3x3) (winograd.hip) for the 8x8 3x3 classes: forward of class 0, grad-x of
// class 0 and of class 2 (its zero-inserted dY), unsplit launches that tile exactly
bool conv_wino(int cls, const ConvGeom& g, int B, bool dgrad) {
  // the direct kernel's split-K factor (small batches) is kept: the Winograd slabs then go to the
  // same consumers (slab sum / the fused BN kernel)
  if (dgrad)  // class 2's grad-x is an 8x8 map (its zero-inserted dY)
    return (cls == 0 || cls == 1 || cls == 2) && wino_ok(g.Co, g.C, B, g.H, g.W, conv_ksplit(cls, g, B, true));
  return (cls == 0 || cls == 1) && wino_ok(g.C, g.Co, B, g.H, g.W, conv_ksplit(cls, g, B, false));
}

// Output-row blocks per image of the stem forward (ConvFwdCfg PSPLIT): enough workgroups for
// the 256 CUs at the small per-GPU batches of the strong-scaling runs.  Every split re-stages
// the image and the 64 x 196 weight image, so more blocks only pay below one workgroup per CU.
// Stem forward + statistics epilogue on 1x MI355X (tools/diag/stem_psplit.py, µs, split 1/2/4;
// profiles/r5/stem_psplit*.jsonl): batch 64 20.8 / 15.9 / 12.1, 128 21.4 / 16.7 / 16.9,
// 256 22.9 / 23.5 / 30.9, 512 34.1 / 43.6 / 58.2 (paired-k stem with float4 weight staging;
// before it, 512: 51.5 / 72.3 / 110 — 1 wave per SIMD from 400+ registers of staging state).
static int g_stem_psplit = 0;  // 0 = by batch (A/B override: conv_set_stem_psplit)
void conv_set_stem_psplit(int p) { g_stem_psplit = (p == 1 || p == 2 || p == 4) ? p : 0; }
int stem_psplit(int B) {
  if (g_stem_psplit) return g_stem_psplit;
  return B >= 256 ? 1 : B >= 128 ? 2 : 4;
}

int conv_fwd_stats_slices(int cls, const ConvGeom& g, int B) {
  static_assert(ConvFwdCfg<3, 3, 1, 1, 8, 8, 8, 64, 1, 2, 2, 4, false>::STATS_OK &&
                    ConvFwdCfg<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false>::STATS_OK &&
                    ConvFwdCfg<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false, 2>::STATS_OK &&
                    ConvFwdCfg<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false, 4>::STATS_OK,
                "statistics epilogue fits every layer1 / stem tile");
  if (cls != 0 && cls != 3) return 0;
  if (conv_ksplit(cls, g, B, false) != 1) return 0;
  if (cls == 3) return B * stem_psplit(B);  // one partial per (image, row block)
  return conv_wino(cls, g, B, false) ? B / wino_imgs(g.H) : B / conv_fwd_imgs(cls);
}
// backward-mode BN partial sums from the grad-x epilogue: the layer1 3x3 class (its BN takes the
// two-kernel large-map path), unsplit grad-x launches only; 0 = none
int conv_dgrad_stats_slices(int cls, const ConvGeom& g, int B) {
  static_assert(ConvFwdCfg<3, 3, 1, 1, 8, 8, 8, 64, 1, 2, 2, 4, true>::STATS2_OK,
                "backward statistics epilogue fits the layer1 grad-x tiles");
  // class 2 (3x3 stride 2) runs the layer1 grad-x kernel on the zero-inserted dY: one image per tile
  if ((cls != 0 && cls != 2) || conv_ksplit(cls, g, B, true) != 1) return 0;
  if (conv_wino(cls, g, B, true)) return B / wino_imgs(g.H);
  return cls == 2 ? B : B / conv_fwd_imgs(cls);
}
// Every class runs its grad-x natively.  The 3x3 stride-2 grad-x runs on the zero-inserted dY
// (exact, 4x the MFMA work of the sub-pixel form; round 2: 2.006 / 2.005 vs MIOpen 1.991 ms at
// batch 512): MIOpen's algorithm choice depends on its on-disk find database and, captured in a
// hipGraph, was found non-deterministic and NaN-producing (round 3 bisection).
bool conv_dgrad_direct(int cls) { return cls >= 0 && cls <= 5 && cls != 3; }

// MFMA-block schedule of the layer1 / layer2 fwd + grad-x kernels: SCH = 2 (pinned MFMA /
// LDS-read interleave): ResNet-18 step on 1x MI355X 2.0175 / 2.0154 -> 1.9981 / 1.9994 ms at
// batch 512, 1.0582 / 1.0627 -> 1.0546 / 1.0569 at batch 64 against the compiler's schedule
// (iglp_opt(0): 2.0043 / 1.0602; the pinned interleave on the stem / 3x3-2 / 1x1-2 forwards
// and 16-channel chunks or two-image layer1 tiles were slower — round 3 A/Bs)
namespace {
struct PendingFwd {  // the downsample conv's forward, held for its block's conv1 (class 2)
  const float* x = nullptr;
  const float* w = nullptr;
  float* y = nullptr;
  float* part = nullptr;
  int B = 0, ks = 1;
  bool defer = false;
  ConvGeom g{};
  hipStream_t s = nullptr;
};
PendingFwd g_pending_fwd;
using CfgC2 = ConvFwdCfg<3, 3, 2, 1, 8, 8, 8, 64, 4, 2, 2, 4, false, 1>;
using CfgC4 = ConvFwdCfg<1, 1, 2, 0, 8, 8, 8, 64, 4, 2, 2, 4, false, 1>;
}  // namespace

void conv_flush_pending_fwd() {
  if (g_pending_fwd.x == nullptr) return;
  const PendingFwd p = g_pending_fwd;
  g_pending_fwd = PendingFwd{};
  run_fwd<1, 1, 2, 0, 8, 8, 8, 64, 4, 2, 2, 4, false, true>(p.x, p.w, p.y, p.B, p.g.C, p.g.Co, p.ks, p.part, p.s,
                                                           nullptr, p.defer);
}

int launch_conv_fwd(const float* x, const float* w, float* y, int B, const ConvGeom& g, float* part, hipStream_t s,
                    bool defer, double* stats_out, float* wino_u, bool pair) {
  const ConvBnStats stats{stats_out, nullptr, nullptr, nullptr, nullptr};
  const int cls = conv_direct_class(g);
  const int ks = conv_ksplit(cls, g, B, false);
  if (cls == 4 && pair && stats_out == nullptr) {  // held for conv1 (ds_fwd_pair_kernel); same return as run_fwd
    conv_flush_pending_fwd();
    int k = ks;
    fwd_part<CfgC4>(x, w, y, part, B, g.C, g.Co, k);
    g_pending_fwd = PendingFwd{x, w, y, part, B, ks, defer, g, s};
    return (k > 1 && defer) ? k : 1;
  }
  if (cls == 2 && g_pending_fwd.x == x && g_pending_fwd.s == s && g_pending_fwd.B == B && stats_out == nullptr) {
    const PendingFwd p = g_pending_fwd;
    g_pending_fwd = PendingFwd{};
    int ka = ks, kb = p.ks;
    const FwdPart a = fwd_part<CfgC2>(x, w, y, part, B, g.C, g.Co, ka);
    const FwdPart b = fwd_part<CfgC4>(p.x, p.w, p.y, p.part, B, p.g.C, p.g.Co, kb);
    const uint3 ga = make_uint3((unsigned)(B / 4), (unsigned)(g.Co / 64), (unsigned)ka);
    const uint3 gb = make_uint3((unsigned)(B / 4), (unsigned)(p.g.Co / 64), (unsigned)kb);
    constexpr size_t lds = CfgC2::LDS_BYTES > CfgC4::LDS_BYTES ? CfgC2::LDS_BYTES : CfgC4::LDS_BYTES;
    static bool attr = false;
    if (!attr) { set_lds(ds_fwd_pair_kernel, lds); attr = true; }
    hipLaunchKernelGGL(ds_fwd_pair_kernel, dim3(ga.x * ga.y * ga.z + gb.x * gb.y * gb.z), dim3(256), lds, s, a, ga, b, gb);
    if (kb > 1 && !p.defer)
      hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((b.slab / 4 + 15) / 16)), dim3(256), 0, s, p.part, p.y,
                         b.slab, kb, nullptr);
    if (ka > 1 && defer) return ka;
    if (ka > 1)
      hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((a.slab / 4 + 15) / 16)), dim3(256), 0, s, part, y,
                         a.slab, ka, nullptr);
    return 1;
  }
  conv_flush_pending_fwd();
  if (wino_u != nullptr && conv_wino(cls, g, B, false)) {
    launch_wino_conv(x, wino_u, y, B, g.C, g.Co, g.H, false, 1, nullptr, ks > 1 ? ConvBnStats{} : stats, ks, part, s);
    return ks > 1 ? wino_slabs(part, y, (int64_t)B * g.Co * g.H * g.W, ks, defer, nullptr, s) : 1;
  }
  switch (cls) {
    case 0:
      return run_fwd<3, 3, 1, 1, 8, 8, 8, 64, 1, 2, 2, 4, false, true, 1, 2>(x, w, y, B, g.C, g.Co, ks, part, s,
                                                                             nullptr, defer, stats);
    case 1:
      return run_fwd<3, 3, 1, 1, 4, 4, 8, 64, 4, 2, 2, 4, false, true, 1, 2>(x, w, y, B, g.C, g.Co, ks, part, s,
                                                                             nullptr, defer);
    case 2:
      return run_fwd<3, 3, 2, 1, 8, 8, 8, 64, 4, 2, 2, 4, false, true>(x, w, y, B, g.C, g.Co, ks, part, s, nullptr,
                                                                       defer);
    case 3:
      switch (stem_psplit(B)) {
        case 4:
          return run_fwd<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false, false, 1, 0, 1, 4>(x, w, y, B, g.C, g.Co, 1, nullptr,
                                                                                        s, nullptr, false, stats);
        case 2:
          return run_fwd<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false, false, 1, 0, 1, 2>(x, w, y, B, g.C, g.Co, 1, nullptr,
                                                                                        s, nullptr, false, stats);
        default:
          return run_fwd<7, 7, 2, 3, 32, 32, 4, 64, 1, 2, 1, 7, false, false>(x, w, y, B, g.C, g.Co, 1, nullptr, s,
                                                                              nullptr, false, stats);
      }
    case 4:
      return run_fwd<1, 1, 2, 0, 8, 8, 8, 64, 4, 2, 2, 4, false, true>(x, w, y, B, g.C, g.Co, ks, part, s, nullptr,
                                                                       defer);
    case 5:
      return run_fwd<1, 1, 2, 0, 4, 4, 8, 64, 16, 2, 2, 4, false, true>(x, w, y, B, g.C, g.Co, ks, part, s, nullptr,
                                                                        defer);
    default: return 1;
  }
}

// A layer1 Winograd grad-W held back by launch_conv_wgrad(pair = true) for the grad-x of the same
// conv (host state only: set and consumed within one conv backward, capture-safe)
namespace {
struct PendingWgrad {
  const float* x = nullptr;
  const float* dy = nullptr;
  float* part = nullptr;
  int B = 0, imgs = 0, cls = -1;
  ConvGeom g{};
  hipStream_t s = nullptr;
};
// two slots: a downsample block's two sibling convs (3x3/2 and 1x1/2) each hold one while the
// BranchLink defers one of their grad-x launches into the other's backward
constexpr int kPendingSlots = 2;
PendingWgrad g_pending[kPendingSlots];
unsigned g_pending_seq[kPendingSlots];
unsigned g_seq = 0;

void launch_pending(const PendingWgrad& p);
// the held-back grad-W of THIS grad-x's conv (same dY, same geometry and stream), or nullptr
PendingWgrad* find_pending(const float* dy, int cls, int B, const ConvGeom& g, hipStream_t s) {
  for (auto& p : g_pending)
    if (p.dy == dy && p.cls == cls && p.s == s && p.B == B && p.g.C == g.C && p.g.Co == g.Co && p.g.H == g.H) return &p;
  return nullptr;
}
// launch (alone) whatever is held for this dY
void flush_pending_dy(const float* dy) {
  for (auto& p : g_pending)
    if (p.dy == dy) {
      const PendingWgrad q = p;
      p = PendingWgrad{};
      launch_pending(q);
    }
}
// hold a grad-W: a free slot, else the oldest one is launched alone first
void hold_pending(const PendingWgrad& q) {
  int k = -1;
  for (int i = 0; i < kPendingSlots; ++i)
    if (g_pending[i].dy == nullptr) { k = i; break; }
  if (k < 0) {
    k = g_pending_seq[0] <= g_pending_seq[1] ? 0 : 1;
    const PendingWgrad old = g_pending[k];
    g_pending[k] = PendingWgrad{};
    launch_pending(old);
  }
  g_pending[k] = q;
  g_pending_seq[k] = ++g_seq;
}

// grad-x of a layer2 class on the Winograd kernel + the held-back direct grad-W, one launch
template <int WH, int IUPS, int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW, int KB>
void run_pair(const float* dy, const float* u, float* dx, int B, int inC, int outC, const float* addend,
              const ConvBnStats& st, int ks, float* part_x, const PendingWgrad& p, hipStream_t s) {
  using G = ConvWgCfg<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  auto k = wino_direct_pair_kernel<WH, IUPS, R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  constexpr size_t lds = kWLds > G::LDS_BYTES ? kWLds : G::LDS_BYTES;
  static bool attr = false;
  if (!attr) { set_lds(k, lds); attr = true; }
  const WinoConvArgs a{dy, u + 16 * (int64_t)inC * outC,  // the grad-x half of the transforms
                       dx, inC, outC, ks > 1 ? nullptr : addend, ks > 1 ? ConvBnStats{} : st, (inC / kWCK) / ks,
                       part_x, (int64_t)B * outC * WH * WH};
  const uint3 ga = make_uint3((unsigned)(B / wino_imgs(WH)), (unsigned)(outC / kWBM), (unsigned)ks);
  const uint3 gw = make_uint3((unsigned)(p.B / p.imgs), (unsigned)(p.g.Co / BM), (unsigned)((p.g.C + CB - 1) / CB));
  const unsigned n = ga.x * ga.y * ga.z + gw.x * gw.y * gw.z;
  hipLaunchKernelGGL(k, dim3(n), dim3(256), lds, s, a, ga, p.x, p.dy, p.part, p.g.C, p.g.Co, p.imgs, gw);
}
// the 1x1 stride-2 grad-x (run_fwd's UPS = 2 path, incl. its split-K slab sum) + the held-back direct
// grad-W of the same conv, one launch
template <int DH, int DW, int DIMGS, int R, int S, int ST, int PD, int H, int W, int CB, int BM, int NW, int NBPW,
          int KB>
int run_direct_pair(const float* dy, const float* w, float* dx, int B, int Cin, int Kout, int ksplit, float* part,
                    const float* addend, const PendingWgrad& p, hipStream_t s) {
  using GF = ConvFwdCfg<1, 1, 1, 0, DH, DW, 8, 64, DIMGS, 2, 2, 4, true, 1>;
  using GW = ConvWgCfg<R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  auto k = direct_pair_kernel<DH, DW, 64, DIMGS, R, S, ST, PD, H, W, CB, BM, NW, NBPW, KB>;
  constexpr size_t lds = GF::LDS_BYTES > GW::LDS_BYTES ? GF::LDS_BYTES : GW::LDS_BYTES;
  static bool attr = false;
  if (!attr) { set_lds(k, lds); attr = true; }
  const int nchunks = (Cin + 7) / 8;
  if (ksplit < 1 || part == nullptr) ksplit = 1;
  const int cps = (nchunks + ksplit - 1) / ksplit;
  ksplit = (nchunks + cps - 1) / cps;
  const int64_t slab = (int64_t)B * Kout * GF::PQ;
  const DirectDgradArgs a{dy, w, dx, part, Cin, Kout, cps, slab, ksplit > 1 ? nullptr : addend};
  const uint3 ga = make_uint3((unsigned)(B / DIMGS), (unsigned)(Kout / 64), (unsigned)ksplit);
  const uint3 gw = make_uint3((unsigned)(p.B / p.imgs), (unsigned)(p.g.Co / BM), (unsigned)((p.g.C + CB - 1) / CB));
  const unsigned n = ga.x * ga.y * ga.z + gw.x * gw.y * gw.z;
  hipLaunchKernelGGL(k, dim3(n), dim3(256), lds, s, a, ga, p.x, p.dy, p.part, p.g.C, p.g.Co, p.imgs, gw);
  if (ksplit > 1)
    hipLaunchKernelGGL((conv_slab_sum_ups_kernel<GF::P, GF::Q>), dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, s,
                       part, dx, slab, ksplit, addend);
  return 1;
}

void launch_pending(const PendingWgrad& p) {
  if (p.cls == 0) launch_wino_wgrad(p.x, p.dy, p.part, p.B, p.g.C, p.g.Co, p.g.H, p.imgs, p.s);
  else if (p.cls == 1) run_wgrad<3, 3, 1, 1, 4, 4, 32, 32, 3, 3, 4>(p.x, p.dy, p.part, nullptr, p.B, p.g.C, p.g.Co, p.imgs, p.s);
  else if (p.cls == 2) run_wgrad<3, 3, 2, 1, 8, 8, 32, 32, 3, 3, 4>(p.x, p.dy, p.part, nullptr, p.B, p.g.C, p.g.Co, p.imgs, p.s);
  else if (p.cls == 4) run_wgrad<1, 1, 2, 0, 8, 8, 32, 32, 1, 1, 4>(p.x, p.dy, p.part, nullptr, p.B, p.g.C, p.g.Co, p.imgs, p.s);
  else run_wgrad<1, 1, 2, 0, 4, 4, 32, 32, 1, 1, 2>(p.x, p.dy, p.part, nullptr, p.B, p.g.C, p.g.Co, p.imgs, p.s);
}
}  // namespace

// every held-back grad-W, oldest first
void conv_flush_pending() {
  while (true) {
    int k = -1;
    for (int i = 0; i < kPendingSlots; ++i)
      if (g_pending[i].dy != nullptr && (k < 0 || g_pending_seq[i] < g_pending_seq[k])) k = i;
    if (k < 0) return;
    const PendingWgrad p = g_pending[k];
    g_pending[k] = PendingWgrad{};
    launch_pending(p);
  }
}

// dx[B, C, H, W] from dy[B, Co, OH, OW]
int launch_conv_dgrad(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, float* part,
                      hipStream_t s, const float* addend, bool defer, const ConvBnStats* bst, float* wino_u) {
  const ConvBnStats stats = bst != nullptr ? *bst : ConvBnStats{nullptr, nullptr, nullptr, nullptr, nullptr};
  const int cls = conv_direct_class(g);
  const int ks = conv_ksplit(cls, g, B, true);
  if (wino_u != nullptr && conv_wino(cls, g, B, true)) {
    if (PendingWgrad* pp = find_pending(dy, cls, B, g, s)) {
      // this conv's grad-W is waiting: both in one launch
      const PendingWgrad p = *pp;
      *pp = PendingWgrad{};
      if (cls == 0)
        launch_wino_bwd_pair(dy, wino_u, dx, B, g.Co, g.C, addend, stats, ks, part, p.x, p.part, p.imgs, s);
      else if (cls == 1)
        run_pair<4, 1, 3, 3, 1, 1, 4, 4, 32, 32, 3, 3, 4>(dy, wino_u, dx, B, g.Co, g.C, addend, stats, ks, part, p, s);
      else
        run_pair<8, 2, 3, 3, 2, 1, 8, 8, 32, 32, 3, 3, 4>(dy, wino_u, dx, B, g.Co, g.C, addend, stats, ks, part, p, s);
    } else {
      flush_pending_dy(dy);  // this conv's own grad-W, not pairable after all
      launch_wino_conv(dy, wino_u, dx, B, g.Co, g.C, g.H, true, cls == 2 ? 2 : 1, addend,
                       ks > 1 ? ConvBnStats{} : stats, ks, part, s);
    }
    return ks > 1 ? wino_slabs(part, dx, (int64_t)B * g.C * g.H * g.W, ks, defer, addend, s) : 1;
  }
  if (PendingWgrad* pp = (cls == 4 || cls == 5) ? find_pending(dy, cls, B, g, s) : nullptr) {
    // the downsample conv's grad-W is waiting: both in one launch
    const PendingWgrad p = *pp;
    *pp = PendingWgrad{};
    return cls == 4
        ? run_direct_pair<4, 4, 4, 1, 1, 2, 0, 8, 8, 32, 32, 1, 1, 4>(dy, w, dx, B, g.Co, g.C, ks, part, addend, p, s)
        : run_direct_pair<2, 2, 16, 1, 1, 2, 0, 4, 4, 32, 32, 1, 1, 2>(dy, w, dx, B, g.Co, g.C, ks, part, addend, p, s);
  }
  flush_pending_dy(dy);
  switch (cls) {
    case 0:
      return run_fwd<3, 3, 1, 1, 8, 8, 8, 64, 1, 2, 2, 4, true, true, 1, 2>(dy, w, dx, B, g.Co, g.C, ks, part, s,
                                                                            addend, defer, stats);
    case 1:
      return run_fwd<3, 3, 1, 1, 4, 4, 8, 64, 4, 2, 2, 4, true, true, 1, 2>(dy, w, dx, B, g.Co, g.C, ks, part, s,
                                                                            addend, defer);
    case 2:  // 3x3 stride 2: the layer1 grad-x kernel on the zero-inserted dY (staged, not stored)
      return run_fwd<3, 3, 1, 1, 8, 8, 8, 64, 1, 2, 2, 4, true, true, 1, 2, 2>(dy, w, dx, B, g.Co, g.C, ks, part, s,
                                                                              addend, defer, stats);
    case 4:
      return run_fwd<1, 1, 1, 0, 4, 4, 8, 64, 4, 2, 2, 4, true, true, 2>(dy, w, dx, B, g.Co, g.C, ks, part, s, addend);
    case 5:
      return run_fwd<1, 1, 1, 0, 2, 2, 8, 64, 16, 2, 2, 4, true, true, 2>(dy, w, dx, B, g.Co, g.C, ks, part, s, addend);
    default: return 1;
  }
}

// part: (B / conv_wgrad_imgs) * Co * C * KH * KW floats of scratch
void launch_conv_wgrad(const float* x, const float* dy, float* part, float* dw, int B, const ConvGeom& g,
                       hipStream_t s, bool pair) {
  // a grad-W held back earlier stays held (its grad-x may come later, e.g. from the BranchLink
  // sibling's backward) unless this one needs its slot
  const int cls = conv_direct_class(g);
  const int imgs = conv_wgrad_imgs(cls, g, B);
  if (cls == 0 && wino_wgrad_ok(g.C, g.Co, g.H)) {
    // held back for this conv's grad-x (launch_conv_dgrad).  ResNet-18 r=4, ms/step
    // (profiles/r6/bench_wino_pair.jsonl): batch 64 0.7758 / 0.7656 -> 0.7498 / 0.7517, 128
    // 0.8676 -> 0.8434, 256 (with the layer2 pairs) 1.0539 / 1.0572 -> 1.0303 / 1.0343; at 512 the
    // pair was slower with the one-wave-per-block grad-W (1.4640 -> 1.4818), faster with the
    // two-wave one (winograd.hip wgrad_red: 1.4143 / 1.4147 -> 1.3934 / 1.3966)
    if (pair && dw == nullptr) {
      hold_pending(PendingWgrad{x, dy, part, B, imgs, cls, g, s});
      return;
    }
    // Winograd-domain grad-W (winograd.hip): same slab layout and slicing as the direct kernel.
    // Layer1 only: ResNet-18 at batch 512 90.7 vs 130.2 µs per step (4 launches), batch 64 31.1 vs
    // 38.5; the 4x4 maps (one tile per lane group and image: a load per 16 MFMAs) measured slower,
    // 142.8 vs 99.0 µs at batch 512 and 64.0 vs 29.5 at batch 64 (profiles/r5)
    launch_wino_wgrad(x, dy, part, B, g.C, g.Co, g.H, imgs, s);
    if (dw != nullptr) {
      const int64_t n = (int64_t)g.Co * g.C * 9;
      hipLaunchKernelGGL(conv_slab_sum_kernel, dim3((unsigned)((n / 4 + 15) / 16)), dim3(256), 0, s, part, dw, n,
                         B / imgs);
    }
    return;
  }
  // the layer2 3x3 classes likewise when their grad-x takes the Winograd kernel: the 3x3 class at
  // every batch (with / without, ms/step: batch 64 0.7381 / 0.7371 vs 0.7493 / 0.7495, 256
  // 1.0539 / 1.0572 vs 1.0700 / 1.0783, 512 1.4433 / 1.4427 vs 1.4566 / 1.4542); the 3x3/2 class
  // (its grad-x comes from the downsample sibling's backward) up to 256 (128 0.8243 vs 0.8303, 256
  // 1.0196 vs 1.0339, 64 0.7295-0.7439 vs 0.7329-0.7385; 512 1.4504 / 1.4453 vs 1.4470 / 1.4431)
  // The 1x1 stride-2 downsample classes (direct grad-x + direct grad-W, direct_pair_kernel) at every
  // batch: 64 0.7218 / 0.7264 vs 0.7301 / 0.7311, 256 1.0125 vs 1.0256, 512 1.4396 / 1.4355 vs
  // 1.4469 / 1.4360.
  if (pair && dw == nullptr &&
      (((cls == 1 || (cls == 2 && B <= 256)) && conv_wino(cls, g, B, true)) || cls == 4 || cls == 5)) {
    hold_pending(PendingWgrad{x, dy, part, B, imgs, cls, g, s});
    return;
  }
  switch (cls) {
    case 0: run_wgrad<3, 3, 1, 1, 8, 8, 32, 32, 3, 3, 4>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    case 1: run_wgrad<3, 3, 1, 1, 4, 4, 32, 32, 3, 3, 4>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    case 2: run_wgrad<3, 3, 2, 1, 8, 8, 32, 32, 3, 3, 4>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    case 3: run_wgrad<7, 7, 2, 3, 32, 32, 3, 32, 5, 1, 4>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    case 4: run_wgrad<1, 1, 2, 0, 8, 8, 32, 32, 1, 1, 4>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    case 5: run_wgrad<1, 1, 2, 0, 4, 4, 32, 32, 1, 1, 2>(x, dy, part, dw, B, g.C, g.Co, imgs, s); break;
    default: break;
  }
}

}  // namespace ndp
