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
#include "ndp_kernels.h"

namespace ndp {

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

// one thread per weight element: dW[co,ci,kh,kw] = sum_{oh,ow valid} dWt[(co,oh,ow),(ci,ih,iw)]
__global__ __launch_bounds__(256) void toeplitz_fold_kernel(const float* __restrict__ dwt, float* __restrict__ dw,
                                                            ConvGeom g) {
  const int nw = g.Co * g.C * g.KH * g.KW;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= nw) return;
  const int kw = idx % g.KW;
  const int kh = (idx / g.KW) % g.KH;
  const int ci = (idx / (g.KW * g.KH)) % g.C;
  const int co = idx / (g.KW * g.KH * g.C);
  const int K = g.C * g.H * g.W;
  float acc = 0.f;
  for (int oh = 0; oh < g.OH; ++oh) {
    const int ih = oh * g.stride - g.pad + kh;
    if (ih < 0 || ih >= g.H) continue;
    for (int ow = 0; ow < g.OW; ++ow) {
      const int iw = ow * g.stride - g.pad + kw;
      if (iw < 0 || iw >= g.W) continue;
      const int n = (co * g.OH + oh) * g.OW + ow;
      acc += dwt[(int64_t)n * K + (ci * g.H + ih) * g.W + iw];
    }
  }
  dw[idx] = acc;
}

void launch_toeplitz_expand(const float* w, float* wb, const ConvGeom& g, hipStream_t s) {
  const int N = g.Co * g.OH * g.OW, K = g.C * g.H * g.W;
  hipLaunchKernelGGL(toeplitz_expand_kernel, dim3((K + 255) / 256, N), dim3(256), 0, s, w, wb, g);
}

void launch_toeplitz_fold(const float* dwb, float* dw, const ConvGeom& g, hipStream_t s) {
  const int nw = g.Co * g.C * g.KH * g.KW;
  hipLaunchKernelGGL(toeplitz_fold_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, dwb, dw, g);
}

}  // namespace ndp
