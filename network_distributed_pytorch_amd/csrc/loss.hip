// Fused softmax cross-entropy (torch.nn.CrossEntropyLoss, mean over non-ignored rows).
//
// PyTorch-ROCm runs the training loss as log_softmax + nll_loss forward and, in backward, a
// zero fill + nll_loss_backward + log_softmax_backward: five launches per step, and its
// nll_loss_forward reduction alone takes ~15 µs at ResNet's 512 x 1000 logits (profiles/r2/).
// Here:
//   fwd: one wave per row (4 rows per 256-thread workgroup): row max, sum of exp(x - max),
//        lse = max + log(sum) (fp32, butterfly order: the same value on every lane),
//        loss_b = lse - x[t], and the row of the saved gradient dl[b, k] = softmax_k - [k == t]
//        (unscaled).  Rows whose target is ignore_index contribute nothing (0 loss, 0 grad).
//        Row losses go to rowloss[b]; the LAST workgroup to finish (agent-scope counter:
//        plain stores -> release fence -> relaxed add; the last one: acquire fence, same
//        idiom as orth.hip) adds them in row order and writes loss = sum / n_valid and
//        inv = 1 / n_valid, then re-arms the counter (hipGraph-replay safe).
//   bwd: dx = dl * (dloss * inv) — one float4 launch.
// Fixed summation order everywhere: bitwise reproducible.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ndp_kernels.h"

namespace ndp {

typedef float f4ce __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kCeRowsPerWg = 4;
constexpr int kCeRegs = 16;  // row length held in registers: K <= 1024

__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ x, const int64_t* __restrict__ tgt,
                                                     int B, int K, int64_t ignore, float* __restrict__ dl,
                                                     float* __restrict__ rowloss, float* __restrict__ loss,
                                                     float* __restrict__ inv, unsigned* __restrict__ ctr,
                                                     float* __restrict__ acc) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x * kCeRowsPerWg + wave;
  if (b < B) {
    const float* xr = x + (int64_t)b * K;
    float* dr = dl + (int64_t)b * K;
    const int64_t t = tgt[b];
    const bool valid = t != ignore;
    const bool in_range = t >= 0 && t < K;
    float m = -INFINITY, s = 0.f, lse;
    if (K <= 64 * kCeRegs) {  // the row in registers: one load pass (ResNet's 1000 classes)
      float v[kCeRegs];
#pragma unroll
      for (int i = 0; i < kCeRegs; ++i) {
        const int k = lane + 64 * i;
        v[i] = k < K ? xr[k] : -INFINITY;
        m = fmaxf(m, v[i]);
      }
      m = wave_max_f(m);
#pragma unroll
      for (int i = 0; i < kCeRegs; ++i) s += lane + 64 * i < K ? expf(v[i] - m) : 0.f;
      s = wave_sum_f(s);
      lse = m + logf(s);
#pragma unroll
      for (int i = 0; i < kCeRegs; ++i) {
        const int k = lane + 64 * i;
        if (k < K) dr[k] = valid ? expf(v[i] - lse) - (k == t ? 1.f : 0.f) : 0.f;
      }
    } else {
      for (int k = lane; k < K; k += 64) m = fmaxf(m, xr[k]);
      m = wave_max_f(m);
      for (int k = lane; k < K; k += 64) s += expf(xr[k] - m);
      s = wave_sum_f(s);
      lse = m + logf(s);
      for (int k = lane; k < K; k += 64)
        dr[k] = valid ? expf(xr[k] - lse) - (k == t ? 1.f : 0.f) : 0.f;
    }
    if (lane == 0)  // sc1 (write-through) store: read back by the last workgroup below
      __hip_atomic_store(rowloss + b, !valid ? 0.f : (in_range ? lse - xr[t] : __builtin_nanf("")), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // last-arriving workgroup: fixed-order mean over the rows.  The row losses cross workgroups
  // through sc1 stores (drained before the ticket) and agent-scope loads — no release / acquire
  // fence: an agent-scope release writes the XCD's whole L2 back (11.2 -> 10.0 µs at batch 512)
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: the loads below are sc1
  __shared__ float red[2][4];
  float a = 0.f, n = 0.f;
  for (int r = threadIdx.x; r < B; r += 256) {
    a += __hip_atomic_load(rowloss + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    n += tgt[r] != ignore ? 1.f : 0.f;
  }
  a = wave_sum_f(a);
  n = wave_sum_f(n);
  if (lane == 0) {
    red[0][wave] = a;
    red[1][wave] = n;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const float cnt = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    loss[0] = tot / cnt;  // 0 / 0 = NaN when every row is ignored, like PyTorch
    if (acc != nullptr) acc[0] += tot / cnt;  // running loss sum (logging): no separate add launch
    inv[0] = 1.f / cnt;
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ dl, const float* __restrict__ g,
                                                     const float* __restrict__ inv, float* __restrict__ dx,
                                                     int64_t n) {
  const float sc = g[0] * inv[0];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (4 * i + 3 < n) {
    const f4ce v = reinterpret_cast<const f4ce*>(dl)[i];
    reinterpret_cast<f4ce*>(dx)[i] = v * sc;
  } else {
    for (int64_t j = 4 * i; j < n; ++j) dx[j] = dl[j] * sc;
  }
}

void launch_ce_fwd(const float* x, const int64_t* tgt, int B, int K, int64_t ignore, float* dl, float* rowloss,
                   float* loss, float* inv, unsigned* ctr, hipStream_t s, float* acc) {
  const unsigned wgs = (unsigned)((B + kCeRowsPerWg - 1) / kCeRowsPerWg);
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(wgs), dim3(256), 0, s, x, tgt, B, K, ignore, dl, rowloss, loss, inv, ctr,
                     acc);
}

void launch_ce_bwd(const float* dl, const float* g, const float* inv, float* dx, int64_t n, hipStream_t s) {
  const int64_t n4 = (n + 3) / 4;
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, dl, g, inv, dx, n);
}

}  // namespace ndp
