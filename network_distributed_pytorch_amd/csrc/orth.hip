// Batched, multi-workgroup, deterministic modified Gram-Schmidt for PowerSGD's P-hat.
//
// Reference: orthogonalize() (ddp_powersgd_guide_cifar10/reducer.py:180-191), a TorchScript
// per-column loop run once per matrix (reducer.py:136-137):
//     col_i /= sqrt(sum(col_i^2)) + eps ;   rest_j -= sum(col_i * rest_j) * col_i
// with the all-reduce mean folded in (reducer.py:128, p_memory /= N).
//
// MI355X design:
//  * ONE launch for every matrix.  Matrix i is split into nwg_i workgroups of 256*RPT rows;
//    each thread keeps its RPT rows x RMAX columns in VGPRs for the whole factorisation
//    (P is read once and written once; every column step is register work + reductions).
//  * One column reduction per step (r cross-workgroup barriers per launch, not 2r - 1): the
//    norm and every projection coefficient of column i come from the same dot products
//    <u_i, v_j>, j >= i, taken before u_i is normalised.
//  * Column reductions: wave butterfly (bitwise-identical in every lane) -> fixed-order LDS
//    combine -> for nwg_i > 1 a fixed-order sum of per-workgroup partial slabs exchanged
//    through the sc1 form of cdna_hip_programming.md §6 Guideline 16 (write-through stores +
//    vmcnt drain + relaxed agent counter; poller: relaxed loads; every slab read an sc1 load,
//    so no fence: round 5's release fence wrote back the L2 at each of the r barriers).  Every workgroup of a matrix, and every
//    rank (same plan), computes the bitwise-identical result: replicas stay consistent.
//  * Partial slabs are double-buffered by barrier parity (a fast workgroup can be at most
//    one barrier ahead).  Counters are never reset (no memset node per launch): every
//    workgroup increments its 64-bit matrix counter exactly once per barrier, so a launch
//    moves it by period = r * nwg and each launch starts on a multiple of the period; a
//    workgroup reads its base on entry (before barrier 0 can complete, so the counter is
//    then in [base, base + nwg)).  Spins are bounded and report through an error word
//    instead of hanging the GPU.
//  * Residency: workgroups are dispatched in grid order, so the barrier can only
//    deadlock if ONE matrix needs more workgroups than the device holds at once.  The
//    plan checks every matrix's workgroup count against orth_coresident_cap() =
//    hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs / 2 (half the device is left to
//    kernels of other streams: backward, RCCL).  A spin that still exceeds `max_spins`
//    sets the error word AND poisons the workgroup's rows of P-hat with NaN, so a
//    timed-out barrier can never silently yield a plausible-but-wrong P-hat; the Python
//    layer reads the error word at its check cadence and raises.
#include <hip/hip_runtime.h>
#include "ndp_kernels.h"

namespace ndp {

__device__ __forceinline__ float wave_sum_o(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int K>
__device__ __forceinline__ void block_sum_o(float (&v)[K], float* red /*[4][K]*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum_o(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) red[wave * K + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((red[k] + red[K + k]) + red[2 * K + k]) + red[3 * K + k];
  __syncthreads();
}

struct OrthCtx {
  float* partial;     // [2][n_items][kMaxRank]
  unsigned long long* ctr;  // [n_mats], 64-bit: never wraps
  unsigned* err;      // [1]
  int n_items;
  unsigned max_spins; // barrier spin bound (s_sleep 2 each) before reporting a timeout
};

// Sum v[] over all workgroups of the matrix (deterministic, identical everywhere).
template <int K>
__device__ __forceinline__ void group_sum(float (&v)[K], float* red, const OrthItem& it, const OrthCtx& cx,
                                          int& bar, unsigned long long base, int* bad) {
  block_sum_o<K>(v, red);
  if (it.nwg == 1) return;
  float* slab = cx.partial + ((size_t)(bar & 1) * cx.n_items + it.slab0) * kMaxRank;
  // payload stored write-through (sc1 = relaxed agent-scope atomic store) and drained by the
  // storing wave; every read of another workgroup's slab below is an sc1 load, so neither a
  // release nor an acquire fence is needed (§6 Guideline 16, sc1 form).  The release fence of
  // the plain-store form wrote back every dirty L2 line at each of the r barriers.
  if (threadIdx.x < K) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if ((int)threadIdx.x == k)
        __hip_atomic_store(slab + it.wg * kMaxRank + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cx.ctr + it.mat, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = base + (unsigned long long)(bar + 1) * (unsigned long long)it.nwg;
    unsigned spins = 0;
    while ((long long)(__hip_atomic_load(cx.ctr + it.mat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > cx.max_spins) {  // report (and poison, below) instead of hanging
        __hip_atomic_fetch_or(cx.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *bad = 1;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: sc1 loads follow
  // sc1 buffer loads (not atomics, which the compiler serialises): all K values of 4 workgroups
  // in flight before their adds (past the slab they return 0 and are not added); the adds keep
  // workgroup order (deterministic)
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, it.nwg * kMaxRank * 4, 0x00020000);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = 0.f;
  int w = 0;
  for (; w < it.nwg; w += 4) {
    float t[4][K];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k)
        t[u][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ((w + u) * kMaxRank + k) * 4, 0, 16));
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (w + u < it.nwg) v[k] += t[u][k];
  }
  ++bar;
}

template <int RMAX, int RPT>
__global__ __launch_bounds__(256) void psgd_orth_mw_kernel(const MatGeom* __restrict__ geom,
                                                           const OrthItem* __restrict__ items,
                                                           float* __restrict__ p, float p_div,
                                                           float eps, OrthCtx cx) {
  __shared__ float red[4 * RMAX];
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;  // published by group_sum's barriers before any read
  const OrthItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const int r = g.r;
  float* P = p + g.p_off;
  const int tid = threadIdx.x;
  __shared__ unsigned long long base_s;
  if (tid == 0 && it.nwg > 1) {
    const unsigned long long period = (unsigned long long)r * (unsigned long long)it.nwg;  // r barriers per launch
    const unsigned long long c0 = __hip_atomic_load(cx.ctr + it.mat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base_s = c0 - c0 % period;
  }
  __syncthreads();
  const unsigned long long base = it.nwg > 1 ? base_s : 0ull;

  float v[RPT][RMAX];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int a = it.row0 + tid + 256 * k;
    const bool ok = a < it.row1;
#pragma unroll
    for (int c = 0; c < RMAX; ++c) v[k][c] = (ok && c < r) ? P[(int64_t)a * r + c] / p_div : 0.f;
  }

  int bar = 0;
  // one reduction per column (r barriers, not 2r - 1): with u = column i before its
  // normalisation, q[j] = <u, v_j> for j >= i gives the norm (j = i) and every projection
  // coefficient at once: v_i = u / (sqrt(q[i]) + eps), v_j -= (q[j] / (sqrt(q[i]) + eps)) v_i
  for (int i = 0; i < r; ++i) {
    float ui[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      ui[k] = 0.f;
#pragma unroll
      for (int c = 0; c < RMAX; ++c)
        if (c == i) ui[k] = v[k][c];
    }
    float q[RMAX];
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      q[j] = 0.f;
#pragma unroll
      for (int k = 0; k < RPT; ++k)
        if (j >= i) q[j] += ui[k] * v[k][j];
    }
    group_sum<RMAX>(q, red, it, cx, bar, base, &bad);
    float qi = 0.f;
#pragma unroll
    for (int c = 0; c < RMAX; ++c)
      if (c == i) qi = q[c];
    const float nrm = sqrtf(qi) + eps;
    float vi[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      vi[k] = ui[k] / nrm;
#pragma unroll
      for (int c = 0; c < RMAX; ++c)
        if (c == i) v[k][c] = vi[k];
    }
#pragma unroll
    for (int j = 0; j < RMAX; ++j) {
      if (j > i && j < r) {
        const float d = q[j] / nrm;
#pragma unroll
        for (int k = 0; k < RPT; ++k) v[k][j] = v[k][j] - d * vi[k];
      }
    }
  }

  __syncthreads();
  const bool poison = bad != 0;
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int a = it.row0 + tid + 256 * k;
    if (a < it.row1) {
#pragma unroll
      for (int c = 0; c < RMAX; ++c)
        if (c < r) P[(int64_t)a * r + c] = poison ? __builtin_nanf("") : v[k][c];
    }
  }
}

int orth_rows_per_thread(int max_rank) {
  if (max_rank <= 8) return 8;
  if (max_rank <= 16) return 4;
  if (max_rank <= 32) return 2;
  return 1;
}

void launch_psgd_orth(const MatGeom* geom, const OrthItem* items, int n_items, int n_mats, float* p,
                      float p_div, float eps, int max_rank, float* partial, unsigned long long* counters,
                      unsigned* err, int n_items_total, unsigned max_spins, hipStream_t s) {
  if (n_items <= 0) return;
  OrthCtx cx{partial, counters, err, n_items_total, max_spins};
  if (max_rank <= 4)
    hipLaunchKernelGGL((psgd_orth_mw_kernel<4, 8>), dim3(n_items), dim3(256), 0, s, geom, items, p, p_div, eps, cx);
  else if (max_rank <= 8)
    hipLaunchKernelGGL((psgd_orth_mw_kernel<8, 8>), dim3(n_items), dim3(256), 0, s, geom, items, p, p_div, eps, cx);
  else if (max_rank <= 16)
    hipLaunchKernelGGL((psgd_orth_mw_kernel<16, 4>), dim3(n_items), dim3(256), 0, s, geom, items, p, p_div, eps, cx);
  else if (max_rank <= 32)
    hipLaunchKernelGGL((psgd_orth_mw_kernel<32, 2>), dim3(n_items), dim3(256), 0, s, geom, items, p, p_div, eps, cx);
  else
    hipLaunchKernelGGL((psgd_orth_mw_kernel<64, 1>), dim3(n_items), dim3(256), 0, s, geom, items, p, p_div, eps, cx);
}

static int occ(const void* fn) {
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, 256, 0) != hipSuccess) blocks = 1;
  return blocks < 1 ? 1 : blocks;
}

int orth_coresident_cap(int max_rank) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return -1;  // no device: the caller falls back to a conservative constant
  int per_cu;
  if (max_rank <= 4) per_cu = occ(reinterpret_cast<const void*>(psgd_orth_mw_kernel<4, 8>));
  else if (max_rank <= 8) per_cu = occ(reinterpret_cast<const void*>(psgd_orth_mw_kernel<8, 8>));
  else if (max_rank <= 16) per_cu = occ(reinterpret_cast<const void*>(psgd_orth_mw_kernel<16, 4>));
  else if (max_rank <= 32) per_cu = occ(reinterpret_cast<const void*>(psgd_orth_mw_kernel<32, 2>));
  else per_cu = occ(reinterpret_cast<const void*>(psgd_orth_mw_kernel<64, 1>));
  return (per_cu * cus) / 2;
}

}  // namespace ndp
