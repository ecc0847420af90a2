// Multi-tensor / flat-arena kernels for gfx950.
//
//  * seg_reduce: ONE launch that performs any number of (strided multi-slab) reduce-copies:
//      - TensorBuffer pack   (reference: tensor_buffer.py:19 torch.cat, :27-32 pack)
//      - TensorBuffer unpack with the all-reduce mean folded in (reducer.py:167-168)
//      - deterministic split-K sum of the PowerSGD P / Q partial slabs
//    The workgroup -> entry map is a block-prefix table searched in scalar registers.
//  * sgd_momentum: dense-arm torch.optim.SGD(momentum) step with the all-reduce mean
//    folded in (ddp_guide_cifar10/ddp_init.py:57-62,111,125) over the flat gradient arena.
//  * add: EF pack  send = g + e  (ddp_powersgd_guide_cifar10/ddp_init.py:156-157).
//  * delay_ns: wall-clock spin used by the link emulator to pace collectives to a
//    1/10/100 Gb budget on the stream (reference README.md:2 experiments).
//  * checksum: deterministic fp64 sum of a flat buffer (cross-rank divergence detector).
#include <hip/hip_runtime.h>
#include "ndp_kernels.h"
#include "seg_block.h"

namespace ndp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
// the entry table's pointers, re-typed as global (address space 1): read through the table they
// would compile to FLAT accesses, which also wait on the scalar-cache counter
#define NDP_GLOBAL __attribute__((address_space(1)))
__device__ __forceinline__ f32x4 ld4(const float NDP_GLOBAL* p) { return *reinterpret_cast<const f32x4 NDP_GLOBAL*>(p); }
__device__ __forceinline__ void st4(float NDP_GLOBAL* p, f32x4 v) { *reinterpret_cast<f32x4 NDP_GLOBAL*>(p) = v; }

__global__ __launch_bounds__(256) void seg_reduce_kernel(const SegEntry* __restrict__ ents,
                                                         const int64_t* __restrict__ prefix,
                                                         int n_ent) {
  seg_reduce_block(ents, prefix, n_ent, blockIdx.x);
}

__global__ __launch_bounds__(256) void sgd_momentum_vec_kernel(float* __restrict__ x,
                                                               const float* __restrict__ g,
                                                               float* __restrict__ buf,
                                                               int64_t n4, float lr, float mu,
                                                               float div) {
  const bool scale = div != 1.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    // gradient and momentum buffer through non-temporal accesses (each touched once per step; the
    // parameters are cached for the next forward), as in powersgd.hip's update pass
    f32x4 gg = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + 4 * i));
    if (scale) gg = gg / div;
    f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(buf + 4 * i));
    f32x4 xx = ld4(x + 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      b[j] = __fadd_rn(__fmul_rn(b[j], mu), gg[j]);
      xx[j] = fmaf(-lr, b[j], xx[j]);
    }
    __builtin_nontemporal_store(b, reinterpret_cast<f32x4*>(buf + 4 * i));
    st4(x + 4 * i, xx);
  }
}

__global__ __launch_bounds__(256) void sgd_momentum_kernel(float* __restrict__ x,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ buf,
                                                           int64_t start, int64_t n, float lr,
                                                           float mu, float div) {
  for (int64_t i = start + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gg = g[i];
    if (div != 1.0f) gg = gg / div;
    const float b = __fadd_rn(__fmul_rn(buf[i], mu), gg);
    buf[i] = b;
    x[i] = fmaf(-lr, b, x[i]);
  }
}

__global__ __launch_bounds__(256) void add_vec_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ b,
                                                      float* __restrict__ o, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    st4(o + 4 * i, ld4(a + 4 * i) + ld4(b + 4 * i));
}

__global__ __launch_bounds__(256) void add_kernel(const float* __restrict__ a,
                                                  const float* __restrict__ b,
                                                  float* __restrict__ o, int64_t start,
                                                  int64_t n) {
  for (int64_t i = start + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    o[i] = a[i] + b[i];
}

__global__ void delay_kernel(int64_t ticks) {
  // s_memrealtime is the 100 MHz constant-rate clock: 1 tick = 10 ns.  Bounded spin.
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

// ---- device-flag ordering between the compute and comm graphs (utils/graph.py) -------
// A cross-queue hipEvent wait is re-evaluated late when the producing queue runs a long
// train of short kernels (measured: comm-graph work started only after the whole compute
// graph).  Instead, the compute graph bumps a counter with one single-lane kernel and the
// comm graph's first kernel of each piece spins on it (agent-scope acquire, s_sleep), so
// the comm queue reacts within microseconds.  Each wait consumes exactly one bump
// (`seen` is private to the waiting queue), so the same captured graphs replay forever.
// A wall-clock-bounded spin (s_memrealtime, 100 MHz) never hangs the GPU: on timeout it sets
// the error word and proceeds.  The error is STICKY — once set, every later wait proceeds at
// once (a broken ordering costs one timeout, not one per wait) — and it is fatal on the
// host: Communicator.check() raises, the bench's health checks fail the attempt and the
// supervisor falls back (bench.py).  A set error word is also mirrored into a pinned host
// word (host_err), which StepRunner reads before every replay: the run stops at the next
// step, not at the next health-check cadence.  Results of a step run after a timed-out
// wait are never reported.
__global__ void flag_signal_kernel(unsigned* ctr) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void flag_wait_kernel(unsigned* ctr, unsigned* seen, unsigned* err, uint64_t max_ticks,
                                 unsigned* host_err) {
  if (threadIdx.x == 0) {
    const unsigned want = __hip_atomic_load(seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;  // sticky
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __hip_atomic_store(seen, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (host_err != nullptr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
      __hip_atomic_store(host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

void launch_flag_signal(unsigned* ctr, hipStream_t s) {
  hipLaunchKernelGGL(flag_signal_kernel, dim3(1), dim3(64), 0, s, ctr);
}

void launch_flag_wait(unsigned* ctr, unsigned* seen, unsigned* err, int64_t timeout_us, hipStream_t s,
                      unsigned* host_err) {
  const uint64_t ticks = (uint64_t)(timeout_us > 0 ? timeout_us : 0) * 100u;  // 100 MHz clock
  hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, s, ctr, seen, err, ticks, host_err);
}

constexpr int kCkBlocks = 256;

__global__ __launch_bounds__(256) void checksum_partial_kernel(const float* __restrict__ x,
                                                               int64_t n,
                                                               double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)kCkBlocks * 256)
    s += (double)x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void checksum_final_kernel(double* out) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < kCkBlocks; ++i) s += out[1 + i];
    out[0] = s;
  }
}

// ---------------------------------- launchers -------------------------------------
static inline unsigned grid_for(int64_t n, int64_t per_block = 256, int64_t cap = 2048) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void launch_seg_reduce(const SegEntry* entries, const int64_t* block_prefix, int n_entries,
                       int64_t n_blocks, hipStream_t s) {
  if (n_entries <= 0 || n_blocks <= 0) return;
  hipLaunchKernelGGL(seg_reduce_kernel, dim3((unsigned)n_blocks), dim3(256), 0, s, entries,
                     block_prefix, n_entries);
}

void launch_sgd_momentum(float* x, const float* g, float* buf, int64_t n, float lr, float mu,
                         float div, hipStream_t s) {
  if (n <= 0) return;
  int64_t done = 0;
  if (aligned16(x) && aligned16(g) && aligned16(buf)) {
    const int64_t n4 = n / 4;
    if (n4 > 0)
      hipLaunchKernelGGL(sgd_momentum_vec_kernel, dim3(grid_for(n4)), dim3(256), 0, s, x, g, buf,
                         n4, lr, mu, div);
    done = n4 * 4;
  }
  if (done < n)
    hipLaunchKernelGGL(sgd_momentum_kernel, dim3(grid_for(n - done)), dim3(256), 0, s, x, g, buf,
                       done, n, lr, mu, div);
}

void launch_add(const float* a, const float* b, float* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  int64_t done = 0;
  if (aligned16(a) && aligned16(b) && aligned16(out)) {
    const int64_t n4 = n / 4;
    if (n4 > 0)
      hipLaunchKernelGGL(add_vec_kernel, dim3(grid_for(n4)), dim3(256), 0, s, a, b, out, n4);
    done = n4 * 4;
  }
  if (done < n)
    hipLaunchKernelGGL(add_kernel, dim3(grid_for(n - done)), dim3(256), 0, s, a, b, out, done, n);
}

void launch_delay_ns(int64_t ns, hipStream_t s) {
  if (ns <= 0) return;
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, (ns + 9) / 10);
}

void launch_checksum(const float* x, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(checksum_partial_kernel, dim3(kCkBlocks), dim3(256), 0, s, x, n, out + 1);
  hipLaunchKernelGGL(checksum_final_kernel, dim3(1), dim3(64), 0, s, out);
}

}  // namespace ndp
