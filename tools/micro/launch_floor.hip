// Per-kernel fixed cost on gfx950 inside a hipGraph: L dependent launches of a kernel that
// does nothing / writes / reads+writes X bytes, replayed R times; prints µs per launch.
// Decides how much a fused (vertical) or grouped (horizontal) launch saves over separate
// kernels in the ResNet step (profiles/r4/launch_floor.md).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/launch_floor.hip -o /tmp/launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_empty(float* p) {
  if (p == nullptr && threadIdx.x == 1000) p[0] = 1.f;  // never true; keeps the argument
}

__global__ __launch_bounds__(256) void k_write(f4* p, int n4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n4) p[i] = f4{1.f, 2.f, 3.f, (float)i};
}

__global__ __launch_bounds__(256) void k_rw(const f4* __restrict__ a, f4* __restrict__ b, int n4) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n4) b[i] = a[i] * 1.0001f;
}

enum Kind { EMPTY, WRITE, RW };

static float run(Kind kind, int grid, size_t bytes, int L, bool graph, float* buf0, float* buf1, hipStream_t s) {
  const int n4 = (int)(bytes / 16);
  auto launch_all = [&]() {
    for (int i = 0; i < L; ++i) {
      if (kind == EMPTY) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, buf0);
      else if (kind == WRITE) hipLaunchKernelGGL(k_write, dim3((n4 + 255) / 256), dim3(256), 0, s, (f4*)buf0, n4);
      else {
        float* a = (i & 1) ? buf1 : buf0;
        float* b = (i & 1) ? buf0 : buf1;
        hipLaunchKernelGGL(k_rw, dim3((n4 + 255) / 256), dim3(256), 0, s, (const f4*)a, (f4*)b, n4);
      }
    }
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 20;
  float ms = 0.f;
  if (graph) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    launch_all();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  } else {
    for (int w = 0; w < 3; ++w) launch_all();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < R; ++r) launch_all();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 1000.f * ms / (R * L);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = 64u << 20;
  float *b0, *b1;
  CK(hipMalloc(&b0, maxb));
  CK(hipMalloc(&b1, maxb));
  CK(hipMemset(b0, 0, maxb));
  CK(hipMemset(b1, 0, maxb));
  const int L = 100;
  printf("| kernel | graph µs/launch | eager µs/launch |\n|---|---:|---:|\n");
  const int grids[] = {1, 256, 1024, 4096};
  for (int g : grids)
    printf("| empty, %d WGs | %.2f | %.2f |\n", g, run(EMPTY, g, 0, L, true, b0, b1, s), run(EMPTY, g, 0, L, false, b0, b1, s));
  const size_t sizes[] = {64u << 10, 1u << 20, 4u << 20, 8u << 20, 32u << 20};
  for (size_t b : sizes)
    printf("| write %zu KiB | %.2f | %.2f |\n", b >> 10, run(WRITE, 0, b, L, true, b0, b1, s),
           run(WRITE, 0, b, L, false, b0, b1, s));
  for (size_t b : sizes)
    printf("| read+write %zu KiB | %.2f | %.2f |\n", b >> 10, run(RW, 0, b, L, true, b0, b1, s),
           run(RW, 0, b, L, false, b0, b1, s));
  CK(hipFree(b0));
  CK(hipFree(b1));
  return 0;
}
