// Winograd F(2x2, 3x3) convolution for ResNet's 3x3 stride-1 pad-1 layers on 8x8 (layer1) and
// 4x4 (layer2) maps, exact fp32 arithmetic on v_mfma_f32_16x16x4_f32 (gfx950).
//
// The direct implicit-GEMM kernels (conv.hip) spend 9 MACs per output pixel per input channel;
// F(2x2, 3x3) spends 4 (16 per 2x2 output tile): Y = A^T [ (G g G^T) (.) (B^T d B) ] A with
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1]
// (Lavin & Gray; the transform constants are 0, +-1, +-0.5: no precision is given up beyond the
// reassociation of fp32 sums — measured 2-3x closer to an fp64 oracle than the direct kernels, and
// what cuDNN / MIOpen themselves run for fp32 3x3 convolutions).  The 16 transform-domain
// products are 16 independent GEMMs  M[e][co][tile] = sum_ci U[e][co][ci] V[e][ci][tile].
//
// gfx950 mapping (one workgroup = 4 waves x 16 output channels; a wave = 16 tiles: one 8x8 image
// or four 4x4 images):
//  * the 16 tiles are the N = 16 columns of a 16x16x4 MFMA, so every lane computes the input
//    transform of ITS OWN tile for its own 4 channels (lane = (tile j, channel quad kq): the B
//    operand of MFMA step t is V[e][4kq+t][j]) — no transform is computed twice and the
//    transformed input never touches LDS or HBM;
//  * a tile's 4x4 input patch = its own 2x2 core (global loads straight into registers, one
//    chunk ahead) + 12 halo values of the 8 neighbour tiles exchanged by DPP row shifts (the 16
//    lanes of a channel quad are one DPP row; lane-constant masks give the zero padding and image
//    boundaries);
//  * the 16 transform-domain accumulators (64 registers) stay in the register file and the
//    output transform is lane-local: two waves per SIMD;
//  * U (the transformed weights, [e][co][ci] with ci contiguous, built once per pass for every
//    Winograd layer of a model by wino_weights_many_kernel, ops/conv.WinoBank) is staged per
//    16-channel chunk in LDS (double-buffered, one barrier per chunk) and read as one
//    ds_read_b128 per 4 MFMAs.
// Epilogues match the direct kernel's: `addend` (a residual-branch gradient added to grad-x),
// and the BatchNorm partial sums of the output (forward: sum / sum of squares; backward mode:
// sum dz / sum dz * xhat with dz = (by > 0) ? v : 0) per (channel, workgroup) in the [c][s][2]
// fp64 layout the BN kernels fold in a fixed order (deterministic).
// Grad-x of the same conv runs this kernel on U' = the transform of the flipped, transposed
// weights, which is a permutation of U (wino_pi), written next to it by the same launch.
// Measured (tools/diag/wino_scan.py, 1x MI355X, batch 512, graph-timed): 64 -> 64 channels on 8x8
// 17.3 us vs 29.9 us direct; 128 -> 128 on 8x8 50.5 vs 89.1 us.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <string>

#include "ndp_kernels.h"
#include "wino_dpp.h"

namespace ndp {

namespace {

template <int H, int IUPS>
__global__ __launch_bounds__(256, 2) void wino_dpp_kernel(WinoConvArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  wino_dpp_body<H, IUPS>(A, make_uint3(blockIdx.x, blockIdx.y, blockIdx.z),
                         make_uint3(gridDim.x, gridDim.y, gridDim.z), smem);
}

// ---- grad-W in the transform domain --------------------------------------------------------
// With Y_tile = A^T (U (.) V) A:  dU_e[co][ci] = sum_(images, tiles) Yh_e[co][tile] V_e[ci][tile],
// Yh = A dY_tile A^T (the 2x2 output gradient of a tile lifted to 4x4), and dW = G^T dU G
// (4x4 -> 3x3): 16 GEMMs with K = tiles, 4 / 9 of the direct grad-W's MACs.  A wave owns a 16 x 16
// (co, ci) block of dW over an image slice: lane (i, kq) lifts the output gradient of channel
// co0 + i and transforms the input of channel ci0 + i for its tile group kq (H = 8: tile row kq,
// 4 tiles; H = 4: tile kq) — the two MFMA operands of the same k — and 16 accumulators (one per e)
// hold the block.  The slice's dW goes back through G^T . G in registers and is written as one
// grad-W slab in the direct kernel's [co][ci][3][3] layout (conv_slab_sum / gradfinish sum the
// slabs in slice order, deterministic).
// RED = 4: the workgroup's 4 waves share ONE block, each over a quarter of the slice's images, and
// are summed through LDS in wave order before the single slab store — 4x fewer (larger) slices
// for the same wave count, i.e. 4x less slab traffic for the grad-W sum.  RED = 1: a wave per
// block (the slice's images all in one wave), for batches the 4-way split does not divide.
struct WinoWgradArgs {
  const float* x;
  const float* dy;
  float* part;
  int Cin, Cout, imgs;
};
constexpr size_t kWgRedLds = (size_t)3 * 16 * 64 * sizeof(f32x4w);  // RED = 4: waves 1..3's blocks
template <int H, int RED = 1>
__device__ __forceinline__ void wino_wgrad_body(const WinoWgradArgs& A, const uint3 bid, float* __restrict__ smem) {
  const float* __restrict__ x = A.x;
  const float* __restrict__ dy = A.dy;
  float* __restrict__ part = A.part;
  const int Cin = A.Cin, Cout = A.Cout;
  int imgs = A.imgs;
  constexpr int TW = H / 2, TPL = TW * TW / 4, HW = H * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 15, kq = lane >> 4;
  // RED waves per block: the block is wave / RED-th of the workgroup's 4 / RED, the images the
  // (wave % RED)-th 1 / RED of the slice's
  const int blk = (int)bid.y * (4 / RED) + wave / RED, nbc = Cin / 16;
  const int cob = blk / nbc, cib = blk - cob * nbc;
  if (cob * 16 >= Cout) return;  // (RED > 1: uniform over the workgroup, before its barrier)
  const int slice = bid.x;
  const int b0 = slice * imgs + (wave % RED) * (imgs / RED);
  imgs /= RED;  // this wave's images
  // tile group kq: H = 8 -> tile row ty = kq (tiles tx = 0..3); H = 4 -> tile (kq / 2, kq % 2)
  const int ty = H == 8 ? kq : kq >> 1, tx0 = H == 8 ? 0 : (kq & 1);
  const float* xp = x + ((int64_t)b0 * Cin + cib * 16 + i) * HW;
  const float* gp = dy + ((int64_t)b0 * Cout + cob * 16 + i) * HW;
  // per image: input rows 2ty - 1 .. 2ty + 2 (zero outside), output-gradient rows 2ty, 2ty + 1
  float xr[2][4][H], gr[2][2][H];
  auto load = [&](int n, float (&xv)[4][H], float (&gv)[2][H]) __attribute__((always_inline)) {
    const float* xa = xp + (int64_t)n * Cin * HW;
    const float* ga = gp + (int64_t)n * Cout * HW;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 2 * ty - 1 + r;
      const bool ok = row >= 0 && row < H;
#pragma unroll
      for (int c4 = 0; c4 < H / 4; ++c4) {
        const f32x4w v = ok ? *reinterpret_cast<const f32x4w*>(xa + row * H + 4 * c4) : f32x4w{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[r][4 * c4 + k] = v[k];
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c4 = 0; c4 < H / 4; ++c4) {
        const f32x4w v = *reinterpret_cast<const f32x4w*>(ga + (2 * ty + r) * H + 4 * c4);
#pragma unroll
        for (int k = 0; k < 4; ++k) gv[r][4 * c4 + k] = v[k];
      }
  };
  f32x4w acc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = f32x4w{0.f, 0.f, 0.f, 0.f};
  auto step = [&](const float (&xv)[4][H], const float (&gv)[2][H]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < TPL; ++s) {
      const int tx = H == 8 ? s : tx0;
      float d[4][4];
      if constexpr (H == 8) {  // tx = s: static columns
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int col = 2 * s - 1 + c;
            d[r][c] = (col >= 0 && col < H) ? xv[r][col < 0 ? 0 : (col >= H ? H - 1 : col)] : 0.f;
          }
      } else {  // tx = kq & 1 (lane constant): columns -1..2 or 1..4 of the 4-wide rows, by select
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          d[r][0] = tx ? xv[r][1] : 0.f;
          d[r][1] = tx ? xv[r][2] : xv[r][0];
          d[r][2] = tx ? xv[r][3] : xv[r][1];
          d[r][3] = tx ? 0.f : xv[r][2];
        }
      }
      float v[16], sd[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // B^T d
        sd[0][c] = d[0][c] - d[2][c];
        sd[1][c] = d[1][c] + d[2][c];
        sd[2][c] = d[2][c] - d[1][c];
        sd[3][c] = d[1][c] - d[3][c];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // (B^T d) B
        v[4 * r + 0] = sd[r][0] - sd[r][2];
        v[4 * r + 1] = sd[r][1] + sd[r][2];
        v[4 * r + 2] = sd[r][2] - sd[r][1];
        v[4 * r + 3] = sd[r][1] - sd[r][3];
      }
      // Yh = A g A^T, A = [1 0; 1 1; 1 -1; 0 -1]
      float g00, g01, g10, g11;
      if constexpr (H == 8) {
        g00 = gv[0][2 * s]; g01 = gv[0][2 * s + 1]; g10 = gv[1][2 * s]; g11 = gv[1][2 * s + 1];
      } else {
        g00 = tx ? gv[0][2] : gv[0][0]; g01 = tx ? gv[0][3] : gv[0][1];
        g10 = tx ? gv[1][2] : gv[1][0]; g11 = tx ? gv[1][3] : gv[1][1];
      }
      const float t[4][2] = {{g00, g01}, {g00 + g10, g01 + g11}, {g00 - g10, g01 - g11}, {-g10, -g11}};
      float yh[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        yh[4 * u + 0] = t[u][0];
        yh[4 * u + 1] = t[u][0] + t[u][1];
        yh[4 * u + 2] = t[u][0] - t[u][1];
        yh[4 * u + 3] = -t[u][1];
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = mfma16(yh[e], v[e], acc[e]);
      __builtin_amdgcn_sched_barrier(0);  // one tile's operands live at a time (else: spills)
    }
  };
  if constexpr (H == 4) {
    load(0, xr[0], gr[0]);
    for (int n = 0; n < imgs; n += 2) {  // two register sets, swapped by unrolling (imgs even or 1)
      if (n + 1 < imgs) load(n + 1, xr[1], gr[1]);
      step(xr[0], gr[0]);
      if (n + 1 >= imgs) break;
      if (n + 2 < imgs) load(n + 2, xr[0], gr[0]);
      step(xr[1], gr[1]);
    }
  } else {  // 8x8: the 48 raw values of a second image in flight spill; two waves per SIMD hide it
    for (int n = 0; n < imgs; ++n) {
      load(n, xr[0], gr[0]);
      step(xr[0], gr[0]);
    }
  }
  if constexpr (RED == 4) {  // waves 1..3 -> LDS, wave 0 adds them in wave order
    auto red = reinterpret_cast<f32x4w (*)[16][64]>(smem);  // [3][16][64]
    if (wave > 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) red[wave - 1][e][lane] = acc[e];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] += red[w][e][lane];
  } else if constexpr (RED == 2) {  // the odd wave of each pair -> LDS, the even one adds it
    auto red = reinterpret_cast<f32x4w (*)[16][64]>(smem);  // [2][16][64]
    if (wave & 1) {
#pragma unroll
      for (int e = 0; e < 16; ++e) red[wave >> 1][e][lane] = acc[e];
    }
    __syncthreads();
    if (wave & 1) return;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] += red[wave >> 1][e][lane];
  }
  // dW = G^T dU G per (co, ci) = (row 4 kq + r, column i) of the block, lane-local
  float* out = part + (int64_t)slice * Cout * Cin * 9;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = cob * 16 + 4 * kq + r, ci = cib * 16 + i;
    float m[4][4];
#pragma unroll
    for (int e = 0; e < 16; ++e) m[e >> 2][e & 3] = acc[e][r];
    float t[3][4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      t[0][v] = m[0][v] + 0.5f * (m[1][v] + m[2][v]);
      t[1][v] = 0.5f * (m[1][v] - m[2][v]);
      t[2][v] = 0.5f * (m[1][v] + m[2][v]) + m[3][v];
    }
    float* o = out + ((int64_t)co * Cin + ci) * 9;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      o[3 * a + 0] = t[a][0] + 0.5f * (t[a][1] + t[a][2]);
      o[3 * a + 1] = 0.5f * (t[a][1] - t[a][2]);
      o[3 * a + 2] = 0.5f * (t[a][1] + t[a][2]) + t[a][3];
    }
  }
}

template <int H, int RED = 1>
__global__ __launch_bounds__(256, 2) void wino_wgrad_kernel(WinoWgradArgs A) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  wino_wgrad_body<H, RED>(A, make_uint3(blockIdx.x, blockIdx.y, 0), smem);
}

// The layer1 backward pair in ONE launch: workgroups [0, n_dgrad) run the grad-x (wino_dpp_body on
// the transposed-weight transform), the rest the Winograd grad-W of the same conv (both read only
// dY / x / U and write disjoint outputs).  At the small per-GPU batches each of the two launches
// fills about half of the CUs; together they run side by side instead of one after the other.
// The grid is linearised x-fastest per part (the hardware's own dispatch order).
template <int RED>
__global__ __launch_bounds__(256, 2) void wino_bwd_pair_kernel(WinoConvArgs A, uint3 ga, WinoWgradArgs W, uint3 gw) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const unsigned na = ga.x * ga.y * ga.z;
  unsigned b = blockIdx.x;
  if (b < na) {
    const uint3 id = make_uint3(b % ga.x, (b / ga.x) % ga.y, b / (ga.x * ga.y));
    wino_dpp_body<8, 1>(A, id, ga, smem);
  } else {
    b -= na;
    wino_wgrad_body<8, RED>(W, make_uint3(b % gw.x, b / gw.x, 0), smem);
  }
}

// u[0 .. 16 Co C):  U[e][co][ci] = (G w[co][ci] G^T)[e]            (forward, ci contiguous)
// u[16 Co C ..):    U'[e][c][k]  = U[pi(e)][k][c]                  (grad-x: the flipped,
//                   transposed weights' transform, k contiguous)
// Workgroup = one transform row uu x a 16 x 16 (co, ci) block; the grad-x copy goes through an
// LDS transpose so both outputs are written with lanes along their contiguous index.
// (WinoBatch: every Winograd layer of a model in one launch — blockIdx.x runs over all layers'
// 16 x 16 blocks, the layer found from the prefix sums in the kernel arguments)
__device__ __forceinline__ void wino_weights_block(const float* __restrict__ w, float* __restrict__ u, int Co, int C,
                                                   int uu, int blk, float (&tr)[4][16][17]) {
  const int nci = C / 16;
  const int cob = blk / nci, cib = blk - cob * nci;
  const int n = Co * C;
  {
    const int col = threadIdx.x >> 4, cil = threadIdx.x & 15;
    const int co = cob * 16 + col, ci = cib * 16 + cil;
    const float* p = w + ((int64_t)co * C + ci) * 9;
    float g[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) g[r][c] = p[3 * r + c];
    float gg[3];  // row uu of G g
#pragma unroll
    for (int c = 0; c < 3; ++c)
      gg[c] = uu == 0 ? g[0][c] : uu == 3 ? g[2][c] : 0.5f * ((g[0][c] + g[2][c]) + (uu == 1 ? g[1][c] : -g[1][c]));
    float o[4] = {gg[0], 0.5f * ((gg[0] + gg[2]) + gg[1]), 0.5f * ((gg[0] + gg[2]) - gg[1]), gg[2]};
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      u[(int64_t)(4 * uu + v) * n + (int64_t)co * C + ci] = o[v];
      tr[v][cil][col] = o[v];
    }
  }
  __syncthreads();
  const int cil = threadIdx.x >> 4, col = threadIdx.x & 15;
  const int co = cob * 16 + col, ci = cib * 16 + cil;
  float* ub = u + 16 * (int64_t)n;
#pragma unroll
  for (int v = 0; v < 4; ++v) ub[(int64_t)wino_pi(4 * uu + v) * n + (int64_t)ci * Co + co] = tr[v][cil][col];
}

__global__ __launch_bounds__(256) void wino_weights_kernel(const float* __restrict__ w, float* __restrict__ u, int Co,
                                                           int C) {
  __shared__ float tr[4][16][17];
  wino_weights_block(w, u, Co, C, blockIdx.y, blockIdx.x, tr);
}

__global__ __launch_bounds__(256) void wino_weights_many_kernel(WinoBatch b) {
  __shared__ float tr[4][16][17];
  const int blk = blockIdx.x;
  int e = 0;
  while (e + 1 < b.n && blk >= b.end[e]) ++e;
  wino_weights_block(b.w[e], b.u[e], b.Co[e], b.C[e], blockIdx.y, blk - (e ? b.end[e - 1] : 0), tr);
}

}  // namespace

// The Winograd path applies to the layer1 3x3 class (8x8, stride 1, pad 1) — forward, and grad-x
// of that class and of the stride-2 8x8 -> 4x4 class (zero-inserted dY, iups = 2) — when the
// launch is unsplit (the direct kernel's split-K serves small batches) and tiles exactly:
// Cin % 16, Cout % 32, B % 4.
bool wino_ok(int inC, int outC, int B, int H, int W, int ks) {
  const int wimgs = wino_imgs(H);
  return H == W && (H == 8 || H == 4) && inC % kWCK == 0 && (inC / kWCK) % ks == 0 && outC % kWBM == 0 &&
         B % wimgs == 0 && (int64_t)(B / wimgs) * (outC / kWBM) * ks >= 128 && !wino_disabled();
}
// images per workgroup: 4 waves x (16 tiles / tiles per image)
int wino_imgs(int H) { return kWImgs * (H == 4 ? 4 : 1); }
int64_t wino_u_numel(int inC, int outC) { return (int64_t)32 * inC * outC; }  // both layouts

static int g_wino = -1;
bool wino_disabled() {
  if (g_wino < 0) {
    const char* e = getenv("NDP_FUSION_OFF");
    const std::string s = std::string(",") + (e ? e : "") + ",";
    g_wino = (s.find(",winograd,") != std::string::npos || s.find(",all,") != std::string::npos) ? 0 : 1;
  }
  return g_wino == 0;
}
void wino_set_enabled(bool on) { g_wino = on ? 1 : 0; }

void launch_wino_weights(const float* w, float* u, int Co, int C, hipStream_t s) {
  hipLaunchKernelGGL(wino_weights_kernel, dim3((unsigned)((Co / 16) * (C / 16)), 4), dim3(256), 0, s, w, u, Co, C);
}

void launch_wino_weights_many(const WinoBatch& b, hipStream_t s) {
  if (b.n <= 0) return;
  hipLaunchKernelGGL(wino_weights_many_kernel, dim3((unsigned)b.end[b.n - 1], 4), dim3(256), 0, s, b);
}

// y[B][outC][8][8] = conv3x3(x[B][inC][8 / iups][8 / iups] (zero-inserted when iups = 2), W) with
// u = launch_wino_weights(W) of the FORWARD conv (transw: this is its grad-x, inC = Co, outC = C,
// and the kernel reads the grad-x half of u)
template <int H, int IUPS>
static void run_wino(const float* x, const float* u, float* y, int B, int inC, int outC, const float* addend,
                     const ConvBnStats& st, int ks, float* part, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(wino_dpp_kernel<H, IUPS>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWLds);
    attr = true;
  }
  const int64_t slab = (int64_t)B * outC * H * H;
  const WinoConvArgs a{x, u, y, inC, outC, ks > 1 ? nullptr : addend, st, (inC / kWCK) / ks, part, slab};
  hipLaunchKernelGGL((wino_dpp_kernel<H, IUPS>),
                     dim3((unsigned)(B / wino_imgs(H)), (unsigned)(outC / kWBM), (unsigned)ks), dim3(256), kWLds, s, a);
}

// y[B][outC][H][H] = conv3x3(x (zero-inserted 4x4 -> 8x8 when iups = 2), W) with u =
// launch_wino_weights(W) of the FORWARD conv (transw: this is its grad-x, inC = Co, outC = C, and
// the kernel reads the grad-x half of u).  ks > 1: split-K into `part` (ks slabs of y's layout);
// the caller sums them (or leaves them to the consuming BN kernel).
void launch_wino_conv(const float* x, const float* u, float* y, int B, int inC, int outC, int H, bool transw,
                      int iups, const float* addend, const ConvBnStats& st, int ks, float* part, hipStream_t s) {
  const float* uk = transw ? u + 16 * (int64_t)inC * outC : u;
  if (H == 4) run_wino<4, 1>(x, uk, y, B, inC, outC, addend, st, ks, part, s);
  else if (iups == 2) run_wino<8, 2>(x, uk, y, B, inC, outC, addend, st, ks, part, s);
  else run_wino<8, 1>(x, uk, y, B, inC, outC, addend, st, ks, part, s);
}

// grad-W slabs part[B / imgs][Co][C][3][3] of the layer1 class.  8x8 maps only: the 4x4
// instantiation (one tile per lane group and image: a load per 16 MFMAs) measured slower than the
// direct grad-W kernel (conv.hip launch_conv_wgrad) and is not built
bool wino_wgrad_ok(int C, int Co, int H) { return H == 8 && C % 16 == 0 && Co % 16 == 0 && !wino_disabled(); }
// the 4-wave reduction at per-GPU batch <= 128 for slices of imgs % 4 == 0 images, and from 256 for
// 16-image slices (conv.hip conv_wgrad_imgs sizes the slices for it: one workgroup per block and slice)
bool wino_wgrad_red(int B, int imgs) { return imgs % 4 == 0 && (B <= 128 || (B >= 256 && imgs == 16)); }
// waves per (co, ci) block: 4 (above); 2 from batch 512 — the slice's images split over two waves
// summed through LDS: twice the workgroups of RED = 1 at the same slab count, two waves per SIMD
// instead of one (the 8x8 kernel keeps one image's operands in flight and relies on a second wave
// to hide the loads).  ResNet-18 r=4 batch 512: alone even (1.4143 / 1.4147 vs 1.4184 / 1.4140 ms),
// with the layer1 grad-x pair it enables 1.3934 / 1.3966; batch 256: 1.0141 vs 0.9998 (kept at 1)
static int wgrad_red(int B, int C, int Co, int imgs) {
  if (wino_wgrad_red(B, imgs)) return 4;
  return (B >= 512 && imgs % 2 == 0 && ((Co / 16) * (C / 16)) % 2 == 0) ? 2 : 1;
}
void launch_wino_wgrad(const float* x, const float* dy, float* part, int B, int C, int Co, int H, int imgs,
                       hipStream_t s) {
  if (H != 8) return;
  const WinoWgradArgs a{x, dy, part, C, Co, imgs};
  const int red = wgrad_red(B, C, Co, imgs);
  if (red == 4) {
    const dim3 grid((unsigned)(B / imgs), (unsigned)((Co / 16) * (C / 16)));
    hipLaunchKernelGGL((wino_wgrad_kernel<8, 4>), grid, dim3(256), kWgRedLds, s, a);
  } else if (red == 2) {
    const dim3 grid((unsigned)(B / imgs), (unsigned)((Co / 16) * (C / 16) / 2));
    hipLaunchKernelGGL((wino_wgrad_kernel<8, 2>), grid, dim3(256), kWgRedLds, s, a);
  } else {
    const dim3 grid((unsigned)(B / imgs), (unsigned)(((Co / 16) * (C / 16) + 3) / 4));
    hipLaunchKernelGGL((wino_wgrad_kernel<8, 1>), grid, dim3(256), 0, s, a);
  }
}

// grad-x (layer1 class, unsplit or split-K into `part_x`) and grad-W slabs of one conv in one launch
void launch_wino_bwd_pair(const float* dy, const float* u, float* dx, int B, int inC, int outC, const float* addend,
                          const ConvBnStats& st, int ks, float* part_x, const float* x, float* part_w, int imgs,
                          hipStream_t s) {
  // grad-x: inC = the forward's Co (dY channels), outC = the forward's C; grad-W of the forward
  // conv C -> Co: x has outC channels, dY inC
  const float* uk = u + 16 * (int64_t)inC * outC;
  const WinoConvArgs a{dy, uk, dx, inC, outC, ks > 1 ? nullptr : addend, ks > 1 ? ConvBnStats{} : st, (inC / kWCK) / ks,
                       part_x, (int64_t)B * outC * 64};
  const uint3 ga = make_uint3((unsigned)(B / wino_imgs(8)), (unsigned)(outC / kWBM), (unsigned)ks);
  const WinoWgradArgs w{x, dy, part_w, outC, inC, imgs};
  const int C = outC, Co = inC;
  const int red = wgrad_red(B, C, Co, imgs);
  const int nb = (Co / 16) * (C / 16);
  const uint3 gw = make_uint3((unsigned)(B / imgs), (unsigned)(red == 4 ? nb : red == 2 ? nb / 2 : (nb + 3) / 4), 1);
  const unsigned n = ga.x * ga.y * ga.z + gw.x * gw.y;
  const size_t lds = kWLds > kWgRedLds ? kWLds : kWgRedLds;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(wino_bwd_pair_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(wino_bwd_pair_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    hipFuncSetAttribute(reinterpret_cast<const void*>(wino_bwd_pair_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr = true;
  }
  if (red == 4) hipLaunchKernelGGL(wino_bwd_pair_kernel<4>, dim3(n), dim3(256), lds, s, a, ga, w, gw);
  else if (red == 2) hipLaunchKernelGGL(wino_bwd_pair_kernel<2>, dim3(n), dim3(256), lds, s, a, ga, w, gw);
  else hipLaunchKernelGGL(wino_bwd_pair_kernel<1>, dim3(n), dim3(256), lds, s, a, ga, w, gw);
}

}  // namespace ndp
