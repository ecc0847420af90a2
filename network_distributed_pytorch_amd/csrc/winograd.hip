// Winograd F(2x2, 3x3) convolution for ResNet's layer1 shape (3x3, stride 1, pad 1, 8x8 maps),
// exact fp32 arithmetic on v_mfma_f32_16x16x4_f32 (gfx950).
//
// The direct implicit-GEMM kernels (conv.hip) spend 9 MACs per output pixel per input channel;
// F(2x2, 3x3) spends 4 (16 per 2x2 output tile): Y = A^T [ (G g G^T) (.) (B^T d B) ] A with
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1]
// (Lavin & Gray; the transform constants are 0, +-1, +-0.5: no precision is given up beyond the
// reassociation of fp32 sums — same class of rounding as the direct kernels' MFMA order, and
// what cuDNN / MIOpen themselves run for fp32 3x3 convolutions).  The 16 transform-domain
// products are 16 independent GEMMs  M[e][co][tile] = sum_ci U[e][co][ci] V[e][ci][tile].
//
// gfx950 mapping (one workgroup = 4 waves = 4 images x 32 output channels):
//  * wave w owns image w of the tile: its 16 2x2 output tiles are the N = 16 columns of a
//    16x16x4 MFMA, so every lane computes the input transform of ITS OWN tile for its own 4
//    channels (lane = (tile j, channel quad kq): the B operand of MFMA step t is V[e][4kq+t][j])
//    straight from the zero-bordered raw input in LDS: the transformed input never touches LDS
//    or HBM, and no transform is computed twice;
//  * all 16 transform-domain accumulators of the 32 output channels stay in AGPRs (16 e x 2
//    channel blocks x 4 = 128 per lane — the 512-entry gfx950 register file at one wave per
//    SIMD), so the output transform is lane-local register arithmetic: no LDS exchange;
//  * U (the transformed weights, [e][co][ci] with ci contiguous, built per pass by
//    wino_weights_kernel) is staged per 16-channel chunk in LDS and read as one ds_read_b128 per
//    4 MFMAs (row stride 20 floats: the 8 lanes of a b128 phase start in distinct 4-bank groups);
//  * global loads of chunk i+1 are issued before the MFMAs of chunk i (register prefetch, two LDS
//    buffers, one barrier per chunk).
// Epilogues match the direct kernel's: `addend` (a residual-branch gradient added to grad-x),
// and the BatchNorm partial sums of the output (forward: sum / sum of squares; backward mode:
// sum dz / sum dz * xhat with dz = (by > 0) ? v : 0) per (channel, 4-image tile) in the
// [c][s][2] fp64 layout the BN kernels fold in a fixed order (deterministic).
// Grad-x of the same conv runs this kernel with U' = the transform of the flipped, transposed
// weights (conv of dY with w'[c][k][r][s] = w[k][c][2-r][2-s]).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <string>

#include "ndp_kernels.h"

namespace ndp {

namespace {

typedef float f32x4w __attribute__((ext_vector_type(4)));
typedef float f32x2w __attribute__((ext_vector_type(2)));

constexpr int kWImgs = 4;      // images per workgroup (one per wave)
constexpr int kWCK = 16;       // input channels per chunk
// Output channels per workgroup: one 16-row MFMA block.  The 16 transform-domain accumulators
// then take 64 AGPRs and the kernel fits two waves per SIMD (two workgroups per CU, single LDS
// buffers): one wave's input transform / staging overlaps the other's MFMAs.  (32 channels =
// 128 AGPRs at one wave per SIMD with double-buffered LDS left the MFMA pipe ~11 % busy: every
// phase of a chunk — global wait, LDS stores, barrier, transform — ran exposed; PMC round 5.)
constexpr int kWBM = 16;
// Raw input planes in LDS: 10 x 10 zero-bordered, each row stored de-interleaved (padded column c
// at (c & 1) * 5 + c / 2), row stride 10, plane stride 100 (= 4 mod 32).  A patch read of a
// half-wave (16 tiles (ty, tx) x 2 channel quads) then lands on 32 distinct banks: tile offsets
// 20 ty + tx cover 16 banks, the second quad (4 planes on) the other 16.  (Interleaved rows put
// the stride-2 tile starts on even banks only: 3-way conflicts, 46-55 % of LDS cycles, PMC.)
constexpr int kWRW = 10;
constexpr int kWPL = 100;
constexpr int kWIMG = kWCK * kWPL;
constexpr int kWXS = kWImgs * kWIMG;       // raw input floats per buffer
constexpr int kWLDU = 20;                  // U row stride (16 ci + 4)
constexpr int kWUS = 16 * kWBM * kWLDU;    // U floats per buffer
constexpr int kWNB = 1;                    // LDS buffers
constexpr int kWUPT = 16 * kWBM * kWCK / 4 / 256;  // U float4 per thread per chunk
constexpr size_t kWLds = (size_t)kWNB * (kWXS + kWUS) * sizeof(float);

__device__ __forceinline__ constexpr int wcpos(int c) { return (c & 1) * 5 + (c >> 1); }

__device__ __forceinline__ f32x4w mfma16(float a, float b, f32x4w c) {
  // D(16x16) += A(16x4) B(4x16); lane l: A[l&15][l>>4], B[l>>4][l&15]; D: col l&15, row 4(l>>4)+reg
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// e-permutation of the flipped-weight transform: G J3 = P G with P swapping rows 0 and 3, so
// G flip(g) G^T = P (G g G^T) P^T, i.e. U'[e] = U[pi(e)] with pi swapping 0 <-> 3 in both 4-digit
// halves of e = 4u + v
__device__ __forceinline__ int wino_pi(int e) {
  const int uu = e >> 2, vv = e & 3;
  return 4 * (uu == 0 ? 3 : uu == 3 ? 0 : uu) + (vv == 0 ? 3 : vv == 3 ? 0 : vv);
}

// u: [16][Cout][Cin] (ci contiguous) — the forward transform, or for grad-x the backward layout
// wino_weights_kernel writes next to it.  IUPS = 2: the input is a 4x4 map staged onto the even
// pixels of the 8x8 interior (grad-x of the stride-2 conv on its zero-inserted dY).
template <int IUPS>
__global__ __launch_bounds__(256, 2) void wino_fwd_kernel(const float* __restrict__ x, const float* __restrict__ u,
                                                       float* __restrict__ y, int Cin, int Cout,
                                                       const float* __restrict__ addend, ConvBnStats st) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Xs = smem;                 // [kWNB][kWXS]
  float* Us = smem + kWNB * kWXS;   // [kWNB][kWUS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, kq = lane >> 4, ty = j >> 2, tx = j & 3;
  const int b0 = blockIdx.x * kWImgs, co0 = blockIdx.y * kWBM;
  const int nchunks = Cin / kWCK;

  for (int i = tid; i < kWNB * kWXS; i += 256) Xs[i] = 0.f;  // zero borders (interiors rewritten per chunk)

  constexpr int IPL = 64 / (IUPS * IUPS), IW = 8 / IUPS;  // input plane floats / row width
  constexpr int XPT = kWImgs * kWCK * IPL / 4 / 256;      // float4 per thread: 4 or 1
  f32x4w rx[XPT], ru[kWUPT];
  auto load = [&](int ch) {
    const int c0 = ch * kWCK;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e4 = tid + 256 * i;
      const int img = e4 / (kWCK * IPL / 4), rem = e4 - img * (kWCK * IPL / 4);
      const int ci = (4 * rem) / IPL, q = 4 * rem - ci * IPL;
      rx[i] = *reinterpret_cast<const f32x4w*>(x + ((int64_t)(b0 + img) * Cin + c0 + ci) * IPL + q);
    }
#pragma unroll
    for (int i = 0; i < kWUPT; ++i) {  // U chunk: 16 e x kWBM co x 16 ci
      const int e4 = tid + 256 * i;
      const int e = e4 / (kWBM * 4), rem = e4 - e * (kWBM * 4), co = rem >> 2, c4 = rem & 3;
      ru[i] = *reinterpret_cast<const f32x4w*>(u + ((int64_t)e * Cout + co0 + co) * Cin + c0 + 4 * c4);
    }
  };
  auto store = [&](int buf) {
    float* X = Xs + buf * kWXS;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e4 = tid + 256 * i;
      const int img = e4 / (kWCK * IPL / 4), rem = e4 - img * (kWCK * IPL / 4);
      const int ci = (4 * rem) / IPL, q = 4 * rem - ci * IPL;
      const int row = q / IW, col = q - row * IW;
      float* d = X + img * kWIMG + ci * kWPL + (IUPS * row + 1) * kWRW;
#pragma unroll
      for (int k = 0; k < 4; ++k) d[wcpos(IUPS * (col + k) + 1)] = rx[i][k];
    }
    float* U = Us + buf * kWUS;
#pragma unroll
    for (int i = 0; i < kWUPT; ++i) {
      const int e4 = tid + 256 * i;
      const int e = e4 / (kWBM * 4), rem = e4 - e * (kWBM * 4), co = rem >> 2, c4 = rem & 3;
      *reinterpret_cast<f32x4w*>(U + (e * kWBM + co) * kWLDU + 4 * c4) = ru[i];
    }
  };

  constexpr int NB = kWBM / 16;  // 16-row channel blocks
  f32x4w acc[16][NB];
#pragma unroll
  for (int e = 0; e < 16; ++e)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[e][b] = f32x4w{0.f, 0.f, 0.f, 0.f};

  load(0);
  __syncthreads();  // zero fill before interior writes
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const int cur = kWNB == 2 ? (ch & 1) : 0;
    if (ch + 1 < nchunks) load(ch + 1);
    const float* X = Xs + cur * kWXS + wave * kWIMG;
    const float* U = Us + cur * kWUS;
    // input transform of this lane's tile for channels 4kq .. 4kq + 3 (all 64 reads issued first)
    float v[4][16];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* p = X + (4 * kq + t) * kWPL + 2 * ty * kWRW + tx;
      float d[1][4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) d[0][r][c] = p[r * kWRW + (c & 1) * 5 + (c >> 1)];
      float s4[4][4];  // B^T d
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s4[0][c] = d[0][0][c] - d[0][2][c];
        s4[1][c] = d[0][1][c] + d[0][2][c];
        s4[2][c] = d[0][2][c] - d[0][1][c];
        s4[3][c] = d[0][1][c] - d[0][3][c];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // (B^T d) B
        v[t][4 * r + 0] = s4[r][0] - s4[r][2];
        v[t][4 * r + 1] = s4[r][1] + s4[r][2];
        v[t][4 * r + 2] = s4[r][2] - s4[r][1];
        v[t][4 * r + 3] = s4[r][1] - s4[r][3];
      }
    }
    // A operands (one ds_read_b128 = 4 MFMA steps) read two e ahead of their MFMAs; the two
    // channel blocks' accumulator chains alternate (16x16x4 f32: 32-cycle issue, 40-cycle
    // dependent latency).  sched_barrier keeps each prefetch ahead of the MFMA group it must
    // overlap — left alone, the scheduler sinks every ds_read next to its first use.
    f32x4w a[3][NB];
    auto lda = [&](int e, int slot) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        a[slot][b] = *reinterpret_cast<const f32x4w*>(U + (e * kWBM + 16 * b + j) * kWLDU + 4 * kq);
    };
    lda(0, 0);
    lda(1, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (e + 2 < 16) lda(e + 2, (e + 2) % 3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[e][b] = mfma16(a[e % 3][b][t], v[t][e], acc[e][b]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (ch + 1 < nchunks) {
      if (kWNB == 1) __syncthreads();  // single buffer: everyone is done reading it
      store(kWNB == 2 ? (cur ^ 1) : 0);
    }
    __syncthreads();
  }

  // output transform Y = A^T M A per (channel, tile), lane-local
  const int img = b0 + wave;
  const bool stats = st.out != nullptr;
  const bool bstats = stats && st.bx != nullptr;
  double ps[NB][4], pq[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * b + 4 * kq + r;
      float m[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) m[e] = acc[e][b][r];
      float t0[4], t1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t0[c] = m[c] + m[4 + c] + m[8 + c];
        t1[c] = m[4 + c] - m[8 + c] - m[12 + c];
      }
      f32x2w y0 = {t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3]};
      f32x2w y1 = {t1[0] + t1[1] + t1[2], t1[1] - t1[2] - t1[3]};
      const int64_t o = ((int64_t)img * Cout + co) * 64 + (2 * ty) * 8 + 2 * tx;
      if (addend != nullptr) {
        y0 += *reinterpret_cast<const f32x2w*>(addend + o);
        y1 += *reinterpret_cast<const f32x2w*>(addend + o + 8);
      }
      *reinterpret_cast<f32x2w*>(y + o) = y0;
      *reinterpret_cast<f32x2w*>(y + o + 8) = y1;
      ps[b][r] = pq[b][r] = 0.0;
      if (bstats) {
        const f32x2w bx0 = *reinterpret_cast<const f32x2w*>(st.bx + o);
        const f32x2w bx1 = *reinterpret_cast<const f32x2w*>(st.bx + o + 8);
        const f32x2w by0 = *reinterpret_cast<const f32x2w*>(st.by + o);
        const f32x2w by1 = *reinterpret_cast<const f32x2w*>(st.by + o + 8);
        const float mu = st.mean[co], is = st.invstd[co];
        const float z0 = by0.x > 0.f ? y0.x : 0.f, z1 = by0.y > 0.f ? y0.y : 0.f;
        const float z2 = by1.x > 0.f ? y1.x : 0.f, z3 = by1.y > 0.f ? y1.y : 0.f;
        ps[b][r] = (double)((z0 + z1) + (z2 + z3));
        pq[b][r] = (double)((z0 * ((bx0.x - mu) * is) + z1 * ((bx0.y - mu) * is)) +
                            (z2 * ((bx1.x - mu) * is) + z3 * ((bx1.y - mu) * is)));
      } else if (stats) {
        ps[b][r] = (double)((y0.x + y0.y) + (y1.x + y1.y));
        pq[b][r] = (double)((y0.x * y0.x + y0.y * y0.y) + (y1.x * y1.x + y1.y * y1.y));
      }
    }
  if (!stats) return;
  // per channel: the 16 tiles of this wave's image (lanes j, fixed xor butterfly), then the 4
  // images in wave order through LDS; S = gridDim.x partials per channel
  double* red = reinterpret_cast<double*>(smem);  // [4 waves][kWBM co][2]; the loop ended on a barrier
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        ps[b][r] += __shfl_xor(ps[b][r], o, 64);
        pq[b][r] += __shfl_xor(pq[b][r], o, 64);
      }
      if (j == 0) {
        const int c = 16 * b + 4 * kq + r;
        red[(wave * kWBM + c) * 2] = ps[b][r];
        red[(wave * kWBM + c) * 2 + 1] = pq[b][r];
      }
    }
  __syncthreads();
  if (tid < kWBM) {
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int w = 0; w < kWImgs; ++w) {
      s0 += red[(w * kWBM + tid) * 2];
      s1 += red[(w * kWBM + tid) * 2 + 1];
    }
    double* dd = st.out + ((int64_t)(co0 + tid) * gridDim.x + blockIdx.x) * 2;
    dd[0] = s0;
    dd[1] = s1;
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
bool wino_ok(int inC, int outC, int B, int H, int W) {
  return H == 8 && W == 8 && inC % kWCK == 0 && outC % kWBM == 0 && B % kWImgs == 0 &&
         (int64_t)(B / kWImgs) * (outC / kWBM) >= 256 && !wino_disabled();
}
int wino_imgs() { return kWImgs; }
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
void launch_wino_conv(const float* x, const float* u, float* y, int B, int inC, int outC, bool transw, int iups,
                      const float* addend, const ConvBnStats& st, hipStream_t s) {
  static bool attr[2] = {false, false};
  const int k = iups == 2 ? 1 : 0;
  if (!attr[k]) {
    hipFuncSetAttribute(k ? reinterpret_cast<const void*>(wino_fwd_kernel<2>)
                          : reinterpret_cast<const void*>(wino_fwd_kernel<1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWLds);
    attr[k] = true;
  }
  const float* uk = transw ? u + 16 * (int64_t)inC * outC : u;
  const dim3 grid((unsigned)(B / kWImgs), (unsigned)(outC / kWBM));
  if (k)
    hipLaunchKernelGGL(wino_fwd_kernel<2>, grid, dim3(256), kWLds, s, x, uk, y, inC, outC, addend, st);
  else
    hipLaunchKernelGGL(wino_fwd_kernel<1>, grid, dim3(256), kWLds, s, x, uk, y, inC, outC, addend, st);
}

}  // namespace ndp
