// Small-map convolutions (input <= 4x4, output <= 2x2: ResNet layer3 / layer4 on 32x32
// inputs) on v_mfma_f32_16x16x4_f32 — exact f32, NCHW, no W_big, no fold, no vendor GEMM.
//
// On a 2x2 or 1x1 map a convolution is a sum over a handful of (input pixel p, output
// pixel q) pairs, each joined by ONE kernel tap t(p, q) (models/conv_gemm.py has the
// Toeplitz view).  With the geometry a template parameter the pair list is a compile-time
// constant, so each direction is a set of small GEMMs over channels, one per pair, all
// accumulating in registers:
//   forward  Y[b, co, q]  = sum_(p,q) sum_ci X[b, ci, p]  W[co, ci, t(p, q)]
//   grad-x   dX[b, ci, p] = sum_(p,q) sum_co dY[b, co, q] W[co, ci, t(p, q)]
//   grad-W   dW[co, ci, t] = sum_b sum_((p,q): t) dY[b, co, q] X[b, ci, p]
// The weight tile is staged from W's own [co][ci][tap] rows (16-B loads of whole rows when
// every tap is used, the used taps only otherwise), the activation tile from the [b][c][pix]
// rows; the tap gather is LDS index arithmetic folded at compile time.  grad-W lands in W's
// layout directly (every KH*KW tap, structural zeros written): no Toeplitz expand / fold.
//
// Row kernel (forward and grad-x): workgroup tile = TM images x TN output channels x every
// output pixel; the 4 waves split the reduction channels of each LDS chunk (wave w owns
// k-steps w*S .. w*S+S-1 of 4 channels) and add their partial tiles through LDS in wave order
// at the end — the whole reduction of a tile inside one workgroup, deterministic, so the
// epilogue sees final values.  Small batches that cannot fill the 256 CUs split the channels
// over gridDim.z instead, as partial slabs summed in z order by the consumer (the fused BN
// kernel, ops/slablink.py, or conv_slab_sum).
// grad-W kernel: tile = TMC out x TNC in channels x every tap; the waves split the images,
// gridDim.z splits the batch into slabs (summed by ops/gradfinish.py, batched).
//
// LDS images are padded so that every ds_read_b32 of an MFMA operand is conflict-free: a
// half-wave reads 16 lanes along one index and 2 along another; either the 16-lane stride
// is = 2 (mod 32) and the 2-lane stride odd, or the 16-lane stride odd and the 2-lane stride
// = 16 (mod 32) — both put the 32 lanes on 32 distinct banks.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <type_traits>

#include "ndp_kernels.h"

namespace ndp {

namespace {

typedef float f32x4s __attribute__((ext_vector_type(4)));

template <int HI_, int WI_, int KH_, int KW_, int ST_, int PD_>
struct Geo {
  static constexpr int HI = HI_, WI = WI_, KH = KH_, KW = KW_, ST = ST_, PD = PD_;
  static constexpr int OH = (HI + 2 * PD - KH) / ST + 1, OW = (WI + 2 * PD - KW) / ST + 1;
  static constexpr int PI = HI * WI, PO = OH * OW, T = KH * KW;
  static constexpr int tap(int i, int o) {
    const int ih = i / WI, iw = i % WI, oh = o / OW, ow = o % OW;
    const int kh = ih - oh * ST + PD, kw = iw - ow * ST + PD;
    return (kh >= 0 && kh < KH && kw >= 0 && kw < KW) ? kh * KW + kw : -1;
  }
  static constexpr bool used(int t) {
    for (int i = 0; i < PI; ++i)
      for (int o = 0; o < PO; ++o)
        if (tap(i, o) == t) return true;
    return false;
  }
  static constexpr int n_used() {
    int n = 0;
    for (int t = 0; t < T; ++t) n += used(t) ? 1 : 0;
    return n;
  }
  static constexpr int slot(int t) {  // compact index of tap t among the used taps (-1: unused)
    if (t < 0 || !used(t)) return -1;
    int n = 0;
    for (int u = 0; u < t; ++u) n += used(u) ? 1 : 0;
    return n;
  }
  static constexpr int utap(int s) {  // the s-th used tap
    for (int t = 0; t < T; ++t)
      if (used(t) && slot(t) == s) return t;
    return -1;
  }
  static constexpr int NU = n_used();
  static constexpr bool ALL = NU == T;
};

// the ResNet small-map geometries (CIFAR inputs; any channel counts)
using G_3x3_2 = Geo<2, 2, 3, 3, 1, 1>;    // 3x3 on 2x2 (layer3)
using G_3x3_4s2 = Geo<4, 4, 3, 3, 2, 1>;  // 3x3 / 2, 4x4 -> 2x2 (layer3 entry)
using G_1x1_4s2 = Geo<4, 4, 1, 1, 2, 0>;  // 1x1 / 2, 4x4 -> 2x2 (layer3 downsample)
using G_3x3_2s2 = Geo<2, 2, 3, 3, 2, 1>;  // 3x3 / 2, 2x2 -> 1x1 (layer4 entry)
using G_3x3_1 = Geo<1, 1, 3, 3, 1, 1>;    // 3x3 on 1x1: the centre tap (layer4)
using G_1x1_2s2 = Geo<2, 2, 1, 1, 2, 0>;  // 1x1 / 2, 2x2 -> 1x1 (layer4 downsample)
using G_1x1_2 = Geo<2, 2, 1, 1, 1, 0>;    // 1x1 on 2x2 (bottleneck conv1 / conv3, layer3)
using G_1x1_1 = Geo<1, 1, 1, 1, 1, 0>;    // 1x1 on 1x1 (bottleneck, layer4)

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

constexpr int cpad(int need, int mod) {  // smallest v >= need with v % 32 == mod
  int v = need;
  while (v % 32 != mod) ++v;
  return v;
}

__device__ __forceinline__ f32x4s mfma16(float a, float b, f32x4s c) {
  // D(16x16) += A(16x4) B(4x16); lane l: A[l&15][l>>4], B[l>>4][l&15]; D: col l&15, row 4*(l>>4)+r
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, 0x7fffffff, 0x00020000);
}
constexpr uint32_t kOOB = 0xffffffffu;  // past the descriptor's range: the load returns 0
__device__ __forceinline__ f32x4s bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4s, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// ---- fused BatchNorm: coefficient finalization (ndp_kernels.h SmBnF / SmBnB) ---------------
// sum over the R row-tile partials of channel k, field j of a [R][C][W] fp64 table: the loads
// of 8 rows are issued together, the adds stay in row order (the same value in every consumer)
template <int W>
__device__ __forceinline__ double part_sum(const double* part, int R, int C, int k, int j) {
  double t = 0.0;
  int r = 0;
  for (; r + 8 <= R; r += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[((int64_t)(r + u) * C + k) * W + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; r < R; ++r) t += part[((int64_t)r * C + k) * W + j];
  return t;
}

// Forward: mean / invstd from the per-row-tile partial sums (fp64, fixed row order: every
// consumer computes bitwise the same value) or the saved statistics; scale = gamma * invstd,
// shift = beta - mean * scale — the same fp32 formulas as csrc/batchnorm.hip, so a mask or an
// activation recomputed in backward from the saved statistics is bitwise the forward's.
__device__ __forceinline__ void bn_fwd_coef(const SmBnF& f, int k, int C, bool writer, float& s, float& h,
                                            float& mean, float& invstd) {
  if (f.part != nullptr) {
    const double sum = part_sum<2>(f.part, f.R, C, k, 0);
    const double sq = part_sum<2>(f.part, f.R, C, k, 1);
    const double M = f.count;
    const double mu = sum / M;
    double var = sq / M - mu * mu;
    if (var < 0.0) var = 0.0;
    mean = (float)mu;
    invstd = (float)(1.0 / sqrt(var + (double)f.eps));
    if (writer) {
      f.save_mean[k] = mean;
      f.save_invstd[k] = invstd;
      if (f.rmean != nullptr) {
        const double unb = M > 1.0 ? var * M / (M - 1.0) : var;
        f.rmean[k] = (float)((1.0 - f.momentum) * (double)f.rmean[k] + f.momentum * mu);
        f.rvar[k] = (float)((1.0 - f.momentum) * (double)f.rvar[k] + f.momentum * unb);
      }
      if (f.nbt != nullptr && k == 0) f.nbt[0] += 1;
    }
  } else {
    mean = f.save_mean[k];
    invstd = f.save_invstd[k];
  }
  s = (f.gamma ? f.gamma[k] : 1.f) * invstd;
  h = (f.beta ? f.beta[k] : 0.f) - mean * s;
}

// Backward: k1 = gamma * invstd, mean dz, mean dz * xhat (dx = k1 (dz - mdz - xhat mdzx))
__device__ __forceinline__ void bn_bwd_coef(const SmBnB& b, int k, int C, bool writer, float& k1, float& mdz,
                                            float& mdzx) {
  const double sdz = part_sum<4>(b.part, b.R, C, k, 0);
  const double sdzx = part_sum<4>(b.part, b.R, C, k, b.j);
  if (writer) {
    if (b.dgamma) b.dgamma[k] = (float)sdzx;
    if (b.dbeta) b.dbeta[k] = (float)sdz;
  }
  k1 = (b.gamma ? b.gamma[k] : 1.f) * b.invstd[k];
  mdz = (float)(sdz / b.count);
  mdzx = (float)(sdzx / b.count);
}

// coefficient table rows per operand transform (LDS, [row][channel])
__host__ __device__ constexpr int coef_rows(int amode, int amask) {
  return amode == 0 ? 0 : amode <= 2 ? 2 : amode == 3 ? 4 : (amask == 2 ? 7 : 5);
}

// fill coef[row * nch + i] for channels k0 + i, i < nch (the operand's transform)
__device__ __forceinline__ void fill_coefs(const SmOps& o, float* coef, int k0, int nch, int C, bool writer) {
  for (int i = threadIdx.x; i < nch; i += blockDim.x) {
    const int k = k0 + i;
    float s, h, mean, invstd;
    if (o.amode >= 1 && o.amode <= 3) {
      bn_fwd_coef(o.af, k, C, writer, s, h, mean, invstd);
      coef[i] = s;
      coef[nch + i] = h;
      if (o.amode == 3) {
        bn_fwd_coef(o.afd, k, C, writer, s, h, mean, invstd);
        coef[2 * nch + i] = s;
        coef[3 * nch + i] = h;
      }
    } else if (o.amode == 4) {
      float k1, mdz, mdzx;
      bn_bwd_coef(o.ab, k, C, writer, k1, mdz, mdzx);
      coef[i] = k1;
      coef[nch + i] = mdz;
      coef[2 * nch + i] = mdzx;
      coef[3 * nch + i] = o.ab.mean[k];
      coef[4 * nch + i] = o.ab.invstd[k];
      if (o.amask == 2) {
        bn_fwd_coef(o.af, k, C, false, s, h, mean, invstd);
        coef[5 * nch + i] = s;
        coef[6 * nch + i] = h;
      }
    }
  }
}

// one operand element through the transform: x (the raw operand), e1 / e2 (the extra tensors:
// amode 2-3 e1 = residual; amode 4 e1 = BN input c, e2 = mask tensor), channel i of the table
__device__ __forceinline__ float xform(const SmOps& o, const float* coef, int nch, int i, float x, float e1,
                                       float e2) {
  if (o.amode == 1) return fmaxf(fmaf(x, coef[i], coef[nch + i]), 0.f);
  if (o.amode == 2) return fmaxf(fmaf(x, coef[i], coef[nch + i]) + e1, 0.f);
  if (o.amode == 3) return fmaxf(fmaf(x, coef[i], coef[nch + i]) + fmaf(e1, coef[2 * nch + i], coef[3 * nch + i]), 0.f);
  // amode 4
  bool m = true;
  if (o.amask == 1) m = e2 > 0.f;
  else if (o.amask == 2) m = fmaf(e1, coef[5 * nch + i], coef[6 * nch + i]) > 0.f;
  const float dz = m ? x : 0.f;
  const float xh = (e1 - coef[3 * nch + i]) * coef[4 * nch + i];
  return coef[i] * (dz - coef[nch + i] - xh * coef[2 * nch + i]);
}

// ---- row kernel: forward (DIR 0) / grad-x (DIR 1) ------------------------------------------
// operand "act": [B][K][PP] (X for the forward, dY for grad-x), K = reduction channels;
// W [Co][C][T]: forward n = co, k = ci; grad-x n = ci, k = co.  out [B][N][PQ].
template <class G, int DIR, int TM, int TN, int S>
struct RowCfg {
  static constexpr int PP = DIR == 0 ? G::PI : G::PO;
  static constexpr int PQ = DIR == 0 ? G::PO : G::PI;
  static constexpr int tapq(int p, int q) { return DIR == 0 ? G::tap(p, q) : G::tap(q, p); }
  static constexpr int TK = 16 * S;  // channels per LDS chunk: 4 waves x S k-steps x 4
  static constexpr int MB = TM / 16, NB = TN / 16;
  // act image [b][k][p]: 16 lanes along b (RS = 2 mod 32), 2 along k (KS odd)
  static constexpr int KS = PP | 1;
  static constexpr int RS = cpad(TK * KS, 2);
  static constexpr int A_SZ = TM * RS;
  // weight image of the used taps (U, compact slot order); KSW = U | 1 (odd; = T when every
  // tap is used, T in {1, 9}, so a W row stays contiguous in LDS)
  //  forward [n][k][u]: 16 lanes along n (RSW = 2 mod 32), 2 along k (stride KSW, odd)
  //  grad-x  [k][n][u]: 16 lanes along n (stride KSW, odd), 2 along k (RSW = 16 mod 32)
  static constexpr int U = G::NU;
  static constexpr int KSW = U | 1;
  static constexpr int RSW = DIR == 0 ? cpad(TK * KSW, 2) : cpad(TN * KSW, 16);
  static constexpr int W_SZ = DIR == 0 ? TN * RSW : TK * RSW;
  static constexpr int STAGE = (A_SZ + W_SZ + 3) / 4 * 4;
  static constexpr int NACC = MB * NB * PQ;  // f32x4 accumulators per wave
  static constexpr int RED = 4 * NACC * 4 * 64;
  static constexpr int BASE = ((2 * STAGE > RED ? 2 * STAGE : RED) + 3) / 4 * 4;  // floats
  static constexpr int ESTAT = 16 * TN * 4;  // doubles: (wave, l4) x column x 4 sums
  // dynamic LDS: BASE floats | coefficient table (runtime rows x K) | ESTAT doubles
  static size_t lds_bytes(int ncoef_floats) {
    return (size_t)(BASE + (ncoef_floats + 3) / 4 * 4) * 4 + (size_t)ESTAT * 8;
  }
  // global loads per chunk: act = TM rows of TK*PP contiguous floats (16-B vectors)
  static constexpr int AV = TM * TK * PP / 4, A_PER = (AV + 255) / 256;
  // weights: whole rows (every tap used) as 16-B vectors, else one float per used tap
  static constexpr int WCH = DIR == 0 ? TK : TN;    // channels along a tile row of W
  static constexpr int WROWS = DIR == 0 ? TN : TK;  // rows (co) of the tile
  static constexpr int WV = G::ALL ? WROWS * WCH * G::T / 4 : WROWS * WCH * U;
  static constexpr int W_PER = (WV + 255) / 256;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "tile");
  static_assert((TK * PP) % 4 == 0 && (!G::ALL || (WCH * G::T) % 4 == 0), "16-B rows");
  static_assert(!G::ALL || KSW == G::T, "contiguous W rows");
  static_assert(PP >= 4 || PP == 1, "act vectors");
};

struct SmRowArgs {
  const float* act;     // [B][K][PP]
  const float* w;       // [Co][C][KH][KW]
  float* out;           // [B][N][PQ]
  float* part;          // split-K slabs [z][B][N][PQ] (gridDim.z > 1)
  int B, K, N, C, cps;  // cps: reduction channels per split
  int64_t slab;
  SmOps ops;            // fused BN operand transform / epilogue (all modes 0: plain)
};

template <class G, int DIR, int TM, int TN, int S>
__global__ __launch_bounds__(256) void sm_row_kernel(SmRowArgs a) {
  using R = RowCfg<G, DIR, TM, TN, S>;
  constexpr int PP = R::PP, PQ = R::PQ, TK = R::TK, U = R::U, MB = R::MB, NB = R::NB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const SmOps& ops = a.ops;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, l4 = lane >> 4;
  const int n0 = blockIdx.x * TN, b0 = blockIdx.y * TM;
  const int kbeg = blockIdx.z * a.cps;
  const int klen = min(a.K, kbeg + a.cps) - kbeg;  // a multiple of 16; the last chunk may be partial
  const int nchunks = (klen + TK - 1) / TK;
  const int amode = ops.amode;
  const bool origin = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;

  // operand transform coefficients for every reduction channel (finalized here)
  float* coef = smem + R::BASE;
  if (amode != 0) {
    fill_coefs(ops, coef, 0, a.K, a.K, origin);
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t ra = rsrc(a.act), rw = rsrc(a.w);
  const __amdgpu_buffer_rsrc_t re1 = rsrc(amode == 4 ? ops.c : ops.res), re2 = rsrc(ops.mtensor);
  const bool ld1 = amode >= 2, ld2 = amode == 4 && ops.amask == 1;
  const bool wmat = ops.mat != nullptr && amode >= 1 && amode <= 3 && blockIdx.x == 0 && gridDim.z == 1;
  // fixed per-thread load coordinates (only a uniform chunk offset moves)
  uint32_t aoff[R::A_PER];
  int adst[R::A_PER], ach[R::A_PER];
#pragma unroll
  for (int v = 0; v < R::A_PER; ++v) {
    const int e = tid + 256 * v;  // vector index in [TM][TK*PP / 4]
    const int row = e / (TK * PP / 4), j = 4 * (e - row * (TK * PP / 4));
    const int b = b0 + row;
    aoff[v] = (e < R::AV && b < a.B) ? (uint32_t)((((int64_t)b * a.K + kbeg) * PP + j) * 4) : kOOB;
    adst[v] = e < R::AV ? row * R::RS + (j / PP) * R::KS + (j % PP) : -1;
    ach[v] = j / PP;  // channel in the chunk (PP == 1: the first of 4)
  }
  uint32_t woff[R::W_PER];
  int wdst[R::W_PER], wkc[R::W_PER];
#pragma unroll
  for (int v = 0; v < R::W_PER; ++v) {
    const int e = tid + 256 * v;
    const bool ok = e < R::WV;
    int row, tsrc, dcol, ch;  // tile row, source float along the W row, destination column, channel
    if constexpr (G::ALL) {
      row = e / (R::WCH * G::T / 4);
      const int j = 4 * (e - row * (R::WCH * G::T / 4));  // float in the row (contiguous in LDS too)
      tsrc = j;
      dcol = j;
      ch = j / G::T;  // a 16-B vector never straddles a 16-channel boundary
    } else {
      row = e / (R::WCH * U);
      const int r2 = e - row * (R::WCH * U);
      ch = r2 / U;
      const int s = r2 - ch * U;
      tsrc = ch * G::T + G::utap(s);
      dcol = ch * R::KSW + s;
    }
    wkc[v] = DIR == 0 ? ch : row;  // reduction channel of this load inside the chunk
    // forward rows: co = n0 + row, floats from ci = kbeg; grad-x rows: co = kbeg + row, from ci = n0
    const int64_t g = DIR == 0 ? ((int64_t)(n0 + row) * a.C + kbeg) * G::T + tsrc
                               : ((int64_t)(kbeg + row) * a.C + n0) * G::T + tsrc;
    woff[v] = ok ? (uint32_t)(g * 4) : kOOB;
    wdst[v] = ok ? row * R::RSW + dcol : -1;
  }
  // per-chunk advance: act TK channels; weights TK reduction channels (forward: along a row,
  // grad-x: TK rows down)
  const uint32_t astep = TK * PP * 4;
  const uint32_t wstep = DIR == 0 ? TK * G::T * 4 : (uint32_t)(TK * a.C * G::T * 4);

  typedef typename std::conditional<G::ALL, f32x4s, float>::type WVec;
  f32x4s rA[R::A_PER], rE1[R::A_PER], rE2[R::A_PER];
  WVec rW[R::W_PER];
  // channels past the split (a partial last chunk) load as zeros: W zero, operand zero
  auto load = [&](int c) {
#pragma unroll
    for (int v = 0; v < R::A_PER; ++v) {
      const uint32_t o = (aoff[v] == kOOB || c * TK + ach[v] >= klen) ? kOOB : aoff[v] + c * astep;
      rA[v] = bload4(ra, o);
      if (ld1) rE1[v] = bload4(re1, o);
      if (ld2) rE2[v] = bload4(re2, o);
    }
#pragma unroll
    for (int v = 0; v < R::W_PER; ++v) {
      const uint32_t o = (woff[v] == kOOB || c * TK + wkc[v] >= klen) ? kOOB : woff[v] + c * wstep;
      if constexpr (G::ALL) rW[v] = bload4(rw, o);
      else rW[v] = bload1(rw, o);
    }
  };
  auto store = [&](int buf, int c) {
    float* As = smem + buf * R::STAGE;
    float* Ws = As + R::A_SZ;
#pragma unroll
    for (int v = 0; v < R::A_PER; ++v) {
      if (adst[v] < 0) continue;
      f32x4s x = rA[v];
      if (amode != 0 && c * TK + ach[v] < klen) {
        const int k = kbeg + c * TK + ach[v];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = xform(ops, coef, a.K, k + (PP >= 4 ? 0 : q), x[q], rE1[v][q], rE2[v][q]);
        if (wmat && aoff[v] != kOOB)
          *reinterpret_cast<f32x4s*>(reinterpret_cast<char*>(ops.mat) + aoff[v] + c * astep) = x;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) As[adst[v] + (PP >= 4 ? q : q * R::KS)] = x[q];
    }
#pragma unroll
    for (int v = 0; v < R::W_PER; ++v) {
      if (wdst[v] < 0) continue;
      if constexpr (G::ALL) {
#pragma unroll
        for (int q = 0; q < 4; ++q) Ws[wdst[v] + q] = rW[v][q];
      } else {
        Ws[wdst[v]] = rW[v];
      }
    }
  };

  f32x4s acc[MB][NB][PQ];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < PQ; ++q) acc[i][j][q] = f32x4s{0.f, 0.f, 0.f, 0.f};

  if (nchunks > 0) {
    load(0);
    store(0, 0);
    __syncthreads();
  }
  for (int c = 0; c < nchunks; ++c) {
    const int cur = c & 1;
    if (c + 1 < nchunks) load(c + 1);  // in flight during this chunk's MFMAs
    const float* As = smem + cur * R::STAGE;
    const float* Ws = As + R::A_SZ;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int kk = (wave * S + s) * 4 + l4;  // the reduction channel this lane feeds
      float af[MB][PP], bf[NB][U];
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int p = 0; p < PP; ++p) af[i][p] = As[(i * 16 + l16) * R::RS + kk * R::KS + p];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int u = 0; u < U; ++u)
          bf[j][u] = DIR == 0 ? Ws[(j * 16 + l16) * R::RSW + kk * R::KSW + u]
                              : Ws[kk * R::RSW + (j * 16 + l16) * R::KSW + u];
      static_for<0, PP * PQ>([&](auto idx) {
        constexpr int p = decltype(idx)::value / PQ, q = decltype(idx)::value % PQ;
        constexpr int u = G::slot(R::tapq(p, q));
        if constexpr (u >= 0) {
#pragma unroll
          for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[i][j][q] = mfma16(af[i][p], bf[j][u], acc[i][j][q]);
        }
      });
    }
    if (c + 1 < nchunks) store(cur ^ 1, c + 1);  // the other buffer was released by the last barrier
    __syncthreads();
  }

  // the 4 waves' partial tiles -> LDS -> wave w finishes register w (rows 4*l4 + w of each
  // 16-row block), adding the waves in order 0..3
  float* red = smem;
  if (nchunks == 0) __syncthreads();
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < PQ; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(((wave * MB + i) * NB + j) * PQ + q) * 256 + r * 64 + lane] = acc[i][j][q][r];
  __syncthreads();
  const bool split = gridDim.z > 1;
  float* dst = split ? a.part + (int64_t)blockIdx.z * a.slab : a.out;
  const int emode = split ? 0 : ops.emode;
  double es[NB][3];
#pragma unroll
  for (int j = 0; j < NB; ++j) es[j][0] = es[j][1] = es[j][2] = 0.0;
  // epilogue BN statistics of the previous layer (emode 2): its saved forward coefficients
  float em[NB], ei[NB], emd[NB], eid[NB], esc[NB], esh[NB];
  if (emode == 2) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = n0 + j * 16 + l16;
      float t0, t1;
      bn_fwd_coef(ops.ef, n, a.N, false, esc[j], esh[j], em[j], ei[j]);
      if (ops.eds) bn_fwd_coef(ops.efd, n, a.N, false, t0, t1, emd[j], eid[j]);
    }
  }
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int b = b0 + i * 16 + 4 * l4 + wave;
    if (b >= a.B) continue;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int n = n0 + j * 16 + l16;
      float v[PQ];
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += red[(((w * MB + i) * NB + j) * PQ + q) * 256 + wave * 64 + lane];
        v[q] = t;
      }
      const int64_t o = ((int64_t)b * a.N + n) * PQ;
      if (!split && ops.eadd != 0) {
#pragma unroll
        for (int q = 0; q < PQ; ++q) {
          const float ad = ops.addend[o + q];
          v[q] += (ops.eadd == 2) ? ((ops.addmask[o + q] > 0.f) ? ad : 0.f) : ad;
        }
      }
      if constexpr (PQ % 4 == 0) {
#pragma unroll
        for (int q = 0; q < PQ; q += 4)
          *reinterpret_cast<f32x4s*>(dst + o + q) = f32x4s{v[q], v[q + 1], v[q + 2], v[q + 3]};
      } else {
#pragma unroll
        for (int q = 0; q < PQ; ++q) dst[o + q] = v[q];
      }
      if (emode == 1) {
#pragma unroll
        for (int q = 0; q < PQ; ++q) {
          es[j][0] += (double)v[q];
          es[j][1] += (double)v[q] * (double)v[q];
        }
      } else if (emode == 2) {
#pragma unroll
        for (int q = 0; q < PQ; ++q) {
          const float cv = ops.ec[o + q];
          bool m = true;
          if (ops.emask == 1) m = ops.emtensor[o + q] > 0.f;
          else if (ops.emask == 2) m = fmaf(cv, esc[j], esh[j]) > 0.f;
          const float dz = m ? v[q] : 0.f;
          es[j][0] += (double)dz;
          es[j][1] += (double)dz * (double)((cv - em[j]) * ei[j]);
          if (ops.eds) es[j][2] += (double)dz * (double)((ops.ecd[o + q] - emd[j]) * eid[j]);
        }
      }
    }
  }
  if (emode != 0) {
    // column sums over this tile's rows: (wave, l4) partials through LDS, fixed order
    double* est = reinterpret_cast<double*>(smem + R::BASE + (coef_rows(amode, ops.amask) * a.K + 3) / 4 * 4);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < 3; ++e) est[((wave * 4 + l4) * TN + j * 16 + l16) * 4 + e] = es[j][e];
    __syncthreads();
    if (tid < TN) {
      double t[3] = {0.0, 0.0, 0.0};
      for (int g = 0; g < 16; ++g)
#pragma unroll
        for (int e = 0; e < 3; ++e) t[e] += est[(g * TN + tid) * 4 + e];
      const int n = n0 + tid;
      if (emode == 1) {
        ops.epart[((int64_t)blockIdx.y * a.N + n) * 2] = t[0];
        ops.epart[((int64_t)blockIdx.y * a.N + n) * 2 + 1] = t[1];
      } else {
        double* pp = ops.epart + ((int64_t)blockIdx.y * a.N + n) * 4;
        pp[0] = t[0];
        pp[1] = t[1];
        pp[2] = t[2];
        pp[3] = 0.0;
      }
    }
  }
}

// ---- grad-W kernel ---------------------------------------------------------------------------
// dW[co][ci][t] (+ slab z) = sum over this split's images b and the pairs (p, q) with tap t of
// G[b][co][q] A[b][ci][p], G = dY (or its BN-backward transform), A = X (or relu(bn(X))).
// MFMA: M = co (16 lanes), N = ci (16 lanes), K = 4 images.
template <class G, int TMC, int TNC, int S>
struct WgCfg {
  static constexpr int PI = G::PI, PO = G::PO, U = G::NU;
  static constexpr int TB = 16 * S;  // images per LDS chunk
  static constexpr int MB = TMC / 16, NB = TNC / 16;
  // dY image [b][co][q]: 16 lanes along co (KSG = PO | 1, odd), 2 along b (RSG = 16 mod 32)
  static constexpr int KSG = PO | 1, RSG = cpad(TMC * KSG, 16), G_SZ = TB * RSG;
  // X image [b][ci][p]: 16 lanes along ci (KSX = PI | 1), 2 along b (RSX = 16 mod 32)
  static constexpr int KSX = PI | 1, RSX = cpad(TNC * KSX, 16), X_SZ = TB * RSX;
  static constexpr int STAGE = (G_SZ + X_SZ + 3) / 4 * 4;
  static constexpr int NACC = MB * NB * U;
  static constexpr int RED = 4 * NACC * 4 * 64;
  static constexpr int BASE = ((2 * STAGE > RED ? 2 * STAGE : RED) + 3) / 4 * 4;
  static constexpr int COEF = 7 * TMC + 2 * TNC;  // dY transform rows x TMC | X transform rows x TNC
  static constexpr size_t LDS_BYTES = (size_t)(BASE + COEF) * 4;
  static constexpr int GV = TB * TMC * PO / 4, G_PER = (GV + 255) / 256;
  static constexpr int XV = TB * TNC * PI / 4, X_PER = (XV + 255) / 256;
  static_assert((TMC * PO) % 4 == 0 && (TNC * PI) % 4 == 0, "16-B rows");
  static_assert(PO >= 4 || PO == 1, "dY vectors");
  static_assert(PI >= 4 || PI == 1, "X vectors");
};

struct SmWgArgs {
  const float* x;   // [B][C][PI]
  const float* dy;  // [B][Co][PO]
  float* out;       // dW [Co][C][T] (or slab base when gridDim.z > 1)
  int B, C, Co, ips;  // ips: images per split
  int64_t slab;
  SmOps xops;       // X transform (amode 0 / 1; saved statistics)
  SmOps gops;       // dY transform (amode 0 / 4)
};

template <class G, int TMC, int TNC, int S>
__global__ __launch_bounds__(256) void sm_wgrad_kernel(SmWgArgs a) {
  using R = WgCfg<G, TMC, TNC, S>;
  constexpr int PI = R::PI, PO = R::PO, U = R::U, TB = R::TB, MB = R::MB, NB = R::NB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, l4 = lane >> 4;
  const int ci0 = blockIdx.x * TNC, co0 = blockIdx.y * TMC;
  const int bbeg = blockIdx.z * a.ips;
  const int bend = min(a.B, bbeg + a.ips);
  const int nchunks = (bend - bbeg + TB - 1) / TB;
  const int gm = a.gops.amode, xm = a.xops.amode;

  // transform coefficients of this tile's channels (never the writer: statistics, dgamma /
  // dbeta belong to the forward consumer / the grad-x kernel)
  float* gcoef = smem + R::BASE;
  float* xcoef = gcoef + 7 * TMC;
  if (gm != 0 || xm != 0) {
    if (gm != 0) fill_coefs(a.gops, gcoef, co0, TMC, a.Co, false);
    if (xm != 0) fill_coefs(a.xops, xcoef, ci0, TNC, a.C, false);
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t rg = rsrc(a.dy), rx = rsrc(a.x);
  const __amdgpu_buffer_rsrc_t rc = rsrc(a.gops.c), rm = rsrc(a.gops.mtensor);
  const bool ldc = gm == 4, ldm = gm == 4 && a.gops.amask == 1;
  uint32_t goff[R::G_PER], xoff[R::X_PER];
  int gdst[R::G_PER], xdst[R::X_PER], gimg[R::G_PER], ximg[R::X_PER], gch[R::G_PER], xch[R::X_PER];
#pragma unroll
  for (int v = 0; v < R::G_PER; ++v) {
    const int e = tid + 256 * v;
    const int bi = e / (TMC * PO / 4), j = 4 * (e - bi * (TMC * PO / 4));
    const bool ok = e < R::GV;
    gimg[v] = ok ? bi : (1 << 20);
    goff[v] = ok ? (uint32_t)((((int64_t)(bbeg + bi) * a.Co + co0) * PO + j) * 4) : kOOB;
    gdst[v] = ok ? bi * R::RSG + (j / PO) * R::KSG + (j % PO) : -1;
    gch[v] = j / PO;
  }
#pragma unroll
  for (int v = 0; v < R::X_PER; ++v) {
    const int e = tid + 256 * v;
    const int bi = e / (TNC * PI / 4), j = 4 * (e - bi * (TNC * PI / 4));
    const bool ok = e < R::XV;
    ximg[v] = ok ? bi : (1 << 20);
    xoff[v] = ok ? (uint32_t)((((int64_t)(bbeg + bi) * a.C + ci0) * PI + j) * 4) : kOOB;
    xdst[v] = ok ? bi * R::RSX + (j / PI) * R::KSX + (j % PI) : -1;
    xch[v] = j / PI;
  }
  const uint32_t gstep = (uint32_t)((int64_t)TB * a.Co * PO * 4), xstep = (uint32_t)((int64_t)TB * a.C * PI * 4);

  f32x4s rG[R::G_PER], rC[R::G_PER], rM[R::G_PER], rX[R::X_PER];
  auto load = [&](int c) {
    const int left = bend - bbeg - c * TB;  // images of this chunk inside the split
#pragma unroll
    for (int v = 0; v < R::G_PER; ++v) {
      const uint32_t o = (goff[v] == kOOB || gimg[v] >= left) ? kOOB : goff[v] + c * gstep;
      rG[v] = bload4(rg, o);
      if (ldc) rC[v] = bload4(rc, o);
      if (ldm) rM[v] = bload4(rm, o);
    }
#pragma unroll
    for (int v = 0; v < R::X_PER; ++v)
      rX[v] = bload4(rx, (xoff[v] == kOOB || ximg[v] >= left) ? kOOB : xoff[v] + c * xstep);
  };
  auto store = [&](int buf, int c) {
    float* Gs = smem + buf * R::STAGE;
    float* Xs = Gs + R::G_SZ;
    const int left = bend - bbeg - c * TB;
#pragma unroll
    for (int v = 0; v < R::G_PER; ++v) {
      if (gdst[v] < 0) continue;
      f32x4s g = rG[v];
      if (gm != 0 && gimg[v] < left) {  // images past the split stay exact zeros
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = xform(a.gops, gcoef, TMC, gch[v] + (PO >= 4 ? 0 : q), g[q], rC[v][q], rM[v][q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Gs[gdst[v] + (PO >= 4 ? q : q * R::KSG)] = g[q];
    }
#pragma unroll
    for (int v = 0; v < R::X_PER; ++v) {
      if (xdst[v] < 0) continue;
      f32x4s x = rX[v];
      if (xm != 0 && ximg[v] < left) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = xform(a.xops, xcoef, TNC, xch[v] + (PI >= 4 ? 0 : q), x[q], 0.f, 0.f);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[xdst[v] + (PI >= 4 ? q : q * R::KSX)] = x[q];
    }
  };

  f32x4s acc[MB][NB][U];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) acc[i][j][u] = f32x4s{0.f, 0.f, 0.f, 0.f};

  if (nchunks > 0) {
    load(0);
    store(0, 0);
    __syncthreads();
  }
  for (int c = 0; c < nchunks; ++c) {
    const int cur = c & 1;
    if (c + 1 < nchunks) load(c + 1);
    const float* Gs = smem + cur * R::STAGE;
    const float* Xs = Gs + R::G_SZ;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int bb = (wave * S + s) * 4 + l4;  // the image this lane feeds (zero rows past B)
      float gf[MB][PO], xf[NB][PI];
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int q = 0; q < PO; ++q) gf[i][q] = Gs[bb * R::RSG + (i * 16 + l16) * R::KSG + q];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int p = 0; p < PI; ++p) xf[j][p] = Xs[bb * R::RSX + (j * 16 + l16) * R::KSX + p];
      static_for<0, PI * PO>([&](auto idx) {
        constexpr int p = decltype(idx)::value / PO, q = decltype(idx)::value % PO;
        constexpr int u = G::slot(G::tap(p, q));
        if constexpr (u >= 0) {
#pragma unroll
          for (int i = 0; i < MB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[i][j][u] = mfma16(gf[i][q], xf[j][p], acc[i][j][u]);
        }
      });
    }
    if (c + 1 < nchunks) store(cur ^ 1, c + 1);
    __syncthreads();
  }

  float* red = smem;
  if (nchunks == 0) __syncthreads();
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(((wave * MB + i) * NB + j) * U + u) * 256 + r * 64 + lane] = acc[i][j][u][r];
  __syncthreads();
  float* dst = a.out + (int64_t)blockIdx.z * a.slab;
#pragma unroll
  for (int i = 0; i < MB; ++i) {
    const int co = co0 + i * 16 + 4 * l4 + wave;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int ci = ci0 + j * 16 + l16;
      float v[G::T];
#pragma unroll
      for (int t = 0; t < G::T; ++t) v[t] = 0.f;
      static_for<0, U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) s += red[(((w * MB + i) * NB + j) * U + u) * 256 + wave * 64 + lane];
        v[G::utap(u)] = s;
      });
      float* o = dst + ((int64_t)co * a.C + ci) * G::T;
#pragma unroll
      for (int t = 0; t < G::T; ++t) o[t] = v[t];
    }
  }
}

// ---- stage-end BN apply / BN-backward statistics ------------------------------------------------
// [B][C][P] tensors; workgroup = 16 channels x 64 images
constexpr int kBnRows = 64;

__global__ __launch_bounds__(256) void sm_bn_apply_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                          int C, int P, SmOps ops) {
  __shared__ float coef[4 * 16];
  const int c0 = blockIdx.x * 16, b0 = blockIdx.y * kBnRows;
  fill_coefs(ops, coef, c0, 16, C, blockIdx.y == 0);  // row block 0 writes the statistics
  __syncthreads();
  const int per = 16 * P;  // floats of one image in this channel block (contiguous)
  for (int e = threadIdx.x; e < kBnRows * per; e += 256) {
    const int r = e / per, f = e - r * per;
    const int b = b0 + r;
    if (b >= B) break;
    const int i = f / P;
    const int64_t o = ((int64_t)b * C + c0) * P + f;
    const float e1 = ops.res != nullptr ? ops.res[o] : 0.f;
    y[o] = xform(ops, coef, 16, i, x[o], e1, 0.f);
  }
}

__global__ __launch_bounds__(256) void sm_bn_bstats_kernel(const float* __restrict__ dy, int B, int C, int P,
                                                           SmOps ops) {
  __shared__ double red[256][3];
  const int c0 = blockIdx.x * 16, b0 = blockIdx.y * kBnRows;
  // thread = (channel i = tid & 15, row group g = tid >> 4): rows b0 + g, b0 + g + 16, ...
  const int i = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = c0 + i;
  float sc, sh, m, is, md = 0.f, idd = 0.f, t0, t1;
  bn_fwd_coef(ops.ef, c, C, false, sc, sh, m, is);
  if (ops.eds) bn_fwd_coef(ops.efd, c, C, false, t0, t1, md, idd);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int r = g; r < kBnRows; r += 16) {
    const int b = b0 + r;
    if (b >= B) break;
    for (int p = 0; p < P; ++p) {
      const int64_t o = ((int64_t)b * C + c) * P + p;
      const float cv = ops.ec[o];
      bool mk = true;
      if (ops.emask == 1) mk = ops.emtensor[o] > 0.f;
      else if (ops.emask == 2) mk = fmaf(cv, sc, sh) > 0.f;
      const float dz = mk ? dy[o] : 0.f;
      s0 += (double)dz;
      s1 += (double)dz * (double)((cv - m) * is);
      if (ops.eds) s2 += (double)dz * (double)((ops.ecd[o] - md) * idd);
    }
  }
  red[threadIdx.x][0] = s0;
  red[threadIdx.x][1] = s1;
  red[threadIdx.x][2] = s2;
  __syncthreads();
  if (threadIdx.x < 16) {
    double t[3] = {0.0, 0.0, 0.0};
    for (int gg = 0; gg < 16; ++gg)
      for (int e = 0; e < 3; ++e) t[e] += red[gg * 16 + threadIdx.x][e];
    double* pp = ops.epart + ((int64_t)blockIdx.y * C + c0 + threadIdx.x) * 4;
    pp[0] = t[0];
    pp[1] = t[1];
    pp[2] = t[2];
    pp[3] = 0.0;
  }
}

// ---- dispatch ----------------------------------------------------------------------------------
template <typename K>
void set_lds_once(K k, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// LDS chunk depth: the largest S (k-steps per wave per chunk) whose double-buffered stage fits
// 80 KB and whose staging registers stay modest — few, large chunks: each chunk costs a barrier
// and a global round trip that its MFMAs must cover (S = 1 left the layer4 GEMMs latency-bound)
constexpr int kSmStageFloats = 20480;
template <class G, int DIR, int TM, int S>
constexpr bool row_fits() {
  using R = RowCfg<G, DIR, TM, 16, S>;
  return 2 * R::STAGE <= kSmStageFloats && R::A_PER * 12 + R::W_PER * (G::ALL ? 4 : 1) <= 128;
}
template <class G, int DIR, int TM>
constexpr int row_s() {
  return row_fits<G, DIR, TM, 8>() ? 8 : row_fits<G, DIR, TM, 4>() ? 4 : row_fits<G, DIR, TM, 2>() ? 2 : 1;
}
template <class G, int S>
constexpr bool wg_fits() {
  using R = WgCfg<G, 16, 32, S>;
  return 2 * R::STAGE <= kSmStageFloats && R::G_PER * 12 + R::X_PER * 4 <= 128;
}
template <class G>
constexpr int wg_s() {
  return wg_fits<G, 8>() ? 8 : wg_fits<G, 4>() ? 4 : wg_fits<G, 2>() ? 2 : 1;
}

constexpr int kSmFill = 256;    // workgroups for one per CU
constexpr int kSmMaxSplit = 4;  // forward / grad-x slabs: the fused BN kernel sums <= 4 (kMaxFusedSlabs)
constexpr size_t kSmMaxLds = 160 * 1024;

int pow2_split(int base, int chunks, int cap) {
  int ks = 1;
  while (ks * 2 <= cap && base * ks < kSmFill && chunks % (ks * 2) == 0) ks *= 2;
  return ks;
}

// images per row tile: 32 when the grid still fills the chip (and the accumulators fit), else 16
template <class G, int DIR>
int row_tm(int B, int N) {
  constexpr int PQ = DIR == 0 ? G::PO : G::PI;
  if (PQ > 4) return 16;
  return ((B + 31) / 32) * (N / 16) >= kSmFill ? 32 : 16;
}

template <class G, int DIR, int TM>
void run_row(const float* act, const float* w, float* out, float* part, int B, int K, int N, int C, int ks,
             const SmOps& ops, hipStream_t s) {
  constexpr int S = row_s<G, DIR, TM>();
  using R = RowCfg<G, DIR, TM, 16, S>;
  auto k = sm_row_kernel<G, DIR, TM, 16, S>;
  static bool attr = false;
  if (!attr) {
    set_lds_once(k, kSmMaxLds);
    attr = true;
  }
  SmRowArgs a{};
  a.act = act;
  a.w = w;
  a.out = out;
  a.part = part;
  a.B = B;
  a.K = K;
  a.N = N;
  a.C = C;
  a.cps = K / ks;
  a.slab = (int64_t)B * N * (DIR == 0 ? G::PO : G::PI);
  a.ops = ops;
  const size_t lds = R::lds_bytes(coef_rows(ops.amode, ops.amask) * K);
  hipLaunchKernelGGL(k, dim3(N / 16, (B + TM - 1) / TM, ks), dim3(256), lds, s, a);
}

template <class G, int DIR>
int row_splits(int B, int K, int N) {
  const int tm = row_tm<G, DIR>(B, N);
  return pow2_split(((B + tm - 1) / tm) * (N / 16), K / 16, kSmMaxSplit);
}

template <class G, int DIR>
int run_row_any(const float* act, const float* w, float* out, float* part, int B, int K, int N, int C,
                const SmOps& ops, hipStream_t s) {
  const int ks = part != nullptr ? row_splits<G, DIR>(B, K, N) : 1;
  if (row_tm<G, DIR>(B, N) == 32) run_row<G, DIR, 32>(act, w, out, part, B, K, N, C, ks, ops, s);
  else run_row<G, DIR, 16>(act, w, out, part, B, K, N, C, ks, ops, s);
  return ks;
}

template <class G>
int wg_splits(int B, int C, int Co) {
  const int base = (C / 32) * (Co / 16);
  int z = 1;
  while (base * z < kSmFill && B / (z * 2) >= 32 && z < 16) z *= 2;
  return z;
}

template <class G>
void run_wgrad(const float* x, const float* dy, float* out, int B, int C, int Co, int splits, const SmOps& xops,
               const SmOps& gops, hipStream_t s) {
  constexpr int S = wg_s<G>();
  using R = WgCfg<G, 16, 32, S>;
  auto k = sm_wgrad_kernel<G, 16, 32, S>;
  static bool attr = false;
  if (!attr) {
    set_lds_once(k, R::LDS_BYTES);
    attr = true;
  }
  SmWgArgs a{};
  a.x = x;
  a.dy = dy;
  a.out = out;
  a.B = B;
  a.C = C;
  a.Co = Co;
  a.ips = (B + splits - 1) / splits;
  a.slab = (int64_t)Co * C * G::T;
  a.xops = xops;
  a.gops = gops;
  hipLaunchKernelGGL(k, dim3(C / 32, Co / 16, splits), dim3(256), R::LDS_BYTES, s, a);
}

// geometry id of a conv (-1: not a small-map geometry this file covers)
int sm_geo(const ConvGeom& g) {
  auto is = [&](int h, int w, int kh, int kw, int st, int pd) {
    return g.H == h && g.W == w && g.KH == kh && g.KW == kw && g.stride == st && g.pad == pd;
  };
  if (is(2, 2, 3, 3, 1, 1)) return 0;
  if (is(4, 4, 3, 3, 2, 1)) return 1;
  if (is(4, 4, 1, 1, 2, 0)) return 2;
  if (is(2, 2, 3, 3, 2, 1)) return 3;
  if (is(1, 1, 3, 3, 1, 1)) return 4;
  if (is(2, 2, 1, 1, 2, 0)) return 5;
  if (is(2, 2, 1, 1, 1, 0)) return 6;
  if (is(1, 1, 1, 1, 1, 0)) return 7;
  return -1;
}

#define NDP_SM_SWITCH(ID, ...)                     \
  switch (ID) {                                    \
    case 0: { using G = G_3x3_2; __VA_ARGS__; }    \
    case 1: { using G = G_3x3_4s2; __VA_ARGS__; }  \
    case 2: { using G = G_1x1_4s2; __VA_ARGS__; }  \
    case 3: { using G = G_3x3_2s2; __VA_ARGS__; }  \
    case 4: { using G = G_3x3_1; __VA_ARGS__; }    \
    case 5: { using G = G_1x1_2s2; __VA_ARGS__; }  \
    case 6: { using G = G_1x1_2; __VA_ARGS__; }    \
    case 7: { using G = G_1x1_1; __VA_ARGS__; }    \
    default: break;                                \
  }

const SmOps kPlain{};

}  // namespace

int sm_class(const ConvGeom& g) {
  const int id = sm_geo(g);
  if (id < 0) return -1;
  // channel tiles of 16 (row kernels, chunks) and 32 (grad-W in-channel tile)
  if (g.C % 32 || g.Co % 32) return -1;
  return id;
}

int sm_splits(const ConvGeom& g, int B, int dir) {
  const int id = sm_class(g);
  if (id < 0) return 1;
  NDP_SM_SWITCH(id, {
    if (dir == 0) return row_splits<G, 0>(B, g.C, g.Co);
    if (dir == 1) return row_splits<G, 1>(B, g.Co, g.C);
    return wg_splits<G>(B, g.C, g.Co);
  })
  return 1;
}

int sm_rowtile(const ConvGeom& g, int B, int dir) {
  const int id = sm_class(g);
  NDP_SM_SWITCH(id, { return dir == 0 ? row_tm<G, 0>(B, g.Co) : row_tm<G, 1>(B, g.C); })
  return 16;
}

int launch_sm_fwd(const float* x, const float* w, float* y, int B, const ConvGeom& g, float* part, hipStream_t s,
                  bool defer) {
  const int id = sm_class(g);
  int ks = 1;
  NDP_SM_SWITCH(id, { ks = run_row_any<G, 0>(x, w, y, part, B, g.C, g.Co, g.C, kPlain, s); break; })
  if (ks <= 1) return 1;
  if (defer) return ks;  // the consuming fused BN kernel sums the slabs
  launch_slab_sum(part, y, (int64_t)B * g.Co * g.OH * g.OW, ks, s);
  return 1;
}

int launch_sm_dgrad(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, float* part, hipStream_t s,
                    const float* addend, bool defer) {
  const int id = sm_class(g);
  int ks = 1;
  SmOps ops{};
  if (addend != nullptr) {  // applied in the epilogue when unsplit, by the slab sum otherwise
    ops.eadd = 1;
    ops.addend = addend;
  }
  NDP_SM_SWITCH(id, { ks = run_row_any<G, 1>(dy, w, dx, part, B, g.Co, g.C, g.C, ops, s); break; })
  if (ks <= 1) return 1;
  if (defer && addend == nullptr) return ks;
  launch_slab_sum(part, dx, (int64_t)B * g.C * g.H * g.W, ks, s, addend);
  return 1;
}

int launch_sm_wgrad(const float* x, const float* dy, float* out, int B, const ConvGeom& g, hipStream_t s) {
  return launch_sm_wgrad_ops(x, dy, out, B, g, kPlain, kPlain, s);
}

void launch_sm_fwd_ops(const float* x, const float* w, float* y, int B, const ConvGeom& g, const SmOps& ops,
                       hipStream_t s) {
  const int id = sm_class(g);
  NDP_SM_SWITCH(id, { run_row_any<G, 0>(x, w, y, nullptr, B, g.C, g.Co, g.C, ops, s); break; })
}

void launch_sm_dgrad_ops(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, const SmOps& ops,
                         hipStream_t s) {
  const int id = sm_class(g);
  NDP_SM_SWITCH(id, { run_row_any<G, 1>(dy, w, dx, nullptr, B, g.Co, g.C, g.C, ops, s); break; })
}

int launch_sm_wgrad_ops(const float* x, const float* dy, float* out, int B, const ConvGeom& g, const SmOps& xops,
                        const SmOps& gops, hipStream_t s) {
  const int id = sm_class(g);
  int z = 1;
  NDP_SM_SWITCH(id, {
    z = wg_splits<G>(B, g.C, g.Co);
    run_wgrad<G>(x, dy, out, B, g.C, g.Co, z, xops, gops, s);
    break;
  })
  return z;
}

int sm_bstats_rows(int B) { return (B + kBnRows - 1) / kBnRows; }

void launch_sm_bn_apply(const float* x, float* y, int B, int C, int P, const SmOps& ops, hipStream_t s) {
  hipLaunchKernelGGL(sm_bn_apply_kernel, dim3(C / 16, (B + kBnRows - 1) / kBnRows), dim3(256), 0, s, x, y, B, C, P,
                     ops);
}

void launch_sm_bn_bstats(const float* dy, int B, int C, int P, const SmOps& ops, hipStream_t s) {
  hipLaunchKernelGGL(sm_bn_bstats_kernel, dim3(C / 16, (B + kBnRows - 1) / kBnRows), dim3(256), 0, s, dy, B, C, P,
                     ops);
}

#undef NDP_SM_SWITCH

}  // namespace ndp
