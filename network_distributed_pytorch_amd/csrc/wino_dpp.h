// The Winograd F(2x2, 3x3) forward / grad-x workgroup body (winograd.hip describes the scheme),
// shared by winograd.hip (its own kernels, the layer1 backward pair) and conv.hip (the layer2
// backward pairs with the direct grad-W kernel).  Device code only; every includer gets its own
// internal-linkage copy.
#pragma once
#include <hip/hip_runtime.h>

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
constexpr int kWLDU = 20;                  // U row stride (16 ci + 4)
constexpr int kWUS = 16 * kWBM * kWLDU;    // U floats per buffer
constexpr int kWUPT = 16 * kWBM * kWCK / 4 / 256;  // U float4 per thread per chunk
constexpr size_t kWLds = (size_t)2 * kWUS * sizeof(float);  // two U buffers

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

// ---- register-halo variant ------------------------------------------------------------------
// The input patch of a tile is its own 2x2 "core" (loaded straight from global memory into
// registers, one chunk ahead) plus the 12 halo values of the 8 neighbouring tiles, exchanged with
// DPP row shifts: a wave's 16 lanes of one channel quad are exactly the 16 tiles of its image
// (lane j = 4 ty + tx), i.e. one DPP row, and out-of-row sources read 0 — the top / bottom zero
// padding for free; the left / right padding is a lane-constant select.  No raw input in LDS: no
// staging stores, no zero fill, no 64 patch reads per chunk (the LDS path's 45 s_waitcnt per
// chunk at lgkmcnt's 15-op depth); only the transformed weights are staged (shared by the 4 waves).
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// (DPP controls: row_shl:n = 0x100 + n, row_shr:n = 0x110 + n; bound_ctrl: out-of-row reads 0)

// H x H output maps (H = 8: layer1; H = 4: layer2, 4 images per wave so the 16 lanes of a channel
// quad are still 16 tiles); IUPS = 2: grad-x of the stride-2 8x8 -> 4x4 conv on its zero-inserted dY
// Split-K (grid z > 1, small batches): workgroup z reduces the input channels [z cps, (z + 1)
// cps) x 16 into slab z of `part` (the output layout; no addend, no statistics) — the consumer sums
// the slabs in z order like the direct kernels' (deterministic).
// (A device function of the workgroup's grid coordinates, so that wino_bwd_pair_kernel can run it
// on one part of a combined grid.)
struct WinoConvArgs {
  const float* x;
  const float* u;
  float* y;
  int Cin, Cout;
  const float* addend;
  ConvBnStats st;
  int cps;
  float* part;
  int64_t slab;
};
template <int H, int IUPS>
__device__ __forceinline__ void wino_dpp_body(const WinoConvArgs& A, const uint3 bid, const uint3 gdim,
                                              float* __restrict__ smem) {
  const float* __restrict__ x = A.x;
  const float* __restrict__ u = A.u;
  float* __restrict__ y = A.y;
  const int Cin = A.Cin, Cout = A.Cout, cps = A.cps;
  const float* __restrict__ addend = A.addend;
  const ConvBnStats& st = A.st;
  float* __restrict__ part = A.part;
  const int64_t slab = A.slab;
  constexpr int TW = H / 2, TPI = TW * TW, IPW = 16 / TPI, HW = H * H;  // tiles per row / image, images per wave
  static_assert((H == 8 || H == 4) && (IUPS == 1 || H == 8), "shapes");
  float* Us = smem;  // [2][kWUS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, kq = lane >> 4;
  const int ii = j / TPI, tj = j - ii * TPI, ty = tj / TW, tx = tj - ty * TW;
  const int b0 = bid.x * kWImgs * IPW, co0 = bid.y * kWBM;
  const int img = b0 + wave * IPW + ii;
  const int nchunks = cps, cz = bid.z * cps;  // chunk range of this split
  constexpr int IPL = HW / (IUPS * IUPS);  // input plane floats

  // core loads: IUPS 1: rows 2ty, 2ty + 1 x columns 2tx, 2tx + 1 of channel 4 kq + t; IUPS 2 (the
  // zero-inserted dY of a stride-2 grad-x): only the core's (0, 0) pixel is nonzero = dY[ty][tx]
  const float* xb = x + ((int64_t)img * Cin + cz * kWCK + 4 * kq) * IPL + (IUPS == 1 ? 2 * H * ty + 2 * tx : TW * ty + tx);
  f32x4w core[2][4];
  auto load_core = [&](int ch, f32x4w (&c)[4]) __attribute__((always_inline)) {
    const float* p = xb + (int64_t)ch * kWCK * IPL;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if constexpr (IUPS == 1) {
        const f32x2w r0 = *reinterpret_cast<const f32x2w*>(p + t * IPL);
        const f32x2w r1 = *reinterpret_cast<const f32x2w*>(p + t * IPL + H);
        c[t] = f32x4w{r0.x, r0.y, r1.x, r1.y};
      } else {
        c[t] = f32x4w{p[t * IPL], 0.f, 0.f, 0.f};
      }
    }
  };
  int ug[kWUPT], ul[kWUPT];
#pragma unroll
  for (int i = 0; i < kWUPT; ++i) {
    const int e4 = tid + 256 * i;
    const int e = e4 / (kWBM * 4), rem = e4 - e * (kWBM * 4), co = rem >> 2, c4 = rem & 3;
    ug[i] = (e * Cout + co0 + co) * Cin + cz * kWCK + 4 * c4;
    ul[i] = (e * kWBM + co) * kWLDU + 4 * c4;
  }
  f32x4w ru[kWUPT];
  auto load_u = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kWUPT; ++i) ru[i] = *reinterpret_cast<const f32x4w*>(u + ug[i] + ch * kWCK);
  };
  auto store_u = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kWUPT; ++i) *reinterpret_cast<f32x4w*>(Us + buf * kWUS + ul[i]) = ru[i];
  };
  // neighbour tiles are lanes j -+ 1 (left / right), j -+ TW (above / below) and j -+ TW -+ 1:
  // lane-constant masks supply the zero padding (and, for H = 4, the image boundaries)
  const bool lok = tx > 0, rok = tx < TW - 1, uok = ty > 0, dok = ty < TW - 1;
  constexpr int U1 = 0x110 + TW, D1 = 0x100 + TW;                          // row_shr / row_shl TW
  constexpr int UL = 0x110 + TW + 1, UR = 0x110 + TW - 1, DL = 0x100 + TW - 1, DR = 0x100 + TW + 1;
  // V[t][e] of this lane's tile for channel 4 kq + t (core c = {c00, c01, c10, c11})
  auto xform = [&](const f32x4w (&c)[4], float (&v)[4][16]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float c00 = c[t][0], c01 = c[t][1], c10 = c[t][2], c11 = c[t][3];
      float d[4][4];
      d[1][1] = c00; d[1][2] = c01; d[2][1] = c10; d[2][2] = c11;
      if constexpr (IUPS == 1) {
        const float u0 = dppf<U1>(c10), u1 = dppf<U1>(c11);          // tile above: its bottom row
        const float w0 = dppf<D1>(c00), w1 = dppf<D1>(c01);          // below: its top row
        const float l1 = dppf<0x111>(c01), l2 = dppf<0x111>(c11);    // left: its right column
        const float r1 = dppf<0x101>(c00), r2 = dppf<0x101>(c10);    // right: its left column
        const float ul = dppf<UL>(c11), ur = dppf<UR>(c10);
        const float dl = dppf<DL>(c01), dr = dppf<DR>(c00);
        d[0][1] = uok ? u0 : 0.f; d[0][2] = uok ? u1 : 0.f;
        d[3][1] = dok ? w0 : 0.f; d[3][2] = dok ? w1 : 0.f;
        d[1][0] = lok ? l1 : 0.f; d[2][0] = lok ? l2 : 0.f;
        d[1][3] = rok ? r1 : 0.f; d[2][3] = rok ? r2 : 0.f;
        d[0][0] = (lok && uok) ? ul : 0.f; d[3][0] = (lok && dok) ? dl : 0.f;
        d[0][3] = (rok && uok) ? ur : 0.f; d[3][3] = (rok && dok) ? dr : 0.f;
      } else {  // only the cores' (0, 0) pixels are nonzero
        d[0][0] = d[0][1] = d[0][2] = d[0][3] = 0.f;
        d[1][0] = d[2][0] = d[3][0] = d[3][2] = 0.f;
        const float w0 = dppf<D1>(c00), r1 = dppf<0x101>(c00), dr = dppf<DR>(c00);
        d[3][1] = dok ? w0 : 0.f;
        d[1][3] = rok ? r1 : 0.f; d[2][3] = 0.f;
        d[3][3] = (rok && dok) ? dr : 0.f;
      }
      float s4[4][4];  // B^T d
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        s4[0][cc] = d[0][cc] - d[2][cc];
        s4[1][cc] = d[1][cc] + d[2][cc];
        s4[2][cc] = d[2][cc] - d[1][cc];
        s4[3][cc] = d[1][cc] - d[3][cc];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // (B^T d) B
        v[t][4 * r + 0] = s4[r][0] - s4[r][2];
        v[t][4 * r + 1] = s4[r][1] + s4[r][2];
        v[t][4 * r + 2] = s4[r][2] - s4[r][1];
        v[t][4 * r + 3] = s4[r][1] - s4[r][3];
      }
    }
  };

  f32x4w acc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = f32x4w{0.f, 0.f, 0.f, 0.f};

  load_core(0, core[0]);
  load_u(0);
  store_u(0);
  __syncthreads();
  auto step = [&](int ch, f32x4w (&cc)[4], f32x4w (&cn)[4]) __attribute__((always_inline)) {
    const bool next = ch + 1 < nchunks;
    if (next) {
      load_core(ch + 1, cn);
      load_u(ch + 1);
    }
    float v[4][16];
    xform(cc, v);
    const float* U = Us + (ch & 1) * kWUS;
    // A operands (one ds_read_b128 = the 4 k-steps of an element) read two elements ahead
    f32x4w a[3];
    auto lda = [&](int e, int slot) __attribute__((always_inline)) {
      a[slot] = *reinterpret_cast<const f32x4w*>(U + (e * kWBM + j) * kWLDU + 4 * kq);
    };
    lda(0, 0);
    lda(1, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (e + 2 < 16) lda(e + 2, (e + 2) % 3);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[e] = mfma16(a[e % 3][t], v[t][e], acc[e]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (next) store_u((ch + 1) & 1);
    __syncthreads();
  };
  for (int ch = 0; ch < nchunks; ch += 2) {  // the two core sets swap (unrolled by two)
    step(ch, core[0], core[1]);
    if (ch + 1 < nchunks) step(ch + 1, core[1], core[0]);
  }
  if (gdim.z > 1) {  // split-K: this slice's partial output
    float* pz = part + (int64_t)bid.z * slab;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 4 * kq + r;
      float m[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) m[e] = acc[e][r];
      float t0[4], t1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t0[c] = m[c] + m[4 + c] + m[8 + c];
        t1[c] = m[4 + c] - m[8 + c] - m[12 + c];
      }
      const int64_t o = ((int64_t)img * Cout + co) * HW + (2 * ty) * H + 2 * tx;
      *reinterpret_cast<f32x2w*>(pz + o) = f32x2w{t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3]};
      *reinterpret_cast<f32x2w*>(pz + o + H) = f32x2w{t1[0] + t1[1] + t1[2], t1[1] - t1[2] - t1[3]};
    }
    return;
  }

  // output transform Y = A^T M A per (channel, tile), lane-local
  const bool stats = st.out != nullptr;
  const bool bstats = stats && st.bx != nullptr;
  double ps[4], pq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + 4 * kq + r;
    float m[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) m[e] = acc[e][r];
    float t0[4], t1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t0[c] = m[c] + m[4 + c] + m[8 + c];
      t1[c] = m[4 + c] - m[8 + c] - m[12 + c];
    }
    f32x2w y0 = {t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3]};
    f32x2w y1 = {t1[0] + t1[1] + t1[2], t1[1] - t1[2] - t1[3]};
    const int64_t o = ((int64_t)img * Cout + co) * HW + (2 * ty) * H + 2 * tx;
    if (addend != nullptr) {
      y0 += *reinterpret_cast<const f32x2w*>(addend + o);
      y1 += *reinterpret_cast<const f32x2w*>(addend + o + H);
    }
    *reinterpret_cast<f32x2w*>(y + o) = y0;
    *reinterpret_cast<f32x2w*>(y + o + H) = y1;
    ps[r] = pq[r] = 0.0;
    if (bstats) {
      const f32x2w bx0 = *reinterpret_cast<const f32x2w*>(st.bx + o);
      const f32x2w bx1 = *reinterpret_cast<const f32x2w*>(st.bx + o + H);
      const f32x2w by0 = *reinterpret_cast<const f32x2w*>(st.by + o);
      const f32x2w by1 = *reinterpret_cast<const f32x2w*>(st.by + o + H);
      const float mu = st.mean[co], is = st.invstd[co];
      const float z0 = by0.x > 0.f ? y0.x : 0.f, z1 = by0.y > 0.f ? y0.y : 0.f;
      const float z2 = by1.x > 0.f ? y1.x : 0.f, z3 = by1.y > 0.f ? y1.y : 0.f;
      ps[r] = (double)((z0 + z1) + (z2 + z3));
      pq[r] = (double)((z0 * ((bx0.x - mu) * is) + z1 * ((bx0.y - mu) * is)) +
                       (z2 * ((bx1.x - mu) * is) + z3 * ((bx1.y - mu) * is)));
    } else if (stats) {
      ps[r] = (double)((y0.x + y0.y) + (y1.x + y1.y));
      pq[r] = (double)((y0.x * y0.x + y0.y * y0.y) + (y1.x * y1.x + y1.y * y1.y));
    }
  }
  if (!stats) return;
  double* red = reinterpret_cast<double*>(smem);  // [4 waves][kWBM co][2]; the loop ended on a barrier
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      ps[r] += __shfl_xor(ps[r], o, 64);
      pq[r] += __shfl_xor(pq[r], o, 64);
    }
    if (j == 0) {
      const int c = 4 * kq + r;
      red[(wave * kWBM + c) * 2] = ps[r];
      red[(wave * kWBM + c) * 2 + 1] = pq[r];
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
    double* dd = st.out + ((int64_t)(co0 + tid) * gdim.x + bid.x) * 2;
    dd[0] = s0;
    dd[1] = s1;
  }
}

}  // namespace
}  // namespace ndp
