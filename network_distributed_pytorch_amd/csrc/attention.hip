// Fused fp32 multi-head attention (flash-style) for DistilBERT on gfx950.
//
// Reference model: HF DistilBERT MultiHeadSelfAttention (used by
// ddp_powersgd_distillBERT_IMDb/ddp_init.py:150): q/sqrt(dh) @ k^T, key-padding mask
// (masked_fill with finfo.min), softmax, dropout(0.1), @ v.  Done eagerly, every layer
// materialises 16x12x512x512 fp32 score tensors (~200 MB) several times per pass.
//
// Here: q, k, v, o are [B, S, H, D] (the linear layers' natural [B, S, H*D] layout: no
// transposes).  D = 64.  All matmuls run on v_mfma_f32_16x16x4_f32 (exact f32).
//   forward : one wave = 16 queries; per 64-key block: S^T = K Q^T (the key on the MFMA
//             row, the query on the lane), online softmax per lane, O^T += V^T P~^T with the
//             S^T accumulator registers used directly as the B operand (no LDS round trip,
//             cdna_hip_programming.md §3 'accumulator tile as the next MFMA's operand').
//             Saves m and log(l) per query (kept apart: for a fully padded row m is
//             finfo.min and m + log(l) would round back to m).
//   backward: delta = rowsum(dO*O); kernel dKdV (one wave = 16 keys, loop over queries);
//             kernel dQ (one wave = 16 queries, loop over keys).  Two kernels, no atomics:
//             deterministic.
//   dropout : counter-based hash of (seed, b*H+h, q, key) — the same mask is regenerated
//             in backward; kept probabilities are scaled by 1/(1-p) like nn.Dropout.
//   LDS     : tiles are staged ONCE, row-major [token][d] (b128 writes, conflict-free).  The
//             operands that need the transposed view (V^T / dO^T / Q^T / K^T rows d as the A
//             operand) are read as 4 ds_read_b32 from the row layout: lane (g, c16) reads
//             row 4g + r, column c16, and with the 68-float row stride rows 4g and 4(g+1)
//             land 16 banks apart, so each 32-lane half covers the 32 banks.  Same LDS bytes
//             as one b128 from a transposed copy, but no transposing scalar stores (8-way
//             bank conflicts: ~60 % of LDS cycles before, PMC round 4) and half the LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ndp_kernels.h"

namespace ndp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  // D(16x16) += A(16x4) B(4x16): lane l holds A[l&15][l>>4], B[l>>4][l&15];
  // D: col = l&15, row = 4*(l>>4) + reg
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int kD = 64;     // head dim
constexpr int kBK = 64;    // keys per block
constexpr int kLD = 68;    // LDS row stride (floats) for K / V^T tiles
constexpr float kNegBig = -3.4028234663852886e38f;  // torch.finfo(float32).min

__device__ __forceinline__ uint32_t hash4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  // small avalanche hash (murmur3 finaliser rounds); counter-based, stateless
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= (c + 0x165667B1u) * 0xC2B2AE3Du;
  h = (h ^ (h >> 15)) * 0x2C1B3C6Du;
  h ^= (d + 0x27D4EB2Fu) * 0x9E3779B1u;
  h = (h ^ (h >> 13)) * 0x297A2D39u;
  return h ^ (h >> 16);
}

__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t bh, uint32_t q, uint32_t k, uint32_t thr) {
  return hash4(seed, bh, q, k) >= thr;  // thr = p * 2^32
}

// Padding-block map: blkv[j] = 1 if key block j (64 keys) holds an attended key; returns
// whether row b attends to any key at all.  A block with no attended key contributes
// exactly nothing (p = exp(finfo.min - m) == 0) unless the whole row is padding (then HF's
// masked softmax is uniform), so such blocks are skipped — exact, not an approximation.
constexpr int kMaxBlk = 64;   // S <= 4096 gets the map; longer sequences never skip
__device__ __forceinline__ bool scan_mask(const int32_t* __restrict__ mask, int b, int S, int* blkv) {
  if (mask == nullptr) return true;
  if (threadIdx.x < kMaxBlk) blkv[threadIdx.x] = 0;
  __syncthreads();
  int any = 0;
  for (int i = threadIdx.x; i < S; i += blockDim.x)
    if (mask[(int64_t)b * S + i] != 0) {
      any = 1;
      if ((i >> 6) < kMaxBlk) blkv[i >> 6] = 1;   // benign same-value race
    }
  return __syncthreads_or(any) != 0;
}

__device__ __forceinline__ bool skip_block(const int32_t* mask, bool row_any, const int* blkv, int k0) {
  return mask != nullptr && row_any && (k0 >> 6) < kMaxBlk && blkv[k0 >> 6] == 0;
}

struct AttnArgs {
  const float* q; const float* k; const float* v; const int32_t* mask;  // mask [B, S] (1 keep), may be null
  float* o; float* lse;          // lse [2][B, H, S]: row max m, then log(l)
  int B, S, H;
  float scale;                   // 1/sqrt(D)
  const int32_t* seedp;          // device-resident seed (graph-replay safe), may be null
  uint32_t drop_thr;             // drop_thr = 0 -> no dropout
  float drop_scale;              // 1/(1-p)
  int64_t ldq;                   // token row stride (floats) of q / k / v: H*D, or 3*H*D for a packed QKV
};

// ---------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void attn_fwd_kernel(AttnArgs a) {
  const uint32_t seed = (a.drop_thr && a.seedp) ? (uint32_t)*a.seedp : 0u;
  __shared__ __attribute__((aligned(16))) float Ks[kBK * kLD];   // K[key][d]
  __shared__ __attribute__((aligned(16))) float Vs[kBK * kLD];   // V[key][d]
  __shared__ float Mk[kBK];                                      // key mask (1 / 0)
  __shared__ int blkv[kMaxBlk];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const bool row_any = scan_mask(a.mask, b, a.S, blkv);
  const int64_t rs = (int64_t)a.H * kD;                       // row stride of [B,S,H,D]
  const int64_t base = (int64_t)b * a.S * rs + (int64_t)h * kD;
  const int64_t qrs = a.ldq;                                  // q / k / v (+ grads) row stride
  const int64_t qbase = (int64_t)b * a.S * qrs + (int64_t)h * kD;
  const int q = blockIdx.x * 64 + wave * 16 + c16;            // this lane's query
  const bool qok = q < a.S;

  // Q^T as the B operand, pre-scaled: lane (g, c16) holds Q[q][16c + 4g + t]
  float Qr[4][4];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    f32x4 v4 = {0.f, 0.f, 0.f, 0.f};
    if (qok) v4 = *reinterpret_cast<const f32x4*>(a.q + qbase + (int64_t)q * qrs + 16 * cc + 4 * g);
#pragma unroll
    for (int t = 0; t < 4; ++t) Qr[cc][t] = v4[t] * a.scale;
  }
  f32x4 O[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) O[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = kNegBig, l = 0.f;

  for (int k0 = 0; k0 < a.S; k0 += kBK) {
    if (skip_block(a.mask, row_any, blkv, k0)) continue;
    __syncthreads();
    // stage K[k0:k0+64][0:64] and V^T
    for (int idx = threadIdx.x; idx < kBK * (kD / 4); idx += 256) {
      const int kr = idx >> 4, dq = (idx & 15) * 4;
      const int key = k0 + kr;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (key < a.S) {
        kv = *reinterpret_cast<const f32x4*>(a.k + qbase + (int64_t)key * qrs + dq);
        vv = *reinterpret_cast<const f32x4*>(a.v + qbase + (int64_t)key * qrs + dq);
      }
      *reinterpret_cast<f32x4*>(&Ks[kr * kLD + dq]) = kv;
      *reinterpret_cast<f32x4*>(&Vs[kr * kLD + dq]) = vv;
    }
    if (threadIdx.x < kBK) {
      const int key = k0 + threadIdx.x;
      Mk[threadIdx.x] = (key < a.S && (a.mask == nullptr || a.mask[(int64_t)b * a.S + key] != 0)) ? 1.f
                        : (key < a.S ? 0.f : -1.f);  // -1: beyond the sequence (excluded)
    }
    __syncthreads();

    // S^T tiles: rows = key (16kt + 4g + reg), col = query (lane c16)
    f32x4 St[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[(16 * kt + c16) * kLD + 16 * cc + 4 * g]);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma16(kf[t], Qr[cc][t], acc);
      }
      St[kt] = acc;
    }
    // mask + block max
    float bmax = kNegBig;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mk = Mk[16 * kt + 4 * g + r];
        float s = St[kt][r];
        if (mk == 0.f) s = kNegBig;          // HF masked_fill(finfo.min)
        if (mk < 0.f) s = -INFINITY;         // padding past S: contributes nothing
        St[kt][r] = s;
        bmax = fmaxf(bmax, s);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    const float mnew = fmaxf(m, bmax);
    const float alpha = __expf(m - mnew);
    float psum = 0.f;
    float P[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(St[kt][r] - mnew);
        psum += p;
        float pd = p;
        if (a.drop_thr) {
          const int key = k0 + 16 * kt + 4 * g + r;
          pd = keep_elem(seed, (uint32_t)bh, (uint32_t)q, (uint32_t)key, a.drop_thr) ? p * a.drop_scale : 0.f;
        }
        P[kt][r] = pd;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
    // O^T[d][q] = alpha * O^T + V^T P~^T   (A = V^T rows d, B = P~^T: lane group g <-> key 4g+r)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4 acc = O[dt] * alpha;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const float* vr = &Vs[(16 * kt + 4 * g) * kLD + 16 * dt + c16];  // V^T[d][key] = V[key][d]
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma16(vr[r * kLD], P[kt][r], acc);
      }
      O[dt] = acc;
    }
  }
  if (!qok) return;
  const float inv = 1.f / l;
  // O^T tile dt: col = query (c16), rows d = 16dt + 4g + reg -> 4 consecutive d per lane
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    *reinterpret_cast<f32x4*>(a.o + base + (int64_t)q * rs + 16 * dt + 4 * g) = O[dt] * inv;
  if (g == 0) {
    const int64_t i = (int64_t)bh * a.S + q;
    a.lse[i] = m;
    a.lse[(int64_t)a.B * a.H * a.S + i] = __logf(l);
  }
}

// ---------------------------------------------------------------------------------------
// backward.  delta[bh][q] = sum_d dO[q][d] * O[q][d]
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(const float* __restrict__ o, const float* __restrict__ dout,
                                                             float* __restrict__ delta, int B, int S, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per (b, s, h) row
  const int lane = threadIdx.x & 63;
  if (row >= B * S * H) return;
  const int64_t off = (int64_t)row * kD + lane;
  float v = o[off] * dout[off];
#pragma unroll
  for (int x = 32; x > 0; x >>= 1) v += __shfl_xor(v, x, 64);
  if (lane == 0) {
    const int h = row % H, bs = row / H, s = bs % S, b = bs / S;
    delta[((int64_t)b * H + h) * S + s] = v;
  }
}

struct AttnBwdArgs {
  const float* q; const float* k; const float* v; const int32_t* mask; const float* dout;
  const float* lse; const float* delta;
  float* dq; float* dk; float* dv;
  int B, S, H;
  float scale;
  const int32_t* seedp;
  uint32_t drop_thr;
  float drop_scale;
  int64_t ldq;                   // token row stride of q / k / v and dq / dk / dv (o / dout: H*D)
};

// Recompute one 16(query) x 64(key) probability tile in the S^T layout used by the forward:
// lane (g, c16): query = q (lane), keys 16kt + 4g + r.
// dK, dV: one wave owns 16 keys (rows = d on MFMA outputs), loops over all queries.
// One accumulator chain per product: 8 independent dK / dV accumulators are already in flight.
// A two-chain variant (even / odd r summed at the end) passed the fp64 tests but spilled (32 ->
// 232 B/lane scratch) and ran 53 % slower: profiles/r5/attn_chains.md (code at commit 831b94e).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void attn_bwd_dkdv_kernel(AttnBwdArgs a) {
  const uint32_t seed = (a.drop_thr && a.seedp) ? (uint32_t)*a.seedp : 0u;
  __shared__ __attribute__((aligned(16))) float Qs[64 * kLD];    // Q[q][d] (scaled)
  __shared__ __attribute__((aligned(16))) float dOs[64 * kLD];   // dO[q][d]
  __shared__ float Ls[64], LLs[64], Ds[64];
  __shared__ int blkv[kMaxBlk];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const int64_t rs = (int64_t)a.H * kD;
  const int64_t base = (int64_t)b * a.S * rs + (int64_t)h * kD;
  const int64_t qrs = a.ldq;                                  // q / k / v (+ grads) row stride
  const int64_t qbase = (int64_t)b * a.S * qrs + (int64_t)h * kD;
  const int key = blockIdx.x * 64 + wave * 16 + c16;             // this lane's key
  const bool kok = key < a.S;
  const bool row_any = scan_mask(a.mask, b, a.S, blkv);
  if (skip_block(a.mask, row_any, blkv, blockIdx.x * 64)) {      // all-padding keys: zero grads
    if (kok)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        *reinterpret_cast<f32x4*>(a.dk + qbase + (int64_t)key * qrs + 16 * dt + 4 * g) = f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(a.dv + qbase + (int64_t)key * qrs + 16 * dt + 4 * g) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    return;
  }
  const bool kmasked = kok && a.mask != nullptr && a.mask[(int64_t)b * a.S + key] == 0;

  // K and V rows of this lane's key as B operands: lane (g, c16): [key][16c + 4g + t]
  float Kr[4][4], Vr[4][4];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
    if (kok) {
      kv = *reinterpret_cast<const f32x4*>(a.k + qbase + (int64_t)key * qrs + 16 * cc + 4 * g);
      vv = *reinterpret_cast<const f32x4*>(a.v + qbase + (int64_t)key * qrs + 16 * cc + 4 * g);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      Kr[cc][t] = kv[t];
      Vr[cc][t] = vv[t];
    }
  }
  f32x4 dK[4], dV[4];   // transposed: rows d (16dt + 4g + r), col = key (lane)
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    dK[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dV[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (int q0 = 0; q0 < a.S; q0 += 64) {
    __syncthreads();
    for (int idx = threadIdx.x; idx < 64 * 16; idx += 256) {
      const int qr = idx >> 4, dq = (idx & 15) * 4;
      const int qq = q0 + qr;
      f32x4 qv = {0.f, 0.f, 0.f, 0.f}, gv = {0.f, 0.f, 0.f, 0.f};
      if (qq < a.S) {
        qv = *reinterpret_cast<const f32x4*>(a.q + qbase + (int64_t)qq * qrs + dq) * a.scale;
        gv = *reinterpret_cast<const f32x4*>(a.dout + base + (int64_t)qq * rs + dq);
      }
      *reinterpret_cast<f32x4*>(&Qs[qr * kLD + dq]) = qv;
      *reinterpret_cast<f32x4*>(&dOs[qr * kLD + dq]) = gv;
    }
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      Ls[threadIdx.x] = qq < a.S ? a.lse[(int64_t)bh * a.S + qq] : INFINITY;
      LLs[threadIdx.x] = qq < a.S ? a.lse[(int64_t)a.B * a.H * a.S + (int64_t)bh * a.S + qq] : 0.f;
      Ds[threadIdx.x] = qq < a.S ? a.delta[(int64_t)bh * a.S + qq] : 0.f;
    }
    __syncthreads();
    // S tiles here: rows = query (16qt + 4g + r), col = key (lane).  A = Q rows, B = K^T (lane key)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const f32x4 qf = *reinterpret_cast<const f32x4*>(&Qs[(16 * qt + c16) * kLD + 16 * cc + 4 * g]);
        const f32x4 gf = *reinterpret_cast<const f32x4*>(&dOs[(16 * qt + c16) * kLD + 16 * cc + 4 * g]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s = mfma16(qf[t], Kr[cc][t], s);       // S[q][key]
          dp = mfma16(gf[t], Vr[cc][t], dp);     // dP_drop[q][key] = dO . V
        }
      }
      float P[4], Pd[4], dS[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * qt + 4 * g + r, qq = q0 + ql;
        float sv = kmasked ? kNegBig : s[r];
        float p = (kok && qq < a.S) ? __expf((sv - Ls[ql]) - LLs[ql]) : 0.f;
        bool keep = true;
        if (a.drop_thr) keep = keep_elem(seed, (uint32_t)bh, (uint32_t)qq, (uint32_t)key, a.drop_thr);
        const float pd = keep ? p * (a.drop_thr ? a.drop_scale : 1.f) : 0.f;
        const float dpp = keep ? dp[r] * (a.drop_thr ? a.drop_scale : 1.f) : 0.f;   // dP = keep*dPd/(1-p)
        P[r] = p;
        Pd[r] = pd;
        dS[r] = kmasked ? 0.f : p * (dpp - Ds[ql]);   // masked_fill: no grad to the score
      }
      // dV^T[d][key] += sum_q dO[q][d] * Pd[q][key]: A = dO^T rows d (lane-group k = query),
      // B = Pd (k = query 4g + r, col = key lane).  dK^T likewise with Q and dS.
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float* gr = &dOs[(16 * qt + 4 * g) * kLD + 16 * dt + c16];  // dO^T[d][q] = dO[q][d]
        const float* qp = &Qs[(16 * qt + 4 * g) * kLD + 16 * dt + c16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dV[dt] = mfma16(gr[r * kLD], Pd[r], dV[dt]);
          dK[dt] = mfma16(qp[r * kLD], dS[r], dK[dt]);
        }
      }
      (void)P;
    }
  }
  if (!kok) return;
  // dK^T tile: col = key (lane), rows d = 16dt + 4g + r.  Q was pre-scaled -> dK = dS^T (Q*scale)
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    *reinterpret_cast<f32x4*>(a.dk + qbase + (int64_t)key * qrs + 16 * dt + 4 * g) = dK[dt];
    *reinterpret_cast<f32x4*>(a.dv + qbase + (int64_t)key * qrs + 16 * dt + 4 * g) = dV[dt];
  }
}

// dQ: one wave owns 16 queries, loops over keys (recomputes P and dP).  4 waves per SIMD: its
// registers fit 128 VGPRs without spilling (160 with AGPRs by default -> 3 waves).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  const uint32_t seed = (a.drop_thr && a.seedp) ? (uint32_t)*a.seedp : 0u;
  __shared__ __attribute__((aligned(16))) float Ks[kBK * kLD];   // K[key][d]
  __shared__ __attribute__((aligned(16))) float Vs[kBK * kLD];   // V[key][d]
  __shared__ float Mk[kBK];
  __shared__ int blkv[kMaxBlk];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c16 = lane & 15;
  const int bh = blockIdx.y, b = bh / a.H, h = bh - (bh / a.H) * a.H;
  const bool row_any = scan_mask(a.mask, b, a.S, blkv);
  const int64_t rs = (int64_t)a.H * kD;
  const int64_t base = (int64_t)b * a.S * rs + (int64_t)h * kD;
  const int64_t qrs = a.ldq;                                  // q / k / v (+ grads) row stride
  const int64_t qbase = (int64_t)b * a.S * qrs + (int64_t)h * kD;
  const int q = blockIdx.x * 64 + wave * 16 + c16;
  const bool qok = q < a.S;
  float Qr[4][4], Gr[4][4];
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    f32x4 qv = {0.f, 0.f, 0.f, 0.f}, gv = {0.f, 0.f, 0.f, 0.f};
    if (qok) {
      qv = *reinterpret_cast<const f32x4*>(a.q + qbase + (int64_t)q * qrs + 16 * cc + 4 * g);
      gv = *reinterpret_cast<const f32x4*>(a.dout + base + (int64_t)q * rs + 16 * cc + 4 * g);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      Qr[cc][t] = qv[t] * a.scale;
      Gr[cc][t] = gv[t];
    }
  }
  const float L = qok ? a.lse[(int64_t)bh * a.S + q] : 0.f;
  const float LL = qok ? a.lse[(int64_t)a.B * a.H * a.S + (int64_t)bh * a.S + q] : 0.f;
  const float Dl = qok ? a.delta[(int64_t)bh * a.S + q] : 0.f;
  f32x4 dQ[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dQ[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.S; k0 += kBK) {
    if (skip_block(a.mask, row_any, blkv, k0)) continue;
    __syncthreads();
    for (int idx = threadIdx.x; idx < kBK * 16; idx += 256) {
      const int kr = idx >> 4, dq = (idx & 15) * 4;
      const int key = k0 + kr;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (key < a.S) {
        kv = *reinterpret_cast<const f32x4*>(a.k + qbase + (int64_t)key * qrs + dq);
        vv = *reinterpret_cast<const f32x4*>(a.v + qbase + (int64_t)key * qrs + dq);
      }
      *reinterpret_cast<f32x4*>(&Ks[kr * kLD + dq]) = kv;
      *reinterpret_cast<f32x4*>(&Vs[kr * kLD + dq]) = vv;
    }
    if (threadIdx.x < kBK) {
      const int key = k0 + threadIdx.x;
      Mk[threadIdx.x] = (key < a.S && (a.mask == nullptr || a.mask[(int64_t)b * a.S + key] != 0)) ? 1.f
                        : (key < a.S ? 0.f : -1.f);
    }
    __syncthreads();
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      // S^T and dP^T tiles: rows = key (16kt + 4g + r), col = query (lane)
      f32x4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const f32x4 kf = *reinterpret_cast<const f32x4*>(&Ks[(16 * kt + c16) * kLD + 16 * cc + 4 * g]);
        const f32x4 vf = *reinterpret_cast<const f32x4*>(&Vs[(16 * kt + c16) * kLD + 16 * cc + 4 * g]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          st = mfma16(kf[t], Qr[cc][t], st);
          dpt = mfma16(vf[t], Gr[cc][t], dpt);
        }
      }
      float dS[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kl = 16 * kt + 4 * g + r, key = k0 + kl;
        const float mk = Mk[kl];
        const float sv = (mk == 0.f) ? kNegBig : st[r];
        const float p = (mk >= 0.f && qok) ? __expf((sv - L) - LL) : 0.f;
        bool keep = true;
        if (a.drop_thr) keep = keep_elem(seed, (uint32_t)bh, (uint32_t)q, (uint32_t)key, a.drop_thr);
        const float dpp = keep ? dpt[r] * (a.drop_thr ? a.drop_scale : 1.f) : 0.f;
        dS[r] = (mk == 0.f) ? 0.f : p * (dpp - Dl);    // masked_fill: no grad to the score
      }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]: A = K^T rows d, B = dS (k = key 4g + r)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float* kp = &Ks[(16 * kt + 4 * g) * kLD + 16 * dt + c16];  // K^T[d][key] = K[key][d]
#pragma unroll
        for (int r = 0; r < 4; ++r) dQ[dt] = mfma16(kp[r * kLD], dS[r], dQ[dt]);
      }
    }
  }
  if (!qok) return;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    *reinterpret_cast<f32x4*>(a.dq + qbase + (int64_t)q * qrs + 16 * dt + 4 * g) = dQ[dt] * a.scale;
}

// ------------------------------------ launchers ------------------------------------------
void launch_attn_fwd(const float* q, const float* k, const float* v, const int32_t* mask, float* o, float* lse,
                     int B, int S, int H, float scale, const int32_t* seed, float p_drop, hipStream_t s,
                     int64_t ldq) {
  AttnArgs a{q, k, v, mask, o, lse, B, S, H, scale, seed, 0u, 1.f, ldq > 0 ? ldq : (int64_t)H * kD};
  if (p_drop > 0.f) {
    a.drop_thr = (uint32_t)fminf(p_drop * 4294967296.0f, 4294967295.0f);
    a.drop_scale = 1.f / (1.f - p_drop);
  }
  hipLaunchKernelGGL(attn_fwd_kernel, dim3((S + 63) / 64, B * H), dim3(256), 0, s, a);
}

void launch_attn_bwd(const float* q, const float* k, const float* v, const int32_t* mask, const float* o,
                     const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv, int B,
                     int S, int H, float scale, const int32_t* seed, float p_drop, hipStream_t s, int64_t ldq) {
  const int rows = B * S * H;
  hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, o, dout, delta, B, S, H);
  AttnBwdArgs a{q, k, v, mask, dout, lse, delta, dq, dk, dv, B, S, H, scale, seed, 0u, 1.f,
                ldq > 0 ? ldq : (int64_t)H * kD};
  if (p_drop > 0.f) {
    a.drop_thr = (uint32_t)fminf(p_drop * 4294967296.0f, 4294967295.0f);
    a.drop_scale = 1.f / (1.f - p_drop);
  }
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((S + 63) / 64, B * H), dim3(256), 0, s, a);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((S + 63) / 64, B * H), dim3(256), 0, s, a);
}

}  // namespace ndp
