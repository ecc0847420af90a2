// Strided / tabled implicit-GEMM convolutions on v_mfma_f32_32x32x2_f32 (exact f32, gfx950).
//
// Two conv families that the direct kernels (conv.hip) do not cover, both NCHW fp32:
//
//  * POINTWISE: 1x1 stride-1 convolutions on any power-of-two map (the bottleneck conv1 /
//    conv3 and the stride-1 downsample of ResNet-50/101/152 — the reference's own models,
//    ddp_guide_cifar10/ddp_init.py:108, ddp_powersgd_guide_cifar10/ddp_init.py:111):
//      forward  Y[co, (b,p)]  = sum_c  W[co, c]  X[c, (b,p)]        M = Co, N = B*HW, K = C
//      grad-x   dX[c, (b,p)]  = sum_co W[co, c]  dY[co, (b,p)]      M = C,  N = B*HW, K = Co
//      grad-W   dW[co, c]     = sum_(b,p) dY[co, (b,p)] X[c, (b,p)] M = Co, N = C,    K = B*HW
//  (Round 3-5 also carried a SMALL-MAP family here — the Toeplitz product of ResNet layer3 /
//  layer4 with the weight gathered through a tap table.  It measured 0.46-0.72x the hipBLASLt
//  Toeplitz GEMMs, stayed off by default and was deleted in round 6: profiles/r3/tg_bench.md.)
//
// One kernel serves all three: C[m, n] = sum_k A[m, k] B[k, n] with every operand index
// split as (i >> sh) * so + (i & (2^sh - 1)) * si — NCHW's (image, pixel) pairs are such
// composites when the map is a power of two.
// Tiles: 64 x 64 x 32, 4 waves of 32 x 32 (one f32x16 accumulator each), operands staged
// in LDS as [m][k] / [n][k] (k contiguous, padded rows: b128 fragment reads), register
// double buffering: the global loads of tile t+1 are
// in flight while the MFMAs of tile t issue; one barrier per tile.  The load mapping walks
// the operand's contiguous index across lanes (template AKF / BNF) so every global access is
// a coalesced 256-B wave transaction.  Split-K (blockIdx.z) writes slabs that
// conv_slab_sum adds in z order: deterministic, no atomics.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "ndp_kernels.h"

namespace ndp {

namespace {

// tile shape (BM, BN, BK) = 64 x 64 x 32, one 32 x 32 accumulator per wave.  Measured and
// removed (profiles/r3/tg_bench.md): 128 x 128 x 16; 64 x 128 / 128 x 64 (two accumulators per
// wave: 3-5x slower on every shape); a 64-deep k-tile; 3-4 deep register prefetch.
struct TgTile {
  int bm, bn, bk;
};
constexpr TgTile kTile64{64, 64, 32};
typedef float f32x16t __attribute__((ext_vector_type(16)));
typedef float f32x4t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t tg_off(const TgIndex& t, int i) {
  return (int64_t)(i >> t.sh) * t.so + (int64_t)(i & ((1 << t.sh) - 1)) * t.si;
}

template <int W>
struct VecT { typedef float __attribute__((ext_vector_type(W))) type; };
template <>
struct VecT<1> { typedef float type; };

// W floats from byte offset `off` of a raw buffer (0 past the descriptor's range)
template <int W>
__device__ __forceinline__ typename VecT<W>::type bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (W == 1) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
  } else {
    return __builtin_bit_cast(typename VecT<W>::type, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  }
}

template <int W>
__device__ __forceinline__ float vget(const typename VecT<W>::type& v, int j) {
  if constexpr (W == 1) return v;
  else return v[j];
}

// Tile TBM x TBN x TBK, 4 waves in 2 x 2, each wave (TBM/2) x (TBN/2) = TM x TN MFMA tiles of
// 32 x 32 (64 x 64 x 32: one tile per wave; 128 x 128 x 16: 2 x 2 tiles per wave, one LDS read
// per MFMA instead of two, half the global-load instructions per FLOP).
// WA / WB: elements per global load of A / B along the operand's unit-stride index (4 =
// one 16-B load; the host checks contiguity, alignment and extents)
// D: register prefetch slots.  The loads of tile t+1 are issued D-1 k-steps before its LDS
// store, so D-1 MFMA phases (~1024 cycles each at one wave per SIMD) cover the memory latency.
template <int TBM, int TBN, int TBK, bool AKF, bool BNF, int WA, int WB, int D>
__global__ __launch_bounds__(256) void tgemm_kernel(TgArgs g) {
  typedef typename VecT<WA>::type VA;
  typedef typename VecT<WB>::type VB;
  constexpr int TM = TBM / 64, TN = TBN / 64;
  // LDS tiles are [m][k] / [n][k] with k contiguous (row stride TBK + 4: 16-B aligned rows, and
  // 16 consecutive rows start 36 (or 68) words apart, i.e. in disjoint 4-bank groups).  Lane
  // (h, l32) feeds MFMA kp with k = h * TBK/2 + kp — any k order works as long as A and B
  // agree — so a lane's whole fragment of a tile is TBK/2 CONSECUTIVE floats: TBK/8
  // ds_read_b128 per operand, all issued before the MFMA chain (a [k][m] layout needs one
  // ds_read_b32 per MFMA, and hipcc interleaved those with the chain, exposing the LDS
  // latency before every MFMA pair).
  constexpr int LDK = TBK + 4;
  __shared__ __attribute__((aligned(16))) float As[2][TBM][LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][TBN][LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm = wave & 1, wn = wave >> 1;
  const int n0 = blockIdx.x * TBN, m0 = blockIdx.y * TBM;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  constexpr int PERA = TBM * TBK / 256, PERB = TBN * TBK / 256;  // elements per thread and tile
  constexpr int NVA = PERA / WA, NVB = PERB / WB;
  constexpr int FA = (AKF ? TBK : TBM) / WA, FB = (BNF ? TBN : TBK) / WB;  // vectors per fast row

  // Fixed per-thread tile coordinates.  Every operand offset splits into a tile-invariant
  // per-element part and a per-tile part that is uniform across the workgroup: tiles start
  // at multiples of TBK and every composite inner extent is a power of two, so
  // off(k0 + kk) = off(k0) + off(kk) for kk < TBK (if the extent E >= TBK the tile stays
  // inside one E-block; if E < TBK, k0 is a multiple of E).  Only a scalar base moves per
  // tile: no per-element index arithmetic in the K loop.
  int ak[NVA], am[NVA], bk[NVB], bn[NVB];
  int64_t aoff[NVA], boff[NVB];
  bool aok[NVA], bok[NVB];
#pragma unroll
  for (int v = 0; v < NVA; ++v) {
    const int e = tid + 256 * v;
    const int fast = (e % FA) * WA, slow = e / FA;
    ak[v] = AKF ? fast : slow;
    am[v] = AKF ? slow : fast;
    const int gm = m0 + am[v];
    aok[v] = gm < g.M;  // WA = 4 along m: M % 4 == 0, a vector is wholly in or out
    aoff[v] = aok[v] ? tg_off(g.am, gm) + tg_off(g.ak, ak[v]) : 0;
  }
#pragma unroll
  for (int v = 0; v < NVB; ++v) {
    const int e = tid + 256 * v;
    const int fast = (e % FB) * WB, slow = e / FB;
    bn[v] = BNF ? fast : slow;
    bk[v] = BNF ? slow : fast;
    const int gn = n0 + bn[v];
    bok[v] = gn < g.N;
    boff[v] = bok[v] ? tg_off(g.bn, gn) + tg_off(g.bk, bk[v]) : 0;
  }

  // D register slots: the global loads of tiles t+1 .. t+D-1 are in flight while tile t's
  // MFMAs run (tile t+1 is stored to the other LDS buffer at the end of the step).
  // Loads are raw BUFFER loads: a masked element gets an offset past the descriptor's range
  // and the hardware returns 0.  A predicated `ok ? *p : 0` (or a select on the loaded value)
  // makes hipcc turn each load into a branch + s_waitcnt vmcnt(0), which drained the prefetch
  // right after issuing it and serialised every k-tile on a full memory round trip (8-10 %
  // MFMA busy, profiles/r3/pmc_r50b512.md).  Offsets are 32-bit bytes (host-checked < 2 GB).
  const __amdgpu_buffer_rsrc_t ra_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.a), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.b), 0, 0x7fffffff, 0x00020000);
  constexpr uint32_t kOOB = 0xffffffffu;
  uint32_t aoffb[NVA], boffb[NVB];
#pragma unroll
  for (int v = 0; v < NVA; ++v) aoffb[v] = aok[v] ? (uint32_t)(aoff[v] * 4) : kOOB;
#pragma unroll
  for (int v = 0; v < NVB; ++v) boffb[v] = bok[v] ? (uint32_t)(boff[v] * 4) : kOOB;
  VA ra[D][NVA];
  VB rb[D][NVB];
  auto load = [&](int k0, int slot) {
    const uint32_t ta = (uint32_t)(tg_off(g.ak, k0) * 4);
    const uint32_t tb = (uint32_t)(tg_off(g.bk, k0) * 4);
#pragma unroll
    for (int v = 0; v < NVA; ++v) {
      const bool ok = (aoffb[v] != kOOB) & (k0 + ak[v] < kend);  // WA = 4 along k: K % 4 == 0
      ra[slot][v] = bload<WA>(ra_src, ok ? aoffb[v] + ta : kOOB);
    }
#pragma unroll
    for (int v = 0; v < NVB; ++v) {
      const bool ok = (boffb[v] != kOOB) & (k0 + bk[v] < kend);
      rb[slot][v] = bload<WB>(rb_src, ok ? boffb[v] + tb : kOOB);
    }
  };
  // A vector along m / n lands in 4 different rows of the [m][k] / [n][k] image.  Written
  // component by component, the 16 lanes of a k-row (rows 4i + j, i = 0..15) hit only 4 bank
  // groups (row stride 36 words: 144 i = 16 i mod 64), i.e. 4-way conflicts (profiles/r3/
  // pmc_tgemm_micro.md).  Write w stores component j = (w + i / 4) & 3 instead: banks
  // 16 (i & 3) + 36 j + k then cover all 64 (2-way at 32 vectors per row).
  auto rot = [](int w, int fast) { return (w + (fast >> 4)) & 3; };
  auto pick = [](const f32x4t& v, int j) { return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : v[3])); };
  auto store = [&](int buf, int slot) {
#pragma unroll
    for (int v = 0; v < NVA; ++v)
#pragma unroll
      for (int w = 0; w < WA; ++w) {
        if (AKF) {
          As[buf][am[v]][ak[v] + w] = vget<WA>(ra[slot][v], w);
        } else if constexpr (WA == 4) {
          const int j = rot(w, am[v]);
          As[buf][am[v] + j][ak[v]] = pick(ra[slot][v], j);
        } else {
          As[buf][am[v]][ak[v]] = vget<WA>(ra[slot][v], w);
        }
      }
#pragma unroll
    for (int v = 0; v < NVB; ++v)
#pragma unroll
      for (int w = 0; w < WB; ++w) {
        if (!BNF) {
          Bs[buf][bn[v]][bk[v] + w] = vget<WB>(rb[slot][v], w);
        } else if constexpr (WB == 4) {
          const int j = rot(w, bn[v]);
          Bs[buf][bn[v] + j][bk[v]] = pick(rb[slot][v], j);
        } else {
          Bs[buf][bn[v]][bk[v]] = vget<WB>(rb[slot][v], w);
        }
      }
  };

  f32x16t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ntiles = kend > kbeg ? (kend - kbeg + TBK - 1) / TBK : 0;
  // One k-tile.  The loop is unrolled by lcm(D, 2) so the register slot / LDS buffer indices
  // are compile-time constants (a runtime `t & 1` index into the register arrays forced hipcc
  // to shuffle them through selects and drain the load queue), and its body is branch-free:
  // loads past the K range are masked to 0 by the buffer descriptor, the extra LDS stores at
  // the end are never read.
  auto step = [&](auto slotc, auto bufc, int t) {
    constexpr int slot = decltype(slotc)::value, cur = decltype(bufc)::value;
    load(kbeg + (t + D) * TBK, slot);  // slot `slot` (tile t) is in LDS already
    // pin the loads at the top of the step: hipcc otherwise sinks them below the LDS stores
    // at the end of the step, which leaves one MFMA phase (not D - 1) to hide their latency
    __builtin_amdgcn_sched_barrier(0);
    // every fragment of the tile in registers first, then the MFMA chain
    f32x4t a[TM][TBK / 8], b[TN][TBK / 8];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < TBK / 8; ++q)
        a[i][q] = *reinterpret_cast<const f32x4t*>(&As[cur][(wm * TM + i) * 32 + l32][h * (TBK / 2) + 4 * q]);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < TBK / 8; ++q)
        b[j][q] = *reinterpret_cast<const f32x4t*>(&Bs[cur][(wn * TN + j) * 32 + l32][h * (TBK / 2) + 4 * q]);
#pragma unroll
    for (int kp = 0; kp < TBK / 2; ++kp)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][kp / 4][kp % 4], b[j][kp / 4][kp % 4], acc[i][j], 0, 0, 0);
    store(cur ^ 1, (slot + 1) % D);  // LDS buffer cur^1 was released by the last barrier
    __syncthreads();
  };
  constexpr int U = D % 2 == 0 ? D : 2 * D;
  // steps t .. t+U-1 of one unrolled round (no exit inside: a mid-round `break` gave the
  // loop two exits, and the rotated loop then copied the prefetch registers between slots
  // each round, i.e. waited for every load in flight: s_waitcnt vmcnt(0) per round)
  auto round = [&](auto self, auto uc, int t) -> void {
    constexpr int u = decltype(uc)::value;
    if constexpr (u < U) {
      step(std::integral_constant<int, u % D>{}, std::integral_constant<int, u % 2>{}, t + u);
      self(self, std::integral_constant<int, u + 1>{}, t);
    }
  };
  // the last ntiles % U steps, one at a time (slot / buffer indices continue the pattern)
  auto tail = [&](auto self, auto uc, int t, int left) -> void {
    constexpr int u = decltype(uc)::value;
    if constexpr (u < U - 1) {
      if (u < left) {
        step(std::integral_constant<int, u % D>{}, std::integral_constant<int, u % 2>{}, t + u);
        self(self, std::integral_constant<int, u + 1>{}, t, left);
      }
    }
  };
  if (ntiles > 0) {
#pragma unroll
    for (int s = 0; s < D; ++s) load(kbeg + s * TBK, s);
    store(0, 0);
    __syncthreads();
    int t = 0;
    for (; t + U <= ntiles; t += U) round(round, std::integral_constant<int, 0>{}, t);
    tail(tail, std::integral_constant<int, 0>{}, t, ntiles - t);
  }

  float* out = g.part != nullptr ? g.part + (int64_t)blockIdx.z * g.slab : g.c;
  const bool add = g.addend != nullptr && g.part == nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + (wn * TN + j) * 32 + l32;
    if (n >= g.N) continue;
    const int64_t noff = tg_off(g.cn, n);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // addends loaded unconditionally (clamped address) before any store: no per-element
      // branch + queue drain
      float ad[16];
      if (add) {  // uniform: one branch around the whole batch of loads
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          ad[r] = g.addend[tg_off(g.cm, m < g.M ? m : 0) + noff];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) ad[r] = 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < g.M) out[tg_off(g.cm, m) + noff] = acc[i][j][r] + ad[r];
      }
    }
  }
}

int ilog2_exact(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return (1 << s) == v ? s : -1;
}

TgIndex plain(int64_t stride) { return TgIndex{0, stride, 30, 0}; }  // i < 2^30: outer part always 0
TgIndex comp(int sh, int64_t outer, int64_t inner) { return TgIndex{outer, inner, sh, 0}; }

constexpr int kTgFill = 256;  // split-K until tiles x splits reaches one workgroup per CU

TgTile tg_tile(int, int) { return kTile64; }

// split-K factor: power of two so that tiles * splits >= kTgFill, each split >= 2 k-tiles
int tg_pick_splits(int M, int N, int K, int cap) {
  const TgTile t = tg_tile(M, N);
  const int tiles = ((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn);
  const int ktiles = (K + t.bk - 1) / t.bk;
  int s = 1;
  while (s * 2 <= cap && tiles * s < kTgFill && ktiles >= 4 * s) s *= 2;
  return s;
}

// 4 = batchnorm.hip kMaxFusedSlabs: forward / grad-x slabs up to 4 are summed inside the fused
// BN kernel that consumes the conv (ops/slablink.py), i.e. at no extra launch
constexpr int kTgCap = 4;
static int tg_cap() { return kTgCap; }

// 16-B loads along `fast` are legal when its 4 consecutive indices are 4 consecutive floats
// (unit inner stride, outer steps and every stride of `slow` multiples of 4 floats), the base
// is 16-B aligned and the fast extent is a multiple of 4 (tile origins are multiples of 32)
bool vec_ok(const TgIndex& fast, const TgIndex& slow, const float* base, int extent) {
  const bool unit = fast.si == 1 && (fast.sh == 30 || (fast.sh >= 2 && fast.so % 4 == 0));
  const bool slow4 = slow.so % 4 == 0 && (slow.sh == 0 || slow.si % 4 == 0);
  return unit && slow4 && (reinterpret_cast<uintptr_t>(base) & 15) == 0 && extent % 4 == 0;
}

template <int BM, int BN, int BK, int DEPTH>
void launch_tile(const TgArgs& a, bool akf, bool bnf, bool va, bool vb, dim3 grid, hipStream_t s) {
#define NDP_TG_LAUNCH(AK, BN_, W1, W2) \
  hipLaunchKernelGGL((tgemm_kernel<BM, BN, BK, AK, BN_, W1, W2, DEPTH>), grid, dim3(256), 0, s, a)
#define NDP_TG_W(AK, BN_)                                  \
  do {                                                     \
    if (va && vb) NDP_TG_LAUNCH(AK, BN_, 4, 4);            \
    else if (va) NDP_TG_LAUNCH(AK, BN_, 4, 1);             \
    else if (vb) NDP_TG_LAUNCH(AK, BN_, 1, 4);             \
    else NDP_TG_LAUNCH(AK, BN_, 1, 1);                     \
  } while (0)
  if (akf && bnf) NDP_TG_W(true, true);
  else if (akf) NDP_TG_W(true, false);
  else if (bnf) NDP_TG_W(false, true);
  else NDP_TG_W(false, false);
#undef NDP_TG_W
#undef NDP_TG_LAUNCH
}

// returns the number of split-K slabs left in a.part (defer), or 1 when final_out is written
int run(TgArgs a, bool akf, bool bnf, int splits, float* final_out, hipStream_t s, bool defer = false) {
  const TgTile tile = tg_tile(a.M, a.N);
  const int ktiles = (a.K + tile.bk - 1) / tile.bk;
  const int per = (ktiles + splits - 1) / splits;
  a.kchunk = per * tile.bk;
  splits = (ktiles + per - 1) / per;
  if (splits <= 1) a.part = nullptr;
  const dim3 grid((a.N + tile.bn - 1) / tile.bn, (a.M + tile.bm - 1) / tile.bm, splits);
  const bool va = vec_ok(akf ? a.ak : a.am, akf ? a.am : a.ak, a.a, akf ? a.K : a.M);
  const bool vb = vec_ok(bnf ? a.bn : a.bk, bnf ? a.bk : a.bn, a.b, bnf ? a.N : a.K);
  launch_tile<kTile64.bm, kTile64.bn, kTile64.bk, 2>(a, akf, bnf, va, vb, grid, s);
  if (splits <= 1) return 1;
  if (defer && a.addend == nullptr) return splits;  // the consumer (fused BN, gradfinish) sums them
  launch_slab_sum(a.part, final_out, a.slab, splits, s, a.addend);
  return 1;
}

}  // namespace

int tg_class(const ConvGeom& g) {
  const int hw = g.H * g.W;
  // 1x1 maps excluded: there the plain hipBLASLt GEMM (Toeplitz path) measured faster
  if (g.KH == 1 && g.KW == 1 && g.stride == 1 && g.pad == 0 && hw > 1 && ilog2_exact(hw) >= 0) return TG_POINTWISE;
  return -1;
}

// slabs `part` must hold for direction dir (0 fwd, 1 grad-x, 2 grad-W); 1 = no scratch
int tg_splits(const ConvGeom& g, int B, int dir) {
  const int cls = tg_class(g);
  const int hw = g.H * g.W;
  if (cls == TG_POINTWISE) {
    if (dir == 0) return tg_pick_splits(g.Co, B * hw, g.C, tg_cap());
    if (dir == 1) return tg_pick_splits(g.C, B * hw, g.Co, tg_cap());
    return tg_pick_splits(g.Co, g.C, B * hw, 64);
  }
  return 1;
}

// y [B, Co, OH, OW] = conv(x [B, C, H, W], w); part: tg_splits(g, B, 0) * numel(y) floats (or null if 1)
// the GEMM description of one direction (operand pointers / scratch left null), and the
// load mappings (A k-fast, B n-fast) the launch uses
TgArgs tg_args(const ConvGeom& g, int B, int dir, bool* akf, bool* bnf) {
  const int hw = g.H * g.W;
  const int sh = ilog2_exact(hw);
  TgArgs a{};
  if (dir == 0) {
    a.am = plain(g.C); a.ak = plain(1);                         // W [Co][C]
    a.bk = plain(hw); a.bn = comp(sh, (int64_t)g.C * hw, 1);    // X [b][c][p]
    a.cm = plain(hw); a.cn = comp(sh, (int64_t)g.Co * hw, 1);   // Y [b][co][p]
    a.M = g.Co; a.N = B * hw; a.K = g.C;
    a.slab = (int64_t)B * g.Co * hw;
    *akf = true; *bnf = hw >= 4;
  } else if (dir == 1) {
    a.am = plain(1); a.ak = plain(g.C);                         // W^T: A[c][co] = W[co][c]
    a.bk = plain(hw); a.bn = comp(sh, (int64_t)g.Co * hw, 1);   // dY [b][co][p]
    a.cm = plain(hw); a.cn = comp(sh, (int64_t)g.C * hw, 1);    // dX [b][c][p]
    a.M = g.C; a.N = B * hw; a.K = g.Co;
    a.slab = (int64_t)B * g.C * hw;
    *akf = false; *bnf = hw >= 4;
  } else {
    a.am = plain(hw); a.ak = comp(sh, (int64_t)g.Co * hw, 1);   // dY as A[co][(b,p)]
    a.bk = comp(sh, (int64_t)g.C * hw, 1); a.bn = plain(hw);    // X as B[(b,p)][c]
    a.cm = plain(g.C); a.cn = plain(1);                         // dW [co][c]
    a.M = g.Co; a.N = g.C; a.K = B * hw;
    a.slab = (int64_t)g.Co * g.C;
    *akf = hw >= 4; *bnf = hw == 1;
  }
  return a;
}

int launch_tg_fwd(const float* x, const float* w, float* y, int B, const ConvGeom& g, float* part, hipStream_t s,
                  bool defer) {
  bool akf, bnf;
  TgArgs a = tg_args(g, B, 0, &akf, &bnf);
  a.a = w;
  a.b = x;
  a.c = y;
  a.part = part;
  return run(a, akf, bnf, tg_splits(g, B, 0), y, s, defer);
}

// dx [B, C, H, W] from dy [B, Co, OH, OW]; part: tg_splits(g, B, 1) * numel(dx) floats
int launch_tg_dgrad(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, float* part,
                    hipStream_t s, const float* addend, bool defer) {
  bool akf, bnf;
  TgArgs a = tg_args(g, B, 1, &akf, &bnf);
  a.a = w;
  a.b = dy;
  a.c = dx;
  a.part = part;
  a.addend = addend;
  return run(a, akf, bnf, tg_splits(g, B, 1), dx, s, defer);
}

// out = dW [Co, C].  part: tg_splits(g, B, 2) * numel(out) floats.  defer: leave the split-K
// slabs in `part` and return how many (1 = `out` final).
int launch_tg_wgrad(const float* x, const float* dy, float* out, int B, const ConvGeom& g, float* part, hipStream_t s,
                    bool defer) {
  bool akf, bnf;
  TgArgs a = tg_args(g, B, 2, &akf, &bnf);
  a.a = dy;
  a.b = x;
  a.c = out;
  a.part = part;
  return run(a, akf, bnf, tg_splits(g, B, 2), out, s, defer);
}

}  // namespace ndp
