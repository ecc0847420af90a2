// PowerSGD compression pipeline on gfx950 (CDNA4) — hand-written HIP, f32 MFMA.
//
// Replaces the reference's per-tensor eager loop
//   P = M Q            (ddp_powersgd_guide_cifar10/reducer.py:121-123)   -> psgd_p_kernel
//   orthogonalize(P)   (reducer.py:136-137, 180-191)                     -> orth.hip
//   Q = M^T P          (reducer.py:140-142)                              -> psgd_q_kernel
//   out = P Q^T, mem = M - out (reducer.py:158-163) + Algorithm-2 momentum/SGD
//                      (ddp_powersgd_guide_cifar10/ddp_init.py:156-178)  -> psgd_update_kernel
// with ONE launch per stage for all matrices (work-item tables from plan.cpp).
//
// Design notes (MI355X):
//  * The GEMMs are tall-skinny (r <= 64) and HBM-bound (~r/2 FLOP/B).  They run on
//    v_mfma_f32_16x16x4_f32 (exact f32, k-ordered fmaf chain), the small operand (Q or P)
//    is staged in LDS and shared by the 4 waves of a workgroup, the big operand (M) is
//    streamed straight to VGPRs with 16-B loads (cdna_hip_programming.md §5 'GEMV' row).
//  * Split-K partials are written to slabs and summed in a fixed order by seg_reduce,
//    so P and Q are bitwise reproducible: every rank computes the identical P-hat and the
//    identical decompressed gradient (SURVEY.md §7.4 hard part 1).  No float atomics.
//  * M = g + e is formed on the fly in the P pass and written back into e, so the Q and
//    update passes read one array; the update pass fuses decompression, error feedback,
//    momentum and the parameter update (one read-modify-write of e, m, x).
#include <hip/hip_runtime.h>

#include <algorithm>
#include "ndp_kernels.h"
#include "seg_block.h"

namespace ndp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  // D(16x16) += A(16x4) * B(4x16); lane l: A[l&15][l>>4], B[l>>4][l&15];
  // D: col = l&15, row = 4*(l>>4) + reg.
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// The per-matrix pointers come from a table in memory, so the compiler cannot prove they are
// global: every HBM stream through them compiled to FLAT loads / stores, which also count on
// lgkmcnt — each scalar-cache wait (s_load of a P-hat row, a table entry) then drained every
// outstanding stream load as well.  GPtrs re-types them as global (address space 1).
#define NDP_GLOBAL __attribute__((address_space(1)))
struct GPtrs {
  const float NDP_GLOBAL* min;
  float NDP_GLOBAL* e;
  const float NDP_GLOBAL* mread;
  float NDP_GLOBAL* out;
  float NDP_GLOBAL* mem;
  float NDP_GLOBAL* mom;
  float NDP_GLOBAL* x;
  float NDP_GLOBAL* g;
};
__device__ __forceinline__ GPtrs gptrs(const MatPtrs& p) {
  return GPtrs{(const float NDP_GLOBAL*)p.min, (float NDP_GLOBAL*)p.e,   (const float NDP_GLOBAL*)p.mread,
               (float NDP_GLOBAL*)p.out,       (float NDP_GLOBAL*)p.mem, (float NDP_GLOBAL*)p.mom,
               (float NDP_GLOBAL*)p.x,         (float NDP_GLOBAL*)p.g};
}
__device__ __forceinline__ f32x4 ld4(const float NDP_GLOBAL* p) { return *reinterpret_cast<const f32x4 NDP_GLOBAL*>(p); }
__device__ __forceinline__ void st4(float NDP_GLOBAL* p, f32x4 v) { *reinterpret_cast<f32x4 NDP_GLOBAL*>(p) = v; }

__device__ __forceinline__ float wave_sum(float v) {
  // xor butterfly: every lane ends with the bitwise-identical total (fp add commutes)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ----------------------------------------------------------------------------------
// P partial:  p_part[chunk][a][c] = sum_{k in chunk} M[a][k] * Q[k][c]
// workgroup = 64 rows x kPK columns of one matrix; wave w owns rows row0+16w..+15.
// Q[k0:k1, :] is staged transposed in LDS: qt[c][k] (row stride kPK+4).
// ----------------------------------------------------------------------------------
template <int NCG>
__global__ __launch_bounds__(256) void psgd_p_kernel(const MatGeom* __restrict__ geom,
                                                     const MatPtrs* __restrict__ ptrs,
                                                     const PItem* __restrict__ items,
                                                     const float* __restrict__ q_warm,
                                                     float* __restrict__ p_part, int fuse_ef) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int LD = kPK + 4;
  constexpr int CW = 16 * NCG;
  const PItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const GPtrs pt = gptrs(ptrs[it.mat]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = g.r;
  const int klen = it.k1 - it.k0;
  const float* Q = q_warm + g.q_off + (int64_t)it.k0 * r;
  const int a0 = it.row0 + wave * 16;
  const int arow = a0 + (lane & 15);
  const bool rowok = arow < g.n;
  const int kq = 4 * (lane >> 4);
  const int64_t rowbase = (int64_t)arow * g.m + it.k0;

  // issue the HBM stream (M = g [+ e]) first, so it is in flight while Q is staged
  f32x4 mv[16];
  f32x4 ev[16];
  if (g.vec) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int kl = 16 * s + kq;
      mv[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      ev[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (rowok && kl < klen) {
        mv[s] = ld4(pt.min + rowbase + kl);
        if (fuse_ef) ev[s] = ld4(pt.e + rowbase + kl);
      }
    }
  }
  for (int idx = tid; idx < kPK * CW; idx += 256) {
    const int b = idx / CW, c = idx - (idx / CW) * CW;
    float v = 0.f;
    if (b < klen && c < r) v = Q[b * r + c];
    smem[c * LD + b] = v;
  }
  __syncthreads();
  if (a0 >= g.n) return;  // no barrier below

  if (g.vec) {
    if (fuse_ef) {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int kl = 16 * s + kq;
        mv[s] = mv[s] + ev[s];  // send = g + e   (ddp_init.py:156-157)
        if (rowok && kl < klen) st4(pt.e + rowbase + kl, mv[s]);
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int kl = 16 * s + kq;
      float t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = 0.f;
        if (rowok && kl + j < klen) {
          v = pt.min[rowbase + kl + j];
          if (fuse_ef) {
            v = v + pt.e[rowbase + kl + j];
            pt.e[rowbase + kl + j] = v;
          }
        }
        t[j] = v;
      }
      mv[s] = f32x4{t[0], t[1], t[2], t[3]};
    }
  }

  float* dst = p_part + g.pp_off + (int64_t)it.chunk * g.n * r;
#pragma unroll
  for (int cg = 0; cg < NCG; ++cg) {
    if (cg * 16 >= r) break;
    const float* qrow = smem + (cg * 16 + (lane & 15)) * LD + kq;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      const f32x4 q0 = ld4(qrow + 16 * s);
      const f32x4 q1 = ld4(qrow + 16 * (s + 1));
      acc0 = mfma4(mv[s].x, q0.x, acc0);
      acc1 = mfma4(mv[s + 1].x, q1.x, acc1);
      acc0 = mfma4(mv[s].y, q0.y, acc0);
      acc1 = mfma4(mv[s + 1].y, q1.y, acc1);
      acc0 = mfma4(mv[s].z, q0.z, acc0);
      acc1 = mfma4(mv[s + 1].z, q1.z, acc1);
      acc0 = mfma4(mv[s].w, q0.w, acc0);
      acc1 = mfma4(mv[s + 1].w, q1.w, acc1);
    }
    const f32x4 acc = acc0 + acc1;
    const int c = cg * 16 + (lane & 15);
    if (c < r) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int a = a0 + 4 * (lane >> 4) + j;
        if (a < g.n) dst[(int64_t)a * r + c] = acc[j];
      }
    }
  }
}

// ----------------------------------------------------------------------------------
// Same stage for plans with max rank <= kUWideMaxRank: item = kPWRows rows x kPKW columns,
// wave = 4 rows, lane = 4 consecutive columns of each 256-column slice, so every wave load
// instruction streams 1 KB of ONE row (the MFMA tile above reads 16 rows x 64 B per
// instruction).  The partial dot products (4 rows x r per lane) are FMA'd on the VALU and
// reduced across the wave by recursive halving: each xor step exchanges half of the
// remaining values, so 4r values cost 4r - 1 shuffles and lane groups end up holding one
// total each (a fixed tree per value: bitwise reproducible).
// ----------------------------------------------------------------------------------
// after the call, v[0] of every lane holds the wave total of value index spread_index<V>(lane)
template <int V>
__device__ __forceinline__ void wave_reduce_spread(float (&v)[V], int lane) {
  static_assert(V >= 1 && V <= 64 && (V & (V - 1)) == 0, "power of two <= 64 values");
  int o = 32;
#pragma unroll
  for (int c = V; c > 1; c >>= 1, o >>= 1) {
    const bool upper = (lane & o) != 0;
#pragma unroll
    for (int k = 0; k < c / 2; ++k) {
      const float send = upper ? v[k] : v[k + c / 2];
      const float keep = upper ? v[k + c / 2] : v[k];
      v[k] = keep + __shfl_xor(send, o, 64);
    }
  }
  for (; o > 0; o >>= 1) v[0] += __shfl_xor(v[0], o, 64);
}

template <int V>
__device__ __forceinline__ int spread_index(int lane) {
  int idx = 0, o = 32;
#pragma unroll
  for (int c = V; c > 1; c >>= 1, o >>= 1)
    if (lane & o) idx += c / 2;
  return idx;
}

// lanes whose spread index is owned by them alone (the lowest lane of each group)
template <int V>
__device__ __forceinline__ bool spread_writer(int lane) {
  return (lane & (64 / V - 1)) == 0;  // the low 6 - log2(V) lane bits were plain butterflies
}

// Lazy error feedback (p_prev != nullptr): the update pass no longer writes e = M - P Q^T
// (reading M back just for that store is 2 of its 6 HBM passes); e keeps M, p_prev keeps the
// step's P-hat rows, and this pass forms e = M_prev - P_prev Qs^T element by element with the
// update's exact arithmetic (Qs = the warm-start Q it reads anyway, the same fmaf chain over
// c), so M = g + e is bitwise the eager formula's.  p_prev = 0 (first step, after a
// checkpoint materialised e) makes the correction an exact zero.
// In-kernel split-K finish (PFin): the item's wave-reduced partial is stored write-through (sc1)
// and drained, the row block's arrival counter is bumped (relaxed, agent scope: no release fence
// is needed for sc1 payloads, and none is wanted — it would write back the L2's dirty e lines),
// and the last arriver sums the chunk partials with sc1 loads in chunk order
// (cdna_hip_programming.md §5 'In-launch split-K reduction', sc1 form).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum_{ch < chunks} base[ch * cstride + o] in chunk order, every load an sc1 buffer load (not an
// atomic: the compiler issues a batch of 8 before the first add — relaxed atomic loads were
// serialised, one memory round trip per chunk).  base is wave-uniform; nbytes bounds the slabs.
__device__ __forceinline__ float chunk_sum_sc1(const float* base, int64_t cstride, int chunks, int64_t o,
                                               int64_t nbytes) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)nbytes, 0x00020000);
  auto ld = [&](int ch) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((ch * cstride + o) * 4), 0, 16));
  };
  float sum = ld(0);
  int ch = 1;
  for (; ch + 8 <= chunks; ch += 8) {
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = ld(ch + j);
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += t[j];
  }
  if (ch < chunks) {  // the last 1..7 chunks, issued together too (loads past nbytes return 0)
    float t[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) t[j] = ld(ch + j);
#pragma unroll
    for (int j = 0; j < 7; ++j)
      if (ch + j < chunks) sum += t[j];
  }
  return sum;
}

// every wave: drain the sc1 partial stores; one lane draws the arrival ticket; true in every
// thread of the block that drew the last of `chunks` tickets
__device__ __forceinline__ bool last_arrival(unsigned long long* ctr, int chunks, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long old = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = (int)((old + 1ull) % (unsigned long long)chunks == 0ull);
  }
  __syncthreads();
  const bool last = *flag != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: the loads after are sc1
  return last;
}

template <int RQ, int NT = 0, int NS = kPKW / 256, int SB = (RQ <= 4 ? NS : (NS < 2 ? NS : 2))>
__global__ __launch_bounds__(256) void psgd_p_wide_kernel(const MatGeom* __restrict__ geom,
                                                          const MatPtrs* __restrict__ ptrs,
                                                          const PItem* __restrict__ items,
                                                          const float* __restrict__ q_warm,
                                                          float* __restrict__ p_part, int fuse_ef,
                                                          const float* __restrict__ p_prev, PFin fin) {
  // NS: 256-column slices per item; SB: slices whose loads are in flight together (RQ = 8
  // with SB = 4 held 228 VGPRs = 2 waves / SIMD; SB = 2 keeps it at 3)
  constexpr int V = 4 * RQ;
  __shared__ int last_flag;
  if ((int)blockIdx.x >= fin.n_items) {  // rank-1 group pack (seg table), same launch
    seg_reduce_block(fin.seg, fin.seg_prefix, fin.n_seg, (int64_t)blockIdx.x - fin.n_items);
    return;
  }
  const PItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const GPtrs pt = gptrs(ptrs[it.mat]);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = g.r, n = g.n, m = g.m;
  const int arow0 = it.row0 + wave * 4;
  const bool active = arow0 < n;  // inactive waves still reach the finish's barriers
  const float* Q = q_warm + g.q_off;
  const bool q4 = (r & 3) == 0 && (g.q_off & 3) == 0;

  float acc[V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  // One load group (SB == NS): the M = g + e rows stay in registers and are stored only after
  // the split-K arrival — the arrival's vmcnt(0) drain then waits for the partial store alone,
  // not for the whole e stream's write acknowledgements.
  constexpr bool kLateE = SB == NS;
  f32x4 late[kLateE ? 4 : 1][kLateE ? SB : 1];
  auto store_e = [&](int i, int b, f32x4 v) {
    if (arow0 + i >= n) return;
    const int64_t o = (int64_t)(arow0 + i) * m + b;
    if (g.vec) {
      if (b < it.k1) {
        if constexpr (NT >= 2) __builtin_nontemporal_store(v, reinterpret_cast<f32x4 NDP_GLOBAL*>(pt.e + o));
        else st4(pt.e + o, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (b + j < it.k1) pt.e[o + j] = v[j];
    }
  };
  auto store_late = [&]() {
    if constexpr (kLateE) {
      if (active && fuse_ef) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int sb = 0; sb < SB; ++sb) store_e(i, it.k0 + 256 * sb + 4 * lane, late[i][sb]);
      }
    }
  };

  if (active) {
#pragma unroll
  for (int s0 = 0; s0 < NS; s0 += SB) {
    // the HBM stream of SB slices first: g and e of the wave's 4 rows (combined below, once
    // the lane's Q rows are in registers: the lazy correction needs them)
    f32x4 mv[4][SB], ev[4][SB];
    if (g.vec) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
          const int b = it.k0 + 256 * (s0 + sb) + 4 * lane;
          const bool ok = arow0 + i < n && b < it.k1;  // vec: k1 - b >= 4 whenever b < k1
          const int64_t o = (int64_t)(arow0 + i) * m + b;
          if constexpr (NT >= 1) {
            mv[i][sb] = ok ? __builtin_nontemporal_load(reinterpret_cast<const f32x4 NDP_GLOBAL*>(pt.min + o))
                           : f32x4{0.f, 0.f, 0.f, 0.f};
            ev[i][sb] = (ok && fuse_ef) ? __builtin_nontemporal_load(reinterpret_cast<const f32x4 NDP_GLOBAL*>(pt.e + o))
                                        : f32x4{0.f, 0.f, 0.f, 0.f};
          } else {
            mv[i][sb] = ok ? ld4(pt.min + o) : f32x4{0.f, 0.f, 0.f, 0.f};
            ev[i][sb] = (ok && fuse_ef) ? ld4(pt.e + o) : f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int sb = 0; sb < SB; ++sb) {
          const int b = it.k0 + 256 * (s0 + sb) + 4 * lane;
          float t[4], u[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            t[j] = u[j] = 0.f;
            if (arow0 + i < n && b + j < it.k1) {
              const int64_t o = (int64_t)(arow0 + i) * m + b + j;
              t[j] = pt.min[o];
              if (fuse_ef) u[j] = pt.e[o];
            }
          }
          mv[i][sb] = f32x4{t[0], t[1], t[2], t[3]};
          ev[i][sb] = f32x4{u[0], u[1], u[2], u[3]};
        }
    }
    // Q rows of this lane's columns (L2-resident: m x r floats per matrix)
#pragma unroll
    for (int sb = 0; sb < SB; ++sb) {
      const int b = it.k0 + 256 * (s0 + sb) + 4 * lane;
      float qv[4][RQ];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool okj = b + j < it.k1;
        if (q4) {
#pragma unroll
          for (int c = 0; c < RQ; c += 4) {
            const f32x4 t = (okj && c < r) ? ld4(Q + (int64_t)(b + j) * r + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 4; ++u) qv[j][c + u] = t[u];
          }
        } else {
#pragma unroll
          for (int c = 0; c < RQ; ++c) qv[j][c] = (okj && c < r) ? Q[(int64_t)(b + j) * r + c] : 0.f;
        }
      }
      if (fuse_ef) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 e4 = ev[i][sb];
          if (p_prev != nullptr) {  // e = M_prev - P_prev Qs^T, psgd_update_wide's arithmetic
            const bool rok = arow0 + i < n;
            const float* pp = p_prev + g.p_off + (int64_t)(rok ? arow0 + i : 0) * r;
            f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < RQ; ++c) {
              if (c >= r) break;
              const float pv = rok ? pp[c] : 0.f;
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] = fmaf(pv, qv[j][c], o[j]);
            }
            e4 = e4 - o;
          }
          mv[i][sb] = mv[i][sb] + e4;  // send = g + e   (ddp_init.py:156-157)
          if constexpr (kLateE) late[i][sb] = mv[i][sb];
          else store_e(i, b, mv[i][sb]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < RQ; ++c) acc[i * RQ + c] = fmaf(mv[i][sb][j], qv[j][c], acc[i * RQ + c]);
    }
  }
  }  // active

  wave_reduce_spread<V>(acc, lane);
  const int idx = spread_index<V>(lane);
  const int i = idx / RQ, c = idx % RQ;
  const int a = arow0 + i;
  const bool wr = active && spread_writer<V>(lane) && c < r && a < n;
  const int chunks = g.p_chunks;
  if (fin.out == nullptr) {  // partials for a separate seg_reduce
    if (wr) p_part[g.pp_off + (int64_t)it.chunk * n * r + (int64_t)a * r + c] = acc[0];
    store_late();
    return;
  }
  if (chunks == 1) {  // unsplit: the item IS the row block's P
    if (wr) fin.out[g.p_off + (int64_t)a * r + c] = acc[0];
    store_late();
    return;
  }
  if (wr) st_sc1(p_part + g.pp_off + (int64_t)it.chunk * n * r + (int64_t)a * r + c, acc[0]);
  const bool last = last_arrival(fin.ctr + it.rb, chunks, &last_flag);
  store_late();
  if (!last) return;
  const int rows = min(kPWRows, n - it.row0);
  for (int t = threadIdx.x; t < rows * r; t += 256) {
    const int64_t o = (int64_t)it.row0 * r + t;  // row-major n x r: the block's rows are contiguous
    fin.out[g.p_off + o] = chunk_sum_sc1(p_part + g.pp_off, (int64_t)n * r, chunks, o, (int64_t)chunks * n * r * 4);
  }
}

// ----------------------------------------------------------------------------------
// Q partial:  q_part[chunk][b][c] = sum_{a in [row0,row1)} M[a][b] * Phat[a][c]
// workgroup = [row0,row1) x 256 columns; wave w owns columns col0+64w..+63.
// Lane l streams M[a][b0+4(l&15) .. +3] for row a = step + (l>>4): 4 rows x 256 B per
// wave instruction.  MFMA j consumes component j (column b0 + 4i + j of row block).
// P-hat rows [row0,row1) are staged in LDS (row stride LDP, bank-conflict padded).
// ----------------------------------------------------------------------------------
template <int NCG, bool kQNT = false>
__global__ __launch_bounds__(256) void psgd_q_kernel(const MatGeom* __restrict__ geom,
                                                     const MatPtrs* __restrict__ ptrs,
                                                     const QItem* __restrict__ items,
                                                     const float* __restrict__ p_hat,
                                                     float* __restrict__ q_part, QFin fin) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CW = 16 * NCG;
  constexpr int LDP = CW + (NCG > 1 ? 16 : 0);
  const QItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const GPtrs pt = gptrs(ptrs[it.mat]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = g.r;
  const int nrows = it.row1 - it.row0;
  const int nrows4 = (nrows + 3) & ~3;
  const int b0 = it.col0 + wave * 64;
  const bool active = b0 < g.m;  // inactive waves still reach the finish's barriers
  const int bl = b0 + 4 * (lane & 15);
  const int rsub = lane >> 4;
  const int cl = lane & 15;
  const float NDP_GLOBAL* Mb = pt.mread + (int64_t)it.row0 * g.m;

  const float* P = p_hat + g.p_off + (int64_t)it.row0 * r;
  auto stage_p = [&]() {
    for (int idx = tid; idx < nrows4 * CW; idx += 256) {
      const int a = idx / CW, c = idx - (idx / CW) * CW;
      float v = 0.f;
      if (a < nrows && c < r) v = P[(int64_t)a * r + c];
      smem[a * LDP + c] = v;
    }
    __syncthreads();
  };
  f32x4 acc[NCG][4];
#pragma unroll
  for (int cg = 0; cg < NCG; ++cg)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[cg][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load_m = [&](int s) -> f32x4 {
    const int al = s + rsub;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (al < nrows) {
      const float NDP_GLOBAL* row = Mb + (int64_t)al * g.m;
      if (g.vec) {
        if (bl < g.m) v = kQNT ? __builtin_nontemporal_load(reinterpret_cast<const f32x4 NDP_GLOBAL*>(row + bl))
                               : ld4(row + bl);
      } else {
        float t[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = (bl + j < g.m) ? row[bl + j] : 0.f;
        v = f32x4{t[0], t[1], t[2], t[3]};
      }
    }
    return v;
  };
  auto consume = [&](int s, f32x4 mv) {
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) {
      const float pv = smem[(s + rsub) * LDP + cg * 16 + cl];
      acc[cg][0] = mfma4(mv.x, pv, acc[cg][0]);
      acc[cg][1] = mfma4(mv.y, pv, acc[cg][1]);
      acc[cg][2] = mfma4(mv.z, pv, acc[cg][2]);
      acc[cg][3] = mfma4(mv.w, pv, acc[cg][3]);
    }
  };

  if (active) {
    // 32-row batches, double-buffered: the next batch's 8 loads are in flight while this one is
    // consumed (round 5 kept 4 loads in flight and paid one memory round trip per 16 rows: the
    // 64-row ResNet items took 4 dependent trips, 2.4 TB/s)
    constexpr int QB = 8;
    f32x4 bufa[QB], bufb[QB];
    auto load_batch = [&](int s0, f32x4 (&b)[QB]) {
#pragma unroll
      for (int u = 0; u < QB; ++u) b[u] = load_m(s0 + 4 * u);  // rows past nrows load 0
    };
    auto consume_batch = [&](int s0, const f32x4 (&b)[QB]) {
#pragma unroll
      for (int u = 0; u < QB; ++u)
        if (s0 + 4 * u < nrows4) consume(s0 + 4 * u, b[u]);  // LDS rows past nrows4 are not staged
    };
    load_batch(0, bufa);
    if (4 * QB < nrows4) load_batch(4 * QB, bufb);
    stage_p();  // the P-hat tile is staged while the first two batches of M are in flight
    for (int s0 = 0; s0 < nrows4; s0 += 2 * 4 * QB) {
      if (s0 > 0 && s0 + 4 * QB < nrows4) load_batch(s0 + 4 * QB, bufb);
      consume_batch(s0, bufa);
      if (s0 + 4 * QB >= nrows4) break;
      if (s0 + 8 * QB < nrows4) load_batch(s0 + 8 * QB, bufa);
      consume_batch(s0 + 4 * QB, bufb);
    }
  } else {
    stage_p();  // every wave reaches the staging barrier
  }

  const int chunks = g.q_chunks;
  // destination: the partial slab (separate seg_reduce / in-kernel finish) or, unsplit, Q itself;
  // matrices split in more than fin.max_chunks row chunks (the DistilBERT embedding: 120) keep
  // the separate seg_reduce — one workgroup summing them all would be the launch's long tail
  const bool direct = fin.out != nullptr && chunks == 1;
  const bool sc1 = fin.out != nullptr && chunks > 1 && chunks <= fin.max_chunks;
  float* dst = direct ? fin.out + g.q_off : q_part + g.qp_off + (int64_t)it.chunk * g.m * r;
  if (active) {
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) {
      const int c = cg * 16 + cl;
      if (c >= r) continue;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int b = b0 + 4 * (4 * rsub + reg) + j;
          if (b < g.m) {
            if (sc1) st_sc1(dst + (int64_t)b * r + c, acc[cg][j][reg]);
            else dst[(int64_t)b * r + c] = acc[cg][j][reg];
          }
        }
      }
    }
  }
  if (!sc1) return;
  __syncthreads();  // every wave is done reading the P-hat tile: smem[0] may carry the flag
  if (!last_arrival(fin.ctr + it.cb, chunks, reinterpret_cast<int*>(smem))) return;
  const int cols = min(kQCols, g.m - it.col0);
  for (int t = threadIdx.x; t < cols * r; t += 256) {
    const int64_t o = (int64_t)it.col0 * r + t;  // row-major m x r: the block's columns are contiguous
    fin.out[g.q_off + o] = chunk_sum_sc1(q_part + g.qp_off, (int64_t)g.m * r, chunks, o,
                                         (int64_t)chunks * g.m * r * 4);
  }
}

// ----------------------------------------------------------------------------------
// Decompress + error feedback (+ momentum + SGD):  out[a][b] = sum_c Phat[a][c] * Qs[b][c]
// computed as D = Qs * Phat^T on MFMA so each lane holds 4 consecutive b of one row a
// (16-B accesses of e / m / x).  Qs = Q_sum / q_div (reducer.py:147).  One designated
// wave per column block also writes Qs into the warm-start buffer (reducer.py:101-111).
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void psgd_update_kernel(
    const MatGeom* __restrict__ geom, const MatPtrs* __restrict__ ptrs,
    const UItem* __restrict__ items, const float* __restrict__ p_hat,
    const float* __restrict__ q_sum, float q_div, float* __restrict__ q_warm, int mode,
    float lr, float momentum) {
  const UItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const GPtrs pt = gptrs(ptrs[it.mat]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = g.r, n = g.n, m = g.m;
  const float* P = p_hat + g.p_off;
  const float* Q = q_sum + g.q_off;

  if (q_warm != nullptr && it.row0 == 0 && wave == 0) {
    float* W = q_warm + g.q_off;
    const int cnt = min(kUCols, m - it.col0) * r;
    const int64_t base = (int64_t)it.col0 * r;
    for (int idx = lane; idx < cnt; idx += 64) W[base + idx] = Q[base + idx] / q_div;
  }

  const int a0 = it.row0 + wave * 16;
  if (a0 >= n) return;
  const int aL = a0 + (lane & 15);
  const int kq = lane >> 4;
  const int nk = (r + 3) >> 2;
  const bool rowok = aL < n;
  const int64_t ro = (int64_t)aL * m;
  // prefetch the HBM stream (M, momentum, parameters) before the MFMA chain
  f32x4 Mv[4], Mm[4], Xv[4];
  if (g.vec) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int b = it.col0 + 16 * t + 4 * kq;
      const bool ok = rowok && b < m;
      Mv[t] = ok ? ld4(pt.mread + ro + b) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (mode != 0) {
        Mm[t] = ok ? ld4(pt.mom + ro + b) : f32x4{0.f, 0.f, 0.f, 0.f};
        Xv[t] = ok ? ld4(pt.x + ro + b) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < nk; ++kc) {
    const int c = 4 * kc + kq;
    const float bv = (rowok && c < r) ? P[(int64_t)aL * r + c] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int b = it.col0 + 16 * t + (lane & 15);
      const float av = (b < m && c < r) ? Q[(int64_t)b * r + c] / q_div : 0.f;
      acc[t] = mfma4(av, bv, acc[t]);
    }
  }
  if (!rowok) return;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int b = it.col0 + 16 * t + 4 * kq;
    if (b >= m) continue;
    const f32x4 o = acc[t];
    if (g.vec) {
      const f32x4 M = Mv[t];
      if (mode == 0) {
        st4(pt.out + ro + b, o);
        st4(pt.mem + ro + b, M - o);
      } else {
        f32x4 mm = Mm[t];
        f32x4 xx = Xv[t];
        st4(pt.e + ro + b, M - o);
#pragma unroll
        for (int j = 0; j < 4; ++j) mm[j] = __fadd_rn(__fmul_rn(mm[j], momentum), o[j]);
        const f32x4 up = o + mm;
#pragma unroll
        for (int j = 0; j < 4; ++j) xx[j] = fmaf(-lr, up[j], xx[j]);
        st4(pt.mom + ro + b, mm);
        st4(pt.x + ro + b, xx);
        if (mode == 2) st4(pt.g + ro + b, up);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (b + j >= m) break;
        const int64_t k = ro + b + j;
        const float M = pt.mread[k];
        if (mode == 0) {
          pt.out[k] = o[j];
          pt.mem[k] = M - o[j];
        } else {
          pt.e[k] = M - o[j];
          const float mm = __fadd_rn(__fmul_rn(pt.mom[k], momentum), o[j]);
          pt.mom[k] = mm;
          const float up = o[j] + mm;
          pt.x[k] = fmaf(-lr, up, pt.x[k]);
          if (mode == 2) pt.g[k] = up;
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------------
// Same stage for plans with max rank <= kUWideMaxRank (every ResNet / DistilBERT config the
// reference runs): 16 x 256 tiles, one wave = 4 rows x 256 columns, lane = 4 consecutive
// columns.  Each wave load instruction streams 1 KB of one row (the MFMA tile above reads 16
// rows x 64 B per instruction), all 12 float4 loads of the HBM stream are issued before any
// use, and the decompression out = P Q^T / N is r fmaf per element on the VALU: Q's 4 x r
// values per lane are loaded once into registers, P's row is wave-uniform (scalar loads).
// ----------------------------------------------------------------------------------
constexpr int kURowsPerWave = kUWideRows / 4;

// p_prev != nullptr (lazy error feedback, modes 1 / 2): e is not written — M is not even read —
// and the column-block-0 workgroup of each row block keeps its P-hat rows in p_prev for the
// next P pass.  mode 3: e -= p_hat Qs^T only (the lazy state materialised: checkpoint, API).
template <int RQ, int NT = 0>
__global__ __launch_bounds__(256) void psgd_update_wide_kernel(
    const MatGeom* __restrict__ geom, const MatPtrs* __restrict__ ptrs,
    const UItem* __restrict__ items, const float* __restrict__ p_hat,
    const float* __restrict__ q_sum, float q_div, float* __restrict__ q_warm, int mode,
    float lr, float momentum, float* __restrict__ p_prev, R1Step r1) {
  if ((int)blockIdx.x >= r1.n_items) {  // the rank-1 group's step, same launch (rank1_step_kernel)
    const int64_t stride = (int64_t)(gridDim.x - r1.n_items) * 256;
    for (int64_t k = (int64_t)(blockIdx.x - r1.n_items) * 256 + threadIdx.x; k < r1.n; k += stride) {
      const float o = r1.buf[k] / r1.div;
      const float mm = __fadd_rn(__fmul_rn(r1.mom[k], momentum), o);
      r1.mom[k] = mm;
      const float up = o + mm;
      r1.x[k] = fmaf(-lr, up, r1.x[k]);
      if (r1.g) r1.g[k] = up;
    }
    return;
  }
  const UItem it = items[blockIdx.x];
  const MatGeom g = geom[it.mat];
  const GPtrs pt = gptrs(ptrs[it.mat]);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = g.r, n = g.n, m = g.m;
  const float* P = p_hat + g.p_off;
  const float* Q = q_sum + g.q_off;

  if (q_warm != nullptr && it.row0 == 0 && wave == 0) {
    float* W = q_warm + g.q_off;
    const int cnt = min(kUWideCols, m - it.col0) * r;
    const int64_t base = (int64_t)it.col0 * r;
    for (int idx = lane; idx < cnt; idx += 64) W[base + idx] = Q[base + idx] / q_div;
  }

  const int arow0 = it.row0 + wave * kURowsPerWave;
  if (arow0 >= n) return;
  const bool lazy = p_prev != nullptr && (mode == 1 || mode == 2);
  if (lazy && it.col0 == 0 && lane < r) {  // this row block's P-hat for the next P pass
#pragma unroll
    for (int i = 0; i < kURowsPerWave; ++i)
      if (arow0 + i < n) p_prev[g.p_off + (int64_t)(arow0 + i) * r + lane] = P[(int64_t)(arow0 + i) * r + lane];
  }
  const int b = it.col0 + 4 * lane;
  const int nb = max(0, min(4, m - b));  // valid columns of this lane (vec: 0 or 4)
  // the HBM stream first: M (= g + e), momentum, parameters of every row of the wave
  f32x4 Mv[kURowsPerWave], Mm[kURowsPerWave], Xv[kURowsPerWave];
  if (g.vec) {
#pragma unroll
    for (int i = 0; i < kURowsPerWave; ++i) {
      const bool ok = nb == 4 && arow0 + i < n;
      const int64_t o = (int64_t)(arow0 + i) * m + b;
      Mv[i] = (ok && !lazy) ? ld4(pt.mread + o) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (mode == 1 || mode == 2) {
        if constexpr (NT >= 1) {
          Mm[i] = ok ? __builtin_nontemporal_load(reinterpret_cast<const f32x4 NDP_GLOBAL*>(pt.mom + o))
                     : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
          Mm[i] = ok ? ld4(pt.mom + o) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        Xv[i] = ok ? ld4(pt.x + o) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // Qs = Q_sum / N for this lane's columns (reducer.py:147)
  float qv[4][RQ];
  const bool q4 = (r & 3) == 0 && (g.q_off & 3) == 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (q4) {
#pragma unroll
      for (int c = 0; c < RQ; c += 4) {
        f32x4 t = (j < nb && c < r) ? ld4(Q + (int64_t)(b + j) * r + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) qv[j][c + u] = t[u] / q_div;
      }
    } else {
#pragma unroll
      for (int c = 0; c < RQ; ++c) qv[j][c] = (j < nb && c < r) ? Q[(int64_t)(b + j) * r + c] / q_div : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < kURowsPerWave; ++i) {
    const int a = arow0 + i;
    if (a >= n) break;  // wave-uniform
    const float* prow = P + (int64_t)a * r;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < RQ; ++c) {
      if (c >= r) break;
      const float pv = prow[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf(pv, qv[j][c], o[j]);
    }
    const int64_t ro = (int64_t)a * m;
    if (g.vec) {
      if (nb != 4) continue;
      const f32x4 M = Mv[i];
      if (mode == 0) {
        st4(pt.out + ro + b, o);
        st4(pt.mem + ro + b, M - o);
      } else if (mode == 3) {
        st4(pt.e + ro + b, M - o);
      } else {
        f32x4 mm = Mm[i];
        f32x4 xx = Xv[i];
        if (!lazy) st4(pt.e + ro + b, M - o);
#pragma unroll
        for (int j = 0; j < 4; ++j) mm[j] = __fadd_rn(__fmul_rn(mm[j], momentum), o[j]);
        const f32x4 up = o + mm;
#pragma unroll
        for (int j = 0; j < 4; ++j) xx[j] = fmaf(-lr, up[j], xx[j]);
        if constexpr (NT >= 2) __builtin_nontemporal_store(mm, reinterpret_cast<f32x4 NDP_GLOBAL*>(pt.mom + ro + b));
        else st4(pt.mom + ro + b, mm);
        st4(pt.x + ro + b, xx);
        if (mode == 2) st4(pt.g + ro + b, up);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= nb) break;
        const int64_t k = ro + b + j;
        const float M = lazy ? 0.f : pt.mread[k];
        if (mode == 0) {
          pt.out[k] = o[j];
          pt.mem[k] = M - o[j];
        } else if (mode == 3) {
          pt.e[k] = M - o[j];
        } else {
          if (!lazy) pt.e[k] = M - o[j];
          const float mm = __fadd_rn(__fmul_rn(pt.mom[k], momentum), o[j]);
          pt.mom[k] = mm;
          const float up = o[j] + mm;
          pt.x[k] = fmaf(-lr, up, pt.x[k]);
          if (mode == 2) pt.g[k] = up;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void rank1_step_kernel(const float* __restrict__ buf, float div,
                                                         float* __restrict__ mom,
                                                         float* __restrict__ x,
                                                         float* __restrict__ g, int64_t n,
                                                         float lr, float momentum) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const float o = buf[k] / div;
    const float mm = __fadd_rn(__fmul_rn(mom[k], momentum), o);
    mom[k] = mm;
    const float up = o + mm;
    x[k] = fmaf(-lr, up, x[k]);
    if (g) g[k] = up;
  }
}

// ---------------------------------- launchers -------------------------------------
static inline void allow_lds(const void* fn, size_t bytes) {
  // gfx950 has 160 KiB of LDS per CU; dynamic requests above 64 KiB must be opted in.
  if (bytes > 65536) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

static inline int ncg_for(int max_rank) {
  const int c = (max_rank + 15) / 16;
  return c <= 1 ? 1 : (c == 2 ? 2 : 4);
}

template <int RQ, int NT>
static void launch_p_wide(int item_cols, unsigned grid, hipStream_t s, const MatGeom* geom, const MatPtrs* ptrs,
                          const PItem* items, const float* q_warm, float* p_part, int fuse_ef, const float* p_prev,
                          PFin fin) {
  if (item_cols == 256)
    hipLaunchKernelGGL((psgd_p_wide_kernel<RQ, NT, 1>), dim3(grid), dim3(256), 0, s, geom, ptrs, items, q_warm, p_part,
                       fuse_ef, p_prev, fin);
  else if (item_cols == 512)
    hipLaunchKernelGGL((psgd_p_wide_kernel<RQ, NT, 2>), dim3(grid), dim3(256), 0, s, geom, ptrs, items, q_warm, p_part,
                       fuse_ef, p_prev, fin);
  else
    hipLaunchKernelGGL((psgd_p_wide_kernel<RQ, NT, 4>), dim3(grid), dim3(256), 0, s, geom, ptrs, items, q_warm, p_part,
                       fuse_ef, p_prev, fin);
}

void launch_psgd_p(const MatGeom* geom, const MatPtrs* ptrs, const PItem* items, int n_items,
                   const float* q_warm, float* p_part, int fuse_ef, int max_rank,
                   hipStream_t s, const float* p_prev, PFin fin, int64_t n_seg_blocks, int item_cols) {
  if (n_items <= 0 && n_seg_blocks <= 0) return;
  fin.n_items = n_items;
  if (fin.seg == nullptr) n_seg_blocks = 0;
  const unsigned grid = (unsigned)(n_items + n_seg_blocks);
  // the item shape follows the plan (plan.cpp): wide 16 x item_cols items up to rank 16;
  // non-temporal g / e loads (read once per step): ResNet-18 r=4 batch 64 0.8306 / 0.8294 ->
  // 0.8245 / 0.8233 ms (profiles/r5/bench_psgd_nt.jsonl)
  if (max_rank <= 4) return launch_p_wide<4, 1>(item_cols, grid, s, geom, ptrs, items, q_warm, p_part, fuse_ef, p_prev, fin);
  if (max_rank <= 8) return launch_p_wide<8, 1>(item_cols, grid, s, geom, ptrs, items, q_warm, p_part, fuse_ef, p_prev, fin);
  if (max_rank <= kUWideMaxRank)
    return launch_p_wide<kUWideMaxRank, 0>(item_cols, grid, s, geom, ptrs, items, q_warm, p_part, fuse_ef, p_prev, fin);
  if (fin.out != nullptr || n_seg_blocks > 0) return;  // the caller checks: wide plans only (bindings.cpp)
  const int ncg = ncg_for(max_rank);
  const size_t lds = sizeof(float) * 16 * ncg * (kPK + 4);
  if (ncg == 4) allow_lds(reinterpret_cast<const void*>(psgd_p_kernel<4>), lds);
  if (ncg == 1)
    hipLaunchKernelGGL(psgd_p_kernel<1>, dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       q_warm, p_part, fuse_ef);
  else if (ncg == 2)
    hipLaunchKernelGGL(psgd_p_kernel<2>, dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       q_warm, p_part, fuse_ef);
  else
    hipLaunchKernelGGL(psgd_p_kernel<4>, dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       q_warm, p_part, fuse_ef);
}

void launch_psgd_q(const MatGeom* geom, const MatPtrs* ptrs, const QItem* items, int n_items,
                   const float* p_hat, float* q_part, int max_rank, hipStream_t s, QFin fin) {
  if (n_items <= 0) return;
  const int ncg = ncg_for(max_rank);
  const int ldp = 16 * ncg + (ncg > 1 ? 16 : 0);
  const size_t lds = sizeof(float) * kQRowsMax * ldp;
  if (ncg == 4) allow_lds(reinterpret_cast<const void*>(psgd_q_kernel<4>), lds);
  // non-temporal M loads (the step's last read of e): ResNet-18 r=4 batch 64 0.796 / 0.808 ->
  // 0.779 / 0.783 ms with the non-temporal slab sums (profiles/r5/bench_psgd_nt.jsonl)
  if (ncg == 1)
    hipLaunchKernelGGL((psgd_q_kernel<1, true>), dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       p_hat, q_part, fin);
  else if (ncg == 2)
    hipLaunchKernelGGL(psgd_q_kernel<2>, dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       p_hat, q_part, fin);
  else
    hipLaunchKernelGGL(psgd_q_kernel<4>, dim3(n_items), dim3(256), lds, s, geom, ptrs, items,
                       p_hat, q_part, fin);
}

void launch_psgd_update(const MatGeom* geom, const MatPtrs* ptrs, const UItem* items,
                        int n_items, const float* p_hat, const float* q_sum, float q_div,
                        float* q_warm, int mode, float lr, float momentum, int max_rank,
                        hipStream_t s, float* p_prev, R1Step r1) {
  r1.n_items = n_items;
  int64_t r1_blocks = r1.n > 0 ? std::min<int64_t>((r1.n + 255) / 256, 512) : 0;
  if (n_items <= 0 && r1_blocks <= 0) return;
  const unsigned grid = (unsigned)(n_items + r1_blocks);
  // the item tiles follow the plan's max rank (plan.cpp): wide 16 x 256 tiles up to rank 16
  // momentum through non-temporal loads / stores (touched once per step, 4 B per parameter): it
  // no longer evicts the next forward's weights and activations from the caches — ResNet-18 r=4
  // batch 64 0.8245 / 0.8233 -> 0.7896 / 0.7855 ms, batch 512 unchanged (1.4905 / 1.4930)
  if (max_rank <= 4)
    hipLaunchKernelGGL((psgd_update_wide_kernel<4, 2>), dim3(grid), dim3(256), 0, s, geom, ptrs,
                       items, p_hat, q_sum, q_div, q_warm, mode, lr, momentum, p_prev, r1);
  else if (max_rank <= 8)
    hipLaunchKernelGGL((psgd_update_wide_kernel<8, 2>), dim3(grid), dim3(256), 0, s, geom, ptrs,
                       items, p_hat, q_sum, q_div, q_warm, mode, lr, momentum, p_prev, r1);
  else if (max_rank <= kUWideMaxRank)
    hipLaunchKernelGGL(psgd_update_wide_kernel<kUWideMaxRank>, dim3(grid), dim3(256), 0, s,
                       geom, ptrs, items, p_hat, q_sum, q_div, q_warm, mode, lr, momentum, p_prev, r1);
  else {
    if (n_items > 0)
      hipLaunchKernelGGL(psgd_update_kernel, dim3(n_items), dim3(256), 0, s, geom, ptrs, items,
                         p_hat, q_sum, q_div, q_warm, mode, lr, momentum);
    if (r1.n > 0) launch_rank1_step(r1.buf, r1.div, r1.mom, r1.x, r1.g, r1.n, lr, momentum, s);
  }
}

void launch_rank1_step(const float* buf, float div, float* mom, float* x, float* g, int64_t n,
                       float lr, float momentum, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(rank1_step_kernel, dim3((unsigned)blocks), dim3(256), 0, s, buf, div, mom,
                     x, g, n, lr, momentum);
}

}  // namespace ndp
