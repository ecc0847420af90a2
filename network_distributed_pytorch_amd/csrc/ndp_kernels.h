// Shared device-table layouts and host launch entry points for the gfx950 kernels.
//
// Every hot op of the reference's PowerSGD step is a grouped
// kernel driven by a device-side table built once per model by the plan builder
// (plan.cpp).  The tables replace the reference's per-tensor Python loops
// (reference: ddp_powersgd_guide_cifar10/reducer.py:86-168).
//
// All launchers take raw device pointers + a hipStream_t and never allocate or
// synchronise, so every call is hipGraph-capturable.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace ndp {

// ---- PowerSGD plan geometry (one per high-rank matrix, 64 B) ----------------------
struct MatGeom {
  int32_t n, m, r;      // matrix = param.view(n, m); r = min(n, m, R)
  int32_t vec;          // 1 -> m % 4 == 0 and every bound pointer 16-B aligned (float4 path)
  int32_t p_off, q_off; // element offsets into the flat P / Q buffers (reference order)
  int32_t pp_off, qp_off;     // element offsets into the P / Q split-K partial scratch
  int32_t p_chunks, q_chunks; // number of split-K slabs for P (over m) and Q (over n)
  int32_t pad[6];
};

// ---- per-matrix bound pointers (64 B) -------------------------------------------
// engine mode : min = grad, e = error memory (M = g + e is written back into e),
//               mread = e, mom = momentum, x = parameter, g = grad (optional write)
// api mode    : min = M (caller's send buffer), e = nullptr, mread = M,
//               out = grad_out, mem = memory_out
struct MatPtrs {
  const float* min;
  float* e;
  const float* mread;
  float* out;
  float* mem;
  float* mom;
  float* x;
  float* g;
};

// Work items.  One workgroup (4 waves) per item.
// rb / cb: ordinal of the item's P row block / Q column block in the plan (the arrival counter
// of the in-kernel split-K finish, PFin / QFin)
struct PItem { int32_t mat, row0, k0, k1, chunk, rb, pad[2]; };   // 64 rows x [k0,k1)
struct QItem { int32_t mat, col0, row0, row1, chunk, cb, pad[2]; }; // [row0,row1) x 256 cols
struct UItem { int32_t mat, row0, col0, pad; };                 // 64 rows x 64 cols
// orth: rows [row0,row1) of matrix `mat`; workgroup `wg` of `nwg`; slab0 = first item of mat
struct OrthItem { int32_t mat, row0, row1, wg, nwg, slab0, pad[2]; };

// Segmented reduce-copy entry: dst[k] = (sum_c src[c*stride + k]) / div
struct SegEntry {
  const float* src;
  float* dst;
  int64_t numel;
  int64_t stride;
  int32_t chunks;
  float div;
  int32_t vec;
  int32_t pad;
};

constexpr int kPRows = 64;    // rows per P item (4 waves x 16)
constexpr int kPK = 256;      // k-chunk of a P item
// plans whose max rank is <= kUWideMaxRank use kPWRows x kPKW P items (psgd_p_wide_kernel)
constexpr int kPWRows = 16;
constexpr int kPKW = 1024;
constexpr int kQCols = 256;   // columns per Q item (4 waves x 64)
constexpr int kQRowsMax = 256;  // max rows per Q item (LDS: 256 x (16*NCG+pad) floats)
constexpr int kURows = 64;
constexpr int kUCols = 64;
// plans whose max rank is <= kUWideMaxRank use 16 x 256 update tiles (psgd_update_wide_kernel)
constexpr int kUWideRows = 16;
constexpr int kUWideCols = 256;
constexpr int kUWideMaxRank = 16;
constexpr int kMaxRank = 64;
constexpr int kSegBlockElems = 2048;  // elements per workgroup in seg_reduce

// ---- launchers (powersgd.hip) --------------------------------------------------
// p_prev (rank <= kUWideMaxRank only): lazy error feedback, e = M_prev - P_prev Qs^T formed here
// In-kernel split-K finish of the P / Q passes: every chunk item stores its
// partial write-through (sc1), drains, and bumps its row / column block's monotonic arrival
// counter; the block's last arriver sums the chunk partials in chunk order (the order of the
// seg_reduce it replaces: bitwise identical) and writes the final P / Q.  out == nullptr: leave
// the partials for a separate seg_reduce.  P's extra blocks [n_items, grid) run a seg table (the
// rank-1 group's pack into the comm buffer), so the P stage is ONE launch.
struct PFin {
  float* out;                    // final P (comm buffer, MatGeom.p_off)
  unsigned long long* ctr;       // [n row blocks]
  const SegEntry* seg;           // optional reduce-copy table run by the extra blocks
  const int64_t* seg_prefix;
  int n_seg;
  int n_items;
};
struct QFin {
  float* out;                    // final Q sums (q_memory, MatGeom.q_off)
  unsigned long long* ctr;       // [n column blocks]
  int max_chunks;                // matrices with more row chunks leave their partials to seg_reduce
};
// the rank-1 (<= 1-D) group's momentum / SGD step, run by the update pass's extra blocks
struct R1Step {
  const float* buf;
  float* mom;
  float* x;
  float* g;
  int64_t n;
  float div;
  int n_items;
};

void launch_psgd_p(const MatGeom* geom, const MatPtrs* ptrs, const PItem* items, int n_items,
                   const float* q_warm, float* p_part, int fuse_ef, int max_rank, hipStream_t s,
                   const float* p_prev = nullptr, PFin fin = PFin{}, int64_t n_seg_blocks = 0,
                   int item_cols = kPKW);
void launch_psgd_q(const MatGeom* geom, const MatPtrs* ptrs, const QItem* items, int n_items,
                   const float* p_hat, float* q_part, int max_rank, hipStream_t s, QFin fin = QFin{});
// partial: 2 * n_items_total * kMaxRank floats; counters: n_mats uint64 (zeroed once, never reset);
// items may be a slice [k0, k0 + n_items) of an n_items_total list (slab0 indexes are global)
void launch_psgd_orth(const MatGeom* geom, const OrthItem* items, int n_items, int n_mats, float* p,
                      float p_div, float eps, int max_rank, float* partial, unsigned long long* counters,
                      unsigned* err, int n_items_total, unsigned max_spins, hipStream_t s);
int orth_rows_per_thread(int max_rank);
// workgroups of ONE matrix the MGS barrier may span: occupancy x CUs / 2 (-1: no device)
int orth_coresident_cap(int max_rank);
constexpr unsigned kOrthMaxSpins = 1u << 25;  // ~seconds of s_sleep 2
// mode 0 = api (out/mem), 1 = engine (EF + momentum + SGD), 2 = engine + write grad,
// 3 = e -= p_hat q_sum^T / q_div only (materialise the lazy error, rank <= kUWideMaxRank);
// p_prev (modes 1 / 2, rank <= kUWideMaxRank): lazy error feedback — e is not written, the
// P-hat rows are kept in p_prev for the next P pass
void launch_psgd_update(const MatGeom* geom, const MatPtrs* ptrs, const UItem* items,
                        int n_items, const float* p_hat, const float* q_sum, float q_div,
                        float* q_warm, int mode, float lr, float momentum, int max_rank,
                        hipStream_t s, float* p_prev = nullptr, R1Step r1 = R1Step{});
// rank-1 (<=1-D) group of the fused engine: out = buf/div; m = lam*m + out; x -= lr*(out+m)
void launch_rank1_step(const float* buf, float div, float* mom, float* x, float* g,
                       int64_t n, float lr, float momentum, hipStream_t s);

// ---- launchers (multitensor.hip) -----------------------------------------------
void launch_seg_reduce(const SegEntry* entries, const int64_t* block_prefix, int n_entries,
                       int64_t n_blocks, hipStream_t s);
// dense arm: b = mu*b + g/div ; x -= lr*b   (torch.optim.SGD(momentum) with zero-init buf)
void launch_sgd_momentum(float* x, const float* g, float* buf, int64_t n, float lr, float mu,
                         float div, hipStream_t s);
// out = a + b  (EF pack: send = g + e)
void launch_add(const float* a, const float* b, float* out, int64_t n, hipStream_t s);
// spin the stream for `ns` nanoseconds of wall time (link-emulation pacing)
void launch_delay_ns(int64_t ns, hipStream_t s);
// device-flag ordering between two queues: signal bumps *ctr; wait spins until *ctr has
// been bumped once more than *seen records (then records it); err |= 1 on spin timeout
void launch_flag_signal(unsigned* ctr, hipStream_t s);
void launch_flag_wait(unsigned* ctr, unsigned* seen, unsigned* err, int64_t timeout_us, hipStream_t s,
                      unsigned* host_err = nullptr);
// deterministic fp64-accumulated checksum of a flat buffer (replica divergence detector)
void launch_checksum(const float* x, int64_t n, double* out, hipStream_t s);

}  // namespace ndp

// ---- fused BatchNorm2d (+residual) (+ReLU), NCHW fp32 (batchnorm.hip) -------------------
namespace ndp {
int bn_slices(int N, int C, int HW);
// doubles of `part` scratch a (N, C, HW) BN needs (large-map slices or the small-map path)
int64_t bn_part_numel(int N, int C, int HW);
// part: C * S * 2 doubles of scratch; rmean/rvar/nbt may be null; training=0 uses running stats;
// single: allow the one-launch small-map path (HW <= 4, N <= 512)
void launch_bn_fwd(const float* x, const float* res, float* y, const float* gamma, const float* beta,
                   float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                   double* part, int N, int C, int HW, int S, float eps, float momentum, int relu,
                   int training, int single, hipStream_t s, const float* xpart = nullptr, int nslab = 0,
                   const double* xstats = nullptr, int xS = 0);
// xstats (nullable, training): [C][xS][2] fp64 partial sums of x from the producing conv's
// epilogue (conv_fwd_stats_slices); the large-map path then skips its statistics pass
// xpart / dypart (nullable): the input x (forward) / dy (backward) is the sum of `nslab`
// split-K slabs of numel(x) floats (a deferred conv sum); the forward also writes the sum to x
void launch_bn_bwd(const float* dy, const float* y, const float* x, const float* gamma, const float* save_mean,
                   const float* save_invstd, float* dx, float* dres, float* dgamma, float* dbeta, double* part,
                   int N, int C, int HW, int S, int relu, int single, hipStream_t s, const float* dypart = nullptr,
                   int nslab = 0, const float* dyadd = nullptr, const float* mbeta = nullptr,
                   const double* dstats = nullptr, int dS = 0);
// dstats (nullable; large-map path, no slabs): [C][dS][2] partial sums of dz and dz * xhat from the
// grad-x epilogue of the conv that produced dy (conv_dgrad bst); the statistics pass is skipped
// mbeta (nullable, relu, two-kernel path only): y was never stored; the ReLU mask is recomputed
// from x as fmaf(x, gamma * invstd, beta - mean * gamma * invstd) > 0 (the forward's own ops)
bool bn_two_kernel_path(int N, int C, int HW, int single);
// the downsample block's BN(x) + BN2(x2) -> ReLU in one launch per direction (batchnorm.hip BnPair)
bool bn_pair_ok(int N, int C, int HW);
void launch_bn_pair_fwd(const float* x, const float* x2, float* y, const float* gamma, const float* beta,
                        float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                        const float* gamma2, const float* beta2, float* rmean2, float* rvar2, int64_t* nbt2,
                        float* save_mean2, float* save_invstd2, int N, int C, int HW, float eps, float momentum,
                        hipStream_t s, const float* xpart, int nslab, const float* x2part, int nslab2);
void launch_bn_pair_bwd(const float* dy, const float* y, const float* x, const float* x2, const float* gamma,
                        const float* save_mean, const float* save_invstd, const float* gamma2,
                        const float* save_mean2, const float* save_invstd2, float* dx, float* dx2, float* dgamma,
                        float* dbeta, float* dgamma2, float* dbeta2, int N, int C, int HW, hipStream_t s,
                        const float* dypart, int nslab, const float* dyadd);
void bn_set_vec4(bool on);
// BN (training) -> ReLU -> MaxPool(3, 2, 1) in one pass without storing the BN output (the
// ResNet stem tail); y / idx: the pooled output and its uint8 window offsets (pool.hip layout)
void launch_bn_relu_maxpool(const float* x, float* y, uint8_t* idx, const float* gamma, const float* beta,
                            float* rmean, float* rvar, int64_t* nbt, float* save_mean, float* save_invstd,
                            double* part, int N, int C, int H, int W, float eps, float momentum, hipStream_t s,
                            const double* xstats = nullptr, int xS = 0);
// dyadd (nullable, with dypart): dy = sum of the slabs + dyadd (added last, as conv_slab_sum does)
}  // namespace ndp

// ---- embedding backward (embedding.hip) -------------------------------------------------
// grad_W [V, D] (dense, zeros for unreferenced rows and `pad`) from ids [T] int64 and
// grad_out [T, D]; perm [T], row_start [V] int32 scratch, row_cnt [V] int32 zeroed once
// at allocation (the kernels re-arm it).  Deterministic (fixed summation order).
namespace ndp {
// column sums of a row-major [M, N] fp32 matrix (N % 4 == 0): Linear bias gradient
// (linear.hip); part: colsum_chunks(M, N) * N floats of scratch
int colsum_chunks(int64_t M, int N);
void launch_colsum(const float* g, int64_t M, int N, float* part, float* out, hipStream_t s);
// dh = g * gelu'(h) (exact GELU) and out = column sums of dh, one pass over g / h (+ slab sum)
void launch_gelu_bwd_colsum(const float* g, const float* h, float* dh, int64_t M, int N, float* part, float* out,
                            hipStream_t s);
void launch_embedding_backward(const int64_t* ids, int T, const float* gout, int V, int D, int pad, int* perm,
                               int* row_start, int* row_cnt, float* gw, hipStream_t s);
}  // namespace ndp

// ---- fused softmax cross-entropy, mean reduction (loss.hip) -----------------------------
// x [B, K] logits, tgt [B] int64; dl [B, K] saved gradient (unscaled softmax - onehot),
// rowloss [B] scratch, loss / inv device scalars, ctr: one zeroed uint32 (re-armed by the kernel)
namespace ndp {
// acc (nullable): acc[0] += loss (a running loss sum)
void launch_ce_fwd(const float* x, const int64_t* tgt, int B, int K, int64_t ignore, float* dl, float* rowloss,
                   float* loss, float* inv, unsigned* ctr, hipStream_t s, float* acc = nullptr);
// dx = dl * (g[0] * inv[0])
void launch_ce_bwd(const float* dl, const float* g, const float* inv, float* dx, int64_t n, hipStream_t s);
}  // namespace ndp

// ---- fused residual add + LayerNorm over the last dim (layernorm.hip) --------------------
namespace ndp {
bool ln_supported(int D);  // D in {256, 512, 768, 1024}
// hash dropout fused into the LayerNorm: mode 0 none, 1 on a (before the residual add; the
// backward also writes da = dropout'(dx)), 2 on the output; keep = hash >= thr (= p * 2^32)
struct LnDrop {
  const int32_t* seed;
  uint32_t thr;
  float scale;  // 1 / (1 - p)
  int mode;
  float* da;
};
// y = LN(a (+ b)) * gamma + beta; s = a (+ b), mean / rstd [R] saved for backward
void launch_ln_fwd(const float* a, const float* b, const float* gamma, const float* beta, float* y, float* s,
                   float* mean, float* rstd, int64_t R, int D, float eps, hipStream_t st, const LnDrop& dp);
int ln_bwd_wgs(int64_t R);
// dx [R, D]; part: ln_bwd_wgs(R) * 2D floats of scratch; dgb: [dgamma | dbeta] (2D floats)
void launch_ln_bwd(const float* dy, const float* s, const float* mean, const float* rstd, const float* gamma,
                   float* dx, float* part, float* dgb, int64_t R, int D, hipStream_t st, const LnDrop& dp);
}  // namespace ndp

// ---- convolutions, NCHW fp32 (conv.hip) -------------------------------------------------
namespace ndp {
struct ConvGeom {
  int32_t C, H, W;        // input channels / spatial
  int32_t Co, KH, KW;     // output channels / kernel
  int32_t stride, pad;
  int32_t OH, OW;         // output spatial
};
// Wt_big [Co*OH*OW, C*H*W] <- W [Co, C, KH, KW]  (transposed Toeplitz form of a small-spatial conv)
void launch_toeplitz_expand(const float* w, float* wb, const ConvGeom& g, hipStream_t s);
// several layers' W_big^T in one launch (by-value kernel arguments)
constexpr int kMaxExpand = 24;
struct ExpandBatch {
  const float* w[kMaxExpand];
  float* wt[kMaxExpand];
  ConvGeom g[kMaxExpand];
  int64_t end[kMaxExpand];  // inclusive prefix sums of the W_big^T row counts N = Co*OH*OW
  int n;
};
void launch_toeplitz_expand_many(const ExpandBatch& b, hipStream_t s);
// several layers' grad-W folds in one launch
struct FoldBatch {
  const float* dwt[kMaxExpand];
  float* dw[kMaxExpand];
  ConvGeom g[kMaxExpand];
  int64_t end[kMaxExpand];  // inclusive prefix sums of the (co, ci) pair counts Co*C
  int n;
};
void launch_toeplitz_fold_many(const FoldBatch& b, hipStream_t s);
// several grad-W slab sums in one launch: dw_e = sum over slices of part_e (numel % 4 == 0)
struct SlabBatch {
  const float* part[kMaxExpand];
  float* dw[kMaxExpand];
  int64_t numel[kMaxExpand];
  int slices[kMaxExpand];
  int64_t end[kMaxExpand];  // inclusive prefix sums of blocks (64 floats per block)
  int n;
  int nt;  // non-temporal slab loads (set by launch_slab_sum_many)
};
void launch_slab_sum_many(const SlabBatch& b, hipStream_t s);
// both of the above in one launch (the end-of-backward grad-W finish)
void launch_gradw_finish(const SlabBatch& sb, const FoldBatch& fb, hipStream_t s);
// dW [Co, C, KH, KW] <- fold of dWt_big [Co*OH*OW, C*H*W]  (fixed-order sum, deterministic)
void launch_toeplitz_fold(const float* dwb, float* dw, const ConvGeom& g, hipStream_t s);
// direct fp32-MFMA convolutions: shape class (-1 = none), images per workgroup / slice
int conv_direct_class(const ConvGeom& g);
int conv_fwd_imgs(int cls);
int conv_wgrad_imgs(int cls, const ConvGeom& g, int B);
bool conv_dgrad_direct(int cls);
// split-K factor (1 = none) of the forward / grad-x kernel for batch B; with ksplit > 1 the
// launchers need `part` scratch of ksplit * (compact output) floats: B * outC * OH * OW
// (the stride-2 1x1 grad-x: B * C * 4 * 4 before its even-pixel scatter)
int conv_ksplit(int cls, const ConvGeom& g, int B, bool dgrad);
// defer: with split-K, skip the slab sum and return the number of slabs left in `part`
// (compact output layout, slab = numel(out)); returns 1 when `y` / `dx` holds the result
// stats (nullable; only where conv_fwd_stats_slices > 0): BatchNorm partial sums of y from the
// epilogue, [Co][S][2] fp64 (sum, sum of squares per channel and batch tile)
// BatchNorm partial sums from the epilogue (out != nullptr): forward mode (bx == nullptr) sums
// the output v and v^2 for the BN that consumes it; backward mode sums dz = v * (by > 0) and
// dz * (bx - mean) * invstd for the BN whose output gradient v is (bx / by: that BN's input and
// ReLU output, mean / invstd its saved statistics) — the BN backward's statistics pass
struct ConvBnStats {
  double* out;
  const float* bx;
  const float* by;
  const float* mean;
  const float* invstd;
};
// wino_u (nullable): the conv's Winograd weight transforms (launch_wino_weights: forward + grad-x
// layouts, 32 * Co * C floats) when conv_wino(cls, g, B, dgrad) — the launch then runs the Winograd kernel
// pair: a downsample conv (class 4) forward may be held back and launched together with the next
// class-2 forward of the same input (ds_fwd_pair_kernel); conv_flush_pending_fwd() launches it alone
int launch_conv_fwd(const float* x, const float* w, float* y, int B, const ConvGeom& g, float* part, hipStream_t s,
                    bool defer = false, double* stats = nullptr, float* wino_u = nullptr, bool pair = false);
void conv_flush_pending_fwd();
// stem forward output-row blocks per image (by batch; A/B override 1 / 2 / 4, 0 = auto)
int stem_psplit(int B);
void conv_set_stem_psplit(int p);
int conv_fwd_stats_slices(int cls, const ConvGeom& g, int B);
// addend (nullable, 3x3 classes): dx += addend in the epilogue / split-K sum; with defer the
// slabs are left unsummed and the consumer adds the addend after them (launch_bn_bwd dyadd)
// bst (nullable; the layer1 3x3 class, unsplit: conv_dgrad_stats_slices): backward-mode BN partial
// sums of dx for the BN whose output gradient dx is
int launch_conv_dgrad(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, float* part,
                      hipStream_t s, const float* addend = nullptr, bool defer = false,
                      const ConvBnStats* bst = nullptr, float* wino_u = nullptr);
int conv_dgrad_stats_slices(int cls, const ConvGeom& g, int B);
// Winograd F(2x2, 3x3) path of the 8x8 3x3 classes (winograd.hip): whether a launch takes it,
// and the U scratch it needs (16 * inC * outC floats)
bool conv_wino(int cls, const ConvGeom& g, int B, bool dgrad);
bool wino_ok(int inC, int outC, int B, int H, int W, int ks);
bool wino_disabled();
void wino_set_enabled(bool on);
int wino_imgs(int H);
int64_t wino_u_numel(int inC, int outC);
void launch_wino_weights(const float* w, float* u, int Co, int C, hipStream_t s);
bool wino_wgrad_red(int B, int imgs);
bool wino_wgrad_ok(int C, int Co, int H);
void launch_wino_wgrad(const float* x, const float* dy, float* part, int B, int C, int Co, int H, int imgs,
                       hipStream_t s);
// several layers' transforms in one launch (ops/conv.py WinoBank)
constexpr int kMaxWino = 16;
struct WinoBatch {
  const float* w[kMaxWino];
  float* u[kMaxWino];
  int Co[kMaxWino];
  int C[kMaxWino];
  int end[kMaxWino];  // inclusive prefix sums of the (Co / 16) * (C / 16) block counts
  int n;
};
void launch_wino_weights_many(const WinoBatch& b, hipStream_t s);
void launch_wino_conv(const float* x, const float* u, float* y, int B, int inC, int outC, int H, bool transw,
                      int iups, const float* addend, const ConvBnStats& st, int ks, float* part, hipStream_t s);
// out[i] = sum_{z < nslab} part[z * n + i] (+ addend[i]) in z order (n % 4 == 0), same order as
// the split-K sums; out may alias addend
void launch_slab_sum(const float* part, float* out, int64_t n, int nslab, hipStream_t s,
                     const float* addend = nullptr);
// part: (B / conv_wgrad_imgs(cls, g, B)) * Co*C*KH*KW floats of scratch.  pair: a layer1 Winograd
// grad-W into `part` (dw == nullptr) may be held back and launched together with the next
// launch_conv_dgrad of the same dY (one wino_bwd_pair_kernel launch); conv_flush_pending() launches
// a held-back grad-W on its own (the caller's end of the conv backward)
void launch_conv_wgrad(const float* x, const float* dy, float* part, float* dw, int B, const ConvGeom& g,
                       hipStream_t s, bool pair = false);
void conv_flush_pending();
void launch_wino_bwd_pair(const float* dy, const float* u, float* dx, int B, int inC, int outC, const float* addend,
                          const ConvBnStats& st, int ks, float* part_x, const float* x, float* part_w, int imgs,
                          hipStream_t s);

// ---- strided / tabled implicit-GEMM convolutions (tgemm.hip) ------------------------------
// operand index i -> element offset (i >> sh) * so + (i & (2^sh - 1)) * si
struct TgIndex {
  int64_t so, si;
  int32_t sh, pad;
};
// C[m, n] (+)= sum_k A[m, k] B[k, n];  A(m,k) = a[am(m) + ak(k)], B(k,n) = b[bk(k) + bn(n)];
// C(m,n) = c[cm(m) + cn(n)]; split z writes part + z * slab when part != null
struct TgArgs {
  const float* a;
  const float* b;
  float* c;
  float* part;
  const float* addend;  // C += addend (same offsets; may alias c); single-split launches only
  TgIndex am, ak, bk, bn, cm, cn;
  int32_t M, N, K, kchunk;
  int64_t slab;
};
constexpr int TG_POINTWISE = 0;  // 1x1 stride-1, power-of-two map of >= 2 pixels
int tg_class(const ConvGeom& g);
// the GEMM description of direction dir (pointers null) + the load mappings of its launch
TgArgs tg_args(const ConvGeom& g, int B, int dir, bool* akf, bool* bnf);
// split-K slabs of direction dir (0 fwd, 1 grad-x, 2 grad-W) for batch B (1 = no scratch)
int tg_splits(const ConvGeom& g, int B, int dir);
// defer: leave the split-K slabs in part and return their count (1 = y / dx final)
int launch_tg_fwd(const float* x, const float* w, float* y, int B, const ConvGeom& g, float* part, hipStream_t s,
                  bool defer = false);
// addend (nullable, may alias dx): dx = grad-x + addend (never deferred)
int launch_tg_dgrad(const float* dy, const float* w, float* dx, int B, const ConvGeom& g, float* part,
                    hipStream_t s, const float* addend = nullptr, bool defer = false);
// POINTWISE: out = dW; SMALL: out = dWbig^T [Co*OH*OW, C*H*W] (fold with toeplitz_fold).
// defer: leave the split-K slabs in part, return their count (1 = out final)
int launch_tg_wgrad(const float* x, const float* dy, float* out, int B, const ConvGeom& g, float* part,
                    hipStream_t s, bool defer = false);
}  // namespace ndp

// ---- fused fp32 attention, q/k/v/o [B, S, H, 64] (attention.hip) ------------------------
namespace ndp {
// mask: [B, S] int32 (nonzero = attend) or null; lse: [B, H, S]; p_drop in [0, 1);
// seed: device int32[1] read by the kernels (so a replayed hipGraph sees fresh seeds)
void launch_attn_fwd(const float* q, const float* k, const float* v, const int32_t* mask, float* o, float* lse,
                     int B, int S, int H, float scale, const int32_t* seed, float p_drop, hipStream_t s,
                     int64_t ldq = 0);
// ldq: token row stride of q / k / v (and dq / dk / dv): 0 = H*64 (contiguous), 3*H*64 for
// views into a packed [B, S, 3, H, 64] QKV projection.  delta: [B, H, S] scratch
void launch_attn_bwd(const float* q, const float* k, const float* v, const int32_t* mask, const float* o,
                     const float* dout, const float* lse, float* delta, float* dq, float* dk, float* dv, int B,
                     int S, int H, float scale, const int32_t* seed, float p_drop, hipStream_t s,
                     int64_t ldq = 0);
}  // namespace ndp

// ---- max-pool 2-D, NCHW fp32, deterministic gather backward (pool.hip) ---------------
namespace ndp {
struct PoolGeom {
  int32_t H, W, OH, OW;
  int32_t KH, KW, stride, pad;
};
// idx: uint8 window offset (kh*KW + kw) of each output's maximum
void launch_maxpool_fwd(const float* x, float* y, uint8_t* idx, int planes, const PoolGeom& g, hipStream_t s);
// BatchNorm backward statistics from the pool backward (stats != nullptr; ResNet stem tail, the
// BN output never stored): per plane (n, c) the sums of dz = dx * mask(x) and dz * xhat into
// stats[(c * N + n) * 2], the mask recomputed from x as bn_relu_maxpool computed its output
struct PoolBnStats {
  const float* x;
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* invstd;
  double* stats;
  int C, N;
};
bool maxpool_bwd_bnstats_ok(const PoolGeom& g);
// the stem BN input gradient straight from the pooled gradient (batchnorm.hip): 16x16 -> 8x8 maps,
// statistics [C][N][2] from the statistics-only pool backward
void launch_stem_pool_bwd_apply(const float* dy, const uint8_t* idx, const float* x, const float* gamma,
                                const float* beta, const float* save_mean, const float* save_invstd,
                                const double* stats, float* dx, float* dgamma, float* dbeta, int N, int C, int H,
                                int W, hipStream_t s);
void launch_maxpool_bwd(const float* dy, const uint8_t* idx, float* dx, int planes, const PoolGeom& g,
                        hipStream_t s,
                        const PoolBnStats& bs = PoolBnStats{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0});
}  // namespace ndp
