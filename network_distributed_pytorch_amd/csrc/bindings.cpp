// pybind11 bindings for the gfx950 kernels and the host plan builder.
//
// Every entry point enqueues on the caller's current HIP stream (so the Python layer can
// place work on a side stream, overlap it with backward and capture it in a hipGraph),
// never synchronises and never allocates.
#include <algorithm>
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <cstring>

#include "ndp_kernels.h"
#include "plan.h"

namespace {

using ndp::MatGeom;
using ndp::MatPtrs;
using ndp::PItem;
using ndp::QItem;
using ndp::SegEntry;
using ndp::UItem;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// surface launch-configuration errors immediately (no device sync)
void check_launch(const char* what) {
  const hipError_t err = hipGetLastError();
  TORCH_CHECK(err == hipSuccess, what, ": ", hipGetErrorString(err));
}

void check_dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device (HIP) tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_f32(const torch::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

template <typename T>
torch::Tensor to_bytes(const std::vector<T>& v) {
  auto t = torch::empty({(int64_t)(v.size() * sizeof(T))}, torch::dtype(torch::kUInt8));
  if (!v.empty()) std::memcpy(t.data_ptr(), v.data(), v.size() * sizeof(T));
  return t;
}

py::dict build_plan(const std::vector<std::pair<int64_t, int64_t>>& shapes, int rank) {
  ndp::Plan pl = ndp::build_plan(shapes, rank);
  py::dict d;
  d["geom"] = to_bytes(pl.geom);
  d["p_items"] = to_bytes(pl.p_items);
  d["q_items"] = to_bytes(pl.q_items);
  d["u_items"] = to_bytes(pl.u_items);
  d["orth_items"] = to_bytes(pl.orth_items);
  d["n_orth_items"] = (int64_t)pl.orth_items.size();
  d["n_mats"] = (int64_t)pl.geom.size();
  d["n_p_items"] = (int64_t)pl.p_items.size();
  d["n_q_items"] = (int64_t)pl.q_items.size();
  d["n_u_items"] = (int64_t)pl.u_items.size();
  d["p_total"] = pl.p_total;
  d["q_total"] = pl.q_total;
  d["pp_total"] = pl.pp_total;
  d["qp_total"] = pl.qp_total;
  d["max_rank"] = pl.max_rank;
  d["n_p_blocks"] = pl.n_p_blocks;
  d["p_cols"] = (int64_t)pl.p_cols;
  d["n_q_blocks"] = pl.n_q_blocks;
  // first work item of every matrix (+ sentinel) in each list: a PowerSGD group of
  // matrices [lo, hi) launches the contiguous item slice [start[lo], start[hi])
  auto starts = [&](auto const& items) {
    py::list out;
    size_t k = 0;
    for (size_t i = 0; i <= pl.geom.size(); ++i) {
      while (k < items.size() && (size_t)items[k].mat < i) ++k;
      out.append((int64_t)k);
    }
    return out;
  };
  d["p_item_start"] = starts(pl.p_items);
  d["q_item_start"] = starts(pl.q_items);
  d["u_item_start"] = starts(pl.u_items);
  d["orth_item_start"] = starts(pl.orth_items);
  py::list rs, poff, qoff, ppoff, qpoff, pch, qch, qrows;
  for (size_t i = 0; i < pl.geom.size(); ++i) {
    rs.append(pl.geom[i].r);
    poff.append(pl.geom[i].p_off);
    qoff.append(pl.geom[i].q_off);
    ppoff.append(pl.geom[i].pp_off);
    qpoff.append(pl.geom[i].qp_off);
    pch.append(pl.geom[i].p_chunks);
    qch.append(pl.geom[i].q_chunks);
    qrows.append(pl.q_rows[i]);
  }
  d["ranks"] = rs;
  d["p_offs"] = poff;
  d["q_offs"] = qoff;
  d["pp_offs"] = ppoff;
  d["qp_offs"] = qpoff;
  d["p_chunks"] = pch;
  d["q_chunks"] = qch;
  d["q_rows"] = qrows;
  return d;
}

// geom bytes (host) with per-matrix `vec` flags patched in
torch::Tensor patch_geom_vec(torch::Tensor geom, const std::vector<int>& vec) {
  TORCH_CHECK(!geom.is_cuda() && geom.scalar_type() == torch::kUInt8, "geom must be host bytes");
  auto out = geom.clone();
  auto* g = reinterpret_cast<MatGeom*>(out.data_ptr());
  const int64_t n = out.numel() / (int64_t)sizeof(MatGeom);
  TORCH_CHECK((int64_t)vec.size() == n, "vec flags size mismatch");
  for (int64_t i = 0; i < n; ++i) g[i].vec = vec[i];
  return out;
}

// ptrs: list of 8-tuples of raw addresses (0 = null) -> host bytes
torch::Tensor make_mat_ptrs(const std::vector<std::vector<int64_t>>& rows) {
  std::vector<MatPtrs> v(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    TORCH_CHECK(rows[i].size() == 8, "MatPtrs row needs 8 addresses");
    int64_t* dst = reinterpret_cast<int64_t*>(&v[i]);
    for (int k = 0; k < 8; ++k) dst[k] = rows[i][k];
  }
  return to_bytes(v);
}

// specs: (src_addr, dst_addr, numel, stride, chunks, div)
py::tuple make_seg_table(const std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t, int, double>>& specs) {
  std::vector<ndp::SegSpec> s;
  s.reserve(specs.size());
  for (const auto& t : specs) {
    ndp::SegSpec x{};
    x.src = (uintptr_t)std::get<0>(t);
    x.dst = (uintptr_t)std::get<1>(t);
    x.numel = std::get<2>(t);
    x.stride = std::get<3>(t);
    x.chunks = std::get<4>(t);
    x.div = (float)std::get<5>(t);
    s.push_back(x);
  }
  ndp::SegTable tab = ndp::build_seg_table(s);
  auto prefix = torch::empty({(int64_t)tab.prefix.size()}, torch::dtype(torch::kInt64));
  if (!tab.prefix.empty())
    std::memcpy(prefix.data_ptr(), tab.prefix.data(), tab.prefix.size() * sizeof(int64_t));
  return py::make_tuple(to_bytes(tab.entries), prefix, (int64_t)tab.entries.size(), tab.n_blocks);
}

// geometry + work list for a standalone batched orthogonalisation: rows of (n, r, p_off)
py::tuple make_orth_geom(const std::vector<std::tuple<int64_t, int64_t, int64_t>>& mats) {
  std::vector<MatGeom> v(mats.size());
  int max_rank = 1;
  for (size_t i = 0; i < mats.size(); ++i) {
    v[i] = MatGeom{};
    v[i].n = (int32_t)std::get<0>(mats[i]);
    v[i].r = (int32_t)std::get<1>(mats[i]);
    TORCH_CHECK(v[i].r >= 1 && v[i].r <= ndp::kMaxRank, "orthogonalize supports 1..64 columns");
    v[i].m = v[i].r;
    v[i].p_off = (int32_t)std::get<2>(mats[i]);
    max_rank = std::max<int>(max_rank, v[i].r);
  }
  auto items = ndp::build_orth_items(v, max_rank);
  return py::make_tuple(to_bytes(v), to_bytes(items), (int64_t)items.size(), max_rank);
}

int64_t n_of(const torch::Tensor& bytes, size_t sz) { return bytes.numel() / (int64_t)sz; }

using OptT = c10::optional<torch::Tensor>;

unsigned long long* ctr_ptr(const torch::Tensor& c, int64_t need, const char* what) {
  check_dev(c, what);
  TORCH_CHECK(c.scalar_type() == torch::kInt64 && c.numel() >= need, what, ": int64 counters, one per block");
  return reinterpret_cast<unsigned long long*>(c.data_ptr());
}

// p_out + p_ctr: in-kernel split-K finish (P written into p_out, wide plans only); seg_*: the
// rank-1 pack run by the same launch's extra blocks
void psgd_p(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor q_warm,
            torch::Tensor p_part, bool fuse_ef, int max_rank, OptT p_prev, OptT p_out, OptT p_ctr,
            OptT seg_entries, OptT seg_prefix, int64_t seg_n, int64_t seg_blocks, int64_t p_cols) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(q_warm, "q_warm"); check_f32(p_part, "p_part");
  const float* pp = nullptr;
  if (p_prev.has_value()) {
    check_f32(*p_prev, "p_prev");
    TORCH_CHECK(fuse_ef && max_rank <= ndp::kUWideMaxRank, "psgd_p: lazy error feedback needs fuse_ef, rank <= 16");
    pp = p_prev->data_ptr<float>();
  }
  const int n_items = (int)n_of(items, sizeof(PItem));
  ndp::PFin fin{};
  if (p_out.has_value()) {
    TORCH_CHECK(max_rank <= ndp::kUWideMaxRank, "psgd_p: in-kernel split-K finish needs rank <= 16");
    TORCH_CHECK(p_ctr.has_value(), "psgd_p: p_out needs p_ctr");
    check_f32(*p_out, "p_out");
    fin.out = p_out->data_ptr<float>();
    fin.ctr = ctr_ptr(*p_ctr, 1, "p_ctr");  // sized n_p_blocks by the plan (parallel/powersgd.py)
  }
  int64_t nsb = 0;
  if (seg_entries.has_value() && seg_n > 0 && seg_blocks > 0) {
    TORCH_CHECK(max_rank <= ndp::kUWideMaxRank, "psgd_p: fused rank-1 pack needs rank <= 16");
    TORCH_CHECK(seg_prefix.has_value(), "psgd_p: seg table needs its prefix");
    check_dev(*seg_entries, "seg_entries"); check_dev(*seg_prefix, "seg_prefix");
    TORCH_CHECK(seg_entries->numel() >= seg_n * (int64_t)sizeof(SegEntry) && seg_prefix->numel() >= seg_n,
                "seg table size mismatch");
    fin.seg = reinterpret_cast<const SegEntry*>(seg_entries->data_ptr());
    fin.seg_prefix = seg_prefix->data_ptr<int64_t>();
    fin.n_seg = (int)seg_n;
    nsb = seg_blocks;
  }
  ndp::launch_psgd_p(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                     reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                     reinterpret_cast<const PItem*>(items.data_ptr()), n_items, q_warm.data_ptr<float>(),
                     p_part.data_ptr<float>(), fuse_ef ? 1 : 0, max_rank, cur_stream(), pp, fin, nsb, (int)p_cols);
  check_launch("launch_psgd_p");
}

void psgd_q(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor p_hat,
            torch::Tensor q_part, int max_rank, OptT q_out, OptT q_ctr, int64_t q_fin_max) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(p_hat, "p_hat"); check_f32(q_part, "q_part");
  ndp::QFin fin{};
  if (q_out.has_value()) {
    TORCH_CHECK(q_ctr.has_value(), "psgd_q: q_out needs q_ctr");
    check_f32(*q_out, "q_out");
    fin.out = q_out->data_ptr<float>();
    fin.ctr = ctr_ptr(*q_ctr, 1, "q_ctr");
    fin.max_chunks = (int)q_fin_max;
  }
  ndp::launch_psgd_q(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                     reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                     reinterpret_cast<const QItem*>(items.data_ptr()),
                     (int)n_of(items, sizeof(QItem)), p_hat.data_ptr<float>(),
                     q_part.data_ptr<float>(), max_rank, cur_stream(), fin);
  check_launch("launch_psgd_q");
}

// scratch: float32 tensor of >= 2*n_items*kMaxRank partials; ctr: int64 tensor of
// >= n_mats + 1 words (64-bit counters, then the uint32 error word in word n_mats)
// items may be a slice of the plan's full item list (one PowerSGD group); n_items_total
// (the full list's length, -1 = this slice) fixes the double-buffered slab layout
void psgd_orth(torch::Tensor geom, torch::Tensor items, torch::Tensor p, double p_div, double eps,
               int max_rank, torch::Tensor scratch, torch::Tensor ctr, int64_t n_items_total,
               int64_t max_spins) {
  check_dev(geom, "geom"); check_dev(items, "items"); check_f32(p, "p"); check_f32(scratch, "scratch");
  check_dev(ctr, "ctr");
  const int n_items = (int)n_of(items, sizeof(ndp::OrthItem));
  const int n_total = n_items_total < 0 ? n_items : (int)n_items_total;
  TORCH_CHECK(n_total >= n_items, "orth: n_items_total smaller than the item slice");
  const int n_mats = (int)n_of(geom, sizeof(MatGeom));
  TORCH_CHECK(scratch.numel() >= 2LL * n_total * ndp::kMaxRank, "orth scratch too small");
  // [n_mats x uint64 barrier counters][uint32 error word]
  TORCH_CHECK(ctr.numel() * ctr.element_size() >= 8LL * n_mats + 4, "orth counters too small");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(ctr.data_ptr()) & 7) == 0, "orth counters: 8-B aligned");
  auto* c = reinterpret_cast<unsigned long long*>(ctr.data_ptr());
  ndp::launch_psgd_orth(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                        reinterpret_cast<const ndp::OrthItem*>(items.data_ptr()), n_items, n_mats,
                        p.data_ptr<float>(), (float)p_div, (float)eps, max_rank,
                        scratch.data_ptr<float>(), c, reinterpret_cast<unsigned*>(c + n_mats), n_total,
                        max_spins < 0 ? ndp::kOrthMaxSpins : (unsigned)max_spins, cur_stream());
  check_launch("launch_psgd_orth");
}

void psgd_update(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor p_hat,
                 torch::Tensor q_sum, double q_div, c10::optional<torch::Tensor> q_warm, int mode,
                 double lr, double momentum, int max_rank, c10::optional<torch::Tensor> p_prev,
                 OptT r1_buf, double r1_div, OptT r1_mom, OptT r1_x, OptT r1_g) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(p_hat, "p_hat"); check_f32(q_sum, "q_sum");
  TORCH_CHECK(mode >= 0 && mode <= 3, "psgd_update: mode 0..3");
  TORCH_CHECK((mode != 3 && !p_prev.has_value()) || max_rank <= ndp::kUWideMaxRank,
              "psgd_update: lazy error feedback / materialise need rank <= 16");
  float* qw = nullptr;
  if (q_warm.has_value()) { check_f32(*q_warm, "q_warm"); qw = q_warm->data_ptr<float>(); }
  float* pp = nullptr;
  if (p_prev.has_value()) { check_f32(*p_prev, "p_prev"); pp = p_prev->data_ptr<float>(); }
  ndp::R1Step r1{};
  if (r1_buf.has_value()) {  // the rank-1 group's step rides in the same launch
    TORCH_CHECK(mode == 1 || mode == 2, "psgd_update: the rank-1 step needs the engine modes 1 / 2");
    TORCH_CHECK(r1_mom.has_value() && r1_x.has_value(), "psgd_update: rank-1 step needs mom and x");
    check_f32(*r1_buf, "r1_buf"); check_f32(*r1_mom, "r1_mom"); check_f32(*r1_x, "r1_x");
    TORCH_CHECK(r1_buf->numel() == r1_mom->numel() && r1_buf->numel() == r1_x->numel(), "rank-1 size mismatch");
    r1.buf = r1_buf->data_ptr<float>();
    r1.mom = r1_mom->data_ptr<float>();
    r1.x = r1_x->data_ptr<float>();
    if (r1_g.has_value()) {
      check_f32(*r1_g, "r1_g");
      TORCH_CHECK(r1_g->numel() == r1_buf->numel(), "rank-1 size mismatch");
      r1.g = r1_g->data_ptr<float>();
    }
    r1.n = r1_buf->numel();
    r1.div = (float)r1_div;
  }
  ndp::launch_psgd_update(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                          reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                          reinterpret_cast<const UItem*>(items.data_ptr()),
                          (int)n_of(items, sizeof(UItem)), p_hat.data_ptr<float>(),
                          q_sum.data_ptr<float>(), (float)q_div, qw, mode, (float)lr,
                          (float)momentum, max_rank, cur_stream(), pp, r1);
  check_launch("launch_psgd_update");
}

void rank1_step(torch::Tensor buf, double div, torch::Tensor mom, torch::Tensor x,
                c10::optional<torch::Tensor> g, double lr, double momentum) {
  check_f32(buf, "buf"); check_f32(mom, "mom"); check_f32(x, "x");
  TORCH_CHECK(buf.numel() == mom.numel() && buf.numel() == x.numel(), "rank1_step size mismatch");
  float* gp = nullptr;
  if (g.has_value()) {
    check_f32(*g, "g");
    TORCH_CHECK(g->numel() == buf.numel(), "rank1_step size mismatch");
    gp = g->data_ptr<float>();
  }
  ndp::launch_rank1_step(buf.data_ptr<float>(), (float)div, mom.data_ptr<float>(),
                         x.data_ptr<float>(), gp, buf.numel(), (float)lr, (float)momentum,
                         cur_stream());
  check_launch("launch_rank1_step");
}

void seg_reduce(torch::Tensor entries, torch::Tensor prefix, int64_t n_entries, int64_t n_blocks) {
  check_dev(entries, "entries"); check_dev(prefix, "prefix");
  TORCH_CHECK(entries.numel() >= n_entries * (int64_t)sizeof(SegEntry) && prefix.numel() >= n_entries,
              "seg table size mismatch");
  ndp::launch_seg_reduce(reinterpret_cast<const SegEntry*>(entries.data_ptr()),
                         prefix.data_ptr<int64_t>(), (int)n_entries, n_blocks, cur_stream());
  check_launch("launch_seg_reduce");
}

void sgd_momentum(torch::Tensor x, torch::Tensor g, torch::Tensor buf, double lr, double mu,
                  double div) {
  check_f32(x, "x"); check_f32(g, "g"); check_f32(buf, "buf");
  TORCH_CHECK(x.numel() == g.numel() && x.numel() == buf.numel(), "sgd_momentum size mismatch");
  ndp::launch_sgd_momentum(x.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(),
                           x.numel(), (float)lr, (float)mu, (float)div, cur_stream());
  check_launch("launch_sgd_momentum");
}

void add(torch::Tensor a, torch::Tensor b, torch::Tensor out) {
  check_f32(a, "a"); check_f32(b, "b"); check_f32(out, "out");
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == out.numel(), "add size mismatch");
  ndp::launch_add(a.data_ptr<float>(), b.data_ptr<float>(), out.data_ptr<float>(), a.numel(),
                  cur_stream());
  check_launch("launch_add");
}

const float* opt_f32(const c10::optional<torch::Tensor>& t, const char* name) {
  if (!t.has_value()) return nullptr;
  check_f32(*t, name);
  return t->data_ptr<float>();
}

// deferred split-K slabs of a conv output (ops/slablink.py): nslab slabs of `numel` floats
const float* slab_input(const c10::optional<torch::Tensor>& part, int64_t nslab, int64_t numel, const char* who) {
  if (!part.has_value() || nslab < 2) return nullptr;
  check_f32(*part, "slab part");
  TORCH_CHECK(numel % 4 == 0 && part->numel() >= nslab * numel, who, ": slab scratch too small");
  return part->data_ptr<float>();
}

// out = sum of nslab split-K slabs (a deferred conv sum that found no fused consumer)
void slab_sum(torch::Tensor part, torch::Tensor out, int64_t nslab) {
  check_f32(out, "out");
  TORCH_CHECK(out.is_contiguous(), "slab_sum: contiguous output");
  const float* p = slab_input(part, nslab, out.numel(), "slab_sum");
  TORCH_CHECK(p != nullptr, "slab_sum: needs >= 2 slabs");
  ndp::launch_slab_sum(p, out.data_ptr<float>(), out.numel(), (int)nslab, cur_stream());
  check_launch("launch_slab_sum");
}

// fused BN(+res)(+relu) forward; returns nothing, writes y / save_mean / save_invstd
void bn_fwd(torch::Tensor x, c10::optional<torch::Tensor> res, torch::Tensor y,
            c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
            c10::optional<torch::Tensor> rmean, c10::optional<torch::Tensor> rvar,
            c10::optional<torch::Tensor> nbt, torch::Tensor save_mean, torch::Tensor save_invstd,
            torch::Tensor part, double eps, double momentum, bool relu, bool training,
            bool single, c10::optional<torch::Tensor> xpart, int64_t nslab,
            c10::optional<torch::Tensor> xstats, int64_t xS) {
  check_f32(x, "x"); check_f32(y, "y"); check_f32(save_mean, "save_mean"); check_f32(save_invstd, "save_invstd");
  check_dev(part, "part");
  TORCH_CHECK(x.dim() >= 2 && x.sizes() == y.sizes(), "bn_fwd: bad shapes");
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int HW = (int)(x.numel() / ((int64_t)N * C));
  const int S = ndp::bn_slices(N, C, HW);
  TORCH_CHECK(part.scalar_type() == torch::kFloat64 && part.numel() >= ndp::bn_part_numel(N, C, HW),
              "bn part too small");
  TORCH_CHECK(save_mean.numel() >= C && save_invstd.numel() >= C, "bn save buffers too small");
  if (res.has_value()) TORCH_CHECK(res->sizes() == x.sizes(), "bn residual shape");
  int64_t* nb = nullptr;
  if (nbt.has_value()) {
    check_dev(*nbt, "nbt");
    TORCH_CHECK(nbt->scalar_type() == torch::kInt64, "num_batches_tracked must be int64");
    nb = nbt->data_ptr<int64_t>();
  }
  const float* xp = slab_input(xpart, nslab, x.numel(), "bn_fwd");
  TORCH_CHECK(xp == nullptr || training, "bn_fwd: deferred conv slabs need training mode");
  const double* xst = nullptr;
  if (xstats.has_value()) {  // [C][xS][2] partial sums from the producing conv's epilogue
    check_dev(*xstats, "xstats");
    TORCH_CHECK(xstats->scalar_type() == torch::kFloat64 && xstats->is_contiguous() && xS > 0 &&
                    xstats->numel() >= (int64_t)C * xS * 2 && training && xp == nullptr,
                "bn_fwd: xstats must hold C * xS * 2 doubles (training, no deferred slabs)");
    xst = xstats->data_ptr<double>();
  }
  ndp::launch_bn_fwd(x.data_ptr<float>(), opt_f32(res, "res"), y.data_ptr<float>(), opt_f32(gamma, "gamma"),
                     opt_f32(beta, "beta"), const_cast<float*>(opt_f32(rmean, "running_mean")),
                     const_cast<float*>(opt_f32(rvar, "running_var")), nb, save_mean.data_ptr<float>(),
                     save_invstd.data_ptr<float>(), part.data_ptr<double>(), N, C, HW, S, (float)eps,
                     (float)momentum, relu ? 1 : 0, training ? 1 : 0, single ? 1 : 0, cur_stream(), xp, (int)nslab,
                     xst, (int)xS);
  check_launch("launch_bn_fwd");
}

// training BN -> ReLU -> MaxPool(3, 2, 1) without storing the BN output (the ResNet stem tail)
void bn_relu_maxpool(torch::Tensor x, torch::Tensor y, torch::Tensor idx, c10::optional<torch::Tensor> gamma,
                     c10::optional<torch::Tensor> beta, c10::optional<torch::Tensor> rmean,
                     c10::optional<torch::Tensor> rvar, c10::optional<torch::Tensor> nbt, torch::Tensor save_mean,
                     torch::Tensor save_invstd, torch::Tensor part, double eps, double momentum,
                     c10::optional<torch::Tensor> xstats, int64_t xS) {
  check_f32(x, "x"); check_f32(y, "y"); check_f32(save_mean, "save_mean"); check_f32(save_invstd, "save_invstd");
  check_dev(part, "part"); check_dev(idx, "idx");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "bn_relu_maxpool: contiguous NCHW x");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(y.is_contiguous() && y.dim() == 4 && y.size(0) == N && y.size(1) == C && y.size(2) == OH &&
                  y.size(3) == OW, "bn_relu_maxpool: y must be [N, C, (H-1)/2+1, (W-1)/2+1]");
  TORCH_CHECK(idx.scalar_type() == torch::kUInt8 && idx.is_contiguous() && idx.sizes() == y.sizes(),
              "bn_relu_maxpool: uint8 idx shaped like y");
  TORCH_CHECK(part.scalar_type() == torch::kFloat64 && part.numel() >= ndp::bn_part_numel(N, C, H * W),
              "bn part too small");
  TORCH_CHECK(save_mean.numel() >= C && save_invstd.numel() >= C, "bn save buffers too small");
  TORCH_CHECK((int64_t)N * C * H * W < (1LL << 31), "bn_relu_maxpool: tensor too large");
  int64_t* nb = nullptr;
  if (nbt.has_value()) {
    check_dev(*nbt, "nbt");
    TORCH_CHECK(nbt->scalar_type() == torch::kInt64, "num_batches_tracked must be int64");
    nb = nbt->data_ptr<int64_t>();
  }
  const double* xst = nullptr;
  if (xstats.has_value()) {
    check_dev(*xstats, "xstats");
    TORCH_CHECK(xstats->scalar_type() == torch::kFloat64 && xstats->is_contiguous() && xS > 0 &&
                    xstats->numel() >= (int64_t)C * xS * 2, "bn_relu_maxpool: xstats must hold C * xS * 2 doubles");
    xst = xstats->data_ptr<double>();
  }
  ndp::launch_bn_relu_maxpool(x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(),
                              opt_f32(gamma, "gamma"), opt_f32(beta, "beta"),
                              const_cast<float*>(opt_f32(rmean, "running_mean")),
                              const_cast<float*>(opt_f32(rvar, "running_var")), nb, save_mean.data_ptr<float>(),
                              save_invstd.data_ptr<float>(), part.data_ptr<double>(), N, C, H, W, (float)eps,
                              (float)momentum, cur_stream(), xst, (int)xS);
  check_launch("launch_bn_relu_maxpool");
}

void bn_bwd(torch::Tensor dy, c10::optional<torch::Tensor> y, torch::Tensor x, c10::optional<torch::Tensor> gamma,
            torch::Tensor save_mean, torch::Tensor save_invstd, torch::Tensor dx, c10::optional<torch::Tensor> dres,
            c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta, torch::Tensor part,
            bool relu, bool single, c10::optional<torch::Tensor> dypart, int64_t nslab,
            c10::optional<torch::Tensor> dyadd, c10::optional<torch::Tensor> mbeta,
            c10::optional<torch::Tensor> dstats, int64_t dS) {
  check_f32(dy, "dy"); check_f32(x, "x"); check_f32(dx, "dx"); check_dev(part, "part");
  if (dyadd.has_value()) {
    check_f32(*dyadd, "dyadd");
    TORCH_CHECK(dyadd->sizes() == dy.sizes() && dyadd->is_contiguous() && dypart.has_value(),
                "bn_bwd: dyadd (the deferred grad-x addend) must match dy and come with dypart");
  }
  TORCH_CHECK(dy.sizes() == x.sizes() && dx.sizes() == x.sizes(), "bn_bwd: bad shapes");
  TORCH_CHECK(!relu || y.has_value() || mbeta.has_value(), "bn_bwd: relu needs y (or mbeta)");
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int HW = (int)(x.numel() / ((int64_t)N * C));
  const int S = ndp::bn_slices(N, C, HW);
  TORCH_CHECK(part.scalar_type() == torch::kFloat64 && part.numel() >= ndp::bn_part_numel(N, C, HW),
              "bn part too small");
  const double* dst = nullptr;
  if (dstats.has_value()) {  // [C][dS][2] partial sums from the producing conv's grad-x epilogue
    check_dev(*dstats, "dstats");
    TORCH_CHECK(dstats->scalar_type() == torch::kFloat64 && dstats->is_contiguous() && dS > 0 &&
                    dstats->numel() >= (int64_t)C * dS * 2 && !dypart.has_value(),
                "bn_bwd: dstats must hold C * dS * 2 doubles (no slabs)");
    dst = dstats->data_ptr<double>();
  }
  if (mbeta.has_value()) {  // ReLU mask recomputed from x: the vectorised two-kernel path only
    check_f32(*mbeta, "mbeta");
    TORCH_CHECK(relu && !y.has_value() && !dypart.has_value() && mbeta->numel() >= C && HW % 4 == 0 &&
                    ndp::bn_two_kernel_path(N, C, HW, single ? 1 : 0),
                "bn_bwd: mbeta needs relu, no y, no slabs, HW % 4 == 0 and the large-map path");
  }
  ndp::launch_bn_bwd(dy.data_ptr<float>(), opt_f32(y, "y"), x.data_ptr<float>(), opt_f32(gamma, "gamma"),
                     save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(), dx.data_ptr<float>(),
                     const_cast<float*>(opt_f32(dres, "dres")), const_cast<float*>(opt_f32(dgamma, "dgamma")),
                     const_cast<float*>(opt_f32(dbeta, "dbeta")), part.data_ptr<double>(), N, C, HW, S,
                     relu ? 1 : 0, single ? 1 : 0, cur_stream(), slab_input(dypart, nslab, dy.numel(), "bn_bwd"),
                     (int)nslab, opt_f32(dyadd, "dyadd"), opt_f32(mbeta, "mbeta"), dst, (int)dS);
  check_launch("launch_bn_bwd");
}

// the downsample block's relu(BN(x) + BN2(x2)) in one launch (training); momentum applies to both
void bn_pair_fwd(torch::Tensor x, torch::Tensor x2, torch::Tensor y, torch::Tensor gamma, torch::Tensor beta,
                 torch::Tensor rmean, torch::Tensor rvar, torch::Tensor nbt, torch::Tensor save_mean,
                 torch::Tensor save_invstd, torch::Tensor gamma2, torch::Tensor beta2, torch::Tensor rmean2,
                 torch::Tensor rvar2, torch::Tensor nbt2, torch::Tensor save_mean2, torch::Tensor save_invstd2,
                 double eps, double momentum, c10::optional<torch::Tensor> xpart, int64_t nslab,
                 c10::optional<torch::Tensor> x2part, int64_t nslab2) {
  for (auto* t : {&x, &x2, &y, &gamma, &beta, &rmean, &rvar, &save_mean, &save_invstd, &gamma2, &beta2, &rmean2,
                  &rvar2, &save_mean2, &save_invstd2})
    check_f32(*t, "bn_pair_fwd operand");
  TORCH_CHECK(x.dim() >= 2 && x.sizes() == y.sizes() && x.sizes() == x2.sizes() && x.is_contiguous() &&
                  x2.is_contiguous() && y.is_contiguous(), "bn_pair_fwd: x, x2, y must be contiguous, one shape");
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int HW = (int)(x.numel() / ((int64_t)N * C));
  TORCH_CHECK(ndp::bn_pair_ok(N, C, HW), "bn_pair_fwd: shape outside the single-launch path (bn_pair_ok)");
  for (auto* t : {&gamma, &beta, &rmean, &rvar, &save_mean, &save_invstd, &gamma2, &beta2, &rmean2, &rvar2,
                  &save_mean2, &save_invstd2})
    TORCH_CHECK(t->numel() >= C, "bn_pair_fwd: per-channel operand too small");
  check_dev(nbt, "nbt"); check_dev(nbt2, "nbt2");
  TORCH_CHECK(nbt.scalar_type() == torch::kInt64 && nbt2.scalar_type() == torch::kInt64, "num_batches_tracked int64");
  ndp::launch_bn_pair_fwd(x.data_ptr<float>(), x2.data_ptr<float>(), y.data_ptr<float>(), gamma.data_ptr<float>(),
                          beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                          nbt.data_ptr<int64_t>(), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                          gamma2.data_ptr<float>(), beta2.data_ptr<float>(), rmean2.data_ptr<float>(),
                          rvar2.data_ptr<float>(), nbt2.data_ptr<int64_t>(), save_mean2.data_ptr<float>(),
                          save_invstd2.data_ptr<float>(), N, C, HW, (float)eps, (float)momentum, cur_stream(),
                          slab_input(xpart, nslab, x.numel(), "bn_pair_fwd"), (int)nslab,
                          slab_input(x2part, nslab2, x.numel(), "bn_pair_fwd"), (int)nslab2);
  check_launch("launch_bn_pair_fwd");
}

void bn_pair_bwd(torch::Tensor dy, torch::Tensor y, torch::Tensor x, torch::Tensor x2, torch::Tensor gamma,
                 torch::Tensor save_mean, torch::Tensor save_invstd, torch::Tensor gamma2, torch::Tensor save_mean2,
                 torch::Tensor save_invstd2, torch::Tensor dx, torch::Tensor dx2, torch::Tensor dgamma,
                 torch::Tensor dbeta, torch::Tensor dgamma2, torch::Tensor dbeta2, c10::optional<torch::Tensor> dypart,
                 int64_t nslab, c10::optional<torch::Tensor> dyadd) {
  for (auto* t : {&dy, &y, &x, &x2, &gamma, &save_mean, &save_invstd, &gamma2, &save_mean2, &save_invstd2, &dx, &dx2,
                  &dgamma, &dbeta, &dgamma2, &dbeta2})
    check_f32(*t, "bn_pair_bwd operand");
  for (auto* t : {&dy, &y, &x2, &dx, &dx2})
    TORCH_CHECK(t->sizes() == x.sizes() && t->is_contiguous(), "bn_pair_bwd: tensors must be contiguous, one shape");
  TORCH_CHECK(x.is_contiguous(), "bn_pair_bwd: contiguous x");
  if (dyadd.has_value()) {
    check_f32(*dyadd, "dyadd");
    TORCH_CHECK(dyadd->sizes() == dy.sizes() && dyadd->is_contiguous() && dypart.has_value(),
                "bn_pair_bwd: dyadd must match dy and come with dypart");
  }
  const int N = (int)x.size(0), C = (int)x.size(1);
  const int HW = (int)(x.numel() / ((int64_t)N * C));
  TORCH_CHECK(ndp::bn_pair_ok(N, C, HW), "bn_pair_bwd: shape outside the single-launch path (bn_pair_ok)");
  ndp::launch_bn_pair_bwd(dy.data_ptr<float>(), y.data_ptr<float>(), x.data_ptr<float>(), x2.data_ptr<float>(),
                          gamma.data_ptr<float>(), save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                          gamma2.data_ptr<float>(), save_mean2.data_ptr<float>(), save_invstd2.data_ptr<float>(),
                          dx.data_ptr<float>(), dx2.data_ptr<float>(), dgamma.data_ptr<float>(),
                          dbeta.data_ptr<float>(), dgamma2.data_ptr<float>(), dbeta2.data_ptr<float>(), N, C, HW,
                          cur_stream(), slab_input(dypart, nslab, dy.numel(), "bn_pair_bwd"), (int)nslab,
                          opt_f32(dyadd, "dyadd"));
  check_launch("launch_bn_pair_bwd");
}

// max-pool 2-D (stride/pad symmetric, dilation 1, floor mode): x [N, C, H, W] -> y, idx [N, C, OH, OW]
static ndp::PoolGeom pool_geom(const torch::Tensor& x, const torch::Tensor& y, int64_t k, int64_t stride,
                               int64_t pad) {
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(1) == y.size(1),
              "maxpool: bad shapes");
  TORCH_CHECK(k >= 1 && k * k <= 256 && stride >= 1 && pad >= 0 && 2 * pad <= k, "maxpool: bad window");
  ndp::PoolGeom g;
  g.H = (int)x.size(2); g.W = (int)x.size(3); g.OH = (int)y.size(2); g.OW = (int)y.size(3);
  g.KH = g.KW = (int)k; g.stride = (int)stride; g.pad = (int)pad;
  TORCH_CHECK(g.OH == (g.H + 2 * g.pad - g.KH) / g.stride + 1 && g.OW == (g.W + 2 * g.pad - g.KW) / g.stride + 1,
              "maxpool: output size mismatch");
  TORCH_CHECK(x.numel() < ((int64_t)1 << 31) - 256, "maxpool: tensor too large (32-bit indexing)");
  return g;
}

void maxpool_fwd(torch::Tensor x, torch::Tensor y, torch::Tensor idx, int64_t k, int64_t stride, int64_t pad) {
  check_f32(x, "x"); check_f32(y, "y"); check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == torch::kUInt8 && idx.sizes() == y.sizes() && idx.is_contiguous(),
              "maxpool: idx must be contiguous uint8 shaped like y");
  const ndp::PoolGeom g = pool_geom(x, y, k, stride, pad);
  ndp::launch_maxpool_fwd(x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(),
                          (int)(x.size(0) * x.size(1)), g, cur_stream());
  check_launch("launch_maxpool_fwd");
}

void maxpool_bwd(torch::Tensor dy, torch::Tensor idx, torch::Tensor dx, int64_t k, int64_t stride, int64_t pad) {
  check_f32(dy, "dy"); check_f32(dx, "dx"); check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == torch::kUInt8 && idx.sizes() == dy.sizes() && idx.is_contiguous(),
              "maxpool: idx must be contiguous uint8 shaped like dy");
  const ndp::PoolGeom g = pool_geom(dx, dy, k, stride, pad);
  ndp::launch_maxpool_bwd(dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(),
                          (int)(dx.size(0) * dx.size(1)), g, cur_stream());
  check_launch("launch_maxpool_bwd");
}

// MaxPool(3, 2, 1) backward of the fused stem tail + its BN's backward statistics ([C][N][2])
// dx = None: statistics only (the routed gradient is re-formed by stem_pool_bwd_apply)
void maxpool_bwd_bnstats(torch::Tensor dy, torch::Tensor idx, c10::optional<torch::Tensor> dx_opt, torch::Tensor x,
                         c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, torch::Tensor mean,
                         torch::Tensor invstd, torch::Tensor stats) {
  check_f32(dy, "dy"); check_f32(x, "x"); check_dev(idx, "idx");
  check_f32(mean, "mean"); check_f32(invstd, "invstd"); check_dev(stats, "stats");
  TORCH_CHECK(idx.scalar_type() == torch::kUInt8 && idx.sizes() == dy.sizes() && idx.is_contiguous(),
              "maxpool: idx must be contiguous uint8 shaped like dy");
  if (dx_opt.has_value()) {
    check_f32(*dx_opt, "dx");
    TORCH_CHECK(x.sizes() == dx_opt->sizes(), "maxpool_bwd_bnstats: x shaped like dx");
  }
  TORCH_CHECK(x.is_contiguous() && x.dim() == 4, "maxpool_bwd_bnstats: contiguous 4-d x");
  const torch::Tensor& dx = x;  // geometry only
  const ndp::PoolGeom g = pool_geom(dx, dy, 3, 2, 1);
  TORCH_CHECK(ndp::maxpool_bwd_bnstats_ok(g), "maxpool_bwd_bnstats: needs the 16x16 -> 8x8 stem window");
  const int N = (int)dx.size(0), C = (int)dx.size(1);
  TORCH_CHECK(stats.scalar_type() == torch::kFloat64 && stats.is_contiguous() && stats.numel() >= (int64_t)C * N * 2,
              "maxpool_bwd_bnstats: stats must hold C * N * 2 doubles");
  TORCH_CHECK(mean.numel() >= C && invstd.numel() >= C, "maxpool_bwd_bnstats: statistics size");
  const ndp::PoolBnStats bs{x.data_ptr<float>(), opt_f32(gamma, "gamma"), opt_f32(beta, "beta"),
                            mean.data_ptr<float>(), invstd.data_ptr<float>(), stats.data_ptr<double>(), C, N};
  ndp::launch_maxpool_bwd(dy.data_ptr<float>(), idx.data_ptr<uint8_t>(),
                          dx_opt.has_value() ? dx_opt->data_ptr<float>() : nullptr, N * C, g, cur_stream(), bs);
  check_launch("launch_maxpool_bwd");
}

// the stem BN's input gradient from the pooled gradient and the statistics-only pool backward
void stem_pool_bwd_apply(torch::Tensor dy, torch::Tensor idx, torch::Tensor x, c10::optional<torch::Tensor> gamma,
                         c10::optional<torch::Tensor> beta, torch::Tensor mean, torch::Tensor invstd,
                         torch::Tensor stats, torch::Tensor dx, c10::optional<torch::Tensor> dgamma,
                         c10::optional<torch::Tensor> dbeta) {
  check_f32(dy, "dy"); check_f32(x, "x"); check_f32(dx, "dx"); check_dev(idx, "idx");
  check_f32(mean, "mean"); check_f32(invstd, "invstd"); check_dev(stats, "stats");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && dx.sizes() == x.sizes() && dx.is_contiguous(),
              "stem_pool_bwd_apply: contiguous x / dx of one shape");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK(H == 16 && W == 16 && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == C && dy.size(2) == 8 &&
                  dy.size(3) == 8 && dy.is_contiguous(),
              "stem_pool_bwd_apply: 16x16 -> 8x8 stem maps");
  TORCH_CHECK(idx.scalar_type() == torch::kUInt8 && idx.sizes() == dy.sizes() && idx.is_contiguous(),
              "stem_pool_bwd_apply: idx must be contiguous uint8 shaped like dy");
  TORCH_CHECK(stats.scalar_type() == torch::kFloat64 && stats.numel() >= (int64_t)C * N * 2 && mean.numel() >= C &&
                  invstd.numel() >= C,
              "stem_pool_bwd_apply: statistics sizes");
  ndp::launch_stem_pool_bwd_apply(dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), x.data_ptr<float>(),
                                  opt_f32(gamma, "gamma"), opt_f32(beta, "beta"), mean.data_ptr<float>(),
                                  invstd.data_ptr<float>(), stats.data_ptr<double>(), dx.data_ptr<float>(),
                                  dgamma.has_value() ? dgamma->data_ptr<float>() : nullptr,
                                  dbeta.has_value() ? dbeta->data_ptr<float>() : nullptr, N, C, H, W, cur_stream());
  check_launch("launch_stem_pool_bwd_apply");
}

int bn_slices(int N, int C, int HW) { return ndp::bn_slices(N, C, HW); }
int64_t bn_part_numel(int N, int C, int HW) { return ndp::bn_part_numel(N, C, HW); }

void delay_ns(int64_t ns) {
  ndp::launch_delay_ns(ns, cur_stream());
  check_launch("launch_delay_ns");
}

// flags: int32 device tensor; indices are element offsets
void flag_signal(torch::Tensor flags, int64_t i) {
  check_dev(flags, "flags");
  TORCH_CHECK(flags.scalar_type() == torch::kInt32 && i >= 0 && i < flags.numel(), "flag_signal: bad flag");
  ndp::launch_flag_signal(reinterpret_cast<unsigned*>(flags.data_ptr<int32_t>()) + i, cur_stream());
  check_launch("launch_flag_signal");
}

// host_err (optional): a pinned host int32 the wait mirrors a set error word into, so the
// host sees a timed-out wait at its next replay without a device synchronisation
void flag_wait(torch::Tensor flags, int64_t i, int64_t seen, int64_t err, int64_t timeout_us,
               c10::optional<torch::Tensor> host_err) {
  check_dev(flags, "flags");
  TORCH_CHECK(flags.scalar_type() == torch::kInt32 && i >= 0 && i < flags.numel() && seen >= 0 &&
                  seen < flags.numel() && err >= 0 && err < flags.numel(),
              "flag_wait: bad flag indices");
  auto* f = reinterpret_cast<unsigned*>(flags.data_ptr<int32_t>());
  unsigned* h = nullptr;
  if (host_err.has_value() && host_err->defined()) {
    TORCH_CHECK(!host_err->is_cuda() && host_err->is_pinned() && host_err->scalar_type() == torch::kInt32,
                "flag_wait: host_err must be a pinned int32 host tensor");
    void* dp = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&dp, host_err->data_ptr(), 0) == hipSuccess,
                "flag_wait: host_err is not device-mapped pinned memory");
    h = static_cast<unsigned*>(dp);
  }
  ndp::launch_flag_wait(f + i, f + seen, f + err, timeout_us, cur_stream(), h);
  check_launch("launch_flag_wait");
}

void checksum(torch::Tensor x, torch::Tensor out) {
  check_f32(x, "x");
  check_dev(out, "out");
  TORCH_CHECK(out.scalar_type() == torch::kFloat64 && out.numel() >= 257,
              "checksum out must be float64[>=257]");
  ndp::launch_checksum(x.data_ptr<float>(), x.numel(), out.data_ptr<double>(), cur_stream());
  check_launch("launch_checksum");
}

// conv geometry from (C, H, W, Co, KH, KW, stride, pad); OH/OW derived
ndp::ConvGeom conv_geom(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 8, "conv geometry needs (C, H, W, Co, KH, KW, stride, pad)");
  ndp::ConvGeom g{};
  g.C = (int32_t)v[0]; g.H = (int32_t)v[1]; g.W = (int32_t)v[2];
  g.Co = (int32_t)v[3]; g.KH = (int32_t)v[4]; g.KW = (int32_t)v[5];
  g.stride = (int32_t)v[6]; g.pad = (int32_t)v[7];
  TORCH_CHECK(g.C > 0 && g.H > 0 && g.W > 0 && g.Co > 0 && g.KH > 0 && g.KW > 0 && g.stride > 0 && g.pad >= 0,
              "bad conv geometry");
  g.OH = (g.H + 2 * g.pad - g.KH) / g.stride + 1;
  g.OW = (g.W + 2 * g.pad - g.KW) / g.stride + 1;
  TORCH_CHECK(g.OH > 0 && g.OW > 0, "conv output is empty");
  return g;
}

void toeplitz_expand(torch::Tensor w, torch::Tensor wb, const std::vector<int64_t>& geom) {
  check_f32(w, "w"); check_f32(wb, "w_big");
  const ndp::ConvGeom g = conv_geom(geom);
  TORCH_CHECK(w.numel() == (int64_t)g.Co * g.C * g.KH * g.KW, "toeplitz_expand: weight size");
  TORCH_CHECK(wb.numel() == (int64_t)g.C * g.H * g.W * g.Co * g.OH * g.OW, "toeplitz_expand: w_big size");
  ndp::launch_toeplitz_expand(w.data_ptr<float>(), wb.data_ptr<float>(), g, cur_stream());
  check_launch("launch_toeplitz_expand");
}

// entries: [(w, w_big, geom)] -> every W_big^T in one launch
void toeplitz_expand_many(const std::vector<std::tuple<torch::Tensor, torch::Tensor, std::vector<int64_t>>>& entries) {
  TORCH_CHECK(!entries.empty() && (int)entries.size() <= ndp::kMaxExpand, "toeplitz_expand_many: 1..",
              ndp::kMaxExpand, " layers");
  ndp::ExpandBatch b{};
  int64_t acc = 0;
  for (const auto& en : entries) {
    const torch::Tensor& w = std::get<0>(en);
    const torch::Tensor& wb = std::get<1>(en);
    check_f32(w, "w"); check_f32(wb, "w_big");
    const ndp::ConvGeom g = conv_geom(std::get<2>(en));
    TORCH_CHECK(w.numel() == (int64_t)g.Co * g.C * g.KH * g.KW, "toeplitz_expand_many: weight size");
    const int64_t nk = (int64_t)g.C * g.H * g.W * g.Co * g.OH * g.OW;
    TORCH_CHECK(wb.numel() == nk, "toeplitz_expand_many: w_big size");
    b.w[b.n] = w.data_ptr<float>();
    b.wt[b.n] = wb.data_ptr<float>();
    b.g[b.n] = g;
    TORCH_CHECK((reinterpret_cast<uintptr_t>(b.wt[b.n]) & 15) == 0, "toeplitz_expand_many: w_big not 16-B aligned");
    acc += (int64_t)g.Co * g.OH * g.OW;
    b.end[b.n] = acc;
    ++b.n;
  }
  ndp::launch_toeplitz_expand_many(b, cur_stream());
  check_launch("launch_toeplitz_expand_many");
}

using FoldEntries = std::vector<std::tuple<torch::Tensor, torch::Tensor, std::vector<int64_t>>>;
using SlabEntries = std::vector<std::tuple<torch::Tensor, torch::Tensor, int64_t>>;

ndp::FoldBatch fold_batch(const FoldEntries& entries) {
  TORCH_CHECK((int)entries.size() <= ndp::kMaxExpand, "toeplitz_fold_many: at most ", ndp::kMaxExpand, " layers");
  ndp::FoldBatch b{};
  int64_t acc = 0;
  for (const auto& en : entries) {
    const torch::Tensor& dwb = std::get<0>(en);
    const torch::Tensor& dw = std::get<1>(en);
    check_f32(dwb, "dw_big"); check_f32(dw, "dw");
    const ndp::ConvGeom g = conv_geom(std::get<2>(en));
    const int64_t nw = (int64_t)g.Co * g.C * g.KH * g.KW;
    TORCH_CHECK(dw.numel() == nw, "toeplitz_fold_many: weight size");
    TORCH_CHECK(dwb.numel() == (int64_t)g.C * g.H * g.W * g.Co * g.OH * g.OW, "toeplitz_fold_many: dw_big size");
    b.dwt[b.n] = dwb.data_ptr<float>();
    b.dw[b.n] = dw.data_ptr<float>();
    TORCH_CHECK(g.KH * g.KW <= 9 && g.H * g.W <= 64, "toeplitz_fold_many: kernel / map too large");
    b.g[b.n] = g;
    acc += (int64_t)g.Co * g.C;
    b.end[b.n] = acc;
    ++b.n;
  }
  return b;
}

ndp::SlabBatch slab_batch(const SlabEntries& entries) {
  TORCH_CHECK((int)entries.size() <= ndp::kMaxExpand, "slab_sum_many: at most ", ndp::kMaxExpand, " entries");
  ndp::SlabBatch b{};
  int64_t blocks = 0;
  for (const auto& en : entries) {
    const torch::Tensor& part = std::get<0>(en);
    const torch::Tensor& dw = std::get<1>(en);
    const int64_t slices = std::get<2>(en);
    check_f32(part, "part"); check_f32(dw, "dw");
    const int64_t n = dw.numel();
    TORCH_CHECK(n % 4 == 0 && slices >= 1 && part.numel() >= slices * n, "slab_sum_many: bad entry");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(part.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(dw.data_ptr()) & 15) == 0,
                "slab_sum_many: 16-B aligned tensors");
    b.part[b.n] = part.data_ptr<float>();
    b.dw[b.n] = dw.data_ptr<float>();
    b.numel[b.n] = n;
    b.slices[b.n] = (int)slices;
    blocks += (n / 4 + 15) / 16;
    b.end[b.n] = blocks;
    ++b.n;
  }
  return b;
}

// entries: [(dw_big, dw, geom)] -> every fold in one launch
void toeplitz_fold_many(const FoldEntries& entries) {
  TORCH_CHECK(!entries.empty(), "toeplitz_fold_many: no entries");
  ndp::launch_toeplitz_fold_many(fold_batch(entries), cur_stream());
  check_launch("launch_toeplitz_fold_many");
}

// entries: [(part, dw, slices)] -> dw = sum_s part[s * numel(dw) :], every entry in one launch
void slab_sum_many(const SlabEntries& entries) {
  TORCH_CHECK(!entries.empty(), "slab_sum_many: no entries");
  ndp::launch_slab_sum_many(slab_batch(entries), cur_stream());
  check_launch("launch_slab_sum_many");
}

// slab_sum_many(slabs) and toeplitz_fold_many(folds) in one launch (bitwise the same results)
void gradw_finish(const SlabEntries& slabs, const FoldEntries& folds) {
  if (slabs.empty() && folds.empty()) return;
  ndp::launch_gradw_finish(slab_batch(slabs), fold_batch(folds), cur_stream());
  check_launch("launch_gradw_finish");
}

void toeplitz_fold(torch::Tensor dwb, torch::Tensor dw, const std::vector<int64_t>& geom) {
  check_f32(dwb, "dw_big"); check_f32(dw, "dw");
  const ndp::ConvGeom g = conv_geom(geom);
  TORCH_CHECK(dw.numel() == (int64_t)g.Co * g.C * g.KH * g.KW, "toeplitz_fold: weight size");
  TORCH_CHECK(dwb.numel() == (int64_t)g.C * g.H * g.W * g.Co * g.OH * g.OW, "toeplitz_fold: dw_big size");
  TORCH_CHECK(g.KH * g.KW <= 9, "toeplitz_fold: kernel too large");
  ndp::launch_toeplitz_fold(dwb.data_ptr<float>(), dw.data_ptr<float>(), g, cur_stream());
  check_launch("launch_toeplitz_fold");
}

// (class, fwd images per workgroup, grad-W images per slice, grad-x direct) or class -1
// (class, fwd images per workgroup, grad-W images per slice, grad-x direct, fwd split-K,
// grad-x split-K) for batch B, or class -1
py::tuple conv_plan(const std::vector<int64_t>& geom, int64_t B) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::conv_direct_class(g);
  if (cls < 0 || B <= 0 || B % ndp::conv_fwd_imgs(cls)) return py::make_tuple(-1, 0, 0, false, 1, 1);
  return py::make_tuple(cls, ndp::conv_fwd_imgs(cls), ndp::conv_wgrad_imgs(cls, g, (int)B),
                        ndp::conv_dgrad_direct(cls), ndp::conv_ksplit(cls, g, (int)B, false),
                        ndp::conv_ksplit(cls, g, (int)B, true));
}

// batch-tile partials of the BatchNorm statistics the forward epilogue can emit (0 = none)
int64_t conv_stats_slices(const std::vector<int64_t>& geom, int64_t B) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::conv_direct_class(g);
  if (cls < 0 || B <= 0 || B % ndp::conv_fwd_imgs(cls)) return 0;
  return ndp::conv_fwd_stats_slices(cls, g, (int)B);
}

float* conv_part(const c10::optional<torch::Tensor>& part, int ks, int64_t slab, const char* who) {
  if (ks <= 1) return nullptr;
  TORCH_CHECK(part.has_value(), who, ": split-K needs a part scratch tensor");
  check_f32(*part, "part");
  TORCH_CHECK(part->numel() >= ks * slab, who, ": part scratch too small");
  return part->data_ptr<float>();
}

void conv_check(const torch::Tensor& t, const char* n, int64_t b, int64_t c, int64_t h, int64_t w) {
  check_f32(t, n);
  TORCH_CHECK(t.dim() == 4 && t.size(0) == b && t.size(1) == c && t.size(2) == h && t.size(3) == w, n,
              ": shape mismatch with the conv geometry");
}

int conv_batch(const torch::Tensor& t, const ndp::ConvGeom& g, int imgs) {
  const int B = (int)t.size(0);
  TORCH_CHECK(ndp::conv_direct_class(g) >= 0, "conv: no direct kernel for this geometry");
  TORCH_CHECK(imgs > 0 && B % imgs == 0, "conv: batch must be a multiple of ", imgs);
  return B;
}

// Winograd weight transforms of w (forward + grad-x layouts, 32 * Co * C floats): the caller's (built once per pass by
// wino_weights and shared by forward and grad-x), or built here
torch::Tensor wino_u_for(const c10::optional<torch::Tensor>& given, const torch::Tensor& w, const ndp::ConvGeom& g,
                         bool needed) {
  if (!needed) return torch::Tensor();
  if (given.has_value()) {
    check_f32(*given, "wino_u");
    TORCH_CHECK(given->numel() == ndp::wino_u_numel(g.C, g.Co), "wino_u: 32 * Co * C floats (both layouts)");
    return *given;
  }
  torch::Tensor u = torch::empty({ndp::wino_u_numel(g.C, g.Co)}, w.options());
  ndp::launch_wino_weights(w.data_ptr<float>(), u.data_ptr<float>(), g.Co, g.C, cur_stream());
  return u;
}

// the forward Winograd weight transform of a 3x3 weight (csrc/winograd.hip)
void wino_weights(torch::Tensor w, torch::Tensor u) {
  check_f32(w, "w"); check_f32(u, "u");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "wino_weights: 3x3 weight");
  TORCH_CHECK(u.numel() == 32 * w.size(0) * w.size(1), "wino_weights: u holds 32 * Co * C floats");
  TORCH_CHECK(w.size(0) % 16 == 0 && w.size(1) % 16 == 0, "wino_weights: channels in multiples of 16");
  ndp::launch_wino_weights(w.data_ptr<float>(), u.data_ptr<float>(), (int)w.size(0), (int)w.size(1), cur_stream());
  check_launch("launch_wino_weights");
}

// every Winograd layer of a model in one launch: [(w, u), ...]
void wino_weights_many(const std::vector<std::pair<torch::Tensor, torch::Tensor>>& items) {
  TORCH_CHECK((int)items.size() <= ndp::kMaxWino, "wino_weights_many: at most ", ndp::kMaxWino, " layers");
  ndp::WinoBatch b{};
  int acc = 0;
  for (const auto& it : items) {
    const torch::Tensor& w = it.first;
    const torch::Tensor& u = it.second;
    check_f32(w, "w"); check_f32(u, "u");
    TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(0) % 16 == 0 && w.size(1) % 16 == 0,
                "wino_weights_many: 3x3 weights, channels in multiples of 16");
    TORCH_CHECK(u.numel() == 32 * w.size(0) * w.size(1), "wino_weights_many: u holds 32 * Co * C floats");
    b.w[b.n] = w.data_ptr<float>();
    b.u[b.n] = u.data_ptr<float>();
    b.Co[b.n] = (int)w.size(0);
    b.C[b.n] = (int)w.size(1);
    acc += (int)(w.size(0) / 16 * (w.size(1) / 16));
    b.end[b.n] = acc;
    ++b.n;
  }
  ndp::launch_wino_weights_many(b, cur_stream());
  check_launch("launch_wino_weights_many");
}

// defer: split-K slabs are left in `part` for the consumer; returns how many (1 = y final)
int64_t conv_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor y, const std::vector<int64_t>& geom,
                 c10::optional<torch::Tensor> part, bool defer, c10::optional<torch::Tensor> stats,
                 c10::optional<torch::Tensor> wino_u, bool pair) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::conv_direct_class(g);
  const int B = conv_batch(x, g, ndp::conv_fwd_imgs(cls));
  conv_check(x, "x", B, g.C, g.H, g.W);
  conv_check(w, "w", g.Co, g.C, g.KH, g.KW);
  conv_check(y, "y", B, g.Co, g.OH, g.OW);
  const int ks = ndp::conv_ksplit(cls, g, B, false);
  float* pp = conv_part(part, ks, y.numel(), "conv_fwd");
  double* st = nullptr;
  if (stats.has_value()) {  // BatchNorm partial sums from the epilogue: [Co][S][2]
    const int S = ndp::conv_fwd_stats_slices(cls, g, B);
    check_dev(*stats, "stats");
    TORCH_CHECK(S > 0, "conv_fwd: no statistics epilogue for this geometry / batch (conv_stats_slices)");
    TORCH_CHECK(stats->scalar_type() == torch::kFloat64 && stats->is_contiguous() &&
                    stats->numel() >= (int64_t)g.Co * S * 2,
                "conv_fwd: stats must hold Co * S * 2 doubles");
    st = stats->data_ptr<double>();
  }
  torch::Tensor wu = wino_u_for(wino_u, w, g, ndp::conv_wino(cls, g, B, false));
  const int left = ndp::launch_conv_fwd(x.data_ptr<float>(), w.data_ptr<float>(), y.data_ptr<float>(), B, g, pp,
                                        cur_stream(), defer, st, wu.defined() ? wu.data_ptr<float>() : nullptr,
                                        pair && x.is_contiguous());
  check_launch("launch_conv_fwd");
  return left;
}

int64_t conv_dgrad(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, const std::vector<int64_t>& geom,
                   c10::optional<torch::Tensor> part, c10::optional<torch::Tensor> addend, bool defer,
                   c10::optional<torch::Tensor> stats, c10::optional<torch::Tensor> bn_x,
                   c10::optional<torch::Tensor> bn_y, c10::optional<torch::Tensor> bn_mean,
                   c10::optional<torch::Tensor> bn_invstd, c10::optional<torch::Tensor> wino_u) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::conv_direct_class(g);
  TORCH_CHECK(cls >= 0 && ndp::conv_dgrad_direct(cls), "conv_dgrad: no direct grad-x kernel for this geometry");
  const int B = conv_batch(dy, g, ndp::conv_fwd_imgs(cls));
  conv_check(dy, "dy", B, g.Co, g.OH, g.OW);
  conv_check(w, "w", g.Co, g.C, g.KH, g.KW);
  conv_check(dx, "dx", B, g.C, g.H, g.W);
  const int ks = ndp::conv_ksplit(cls, g, B, true);
  // partial slabs are compact [B][C][OH*OW]-pixel tiles of the transposed product (for the
  // stride-2 1x1 class the 4x4 map, before the even-pixel scatter)
  const int64_t slab = (int64_t)B * g.C * ((cls == 4 || cls == 5) ? g.OH * g.OW : g.H * g.W);
  float* pp = conv_part(part, ks, slab, "conv_dgrad");
  const float* ap = nullptr;
  if (addend.has_value()) {
    conv_check(*addend, "addend", B, g.C, g.H, g.W);
    TORCH_CHECK((reinterpret_cast<uintptr_t>(addend->data_ptr()) & 15) == 0, "conv_dgrad: 16-B aligned addend");
    ap = addend->data_ptr<float>();
  }
  ndp::ConvBnStats bst{nullptr, nullptr, nullptr, nullptr, nullptr};
  if (stats.has_value()) {  // backward-mode BN partial sums of dx: [C][S][2]
    const int S = ndp::conv_dgrad_stats_slices(cls, g, B);
    TORCH_CHECK(S > 0, "conv_dgrad: no statistics epilogue for this geometry / batch (conv_dgrad_stats_slices)");
    check_dev(*stats, "stats");
    TORCH_CHECK(stats->scalar_type() == torch::kFloat64 && stats->is_contiguous() &&
                    stats->numel() >= (int64_t)g.C * S * 2, "conv_dgrad: stats must hold C * S * 2 doubles");
    TORCH_CHECK(bn_x.has_value() && bn_y.has_value() && bn_mean.has_value() && bn_invstd.has_value(),
                "conv_dgrad: stats need the BN's x, y, mean, invstd");
    conv_check(*bn_x, "bn_x", B, g.C, g.H, g.W);
    conv_check(*bn_y, "bn_y", B, g.C, g.H, g.W);
    check_f32(*bn_mean, "bn_mean"); check_f32(*bn_invstd, "bn_invstd");
    TORCH_CHECK(bn_mean->numel() >= g.C && bn_invstd->numel() >= g.C, "conv_dgrad: BN statistics size");
    bst = ndp::ConvBnStats{stats->data_ptr<double>(), bn_x->data_ptr<float>(), bn_y->data_ptr<float>(),
                           bn_mean->data_ptr<float>(), bn_invstd->data_ptr<float>()};
  }
  torch::Tensor wu = wino_u_for(wino_u, w, g, ndp::conv_wino(cls, g, B, true));
  const int left = ndp::launch_conv_dgrad(dy.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(), B, g, pp,
                                          cur_stream(), ap, defer && cls != 4 && cls != 5, bst.out ? &bst : nullptr,
                                          wu.defined() ? wu.data_ptr<float>() : nullptr);
  check_launch("launch_conv_dgrad");
  return left;
}

// dw None: write the per-slice partial slabs only (the caller sums them, batched)
void conv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor part, c10::optional<torch::Tensor> dw_opt,
                const std::vector<int64_t>& geom, bool pair) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::conv_direct_class(g);
  TORCH_CHECK(cls >= 0, "conv_wgrad: no direct kernel for this geometry");
  const int imgs = ndp::conv_wgrad_imgs(cls, g, (int)x.size(0));
  const int B = conv_batch(x, g, imgs);
  conv_check(x, "x", B, g.C, g.H, g.W);
  conv_check(dy, "dy", B, g.Co, g.OH, g.OW);
  float* dwp = nullptr;
  if (dw_opt.has_value()) {
    conv_check(*dw_opt, "dw", g.Co, g.C, g.KH, g.KW);
    dwp = dw_opt->data_ptr<float>();
  }
  check_f32(part, "part");
  TORCH_CHECK(part.numel() >= (int64_t)(B / imgs) * g.Co * g.C * g.KH * g.KW, "conv_wgrad: partial scratch too small");
  ndp::launch_conv_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), part.data_ptr<float>(), dwp, B, g, cur_stream(),
                         pair && dy.is_contiguous() && x.is_contiguous());
  check_launch("launch_conv_wgrad");
}

// ---- strided / tabled implicit-GEMM convolutions (tgemm.hip) -----------------------------
// (class, fwd slabs, grad-x slabs, grad-W slabs) for batch B, or class -1 (no tgemm path)
py::tuple tg_plan(const std::vector<int64_t>& geom, int64_t B) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int cls = ndp::tg_class(g);
  const int64_t ny = B * g.Co * g.OH * g.OW, nx = B * g.C * g.H * g.W;
  const int64_t nw = (int64_t)g.Co * g.C;
  // split-K slab sums run on float4: every output must hold a multiple of 4 floats
  if (cls < 0 || B <= 0 || ny % 4 || nx % 4 || nw % 4) return py::make_tuple(-1, 1, 1, 1);
  // tgemm addresses its operands with 32-bit byte offsets of raw buffer descriptors
  if (std::max(std::max(ny, nx), (int64_t)g.Co * g.C * g.KH * g.KW) * 4 >= (1LL << 31)) return py::make_tuple(-1, 1, 1, 1);
  return py::make_tuple(cls, ndp::tg_splits(g, (int)B, 0), ndp::tg_splits(g, (int)B, 1), ndp::tg_splits(g, (int)B, 2));
}

// the GEMM description tgemm launches for (geom, B, dir) — host-side, for the CPU emulation
// test of the index algebra (tests/test_tgemm_cpu.py)
py::dict tg_describe(const std::vector<int64_t>& geom, int64_t B, int64_t dir) {
  const ndp::ConvGeom g = conv_geom(geom);
  TORCH_CHECK(ndp::tg_class(g) >= 0, "tg_describe: no tgemm path");
  bool akf = false, bnf = false;
  const ndp::TgArgs a = ndp::tg_args(g, (int)B, (int)dir, &akf, &bnf);
  auto idx = [](const ndp::TgIndex& t) { return py::make_tuple(t.so, t.si, t.sh); };
  py::dict d;
  d["am"] = idx(a.am); d["ak"] = idx(a.ak); d["bk"] = idx(a.bk); d["bn"] = idx(a.bn);
  d["cm"] = idx(a.cm); d["cn"] = idx(a.cn);
  d["M"] = a.M; d["N"] = a.N; d["K"] = a.K; d["slab"] = a.slab;
  d["akf"] = akf; d["bnf"] = bnf;
  d["splits"] = ndp::tg_splits(g, (int)B, (int)dir);
  return d;
}

static int tg_batch(const torch::Tensor& t, const ndp::ConvGeom& g, const char* who) {
  TORCH_CHECK(ndp::tg_class(g) >= 0, who, ": no tgemm path for this geometry");
  const int64_t B = t.size(0);
  TORCH_CHECK(std::max(B * g.C * g.H * g.W, B * g.Co * g.OH * g.OW) * 4 < (1LL << 31), who,
              ": operands >= 2 GB (tgemm uses 32-bit buffer offsets)");
  return (int)B;
}

static float* tg_part(const c10::optional<torch::Tensor>& part, int splits, int64_t slab, const char* who) {
  if (splits <= 1) return nullptr;
  TORCH_CHECK(part.has_value(), who, ": split-K needs a part scratch tensor");
  check_f32(*part, "part");
  TORCH_CHECK(part->numel() >= splits * slab && slab % 4 == 0, who, ": part scratch too small / slab % 4");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(part->data_ptr()) & 15) == 0, who, ": 16-B aligned part");
  return part->data_ptr<float>();
}

int64_t tg_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor y, const std::vector<int64_t>& geom,
               c10::optional<torch::Tensor> part, bool defer) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int B = tg_batch(x, g, "tg_fwd");
  conv_check(x, "x", B, g.C, g.H, g.W);
  conv_check(w, "w", g.Co, g.C, g.KH, g.KW);
  conv_check(y, "y", B, g.Co, g.OH, g.OW);
  float* pp = tg_part(part, ndp::tg_splits(g, B, 0), y.numel(), "tg_fwd");
  const int left = ndp::launch_tg_fwd(x.data_ptr<float>(), w.data_ptr<float>(), y.data_ptr<float>(), B, g, pp,
                                      cur_stream(), defer);
  check_launch("launch_tg_fwd");
  return left;
}

int64_t tg_dgrad(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, const std::vector<int64_t>& geom,
                 c10::optional<torch::Tensor> part, c10::optional<torch::Tensor> addend, bool defer) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int B = tg_batch(dy, g, "tg_dgrad");
  conv_check(dy, "dy", B, g.Co, g.OH, g.OW);
  conv_check(w, "w", g.Co, g.C, g.KH, g.KW);
  conv_check(dx, "dx", B, g.C, g.H, g.W);
  float* pp = tg_part(part, ndp::tg_splits(g, B, 1), dx.numel(), "tg_dgrad");
  const float* ap = nullptr;
  if (addend.has_value()) {
    conv_check(*addend, "addend", B, g.C, g.H, g.W);
    TORCH_CHECK((reinterpret_cast<uintptr_t>(addend->data_ptr()) & 15) == 0, "tg_dgrad: 16-B aligned addend");
    ap = addend->data_ptr<float>();
  }
  const int left = ndp::launch_tg_dgrad(dy.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(), B, g, pp,
                                        cur_stream(), ap, defer);
  check_launch("launch_tg_dgrad");
  return left;
}

// out: dW [Co, C, 1, 1]; returns the number of slabs left in part (defer) or 1
int64_t tg_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor out, const std::vector<int64_t>& geom,
                 c10::optional<torch::Tensor> part, bool defer) {
  const ndp::ConvGeom g = conv_geom(geom);
  const int B = tg_batch(x, g, "tg_wgrad");
  conv_check(x, "x", B, g.C, g.H, g.W);
  conv_check(dy, "dy", B, g.Co, g.OH, g.OW);
  check_f32(out, "out");
  const int64_t n = (int64_t)g.Co * g.C;
  TORCH_CHECK(out.numel() == n, "tg_wgrad: out must hold ", n, " floats");
  float* pp = tg_part(part, ndp::tg_splits(g, B, 2), n, "tg_wgrad");
  const int left = ndp::launch_tg_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), out.data_ptr<float>(), B, g, pp,
                                        cur_stream(), defer);
  check_launch("launch_tg_wgrad");
  return left;
}

// db = g.sum(0) for g [M, N] contiguous fp32, N % 4 == 0 (deterministic, graph-safe)
// part (optional, >= colsum_chunks(M, N) * N floats): write the per-chunk partials there and
// leave the final fixed-order sum to the caller (ops/gradfinish.py batches it); returns the
// chunk count (0: summed into out here)
static float* deferred_part(const c10::optional<torch::Tensor>& part, int64_t need, const char* what) {
  if (!part.has_value()) return nullptr;
  check_f32(*part, what);
  TORCH_CHECK(part->is_contiguous() && part->numel() >= need, what, ": partial buffer too small");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(part->data_ptr()) & 15) == 0, what, ": 16-B aligned partials");
  return part->data_ptr<float>();
}

int64_t colsum(torch::Tensor g, torch::Tensor out, c10::optional<torch::Tensor> part_out) {
  check_f32(g, "g"); check_f32(out, "out");
  TORCH_CHECK(g.dim() == 2 && g.size(1) % 4 == 0 && out.numel() == g.size(1), "colsum: g [M, N] with N % 4 == 0");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0, "colsum: 16-B aligned input");
  const int64_t M = g.size(0);
  const int N = (int)g.size(1);
  const int chunks = ndp::colsum_chunks(M, N);
  float* dp = deferred_part(part_out, (int64_t)chunks * N, "colsum");
  torch::Tensor part;
  if (dp == nullptr) part = torch::empty({(int64_t)chunks * N}, g.options());
  ndp::launch_colsum(g.data_ptr<float>(), M, N, dp ? dp : part.data_ptr<float>(), dp ? nullptr : out.data_ptr<float>(),
                     cur_stream());
  check_launch("launch_colsum");
  return dp ? chunks : 0;
}

// DistilBERT FFN: dh = g * gelu'(h) and db = column sums of dh in one pass
int64_t gelu_bwd_colsum(torch::Tensor g, torch::Tensor h, torch::Tensor dh, torch::Tensor db,
                        c10::optional<torch::Tensor> part_out) {
  check_f32(g, "g"); check_f32(h, "h"); check_f32(dh, "dh"); check_f32(db, "db");
  TORCH_CHECK(g.dim() == 2 && g.size(1) % 4 == 0 && h.sizes() == g.sizes() && dh.sizes() == g.sizes() &&
                  db.numel() == g.size(1),
              "gelu_bwd_colsum: g / h / dh [M, N] with N % 4 == 0, db [N]");
  for (auto* t : {&g, &h, &dh})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gelu_bwd_colsum: 16-B aligned tensors");
  const int64_t M = g.size(0);
  const int N = (int)g.size(1);
  const int chunks = ndp::colsum_chunks(M, N);
  float* dp = deferred_part(part_out, (int64_t)chunks * N, "gelu_bwd_colsum");
  torch::Tensor part;
  if (dp == nullptr) part = torch::empty({(int64_t)chunks * N}, g.options());
  ndp::launch_gelu_bwd_colsum(g.data_ptr<float>(), h.data_ptr<float>(), dh.data_ptr<float>(), M, N,
                              dp ? dp : part.data_ptr<float>(), dp ? nullptr : db.data_ptr<float>(), cur_stream());
  check_launch("launch_gelu_bwd_colsum");
  return dp ? chunks : 0;
}

// fused cross-entropy forward: loss (0-d), dl [B, K] saved gradient; scratch = rowloss [B] + inv [1]
void ce_fwd(torch::Tensor x, torch::Tensor tgt, torch::Tensor dl, torch::Tensor scratch, torch::Tensor loss,
            torch::Tensor ctr, int64_t ignore_index, c10::optional<torch::Tensor> acc) {
  check_f32(x, "logits"); check_f32(dl, "dl"); check_f32(scratch, "scratch"); check_f32(loss, "loss");
  float* ap = nullptr;
  if (acc.has_value()) {  // running loss sum: acc += loss inside the kernel
    check_f32(*acc, "acc");
    TORCH_CHECK(acc->numel() == 1, "ce_fwd: acc must be a one-element fp32 tensor");
    ap = acc->data_ptr<float>();
  }
  check_dev(tgt, "target"); check_dev(ctr, "ctr");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && dl.sizes() == x.sizes() && dl.is_contiguous(),
              "ce_fwd: logits / dl must be contiguous [B, K]");
  TORCH_CHECK(tgt.scalar_type() == torch::kInt64 && tgt.is_contiguous() && tgt.numel() == x.size(0),
              "ce_fwd: target must be contiguous int64 [B]");
  TORCH_CHECK(scratch.numel() >= x.size(0) + 1 && loss.numel() == 1, "ce_fwd: scratch / loss size");
  TORCH_CHECK(ctr.scalar_type() == torch::kInt32 && ctr.numel() >= 1, "ce_fwd: int32 counter");
  TORCH_CHECK(x.size(0) >= 1 && x.size(0) < (1LL << 31) && x.size(1) >= 1, "ce_fwd: empty batch");
  const int B = (int)x.size(0);
  float* sp = scratch.data_ptr<float>();
  ndp::launch_ce_fwd(x.data_ptr<float>(), tgt.data_ptr<int64_t>(), B, (int)x.size(1), ignore_index,
                     dl.data_ptr<float>(), sp, loss.data_ptr<float>(), sp + B,
                     reinterpret_cast<unsigned*>(ctr.data_ptr<int32_t>()), cur_stream(), ap);
  check_launch("launch_ce_fwd");
}

void ce_bwd(torch::Tensor dl, torch::Tensor g, torch::Tensor scratch, torch::Tensor dx) {
  check_f32(dl, "dl"); check_f32(g, "grad"); check_f32(scratch, "scratch"); check_f32(dx, "dx");
  TORCH_CHECK(dl.is_contiguous() && dx.is_contiguous() && dx.sizes() == dl.sizes() && dl.dim() == 2, "ce_bwd: shapes");
  TORCH_CHECK(g.numel() == 1 && scratch.numel() >= dl.size(0) + 1, "ce_bwd: scalar grad / scratch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(dl.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(dx.data_ptr()) & 15) == 0,
              "ce_bwd: 16-B aligned tensors");
  ndp::launch_ce_bwd(dl.data_ptr<float>(), g.data_ptr<float>(), scratch.data_ptr<float>() + dl.size(0),
                     dx.data_ptr<float>(), dl.numel(), cur_stream());
  check_launch("launch_ce_bwd");
}

// fused residual add + LayerNorm (last dim D): y, s (= a + b), mean, rstd are outputs
// LayerNorm hash dropout: mode 0 none / 1 on the input a / 2 on the output (layernorm.hip)
static ndp::LnDrop ln_drop(int64_t mode, double p, const c10::optional<torch::Tensor>& seed,
                           const c10::optional<torch::Tensor>& da, int64_t numel) {
  ndp::LnDrop d{nullptr, 0u, 1.f, 0, nullptr};
  if (mode == 0 || p <= 0.0) return d;
  TORCH_CHECK(mode == 1 || mode == 2, "ln: dropout mode 0 / 1 / 2");
  TORCH_CHECK(p < 1.0, "ln: dropout p < 1");
  TORCH_CHECK(seed.has_value() && seed->is_cuda() && seed->scalar_type() == torch::kInt32 && seed->numel() >= 1,
              "ln: dropout needs a device int32 seed");
  d.seed = seed->data_ptr<int32_t>();
  const double t = p * 4294967296.0;
  d.thr = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  d.scale = (float)(1.0 / (1.0 - p));
  d.mode = (int)mode;
  if (da.has_value()) {
    check_f32(*da, "da");
    TORCH_CHECK(da->is_contiguous() && da->numel() == numel, "ln: da [R, D]");
    d.da = da->data_ptr<float>();
  }
  return d;
}

void ln_fwd(torch::Tensor a, c10::optional<torch::Tensor> b, torch::Tensor gamma, torch::Tensor beta, torch::Tensor y,
            torch::Tensor s, torch::Tensor mean, torch::Tensor rstd, double eps, int64_t drop_mode, double p,
            c10::optional<torch::Tensor> seed) {
  check_f32(a, "a"); check_f32(gamma, "gamma"); check_f32(beta, "beta"); check_f32(y, "y"); check_f32(s, "s");
  check_f32(mean, "mean"); check_f32(rstd, "rstd");
  const int D = (int)a.size(-1);
  TORCH_CHECK(ndp::ln_supported(D) && gamma.numel() == D && beta.numel() == D, "ln_fwd: unsupported D");
  const int64_t R = a.numel() / D;
  for (auto* t : {&a, &y, &s}) TORCH_CHECK(t->is_contiguous() && t->numel() == R * D, "ln_fwd: contiguous [R, D]");
  if (b.has_value()) {
    check_f32(*b, "b");
    TORCH_CHECK(b->is_contiguous() && b->sizes() == a.sizes(), "ln_fwd: residual shape");
  }
  TORCH_CHECK(mean.numel() == R && rstd.numel() == R, "ln_fwd: stats size");
  ndp::launch_ln_fwd(a.data_ptr<float>(), opt_f32(b, "b"), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                     y.data_ptr<float>(), s.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), R, D,
                     (float)eps, cur_stream(), ln_drop(drop_mode, p, seed, c10::nullopt, R * D));
  check_launch("launch_ln_fwd");
}

int64_t ln_bwd(torch::Tensor dy, torch::Tensor s, torch::Tensor mean, torch::Tensor rstd, torch::Tensor gamma,
               torch::Tensor dx, torch::Tensor dgb, int64_t drop_mode, double p, c10::optional<torch::Tensor> seed,
               c10::optional<torch::Tensor> da, c10::optional<torch::Tensor> part_out) {
  check_f32(dy, "dy"); check_f32(s, "s"); check_f32(mean, "mean"); check_f32(rstd, "rstd"); check_f32(gamma, "gamma");
  check_f32(dx, "dx"); check_f32(dgb, "dgb");
  const int D = (int)s.size(-1);
  const int64_t R = s.numel() / D;
  TORCH_CHECK(ndp::ln_supported(D) && gamma.numel() == D && dgb.numel() == 2 * D, "ln_bwd: unsupported D");
  for (auto* t : {&dy, &s, &dx}) TORCH_CHECK(t->is_contiguous() && t->numel() == R * D, "ln_bwd: contiguous [R, D]");
  const ndp::LnDrop dp = ln_drop(drop_mode, p, seed, da, R * D);
  TORCH_CHECK(dp.mode != 1 || dp.da != nullptr, "ln_bwd: input dropout needs da");
  const int wgs = ndp::ln_bwd_wgs(R);
  float* pp = deferred_part(part_out, (int64_t)wgs * 2 * D, "ln_bwd");
  torch::Tensor part;
  if (pp == nullptr) part = torch::empty({(int64_t)wgs * 2 * D}, s.options());
  ndp::launch_ln_bwd(dy.data_ptr<float>(), s.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                     gamma.data_ptr<float>(), dx.data_ptr<float>(), pp ? pp : part.data_ptr<float>(),
                     pp ? nullptr : dgb.data_ptr<float>(), R, D, cur_stream(), dp);
  check_launch("launch_ln_bwd");
  return pp ? wgs : 0;
}

void embedding_backward(torch::Tensor ids, torch::Tensor gout, torch::Tensor gw, int64_t pad, torch::Tensor perm,
                        torch::Tensor row_start, torch::Tensor row_cnt) {
  check_dev(ids, "ids"); check_f32(gout, "grad_out"); check_f32(gw, "grad_weight");
  check_dev(perm, "perm"); check_dev(row_start, "row_start"); check_dev(row_cnt, "row_cnt");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.is_contiguous(), "embedding_backward: ids must be contiguous int64");
  TORCH_CHECK(gw.dim() == 2 && gw.size(1) % 4 == 0, "embedding_backward: grad_weight [V, D] with D % 4 == 0");
  const int64_t T = ids.numel(), V = gw.size(0), D = gw.size(1);
  TORCH_CHECK(gout.numel() == T * D, "embedding_backward: grad_out must be [T, D]");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(gout.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(gw.data_ptr()) & 15) == 0,
              "embedding_backward: 16-B aligned grad tensors");
  for (auto* t : {&perm, &row_start, &row_cnt})
    TORCH_CHECK(t->scalar_type() == torch::kInt32 && t->is_contiguous(), "embedding_backward: int32 scratch");
  TORCH_CHECK(perm.numel() >= T && row_start.numel() >= V && row_cnt.numel() >= V, "embedding_backward: scratch too small");
  TORCH_CHECK(T < (1LL << 29) && V < (1LL << 31), "embedding_backward: too many tokens / rows");
  ndp::launch_embedding_backward(ids.data_ptr<int64_t>(), (int)T, gout.data_ptr<float>(), (int)V, (int)D, (int)pad,
                                 perm.data_ptr<int32_t>(), row_start.data_ptr<int32_t>(), row_cnt.data_ptr<int32_t>(),
                                 gw.data_ptr<float>(), cur_stream());
  check_launch("launch_embedding_backward");
}

// q/k/v/o: [B, S, H, 64] fp32 contiguous (== the [B, S, H*64] projections); mask [B, S] int32 or None
void attn_check(const torch::Tensor& t, const char* n, const torch::Tensor& q) {
  check_f32(t, n);
  TORCH_CHECK(t.sizes() == q.sizes() && t.is_contiguous(), n, ": contiguous [B, S, H, 64] like q");
}

// q / k / v (and dq / dk / dv): [B, S, H, 64] with unit element / 64-float head strides and
// a common token row stride ld (H*64 contiguous, 3*H*64 for views into a packed QKV)
int64_t attn_ld(const torch::Tensor& t, const char* n, const torch::Tensor& q) {
  TORCH_CHECK(t.is_cuda(), n, " must be a device (HIP) tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 && t.sizes() == q.sizes(), n, ": fp32 [B, S, H, 64] like q");
  const int64_t S = t.size(1), H = t.size(2), ld = t.stride(1);
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) == 64 && t.stride(0) == S * ld && ld >= H * 64 && ld % 4 == 0 &&
                  (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0,
              n, ": needs [B, S, H, 64] rows with a 16-B aligned token stride");
  return ld;
}

const int32_t* attn_seed(const c10::optional<torch::Tensor>& seed, double p_drop) {
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "attn: p_drop in [0, 1)");
  if (p_drop == 0.0) return nullptr;
  TORCH_CHECK(seed.has_value(), "attn: dropout needs a device seed tensor");
  check_dev(*seed, "seed");
  TORCH_CHECK(seed->scalar_type() == torch::kInt32 && seed->numel() >= 1, "attn: seed must be int32[1]");
  return seed->data_ptr<int32_t>();
}

void attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, c10::optional<torch::Tensor> mask, torch::Tensor o,
              torch::Tensor lse, double scale, c10::optional<torch::Tensor> seed, double p_drop) {
  TORCH_CHECK(q.dim() == 4 && q.size(3) == 64, "attn: q must be [B, S, H, 64]");
  const int64_t ld = attn_ld(q, "q", q);
  TORCH_CHECK(attn_ld(k, "k", q) == ld && attn_ld(v, "v", q) == ld, "attn: q / k / v need one token stride");
  attn_check(o, "o", q); check_f32(lse, "lse");
  const int B = (int)q.size(0), S = (int)q.size(1), H = (int)q.size(2);
  TORCH_CHECK(lse.numel() >= 2 * (int64_t)B * H * S, "attn: lse must hold 2*B*H*S floats");
  const int32_t* mp = nullptr;
  if (mask.has_value()) {
    check_dev(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == torch::kInt32 && mask->is_contiguous() && mask->numel() == (int64_t)B * S,
                "attn: mask must be int32 [B, S]");
    mp = mask->data_ptr<int32_t>();
  }
  const int32_t* sp = attn_seed(seed, p_drop);
  ndp::launch_attn_fwd(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), mp, o.data_ptr<float>(),
                       lse.data_ptr<float>(), B, S, H, (float)scale, sp, (float)p_drop, cur_stream(), ld);
  check_launch("launch_attn_fwd");
}

void attn_bwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, c10::optional<torch::Tensor> mask, torch::Tensor o,
              torch::Tensor dout, torch::Tensor lse, torch::Tensor delta, torch::Tensor dq, torch::Tensor dk,
              torch::Tensor dv, double scale, c10::optional<torch::Tensor> seed, double p_drop) {
  TORCH_CHECK(q.dim() == 4 && q.size(3) == 64, "attn: q must be [B, S, H, 64]");
  const int64_t ld = attn_ld(q, "q", q);
  for (auto* t : {&k, &v, &dq, &dk, &dv})
    TORCH_CHECK(attn_ld(*t, "q/k/v grads", q) == ld, "attn: q / k / v and their grads need one token stride");
  attn_check(o, "o", q); attn_check(dout, "dout", q);
  check_f32(lse, "lse"); check_f32(delta, "delta");
  const int B = (int)q.size(0), S = (int)q.size(1), H = (int)q.size(2);
  TORCH_CHECK(lse.numel() >= 2 * (int64_t)B * H * S && delta.numel() >= (int64_t)B * H * S,
              "attn: lse/delta too small");
  const int32_t* mp = nullptr;
  if (mask.has_value()) {
    check_dev(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == torch::kInt32 && mask->is_contiguous() && mask->numel() == (int64_t)B * S,
                "attn: mask must be int32 [B, S]");
    mp = mask->data_ptr<int32_t>();
  }
  const int32_t* sp = attn_seed(seed, p_drop);
  ndp::launch_attn_bwd(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), mp, o.data_ptr<float>(),
                       dout.data_ptr<float>(), lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr<float>(),
                       dk.data_ptr<float>(), dv.data_ptr<float>(), B, S, H, (float)scale, sp,
                       (float)p_drop, cur_stream(), ld);
  check_launch("launch_attn_bwd");
}

}  // namespace

void register_comm(py::module& m);  // comm.cpp
// ---- HIP-IPC one-shot all-reduce (ipc.hip; registered here so pybind11 stays g++-only) ----
namespace ndp {
void* ipc_new(int rank, int nranks, int device, int64_t capacity_bytes);
void ipc_delete(void* c);
std::string ipc_handle(void* c);
void ipc_open(void* c, const std::vector<std::string>& h);
void ipc_all_reduce_many(void* c, const std::vector<at::Tensor>& ts, const std::string& op, int64_t stream);
int64_t ipc_error(void* c);
void ipc_check(void* c);
void ipc_destroy(void* c);
std::string ipc_bus_id(void* c);
int64_t ipc_info(void* c, int what);
}  // namespace ndp

struct IpcCommPy {
  void* c;
  IpcCommPy(int rank, int nranks, int device, int64_t cap) : c(ndp::ipc_new(rank, nranks, device, cap)) {}
  ~IpcCommPy() { ndp::ipc_delete(c); }  // buffers are released by destroy() (graphs may still use them)
};

void register_ipc(py::module& m) {
  py::class_<IpcCommPy, std::shared_ptr<IpcCommPy>>(m, "IpcComm")
      .def(py::init<int, int, int, int64_t>(), py::arg("rank"), py::arg("nranks"), py::arg("device"),
           py::arg("capacity_bytes") = 8 << 20)
      .def("handle", [](IpcCommPy& s) { return py::bytes(ndp::ipc_handle(s.c)); })
      .def("open", [](IpcCommPy& s, const std::vector<std::string>& h) { ndp::ipc_open(s.c, h); })
      .def("all_reduce", [](IpcCommPy& s, torch::Tensor t, const std::string& op, int64_t stream) {
            ndp::ipc_all_reduce_many(s.c, {t}, op, stream);
          }, py::arg("t"), py::arg("op") = "sum", py::arg("stream") = 0)
      .def("all_reduce_many", [](IpcCommPy& s, const std::vector<torch::Tensor>& ts, const std::string& op,
                                 int64_t stream) { ndp::ipc_all_reduce_many(s.c, ts, op, stream); },
           py::arg("ts"), py::arg("op") = "sum", py::arg("stream") = 0)
      .def("error", [](IpcCommPy& s) { return ndp::ipc_error(s.c); })
      .def("check", [](IpcCommPy& s) { ndp::ipc_check(s.c); })
      .def("destroy", [](IpcCommPy& s) { ndp::ipc_destroy(s.c); })
      .def("bus_id", [](IpcCommPy& s) { return ndp::ipc_bus_id(s.c); })
      .def_property_readonly("rank", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 0); })
      .def_property_readonly("nranks", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 1); })
      .def_property_readonly("device", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 2); })
      .def_property_readonly("capacity", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 3); })
      .def_property_readonly("alive", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 4) != 0; })
      .def_property_readonly("uncached", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 5) != 0; })
      .def_property_readonly("launches", [](IpcCommPy& s) { return ndp::ipc_info(s.c, 6); });
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "network_distributed_pytorch_amd native gfx950 kernels + plan builder";
  m.attr("SIZEOF_MATGEOM") = (int)sizeof(MatGeom);
  m.attr("SIZEOF_MATPTRS") = (int)sizeof(MatPtrs);
  m.attr("SIZEOF_SEGENTRY") = (int)sizeof(SegEntry);
  m.attr("MAX_RANK") = ndp::kMaxRank;
  m.def("build_plan", &build_plan, "Build the PowerSGD execution plan (host)");
  m.def("patch_geom_vec", &patch_geom_vec);
  m.def("make_mat_ptrs", &make_mat_ptrs);
  m.def("make_seg_table", &make_seg_table);
  m.def("make_orth_geom", &make_orth_geom);
  m.def("psgd_p", &psgd_p, py::arg("geom"), py::arg("ptrs"), py::arg("items"), py::arg("q_warm"), py::arg("p_part"),
        py::arg("fuse_ef"), py::arg("max_rank"), py::arg("p_prev") = OptT(), py::arg("p_out") = OptT(),
        py::arg("p_ctr") = OptT(), py::arg("seg_entries") = OptT(), py::arg("seg_prefix") = OptT(),
        py::arg("seg_n") = 0, py::arg("seg_blocks") = 0, py::arg("p_cols") = (int64_t)ndp::kPKW);
  m.def("psgd_q", &psgd_q, py::arg("geom"), py::arg("ptrs"), py::arg("items"), py::arg("p_hat"), py::arg("q_part"),
        py::arg("max_rank"), py::arg("q_out") = OptT(), py::arg("q_ctr") = OptT(), py::arg("q_fin_max") = 1 << 30);
  m.def("psgd_orth", &psgd_orth, py::arg("geom"), py::arg("items"), py::arg("p"), py::arg("p_div"),
        py::arg("eps"), py::arg("max_rank"), py::arg("scratch"), py::arg("ctr"), py::arg("n_items_total") = -1,
        py::arg("max_spins") = -1);
  m.def("orth_coresident_cap", &ndp::orth_coresident_cap);
  m.def("psgd_update", &psgd_update, py::arg("geom"), py::arg("ptrs"), py::arg("items"), py::arg("p_hat"),
        py::arg("q_sum"), py::arg("q_div"), py::arg("q_warm"), py::arg("mode"), py::arg("lr"), py::arg("momentum"),
        py::arg("max_rank"), py::arg("p_prev") = c10::optional<torch::Tensor>(), py::arg("r1_buf") = OptT(),
        py::arg("r1_div") = 1.0, py::arg("r1_mom") = OptT(), py::arg("r1_x") = OptT(), py::arg("r1_g") = OptT());
  m.def("rank1_step", &rank1_step);
  m.def("seg_reduce", &seg_reduce);
  m.def("sgd_momentum", &sgd_momentum);
  m.def("add", &add);
  m.def("delay_ns", &delay_ns);
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("res"), py::arg("y"), py::arg("gamma"), py::arg("beta"),
        py::arg("rmean"), py::arg("rvar"), py::arg("nbt"), py::arg("save_mean"), py::arg("save_invstd"),
        py::arg("part"), py::arg("eps"), py::arg("momentum"), py::arg("relu"), py::arg("training"),
        py::arg("single"), py::arg("xpart") = py::none(), py::arg("nslab") = 0, py::arg("xstats") = py::none(),
        py::arg("xS") = 0);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("gamma"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("dx"), py::arg("dres"), py::arg("dgamma"), py::arg("dbeta"), py::arg("part"),
        py::arg("relu"), py::arg("single"), py::arg("dypart") = py::none(), py::arg("nslab") = 0,
        py::arg("dyadd") = py::none(), py::arg("mbeta") = py::none(), py::arg("dstats") = py::none(),
        py::arg("dS") = 0);
  m.def("bn_relu_maxpool", &bn_relu_maxpool, py::arg("x"), py::arg("y"), py::arg("idx"), py::arg("gamma"),
        py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("nbt"), py::arg("save_mean"),
        py::arg("save_invstd"), py::arg("part"), py::arg("eps"), py::arg("momentum"), py::arg("xstats") = py::none(),
        py::arg("xS") = 0);
  m.def("bn_two_kernel_path", [](int64_t N, int64_t C, int64_t HW, bool single) {
    return ndp::bn_two_kernel_path((int)N, (int)C, (int)HW, single ? 1 : 0);
  });
  m.def("bn_set_vec4", &ndp::bn_set_vec4);
  m.def("bn_pair_ok", &ndp::bn_pair_ok);
  m.def("bn_pair_fwd", &bn_pair_fwd);
  m.def("bn_pair_bwd", &bn_pair_bwd);
  m.def("wino_set_enabled", &ndp::wino_set_enabled);
  m.def("conv_set_stem_psplit", &ndp::conv_set_stem_psplit);
  m.def("bn_slices", &bn_slices);
  m.def("slab_sum", &slab_sum);
  m.def("bn_part_numel", &bn_part_numel);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("maxpool_bwd_bnstats", &maxpool_bwd_bnstats, py::arg("dy"), py::arg("idx"), py::arg("dx"), py::arg("x"),
        py::arg("gamma"), py::arg("beta"), py::arg("mean"), py::arg("invstd"), py::arg("stats"));
  m.def("stem_pool_bwd_apply", &stem_pool_bwd_apply);
  m.def("checksum", &checksum);
  m.def("flag_signal", &flag_signal);
  m.def("flag_wait", &flag_wait, py::arg("flags"), py::arg("i"), py::arg("seen"), py::arg("err"),
        py::arg("timeout_us"), py::arg("host_err") = c10::optional<torch::Tensor>());
  m.def("toeplitz_expand", &toeplitz_expand);
  m.def("toeplitz_fold", &toeplitz_fold);
  m.def("toeplitz_expand_many", &toeplitz_expand_many);
  m.def("toeplitz_fold_many", &toeplitz_fold_many);
  m.def("slab_sum_many", &slab_sum_many);
  m.def("gradw_finish", &gradw_finish, py::arg("slabs"), py::arg("folds"));
  m.def("conv_plan", &conv_plan, py::arg("geom"), py::arg("batch"));
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("geom"), py::arg("part") = py::none(),
        py::arg("defer") = false, py::arg("stats") = py::none(), py::arg("wino_u") = py::none(),
        py::arg("pair") = false);
  m.def("conv_flush_pending_fwd", []() {
    ndp::conv_flush_pending_fwd();
    check_launch("conv_flush_pending_fwd");
  });
  m.def("wino_weights", &wino_weights);
  m.def("wino_weights_many", &wino_weights_many);
  m.def("conv_wino", [](const std::vector<int64_t>& geom, int64_t B, bool dgrad) {
    const ndp::ConvGeom g = conv_geom(geom);
    const int cls = ndp::conv_direct_class(g);
    return cls >= 0 && B > 0 && B % ndp::conv_fwd_imgs(cls) == 0 && ndp::conv_wino(cls, g, (int)B, dgrad);
  });
  m.def("conv_stats_slices", &conv_stats_slices, py::arg("geom"), py::arg("batch"));
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("geom"),
        py::arg("part") = py::none(), py::arg("addend") = py::none(), py::arg("defer") = false,
        py::arg("stats") = py::none(), py::arg("bn_x") = py::none(), py::arg("bn_y") = py::none(),
        py::arg("bn_mean") = py::none(), py::arg("bn_invstd") = py::none(), py::arg("wino_u") = py::none());
  m.def("conv_dgrad_stats_slices", [](const std::vector<int64_t>& geom, int64_t B) -> int64_t {
    const ndp::ConvGeom g = conv_geom(geom);
    const int cls = ndp::conv_direct_class(g);
    if (cls < 0 || B <= 0 || B % ndp::conv_fwd_imgs(cls)) return 0;
    return ndp::conv_dgrad_stats_slices(cls, g, (int)B);
  }, py::arg("geom"), py::arg("batch"));
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("part"), py::arg("dw"), py::arg("geom"),
        py::arg("pair") = false);
  m.def("conv_flush_pending", []() {
    ndp::conv_flush_pending();
    check_launch("conv_flush_pending");
  });
  m.def("tg_plan", &tg_plan);
  m.def("tg_describe", &tg_describe);
  m.def("tg_fwd", &tg_fwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("geom"), py::arg("part") = py::none(),
        py::arg("defer") = false);
  m.def("tg_dgrad", &tg_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("geom"),
        py::arg("part") = py::none(), py::arg("addend") = py::none(), py::arg("defer") = false);
  m.def("tg_wgrad", &tg_wgrad, py::arg("x"), py::arg("dy"), py::arg("out"), py::arg("geom"),
        py::arg("part") = py::none(), py::arg("defer") = false);
  m.def("embedding_backward", &embedding_backward);
  m.def("colsum", &colsum, py::arg("g"), py::arg("out"), py::arg("part") = c10::optional<torch::Tensor>());
  m.def("gelu_bwd_colsum", &gelu_bwd_colsum, py::arg("g"), py::arg("h"), py::arg("dh"), py::arg("db"),
        py::arg("part") = c10::optional<torch::Tensor>());
  m.def("ce_fwd", &ce_fwd, py::arg("x"), py::arg("tgt"), py::arg("dl"), py::arg("scratch"), py::arg("loss"),
        py::arg("ctr"), py::arg("ignore_index"), py::arg("acc") = py::none());
  m.def("ln_fwd", &ln_fwd, py::arg("a"), py::arg("b"), py::arg("gamma"), py::arg("beta"), py::arg("y"), py::arg("s"),
        py::arg("mean"), py::arg("rstd"), py::arg("eps"), py::arg("drop_mode") = 0, py::arg("p") = 0.0,
        py::arg("seed") = c10::optional<torch::Tensor>());
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("s"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"),
        py::arg("dx"), py::arg("dgb"), py::arg("drop_mode") = 0, py::arg("p") = 0.0,
        py::arg("seed") = c10::optional<torch::Tensor>(), py::arg("da") = c10::optional<torch::Tensor>(),
        py::arg("part") = c10::optional<torch::Tensor>());
  m.def("ln_bwd_wgs", [](int64_t R) { return (int64_t)ndp::ln_bwd_wgs(R); });
  m.def("colsum_chunks", [](int64_t M, int64_t N) { return (int64_t)ndp::colsum_chunks(M, (int)N); });
  m.def("ce_bwd", &ce_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  register_comm(m);
  register_ipc(m);
}
