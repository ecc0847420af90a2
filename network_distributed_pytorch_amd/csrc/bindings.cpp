// pybind11 bindings for the gfx950 kernels and the host plan builder.
//
// Every entry point enqueues on the caller's current HIP stream (so the Python layer can
// place work on a side stream, overlap it with backward and capture it in a hipGraph),
// never synchronises and never allocates.
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

void psgd_p(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor q_warm,
            torch::Tensor p_part, bool fuse_ef, int max_rank) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(q_warm, "q_warm"); check_f32(p_part, "p_part");
  ndp::launch_psgd_p(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                     reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                     reinterpret_cast<const PItem*>(items.data_ptr()),
                     (int)n_of(items, sizeof(PItem)), q_warm.data_ptr<float>(),
                     p_part.data_ptr<float>(), fuse_ef ? 1 : 0, max_rank, cur_stream());
  check_launch("launch_psgd_p");
}

void psgd_q(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor p_hat,
            torch::Tensor q_part, int max_rank) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(p_hat, "p_hat"); check_f32(q_part, "q_part");
  ndp::launch_psgd_q(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                     reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                     reinterpret_cast<const QItem*>(items.data_ptr()),
                     (int)n_of(items, sizeof(QItem)), p_hat.data_ptr<float>(),
                     q_part.data_ptr<float>(), max_rank, cur_stream());
  check_launch("launch_psgd_q");
}

// scratch: float32 tensor of >= 2*n_items*kMaxRank partials; ctr: int32 tensor of
// >= n_mats + 1 words (counters, then the error word at index n_mats)
void psgd_orth(torch::Tensor geom, torch::Tensor items, torch::Tensor p, double p_div, double eps,
               int max_rank, torch::Tensor scratch, torch::Tensor ctr) {
  check_dev(geom, "geom"); check_dev(items, "items"); check_f32(p, "p"); check_f32(scratch, "scratch");
  check_dev(ctr, "ctr");
  const int n_items = (int)n_of(items, sizeof(ndp::OrthItem));
  const int n_mats = (int)n_of(geom, sizeof(MatGeom));
  TORCH_CHECK(scratch.numel() >= 2LL * n_items * ndp::kMaxRank, "orth scratch too small");
  TORCH_CHECK(ctr.numel() * ctr.element_size() >= 4LL * (n_mats + 1), "orth counters too small");
  auto* c = reinterpret_cast<unsigned*>(ctr.data_ptr());
  ndp::launch_psgd_orth(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                        reinterpret_cast<const ndp::OrthItem*>(items.data_ptr()), n_items, n_mats,
                        p.data_ptr<float>(), (float)p_div, (float)eps, max_rank,
                        scratch.data_ptr<float>(), c, c + n_mats, cur_stream());
  check_launch("launch_psgd_orth");
}

void psgd_update(torch::Tensor geom, torch::Tensor ptrs, torch::Tensor items, torch::Tensor p_hat,
                 torch::Tensor q_sum, double q_div, c10::optional<torch::Tensor> q_warm, int mode,
                 double lr, double momentum) {
  check_dev(geom, "geom"); check_dev(ptrs, "ptrs"); check_dev(items, "items");
  check_f32(p_hat, "p_hat"); check_f32(q_sum, "q_sum");
  float* qw = nullptr;
  if (q_warm.has_value()) { check_f32(*q_warm, "q_warm"); qw = q_warm->data_ptr<float>(); }
  ndp::launch_psgd_update(reinterpret_cast<const MatGeom*>(geom.data_ptr()),
                          reinterpret_cast<const MatPtrs*>(ptrs.data_ptr()),
                          reinterpret_cast<const UItem*>(items.data_ptr()),
                          (int)n_of(items, sizeof(UItem)), p_hat.data_ptr<float>(),
                          q_sum.data_ptr<float>(), (float)q_div, qw, mode, (float)lr,
                          (float)momentum, cur_stream());
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

void delay_ns(int64_t ns) { ndp::launch_delay_ns(ns, cur_stream()); }

void checksum(torch::Tensor x, torch::Tensor out) {
  check_f32(x, "x");
  check_launch("launch_delay_ns");
  check_dev(out, "out");
  TORCH_CHECK(out.scalar_type() == torch::kFloat64 && out.numel() >= 257,
              "checksum out must be float64[>=257]");
  ndp::launch_checksum(x.data_ptr<float>(), x.numel(), out.data_ptr<double>(), cur_stream());
  check_launch("launch_checksum");
}

}  // namespace

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
  m.def("psgd_p", &psgd_p);
  m.def("psgd_q", &psgd_q);
  m.def("psgd_orth", &psgd_orth);
  m.def("psgd_update", &psgd_update);
  m.def("rank1_step", &rank1_step);
  m.def("seg_reduce", &seg_reduce);
  m.def("sgd_momentum", &sgd_momentum);
  m.def("add", &add);
  m.def("delay_ns", &delay_ns);
  m.def("checksum", &checksum);
}
