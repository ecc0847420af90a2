// PowerSGD execution-plan builder (host C++).
//
// The reference re-derives its P/Q layout every call with Python loops
// (ddp_powersgd_guide_cifar10/reducer.py:72-98) and allocates p_memory / q_memory once
// (reducer.py:82-84).  Here the layout and the load-balanced work lists for every
// grouped kernel are computed ONCE per parameter set:
//   * P / Q buffer offsets in reference order (so the all-reduced payload and its byte
//     count are identical to the reference: SURVEY.md §2.7);
//   * P items  : (matrix, 64-row block, 256-wide k-chunk; 16 x 1024 up to rank 16) -> split-K over m;
//   * Q items  : (matrix, 256-col block, row chunk)          -> split-K over n;
//   * U items  : (matrix, 16x256 tile; 64x64 above rank 16)  -> fused decompress/update;
//   * split-K slab offsets for the deterministic seg_reduce.
#include <cstdlib>
#include "plan.h"

#include <algorithm>
#include <stdexcept>

namespace ndp {

// columns per wide P item: 1024 (default), 512 or 256 (NDP_PSGD_PKW, A/B).  Round 5 measured
// narrower items slower (profiles/r5/bench_psgd_pkw_ab.jsonl) with a kernel that still looped over
// 1024 columns (3/4 of its loads masked off); the kernel now has one instance per width.
// Default by the plan's max rank (tools/psgd_bench.py, round 6): rank <= 8 -> 512 (ResNet-18 r=4
// reducer 112.0 -> 106.4 µs; 256: 109.1.  DistilBERT r=8: 676 µs at 1024 against 700 at 512 until
// the P pass kept its single load group's e stores past the split-K arrival; since, 1024: 685.7 /
// 686.1 / 684.7 / 686.7, 512: 678.7 / 679.1, 256: 808.7 / 806.8 — profiles/r6/psgd_pkw_bert8.jsonl),
// else 1024.
int64_t p_item_cols(int plan_rank) {
  const int64_t dflt = plan_rank <= 8 ? 512 : kPKW;
  const char* e = getenv("NDP_PSGD_PKW");
  const int64_t v = e ? atoll(e) : dflt;
  return (v == 256 || v == 512 || v == 1024) ? v : dflt;
}

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

Plan build_plan(const std::vector<std::pair<int64_t, int64_t>>& shapes, int rank) {
  if (rank < 1 || rank > kMaxRank)
    throw std::invalid_argument("PowerSGD rank must be in [1, 64]");
  Plan pl;
  pl.max_rank = 0;
  int64_t p_off = 0, q_off = 0, pp_off = 0, qp_off = 0;
  int plan_rank = 1;  // max over matrices of min(n, m, rank): picks the update tile shape
  for (const auto& s : shapes) plan_rank = std::max<int>(plan_rank, (int)std::min<int64_t>(std::min(s.first, s.second), rank));
  const bool wide = plan_rank <= kUWideMaxRank;
  const int64_t u_rows = wide ? kUWideRows : kURows, u_cols = wide ? kUWideCols : kUCols;
  for (size_t i = 0; i < shapes.size(); ++i) {
    const int64_t n = shapes[i].first, m = shapes[i].second;
    if (n < 1 || m < 1) throw std::invalid_argument("empty matrix in PowerSGD plan");
    if (n > (1LL << 30) || m > (1LL << 30)) throw std::invalid_argument("matrix too large");
    const int64_t r = std::min<int64_t>(std::min(n, m), rank);
    MatGeom g{};
    g.n = (int32_t)n;
    g.m = (int32_t)m;
    g.r = (int32_t)r;
    g.vec = 0;
    g.p_off = (int32_t)p_off;
    g.q_off = (int32_t)q_off;
    const int64_t p_rows = wide ? kPWRows : kPRows, p_k = wide ? p_item_cols(plan_rank) : kPK;
    g.p_chunks = (int32_t)cdiv(m, p_k);
    // Q split over n: 64-row chunks, but at most 64 chunks (cap the slab scratch), and
    // never more rows than the LDS tile holds.
    int64_t rc = 64;
    if (cdiv(n, rc) > 64) rc = std::min<int64_t>(kQRowsMax, ((cdiv(n, 64) + 3) / 4) * 4);
    if (rc > n) rc = n;
    g.q_chunks = (int32_t)cdiv(n, rc);
    g.pp_off = (int32_t)pp_off;
    g.qp_off = (int32_t)qp_off;
    pl.geom.push_back(g);
    pl.q_rows.push_back((int32_t)rc);

    for (int64_t row0 = 0; row0 < n; row0 += p_rows, ++pl.n_p_blocks)
      for (int64_t c = 0; c < g.p_chunks; ++c) {
        PItem it{};
        it.mat = (int32_t)i;
        it.row0 = (int32_t)row0;
        it.k0 = (int32_t)(c * p_k);
        it.k1 = (int32_t)std::min<int64_t>(m, (c + 1) * p_k);
        it.chunk = (int32_t)c;
        it.rb = (int32_t)pl.n_p_blocks;  // arrival counter of the in-kernel split-K finish
        pl.p_items.push_back(it);
      }
    // a column block's row chunks are consecutive in the grid, so the in-kernel finishes
    // (last arriver per column block) are spread over the launch instead of all at its end
    const int32_t cb0 = (int32_t)pl.n_q_blocks;
    for (int64_t col0 = 0; col0 < m; col0 += kQCols)
      for (int64_t c = 0; c < g.q_chunks; ++c) {
        QItem it{};
        it.mat = (int32_t)i;
        it.col0 = (int32_t)col0;
        it.row0 = (int32_t)(c * rc);
        it.row1 = (int32_t)std::min<int64_t>(n, (c + 1) * rc);
        it.chunk = (int32_t)c;
        it.cb = cb0 + (int32_t)(col0 / kQCols);
        pl.q_items.push_back(it);
      }
    pl.n_q_blocks += cdiv(m, kQCols);
    for (int64_t row0 = 0; row0 < n; row0 += u_rows)
      for (int64_t col0 = 0; col0 < m; col0 += u_cols) {
        UItem it{};
        it.mat = (int32_t)i;
        it.row0 = (int32_t)row0;
        it.col0 = (int32_t)col0;
        pl.u_items.push_back(it);
      }

    p_off += n * r;
    q_off += m * r;
    pp_off += g.p_chunks * n * r;
    qp_off += g.q_chunks * m * r;
    pl.max_rank = std::max<int>(pl.max_rank, (int)r);
    if (p_off > (1LL << 31) - 1 || q_off > (1LL << 31) - 1 || pp_off > (1LL << 31) - 1 ||
        qp_off > (1LL << 31) - 1)
      throw std::invalid_argument("PowerSGD plan exceeds int32 offsets");
  }
  pl.p_cols = wide ? (int32_t)p_item_cols(plan_rank) : (int32_t)kPK;
  pl.p_total = p_off;
  pl.q_total = q_off;
  pl.pp_total = pp_off;
  pl.qp_total = qp_off;
  if (pl.max_rank == 0) pl.max_rank = 1;
  pl.orth_items = build_orth_items(pl.geom, pl.max_rank);
  return pl;
}

std::vector<OrthItem> build_orth_items(const std::vector<MatGeom>& geom, int max_rank) {
  const int64_t rows_per_wg = 256LL * orth_rows_per_thread(max_rank);
  std::vector<OrthItem> items;
  for (size_t i = 0; i < geom.size(); ++i) {
    const int64_t n = geom[i].n;
    const int64_t nwg = std::max<int64_t>(1, cdiv(n, rows_per_wg));
    const int32_t slab0 = (int32_t)items.size();
    for (int64_t w = 0; w < nwg; ++w) {
      OrthItem it{};
      it.mat = (int32_t)i;
      it.row0 = (int32_t)(w * rows_per_wg);
      it.row1 = (int32_t)std::min<int64_t>(n, (w + 1) * rows_per_wg);
      it.wg = (int32_t)w;
      it.nwg = (int32_t)nwg;
      it.slab0 = slab0;
      items.push_back(it);
    }
  }
  // every workgroup of ONE matrix must be co-resident (spin barriers; grid-order dispatch
  // means other matrices' workgroups always drain): check against the measured occupancy
  // of the kernel instance (orth.hip), or a conservative constant without a device
  int cap = orth_coresident_cap(max_rank);
  if (cap <= 0) cap = 64;
  for (const OrthItem& it : items)
    if (it.nwg > cap)
      throw std::invalid_argument("orthogonalisation: a matrix needs more workgroups than can be co-resident");
  return items;
}

SegTable build_seg_table(const std::vector<SegSpec>& specs) {
  SegTable t;
  int64_t blocks = 0;
  for (const SegSpec& s : specs) {
    if (s.numel <= 0) continue;
    SegEntry e{};
    e.src = reinterpret_cast<const float*>(s.src);
    e.dst = reinterpret_cast<float*>(s.dst);
    e.numel = s.numel;
    e.stride = s.stride;
    e.chunks = s.chunks < 1 ? 1 : s.chunks;
    e.div = s.div;
    e.vec = ((s.src & 15) == 0 && (s.dst & 15) == 0 && (e.chunks == 1 || (s.stride & 3) == 0))
                ? 1 : 0;
    t.entries.push_back(e);
    t.prefix.push_back(blocks);
    blocks += cdiv(s.numel, kSegBlockElems);
  }
  t.n_blocks = blocks;
  return t;
}

}  // namespace ndp
