#pragma once
#include <cstdint>
#include <utility>
#include <vector>

#include "ndp_kernels.h"

namespace ndp {

struct Plan {
  std::vector<MatGeom> geom;
  std::vector<int32_t> q_rows;  // rows per Q split-K chunk, per matrix
  std::vector<PItem> p_items;
  int64_t n_p_blocks = 0;  // P row blocks / Q column blocks (in-kernel split-K arrival counters)
  int64_t n_q_blocks = 0;
  std::vector<QItem> q_items;
  std::vector<UItem> u_items;
  std::vector<OrthItem> orth_items;
  int64_t p_total = 0, q_total = 0, pp_total = 0, qp_total = 0;
  int max_rank = 1;
  int32_t p_cols = kPKW;  // columns per P item (wide plans)
};

// shapes[i] = (n_i, m_i) of every >1-D tensor, in model.parameters() order
Plan build_plan(const std::vector<std::pair<int64_t, int64_t>>& shapes, int rank);

// multi-workgroup MGS work list for the given matrices (rows split in 256*RPT blocks)
std::vector<OrthItem> build_orth_items(const std::vector<MatGeom>& geom, int max_rank);

struct SegSpec {
  uintptr_t src, dst;
  int64_t numel, stride;
  int32_t chunks;
  float div;
};

struct SegTable {
  std::vector<SegEntry> entries;
  std::vector<int64_t> prefix;
  int64_t n_blocks = 0;
};

SegTable build_seg_table(const std::vector<SegSpec>& specs);

}  // namespace ndp
