// Host-side AddressSanitizer / UBSan fuzz of the PowerSGD plan builder (csrc/plan.cpp):
// random model shapes and ranks -> build_plan / build_orth_items / build_seg_table, with
// the invariants the GPU kernels rely on checked on every plan (sanitizers
// on host code only — GPU ASan is not available on this pool).
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer \
//       -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Inetwork_distributed_pytorch_amd/csrc \
//       tools/asan/plan_fuzz.cpp network_distributed_pytorch_amd/csrc/plan.cpp -o /tmp/plan_fuzz
#include <cstdio>
#include <cstdlib>
#include <random>

#include "plan.h"

namespace ndp {
// the device-occupancy query lives in orth.hip; on the host fuzz use the conservative path
int orth_coresident_cap(int) { return -1; }
int orth_rows_per_thread(int max_rank) {
  if (max_rank <= 8) return 8;
  if (max_rank <= 16) return 4;
  if (max_rank <= 32) return 2;
  return 1;
}
}  // namespace ndp

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "invariant failed: %s (line %d)\n", #c, __LINE__); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
  std::mt19937_64 rng(1234);
  int64_t plans = 0;
  for (int it = 0; it < iters; ++it) {
    const int n_mats = 1 + (int)(rng() % 60);
    const int rank = 1 + (int)(rng() % 64);
    std::vector<std::pair<int64_t, int64_t>> shapes;
    for (int i = 0; i < n_mats; ++i) {
      const int64_t n = 1 + (int64_t)(rng() % (rng() % 4 == 0 ? 40000 : 600));
      const int64_t m = 1 + (int64_t)(rng() % (rng() % 4 == 0 ? 5000 : 600));
      shapes.emplace_back(n, m);
    }
    ndp::Plan pl;
    try {
      pl = ndp::build_plan(shapes, rank);
    } catch (const std::exception&) {
      continue;  // e.g. a matrix whose MGS needs more workgroups than the conservative cap
    }
    ++plans;
    CHECK((int)pl.geom.size() == n_mats);
    int64_t p_off = 0, q_off = 0;
    for (int i = 0; i < n_mats; ++i) {
      const ndp::MatGeom& g = pl.geom[i];
      CHECK(g.n == shapes[i].first && g.m == shapes[i].second);
      CHECK(g.r >= 1 && g.r <= rank && g.r <= g.n && g.r <= g.m);
      CHECK(g.p_off == p_off && g.q_off == q_off);
      p_off += g.n * g.r;
      q_off += g.m * g.r;
    }
    CHECK(pl.p_total == p_off && pl.q_total == q_off);
    for (const auto& it2 : pl.p_items) CHECK(it2.mat >= 0 && it2.mat < n_mats && it2.k0 < it2.k1);
    for (const auto& it2 : pl.q_items) CHECK(it2.mat >= 0 && it2.mat < n_mats && it2.row0 < it2.row1);
    for (const auto& it2 : pl.orth_items) {
      CHECK(it2.mat >= 0 && it2.mat < n_mats && it2.row0 < it2.row1 && it2.wg < it2.nwg);
      CHECK(it2.row1 <= pl.geom[it2.mat].n);
    }
    std::vector<ndp::SegSpec> specs;
    for (int i = 0; i < n_mats; ++i)
      specs.push_back({(uintptr_t)(16 * (i + 1)), (uintptr_t)(16 * (i + 7)), shapes[i].first * (i % 3 + 1),
                       shapes[i].first, (int32_t)(i % 4 + 1), 1.f});
    const ndp::SegTable t = ndp::build_seg_table(specs);
    CHECK(t.entries.size() == t.prefix.size());
  }
  std::printf("plan_fuzz ok: %lld plans\n", (long long)plans);
  return 0;
}
