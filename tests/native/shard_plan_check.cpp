// Host check of the multi-device row bookkeeping (csrc/shard_plan.h), built by
// tests/test_shard_plan.py with the host sanitizers.  Prints one line per (N, ndev):
// "N ndev r0:r1 r0:r1 ..." for the Python side to compare with scsopt.shard.row_range, and exits
// non-zero if a structural property fails.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../selfconcordantsmoothoptimization.jl_amd/csrc/shard_plan.h"

using namespace scs;

static int fails = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s at line %d\n", #c, __LINE__);      \
      ++fails;                                                         \
    }                                                                  \
  } while (0)

int main() {
  const long long Ns[] = {1, 7, 8, 9, 1000, 3001, 1048576, 4194304, 4194311};
  for (long long N : Ns)
    for (int nd = 1; nd <= 8; ++nd) {
      if (N < nd) continue;
      const std::vector<RowBlock> p = row_plan(N, nd);
      CHECK((int)p.size() == nd);
      CHECK(p.front().r0 == 0 && p.back().r1 == N);
      for (int d = 0; d < nd; ++d) {
        CHECK(p[d].rows() >= N / nd && p[d].rows() <= N / nd + 1);
        if (d) CHECK(p[d].r0 == p[d - 1].r1);
      }
      // every row has exactly one owner
      for (long long r : {0LL, N / 2, N - 1}) CHECK(row_owner(p, r) >= 0 && p[row_owner(p, r)].r0 <= r);
      CHECK(row_owner(p, N) == -1 && row_owner(p, -1) == -1);
      // windows: the pieces tile the window exactly, in order, each inside its device's block
      const long long wins[][2] = {{0, N}, {N / 3, N / 3 + 1}, {N / 5, N - N / 5}, {N - 1, 1}, {0, 0}};
      for (const auto& w : wins) {
        const std::vector<RowPiece> pc = window_pieces(p, w[0], w[1]);
        long long cov = 0;
        for (size_t k = 0; k < pc.size(); ++k) {
          CHECK(pc[k].off == cov);
          CHECK(pc[k].local0 >= 0 && pc[k].local0 + pc[k].n <= p[pc[k].dev].rows());
          CHECK(p[pc[k].dev].r0 + pc[k].local0 == w[0] + pc[k].off);
          cov += pc[k].n;
        }
        CHECK(cov == w[1]);
      }
      std::printf("%lld %d", N, nd);
      for (const RowBlock& b : p) std::printf(" %lld:%lld", (long long)b.r0, (long long)b.r1);
      std::printf("\n");
    }
  // out-of-range arguments give empty blocks, not UB
  CHECK(row_block(10, 0, 0).rows() == 0 && row_block(10, 2, 5).rows() == 0);
  return fails ? 1 : 0;
}
