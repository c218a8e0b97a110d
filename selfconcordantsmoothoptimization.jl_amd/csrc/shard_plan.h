// Host-only bookkeeping of a multi-device context (scs_create_multi): which rows of the
// caller's N_global x m problem each device holds, and how a caller's arguments map onto
// them.  Pure C++ (no HIP), so tests/test_shard_plan.py compiles it with the host
// sanitizers and checks it without a GPU.
//
// The split is scsopt.shard.row_range's: contiguous, balanced blocks, the first N % ndev
// devices holding one more row -- the same rows a one-process-per-GPU run gives each rank,
// so both launch modes shard identically.
#pragma once
#include <stdint.h>

#include <vector>

namespace scs {

struct RowBlock {
  int64_t r0 = 0, r1 = 0;   // rows [r0, r1) of the global problem
  int64_t rows() const { return r1 - r0; }
};

inline RowBlock row_block(int64_t N, int ndev, int d) {
  RowBlock b;
  if (ndev < 1 || d < 0 || d >= ndev || N < 0) return b;
  const int64_t base = N / ndev, rem = N % ndev;
  b.r0 = (int64_t)d * base + (d < rem ? d : rem);
  b.r1 = b.r0 + base + (d < rem ? 1 : 0);
  return b;
}

inline std::vector<RowBlock> row_plan(int64_t N, int ndev) {
  std::vector<RowBlock> p;
  for (int d = 0; d < ndev; ++d) p.push_back(row_block(N, ndev, d));
  return p;
}

// The device holding global row r (-1 when r is outside [0, N)).
inline int row_owner(const std::vector<RowBlock>& plan, int64_t r) {
  for (int d = 0; d < (int)plan.size(); ++d)
    if (r >= plan[d].r0 && r < plan[d].r1) return d;
  return -1;
}

// A caller's row window [q0, q0 + nq) (scs_get_data) cut into the pieces each device holds:
// (device, first local row, rows, offset of the piece in the window).
struct RowPiece {
  int dev = 0;
  int64_t local0 = 0, n = 0, off = 0;
};

inline std::vector<RowPiece> window_pieces(const std::vector<RowBlock>& plan, int64_t q0, int64_t nq) {
  std::vector<RowPiece> out;
  const int64_t q1 = q0 + nq;
  for (int d = 0; d < (int)plan.size(); ++d) {
    const int64_t a = q0 > plan[d].r0 ? q0 : plan[d].r0;
    const int64_t b = q1 < plan[d].r1 ? q1 : plan[d].r1;
    if (a >= b) continue;
    RowPiece p;
    p.dev = d;
    p.local0 = a - plan[d].r0;
    p.n = b - a;
    p.off = a - q0;
    out.push_back(p);
  }
  return out;
}

}  // namespace scs
