// combine.h — lane codec of the in-library RCCL combine (mbx_combine=rccl).
//
// A sharded global aggregate (COUNT / exact int128 SUM over
// row-range shards) leaves one partial row per shard device.  Each partial
// value travels as three int64 lanes {lo, hi, flags} (flags bit 0: non-NULL),
// so COUNT, SUM as HUGEINT / DECIMAL(38,s) and integer MIN / MAX share one
// ncclInt64 all-gather; no RCCL reduction op adds 128-bit integers, so the
// gathered lanes are combined carry-correct afterwards (CombineColumn, on
// device 0 by the combine kernel, and on the host by the CPU tests through
// duckdb_mbx_combine_lanes).  A COUNT-only row needs no int128: its lanes are
// the counts themselves, summed into device 0 by one ncclInt64 reduce.  Every rank
// appends its device error word, so a shard's overflow is raised as on one
// device.  Shared by the kernels (rccl_combine.cpp) and the host (shim.cpp).
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define MBX_HD __host__ __device__
#else
#define MBX_HD
#endif

namespace mbx {
namespace rc {

constexpr int kMaxCols = 32;  // partial columns one combine carries

// how the ranks' values of a partial column combine
enum Kind : int8_t {
  K_SUM = 0,  // COUNT, COUNT(*), SUM: int128 add; NULL only if every rank's is NULL
  K_MIN = 1,
  K_MAX = 2,
};

// int64 lanes per rank: 3 per column (or 1 per column for a COUNT-only row), then the error word
MBX_HD inline int LanesPerRank(int ncols, bool counts_only) { return (counts_only ? ncols : 3 * ncols) + 1; }

// int64 lanes per dense GROUP BY slot: presence, then {lo, hi, flags} per column
MBX_HD inline int SlotLanes(int ncols) { return 1 + 3 * ncols; }

MBX_HD inline int Cmp128(int64_t alo, int64_t ahi, int64_t blo, int64_t bhi) {
  if (ahi != bhi) return ahi < bhi ? -1 : 1;
  const uint64_t a = (uint64_t)alo, b = (uint64_t)blo;
  return a < b ? -1 : a > b ? 1 : 0;
}

// (lo, hi) += (blo, bhi), two's complement int128 with the carry of the low word
MBX_HD inline void Add128(int64_t &lo, int64_t &hi, int64_t blo, int64_t bhi) {
  const uint64_t l = (uint64_t)lo + (uint64_t)blo;
  const uint64_t carry = l < (uint64_t)lo ? 1u : 0u;
  hi = (int64_t)((uint64_t)hi + (uint64_t)bhi + carry);
  lo = (int64_t)l;
}

// out[0..2] = column j combined over nranks ranks; rank r's lanes start at g + r * stride
MBX_HD inline void CombineColumn(const int64_t *g, int nranks, int stride, int j, int8_t kind, int64_t *out) {
  int64_t lo = 0, hi = 0, fl = 0;
  for (int r = 0; r < nranks; r++) {
    const int64_t *x = g + (int64_t)r * stride + 3 * j;
    if (!(x[2] & 1)) continue;  // a NULL partial (SUM / MIN / MAX of no valid row)
    if (kind == K_SUM) {
      Add128(lo, hi, x[0], x[1]);
    } else if (!(fl & 1) || (kind == K_MIN ? Cmp128(x[0], x[1], lo, hi) < 0 : Cmp128(x[0], x[1], lo, hi) > 0)) {
      lo = x[0], hi = x[1];
    }
    fl |= 1;
  }
  out[0] = lo, out[1] = hi, out[2] = fl;
}

}  // namespace rc
}  // namespace mbx
