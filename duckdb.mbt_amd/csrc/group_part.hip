// group_part.hip — GROUP BY one integer key over a key range too wide for
// one LDS table (the zone map bounds it to (1024, PartGroupMaxRange]): rows are
// partitioned by key range, then every partition is reduced in LDS.
//
// Why not per-row global atomics (the hash path's group_reduce): on MI355X a
// global atomic executes at the memory side, one request per lane when the
// lanes hit scattered rows (MI355X_MICROARCH.md §Global float atomics; the
// integer form behaves alike), so a row-at-a-time reduction of 1e9 rows into
// 1e5 groups ran 205 ms for its atomics alone (profiles/r06_hash/).  Here
// every row's aggregate update is an LDS atomic, and HBM sees three streams:
//   1. pg_hist     each workgroup counts its contiguous row chunk's rows per
//                  partition (partition = (key - kmin) >> shift) in LDS;
//                  keys only;
//   2. (scan)      exclusive prefix over [partition][workgroup] counts:
//                  partition p's rows land in one contiguous run, every
//                  workgroup its own sub-run;
//   3. pg_scatter  the same chunks again, in tiles counting-sorted by
//                  partition in LDS and stored run by run into the workgroup's
//                  sub-run of each partition: one 8-byte record per row
//                  ((v << shift) | index in partition) when the value's zone map
//                  leaves its top bits free, else a u16 index + the values;
//   4. pg_reduce   the partitioned rows in fixed-size pieces (grid = pieces):
//                  each piece walks the partitions it overlaps, adds its rows
//                  into an LDS table of the partition's keys (COUNT, int64
//                  sums made overflow-free by the piece size, MIN / MAX), and
//                  flushes the non-empty keys with one carry-correct int128
//                  atomic set per key into the dense per-key states.
// HBM bytes per row with one INT64 key and value (c3h): 8 (hist) + 16 + 8
// (scatter) + 8 (reduce) = 40 B against the 16 B the query names.  F3h (the
// second half of this file) does the same over a hashed partition function
// for keys too sparse for dense states.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "device.h"
#include "knobs.h"
#include "phys.h"

namespace mbx {
namespace dev {

namespace {
constexpr int kReduceThreads = 1024;  // the reduce pass: one 16-wave workgroup per CU (its LDS table bounds it)

__device__ __forceinline__ void state_add(AggState *st, unsigned long long cnt, long long sum, long long mn,
                                          long long mx, bool mm) {
  atomicAdd(&st->count, cnt);
  const unsigned long long lo = (unsigned long long)sum;
  const unsigned long long old = atomicAdd(&st->sum_lo, lo);
  const unsigned long long carry = old + lo < old ? 1ull : 0ull;
  const unsigned long long hi = (unsigned long long)(sum >> 63) + carry;
  if (hi) atomicAdd((unsigned long long *)&st->sum_hi, hi);
  if (mm) {
    atomicMin(&st->min_i, mn);
    atomicMax(&st->max_i, mx);
  }
}
}  // namespace

// rows [w * chunk, min(n, (w + 1) * chunk)) of workgroup w
// a row's partition: (key - kmin) >> shift, or with HASHED the top `shift`
// bits of the key's hash (F3h)
__device__ __forceinline__ uint64_t pg_mix(uint64_t x) {  // splitmix64's finaliser
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
template <bool HASHED>
__device__ __forceinline__ int pg_part(int64_t k, int64_t kmin, int shift) {
  return HASHED ? (int)(pg_mix((uint64_t)k) >> (64 - shift)) : (int)((uint64_t)(k - kmin) >> shift);
}

template <typename TK, bool HASHED = false>
__global__ __launch_bounds__(1024) void pg_hist_kernel(const TK *__restrict__ key, int64_t n, int64_t chunk,
                                                      int64_t kmin, int shift, int np,
                                                      unsigned int *__restrict__ hist /* [np][grid] */) {
  extern __shared__ unsigned int h[];
  for (int p = threadIdx.x; p < np; p += blockDim.x) h[p] = 0;
  __syncthreads();
  // (one row per lane per load: 16-byte row pairs measured slower here and in
  // the scatter -- 1.32 vs 1.23 ms and 6.77 vs 6.15 ms at 1e6 keys)
  const int64_t b = (int64_t)blockIdx.x * chunk, e = min(n, b + chunk);
  const int64_t B = blockDim.x;
  int64_t i = b + threadIdx.x;
  for (; i + 3 * B < e; i += 4 * B) {  // four rows in flight per lane
    int64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; u++) k[u] = (int64_t)key[i + u * B];
#pragma unroll
    for (int u = 0; u < 4; u++) atomicAdd(&h[pg_part<HASHED>(k[u], kmin, shift)], 1u);
  }
  for (; i < e; i += B) atomicAdd(&h[pg_part<HASHED>((int64_t)key[i], kmin, shift)], 1u);
  __syncthreads();
  for (int p = threadIdx.x; p < np; p += blockDim.x) hist[(size_t)p * gridDim.x + blockIdx.x] = h[p];
}

// Rows of a workgroup's chunk in tiles of kTile: each tile is counting-sorted
// by partition in LDS (a returning LDS add gives a row its rank in its
// partition, a block scan the partitions' bases), staged there, and written
// out in staged order, so consecutive lanes store consecutive slots of one
// partition's run (coalesced) instead of one scattered 2- and 8-byte store per
// row.  The key leaves as its index inside the partition (u16) -- or, with
// PACK (one INT64 value column whose zone map leaves its top bits unused),
// inside the value's low bits: one 8-byte record per row, (v << shift) | index.
// TILE rows per tile, 8 per thread: 8192-row tiles in one 16-wave workgroup
// per CU where the staging fits LDS (longer runs per partition), else 4096-row
// tiles in two 8-wave workgroups per CU (one stages while the other stores)
constexpr int kScatterThreads = 512, kTile = 4096;

template <typename TK, typename TV, int NV, bool PACK, int TILE>
__global__ __launch_bounds__(TILE / 8) void pg_scatter_kernel(
    const TK *__restrict__ key, const TV *__restrict__ v0, const TV *__restrict__ v1, int64_t n, int64_t chunk,
    int64_t kmin, int shift, int np, const unsigned int *__restrict__ off /* [np][grid] */, uint16_t *__restrict__ ok,
    TV *__restrict__ ov0, TV *__restrict__ ov1) {
  constexpr int kTile = TILE, kScatterThreads = TILE / 8;
  constexpr int RPT = kTile / kScatterThreads;  // rows per thread and tile
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  TV *sv0 = (TV *)lds;                            // staged values
  TV *sv1 = sv0 + (NV >= 2 ? kTile : 0);
  uint16_t *sk = (uint16_t *)(sv0 + (size_t)kTile * (NV >= 2 ? 2 : NV));  // staged keys (index in partition)
  uint16_t *sp = sk + kTile;                      // staged rows' partitions
  unsigned int *cur = (unsigned int *)(sp + kTile);  // this workgroup's next global slot per partition
  unsigned int *cnt = cur + np;                   // tile: rows per partition
  unsigned int *base = cnt + np;                  // tile: exclusive scan of cnt
  unsigned int *wsum = base + np;                 // scan: per-wave totals
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = kScatterThreads / 64;
  for (int p = t; p < np; p += kScatterThreads) cur[p] = off[(size_t)p * gridDim.x + blockIdx.x];
  const uint32_t lmask = (1u << shift) - 1u;
  const int64_t b = (int64_t)blockIdx.x * chunk, e = min(n, b + chunk);
  // the next tile is loaded into registers while this one's rows are stored
  // (straight-line loads and stores, as in pg_hscatter: a row past the chunk
  // loads the chunk's last row and stores into the pad slot after each array)
  uint32_t rel[RPT];
  TV a[RPT], c[RPT];
  auto load = [&](int64_t tb) {
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      const int64_t r = min(tb + u * kScatterThreads + t, e - 1);
      rel[u] = (uint32_t)((int64_t)key[r] - kmin);
      if (NV >= 1) a[u] = v0[r];
      if (NV >= 2) c[u] = v1[r];
    }
  };
  if (b < e) load(b);
  for (int64_t tb = b; tb < e; tb += kTile) {
    const int tn = (int)min((int64_t)kTile, e - tb);
    for (int p = t; p < np; p += kScatterThreads) cnt[p] = 0;
    __syncthreads();
    unsigned int rank[RPT];
    auto row_of = [&](int u) { return u * kScatterThreads + t; };
#pragma unroll
    for (int u = 0; u < RPT; u++)
      if (row_of(u) < tn) rank[u] = atomicAdd(&cnt[rel[u] >> shift], 1u);
    __syncthreads();
    // exclusive scan of cnt[0, np): each thread a run of consecutive entries,
    // then the runs' totals across the block
    const int per = (np + kScatterThreads - 1) / kScatterThreads, p0 = min(np, t * per), p1 = min(np, p0 + per);
    unsigned int run = 0;
    for (int p = p0; p < p1; p++) run += cnt[p];
    unsigned int incl = run;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      const unsigned int y = __shfl_up(incl, m, 64);
      if (lane >= m) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned int before = incl - run;
    for (int k = 0; k < w; k++) before += wsum[k];
    for (int p = p0; p < p1; p++) {
      base[p] = before;
      before += cnt[p];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      if (row_of(u) >= tn) continue;
      const int pp = (int)(rel[u] >> shift);
      const unsigned int pos = base[pp] + rank[u];
      sp[pos] = (uint16_t)pp;
      if (PACK) {
        sv0[pos] = (TV)(((uint64_t)a[u] << shift) | (uint64_t)(rel[u] & lmask));
        continue;
      }
      sk[pos] = (uint16_t)(rel[u] & lmask);
      if (NV >= 1) sv0[pos] = a[u];
      if (NV >= 2) sv1[pos] = c[u];
    }
    __syncthreads();
    load(min(tb + kTile, e - 1));
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      const int j = u * kScatterThreads + t;
      const int jj = min(j, tn - 1);
      const int pp = sp[jj];
      const size_t dst = j < tn ? (size_t)(cur[pp] + (unsigned int)j - base[pp]) : (size_t)n;  // (n: the pad slot)
      if (!PACK) ok[dst] = sk[jj];
      if (NV >= 1) ov0[dst] = sv0[jj];
      if (NV >= 2) ov1[dst] = sv1[jj];
    }
    __syncthreads();
    for (int p = t; p < np; p += kScatterThreads) cur[p] += cnt[p];
  }
}

// the reduce passes' piece: at most 2^20 rows, and the piece count a multiple
// of the CU count, so the last round of workgroups is not a partial one
// (1e9 rows: 1024 pieces of 976 563 rows instead of 954 of 2^20)
static int64_t BalancedPiece(int64_t n) {
  const int64_t cus = NumCUs(), target = (int64_t)1 << 20;
  const int64_t rounds = std::max<int64_t>(1, (n + cus * target - 1) / (cus * target));
  const int64_t pieces = cus * rounds;
  return std::max<int64_t>(4096, (n + pieces - 1) / pieces);
}

// an array of `bytes` plus one 16-byte pad slot, rounded up to 256 bytes
static size_t PadUp(size_t bytes) { return (bytes + 16 + 255) & ~(size_t)255; }

size_t ScatterLds(int np, int nv, int vb, int tile) {
  return (size_t)tile * vb * (nv >= 2 ? 2 : nv) + (size_t)tile * 4 + (size_t)np * 12 + 64;
}

// PC (value columns with piece x max|v| < 2^41): a row adds 2^42 + v to one
// 64-bit word, so COUNT and the sum share one LDS atomic (count = the word
// rounded to a multiple of 2^42, sum = the rest)
constexpr int kPcShift = 42;
__device__ __forceinline__ void pc_split(unsigned long long w, unsigned int *c, long long *sum) {
  const long long q = (long long)(w + (1ull << (kPcShift - 1))) >> kPcShift;
  *c = (unsigned int)q;
  *sum = (long long)(w - ((unsigned long long)q << kPcShift));
}

// Piece q = rows [q * piece, min(n, (q + 1) * piece)) of the partitioned
// arrays; start[p] = first row of partition p (start[np] = n).  LDS: the
// partition's table of KP keys -- COUNT(*) u32, then per value column its int64
// sum (and min / max).
template <typename TV, int NV, bool MM, bool PACK, bool PC>
__global__ __launch_bounds__(1024) void pg_reduce_kernel(const uint16_t *__restrict__ rk, const TV *__restrict__ rv0,
                                                        const TV *__restrict__ rv1, int64_t n, int64_t piece,
                                                        const unsigned int *__restrict__ start, int np, int shift,
                                                        int64_t range, unsigned long long *__restrict__ cstar,
                                                        AggState *__restrict__ st0, AggState *__restrict__ st1) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int KP = 1 << shift;
  unsigned int *cnt = (unsigned int *)lds;
  long long *sum0 = (long long *)(lds + (size_t)KP * 4);
  long long *sum1 = sum0 + KP;
  long long *mn0 = sum0 + (NV >= 2 ? 2 : 1) * KP, *mx0 = mn0 + KP, *mn1 = mx0 + KP, *mx1 = mn1 + KP;
  const int64_t a = (int64_t)blockIdx.x * piece, z = min(n, a + piece);
  if (a >= z) return;
  // the first partition that ends after a (start is ascending; np <= 4096)
  int lo = 0, hi = np - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)start[mid + 1] <= a) lo = mid + 1;
    else hi = mid;
  }
  for (int p = lo; p < np && (int64_t)start[p] < z; p++) {
    const int64_t s0 = max(a, (int64_t)start[p]), s1 = min(z, (int64_t)start[p + 1]);
    if (s0 >= s1) continue;
    for (int j = threadIdx.x; j < KP; j += blockDim.x) {
      cnt[j] = 0;
      if (NV >= 1) sum0[j] = 0;
      if (NV >= 2) sum1[j] = 0;
      if (MM) {
        mn0[j] = INT64_MAX, mx0[j] = INT64_MIN;
        if (NV >= 2) mn1[j] = INT64_MAX, mx1[j] = INT64_MIN;
      }
    }
    __syncthreads();
    const uint32_t base = (uint32_t)p << shift;
    auto add = [&](uint32_t k, TV x, TV y) {
      const int j = (int)k;  // the key's index inside partition p
      if (PC) {
        atomicAdd((unsigned long long *)&sum0[j], (1ull << kPcShift) + (unsigned long long)(long long)x);
      } else {
        atomicAdd(&cnt[j], 1u);
        if (NV >= 1) atomicAdd((unsigned long long *)&sum0[j], (unsigned long long)(long long)x);
      }
      if (NV >= 2) atomicAdd((unsigned long long *)&sum1[j], (unsigned long long)(long long)y);
      if (MM) {
        atomicMin(&mn0[j], (long long)x), atomicMax(&mx0[j], (long long)x);
        if (NV >= 2) atomicMin(&mn1[j], (long long)y), atomicMax(&mx1[j], (long long)y);
      }
    };
    if (PACK) {
      // 8-byte records two per lane (16-byte loads) from the first even row
      auto one = [&](TV r) { add((uint32_t)r & (uint32_t)(KP - 1), (TV)((int64_t)r >> shift), (TV)0); };
      const int64_t ev = (s0 + 1) & ~(int64_t)1;
      if (threadIdx.x == 0 && ev > s0) one(rv0[s0]);
      const int64_t B2 = 2 * (int64_t)blockDim.x;
      int64_t i = ev + 2 * threadIdx.x;
      typedef TV PV __attribute__((ext_vector_type(2)));
      for (; i + 3 * B2 + 1 < s1; i += 4 * B2) {
        PV x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = *(const PV *)(rv0 + i + u * B2);
#pragma unroll
        for (int u = 0; u < 4; u++) one(x[u].x), one(x[u].y);
      }
      for (; i < s1; i += B2) {
        one(rv0[i]);
        if (i + 1 < s1) one(rv0[i + 1]);
      }
      __syncthreads();
      goto flush;
    }
    {
    const int64_t B = blockDim.x;
    int64_t i = s0 + threadIdx.x;
    for (; i + 3 * B < s1; i += 4 * B) {
      uint32_t k[4];  // (u16 in memory)
      TV x[4], y[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (PACK) {
          const TV r = rv0[i + u * B];
          k[u] = (uint32_t)r & (uint32_t)(KP - 1);
          x[u] = (TV)((int64_t)r >> shift);
          continue;
        }
        k[u] = rk[i + u * B];
        if (NV >= 1) x[u] = rv0[i + u * B];
        if (NV >= 2) y[u] = rv1[i + u * B];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) add(k[u], NV >= 1 ? x[u] : (TV)0, NV >= 2 ? y[u] : (TV)0);
    }
    for (; i < s1; i += B) add(rk[i], NV >= 1 ? rv0[i] : (TV)0, NV >= 2 ? rv1[i] : (TV)0);
    __syncthreads();
    }
  flush:
    for (int j = threadIdx.x; j < KP; j += blockDim.x) {
      unsigned int c;
      long long s0j = 0;
      if (PC) pc_split((unsigned long long)sum0[j], &c, &s0j);
      else c = cnt[j], s0j = NV >= 1 ? sum0[j] : 0;
      const int64_t key = (int64_t)base + j;
      if (!c || key >= range) continue;
      atomicAdd(&cstar[key], (unsigned long long)c);
      if (NV >= 1) state_add(&st0[key], c, s0j, MM ? mn0[j] : 0, MM ? mx0[j] : 0, MM);
      if (NV >= 2) state_add(&st1[key], c, sum1[j], MM ? mn1[j] : 0, MM ? mx1[j] : 0, MM);
    }
    __syncthreads();
  }
}

// ---- F3h: the same over a hashed partition function (sparse integer keys) ----
// Records are the full key (stored as key ^ 2^63, so that 0 marks an empty
// table slot and INT64_MIN has a slot of its own) and, with one value column,
// the value: 16-byte records written by one store each.  The reduce pass keeps
// an LDS hash table per partition piece (open addressing, kHashSlots slots)
// and flushes its groups into a global table of kHashGlobal slots per
// partition; a table that fills up sets *overflow and the caller answers the
// query on the hash path instead.
constexpr int kHashParts = 9;      // log2 partitions
// the hashed scatter: 8192-row tiles in one 16-wave workgroup per CU, so a
// tile's run per partition averages 16 records (256 B) -- 4096-row tiles
// (8-record runs) in two workgroups per CU ran 8.70 vs 7.92 ms at 1e6 keys;
// 256 partitions (32-record runs) 8.42 ms of scatter but a slower reduce
constexpr int kHTile = 8192, kHThreads = 1024, kHBlocksPerCU = 1;
constexpr int kHashSlots = 4096;   // LDS table of a piece
constexpr int kHashGlobal = 8192;  // global table per partition
constexpr uint64_t kMsb = 0x8000000000000000ull;

template <typename TK, typename TV, int NV>
__global__ __launch_bounds__(kHThreads) void pg_hscatter_kernel(
    const TK *__restrict__ key, const TV *__restrict__ v0, int64_t n, int64_t chunk, int pbits, int np,
    const unsigned int *__restrict__ off, int64_t *__restrict__ rec /* [n][NV + 1] */) {
  constexpr int kTile = kHTile, kScatterThreads = kHThreads;
  constexpr int RPT = kTile / kScatterThreads, RS = NV + 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int64_t *srec = (int64_t *)lds;                                   // staged records
  uint16_t *sp = (uint16_t *)(srec + (size_t)kTile * RS);           // staged rows' partitions
  unsigned int *cur = (unsigned int *)(sp + kTile);
  unsigned int *cnt = cur + np, *base = cnt + np, *wsum = base + np;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int p = t; p < np; p += kScatterThreads) cur[p] = off[(size_t)p * gridDim.x + blockIdx.x];
  const int64_t b = (int64_t)blockIdx.x * chunk, e = min(n, b + chunk);
  // the next tile's rows are loaded into registers while the current tile's
  // staged records are stored, so the read and write streams overlap
  // Loads and stores are straight-line (no lane branches), so the compiler's
  // wait for the prefetched rows counts past the stores issued after them
  // instead of draining them: a row past the chunk loads the chunk's last row
  // and stores into the pad slot after the records.
  int64_t kk[RPT], vv[RPT];
  auto load = [&](int64_t tb) {
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      const int64_t r = min(tb + u * kScatterThreads + t, e - 1);
      kk[u] = (int64_t)key[r];
      if (NV >= 1) vv[u] = (int64_t)v0[r];
    }
  };
  if (b < e) load(b);
  for (int64_t tb = b; tb < e; tb += kTile) {
    const int tn = (int)min((int64_t)kTile, e - tb);
    for (int p = t; p < np; p += kScatterThreads) cnt[p] = 0;
    __syncthreads();
    int pp[RPT];
    unsigned int rank[RPT];
#pragma unroll
    for (int u = 0; u < RPT; u++)
      if (u * kScatterThreads + t < tn) pp[u] = pg_part<true>(kk[u], 0, pbits);
#pragma unroll
    for (int u = 0; u < RPT; u++)
      if (u * kScatterThreads + t < tn) rank[u] = atomicAdd(&cnt[pp[u]], 1u);
    __syncthreads();
    const int per = (np + kScatterThreads - 1) / kScatterThreads, p0 = min(np, t * per), p1 = min(np, p0 + per);
    unsigned int run = 0;
    for (int p = p0; p < p1; p++) run += cnt[p];
    unsigned int incl = run;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      const unsigned int y = __shfl_up(incl, m, 64);
      if (lane >= m) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned int before = incl - run;
    for (int k = 0; k < w; k++) before += wsum[k];
    for (int p = p0; p < p1; p++) {
      base[p] = before;
      before += cnt[p];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      if (u * kScatterThreads + t >= tn) continue;
      const unsigned int pos = base[pp[u]] + rank[u];
      sp[pos] = (uint16_t)pp[u];
      srec[(size_t)pos * RS] = (int64_t)((uint64_t)kk[u] ^ kMsb);
      if (NV >= 1) srec[(size_t)pos * RS + 1] = vv[u];
    }
    __syncthreads();
    load(min(tb + kTile, e - 1));  // (the last tile re-reads a row: no branch)
#pragma unroll
    for (int u = 0; u < RPT; u++) {
      const int j = u * kScatterThreads + t;
      const int jj = min(j, tn - 1);
      const int q = sp[jj];
      const size_t dst = j < tn ? (size_t)(cur[q] + (unsigned int)j - base[q]) : (size_t)n;  // (n: the pad slot)
      if (NV >= 1) {
        typedef int64_t P __attribute__((ext_vector_type(2)));
        *(P *)(rec + dst * 2) = *(const P *)(srec + (size_t)jj * 2);
      } else {
        rec[dst] = srec[jj];
      }
    }
    __syncthreads();
    for (int p = t; p < np; p += kScatterThreads) cur[p] += cnt[p];
  }
}

template <int NV, bool MM, bool PC>
__global__ __launch_bounds__(1024) void pg_hreduce_kernel(const int64_t *__restrict__ rec, int64_t n, int64_t piece,
                                                         const unsigned int *__restrict__ start, int np,
                                                         unsigned long long *__restrict__ gkeys,
                                                         unsigned long long *__restrict__ gcs,
                                                         AggState *__restrict__ gst, int *__restrict__ overflow) {
  constexpr int RS = NV + 1, C = kHashSlots;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned long long *tk = (unsigned long long *)lds;  // C + 1 slots: key ^ 2^63 (0: empty); slot C: INT64_MIN
  long long *sum = (long long *)(tk + C + 1);
  long long *mn = sum + C + 1, *mx = mn + C + 1;
  unsigned int *cnt = (unsigned int *)(lds + (size_t)(C + 1) * 8 * (NV >= 1 ? (MM ? 4 : 2) : 1));
  __shared__ int full;
  const int64_t a = (int64_t)blockIdx.x * piece, z = min(n, a + piece);
  if (a >= z) return;
  int lo = 0, hi = np - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)start[mid + 1] <= a) lo = mid + 1;
    else hi = mid;
  }
  if (threadIdx.x == 0) full = 0;
  for (int p = lo; p < np && (int64_t)start[p] < z; p++) {
    const int64_t s0 = max(a, (int64_t)start[p]), s1 = min(z, (int64_t)start[p + 1]);
    if (s0 >= s1) continue;
    for (int j = threadIdx.x; j <= C; j += blockDim.x) {
      tk[j] = 0, cnt[j] = 0;
      if (NV >= 1) sum[j] = 0;
      if (MM) mn[j] = INT64_MAX, mx[j] = INT64_MIN;
    }
    __syncthreads();
    typedef int64_t P __attribute__((ext_vector_type(2)));
    auto load = [&](int64_t i) {
      P r;
      if (NV >= 1) r = *(const P *)(rec + (size_t)i * 2);  // one 16-byte record
      else r.x = rec[i], r.y = 0;
      return r;
    };
    // a row's slot: its key's first probe is a compare-and-swap issued for
    // every row of the batch at once (their returns overlap), then each row
    // walks on only if that slot holds another key
    auto probe = [&](unsigned long long t, int h, unsigned long long c) {
      int probes = 1;
      while (c != 0 && c != t) {
        h = (h + 1) & (C - 1);
        if (probes++ == C) return -1;
        c = atomicCAS(&tk[h], 0ull, t);
      }
      return h;
    };
    auto update = [&](int slot, int64_t v) {
      if (PC) {
        atomicAdd((unsigned long long *)&sum[slot], (1ull << kPcShift) + (unsigned long long)v);
      } else {
        atomicAdd(&cnt[slot], 1u);
        if (NV >= 1) atomicAdd((unsigned long long *)&sum[slot], (unsigned long long)v);
      }
      if (NV >= 1 && MM) atomicMin(&mn[slot], (long long)v), atomicMax(&mx[slot], (long long)v);
    };
    auto first = [&](unsigned long long t) { return (int)(pg_mix(t) & (C - 1)); };
    auto add = [&](P r) {
      const unsigned long long t = (unsigned long long)r.x;
      int slot = C;  // (t == 0: the key INT64_MIN, slot C)
      if (t) {
        const int h = first(t);
        slot = probe(t, h, atomicCAS(&tk[h], 0ull, t));
      }
      if (slot < 0) full = 1;
      else update(slot, r.y);
    };
    // four records in flight per lane, and their first probes too: the
    // compare-and-swap waits on its return
    const int64_t B = blockDim.x;
    int64_t i = s0 + threadIdx.x;
    for (; i + 3 * B < s1; i += 4 * B) {
      P r[4];
#pragma unroll
      for (int u = 0; u < 4; u++) r[u] = load(i + u * B);
      int h[4];
      unsigned long long c[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const unsigned long long t = (unsigned long long)r[u].x;
        h[u] = t ? first(t) : C;
        c[u] = t ? atomicCAS(&tk[h[u]], 0ull, t) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const unsigned long long t = (unsigned long long)r[u].x;
        const int slot = t ? probe(t, h[u], c[u]) : C;
        if (slot < 0) full = 1;
        else update(slot, r[u].y);
      }
    }
    for (; i < s1; i += B) add(load(i));
    __syncthreads();
    if (full) {
      if (threadIdx.x == 0) atomicOr(overflow, 1);
      return;  // (uniform: every thread read the same flag after the barrier)
    }
    // the piece's groups into partition p's global table (slot p << log2(G);
    // INT64_MIN's group in the one slot after every partition's)
    const size_t gb = (size_t)p * kHashGlobal;
    for (int j = threadIdx.x; j <= C; j += blockDim.x) {
      unsigned int c;
      long long sj = 0;
      if (PC) pc_split((unsigned long long)sum[j], &c, &sj);
      else c = cnt[j], sj = NV >= 1 ? sum[j] : 0;
      if (!c) continue;
      size_t g = (size_t)np * kHashGlobal;
      if (j < C) {
        const unsigned long long t = tk[j];
        int h = (int)((pg_mix(t) >> 20) & (kHashGlobal - 1)), probes = 0;
        for (;;) {
          const unsigned long long o = atomicCAS(&gkeys[gb + h], 0ull, t);
          if (o == 0 || o == t) break;
          h = (h + 1) & (kHashGlobal - 1);
          if (++probes == kHashGlobal) {
            h = -1;
            break;
          }
        }
        if (h < 0) {
          atomicOr(overflow, 1);
          continue;
        }
        g = gb + h;
      }
      atomicAdd(&gcs[g], (unsigned long long)c);
      if (NV >= 1) state_add(&gst[g], c, sj, MM ? mn[j] : 0, MM ? mx[j] : 0, MM);
    }
    __syncthreads();
  }
}

bool PartGroupHashed(const PartGroupDesc &d, unsigned long long *gkeys, int *overflow, hipStream_t s) {
  if (d.n <= 0 || d.n >= ((int64_t)1 << 32) || d.nv < 0 || d.nv > 1) return false;
  if (d.kphys != P_I32 && d.kphys != P_I64) return false;
  if (d.nv > 0 && d.vphys != P_I32 && d.vphys != P_I64) return false;
  const int pbits = kHashParts, np = 1 << pbits;
  int64_t piece = BalancedPiece(d.n);
  if (d.nv > 0 && d.vmaxabs > 0) {
    const uint64_t cap = ((uint64_t)1 << 62) / d.vmaxabs;
    if (cap < 4096) return false;
    piece = std::min<int64_t>(piece, (int64_t)cap);
  }
  const int grid = NumCUs() * kHBlocksPerCU;  // (kHThreads workgroups in the hist and scatter passes)
  const int64_t chunk = (((d.n + grid - 1) / grid) + 255) & ~(int64_t)255;
  unsigned int *hist = (unsigned int *)d.scratch_hist, *off = hist + (size_t)np * grid;
  unsigned int *start = (unsigned int *)d.scratch_start;
  int64_t *rec = (int64_t *)d.scratch_rows;
  const size_t hl = (size_t)np * 4;
  if (d.kphys == P_I64)
    hipLaunchKernelGGL((pg_hist_kernel<int64_t, true>), dim3(grid), dim3(kHThreads), hl, s,
                       (const int64_t *)d.key, d.n, chunk, (int64_t)0, pbits, np, hist);
  else
    hipLaunchKernelGGL((pg_hist_kernel<int32_t, true>), dim3(grid), dim3(kHThreads), hl, s,
                       (const int32_t *)d.key, d.n, chunk, (int64_t)0, pbits, np, hist);
  size_t tmp = 0;
  const int nh = np * grid;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, hist, off, nh, s);
  if (tmp > d.scratch_scan_bytes) throw std::runtime_error("PartGroupHashed: scan scratch too small");
  (void)hipcub::DeviceScan::ExclusiveSum(d.scratch_scan, tmp, hist, off, nh, s);
  (void)hipMemcpy2DAsync(start, 4, off, (size_t)grid * 4, 4, np, hipMemcpyDeviceToDevice, s);
  (void)hipMemsetD32Async((hipDeviceptr_t)(start + np), (int)(unsigned int)d.n, 1, s);
  const size_t sl = (size_t)kHTile * 8 * (d.nv + 1) + (size_t)kHTile * 2 + (size_t)np * 12 + 64;
#define PHS(TK, TV, NV)                                                                                             \
  {                                                                                                                 \
    (void)hipFuncSetAttribute((const void *)pg_hscatter_kernel<TK, TV, NV>,                                         \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sl);                                 \
    hipLaunchKernelGGL((pg_hscatter_kernel<TK, TV, NV>), dim3(grid), dim3(kHThreads), sl, s,                       \
                       (const TK *)d.key, (const TV *)d.v0, d.n, chunk, pbits, np, off, rec);                       \
  }
#define PHSV(TK)                                                                                                    \
  if (d.nv == 0) PHS(TK, int64_t, 0)                                                                                \
  else if (d.vphys == P_I64) PHS(TK, int64_t, 1)                                                                    \
  else PHS(TK, int32_t, 1)
  if (d.kphys == P_I64) { PHSV(int64_t) } else { PHSV(int32_t) }
#undef PHSV
#undef PHS
  const int64_t total = (int64_t)np * kHashGlobal + 1;
  (void)hipMemsetAsync(gkeys, 0, (size_t)total * 8, s);
  (void)hipMemsetAsync(overflow, 0, 4, s);
  InitAggStatesCounts(d.st0, total, d.cstar, total, s);
  const int npieces = (int)((d.n + piece - 1) / piece);
  const size_t rl = (size_t)(kHashSlots + 1) * (8 * (d.nv >= 1 ? (d.mm ? 4 : 2) : 1) + 4) + 16;
  const bool pc = d.nv == 1 && (unsigned __int128)d.vmaxabs * (uint64_t)piece < ((unsigned __int128)1 << (kPcShift - 1)) &&
                  !Knob("MBX_PG_NO_PC");
#define PHR(NV, MM, PC)                                                                                             \
  {                                                                                                                 \
    (void)hipFuncSetAttribute((const void *)pg_hreduce_kernel<NV, MM, PC>,                                          \
                              hipFuncAttributeMaxDynamicSharedMemorySize,                                           \
                              (int)rl);  /* (the kernel's own static LDS word counts against 160 KiB) */            \
    hipLaunchKernelGGL((pg_hreduce_kernel<NV, MM, PC>), dim3(npieces), dim3(kReduceThreads), rl, s, rec, d.n,      \
                       piece, start, np, gkeys, d.cstar, d.st0, overflow);                                          \
  }
  if (d.nv == 0) PHR(0, false, false)
  else if (d.mm) { if (pc) PHR(1, true, true) else PHR(1, true, false) }
  else { if (pc) PHR(1, false, true) else PHR(1, false, false) }
#undef PHR
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess && Knob("MBX_PG_DEBUG")) fprintf(stderr, "[mbx] F3h: %s\n", hipGetErrorString(err));
  return err == hipSuccess;
}

int64_t PartGroupHashedSlots() { return ((int64_t)1 << kHashParts) * kHashGlobal + 1; }

void PartGroupHashedScratch(int64_t n, int nv, size_t *hist_bytes, size_t *start_bytes, size_t *rows_bytes,
                            size_t *scan_bytes) {
  const int np = 1 << kHashParts;
  const int grid = NumCUs() * kHBlocksPerCU;
  *hist_bytes = (size_t)np * grid * 4 * 2;
  *start_bytes = (size_t)(np + 1) * 4;
  *rows_bytes = (size_t)n * 8 * (nv + 1) + 256;
  size_t tmp = 0;
  unsigned int *dummy = nullptr;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, dummy, dummy, np * grid, (hipStream_t)0);
  *scan_bytes = tmp ? tmp : 16;
}

int PartGroupShift(int nv, bool mm) {
  // the largest partition table (power of two) that fits the LDS budget
  const int per_key = 4 + 8 * nv + (mm ? 16 * nv : 0);
  int shift = 15;
  while (shift > 10 && ((size_t)per_key << shift) > (size_t)128 * 1024) shift--;
  return shift;
}

int64_t PartGroupMaxRange(int nv, bool mm) { return (int64_t)kPartGroupMaxParts << PartGroupShift(nv, mm); }

bool PartGroup(const PartGroupDesc &d, hipStream_t s) {
  if (d.range <= 0 || d.range > PartGroupMaxRange(d.nv, d.mm) || d.n <= 0 || d.n >= ((int64_t)1 << 32)) return false;
  if (d.nv < 0 || d.nv > 2 || (d.kphys != P_I32 && d.kphys != P_I64)) return false;
  if (d.nv > 0 && d.vphys != P_I32 && d.vphys != P_I64) return false;
  const int shift = PartGroupShift(d.nv, d.mm);
  const int np = (int)((d.range + (1 << shift) - 1) >> shift);
  // int64 LDS sums stay exact over a piece: piece x max|v| < 2^62
  int64_t piece = BalancedPiece(d.n);
  if (d.nv > 0 && d.vmaxabs > 0) {
    const uint64_t cap = ((uint64_t)1 << 62) / d.vmaxabs;
    if (cap < 4096) return false;
    piece = std::min<int64_t>(piece, (int64_t)cap);
  }
  const int vb = d.vphys == P_I64 ? 8 : 4;
  // the scatter's tile: 8192 rows in one 16-wave workgroup per CU where the
  // staging fits LDS (c3h at 1e6 keys 9.33 vs 10.20 ms of kernels, 1e5 keys
  // 8.18 vs 8.23: longer runs per partition), else 4096-row tiles in two
  // workgroups per CU (MBX_PG_TILE=4096 forces these: A/B)
  int tile = ScatterLds(np, d.nv, vb, 8192) <= (size_t)150 * 1024 ? 8192 : kTile;
  if (const char *t = Knob("MBX_PG_TILE"))
    if (atoi(t) == 4096) tile = kTile;
  const int sthreads = tile / 8;
  const int grid = NumCUs() * (tile == 4096 ? 2 : 1);
  const int64_t chunk = (((d.n + grid - 1) / grid) + 255) & ~(int64_t)255;  // 2-row aligned pairs in every chunk
  // one INT64 value column whose |v| leaves shift + 1 top bits unused: the
  // partition index rides in the value's low bits (8-byte records)
  const bool pack = d.nv == 1 && d.vphys == P_I64 && d.vmaxabs < ((uint64_t)1 << (62 - shift));
  unsigned int *hist = (unsigned int *)d.scratch_hist;  // [np][grid] counts
  unsigned int *off = hist + (size_t)np * grid;         // ... and their exclusive scan
  unsigned int *start = (unsigned int *)d.scratch_start;  // [np + 1]
  uint16_t *rk = (uint16_t *)d.scratch_rows;  // (each array with its pad slot: PartGroupScratch)
  void *rv0 = (char *)d.scratch_rows + PadUp((size_t)d.n * 2);
  void *rv1 = (char *)rv0 + PadUp((size_t)d.n * vb);
  const size_t hl = (size_t)np * 4;
  if (d.kphys == P_I64)
    hipLaunchKernelGGL(pg_hist_kernel<int64_t>, dim3(grid), dim3(sthreads), hl, s, (const int64_t *)d.key,
                       d.n, chunk, d.kmin, shift, np, hist);
  else
    hipLaunchKernelGGL(pg_hist_kernel<int32_t>, dim3(grid), dim3(sthreads), hl, s, (const int32_t *)d.key,
                       d.n, chunk, d.kmin, shift, np, hist);
  const size_t sl = ScatterLds(np, d.nv, vb, tile);
  // partition p starts at the offset of its first workgroup's sub-run
  size_t tmp = 0;
  const int nh = np * grid;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, hist, off, nh, s);
  if (tmp > d.scratch_scan_bytes) throw std::runtime_error("PartGroup: scan scratch too small");
  (void)hipcub::DeviceScan::ExclusiveSum(d.scratch_scan, tmp, hist, off, nh, s);
  (void)hipMemcpy2DAsync(start, 4, off, (size_t)grid * 4, 4, np, hipMemcpyDeviceToDevice, s);
  (void)hipMemsetD32Async((hipDeviceptr_t)(start + np), (int)(unsigned int)d.n, 1, s);
#define PGS1(TK, TV, NV, PK, T)                                                                                     \
  {                                                                                                                 \
    (void)hipFuncSetAttribute((const void *)pg_scatter_kernel<TK, TV, NV, PK, T>,                                   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sl);                                 \
    hipLaunchKernelGGL((pg_scatter_kernel<TK, TV, NV, PK, T>), dim3(grid), dim3(T / 8), sl, s, (const TK *)d.key, \
                       (const TV *)d.v0, (const TV *)d.v1, d.n, chunk, d.kmin, shift, np, off, rk, (TV *)rv0,      \
                       (TV *)rv1);                                                                                  \
  }
#define PGS(TK, TV, NV, PK)                                                                                         \
  if (tile == 8192) PGS1(TK, TV, NV, PK, 8192) else PGS1(TK, TV, NV, PK, 4096)
#define PGSV(TK)                                                                                                    \
  if (d.vphys == P_I64) {                                                                                           \
    if (d.nv == 0) PGS(TK, int64_t, 0, false)                                                                       \
    else if (d.nv == 1) { if (pack) PGS(TK, int64_t, 1, true) else PGS(TK, int64_t, 1, false) }                     \
    else PGS(TK, int64_t, 2, false)                                                                                 \
  } else {                                                                                                          \
    if (d.nv == 0) PGS(TK, int32_t, 0, false)                                                                       \
    else if (d.nv == 1) PGS(TK, int32_t, 1, false)                                                                  \
    else PGS(TK, int32_t, 2, false)                                                                                 \
  }
  if (d.kphys == P_I64) { PGSV(int64_t) } else { PGSV(int32_t) }
#undef PGSV
#undef PGS
#undef PGS1
  InitAggStatesCounts(d.st0, d.nv >= 2 ? 2 * d.range : d.range, d.cstar, d.range, s);
  const int npieces = (int)((d.n + piece - 1) / piece);
  const bool pc = d.nv >= 1 && (unsigned __int128)d.vmaxabs * (uint64_t)piece < ((unsigned __int128)1 << (kPcShift - 1)) &&
                  !Knob("MBX_PG_NO_PC");
  const size_t rl = ((size_t)4 << shift) +
                    ((size_t)8 << shift) * (size_t)(d.nv == 0 ? 0 : d.nv + (d.mm ? 2 * d.nv : 0));
#define PGR1(TV, NV, MM, PK, PC)                                                                                    \
  {                                                                                                                 \
    (void)hipFuncSetAttribute((const void *)pg_reduce_kernel<TV, NV, MM, PK, PC>,                                   \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)rl);                                 \
    hipLaunchKernelGGL((pg_reduce_kernel<TV, NV, MM, PK, PC>), dim3(npieces), dim3(kReduceThreads), rl, s, rk,   \
                       (const TV *)rv0,                                                                             \
                       (const TV *)rv1, d.n, piece, start, np, shift, d.range, d.cstar, d.st0,                      \
                       d.st0 + d.range);                                                                            \
  }
#define PGR(TV, NV, MM, PK)                                                                                         \
  if (NV >= 1 && pc) PGR1(TV, NV, MM, PK, true) else PGR1(TV, NV, MM, PK, false)
#define PGRV(TV)                                                                                                    \
  if (d.nv == 0) PGR(TV, 0, false, false)                                                                           \
  else if (d.nv == 1) { if (d.mm) PGR(TV, 1, true, false) else PGR(TV, 1, false, false) }                            \
  else { if (d.mm) PGR(TV, 2, true, false) else PGR(TV, 2, false, false) }
  if (d.vphys == P_I64) {
    if (pack) {
      if (d.mm) PGR(int64_t, 1, true, true) else PGR(int64_t, 1, false, true)
    } else {
      PGRV(int64_t)
    }
  } else {
    PGRV(int32_t)
  }
#undef PGRV
#undef PGR
#undef PGR1
  return hipGetLastError() == hipSuccess;
}

void PartGroupScratch(int64_t n, int64_t range, int nv, bool mm, int vphys, size_t *hist_bytes, size_t *start_bytes,
                      size_t *rows_bytes, size_t *scan_bytes) {
  const int shift = PartGroupShift(nv, mm);
  const int np = (int)std::max<int64_t>(1, (range + (1 << shift) - 1) >> shift);
  const int grid = NumCUs() * (kScatterThreads == 512 ? 2 : 1);
  const int vb = vphys == P_I64 ? 8 : 4;
  *hist_bytes = (size_t)np * grid * 4 * 2;  // counts and their scan
  *start_bytes = (size_t)(np + 1) * 4;
  *rows_bytes = PadUp((size_t)n * 2) + (size_t)std::max(nv, 0) * PadUp((size_t)n * vb);
  size_t tmp = 0;
  unsigned int *dummy = nullptr;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, dummy, dummy, np * grid, (hipStream_t)0);
  *scan_bytes = tmp ? tmp : 16;
}

}  // namespace dev
}  // namespace mbx
