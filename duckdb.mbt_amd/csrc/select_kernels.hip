// select_kernels.hip — one-pass, order-preserving filter -> compaction
// (SELECT <cols> FROM t WHERE <range conjunction>) for gfx950.
//
// Why one pass: the two-pass form (kernels.hip: filter_bits_lds -> scan ->
// compact_lds) reads every predicate column twice when the predicate column
// is also an output (SELECT x FROM t WHERE x > 24: 16 GB read + 4.2 GB
// written per 1e9 rows).  select_rounds (below) reads each needed column from
// HBM once and places every workgroup's rows by a round-synchronous prefix.
// The count-first two-pass form (filter_count_lds -> scan ->
// compact_recomp_lds, at the end of this file) serves small inputs.
#include <hip/hip_runtime.h>

#include <atomic>
#include <climits>
#include <stdexcept>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "device.h"
#include "types.h"
#include "knobs.h"

namespace mbx {
namespace dev {

// hipFuncAttributeMaxDynamicSharedMemorySize once per (kernel, device): the
// attribute belongs to a device, and the shard workers of one process launch
// on several devices at once (a per-process flag would skip devices and race)
static void EnsureMaxLds(const void *fn, std::atomic<uint64_t> &done, int bytes) {
  int d = 0;
  (void)hipGetDevice(&d);
  const uint64_t bit = 1ull << (d & 63);
  if (done.load(std::memory_order_acquire) & bit) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done.fetch_or(bit, std::memory_order_acq_rel);
}

namespace {

typedef long long sl_v2i64 __attribute__((ext_vector_type(2)));
typedef int sl_v4i32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int64_t sl_wave_sum(int64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// 4 consecutive values (rows 4 lane .. 4 lane + 3 of a step) of a 4- or
// 8-byte column slice held in LDS, widened to int64 (sign-extended for 4 B).
__device__ __forceinline__ void sl_read4(const unsigned char *slice, int w, int lane, int64_t v[4]) {
  if (w == 8) {
    const sl_v2i64 a = *(const sl_v2i64 *)(slice + lane * 32), b = *(const sl_v2i64 *)(slice + lane * 32 + 16);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
  } else {
    const sl_v4i32 a = *(const sl_v4i32 *)(slice + lane * 16);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
}

// a value every lane holds alike (read from LDS), moved to an SGPR so that the
// branches on it stay scalar
__device__ __forceinline__ int64_t sl_uni(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)((uint64_t)hi << 32 | lo);
}

}  // namespace

// ---------------------------------------------------------------------------
// Round-synchronous one-pass compaction (select_rounds; see device.h).
//
// One persistent workgroup per CU (G of them), 9 waves with fixed roles:
//  * waves 0-3, loaders: stream their steps of every loaded column through an
//    LDS-DMA ring (as filter_agg_lds does), evaluate the predicates and write
//    each selected value straight into the wave's staging ring in LDS (its
//    rank from the ballots).  Tile t = r G + g of round r is 4 S consecutive
//    steps (loader w owns steps [4 S t + w S, 4 S t + (w + 1) S)).  At the end
//    of a round the last loader to arrive (an LDS atomic) publishes the
//    workgroup's round count as one 8-byte {count, epoch} granule with an sc1
//    store: data and flag in one word, no ordering needed.
//  * wave 8, coordinator: polls the G granules of the oldest unresolved
//    rounds (sc1 loads, SR_PW rounds per poll); once a round is complete it
//    knows the round's total and the workgroup's exclusive prefix, so the
//    tile's output position is running + prefix.  It hands that to the
//    storers through LDS.  No look-back chains: every coordinator reads every
//    round's G counts once (2 KB), and nothing waits on a ticket.
//  * waves 4-7, storers: storer s moves loader s's staged values of the round
//    to base + Σ counts of loaders < s with contiguous 8/4-byte stores, then
//    frees the staging rows.  Stores never share a vmcnt queue with the DMA.
// Loaders run ahead of the storers by as many rounds as the staging rings
// and the SR_MR meta slots allow, which hides the poll latency.
// Progress: the workgroup at the lowest round only waits for rounds every
// other workgroup has already published, provided all G workgroups are
// resident (G = #CUs, LDS padded past half a CU, so one per CU).  Should a
// workgroup never be scheduled, a coordinator that sees no progress for
// SR_TIMEOUT gives up: it writes the launch's epoch into the abort word, every
// wave leaves its loop (loaders drain their DMA first), and the host falls
// back to the two-pass form.
// ---------------------------------------------------------------------------
namespace {
constexpr int SR_MR = 32;                    // rounds in flight inside a workgroup (meta slots)
// staged validity of a NULL-able output: one 0/1 byte per staged row (16-bit
// entries measured no faster for SELECT vn ... WHERE x > 24, 4.06 ms either
// way, and their larger rows halved the staging ring of three-column shapes:
// SELECT vn ... WHERE xn > 24 AND k < 16 4.83 -> 5.45 ms)
typedef uint8_t sr_vb_t;
constexpr int SR_VB = sizeof(sr_vb_t);
constexpr int SR_PW = 4;                     // most rounds polled per coordinator poll (runtime: pwmax)
constexpr long long SR_TIMEOUT = 10000000;   // s_memrealtime ticks (100 MHz): 100 ms without progress
struct SrShared {
  unsigned long long arr[SR_MR];  // (count << 16) + arrivals of the round's loaders
  uint32_t cnt[SR_MR][8];         // each loader's count of the round
  long long base[SR_MR];          // output row of the workgroup's tile of the round
  uint32_t btag[SR_MR];           // round + 1 once base is set
  uint32_t tail[8];               // staging rows freed, per loader (monotonic)
  uint32_t sdone[8];              // rounds finished, per storer
  uint32_t abort_;
  unsigned long long pubt[SR_MR];  // MBX_SR_DEBUG: clock64 when the round's granule was published
};
// Control words in LDS are read and written with inline-asm ds_* ops: the
// compiler puts an s_waitcnt vmcnt(0) in front of every atomic or volatile LDS
// access once LDS-DMA is in flight (it cannot prove they do not alias the DMA
// targets), which would drain a loader's whole ring at every check.  Each op
// waits for itself (lgkmcnt(0)), so program order is LDS order.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
// (reads return the value as a wave-uniform scalar: every control word is
// uniform, and a VGPR result would make the branches on it divergent)
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ long long lds_ld(const long long *p) {
  long long v;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return sl_uni(v);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st(long long *p, long long v) {
  asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st(unsigned long long *p, unsigned long long v) {
  asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
// a control-word store whose completion nobody in this wave waits for (the
// wave's later LDS ops stay in order behind it; the reader polls)
__device__ __forceinline__ void lds_st_nw(uint32_t *p, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
template <int N>
__device__ __forceinline__ void sr_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ unsigned long long lds_add_rtn(unsigned long long *p, unsigned long long v) {
  unsigned long long old;
  asm volatile("ds_add_rtn_u64 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(lds_addr(p)), "v"(v) : "memory");
  return old;
}
}  // namespace

// A storer's copy of staged rows t0w .. t0w + c - 1 (ring positions & mask) to
// dst[0 .. c): 4 rows per lane per pass, so the 4 staging reads share one LDS
// wait.
// a storer's output store: non-temporal (the rows are written once and not
// read back by this kernel; plain stores measured the same time and the same
// WRITE_SIZE, profiles/r04_shapes_store_flavour_ab.log)
template <typename T>
__device__ __forceinline__ void sr_store(T v, T *p) {
  __builtin_nontemporal_store(v, p);
}

template <typename TS, typename TD>
__device__ __forceinline__ void sr_copy(const TS *st, uint32_t t0w, uint32_t mask, uint32_t c, int lane, TD *dst) {
  uint32_t i = lane;
  // whole 4-row groups only: with one 256-row step per round (8 loaders,
  // S = 1) a loader's range is ~130 rows, and guarded 4-row passes over such
  // ranges measured slower than the one-row loop (SELECT v ... WHERE xn > 24
  // 3.70 vs 3.57 ms, profiles/r04_storer_copy_ab.log)
  for (; i + 192 < c; i += 256) {
    TS x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = st[(t0w + i + 64 * u) & mask];
#pragma unroll
    for (int u = 0; u < 4; u++) sr_store((TD)x[u], dst + i + 64 * u);
  }
  for (; i < c; i += 64) sr_store((TD)st[(t0w + i) & mask], dst + i);
}

// A storer's copy of a sentinel-staged NULL-able output (SelectDesc::col
// vsent): the value (0 under NULL), its validity byte, and with Z the zone map
// of the valid rows.
template <typename TS, typename TD, bool Z>
__device__ __forceinline__ void sr_copy_sent(const TS *st, uint32_t t0w, uint32_t mask, uint32_t c, int lane, TD *dst,
                                             uint8_t *vd, TS sent, long long &mn, long long &mx, uint32_t &nv) {
  uint32_t b = 0;
  // whole passes of 256 rows, 4 per lane (rows b + lane + 64 u): the 4 staging
  // reads share one LDS wait.  The validity of the pass comes back as 4 ballots
  // (bit l of ballot u = row b + 64 u + l), from which lane l writes the bytes
  // of rows b + 4 l .. b + 4 l + 3 as one 4-byte store (nibble -> bytes by one
  // multiply), so a pass stores its 256 validity bytes with one instruction
  // instead of four (which measured the same).  The rows after
  // the last whole pass take the one-row loop: guarded partial passes measured
  // slower on ~130-row ranges (SELECT vn ... WHERE x > 24 4.81 vs 4.06 ms,
  // profiles/r04_storer_copy_ab.log)
  for (; b + 256 <= c; b += 256) {
    TS x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) x[u] = st[(t0w + b + lane + 64 * u) & mask];
    unsigned long long bal[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const bool ok = x[u] != sent;
      sr_store((TD)(ok ? x[u] : (TS)0), dst + b + lane + 64 * u);
      bal[u] = __ballot(ok);
      if constexpr (Z) {
        mn = ok && (long long)x[u] < mn ? (long long)x[u] : mn;
        mx = ok && (long long)x[u] > mx ? (long long)x[u] : mx;
        nv += ok;
      }
    }
    {
      // vd = D.vdst[o] + pos with pos any prefix count, so this dword store is
      // generally not 4-byte aligned: it relies on the unaligned global access
      // mode the ROCm runtime configures for gfx9 (SH_MEM_CONFIG alignment_mode
      // UNALIGNED, ROCm's default)
      const int q = lane >> 4;
      const unsigned long long bw = q == 0 ? bal[0] : q == 1 ? bal[1] : q == 2 ? bal[2] : bal[3];
      const uint32_t nib = (uint32_t)(bw >> ((4 * lane) & 63)) & 0xFu;
      sr_store((nib * 0x00204081u) & 0x01010101u, (uint32_t *)(vd + b + 4 * lane));
    }
  }
  for (uint32_t i = b + lane; i < c; i += 64) {
    const TS x = st[(t0w + i) & mask];
    const bool ok = x != sent;
    sr_store((TD)(ok ? x : (TS)0), dst + i);
    sr_store((uint8_t)ok, vd + i);
    if constexpr (Z) {
      mn = ok && (long long)x < mn ? (long long)x : mn;
      mx = ok && (long long)x > mx ? (long long)x : mx;
      nv += ok;
    }
  }
}

// A storer's copy of its two loaders' ranges of a round as one stream (8
// loaders, one sentinel-staged NULL-able output): rows i < cA come from loader A's staging and go to
// dA + i, the rest from B's to dB + i - cA.  4 rows per lane per pass over the
// joined ranges, so the ~2 x 130 rows of a one-step round take 2 LDS waits
// instead of 6 (each range's last pass was mostly empty).  SENT: a
// sentinel-staged NULL-able output (0 and a validity byte of 0 under NULL).
template <typename TS, typename TD, bool SENT>
__device__ __forceinline__ void sr_copy2(const TS *stA, uint32_t tA, TD *dA, uint8_t *vA, uint32_t cA, const TS *stB,
                                         uint32_t tB, TD *dB, uint8_t *vB, uint32_t cB, uint32_t mask, int lane, TS sent) {
  const uint32_t c = cA + cB;
  for (uint32_t i = lane; i < c; i += 256) {
    TS x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {  // one LDS read per row (reads past c stay inside the staging ring, unused)
      const uint32_t r = i + 64 * u;
      const TS *p = r < cA ? stA + ((tA + r) & mask) : stB + ((tB + r - cA) & mask);
      x[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t r = i + 64 * u;
      if (r < c) {
        const bool a = r < cA;
        TD *d = a ? dA + r : dB + (r - cA);
        if constexpr (SENT) {
          const bool ok = x[u] != sent;
          __builtin_nontemporal_store((TD)(ok ? x[u] : (TS)0), d);
          __builtin_nontemporal_store((uint8_t)ok, a ? vA + r : vB + (r - cA));
        } else {
          __builtin_nontemporal_store((TD)x[u], d);
        }
      }
    }
  }
}

// NC loaded columns; bit c of WM: column c is 8 bytes wide (else 4).
template <int NC, int WM>
struct SrCols {
  static constexpr int w(int c) { return (WM >> c) & 1 ? 8 : 4; }
  static constexpr int off(int c) { return c == 0 ? 0 : off(c - 1) + w(c - 1) * 256; }
  static constexpr int ni() { return off(NC) / 1024; }
};

// Staging: every loaded column that feeds an output (bit c of D's staged mask)
// has an array of stg + 64 entries per loader (the 64 extra are each lane's
// dump slot for unselected rows, so the writes need no exec masking).
// A step is H x 256 consecutive rows (sub-step h = rows 256 h .. 256 h + 255
// of it); a loader handles its H sub-steps in one pass, so their dependency
// chains interleave (one loader wave per SIMD cannot hide its own latencies).
// NL loader waves (4 or 8: two per SIMD hide each other's latencies), 4
// storers (storer s drains loaders s, s + 4, ...) and one coordinator.
// VAL: some columns carry validity words.  A sub-step's 32 B of words per
// NULL-able column ride a second ring (one exec-masked LDS-DMA instruction
// each, counted exactly in the wait); a NULL fails a predicate, and a NULL-able
// output stages one validity byte per selected row, which its storer writes to
// D.vdst (PackValidityBytes turns those into the output's bitmap).  Three
// storer-side bitmap builders (a ballot per 64 rows; one word per lane from
// the staged bytes; bits ORed into an LDS ring by the loaders) measured 5.5-6.5
// ms against 4.25 + 0.14-0.22 ms for this form on `SELECT vn ... WHERE x > 24`
// at 1e9 rows: the storers of this shape are nearly as busy as the loaders.
template <int NC, int WM, int DEPTH, int H, int NL, bool VAL, int NS = 4>
__global__ __launch_bounds__((NL + NS + 1) * 64) void select_rounds_kernel(SelectDesc D, int64_t n, int64_t nrounds, int S, int stg,
                                                            unsigned long long *ctl, uint32_t epoch, int sleep_,
                                                            int test_stall, int pwmax) {
  typedef SrCols<NC, WM> L;
  extern __shared__ __attribute__((aligned(16))) unsigned char sr_lds[];
  __shared__ SrShared sm;
  constexpr int SB1 = L::off(NC);  // one 256-row sub-step of every loaded column
  constexpr int SB = H * SB1;       // a ring slot: one step
  constexpr int NI = H * L::ni();   // LDS-DMA instructions per step
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int G = gridDim.x, g = blockIdx.x;
  const int64_t nsteps = n / (256 * H);
  unsigned long long *gran = ctl + 8;  // ctl[0]: abort word, ctl[1]: total, granules from ctl[8]
  {
    uint32_t *z = (uint32_t *)&sm;
    for (int i = threadIdx.x; i < (int)(sizeof(SrShared) / 4); i += blockDim.x) z[i] = 0;
  }
  // staged columns: the byte offset of column c's array in a loader's staging
  // area, and its staged width (4 for an 8-byte column the zone map proves
  // fits int32: half the LDS per staged row; the storer sign-extends)
  int soff[NC];
  bool st8[NC];
  uint32_t smask = 0;
  int rowb = 0;
  for (int o = 0; o < D.nout; o++) smask |= 1u << D.out_col[o];
#pragma unroll
  for (int c = 0; c < NC; c++) {
    soff[c] = rowb * (stg + 64);
    st8[c] = L::w(c) == 8 && !D.col[c].narrow;
    if ((smask >> c) & 1) rowb += st8[c] ? 8 : 4;
  }
  // NULL-able columns: slot offset of their words in the validity ring, and
  // (staged outputs) the byte offset of their staged validity bytes (0/1, one
  // per staged row, indexed like the staged values)
  int voff[NC], vsoff[NC];
  bool hv[NC];
  int nv = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    hv[c] = VAL && D.col[c].valid != nullptr;
    voff[c] = 32 * nv;
    nv += hv[c];
    vsoff[c] = rowb * (stg + 64);
    if (hv[c] && ((smask >> c) & 1) && !D.col[c].vsent) rowb += SR_VB;
  }
  constexpr int VSB = VAL ? H * NC * 32 : 0;  // validity ring slot: 4 words per sub-step and NULL-able column
  unsigned char *stage0 = sr_lds + (size_t)NL * DEPTH * SB + (size_t)NL * DEPTH * VSB;
  const uint32_t mask = (uint32_t)stg - 1;
  const uint64_t lt = (1ull << lane) - 1;
  __syncthreads();  // the only barrier: the roles diverge below

  if (w < NL) {
    // ------------------------------------------------------------ loader
    if (nrounds == 0) return;
    unsigned char *ring = sr_lds + (size_t)w * DEPTH * SB;
    unsigned char *vring = sr_lds + (size_t)NL * DEPTH * SB + (size_t)w * DEPTH * VSB;
    unsigned char *mystage = stage0 + (size_t)w * (stg + 64) * rowb;
    const int64_t qstride = (int64_t)G * NL * S;  // steps between a wave's tiles of consecutive rounds
    const unsigned char *colp[NC];
    int64_t lo[NC];
    uint64_t span[NC];
    uint32_t pmask = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      colp[c] = (const unsigned char *)D.col[c].data + lane * 16;
      lo[c] = D.col[c].lo;
      span[c] = D.col[c].span;
      pmask |= (D.col[c].is_pred ? 1u : 0u) << c;
    }
    int64_t iq = ((int64_t)g * NL + w) * S, ir = 0;  // the next step to issue: round ir, step iq
    int is = 0;
    auto issue = [&](int slot) {  // dead steps re-load step 0: a fixed count per slot
      const int64_t q = ir < nrounds && iq + is < nsteps ? iq + is : 0;
      if (++is == S) {
        is = 0;
        ir++;
        iq += qstride;
      }
#pragma unroll
      for (int h = 0; h < H; h++) {
        unsigned char *dst = ring + slot * SB + h * SB1;
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const unsigned char *src = colp[c] + (q * H + h) * (L::w(c) * 256);
          __builtin_amdgcn_global_load_lds((const void *)src, (void *)(dst + L::off(c)), 16, 0, 2);
          if (L::w(c) == 8)
            __builtin_amdgcn_global_load_lds((const void *)(src + 1024), (void *)(dst + L::off(c) + 1024), 16, 0, 2);
        }
      }
      if constexpr (VAL) {
#pragma unroll
        for (int h = 0; h < H; h++)
#pragma unroll
          for (int c = 0; c < NC; c++)
            if (hv[c] && lane < 2)
              __builtin_amdgcn_global_load_lds((const void *)(D.col[c].valid + (q * H + h) * 4 + lane * 2),
                                               (void *)(vring + slot * VSB + h * NC * 32 + voff[c]), 16, 0, 2);
      }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; d++) issue(d);
    int k = 0;
    uint32_t head = 0, tail_seen = 0;
    bool quit = false;
    // MBX_SR_DEBUG (D.dbg): cycles in total, waiting on the DMA, on staging room, on meta slots
    const bool dbg = D.dbg != nullptr;
    unsigned long long t_all = dbg ? clock64() : 0, d_dma = 0, d_stg = 0, d_meta = 0, t0 = 0;
    int64_t qb = ((int64_t)g * NL + w) * S;  // this round's first step
    // zone map of the selected rows of the D.zmask output columns (CREATE
    // TABLE AS keeps it as the new column's statistics), NULL rows skipped:
    // folded from the values already in registers (4-byte columns in 32-bit
    // ops); the non-NULL count only for NULL-able columns (otherwise it is the
    // selected count)
    const uint32_t zmask = NL == 8 && D.zstats && !D.zstore ? (uint32_t)D.zmask & smask : 0u;  // (4 loaders: the storers fold it)
    long long zmn[NC], zmx[NC];
    int zmn4[NC], zmx4[NC];
    uint32_t zcnt[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) zmn[c] = LLONG_MAX, zmx[c] = LLONG_MIN, zmn4[c] = INT_MAX, zmx4[c] = INT_MIN, zcnt[c] = 0;
    for (int64_t r = 0; r < nrounds && !quit; r++, qb += qstride) {
      const int slot = (int)(r % SR_MR);
      if (r >= SR_MR) {  // meta slot reuse: every storer is done with round r - SR_MR
        const uint32_t need = (uint32_t)(r - SR_MR + 1);
        if (dbg) t0 = clock64();
        while (true) {
          uint32_t m = lds_ld(&sm.sdone[0]);
#pragma unroll
          for (int q = 1; q < NS; q++) m = min(m, lds_ld(&sm.sdone[q]));
          if (__builtin_amdgcn_readfirstlane(m) >= need) break;
          if (lds_ld(&sm.abort_)) { quit = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (dbg) d_meta += clock64() - t0;
        if (quit) break;
      }
      const int64_t live_steps = nsteps - qb;  // steps s < live_steps hold data
      uint32_t rc = 0;
      for (int s = 0; s < S; s++) {
        if (dbg) t0 = clock64();
        if constexpr (VAL) {
          switch (nv) {  // wave-uniform: the exact count of the instructions issued after this slot's
            case 1: sr_wait<(NI + H) * (DEPTH - 1)>(); break;
            case 2: sr_wait<(NI + 2 * H) * (DEPTH - 1)>(); break;
            case 3: sr_wait<(NI + 3 * H) * (DEPTH - 1)>(); break;
            default: sr_wait<(NI + 4 * H) * (DEPTH - 1)>(); break;
          }
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
        }
        if (dbg) d_dma += clock64() - t0;
        const unsigned char *src = ring + k * SB;
        int64_t v[H][NC][4];
#pragma unroll
        for (int h = 0; h < H; h++)
#pragma unroll
          for (int c = 0; c < NC; c++) sl_read4(src + h * SB1 + L::off(c), L::w(c), lane, v[h][c]);
        // validity of rows 256 h + 4 lane .. + 3 per column (bit e), all valid without words
        uint32_t vmc[H][NC];
#pragma unroll
        for (int h = 0; h < H; h++)
#pragma unroll
          for (int c = 0; c < NC; c++) {
            vmc[h][c] = 0xFu;
            if constexpr (VAL) {
              if (hv[c])
                vmc[h][c] = (uint32_t)(*(const uint64_t *)(vring + k * VSB + h * NC * 32 + voff[c] + (lane >> 4) * 8) >>
                                       (4 * (lane & 15))) &
                            0xFu;
            }
          }
        // ok[h][e]: row 256 h + 4 lane + e passes (kept as lane masks: each ballot is the compare's own mask)
        const bool live = s < live_steps;
        bool ok[H][4];
#pragma unroll
        for (int h = 0; h < H; h++)
#pragma unroll
          for (int e = 0; e < 4; e++) ok[h][e] = live;
#pragma unroll
        for (int c = 0; c < NC; c++) {
          if (NC > 1 && !((pmask >> c) & 1)) continue;  // a lone column is the predicate column
#pragma unroll
          for (int h = 0; h < H; h++)
#pragma unroll
            for (int e = 0; e < 4; e++) ok[h][e] = ok[h][e] & ((uint64_t)(v[h][c][e]) - (uint64_t)(lo[c]) <= span[c]);
          if constexpr (VAL) {  // a NULL fails the predicate
#pragma unroll
            for (int h = 0; h < H; h++)
#pragma unroll
              for (int e = 0; e < 4; e++) ok[h][e] = ok[h][e] & (((vmc[h][c] >> e) & 1u) != 0);
          }
        }
        unsigned long long b[H][4];
        uint32_t hc[H];  // selected rows per sub-step
        uint32_t cnt = 0;
#pragma unroll
        for (int h = 0; h < H; h++) {
          hc[h] = 0;
#pragma unroll
          for (int e = 0; e < 4; e++) {
            b[h][e] = __ballot(ok[h][e]);
            hc[h] += (uint32_t)__popcll(b[h][e]);
          }
          cnt += hc[h];
        }
        if (cnt) {
          if (head + 256u * H - tail_seen > (uint32_t)stg) {  // staging full: wait for the storer
            if (dbg) t0 = clock64();
            while (true) {
              tail_seen = lds_ld(&sm.tail[w]);
              if (head + 256u * H - tail_seen <= (uint32_t)stg) break;
              if (lds_ld(&sm.abort_)) { quit = true; break; }
              __builtin_amdgcn_s_sleep(1);
            }
            if (dbg) d_stg += clock64() - t0;
            if (quit) break;
          }
          uint32_t hb = head;
#pragma unroll
          for (int h = 0; h < H; h++) {
            // rank of row (h, lane, e): earlier sub-steps, selected rows of lower lanes (mbcnt),
            // then this lane's earlier rows
            uint32_t rk = hb;
#pragma unroll
            for (int e = 0; e < 4; e++)
              rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(b[h][e] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b[h][e], rk));
            uint32_t idx[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
              idx[e] = ok[h][e] ? (rk & mask) : (uint32_t)stg + lane;
              rk += ok[h][e];
            }
#pragma unroll
            for (int c = 0; c < NC; c++) {
              if (!((smask >> c) & 1)) continue;
              unsigned char *st = mystage + soff[c];
              int64_t sv[4];  // the staged values: a NULL row of a sentinel-staged column as D.col[c].sent
#pragma unroll
              for (int e = 0; e < 4; e++) {
                sv[e] = v[h][c][e];
                if constexpr (VAL) {
                  if (hv[c] && D.col[c].vsent) sv[e] = ((vmc[h][c] >> e) & 1u) ? sv[e] : D.col[c].sent;
                }
              }
              if (st8[c]) {
#pragma unroll
                for (int e = 0; e < 4; e++) ((int64_t *)st)[idx[e]] = sv[e];
              } else {
#pragma unroll
                for (int e = 0; e < 4; e++) ((int32_t *)st)[idx[e]] = (int32_t)sv[e];
              }
              if constexpr (VAL) {
                if (hv[c] && !D.col[c].vsent) {  // one 0/1 byte per staged row (unselected rows: the dump slot)
                  sr_vb_t *vb = (sr_vb_t *)(mystage + vsoff[c]);
#pragma unroll
                  for (int e = 0; e < 4; e++) vb[idx[e]] = (sr_vb_t)((vmc[h][c] >> e) & 1u);
                }
              }
              if ((zmask >> c) & 1) {
#pragma unroll
                for (int e = 0; e < 4; e++) {
                  const bool z = ok[h][e] && ((vmc[h][c] >> e) & 1u);
                  if (L::w(c) == 4) {
                    const int x = (int)v[h][c][e];
                    zmn4[c] = min(zmn4[c], z ? x : INT_MAX);
                    zmx4[c] = max(zmx4[c], z ? x : INT_MIN);
                  } else {
                    const long long x = v[h][c][e];
                    zmn[c] = z && x < zmn[c] ? x : zmn[c];
                    zmx[c] = z && x > zmx[c] ? x : zmx[c];
                  }
                  if (hv[c]) zcnt[c] += z;
                }
              }
            }
            hb += hc[h];
          }
          head = __builtin_amdgcn_readfirstlane(head + cnt);  // wave-uniform: keeps the room check scalar
          rc += cnt;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read (and staging written) before the DMA reuses it
        issue(k);
        k = k + 1 == DEPTH ? 0 : k + 1;
      }
      if (quit) break;
      if (lane == 0) {
        lds_st(&sm.cnt[slot][w], rc);
        const unsigned long long old =
            (unsigned long long)sl_uni((int64_t)lds_add_rtn(&sm.arr[slot], ((unsigned long long)rc << 16) + 1));
        if ((old & 0xffff) == NL - 1 && g != test_stall) {  // the last loader of the round publishes the workgroup's count
          lds_st(&sm.arr[slot], 0ull);
          const unsigned long long tot = (old >> 16) + rc;
          __hip_atomic_store(&gran[r * G + g], ((unsigned long long)epoch << 32) | tot, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          if (dbg) {
            lds_st(&sm.pubt[slot], (unsigned long long)clock64());
            if (D.dbg_ts) D.dbg_ts[r * G + g] = __builtin_amdgcn_s_memrealtime();  // MBX_SR_DEBUG=2: publish times
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
    if (zmask) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (!((zmask >> c) & 1)) continue;
        long long a = L::w(c) == 4 ? (long long)zmn4[c] : zmn[c], b = L::w(c) == 4 ? (long long)zmx4[c] : zmx[c];
        uint32_t n = zcnt[c];
#pragma unroll
        for (int off = 32; off; off >>= 1) {
          const long long a2 = __shfl_xor(a, off), b2 = __shfl_xor(b, off);
          a = a2 < a ? a2 : a;
          b = b2 > b ? b2 : b;
          n += __shfl_xor(n, off);
        }
        if (lane == 0) {
          atomicMin(&D.zstats[3 * c], a);
          atomicMax(&D.zstats[3 * c + 1], b);
          atomicAdd((unsigned long long *)&D.zstats[3 * c + 2], (unsigned long long)n);
        }
      }
    }
    if (dbg && lane == 0) {
      atomicAdd(&D.dbg[0], clock64() - t_all);
      atomicAdd(&D.dbg[1], d_dma);
      atomicAdd(&D.dbg[2], d_stg);
      atomicAdd(&D.dbg[3], d_meta);
    }
    return;
  }
  if (w < NL + NS) {
    // ------------------------------------------------------------ storer
    const int sw = w - NL;
    constexpr int PER = NL / NS;  // loaders per storer: sw, sw + NS, ...
    uint32_t tail[PER];
#pragma unroll
    for (int j = 0; j < PER; j++) tail[j] = 0;
    const bool dbg = D.dbg != nullptr;
    unsigned long long t_all = dbg ? clock64() : 0, d_wait = 0, d_copy = 0, t0 = 0, t1 = 0;
    // Output stores are non-temporal: the rows are written once and not read
    // back by this kernel (sel 2.055 -> 2.025 ms, SELECT k, v 4.61 -> 4.44,
    // SELECT v 3.40 -> 3.30 at 1e9 rows).
    // D.zstore: the zone map of the D.zmask columns is folded here, per
    // output, from the values the copy loads anyway (else by the loaders)
    // (8 loaders: the loaders fold it, so the storer's copy of the map is not
    // compiled -- its registers pushed the NULL-able 8-loader instances past
    // 128 VGPRs into scratch)
    const uint32_t zsmask = NL == 4 && D.zstats && D.zstore ? (uint32_t)D.zmask & smask : 0u;
    static_assert(NL % NS == 0, "every storer drains the same number of loaders");
    long long zmn[SL_MAX_OUT], zmx[SL_MAX_OUT];
    uint32_t zcnt[SL_MAX_OUT];
#pragma unroll
    for (int o = 0; o < SL_MAX_OUT; o++) zmn[o] = LLONG_MAX, zmx[o] = LLONG_MIN, zcnt[o] = 0;
    for (int64_t r = 0; r < nrounds; r++) {
      const int slot = (int)(r % SR_MR);
      bool quit = false;
      if (dbg) t0 = clock64();
      while (lds_ld(&sm.btag[slot]) != (uint32_t)(r + 1)) {
        if (lds_ld(&sm.abort_)) { quit = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (dbg) d_wait += clock64() - t0;
      if (quit) break;
      int64_t pos = lds_ld(&sm.base[slot]);
      // the round's loader counts in one LDS read (lane q: loader q's count),
      // the prefix taken by readlanes: one LDS round trip per round instead of
      // one per earlier loader (up to 8 waited reads for storer 3's second loader)
      uint32_t cl;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(cl) : "v"(lds_addr(&sm.cnt[slot][lane & 7])) : "memory");
      if (dbg) t1 = clock64();
      int q = 0;
      // 8 loaders, one output without staged validity bytes: both loaders'
      // ranges in one stream (sr_copy2)
      bool merged = false;
      if constexpr (PER == 2) {
        const int oc = D.out_col[0];
        bool vs = false, vbyte = false;
        if constexpr (VAL) {
          vs = D.vdst[0] && D.col[oc].vsent;
          vbyte = D.vdst[0] && !D.col[oc].vsent;
        }
        // (sentinel-staged NULL-able outputs only: SELECT vn ... WHERE x > 24 3.91 -> 3.62 ms, but the
        // NULL-free SELECT v ... WHERE x > 24 3.27 -> 3.46, profiles/r04_storer_merged_ab.log)
        if (D.nout == 1 && vs && !vbyte && !((zsmask >> oc) & 1)) {
          merged = true;
          const int lA = sw, lB = sw + NS;
          int64_t pA = pos, pB;
          for (int qq = 0; qq < lA; qq++) pA += (uint32_t)__builtin_amdgcn_readlane((int)cl, qq);
          pB = pA;
          for (int qq = lA; qq < lB; qq++) pB += (uint32_t)__builtin_amdgcn_readlane((int)cl, qq);
          const uint32_t cA = (uint32_t)__builtin_amdgcn_readlane((int)cl, lA);
          const uint32_t cB = (uint32_t)__builtin_amdgcn_readlane((int)cl, lB);
          int so = 0;
          bool s8 = false;
#pragma unroll
          for (int cc = 0; cc < NC; cc++)
            if (cc == oc) so = soff[cc], s8 = st8[cc];
          const unsigned char *sA = stage0 + (size_t)lA * (stg + 64) * rowb + so;
          const unsigned char *sB = stage0 + (size_t)lB * (stg + 64) * rowb + so;
          uint8_t *vA = vs ? D.vdst[0] + pA : nullptr, *vB = vs ? D.vdst[0] + pB : nullptr;
          if (s8) {
            if (vs) sr_copy2<int64_t, int64_t, true>((const int64_t *)sA, tail[0], (int64_t *)D.dst[0] + pA, vA, cA, (const int64_t *)sB, tail[1], (int64_t *)D.dst[0] + pB, vB, cB, mask, lane, D.col[oc].sent);
            else sr_copy2<int64_t, int64_t, false>((const int64_t *)sA, tail[0], (int64_t *)D.dst[0] + pA, vA, cA, (const int64_t *)sB, tail[1], (int64_t *)D.dst[0] + pB, vB, cB, mask, lane, 0);
          } else if (D.col[oc].w == 8) {  // staged narrow: sign-extend back to int64
            if (vs) sr_copy2<int32_t, int64_t, true>((const int32_t *)sA, tail[0], (int64_t *)D.dst[0] + pA, vA, cA, (const int32_t *)sB, tail[1], (int64_t *)D.dst[0] + pB, vB, cB, mask, lane, (int32_t)D.col[oc].sent);
            else sr_copy2<int32_t, int64_t, false>((const int32_t *)sA, tail[0], (int64_t *)D.dst[0] + pA, vA, cA, (const int32_t *)sB, tail[1], (int64_t *)D.dst[0] + pB, vB, cB, mask, lane, 0);
          } else {
            if (vs) sr_copy2<int32_t, int32_t, true>((const int32_t *)sA, tail[0], (int32_t *)D.dst[0] + pA, vA, cA, (const int32_t *)sB, tail[1], (int32_t *)D.dst[0] + pB, vB, cB, mask, lane, (int32_t)D.col[oc].sent);
            else sr_copy2<int32_t, int32_t, false>((const int32_t *)sA, tail[0], (int32_t *)D.dst[0] + pA, vA, cA, (const int32_t *)sB, tail[1], (int32_t *)D.dst[0] + pB, vB, cB, mask, lane, 0);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read before it is freed
          tail[0] += cA;
          tail[1] += cB;
          if (lane == 0) {
            lds_st_nw(&sm.tail[lA], tail[0]);
            lds_st_nw(&sm.tail[lB], tail[1]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < PER && !merged; j++) {
        const int l = sw + NS * j;
        for (; q < l; q++) pos += (uint32_t)__builtin_amdgcn_readlane((int)cl, q);
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cl, l);
        const unsigned char *mystage = stage0 + (size_t)l * (stg + 64) * rowb;
#pragma unroll
        for (int o = 0; o < SL_MAX_OUT; o++) {
          if (o >= D.nout) break;
          const int oc = D.out_col[o];
          int so = 0, vo = 0;
          bool s8 = false;
#pragma unroll
          for (int cc = 0; cc < NC; cc++)
            if (cc == oc) so = soff[cc], s8 = st8[cc], vo = vsoff[cc];
          const sr_vb_t *vb = nullptr;
          bool vs = false;  // a sentinel-staged NULL-able output: validity from the staged values
          if constexpr (VAL) {
            vs = D.vdst[o] && D.col[oc].vsent;
            if (D.vdst[o] && !vs) vb = (const sr_vb_t *)(mystage + vo);
          }
          const uint32_t t0w = tail[j];
          if (vs) {
            const bool z = (zsmask >> oc) & 1;
            uint8_t *vd = D.vdst[o] + pos;
            if (s8) {
              const int64_t *st = (const int64_t *)(mystage + so);
              if (z) sr_copy_sent<int64_t, int64_t, true>(st, t0w, mask, c, lane, (int64_t *)D.dst[o] + pos, vd, D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
              else sr_copy_sent<int64_t, int64_t, false>(st, t0w, mask, c, lane, (int64_t *)D.dst[o] + pos, vd, D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
            } else if (D.col[oc].w == 8) {
              const int32_t *st = (const int32_t *)(mystage + so);
              if (z) sr_copy_sent<int32_t, int64_t, true>(st, t0w, mask, c, lane, (int64_t *)D.dst[o] + pos, vd, (int32_t)D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
              else sr_copy_sent<int32_t, int64_t, false>(st, t0w, mask, c, lane, (int64_t *)D.dst[o] + pos, vd, (int32_t)D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
            } else {
              const int32_t *st = (const int32_t *)(mystage + so);
              if (z) sr_copy_sent<int32_t, int32_t, true>(st, t0w, mask, c, lane, (int32_t *)D.dst[o] + pos, vd, (int32_t)D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
              else sr_copy_sent<int32_t, int32_t, false>(st, t0w, mask, c, lane, (int32_t *)D.dst[o] + pos, vd, (int32_t)D.col[oc].sent, zmn[o], zmx[o], zcnt[o]);
            }
          } else if ((zsmask >> oc) & 1) {  // the copy also folds the output's zone map (NULL rows skipped)
            long long mn = zmn[o], mx = zmx[o];
            uint32_t nv = 0;
            if (s8) {
              const int64_t *st = (const int64_t *)(mystage + so);
              int64_t *dst = (int64_t *)D.dst[o] + pos;
              for (uint32_t i = lane; i < c; i += 64) {
                const uint32_t k = (t0w + i) & mask;
                const long long x = st[k];
                __builtin_nontemporal_store((int64_t)x, dst + i);
                const bool ok = VAL ? (!vb || vb[k] != 0) : true;
                mn = ok && x < mn ? x : mn;
                mx = ok && x > mx ? x : mx;
                nv += ok;
              }
            } else {  // 4 bytes staged: an int32 column, or a narrow-staged int64 one
              const int32_t *st = (const int32_t *)(mystage + so);
              const bool w8 = D.col[oc].w == 8;
              for (uint32_t i = lane; i < c; i += 64) {
                const uint32_t k = (t0w + i) & mask;
                const int32_t x = st[k];
                if (w8) __builtin_nontemporal_store((int64_t)x, (int64_t *)D.dst[o] + pos + i);
                else __builtin_nontemporal_store(x, (int32_t *)D.dst[o] + pos + i);
                const bool ok = VAL ? (!vb || vb[k] != 0) : true;
                mn = ok && x < mn ? x : mn;
                mx = ok && x > mx ? x : mx;
                nv += ok;
              }
            }
            zmn[o] = mn, zmx[o] = mx, zcnt[o] += nv;
          } else if (s8) {
            sr_copy<int64_t, int64_t>((const int64_t *)(mystage + so), t0w, mask, c, lane, (int64_t *)D.dst[o] + pos);
          } else if (D.col[oc].w == 8) {  // staged narrow: sign-extend back to int64
            sr_copy<int32_t, int64_t>((const int32_t *)(mystage + so), t0w, mask, c, lane, (int64_t *)D.dst[o] + pos);
          } else {
            sr_copy<int32_t, int32_t>((const int32_t *)(mystage + so), t0w, mask, c, lane, (int32_t *)D.dst[o] + pos);
          }
          if constexpr (VAL) {
            if (vb) {
              uint8_t *vd = D.vdst[o] + pos;
              for (uint32_t i = lane; i < c; i += 64) sr_store((uint8_t)vb[(t0w + i) & mask], vd + i);
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read before it is freed
        tail[j] += c;
        if (lane == 0) lds_st_nw(&sm.tail[l], tail[j]);
      }
      if (dbg) d_copy += clock64() - t1;
      if (lane == 0) lds_st_nw(&sm.sdone[sw], (uint32_t)(r + 1));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last control stores land before the wave ends
    if (zsmask) {
#pragma unroll
      for (int o = 0; o < SL_MAX_OUT; o++) {
        if (o >= D.nout) break;
        const int oc = D.out_col[o];
        if (!((zsmask >> oc) & 1)) continue;
        long long a = zmn[o], b = zmx[o];
        uint32_t n = zcnt[o];
#pragma unroll
        for (int off = 32; off; off >>= 1) {
          const long long a2 = __shfl_xor(a, off), b2 = __shfl_xor(b, off);
          a = a2 < a ? a2 : a;
          b = b2 > b ? b2 : b;
          n += __shfl_xor(n, off);
        }
        if (lane == 0) {
          atomicMin(&D.zstats[3 * oc], a);
          atomicMax(&D.zstats[3 * oc + 1], b);
          atomicAdd((unsigned long long *)&D.zstats[3 * oc + 2], (unsigned long long)n);
        }
      }
    }
    if (dbg && lane == 0) {
      atomicAdd(&D.dbg[4], clock64() - t_all);
      atomicAdd(&D.dbg[5], d_wait);
      atomicAdd(&D.dbg[13], d_copy);
    }
    return;
  }
  // -------------------------------------------------------------- coordinator
  int64_t running = 0, r0 = 0;
  long long last = (long long)__builtin_amdgcn_s_memrealtime();
  bool aborted = false;
  // MBX_SR_DEBUG: total cycles, polls, polls without progress, cycles in poll loads,
  // rounds resolved, most rounds in one poll, publish -> resolve cycles
  const bool dbg = D.dbg != nullptr;
  unsigned long long t_all = dbg ? clock64() : 0, c_polls = 0, c_fail = 0, c_load = 0, c_res = 0, c_max = 0, c_lag = 0,
                     t0 = 0;
  while (r0 < nrounds) {
    if (__hip_atomic_load(&ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned long long)epoch) {
      aborted = true;  // another workgroup gave up
      break;
    }
    const int pw = (int)(nrounds - r0 < pwmax ? nrounds - r0 : pwmax);
    if (dbg) t0 = clock64();
    unsigned long long x[SR_PW][4];
#pragma unroll
    for (int i = 0; i < SR_PW; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int idx = 4 * lane + j;
        x[i][j] = (i < pw && idx < G)
                      ? __hip_atomic_load(&gran[(r0 + i) * G + idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : ((unsigned long long)epoch << 32);
      }
    if (dbg) {
      unsigned long long acc = 0;
#pragma unroll
      for (int i = 0; i < SR_PW; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc ^= x[i][j];
      if (__ballot(acc == 0x5a5a5a5a5a5aull)) c_polls += 0;  // uses the loads: the clock below waits for them
      c_load += clock64() - t0;
      c_polls++;
    }
    int prog = 0;
#pragma unroll
    for (int i = 0; i < SR_PW; i++) {
      if (i >= pw) break;
      bool mine = true;
      int64_t sa = 0, sb = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        mine = mine && (uint32_t)(x[i][j] >> 32) == epoch;
        const int64_t c = (int64_t)(uint32_t)x[i][j];
        sa += c;
        if (4 * lane + j < g) sb += c;
      }
      if (__ballot(!mine)) break;  // the round is not complete yet
      sa = sl_wave_sum(sa);
      sb = sl_wave_sum(sb);
      if (lane == 0) {
        const int slot = (int)((r0 + i) % SR_MR);
        lds_st(&sm.base[slot], (long long)(running + sb));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lds_st(&sm.btag[slot], (uint32_t)(r0 + i + 1));
      }
      if (dbg) c_lag += clock64() - (unsigned long long)lds_ld((const long long *)&sm.pubt[(r0 + i) % SR_MR]);
      running += sa;
      prog++;
    }
    r0 += prog;
    if (dbg) {
      c_res += prog;
      c_max = c_max > (unsigned long long)prog ? c_max : (unsigned long long)prog;
      c_fail += prog == 0;
    }
    const long long now = (long long)__builtin_amdgcn_s_memrealtime();
    if (prog) {
      last = now;
    } else {
      if (now - last > SR_TIMEOUT) {
        if (lane == 0)
          __hip_atomic_store(&ctl[0], (unsigned long long)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        aborted = true;
        break;
      }
      for (int i = 0; i < sleep_; i++) __builtin_amdgcn_s_sleep(8);
    }
  }
  if (dbg && lane == 0) {
    atomicAdd(&D.dbg[6], clock64() - t_all);
    atomicAdd(&D.dbg[7], c_polls);
    atomicAdd(&D.dbg[8], c_fail);
    atomicAdd(&D.dbg[9], c_load);
    atomicAdd(&D.dbg[10], c_res);
    atomicMax(&D.dbg[11], c_max);
    atomicAdd(&D.dbg[12], c_lag);
  }
  if (aborted) {
    if (lane == 0) lds_st(&sm.abort_, 1u);
    return;
  }
  if (g != 0) return;
  // workgroup 0: the rows after the last full step (guarded loads, 256 per pass), and the total.
  // The zone map of the D.zmask outputs folds these rows too, whichever role
  // (loaders or storers) folded the full steps: the host takes the map as the
  // statistics of every selected row (DCol::zn = the total)
  const uint32_t tzm = D.zstats ? (uint32_t)D.zmask & smask : 0u;
  long long tmn[NC], tmx[NC];
  uint32_t tnv[NC];
#pragma unroll
  for (int c = 0; c < NC; c++) tmn[c] = LLONG_MAX, tmx[c] = LLONG_MIN, tnv[c] = 0;
  int64_t tcnt = 0;
  for (int64_t base = nsteps * 256 * H; base < n; base += 256) {
    bool ok[4];
    const int64_t i0 = base + 4 * lane;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t i = i0 + e;
      ok[e] = i < n;
      for (int c = 0; c < D.ncol && ok[e]; c++) {
        if (!D.col[c].is_pred) continue;
        const int64_t xv = D.col[c].w == 8 ? ((const int64_t *)D.col[c].data)[i]
                                           : (int64_t)((const int32_t *)D.col[c].data)[i];
        ok[e] = (uint64_t)(xv) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
        if (VAL && D.col[c].valid) ok[e] = ok[e] && ((D.col[c].valid[i >> 6] >> (i & 63)) & 1);
      }
    }
    unsigned long long bb[4];
#pragma unroll
    for (int e = 0; e < 4; e++) bb[e] = __ballot(ok[e]);
    int64_t pos = running + tcnt + __popcll(bb[0] & lt) + __popcll(bb[1] & lt) + __popcll(bb[2] & lt) +
                  __popcll(bb[3] & lt);
    for (int e = 0; e < 4; e++) {
      if (!ok[e]) continue;
      for (int o = 0; o < D.nout; o++) {
        const int c = D.out_col[o];
        if (D.col[c].w == 8) ((int64_t *)D.dst[o])[pos] = ((const int64_t *)D.col[c].data)[i0 + e];
        else ((int32_t *)D.dst[o])[pos] = ((const int32_t *)D.col[c].data)[i0 + e];
        if (VAL && D.vdst[o]) D.vdst[o][pos] = (uint8_t)((D.col[c].valid[(i0 + e) >> 6] >> ((i0 + e) & 63)) & 1);
      }
      pos++;
    }
    if (tzm) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (!((tzm >> c) & 1)) continue;
        for (int e = 0; e < 4; e++) {
          if (!ok[e]) continue;
          const int64_t i = i0 + e;
          const bool vz = !(VAL && D.col[c].valid) || ((D.col[c].valid[i >> 6] >> (i & 63)) & 1);
          if (!vz) continue;
          const long long x = D.col[c].w == 8 ? ((const int64_t *)D.col[c].data)[i]
                                              : (long long)((const int32_t *)D.col[c].data)[i];
          tmn[c] = x < tmn[c] ? x : tmn[c];
          tmx[c] = x > tmx[c] ? x : tmx[c];
          tnv[c]++;
        }
      }
    }
    tcnt += __popcll(bb[0]) + __popcll(bb[1]) + __popcll(bb[2]) + __popcll(bb[3]);
  }
  if (tzm) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      if (!((tzm >> c) & 1)) continue;
      long long a = tmn[c], b = tmx[c];
      uint32_t nz = tnv[c];
#pragma unroll
      for (int off = 32; off; off >>= 1) {
        const long long a2 = __shfl_xor(a, off), b2 = __shfl_xor(b, off);
        a = a2 < a ? a2 : a;
        b = b2 > b ? b2 : b;
        nz += __shfl_xor(nz, off);
      }
      if (lane == 0 && nz) {
        atomicMin(&D.zstats[3 * c], a);
        atomicMax(&D.zstats[3 * c + 1], b);
        atomicAdd((unsigned long long *)&D.zstats[3 * c + 2], (unsigned long long)nz);
      }
    }
  }
  if (lane == 0) ctl[1] = (unsigned long long)(running + tcnt);
}

static SelectRoundsPlan PlanSelectRoundsNL(const SelectDesc &d, int64_t nrows, int force_nl);
SelectRoundsPlan PlanSelectRounds(const SelectDesc &d, int64_t nrows) {
  SelectRoundsPlan p = PlanSelectRoundsNL(d, nrows, 0);
  if (!p.ok && p.NL == 8) p = PlanSelectRoundsNL(d, nrows, 4);  // 8 loaders leave too little staging: 4
  return p;
}
static SelectRoundsPlan PlanSelectRoundsNL(const SelectDesc &d, int64_t nrows, int force_nl) {
  SelectRoundsPlan p;
  memset(&p, 0, sizeof(p));
  if (d.ncol < 1 || d.ncol > SL_MAX_COL || d.nout < 1 || d.nout > SL_MAX_OUT) return p;
  uint32_t smask = 0;
  for (int k = 0; k < d.nout; k++) smask |= 1u << d.out_col[k];
  int rowb = 0;  // staged bytes per row: every distinct loaded column an output reads (+SR_VB if NULL-able)
  bool vout = false;
  for (int c = 0; c < d.ncol; c++) {
    if (d.col[c].w != 4 && d.col[c].w != 8) return p;
    p.ni += d.col[c].w / 4;
    if (d.col[c].w == 8) p.wm |= 1 << c;
    if ((smask >> c) & 1) rowb += d.col[c].w == 8 && !d.col[c].narrow ? 8 : 4;
    if (d.col[c].valid) {
      p.nv++;
      if (((smask >> c) & 1) && !d.col[c].vsent) rowb += SR_VB, vout = true;  // (a sentinel-staged output: no byte)
    }
  }
  p.nc = d.ncol;
  // Ring and staging share the CU's LDS.  Sub-steps per step (H) and ring depth
  // per H: H = 1 with a 3-deep ring for one- and two-slot columns sets, else 2;
  // H = 2 with a 2-deep ring.  H is the one that leaves the larger staging ring
  // (the staging ring is what hides the round latency; ties go to H = 2, whose
  // two interleaved sub-steps cost the loader fewer cycles per row).
  int want_h = 0, want_s = 0, want_stg = 4096, want_depth = 0;
  // One-column shapes staged in 4 bytes (INT32, or INT64 the zone map proves
  // fits int32) leave LDS for 8 loader waves (two per SIMD: each hides the
  // other's latencies) with a 3-deep ring and 2048 staged rows each
  // (profiles/r02_select_rounds_sweep.log).  MBX_SR_NL=4|8 overrides.
  // (+SR_VB staged bytes per row for a NULL-able output's validity).  Two
  // columns without a NULL-able output take 8 loaders too, at H = 1 with a
  // 1024-row staging ring each (SELECT v ... WHERE xn > 24: 3.83 -> 3.59 ms;
  // SELECT v ... WHERE x > 24: 3.45 -> 3.39); with one (SELECT vn ... WHERE
  // x > 24) the validity staging leaves too little LDS (4.07 -> 4.34 ms).
  p.NL = (p.nc == 1 && rowb <= 4 + p.nv * SR_VB) || (p.nc == 2 && !vout) ? 8 : 4;
  if (const char *e = Knob("MBX_SR_NL")) p.NL = atoi(e) == 8 && p.nc <= 2 ? 8 : 4;
  if (force_nl) p.NL = force_nl;
  p.NS = 4;  // storer waves (every instance has 4; the kernel takes NS as a parameter)
  if (p.NL == 8) want_h = 1, want_depth = p.nc == 1 || p.ni <= 2 ? 3 : 2;  // (the depths SrDepth instantiates)
  if (const char *e = Knob("MBX_SR_H")) want_h = atoi(e) == 1 ? 1 : 2;
  if (p.nv && p.NL == 8) want_h = 1;  // the 8-loader NULL-able form is H = 1 only
  if (p.nc == 2 && p.NL == 8 && want_h == 2) p.NL = 4, want_depth = 0;  // (two columns: 8 loaders at H = 1 only)
  if (const char *e = Knob("MBX_SR_S")) want_s = atoi(e) > 0 ? atoi(e) : 0;
  if (const char *e = Knob("MBX_SR_STG")) want_stg = atoi(e) >= 256 ? atoi(e) : 4096;
  if (const char *e = Knob("MBX_SR_DEPTH")) {
    const int v = atoi(e);
    if (p.nc == 1 && !p.nv && (v == 2 || v == 3 || v == 4 || v == 6)) want_depth = v;  // single-column shapes only (sweeps)
  }
  int best_stg = 0;
  for (int h = 2; h >= 1; h--) {
    if (want_h && h != want_h) continue;
    const int depth = want_depth ? want_depth : h == 2 ? 2 : (p.ni <= 2 ? 3 : 2);
    const size_t ring = (size_t)p.NL * depth * p.ni * 1024 * h + (p.nv ? (size_t)p.NL * depth * p.nc * 32 * h : 0);
    if (ring + 2048 >= (size_t)160 * 1024) continue;
    const size_t budget = (size_t)160 * 1024 - 2048 - ring;  // static meta (1.5 KB) + margin
    int stg = want_stg;
    while (stg >= 256 * h && (size_t)p.NL * (stg + 64) * rowb > budget) stg >>= 1;
    if (stg < 256 * h || (stg & (stg - 1))) continue;
    if (stg > best_stg) {
      best_stg = stg;
      p.H = h;
      p.depth = depth;
      p.lds = ring + (size_t)p.NL * (stg + 64) * rowb;
    }
  }
  if (!best_stg) return p;
  p.stg = best_stg;
  // a round is a quarter of the staging ring (1..4 steps)
  p.S = want_s ? want_s : std::max(1, std::min(4, p.stg / (1024 * p.H)));
  if (p.S * 256 * p.H > p.stg) p.S = p.stg / (256 * p.H);
  if (p.S < 1) return p;
  p.G = NumCUs() < 256 ? NumCUs() : 256;
  const int64_t nsteps = nrows / (256 * p.H);
  const int64_t ntiles = (nsteps + p.NL * p.S - 1) / (p.NL * p.S);
  p.nrounds = (ntiles + p.G - 1) / p.G;
  if (p.lds < (size_t)96 * 1024) p.lds = (size_t)96 * 1024;  // one workgroup per CU
  p.sleep = 1;
  if (const char *e = Knob("MBX_SR_SLEEP")) p.sleep = atoi(e) >= 0 ? atoi(e) : 1;
  p.pw = 2;  // rounds per coordinator poll (1..4)
  if (const char *e = Knob("MBX_SR_PW")) p.pw = std::max(1, std::min(4, atoi(e)));
  // tests: workgroup MBX_SR_TEST_STALL never publishes, as if it were never
  // scheduled, so every coordinator times out and the launch aborts
  p.test_stall = -1;
  if (const char *e = Knob("MBX_SR_TEST_STALL")) p.test_stall = atoi(e);
  p.ok = true;
  return p;
}

size_t SelectRoundsCtlBytes(const SelectRoundsPlan &p) { return (size_t)(8 + p.nrounds * p.G) * 8; }

namespace {
template <int NC, int WM, int DP, int H, int NL, bool VAL = false, int NS = 4>
void SrLaunchNL(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl, uint32_t epoch,
                hipStream_t s) {
  // the plan's layout must be this instance's: a mismatch (a planner rule
  // without a matching instance) would place rows wrongly, so it never launches
  if (p.NL != NL || p.NS != NS || p.H != H || p.depth != DP)
    throw std::logic_error("select_rounds: plan has no matching kernel");
  static std::atomic<uint64_t> attr{0};
  EnsureMaxLds((const void *)select_rounds_kernel<NC, WM, DP, H, NL, VAL, NS>, attr, 160 * 1024 - 2048);
  hipLaunchKernelGGL((select_rounds_kernel<NC, WM, DP, H, NL, VAL, NS>), dim3((unsigned)p.G), dim3((NL + NS + 1) * 64),
                     p.lds, s,
                     d, nrows, p.nrounds, p.S, p.stg, ctl, epoch, p.sleep, p.test_stall, p.pw);
}
template <int NC, int WM, int DP, int H>
void SrLaunchH(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl, uint32_t epoch,
               hipStream_t s) {
  if constexpr (NC == 1 || (NC == 2 && H == 1)) {
    if (p.NL == 8) return SrLaunchNL<NC, WM, DP, H, 8>(d, p, nrows, ctl, epoch, s);
  }
  SrLaunchNL<NC, WM, DP, H, 4>(d, p, nrows, ctl, epoch, s);
}
template <int NC, int WM>
void SrDepth(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl, uint32_t epoch,
             hipStream_t s) {
  constexpr int ni = SrCols<NC, WM>::ni();
  if (p.nv) {  // NULL-able columns: 8 loaders for one column only; H = 2 with a 2-deep ring, or H = 1
    if constexpr (NC == 1) {
      if (p.NL == 8) return SrLaunchNL<NC, WM, 3, 1, 8, true>(d, p, nrows, ctl, epoch, s);
    }
    if constexpr (NC == 2) {  // two columns: 8 loaders with H = 1 (the planner's ring depth for ni)
      if (p.NL == 8) return SrLaunchNL<NC, WM, (ni <= 2 ? 3 : 2), 1, 8, true>(d, p, nrows, ctl, epoch, s);
      // (6 loaders + 6 storers, one loader range per storer, measured no better
      // for SELECT vn ... WHERE x > 24 -- 3.57-3.61 vs 3.61-3.65 ms -- and
      // slower for SELECT v ... WHERE xn > 24, 3.49-3.51 vs 3.31-3.40 ms:
      // profiles/r05_seln_ab/; the instance was removed, NS stays a parameter)
    }
    if (p.H == 2) return SrLaunchNL<NC, WM, 2, 2, 4, true>(d, p, nrows, ctl, epoch, s);
    if (ni <= 2) return SrLaunchNL<NC, WM, 3, 1, 4, true>(d, p, nrows, ctl, epoch, s);
    return SrLaunchNL<NC, WM, 2, 1, 4, true>(d, p, nrows, ctl, epoch, s);
  }
  if (p.H == 1 && ni <= 2) {  // 3-deep ring at H = 1
    if constexpr (NC == 1) {
      if (p.depth == 2) return SrLaunchH<NC, WM, 2, 1>(d, p, nrows, ctl, epoch, s);
      if (p.depth == 4) return SrLaunchH<NC, WM, 4, 1>(d, p, nrows, ctl, epoch, s);
      if (p.depth == 6) return SrLaunchH<NC, WM, 6, 1>(d, p, nrows, ctl, epoch, s);
    }
    return SrLaunchH<NC, WM, 3, 1>(d, p, nrows, ctl, epoch, s);
  }
  if (p.H == 1) return SrLaunchH<NC, WM, 2, 1>(d, p, nrows, ctl, epoch, s);
  if constexpr (NC == 1) {
    if (p.depth == 3) return SrLaunchH<NC, WM, 3, 2>(d, p, nrows, ctl, epoch, s);
    if (p.depth == 4) return SrLaunchH<NC, WM, 4, 2>(d, p, nrows, ctl, epoch, s);
    if (p.depth == 6) return SrLaunchH<NC, WM, 6, 2>(d, p, nrows, ctl, epoch, s);
  }
  SrLaunchH<NC, WM, 2, 2>(d, p, nrows, ctl, epoch, s);
}
template <int NC, int WM = 0>
void SrDispatch(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl,
                uint32_t epoch, hipStream_t s) {
  if constexpr (WM < (1 << NC)) {
    if (p.wm == WM) return SrDepth<NC, WM>(d, p, nrows, ctl, epoch, s);
    SrDispatch<NC, WM + 1>(d, p, nrows, ctl, epoch, s);
  }
}
}  // namespace

// validity bytes (0/1) -> bits: each lane packs 16 consecutive bytes (one
// 16-byte load, so a wave reads 1 KiB contiguously) into 16 bits - bit i of
// (y * 0x0102040810204080) >> 56 is byte i of y - and 4 neighbouring lanes
// merge theirs into one output word by two shuffles.  (One thread per word
// with eight 8-byte loads 64 bytes apart measured 0.15 ms for 5.2e8 bytes.)
__global__ __launch_bounds__(256) void pack_validity_bytes_kernel(const uint8_t *__restrict__ b, int64_t n,
                                                                  uint64_t *__restrict__ bits) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t base = t * 16;
  uint64_t x = 0;
  if (base + 16 <= n) {
    const uint4 y = *(const uint4 *)(b + base);
    const uint64_t lo = ((uint64_t)y.y << 32) | y.x, hi = ((uint64_t)y.w << 32) | y.z;
    x = ((lo * 0x0102040810204080ull) >> 56) | (((hi * 0x0102040810204080ull) >> 56) << 8);
  } else if (base < n) {
    for (int64_t i = base; i < n; i++) x |= (uint64_t)(b[i] & 1) << (i - base);
  }
  x <<= 16 * (threadIdx.x & 3);
  x |= __shfl_xor(x, 1);
  x |= __shfl_xor(x, 2);
  if ((threadIdx.x & 3) == 0 && base < n) bits[t >> 2] = x;
}

void PackValidityBytes(const uint8_t *bytes, int64_t n, uint64_t *bits, hipStream_t s) {
  if (n <= 0) return;
  const int64_t words = (n + 63) / 64;
  hipLaunchKernelGGL(pack_validity_bytes_kernel, dim3((unsigned)((words * 4 + 255) / 256)), dim3(256), 0, s, bytes, n,
                     bits);
}

hipError_t SelectRounds(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl,
                        uint32_t epoch, hipStream_t s) {
  if (!p.ok) throw std::runtime_error("SelectRounds: unsupported shape");
  (void)hipGetLastError();  // an earlier, unrelated sticky error must not be taken for this launch's
  try {
    switch (p.nc) {
      case 1: SrDispatch<1>(d, p, nrows, ctl, epoch, s); break;
      case 2: SrDispatch<2>(d, p, nrows, ctl, epoch, s); break;
      case 3: SrDispatch<3>(d, p, nrows, ctl, epoch, s); break;
      default: SrDispatch<4>(d, p, nrows, ctl, epoch, s); break;
    }
  } catch (const std::logic_error &) {
    return hipErrorInvalidConfiguration;  // nothing launched: the caller takes the two-pass form
  }
  return hipGetLastError();  // the launch's own error (LDS / resource limits): the caller falls back
}

// ---------------------------------------------------------------------------
// Count-first compaction (see device.h): chunk-owned steps in both passes.
// ---------------------------------------------------------------------------
int64_t CountChunks(int64_t nrows) { return ((nrows >> 8) + FC_CHUNK - 1) / FC_CHUNK; }

// Pass 1 counts every K1 steps (K1 divides FC_CHUNK; MBX_FK_CHUNK, default
// FC_CHUNK: 1.29 ms at 1e9 INT64 rows vs 1.36 for K1 = 1, which walks the steps
// grid-stride like the fused filter-aggregate); pass 2 reads the offset of
// chunk c at entry c * FC_CHUNK / K1 of the scanned counts.
static int FkChunk() {
  const char *e = Knob("MBX_FK_CHUNK");
  const int v = e ? atoi(e) : FC_CHUNK;
  return (v == 1 || v == 2 || v == 4) ? v : FC_CHUNK;
}
int64_t CountEntries(int64_t nrows) {  // pass-1 count entries over the full steps (+1 for the partial step)
  const int64_t steps = nrows >> 8;
  return ((steps + FC_CHUNK - 1) / FC_CHUNK) * (FC_CHUNK / FkChunk());
}

namespace {
// sequence position p of wave wv -> its step (chunk wv + (p / K) NW, step p % K
// of that chunk), or -1 past the wave's last chunk / past the last full step
template <int K>
__device__ __forceinline__ int64_t cc_step(int64_t p, int64_t wv, int64_t nw, int64_t nchunks, int64_t nsteps) {
  const int64_t c = wv + (p / K) * nw;
  const int64_t st = c * K + p % K;
  return c < nchunks && st < nsteps ? st : -1;
}
}  // namespace

// pass 1: NI LDS-DMA instructions (KiB of predicate slices) per step, one
// count per K1 steps
template <int NI, int DEPTH, int K1>
__global__ __launch_bounds__(256) void filter_count_lds_kernel(FilterMultiDesc D, int64_t n, uint32_t *counts,
                                                               int slot_bytes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fk_lds[];
  const int SB = slot_bytes;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = fk_lds + (size_t)w * DEPTH * SB;
  int off[FM_MAX];
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      off[c] = o;
      if (c < D.ncol) o += D.col[c].phys == P_I64 ? 2048 : 1024;
    }
  }
  const int64_t nsteps = n >> 8;
  const int64_t nchunks = ((nsteps + FC_CHUNK - 1) / FC_CHUNK) * (FC_CHUNK / K1);  // count entries
  const int64_t nw = (int64_t)gridDim.x * 4, wv = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t p, int d) {
    int64_t q = cc_step<K1>(p, wv, nw, nchunks, nsteps);
    if (q < 0) q = 0;
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FM_MAX; c++) {
      if (c >= D.ncol) break;
      const int B = D.col[c].phys == P_I64 ? 2048 : 1024;
      const unsigned char *src = (const unsigned char *)D.col[c].data + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)(dst + off[c]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + off[c] + 1024), 16, 0, 2);
    }
  };
  if (wv < nchunks) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) issue(d, d);
    int k = 0;
    uint32_t acc = 0;
    for (int64_t p = 0;; p++) {
      const int64_t c = wv + (p / K1) * nw;
      if (c >= nchunks) break;
      const int64_t st = c * K1 + p % K1;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (DEPTH - 1)) : "memory");
      const unsigned char *src = ring + k * SB;
      bool ok[4] = {st < nsteps, st < nsteps, st < nsteps, st < nsteps};
#pragma unroll
      for (int c2 = 0; c2 < FM_MAX; c2++) {
        if (c2 >= D.ncol) break;
        int64_t v[4];
        sl_read4(src + off[c2], D.col[c2].phys == P_I64 ? 8 : 4, lane, v);
#pragma unroll
        for (int e = 0; e < 4; e++) ok[e] = ok[e] && (uint64_t)(v[e]) - (uint64_t)(D.col[c2].lo) <= D.col[c2].span;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(p + DEPTH, k);
#pragma unroll
      for (int e = 0; e < 4; e++) acc += (uint32_t)__popcll(__ballot(ok[e]));
      if (p % K1 == K1 - 1) {
        if (lane == 0) counts[c] = acc;
        acc = 0;
      }
      k = k + 1 == DEPTH ? 0 : k + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // the partial last step's count after the chunks (always written)
  if (blockIdx.x == 0 && w == 0) {
    bool ok[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t i = (nsteps << 8) + 4 * lane + e;
      ok[e] = i < n;
      for (int c = 0; c < D.ncol && ok[e]; c++) {
        const int64_t x = D.col[c].phys == P_I64 ? ((const int64_t *)D.col[c].data)[i]
                                                 : (int64_t)((const int32_t *)D.col[c].data)[i];
        ok[e] = (uint64_t)(x) - (uint64_t)(D.col[c].lo) <= D.col[c].span;
      }
    }
    uint32_t t = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) t += (uint32_t)__popcll(__ballot(ok[e]));
    if (lane == 0) counts[nchunks] = t;
  }
}

void FilterCountChunks(const FilterMultiDesc &d, int64_t nrows, uint32_t *counts, hipStream_t s) {
  int ni = 0;
  for (int c = 0; c < d.ncol; c++) {
    if (d.col[c].valid) throw std::runtime_error("FilterCountChunks: NULL-able predicate column");
    ni += d.col[c].phys == P_I64 ? 2 : 1;
  }
  const int slot = ni * 1024;
  int gpc = 3;
  if (const char *e = Knob("MBX_FK_BLOCKS_PER_CU")) gpc = atoi(e) > 0 ? atoi(e) : 3;
  const int64_t chunks = CountEntries(nrows);
  int64_t grid = (int64_t)NumCUs() * gpc;
  if (grid > chunks / 4 + 1) grid = chunks / 4 + 1;
  int dp = 0;
  if (const char *e = Knob("MBX_FK_DEPTH")) dp = atoi(e);
  const int k1 = FkChunk();
#define FK1(L, DP, K)                                                                                         \
  hipLaunchKernelGGL((filter_count_lds_kernel<L, DP, K>), dim3((unsigned)grid), dim3(256), (size_t)4 * DP * slot, s, \
                     d, nrows, counts, slot)
#define FK(L, DP) \
  if (k1 == 8) FK1(L, DP, 8); else if (k1 == 4) FK1(L, DP, 4); else if (k1 == 2) FK1(L, DP, 2); else FK1(L, DP, 1)
#define FKD(L, DEF) \
  if ((dp ? dp : DEF) <= 2) FK(L, 2); else if ((dp ? dp : DEF) <= 3) FK(L, 3); else if ((dp ? dp : DEF) <= 4) FK(L, 4); else FK(L, 6);
  switch (ni) {
    case 1: FKD(1, 6); break;
    case 2: FKD(2, 6); break;
    case 3: FKD(3, 3); break;
    case 4: FKD(4, 3); break;
    case 5: FK(5, 2); break;
    case 6: FK(6, 2); break;
    case 7: FK(7, 2); break;
    default: FK(8, 2); break;
  }
#undef FKD
#undef FK
#undef FK1
  (void)hipGetLastError();
}

// pass 2: NLD KiB of output slices per step; predicates re-evaluated on them
template <int NLD, int DEPTH>
__global__ __launch_bounds__(256) void compact_recomp_lds_kernel(CompactDesc D, int64_t n,
                                                                 const int64_t *__restrict__ offs, int stride) {
  extern __shared__ __attribute__((aligned(16))) unsigned char cr_lds[];
  constexpr int SB = NLD * 1024;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned char *ring = cr_lds + (size_t)w * DEPTH * SB;
  unsigned char *stage = cr_lds + (size_t)4 * DEPTH * SB + (size_t)w * 2048;
  int off[FC_MAX_OUT];
  {
    int o = 0;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      off[c] = o;
      if (c < D.nout) o += D.ow[c] * 256;
    }
  }
  const uint64_t lt = (1ull << lane) - 1;
  const int64_t nsteps = n >> 8, nchunks = (nsteps + FC_CHUNK - 1) / FC_CHUNK;
  const int64_t nw = (int64_t)gridDim.x * 4, wv = (int64_t)blockIdx.x * 4 + w;
  auto issue = [&](int64_t p, int d) {
    int64_t q = cc_step<FC_CHUNK>(p, wv, nw, nchunks, nsteps);
    if (q < 0) q = 0;
    unsigned char *dst = ring + d * SB;
#pragma unroll
    for (int c = 0; c < FC_MAX_OUT; c++) {
      if (c >= D.nout) break;
      const int B = D.ow[c] * 256;
      const unsigned char *src = (const unsigned char *)D.src[c] + q * B;
      __builtin_amdgcn_global_load_lds((const void *)(src + lane * 16), (void *)(dst + off[c]), 16, 0, 2);
      if (B == 2048)
        __builtin_amdgcn_global_load_lds((const void *)(src + 1024 + lane * 16), (void *)(dst + off[c] + 1024), 16, 0, 2);
    }
  };
  if (wv < nchunks) {
#pragma unroll
    for (int d = 0; d < DEPTH; d++) issue(d, d);
    int k = 0;
    int64_t run = 0;
    for (int64_t p = 0;; p++) {
      const int64_t c = wv + (p / FC_CHUNK) * nw;
      if (c >= nchunks) break;
      const int64_t st = c * FC_CHUNK + p % FC_CHUNK;
      if (p % FC_CHUNK == 0) run = offs[c * stride];
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD * (DEPTH - 1)) : "memory");
      const unsigned char *src = ring + k * SB;
      int64_t v[FC_MAX_OUT][4];
#pragma unroll
      for (int c2 = 0; c2 < FC_MAX_OUT; c2++) {
        if (c2 >= D.nout) break;
        sl_read4(src + off[c2], D.ow[c2], lane, v[c2]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(p + DEPTH, k);
      k = k + 1 == DEPTH ? 0 : k + 1;
      if (st >= nsteps) continue;  // wave-uniform: past the last full step
      bool ok[4] = {true, true, true, true};
#pragma unroll
      for (int j = 0; j < FM_MAX; j++) {
        if (j >= D.npred) break;
        int64_t pv[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          // the predicate's column among the outputs (a uniform index)
          int64_t x = v[0][e];
#pragma unroll
          for (int c2 = 1; c2 < FC_MAX_OUT; c2++)
            if (c2 == D.pred_out[j]) x = v[c2][e];
          pv[e] = x;
        }
#pragma unroll
        for (int e = 0; e < 4; e++) ok[e] = ok[e] && (uint64_t)(pv[e]) - (uint64_t)(D.pred_lo[j]) <= D.pred_span[j];
      }
      const unsigned long long b0 = __ballot(ok[0]), b1 = __ballot(ok[1]), b2 = __ballot(ok[2]), b3 = __ballot(ok[3]);
      const int cnt = __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
      if (cnt == 0) continue;
      const unsigned m = (unsigned)ok[0] | (unsigned)ok[1] << 1 | (unsigned)ok[2] << 2 | (unsigned)ok[3] << 3;
      const int r0 = __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
#pragma unroll
      for (int c2 = 0; c2 < FC_MAX_OUT; c2++) {
        if (c2 >= D.nout) break;
        int r = r0;
        if (D.ow[c2] == 8) {
#pragma unroll
          for (int e = 0; e < 4; e++)
            if ((m >> e) & 1u) ((int64_t *)stage)[r++] = v[c2][e];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          int64_t *dst = (int64_t *)D.dst[c2] + run;
          for (int i = lane; i < cnt; i += 64) dst[i] = ((const int64_t *)stage)[i];
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++)
            if ((m >> e) & 1u) ((int32_t *)stage)[r++] = (int32_t)v[c2][e];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          int32_t *dst = (int32_t *)D.dst[c2] + run;
          for (int i = lane; i < cnt; i += 64) dst[i] = ((const int32_t *)stage)[i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      run += cnt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // the partial last step: block 0, wave 0, guarded loads, after every chunk
  if (blockIdx.x == 0 && w == 0 && (n & 255)) {
    bool ok[4];
    const int64_t i0 = (nsteps << 8) + 4 * lane;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t i = i0 + e;
      ok[e] = i < n;
      for (int j = 0; j < D.npred && ok[e]; j++) {
        const int c = D.pred_out[j];
        const int64_t x = D.ow[c] == 8 ? ((const int64_t *)D.src[c])[i] : (int64_t)((const int32_t *)D.src[c])[i];
        ok[e] = (uint64_t)(x) - (uint64_t)(D.pred_lo[j]) <= D.pred_span[j];
      }
    }
    unsigned long long bb[4];
#pragma unroll
    for (int e = 0; e < 4; e++) bb[e] = __ballot(ok[e]);
    int64_t pos = offs[nchunks * stride] + __popcll(bb[0] & lt) + __popcll(bb[1] & lt) + __popcll(bb[2] & lt) +
                  __popcll(bb[3] & lt);
    for (int e = 0; e < 4; e++) {
      if (!ok[e]) continue;
      for (int c = 0; c < D.nout; c++) {
        if (D.ow[c] == 8) ((int64_t *)D.dst[c])[pos] = ((const int64_t *)D.src[c])[i0 + e];
        else ((int32_t *)D.dst[c])[pos] = ((const int32_t *)D.src[c])[i0 + e];
      }
      pos++;
    }
  }
}

void CompactRecompute(const CompactDesc &d, int64_t nrows, const int64_t *chunk_offsets, hipStream_t s) {
  int nld = 0;
  for (int c = 0; c < d.nout; c++) {
    if (d.ow[c] != 4 && d.ow[c] != 8) throw std::runtime_error("CompactRecompute: outputs must be 4 or 8 bytes");
    nld += d.ow[c] / 4;
  }
  if (nld < 1 || nld > 8 || d.npred < 1 || d.npred > FM_MAX) throw std::runtime_error("CompactRecompute: shape");
  int gpc = 3;
  if (const char *e = Knob("MBX_CR_BLOCKS_PER_CU")) gpc = atoi(e) > 0 ? atoi(e) : 3;
  const int64_t chunks = CountChunks(nrows);
  int64_t grid = (int64_t)NumCUs() * gpc;
  if (grid > chunks / 4 + 1) grid = chunks / 4 + 1;
  int dp = 0;
  if (const char *e = Knob("MBX_CR_DEPTH")) dp = atoi(e);
#define CR(L, DP)                                                                                               \
  hipLaunchKernelGGL((compact_recomp_lds_kernel<L, DP>), dim3((unsigned)grid), dim3(256),                      \
                     (size_t)4 * DP * L * 1024 + 4 * 2048, s, d, nrows, chunk_offsets, FC_CHUNK / FkChunk())
#define CRD(L, DEF) \
  if ((dp ? dp : DEF) <= 2) CR(L, 2); else if ((dp ? dp : DEF) <= 3) CR(L, 3); else if ((dp ? dp : DEF) <= 4) CR(L, 4); else CR(L, 6);
  switch (nld) {
    case 1: CRD(1, 6); break;
    case 2: CRD(2, 3); break;
    case 3: CRD(3, 2); break;
    case 4: CRD(4, 2); break;
    case 5: CR(5, 2); break;
    case 6: CR(6, 2); break;
    case 7: CR(7, 2); break;
    default: CR(8, 2); break;
  }
#undef CRD
#undef CR
  (void)hipGetLastError();
}

}  // namespace dev
}  // namespace mbx
