// device.h — host-callable launchers for the gfx950 kernels in kernels.hip.
// Everything here is asynchronous on the given stream unless stated.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "vm.h"

namespace mbx {
namespace dev {

// validity[w] = ~nullbits[w] over the words covering n rows (tail bits cleared)
void InvertNullBits(uint64_t *bits, int64_t n, hipStream_t s);

// --- expression VM --------------------------------------------------------
// Predicate pass: one bit per row into sel_bits (4 x u64 words per 256-row
// tile) and the selected-row count of every tile into tile_counts.
void VmFilter(const VmProgram &p, const VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
              uint64_t *sel_bits, uint32_t *tile_counts, int32_t *err, hipStream_t s);
// Projection pass over all rows (sel_bits == null) or over the selected rows,
// written densely at tile_offsets[tile] + rank.
void VmProject(const VmProgram &p, const VmCols &cols, int64_t nrows, int64_t range_start, int64_t range_step,
               const uint64_t *sel_bits, const int64_t *tile_offsets, const VmOuts &outs, int32_t *err,
               hipStream_t s);
// Exclusive scan of tile counts -> int64 offsets; total written to *total (device).
void ScanTileCounts(const uint32_t *counts, int64_t *offsets, int64_t n, int64_t *total, hipStream_t s);

// --- aggregate state (one per aggregate and group slot), 64 bytes -------
struct AggState {
  unsigned long long count;
  unsigned long long sum_lo;
  long long sum_hi;
  long long min_i, max_i;
  double sum_f;
  unsigned long long min_f, max_f;  // order-preserving encoded doubles
};

// --- fused scan -> filter -> aggregate (no GROUP BY; configs C2, C5) -------
// Predicate lo <= p[i] <= hi on column p (P_I32 / P_I64, no nulls) or none;
// aggregate column a (P_I32 / P_I64; == p allowed) or none (COUNT(*) only).
// count_star += selected rows; st accumulates count/sum/min/max of a.
// One workgroup's partial of the fused filter-aggregate (count, int128 sum as
// lo/hi, min, max) — same layout as the kernel's accumulator.
struct AggPartial {
  uint64_t cnt;
  uint64_t slo;
  int64_t shi;
  int64_t mn, mx;
};
// Launches the fused filter-aggregate.  With `partials` (room for
// kMaxAggPartials) the default LDS-DMA kernel writes one AggPartial per
// workgroup and the call returns how many; the emit kernel reduces them
// (EmitDesc::partials), so no state initialisation and no atomics are
// needed.  Otherwise (or for shapes the LDS kernel does not take) it zeroes
// st/cstar itself, accumulates with atomics and returns 0.
constexpr int kMaxAggPartials = 4096;

// Fused filter-aggregate over several columns: a conjunction of range
// predicates on up to 4 int32/int64 columns (no NULLs) and at most one
// aggregated column (which may also carry a predicate).  Always writes
// per-workgroup partials (returns their count, > 0).
#define FM_MAX 4
struct FilterMultiCol {
  const void *data;
  int32_t phys;     // P_I32 / P_I64
  int32_t is_pred;  // 1: lo <= x <= lo + span
  int64_t lo;
  uint64_t span;
  const uint64_t *valid;  // FilterBits only: validity words (NULL fails the predicate); nullptr = no NULLs
};
struct FilterMultiDesc {
  int32_t ncol;
  int32_t agg;  // index into col[] of the aggregated column, -1: COUNT only
  int32_t mm;
  int32_t narrow;   // set by FilterMultiPartials from maxabs and its grid
  int32_t mm32;     // set by FilterMultiPartials: MIN/MAX in int32 (|value| < 2^31 by the zone map)
  uint64_t maxabs;  // zone-map bound on |aggregated value|, ~0 = unknown
  FilterMultiCol col[FM_MAX];
};
int FilterMultiPartials(const FilterMultiDesc &d, int64_t nrows, AggPartial *partials, hipStream_t s);
int FilterAggStates(const void *pcol, int pphys, int64_t lo, int64_t hi, bool has_pred, const void *acol, int aphys,
                    int64_t nrows, AggState *st, unsigned long long *cstar, int grid_blocks, hipStream_t s,
                    bool need_minmax = true, uint64_t sum_maxabs = ~0ull, AggPartial *partials = nullptr);

// --- fused GROUP BY on a small-range integer key (config C3) -------------
// key in [kmin, kmin + nk) (the NULL group in slot nk - 1 when the key has
// NULLs); up to 2 value columns of one phys.  vm: NULL-able columns (bit 0
// value 0, bit 1 value 1, bit 2 the key); any: + the valid-row count tables
size_t GroupDirectLds(int nk, int R, int nv, bool mm, int vm = 0);
// validity words (LSB-first, 16-B aligned) of the NULL-able columns, or nullptr
struct GroupValidity {
  const uint64_t *key, *v0, *v1;
};
// Optional fused range predicates of the direct GROUP BY (a conjunction):
// rows with lo <= p <= lo + span for every entry.  src: 1 = its own column
// `col` (int32/int64, loaded as an extra slice), 2 = the key column, 3 = value
// column 0.
#define GROUP_MAX_PRED 3
struct GroupPred {
  int32_t src;
  int32_t phys;
  const void *col;
  int64_t lo;
  uint64_t span;
};
struct GroupPreds {
  int32_t n;
  int32_t xcd;  // group_direct_lds: 1 = XCD-grouped step windows (blocks b, b+8, ... share an XCD)
  GroupPred p[GROUP_MAX_PRED];
};
// Per-workgroup partial records of group_direct_lds (key-major, GroupPartialWords
// u64 each: COUNT(*), then per value column its valid-row count, sum lo / hi
// and, with MIN/MAX, min / max), reduced by GroupPartialsCompact.
constexpr int kGroupPartialKeys = 128;
__host__ __device__ constexpr int GroupPartialWords(int nv, bool mm) { return 1 + nv * (mm ? 5 : 3); }
struct GroupPartialsOut {
  void *buf;            // room for the records
  size_t bytes;
  int64_t state_slots;  // AggStates at st0 (st1 follows st0) that the call initialises when it uses atomics
  bool used;            // set: the records were written (GroupPartialsCompact must follow)
  int blocks;           // set: workgroups that wrote records
};
// The records reduced into cstar / st0 / st1 for every key (empty keys as
// initialised), then the non-empty keys compacted as CompactSlots does; with
// emit, the same launch then writes that relation as EmitAggRelation would
// (emit->slot_list / n_list: slot_list / n_out).
struct EmitDesc;
void GroupPartialsCompact(const GroupPartialsOut &po, int nv, bool mm, int nk, unsigned long long *count_star,
                          AggState *st0, AggState *st1, int32_t *slot_list, int64_t *n_out, hipStream_t s,
                          const EmitDesc *emit = nullptr);
// false only when a predicate was given and the shape needs the segmented kernel.
// po: the caller did not initialise cstar / st0 / st1: the call does (atomic
// forms) or writes per-workgroup records instead (po->used).
bool GroupByDirectStates(const void *kcol, int kphys, int64_t kmin, int nk, const void *v0, const void *v1, int vphys,
                         int nv, bool mm, int64_t nrows, int64_t seg_rows, int R, unsigned long long *cstar,
                         AggState *st0, AggState *st1, int grid_blocks, hipStream_t s,
                         const GroupPreds *pred = nullptr, uint64_t vmaxabs = ~0ull /* (unused) */,
                         const GroupValidity *valid = nullptr,  // NULL-able key / values: false if unsupported
                         GroupPartialsOut *po = nullptr);

// --- GROUP BY one integer key over a wide range (group_part.hip) ----------
// Keys in [kmin, kmin + range) without NULLs, up to 2 value columns of one
// phys without NULLs; rows partitioned by key range (hist, scan, scatter),
// each partition reduced in an LDS table.  Writes COUNT(*) into cstar[range]
// and the states of value column j into st0[j * range ..] (every key: empty
// keys as InitAggStatesCounts leaves them).  false: the shape does not fit
// (range above PartGroupMaxRange, n >= 2^32, a value bound that would make the
// pieces too small).
constexpr int kPartGroupMaxParts = 4096;
int PartGroupShift(int nv, bool mm);          // log2 keys per partition
int64_t PartGroupMaxRange(int nv, bool mm);
struct PartGroupDesc {
  const void *key;
  int kphys;
  int64_t kmin, range;
  const void *v0, *v1;
  int vphys, nv;
  bool mm;
  int64_t n;
  uint64_t vmaxabs;  // max |value| (zone maps); 0 = no value columns
  unsigned long long *cstar;
  AggState *st0;  // [nv >= 2 ? 2 * range : range]
  void *scratch_hist, *scratch_start, *scratch_rows, *scratch_scan;
  size_t scratch_scan_bytes;
};
void PartGroupScratch(int64_t n, int64_t range, int nv, bool mm, int vphys, size_t *hist_bytes, size_t *start_bytes,
                      size_t *rows_bytes, size_t *scan_bytes);
bool PartGroup(const PartGroupDesc &d, hipStream_t s);
// F3h: the same with a hashed partition function, for integer keys too sparse
// for dense states (<= 1 value column): groups land in a global hash table of
// PartGroupHashedSlots() slots -- gkeys[slot] = key ^ 2^63 (0: empty, except
// the last slot, INT64_MIN's group), cstar / st0 per slot.  *overflow (device)
// becomes non-zero when a table filled up: the result is then incomplete and
// the caller must answer the query another way.
bool PartGroupHashed(const PartGroupDesc &d, unsigned long long *gkeys, int *overflow, hipStream_t s);
int64_t PartGroupHashedSlots();
void PartGroupHashedScratch(int64_t n, int nv, size_t *hist_bytes, size_t *start_bytes, size_t *rows_bytes,
                            size_t *scan_bytes);

// --- generic aggregation over compacted columns ---------------------------
// vclass: VC_I64 / VC_I128 / VC_F64 of the input column (phys given)
void ReduceColumn(const void *col, int phys, const uint64_t *valid, int64_t n, AggState *out, hipStream_t s);
// min/max of an integer key column (for group planning); writes {min,max,nonnull count}
void KeyRange(const void *col, int phys, const uint64_t *valid, int64_t n, long long *out3, hipStream_t s);
// Direct-index grouping: slot = valid ? key - kmin : nslots-1 (NULL group).
// For every aggregate column: AggState per slot; count_star per slot.
void GroupAssign(const void *kcol, int kphys, const uint64_t *kvalid, int64_t kmin, int64_t nslots, int64_t n,
                 int32_t *slot_of_row, unsigned long long *count_star, hipStream_t s);
void GroupReduceColumn(const int32_t *slot_of_row, const void *col, int phys, const uint64_t *valid, int64_t n,
                       AggState *states, hipStream_t s);
void InitAggStates(AggState *st, int64_t n, hipStream_t s);
void InitAggStatesCounts(AggState *st, int64_t n, unsigned long long *cs, int64_t nc, hipStream_t s);
// Compact non-empty slots into the aggregate relation (index list).
void CompactSlots(const unsigned long long *count_star, int64_t nslots, int32_t *slot_list, int64_t *n_out,
                  hipStream_t s);

// --- sort / gather -------------------------------------------------------
// Order-preserving u64 keys of a column (asc; desc flips; nulls per flag).
void SortKeyU64(const void *col, int phys, const uint64_t *valid, int64_t n, const int64_t *perm, bool desc,
                bool nulls_first, uint64_t *keys, hipStream_t s);
void SortPairs(uint64_t *keys_in, int64_t *vals_in, uint64_t *keys_out, int64_t *vals_out, int64_t n, hipStream_t s,
               int end_bit = 64);
void SortKeyNull(const uint64_t *valid, int64_t n, const int64_t *perm, bool nulls_first, uint64_t *keys,
                 hipStream_t s);
void SortKeyStr(const int64_t *offsets, const char *chars, const uint64_t *valid, int64_t n, const int64_t *perm,
                int64_t chunk, bool desc, uint64_t *keys, hipStream_t s);
void StrMaxLen(const int64_t *offsets, int64_t n, unsigned long long *out, hipStream_t s);
void Iota(int64_t *p, int64_t n, int64_t start, hipStream_t s);
// out[i] = in[idx[i]] for fixed-width phys; validity likewise (bitmap)
void GatherFixed(const void *in, int phys, const uint64_t *in_valid, const int64_t *idx, int64_t n, void *out,
                 uint32_t *out_valid, hipStream_t s);
void GatherSlots(const void *in, int elem_bytes, const int32_t *idx, int64_t n, void *out, hipStream_t s);

// --- strings ---------------------------------------------------------------
// codes[i] >= 0: row of the source string column; < 0: -(k+1) into pool.
void StringLengths(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off,
                   const int64_t *pool_off, int64_t *lens, hipStream_t s);
void ScanLengths(const int64_t *lens, int64_t *offsets, int64_t n, hipStream_t s);  // offsets[n+1]
void StringCopy(const int64_t *codes, const uint64_t *valid, int64_t n, const int64_t *src_off, const char *src_chars,
                const int64_t *pool_off, const char *pool_chars, const int64_t *out_off, char *out_chars,
                hipStream_t s);

// --- ingest / stats ----------------------------------------------------------
// min/max/null count over rows [0, n) of a fixed-width integer-like column.
void ColumnStats(const void *col, int phys, const uint64_t *valid, int64_t n, long long *out3, hipStream_t s);
// Synthetic column: out[i] = splitmix64(seed + start + i) mod m + add  (int64 or int32)
void Synth(void *out, int phys, int64_t n, int64_t seed, int64_t start, int64_t m, int64_t add, hipStream_t s);
// Copy a bitmap range: dst bits [dst_off, dst_off+n) = src bits [0, n) (src null -> all ones)
void BitmapAppend(uint64_t *dst, int64_t dst_off, const uint64_t *src, int64_t n, hipStream_t s);
// HBM calibration: out = in (float4 copy), nbytes multiple of 16
void CopyKernel(const void *in, void *out, int64_t nbytes, hipStream_t s);
// best-of-iters GB/s of {float4 copy (read+write bytes), nt int64 read, plain int64 read}
constexpr int kCalibrateShapes = 8;  // HbmCalibrate's measured shapes (kernels.hip)
void HbmCalibrate(void *buf_a, void *buf_b, int64_t bytes, int iters, double out[kCalibrateShapes], hipStream_t s);
// clock stamps of the last stamped launch (libduckdb_mb_amd_clk.so only; 0 otherwise)
int ReadClockStamps(uint64_t *out, int cap, hipStream_t s);

int NumCUs();

}  // namespace dev
}  // namespace mbx

namespace mbx {
namespace dev {

// --- aggregate relation emission ---------------------------------------------
struct EmitAgg {
  int32_t kind;      // AggKind
  int32_t in_class;  // VClass of the aggregated column
  int32_t out_phys;  // Phys of the result column
  int32_t avg_scale; // decimal scale for AVG
  AggState *states;  // per slot (null for COUNT_STAR)
  void *out;
  uint32_t *valid;   // zeroed bitmap words
};
#define EMIT_MAX_AGGS 16
#define EMIT_MAX_CKEYS 4
struct EmitDesc {
  int32_t nagg;
  EmitAgg a[EMIT_MAX_AGGS];
  const unsigned long long *cstar;  // per slot
  const int32_t *slot_list;         // null: slots 0..nslots-1 all emitted
  const int64_t *n_list;            // device count of slot_list (if slot_list)
  int64_t nslots;
  int32_t has_key;
  int32_t key_phys;
  int64_t kmin;
  int64_t null_slot;  // -1 if none
  // has_key with key_msb: the key of slot sl is key_msb[sl] ^ 2^63 (the hashed
  // wide GROUP BY's table) instead of kmin + sl
  const unsigned long long *key_msb;
  void *key_out;
  uint32_t *key_valid;
  // composite keys (instead of has_key): key q of slot sl is kmin + digit,
  // digit = (sl / stride) % radix; NULL when nullable and digit == radix - 1
  int32_t nkeys_c;
  struct {
    void *out;
    uint32_t *valid;
    int32_t phys, nullable;
    int64_t kmin, radix, stride;
  } kc[EMIT_MAX_CKEYS];
  // optional: reduce these per-workgroup partials into slot 0 first
  // (states of every aggregate and cstar[0]); emit then runs one workgroup
  const AggPartial *partials;
  int32_t npartials;
};
void EmitAggRelation(const EmitDesc &d, hipStream_t s);

// ---- hash GROUP BY (any number of fixed-width / VARCHAR keys) --------------
struct HashKeyCol {
  const void *data;
  const uint64_t *validity;
  const int64_t *offsets;  // P_STR
  const char *chars;       // P_STR
  int32_t phys;
};
#define HASH_MAX_KEYS 8
struct HashKeys {
  int32_t nk;
  HashKeyCol k[HASH_MAX_KEYS];
};
// Open-addressing table (cap = power of two >= 2n, 8 B/entry: 24-bit hash
// tag | 40-bit representative row).  Produces slot_of_row in [0, ngroups)
// (dense group ids in table order), rep_row[g], count_star[g] and
// *ngroups (device).  Scratch: table (cap x 8 B), entry ids (cap x 4 B).
// Scratch allocator the helpers below use (set per call by the executor to
// the connection's caching pool; the helpers run on that connection's stream).
typedef void *(*TempAllocFn)(size_t bytes, void *ctx);
typedef void (*TempFreeFn)(void *p, size_t bytes, void *ctx);
void SetTempAllocator(TempAllocFn a, TempFreeFn f, void *ctx);
void CountSlots(const int32_t *slot_of_row, int64_t n, unsigned long long *count_star, hipStream_t s);
void HashGroupAssign(const HashKeys &k, int64_t n, unsigned long long *table, int64_t cap, int32_t *slot_of_row,
                     int32_t *gid_of_entry, int64_t *rep_row, unsigned long long *count_star, int64_t *ngroups,
                     int32_t *err, hipStream_t s);

// Small results: one kernel copies every result buffer (and the device error
// word) into coherent pinned host memory, replacing a DMA per buffer.
struct HostCopySeg {
  const void *src;
  void *dst;
  int64_t bytes;
};
#define HOSTCOPY_MAX 32
struct HostCopyDesc {
  int32_t nseg;
  HostCopySeg seg[HOSTCOPY_MAX];
  const int32_t *err_src;
  int32_t *err_dst;
};
void HostCopy(const HostCopyDesc &d, hipStream_t s);
// Arrow wire layout of a fixed-width (1/4/8-byte) column: vals[i] = src[i], or
// 0 where the validity bit is clear; vbytes[i] = validity (may be nullptr;
// valid == nullptr means no NULLs).
void ArrowWire(const void *src, const uint64_t *valid, int64_t n, int width, void *vals, uint8_t *vbytes,
               hipStream_t s);

// Filter -> compaction in two streaming passes (order preserving), for a
// conjunction of range predicates over NULL-free int32/int64 columns and
// NULL-free 1/2/4/8/16-byte output columns.  A "step" is 256 consecutive rows.
//  1. FilterBits: predicate columns through an LDS-DMA ring; per step four
//     ballot words (bit L of word e <-> row 256 s + 4 L + e, the lane layout
//     of both passes).
//  2. ScanStepBits -> each step's first output position (exclusive scan of
//     the words' popcounts).
//  3. CompactColumns: output columns through an LDS-DMA ring; each selected
//     row goes to offset[step] + its rank inside the step.
#define FC_MAX_OUT 8
struct CompactDesc {
  int32_t nout;
  const void *src[FC_MAX_OUT];
  void *dst[FC_MAX_OUT];
  int32_t ow[FC_MAX_OUT];  // 1, 2, 4, 8 or 16 bytes (4/8 only: the register kernel; else the generic one)
  // CompactRecompute only: the range predicates, each over one of the output
  // columns (pred_out[j]; 4/8-byte integer, sign-extended), evaluated again
  // from the slices pass 2 loads anyway
  int32_t npred;
  int32_t pred_out[FM_MAX];
  int64_t pred_lo[FM_MAX];
  uint64_t pred_span[FM_MAX];
};
void FilterBits(const FilterMultiDesc &d, int64_t nrows, unsigned long long *bits, hipStream_t s);
// exclusive scan of the steps' selected-row counts (popcounts of their ballot words)
void ScanStepBits(const unsigned long long *bits, int64_t *offsets, int64_t steps, int64_t *total, hipStream_t s);
// Validity of the compacted rows: bit offset[step] + rank of every selected
// row of valid_in (64-bit words, bit r = row r) into valid_out, which must be
// zeroed (a step's first and last output words are OR'd, shared with its
// neighbours).
void CompactValidity(const unsigned long long *bits, const int64_t *step_offsets, int64_t nrows,
                     const uint64_t *valid_in, uint64_t *valid_out, hipStream_t s);
void CompactColumns(const CompactDesc &d, int64_t nrows, const unsigned long long *bits, const int64_t *step_offsets,
                    hipStream_t s);
void RebaseOffsets(const int64_t *src, int64_t *dst, int64_t n, int64_t delta, hipStream_t s);

// Values as text in the string wire layout (text_kernels.hip): lengths (text +
// NUL) of every row, then, at each row's exclusive-scan offset, its text and a
// NUL; vbytes (optional) gets the validity byte of every row.
enum TextKind { TEXT_INT = 0, TEXT_BOOL = 1, TEXT_DECIMAL = 2 };
struct TextCol {
  const void *data;
  const uint64_t *valid;
  int32_t phys;   // P_U8 .. P_I128
  int32_t kind;   // TextKind
  int32_t scale;  // TEXT_DECIMAL
};
void TextLengths(const TextCol &c, int64_t n, uint32_t *lens, hipStream_t s);
void TextWrite(const TextCol &c, int64_t n, const int64_t *offsets, char *chars, uint8_t *vbytes, hipStream_t s);
void OffsetsU32(const int64_t *offsets, uint32_t *out, int64_t m, hipStream_t s);

// Count-first compaction, for a conjunction of range predicates whose columns
// are all among the (NULL-free, 4/8-byte) outputs, e.g. SELECT x FROM t WHERE
// x > 24.  A chunk is FC_CHUNK consecutive 256-row steps, owned by one wave in
// both passes (so a wave's stores of a chunk form one contiguous run).
//  1. FilterCountChunks: predicate columns through an LDS-DMA ring; one
//     uint32 count per K1 steps (no per-row bits; K1 = FC_CHUNK by default,
//     one count per chunk), the partial last step's count in counts[CountEntries].
//  2. ScanTileCounts over CountEntries + 1 entries -> offsets and the total.
//  3. CompactRecompute: output columns through an LDS-DMA ring; the predicates
//     are evaluated again on the loaded slices (no bits to read), each selected
//     row goes to offsets[chunk] + its rank in the chunk.
#define FC_CHUNK 8
int64_t CountChunks(int64_t nrows);   // pass-2 chunks of full steps
int64_t CountEntries(int64_t nrows);  // pass-1 count entries (the count array has one more)
void FilterCountChunks(const FilterMultiDesc &d, int64_t nrows, uint32_t *counts, hipStream_t s);
void CompactRecompute(const CompactDesc &d, int64_t nrows, const int64_t *chunk_offsets, hipStream_t s);

// One-pass filter -> compaction (select_kernels.hip, select_rounds): every
// loaded column (the union of the predicate and output columns, 4 or 8 bytes)
// is read from HBM once.  Outputs must have room for every row (the selected
// count is not known up front).
#define SL_MAX_COL 4
#define SL_MAX_OUT 4
struct SelectDesc {
  int32_t ncol;
  int32_t nout;
  struct {
    const void *data;
    int32_t w;        // 4 or 8
    int32_t is_pred;  // lo <= x <= lo + span (x sign-extended for 4 B)
    int32_t narrow;   // select_rounds: an 8-byte column whose values fit int32 (zone map) is staged as int32
    int64_t lo;
    uint64_t span;
    const uint64_t *valid;  // select_rounds: validity words (NULL fails a predicate; outputs carry it), or nullptr
    // select_rounds, a NULL-able output column: 1 = a NULL row is staged as the
    // value `sent` (outside the zone map of the valid rows, in the staged
    // width) instead of with a validity byte of its own; the storer writes
    // validity = (staged != sent) and 0 under NULL
    int32_t vsent;
    int64_t sent;
  } col[SL_MAX_COL];
  int32_t out_col[SL_MAX_OUT];  // index into col[]
  void *dst[SL_MAX_OUT];
  uint8_t *vdst[SL_MAX_OUT];  // select_rounds: one validity byte per output row of a NULL-able output, or nullptr
  // select_rounds: nullptr, or the zone map of the selected rows of every
  // output column c with bit c of zmask: zstats[3c .. 3c + 2] = {min, max,
  // non-NULL count (NULL-able columns only)} (values sign-extended), folded in
  // with atomics - the caller sets them to {INT64_MAX, INT64_MIN, 0} first
  long long *zstats;
  int32_t zmask;
  int32_t zstore;  // 1: the storers fold the zone maps while copying, 0: the loaders
  unsigned long long *dbg;     // nullptr, or 14 counters (MBX_SR_DEBUG)
  unsigned long long *dbg_ts;  // MBX_SR_DEBUG=2: s_memrealtime of every (round, workgroup) publish
};

// Round-synchronous one-pass filter -> compaction (select_kernels.hip,
// select_rounds), one persistent workgroup per CU.  Round r's tile of workgroup g is 4 S steps; a
// workgroup's round count is published as an 8-byte {count, epoch} granule
// and every workgroup reads each round's G granules to place its tile.  ctl:
// SelectRoundsCtlBytes(plan) bytes, zeroed once when allocated and reused
// with a fresh epoch per launch (never 0, never reused).  After the launch
// ctl[0] == epoch means a workgroup gave up (no progress for 100 ms: a
// workgroup was never scheduled) and the outputs are garbage; otherwise
// ctl[1] is the selected-row count.
struct SelectRoundsPlan {
  bool ok;
  int nc, wm, ni, depth, S, H, NL, stg, G, sleep, test_stall, pw;  // wm: bit c = column c is 8 bytes; H: 256-row sub-steps per step
  int NS;  // storer waves (4; 6 with 6 loaders)
  int nv;  // loaded columns with validity words (their 32 B per step ride a second ring)
  int64_t nrounds;
  size_t lds;
};
SelectRoundsPlan PlanSelectRounds(const SelectDesc &d, int64_t nrows);
size_t SelectRoundsCtlBytes(const SelectRoundsPlan &p);
hipError_t SelectRounds(const SelectDesc &d, const SelectRoundsPlan &p, int64_t nrows, unsigned long long *ctl,
                  uint32_t epoch, hipStream_t s);
// bits[i / 64] bit i % 64 = bytes[i] (0/1), for the n output rows of a NULL-able select_rounds output
void PackValidityBytes(const uint8_t *bytes, int64_t n, uint64_t *bits, hipStream_t s);

}  // namespace dev
}  // namespace mbx
