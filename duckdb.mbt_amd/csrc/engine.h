// engine.h — catalog, device column chunks, results and handles behind the
// duckdb_mb_* C-ABI (the objects the reference keeps inside libduckdb).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "plan.h"
#include "types.h"

namespace mbx {

// One column of a device-resident table: Arrow-layout values buffer (256-B
// aligned, allocated with hipMalloc) and an LSB-first validity bitmap in
// 64-bit words (bit = 1 -> valid; same bit order as DuckDB's
// duckdb_validity_row_is_valid, reference duckdb_native.c:530-534).  A null
// validity pointer means "all rows valid".  Strings keep int64 offsets[n+1]
// plus a chars buffer.
struct DevColumn {
  LogicalType type;
  Phys phys = P_I64;
  void *data = nullptr;
  uint64_t *validity = nullptr;
  int64_t *offsets = nullptr;  // P_STR
  char *chars = nullptr;       // P_STR
  int64_t chars_len = 0, chars_cap = 0;
  int64_t capacity = 0;  // rows
  // owners of the buffers above (hipFree, or back to the device pool for the
  // blocks CREATE TABLE AS took over from its query): a result that still
  // reads the column without a copy (a stream, an Arrow result, a LIMIT
  // slice) holds them too, so an append that regrows the column, or a DROP,
  // never frees memory a live result reads
  std::shared_ptr<void> data_owner, validity_owner, offsets_owner, chars_owner;
  // zone-map statistics over all rows (kept by ingest; used by the planner
  // to pick overflow-free accumulators and direct-index group tables)
  bool stats_valid = false;
  i128 imin = 0, imax = 0;
  int64_t null_count = 0;
};

struct Table {
  std::string name;
  std::vector<std::string> col_names;
  std::vector<DevColumn> cols;
  int64_t nrows = 0;
  int device = 0;
  // Sharded table (a connection opened with "gpu_devices"): part i holds a
  // contiguous run of rows on shard i's device; the table's row order is part
  // 0's rows, then part 1's, ...  `cols` then carries only names and types, and
  // nrows is the sum over the parts.
  std::vector<std::shared_ptr<Table>> parts;
  bool sharded() const { return !parts.empty(); }
  ~Table();
};
typedef std::shared_ptr<Table> TablePtr;

struct Catalog {
  std::map<std::string, TablePtr> tables;  // lower-cased name
  int device = 0;
  uint64_t version = 0;  // bumped by CREATE / DROP (a bound plan names TablePtrs)
  TablePtr Find(const std::string &name) const;
};

// Host copy of a result column (after the single D2H of a query).
// Host buffers of materialized results.  Blocks of 1 MiB and more come from a
// process-wide cache of recycled blocks (mmap'd with MADV_HUGEPAGE and
// page-locked for DMA when new, hipHostRegister):
// a 1e6-group result is ~60 MB of host columns, and fresh pages from malloc
// (page faults on first touch, munmap at destroy) cost more than its kernels.
namespace result_blocks {
void *Get(size_t bytes);
void Put(void *p, size_t bytes);
}  // namespace result_blocks
template <class T>
struct ResultAlloc {
  typedef T value_type;
  ResultAlloc() = default;
  template <class U>
  ResultAlloc(const ResultAlloc<U> &) {}
  T *allocate(size_t n) { return (T *)result_blocks::Get(n * sizeof(T)); }
  void deallocate(T *p, size_t n) { result_blocks::Put(p, n * sizeof(T)); }
  // resize() leaves new elements uninitialised (every caller writes them: a
  // DMA or a fill loop), so a 32 MB column is not zeroed before its copy
  template <class U>
  void construct(U *p) noexcept {
    ::new ((void *)p) U;
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new ((void *)p) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const ResultAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const ResultAlloc<U> &) const { return false; }
};
template <class T>
using ResultVec = std::vector<T, ResultAlloc<T>>;

struct HostColumn {
  std::string name;
  LogicalType type;
  Phys phys = P_I64;
  ResultVec<uint8_t> data;           // fixed-width values
  ResultVec<uint8_t> valid;          // 1 byte per row (1 = valid)
  std::vector<int64_t> offsets;      // P_STR
  std::string chars;                 // P_STR
  // cell text formatted on the device (large integer / BOOLEAN / DECIMAL /
  // HUGEINT results of duckdb_mb_query and stream batches): row i's text is
  // text[text_off[i], text_off[i + 1] - 1) (each row's text is followed by a NUL)
  ResultVec<uint32_t> text_off;
  ResultVec<char> text;
  Value Get(int64_t row) const;
  // Text of a non-NULL integer/BOOLEAN/DECIMAL cell written into out (>= 48
  // bytes), spelled as FormatValue(Get(row)); -1 for the other types.
  int FormatInto(int64_t row, char *out) const;
  bool IsNull(int64_t row) const { return !valid.empty() && !valid[row]; }
};

struct MaterializedResult {
  std::vector<HostColumn> cols;
  int64_t nrows = 0;
  std::vector<std::string> formatted;  // optional cache
};
typedef std::shared_ptr<MaterializedResult> ResultPtr;

struct QueryProfile {
  struct Kernel {
    std::string name;
    double ms = 0;
    double bytes = 0;  // algorithmic bytes moved
    int64_t rows = 0;
    int shard = -1, device = -1;  // the shard engine that ran it (gpu_devices), -1: the connection's own
  };
  std::vector<Kernel> kernels;
  double total_ms = 0;
};

struct Database;

// Options a connection was opened with (Config::set keys, reference
// duckdb_native.c:714-747 passes them to duckdb_set_config).
struct Options {
  int device = -1;            // "gpu_device" (default: current HIP device)
  bool profile = false;       // "mbx_profile"
  int threads = 0;            // "threads" (accepted; CPU-side only)
  bool allow_no_gpu = false;  // "mbx_allow_no_gpu": host-constant queries only (tests)
  int64_t appender_flush_rows = 1 << 20;  // "mbx_appender_flush_rows"
  // "gpu_devices": a comma-separated device list (or "all"); two or more
  // entries shard every table across them (a device may repeat: two shards on
  // one GPU, for tests)
  std::vector<int> devices;
  // "mbx_shard_rows": appends fill part i of a sharded table up to this many
  // rows before moving on to part i + 1 (0: appends go to the last part)
  int64_t shard_rows = 0;
  // "mbx_force_peer" (tests): shards on the same device still exchange row
  // results by peer DMA (hipMemcpyPeerAsync), as distinct devices do
  bool force_peer = false;
  // "mbx_combine" = "rccl" (default) | "host": a sharded global aggregate, or
  // a GROUP BY on one integer key, over distinct devices combines its partials
  // with RCCL collectives on the shard devices (rccl_combine.h), once the
  // communicators opened at connect have passed their multi-rank check;
  // "host" (and every shape or device list RCCL does not cover: floating-point
  // partials, non-integer or several keys, same-device shards) merges the
  // partials on the host
  bool combine_rccl = true;
  // "mbx_combine" = "rccl_loopback" (tests only, MBX_EXPERIMENTS=1): the RCCL
  // combine with its two collectives replaced by device copies between the
  // shards' lane buffers, so it runs over same-device shards on one GPU
  bool rccl_loopback = false;
  std::map<std::string, std::string> raw;
};

struct Engine;        // per-connection executor state (device stream, scratch)
namespace rc {
struct Comms;  // RCCL communicators over the shard devices (rccl_combine.h)
struct Init;   // their open, in flight on a helper thread
}
struct ShardWorkers;  // persistent per-shard host threads (executor.cpp)

// Counters of the multi-device path (duckdb_mbx_shard_stats).
struct ShardStats {
  int64_t dispatches = 0;    // ForShards calls (one per sharded statement step)
  int64_t peer_links = 0;    // device pairs with peer access enabled at connect
  int64_t peer_copies = 0;   // buffers moved between shards by peer DMA
  int64_t peer_bytes = 0;
  int64_t host_results = 0;  // sharded aggregates finished on the host (no re-upload)
  double last_dispatch_us = 0;  // wall time of the last ForShards (all shards' work)
  double last_combine_us = 0;   // host merge of the last sharded aggregate
  // the last ForShards, per shard (duckdb_mbx_shard_timings), in us from the
  // dispatch: the worker picked the job up (wake), its plan + launches were
  // queued (launch), its result reached the host (done: kernel + D2H + sync)
  struct Timing {
    int device = -1;
    double wake_us = 0, launch_us = 0, done_us = 0;
  };
  std::vector<Timing> last;
  // the per-shard partial relations of the last sharded aggregate, as they
  // came back from each device before the merge (duckdb_mbx_shard_partial)
  std::vector<ResultPtr> last_partials;
  // mbx_combine=rccl: sharded aggregates combined by RCCL collectives on the
  // shard devices instead of the host merge; fallbacks = combines RCCL should
  // have run but could not (communicators unavailable, a collective failed or
  // timed out); unsupported = shapes / layouts it never covers (host merge)
  int64_t rccl_combines = 0, rccl_fallbacks = 0, rccl_unsupported = 0;
  int64_t rccl_reduces = 0, rccl_allgathers = 0;  // the collective each combine ran
  std::string last_collective;
  bool rccl_prepared_at_connect = false;  // the open started at connect (helper thread)
  double rccl_first_wait_ms = -1;         // how long the first combine waited for it (-1: not yet)
  int64_t rccl_loopbacks = 0;  // of rccl_combines, through the test loopback
  int64_t rccl_group_combines = 0;  // of rccl_combines, GROUP BY relations
  int64_t rccl_errors = 0;     // combines that raised a shard's device error
  int64_t rccl_timeouts = 0;   // collectives aborted after MBX_RCCL_TIMEOUT_MS (then host merge)
  double last_rccl_us = 0;
  std::string rccl_note;  // why the last rccl request fell back (empty: it ran)
};

struct Connection {
  Options opts;
  Catalog catalog;
  std::shared_ptr<Engine> engine;
  QueryProfile last_profile;
  std::vector<QueryProfile::Kernel> profile_history;  // drained by duckdb_mbx_profile_drain
  // gpu_devices: one shard connection (own device, stream, pool and catalog of
  // the table parts) per entry; this connection's engine (on the first device)
  // combines their results
  std::vector<std::unique_ptr<Connection>> shards;
  std::shared_ptr<ShardWorkers> workers;  // declared after shards: stopped before they go
  std::shared_ptr<rc::Comms> rccl;        // mbx_combine=rccl: the communicators, once waited for
  std::shared_ptr<rc::Init> rccl_init;    // their open (started at connect over distinct devices)
  bool rccl_tried = false;
  ShardStats shard_stats;
  int64_t shard_stats_t0 = 0;  // steady-clock ns at the start of the current ForShards
  bool sharded() const { return !shards.empty(); }
  ~Connection();
};
// Opens the shard connections of c (opts.devices) and enables peer access
// between their devices.
void OpenShards(Connection &c);

// A SELECT result left on the device; streams copy it back in batches.
struct DeviceResult;
typedef std::shared_ptr<DeviceResult> DeviceResultPtr;
struct StreamSource {
  std::vector<std::string> names;
  std::vector<LogicalType> types;
  int64_t nrows = 0;
  ResultPtr host;       // host-side result (DDL, constant SELECTs)
  DeviceResultPtr dev;  // device-resident SELECT result
};
StreamSource RunStatementStream(Connection &c, const Statement &st, const std::vector<Value> &params);
StreamSource RunBoundStream(Connection &c, const BoundSelect &b);  // a bound SELECT as a stream source
// rows [start, start + n) of a device result, materialized on the host
ResultPtr FetchDeviceRows(Connection &c, DeviceResult &d, int64_t start, int64_t n);
// Arrow wire form of a 1/4/8-byte device column, NULLs allowed: values with
// NULL slots zeroed into vals, validity bytes into vbytes (if not nullptr).
bool CopyDeviceColumnWire(Connection &c, DeviceResult &d, int col, int phys, void *vals, uint8_t *vbytes);
bool DeviceColumnWireOk(const DeviceResult &d, int col, int phys);  // its precondition
// String wire form ([text \0]..., NULL = "") of an integer / BOOLEAN / DECIMAL /
// HUGEINT device column, formatted on the device: dst(chars) returns where the
// chars (then, when vbytes, n validity bytes) go, or nullptr to give up.
bool DeviceColumnTextOk(const DeviceResult &d, int col);
bool CopyDeviceColumnText(Connection &c, DeviceResult &d, int col, const std::function<uint8_t *(int64_t)> &dst,
                          bool vbytes);

// Runs one statement; returns a materialized result (empty for DDL).
ResultPtr RunStatement(Connection &c, const std::string &sql, const std::vector<Value> &params, int *n_params_out);
ResultPtr RunParsed(Connection &c, const Statement &st, const std::vector<Value> &params);
std::string Explain(Connection &c, const std::string &sql);

// Executor entry points (executor.cpp).
std::shared_ptr<Engine> CreateEngine(int device, bool allow_no_gpu);
ResultPtr ExecuteSelect(Connection &c, const BoundSelect &s);
DeviceResultPtr ExecuteSelectDevice(Connection &c, const BoundSelect &s, StreamSource *meta);
void ExecuteInsertSelect(Connection &c, Table &t, const BoundSelect &s, const std::vector<int> &col_map);
// A table of c: on a sharded connection its parts are created on every shard
// (and registered in the shards' catalogs under the same name).
TablePtr CreateDeviceTable(Connection &c, const std::string &name, const std::vector<std::string> &names,
                           const std::vector<LogicalType> &types);
void DropDeviceTable(Table &t);
int DeviceCount();

// Host staging -> device append (appender, INSERT VALUES).
struct HostBatch {
  std::vector<HostColumn> cols;
  int64_t nrows = 0;
};
void AppendHostBatch(Connection &c, Table &t, const HostBatch &b);
// pinned host memory for appender staging (hipHostMalloc / hipHostFree)
void *HostPinnedAlloc(size_t bytes);
void HostPinnedFree(void *p);
// raw little-endian bytes of a (non-NULL) value already cast to the column type
void ValueToRaw(const Value &v, Phys phys, uint8_t *dst);
// Appends n rows given as host columns in their physical layout (valid[c]:
// per-row bytes or NULL).  sync=false leaves the DMA and the zone-map
// reduction in flight on the connection's stream (the appender's pinned
// double buffer); the next device statement settles them first.
void AppendRawColumns(Connection &c, Table &t, const std::vector<const void *> &vals,
                      const std::vector<const uint8_t *> &valid, int64_t n, bool sync = true);
// waits for in-flight appends and folds their zone-map statistics
void SettleAppends(Connection &c);
void HostColumnPush(HostColumn &col, const Value &v);  // v already of col.type (or NULL)
void HbmCalibrateConn(Connection &c, int64_t bytes, int iters, double out[8]);
// in-kernel clock stamps of the last stamped launch (libduckdb_mb_amd_clk.so)
int ClockStampsConn(Connection &c, uint64_t *out, int cap);
// the connection's RCCL combine as JSON (duckdb_mbx_rccl_info)
std::string RcclInfoJson(Connection &c);
// rc::SelfTest over devs as JSON (duckdb_mbx_rccl_selftest_ex); *err ("" when
// it passed) and the wall us in *us
std::string RcclSelfTestJson(const std::vector<int> &devs, std::string *err, double *us);
// adds this connection's (and its shards') select_rounds counters to out:
// launches, aborts (a workgroup never scheduled: the two-pass form reran), launch failures
void EngineCounters(const Connection &c, int64_t out[3]);

}  // namespace mbx
