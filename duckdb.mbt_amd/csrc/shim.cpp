// shim.cpp — the 89 duckdb_mb_* C-ABI entry points (include/duckdb_mb.h).
//
// Same names, parameter types, ownership and error conventions as the
// reference shim /root/reference/src/duckdb_native.c (each function cites the
// definition it replaces).  Instead of forwarding to libduckdb, statements go
// to the MI355X engine (engine.cpp / executor.cpp / kernels.hip).
//
// Deliberate differences (documented in DESIGN.md):
//  * the last-error string is thread_local (reference: process-global static,
//    duckdb_native.c:22-40) — identical for the single-threaded MoonBit caller;
//  * duckdb_mb_query_arrow does not read freed memory on error
//    (reference use-after-free at duckdb_native.c:2258-2260);
//  * arrow buffer sizes are computed in 64 bits and refused at 2^28 bytes (the
//    MoonBit byte-object length field; see MbTooBig)
//    (reference int32 overflow at duckdb_native.c:2404).
#include <hip/hip_runtime_api.h>

#include <immintrin.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/duckdb_mb.h"
#include "combine.h"
#include "engine.h"
#include "jit.h"
#include "knobs.h"
#include "hostlink.h"

using namespace mbx;

// ---------------------------------------------------------------------------
// MoonBit byte objects.  Layout of the MoonBit runtime (moonbit.h): an 8-byte
// header {int32 rc; uint32 meta} precedes the payload and the array length is
// the low 28 bits of meta (Moonbit_array_length).  Inside a MoonBit program
// the runtime's strong moonbit_make_bytes_raw wins over this weak one.
// ---------------------------------------------------------------------------
namespace {
struct MbHeader {
  int32_t rc;
  uint32_t meta;
};
inline int32_t MbLen(const uint8_t *b) {
  if (!b) return 0;
  return (int32_t)(((const MbHeader *)b - 1)->meta & ((1u << 28) - 1));
}
}  // namespace

extern "C" __attribute__((weak)) moonbit_bytes_t moonbit_make_bytes_raw(int32_t len) {
  if (len < 0) len = 0;
  MbHeader *h = (MbHeader *)calloc(1, sizeof(MbHeader) + (size_t)len + 1);
  if (!h) return nullptr;
  h->rc = 1;
  h->meta = (uint32_t)len & ((1u << 28) - 1);
  return (moonbit_bytes_t)(h + 1);
}

extern "C" moonbit_bytes_t duckdb_mbx_bytes_new(const uint8_t *data, int32_t len) {
  moonbit_bytes_t b = moonbit_make_bytes_raw(len);
  if (b && len > 0 && data) memcpy(b, data, (size_t)len);
  return b;
}
extern "C" int32_t duckdb_mbx_bytes_len(moonbit_bytes_t b) { return MbLen(b); }
extern "C" void duckdb_mbx_bytes_free(moonbit_bytes_t b) {
  if (b) free((MbHeader *)b - 1);
}
// Drops a Bytes this library allocated and will not return (an error path):
// the MoonBit runtime's own moonbit_decref when linked into a MoonBit program,
// else (this weak definition, test harnesses) the matching free.
extern "C" __attribute__((weak)) void moonbit_decref(void *obj) {
  if (obj) free((MbHeader *)obj - 1);
}

// A MoonBit byte object's length is the low 28 bits of its header word, so a
// getter buffer must stay below 2^28 bytes (a longer one would read back with a
// truncated length): refused with an error instead.
constexpr int64_t kMbMaxBytes = (1 << 28) - 1;
static void SetError(const std::string &msg);
static bool MbTooBig(int64_t total) {
  if (total <= kMbMaxBytes) return false;
  SetError("Invalid Input Error: arrow buffer of " + std::to_string(total) +
           " bytes exceeds the 2^28-byte limit of one MoonBit Bytes object");
  return true;
}

static moonbit_bytes_t MakeBytes(const char *data, size_t len) {
  moonbit_bytes_t b = moonbit_make_bytes_raw((int32_t)len);
  if (b && len && data) memcpy(b, data, len);
  return b;
}
static moonbit_bytes_t MakeBytes(const std::string &s) { return MakeBytes(s.data(), s.size()); }
static std::string BytesStr(moonbit_bytes_t b) {
  if (!b) return std::string();
  return std::string((const char *)b, (size_t)MbLen(b));
}

// ---------------------------------------------------------------------------
// handles
// ---------------------------------------------------------------------------
struct duckdb_mb_connection {
  Connection conn;
};
struct duckdb_mb_result {
  ResultPtr r;
};
// A stream reads a device-resident SELECT result back in batches of
// kStreamBatch rows (one pinned D2H each) and serves 2048-row chunks from the
// current batch; host-side results (DDL, constant SELECTs) are served as is.
struct duckdb_mb_stream {
  duckdb_mb_connection *conn = nullptr;
  std::vector<std::string> names;
  std::vector<LogicalType> types;
  int64_t nrows = 0;
  DeviceResultPtr dev;
  ResultPtr r;  // host result, or the current batch of a device result
  int64_t batch_start = 0;
  int64_t pos = 0;
};
struct duckdb_mb_chunk {
  ResultPtr r;
  int64_t start = 0, n = 0;
  duckdb_mb_stream *stream = nullptr;
};
struct duckdb_mb_config {
  Options opts;
  char error[256];
};
struct duckdb_mb_statement {
  duckdb_mb_connection *conn = nullptr;
  Statement st;
  std::vector<Value> params;
  char error[256];
  // bound-plan cache (SELECT): the plan of the last execute and the constant
  // node of each parameter; re-executed with new values of the same types (and
  // an unchanged catalog) by overwriting those nodes instead of binding again
  BoundSelectPtr plan;
  std::vector<std::pair<BExprPtr, int>> plan_params;
  std::vector<LogicalType> plan_types;
  std::vector<bool> plan_nulls;
  uint64_t plan_version = 0;
  uint64_t binds = 0, reuses = 0;  // statistics (duckdb_mbx_statement_plan_stats)
};
struct duckdb_mb_appender {
  duckdb_mb_connection *conn = nullptr;
  TablePtr table;
  HostBatch batch;  // VARCHAR tables: rows staged in host vectors
  size_t col = 0;
  char error[256];
  // Fixed-width tables stage rows in two pinned buffers per column: while one
  // fills, the other's DMA into the device column (and its zone-map
  // reduction) is in flight on the connection's stream.
  bool pinned = false;
  std::vector<char *> pbuf[2];
  std::vector<int> pw;                        // bytes per value, per column
  std::vector<std::vector<uint8_t>> pvalid;   // per column: empty (all valid) or a byte per row
  int pcur = 0;
  int64_t prow = 0, pcap = 0;
  // columnar bulk ingest
  std::vector<const void *> raw_vals;
  std::vector<const uint8_t *> raw_valid;
  std::vector<int64_t> raw_count;
  ~duckdb_mb_appender() {
    for (int b = 0; b < 2; b++)
      for (char *p : pbuf[b]) HostPinnedFree(p);
  }
};
// The query's result stays on the device: fixed-width getters of columns
// without NULLs DMA straight into the returned Bytes; the others materialize
// the result on the host once (lazily) and convert per cell like the
// reference's duckdb_value_* calls.
struct duckdb_mb_arrow_result {
  duckdb_mb_connection *conn = nullptr;
  DeviceResultPtr dev;
  std::vector<std::string> names;
  std::vector<LogicalType> types;
  ResultPtr r;  // host copy (lazy for device results)
  char error[256];
  int32_t column_count = 0, row_count = 0;
};

static thread_local std::string g_last_error;
static thread_local bool g_has_error = false;

static void SetError(const char *m) {
  if (!m) {
    g_last_error.clear();
    g_has_error = false;
    return;
  }
  g_last_error = m;
  g_has_error = true;
}
static void SetError(const std::string &m) { SetError(m.c_str()); }
static void CopyErr(char *dst, const std::string &m) {
  strncpy(dst, m.c_str(), 255);
  dst[255] = '\0';
}

extern "C" {

// ---- connection -------------------------------------------------------------
static duckdb_mb_connection *OpenConn(moonbit_bytes_t path, const Options &opts) {
  try {
    auto *h = new duckdb_mb_connection();
    h->conn.opts = opts;
    if (opts.devices.size() >= 2) h->conn.opts.device = opts.devices[0];  // the combining device
    h->conn.engine = CreateEngine(h->conn.opts.device, opts.allow_no_gpu);
    h->conn.catalog.device = h->conn.opts.device;
    if (opts.devices.size() >= 2) OpenShards(h->conn);
    (void)path;  // ":memory:" and file paths both open a volatile device-resident database
    return h;
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

duckdb_mb_connection *duckdb_mb_connect(moonbit_bytes_t path) {  // ref duckdb_native.c:67-131
  Options o;
  return OpenConn(path, o);
}

void duckdb_mb_disconnect(duckdb_mb_connection *h) {  // ref :133-140
  jit::JoinPending();
  delete h;
}

int32_t duckdb_mb_is_null_conn(duckdb_mb_connection *h) { return h == nullptr ? 1 : 0; }  // ref :248

moonbit_bytes_t duckdb_mb_last_error(void) {  // ref :240-246
  if (!g_has_error) return moonbit_make_bytes_raw(0);
  return MakeBytes(g_last_error);
}

// ---- materialized query --------------------------------------------------
duckdb_mb_result *duckdb_mb_query(duckdb_mb_connection *h, moonbit_bytes_t sql) {  // ref :142-172
  if (!h) {
    SetError("connection is null");
    return nullptr;
  }
  try {
    ResultPtr r = RunStatement(h->conn, BytesStr(sql), {}, nullptr);
    auto *res = new duckdb_mb_result();
    res->r = r;
    return res;
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

void duckdb_mb_result_destroy(duckdb_mb_result *r) { delete r; }  // ref :174-180

int32_t duckdb_mb_result_column_count(duckdb_mb_result *r) {  // ref :182-187
  return r ? (int32_t)r->r->cols.size() : 0;
}
int32_t duckdb_mb_result_row_count(duckdb_mb_result *r) {  // ref :189-194
  return r ? (int32_t)r->r->nrows : 0;
}
moonbit_bytes_t duckdb_mb_result_column_name(duckdb_mb_result *r, int32_t col) {  // ref :196-206
  if (!r || col < 0 || col >= (int32_t)r->r->cols.size()) return moonbit_make_bytes_raw(0);
  return MakeBytes(r->r->cols[col].name);
}
int32_t duckdb_mb_result_column_type(duckdb_mb_result *r, int32_t col) {  // ref :208-213
  if (!r || col < 0 || col >= (int32_t)r->r->cols.size()) return T_INVALID;
  return r->r->cols[col].type.id;
}
static bool InRange(const ResultPtr &r, int32_t col, int64_t row) {
  return col >= 0 && col < (int32_t)r->cols.size() && row >= 0 && row < r->nrows;
}
int32_t duckdb_mb_result_is_null(duckdb_mb_result *r, int32_t col, int32_t row) {  // ref :215-222
  if (!r || !InRange(r->r, col, row)) return 1;
  return r->r->cols[col].IsNull(row) ? 1 : 0;
}
moonbit_bytes_t duckdb_mb_result_value(duckdb_mb_result *r, int32_t col, int32_t row) {  // ref :224-238
  if (!r || !InRange(r->r, col, row)) return moonbit_make_bytes_raw(0);
  const HostColumn &c = r->r->cols[col];
  if (c.IsNull(row)) return moonbit_make_bytes_raw(0);
  char buf[48];
  const int n = c.FormatInto(row, buf);
  if (n >= 0) return MakeBytes(buf, (size_t)n);
  return MakeBytes(FormatValue(c.Get(row)));
}
int32_t duckdb_mb_is_null_result(duckdb_mb_result *r) { return r == nullptr ? 1 : 0; }  // ref :252

// ---- streaming --------------------------------------------------------------
// Whitelist of streamable types, reference duckdb_native.c:271-303.
static bool StreamSupported(TypeId t) {
  switch (t) {
    case T_BOOLEAN: case T_TINYINT: case T_SMALLINT: case T_INTEGER: case T_BIGINT: case T_UTINYINT:
    case T_USMALLINT: case T_UINTEGER: case T_UBIGINT: case T_FLOAT: case T_DOUBLE: case T_VARCHAR: case T_BLOB:
    case T_DATE: case T_TIME: case T_TIMESTAMP: case T_INTERVAL: case T_HUGEINT:
      return true;
    default:
      return false;
  }
}

static duckdb_mb_stream *StreamFrom(duckdb_mb_connection *h, StreamSource src) {  // ref :320-353
  for (auto &t : src.types)
    if (!StreamSupported(t.id)) {
      SetError("streaming query has unsupported column type");
      return nullptr;
    }
  auto *s = new duckdb_mb_stream();
  s->conn = h;
  s->names = std::move(src.names);
  s->types = std::move(src.types);
  s->nrows = src.nrows;
  s->dev = src.dev;
  s->r = src.host;
  return s;
}

duckdb_mb_stream *duckdb_mb_query_stream(duckdb_mb_connection *h, moonbit_bytes_t sql) {  // ref :355-397
  if (!h) {
    SetError("connection is null");
    return nullptr;
  }
  try {
    Statement st = ParseSQL(BytesStr(sql));
    return StreamFrom(h, RunStatementStream(h->conn, st, {}));
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

void duckdb_mb_stream_destroy(duckdb_mb_stream *s) { delete s; }  // ref :426-438
int32_t duckdb_mb_is_null_stream(duckdb_mb_stream *s) { return s == nullptr ? 1 : 0; }  // ref :440
int32_t duckdb_mb_stream_column_count(duckdb_mb_stream *s) {  // ref :444-449
  return s ? (int32_t)s->names.size() : 0;
}
moonbit_bytes_t duckdb_mb_stream_column_name(duckdb_mb_stream *s, int32_t col) {  // ref :451-464
  if (!s || col < 0 || col >= (int32_t)s->names.size()) return moonbit_make_bytes_raw(0);
  return MakeBytes(s->names[col]);
}

// DuckDB's standard vector size: result chunks carry at most 2048 rows.
static const int64_t kVectorSize = 2048;
// rows per device->host batch of a streamed device result (32 vectors)
static const int64_t kStreamBatch = 32 * kVectorSize;

duckdb_mb_chunk *duckdb_mb_stream_fetch_chunk(duckdb_mb_stream *s) {  // ref :466-490
  if (!s) {
    SetError("stream is null");
    return nullptr;
  }
  if (s->pos >= s->nrows) {
    SetError(nullptr);  // end of stream: NULL chunk with an empty error
    return nullptr;
  }
  if (s->dev && (!s->r || s->pos >= s->batch_start + s->r->nrows)) {
    try {
      s->r = FetchDeviceRows(s->conn->conn, *s->dev, s->pos, std::min(kStreamBatch, s->nrows - s->pos));
      s->batch_start = s->pos;
    } catch (std::exception &e) {
      SetError(e.what());
      return nullptr;
    }
  }
  auto *c = new duckdb_mb_chunk();
  c->r = s->r;
  c->start = s->pos - s->batch_start;
  c->n = std::min(kVectorSize, s->nrows - s->pos);
  c->stream = s;
  s->pos += c->n;
  return c;
}

void duckdb_mb_chunk_destroy(duckdb_mb_chunk *c) { delete c; }  // ref :492-500
int32_t duckdb_mb_is_null_chunk(duckdb_mb_chunk *c) { return c == nullptr ? 1 : 0; }  // ref :502
int32_t duckdb_mb_chunk_row_count(duckdb_mb_chunk *c) { return c ? (int32_t)c->n : 0; }  // ref :506-511
int32_t duckdb_mb_chunk_column_count(duckdb_mb_chunk *c) {  // ref :513-518
  return c ? (int32_t)c->r->cols.size() : 0;
}
int32_t duckdb_mb_chunk_is_null(duckdb_mb_chunk *c, int32_t col, int32_t row) {  // ref :520-535
  if (!c || col < 0 || col >= (int32_t)c->r->cols.size() || row < 0 || row >= c->n) return 1;
  return c->r->cols[col].IsNull(c->start + row) ? 1 : 0;
}
moonbit_bytes_t duckdb_mb_chunk_value(duckdb_mb_chunk *c, int32_t col, int32_t row) {  // ref :537-667
  if (!c || col < 0 || col >= (int32_t)c->r->cols.size() || row < 0 || row >= c->n) return moonbit_make_bytes_raw(0);
  const HostColumn &hc = c->r->cols[col];
  if (hc.IsNull(c->start + row)) return moonbit_make_bytes_raw(0);
  char buf[48];
  const int n = hc.FormatInto(c->start + row, buf);
  if (n >= 0) return MakeBytes(buf, (size_t)n);
  return MakeBytes(FormatValue(hc.Get(c->start + row)));
}

// ---- configuration -----------------------------------------------------------
duckdb_mb_config *duckdb_mb_config_create(void) {  // ref :678-695
  auto *c = new duckdb_mb_config();
  c->error[0] = '\0';
  return c;
}
void duckdb_mb_config_destroy(duckdb_mb_config *c) { delete c; }  // ref :697-705
moonbit_bytes_t duckdb_mb_config_error(duckdb_mb_config *c) {  // ref :707-712
  if (!c) return MakeBytes("", 0);
  return MakeBytes(c->error, strlen(c->error));
}

static bool IsInt(const std::string &v, long long *out) {
  char *end = nullptr;
  long long x = strtoll(v.c_str(), &end, 10);
  if (v.empty() || *end) return false;
  *out = x;
  return true;
}

int32_t duckdb_mb_config_set(duckdb_mb_config *c, moonbit_bytes_t key, moonbit_bytes_t value) {  // ref :714-747
  if (!c) return 0;
  std::string k = BytesStr(key), v = BytesStr(value);
  std::string kl = k;
  for (auto &ch : kl) ch = (char)tolower((unsigned char)ch);
  long long x;
  bool ok = true;
  if (kl == "gpu_device") {
    ok = IsInt(v, &x) && x >= 0;
    if (ok) c->opts.device = (int)x;
  } else if (kl == "gpu_devices") {  // shard every table across these devices
    std::vector<int> devs;
    std::string vl = v;
    for (auto &ch : vl) ch = (char)tolower((unsigned char)ch);
    if (vl == "all") {
      for (int d = 0; d < DeviceCount(); d++) devs.push_back(d);
      ok = !devs.empty();
    } else {
      size_t at = 0;
      while (ok && at <= v.size()) {
        size_t comma = v.find(',', at);
        if (comma == std::string::npos) comma = v.size();
        std::string item = v.substr(at, comma - at);
        while (!item.empty() && item.front() == ' ') item.erase(item.begin());
        while (!item.empty() && item.back() == ' ') item.pop_back();
        ok = IsInt(item, &x) && x >= 0 && devs.size() < 64;
        if (ok) devs.push_back((int)x);
        at = comma + 1;
      }
    }
    if (ok) {
      c->opts.devices = devs.size() >= 2 ? devs : std::vector<int>();
      c->opts.device = devs[0];
    }
  } else if (kl == "mbx_shard_rows") {
    ok = IsInt(v, &x) && x >= 0;
    if (ok) c->opts.shard_rows = x;
  } else if (kl == "mbx_combine") {
    // rccl_loopback: the test-only stand-in for the collectives (rccl_combine.h)
    ok = v == "host" || v == "rccl" || (v == "rccl_loopback" && mbx::Knob("MBX_EXPERIMENTS"));
    if (ok) c->opts.combine_rccl = v != "host", c->opts.rccl_loopback = v == "rccl_loopback";
  } else if (kl == "mbx_force_peer") {
    c->opts.force_peer = v == "true" || v == "1";
  } else if (kl == "mbx_profile") {
    c->opts.profile = v == "true" || v == "1";
  } else if (kl == "mbx_allow_no_gpu") {
    c->opts.allow_no_gpu = v == "true" || v == "1";
  } else if (kl == "mbx_appender_flush_rows") {
    ok = IsInt(v, &x) && x > 0;
    if (ok) c->opts.appender_flush_rows = x;
  } else if (kl == "threads" || kl == "worker_threads") {
    ok = IsInt(v, &x) && x > 0;
    if (ok) c->opts.threads = (int)x;
  } else if (kl == "access_mode") {
    std::string vl = v;
    for (auto &ch : vl) ch = (char)tolower((unsigned char)ch);
    ok = vl == "automatic" || vl == "read_only" || vl == "read_write";
  } else if (kl == "memory_limit" || kl == "max_memory" || kl == "default_order" || kl == "default_null_order" ||
             kl == "enable_external_access" || kl == "allow_unsigned_extensions" || kl == "temp_directory" ||
             kl == "preserve_insertion_order" || kl == "enable_object_cache" || kl == "max_temp_directory_size" ||
             kl == "enable_progress_bar" || kl == "autoload_known_extensions" || kl == "autoinstall_known_extensions") {
    ok = true;
  } else {
    ok = false;
  }
  if (!ok) {
    CopyErr(c->error, "duckdb_set_config failed");
    return 0;
  }
  c->opts.raw[kl] = v;
  return 1;
}

duckdb_mb_connection *duckdb_mb_connect_with_config(moonbit_bytes_t path, duckdb_mb_config *c) {  // ref :749-806
  if (!c) {
    SetError("config is null");
    return nullptr;
  }
  return OpenConn(path, c->opts);
}

// ---- prepared statements -------------------------------------------------------
duckdb_mb_statement *duckdb_mb_prepare(duckdb_mb_connection *h, moonbit_bytes_t sql) {  // ref :816-854
  if (!h) return nullptr;
  try {
    auto *s = new duckdb_mb_statement();
    s->conn = h;
    s->st = ParseSQL(BytesStr(sql));
    s->params.assign(s->st.n_params, Value());  // type INVALID = unbound
    s->error[0] = '\0';
    return s;
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

void duckdb_mb_statement_destroy(duckdb_mb_statement *s) { delete s; }  // ref :856-864
moonbit_bytes_t duckdb_mb_statement_error(duckdb_mb_statement *s) {  // ref :866-871
  if (!s) return MakeBytes("", 0);
  return MakeBytes(s->error, strlen(s->error));
}

static int32_t Bind(duckdb_mb_statement *s, int32_t index, const Value &v) {
  if (!s) return 0;
  if (index < 1 || index > (int32_t)s->params.size()) {
    CopyErr(s->error, "Can not bind to parameter number " + std::to_string(index) + ", statement only has " +
                          std::to_string(s->params.size()) + " parameter(s)");
    return 0;
  }
  s->params[index - 1] = v;
  return 1;
}

int32_t duckdb_mb_bind_int(duckdb_mb_statement *s, int32_t i, int32_t v) { return Bind(s, i, Value::Int(T_INTEGER, v)); }  // ref :873
int32_t duckdb_mb_bind_bigint(duckdb_mb_statement *s, int32_t i, int64_t v) { return Bind(s, i, Value::Int(T_BIGINT, v)); }  // ref :890
int32_t duckdb_mb_bind_double(duckdb_mb_statement *s, int32_t i, double v) { return Bind(s, i, Value::Double(v)); }  // ref :907
int32_t duckdb_mb_bind_varchar(duckdb_mb_statement *s, int32_t i, moonbit_bytes_t v) {  // ref :924
  return Bind(s, i, Value::Varchar(BytesStr(v)));
}
int32_t duckdb_mb_bind_bool(duckdb_mb_statement *s, int32_t i, bool v) { return Bind(s, i, Value::Bool(v)); }  // ref :950
int32_t duckdb_mb_bind_null(duckdb_mb_statement *s, int32_t i) {  // ref :967
  return Bind(s, i, Value::Null(LogicalType(T_SQLNULL)));
}
int32_t duckdb_mb_clear_bindings(duckdb_mb_statement *s) {  // ref :983-989
  if (!s) return 0;
  for (auto &p : s->params) p = Value();
  return 1;
}

// The bound plan of a SELECT statement for its current parameters: the cached
// one with the parameter nodes overwritten when the parameter types and the
// catalog are unchanged (MBX_PLAN_CACHE=0 disables), else a fresh bind.
static BoundSelectPtr PlanFor(duckdb_mb_statement *s) {
  Connection &c = s->conn->conn;
  const char *pc = Knob("MBX_PLAN_CACHE");
  const bool off = pc && atoi(pc) == 0;
  bool same = !off && s->plan && s->plan_version == c.catalog.version && s->plan_types.size() == s->params.size();
  for (size_t i = 0; same && i < s->params.size(); i++)
    same = s->params[i].type == s->plan_types[i] && s->params[i].is_null == s->plan_nulls[i] &&
           s->params[i].type.id != T_INVALID;
  if (same) {
    for (auto &pn : s->plan_params) pn.first->cval = CastValue(s->params[pn.second], pn.first->type);
    s->reuses++;
    return s->plan;
  }
  bool patchable = false;
  std::vector<std::pair<BExprPtr, int>> nodes;
  BoundSelectPtr b = BindSelectCapture(*s->st.select, c.catalog, s->params, &patchable, &nodes);
  s->binds++;
  s->plan.reset();
  if (patchable && !off) {
    s->plan = b;
    s->plan_params = nodes;
    s->plan_version = c.catalog.version;
    s->plan_types.clear();
    s->plan_nulls.clear();
    for (auto &v : s->params) {
      s->plan_types.push_back(v.type);
      s->plan_nulls.push_back(v.is_null);
    }
  }
  return b;
}

duckdb_mb_result *duckdb_mb_execute_prepared(duckdb_mb_statement *s) {  // ref :991-1016
  if (!s) {
    SetError("statement is null");
    return nullptr;
  }
  try {
    ResultPtr r = s->st.kind == Statement::SELECT ? ExecuteSelect(s->conn->conn, *PlanFor(s))
                                                   : RunParsed(s->conn->conn, s->st, s->params);
    auto *res = new duckdb_mb_result();
    res->r = r;
    return res;
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

duckdb_mb_stream *duckdb_mb_execute_prepared_stream(duckdb_mb_statement *s) {  // ref :399-424
  if (!s) {
    SetError("statement is null");
    return nullptr;
  }
  try {
    if (s->st.kind == Statement::SELECT) return StreamFrom(s->conn, RunBoundStream(s->conn->conn, *PlanFor(s)));
    return StreamFrom(s->conn, RunStatementStream(s->conn->conn, s->st, s->params));
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

int32_t duckdb_mb_is_null_statement(duckdb_mb_statement *s) { return s == nullptr ? 1 : 0; }  // ref :1018

int32_t duckdb_mbx_statement_plan_stats(duckdb_mb_statement *s, int64_t *out2) {
  if (!s || !out2) return 0;
  out2[0] = (int64_t)s->binds;
  out2[1] = (int64_t)s->reuses;
  return 1;
}

int32_t duckdb_mb_bind_date(duckdb_mb_statement *s, int32_t i, int32_t days) {  // ref :1261
  return Bind(s, i, Value::Int(T_DATE, days));
}
int32_t duckdb_mb_bind_timestamp(duckdb_mb_statement *s, int32_t i, int64_t micros) {  // ref :1279
  return Bind(s, i, Value::Int(T_TIMESTAMP, micros));
}
int32_t duckdb_mb_bind_blob(duckdb_mb_statement *s, int32_t i, moonbit_bytes_t data, int32_t length) {  // ref :1377
  Value v = Value::Varchar(std::string((const char *)data, data ? (size_t)std::max(length, 0) : 0));
  v.type = LogicalType(T_BLOB);
  return Bind(s, i, v);
}
static i128 HugeFromParts(int64_t lower, int64_t upper) {
  return (i128)(((u128)(uint64_t)upper << 64) | (uint64_t)lower);
}
int32_t duckdb_mb_bind_decimal(duckdb_mb_statement *s, int32_t i, uint8_t width, uint8_t scale, int64_t lower,
                               int64_t upper) {  // ref :1421-1445
  if (width < 1 || width > 38 || scale > width) {
    if (s) CopyErr(s->error, "Invalid Input Error: invalid decimal width/scale");
    return 0;
  }
  return Bind(s, i, Value::Decimal(width, scale, HugeFromParts(lower, upper)));
}
int32_t duckdb_mb_bind_interval(duckdb_mb_statement *s, int32_t i, int32_t months, int32_t days, int64_t micros) {  // ref :1487
  Value v;
  v.type = LogicalType(T_INTERVAL);
  v.is_null = false;
  v.iv.months = months;
  v.iv.days = days;
  v.iv.micros = micros;
  return Bind(s, i, v);
}
static int32_t Unsupported(char *err, const char *what) {
  if (err) CopyErr(err, std::string("Not implemented Error: ") + what + " is not supported by the MI355X backend");
  return 0;
}
int32_t duckdb_mb_bind_list_varchar(duckdb_mb_statement *s, int32_t, moonbit_bytes_t *, int32_t) {  // ref :1539
  return Unsupported(s ? s->error : nullptr, "LIST parameters");
}
int32_t duckdb_mb_bind_struct_varchar(duckdb_mb_statement *s, int32_t, moonbit_bytes_t *, moonbit_bytes_t *, int32_t) {  // ref :1597
  return Unsupported(s ? s->error : nullptr, "STRUCT parameters");
}
int32_t duckdb_mb_bind_map_varchar_varchar(duckdb_mb_statement *s, int32_t, moonbit_bytes_t *, moonbit_bytes_t *, int32_t) {  // ref :1666
  return Unsupported(s ? s->error : nullptr, "MAP parameters");
}

// ---- appender ----------------------------------------------------------------
duckdb_mb_appender *duckdb_mb_appender_create(duckdb_mb_connection *h, moonbit_bytes_t schema, moonbit_bytes_t table) {  // ref :1032-1081
  if (!h) return nullptr;
  std::string sc = BytesStr(schema), tn = BytesStr(table);
  TablePtr t = h->conn.catalog.Find(tn);
  if (!t || (!sc.empty() && sc != "main")) {
    SetError("Catalog Error: Table \"" + (sc.empty() ? std::string("main") : sc) + "." + tn + "\" could not be found");
    return nullptr;
  }
  auto *a = new duckdb_mb_appender();
  a->conn = h;
  a->table = t;
  a->error[0] = '\0';
  a->pinned = !t->cols.empty();
  for (auto &c : t->cols) {
    HostColumn hc;
    hc.type = c.type;
    hc.phys = c.phys;
    if (hc.phys == P_STR) hc.offsets.push_back(0);
    a->batch.cols.push_back(hc);
    if (c.phys == P_STR) a->pinned = false;
    a->pw.push_back(c.phys == P_STR ? 0 : PhysSize(c.phys));
  }
  a->pvalid.resize(t->cols.size());
  return a;
}

// the current pinned buffer's complete rows -> the device (async unless
// sync); then the other buffer, whose DMA the append path has settled
static bool FlushPinned(duckdb_mb_appender *a, bool sync) {
  if (a->prow > 0) {
    std::vector<const void *> vals;
    std::vector<const uint8_t *> valid;
    for (size_t c = 0; c < a->pw.size(); c++) {
      vals.push_back(a->pbuf[a->pcur][c]);
      valid.push_back(a->pvalid[c].empty() ? nullptr : a->pvalid[c].data());
    }
    try {
      AppendRawColumns(a->conn->conn, *a->table, vals, valid, a->prow, sync);
    } catch (std::exception &e) {
      CopyErr(a->error, e.what());
      return false;
    }
    a->pcur ^= 1;
    a->prow = 0;
    for (auto &v : a->pvalid) v.clear();
  }
  if (sync) {
    try {
      SettleAppends(a->conn->conn);
    } catch (std::exception &e) {
      CopyErr(a->error, e.what());
      return false;
    }
  }
  return true;
}

// pinned slot of the current row for column `c` (allocated on first use)
static uint8_t *PinnedSlot(duckdb_mb_appender *a, size_t c) {
  if (a->pcap == 0) {
    int64_t row_bytes = 0;
    for (int w : a->pw) row_bytes += w;
    // the flush size, capped at 32 MB of pinned staging per buffer
    a->pcap = std::max<int64_t>(1, std::min<int64_t>(a->conn->conn.opts.appender_flush_rows,
                                                     std::max<int64_t>(1024, ((int64_t)32 << 20) / row_bytes)));
    for (int b = 0; b < 2; b++)
      for (int w : a->pw) a->pbuf[b].push_back((char *)HostPinnedAlloc((size_t)a->pcap * w));
  }
  return (uint8_t *)a->pbuf[a->pcur][c] + (size_t)a->prow * a->pw[c];
}

static void PinnedValid(duckdb_mb_appender *a, size_t c, bool valid) {
  auto &v = a->pvalid[c];
  if (valid && v.empty()) return;
  if (v.empty()) v.assign((size_t)a->prow, 1);
  v.resize((size_t)a->prow);  // drop a stale byte of an abandoned partial row
  v.push_back(valid ? 1 : 0);
}

static bool FlushAppender(duckdb_mb_appender *a) {
  if (a->pinned) return FlushPinned(a, true);
  // a partial row (destroy with a row half appended) stays out of the flush
  for (auto &hc : a->batch.cols) {
    const size_t n = (size_t)a->batch.nrows;
    if (hc.phys == P_STR) {
      if (hc.offsets.size() > n + 1) {
        hc.offsets.resize(n + 1);
        hc.chars.resize((size_t)hc.offsets[n]);
      }
    } else if (hc.data.size() > n * PhysSize(hc.phys)) {
      hc.data.resize(n * PhysSize(hc.phys));
    }
    if (hc.valid.size() > n) hc.valid.resize(n);
  }
  if (a->batch.nrows == 0) return true;
  try {
    AppendHostBatch(a->conn->conn, *a->table, a->batch);
  } catch (std::exception &e) {
    CopyErr(a->error, e.what());
    return false;
  }
  for (auto &hc : a->batch.cols) {
    hc.data.clear();
    hc.valid.clear();
    hc.chars.clear();
    hc.offsets.clear();
    if (hc.phys == P_STR) hc.offsets.push_back(0);
  }
  a->batch.nrows = 0;
  return true;
}

void duckdb_mb_appender_destroy(duckdb_mb_appender *a) {  // ref :1083-1091 (destroy flushes)
  if (!a) return;
  FlushAppender(a);
  delete a;
}
moonbit_bytes_t duckdb_mb_appender_error(duckdb_mb_appender *a) {  // ref :1093-1098
  if (!a) return MakeBytes("", 0);
  return MakeBytes(a->error, strlen(a->error));
}
int32_t duckdb_mb_begin_row(duckdb_mb_appender *a) {  // ref :1100-1114
  if (!a) return 0;
  return 1;
}

// Values go straight into the batch's column buffers (a flush happens only at
// a row boundary, so a partial row never reaches the device); the integer
// appends into a column of their own width skip the Value round trip.
static int32_t AppendValue(duckdb_mb_appender *a, const Value &v) {
  if (!a) return 0;
  if (a->col >= a->table->cols.size()) {
    CopyErr(a->error, "Too many appends for chunk!");
    return 0;
  }
  try {
    Value cv = CastValue(v, a->table->cols[a->col].type);
    if (a->pinned) {
      if (cv.is_null) {
        memset(PinnedSlot(a, a->col), 0, a->pw[a->col]);
        PinnedValid(a, a->col, false);
      } else {
        ValueToRaw(cv, a->batch.cols[a->col].phys, PinnedSlot(a, a->col));
        PinnedValid(a, a->col, true);
      }
    } else {
      HostColumnPush(a->batch.cols[a->col], cv);
    }
  } catch (std::exception &e) {
    CopyErr(a->error, e.what());
    return 0;
  }
  a->col++;
  return 1;
}

// 1: appended; -1: not this column's exact type (or it has NULLs) -> AppendValue
static inline int32_t AppendRaw(duckdb_mb_appender *a, const void *v, int sz, TypeId tid, Phys phys) {
  if (a && a->col < a->batch.cols.size()) {
    HostColumn &hc = a->batch.cols[a->col];
    if (a->pinned && hc.phys == phys && hc.type.id == tid) {
      memcpy(PinnedSlot(a, a->col), v, sz);
      PinnedValid(a, a->col, true);
      a->col++;
      return 1;
    }
    if (hc.phys == phys && hc.type.id == tid && hc.valid.empty()) {
      const size_t at = hc.data.size();
      hc.data.resize(at + sz);
      memcpy(hc.data.data() + at, v, sz);
      a->col++;
      return 1;
    }
  }
  return -1;
}

int32_t duckdb_mb_append_int(duckdb_mb_appender *a, int32_t v) {  // ref :1116
  const int32_t r = AppendRaw(a, &v, 4, T_INTEGER, P_I32);
  return r >= 0 ? r : AppendValue(a, Value::Int(T_INTEGER, v));
}
int32_t duckdb_mb_append_bigint(duckdb_mb_appender *a, int64_t v) {  // ref :1132
  const int32_t r = AppendRaw(a, &v, 8, T_BIGINT, P_I64);
  return r >= 0 ? r : AppendValue(a, Value::Int(T_BIGINT, v));
}
int32_t duckdb_mb_append_double(duckdb_mb_appender *a, double v) { return AppendValue(a, Value::Double(v)); }  // ref :1148
int32_t duckdb_mb_append_varchar(duckdb_mb_appender *a, moonbit_bytes_t v) {  // ref :1164
  return AppendValue(a, Value::Varchar(BytesStr(v)));
}
int32_t duckdb_mb_append_bool(duckdb_mb_appender *a, bool v) { return AppendValue(a, Value::Bool(v)); }  // ref :1189
int32_t duckdb_mb_append_null(duckdb_mb_appender *a) {  // ref :1205
  if (!a) return 0;
  if (a->col >= a->table->cols.size()) {
    CopyErr(a->error, "Too many appends for chunk!");
    return 0;
  }
  if (a->pinned) {
    memset(PinnedSlot(a, a->col), 0, a->pw[a->col]);
    PinnedValid(a, a->col, false);
  } else {
    HostColumnPush(a->batch.cols[a->col], Value::Null(a->table->cols[a->col].type));
  }
  a->col++;
  return 1;
}
int32_t duckdb_mb_end_row(duckdb_mb_appender *a) {  // ref :1221-1235
  if (!a) return 0;
  if (a->col != a->table->cols.size()) {
    CopyErr(a->error, "Call to EndRow before all columns have been appended to!");
    return 0;
  }
  a->col = 0;
  if (a->pinned) {
    if (++a->prow >= a->pcap) return FlushPinned(a, false) ? 1 : 0;
    return 1;
  }
  a->batch.nrows++;
  if (a->batch.nrows >= a->conn->conn.opts.appender_flush_rows) return FlushAppender(a) ? 1 : 0;
  return 1;
}
int32_t duckdb_mb_flush(duckdb_mb_appender *a) {  // ref :1237-1251
  if (!a) return 0;
  if (a->col != 0) {
    CopyErr(a->error, "Failed to flush appender: Incomplete append to row!");
    return 0;
  }
  return FlushAppender(a) ? 1 : 0;
}
int32_t duckdb_mb_is_null_appender(duckdb_mb_appender *a) { return a == nullptr ? 1 : 0; }  // ref :1253

int32_t duckdb_mb_append_date(duckdb_mb_appender *a, int32_t days) {  // ref :1313 (reference appends an approximate
  return AppendValue(a, Value::Int(T_DATE, days));  // "YYYY-MM-DD" string; here the exact DATE)
}
int32_t duckdb_mb_append_timestamp(duckdb_mb_appender *a, int64_t micros) {  // ref :1350
  return AppendValue(a, Value::Int(T_TIMESTAMP, micros));
}
int32_t duckdb_mb_append_blob(duckdb_mb_appender *a, moonbit_bytes_t data, int32_t length) {  // ref :1397
  Value v = Value::Varchar(std::string((const char *)data, data ? (size_t)std::max(length, 0) : 0));
  v.type = LogicalType(T_BLOB);
  return AppendValue(a, v);
}
int32_t duckdb_mb_append_decimal(duckdb_mb_appender *a, uint8_t width, uint8_t scale, int64_t lower,
                                 int64_t upper) {  // ref :1447-1481
  if (width < 1 || width > 38 || scale > width) {
    if (a) CopyErr(a->error, "failed to create decimal value");
    return 0;
  }
  return AppendValue(a, Value::Decimal(width, scale, HugeFromParts(lower, upper)));
}
int32_t duckdb_mb_append_interval(duckdb_mb_appender *a, int32_t months, int32_t days, int64_t micros) {  // ref :1511
  Value v;
  v.type = LogicalType(T_INTERVAL);
  v.is_null = false;
  v.iv.months = months;
  v.iv.days = days;
  v.iv.micros = micros;
  return AppendValue(a, v);
}
int32_t duckdb_mb_append_list_varchar(duckdb_mb_appender *a, moonbit_bytes_t *, int32_t) {  // ref :1735
  return Unsupported(a ? a->error : nullptr, "LIST values");
}
int32_t duckdb_mb_append_struct_varchar(duckdb_mb_appender *a, moonbit_bytes_t *, moonbit_bytes_t *, int32_t) {  // ref :1792
  return Unsupported(a ? a->error : nullptr, "STRUCT values");
}
int32_t duckdb_mb_append_map_varchar_varchar(duckdb_mb_appender *a, moonbit_bytes_t *, moonbit_bytes_t *, int32_t) {  // ref :1860
  return Unsupported(a ? a->error : nullptr, "MAP values");
}

// ---- columnar bulk ingest (extension) ---------------------------------------------
int32_t duckdb_mbx_append_column(duckdb_mb_appender *a, int32_t col, const void *values, const uint8_t *validity,
                                 int64_t count) {
  if (!a) return 0;
  size_t nc = a->table->cols.size();
  if (col < 0 || (size_t)col >= nc) {
    CopyErr(a->error, "append_column: column index out of range");
    return 0;
  }
  if (a->table->cols[col].phys == P_STR || a->table->cols[col].phys == P_INTERVAL) {
    CopyErr(a->error, "append_column: only fixed-width columns are supported");
    return 0;
  }
  if (a->raw_vals.size() != nc) {
    a->raw_vals.assign(nc, nullptr);
    a->raw_valid.assign(nc, nullptr);
    a->raw_count.assign(nc, -1);
  }
  a->raw_vals[col] = values;
  a->raw_valid[col] = validity;
  a->raw_count[col] = count;
  return 1;
}

// ---- DataChunk / Vector / LogicalType (ref duckdb_native.c:1926-2132) ---------
// A logical type handle points at an MbxLogicalType; a vector handle at an
// MbxVector (host arrays of kVectorSize rows: values, and a validity mask of
// 64-bit words, bit = 1 -> valid, all set by create/reset so a caller may clear
// bits directly); a data chunk at an MbxChunk.
namespace {
struct MbxLogicalType {
  LogicalType t;
};
struct MbxVector {
  LogicalType t;
  Phys phys = P_I64;
  int w = 8;
  std::vector<uint64_t> data;  // kVectorSize * w bytes, 8-byte aligned
  std::vector<uint64_t> valid;
};
struct MbxChunk {
  std::vector<MbxVector> vecs;
  idx_t size = 0;
};
constexpr idx_t kChunkRows = 2048;  // DuckDB's STANDARD_VECTOR_SIZE

duckdb_mb_logical_type *NewMbType(const LogicalType &t) {
  auto *lt = new MbxLogicalType{t};
  auto *mb = (duckdb_mb_logical_type *)malloc(sizeof(duckdb_mb_logical_type));
  mb->type = (duckdb_logical_type)lt;
  return mb;
}
}  // namespace

duckdb_mb_logical_type *duckdb_mb_create_logical_type(duckdb_type type_id) {  // ref :1944-1956
  switch (type_id) {
    case T_BOOLEAN: case T_TINYINT: case T_SMALLINT: case T_INTEGER: case T_BIGINT: case T_UTINYINT:
    case T_USMALLINT: case T_UINTEGER: case T_UBIGINT: case T_FLOAT: case T_DOUBLE: case T_HUGEINT:
    case T_VARCHAR: case T_DATE: case T_TIMESTAMP: case T_TIME:
      return NewMbType(LogicalType((TypeId)type_id));
    case T_DECIMAL:
      return NewMbType(LogicalType::Decimal(18, 3));  // duckdb_create_logical_type(DECIMAL): DECIMAL(18,3)
    default:
      SetError("Not implemented Error: logical type id " + std::to_string(type_id) + " is not supported");
      return nullptr;
  }
}
duckdb_mb_logical_type *duckdb_mb_create_list_type(duckdb_mb_logical_type *) {  // ref :1958-1973
  SetError("Not implemented Error: LIST types are not supported by the MI355X backend");
  return nullptr;
}
duckdb_mb_logical_type *duckdb_mb_create_struct_type(duckdb_logical_type *, const char **, idx_t) {  // ref :1975-1990
  SetError("Not implemented Error: STRUCT types are not supported by the MI355X backend");
  return nullptr;
}
duckdb_mb_logical_type *duckdb_mb_create_map_type(duckdb_logical_type *, duckdb_logical_type *) {  // ref :1992-2009
  SetError("Not implemented Error: MAP types are not supported by the MI355X backend");
  return nullptr;
}
void duckdb_mb_destroy_logical_type(duckdb_mb_logical_type *mb) {  // ref :2011-2019
  if (!mb) return;
  delete (MbxLogicalType *)mb->type;
  free(mb);
}
int32_t duckdb_mb_is_null_logical_type(duckdb_mb_logical_type *mb) { return mb == nullptr ? 1 : 0; }  // ref :2021

duckdb_mb_data_chunk *duckdb_mb_create_data_chunk(duckdb_logical_type *types, idx_t column_count) {  // ref :2029-2043
  if (!types && column_count) return nullptr;
  auto *ch = new MbxChunk();
  for (idx_t i = 0; i < column_count; i++) {
    if (!types[i]) {
      delete ch;
      return nullptr;
    }
    MbxVector v;
    v.t = ((MbxLogicalType *)types[i])->t;
    v.phys = PhysOf(v.t);
    v.w = v.phys == P_STR ? 16 : PhysSize(v.phys);  // VARCHAR: a duckdb_string_t-sized slot per row
    v.data.assign((kChunkRows * v.w + 7) / 8, 0);
    v.valid.assign(kChunkRows / 64, ~0ull);
    ch->vecs.push_back(std::move(v));
  }
  auto *mb = (duckdb_mb_data_chunk *)malloc(sizeof(duckdb_mb_data_chunk));
  mb->chunk = (duckdb_data_chunk)ch;
  return mb;
}
void duckdb_mb_destroy_data_chunk(duckdb_mb_data_chunk *mb) {  // ref :2045-2053
  if (!mb) return;
  delete (MbxChunk *)mb->chunk;
  free(mb);
}
duckdb_vector duckdb_mb_data_chunk_get_vector(duckdb_mb_data_chunk *mb, idx_t col) {  // ref :2055-2061
  if (!mb || !mb->chunk) return nullptr;
  MbxChunk &ch = *(MbxChunk *)mb->chunk;
  if (col >= ch.vecs.size()) return nullptr;
  return (duckdb_vector)&ch.vecs[col];
}
void duckdb_mb_data_chunk_set_size(duckdb_mb_data_chunk *mb, idx_t size) {  // ref :2063-2068
  if (!mb || !mb->chunk) return;
  ((MbxChunk *)mb->chunk)->size = std::min<idx_t>(size, kChunkRows);
}
void duckdb_mb_data_chunk_reset(duckdb_mb_data_chunk *mb) {  // ref :2070-2075
  if (!mb || !mb->chunk) return;
  MbxChunk &ch = *(MbxChunk *)mb->chunk;
  ch.size = 0;
  for (auto &v : ch.vecs) std::fill(v.valid.begin(), v.valid.end(), ~0ull);
}
int32_t duckdb_mb_is_null_data_chunk(duckdb_mb_data_chunk *mb) { return mb == nullptr ? 1 : 0; }  // ref :2077
void *duckdb_mb_vector_get_data(duckdb_vector v) { return v ? ((MbxVector *)v)->data.data() : nullptr; }  // ref :2085
uint64_t *duckdb_mb_vector_get_validity(duckdb_vector v) {  // ref :2089
  return v ? ((MbxVector *)v)->valid.data() : nullptr;
}
duckdb_vector duckdb_mb_list_vector_get_child(duckdb_vector) {  // ref :2093
  SetError("Not implemented Error: LIST vectors are not supported by the MI355X backend");
  return nullptr;
}
duckdb_state duckdb_mb_list_vector_set_size(duckdb_vector, idx_t) { return DuckDBError; }  // ref :2097
duckdb_state duckdb_mb_list_vector_reserve(duckdb_vector, idx_t) { return DuckDBError; }   // ref :2101

// A vector's bytes into the pinned staging buffer, which only the DMA engine
// reads afterwards: memcpy.  Non-temporal stores (no read-for-ownership of the
// destination lines) measured no better on two boxes -- 1e8-row C4 ingest 17.2
// (memcpy) vs 17.1 (SSE2 streaming) vs 17.4 GB/s (AVX-512 streaming), then
// 17.5 vs 16.9 vs 14.1 GB/s (profiles/r06_chunk/, r06_final/chunk/) -- and stay
// as experiments: MBX_CHUNK_COPY = sse / avx512 (both ends 16-byte aligned).
__attribute__((target("avx512f"))) static void StreamNt64(void *dst, const void *src, size_t bytes) {
  char *d = (char *)dst;
  const char *p = (const char *)src;
  size_t n = bytes / 64;
  if (((uintptr_t)d & 63) == 0) {
    for (; n >= 4; n -= 4, d += 256, p += 256) {
      const __m512i a = _mm512_loadu_si512(p), b = _mm512_loadu_si512(p + 64), c = _mm512_loadu_si512(p + 128),
                    e = _mm512_loadu_si512(p + 192);
      _mm512_stream_si512((__m512i *)d, a), _mm512_stream_si512((__m512i *)(d + 64), b);
      _mm512_stream_si512((__m512i *)(d + 128), c), _mm512_stream_si512((__m512i *)(d + 192), e);
    }
    for (; n; n--, d += 64, p += 64) _mm512_stream_si512((__m512i *)d, _mm512_loadu_si512(p));
  }
  const size_t rest = bytes - (size_t)(d - (char *)dst);
  for (size_t i = 0; i + 16 <= rest; i += 16) _mm_stream_si128((__m128i *)(d + i), _mm_loadu_si128((const __m128i *)(p + i)));
  if (rest & 15) memcpy(d + (rest & ~(size_t)15), p + (rest & ~(size_t)15), rest & 15);
  _mm_sfence();
}

static void StreamToPinned(void *dst, const void *src, size_t bytes) {
  static const int mode = [] {
    const char *m = Knob("MBX_CHUNK_COPY");
    if (m && !strcmp(m, "sse")) return 1;
    if (m && !strcmp(m, "avx512")) return __builtin_cpu_supports("avx512f") ? 2 : 1;
    return 0;
  }();
  if (mode == 0 || (((uintptr_t)dst | (uintptr_t)src) & 15)) {
    memcpy(dst, src, bytes);
    return;
  }
  if (mode == 2) {
    StreamNt64(dst, src, bytes);
    return;
  }
  __m128i *d = (__m128i *)dst;
  const __m128i *p = (const __m128i *)src;
  size_t n = bytes / 16;
  for (; n >= 4; n -= 4, d += 4, p += 4) {
    const __m128i a = _mm_load_si128(p), b = _mm_load_si128(p + 1), c = _mm_load_si128(p + 2),
                  e = _mm_load_si128(p + 3);
    _mm_stream_si128(d, a), _mm_stream_si128(d + 1, b), _mm_stream_si128(d + 2, c), _mm_stream_si128(d + 3, e);
  }
  for (; n; n--) _mm_stream_si128(d++, _mm_load_si128(p++));
  if (bytes & 15) memcpy(d, p, bytes & 15);
  _mm_sfence();  // the stores are globally visible before the buffer's DMA is queued
}

// whether rows [lo, hi) of an LSB-first validity bitmap are all valid, a word at a time
static bool AllValid(const uint64_t *w, int64_t lo, int64_t hi) {
  while (lo < hi) {
    const int64_t k = lo >> 6, b = lo & 63, e = std::min<int64_t>(64, b + (hi - lo));
    const uint64_t mask = (e - b == 64) ? ~0ull : (((1ull << (e - b)) - 1) << b);
    if ((w[k] & mask) != mask) return false;
    lo += e - b;
  }
  return true;
}

int32_t duckdb_mb_append_data_chunk(duckdb_mb_appender *a, duckdb_mb_data_chunk *mb) {  // ref :2109-2132
  if (!a) return 0;
  if (!mb || !mb->chunk) {
    CopyErr(a->error, "data_chunk is null");
    return 0;
  }
  MbxChunk &ch = *(MbxChunk *)mb->chunk;
  const size_t nc = a->table->cols.size();
  if (ch.vecs.size() != nc) {
    CopyErr(a->error, "Invalid Input Error: Appender: the data chunk has " + std::to_string(ch.vecs.size()) +
                          " columns but the table has " + std::to_string(nc));
    return 0;
  }
  if (a->col != 0) {
    CopyErr(a->error, "Failed to append data chunk: Incomplete append to row!");
    return 0;
  }
  for (size_t c = 0; c < nc; c++)
    if (ch.vecs[c].phys == P_STR) {
      CopyErr(a->error, "Not implemented Error: VARCHAR vectors in append_data_chunk");
      return 0;
    }
  const int64_t n = (int64_t)ch.size;
  auto row_valid = [&](size_t c, int64_t r) { return (ch.vecs[c].valid[r >> 6] >> (r & 63)) & 1; };
  try {
    bool exact = a->pinned;
    for (size_t c = 0; exact && c < nc; c++) exact = ch.vecs[c].t == a->table->cols[c].type;
    if (exact) {  // whole-vector copies into the pinned double buffer
      int64_t off = 0;
      while (off < n) {
        PinnedSlot(a, 0);  // allocates the buffers on first use
        const int64_t m = std::min<int64_t>(n - off, a->pcap - a->prow);
        for (size_t c = 0; c < nc; c++) {
          const int w = a->pw[c];
          StreamToPinned((char *)a->pbuf[a->pcur][c] + (size_t)a->prow * w,
                         (const char *)ch.vecs[c].data.data() + (size_t)off * w, (size_t)m * w);
          const bool all = AllValid(ch.vecs[c].valid.data(), off, off + m);
          auto &pv = a->pvalid[c];
          if (!all || !pv.empty()) {
            if (pv.empty()) pv.assign((size_t)a->prow, 1);
            pv.resize((size_t)a->prow);
            for (int64_t r = off; r < off + m; r++) pv.push_back((uint8_t)row_valid(c, r));
          }
        }
        a->prow += m;
        off += m;
        if (a->prow >= a->pcap && !FlushPinned(a, false)) return 0;
      }
      return 1;
    }
    // other types: value by value through the appender's casts
    for (int64_t r = 0; r < n; r++) {
      for (size_t c = 0; c < nc; c++) {
        const MbxVector &v = ch.vecs[c];
        Value x = Value::Null(v.t);
        if (row_valid(c, r)) {
          HostColumn hc;
          hc.type = v.t;
          hc.phys = v.phys;
          hc.data.assign((const uint8_t *)v.data.data() + (size_t)r * v.w, (const uint8_t *)v.data.data() + (size_t)(r + 1) * v.w);
          x = hc.Get(0);
        }
        if (!AppendValue(a, x)) return 0;
      }
      if (!duckdb_mb_end_row(a)) return 0;
    }
    return 1;
  } catch (std::exception &e) {
    CopyErr(a->error, e.what());
    return 0;
  }
}

int32_t duckdb_mbx_append_commit(duckdb_mb_appender *a, int64_t count) {
  if (!a) return 0;
  size_t nc = a->table->cols.size();
  if (a->raw_vals.size() != nc) {
    CopyErr(a->error, "append_commit: no columns staged");
    return 0;
  }
  for (size_t i = 0; i < nc; i++)
    if (a->raw_count[i] != count || !a->raw_vals[i]) {
      CopyErr(a->error, "append_commit: every column must be staged with the same row count");
      return 0;
    }
  if (!FlushAppender(a)) return 0;  // keep row order: staged rows first
  try {
    std::vector<const void *> vals(a->raw_vals.begin(), a->raw_vals.end());
    std::vector<const uint8_t *> valid(a->raw_valid.begin(), a->raw_valid.end());
    AppendRawColumns(a->conn->conn, *a->table, vals, valid, count);
  } catch (std::exception &e) {
    CopyErr(a->error, e.what());
    return 0;
  }
  a->raw_vals.clear();
  a->raw_valid.clear();
  a->raw_count.clear();
  return 1;
}

// ---- "arrow" read-back ---------------------------------------------------------
duckdb_mb_arrow_result *duckdb_mb_query_arrow(duckdb_mb_connection *h, moonbit_bytes_t sql) {  // ref :2219-2268
  if (!h) {
    SetError("invalid connection handle");
    return nullptr;
  }
  try {
    Statement st = ParseSQL(BytesStr(sql));
    StreamSource src = RunStatementStream(h->conn, st, {});
    auto *a = new duckdb_mb_arrow_result();
    a->conn = h;
    a->dev = src.dev;
    a->r = src.host;
    a->names = std::move(src.names);
    a->types = std::move(src.types);
    a->error[0] = '\0';
    a->column_count = (int32_t)a->names.size();
    a->row_count = (int32_t)src.nrows;
    return a;
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}

int32_t duckdb_mb_arrow_column_count(duckdb_mb_arrow_result *a) { return a ? a->column_count : 0; }  // ref :2270
int32_t duckdb_mb_arrow_row_count(duckdb_mb_arrow_result *a) { return a ? a->row_count : 0; }        // ref :2277

moonbit_bytes_t duckdb_mb_arrow_schema(duckdb_mb_arrow_result *a) {  // ref :2285-2355
  if (!a || a->column_count <= 0) return MakeBytes("[]", 2);
  std::string j = "[";
  for (int32_t i = 0; i < a->column_count; i++) {
    const LogicalType &ty = a->types[i];
    const char *tid = "string";
    switch (ty.id) {
      case T_BOOLEAN: tid = "bool"; break;
      case T_TINYINT: case T_SMALLINT: case T_INTEGER: tid = "int32"; break;
      case T_BIGINT: tid = "int64"; break;
      case T_FLOAT: case T_DOUBLE: tid = "double"; break;
      default: tid = "string"; break;
    }
    j += std::string(i ? "," : "") + "{\"name\":\"" + a->names[i] + "\",\"nullable\":true,\"type_id\":\"" + tid + "\"}";
  }
  j += "]";
  return MakeBytes(j);
}

// The per-cell conversions of the reference's duckdb_value_int64 /
// duckdb_value_double / duckdb_value_boolean: a failed cast yields 0.
static int64_t CellI64(const HostColumn &c, int64_t row) {
  Value v = c.Get(row);
  if (v.is_null) return 0;
  Value x = CastValue(v, LogicalType(T_BIGINT), true);
  return x.is_null ? 0 : (int64_t)x.i;
}
static double CellF64(const HostColumn &c, int64_t row) {
  Value v = c.Get(row);
  if (v.is_null) return 0.0;
  Value x = CastValue(v, LogicalType(T_DOUBLE), true);
  return x.is_null ? 0.0 : x.d;
}
static uint8_t CellBool(const HostColumn &c, int64_t row) {
  Value v = c.Get(row);
  if (v.is_null) return 0;
  Value x = CastValue(v, LogicalType(T_BOOLEAN), true);
  return x.is_null ? 0 : (x.i ? 1 : 0);
}

static bool ArrowOk(duckdb_mb_arrow_result *a, int32_t col) {
  return a && col >= 0 && col < a->column_count && a->row_count > 0;
}
// [i32 count][values][validity bytes if nullable] straight from a device
// column of exactly this type (NULL slots zeroed on the device), or nullptr
static moonbit_bytes_t ArrowDirectBuffer(duckdb_mb_arrow_result *a, int32_t col, TypeId t, Phys ph, int width,
                                         bool nullable = false) {
  if (!ArrowOk(a, col) || !a->dev || a->r || a->types[col].id != t || !DeviceColumnWireOk(*a->dev, col, ph))
    return nullptr;
  const int64_t n = a->row_count;
  const int64_t total = 4 + n * width + (nullable ? n : 0);
  if (MbTooBig(total)) return nullptr;
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)total);
  memcpy(out, &a->row_count, 4);
  uint8_t *vb = nullable ? out + 4 + n * width : nullptr;
  try {
    CopyDeviceColumnWire(a->conn->conn, *a->dev, col, ph, out + 4, vb);
  } catch (std::exception &e) {
    SetError(e.what());
    memset(out + 4, 0, (size_t)(total - 4));
  }
  return out;
}
// the same layout from a host column of exactly this type
static bool ArrowHostExact(const HostColumn &c, int64_t n, TypeId t, Phys ph, int width, bool nullable,
                           uint8_t *vals) {
  if (c.type.id != t || c.phys != ph || (int64_t)c.data.size() < n * width) return false;
  memcpy(vals, c.data.data(), (size_t)(n * width));
  uint8_t *vb = vals + n * width;
  if (c.valid.empty()) {
    if (nullable) memset(vb, 1, (size_t)n);
    return true;
  }
  for (int64_t i = 0; i < n; i++) {
    if (!c.valid[i]) memset(vals + i * width, 0, (size_t)width);
    if (nullable) vb[i] = c.valid[i];
  }
  return true;
}
static const MaterializedResult &ArrowHost(duckdb_mb_arrow_result *a) {
  if (a->r) return *a->r;
  try {
    a->r = FetchDeviceRows(a->conn->conn, *a->dev, 0, a->row_count);
  } catch (std::exception &e) {
    // a failed read-back must not cross the C ABI: serve all-NULL columns
    SetError(e.what());
    auto r = std::make_shared<MaterializedResult>();
    r->nrows = a->row_count;
    for (size_t i = 0; i < a->types.size(); i++) {
      HostColumn hc;
      hc.name = a->names[i];
      hc.type = a->types[i];
      hc.phys = PhysOf(a->types[i]);
      hc.data.assign((size_t)a->row_count * 16, 0);
      hc.valid.assign((size_t)a->row_count, 0);
      if (hc.phys == P_STR) hc.offsets.assign((size_t)a->row_count + 1, 0);
      r->cols.push_back(std::move(hc));
    }
    a->r = r;
  }
  return *a->r;
}

static moonbit_bytes_t ArrowFixed(duckdb_mb_arrow_result *a, int32_t col, int width, bool nullable) {
  if (!ArrowOk(a, col)) return MakeBytes("", 0);
  int64_t n = a->row_count;
  int64_t total = 4 + n * width + (nullable ? n : 0);
  if (MbTooBig(total)) return MakeBytes("", 0);
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)total);
  int32_t cnt = (int32_t)n;
  memcpy(out, &cnt, 4);
  uint8_t *vals = out + 4;
  uint8_t *valid = out + 4 + n * width;
  const HostColumn &c = ArrowHost(a).cols[col];
  if (width == 4 && ArrowHostExact(c, n, T_INTEGER, P_I32, 4, nullable, vals)) return out;
  if (width == 1 && ArrowHostExact(c, n, T_BOOLEAN, P_U8, 1, nullable, vals)) return out;
  for (int64_t i = 0; i < n; i++) {
    bool null = c.IsNull(i);
    if (nullable) valid[i] = null ? 0 : 1;
    if (width == 4) {
      int32_t x = null ? 0 : (int32_t)CellI64(c, i);
      memcpy(vals + 4 * i, &x, 4);
    } else if (width == 8 && c.type.id != T_DOUBLE && c.type.id != T_FLOAT && c.phys != P_F64) {
      // int64 getter
      int64_t x = null ? 0 : CellI64(c, i);
      memcpy(vals + 8 * i, &x, 8);
    } else if (width == 8) {
      double x = null ? 0.0 : CellF64(c, i);
      memcpy(vals + 8 * i, &x, 8);
    } else {
      vals[i] = null ? 0 : CellBool(c, i);
    }
  }
  return out;
}

static moonbit_bytes_t ArrowF64(duckdb_mb_arrow_result *a, int32_t col, bool nullable) {
  if (!ArrowOk(a, col)) return MakeBytes("", 0);
  int64_t n = a->row_count;
  int64_t total = 4 + n * 8 + (nullable ? n : 0);
  if (MbTooBig(total)) return MakeBytes("", 0);
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)total);
  int32_t cnt = (int32_t)n;
  memcpy(out, &cnt, 4);
  const HostColumn &c = ArrowHost(a).cols[col];
  if (ArrowHostExact(c, n, T_DOUBLE, P_F64, 8, nullable, out + 4)) return out;
  for (int64_t i = 0; i < n; i++) {
    bool null = c.IsNull(i);
    double x = null ? 0.0 : CellF64(c, i);
    memcpy(out + 4 + 8 * i, &x, 8);
    if (nullable) out[4 + n * 8 + i] = null ? 0 : 1;
  }
  return out;
}

static moonbit_bytes_t ArrowStr(duckdb_mb_arrow_result *a, int32_t col, bool nullable) {
  if (!ArrowOk(a, col)) return MakeBytes("", 0);
  int64_t n = a->row_count;
  if (a->dev && !a->r && n > 0 && DeviceColumnTextOk(*a->dev, col)) {
    // integer / BOOLEAN / DECIMAL / HUGEINT: formatted on the device, one DMA into the Bytes
    moonbit_bytes_t out = nullptr;
    int64_t total = 0;
    try {
      const bool ok = CopyDeviceColumnText(a->conn->conn, *a->dev, col, [&](int64_t chars) -> uint8_t * {
        total = 8 + chars + (nullable ? n : 0);
        if (MbTooBig(total)) return nullptr;
        out = moonbit_make_bytes_raw((int32_t)total);
        const int32_t h[2] = {(int32_t)n, (int32_t)chars};
        memcpy(out, h, 8);
        return out + 8;
      }, nullable);
      if (ok) return out;
      if (!out) return MakeBytes("", 0);  // over the 2^28-byte limit of one MoonBit Bytes (MbTooBig set the error)
    } catch (std::exception &e) {
      // never hand back a buffer whose header claims n strings it does not hold:
      // drop it, keep the error, return the empty Bytes of the other failures
      SetError(e.what());
      if (out) moonbit_decref(out);
      return MakeBytes("", 0);
    }
  }
  const HostColumn &c = ArrowHost(a).cols[col];
  std::string data;
  for (int64_t i = 0; i < n; i++) {
    if (!c.IsNull(i)) {
      char buf[48];
      const int k = c.FormatInto(i, buf);
      if (k >= 0) data.append(buf, (size_t)k);
      else data += FormatValue(c.Get(i));
    }
    data.push_back('\0');
  }
  int64_t total = 8 + (int64_t)data.size() + (nullable ? n : 0);
  if (MbTooBig(total)) return MakeBytes("", 0);
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)total);
  int32_t h[2] = {(int32_t)n, (int32_t)data.size()};
  memcpy(out, h, 8);
  memcpy(out + 8, data.data(), data.size());
  if (nullable)
    for (int64_t i = 0; i < n; i++) out[8 + data.size() + i] = c.IsNull(i) ? 0 : 1;
  return out;
}

moonbit_bytes_t duckdb_mb_arrow_get_column_int32(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2359
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_INTEGER, P_I32, 4)) return d;
  return ArrowFixed(a, col, 4, false);
}
moonbit_bytes_t duckdb_mb_arrow_get_column_int64(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2392
  if (!ArrowOk(a, col)) return MakeBytes("", 0);
  int64_t n = a->row_count;
  if (MbTooBig(4 + n * 8)) return MakeBytes("", 0);
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_BIGINT, P_I64, 8)) return d;
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)(4 + n * 8));
  int32_t cnt = (int32_t)n;
  memcpy(out, &cnt, 4);
  const HostColumn &c = ArrowHost(a).cols[col];
  if (!ArrowHostExact(c, n, T_BIGINT, P_I64, 8, false, out + 4)) {
    for (int64_t i = 0; i < n; i++) {
      int64_t x = c.IsNull(i) ? 0 : CellI64(c, i);
      memcpy(out + 4 + 8 * i, &x, 8);
    }
  }
  return out;
}
moonbit_bytes_t duckdb_mb_arrow_get_column_double(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2424
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_DOUBLE, P_F64, 8)) return d;
  return ArrowF64(a, col, false);
}
moonbit_bytes_t duckdb_mb_arrow_get_column_string(duckdb_mb_arrow_result *a, int32_t col) { return ArrowStr(a, col, false); }  // ref :2456
moonbit_bytes_t duckdb_mb_arrow_get_column_bool(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2516
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_BOOLEAN, P_U8, 1)) return d;
  return ArrowFixed(a, col, 1, false);
}
moonbit_bytes_t duckdb_mb_arrow_get_column_int32_nullable(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2572
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_INTEGER, P_I32, 4, true)) return d;
  return ArrowFixed(a, col, 4, true);
}
moonbit_bytes_t duckdb_mb_arrow_get_column_int64_nullable(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2611
  if (!ArrowOk(a, col)) return MakeBytes("", 0);
  int64_t n = a->row_count;
  if (MbTooBig(4 + n * 9)) return MakeBytes("", 0);
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_BIGINT, P_I64, 8, true)) return d;
  moonbit_bytes_t out = moonbit_make_bytes_raw((int32_t)(4 + n * 9));
  int32_t cnt = (int32_t)n;
  memcpy(out, &cnt, 4);
  const HostColumn &c = ArrowHost(a).cols[col];
  if (ArrowHostExact(c, n, T_BIGINT, P_I64, 8, true, out + 4)) return out;
  for (int64_t i = 0; i < n; i++) {
    bool null = c.IsNull(i);
    int64_t x = null ? 0 : CellI64(c, i);
    memcpy(out + 4 + 8 * i, &x, 8);
    out[4 + 8 * n + i] = null ? 0 : 1;
  }
  return out;
}
moonbit_bytes_t duckdb_mb_arrow_get_column_double_nullable(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2649
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_DOUBLE, P_F64, 8, true)) return d;
  return ArrowF64(a, col, true);
}
moonbit_bytes_t duckdb_mb_arrow_get_column_string_nullable(duckdb_mb_arrow_result *a, int32_t col) { return ArrowStr(a, col, true); }  // ref :2687
moonbit_bytes_t duckdb_mb_arrow_get_column_bool_nullable(duckdb_mb_arrow_result *a, int32_t col) {  // ref :2761
  if (moonbit_bytes_t d = ArrowDirectBuffer(a, col, T_BOOLEAN, P_U8, 1, true)) return d;
  return ArrowFixed(a, col, 1, true);
}

void duckdb_mb_arrow_destroy(duckdb_mb_arrow_result *a) { delete a; }  // ref :2548
int32_t duckdb_mb_is_null_arrow_result(duckdb_mb_arrow_result *a) { return a == nullptr ? 1 : 0; }  // ref :2556
double duckdb_mb_bytes_to_double(const char *bytes, int32_t offset) {  // ref :2561-2565
  double r;
  memcpy(&r, bytes + offset, sizeof(double));
  return r;
}

// ---- extensions ----------------------------------------------------------------
int32_t duckdb_mbx_device_count(void) { return DeviceCount(); }
const char *duckdb_mbx_version(void) { return "duckdb.mbt-amd 0.1.0 (gfx950, HIP)"; }

char *duckdb_mbx_explain(duckdb_mb_connection *h, const char *sql, int64_t len) {
  if (!h || !sql) {
    SetError("connection is null");
    return nullptr;
  }
  try {
    std::string s = Explain(h->conn, std::string(sql, (size_t)len));
    return strdup(s.c_str());
  } catch (std::exception &e) {
    SetError(e.what());
    return nullptr;
  }
}
void duckdb_mbx_free(void *p) { free(p); }

// Compiles (hipRTC, gfx950, no GPU needed) the specialised filter and
// projection kernels of a small fixed program covering loads, constants,
// integer / 128-bit / double arithmetic, comparisons and three-valued logic.
// Returns NULL when both compile, else the compiler log (free with
// duckdb_mbx_free).  MBX_JIT_DUMP=1 prints the generated sources.
void duckdb_mbx_jit_join(void) { jit::JoinPending(); }

char *duckdb_mbx_jit_selftest(void) {
  VmProgram p;
  memset(&p, 0, sizeof(p));
  dev::VmCols cols;
  memset(&cols, 0, sizeof(cols));
  cols.n = 2;
  cols.c[0].phys = P_I64;
  cols.c[1].phys = P_I32;
  auto ins = [&](int op, int d, int a, int b = 0, int c = 0, int aux = 0) {
    VmIns &I = p.ins[p.n_ins++];
    I.op = (uint8_t)op;
    I.dst = (uint8_t)d;
    I.a = (uint8_t)a;
    I.b = (uint8_t)b;
    I.c = (uint8_t)c;
    I.aux = (uint16_t)aux;
  };
  p.n_const = 2;
  p.consts[0].lo = 24;
  p.consts[1].lo = 16;
  ins(V_LOADCOL, 0, 0);
  ins(V_CONST, 1, 0);
  ins(V_CMP_I, 2, 0, 1, 0, 4);  // x > 24
  ins(V_LOADCOL, 3, 1);
  ins(V_CONST, 4, 1);
  ins(V_CMP_I, 5, 3, 4, 0, 2);  // k < 16
  ins(V_AND, 2, 2, 5);
  ins(V_ADD_I, 6, 0, 3);       // x + k
  ins(V_I2L, 7, 6);
  ins(V_MUL_L, 7, 7, 7);
  ins(V_I2F, 8, 6);
  ins(V_DIV_F, 8, 8, 8);
  ins(V_SELECT, 9, 2, 6, 0);
  p.n_regs = 10;
  p.pred_reg = 2;
  p.n_out = 3;
  p.out_reg[0] = 9;
  p.out_phys[0] = P_I64;
  p.out_reg[1] = 7;
  p.out_phys[1] = P_I128;
  p.out_reg[2] = 8;
  p.out_phys[2] = P_F64;
  std::string log;
  for (bool filter : {true, false}) {
    std::string src = jit::Source(p, cols, filter);
    if (Knob("MBX_JIT_DUMP")) fprintf(stderr, "%s\n", src.c_str());
    std::string r = jit::CompileCheck(src);
    if (!r.empty()) log += std::string(filter ? "[filter] " : "[project] ") + r;
  }
  // the fused aggregate kernel: SUM(x + k) (int), SUM(double), COUNT(*) WHERE x > 24 AND k < 16
  p.n_out = 3;
  p.out_reg[0] = 6;
  p.out_class[0] = VC_I64;
  p.out_reg[1] = 8;
  p.out_class[1] = VC_F64;
  p.out_reg[2] = 255;
  {
    std::string src = jit::AggSourceForTest(p, cols);
    if (Knob("MBX_JIT_DUMP")) fprintf(stderr, "%s\n", src.c_str());
    std::string r = jit::CompileCheck(src);
    if (!r.empty()) log += "[aggregate] " + r;
  }
  // the fused GROUP BY kernel: keys (x nullable-less, k), SUM(x + k) and COUNT(*)
  {
    VmProgram q = p;
    q.n_out = 2;
    q.out_reg[0] = 6;
    q.out_class[0] = VC_I64;
    q.out_phys[0] = 3;
    q.out_reg[1] = 255;
    jit::GroupSpec g;
    memset(&g, 0, sizeof(g));
    g.nkeys = 2;
    g.key_reg[0] = 0;
    g.key_reg[1] = 3;
    g.key_nullable[1] = 1;
    std::string src = jit::GroupSourceForTest(q, cols, g);
    if (Knob("MBX_JIT_DUMP")) fprintf(stderr, "%s\n", src.c_str());
    std::string r = jit::CompileCheck(src);
    if (!r.empty()) log += "[group] " + r;
  }
  if (log.empty()) return nullptr;
  char *out = (char *)malloc(log.size() + 1);
  memcpy(out, log.c_str(), log.size() + 1);
  return out;
}

int32_t duckdb_mbx_hbm_calibrate_ex(duckdb_mb_connection *h, int64_t bytes, int32_t iters, double *out, int32_t nout) {
  if (!h || !out || nout <= 0) return 0;
  try {
    double all[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HbmCalibrateConn(h->conn, bytes, iters, all);
    const int k = nout < 8 ? nout : 8;
    for (int i = 0; i < k; i++) out[i] = all[i];
    return k;
  } catch (std::exception &e) {
    SetError(e.what());
    return 0;
  }
}
// Arrow getter copies of 2-32 MiB (an 8 MB 1e6-row INT64 slice is one): the
// method from now on, process-wide -- -1 the measured choice (default), 0 the
// runtime's copy, 1 a registered destination, 2 the pinned bounce.  Returns 1.
int32_t duckdb_mbx_set_link_mode(int32_t mode) {
  mbx::SetLinkMode(mode);
  return 1;
}

// Per device and power-of-two size class of those copies: each method's trial
// medians (GB/s), the method kept and the calls served, as JSON (malloc'd;
// free with duckdb_mbx_free).
char *duckdb_mbx_link_stats(void) { return strdup(mbx::LinkStatsJson().c_str()); }

// In-kernel clock stamps of the last filter_agg_lds / group_direct_lds /
// two-array ring launch: {memtime, realtime} at the start and the end of each
// of the first cap workgroups' main loop (libduckdb_mb_amd_clk.so, `make
// clockdiag`); returns the workgroups copied, 0 from the product library.
int32_t duckdb_mbx_clock_stamps(duckdb_mb_connection *h, uint64_t *out4, int32_t cap) {
  if (!h || !out4 || cap <= 0) return 0;
  try {
    return ClockStampsConn(h->conn, out4, cap);
  } catch (std::exception &e) {
    SetError(e.what());
    return 0;
  }
}
int32_t duckdb_mbx_hbm_calibrate(duckdb_mb_connection *h, int64_t bytes, int32_t iters, double *out3) {
  return duckdb_mbx_hbm_calibrate_ex(h, bytes, iters, out3, 3) == 3 ? 1 : 0;
}

char *duckdb_mbx_last_profile(duckdb_mb_connection *h) {
  if (!h) return nullptr;
  const QueryProfile &p = h->conn.last_profile;
  std::string j = "{\"total_ms\":" + std::to_string(p.total_ms) + ",\"kernels\":[";
  for (size_t i = 0; i < p.kernels.size(); i++) {
    const auto &k = p.kernels[i];
    char buf[256];
    snprintf(buf, sizeof(buf), "%s{\"name\":\"%s\",\"ms\":%.6f,\"bytes\":%.0f,\"rows\":%lld}", i ? "," : "",
             k.name.c_str(), k.ms, k.bytes, (long long)k.rows);
    j += buf;
  }
  j += "]}";
  return strdup(j.c_str());
}

char *duckdb_mbx_profile_drain(duckdb_mb_connection *h) {
  if (!h) return nullptr;
  std::string j = "[";
  for (size_t i = 0; i < h->conn.profile_history.size(); i++) {
    const auto &k = h->conn.profile_history[i];
    char buf[256];
    snprintf(buf, sizeof(buf),
             "%s{\"name\":\"%s\",\"ms\":%.6f,\"bytes\":%.0f,\"rows\":%lld,\"shard\":%d,\"device\":%d}",
             i ? "," : "", k.name.c_str(), k.ms, k.bytes, (long long)k.rows, k.shard, k.device);
    j += buf;
  }
  j += "]";
  h->conn.profile_history.clear();
  return strdup(j.c_str());
}

// Every cell of a result as text in ONE call: the same strings and NULL flags
// that duckdb_mb_result_is_null / duckdb_mb_result_value return cell by cell
// (the per-cell loop of Connection::query, duckdb_native.mbt:477-497), for
// hosts whose per-call FFI cost dwarfs the formatting.  Layout (little endian):
//   i64 nrows, i64 ncols, u8 null[nrows*ncols] (row-major), zero padding to 8,
//   i64 offsets[nrows*ncols + 1], chars.
// Returns a malloc'd buffer (free with duckdb_mbx_free) and its size in *len.
char *duckdb_mbx_result_text(duckdb_mb_result *r, int64_t *len) {
  if (!r || !r->r || !len) return nullptr;
  const MaterializedResult &m = *r->r;
  const int64_t nr = m.nrows, nc = (int64_t)m.cols.size(), ncell = nr * nc;
  std::string chars;
  std::vector<int64_t> off((size_t)ncell + 1, 0);
  std::vector<uint8_t> nul((size_t)ncell, 0);
  for (int64_t row = 0; row < nr; row++)
    for (int64_t col = 0; col < nc; col++) {
      const HostColumn &c = m.cols[col];
      const int64_t i = row * nc + col;
      if (c.IsNull(row)) {
        nul[i] = 1;
      } else {
        char buf[48];
        const int n = c.FormatInto(row, buf);
        if (n >= 0) chars.append(buf, (size_t)n);
        else chars += FormatValue(c.Get(row));
      }
      off[i + 1] = (int64_t)chars.size();
    }
  const size_t head = 16 + (((size_t)ncell + 7) & ~(size_t)7);
  const size_t total = head + off.size() * 8 + chars.size();
  char *buf = (char *)malloc(total ? total : 1);
  if (!buf) return nullptr;
  memset(buf, 0, head);
  memcpy(buf, &nr, 8);
  memcpy(buf + 8, &nc, 8);
  if (ncell) memcpy(buf + 16, nul.data(), (size_t)ncell);
  memcpy(buf + head, off.data(), off.size() * 8);
  if (!chars.empty()) memcpy(buf + head + off.size() * 8, chars.data(), chars.size());
  *len = (int64_t)total;
  return buf;
}

// Counters of the in-library multi-device path (gpu_devices): out[0] shards,
// [1] peer-access links enabled at connect, [2] ForShards dispatches, [3] peer
// DMA copies, [4] peer DMA bytes, [5] sharded aggregates finished on the host;
// outd[0] the last dispatch's wall time (us), outd[1] the last host merge (us).
// Returns the number of int64 counters written (0 for a null handle).
int32_t duckdb_mbx_shard_stats(duckdb_mb_connection *h, int64_t *out6, double *outd2) {
  if (!h) return 0;
  const ShardStats &st = h->conn.shard_stats;
  if (out6) {
    out6[0] = (int64_t)h->conn.shards.size();
    out6[1] = st.peer_links;
    out6[2] = st.dispatches;
    out6[3] = st.peer_copies;
    out6[4] = st.peer_bytes;
    out6[5] = st.host_results;
  }
  if (outd2) {
    outd2[0] = st.last_dispatch_us;
    outd2[1] = st.last_combine_us;
  }
  return 6;
}

// The last sharded dispatch (ForShards), per shard: out[4 i .. 4 i + 3] =
// {device, wake_us, launch_us, done_us}, times in us since the dispatch began
// (the worker picked the job up; its plan and launches were queued; its
// result reached the host, i.e. kernel + D2H + synchronisation).  Writes at
// most cap shards; returns the shard count of that dispatch (0: none yet).
int32_t duckdb_mbx_shard_timings(duckdb_mb_connection *h, double *out, int32_t cap) {
  if (!h) return 0;
  const auto &last = h->conn.shard_stats.last;
  for (int32_t i = 0; out && i < cap && i < (int32_t)last.size(); i++) {
    out[4 * i] = last[i].device;
    out[4 * i + 1] = last[i].wake_us;
    out[4 * i + 2] = last[i].launch_us;
    out[4 * i + 3] = last[i].done_us;
  }
  return (int32_t)last.size();
}

// Shard i's partial aggregate relation of the last sharded aggregate (groups,
// then the decomposed partials: COUNT, SUM as HUGEINT / DECIMAL(38,s) /
// DOUBLE, MIN, MAX; AVG as SUM then COUNT), as it came back from its device
// before the merge.  A result handle for the duckdb_mb_result_* accessors
// (free with duckdb_mb_result_destroy); NULL if there is none.
duckdb_mb_result *duckdb_mbx_shard_partial(duckdb_mb_connection *h, int32_t shard) {
  if (!h || shard < 0 || shard >= (int32_t)h->conn.shard_stats.last_partials.size()) return nullptr;
  const ResultPtr &p = h->conn.shard_stats.last_partials[shard];
  if (!p) return nullptr;
  auto *r = new duckdb_mb_result;
  r->r = p;
  return r;
}

// mbx_combine=rccl counters: out2 = {sharded aggregates RCCL combined,
// requests that fell back to the host merge}; out_us1 = the last RCCL
// combine's collective + D2H wall time on device 0 (us).  Either may be NULL.
int32_t duckdb_mbx_rccl_stats(duckdb_mb_connection *h, int64_t *out2, double *out_us1) {
  if (!h) return 0;
  const ShardStats &st = h->conn.shard_stats;
  if (out2) out2[0] = st.rccl_combines, out2[1] = st.rccl_fallbacks;
  if (out_us1) out_us1[0] = st.last_rccl_us;
  return 2;
}

// Why the last mbx_combine=rccl request fell back to the host merge ("" when
// it ran); malloc'd, free with duckdb_mbx_free.
char *duckdb_mbx_rccl_note(duckdb_mb_connection *h) {
  return strdup(h ? h->conn.shard_stats.rccl_note.c_str() : "");
}

// mbx_combine counters, up to cap of {RCCL combines, fallbacks to the host
// merge, combines through the test loopback, combines that raised a shard's
// device error, collectives aborted after the timeout, combines of GROUP BY
// relations}; returns how many were written.
int32_t duckdb_mbx_rccl_stats_ex(duckdb_mb_connection *h, int64_t *out, int32_t cap) {
  if (!h || !out) return 0;
  const ShardStats &st = h->conn.shard_stats;
  const int64_t v[9] = {st.rccl_combines,        st.rccl_fallbacks,   st.rccl_loopbacks,
                        st.rccl_errors,          st.rccl_timeouts,    st.rccl_group_combines,
                        st.rccl_unsupported,     st.rccl_reduces,     st.rccl_allgathers};
  int32_t n = 0;
  for (; n < cap && n < 9; n++) out[n] = v[n];
  return n;
}

char *duckdb_mbx_rccl_info(duckdb_mb_connection *h) {
  return strdup(h ? RcclInfoJson(h->conn).c_str() : "{}");
}

// Switches a connection's combine between the host merge (0) and RCCL (1), as
// Config::set("mbx_combine", ...) at connect would; 2 is the test loopback
// (accepted only with MBX_EXPERIMENTS=1).  Returns 1 (0: refused).
int32_t duckdb_mbx_set_combine(duckdb_mb_connection *h, int32_t mode) {
  if (!h || mode < 0 || mode > 2) return 0;
  if (mode == 2 && !mbx::Knob("MBX_EXPERIMENTS")) return 0;
  h->conn.opts.combine_rccl = mode != 0;
  h->conn.opts.rccl_loopback = mode == 2;
  return 1;
}

// The RCCL library calls of the combine on hardware with one GPU (the combine
// itself needs one device per rank): a one-rank communicator on `device`, one
// grouped ncclReduce and one ncclAllGather of 97 int64 lanes, checked.  Returns
// 1 and the wall us in *us_out; 0 and the reason via duckdb_mb_last_error.
int32_t duckdb_mbx_rccl_selftest(int32_t device, double *us_out) {
  std::string err;
  double us = 0;
  RcclSelfTestJson({device}, &err, &us);
  if (us_out) *us_out = us;
  if (!err.empty()) {
    SetError(err.c_str());
    return 0;
  }
  return 1;
}

char *duckdb_mbx_rccl_selftest_ex(const int32_t *devices, int32_t n) {
  std::vector<int> devs;
  for (int32_t i = 0; devices && i < n; i++) devs.push_back(devices[i]);
  std::string err;
  double us = 0;
  return strdup(RcclSelfTestJson(devs, &err, &us).c_str());
}

// The RCCL combine's lane arithmetic on the host (combine.h; CPU tests):
// gathered = nranks x (3 ncols + 1) lanes, kinds[ncols] (0 sum, 1 min, 2 max);
// out = 3 ncols lanes {lo, hi, non-NULL}.  Returns 1 (0: bad arguments).
int32_t duckdb_mbx_combine_lanes(const int64_t *gathered, int32_t nranks, int32_t ncols, const int8_t *kinds,
                                 int64_t *out) {
  if (!gathered || !kinds || !out || nranks < 1 || ncols < 1 || ncols > rc::kMaxCols) return 0;
  for (int j = 0; j < ncols; j++)
    rc::CombineColumn(gathered, nranks, rc::LanesPerRank(ncols, false), j, kinds[j], out + 3 * j);
  return 1;
}

// out3 = {select_rounds launches, aborts (a persistent workgroup was never
// scheduled within 100 ms: the query reran in the two-pass form), launch
// failures (the two-pass form ran instead)} over the connection and its shards.
int32_t duckdb_mbx_engine_stats(duckdb_mb_connection *h, int64_t *out3) {
  if (!h || !out3) return 0;
  out3[0] = out3[1] = out3[2] = 0;
  EngineCounters(h->conn, out3);
  return 3;
}

int32_t duckdb_mbx_result_raw(duckdb_mb_result *r, int32_t col, int32_t row, void *out, int32_t out_len) {
  if (!r || !InRange(r->r, col, row) || !out) return 0;
  const HostColumn &c = r->r->cols[col];
  if (c.IsNull(row) || c.phys == P_STR) return 0;
  int sz = PhysSize(c.phys);
  if (out_len < sz) return 0;
  memcpy(out, c.data.data() + (size_t)row * sz, sz);
  return sz;
}

}  // extern "C"
