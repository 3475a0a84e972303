// engine.cpp — statement dispatch (DDL / DML / SELECT) and host result columns.
#include "engine.h"

#include <hip/hip_runtime_api.h>

#include <cstring>
#include <sys/mman.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <new>

namespace mbx {

namespace result_blocks {
// size classes: 1 MiB steps below 16 MiB, then eighths of a power of two
static size_t ClassOf(size_t b) {
  const size_t mib = (size_t)1 << 20;
  if (b <= 16 * mib) return (b + mib - 1) & ~(mib - 1);
  size_t p = 16 * mib;
  while (p * 2 < b) p *= 2;
  const size_t step = p / 8;
  return (b + step - 1) / step * step;
}
constexpr size_t kMinBlock = (size_t)1 << 20;
constexpr size_t kCacheCap = (size_t)2 << 30;  // bytes kept for reuse, process-wide
static std::mutex mu;
static std::multimap<size_t, void *> cache;
static size_t cached = 0;

void *Get(size_t bytes) {
  if (bytes < kMinBlock) {
    void *p = malloc(bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    return p;
  }
  const size_t c = ClassOf(bytes);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(c);
    if (it != cache.end()) {
      void *p = it->second;
      cache.erase(it);
      cached -= c;
      return p;
    }
  }
  void *p = mmap(nullptr, c, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw std::bad_alloc();
  (void)madvise(p, c, MADV_HUGEPAGE);
  // page-locked once for its lifetime in the cache: a result's columns are
  // DMA targets (a failed registration leaves a pageable block, still valid)
  (void)hipHostRegister(p, c, hipHostRegisterPortable);
  (void)hipGetLastError();
  return p;
}

void Put(void *p, size_t bytes) {
  if (!p) return;
  if (bytes < kMinBlock) {
    free(p);
    return;
  }
  const size_t c = ClassOf(bytes);
  {
    std::lock_guard<std::mutex> g(mu);
    if (cached + c <= kCacheCap) {
      cache.emplace(c, p);
      cached += c;
      return;
    }
  }
  (void)hipHostUnregister(p);
  (void)hipGetLastError();
  munmap(p, c);
}
}  // namespace result_blocks

static std::string Lower(std::string s) {
  for (auto &c : s) c = (char)tolower((unsigned char)c);
  return s;
}

Connection::~Connection() {
  catalog.tables.clear();  // free device columns before the engine stream
  engine.reset();
}

Value HostColumn::Get(int64_t row) const {
  Value v;
  v.type = type;
  if (IsNull(row)) {
    v.is_null = true;
    return v;
  }
  v.is_null = false;
  const uint8_t *p = data.data();
  switch (phys) {
    case P_U8: v.i = p[row]; break;
    case P_I8: v.i = ((const int8_t *)p)[row]; break;
    case P_I16: v.i = ((const int16_t *)p)[row]; break;
    case P_U16: v.i = ((const uint16_t *)p)[row]; break;
    case P_I32: v.i = ((const int32_t *)p)[row]; break;
    case P_U32: v.i = ((const uint32_t *)p)[row]; break;
    case P_I64: v.i = ((const int64_t *)p)[row]; break;
    case P_U64: v.i = (i128)((const uint64_t *)p)[row]; break;
    case P_I128: {
      uint64_t lo;
      int64_t hi;
      memcpy(&lo, p + 16 * row, 8);
      memcpy(&hi, p + 16 * row + 8, 8);
      v.i = (i128)(((u128)(uint64_t)hi << 64) | lo);
      break;
    }
    case P_F32: v.d = ((const float *)p)[row]; break;
    case P_F64: v.d = ((const double *)p)[row]; break;
    case P_STR: v.s = chars.substr(offsets[row], offsets[row + 1] - offsets[row]); break;
    case P_INTERVAL: memcpy(&v.iv, p + 16 * row, 16); break;
  }
  return v;
}

int HostColumn::FormatInto(int64_t row, char *out) const {
  if (!text_off.empty()) {  // formatted on the device with the result
    const uint32_t b = text_off[row], n = text_off[row + 1] - b - 1;
    memcpy(out, text.data() + b, n);
    return (int)n;
  }
  const uint8_t *p = data.data();
  i128 x;
  switch (phys) {
    case P_U8: x = p[row]; break;
    case P_I8: x = ((const int8_t *)p)[row]; break;
    case P_I16: x = ((const int16_t *)p)[row]; break;
    case P_U16: x = ((const uint16_t *)p)[row]; break;
    case P_I32: x = ((const int32_t *)p)[row]; break;
    case P_U32: x = ((const uint32_t *)p)[row]; break;
    case P_I64: x = ((const int64_t *)p)[row]; break;
    case P_U64: x = (i128)((const uint64_t *)p)[row]; break;
    case P_I128: {
      uint64_t lo;
      int64_t hi;
      memcpy(&lo, p + 16 * row, 8);
      memcpy(&hi, p + 16 * row + 8, 8);
      x = (i128)(((u128)(uint64_t)hi << 64) | lo);
      break;
    }
    default: return -1;
  }
  switch (type.id) {
    case T_BOOLEAN:
      if (x) { memcpy(out, "true", 4); return 4; }
      memcpy(out, "false", 5);
      return 5;
    case T_TINYINT: case T_SMALLINT: case T_INTEGER: case T_BIGINT: case T_UTINYINT:
    case T_USMALLINT: case T_UINTEGER: case T_UBIGINT: case T_HUGEINT:
      return FormatI128Into(x, out);
    case T_DECIMAL: {  // same spelling as FormatDecimal: [-]int.frac, frac zero-padded to scale
      const int scale = type.scale;
      if (scale == 0) return FormatI128Into(x, out);
      const bool neg = x < 0;
      char dig[48];
      int n = FormatI128Into(neg ? (i128)(~(u128)x + 1) : x, dig);
      int o = 0;
      if (neg) out[o++] = '-';
      if (n <= scale) {
        out[o++] = '0';
        out[o++] = '.';
        for (int i = n; i < scale; i++) out[o++] = '0';
        memcpy(out + o, dig, (size_t)n);
        return o + n;
      }
      memcpy(out + o, dig, (size_t)(n - scale));
      o += n - scale;
      out[o++] = '.';
      memcpy(out + o, dig + n - scale, (size_t)scale);
      return o + scale;
    }
    default: return -1;
  }
}

void HostColumnPush(HostColumn &c, const Value &v) {
  bool null = v.is_null;
  if (null || !c.valid.empty()) {
    if (c.valid.empty()) {
      int64_t n = c.phys == P_STR ? (int64_t)c.offsets.size() - 1 : (int64_t)(c.data.size() / std::max(PhysSize(c.phys), 1));
      c.valid.assign(n, 1);
    }
    c.valid.push_back(null ? 0 : 1);
  }
  if (c.phys == P_STR) {
    if (c.offsets.empty()) c.offsets.push_back(0);
    if (!null) c.chars += v.s;
    c.offsets.push_back((int64_t)c.chars.size());
    return;
  }
  int sz = PhysSize(c.phys);
  size_t at = c.data.size();
  c.data.resize(at + sz);
  uint8_t *p = c.data.data() + at;
  if (null) {
    memset(p, 0, sz);
    return;
  }
  switch (c.phys) {
    case P_U8: case P_I8: { int8_t x = (int8_t)v.i; memcpy(p, &x, 1); break; }
    case P_I16: case P_U16: { int16_t x = (int16_t)v.i; memcpy(p, &x, 2); break; }
    case P_I32: case P_U32: { int32_t x = (int32_t)v.i; memcpy(p, &x, 4); break; }
    case P_I64: case P_U64: { int64_t x = (int64_t)v.i; memcpy(p, &x, 8); break; }
    case P_I128: {
      uint64_t lo = (uint64_t)(u128)v.i;
      int64_t hi = (int64_t)(uint64_t)((u128)v.i >> 64);
      memcpy(p, &lo, 8);
      memcpy(p + 8, &hi, 8);
      break;
    }
    case P_F32: { float x = (float)v.d; memcpy(p, &x, 4); break; }
    case P_F64: memcpy(p, &v.d, 8); break;
    case P_INTERVAL: memcpy(p, &v.iv, 16); break;
    default: break;
  }
}

void ValueToRaw(const Value &v, Phys phys, uint8_t *p) {
  switch (phys) {
    case P_U8: case P_I8: { int8_t x = (int8_t)v.i; memcpy(p, &x, 1); break; }
    case P_I16: case P_U16: { int16_t x = (int16_t)v.i; memcpy(p, &x, 2); break; }
    case P_I32: case P_U32: { int32_t x = (int32_t)v.i; memcpy(p, &x, 4); break; }
    case P_I64: case P_U64: { int64_t x = (int64_t)v.i; memcpy(p, &x, 8); break; }
    case P_I128: {
      uint64_t lo = (uint64_t)(u128)v.i;
      int64_t hi = (int64_t)(uint64_t)((u128)v.i >> 64);
      memcpy(p, &lo, 8);
      memcpy(p + 8, &hi, 8);
      break;
    }
    case P_F32: { float x = (float)v.d; memcpy(p, &x, 4); break; }
    case P_F64: memcpy(p, &v.d, 8); break;
    case P_INTERVAL: memcpy(p, &v.iv, 16); break;
    default: break;
  }
}

static ResultPtr CountResult(int64_t n) {
  auto r = std::make_shared<MaterializedResult>();
  HostColumn hc;
  hc.name = "Count";
  hc.type = LogicalType(T_BIGINT);
  hc.phys = P_I64;
  HostColumnPush(hc, Value::Int(T_BIGINT, n));
  r->cols.push_back(hc);
  r->nrows = 1;
  return r;
}

static bool IsBareValues(const Select &s) {
  return s.from.kind == TableRef::VALUES && s.list.size() == 1 && s.list[0]->kind == Expr::STAR && !s.where &&
         s.group_by.empty() && !s.having && s.order_by.empty() && !s.limit && !s.offset && s.union_all.empty();
}

StreamSource RunStatementStream(Connection &c, const Statement &st, const std::vector<Value> &params) {
  StreamSource src;
  if (st.kind == Statement::SELECT) {
    BoundSelectPtr b = BindSelect(*st.select, c.catalog, params);
    return RunBoundStream(c, *b);
  } else {
    src.host = RunParsed(c, st, params);
  }
  src.names.clear();
  src.types.clear();
  for (auto &hc : src.host->cols) {
    src.names.push_back(hc.name);
    src.types.push_back(hc.type);
  }
  src.nrows = src.host->nrows;
  return src;
}

StreamSource RunBoundStream(Connection &c, const BoundSelect &b) {
  StreamSource src;
  src.dev = ExecuteSelectDevice(c, b, &src);
  if (src.dev) return src;
  src.host = ExecuteSelect(c, b);
  for (auto &hc : src.host->cols) {
    src.names.push_back(hc.name);
    src.types.push_back(hc.type);
  }
  src.nrows = src.host->nrows;
  return src;
}

ResultPtr RunParsed(Connection &c, const Statement &st, const std::vector<Value> &params) {
  switch (st.kind) {
    case Statement::NOP:
      return std::make_shared<MaterializedResult>();
    case Statement::SELECT: {
      BoundSelectPtr b = BindSelect(*st.select, c.catalog, params);
      return ExecuteSelect(c, *b);
    }
    case Statement::CREATE_TABLE:
    case Statement::CREATE_TABLE_AS: {
      std::string key = Lower(st.table);
      if (c.catalog.Find(key)) {
        if (st.if_not_exists) return std::make_shared<MaterializedResult>();
        if (!st.or_replace) ThrowError("Catalog", "Table with name \"" + st.table + "\" already exists!");
      }
      if (st.kind == Statement::CREATE_TABLE) {
        std::vector<std::string> names;
        std::vector<LogicalType> types;
        for (auto &cd : st.columns) {
          for (auto &n : names)
            if (Lower(n) == Lower(cd.name)) ThrowError("Catalog", "Column with name " + cd.name + " already exists!");
          names.push_back(cd.name);
          types.push_back(cd.type);
        }
        c.catalog.tables[key] = CreateDeviceTable(c, st.table, names, types);
        c.catalog.version++;
        return std::make_shared<MaterializedResult>();
      }
      BoundSelectPtr b = BindSelect(*st.select, c.catalog, params);
      std::vector<LogicalType> types = b->OutTypes();
      std::vector<std::string> names;
      for (size_t i = 0; i < types.size(); i++) {
        if (b->names[i].rfind("__order_", 0) == 0) {
          types.resize(i);
          break;
        }
        names.push_back(b->names[i]);
      }
      for (auto &t : types)
        if (t.id == T_SQLNULL) t = LogicalType(T_INTEGER);
      TablePtr t = CreateDeviceTable(c, st.table, names, types);
      std::vector<int> map;
      for (size_t i = 0; i < types.size(); i++) map.push_back((int)i);
      ExecuteInsertSelect(c, *t, *b, map);
      c.catalog.tables[key] = t;
      c.catalog.version++;
      return CountResult(t->nrows);
    }
    case Statement::INSERT: {
      TablePtr t = c.catalog.Find(st.table);
      if (!t) ThrowError("Catalog", "Table with name " + st.table + " does not exist!");
      std::vector<int> targets;
      if (st.insert_columns.empty()) {
        for (size_t i = 0; i < t->cols.size(); i++) targets.push_back((int)i);
      } else {
        for (auto &n : st.insert_columns) {
          int f = -1;
          for (size_t i = 0; i < t->col_names.size(); i++)
            if (Lower(t->col_names[i]) == Lower(n)) f = (int)i;
          if (f < 0) ThrowError("Binder", "Table \"" + t->name + "\" does not have a column with name \"" + n + "\"");
          targets.push_back(f);
        }
      }
      int64_t before = t->nrows;
      if (IsBareValues(*st.select)) {
        // constant rows: cast to the table types on the host, upload once
        HostBatch b;
        for (size_t i = 0; i < t->cols.size(); i++) {
          HostColumn hc;
          hc.type = t->cols[i].type;
          hc.phys = t->cols[i].phys;
          if (hc.phys == P_STR) hc.offsets.push_back(0);
          b.cols.push_back(hc);
        }
        BoundSelectPtr bs = BindSelect(*st.select, c.catalog, params);
        for (auto &row : bs->src.rows) {
          if (row.size() != targets.size())
            ThrowError("Binder", "table " + t->name + " has " + std::to_string(t->cols.size()) + " columns but " +
                                     std::to_string(row.size()) + " values were supplied");
          std::vector<Value> full(t->cols.size());
          for (size_t i = 0; i < t->cols.size(); i++) full[i] = Value::Null(t->cols[i].type);
          for (size_t k = 0; k < targets.size(); k++) full[targets[k]] = row[k];
          for (size_t i = 0; i < t->cols.size(); i++) HostColumnPush(b.cols[i], CastValue(full[i], t->cols[i].type));
          b.nrows++;
        }
        AppendHostBatch(c, *t, b);
        return CountResult(t->nrows - before);
      }
      BoundSelectPtr bs = BindSelect(*st.select, c.catalog, params);
      size_t nvis = 0;
      for (auto &n : bs->names)
        if (n.rfind("__order_", 0) != 0) nvis++;
      if (nvis != targets.size())
        ThrowError("Binder", "table " + t->name + " has " + std::to_string(targets.size()) + " columns but " +
                                 std::to_string(nvis) + " values were supplied");
      std::vector<int> map(t->cols.size(), -1);
      for (size_t k = 0; k < targets.size(); k++) map[targets[k]] = (int)k;
      ExecuteInsertSelect(c, *t, *bs, map);
      return CountResult(t->nrows - before);
    }
    case Statement::DROP_TABLE: {
      std::string key = Lower(st.table);
      if (!c.catalog.Find(key)) {
        if (st.if_exists) return std::make_shared<MaterializedResult>();
        ThrowError("Catalog", "Table with name " + st.table + " does not exist!");
      }
      c.catalog.tables.erase(key);
      c.catalog.version++;
      for (auto &sc : c.shards) sc->catalog.tables.erase(key);  // the parts of a sharded table
      return std::make_shared<MaterializedResult>();
    }
  }
  return std::make_shared<MaterializedResult>();
}

ResultPtr RunStatement(Connection &c, const std::string &sql, const std::vector<Value> &params, int *n_params_out) {
  Statement st = ParseSQL(sql);
  if (n_params_out) *n_params_out = st.n_params;
  return RunParsed(c, st, params);
}

std::string Explain(Connection &c, const std::string &sql) {
  Statement st = ParseSQL(sql);
  if (st.kind != Statement::SELECT) return "statement kind " + std::to_string((int)st.kind) + "\n";
  std::vector<Value> params(st.n_params);
  for (auto &p : params) p = Value::Null(LogicalType(T_INTEGER));
  BoundSelectPtr b = BindSelect(*st.select, c.catalog, params);
  return ExplainSelect(*b) + (IsHostConstantSelect(*b) ? "[host-constant]\n" : "[device]\n");
}

}  // namespace mbx
