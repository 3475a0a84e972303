// types.h — logical types, scalar values and 128-bit integer helpers shared by
// the binder, the executor and the C-ABI shim.
//
// Type ids are DuckDB's C-API ids, which the reference maps to its ColumnType
// enum in /root/reference/src/duckdb_parsing.mbt:8-52 (column_type_from_id).
#pragma once

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "phys.h"

namespace mbx {

typedef __int128 i128;
typedef unsigned __int128 u128;

enum TypeId : int32_t {
  T_INVALID = 0,
  T_BOOLEAN = 1,
  T_TINYINT = 2,
  T_SMALLINT = 3,
  T_INTEGER = 4,
  T_BIGINT = 5,
  T_UTINYINT = 6,
  T_USMALLINT = 7,
  T_UINTEGER = 8,
  T_UBIGINT = 9,
  T_FLOAT = 10,
  T_DOUBLE = 11,
  T_TIMESTAMP = 12,
  T_DATE = 13,
  T_TIME = 14,
  T_INTERVAL = 15,
  T_HUGEINT = 16,
  T_VARCHAR = 17,
  T_BLOB = 18,
  T_DECIMAL = 19,
  T_SQLNULL = 36,
};



// Register class of the device expression VM.
enum VClass : uint8_t { VC_I64 = 0, VC_I128 = 1, VC_F64 = 2, VC_STR = 3 };

struct LogicalType {
  TypeId id = T_INVALID;
  uint8_t width = 0;  // DECIMAL only
  uint8_t scale = 0;  // DECIMAL only
  LogicalType() {}
  LogicalType(TypeId i) : id(i) {}
  static LogicalType Decimal(int w, int s) {
    LogicalType t(T_DECIMAL);
    t.width = (uint8_t)w;
    t.scale = (uint8_t)s;
    return t;
  }
  bool operator==(const LogicalType &o) const {
    return id == o.id && (id != T_DECIMAL || (width == o.width && scale == o.scale));
  }
  bool operator!=(const LogicalType &o) const { return !(*this == o); }
  std::string ToString() const;
};

Phys PhysOf(const LogicalType &t);
int PhysSize(Phys p);  // bytes per value (0 for strings)
VClass ClassOf(const LogicalType &t);
bool IsIntegral(TypeId t);  // signed/unsigned integers + HUGEINT
bool IsNumeric(TypeId t);   // integral + DECIMAL + FLOAT + DOUBLE
bool IsSignedIntegral(TypeId t);
int IntegralRank(TypeId t);  // order for implicit widening
bool IntegralRange(TypeId t, i128 *lo, i128 *hi);

// ---- scalar value ---------------------------------------------------------
struct Interval {
  int32_t months = 0, days = 0;
  int64_t micros = 0;
};

struct Value {
  LogicalType type;
  bool is_null = true;
  i128 i = 0;       // all integer-like types, DECIMAL (unscaled), DATE, TIME, TIMESTAMP, BOOLEAN
  double d = 0;     // FLOAT / DOUBLE
  std::string s;    // VARCHAR / BLOB
  Interval iv;      // INTERVAL

  static Value Null(LogicalType t = LogicalType(T_SQLNULL)) {
    Value v;
    v.type = t;
    v.is_null = true;
    return v;
  }
  static Value Int(TypeId t, i128 x) {
    Value v;
    v.type = LogicalType(t);
    v.is_null = false;
    v.i = x;
    return v;
  }
  static Value Bool(bool b) { return Int(T_BOOLEAN, b ? 1 : 0); }
  static Value Double(double x) {
    Value v;
    v.type = LogicalType(T_DOUBLE);
    v.is_null = false;
    v.d = x;
    return v;
  }
  static Value Float(float x) {
    Value v;
    v.type = LogicalType(T_FLOAT);
    v.is_null = false;
    v.d = x;
    return v;
  }
  static Value Decimal(int w, int s, i128 x) {
    Value v;
    v.type = LogicalType::Decimal(w, s);
    v.is_null = false;
    v.i = x;
    return v;
  }
  static Value Varchar(const std::string &x) {
    Value v;
    v.type = LogicalType(T_VARCHAR);
    v.is_null = false;
    v.s = x;
    return v;
  }
};

// DuckDB-compatible text rendering (what duckdb_value_varchar returns).
std::string FormatValue(const Value &v);
std::string FormatI128(i128 x);
// Writes the decimal text of x into out (>= 41 bytes); returns its length.
int FormatI128Into(i128 x, char *out);
std::string FormatDecimal(i128 x, int scale);
std::string FormatDouble(double x);
std::string FormatFloat(float x);
std::string FormatDate(int32_t days);
std::string FormatTime(int64_t micros);
std::string FormatTimestamp(int64_t micros);
std::string FormatInterval(const Interval &iv);

// Calendar helpers (proleptic Gregorian, days since 1970-01-01).
int32_t DaysFromCivil(int64_t y, unsigned m, unsigned d);
void CivilFromDays(int64_t z, int64_t *y, unsigned *m, unsigned *d);
bool ParseDate(const std::string &s, int32_t *days);
bool ParseTime(const std::string &s, int64_t *micros);
bool ParseTimestamp(const std::string &s, int64_t *micros);
bool ParseInterval(const std::string &s, Interval *iv);

// Errors carry DuckDB's "<Kind> Error: message" text.
struct EngineError : std::runtime_error {
  explicit EngineError(const std::string &m) : std::runtime_error(m) {}
};
[[noreturn]] void ThrowError(const std::string &kind, const std::string &msg);

i128 Pow10(int k);  // k in [0, 38]
bool ParseI128(const std::string &s, i128 *out);

}  // namespace mbx
