// binder.cpp — name resolution, DuckDB type rules, constant folding.
//
// Typing rules follow DuckDB's binder for the shapes the reference exercises
// (SURVEY.md §8(c)): integer literals are INTEGER/BIGINT/HUGEINT by magnitude,
// decimal literals DECIMAL(digits, fraction digits), COUNT -> BIGINT,
// SUM(integer) -> HUGEINT, SUM(DECIMAL(p,s)) -> DECIMAL(38,s), AVG -> DOUBLE,
// '/' -> DOUBLE, '%' truncated, integer arithmetic overflow is an error,
// division/modulo by zero -> NULL.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <functional>
#include <limits>
#include <set>

#include "engine.h"
#include "plan.h"

namespace mbx {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
static std::string Lower(std::string s) {
  for (auto &c : s) c = (char)tolower((unsigned char)c);
  return s;
}

int64_t BoundSource::RangeCount() const {
  if (kind != RANGE) return 0;
  i128 a = range_start, b = range_stop, st = range_step;
  if (st == 0) return 0;
  if (range_inclusive) b += st > 0 ? 1 : -1;
  if (st > 0) return b > a ? (int64_t)((b - a + st - 1) / st) : 0;
  return a > b ? (int64_t)((a - b + (-st) - 1) / (-st)) : 0;
}

std::vector<LogicalType> BoundSelect::OutTypes() const {
  std::vector<LogicalType> t;
  for (auto &o : outputs) t.push_back(o->type);
  return t;
}

static BExprPtr MkConst(const Value &v) {
  auto e = std::make_shared<BExpr>();
  e->kind = BExpr::CONST;
  e->cval = v;
  e->type = v.type.id == T_SQLNULL ? LogicalType(T_SQLNULL) : v.type;
  return e;
}
static BExprPtr MkCol(int c, const LogicalType &t) {
  auto e = std::make_shared<BExpr>();
  e->kind = BExpr::COL;
  e->col = c;
  e->type = t;
  return e;
}
static BExprPtr MkFunc(BOp op, const LogicalType &t, std::vector<BExprPtr> ch) {
  auto e = std::make_shared<BExpr>();
  e->kind = BExpr::FUNC;
  e->op = op;
  e->type = t;
  e->ch = std::move(ch);
  return e;
}

bool IsConstTree(const BExpr &e) {
  if (e.kind == BExpr::COL) return false;
  for (auto &c : e.ch)
    if (!IsConstTree(*c)) return false;
  return true;
}

static BExprPtr Fold(BExprPtr e) {
  if (e->kind == BExpr::FUNC && IsConstTree(*e)) {
    Value v = EvalConst(*e);
    if (v.is_null) v.type = e->type;
    auto c = MkConst(v);
    c->type = e->type;
    c->cval.type = e->type;
    return c;
  }
  return e;
}

static BExprPtr CastTo(BExprPtr e, const LogicalType &t) {
  if (e->type == t) return e;
  if (e->kind == BExpr::CONST) {
    Value v = CastValue(e->cval, t);
    auto c = MkConst(v);
    c->type = t;
    c->cval.type = t;
    return c;
  }
  return MkFunc(B_CAST, t, {e});
}

static int DecimalWidthOfIntegral(TypeId t) {
  switch (t) {
    case T_BOOLEAN: return 1;
    case T_TINYINT: case T_UTINYINT: return 3;
    case T_SMALLINT: case T_USMALLINT: return 5;
    case T_INTEGER: case T_UINTEGER: return 10;
    case T_BIGINT: return 19;
    case T_UBIGINT: return 20;
    default: return 38;
  }
}

static LogicalType AsDecimal(const LogicalType &t) {
  if (t.id == T_DECIMAL) return t;
  return LogicalType::Decimal(std::min(38, DecimalWidthOfIntegral(t.id)), 0);
}

LogicalType MaxType(const LogicalType &a, const LogicalType &b) {
  if (a.id == T_SQLNULL) return b;
  if (b.id == T_SQLNULL) return a;
  if (a == b) return a;
  if (a.id == T_VARCHAR || b.id == T_VARCHAR) return LogicalType(T_VARCHAR);
  if (a.id == T_DOUBLE || b.id == T_DOUBLE) return LogicalType(T_DOUBLE);
  if (a.id == T_FLOAT || b.id == T_FLOAT) {
    if (IsNumeric(a.id) && IsNumeric(b.id)) return LogicalType(T_DOUBLE);
  }
  if (a.id == T_DECIMAL || b.id == T_DECIMAL) {
    if (!IsNumeric(a.id) && a.id != T_BOOLEAN) ThrowError("Binder", "Cannot mix types " + a.ToString() + " and " + b.ToString());
    if (!IsNumeric(b.id) && b.id != T_BOOLEAN) ThrowError("Binder", "Cannot mix types " + a.ToString() + " and " + b.ToString());
    LogicalType da = AsDecimal(a), db = AsDecimal(b);
    int scale = std::max(da.scale, db.scale);
    int ip = std::max(da.width - da.scale, db.width - db.scale);
    int w = ip + scale;
    if (w > 38) return LogicalType(T_DOUBLE);
    return LogicalType::Decimal(w, scale);
  }
  if ((IsIntegral(a.id) || a.id == T_BOOLEAN) && (IsIntegral(b.id) || b.id == T_BOOLEAN)) {
    if (a.id == T_BOOLEAN) return b;
    if (b.id == T_BOOLEAN) return a;
    bool sa = IsSignedIntegral(a.id), sb = IsSignedIntegral(b.id);
    int ra = IntegralRank(a.id), rb = IntegralRank(b.id);
    if (sa == sb) return ra >= rb ? a : b;
    // mixed signedness: signed type one rank above the unsigned one
    int ru = sa ? rb : ra, rs = sa ? ra : rb;
    int r = std::max(rs, ru + 1);
    static const TypeId bySigned[] = {T_BOOLEAN, T_TINYINT, T_SMALLINT, T_INTEGER, T_BIGINT, T_HUGEINT};
    return LogicalType(bySigned[std::min(r, 5)]);
  }
  if (a.id == T_TIMESTAMP && b.id == T_DATE) return a;
  if (a.id == T_DATE && b.id == T_TIMESTAMP) return b;
  ThrowError("Binder", "Cannot mix values of type " + a.ToString() + " and " + b.ToString() +
                            " - an explicit cast is required");
}

// ---------------------------------------------------------------------------
// host evaluation (constant folding)
// ---------------------------------------------------------------------------
static std::string IntTypeName(TypeId t) {
  switch (t) {
    case T_TINYINT: return "INT8";
    case T_SMALLINT: return "INT16";
    case T_INTEGER: return "INT32";
    case T_BIGINT: return "INT64";
    case T_HUGEINT: return "INT128";
    case T_UTINYINT: return "UINT8";
    case T_USMALLINT: return "UINT16";
    case T_UINTEGER: return "UINT32";
    case T_UBIGINT: return "UINT64";
    default: return LogicalType(t).ToString();
  }
}

static i128 DecimalLimit(int width) { return Pow10(width); }

static i128 RoundDiv(i128 v, i128 d) {  // round half away from zero
  i128 q = v / d, r = v % d;
  if (r < 0) r = -r;
  if (2 * r >= d) q += v < 0 ? -1 : 1;
  return q;
}

static bool DoubleToI128(double x, i128 *out) {
  if (std::isnan(x) || std::isinf(x)) return false;
  double r = std::nearbyint(x);
  if (r >= 1.7014118346046923e38 || r < -1.7014118346046923e38) return false;
  *out = (i128)r;
  return true;
}

static double I128ToDouble(i128 v) { return (double)v; }

Value CastValue(const Value &v, const LogicalType &to, bool try_cast) {
  Value out;
  out.type = to;
  if (v.is_null) {
    out.is_null = true;
    return out;
  }
  out.is_null = false;
  const LogicalType &from = v.type;
  if (from == to) {
    out = v;
    out.type = to;
    return out;
  }
  auto fail = [&](const std::string &msg) -> Value {
    if (try_cast) {
      Value n;
      n.type = to;
      n.is_null = true;
      return n;
    }
    ThrowError("Conversion", msg);
  };
  auto range_fail = [&](const std::string &sv) -> Value {
    return fail("Type " + IntTypeName(from.id) + " with value " + sv +
                " can't be cast because the value is out of range for the destination type " + IntTypeName(to.id));
  };
  // ---- to VARCHAR
  if (to.id == T_VARCHAR) {
    out.s = FormatValue(v);
    return out;
  }
  // ---- from VARCHAR
  if (from.id == T_VARCHAR || from.id == T_BLOB) {
    std::string s = v.s;
    auto trim = [](std::string x) {
      size_t a = 0, b = x.size();
      while (a < b && isspace((unsigned char)x[a])) a++;
      while (b > a && isspace((unsigned char)x[b - 1])) b--;
      return x.substr(a, b - a);
    };
    std::string t = trim(s);
    auto conv_fail = [&]() -> Value {
      return fail("Could not convert string '" + s + "' to " + IntTypeName(to.id));
    };
    if (to.id == T_BLOB) {
      out.s = s;
      return out;
    }
    if (IsIntegral(to.id)) {
      i128 x;
      if (!ParseI128(t, &x)) {
        // DuckDB accepts "1.0"-like strings for integers by rounding decimals
        char *end = nullptr;
        double d = strtod(t.c_str(), &end);
        if (t.empty() || *end != 0 || !DoubleToI128(d, &x)) return conv_fail();
      }
      i128 lo, hi;
      IntegralRange(to.id, &lo, &hi);
      if (x < lo || x > hi) return conv_fail();
      out.i = x;
      return out;
    }
    if (to.id == T_BOOLEAN) {
      std::string l = Lower(t);
      if (l == "true" || l == "t" || l == "1" || l == "yes" || l == "y") out.i = 1;
      else if (l == "false" || l == "f" || l == "0" || l == "no" || l == "n") out.i = 0;
      else return fail("Could not convert string '" + s + "' to BOOL");
      return out;
    }
    if (to.id == T_DOUBLE || to.id == T_FLOAT) {
      std::string l = Lower(t);
      if (l == "nan" || l == "+nan" || l == "-nan") out.d = std::numeric_limits<double>::quiet_NaN();
      else if (l == "inf" || l == "infinity" || l == "+inf" || l == "+infinity") out.d = INFINITY;
      else if (l == "-inf" || l == "-infinity") out.d = -INFINITY;
      else {
        char *end = nullptr;
        double d = strtod(t.c_str(), &end);
        if (t.empty() || *end != 0) return fail("Could not convert string '" + s + "' to " + to.ToString());
        out.d = d;
      }
      if (to.id == T_FLOAT) out.d = (float)out.d;
      return out;
    }
    if (to.id == T_DECIMAL) {
      // parse exact decimal
      std::string x = t;
      bool neg = false;
      size_t p = 0;
      if (p < x.size() && (x[p] == '-' || x[p] == '+')) neg = x[p++] == '-';
      std::string ip, fp;
      bool dot = false;
      for (; p < x.size(); p++) {
        if (x[p] == '.' && !dot) dot = true;
        else if (isdigit((unsigned char)x[p])) (dot ? fp : ip).push_back(x[p]);
        else return fail("Could not convert string '" + s + "' to " + to.ToString());
      }
      if (ip.empty() && fp.empty()) return fail("Could not convert string '" + s + "' to " + to.ToString());
      Value d;
      d.is_null = false;
      int sc = (int)fp.size();
      i128 raw = 0;
      if (!ParseI128((ip.empty() ? "0" : ip) + fp, &raw)) return fail("Could not convert string '" + s + "' to " + to.ToString());
      d.type = LogicalType::Decimal(38, std::min(sc, 38));
      d.i = neg ? -raw : raw;
      return CastValue(d, to, try_cast);
    }
    if (to.id == T_DATE) {
      int32_t days;
      if (!ParseDate(t, &days)) {
        int64_t us;
        if (ParseTimestamp(t, &us)) {
          days = (int32_t)(us / 86400000000LL - (us % 86400000000LL < 0 ? 1 : 0));
        } else {
          return fail("invalid date field format: \"" + s + "\", expected format is (YYYY-MM-DD)");
        }
      }
      out.i = days;
      return out;
    }
    if (to.id == T_TIME) {
      int64_t us;
      if (!ParseTime(t, &us)) return fail("invalid time field format: \"" + s + "\", expected format is ([YYYY-MM-DD ]HH:MM:SS[.MS])");
      out.i = us;
      return out;
    }
    if (to.id == T_TIMESTAMP) {
      int64_t us;
      if (!ParseTimestamp(t, &us)) return fail("invalid timestamp field format: \"" + s + "\", expected format is (YYYY-MM-DD HH:MM:SS[.US][±HH:MM| ZONE])");
      out.i = us;
      return out;
    }
    if (to.id == T_INTERVAL) {
      if (!ParseInterval(t, &out.iv)) return fail("Could not convert string '" + s + "' to INTERVAL");
      return out;
    }
    return fail("Unimplemented type for cast (VARCHAR -> " + to.ToString() + ")");
  }
  // ---- numeric sources
  bool from_int = IsIntegral(from.id) || from.id == T_BOOLEAN;
  if (from_int || from.id == T_DECIMAL) {
    i128 x = v.i;
    int fscale = from.id == T_DECIMAL ? from.scale : 0;
    if (IsIntegral(to.id) || to.id == T_BOOLEAN) {
      if (to.id == T_BOOLEAN) {
        out.i = x != 0;
        return out;
      }
      if (fscale) x = RoundDiv(x, Pow10(fscale));
      i128 lo, hi;
      IntegralRange(to.id, &lo, &hi);
      if (x < lo || x > hi) {
        return range_fail(from.id == T_DECIMAL ? FormatDecimal(v.i, fscale) : FormatI128(v.i));
      }
      out.i = x;
      return out;
    }
    if (to.id == T_DECIMAL) {
      int ds = to.scale - fscale;
      i128 r;
      if (ds >= 0) {
        i128 m = Pow10(ds);
        if (__builtin_mul_overflow(x, m, &r)) return fail("Could not cast value to " + to.ToString());
      } else {
        r = RoundDiv(x, Pow10(-ds));
      }
      i128 lim = DecimalLimit(to.width);
      if (r >= lim || r <= -lim) {
        std::string sv = from.id == T_DECIMAL ? FormatDecimal(v.i, fscale) : FormatI128(v.i);
        return fail("Could not cast value " + sv + " to " + to.ToString());
      }
      out.i = r;
      return out;
    }
    if (to.id == T_DOUBLE || to.id == T_FLOAT) {
      double d = I128ToDouble(x);
      if (fscale) d = d / (double)Pow10(fscale);
      if (fscale) {
        // exact decimal -> double (round-trip via string like DuckDB's cast)
        d = strtod(FormatDecimal(x, fscale).c_str(), nullptr);
      }
      out.d = to.id == T_FLOAT ? (double)(float)d : d;
      return out;
    }
    if (to.id == T_DATE || to.id == T_TIMESTAMP || to.id == T_TIME)
      return fail("Unimplemented type for cast (" + from.ToString() + " -> " + to.ToString() + ")");
  }
  if (from.id == T_DOUBLE || from.id == T_FLOAT) {
    double d = v.d;
    if (IsIntegral(to.id)) {
      i128 x;
      i128 lo, hi;
      IntegralRange(to.id, &lo, &hi);
      if (!DoubleToI128(d, &x) || x < lo || x > hi)
        return fail("Type DOUBLE with value " + FormatDouble(d) +
                    " can't be cast because the value is out of range for the destination type " + IntTypeName(to.id));
      out.i = x;
      return out;
    }
    if (to.id == T_BOOLEAN) {
      out.i = d != 0;
      return out;
    }
    if (to.id == T_DOUBLE || to.id == T_FLOAT) {
      out.d = to.id == T_FLOAT ? (double)(float)d : d;
      return out;
    }
    if (to.id == T_DECIMAL) {
      double scaled = d * (double)Pow10(to.scale);
      i128 x;
      if (!DoubleToI128(scaled, &x) || x >= DecimalLimit(to.width) || x <= -DecimalLimit(to.width))
        return fail("Could not cast value " + FormatDouble(d) + " to " + to.ToString());
      out.i = x;
      return out;
    }
  }
  if (from.id == T_DATE && to.id == T_TIMESTAMP) {
    out.i = v.i * 86400000000LL;
    return out;
  }
  if (from.id == T_TIMESTAMP && to.id == T_DATE) {
    int64_t us = (int64_t)v.i;
    out.i = us / 86400000000LL - ((us % 86400000000LL) < 0 ? 1 : 0);
    return out;
  }
  if (from.id == T_TIMESTAMP && to.id == T_TIME) {
    int64_t us = (int64_t)(v.i % 86400000000LL);
    if (us < 0) us += 86400000000LL;
    out.i = us;
    return out;
  }
  if (from.id == T_SQLNULL) {
    out.is_null = true;
    return out;
  }
  return fail("Unimplemented type for cast (" + from.ToString() + " -> " + to.ToString() + ")");
}

static int Cmp3(const Value &a, const Value &b) {
  // a, b have the same type
  switch (ClassOf(a.type)) {
    case VC_F64: {
      double x = a.d, y = b.d;
      // DuckDB orders NaN above everything and NaN == NaN
      bool nx = std::isnan(x), ny = std::isnan(y);
      if (nx || ny) return nx == ny ? 0 : (nx ? 1 : -1);
      return x < y ? -1 : x > y ? 1 : 0;
    }
    case VC_STR:
      return a.s < b.s ? -1 : a.s > b.s ? 1 : 0;
    default:
      if (a.type.id == T_INTERVAL) {
        i128 x = (i128)a.iv.months * 30 * 86400000000LL + (i128)a.iv.days * 86400000000LL + a.iv.micros;
        i128 y = (i128)b.iv.months * 30 * 86400000000LL + (i128)b.iv.days * 86400000000LL + b.iv.micros;
        return x < y ? -1 : x > y ? 1 : 0;
      }
      return a.i < b.i ? -1 : a.i > b.i ? 1 : 0;
  }
}

static i128 CheckedIntResult(BOp op, const LogicalType &t, i128 r, i128 a, i128 b, bool ovf) {
  i128 lo, hi;
  bool dec = t.id == T_DECIMAL;
  if (dec) {
    Phys p = PhysOf(t);
    if (p == P_I128) {
      lo = (i128)((u128)1 << 127);
      hi = (i128)(((u128)1 << 127) - 1);
    } else {
      lo = INT64_MIN;
      hi = INT64_MAX;
    }
  } else if (!IntegralRange(t.id, &lo, &hi)) {
    lo = INT64_MIN;
    hi = INT64_MAX;
  }
  if (ovf || r < lo || r > hi) {
    const char *nm = op == B_ADD ? "addition" : op == B_SUB ? "subtraction" : op == B_MUL ? "multiplication" : "negation";
    const char *sym = op == B_ADD ? "+" : op == B_SUB ? "-" : op == B_MUL ? "*" : "-";
    std::string tn = dec ? (PhysOf(t) == P_I128 ? "INT128" : "INT64") : IntTypeName(t.id);
    ThrowError("Out of Range", std::string("Overflow in ") + nm + " of " + tn + " (" + FormatI128(a) + " " + sym +
                                   " " + FormatI128(b) + ")!");
  }
  return r;
}

Value EvalConst(const BExpr &e) {
  if (e.kind == BExpr::CONST) {
    Value v = e.cval;
    if (v.is_null) v.type = e.type;
    return v;
  }
  if (e.kind == BExpr::COL) ThrowError("Internal", "column reference in constant expression");
  std::vector<Value> a;
  // short-circuit forms first
  switch (e.op) {
    case B_CASE: {
      size_t n = e.ch.size();
      for (size_t i = 0; i + 1 < n; i += 2) {
        Value c = EvalConst(*e.ch[i]);
        if (!c.is_null && c.i) return CastValue(EvalConst(*e.ch[i + 1]), e.type);
      }
      if (n % 2 == 1) return CastValue(EvalConst(*e.ch[n - 1]), e.type);
      return Value::Null(e.type);
    }
    case B_COALESCE: {
      for (auto &c : e.ch) {
        Value v = EvalConst(*c);
        if (!v.is_null) return CastValue(v, e.type);
      }
      return Value::Null(e.type);
    }
    case B_AND: {
      Value x = EvalConst(*e.ch[0]), y = EvalConst(*e.ch[1]);
      if ((!x.is_null && !x.i) || (!y.is_null && !y.i)) return Value::Bool(false);
      if (x.is_null || y.is_null) return Value::Null(LogicalType(T_BOOLEAN));
      return Value::Bool(true);
    }
    case B_OR: {
      Value x = EvalConst(*e.ch[0]), y = EvalConst(*e.ch[1]);
      if ((!x.is_null && x.i) || (!y.is_null && y.i)) return Value::Bool(true);
      if (x.is_null || y.is_null) return Value::Null(LogicalType(T_BOOLEAN));
      return Value::Bool(false);
    }
    default:
      break;
  }
  for (auto &c : e.ch) a.push_back(EvalConst(*c));
  switch (e.op) {
    case B_ISNULL: return Value::Bool(a[0].is_null);
    case B_ISNOTNULL: return Value::Bool(!a[0].is_null);
    case B_DISTINCT:
    case B_NOT_DISTINCT: {
      bool same;
      if (a[0].is_null || a[1].is_null) same = a[0].is_null && a[1].is_null;
      else same = Cmp3(a[0], a[1]) == 0;
      return Value::Bool(e.op == B_DISTINCT ? !same : same);
    }
    case B_CAST:
      return CastValue(a[0], e.type);
    default:
      break;
  }
  for (auto &v : a)
    if (v.is_null) return Value::Null(e.type);
  switch (e.op) {
    case B_NOT: return Value::Bool(!a[0].i);
    case B_EQ: return Value::Bool(Cmp3(a[0], a[1]) == 0);
    case B_NE: return Value::Bool(Cmp3(a[0], a[1]) != 0);
    case B_LT: return Value::Bool(Cmp3(a[0], a[1]) < 0);
    case B_LE: return Value::Bool(Cmp3(a[0], a[1]) <= 0);
    case B_GT: return Value::Bool(Cmp3(a[0], a[1]) > 0);
    case B_GE: return Value::Bool(Cmp3(a[0], a[1]) >= 0);
    case B_CONCAT: {
      Value r = Value::Varchar(a[0].s + a[1].s);
      return r;
    }
    case B_LENGTH: return Value::Int(T_BIGINT, (i128)a[0].s.size());
    case B_LOWER: return Value::Varchar(Lower(a[0].s));
    case B_UPPER: {
      std::string s = a[0].s;
      for (auto &c : s) c = (char)toupper((unsigned char)c);
      return Value::Varchar(s);
    }
    case B_SYNTH: {
      uint64_t z = (uint64_t)(int64_t)a[0].i + (uint64_t)(int64_t)a[1].i;
      z += 0x9E3779B97F4A7C15ULL;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
      z ^= z >> 31;
      uint64_t m = (uint64_t)(int64_t)a[2].i;
      if (m == 0) return Value::Null(e.type);
      return Value::Int(T_BIGINT, (i128)(z % m));
    }
    default:
      break;
  }
  // arithmetic
  const LogicalType &t = e.type;
  VClass vc = ClassOf(t);
  if (t.id == T_DATE || t.id == T_TIMESTAMP) {
    // date/timestamp +/- interval (children: [date|timestamp, interval])
    const Value &d = a[0];
    const Interval &iv = a[1].iv;
    int sgn = e.op == B_SUB ? -1 : 1;
    int64_t us = d.type.id == T_DATE ? (int64_t)d.i * 86400000000LL : (int64_t)d.i;
    int64_t days = us / 86400000000LL, rem = us % 86400000000LL;
    if (rem < 0) {
      rem += 86400000000LL;
      days--;
    }
    if (iv.months) {
      int64_t y;
      unsigned m, dd;
      CivilFromDays(days, &y, &m, &dd);
      int64_t mm = (int64_t)m - 1 + sgn * (int64_t)iv.months;
      y += mm >= 0 ? mm / 12 : (mm - 11) / 12;
      mm = ((mm % 12) + 12) % 12;
      static const int dm[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
      bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
      unsigned lim = (unsigned)(dm[mm] + (mm == 1 && leap));
      days = DaysFromCivil(y, (unsigned)mm + 1, std::min(dd, lim));
    }
    days += sgn * (int64_t)iv.days;
    int64_t total = days * 86400000000LL + rem + sgn * iv.micros;
    if (t.id == T_DATE) return Value::Int(T_DATE, total / 86400000000LL - (total % 86400000000LL < 0 ? 1 : 0));
    Value r = Value::Int(T_TIMESTAMP, total);
    return r;
  }
  if (vc == VC_F64) {
    double x = a[0].d, y = e.ch.size() > 1 ? a[1].d : 0;
    double r = 0;
    switch (e.op) {
      case B_ADD: r = x + y; break;
      case B_SUB: r = x - y; break;
      case B_MUL: r = x * y; break;
      case B_DIV:
        if (y == 0) return Value::Null(t);
        r = x / y;
        break;
      case B_MOD:
        if (y == 0) return Value::Null(t);
        r = std::fmod(x, y);
        break;
      case B_IDIV:
        if (y == 0) return Value::Null(t);
        r = std::trunc(x / y);
        break;
      case B_NEG: r = -x; break;
      case B_ABS: r = std::fabs(x); break;
      default: ThrowError("Internal", "bad float op");
    }
    Value v = Value::Double(t.id == T_FLOAT ? (double)(float)r : r);
    v.type = t;
    return v;
  }
  // integer / decimal
  i128 x = a[0].i, y = e.ch.size() > 1 ? a[1].i : 0, r = 0;
  bool ovf = false;
  switch (e.op) {
    case B_ADD: ovf = __builtin_add_overflow(x, y, &r); break;
    case B_SUB: ovf = __builtin_sub_overflow(x, y, &r); break;
    case B_MUL: ovf = __builtin_mul_overflow(x, y, &r); break;
    case B_IDIV:
    case B_DIV:
      if (y == 0) return Value::Null(t);
      r = x / y;
      break;
    case B_MOD:
      if (y == 0) return Value::Null(t);
      r = x % y;
      break;
    case B_NEG: ovf = __builtin_sub_overflow((i128)0, x, &r); break;
    case B_ABS: r = x < 0 ? -x : x; break;
    default: ThrowError("Internal", "bad integer op");
  }
  r = CheckedIntResult(e.op, t, r, x, y, ovf);
  Value v;
  v.type = t;
  v.is_null = false;
  v.i = r;
  return v;
}

// ---------------------------------------------------------------------------
// expression printing (column names, EXPLAIN)
// ---------------------------------------------------------------------------
static const char *OpSym(BOp op) {
  switch (op) {
    case B_ADD: return "+";
    case B_SUB: return "-";
    case B_MUL: return "*";
    case B_DIV: return "/";
    case B_IDIV: return "//";
    case B_MOD: return "%";
    case B_EQ: return "=";
    case B_NE: return "!=";
    case B_LT: return "<";
    case B_LE: return "<=";
    case B_GT: return ">";
    case B_GE: return ">=";
    case B_AND: return "AND";
    case B_OR: return "OR";
    case B_CONCAT: return "||";
    default: return "?";
  }
}

std::string ExprToString(const BExpr &e) {
  switch (e.kind) {
    case BExpr::CONST:
      return e.cval.is_null ? "NULL" : (e.type.id == T_VARCHAR ? "'" + e.cval.s + "'" : FormatValue(e.cval));
    case BExpr::COL:
      return "#" + std::to_string(e.col);
    default:
      break;
  }
  std::string s;
  switch (e.op) {
    case B_CAST: return "CAST(" + ExprToString(*e.ch[0]) + " AS " + e.type.ToString() + ")";
    case B_NOT: return "(NOT " + ExprToString(*e.ch[0]) + ")";
    case B_NEG: return "-(" + ExprToString(*e.ch[0]) + ")";
    case B_ABS: return "abs(" + ExprToString(*e.ch[0]) + ")";
    case B_ISNULL: return "(" + ExprToString(*e.ch[0]) + " IS NULL)";
    case B_ISNOTNULL: return "(" + ExprToString(*e.ch[0]) + " IS NOT NULL)";
    case B_CASE: s = "CASE"; for (auto &c : e.ch) s += " " + ExprToString(*c); return s + " END";
    case B_COALESCE: s = "coalesce("; break;
    case B_SYNTH: s = "mbx_synth("; break;
    case B_LENGTH: s = "length("; break;
    case B_LOWER: s = "lower("; break;
    case B_UPPER: s = "upper("; break;
    case B_DISTINCT: return "(" + ExprToString(*e.ch[0]) + " IS DISTINCT FROM " + ExprToString(*e.ch[1]) + ")";
    case B_NOT_DISTINCT: return "(" + ExprToString(*e.ch[0]) + " IS NOT DISTINCT FROM " + ExprToString(*e.ch[1]) + ")";
    default:
      return "(" + ExprToString(*e.ch[0]) + " " + OpSym(e.op) + " " + ExprToString(*e.ch[1]) + ")";
  }
  for (size_t i = 0; i < e.ch.size(); i++) s += (i ? ", " : "") + ExprToString(*e.ch[i]);
  return s + ")";
}

static bool BoundEq(const BExpr &a, const BExpr &b) {
  if (a.kind != b.kind || a.type != b.type) return false;
  if (a.kind == BExpr::COL) return a.col == b.col;
  if (a.kind == BExpr::CONST) {
    if (a.cval.is_null != b.cval.is_null) return false;
    if (a.cval.is_null) return true;
    return FormatValue(a.cval) == FormatValue(b.cval);
  }
  if (a.op != b.op || a.ch.size() != b.ch.size()) return false;
  for (size_t i = 0; i < a.ch.size(); i++)
    if (!BoundEq(*a.ch[i], *b.ch[i])) return false;
  return true;
}

// ---------------------------------------------------------------------------
// the binder
// ---------------------------------------------------------------------------
namespace {

struct ScopeCol {
  std::string name, qualifier;
  LogicalType type;
};

// BindSelectCapture: the constant node of every parameter reference, in bind order
static thread_local std::vector<std::pair<BExprPtr, int>> *g_param_nodes = nullptr;

struct BindCtx {
  std::vector<ScopeCol> scope;
  const std::vector<Value> *params = nullptr;
  // aggregate mode
  bool agg_mode = false;
  std::vector<BExprPtr> *groups = nullptr;
  std::vector<AggSpec> *aggs = nullptr;
  bool in_agg_arg = false;
  // select-list aliases usable in GROUP BY / ORDER BY
  const std::vector<ExprPtr> *select_list = nullptr;
};

std::string ColumnName(const Expr &e);

std::string ConstText(const Value &v) {
  if (v.is_null) return "NULL";
  if (v.type.id == T_VARCHAR) return "'" + v.s + "'";
  return FormatValue(v);
}

std::string ColumnName(const Expr &e) {
  if (!e.alias.empty()) return e.alias;
  switch (e.kind) {
    case Expr::COLREF: return e.name;
    case Expr::CONST: return ConstText(e.val);
    case Expr::FUNC: {
      std::string n = Lower(e.name);
      if (e.star && n == "count") return "count_star()";
      std::string s = n + "(" + (e.distinct ? "DISTINCT " : "");
      for (size_t i = 0; i < e.args.size(); i++) s += (i ? ", " : "") + ColumnName(*e.args[i]);
      return s + ")";
    }
    case Expr::BINARY: {
      std::string op = e.op;
      if (op == "<>") op = "!=";
      return "(" + ColumnName(*e.args[0]) + " " + op + " " + ColumnName(*e.args[1]) + ")";
    }
    case Expr::UNARY:
      if (e.op == "NOT") return "(NOT " + ColumnName(*e.args[0]) + ")";
      return "-(" + ColumnName(*e.args[0]) + ")";
    case Expr::CAST: return "CAST(" + ColumnName(*e.args[0]) + " AS " + e.cast.type.ToString() + ")";
    case Expr::ISNULL: return "(" + ColumnName(*e.args[0]) + (e.negated ? " IS NOT NULL)" : " IS NULL)");
    default: return e.text.empty() ? "?column?" : e.text;
  }
}

bool IsAggName(const std::string &n) {
  return n == "count" || n == "sum" || n == "min" || n == "max" || n == "avg" || n == "mean" ||
         n == "count_star";
}

bool ContainsAgg(const Expr &e) {
  if (e.kind == Expr::FUNC && IsAggName(Lower(e.name))) return true;
  for (auto &a : e.args)
    if (a && ContainsAgg(*a)) return true;
  return false;
}

BExprPtr BindExpr(const Expr &e, BindCtx &ctx);

BExprPtr BindCompare(BOp op, BExprPtr l, BExprPtr r, bool l_strlit = false, bool r_strlit = false) {
  LogicalType t;
  // string literal vs typed value: cast the literal to the other side's type
  if (l_strlit && r->type.id != T_VARCHAR && r->type.id != T_SQLNULL) t = r->type;
  else if (r_strlit && l->type.id != T_VARCHAR && l->type.id != T_SQLNULL) t = l->type;
  else t = MaxType(l->type, r->type);
  if (t.id == T_SQLNULL) t = LogicalType(T_INTEGER);
  return Fold(MkFunc(op, LogicalType(T_BOOLEAN), {CastTo(l, t), CastTo(r, t)}));
}

bool IsStrLit(const Expr &e) { return e.kind == Expr::CONST && e.name == "string_literal"; }

BExprPtr BindArith(const std::string &opname, BExprPtr l, BExprPtr r) {
  LogicalType lt = l->type, rt = r->type;
  if (lt.id == T_SQLNULL) lt = rt.id == T_SQLNULL ? LogicalType(T_INTEGER) : rt;
  if (rt.id == T_SQLNULL) rt = lt;
  BOp op = opname == "+" ? B_ADD : opname == "-" ? B_SUB : opname == "*" ? B_MUL : opname == "/" ? B_DIV
           : opname == "//" ? B_IDIV : B_MOD;
  // date/timestamp +/- interval, date +/- integer
  if ((lt.id == T_DATE || lt.id == T_TIMESTAMP) && (op == B_ADD || op == B_SUB)) {
    if (rt.id == T_INTERVAL) {
      LogicalType res = lt.id == T_DATE ? LogicalType(T_TIMESTAMP) : lt;
      return Fold(MkFunc(op, res, {l, r}));
    }
    if (IsIntegral(rt.id) && lt.id == T_DATE) {
      Value iv;
      // date + n days
      auto ivc = MkFunc(B_CAST, LogicalType(T_INTERVAL), {r});
      if (r->kind == BExpr::CONST && !r->cval.is_null) {
        Value x;
        x.type = LogicalType(T_INTERVAL);
        x.is_null = false;
        x.iv.days = (int32_t)r->cval.i;
        ivc = MkConst(x);
      }
      return Fold(MkFunc(B_CAST, LogicalType(T_DATE), {Fold(MkFunc(op, LogicalType(T_TIMESTAMP), {l, ivc}))}));
    }
  }
  if (!IsNumeric(lt.id) && lt.id != T_BOOLEAN) ThrowError("Binder", "No function matches '" + opname + "(" + lt.ToString() + ", " + rt.ToString() + ")'");
  if (!IsNumeric(rt.id) && rt.id != T_BOOLEAN) ThrowError("Binder", "No function matches '" + opname + "(" + lt.ToString() + ", " + rt.ToString() + ")'");
  if (op == B_DIV) {
    LogicalType d(T_DOUBLE);
    return Fold(MkFunc(op, d, {CastTo(l, d), CastTo(r, d)}));
  }
  LogicalType res;
  if (lt.id == T_DOUBLE || rt.id == T_DOUBLE || lt.id == T_FLOAT || rt.id == T_FLOAT) {
    res = (lt.id == T_FLOAT && rt.id == T_FLOAT) ? LogicalType(T_FLOAT) : LogicalType(T_DOUBLE);
    return Fold(MkFunc(op, res, {CastTo(l, res), CastTo(r, res)}));
  }
  if (lt.id == T_DECIMAL || rt.id == T_DECIMAL) {
    LogicalType dl = AsDecimal(lt), dr = AsDecimal(rt);
    if (op == B_MUL) {
      int s = dl.scale + dr.scale;
      int w = dl.width + dr.width;
      if (w > 38) w = 38;
      if (s > 38) ThrowError("Binder", "Decimal multiplication scale too large");
      res = LogicalType::Decimal(w, s);
      // operands keep their scale; widen their storage only
      return Fold(MkFunc(op, res, {CastTo(l, dl), CastTo(r, dr)}));
    }
    if (op == B_IDIV) {
      LogicalType d(T_DOUBLE);
      return Fold(MkFunc(B_CAST, LogicalType(T_BIGINT), {Fold(MkFunc(B_IDIV, d, {CastTo(l, d), CastTo(r, d)}))}));
    }
    int s = std::max(dl.scale, dr.scale);
    int ip = std::max(dl.width - dl.scale, dr.width - dr.scale);
    int w = ip + s + (op == B_MOD ? 0 : 1);
    if (w > 38) w = 38;
    res = LogicalType::Decimal(w, s);
    return Fold(MkFunc(op, res, {CastTo(l, res), CastTo(r, res)}));
  }
  // integers (BOOLEAN arithmetic is not allowed in DuckDB; treat as error)
  if (lt.id == T_BOOLEAN || rt.id == T_BOOLEAN)
    ThrowError("Binder", "No function matches '" + opname + "(" + lt.ToString() + ", " + rt.ToString() + ")'");
  res = MaxType(lt, rt);
  return Fold(MkFunc(op, res, {CastTo(l, res), CastTo(r, res)}));
}

BExprPtr BindAggregate(const Expr &e, BindCtx &ctx) {
  std::string n = Lower(e.name);
  if (!ctx.agg_mode || ctx.in_agg_arg)
    ThrowError("Binder", "aggregate function calls cannot be nested or appear here: " + ColumnName(e));
  AggSpec a;
  a.distinct = e.distinct;
  if (e.star || n == "count_star") {
    a.kind = A_COUNT_STAR;
    a.type = LogicalType(T_BIGINT);
  } else {
    if (e.args.size() != 1) ThrowError("Binder", "No function matches the given name and argument types '" + n + "'");
    BindCtx sub = ctx;
    sub.agg_mode = false;
    sub.in_agg_arg = true;
    BExprPtr arg = BindExpr(*e.args[0], sub);
    a.arg = arg;
    LogicalType at = arg->type;
    if (at.id == T_SQLNULL) {
      at = LogicalType(T_INTEGER);
      a.arg = CastTo(arg, at);
    }
    if (n == "count") {
      a.kind = A_COUNT;
      a.type = LogicalType(T_BIGINT);
    } else if (n == "sum") {
      a.kind = A_SUM;
      if (IsIntegral(at.id) || at.id == T_BOOLEAN) a.type = LogicalType(T_HUGEINT);
      else if (at.id == T_DECIMAL) a.type = LogicalType::Decimal(38, at.scale);
      else if (at.id == T_FLOAT || at.id == T_DOUBLE) {
        a.type = LogicalType(T_DOUBLE);
        a.arg = CastTo(a.arg, a.type);
      } else ThrowError("Binder", "No function matches the given name and argument types 'sum(" + at.ToString() + ")'");
    } else if (n == "avg" || n == "mean") {
      a.kind = A_AVG;
      if (!IsNumeric(at.id)) ThrowError("Binder", "No function matches the given name and argument types 'avg(" + at.ToString() + ")'");
      if (at.id == T_FLOAT) a.arg = CastTo(a.arg, LogicalType(T_DOUBLE));
      a.type = LogicalType(T_DOUBLE);
    } else if (n == "min" || n == "max") {
      a.kind = n == "min" ? A_MIN : A_MAX;
      a.type = at;
    }
  }
  if (a.distinct && a.kind != A_COUNT && a.kind != A_MIN && a.kind != A_MAX)
    ThrowError("Not implemented", "DISTINCT aggregates are not supported by the MI355X backend");
  if (a.distinct) a.distinct = a.kind == A_COUNT;  // MIN/MAX DISTINCT == MIN/MAX
  int ng = (int)ctx.groups->size();
  // reuse identical aggregates
  for (size_t i = 0; i < ctx.aggs->size(); i++) {
    const AggSpec &o = (*ctx.aggs)[i];
    if (o.kind == a.kind && o.distinct == a.distinct &&
        ((!o.arg && !a.arg) || (o.arg && a.arg && BoundEq(*o.arg, *a.arg))))
      return MkCol(ng + (int)i, o.type);
  }
  ctx.aggs->push_back(a);
  return MkCol(ng + (int)ctx.aggs->size() - 1, a.type);
}

BExprPtr BindFunction(const Expr &e, BindCtx &ctx) {
  std::string n = Lower(e.name);
  if (IsAggName(n)) return BindAggregate(e, ctx);
  std::vector<BExprPtr> args;
  for (auto &a : e.args) args.push_back(BindExpr(*a, ctx));
  auto need = [&](size_t k) {
    if (args.size() != k) ThrowError("Binder", "No function matches the given name and argument types '" + n + "'");
  };
  if (n == "coalesce" || n == "ifnull") {
    if (args.empty()) ThrowError("Binder", "coalesce requires arguments");
    LogicalType t(T_SQLNULL);
    for (auto &a : args) t = MaxType(t, a->type);
    if (t.id == T_SQLNULL) t = LogicalType(T_INTEGER);
    for (auto &a : args) a = CastTo(a, t);
    return Fold(MkFunc(B_COALESCE, t, args));
  }
  if (n == "abs") {
    need(1);
    return Fold(MkFunc(B_ABS, args[0]->type, args));
  }
  if (n == "concat") {
    BExprPtr acc;
    for (auto &a : args) {
      BExprPtr s = CastTo(a, LogicalType(T_VARCHAR));
      // concat() treats NULL as empty string
      s = MkFunc(B_COALESCE, LogicalType(T_VARCHAR), {s, MkConst(Value::Varchar(""))});
      acc = acc ? MkFunc(B_CONCAT, LogicalType(T_VARCHAR), {acc, s}) : s;
    }
    return Fold(acc ? acc : MkConst(Value::Varchar("")));
  }
  if (n == "length" || n == "strlen" || n == "len") {
    need(1);
    return Fold(MkFunc(B_LENGTH, LogicalType(T_BIGINT), {CastTo(args[0], LogicalType(T_VARCHAR))}));
  }
  if (n == "lower" || n == "lcase" || n == "upper" || n == "ucase") {
    need(1);
    return Fold(MkFunc(n[0] == 'l' ? B_LOWER : B_UPPER, LogicalType(T_VARCHAR), {CastTo(args[0], LogicalType(T_VARCHAR))}));
  }
  if (n == "mbx_synth") {
    // mbx_synth(seed, i, m) = splitmix64(seed + i) mod m  (synthetic column
    // generator of the benchmark configurations)
    need(3);
    LogicalType b(T_BIGINT);
    return Fold(MkFunc(B_SYNTH, b, {CastTo(args[0], b), CastTo(args[1], b), CastTo(args[2], b)}));
  }
  if (n == "least" || n == "greatest") {
    if (args.empty()) ThrowError("Binder", n + " requires arguments");
    LogicalType t(T_SQLNULL);
    for (auto &a : args) t = MaxType(t, a->type);
    BExprPtr acc = CastTo(args[0], t);
    for (size_t i = 1; i < args.size(); i++) {
      BExprPtr b = CastTo(args[i], t);
      BExprPtr cond = MkFunc(n == "least" ? B_LT : B_GT, LogicalType(T_BOOLEAN), {acc, b});
      acc = Fold(MkFunc(B_CASE, t, {cond, acc, b}));
    }
    return acc;
  }
  ThrowError("Catalog", "Scalar Function with name " + n + " does not exist!");
}

BExprPtr BindExprInner(const Expr &e, BindCtx &ctx);

// In aggregate mode, any sub-expression equal to a GROUP BY expression
// becomes a reference to that group column.
// expression nesting bound of the binder's recursion (DuckDB's
// max_expression_depth default): a deep left-leaning chain such as
// 1 + 1 + ... parses iteratively but binds recursively
static thread_local int g_bind_depth = 0;
struct BindDepth {
  BindDepth() {
    if (++g_bind_depth > 1000) {
      g_bind_depth = 0;  // the binder unwinds through the throw
      ThrowError("Binder", "Max expression depth limit of 1000 exceeded. Use \"SET max_expression_depth TO x\" to "
                           "increase the maximum expression depth.");
    }
  }
  ~BindDepth() {
    if (g_bind_depth > 0) g_bind_depth--;
  }
};

BExprPtr BindExpr(const Expr &e, BindCtx &ctx) {
  BindDepth depth_guard;
  if (ctx.agg_mode && !ctx.in_agg_arg && !ContainsAgg(e) && e.kind != Expr::CONST && e.kind != Expr::PARAM) {
    BindCtx sub = ctx;
    sub.agg_mode = false;
    BExprPtr b;
    try {
      b = BindExprInner(e, sub);
    } catch (EngineError &) {
      b = nullptr;
    }
    if (b) {
      for (size_t g = 0; g < ctx.groups->size(); g++)
        if (BoundEq(*b, *(*ctx.groups)[g])) return MkCol((int)g, b->type);
      if (IsConstTree(*b)) return b;
      if (e.kind == Expr::COLREF)
        ThrowError("Binder", "column \"" + e.name + "\" must appear in the GROUP BY clause or must be part of an aggregate function.");
    }
  }
  return BindExprInner(e, ctx);
}

BExprPtr BindExprInner(const Expr &e, BindCtx &ctx) {
  switch (e.kind) {
    case Expr::CONST: {
      auto c = MkConst(e.val);
      if (e.val.is_null) c->type = LogicalType(T_SQLNULL);
      return c;
    }
    case Expr::PARAM: {
      if (!ctx.params || e.param_index < 1 || e.param_index > (int)ctx.params->size() ||
          (*ctx.params)[e.param_index - 1].type.id == T_INVALID)
        ThrowError("Invalid Input", "Values were not provided for the following prepared statement parameters: " +
                                        std::to_string(e.param_index));
      Value v = (*ctx.params)[e.param_index - 1];
      auto c = MkConst(v);
      if (v.is_null) c->type = LogicalType(T_SQLNULL);
      if (g_param_nodes) g_param_nodes->push_back({c, e.param_index - 1});
      return c;
    }
    case Expr::COLREF: {
      int found = -1;
      for (size_t i = 0; i < ctx.scope.size(); i++) {
        const ScopeCol &sc = ctx.scope[i];
        if (Lower(sc.name) == Lower(e.name) && (e.qualifier.empty() || Lower(sc.qualifier) == Lower(e.qualifier))) {
          if (found >= 0) ThrowError("Binder", "Ambiguous reference to column name \"" + e.name + "\"");
          found = (int)i;
        }
      }
      if (found < 0) {
        // select-list alias (DuckDB allows aliases in WHERE/GROUP BY)
        if (ctx.select_list) {
          for (auto &s : *ctx.select_list)
            if (!s->alias.empty() && Lower(s->alias) == Lower(e.name) && e.qualifier.empty()) {
              BindCtx sub = ctx;
              sub.select_list = nullptr;
              return BindExpr(*s, sub);
            }
        }
        ThrowError("Binder", "Referenced column \"" + e.name + "\" not found in FROM clause!");
      }
      return MkCol(found, ctx.scope[found].type);
    }
    case Expr::STAR:
      ThrowError("Binder", "* is not allowed here");
    case Expr::UNARY: {
      BExprPtr a = BindExpr(*e.args[0], ctx);
      if (e.op == "NOT") {
        return Fold(MkFunc(B_NOT, LogicalType(T_BOOLEAN), {CastTo(a, LogicalType(T_BOOLEAN))}));
      }
      LogicalType t = a->type.id == T_SQLNULL ? LogicalType(T_INTEGER) : a->type;
      if (!IsNumeric(t.id) && t.id != T_INTERVAL) ThrowError("Binder", "No function matches '-(" + t.ToString() + ")'");
      return Fold(MkFunc(B_NEG, t, {CastTo(a, t)}));
    }
    case Expr::BINARY: {
      const std::string &op = e.op;
      if (op == "AND" || op == "OR") {
        LogicalType b(T_BOOLEAN);
        BExprPtr l = CastTo(BindExpr(*e.args[0], ctx), b), r = CastTo(BindExpr(*e.args[1], ctx), b);
        return Fold(MkFunc(op == "AND" ? B_AND : B_OR, b, {l, r}));
      }
      BExprPtr l = BindExpr(*e.args[0], ctx), r = BindExpr(*e.args[1], ctx);
      if (op == "=" || op == "<>" || op == "<" || op == "<=" || op == ">" || op == ">=" ||
          op == "IS DISTINCT FROM" || op == "IS NOT DISTINCT FROM") {
        BOp bo = op == "=" ? B_EQ : op == "<>" ? B_NE : op == "<" ? B_LT : op == "<=" ? B_LE : op == ">" ? B_GT
                 : op == ">=" ? B_GE : op == "IS DISTINCT FROM" ? B_DISTINCT : B_NOT_DISTINCT;
        return BindCompare(bo, l, r, IsStrLit(*e.args[0]), IsStrLit(*e.args[1]));
      }
      if (op == "||") {
        LogicalType v(T_VARCHAR);
        return Fold(MkFunc(B_CONCAT, v, {CastTo(l, v), CastTo(r, v)}));
      }
      return BindArith(op, l, r);
    }
    case Expr::FUNC:
      return BindFunction(e, ctx);
    case Expr::CAST: {
      BExprPtr a = BindExpr(*e.args[0], ctx);
      if (a->type.id == T_SQLNULL) {
        auto c = MkConst(Value::Null(e.cast.type));
        c->type = e.cast.type;
        return c;
      }
      return Fold(CastTo(a, e.cast.type));
    }
    case Expr::ISNULL: {
      BExprPtr a = BindExpr(*e.args[0], ctx);
      return Fold(MkFunc(e.negated ? B_ISNOTNULL : B_ISNULL, LogicalType(T_BOOLEAN), {a}));
    }
    case Expr::BETWEEN: {
      BExprPtr x = BindExpr(*e.args[0], ctx);
      BExprPtr lo = BindCompare(B_GE, x, BindExpr(*e.args[1], ctx), false, IsStrLit(*e.args[1]));
      BExprPtr hi = BindCompare(B_LE, x, BindExpr(*e.args[2], ctx), false, IsStrLit(*e.args[2]));
      BExprPtr r = Fold(MkFunc(B_AND, LogicalType(T_BOOLEAN), {lo, hi}));
      if (e.negated) r = Fold(MkFunc(B_NOT, LogicalType(T_BOOLEAN), {r}));
      return r;
    }
    case Expr::INLIST: {
      BExprPtr x = BindExpr(*e.args[0], ctx);
      BExprPtr acc;
      for (size_t i = 1; i < e.args.size(); i++) {
        BExprPtr c = BindCompare(B_EQ, x, BindExpr(*e.args[i], ctx), false, IsStrLit(*e.args[i]));
        acc = acc ? Fold(MkFunc(B_OR, LogicalType(T_BOOLEAN), {acc, c})) : c;
      }
      if (e.negated) acc = Fold(MkFunc(B_NOT, LogicalType(T_BOOLEAN), {acc}));
      return acc;
    }
    case Expr::CASE: {
      std::vector<BExprPtr> ch;
      size_t i = 0;
      BExprPtr operand;
      if (e.case_operand) operand = BindExpr(*e.args[i++], ctx);
      size_t end = e.args.size() - (e.has_else ? 1 : 0);
      std::vector<BExprPtr> conds, vals;
      for (; i + 1 < end + 1 && i < end; i += 2) {
        BExprPtr w = BindExpr(*e.args[i], ctx);
        if (operand) w = BindCompare(B_EQ, operand, w, false, IsStrLit(*e.args[i]));
        conds.push_back(CastTo(w, LogicalType(T_BOOLEAN)));
        vals.push_back(BindExpr(*e.args[i + 1], ctx));
      }
      BExprPtr els = e.has_else ? BindExpr(*e.args.back(), ctx) : nullptr;
      LogicalType t(T_SQLNULL);
      for (auto &v : vals) t = MaxType(t, v->type);
      if (els) t = MaxType(t, els->type);
      if (t.id == T_SQLNULL) t = LogicalType(T_INTEGER);
      for (size_t k = 0; k < conds.size(); k++) {
        ch.push_back(conds[k]);
        ch.push_back(CastTo(vals[k], t));
      }
      if (els) ch.push_back(CastTo(els, t));
      return Fold(MkFunc(B_CASE, t, ch));
    }
  }
  ThrowError("Internal", "unhandled expression kind");
}

int64_t ConstInt(const Expr &e, const std::vector<Value> &params, const char *what) {
  BindCtx ctx;
  ctx.params = &params;
  BExprPtr b = BindExpr(e, ctx);
  if (!IsConstTree(*b)) ThrowError("Binder", std::string(what) + " must be a constant");
  Value v = EvalConst(*b);
  if (v.is_null) ThrowError("Binder", std::string(what) + " cannot be NULL");
  Value iv = CastValue(v, LogicalType(T_BIGINT));
  return (int64_t)iv.i;
}

}  // namespace

// ---------------------------------------------------------------------------
static BoundSelectPtr BindSelectOne(const Select &sel, Catalog &cat, const std::vector<Value> &params);

static void BindSource(const TableRef &tr, BoundSource &src, Catalog &cat, const std::vector<Value> &params) {
  switch (tr.kind) {
    case TableRef::NONE:
      src.kind = BoundSource::ONE_ROW;
      break;
    case TableRef::TABLE: {
      TablePtr t = cat.Find(tr.name);
      if (!t) ThrowError("Catalog", "Table with name " + tr.name + " does not exist!\nDid you mean \"" + tr.name + "\"?");
      src.kind = BoundSource::TABLE;
      src.table = t;
      for (size_t i = 0; i < t->cols.size(); i++) {
        src.col_types.push_back(t->cols[i].type);
        src.col_names.push_back(t->col_names[i]);
      }
      src.alias = tr.alias.empty() ? t->name : tr.alias;
      break;
    }
    case TableRef::RANGE: {
      src.kind = BoundSource::RANGE;
      std::vector<int64_t> a;
      for (auto &x : tr.args) a.push_back(ConstInt(*x, params, "range argument"));
      if (a.empty() || a.size() > 3) ThrowError("Binder", "range requires 1 to 3 arguments");
      if (a.size() == 1) {
        src.range_start = 0;
        src.range_stop = a[0];
      } else {
        src.range_start = a[0];
        src.range_stop = a[1];
        if (a.size() == 3) src.range_step = a[2];
      }
      if (src.range_step == 0) ThrowError("Binder", "interval cannot be 0!");
      src.range_inclusive = tr.name == "generate_series";
      src.col_types.push_back(LogicalType(T_BIGINT));
      src.col_names.push_back(tr.name);
      src.alias = tr.alias.empty() ? tr.name : tr.alias;
      break;
    }
    case TableRef::VALUES: {
      src.kind = BoundSource::VALUES;
      size_t ncol = tr.rows[0].size();
      std::vector<std::vector<Value>> vals;
      std::vector<LogicalType> types(ncol, LogicalType(T_SQLNULL));
      for (auto &row : tr.rows) {
        if (row.size() != ncol) ThrowError("Binder", "VALUES lists must all be the same length");
        std::vector<Value> vr;
        for (size_t c = 0; c < ncol; c++) {
          BindCtx ctx;
          ctx.params = &params;
          BExprPtr b = BindExpr(*row[c], ctx);
          if (!IsConstTree(*b)) ThrowError("Binder", "VALUES entries must be constant");
          Value v = EvalConst(*b);
          if (v.is_null) v.type = b->type;
          types[c] = MaxType(types[c], b->type);
          vr.push_back(v);
        }
        vals.push_back(vr);
      }
      for (auto &t : types)
        if (t.id == T_SQLNULL) t = LogicalType(T_INTEGER);
      for (auto &vr : vals)
        for (size_t c = 0; c < ncol; c++) vr[c] = CastValue(vr[c], types[c]);
      src.rows = vals;
      src.col_types = types;
      for (size_t c = 0; c < ncol; c++) src.col_names.push_back("col" + std::to_string(c));
      src.alias = tr.alias.empty() ? "valueslist" : tr.alias;
      break;
    }
    case TableRef::SUBQUERY: {
      src.kind = BoundSource::SUBQUERY;
      src.sub = BindSelect(*tr.sub, cat, params);
      src.col_types = src.sub->OutTypes();
      src.col_names = src.sub->names;
      src.alias = tr.alias.empty() ? "unnamed_subquery" : tr.alias;
      break;
    }
  }
  if (!tr.col_aliases.empty()) {
    if (tr.col_aliases.size() > src.col_names.size())
      ThrowError("Binder", "table \"" + src.alias + "\" has " + std::to_string(src.col_names.size()) +
                                " columns available but " + std::to_string(tr.col_aliases.size()) + " columns specified");
    for (size_t i = 0; i < tr.col_aliases.size(); i++) src.col_names[i] = tr.col_aliases[i];
  }
}

static BoundSelectPtr BindSelectOne(const Select &sel, Catalog &cat, const std::vector<Value> &params) {
  auto bs = std::make_shared<BoundSelect>();
  BindSource(sel.from, bs->src, cat, params);
  BindCtx base;
  base.params = &params;
  for (size_t i = 0; i < bs->src.col_names.size(); i++)
    base.scope.push_back({bs->src.col_names[i], bs->src.alias, bs->src.col_types[i]});
  base.select_list = &sel.list;

  // expand *
  std::vector<ExprPtr> list;
  for (auto &e : sel.list) {
    if (e->kind == Expr::STAR) {
      if (bs->src.kind == BoundSource::ONE_ROW) ThrowError("Binder", "SELECT * expression without FROM clause!");
      for (size_t i = 0; i < bs->src.col_names.size(); i++) {
        auto c = std::make_shared<Expr>();
        c->kind = Expr::COLREF;
        c->name = bs->src.col_names[i];
        list.push_back(c);
      }
    } else {
      list.push_back(e);
    }
  }

  if (sel.where) {
    if (ContainsAgg(*sel.where)) ThrowError("Binder", "WHERE clause cannot contain aggregates!");
    BindCtx ctx = base;
    ctx.select_list = nullptr;
    BExprPtr w = BindExpr(*sel.where, ctx);
    bs->where = CastTo(w, LogicalType(T_BOOLEAN));
  }

  bool has_agg = !sel.group_by.empty() || sel.having;
  for (auto &e : list)
    if (ContainsAgg(*e)) has_agg = true;
  bs->is_agg = has_agg || sel.distinct;

  std::vector<std::string> names;
  for (auto &e : list) names.push_back(ColumnName(*e));

  if (bs->is_agg) {
    BindCtx gctx = base;
    for (auto &g : sel.group_by) {
      if (g->kind == Expr::STAR) {  // GROUP BY ALL: every non-aggregate select item
        for (auto &e : list)
          if (!ContainsAgg(*e)) bs->groups.push_back(BindExpr(*e, gctx));
        continue;
      }
      if (g->kind == Expr::CONST && !g->val.is_null && IsIntegral(g->val.type.id)) {
        int64_t k = (int64_t)g->val.i;
        if (k < 1 || k > (int64_t)list.size()) ThrowError("Binder", "GROUP BY term out of range");
        bs->groups.push_back(BindExpr(*list[k - 1], gctx));
        continue;
      }
      bs->groups.push_back(BindExpr(*g, gctx));
    }
    if (sel.distinct && sel.group_by.empty()) {
      for (auto &e : list) bs->groups.push_back(BindExpr(*e, gctx));
    }
    BindCtx actx = base;
    actx.agg_mode = true;
    actx.groups = &bs->groups;
    actx.aggs = &bs->aggs;
    for (auto &e : list) bs->outputs.push_back(BindExpr(*e, actx));
    if (sel.having) bs->having = CastTo(BindExpr(*sel.having, actx), LogicalType(T_BOOLEAN));
  } else {
    for (auto &e : list) bs->outputs.push_back(BindExpr(*e, base));
  }
  for (auto &o : bs->outputs)
    if (o->type.id == T_SQLNULL) {
      // DuckDB materializes an untyped NULL column as INTEGER
      o = CastTo(o, LogicalType(T_INTEGER));
      if (o->kind == BExpr::CONST) o->type = LogicalType(T_INTEGER);
    }
  bs->names = names;
  return bs;
}

BoundSelectPtr BindSelect(const Select &sel, Catalog &cat, const std::vector<Value> &params) {
  BoundSelectPtr first = BindSelectOne(sel, cat, params);
  for (auto &u : sel.union_all) {
    BoundSelectPtr b = BindSelect(*u, cat, params);
    if (b->outputs.size() != first->outputs.size())
      ThrowError("Binder", "Set operations can only apply to expressions with the same number of result columns");
    first->union_all.push_back(b);
  }
  if (!first->union_all.empty()) {
    for (size_t c = 0; c < first->outputs.size(); c++) {
      LogicalType t = first->outputs[c]->type;
      for (auto &b : first->union_all) t = MaxType(t, b->outputs[c]->type);
      first->outputs[c] = CastTo(first->outputs[c], t);
      for (auto &b : first->union_all) b->outputs[c] = CastTo(b->outputs[c], t);
    }
  }
  // ORDER BY over output columns (alias, position, or an output expression)
  for (auto &oi : sel.order_by) {
    BoundOrder bo;
    bo.desc = oi.desc;
    bo.nulls_first = oi.nulls_first < 0 ? false : oi.nulls_first == 1;  // DuckDB default NULLS LAST
    const Expr &e = *oi.expr;
    int idx = -1;
    if (e.kind == Expr::CONST && !e.val.is_null && IsIntegral(e.val.type.id)) {
      idx = (int)e.val.i - 1;
      if (idx < 0 || idx >= (int)first->outputs.size()) ThrowError("Binder", "ORDER term out of range");
    } else if (e.kind == Expr::COLREF && e.qualifier.empty()) {
      for (size_t i = 0; i < first->names.size(); i++)
        if (Lower(first->names[i]) == Lower(e.name)) {
          idx = (int)i;
          break;
        }
    }
    if (idx < 0) {
      // expression text equal to an output name
      std::string nm = ColumnName(e);
      for (size_t i = 0; i < first->names.size(); i++)
        if (first->names[i] == nm) {
          idx = (int)i;
          break;
        }
    }
    if (idx < 0) {
      if (!first->union_all.empty()) ThrowError("Binder", "ORDER BY of a UNION must refer to an output column");
      // hidden sort key: bind over the source (or the aggregate relation)
      BindCtx ctx;
      ctx.params = &params;
      for (size_t i = 0; i < first->src.col_names.size(); i++)
        ctx.scope.push_back({first->src.col_names[i], first->src.alias, first->src.col_types[i]});
      if (first->is_agg) {
        ctx.agg_mode = true;
        ctx.groups = &first->groups;
        ctx.aggs = &first->aggs;
      }
      BExprPtr b = BindExpr(e, ctx);
      first->outputs.push_back(b);
      first->names.push_back("__order_" + std::to_string(first->outputs.size()));
      idx = (int)first->outputs.size() - 1;
    }
    bo.expr = MkCol(idx, first->outputs[idx]->type);
    first->order.push_back(bo);
  }
  if (sel.limit) first->limit = ConstInt(*sel.limit, params, "LIMIT");
  if (sel.offset) first->offset = ConstInt(*sel.offset, params, "OFFSET");
  if (first->limit < -1) ThrowError("Binder", "LIMIT cannot be negative");
  return first;
}

bool IsHostConstantSelect(const BoundSelect &s) {
  if (s.src.kind != BoundSource::ONE_ROW) return false;
  if (s.where && !IsConstTree(*s.where)) return false;
  for (auto &u : s.union_all)
    if (!IsHostConstantSelect(*u)) return false;
  return true;
}

std::string ExplainSelect(const BoundSelect &s, int ind) {
  std::string pad(ind, ' ');
  std::string out;
  out += pad + "SELECT";
  for (size_t i = 0; i < s.outputs.size(); i++)
    out += (i ? ", " : " ") + ExprToString(*s.outputs[i]) + " AS " + s.names[i] + " :: " + s.outputs[i]->type.ToString();
  out += "\n";
  switch (s.src.kind) {
    case BoundSource::ONE_ROW: out += pad + "  FROM <one row>\n"; break;
    case BoundSource::RANGE:
      out += pad + "  FROM RANGE(" + std::to_string(s.src.range_start) + ", " + std::to_string(s.src.range_stop) + ", " +
             std::to_string(s.src.range_step) + (s.src.range_inclusive ? ", inclusive" : "") + ")\n";
      break;
    case BoundSource::TABLE: out += pad + "  FROM TABLE " + s.src.table->name + "\n"; break;
    case BoundSource::VALUES: out += pad + "  FROM VALUES[" + std::to_string(s.src.rows.size()) + " rows]\n"; break;
    case BoundSource::SUBQUERY: out += pad + "  FROM (\n" + ExplainSelect(*s.src.sub, ind + 4) + pad + "  )\n"; break;
  }
  if (s.where) out += pad + "  WHERE " + ExprToString(*s.where) + "\n";
  if (s.is_agg) {
    out += pad + "  AGGREGATE groups=[";
    for (size_t i = 0; i < s.groups.size(); i++) out += (i ? ", " : "") + ExprToString(*s.groups[i]);
    out += "] aggs=[";
    static const char *an[] = {"count_star", "count", "sum", "min", "max", "avg"};
    for (size_t i = 0; i < s.aggs.size(); i++)
      out += (i ? ", " : "") + std::string(an[s.aggs[i].kind]) + "(" + (s.aggs[i].arg ? ExprToString(*s.aggs[i].arg) : "") +
             ") :: " + s.aggs[i].type.ToString();
    out += "]\n";
  }
  if (s.having) out += pad + "  HAVING " + ExprToString(*s.having) + "\n";
  for (auto &o : s.order) out += pad + "  ORDER BY " + ExprToString(*o.expr) + (o.desc ? " DESC" : " ASC") + "\n";
  if (s.limit >= 0) out += pad + "  LIMIT " + std::to_string(s.limit) + " OFFSET " + std::to_string(s.offset) + "\n";
  for (auto &u : s.union_all) out += pad + "UNION ALL\n" + ExplainSelect(*u, ind);
  return out;
}

TablePtr Catalog::Find(const std::string &name) const {
  auto it = tables.find(Lower(name));
  return it == tables.end() ? nullptr : it->second;
}

}  // namespace mbx

namespace mbx {

static void CollectExprNodes(const BExpr *e, std::set<const BExpr *> &out) {
  if (!e || !out.insert(e).second) return;
  for (auto &c : e->ch) CollectExprNodes(c.get(), out);
}

static void CollectPlanNodes(const BoundSelect &s, std::set<const BExpr *> &out) {
  CollectExprNodes(s.where.get(), out);
  CollectExprNodes(s.having.get(), out);
  for (auto &g : s.groups) CollectExprNodes(g.get(), out);
  for (auto &a : s.aggs) CollectExprNodes(a.arg.get(), out);
  for (auto &o : s.outputs) CollectExprNodes(o.get(), out);
  for (auto &o : s.order) CollectExprNodes(o.expr.get(), out);
  if (s.src.sub) CollectPlanNodes(*s.src.sub, out);
  for (auto &u : s.union_all) CollectPlanNodes(*u, out);
}

BoundSelectPtr BindSelectCapture(const Select &sel, Catalog &cat, const std::vector<Value> &params, bool *patchable,
                                 std::vector<std::pair<BExprPtr, int>> *nodes) {
  nodes->clear();
  g_param_nodes = nodes;
  BoundSelectPtr b;
  try {
    b = BindSelect(sel, cat, params);
  } catch (...) {
    g_param_nodes = nullptr;
    throw;
  }
  g_param_nodes = nullptr;
  // patchable when every parameter the statement has was bound into a node that
  // is still in the plan (not folded away, not a LIMIT/VALUES/range argument)
  std::set<const BExpr *> live;
  CollectPlanNodes(*b, live);
  std::vector<bool> seen(params.size(), false);
  bool ok = true;
  for (auto &pn : *nodes) {
    if (!live.count(pn.first.get())) ok = false;
    if (pn.second >= 0 && pn.second < (int)seen.size()) seen[pn.second] = true;
  }
  for (bool x : seen) ok = ok && x;
  *patchable = ok;
  return b;
}

}  // namespace mbx
