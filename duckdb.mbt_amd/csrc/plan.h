// plan.h — bound (typed) plans produced by the binder and run by the executor.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "sql.h"
#include "types.h"

namespace mbx {

enum BOp : uint8_t {
  B_ADD, B_SUB, B_MUL, B_DIV, B_IDIV, B_MOD, B_NEG, B_ABS,
  B_EQ, B_NE, B_LT, B_LE, B_GT, B_GE, B_DISTINCT, B_NOT_DISTINCT,
  B_AND, B_OR, B_NOT, B_ISNULL, B_ISNOTNULL,
  B_CAST, B_CASE, B_COALESCE, B_CONCAT, B_SYNTH, B_LENGTH, B_LOWER, B_UPPER,
};

enum AggKind : uint8_t { A_COUNT_STAR, A_COUNT, A_SUM, A_MIN, A_MAX, A_AVG };

struct BExpr;
typedef std::shared_ptr<BExpr> BExprPtr;

struct BExpr {
  enum Kind { CONST, COL, FUNC } kind = CONST;
  LogicalType type;
  Value cval;  // CONST
  int col = -1;  // COL: column of the input relation
  BOp op = B_ADD;
  std::vector<BExprPtr> ch;
  // CASE: ch = [when0, then0, when1, then1, ..., else]
};

struct AggSpec {
  AggKind kind;
  BExprPtr arg;  // over the source relation (null for COUNT(*))
  LogicalType type;  // result type
  bool distinct = false;
};

struct Table;  // engine.h

struct BoundSource {
  enum Kind { ONE_ROW, RANGE, TABLE, VALUES, SUBQUERY } kind = ONE_ROW;
  int64_t range_start = 0, range_stop = 0, range_step = 1;
  bool range_inclusive = false;
  std::shared_ptr<Table> table;
  std::vector<std::vector<Value>> rows;  // VALUES, already cast to col_types
  std::shared_ptr<struct BoundSelect> sub;
  std::vector<LogicalType> col_types;
  std::vector<std::string> col_names;
  std::string alias;
  int64_t RangeCount() const;
};

struct BoundOrder {
  BExprPtr expr;  // over the output columns of the select
  bool desc = false;
  bool nulls_first = false;
};

struct BoundSelect {
  BoundSource src;
  BExprPtr where;  // over source columns
  bool is_agg = false;
  std::vector<BExprPtr> groups;  // over source columns
  std::vector<AggSpec> aggs;
  // Outputs.  Non-aggregate: over source columns.  Aggregate: over the
  // aggregate relation [groups..., aggs...].
  std::vector<BExprPtr> outputs;
  std::vector<std::string> names;
  BExprPtr having;  // over aggregate relation
  bool distinct = false;
  std::vector<BoundOrder> order;  // over outputs
  int64_t limit = -1, offset = 0;
  std::vector<std::shared_ptr<BoundSelect>> union_all;
  std::vector<LogicalType> OutTypes() const;
};
typedef std::shared_ptr<BoundSelect> BoundSelectPtr;

struct Catalog;

// Binds a parsed SELECT against the catalog.  `params` are the prepared
// statement bindings (1-based index -> value); missing ones raise.
BoundSelectPtr BindSelect(const Select &sel, Catalog &cat, const std::vector<Value> &params);
// BindSelect that also returns the constant node each parameter was bound into
// (node, 0-based parameter index); *patchable is true when every parameter
// lives in such a node of the plan, so a re-execution with new values of the
// same types may overwrite those nodes' values instead of binding again.
BoundSelectPtr BindSelectCapture(const Select &sel, Catalog &cat, const std::vector<Value> &params, bool *patchable,
                                 std::vector<std::pair<BExprPtr, int>> *nodes);

// Host scalar evaluation for constant folding (no column references).
Value EvalConst(const BExpr &e);
Value CastValue(const Value &v, const LogicalType &to, bool try_cast = false);
LogicalType MaxType(const LogicalType &a, const LogicalType &b);  // implicit common super type
bool IsConstTree(const BExpr &e);
std::string ExplainSelect(const BoundSelect &s, int indent = 0);
std::string ExprToString(const BExpr &e);

// Fully-constant select (source ONE_ROW, no aggregates over data and all
// union branches constant): evaluated entirely by the binder.
bool IsHostConstantSelect(const BoundSelect &s);

}  // namespace mbx
