// sql.h — the SQL subset accepted by the MI355X backend (parse tree).
//
// The reference passes SQL text straight to libduckdb
// (/root/reference/src/duckdb_native.c:142-172 duckdb_mb_query -> duckdb_query).
// This parser covers the statements the reference's tests and the benchmark
// configurations issue: SELECT [DISTINCT] ... FROM {table | range(..) [tbl(col)]
// | (VALUES ..) t(cols) | (subquery)} [WHERE] [GROUP BY] [HAVING] [ORDER BY]
// [LIMIT/OFFSET] [UNION ALL ...], CREATE TABLE [AS SELECT], INSERT INTO ...
// VALUES/SELECT, DROP TABLE.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "types.h"

namespace mbx {

struct Select;
typedef std::shared_ptr<Select> SelectPtr;

struct TypeSpec {
  LogicalType type;
  bool set = false;
};

struct Expr;
typedef std::shared_ptr<Expr> ExprPtr;

struct Expr {
  enum Kind {
    CONST,     // val
    COLREF,    // name (optionally qualifier)
    STAR,      // * (select list or COUNT(*))
    UNARY,     // op in {"-", "+", "NOT"}, args[0]
    BINARY,    // op, args[0], args[1]
    FUNC,      // name(args)
    CAST,      // args[0]::cast
    CASE,      // args = [operand?] (when, then)* [else]; case_operand/has_else flags
    PARAM,     // ? / $n
    ISNULL,    // args[0] IS [NOT] NULL  (negated)
    BETWEEN,   // args[0] [NOT] BETWEEN args[1] AND args[2]
    INLIST,    // args[0] [NOT] IN (args[1..])
  };
  Kind kind = CONST;
  Value val;
  std::string name, qualifier, op;
  std::vector<ExprPtr> args;
  TypeSpec cast;
  bool negated = false;
  bool distinct = false;
  bool star = false;         // COUNT(*)
  bool case_operand = false; // CASE x WHEN ...
  bool has_else = false;
  int param_index = 0;       // 1-based
  std::string alias;
  std::string text;          // original text for column naming
};

struct TableRef {
  enum Kind { NONE, TABLE, RANGE, VALUES, SUBQUERY } kind = NONE;
  std::string name;  // table name or function name (range / generate_series)
  std::vector<ExprPtr> args;
  std::vector<std::vector<ExprPtr>> rows;
  SelectPtr sub;
  std::string alias;
  std::vector<std::string> col_aliases;
};

struct OrderItem {
  ExprPtr expr;
  bool desc = false;
  int nulls_first = -1;  // -1 default
};

struct Select {
  bool distinct = false;
  std::vector<ExprPtr> list;
  TableRef from;
  ExprPtr where;
  std::vector<ExprPtr> group_by;
  ExprPtr having;
  std::vector<OrderItem> order_by;
  ExprPtr limit, offset;
  std::vector<SelectPtr> union_all;  // further branches (UNION ALL)
};

struct ColumnDef {
  std::string name;
  LogicalType type;
  bool not_null = false;
};

struct Statement {
  enum Kind { SELECT, CREATE_TABLE, CREATE_TABLE_AS, INSERT, DROP_TABLE, NOP } kind = SELECT;
  SelectPtr select;
  std::string table;
  std::string schema;
  std::vector<ColumnDef> columns;
  std::vector<std::string> insert_columns;
  bool if_not_exists = false, if_exists = false, or_replace = false;
  int n_params = 0;
};

// Parses exactly one statement (a trailing ';' is allowed).  Throws
// EngineError("Parser Error: ...") on malformed input.
Statement ParseSQL(const std::string &sql);
LogicalType ParseTypeName(const std::string &name, int p1, int p2, bool has_p1, bool has_p2);

}  // namespace mbx
