// sql.cpp — lexer and recursive-descent parser for the accepted SQL subset.
#include "sql.h"

#include <cctype>
#include <cstdlib>

namespace mbx {

namespace {

struct Tok {
  enum K { END, IDENT, QIDENT, NUM, STR, OP, PARAM } k = END;
  std::string s;  // identifier (lower-cased for IDENT), number text, string value, operator
  std::string raw;
  size_t pos = 0;
};

std::string Lower(std::string s) {
  for (auto &c : s) c = (char)tolower((unsigned char)c);
  return s;
}

std::vector<Tok> Lex(const std::string &q) {
  std::vector<Tok> out;
  size_t i = 0, n = q.size();
  while (i < n) {
    char c = q[i];
    if (isspace((unsigned char)c)) {
      i++;
      continue;
    }
    if (c == '-' && i + 1 < n && q[i + 1] == '-') {
      while (i < n && q[i] != '\n') i++;
      continue;
    }
    if (c == '/' && i + 1 < n && q[i + 1] == '*') {
      size_t e = q.find("*/", i + 2);
      i = e == std::string::npos ? n : e + 2;
      continue;
    }
    Tok t;
    t.pos = i;
    if (isalpha((unsigned char)c) || c == '_') {
      size_t st = i;
      while (i < n && (isalnum((unsigned char)q[i]) || q[i] == '_' || q[i] == '$')) i++;
      t.k = Tok::IDENT;
      t.raw = q.substr(st, i - st);
      t.s = Lower(t.raw);
    } else if (c == '"') {
      size_t st = ++i;
      std::string v;
      while (i < n) {
        if (q[i] == '"') {
          if (i + 1 < n && q[i + 1] == '"') {
            v.push_back('"');
            i += 2;
            continue;
          }
          break;
        }
        v.push_back(q[i++]);
      }
      if (i >= n) ThrowError("Parser", "unterminated quoted identifier at or near \"" + q.substr(st - 1) + "\"");
      i++;
      t.k = Tok::QIDENT;
      t.s = t.raw = v;
    } else if (isdigit((unsigned char)c) || (c == '.' && i + 1 < n && isdigit((unsigned char)q[i + 1]))) {
      size_t st = i;
      while (i < n && (isdigit((unsigned char)q[i]) || q[i] == '_')) i++;
      if (i < n && q[i] == '.') {
        i++;
        while (i < n && isdigit((unsigned char)q[i])) i++;
      }
      if (i < n && (q[i] == 'e' || q[i] == 'E')) {
        size_t save = i;
        i++;
        if (i < n && (q[i] == '+' || q[i] == '-')) i++;
        if (i < n && isdigit((unsigned char)q[i])) {
          while (i < n && isdigit((unsigned char)q[i])) i++;
        } else {
          i = save;
        }
      }
      t.k = Tok::NUM;
      t.s = t.raw = q.substr(st, i - st);
    } else if (c == '\'' || ((c == 'e' || c == 'E') && i + 1 < n && q[i + 1] == '\'')) {
      bool esc = c != '\'';
      if (esc) i++;
      i++;
      std::string v;
      while (true) {
        if (i >= n) ThrowError("Parser", "unterminated quoted string at or near \"" + q.substr(t.pos) + "\"");
        if (q[i] == '\'') {
          if (i + 1 < n && q[i + 1] == '\'') {
            v.push_back('\'');
            i += 2;
            continue;
          }
          i++;
          // adjacent string literals separated by whitespace+newline concatenate
          break;
        }
        if (esc && q[i] == '\\' && i + 1 < n) {
          char e = q[i + 1];
          v.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e);
          i += 2;
          continue;
        }
        v.push_back(q[i++]);
      }
      t.k = Tok::STR;
      t.s = v;
    } else if (c == '?') {
      i++;
      t.k = Tok::PARAM;
      t.s = "";
    } else if (c == '$' && i + 1 < n && isdigit((unsigned char)q[i + 1])) {
      size_t st = ++i;
      while (i < n && isdigit((unsigned char)q[i])) i++;
      t.k = Tok::PARAM;
      t.s = q.substr(st, i - st);
    } else {
      static const char *ops[] = {"::", "<=", ">=", "<>", "!=", "==", "||", "//", "**", "(", ")", ",", ";", "*", "+",
                                  "-",  "/",  "%",  "<",  ">",  "=",  ".",  "[",  "]",  ":"};
      bool found = false;
      for (const char *o : ops) {
        size_t L = strlen(o);
        if (q.compare(i, L, o) == 0) {
          t.k = Tok::OP;
          t.s = o;
          i += L;
          found = true;
          break;
        }
      }
      if (!found) ThrowError("Parser", std::string("syntax error at or near \"") + c + "\"");
    }
    if (t.raw.empty()) t.raw = t.s;
    out.push_back(t);
  }
  Tok e;
  e.k = Tok::END;
  e.pos = n;
  out.push_back(e);
  return out;
}

bool IsReserved(const std::string &s) {
  static const char *kw[] = {"select", "from",  "where", "group", "by",     "having", "order", "limit", "offset",
                             "union",  "all",   "as",    "on",    "and",    "or",     "not",   "is",    "null",
                             "in",     "between", "case", "when", "then",   "else",   "end",   "asc",   "desc",
                             "nulls",  "values", "distinct", "cast", "create", "table", "insert", "into", "drop",
                             "join",   "inner", "left", "right", "cross", "using", "like", "except", "intersect",
                             "window", "qualify", "filter", "over", "true", "false", "with", nullptr};
  for (int i = 0; kw[i]; i++)
    if (s == kw[i]) return true;
  return false;
}

class Parser {
 public:
  Parser(const std::string &q) : q_(q), t_(Lex(q)) {}

  Statement ParseStatement() {
    Statement st;
    if (IsKw("select") || IsOp("(") || IsKw("values") || IsKw("from")) {
      st.kind = Statement::SELECT;
      st.select = ParseSelectUnion();
    } else if (AcceptKw("create")) {
      if (AcceptKw("or")) {
        ExpectKw("replace");
        st.or_replace = true;
      }
      AcceptKw("temp") || AcceptKw("temporary");
      ExpectKw("table");
      if (AcceptKw("if")) {
        ExpectKw("not");
        ExpectKw("exists");
        st.if_not_exists = true;
      }
      ParseQualifiedName(&st.schema, &st.table);
      if (AcceptKw("as")) {
        st.kind = Statement::CREATE_TABLE_AS;
        st.select = ParseSelectUnion();
      } else {
        st.kind = Statement::CREATE_TABLE;
        ExpectOp("(");
        do {
          if (IsKw("primary") || IsKw("unique") || IsKw("check") || IsKw("foreign") || IsKw("constraint")) {
            SkipParens();
            continue;
          }
          ColumnDef cd;
          cd.name = Ident();
          cd.type = ParseType();
          while (!IsOp(",") && !IsOp(")")) {
            if (AcceptKw("not")) {
              ExpectKw("null");
              cd.not_null = true;
            } else if (AcceptKw("null") || AcceptKw("unique")) {
            } else if (AcceptKw("primary")) {
              ExpectKw("key");
              cd.not_null = true;
            } else if (AcceptKw("default")) {
              ThrowError("Not implemented", "DEFAULT values are not supported by the MI355X backend");
            } else {
              ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\"");
            }
          }
          st.columns.push_back(cd);
        } while (AcceptOp(","));
        ExpectOp(")");
      }
    } else if (AcceptKw("insert")) {
      st.kind = Statement::INSERT;
      ExpectKw("into");
      ParseQualifiedName(&st.schema, &st.table);
      if (IsOp("(") && !PeekKwAfterParen("select")) {
        ExpectOp("(");
        do st.insert_columns.push_back(Ident());
        while (AcceptOp(","));
        ExpectOp(")");
      }
      st.select = ParseSelectUnion();
    } else if (AcceptKw("drop")) {
      st.kind = Statement::DROP_TABLE;
      ExpectKw("table");
      if (AcceptKw("if")) {
        ExpectKw("exists");
        st.if_exists = true;
      }
      ParseQualifiedName(&st.schema, &st.table);
    } else if (AcceptKw("begin") || AcceptKw("commit") || AcceptKw("rollback") || AcceptKw("checkpoint")) {
      AcceptKw("transaction");
      st.kind = Statement::NOP;
    } else {
      ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\"");
    }
    AcceptOp(";");
    if (Cur().k != Tok::END) ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\"");
    st.n_params = n_params_;
    return st;
  }

 private:
  const std::string &q_;
  std::vector<Tok> t_;
  size_t p_ = 0;
  int n_params_ = 0;

  const Tok &Cur() const { return t_[p_]; }
  const Tok &Peek(int k = 1) const { return t_[std::min(p_ + k, t_.size() - 1)]; }
  bool IsKw(const char *k) const { return Cur().k == Tok::IDENT && Cur().s == k; }
  bool IsOp(const char *o) const { return Cur().k == Tok::OP && Cur().s == o; }
  bool AcceptKw(const char *k) {
    if (IsKw(k)) {
      p_++;
      return true;
    }
    return false;
  }
  bool AcceptOp(const char *o) {
    if (IsOp(o)) {
      p_++;
      return true;
    }
    return false;
  }
  void ExpectKw(const char *k) {
    if (!AcceptKw(k)) ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\" (expected " + k + ")");
  }
  void ExpectOp(const char *o) {
    if (!AcceptOp(o)) ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\" (expected " + o + ")");
  }
  bool PeekKwAfterParen(const char *k) const {
    return Cur().k == Tok::OP && Cur().s == "(" && Peek().k == Tok::IDENT && Peek().s == k;
  }
  void SkipParens() {
    int depth = 0;
    while (Cur().k != Tok::END) {
      if (IsOp("(")) depth++;
      if (IsOp(")")) {
        if (depth == 0) return;
        depth--;
      }
      if (IsOp(",") && depth == 0) return;
      p_++;
    }
  }
  std::string Ident() {
    if (Cur().k == Tok::QIDENT) return t_[p_++].s;
    if (Cur().k == Tok::IDENT) return t_[p_++].s;
    ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\" (expected identifier)");
  }
  void ParseQualifiedName(std::string *schema, std::string *name) {
    std::string a = Ident();
    if (AcceptOp(".")) {
      *schema = a;
      *name = Ident();
    } else {
      *name = a;
    }
  }

  int64_t IntArg() {
    bool neg = AcceptOp("-");
    if (Cur().k != Tok::NUM) ThrowError("Parser", "expected integer near \"" + Cur().raw + "\"");
    int64_t v = std::stoll(t_[p_++].s);
    return neg ? -v : v;
  }

  LogicalType ParseType() {
    std::string nm = Ident();
    if (nm == "double" && AcceptKw("precision")) {
    }
    if ((nm == "character" || nm == "char") && AcceptKw("varying")) nm = "varchar";
    int p1 = 0, p2 = 0;
    bool h1 = false, h2 = false;
    if (AcceptOp("(")) {
      p1 = (int)IntArg();
      h1 = true;
      if (AcceptOp(",")) {
        p2 = (int)IntArg();
        h2 = true;
      }
      ExpectOp(")");
    }
    if (AcceptOp("[")) ThrowError("Not implemented", "LIST types are not supported by the MI355X backend");
    return ParseTypeName(nm, p1, p2, h1, h2);
  }

  // ---- SELECT -------------------------------------------------------------
  SelectPtr ParseSelectUnion() {
    SelectPtr first = ParseSelectCore();
    while (IsKw("union")) {
      p_++;
      if (!AcceptKw("all")) ThrowError("Not implemented", "UNION (distinct) is not supported; use UNION ALL");
      SelectPtr nxt = ParseSelectCore();
      first->union_all.push_back(nxt);
    }
    // ORDER BY / LIMIT after a union apply to the whole union: attach to first
    ParseOrderLimit(first.get());
    return first;
  }

  SelectPtr ParseSelectCore() {
    if (IsOp("(") && (Peek().k == Tok::IDENT && (Peek().s == "select" || Peek().s == "values"))) {
      ExpectOp("(");
      SelectPtr s = ParseSelectUnion();
      ExpectOp(")");
      return s;
    }
    auto s = std::make_shared<Select>();
    if (AcceptKw("values")) {
      // bare VALUES list as a query
      s->from.kind = TableRef::VALUES;
      ParseValuesRows(&s->from);
      auto star = std::make_shared<Expr>();
      star->kind = Expr::STAR;
      s->list.push_back(star);
      return s;
    }
    ExpectKw("select");
    if (AcceptKw("distinct")) s->distinct = true;
    AcceptKw("all");
    do {
      ExprPtr e = ParseExpr();
      if (AcceptKw("as")) {
        e->alias = Ident();
      } else if (Cur().k == Tok::QIDENT || (Cur().k == Tok::IDENT && !IsReserved(Cur().s))) {
        e->alias = Ident();
      }
      s->list.push_back(e);
    } while (AcceptOp(","));
    if (AcceptKw("from")) ParseFrom(&s->from);
    if (AcceptKw("where")) s->where = ParseExpr();
    if (AcceptKw("group")) {
      ExpectKw("by");
      if (AcceptKw("all")) {
        auto all = std::make_shared<Expr>();
        all->kind = Expr::STAR;
        s->group_by.push_back(all);
      } else {
        do s->group_by.push_back(ParseExpr());
        while (AcceptOp(","));
      }
    }
    if (AcceptKw("having")) s->having = ParseExpr();
    return s;
  }

  void ParseOrderLimit(Select *s) {
    if (AcceptKw("order")) {
      ExpectKw("by");
      do {
        OrderItem it;
        it.expr = ParseExpr();
        if (AcceptKw("desc")) it.desc = true;
        else AcceptKw("asc");
        if (AcceptKw("nulls")) {
          if (AcceptKw("first")) it.nulls_first = 1;
          else {
            ExpectKw("last");
            it.nulls_first = 0;
          }
        }
        s->order_by.push_back(it);
      } while (AcceptOp(","));
    }
    for (int k = 0; k < 2; k++) {
      if (AcceptKw("limit")) s->limit = ParseExpr();
      if (AcceptKw("offset")) s->offset = ParseExpr();
    }
  }

  void ParseValuesRows(TableRef *tr) {
    do {
      ExpectOp("(");
      std::vector<ExprPtr> row;
      do row.push_back(ParseExpr());
      while (AcceptOp(","));
      ExpectOp(")");
      tr->rows.push_back(row);
    } while (AcceptOp(","));
  }

  void ParseAlias(TableRef *tr) {
    if (AcceptKw("as") || Cur().k == Tok::QIDENT || (Cur().k == Tok::IDENT && !IsReserved(Cur().s))) {
      tr->alias = Ident();
      if (AcceptOp("(")) {
        do tr->col_aliases.push_back(Ident());
        while (AcceptOp(","));
        ExpectOp(")");
      }
    }
  }

  void ParseFrom(TableRef *tr) {
    if (AcceptOp("(")) {
      if (AcceptKw("values")) {
        tr->kind = TableRef::VALUES;
        ParseValuesRows(tr);
      } else {
        tr->kind = TableRef::SUBQUERY;
        tr->sub = ParseSelectUnion();
      }
      ExpectOp(")");
      ParseAlias(tr);
    } else {
      std::string schema, name;
      ParseQualifiedName(&schema, &name);
      if (IsOp("(")) {
        ExpectOp("(");
        tr->kind = TableRef::RANGE;
        tr->name = name;
        if (!IsOp(")")) {
          do tr->args.push_back(ParseExpr());
          while (AcceptOp(","));
        }
        ExpectOp(")");
        if (name != "range" && name != "generate_series")
          ThrowError("Catalog", "Table Function with name " + name + " does not exist!");
      } else {
        tr->kind = TableRef::TABLE;
        tr->name = name;
      }
      ParseAlias(tr);
    }
    if (IsOp(",") || IsKw("join") || IsKw("inner") || IsKw("left") || IsKw("cross"))
      ThrowError("Not implemented", "joins are not supported by the MI355X backend");
  }

  // ---- expressions ---------------------------------------------------------
  ExprPtr Mk(Expr::Kind k) {
    auto e = std::make_shared<Expr>();
    e->kind = k;
    return e;
  }
  ExprPtr Bin(const std::string &op, ExprPtr a, ExprPtr b) {
    auto e = Mk(Expr::BINARY);
    e->op = op;
    e->args = {a, b};
    return e;
  }

  // recursion guard (nested parentheses, NOT NOT ..., - - ...): DuckDB's
  // max_expression_depth default
  static constexpr int kMaxDepth = 1000;
  int depth_ = 0;
  struct DepthGuard {
    int &d;
    explicit DepthGuard(int &x) : d(x) {
      if (++d > kMaxDepth)
        ThrowError("Parser", "Max expression depth limit of " + std::to_string(kMaxDepth) + " exceeded");
    }
    ~DepthGuard() { d--; }
  };

  ExprPtr ParseExpr() {
    DepthGuard g(depth_);
    size_t st = Cur().pos;
    ExprPtr e = ParseOr();
    size_t en = Cur().pos;
    if (e->text.empty()) {
      std::string tx = q_.substr(st, en - st);
      while (!tx.empty() && isspace((unsigned char)tx.back())) tx.pop_back();
      e->text = tx;
    }
    return e;
  }
  ExprPtr ParseOr() {
    ExprPtr l = ParseAnd();
    while (AcceptKw("or")) l = Bin("OR", l, ParseAnd());
    return l;
  }
  ExprPtr ParseAnd() {
    ExprPtr l = ParseNot();
    while (AcceptKw("and")) l = Bin("AND", l, ParseNot());
    return l;
  }
  ExprPtr ParseNot() {
    DepthGuard g(depth_);
    if (AcceptKw("not")) {
      auto e = Mk(Expr::UNARY);
      e->op = "NOT";
      e->args = {ParseNot()};
      return e;
    }
    return ParseCmp();
  }
  ExprPtr ParseCmp() {
    ExprPtr l = ParseConcat();
    while (true) {
      if (Cur().k == Tok::OP &&
          (Cur().s == "=" || Cur().s == "==" || Cur().s == "<>" || Cur().s == "!=" || Cur().s == "<" ||
           Cur().s == "<=" || Cur().s == ">" || Cur().s == ">=")) {
        std::string op = t_[p_++].s;
        if (op == "==") op = "=";
        if (op == "!=") op = "<>";
        l = Bin(op, l, ParseConcat());
        continue;
      }
      if (IsKw("is")) {
        p_++;
        bool neg = AcceptKw("not");
        if (AcceptKw("null")) {
          auto e = Mk(Expr::ISNULL);
          e->negated = neg;
          e->args = {l};
          l = e;
          continue;
        }
        if (AcceptKw("distinct")) {
          ExpectKw("from");
          auto e = Bin(neg ? "IS NOT DISTINCT FROM" : "IS DISTINCT FROM", l, ParseConcat());
          l = e;
          continue;
        }
        ThrowError("Parser", "syntax error at or near \"" + Cur().raw + "\"");
      }
      bool neg = false;
      size_t save = p_;
      if (IsKw("not") && (Peek().s == "between" || Peek().s == "in" || Peek().s == "like")) {
        p_++;
        neg = true;
      }
      if (AcceptKw("between")) {
        auto e = Mk(Expr::BETWEEN);
        e->negated = neg;
        ExprPtr lo = ParseConcat();
        ExpectKw("and");
        ExprPtr hi = ParseConcat();
        e->args = {l, lo, hi};
        l = e;
        continue;
      }
      if (AcceptKw("in")) {
        auto e = Mk(Expr::INLIST);
        e->negated = neg;
        ExpectOp("(");
        e->args.push_back(l);
        do e->args.push_back(ParseExpr());
        while (AcceptOp(","));
        ExpectOp(")");
        l = e;
        continue;
      }
      if (AcceptKw("like")) ThrowError("Not implemented", "LIKE is not supported by the MI355X backend");
      p_ = save;
      break;
    }
    return l;
  }
  ExprPtr ParseConcat() {
    ExprPtr l = ParseAdd();
    while (AcceptOp("||")) l = Bin("||", l, ParseAdd());
    return l;
  }
  ExprPtr ParseAdd() {
    ExprPtr l = ParseMul();
    while (IsOp("+") || IsOp("-")) {
      std::string op = t_[p_++].s;
      l = Bin(op, l, ParseMul());
    }
    return l;
  }
  ExprPtr ParseMul() {
    ExprPtr l = ParseUnary();
    while (IsOp("*") || IsOp("/") || IsOp("%") || IsOp("//")) {
      std::string op = t_[p_++].s;
      l = Bin(op, l, ParseUnary());
    }
    return l;
  }
  ExprPtr ParseUnary() {
    DepthGuard g(depth_);
    if (IsOp("-") || IsOp("+")) {
      std::string op = t_[p_++].s;
      ExprPtr a = ParseUnary();
      if (op == "+") return a;
      // fold "-<numeric literal>" into the literal (keeps BIGINT minimum a BIGINT)
      if (a->kind == Expr::CONST && !a->val.is_null && a->cast.set == false &&
          (a->val.type.id == T_INTEGER || a->val.type.id == T_BIGINT || a->val.type.id == T_HUGEINT ||
           a->val.type.id == T_DECIMAL || a->val.type.id == T_DOUBLE) &&
          a->op == "literal") {
        Value v = a->val;
        if (v.type.id == T_DOUBLE) {
          v.d = -v.d;
        } else {
          v.i = -v.i;
          if (v.type.id != T_DECIMAL) v.type = LogicalType(IntLiteralType(v.i));
        }
        auto c = Mk(Expr::CONST);
        c->val = v;
        c->op = "literal";
        return c;
      }
      auto e = Mk(Expr::UNARY);
      e->op = "-";
      e->args = {a};
      return e;
    }
    return ParsePostfix();
  }
  static TypeId IntLiteralType(i128 v) {
    if (v >= INT32_MIN && v <= INT32_MAX) return T_INTEGER;
    if (v >= INT64_MIN && v <= INT64_MAX) return T_BIGINT;
    return T_HUGEINT;
  }
  ExprPtr ParsePostfix() {
    ExprPtr e = ParsePrimary();
    while (AcceptOp("::")) {
      auto c = Mk(Expr::CAST);
      c->cast.type = ParseType();
      c->cast.set = true;
      c->args = {e};
      e = c;
    }
    return e;
  }

  ExprPtr NumLiteral(const std::string &txt) {
    auto c = Mk(Expr::CONST);
    c->op = "literal";
    std::string s;
    for (char ch : txt)
      if (ch != '_') s.push_back(ch);
    bool has_dot = s.find('.') != std::string::npos;
    bool has_e = s.find_first_of("eE") != std::string::npos;
    if (has_e) {
      c->val = Value::Double(strtod(s.c_str(), nullptr));
      return c;
    }
    if (!has_dot) {
      i128 v;
      if (ParseI128(s, &v)) {
        c->val = Value::Int(IntLiteralType(v), v);
      } else {
        c->val = Value::Double(strtod(s.c_str(), nullptr));
      }
      return c;
    }
    // decimal literal: DECIMAL(width, scale) where width counts all digits
    size_t dot = s.find('.');
    std::string ip = s.substr(0, dot), fp = s.substr(dot + 1);
    size_t nz = 0;
    while (nz < ip.size() && ip[nz] == '0') nz++;
    ip = ip.substr(nz);
    int scale = (int)fp.size();
    int width = (int)(ip.size() + fp.size());
    if (width < scale) width = scale;
    if (width == 0) width = 1;
    if (width > 38) {
      c->val = Value::Double(strtod(s.c_str(), nullptr));
      return c;
    }
    i128 v = 0;
    ParseI128((ip.empty() ? std::string("0") : ip) + fp, &v);
    c->val = Value::Decimal(width, scale, v);
    return c;
  }

  ExprPtr ParsePrimary() {
    const Tok &t = Cur();
    size_t st = t.pos;
    if (t.k == Tok::NUM) {
      p_++;
      return NumLiteral(t.s);
    }
    if (t.k == Tok::STR) {
      p_++;
      auto c = Mk(Expr::CONST);
      c->op = "literal";
      c->val = Value::Varchar(t.s);
      // string literals carry STRING_LITERAL semantics: implicitly castable
      c->name = "string_literal";
      return c;
    }
    if (t.k == Tok::PARAM) {
      p_++;
      auto e = Mk(Expr::PARAM);
      if (t.s.empty()) {
        e->param_index = ++n_params_;
      } else {
        e->param_index = atoi(t.s.c_str());
        if (e->param_index > n_params_) n_params_ = e->param_index;
      }
      return e;
    }
    if (AcceptOp("(")) {
      if (IsKw("select")) ThrowError("Not implemented", "scalar subqueries are not supported by the MI355X backend");
      ExprPtr e = ParseExpr();
      ExpectOp(")");
      return e;
    }
    if (AcceptOp("*")) return Mk(Expr::STAR);
    if (t.k == Tok::IDENT || t.k == Tok::QIDENT) {
      if (t.k == Tok::IDENT) {
        if (t.s == "null") {
          p_++;
          auto c = Mk(Expr::CONST);
          c->val = Value::Null();
          return c;
        }
        if (t.s == "true" || t.s == "false") {
          p_++;
          auto c = Mk(Expr::CONST);
          c->val = Value::Bool(t.s == "true");
          return c;
        }
        if (t.s == "case") return ParseCase();
        if (t.s == "cast" || t.s == "try_cast") {
          p_++;
          ExpectOp("(");
          auto c = Mk(Expr::CAST);
          c->args = {ParseExpr()};
          ExpectKw("as");
          c->cast.type = ParseType();
          c->cast.set = true;
          ExpectOp(")");
          return c;
        }
        if ((t.s == "date" || t.s == "time" || t.s == "timestamp" || t.s == "interval") && Peek().k == Tok::STR) {
          p_++;
          std::string sv = t_[p_++].s;
          auto c = Mk(Expr::CAST);
          auto lit = Mk(Expr::CONST);
          lit->val = Value::Varchar(sv);
          lit->name = "string_literal";
          c->args = {lit};
          c->cast.set = true;
          c->cast.type = ParseTypeName(t.s, 0, 0, false, false);
          return c;
        }
        if (t.s == "interval" && Peek().k == Tok::NUM) {
          p_++;
          std::string num = t_[p_++].s;
          std::string unit = Ident();
          auto c = Mk(Expr::CAST);
          auto lit = Mk(Expr::CONST);
          lit->val = Value::Varchar(num + " " + unit);
          lit->name = "string_literal";
          c->args = {lit};
          c->cast.set = true;
          c->cast.type = LogicalType(T_INTERVAL);
          return c;
        }
      }
      std::string a = Ident();
      if (IsOp("(")) {
        p_++;
        auto f = Mk(Expr::FUNC);
        f->name = a;
        if (AcceptOp("*")) {
          f->star = true;
        } else if (!IsOp(")")) {
          if (AcceptKw("distinct")) f->distinct = true;
          do f->args.push_back(ParseExpr());
          while (AcceptOp(","));
        }
        ExpectOp(")");
        if (IsKw("over") || IsKw("filter"))
          ThrowError("Not implemented", "window functions / FILTER are not supported by the MI355X backend");
        return f;
      }
      auto c = Mk(Expr::COLREF);
      if (AcceptOp(".")) {
        if (AcceptOp("*")) {
          auto s = Mk(Expr::STAR);
          s->qualifier = a;
          return s;
        }
        c->qualifier = a;
        c->name = Ident();
      } else {
        c->name = a;
      }
      (void)st;
      return c;
    }
    ThrowError("Parser", "syntax error at or near \"" + (t.k == Tok::END ? std::string("end of input") : t.raw) + "\"");
  }

  ExprPtr ParseCase() {
    ExpectKw("case");
    auto e = Mk(Expr::CASE);
    if (!IsKw("when")) {
      e->case_operand = true;
      e->args.push_back(ParseExpr());
    }
    while (AcceptKw("when")) {
      e->args.push_back(ParseExpr());
      ExpectKw("then");
      e->args.push_back(ParseExpr());
    }
    if (AcceptKw("else")) {
      e->has_else = true;
      e->args.push_back(ParseExpr());
    }
    ExpectKw("end");
    return e;
  }
};

}  // namespace

LogicalType ParseTypeName(const std::string &nm, int p1, int p2, bool h1, bool h2) {
  if (nm == "boolean" || nm == "bool" || nm == "logical") return LogicalType(T_BOOLEAN);
  if (nm == "tinyint" || nm == "int1") return LogicalType(T_TINYINT);
  if (nm == "smallint" || nm == "int2" || nm == "short") return LogicalType(T_SMALLINT);
  if (nm == "integer" || nm == "int" || nm == "int4" || nm == "signed") return LogicalType(T_INTEGER);
  if (nm == "bigint" || nm == "int8" || nm == "long") return LogicalType(T_BIGINT);
  if (nm == "hugeint" || nm == "int128") return LogicalType(T_HUGEINT);
  if (nm == "utinyint") return LogicalType(T_UTINYINT);
  if (nm == "usmallint") return LogicalType(T_USMALLINT);
  if (nm == "uinteger") return LogicalType(T_UINTEGER);
  if (nm == "ubigint") return LogicalType(T_UBIGINT);
  if (nm == "float" || nm == "real" || nm == "float4") return LogicalType(T_FLOAT);
  if (nm == "double" || nm == "float8") return LogicalType(T_DOUBLE);
  if (nm == "decimal" || nm == "numeric" || nm == "dec") {
    int w = h1 ? p1 : 18, s = h2 ? p2 : (h1 ? 0 : 3);
    if (w < 1 || w > 38) ThrowError("Parser", "Width must be between 1 and 38!");
    if (s < 0 || s > w) ThrowError("Parser", "Scale must be between 0 and the width!");
    return LogicalType::Decimal(w, s);
  }
  if (nm == "varchar" || nm == "text" || nm == "string" || nm == "char" || nm == "bpchar" || nm == "nvarchar")
    return LogicalType(T_VARCHAR);
  if (nm == "blob" || nm == "bytea" || nm == "binary" || nm == "varbinary") return LogicalType(T_BLOB);
  if (nm == "date") return LogicalType(T_DATE);
  if (nm == "time") return LogicalType(T_TIME);
  if (nm == "timestamp" || nm == "datetime") return LogicalType(T_TIMESTAMP);
  if (nm == "interval") return LogicalType(T_INTERVAL);
  ThrowError("Catalog", "Type with name " + nm + " does not exist!");
}

Statement ParseSQL(const std::string &sql) {
  Parser p(sql);
  return p.ParseStatement();
}

}  // namespace mbx
