#!/usr/bin/env python3
"""Extracts the assertions of the reference's native and arrow tests into
tests/golden/native_cases.json (data only: SQL text, the calls a test makes in
order, and the values it asserts).

Sources (read as text; nothing of the reference is executed):
  /root/reference/src/duckdb_test.mbt        native query / stream / prepared /
                                              appender / typed-result tests
  /root/reference/src/duckdb_arrow_test.mbt  arrow schema / column getter tests

Every `test "name" { ... }` block becomes one case with:
  file, line, name, kind     kind: stream | prepare | appender | arrow | query |
                             helper (pure MoonBit helpers, nothing to run) |
                             out_of_scope (LIST/STRUCT/MAP)
  sql                        the SQL string literals, in source order
  ops                        [method, [args...]] of every statement / appender
                             call (bind_*, clear_bindings, begin_row,
                             append_*, end_row, flush), in source order
  cells                      [row, col, "text" | null | {"one_of": [...]} |
                             {"contains": "..."}] from `value.cell(r, c) {
                             Some(v) => if v != "text" [&& v != "alt"]`,
                             `... if !v.contains("x")` and `None => ()`
  row_count                  from `row_count() != N`
  stream                     {"count": N, "columns": [...]} from a stream test
  arrow                      {"getter", "col", "length", "values": {i: v},
                             "ranges": {i: [lo, hi]}, "fields": N,
                             "types": {i: type_id}, "names": {i: name}}
  partial                    true when the block asserts values in a loop or
                             through code this extractor does not read (those
                             values stay restated by hand in tests/test_gpu_*.py)
Run in the development container (where /root/reference exists); the GPU box
only reads the committed JSON.
"""
import json
import os
import re
import sys

REF = "/root/reference/src"
FILES = ["duckdb_test.mbt", "duckdb_arrow_test.mbt"]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native_cases.json")

STR = r'"((?:[^"\\]|\\.)*)"'
SQL_START = re.compile(r"^\s*(SELECT|CREATE|INSERT|WITH|DROP|FROM)\b", re.I)


def unescape(s):
    # MoonBit escapes: JSON's, plus \' and string interpolation "\{expr}"
    out, i = "", 0
    simple = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'", "{": "{", "b": "\b"}
    while i < len(s):
        if s[i] == "\\" and i + 1 < len(s):
            e = s[i + 1]
            if e in simple:
                out += simple[e]
                i += 2
                continue
            if e == "u":
                out += chr(int(s[i + 2:i + 6], 16))
                i += 6
                continue
        out += s[i]
        i += 1
    return out


def blocks(text):
    """(line, name, body) of every top-level test block."""
    for m in re.finditer(r'^test "([^"]+)" \{\n', text, re.M):
        start = m.end()
        depth, i = 1, start
        while depth:
            ch = text[i]
            if ch == '"':  # skip string literals (they may hold braces)
                i += 1
                while text[i] != '"':
                    i += 2 if text[i] == "\\" else 1
            elif ch == "{":
                depth += 1
            elif ch == "}":
                depth -= 1
            i += 1
        yield text.count("\n", 0, m.start()) + 1, m.group(1), text[start:i - 1]


def literal(tok):
    tok = tok.strip()
    if tok.startswith('"'):
        return unescape(tok[1:-1])
    if tok in ("true", "false"):
        return tok == "true"
    if re.fullmatch(r"-?\d+L?", tok):
        return int(tok.rstrip("L"))
    if re.fullmatch(r"-?\d+\.\d*(e-?\d+)?", tok):
        return float(tok)
    m = re.fullmatch(r"(\w+)\((.*)\)", tok, re.S)
    if m:  # a helper call, e.g. date_from_ymd(2024, 6, 3)
        return {"call": m.group(1), "args": split_args(m.group(2))}
    return {"expr": tok}  # something the extractor does not evaluate


def split_args(s):
    out, depth, cur, q = [], 0, "", False
    for ch in s:
        if ch == '"':
            q = not q
        if not q and ch in "([":
            depth += 1
        if not q and ch in ")]":
            depth -= 1
        if not q and depth == 0 and ch == ",":
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [literal(a) for a in out]


LIT = r'"(?:[^"\\]|\\.)*"|-?\d+\.\d+|-?\d+|true|false'


def var_facts(body, var):
    """length / element / range assertions on one MoonBit array variable"""
    f = {}
    m = re.search(r"\b" + var + r"\.length\(\) != (\d+)", body)
    if m:
        f["length"] = int(m.group(1))
    vals = {}
    for i, v in re.findall(r"\b" + var + r"\[(\d+)\] != (" + LIT + r")", body):
        vals[int(i)] = literal(v)
    if vals:
        f["values"] = vals
    ranges = {}
    for m in re.finditer(r"let (\w+) = " + var + r"\[(\d+)\][^\n]*\n\s*if \1 < (-?[\d.]+) \|\| \1 > (-?[\d.]+)", body):
        ranges[int(m.group(2))] = [float(m.group(3)), float(m.group(4))]
    if ranges:
        f["ranges"] = ranges
    return f


def arrow_facts(body):
    a = {"getters": []}
    for m in re.finditer(r"let (?:\((\w+), (\w+)\)|(\w+)) = result\.get_column_(\w+)\((\d+)\)", body):
        g = {"getter": m.group(4), "col": int(m.group(5))}
        if m.group(3):
            g["values"] = var_facts(body, m.group(3))
        else:
            g["values"] = var_facts(body, m.group(1))
            g["validity"] = var_facts(body, m.group(2))
        a["getters"].append(g)
    for what, call in (("column_count", "column_count"), ("row_count", "row_count")):
        m = re.search(r"let (\w+) = result\." + call + r"\(\)", body)
        if m:
            m2 = re.search(r"\b" + m.group(1) + r" != (\d+)", body)
            if m2:
                a[what] = int(m2.group(1))
    m = re.search(r"fields\.length\(\) != (\d+)", body)
    if m:
        a["fields"] = int(m.group(1))
    alias = dict((v, int(i)) for v, i in re.findall(r"let (\w+) = fields\[(\d+)\]", body))
    types, names = {}, {}
    for f, v in re.findall(r"(fields\[\d+\]|\w+)\.type_id != " + STR, body):
        idx = int(f[7:-1]) if f.startswith("fields[") else alias.get(f)
        if idx is not None:
            types[idx] = unescape(v)
    for f, v in re.findall(r"(fields\[\d+\]|\w+)\.name != " + STR, body):
        idx = int(f[7:-1]) if f.startswith("fields[") else alias.get(f)
        if idx is not None:
            names[idx] = unescape(v)
    if types:
        a["types"] = types
    if names:
        a["names"] = names
    a["expect_error"] = bool(re.search(r"Ok\(_\)\s*=>\s*fail\(", body))
    return a


def kind_of(name, body):
    n = name.lower()
    if any(k in n for k in ("list", "struct", "map")):
        return "out_of_scope"
    if "helpers" in n or "decimal 128" in n or "decimal from" in n or "decimal to" in n or "decimal negative" in n:
        return "helper"
    if "arrow" in n:
        return "arrow"
    if "stream" in n:
        return "stream"
    if "appender" in n:
        return "appender"
    if "prepare" in n:
        return "prepare"
    return "query"


def extract(fname, line, name, body):
    c = {"file": f"src/{fname}", "line": line, "name": name, "kind": kind_of(name, body)}
    c["sql"] = [unescape(s) for s in re.findall(STR, body) if SQL_START.match(unescape(s))]
    lets = dict(re.findall(r"let (\w+) = ([^\n]+?)\s*\n", body))
    ops = []
    for m in re.finditer(r"\b(?:stmt|app|appender|s|a)\.(bind_\w+|clear_bindings|begin_row|end_row|append_\w+|flush)"
                         r"\(((?:[^()]|\([^()]*\))*)\)", body):
        args = split_args(m.group(2))
        # a variable bound by `let x = helper(...)` in the same test
        args = [literal(lets[a["expr"]]) if isinstance(a, dict) and a.get("expr") in lets else a for a in args]
        ops.append([m.group(1), args])
    c["ops"] = ops
    cells = []
    for m in re.finditer(r"\.cell\((\d+),\s*(\d+)\)\s*\{\s*(Some\(v\)\s*=>\s*if (v != " + STR + r"(?:\s*&&\s*v != " + STR +
                         r")*)|None\s*=>\s*\(\))", body):
        if m.group(4) is None:
            want = None
        else:
            alts = [unescape(x) for x in re.findall(STR, m.group(4))]
            want = alts[0] if len(alts) == 1 else {"one_of": alts}  # `v != "5" && v != "5.0"`
        cells.append([int(m.group(1)), int(m.group(2)), want])
    for m in re.finditer(r"\.cell\((\d+),\s*(\d+)\)\s*\{\s*Some\(v\)\s*=>(?:(?!\.cell\().)*?if !v\.contains\(" + STR + r"\)",
                         body, re.S):
        cells.append([int(m.group(1)), int(m.group(2)), {"contains": unescape(m.group(3))}])
    c["cells"] = cells
    rc = re.findall(r"row_count\(\) != (\d+)", body)
    if rc:
        c["row_count"] = int(rc[0])
    if c["kind"] == "stream":
        st = {}
        m = re.search(r"\bcount != (\d+)", body)
        if m:
            st["count"] = int(m.group(1))
        cols = re.findall(r"columns\[(\d+)\] != " + STR, body)
        if cols:
            st["columns"] = [unescape(v) for _, v in sorted(cols)]
        m = re.search(r"columns\.length\(\) != (\d+)", body)
        if m:
            st["ncols"] = int(m.group(1))
        c["stream"] = st
    if c["kind"] == "arrow":
        c["arrow"] = arrow_facts(body)
    loops = bool(re.search(r"\bfor \w+ = ", body))
    reads_other = bool(re.search(r"\.(get_\w+|to_typed|get_value)\(", body)) and c["kind"] in ("query", "appender",
                                                                                             "prepare")
    c["partial"] = loops or reads_other
    return c


def main():
    cases = []
    for f in FILES:
        text = open(os.path.join(REF, f)).read()
        for line, name, body in blocks(text):
            cases.append(extract(f, line, name, body))
    json.dump({"source": FILES, "generator": "tests/golden/make_native_cases.py", "cases": cases},
              open(OUT, "w"), indent=1, sort_keys=True)
    kinds = {}
    for c in cases:
        kinds[c["kind"]] = kinds.get(c["kind"], 0) + 1
    print(f"wrote {len(cases)} cases to {OUT}: {kinds}")


if __name__ == "__main__":
    sys.exit(main())
