#!/usr/bin/env python3
"""Where the C4 Arrow read-back time goes: per 1e6-row slice, the query
(parse + LIMIT/OFFSET + D2H into the result), the int64 wire-buffer getter,
and the Python-side copy of the returned Bytes.  GPU only."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
c = m.connect().value
n = 20_000_000
c.query(f"CREATE TABLE c4 AS SELECT i * 2654435761 AS v FROM range({n}) tbl(i)")
lib = m.lib
t = {"query": 0.0, "getter": 0.0, "py_copy": 0.0, "free": 0.0}
for rep in range(2):
    for k in range(0, n, 1_000_000):
        sql = f"SELECT v FROM c4 LIMIT 1000000 OFFSET {k}"
        a = m._Arg(sql)
        t0 = time.perf_counter()
        h = lib.duckdb_mb_query_arrow(c._h, a.p)
        t1 = time.perf_counter()
        p = lib.duckdb_mb_arrow_get_column_int64(h, 0)
        t2 = time.perf_counter()
        ln = lib.duckdb_mbx_bytes_len(p)
        b = ctypes.string_at(p, ln)
        t3 = time.perf_counter()
        lib.duckdb_mbx_bytes_free(p)
        lib.duckdb_mb_arrow_destroy(h)
        t4 = time.perf_counter()
        if rep:
            t["query"] += t1 - t0
            t["getter"] += t2 - t1
            t["py_copy"] += t3 - t2
            t["free"] += t4 - t3
slices = n // 1_000_000
print(json.dumps({k: v / slices * 1e3 for k, v in t.items()} | {"unit": "ms per 1e6-row slice (8 MB)"}))
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c2 = m.connect_with_config(cfg).value
c2.query(f"CREATE TABLE c4 AS SELECT i * 2654435761 AS v FROM range({n}) tbl(i)")
c2.query("SELECT v FROM c4 LIMIT 1000000 OFFSET 3000000")
print(json.dumps(c2.last_profile()))
