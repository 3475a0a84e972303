#!/usr/bin/env python3
"""Arrow string getter of device columns: formatted by the text kernels vs the
host per-cell path (the result materialized first), 1e6-row slices (the
MoonBit decoder cap).  GPU only.  Usage: text_getter_bench.py [rows]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(11, i, 2000000000) - 1000000000 AS DECIMAL(15,2)) AS d, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS b FROM range({n}) tbl(i)")
c.query(f"CREATE TABLE h AS SELECT CAST(mbx_synth(9, i, 1099511627776) AS HUGEINT) * 100000000000000000000 AS h "
        f"FROM range({n}) tbl(i)")
out = {"rows": n}
for name, sql in (("decimal_15_2", "SELECT d FROM t"), ("bigint", "SELECT b FROM t"), ("hugeint_1e31", "SELECT h FROM h")):
    for path in ("device", "host"):
        ts, nbytes = [], 0
        for rep in range(7):
            a = c.query_arrow(sql).value
            if path == "host":
                m._take(m.lib.duckdb_mb_arrow_get_column_double(a._h, 0))  # materializes the result on the host
            c.profile_drain()
            t0 = time.perf_counter()
            b = m._take(m.lib.duckdb_mb_arrow_get_column_string(a._h, 0))
            ts.append(time.perf_counter() - t0)
            nbytes = len(b)
            ks = c.profile_drain()
            a.close()
        out[f"{name} {path}"] = {"median_ms": statistics.median(ts[2:]) * 1e3, "bytes": nbytes,
                                 "kernels_ms": {k["name"]: round(k["ms"], 4) for k in ks}}
print(json.dumps(out, indent=1))
