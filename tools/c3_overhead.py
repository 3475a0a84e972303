#!/usr/bin/env python3
"""Where the C3 step's time goes beyond the GROUP BY kernel: end-to-end query
(raw handle), plus the one-call cell pull, with and without the per-kernel
event profile.  GPU only.  Usage: c3_overhead.py [rows]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
out = {}
for prof in ("false", "true"):
    cfg = m.Config.create()
    cfg.set("mbx_profile", prof)
    c = m.connect_with_config(cfg).value
    c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
            f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    sql = "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k"
    q_only, q_cells = [], []
    for i in range(25):
        t0 = time.perf_counter()
        rr = c.query_raw(sql)
        t1 = time.perf_counter()
        rr.cells()
        t2 = time.perf_counter()
        rr.close()
        q_only.append(t1 - t0)
        q_cells.append(t2 - t0)
    r = {"query_ms": statistics.median(q_only[5:]) * 1e3, "query_plus_cells_ms": statistics.median(q_cells[5:]) * 1e3}
    if prof == "true":
        c.profile_drain()
        c.query_raw(sql).close()
        r["kernels"] = c.last_profile()["kernels"]
    out[f"profile={prof}"] = r
    print(prof, json.dumps(r), flush=True)
    c.close()
