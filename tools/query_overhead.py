#!/usr/bin/env python3
"""Per-query host overhead of the fused C2 path: end-to-end time of
duckdb_mb_query (+ result cell read) vs the kernel time, with and without
the per-kernel event profile.  GPU only.  Usage: query_overhead.py [rows]"""
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
out = {}
for prof in ("false", "true"):
    cfg = m.Config.create()
    cfg.set("mbx_profile", prof)
    c = m.connect_with_config(cfg).value
    c.query(f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    for sql in ("SELECT COUNT(*) FROM t WHERE x > 24", "SELECT 1"):
        ts = []
        for i in range(300):
            t0 = time.perf_counter()
            rr = c.query_raw(sql)
            rr.value(0, 0)
            rr.close()
            ts.append(time.perf_counter() - t0)
        out[f"profile={prof} {sql}"] = {"median_us": statistics.median(ts[50:]) * 1e6, "min_us": min(ts) * 1e6}
    # the C3 shape: a 32-key GROUP BY whose 96 cells come back as text in one call
    c.query(f"CREATE TABLE t3 AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
            f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
    for sql in ("SELECT k, SUM(v), COUNT(*) FROM t3 GROUP BY k",):
        ts = []
        for i in range(300):
            t0 = time.perf_counter()
            rr = c.query_raw(sql)
            rr.cells()
            rr.close()
            ts.append(time.perf_counter() - t0)
        out[f"profile={prof} {sql}"] = {"median_us": statistics.median(ts[50:]) * 1e6, "min_us": min(ts) * 1e6}
    if prof == "false":
        # prepared re-execution: bound-plan cache on / off (MBX_PLAN_CACHE=0)
        st = c.prepare("SELECT COUNT(*) FROM t WHERE x > ?").value
        for cache in ("1", "0"):
            os.environ["MBX_PLAN_CACHE"] = cache
            ts = []
            for i in range(300):
                st.bind_bigint(1, 24 + (i & 1))
                t0 = time.perf_counter()
                rr = m.lib.duckdb_mb_execute_prepared(st._h)
                m.lib.duckdb_mb_result_destroy(rr)
                ts.append(time.perf_counter() - t0)
            out[f"prepared execute, plan cache={cache}"] = {"median_us": statistics.median(ts[50:]) * 1e6,
                                                            "min_us": min(ts) * 1e6, "stats": st.plan_stats()}
        os.environ.pop("MBX_PLAN_CACHE")
        st.close()
    if prof == "true":
        c.profile_drain()
        c.query_raw("SELECT COUNT(*) FROM t WHERE x > 24").close()
        out["profile kernels"] = c.last_profile()
    c.close()
print(json.dumps(out, indent=1))
