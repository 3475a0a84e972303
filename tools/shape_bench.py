#!/usr/bin/env python3
"""Kernel-level timing of query shapes around the hot path (filter -> project
-> aggregate variants) on a C3-style table.  GPU only.  Usage: shape_bench.py [rows]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
# NULLABLE=1 adds NULL-able twins of x and v (10 % / 14 % NULLs) for the seln_* shapes
extra = (", CASE WHEN mbx_synth(13, i, 10) = 0 THEN NULL ELSE mbx_synth(42, i, 50) + 1 END AS xn, "
         "CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn"
         if os.environ.get("NULLABLE") else "")
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, CAST(mbx_synth(8, i, 4) AS INTEGER) AS k2, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x{extra} FROM range({n}) tbl(i)")
shapes = {
    "c2_count": "SELECT COUNT(*) FROM t WHERE x > 24",
    "c3": "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k",
    "c3_where": "SELECT k, SUM(v), COUNT(*) FROM t WHERE x > 24 GROUP BY k",
    "c3_where2": "SELECT k, SUM(v), COUNT(*) FROM t WHERE x > 24 AND k2 = 1 GROUP BY k",
    "c3_project": "SELECT k, SUM(v * 2), COUNT(*) FROM t GROUP BY k",
    "multi_key": "SELECT k, k2, SUM(v), COUNT(*) FROM t GROUP BY k, k2",
    "filter_sum_expr": "SELECT SUM(v + x) FROM t WHERE x > 24 AND k < 16",
    "filter_multi": "SELECT COUNT(*), SUM(v) FROM t WHERE x > 24 AND k < 16",
    "c3_jit": "SELECT k, SUM(v * 1), COUNT(*) FROM t GROUP BY k",
    "c3_where_jit": "SELECT k, SUM(v * 1), COUNT(*) FROM t WHERE x > 24 GROUP BY k",
    "group_expr2": "SELECT k, k2, SUM(v + x), MIN(v), COUNT(*) FROM t WHERE x + k2 > 24 GROUP BY k, k2",
    "filter_multi3": "SELECT SUM(v), MIN(v), MAX(v) FROM t WHERE x BETWEEN 10 AND 40 AND k < 16 AND k2 = 1",
    "wide_key": "SELECT v % 1000003, COUNT(*) FROM t GROUP BY v % 1000003",
    # selection compaction kept on the device (STREAM: the result stays in HBM; no batch is fetched)
    "sel": "STREAM SELECT x FROM t WHERE x > 24",
    "sel2": "STREAM SELECT k, v FROM t WHERE x > 24",
    "selv": "STREAM SELECT v FROM t WHERE x > 24",
    "sel3": "STREAM SELECT v FROM t WHERE x > 24 AND k < 16",
    "compact": "CREATE OR REPLACE TABLE tc AS SELECT x FROM t WHERE x > 24",
    "compact2": "CREATE OR REPLACE TABLE tc AS SELECT k, v FROM t WHERE x > 24",
    "compact_expr": "CREATE OR REPLACE TABLE tc AS SELECT v + x AS y FROM t WHERE x > 24 AND k < 16",
    # NULLABLE=1: a NULL-able predicate column, NULL-able outputs
    "seln_pred": "STREAM SELECT v FROM t WHERE xn > 24",
    "seln_out": "STREAM SELECT vn FROM t WHERE x > 24",
    "seln_both": "STREAM SELECT vn FROM t WHERE xn > 24 AND k < 16",
    "c2n": "SELECT COUNT(*) FROM t WHERE xn > 24",
    "c5n": "SELECT COUNT(*), SUM(xn) FROM t WHERE xn > 24",
    "c5n_sumv": "SELECT COUNT(vn), SUM(vn) FROM t WHERE x > 24",
    "c3n": "SELECT k, SUM(vn), COUNT(*) FROM t GROUP BY k",
    "c3n_where": "SELECT k, SUM(v), COUNT(*) FROM t WHERE xn > 24 GROUP BY k",
}
if os.environ.get("SHAPES"):
    shapes = {k: v for k, v in shapes.items() if k in os.environ["SHAPES"].split(",")}
out = {}
for name, sql in shapes.items():
    walls, kern = [], []
    if os.environ.get("JIT_WAIT"):  # let a run-time compiled kernel finish building first
        try:
            (c.query_stream(sql[7:]).value if sql.startswith("STREAM ") else c.query_raw(sql)).close()
        except Exception:  # noqa: BLE001
            pass
        time.sleep(float(os.environ["JIT_WAIT"]))
    for i in range(int(os.environ.get("REPS", "5"))):
        t0 = time.perf_counter()
        try:
            if sql.startswith("STREAM "):
                rr = c.query_stream(sql[7:]).value
            else:
                rr = c.query_raw(sql)  # engine time: no per-cell pull of the result
        except Exception as ex:  # noqa: BLE001
            out[name] = {"error": str(ex)}
            break
        walls.append(time.perf_counter() - t0)
        rr.close()
        prof = c.last_profile()
        kern.append({k["name"]: k["ms"] for k in prof["kernels"]})
    else:
        med = {k: statistics.median(d[k] for d in kern[1:] if k in d) for k in kern[-1]}
        out[name] = {"wall_ms_median": statistics.median(walls[1:]) * 1e3, "kernels_last": kern[-1], "kernels_median": med}
    print(name, json.dumps(out[name]), flush=True)
