#!/usr/bin/env python3
"""Environment-knob sweep over query shapes (GPU only): builds shape_bench.py's
table (k, k2 INT32; v, x INT64) once, then for every config of GRID (a JSON
list of env dicts, read by the library at each launch) times each shape's
kernels (median of 4 after one warm-up) from the per-query profile.
Usage: GRID='[{}, {"MBX_FM_DEPTH": 3}]' sweep_env.py rows shape [shape ...]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

SQL = {
    "filter_multi": "SELECT COUNT(*), SUM(v) FROM t WHERE x > 24 AND k < 16",
    "filter_multi3": "SELECT SUM(v), MIN(v), MAX(v) FROM t WHERE x BETWEEN 10 AND 40 AND k < 16 AND k2 = 1",
    "c3_where": "SELECT k, SUM(v), COUNT(*) FROM t WHERE x > 24 GROUP BY k",
    "c3_where2": "SELECT k, SUM(v), COUNT(*) FROM t WHERE x > 24 AND k2 = 1 GROUP BY k",
    "c3": "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k",
    "c3_mm": "SELECT k, SUM(v), MIN(v), MAX(v), COUNT(*) FROM t GROUP BY k",
    "c3_two": "SELECT k, SUM(v), SUM(x), COUNT(*) FROM t GROUP BY k",
    "c5": "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24",
    "filter_mm": "SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM t WHERE x > 24 AND k < 16",
    "filter_cnt2": "SELECT COUNT(*) FROM t WHERE x > 24 AND k < 16",
    "filter_wide": "SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM t WHERE x > 24 AND k < 16",
    # NULLABLE=1
    "c2n": "SELECT COUNT(*) FROM t WHERE xn > 24",
    "c5n": "SELECT COUNT(*), SUM(xn) FROM t WHERE xn > 24",
    "c5n_sumv": "SELECT COUNT(vn), SUM(vn) FROM t WHERE x > 24",
    "c3n": "SELECT k, SUM(vn), COUNT(*) FROM t GROUP BY k",
    "c3n_where": "SELECT k, SUM(vn), COUNT(*) FROM t WHERE x > 24 GROUP BY k",
    "c3n_mm": "SELECT k, COUNT(vn), SUM(vn), MIN(vn), MAX(vn) FROM t GROUP BY k",
}
m = ge._load()
n = int(sys.argv[1])
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
extra = (", CASE WHEN mbx_synth(13, i, 10) = 0 THEN NULL ELSE mbx_synth(42, i, 50) + 1 END AS xn, "
         "CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 END AS vn"
         if os.environ.get("NULLABLE") else "")
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, CAST(mbx_synth(8, i, 4) AS INTEGER) AS k2, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x{extra} FROM range({n}) tbl(i)")
base_env = dict(os.environ)
for shape in sys.argv[2:]:
    ref = None
    for conf in json.loads(os.environ.get("GRID", "[{}]")):
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update({k: str(v) for k, v in conf.items()})
        ms, rows = [], None
        for i in range(5):
            rr = c.query_raw(SQL[shape])
            rows = [[rr.value(col, r) for col in range(rr.column_count())] for r in range(rr.row_count())]
            rr.close()
            ks = c.last_profile()["kernels"]
            if i:
                ms.append(sum(k["ms"] for k in ks))
            if i == 0 and os.environ.get("MBX_JIT") != "0":
                time.sleep(float(os.environ.get("JIT_WAIT", "0")))
        ref = ref or rows
        print(json.dumps({"shape": shape, "conf": conf, "ms_median": statistics.median(ms),
                          "kernels": [k["name"] for k in ks], "same_result": rows == ref}), flush=True)
