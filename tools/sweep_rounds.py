#!/usr/bin/env python3
"""select_rounds launch-shape sweep at 1e9 rows (GPU only): each config is set
through the MBX_SR_* environment (read per launch), timed over 5 queries by the
per-kernel profile; MBX_SR_DEBUG prints the per-role cycle split to stderr.
Usage: sweep_rounds.py [rows] [shape ...]"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
SQL = {"sel": "SELECT x FROM t WHERE x > 24", "sel2": "SELECT k, v FROM t WHERE x > 24",
       "sel3": "SELECT v FROM t WHERE x > 24 AND k < 16"}
shapes = sys.argv[2:] or ["sel"]
grid = json.loads(os.environ.get("GRID", '[{}]'))
for shape in shapes:
    for conf in grid:
        for k in [k for k in os.environ if k.startswith("MBX_SR_") and k != "MBX_SR_DEBUG"]:
            del os.environ[k]
        os.environ.update({k: str(v) for k, v in conf.items()})
        ms = []
        for i in range(5):
            r = c.query_stream(SQL[shape]).value
            r.close()
            ks = {k["name"]: k["ms"] for k in c.last_profile()["kernels"]}
            ms.append(sum(v for k, v in ks.items() if k.startswith("select") or k in ("filter_count", "filter_bits", "compact")))
        print(json.dumps({"shape": shape, "conf": conf, "ms_median": statistics.median(ms[1:]), "ms": ms,
                          "kernels": list(ks)}), flush=True)
