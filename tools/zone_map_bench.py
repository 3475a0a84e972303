#!/usr/bin/env python3
"""Zone-map kernel time per CTAS: CREATE OR REPLACE TABLE over range(n) with a
generated INT64 (and INT32) column, REPS times; prints the median `zone_map`
profile entries (ms) per column type.  GPU only.  Usage: zone_map_bench.py [rows]"""
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
out = {}
for name, expr in [("int64", "mbx_synth(42, i, 50) + 1"), ("int32", "CAST(mbx_synth(7, i, 32) AS INTEGER)")]:
    ms = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        r = c.query_raw(f"CREATE OR REPLACE TABLE zm AS SELECT {expr} AS x FROM range({n}) tbl(i)")
        r.close()
        ms += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == "zone_map"]
    out[name] = {"zone_map_ms_median": statistics.median(ms[1:]) if len(ms) > 1 else None, "all": ms}
print(json.dumps(out), flush=True)
