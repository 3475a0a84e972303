#!/usr/bin/env python3
"""C3 placement probe for PMC passes: builds the C3 table either alone
("alone") or after the 8 GB C2 table ("after_c2", the order bench.py's
extra.c3 uses), then runs the C3 GROUP BY K times.  Run it under
`rocprofv3 --pmc <TCP_UTCL1_* / TCC_* counters>` once per mode; the counters of
the group_direct launches tell translation misses from channel effects.
Prints one JSON line with the kernel's median ms (HIP events).
Usage: c3_tlb_probe.py alone|after_c2 [K]"""
import importlib.util
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
m = importlib.util.module_from_spec(spec)
sys.modules["duckdb_mbt_amd"] = m
spec.loader.exec_module(m)

C2 = "CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range(1000000000) tbl(i)"
C3 = ("CREATE TABLE g AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
      "mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range(1000000000) tbl(i)")
Q = "SELECT k, SUM(v), COUNT(*) FROM g GROUP BY k"

mode = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
for kv in os.environ.get("C3_CFG", "").split(","):
    if "=" in kv:
        cfg.set(*kv.split("=", 1))
c = m.connect_with_config(cfg).value
if mode == "after_c2":
    assert isinstance(c.query(C2), m.Ok)
assert isinstance(c.query(C3), m.Ok)
for _ in range(2):
    c.query_raw(Q).close()
c.profile_drain()
for _ in range(k):
    c.query_raw(Q).close()
ks = sorted(x["ms"] for x in c.profile_drain() if x["name"] == "group_direct")
print(json.dumps({"mode": mode, "cfg": os.environ.get("C3_CFG", ""), "group_direct_ms_median": round(ks[len(ks) // 2], 4),
                  "min": round(ks[0], 4), "max": round(ks[-1], 4), "k": k}), flush=True)
c.close()
