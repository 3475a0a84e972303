#!/usr/bin/env python3
"""A/B of run-time compiled aggregate kernel shapes in ONE process (interleaved
rounds): MBX_JIT_U units per thread, MBX_JIT_PAIRS (units of 2 rows with
vector loads, or single rows), MBX_JIT_BPC blocks per CU.  SWEEP_VARIANTS
= "U:PAIRS:BPC,..." overrides the list.  GPU only."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MBX_JIT"] = "sync"
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
sql = os.environ.get("SWEEP_SQL", "SELECT SUM(v + x) FROM t WHERE x > 24 AND k < 16")
variants = [tuple(v.split(":")) for v in os.environ.get(
    "SWEEP_VARIANTS", "4:0:8,8:0:8,4:0:4,8:0:4,4:0:2,8:0:2,4:1:4,2:1:4").split(",")]
times = {v: [] for v in variants}
ref = None
for rnd in range(7):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        os.environ["MBX_JIT_U"] = v[0]
        os.environ["MBX_JIT_PAIRS"] = v[1]
        os.environ["MBX_JIT_BPC"] = v[2]
        r = c.query(sql)
        assert isinstance(r, m.Ok), r
        ref = ref or r.value.rows
        assert r.value.rows == ref
        times[v] += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == "jit_aggregate"]
res = sorted((statistics.median(t), f"U{v[0]}{'_pairs' if v[1] == '1' else ''}_b{v[2]}") for v, t in times.items() if t)
print(json.dumps({"sql": sql, "rows": n, "median_ms": res}))
