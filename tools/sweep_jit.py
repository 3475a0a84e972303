#!/usr/bin/env python3
"""A/B of run-time compiled aggregate kernel shapes in ONE process (interleaved
rounds): MBX_JIT_U rows per thread, MBX_JIT_LEAN.  GPU only."""
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
variants = [("1", ""), ("2", ""), ("4", ""), ("8", ""), ("4", "1"), ("2", "1")]
times = {v: [] for v in variants}
ref = None
for rnd in range(7):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        os.environ["MBX_JIT_U"] = v[0]
        if v[1]:
            os.environ["MBX_JIT_LEAN"] = "1"
        else:
            os.environ.pop("MBX_JIT_LEAN", None)
        r = c.query(sql)
        assert isinstance(r, m.Ok), r
        ref = ref or r.value.rows
        assert r.value.rows == ref
        times[v] += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == "jit_aggregate"]
res = sorted((statistics.median(t), f"U{v[0]}{'_lean' if v[1] else ''}") for v, t in times.items() if t)
print(json.dumps({"sql": sql, "rows": n, "median_ms": res}))
