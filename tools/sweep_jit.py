#!/usr/bin/env python3
"""A/B of run-time compiled kernel shapes in ONE process (interleaved rounds).
GPU only.  Environment:
  SWEEP_SQL       the query (default: the fused aggregate shape)
  SWEEP_KERNEL    profiled kernel name to time (default jit_aggregate)
  SWEEP_VARIANTS  variants separated by ',', each a ':'-separated list of
                  NAME=value settings (e.g. MBX_JIT_U=4:MBX_JIT_BPC=4)
Usage: sweep_jit.py [rows]"""
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
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, CAST(mbx_synth(8, i, 4) AS INTEGER) AS k2, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
sql = os.environ.get("SWEEP_SQL", "SELECT SUM(v + x) FROM t WHERE x > 24 AND k < 16")
kernel = os.environ.get("SWEEP_KERNEL", "jit_aggregate")
spec = os.environ.get("SWEEP_VARIANTS", "MBX_JIT_U=4:MBX_JIT_BPC=8,MBX_JIT_U=8:MBX_JIT_BPC=8,MBX_JIT_U=4:MBX_JIT_BPC=4,"
                      "MBX_JIT_U=8:MBX_JIT_BPC=4,MBX_JIT_U=4:MBX_JIT_BPC=2,MBX_JIT_U=2:MBX_JIT_PAIRS=1:MBX_JIT_BPC=4")
variants = [tuple(tuple(kv.split("=", 1)) for kv in v.split(":") if kv) for v in spec.split(",")]
names = sorted({k for v in variants for k, _ in v})
times = {v: [] for v in variants}
ref = None
for rnd in range(7):
    for v in (variants if rnd % 2 == 0 else variants[::-1]):
        for k in names:
            os.environ.pop(k, None)
        for k, val in v:
            os.environ[k] = val
        r = c.query(sql)
        assert isinstance(r, m.Ok), r
        ref = ref or r.value.rows
        assert r.value.rows == ref
        times[v] += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == kernel]
res = sorted((statistics.median(t), ":".join(f"{k}={val}" for k, val in v)) for v, t in times.items() if t)
print(json.dumps({"sql": sql, "rows": n, "kernel": kernel, "median_ms": res}))
