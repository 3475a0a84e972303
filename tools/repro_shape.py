#!/usr/bin/env python3
"""Runs ONE query shape from tools/shape_bench.py at a given size in a fresh
process (debug aid).  Usage: repro_shape.py <rows> <sql>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1])
sql = sys.argv[2]
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
r = c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, CAST(mbx_synth(8, i, 4) AS INTEGER) AS k2, "
            f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
assert isinstance(r, m.Ok), r.error.message
r = c.query(sql)
print(n, sql, "->", "OK" if isinstance(r, m.Ok) else r.error.message, flush=True)
if isinstance(r, m.Ok):
    print(r.value.rows[:3], c.last_profile()["kernels"], flush=True)
sys.exit(0 if isinstance(r, m.Ok) else 3)
