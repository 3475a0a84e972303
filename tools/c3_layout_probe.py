#!/usr/bin/env python3
"""C3 kernel time vs what else is resident in HBM: the C3 table alone, after
an 8 GB C2 table, before it, and after that table is dropped; and the C2
kernel with its table created first or after the C3 table.  One JSON line."""
import json
import os
import sys
import importlib.util

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
m = importlib.util.module_from_spec(spec)
sys.modules["duckdb_mbt_amd"] = m
spec.loader.exec_module(m)

C2 = "CREATE TABLE {n} AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range(1000000000) tbl(i)"
C3 = ("CREATE TABLE {n} AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
      "mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range(1000000000) tbl(i)")


def conn():
    cfg = m.Config.create()
    cfg.set("mbx_profile", "true")
    return m.connect_with_config(cfg).value


def kernel_ms(c, sql, name, k=15):
    for _ in range(3):
        c.query_raw(sql).close()
    c.profile_drain()
    for _ in range(k):
        c.query_raw(sql).close()
    ks = sorted(x["ms"] for x in c.profile_drain() if x["name"] == name)
    return round(ks[len(ks) // 2], 4)


def c3_ms(c, t, k=15):
    return kernel_ms(c, f"SELECT k, SUM(v), COUNT(*) FROM {t} GROUP BY k", "group_direct", k)


def c2_ms(c, t, k=15):
    return kernel_ms(c, f"SELECT COUNT(*) FROM {t} WHERE x > 24", "filter_agg", k)


out = {}
c = conn()
c.query(C3.format(n="g"))
out["c3_alone"] = c3_ms(c, "g")
c.query(C2.format(n="t"))
out["c3_then_c2_resident"] = c3_ms(c, "g")
out["c2_after_c3 (C2 kernel)"] = c2_ms(c, "t")
c.close()
c = conn()
c.query(C2.format(n="t"))
out["c2_first (C2 kernel)"] = c2_ms(c, "t")
c.query(C3.format(n="g"))
out["c2_then_c3"] = c3_ms(c, "g")
c.query("DROP TABLE t")
out["c2_then_c3_c2_dropped"] = c3_ms(c, "g")
c.hbm_calibrate(2 << 30, 3)
out["after_calibrate"] = c3_ms(c, "g")
c.close()
print(json.dumps(out), flush=True)
