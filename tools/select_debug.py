#!/usr/bin/env python3
"""One-pass select: cycle split of the controller work (MBX_SL_DEBUG), 1e9 rows.  GPU only."""
import os
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
for sql in os.environ.get("SQLS", "SELECT x FROM t WHERE x > 24|SELECT k, v FROM t WHERE x > 24").split("|"):
    for rep in range(3):
        os.environ["MBX_SL_DEBUG"] = "1" if rep == 2 else ""
        if rep < 2:
            os.environ.pop("MBX_SL_DEBUG")
        st = c.query_stream(sql).value
        st.close()
        ks = [(k["name"], round(k["ms"], 3)) for k in c.last_profile()["kernels"]]
        print(sql, rep, ks, flush=True)
