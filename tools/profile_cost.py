#!/usr/bin/env python3
"""What the per-kernel HIP-event profile (mbx_profile, on in bench.py's timed
loop) costs end to end: the C2 query at 1e9 rows on two connections over the
same table data shape, profile off and on, alternated in rounds.  GPU only."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
conns = {}
for prof in ("false", "true"):
    cfg = m.Config.create()
    cfg.set("mbx_profile", prof)
    c = m.connect_with_config(cfg).value
    c.query(f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
    conns[prof] = c
sql = "SELECT COUNT(*) FROM t WHERE x > 24"
res = {"false": [], "true": []}
for rnd in range(6):
    for prof in ("false", "true") if rnd % 2 == 0 else ("true", "false"):
        c = conns[prof]
        for i in range(10):
            c.query_raw(sql).close()
        ts = []
        for i in range(100):
            t0 = time.perf_counter()
            rr = c.query_raw(sql)
            rr.value(0, 0)
            rr.close()
            ts.append(time.perf_counter() - t0)
        res[prof].append(statistics.median(ts) * 1e6)
        print(json.dumps({"round": rnd, "profile": prof, "median_us": res[prof][-1]}), flush=True)
print(json.dumps({k: {"round_medians_us": v, "median_us": statistics.median(v)} for k, v in res.items()}))
