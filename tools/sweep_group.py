#!/usr/bin/env python3
"""A/B sweep of the fused GROUP BY (group_direct) launch variants on the C3
table in ONE process: interleaved rounds, median/min kernel time.  GPU only.
Variants: MBX_GD_VARIANT = "d<depth>_g<blocks per CU>" (LDS-DMA) or "seg",
with options "+r<replicas>", "+x1" (XCD-grouped step windows) and "+atomic"
(the table flush through global atomics instead of per-workgroup records)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

m = ge._load()
cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({n}) tbl(i)")
variants = os.environ.get("SWEEP_VARIANTS", "seg,d2_g1,d3_g1,d4_g1,d2_g2,d3_g2").split(",")
rounds = int(os.environ.get("SWEEP_ROUNDS", "7"))
sqls = {"c3": "SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k", "count": "SELECT k, COUNT(*) FROM t GROUP BY k"}
if os.environ.get("SWEEP_SQLS"):
    sqls = {k: v for k, v in sqls.items() if k in os.environ["SWEEP_SQLS"].split(",")}
res = {}
ref = {}
for name, sql in sqls.items():
    times = {v: [] for v in variants}
    for rnd in range(rounds):
        for v in (variants if rnd % 2 == 0 else variants[::-1]):
            os.environ["MBX_GD_VARIANT"] = v.split("+")[0]
            os.environ.pop("MBX_GD_R", None)
            os.environ.pop("MBX_GD_XCD", None)
            os.environ.pop("MBX_GD_ATOMIC_FLUSH", None)
            for opt in v.split("+")[1:]:
                if opt == "atomic":
                    os.environ["MBX_GD_ATOMIC_FLUSH"] = "1"  # the table flush through global atomics
                if opt.startswith("x"):
                    os.environ["MBX_GD_XCD"] = opt[1:]  # x1: XCD-grouped step windows
                if opt.startswith("r"):
                    os.environ["MBX_GD_R"] = opt[1:]
            r = c.query(sql)
            assert isinstance(r, m.Ok), r
            rows = sorted(r.value.rows)
            assert ref.setdefault(name, rows) == rows, (name, v)  # every variant gives the same answer
            times[v] += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == "group_direct"]
    bpr = 12 if name == "c3" else 4
    table = sorted((statistics.median(t), min(t), v) for v, t in times.items())
    res[name] = [{"variant": v, "median_ms": md, "min_ms": mn, "gbs_median": n * bpr / md / 1e6} for md, mn, v in table]
    print(name, json.dumps(res[name]), flush=True)
os.environ.pop("MBX_GD_VARIANT", None)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"rows": n, "sweep": res}, open(os.path.join(ROOT, "gpurun_out", "sweep_group.json"), "w"), indent=1)
