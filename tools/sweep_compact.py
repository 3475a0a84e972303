#!/usr/bin/env python3
"""Launch-shape sweep of the two-pass filter -> compaction (filter_bits, compact)
on a C3-style table, interleaved rounds, median kernel times.  GPU only.
Variants: "fb<blocks/CU>d<depth>_cp<blocks/CU>d<depth>" (0 = built-in default).
Usage: sweep_compact.py [rows]"""
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
c.query(f"CREATE TABLE t AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
        f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v, mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
sqls = {"sel": "SELECT x FROM t WHERE x > 24", "sel2": "SELECT k, v FROM t WHERE x > 24",
        "sel3": "SELECT v FROM t WHERE x > 24 AND k < 16"}
variants = os.environ.get("SWEEP_VARIANTS", "fb3d0_cp3d0,fb1d6_cp1d6,fb2d3_cp2d3,fb1d4_cp2d2").split(",")
rounds = int(os.environ.get("SWEEP_ROUNDS", "5"))
res = {}
for name, sql in sqls.items():
    times = {v: {"filter_bits": [], "compact": []} for v in variants}
    for rnd in range(rounds):
        for v in (variants if rnd % 2 == 0 else variants[::-1]):
            fb, cp = v.split("_")
            os.environ["MBX_FB_BLOCKS_PER_CU"] = fb[2:].split("d")[0]
            os.environ["MBX_FB_DEPTH"] = fb.split("d")[1]
            os.environ["MBX_CP_BLOCKS_PER_CU"] = cp[2:].split("d")[0]
            os.environ["MBX_CP_DEPTH"] = cp.split("d")[1]
            st = c.query_stream(sql).value  # the result stays in HBM
            st.close()
            for k in c.last_profile()["kernels"]:
                if k["name"] in times[v]:
                    times[v][k["name"]].append(k["ms"])
    res[name] = {v: {kn: statistics.median(t) for kn, t in d.items() if t} for v, d in times.items()}
    print(name, json.dumps(res[name]), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump({"rows": n, "sweep": res}, open(os.path.join(ROOT, "gpurun_out", "sweep_compact.json"), "w"), indent=1)
