#!/usr/bin/env python3
"""A/B sweep of the fused filter-aggregate kernel launch variants in ONE
process (cdna_hip_programming.md §5.4 rule 24): interleaved rounds, median and
min kernel time per variant, plus the HBM calibration kernels.  GPU only."""
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
c.query(f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({n}) tbl(i)")
cal = c.hbm_calibrate(4 << 30, 5)
print(json.dumps({"calibration": cal}), flush=True)
variants = [f"u{u}_{nt}_{ch}_g{g}" for u in (2, 4, 8) for nt in ("nt", "pl") for ch in ("gs", "ch") for g in (4, 8, 16)]
if os.environ.get("SWEEP_VARIANTS"):
    variants = os.environ["SWEEP_VARIANTS"].split(",")
rounds = int(os.environ.get("SWEEP_ROUNDS", "5"))
sqls = {"count": "SELECT COUNT(*) FROM t WHERE x > 24", "count_sum": "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24",
        "count_sum_min_max": "SELECT COUNT(*), SUM(x), MIN(x), MAX(x) FROM t WHERE x > 24"}
if os.environ.get("SWEEP_SQLS"):
    sqls = {k: v for k, v in sqls.items() if k in os.environ["SWEEP_SQLS"].split(",")}
res = {}
for name, sql in sqls.items():
    times = {v: [] for v in variants}
    for rnd in range(rounds):
        order = variants if rnd % 2 == 0 else variants[::-1]
        for v in order:
            os.environ["MBX_FA_VARIANT"] = v.split("+")[0]
            os.environ["MBX_FA_COUNT_AS_SUM"] = "1" if v.endswith("+cas") else "0"
            r = c.query(sql)
            assert isinstance(r, m.Ok), r
            times[v] += [k["ms"] for k in c.last_profile()["kernels"] if k["name"] == "filter_agg"]
    table = sorted(((statistics.median(t), min(t), v) for v, t in times.items()))
    res[name] = [{"variant": v, "median_ms": md, "min_ms": mn, "gbs_median": n * 8 / md / 1e6} for md, mn, v in table]
    print(name, json.dumps(res[name][:6]), flush=True)
os.environ.pop("MBX_FA_VARIANT", None)
json.dump({"rows": n, "calibration": cal, "sweep": res}, open(os.path.join(ROOT, "gpurun_out", "sweep_filter.json"), "w"), indent=1)
