#!/usr/bin/env python3
"""C3's missing roofline share, looked for in the clock (VERDICT r4 item 2;
MI355X_MICROARCH.md DVFS item 6).  Loads the clock-stamp diagnostic build
(libduckdb_mb_amd_clk.so, `make -C duckdb.mbt_amd clockdiag`; set
DUCKDB_MB_AMD_LIB to it), builds the C2 table and then the C3 table (the order
of bench.py's extra.c3), and for each kernel and launch cadence records per
launch the kernel time (HIP events) and the in-kernel clock of every
workgroup (d s_memtime / d s_memrealtime x 100 MHz around the main loop):

  kernels   c3 = group_direct_lds (SELECT k, SUM(v), COUNT(*) ... GROUP BY k),
            c2 = filter_agg_lds (SELECT COUNT(*) ... WHERE x > 24),
            ring2 = the two-array ring read of C3's shape with no atomics
            (duckdb_mbx_hbm_calibrate_ex slot 7, timed by its own events)
  cadence   b2b (back to back), gap1 / gap10 / gap100 (1 / 10 / 100 ms idle
            before each launch)

Before each kernel's series: >= 2 s of back-to-back launches.  One JSON line
per (kernel, cadence) on stdout.  With an argument "pmc" it instead runs only
the c3 b2b series with the product library, for a rocprofv3 --pmc
GRBM_GUI_ACTIVE pass (effective clock = GRBM_GUI_ACTIVE / 8 / kernel time).
Usage: c3_clock.py [pmc] [launches]"""
import importlib.util
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
m = importlib.util.module_from_spec(spec)
sys.modules["duckdb_mbt_amd"] = m
spec.loader.exec_module(m)

N = 1_000_000_000
C2 = f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range({N}) tbl(i)"
C3 = (f"CREATE TABLE g AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
      f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({N}) tbl(i)")
Q = {"c3": ("SELECT k, SUM(v), COUNT(*) FROM g GROUP BY k", "group_direct", 12.0 * N),
     "c2": ("SELECT COUNT(*) FROM t WHERE x > 24", "filter_agg", 8.0 * N)}
GAPS = {"b2b": 0.0, "gap1": 0.001, "gap10": 0.010, "gap100": 0.100}

args = [a for a in sys.argv[1:]]
pmc = bool(args) and args[0] == "pmc"
if pmc:
    args = args[1:]
K = int(args[0]) if args else 15

cfg = m.Config.create()
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
assert isinstance(c.query(C2), m.Ok)
assert isinstance(c.query(C3), m.Ok)
ncu = 256


def launch(kind):
    """one launch: (kernel ms, per-workgroup clocks)"""
    if kind == "ring2":
        cal = c.hbm_calibrate(12_000_000_000, 1)  # the last stamped launch is the ring2 shape (slot 7)
        ms = 12_000_000_000 / (cal["ring_read2_gbs"] * 1e9) * 1e3
    else:
        sql, kname, _ = Q[kind]
        c.query_raw(sql).close()
        ks = [x["ms"] for x in c.last_profile()["kernels"] if x["name"] == kname]
        ms = ks[-1] if ks else None
    return ms, c.clock_stamps(ncu)


def series(kind, gap):
    t_end = time.time() + 2.0
    while time.time() < t_end:  # >= 2 s of back-to-back launches first
        launch(kind)
    rows = []
    for _ in range(K):
        if gap:
            time.sleep(gap)
        ms, clk = launch(kind)
        g = sorted(x["ghz"] for x in clk)
        rows.append({"ms": ms, "ghz_med": g[len(g) // 2] if g else None, "ghz_min": g[0] if g else None,
                     "ghz_max": g[-1] if g else None,
                     "loop_us_med": statistics.median(x["loop_us"] for x in clk) if clk else None})
    return rows


kinds = ["c3"] if pmc else ["c3", "c2", "ring2", "c3"]
gaps = ["b2b"] if pmc else list(GAPS)
for kind in kinds:
    for gname in gaps:
        rows = series(kind, GAPS[gname])
        ms = [r["ms"] for r in rows if r["ms"]]
        gh = [r["ghz_med"] for r in rows if r["ghz_med"]]
        alg = 12.0 * N if kind in ("c3", "ring2") else 8.0 * N
        out = {"kernel": kind, "cadence": gname, "launches": len(rows),
               "ms_median": statistics.median(ms) if ms else None, "ms_min": min(ms) if ms else None,
               "ms_max": max(ms) if ms else None,
               "tbs_median": alg / (statistics.median(ms) * 1e-3) / 1e12 if ms else None,
               "clock_ghz_median": statistics.median(gh) if gh else None,
               "clock_ghz_min": min(gh) if gh else None, "clock_ghz_max": max(gh) if gh else None,
               "per_launch": rows}
        print(json.dumps(out), flush=True)
c.close()
