#!/usr/bin/env python3
"""Where a C3 step's time goes: the C2 table, then the C3 table (the bench's
extra.c3 order), then K steps of the C3 query exactly as bench.py's step runs
them (query_raw + result_text), each step's wall time and every kernel the
profile saw in it.  One JSON line."""
import importlib.util
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
m = importlib.util.module_from_spec(spec)
sys.modules["duckdb_mbt_amd"] = m
spec.loader.exec_module(m)
sys.path.insert(0, HERE)
import bench  # noqa: E402

cfg = m.Config.create()
cfg.set("gpu_device", "0")
cfg.set("mbx_profile", "true")
c = m.connect_with_config(cfg).value
out = {}
if len(sys.argv) < 2 or sys.argv[1] != "alone":
    c.query(bench.workload("c2", 0, 1_000_000_000)["setup"])
w = bench.workload("c3", 0, 1_000_000_000)
c.query(w["setup"])
step = bench.make_step(c, "c3", w["sql"])
for _ in range(3):
    step()
c.profile_drain()
steps = []
for _ in range(6):
    t0 = time.perf_counter()
    step()
    wall = (time.perf_counter() - t0) * 1e3
    ks = c.profile_drain()
    steps.append({"wall_ms": round(wall, 4), "kernels": [(k["name"], round(k["ms"], 4)) for k in ks]})
out["steps"] = steps
t0 = time.perf_counter()
for _ in range(20):
    step()
out["mean_ms_20"] = (time.perf_counter() - t0) / 20 * 1e3
print(json.dumps(out), flush=True)
c.close()
