"""Where the time of a high-cardinality GROUP BY query goes outside its
kernels: the c3h / c3s statement over ROWS rows with G groups, timed per query
(wall) next to its kernels (the engine's event profile).  Run under
`rocprofv3 --hip-trace --kernel-trace --stats` for the HIP API split.
usage: python tools/c3h_host_probe.py [rows] [groups...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import load_mbx  # noqa: E402

mbx = load_mbx()

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
groups = [int(g) for g in sys.argv[2:]] or [100_000, 1_000_000]
cfg = mbx.Config.create()
cfg.set("gpu_device", "0")
cfg.set("mbx_profile", "true")
conn = mbx.connect_with_config(cfg).value
for g in groups:
    conn.query(f"CREATE OR REPLACE TABLE th AS SELECT mbx_synth(7, i, {g}) AS k, "
               f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range(0, {rows}) tbl(i)")
    sql = "SELECT k, SUM(v), COUNT(*) FROM th GROUP BY k"
    for rep in range(6):
        conn.profile_drain()
        t0 = time.perf_counter()
        rr = conn.query_raw(sql)
        t1 = time.perf_counter()
        n = rr.row_count()
        rr.close()
        t2 = time.perf_counter()
        kern = conn.profile_drain()
        ks = {}
        for k in kern:
            ks[k["name"]] = ks.get(k["name"], 0.0) + k["ms"]
        print(f"groups {g} rep {rep}: query {1e3 * (t1 - t0):.3f} ms, destroy {1e3 * (t2 - t1):.3f} ms, "
              f"rows {n}, kernels {sum(ks.values()):.3f} ms {ks}", flush=True)
