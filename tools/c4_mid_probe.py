#!/usr/bin/env python3
"""8 MB Arrow read-back per method: 1e8 INT64 rows, read back in 1e6-row
slices (query_arrow + duckdb_mb_arrow_get_column_int64, as bench.py's C4 leg),
getter time per slice.  The method comes from MBX_LINK_MID_MODE (0 runtime
copy, 1 registered destination, 2 pinned bounce; unset = the adaptive choice);
run it once per mode.  One JSON line: getter GB/s (mean over the slices), the
median / min slice and the first 12 slices' GB/s (the adaptive trial phase)."""
import ctypes
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
c = m.connect().value
assert isinstance(c.query(f"CREATE TABLE c4 AS SELECT i * 2654435761 % 9223372036854775807 AS v FROM range({n}) tbl(i)"),
                  m.Ok)
rates = []
for rep in range(2):
    for k in range(0, n, 1_000_000):
        a = c.query_arrow(f"SELECT v FROM c4 LIMIT 1000000 OFFSET {k}").value
        t0 = time.perf_counter()
        bp = m.lib.duckdb_mb_arrow_get_column_int64(a._h, 0)
        dt = time.perf_counter() - t0
        ln = m.lib.duckdb_mbx_bytes_len(bp)
        assert ln == 4 + 8 * min(1_000_000, n - k)
        m.lib.duckdb_mbx_bytes_free(bp)
        a.close()
        rates.append((ln - 4) / dt / 1e9)
print(json.dumps({"mode": os.environ.get("MBX_LINK_MID_MODE", "adaptive"), "slices": len(rates),
                  "getter_gbs_mean": len(rates) / sum(1 / r for r in rates),
                  "median_gbs": statistics.median(rates), "max_gbs": max(rates),
                  "first12": [round(r, 1) for r in rates[:12]]}), flush=True)
c.close()
