#!/usr/bin/env python3
"""Fixed per-query cost of the in-library multi-device path (gpu_devices).

A tiny table (rows_per_shard rows per shard, so the kernels take a few
microseconds) is queried through duckdb_mb_query by an unsharded connection
and by connections with 2/4/8 shards listed on device 0; the difference in
per-query wall time is the sharding overhead: waking the persistent shard
workers, per-shard launches and the small D2H each, and the host merge.  The
library's own counters (duckdb_mbx_shard_stats) give the last dispatch and
merge times.  Prints one JSON line.

Usage: python tools/shard_overhead.py [--iters 2000] [--rows-per-shard 4096]
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_mbx():
    spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules["duckdb_mbt_amd"] = m
    spec.loader.exec_module(m)
    return m


def per_query_us(conn, sql, iters):
    for _ in range(50):
        conn.query_raw(sql).close()
    samples = []
    for _ in range(5):
        t0 = time.perf_counter()
        for _ in range(iters // 5):
            r = conn.query_raw(sql)
            r.value(0, 0)
            r.close()
        samples.append((time.perf_counter() - t0) / (iters // 5) * 1e6)
    return statistics.median(samples), samples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--rows-per-shard", type=int, default=4096)
    args = ap.parse_args()
    mbx = load_mbx()
    out = {"what": "per-query wall time through duckdb_mb_query (ctypes), tiny table; sharded = gpu_devices "
                   "listing device 0 k times", "rows_per_shard": args.rows_per_shard, "iters": args.iters,
           "queries": {}}
    for sql in ("SELECT COUNT(*) FROM t WHERE x > 24", "SELECT k, SUM(x), COUNT(*) FROM t GROUP BY k"):
        res = {}
        base = None
        for k in (1, 2, 4, 8):
            cfg = mbx.Config.create()
            if k > 1:
                cfg.set("gpu_devices", ",".join(["0"] * k))
            conn = mbx.connect_with_config(cfg).value
            n = args.rows_per_shard * k
            conn.query(f"CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x, CAST(mbx_synth(7, i, 32) AS INTEGER) "
                       f"AS k FROM range({n}) tbl(i)")
            us, samples = per_query_us(conn, sql, args.iters)
            st = conn.shard_stats() if k > 1 else {}
            if k == 1:
                base = us
            res[str(k)] = {"us_per_query": us, "samples_us": samples,
                           "overhead_vs_unsharded_us": us - base,
                           "last_dispatch_us": st.get("last_dispatch_us"),
                           "last_host_merge_us": st.get("last_combine_us"),
                           "host_results": st.get("host_results")}
            if k > 1:
                res[str(k)]["split_us"] = split(conn, sql)
            conn.close()
        out["queries"][sql] = res
    print(json.dumps(out), flush=True)


def split(conn, sql, iters=400):
    """Median over `iters` queries of where a sharded dispatch's time goes
    (duckdb_mbx_shard_timings / shard_stats): the slowest worker's wake-up,
    the last shard's launches queued, the last shard's partial on the host
    (its D2H + synchronisation), the whole dispatch, and the host merge after
    it; wall = the query's wall time through the C-ABI."""
    keys = ("wake_max", "launch_max", "done_max", "done_min", "dispatch", "merge", "wall")
    rows = {k: [] for k in keys}
    for _ in range(iters):
        t0 = time.perf_counter()
        r = conn.query_raw(sql)
        r.value(0, 0)
        r.close()
        wall = (time.perf_counter() - t0) * 1e6
        tm = conn.shard_timings()
        st = conn.shard_stats()
        rows["wake_max"].append(max(t["wake_us"] for t in tm))
        rows["launch_max"].append(max(t["launch_us"] for t in tm))
        rows["done_max"].append(max(t["done_us"] for t in tm))
        rows["done_min"].append(min(t["done_us"] for t in tm))
        rows["dispatch"].append(st["last_dispatch_us"])
        rows["merge"].append(st["last_combine_us"])
        rows["wall"].append(wall)
    return {k: round(statistics.median(v), 2) for k, v in rows.items()}


if __name__ == "__main__":
    main()
