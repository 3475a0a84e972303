"""C4 host-link breakdown on the GPU box: per-batch ingest time (append_column +
commit), and Arrow int64 read-back time per slice size with the getter alone
timed (query + getter separately).  Prints one line per measurement."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes
import importlib.util

_spec = importlib.util.spec_from_file_location(
    "duckdb_mbt_amd", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "duckdb.mbt_amd", "__init__.py"))
mbx = importlib.util.module_from_spec(_spec)
sys.modules["duckdb_mbt_amd"] = mbx
_spec.loader.exec_module(mbx)
lib = mbx.lib


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    batch = 10_000_000
    i = np.arange(n, dtype=np.uint64)
    v = ((i * np.uint64(2654435761)) & np.uint64(2**63 - 1)).astype(np.int64)
    cfg = mbx.Config.create()
    cfg.set("gpu_device", "0")
    conn = mbx.connect_with_config(cfg).value
    for rep in range(2):
        t = f"c4_{rep}"
        conn.query(f"CREATE TABLE {t} (v BIGINT)")
        ap = conn.create_appender("main", t).value
        per = []
        t0 = time.perf_counter()
        for s in range(0, n, batch):
            a = time.perf_counter()
            ap.append_column(0, v[s:s + batch])
            b = time.perf_counter()
            ap.commit(min(batch, n - s))
            c = time.perf_counter()
            per.append((round((b - a) * 1e3, 2), round((c - b) * 1e3, 2)))
        ap.close()
        tot = time.perf_counter() - t0
        print(f"ingest rep{rep}: {n * 8 / tot / 1e9:.1f} GB/s total {tot * 1e3:.1f} ms; (append, commit) ms per batch {per}",
              flush=True)
    grid = [{}]
    if os.environ.get("C4P_GRID"):
        grid = [{}, {"MBX_LINK_THREADS": "0"}, {"MBX_LINK_MIN": "1"}, {"MBX_LINK_MIN": "1", "MBX_LINK_HUGE": "0"},
                {"MBX_LINK_MIN": "1", "MBX_LINK_THREADS": "2"}, {}, {"MBX_LINK_THREADS": "0"}]
    for env in grid:
        for k in ("MBX_LINK_THREADS", "MBX_LINK_HUGE", "MBX_LINK_MIN"):
            os.environ.pop(k, None)
        os.environ.update(env)
        print(f"-- {env}", flush=True)
        readback(conn, v, n)


def readback(conn, v, n):
    for rows in (1_000_000, 4_000_000, 16_000_000, 32_000_000):
        tq = tg = 0.0
        ok = True
        for k in range(0, n, rows):
            a = time.perf_counter()
            ar = conn.query_arrow(f"SELECT v FROM c4_1 LIMIT {rows} OFFSET {k}").value
            b = time.perf_counter()
            bp = lib.duckdb_mb_arrow_get_column_int64(ar._h, 0)  # the C getter alone (no Python-side copy)
            c = time.perf_counter()
            tq += b - a
            tg += c - b
            m = min(rows, n - k)
            ln = lib.duckdb_mbx_bytes_len(bp)
            got = np.ctypeslib.as_array(ctypes.cast(bp, ctypes.POINTER(ctypes.c_uint8)), shape=(ln,))
            ok &= ln == 4 + 8 * m and np.array_equal(got[4:].view(np.int64), v[k:k + m])
            lib.duckdb_mbx_bytes_free(bp)
            ar.close()
        print(f"readback slice {rows}: query {tq * 1e3:.1f} ms, getter {tg * 1e3:.1f} ms = {n * 8 / tg / 1e9:.1f} GB/s "
              f"getter-only, {n * 8 / (tq + tg) / 1e9:.1f} GB/s with queries, exact={ok}", flush=True)


if __name__ == "__main__":
    main()
