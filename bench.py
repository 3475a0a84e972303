#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: rows/s of scan+filter over a 1e9-row
INT64 column per GPU (config C2: `SELECT COUNT(*) FROM t WHERE x > 24`,
x = splitmix64(42 + i) mod 50 + 1, selectivity 26/50), plus achieved HBM GB/s
of the fused filter-aggregate kernel against the MI355X HBM roofline.

One step = one `duckdb_mb_query` of that SQL through the C-ABI boundary
(parse -> bind -> fused gfx950 kernel over the device-resident column ->
8-byte D2H -> result cell), with the column already resident in HBM.

Multi-GPU (default): the product's own path.  One process opens devices
0..N-1 through the library's `gpu_devices` Config::set key (what a MoonBit
caller gets from duckdb_mb_query); the library shards the table by row range,
runs every shard's fused kernel on its own device and stream from a
persistent host worker, and combines the partial aggregates with RCCL on the
shard devices (a reduce to device 0 for COUNT, all-gather + carry-correct int128 combine
kernel for SUM; the library's default `mbx_combine`), or exactly on the host
where RCCL does not apply (same-device shards, GROUP BY).  The other combine
is timed right after the headline (`multi_device.combine_ab`).  Under the driver's `torch.distributed.run --nproc-per-node N`
launch, rank 0 drives all N devices and the other ranks only join the gloo
barriers.  `--ranks` keeps the one-process-per-GPU form (each rank its own
connection and 1e9-row shard, combined by an RCCL all-reduce / all-gather
inside the timed step).  Scaling is weak (fixed rows per GPU); value = total
rows / max-over-ranks time.  `--shards-per-gpu S` lists each device S times
(rehearses the multi-device combine on one GPU).

The 1-GPU C2 line also carries C3 and sel under "extra" (same clock
discipline, full-size parity) unless --extra says otherwise.

--config sel is the materialising form of C2's scan (`SELECT x FROM t WHERE
x > 24`): the passing rows compacted in row order into a device-resident
result (the reference's query_arrow path, rows counted through
duckdb_mb_arrow_row_count), checked row for row against the oracle.

--config c3n is C3 with 1/7 NULL keys and values; c3h the same GROUP BY over
--groups (1e5) dense INT64 keys (F3, partitioned in LDS); c3s over sparse keys
(F3h, hashed partitions).

Usage: python bench.py [--gpus N] [--shards-per-gpu S] [--ranks] [--steps K] [--warmup W]
                       [--rows R] [--config c1|c2|c2d|c3|c3n|c3h|c3s|c4|c5|sel] [--groups G]
                       [--extra c3,sel,c3n,c3h,c3s] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))

METRIC = "rows/sec scan+filter 1e9-row INT64 at 1/2/4/8 GPUs; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured float4 copy)


def load_mbx():
    import importlib.util
    spec = importlib.util.spec_from_file_location("duckdb_mbt_amd", os.path.join(HERE, "duckdb.mbt_amd", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules["duckdb_mbt_amd"] = m
    spec.loader.exec_module(m)
    return m


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def guard_stdout():
    """The contract's stdout carries the JSON line only.  Libraries in this
    process may write to file descriptor 1 themselves (RCCL prints its version
    banner when a communicator is created, e.g. by the in-library combine); so
    fd 1 is pointed at stderr, and Python's sys.stdout -- where the JSON line is
    printed -- keeps a private duplicate of the original stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    sys.stdout = out


def main():
    guard_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--shards-per-gpu", type=int, default=1,
                    help="in-library shards per device (gpu_devices lists each device this many times); "
                         "with --gpus 1 this rehearses the multi-device combine on one GPU")
    ap.add_argument("--ranks", action="store_true",
                    help="one process per GPU (torch.distributed) combining with RCCL instead of the "
                         "library's in-process gpu_devices sharding")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=None,
                    help="rows per GPU (default 1e9; 1.25e9 for c5 = 1e10 over 8 GPUs)")
    ap.add_argument("--config", default="c2",
                    choices=["c1", "c2", "c2d", "c3", "c3n", "c3h", "c3s", "c4", "c5", "sel"])
    ap.add_argument("--groups", type=int, default=100_000,
                    help="c3h: distinct INT64 keys of the hash GROUP BY (1e5 and 1e6 are the measured points)")
    ap.add_argument("--extra", default="auto",
                    help="comma-separated sub-benchmarks (c3, sel, c3n, c3h, c3s) reported under the headline "
                         "line's \"extra\" key; auto = all five for the 1-GPU C2 line, none otherwise")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rendezvous plumbing only (CPU, gloo): every rank joins, all-reduces its "
                         "rank id and rank 0 prints the JSON skeleton; no GPU is touched")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="--ranks only: nccl (= RCCL over xGMI) for real runs; gloo to rehearse N>1 on fewer GPUs")
    args = ap.parse_args()
    if args.rows is None:
        args.rows = 1_250_000_000 if args.config == "c5" else 1_000_000_000

    if args.ranks and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --ranks --gpus N` started bare: become the launcher of N ranks.
        # Nothing above has touched the GPU (no torch import yet), and the
        # ranks run as child processes (no exec), one per GPU.
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    if args.config in ("c1", "c4") and not args.dry_run:
        if rank == 0:
            return run_single_device_config(args)
        return None
    # N > 1 under a launcher: before anything touches a GPU, every rank counts
    # the devices it can see and a gloo all-gather of the counts decides the
    # form -- the in-library shards when rank 0 sees all N devices, else one
    # device per rank with an RCCL combine (no re-exec either way)
    form, vote = ("ranks" if args.ranks else "in-library"), None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        form, vote = vote_form(args, world, rank)
        if form is None:
            if rank == 0:
                log(f"[bench] {vote['reason']}")
            dist.destroy_process_group()
            raise SystemExit(2)
    if args.dry_run:
        return dry_run(args, world, rank, form, vote)
    if form == "ranks":
        return run_ranks(args, world, rank, local_rank, vote)
    return run_inlib(args, world, rank, vote)


def visible_devices(world):
    """GPUs this process can see, counted without initialising HIP:
    MBX_BENCH_VISIBLE_GPUS (tests simulate a launch's visibility with it), else
    torch.cuda.device_count() (it honours HIP/ROCR/CUDA_VISIBLE_DEVICES and does
    not initialise the GPU on this image).  A CPU dry run has nothing to count:
    it rehearses a full node (world devices)."""
    env = os.environ.get("MBX_BENCH_VISIBLE_GPUS")
    if env is not None:
        return int(env)
    import torch
    n = torch.cuda.device_count()
    return n if n > 0 else -world  # negative: no GPU (a CPU rehearsal)


def choose_form(counts, world, ranks_flag, dry_run=False):
    """The multi-GPU form from every rank's visible-device count: (form, reason);
    form None = no usable layout (a rank sees no GPU)."""
    c = [(-x if x < 0 and dry_run else x) for x in counts]
    if min(c) < 1:
        bad = [r for r, x in enumerate(c) if x < 1]
        return None, f"rank(s) {bad} see no GPU (visible-device counts {counts}): no usable layout"
    if ranks_flag:
        return "ranks", "--ranks asked for one process per GPU"
    if c[0] >= world:
        return "in-library", (f"rank 0 sees {c[0]} >= {world} devices: one process drives devices 0..{world - 1} "
                              f"through gpu_devices; the other ranks only join the barriers")
    return "ranks", (f"rank 0 sees {c[0]} < {world} devices (counts {c}): one device per rank, each rank its own "
                     f"connection and shard, global aggregate combined by RCCL")


def vote_form(args, world, rank):
    """gloo all-gather of every rank's visible-device count (no GPU touched) and
    the form all ranks then take: (form, vote dict)."""
    import torch
    import torch.distributed as dist
    mine = visible_devices(world)
    t = torch.tensor([mine], dtype=torch.int64)
    outs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, t)
    counts = [int(o.item()) for o in outs]
    form, reason = choose_form(counts, world, args.ranks, args.dry_run)
    return form, {"visible_devices_per_rank": counts, "min": min(counts), "max": max(counts), "form": form,
                  "reason": reason}


def dev_map(devs):
    """Device ids as the library sees them.  MBX_BENCH_DEVICE_MOD=k (a
    rehearsal of the N-GPU line on a box with k GPUs) maps device d to d mod k:
    the shards then share devices, so the combine is the host merge and the
    RCCL self-test reports the list it refuses -- every other part of the
    N > 1 line (timed loop, per-shard parity, combine A/B, the 1 -> N curve)
    runs as on a node with N GPUs."""
    k = int(os.environ.get("MBX_BENCH_DEVICE_MOD", "0") or 0)
    return [d % k for d in devs] if k > 0 else list(devs)


def inlib_plan(args, world):
    """The in-library layout: the devices (one process, `gpu_devices` through
    Config::set, ref duckdb_native.c:714-747), each listed --shards-per-gpu
    times; rows per GPU fixed (weak scaling)."""
    ngpu = world if world > 1 else args.gpus
    spg = max(1, args.shards_per_gpu)
    devices = dev_map([d for d in range(ngpu) for _ in range(spg)])
    nshards = len(devices)
    par = (f"in-library row-range shards: gpu_devices={','.join(map(str, devices))} "
           f"({ngpu} GPU x {spg} shard(s), one engine + stream + persistent host worker per shard), "
           f"per-shard partial aggregates combined by the library's default: an RCCL reduce to device 0 (COUNT) / "
           f"all-gather + int128 combine kernel (SUM) over the shard devices when they are distinct, else an exact "
           f"host merge") if nshards > 1 \
        else "row-range shards x1"
    return {"ngpu": ngpu, "shards_per_gpu": spg, "devices": devices, "nshards": nshards,
            "rows_total": args.rows * ngpu, "parallelism": par}


# c3n: C3 with NULLs -- 1/7 of the keys and 1/7 of the values NULL (the
# generator of tests/test_gpu_group_nulls.py and oracle.c orc_synth_groupby_nulls)
C3N_SEEDS = [7, 19, 9, 23, 31, 29]
C3N_MODS = [32, 7, 1 << 40, 7, 1 << 40, 0]
C3N_ADDS = [-(1 << 39), -(1 << 39)]
C3S_MULT = 2654435761


def workload(config, start, n, groups=100_000):
    """SQL and accounting of one bench config over rows [start, start + n)."""
    w = {"c2like": config in ("c2", "c2d")}
    if config == "c3n":
        w["table"] = "t3n"
        w["setup"] = (f"CREATE TABLE t3n AS SELECT CASE WHEN mbx_synth(19, i, 7) = 0 THEN NULL "
                      f"ELSE CAST(mbx_synth(7, i, 32) AS INTEGER) END AS k, "
                      f"CASE WHEN mbx_synth(23, i, 7) = 0 THEN NULL ELSE mbx_synth(9, i, 1099511627776) - 549755813888 "
                      f"END AS v FROM range({start}, {start + n}) tbl(i)")
        w["sql"] = "SELECT k, SUM(v), COUNT(*) FROM t3n GROUP BY k"
        w["kernel"] = "group_direct"
        w["pmc_keys"] = ["group_direct_nulls"]
        w["bytes_per_row"] = 12.25  # 4 B key + 8 B value + the two columns' validity bits
        w["workload"] = ("C3 with NULLs: SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k over 1e9 rows (INT32 key, 32 "
                         "groups + the NULL group; 1/7 of keys and 1/7 of values NULL)")
        w["data"] = ("synthetic: k = splitmix64(7 + i) mod 32 (INT32, NULL where splitmix64(19 + i) mod 7 = 0), "
                     "v = splitmix64(9 + i) mod 2^40 - 2^39 (INT64, NULL where splitmix64(23 + i) mod 7 = 0), "
                     "generated on device (no dataset)")
        return w
    if config == "c3s":
        # the same GROUP BY over sparse keys (g x 2654435761): hashed partitions (F3h)
        w["table"] = "ts"
        w["setup"] = (f"CREATE TABLE ts AS SELECT mbx_synth(7, i, {groups}) * {C3S_MULT} AS k, "
                      f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({start}, {start + n}) tbl(i)")
        w["sql"] = "SELECT k, SUM(v), COUNT(*) FROM ts GROUP BY k"
        w["kernel"] = "*"
        w["pmc_keys"] = ["pg_hist_hashed", "pg_hscatter", "pg_hreduce"]
        w["bytes_per_row"] = 16
        w["workload"] = (f"sparse-key GROUP BY: SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k over 1e9 rows "
                         f"({groups} distinct INT64 keys spread over 2.6e14, INT64 value)")
        w["data"] = (f"synthetic: k = (splitmix64(7 + i) mod {groups}) x {C3S_MULT} (INT64), "
                     f"v = splitmix64(9 + i) mod 2^40 - 2^39 (INT64), generated on device (no dataset)")
        return w
    if config == "c3h":
        w["table"] = "th"
        w["setup"] = (f"CREATE TABLE th AS SELECT mbx_synth(7, i, {groups}) AS k, "
                      f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({start}, {start + n}) tbl(i)")
        w["sql"] = "SELECT k, SUM(v), COUNT(*) FROM th GROUP BY k"
        w["kernel"] = "*"  # every kernel of the statement: the partitioned GROUP BY is a pipeline
        w["pmc_keys"] = ["pg_hist", "pg_scatter", "pg_reduce"]
        w["bytes_per_row"] = 16
        w["workload"] = (f"hash GROUP BY: SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k over 1e9 rows "
                         f"({groups} distinct INT64 keys, INT64 value)")
        w["data"] = (f"synthetic: k = splitmix64(7 + i) mod {groups} (INT64), v = splitmix64(9 + i) mod 2^40 - 2^39 "
                     f"(INT64), generated on device (no dataset)")
        return w
    if config in ("c2", "c2d", "c5", "sel"):
        # c2d: C2 over DECIMAL(15,2) (raw = 100 x; x > 24 is raw > 2400)
        xexpr = "CAST(mbx_synth(42, i, 50) + 1 AS DECIMAL(15,2))" if config == "c2d" else "mbx_synth(42, i, 50) + 1"
        w["table"] = "t"
        w["setup"] = f"CREATE TABLE t AS SELECT {xexpr} AS x FROM range({start}, {start + n}) tbl(i)"
        w["sql"] = {"c5": "SELECT COUNT(*), SUM(x) FROM t WHERE x > 24",
                    "sel": "SELECT x FROM t WHERE x > 24"}.get(config, "SELECT COUNT(*) FROM t WHERE x > 24")
        w["kernel"] = "select_rounds" if config == "sel" else "filter_agg"
        w["bytes_per_row"] = 8
        w["workload"] = {
            "c2": "C2: SELECT COUNT(*) FROM t WHERE x > 24 over a device-resident 1e9-row INT64 column per GPU",
            "sel": "C2 materialised (sel): SELECT x FROM t WHERE x > 24, the passing rows compacted in row order "
                   "into a device-resident result (query_arrow + arrow_row_count), 1e9 INT64 rows per GPU",
            "c2d": "C2 DECIMAL(15,2) variant: SELECT COUNT(*) FROM t WHERE x > 24 (raw int64 > 2400) per GPU",
            "c5": "C5: SELECT COUNT(*), SUM(x) FROM t WHERE x > 24, rows sharded per GPU"}[config]
        w["data"] = ("synthetic: x = splitmix64(42 + i) mod 50 + 1 generated on device (no dataset)"
                     + (", stored as DECIMAL(15,2) (int64 raw = 100 x)" if config == "c2d" else ""))
    else:
        w["table"] = "t3"
        w["setup"] = (f"CREATE TABLE t3 AS SELECT CAST(mbx_synth(7, i, 32) AS INTEGER) AS k, "
                      f"mbx_synth(9, i, 1099511627776) - 549755813888 AS v FROM range({start}, {start + n}) tbl(i)")
        w["sql"] = "SELECT k, SUM(v), COUNT(*) FROM t3 GROUP BY k"
        w["kernel"] = "group_direct"
        w["bytes_per_row"] = 12
        w["workload"] = ("C3: SELECT k, SUM(v), COUNT(*) FROM t GROUP BY k over 1e9 rows (INT32 key, 32 groups; "
                         "INT64 value)")
        w["data"] = ("synthetic: k = splitmix64(7 + i) mod 32 (INT32), v = splitmix64(9 + i) mod 2^40 - 2^39 "
                     "(INT64), generated on device (no dataset)")
    return w


def decode_c3(out):
    """C3 result cells (strings, NULL flags) -> (key or None, COUNT, SUM) ints."""
    if not (isinstance(out, tuple) and len(out) == 3 and out[0] == "c3cells"):
        return out
    _, rows, nulls = out
    return [(None if nl[0] else int(rw[0]), int(rw[2]), None if nl[1] else int(rw[1])) for rw, nl in zip(rows, nulls)]


def make_step(conn, config, sql, decode=True):
    """One step: one duckdb_mb_query of `sql` through the C-ABI and its result
    cells as text, as Connection::query pulls them (C3: every cell's text in
    one duckdb_mbx_result_text call rather than 2 ctypes calls per cell; sel:
    query_arrow, the result left in HBM).  decode=False leaves C3's cells as
    text for decode_c3 after the timed loop (the ranks form decodes inside it:
    its RCCL combine needs the integers)."""
    def step():
        if config == "sel":
            a = conn.query_arrow(sql).value  # the result stays in HBM until a getter pulls it
            rows = a.row_count()
            a.close()
            return [rows]
        rr = conn.query_raw(sql)
        if config in ("c3h", "c3s") and not decode:
            # 1e5+ groups: the step ends at the materialised result (the
            # library's D2H and cell text); the cells are pulled once after
            # the timed loop for parity (a Python list of 3e5 strings per
            # step would time the interpreter, not the query)
            rows = rr.row_count()
            rr.close()
            return ("c3hrows", rows)
        if config in ("c3", "c3n", "c3h", "c3s"):
            rows, nulls = rr.cells()
            cells = ("c3cells", rows, nulls)
            if decode:
                cells = decode_c3(cells)
        else:
            cells = [rr.value(c, 0) for c in range(rr.column_count())]
        rr.close()
        return cells
    return step


def parity_check(conn, config, sql, out, start, n, threads, groups=100_000):
    """The GPU answer over rows [start, start + n) against the CPU oracle at full
    size (test infrastructure: checker only, outside the timed loop)."""
    sys.path.insert(0, HERE)
    from oracle import Oracle
    orc = Oracle()
    if config in ("c2", "c2d", "c5"):
        oc, osum = orc.synth_filter_count(42, start, n, 50, 1, 25, 2**63 - 1, threads)
        par = {"gpu_count": int(out[0]), "oracle_count": oc, "match": int(out[0]) == oc}
        if config == "c5":
            par.update({"gpu_sum": int(out[1]), "oracle_sum": osum, "match": par["match"] and int(out[1]) == osum})
        return par, (oc, osum)
    if config == "c3":
        oc, osum = orc.synth_groupby(7, 9, start, n, 32, 1 << 40, -(1 << 39), threads)
        exp = [(k, oc[k], osum[k]) for k in range(32) if oc[k]]
        got = sorted(out, key=lambda g: (g[0] is None, g[0]))
        return {"groups": len(got), "oracle_groups": len(exp), "match": got == exp,
                "checked": "every group's COUNT and exact int128 SUM over all rows"}, exp
    if config == "c3n":
        g = orc.synth_groupby_nulls(C3N_SEEDS, C3N_MODS, C3N_ADDS, start, n, threads)
        exp = [(e[0], e[1], e[3]) for e in g]  # (key or None, COUNT(*), SUM(v) or None)
        got = sorted(out, key=lambda x: (x[0] is None, x[0] if x[0] is not None else 0))
        return {"groups": len(got), "oracle_groups": len(exp), "match": got == exp,
                "checked": "every group's COUNT(*) and exact int128 SUM over the valid values, the NULL key's "
                           "group included, over all rows (oracle.c orc_synth_groupby_nulls)"}, exp
    if config in ("c3h", "c3s"):
        mult = C3S_MULT if config == "c3s" else 1
        oc, osum = orc.synth_groupby(7, 9, start, n, groups, 1 << 40, -(1 << 39), min(threads, 32))
        exp = [(k * mult, oc[k], osum[k]) for k in range(groups) if oc[k]]
        got = sorted(out, key=lambda g: (g[0] is None, g[0]))
        return {"groups": len(got), "oracle_groups": len(exp), "match": got == exp,
                "checked": f"every one of the {len(exp)} groups' COUNT and exact int128 SUM over all rows"}, exp
    # sel: the full compacted column (one more query, pulled through the int64
    # Arrow getter in slices) against the oracle's order-preserving selection
    import numpy as np
    x = orc.synth_i64(n, 42, start, 50, 1)
    exp = orc.select_i64(x, 25, 2**63 - 1, threads)
    del x
    sel_rows = int(out[0])
    ok = sel_rows == len(exp)
    sl = 25_000_000  # an Arrow Bytes holds < 2^28 bytes (MoonBit header): read the result in slices
    for k in range(0, sel_rows, sl):
        a = conn.query_arrow(f"{sql} LIMIT {sl} OFFSET {k}").value
        raw = a.raw_int64_bytes(0)
        a.close()
        cnt = int.from_bytes(raw[:4], "little", signed=True) if len(raw) >= 4 else -1
        ok = ok and cnt == min(sl, sel_rows - k) and \
            bool(np.array_equal(np.frombuffer(raw, dtype=np.int64, offset=4, count=cnt), exp[k:k + cnt]))
    par = {"gpu_rows": sel_rows, "oracle_rows": int(len(exp)), "match": bool(ok),
           "checked": "every output value at its position (Arrow int64 getter, 25M-row LIMIT/OFFSET "
                      "slices) vs the oracle's select_i64 over the same generator"}
    return par, None


def csrc_digest():
    """sha256 over the library's sources (duckdb.mbt_amd/csrc/*.{hip,cpp,h},
    names and contents, sorted): which build a stored PMC measurement
    describes.  tools/pmc_traffic.py stamps its entries with it."""
    import hashlib
    d = os.path.join(HERE, "duckdb.mbt_amd", "csrc")
    h = hashlib.sha256()
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".cpp", ".h")):
            h.update(name.encode() + b"\0")
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
            h.update(b"\0")
    return h.hexdigest()


def pmc_traffic_entry(kernel, n):
    """(HBM bytes per launch from the stored PMC passes, their provenance):
    the bytes only while the stored entry was measured at this row count AND
    on sources that hash to this build's csrc_digest(), else None."""
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    src = {"file": "profiles/pmc_traffic.json", "entry": kernel}
    try:
        table = json.load(open(pmc))
    except Exception as ex:  # noqa: BLE001
        src["why_null"] = f"unreadable: {ex}"
        return None, src
    # a row count other than the default 1e9 has its own entry ("<kernel>@<rows>", e.g. C5's shard)
    if n != 1_000_000_000 and f"{kernel}@{n}" in table:
        kernel = f"{kernel}@{n}"
        src["entry"] = kernel
    ent = table.get(kernel)
    if not ent:
        src["why_null"] = "no entry for this kernel"
        return None, src
    src.update({"git_head": ent.get("git_head"), "date": ent.get("date"), "csrc_sha256": ent.get("csrc_sha256"),
                "counters": "FETCH_SIZE x1024 x2 + WRITE_SIZE x1024, separate rocprofv3 --pmc passes"})
    here = csrc_digest()
    src["this_build_csrc_sha256"] = here
    if ent.get("csrc_sha256") != here:
        src["why_null"] = "measured on other sources than this build's (csrc digest differs)"
        return None, src
    if n != ent.get("rows", 1_000_000_000):  # the PMC passes run at the default 1e9-row size
        src["why_null"] = f"measured at {ent.get('rows', 1_000_000_000)} rows per launch, not {n}"
        return None, src
    return ent.get("hbm_bytes_per_launch"), src


def pmc_traffic(kernel, n):
    return pmc_traffic_entry(kernel, n)[0]


def pmc_traffic_keys(keys, n):
    """The traffic of a statement whose work is several kernels (c3h's three
    passes): the sum of their stored per-launch bytes, or None if any is
    missing or stale; the provenance of each."""
    tot, srcs = 0.0, []
    for k in keys:
        b, src = pmc_traffic_entry(k, n)
        srcs.append(src)
        tot = None if (tot is None or b is None) else tot + b
    return tot, (srcs[0] if len(srcs) == 1 else {"entries": srcs})


def time_steps(step, steps, warmup, barrier=None, sync=None):
    """W untimed warmup steps, then EXACTLY K steps bracketed by the barrier and
    a device synchronisation on both sides; returns (elapsed s, last output)."""
    out = None
    for _ in range(warmup):
        out = step()
    if barrier:
        barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    if barrier:
        barrier()
    if sync:
        sync()
    return time.perf_counter() - t0, out


def kernel_stats(kern, kernel, nshards, steps):
    """HIP-event durations of `kernel` over the timed loop (shard engines'
    launches included; `kern` = the drained profile, or a connection to drain):
    mean per launch and, per step, the slowest shard."""
    if not isinstance(kern, list):
        kern = kern.profile_drain()
    if kernel == "*":  # a multi-kernel pipeline: every kernel of the statement, per step
        ks = [k["ms"] for k in kern]
        per = sum(ks) / steps if steps and ks else None
        return per, per, ks
    ks = [k["ms"] for k in kern if k["name"] == kernel]
    if not ks:
        return None, None, []
    per_step = [max(ks[i:i + nshards]) for i in range(0, len(ks) - nshards + 1, nshards)][:steps]
    return sum(ks) / len(ks), (sum(per_step) / len(per_step) if per_step else None), ks


def run_inlib(args, world, rank, vote=None):
    """The product's multi-GPU path: ONE process opens every device through the
    library's own `gpu_devices` key and runs the query through duckdb_mb_query;
    the library shards the table, runs every shard on its own device/stream
    from a persistent host worker, and merges the partials.  Under the
    driver's torch.distributed launch (one process per GPU, gloo world group
    set up by the vote) rank 0 drives all devices and the other ranks only
    join the barriers."""
    plan = inlib_plan(args, world)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rank != 0:
            dist.barrier()  # rank 0's timed region starts
            dist.barrier()  # ... and ends
            import torch
            t_all = torch.tensor([0.0], dtype=torch.float64)
            dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
            dist.barrier()
            dist.destroy_process_group()
            return None
    import torch
    mbx = load_mbx()
    selftest = None
    if plan["ngpu"] > 1:
        # the RCCL calls of the combine over every GPU of the run, before any
        # table exists: a fresh ncclCommInitAll over devices 0..N-1 and the
        # multi-rank reduce / all-gather check, with what RCCL reports per rank
        selftest = guarded(lambda: mbx.rccl_selftest(dev_map(range(plan["ngpu"]))), RCCL_LEG_TIMEOUT_S)
        log(f"[bench] rccl self-test over devices 0..{plan['ngpu'] - 1}: {json.dumps(selftest)}")
    cfg = mbx.Config.create()
    if plan["nshards"] > 1:
        cfg.set("gpu_devices", ",".join(map(str, plan["devices"])))
    else:
        cfg.set("gpu_device", "0")
    cfg.set("mbx_profile", "true")
    r = mbx.connect_with_config(cfg)
    if isinstance(r, mbx.Err):
        fail(dist, f"connect over gpu_devices={plan['devices']} failed: {r.error.message}")
    conn = r.value
    n_total = plan["rows_total"]
    w = workload(args.config, 0, n_total, args.groups)
    t0 = time.time()
    res = conn.query(w["setup"])
    if isinstance(res, mbx.Err):
        fail(dist, f"setup failed: {res.error.message}")
    log(f"[rank {rank}] setup {time.time() - t0:.2f}s: {n_total} rows over {plan['nshards']} shard(s)")
    step = make_step(conn, args.config, w["sql"], decode=False)
    try:
        for _ in range(args.warmup):
            step()
        conn.profile_drain()
        barrier = dist.barrier if dist else None
        sr0 = conn.engine_stats()
        cb0 = conn.rccl_stats()
        elapsed, out = time_steps(step, args.steps, 0, barrier,
                                  torch.cuda.synchronize if torch.cuda.is_available() else None)
        kern_timed = None
        log(f"[bench] timed loop done: {elapsed / args.steps * 1e3:.3f} ms/step")
        if isinstance(out, tuple) and out[0] == "c3hrows":  # the cells of the same query, pulled once
            kern_timed = conn.profile_drain()
            out = make_step(conn, args.config, w["sql"], decode=True)()
            conn.profile_drain()
            log(f"[bench] c3h: {len(out)} groups pulled for parity")
        out = decode_c3(out)
        sr_out = sel_outcomes(conn, sr0)
        cb1 = conn.rccl_stats()
        cb_out = combine_delta(cb0, cb1)
    except Exception as ex:  # noqa: BLE001 - a shard's error names the shard and its device
        fail(dist, f"query failed: {ex}")
    kern = conn.profile_drain() if kern_timed is None else kern_timed
    avg_k, step_k, _ = kernel_stats(kern, w["kernel"], plan["nshards"], args.steps)
    split = kernel_split(kern, args.steps)
    sstats = conn.shard_stats() if plan["nshards"] > 1 else None
    if dist:
        t_all = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)
        elapsed = float(t_all.item())
    threads = len(os.sched_getaffinity(0))
    shard_par = None
    log("[bench] parity check against the oracle")
    if sstats and args.config in ("c2", "c2d", "c5", "c3"):
        parity, shard_par = sharded_parity(conn, args.config, out, n_total, plan["nshards"], threads)
    else:
        parity, _ = parity_check(conn, args.config, w["sql"], out, 0, n_total, threads, args.groups)
    if sstats:
        parity["checked"] = (f"the global answer over all {n_total} rows ({plan['nshards']} shards, merged in the "
                             f"library) vs the oracle over the same rows"
                             + ("; every shard's partial vs the oracle over its own row range" if shard_par else ""))
    result = headline(args, w, plan["ngpu"], elapsed, avg_k, n_total, args.rows // plan["shards_per_gpu"],
                      plan["parallelism"], parity,
                      sel_rows=int(out[0]) if args.config == "sel" else None)
    if vote:
        result["config"]["form"] = vote
    if args.config in ("c3h", "c3n", "c3s"):
        # the statement's kernels, ms per step (HIP events per profiled scope)
        result["kernel_split_ms_per_step"] = split
    stuck = False
    if sstats:
        ms = elapsed / args.steps * 1e3
        md = {
            "path": "in-library (gpu_devices)", "shards": plan["nshards"], "devices": plan["devices"],
            "rows_per_shard": n_total // plan["nshards"],
            "kernel_ms_per_launch_avg": avg_k, "slowest_shard_kernel_ms_per_step": step_k,
            "kernel_ms_per_shard": per_shard_kernel_ms(kern, w["kernel"], plan["nshards"]),
            "combine_overhead_ms_per_step": (ms - step_k) if step_k else None,
            "peer_links": sstats["peer_links"], "host_results": sstats["host_results"],
            "note": ("shards on one device run concurrently, so per-launch times overlap"
                     if plan["shards_per_gpu"] > 1 else "one shard per device")}
        md["split_us"] = overhead_split(conn, step, 10)
        if shard_par is not None:
            md["shard_parity"] = [{k: v for k, v in e.items() if k != "oracle"} for e in shard_par]
        # the timed loop ran the library's default combine (RCCL over the shard
        # devices when they are distinct): which collective every step ran, and
        # the communicators as RCCL reports them (rank count and rank of each)
        md["combine"] = {"timed_loop": cb_out, "mode": "rccl" if cb_out["ran_rccl_steps"] else "host merge",
                         "rccl": rccl_evidence(conn.rccl_info(), plan["devices"])}
        if selftest is not None:
            md["rccl_selftest"] = selftest
        if args.config in ("c2", "c2d", "c5", "c3"):
            # the other mode, timed right after
            md["combine_ab"] = guarded(
                lambda: combine_leg(conn, step, args, n_total, "host" if cb_out["ran_rccl_steps"] else "rccl"),
                RCCL_LEG_TIMEOUT_S)
            stuck = md["combine_ab"].get("error", "").startswith("timeout")
        if not stuck and plan["ngpu"] > 1 and args.config in ("c2", "c2d", "c5", "c3") and shard_par is not None:
            # the 1 -> N curve from this one run: the same query over device
            # prefixes 1, 2, 4 ... of 0..N-1, each its own connection and table
            md["curve"] = guarded(lambda: curve_legs(mbx, args, plan, result, shard_par), CURVE_TIMEOUT_S)
        result["multi_device"] = md
    calibrate_into(conn, result, args.config)
    if args.config == "sel":
        # every timed step must have run the one-pass kernel (per shard): a fallback fails parity loudly
        result["select_rounds"] = sr_out
        result["fallbacks"] = sr_out["fallbacks"]
        if sr_out["fallbacks"] or sr_out["select_rounds_launches"] < args.steps * plan["nshards"]:
            result["parity"]["match"] = False
            result["parity"]["fallback_error"] = f"select_rounds outcomes in the timed loop: {sr_out}"
    extras = args.extra
    if extras == "auto":
        extras = "c3,sel,c3n,c3h,c3s" if (args.config == "c2" and plan["nshards"] == 1) else ""
    if extras:
        result["extra"] = {}
        ceil = result["roofline"].get("measured_ceilings_gbs", {})
        for ex in [e for e in extras.split(",") if e]:
            r = result["extra"][ex] = sub_bench(conn, ex, plan, args)
            # against this box's ceiling of the same shape: C3's two-array ring read
            # (4 + 8 B per row, 2-deep 3 KiB slots); sel's half-writing ring copy
            shape = {"c3": "ring_read2_gbs", "c3n": "ring_read2_gbs", "sel": "ring_copy_half_gbs"}.get(ex)
            if shape and isinstance(ceil.get(shape), float) and r.get("achieved_gbs"):
                r["measured_ceiling_gbs"] = ceil[shape]
                r["ceiling_shape"] = shape
                r["frac_of_measured"] = r["achieved_gbs"] / ceil[shape]
    if plan["nshards"] == 1 and args.config == "c2" and extras:
        # the RCCL calls of the in-library combine, on this one-GPU box: a one-rank
        # communicator, a grouped reduce and all-gather (outside the timed loop)
        try:
            result["extra"]["rccl_selftest"] = mbx.rccl_selftest([0])
        except Exception as ex:  # noqa: BLE001
            result["extra"]["rccl_selftest"] = {"ok": False, "error": str(ex)}
    log("[bench] parity done")
    if not args.no_cpu and plan["nshards"] == 1 and args.config in ("c2", "c2d", "c3", "c3n", "c3h", "c3s", "c5", "sel"):
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds,
                                              {"c2d": "c2", "c3n": "c3", "c3s": "c3h"}.get(args.config, args.config),
                                              args.groups)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if not stuck:
        conn.close()
    print(json.dumps(result), flush=True)
    bad = not result["parity"].get("match", True) or (shard_par and not all(p["match"] for p in shard_par))
    if bad:
        log("[bench] PARITY FAILURE: " + json.dumps(result["parity"]) +
            (" shards: " + json.dumps([p for p in shard_par if not p["match"]]) if shard_par else ""))
    if stuck:
        # the second leg's thread is still inside the library: the headline line
        # is out, so leave without joining it (interpreter teardown would wait)
        # a hung leg is a failed run even when the headline's parity matched
        log("[bench] the second combine leg did not finish; exiting (status 4) without closing the connection")
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3 if bad else 4)
    if bad:
        raise SystemExit(3)
    return result


RCCL_LEG_TIMEOUT_S = float(os.environ.get("MBX_BENCH_RCCL_TIMEOUT_S", "120"))
CURVE_TIMEOUT_S = float(os.environ.get("MBX_BENCH_CURVE_TIMEOUT_S", "300"))


ZERO_RCCL_STATS = {"rccl_combines": 0, "rccl_reduces": 0, "rccl_allgathers": 0, "rccl_fallbacks": 0,
                   "rccl_unsupported": 0, "rccl_timeouts": 0, "last_rccl_us": 0.0, "note": ""}


def combine_delta(cb0, cb1):
    """What the combine did between two rccl_stats() snapshots: steps RCCL
    combined (and with which collective), steps that fell back to the host
    merge (RCCL should have run) and steps whose shape RCCL never covers."""
    d = lambda k: cb1[k] - cb0[k]  # noqa: E731
    return {"ran_rccl_steps": d("rccl_combines"), "ncclReduce_steps": d("rccl_reduces"),
            "ncclAllGather_steps": d("rccl_allgathers"), "host_merge_steps": d("rccl_fallbacks") + d("rccl_unsupported"),
            "fallback_steps": d("rccl_fallbacks"), "unsupported_steps": d("rccl_unsupported"),
            "note": cb1["note"], "rccl_timeouts": cb1["rccl_timeouts"],
            "last_collective_d2h_us": cb1["last_rccl_us"]}


def rccl_evidence(info, devices):
    """The connection's communicators as RCCL reports them (duckdb_mbx_rccl_info)
    and whether they prove an N-rank RCCL: every rank's ncclCommCount equal to
    the number of distinct shard devices and its ncclCommUserRank its index."""
    ranks = info.get("ranks") or []
    n = len(devices)
    info = dict(info)
    info["saw_nranks"] = sorted({r["count"] for r in ranks}) if ranks else []
    info["proves_n_ranks"] = (len(ranks) == n and len(set(devices)) == n and
                              all(r["count"] == n and r["user_rank"] == i for i, r in enumerate(ranks)))
    return info


def curve_legs(mbx, args, plan, result, shard_par):
    """The 1 -> N scaling points from one N-GPU process: for every power-of-two
    prefix p < N of devices 0..N-1 (each listed --shards-per-gpu times), its
    own connection and a table of p x rows-per-GPU rows (the same rows as the
    headline's first p x S shards), warmup, K timed steps, the kernel's HIP
    events, and parity: the global answer and every shard's partial against
    the oracle values the headline's shard parity already computed over those
    same row ranges.  The headline's own N point closes the curve."""
    import torch
    curve = []
    for p, devices in curve_points(plan["ngpu"], plan["shards_per_gpu"]):
        nsh = len(devices)
        n = args.rows * p
        cfg = mbx.Config.create()
        if nsh > 1:
            cfg.set("gpu_devices", ",".join(map(str, devices)))
        else:
            cfg.set("gpu_device", "0")
        cfg.set("mbx_profile", "true")
        r = mbx.connect_with_config(cfg)
        if isinstance(r, mbx.Err):
            curve.append({"gpus": p, "error": r.error.message})
            continue
        conn = r.value
        try:
            w = workload(args.config, 0, n)
            res = conn.query(w["setup"])
            if isinstance(res, mbx.Err):
                raise RuntimeError(res.error.message)
            step = make_step(conn, args.config, w["sql"], decode=False)
            for _ in range(args.warmup):
                step()
            conn.profile_drain()
            cb0 = conn.rccl_stats()
            elapsed, out = time_steps(step, args.steps, 0, None, torch.cuda.synchronize)
            out = decode_c3(out)
            cb1 = conn.rccl_stats()
            avg_k, step_k, _ = kernel_stats(conn, w["kernel"], nsh, args.steps)
            exp = shard_par[:nsh]
            if args.config == "c3":
                groups = {}
                for e in exp:
                    for k, c_, s_ in e["oracle"]:
                        gc, gs = groups.get(k, (0, 0))
                        groups[k] = (gc + c_, gs + s_)
                want = [(k, groups[k][0], groups[k][1]) for k in sorted(groups)]
                got = sorted(out, key=lambda g: (g[0] is None, g[0]))
                par = {"groups": len(got), "oracle_groups": len(want), "match": got == want}
            else:
                oc = sum(e["oracle_count"] for e in exp)
                par = {"gpu_count": int(out[0]), "oracle_count": oc, "match": int(out[0]) == oc}
                if args.config == "c5":
                    osum = sum(e["oracle_sum"] for e in exp)
                    par.update({"gpu_sum": int(out[1]), "oracle_sum": osum,
                                "match": par["match"] and int(out[1]) == osum})
            if nsh > 1:
                sp = shard_partials_vs(conn, args.config, exp)
                par["shards_match"] = all(x["match"] for x in sp)
                par["match"] = par["match"] and par["shards_match"]
            pt = {"gpus": p, "shards": nsh, "devices": devices, "rows": n, "ms_per_step": elapsed / args.steps * 1e3,
                  "value": n * args.steps / elapsed, "unit": "rows/s", "kernel_ms_avg": avg_k,
                  "slowest_shard_kernel_ms_per_step": step_k, "parity": par,
                  "combine": combine_delta(cb0, cb1)}
            if nsh > 1:
                pt["rccl"] = rccl_evidence(conn.rccl_info(), devices)
            curve.append(pt)
        except Exception as ex:  # noqa: BLE001 - one point must not lose the others
            curve.append({"gpus": p, "error": str(ex)})
        finally:
            conn.close()
    curve.append({"gpus": plan["ngpu"], "shards": plan["nshards"], "devices": plan["devices"],
                  "rows": plan["rows_total"], "ms_per_step": result["ms_per_step"], "value": result["value"],
                  "unit": "rows/s", "kernel_ms_avg": result["roofline"]["kernel_ms_avg"],
                  "parity": {"match": result["parity"].get("match")}, "the_headline": True})
    base = next((c["value"] for c in curve if c.get("gpus") == 1 and c.get("value")), None)
    for c in curve:
        if base and c.get("value"):
            c["speedup_vs_1"] = c["value"] / base
    return {"points": curve, "scaling": "weak (rows per GPU fixed)",
            "definition": "one process; each point its own connection over devices 0..p-1 and table of p x rows "
                          "per GPU, the same clock discipline as the headline (warmup, K timed steps, "
                          "synchronised); parity against the headline's per-shard oracle values"}


def curve_points(ngpu, spg):
    """The curve's prefixes below the headline's N: (p, gpu_devices list) for
    p = 1, 2, 4, ... < N, each device listed spg times."""
    pts, p = [], 1
    while p < ngpu:
        pts.append((p, dev_map([d for d in range(p) for _ in range(spg)])))
        p *= 2
    return pts


def shard_partials_vs(conn, config, exp):
    """Every shard's partial (duckdb_mbx_shard_partial) of the last sharded
    aggregate against its oracle entry (sharded_parity's)."""
    outp = []
    for i, e in enumerate(exp):
        rr = conn.shard_partial(i)
        if rr is None:
            outp.append({"shard": i, "match": False, "error": "no partial"})
            continue
        if config == "c3":
            rows, nulls = rr.cells()
            got = sorted((None if nl[0] else int(rw[0]), int(rw[2]), None if nl[1] else int(rw[1]))
                         for rw, nl in zip(rows, nulls))
            ok = got == e["oracle"]
        else:
            ok = int(rr.value(0, 0)) == e["oracle_count"]
            if config == "c5":
                ok = ok and int(rr.value(1, 0)) == e["oracle_sum"]
        rr.close()
        outp.append({"shard": i, "match": ok})
    return outp


def guarded(fn, timeout_s):
    """fn() on a daemon thread, given timeout_s seconds: its dict, an {"error"}
    dict if it raised, or {"error": "timeout ..."} if it is still running (a
    collective that never completes must not cost the headline line)."""
    import threading
    box = {}

    def run():
        try:
            box["r"] = fn()
        except Exception as ex:  # noqa: BLE001
            box["r"] = {"error": str(ex)}
    th = threading.Thread(target=run, daemon=True)
    th.start()
    th.join(timeout_s)
    if th.is_alive():
        return {"error": f"timeout: the leg did not finish within {timeout_s:.0f} s"}
    return box["r"]


def fail(dist, msg):
    """A failure before the JSON line: the message (naming the shard and device
    when a shard raised it) on stderr, every rank released, exit status 2."""
    log(f"[bench] FAILED: {msg}")
    if dist is not None:
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
    raise SystemExit(2)


def kernel_split(kern, steps):
    """ms per step of every profiled kernel scope of the timed loop, by name."""
    acc = {}
    for k in kern:
        acc[k["name"]] = acc.get(k["name"], 0.0) + k["ms"]
    return {n: v / steps for n, v in sorted(acc.items(), key=lambda t: -t[1])} if steps else {}


def per_shard_kernel_ms(kern, kernel, nshards):
    """Mean HIP-event duration of `kernel` per shard (from the profile's shard tags)."""
    acc = {}
    for k in kern:
        if k["name"] == kernel and k.get("shard", -1) >= 0:
            acc.setdefault(k["shard"], []).append(k["ms"])
    return [{"shard": i, "device": next((k["device"] for k in kern if k.get("shard") == i), None),
             "kernel_ms_avg": (sum(acc[i]) / len(acc[i])) if i in acc else None, "launches": len(acc.get(i, []))}
            for i in range(nshards)]


def overhead_split(conn, step, reps):
    """Where a sharded step's host time goes, from `reps` untimed steps after the
    timed loop (medians): until every worker took the job (dispatch), until its
    launches were queued, its kernel + D2H + synchronisation, and the merge."""
    import statistics
    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        wall = (time.perf_counter() - t0) * 1e6
        st = conn.shard_stats()
        tm = conn.shard_timings()
        if not tm:
            continue
        rows.append({"wall": wall, "dispatch": max(t["wake_us"] for t in tm),
                     "launch": max(t["launch_us"] - t["wake_us"] for t in tm),
                     "kernel_d2h": max(t["done_us"] - t["launch_us"] for t in tm),
                     "all_done": max(t["done_us"] for t in tm), "merge": st["last_combine_us"],
                     "dispatch_wall": st["last_dispatch_us"], "per_shard": tm})
    if not rows:
        return None
    med = {k: statistics.median(r[k] for r in rows) for k in
           ("wall", "dispatch", "launch", "kernel_d2h", "all_done", "merge", "dispatch_wall")}
    return {"step_wall_us": med["wall"], "dispatch_us": med["dispatch"], "launch_us": med["launch"],
            "kernel_d2h_sync_us": med["kernel_d2h"], "all_shards_done_us": med["all_done"],
            "host_merge_us": med["merge"], "dispatch_wall_us": med["dispatch_wall"],
            "rest_us": med["wall"] - med["dispatch_wall"] - med["merge"],
            "last_step_per_shard": rows[-1]["per_shard"], "reps": len(rows),
            "definition": "medians over untimed steps after the timed loop; dispatch = until the last worker took "
                          "the job; launch = plan + launches queued (max over shards); kernel_d2h_sync = launch "
                          "queued -> partial on the host (max over shards); rest = parse/bind/result outside the "
                          "sharded dispatch and merge"}


def sharded_parity(conn, config, out, n_total, nshards, threads):
    """Every shard's partial (duckdb_mbx_shard_partial) vs the oracle over the
    shard's own row range (CTAS splits range(n) evenly: part i = rows
    [n i / S, n (i + 1) / S)), and the global answer vs the sum of those
    oracles (checker only, outside the timed loop)."""
    sys.path.insert(0, HERE)
    from oracle import Oracle
    orc = Oracle()
    shard_par, g_cnt, g_sum, g_groups = [], 0, 0, {}
    for i in range(nshards):
        lo, hi = n_total * i // nshards, n_total * (i + 1) // nshards
        rr = conn.shard_partial(i)
        if config == "c3":
            oc, osum = orc.synth_groupby(7, 9, lo, hi - lo, 32, 1 << 40, -(1 << 39), threads)
            exp = [(k, oc[k], osum[k]) for k in range(32) if oc[k]]
            for k, c_, s_ in exp:
                gc, gs = g_groups.get(k, (0, 0))
                g_groups[k] = (gc + c_, gs + s_)
            got = None
            if rr is not None:
                rows, nulls = rr.cells()
                got = sorted((None if nl[0] else int(rw[0]), int(rw[2]), None if nl[1] else int(rw[1]))
                             for rw, nl in zip(rows, nulls))
            shard_par.append({"shard": i, "rows": [lo, hi], "groups": len(got or []), "match": got == exp,
                              "oracle": exp})
        else:
            oc, osum = orc.synth_filter_count(42, lo, hi - lo, 50, 1, 25, 2**63 - 1, threads)
            g_cnt += oc
            g_sum += osum
            got_c = int(rr.value(0, 0)) if rr is not None else None
            ent = {"shard": i, "rows": [lo, hi], "count": got_c, "oracle_count": oc}
            ok = got_c == oc
            if config == "c5" and rr is not None:
                ent["sum"] = int(rr.value(1, 0))
                ent["oracle_sum"] = osum
                ok = ok and ent["sum"] == osum
            ent["match"] = ok
            shard_par.append(ent)
        if rr is not None:
            rr.close()
    if config == "c3":
        exp = [(k, g_groups[k][0], g_groups[k][1]) for k in sorted(g_groups)]
        got = sorted(out, key=lambda g: (g[0] is None, g[0]))
        par = {"groups": len(got), "oracle_groups": len(exp), "match": got == exp}
    else:
        par = {"gpu_count": int(out[0]), "oracle_count": g_cnt, "match": int(out[0]) == g_cnt}
        if config == "c5":
            par.update({"gpu_sum": int(out[1]), "oracle_sum": g_sum, "match": par["match"] and int(out[1]) == g_sum})
    return par, shard_par


def combine_leg(conn, step, args, n_total, mode):
    """The same query with the other combine (`mode`: "host" after an RCCL
    headline, "rccl" after a host-merge one), timed with the same discipline
    right after the headline: warmup (RCCL communicators are created on first
    use), K timed steps, the global answer vs the headline mode's.  On
    same-device shards RCCL cannot run (one rank per device) and the library
    falls back to the host merge: reported as such."""
    import torch
    before = conn.rccl_info().get("mode", "rccl")
    try:
        conn.set_combine(mode)
        for _ in range(max(1, args.warmup)):
            step()
        st0 = conn.rccl_stats()
        conn.profile_drain()
        elapsed, out = time_steps(step, args.steps, 0, None, torch.cuda.synchronize)
        out = decode_c3(out)
        st1 = conn.rccl_stats()
        conn.profile_drain()
        conn.set_combine(before)
        exp = decode_c3(step())  # the headline mode again: its answer over the same rows
        return {"mode": mode, "headline_mode": before, **combine_delta(st0, st1),
                "ms_per_step": elapsed / args.steps * 1e3,
                "value": n_total * args.steps / elapsed, "unit": "rows/s",
                "last_collective_d2h_us": st1["last_rccl_us"],
                "parity": {mode: [str(x) for x in out], "default": [str(x) for x in exp],
                           "match": [str(x) for x in out] == [str(x) for x in exp]}}
    except Exception as ex:  # noqa: BLE001 - the second leg must not lose the headline line
        conn.set_combine(before)
        return {"error": str(ex)}


def sel_outcomes(conn, before):
    """select_rounds outcomes since `before` (duckdb_mbx_engine_stats): launches,
    aborts (a persistent workgroup never scheduled: the two-pass form reran)
    and launch failures; fallbacks = aborts + failures."""
    st = conn.engine_stats()
    if before:
        st = {k: st[k] - before.get(k, 0) for k in st}
    st["fallbacks"] = st["select_rounds_aborts"] + st["select_rounds_launch_failures"]
    return st


def headline(args, w, ngpu, elapsed, avg_kernel_ms, n_rows_step, launch_rows, parallelism, parity, sel_rows=None):
    """The contract's JSON line (value = all rows every step ÷ time)."""
    value = n_rows_step * args.steps / elapsed
    alg_bytes = launch_rows * w["bytes_per_row"] + (sel_rows * 8 if sel_rows is not None else 0)
    achieved = (alg_bytes / (avg_kernel_ms * 1e-3)) / 1e9 if avg_kernel_ms else None
    return {
        "metric": METRIC,
        "value": value,
        "unit": "rows/s",
        "n_gpus": ngpu,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": w["data"],
        "config": {"workload": w["workload"], "rows_per_gpu": args.rows, "sql": w["sql"], "parallelism": parallelism},
        "roofline": {
            "bound": "hbm",
            "kernel": w["kernel"],
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": pmc_traffic_keys(w.get("pmc_keys", [w["kernel"]]), launch_rows)[0],
            "traffic_source": pmc_traffic_keys(w.get("pmc_keys", [w["kernel"]]), launch_rows)[1],
            "algorithmic_bytes_per_launch": alg_bytes,
            "kernel_ms_avg": avg_kernel_ms,
            "timing": "hipEventRecord pairs on the engine stream around every launch in the timed loop",
        },
        "parity": parity,
    }


def calibrate_into(conn, result, config):
    """This box's measured ceilings beside the spec peak; outside the timed loop."""
    achieved = result["roofline"]["achieved"]
    try:
        cal = conn.hbm_calibrate(2 << 30, 3)
        # sel reads 8 B and writes ~4.2 B per row: the half-writing ring copy is its shape
        best = (max(cal["ring_read_gbs"], cal["read_nt_gbs"]) if config != "sel" else
                max(cal["ring_copy_half_gbs"], cal["ring_copy_gbs"], cal["copy_nt4_gbs"]))
        result["roofline"]["measured_ceilings_gbs"] = {k: round(v, 1) for k, v in cal.items() if k != "bytes"}
        result["roofline"]["frac_of_measured"] = (achieved / best) if achieved and best else None
    except Exception as ex:  # noqa: BLE001 - a calibration failure must not lose the bench line
        result["roofline"]["measured_ceilings_gbs"] = {"error": str(ex)}


def sub_bench(conn, config, plan, args):
    """A secondary config (C3, C3 with NULLs, the wide / sparse-key GROUP BYs,
    sel) on the same connection and clock discipline as the headline: its own
    table (sel reads the headline's), warmup, timed steps, kernel HIP events and
    full-size parity."""
    try:
        n_total = plan["rows_total"]
        w = workload(config, 0, n_total, args.groups)
        own_table = config != "sel"
        if own_table:
            res = conn.query(w["setup"])
            if not hasattr(res, "value"):
                return {"error": str(res.error.message)}
        step = make_step(conn, config, w["sql"], decode=False)
        for _ in range(args.warmup):
            step()
        conn.profile_drain()
        import torch
        before = conn.engine_stats()
        elapsed, out = time_steps(step, args.steps, 0, None, torch.cuda.synchronize)
        kern = conn.profile_drain()
        if isinstance(out, tuple) and out[0] == "c3hrows":  # the cells, pulled once after the timed loop
            out = make_step(conn, config, w["sql"], decode=True)()
            conn.profile_drain()
        out = decode_c3(out)
        outcomes = sel_outcomes(conn, before) if config == "sel" else None
        avg_k, _, _ = kernel_stats(kern, w["kernel"], plan["nshards"], args.steps)
        launch_rows = n_total // plan["nshards"]
        sel_rows = int(out[0]) if config == "sel" else None
        alg = launch_rows * w["bytes_per_row"] + (sel_rows * 8 if sel_rows is not None else 0)
        ach = alg / (avg_k * 1e-3) / 1e9 if avg_k else None
        parity, _ = parity_check(conn, config, w["sql"], out, 0, n_total, len(os.sched_getaffinity(0)), args.groups)
        if own_table:
            conn.query(f"DROP TABLE {w['table']}")
        keys = w.get("pmc_keys", [w["kernel"]])
        r = {"workload": w["workload"], "sql": w["sql"], "steps": args.steps, "warmup": args.warmup,
             "ms_per_step": elapsed / args.steps * 1e3, "value": n_total * args.steps / elapsed, "unit": "rows/s",
             "kernel": w["kernel"], "kernel_ms_avg": avg_k, "algorithmic_bytes_per_launch": alg,
             "achieved_gbs": ach, "frac": ach / HBM_PEAK_GBS if ach else None,
             "traffic": pmc_traffic_keys(keys, launch_rows)[0],
             "traffic_source": pmc_traffic_keys(keys, launch_rows)[1], "parity": parity}
        if config in ("c3h", "c3s", "c3n"):
            r["kernel_split_ms_per_step"] = kernel_split(kern, args.steps)
        if outcomes is not None:
            # every timed step must have run the one-pass kernel: an abort (a persistent workgroup
            # never scheduled, the two-pass form reran) or a launch failure is a fallback
            r["select_rounds"] = outcomes
            r["fallbacks"] = outcomes["fallbacks"]
            if outcomes["fallbacks"] or outcomes["select_rounds_launches"] < args.steps:
                r["parity"]["match"] = False
                r["parity"]["fallback_error"] = (f"{outcomes['fallbacks']} select_rounds fallback(s) / "
                                                 f"{outcomes['select_rounds_launches']} launches in "
                                                 f"{args.steps} timed steps")
                log("[bench] sel: select_rounds fell back in the timed loop: " + json.dumps(outcomes))
        return r
    except Exception as ex:  # noqa: BLE001 - a sub-benchmark failure must not lose the headline line
        return {"error": str(ex)}


def run_single_device_config(args):
    import torch  # noqa: F401  (device init order as in the other paths)
    mbx = load_mbx()
    if args.config == "c1":
        return bench_c1()
    cfg = mbx.Config.create()
    cfg.set("gpu_device", "0")
    cfg.set("mbx_profile", "true")
    conn = mbx.connect_with_config(cfg).value
    return bench_c4(mbx, conn, min(args.rows, 100_000_000), args)


def run_ranks(args, world, rank, local_rank, vote=None):
    """One process per GPU (torch.distributed): every rank holds its own
    1e9-row shard (rows [r*N, (r+1)*N) of the same generator) in its own
    connection, and the global aggregate is combined with an RCCL collective
    inside the timed step (distributed.py).  The world group is gloo (the
    vote, barriers, timing); the combine runs on an RCCL group (backend
    "nccl") over the ranks' devices, or on the gloo group to rehearse."""
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    device = local_rank % max(ndev, 1)  # == local_rank on a full node; 0 when each rank sees one device
    torch.cuda.set_device(device)
    coll_dev, group = "cpu", None
    if world > 1 and args.dist_backend == "nccl":
        coll_dev = "cuda"
        group = dist.new_group(backend="nccl")
    mbx = load_mbx()
    import importlib.util
    spec = importlib.util.spec_from_file_location("duckdb_mbt_amd_distributed",
                                                  os.path.join(HERE, "duckdb.mbt_amd", "distributed.py"))
    mbx_dist = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mbx_dist)

    cfg = mbx.Config.create()
    cfg.set("gpu_device", str(device))
    cfg.set("mbx_profile", "true")
    r = mbx.connect_with_config(cfg)
    if isinstance(r, mbx.Err):
        fail(dist if world > 1 else None, f"rank {rank}: connect to device {device} failed: {r.error.message}")
    conn = r.value
    n = args.rows
    start = rank * n
    w = workload(args.config, start, n)
    c2like = w["c2like"]
    t0 = time.time()
    res = conn.query(w["setup"])
    if isinstance(res, mbx.Err):
        fail(dist if world > 1 else None, f"rank {rank} (device {device}): setup failed: {res.error.message}")
    log(f"[rank {rank}] setup {time.time() - t0:.2f}s: {n} rows")
    step = make_step(conn, args.config, w["sql"])
    gcount = gsum = ggroups = None

    def combine(out):
        # the one exchange of the path: the global aggregate over all shards.
        # C2/C5 start it asynchronously (RCCL's stream) so that it overlaps the
        # next step's query on the engine stream; every step's global answer is
        # collected inside the timed region (finish_combines).
        if world == 1 or args.config == "sel":
            return None
        if c2like:
            return mbx_dist.allreduce_count_async(int(out[0]), device=coll_dev, group=group)  # COUNT(*)
        if args.config == "c5":
            return mbx_dist.global_count_sum_async(int(out[0]), int(out[1]) if out[1] else None, device=coll_dev,
                                                   group=group)
        return mbx_dist.global_group_count_sum(out, device=coll_dev, group=group)  # C3: 32 x (key, count, sum)

    def finish_combines(pending):
        nonlocal gcount, gsum, ggroups
        for p in pending:
            if p is None:
                continue
            r = p.result() if hasattr(p, "result") else p
            if c2like:
                gcount = r
            elif args.config == "c5":
                gcount, gsum = r
            else:
                ggroups = r

    try:
        # warmup includes the collective, so communicator setup is never timed
        finish_combines([combine(step()) for _ in range(args.warmup)])
        conn.profile_drain()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        pending = []
        out = None
        for _ in range(args.steps):
            out = step()
            pending.append(combine(out))
        finish_combines(pending)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
    except Exception as ex:  # noqa: BLE001
        fail(dist if world > 1 else None, f"rank {rank} (device {device}): {ex}")
    kern = conn.profile_drain()
    avg_k, _, _ = kernel_stats(kern, w["kernel"], 1, args.steps)
    t_all = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t_all, op=dist.ReduceOp.MAX)  # (gloo world group)
    elapsed = float(t_all.item())
    parity, orc = parity_check(conn, args.config, w["sql"], out, start, n, host_share(world))
    if world > 1 and args.config in ("c2", "c2d", "c5"):
        # global answer (combined over RCCL in the timed loop) vs the sum of the shard oracles
        g_oracle, g_osum = mbx_dist.global_count_sum(orc[0], orc[1], device=coll_dev, group=group)
        parity["global_count"] = gcount
        parity["global_oracle_count"] = g_oracle
        parity["match"] = parity["match"] and gcount == g_oracle
        if args.config == "c5":
            parity["global_sum"] = gsum
            parity["global_oracle_sum"] = g_osum
            parity["match"] = parity["match"] and gsum == g_osum
    if world > 1 and args.config == "c3":
        g_exp = mbx_dist.global_group_count_sum(orc, device=coll_dev, group=group)
        parity["global_groups"] = len(ggroups)
        parity["global_oracle_groups"] = len(g_exp)
        parity["match"] = parity["match"] and ggroups == g_exp
    # every rank's own line items, gathered to rank 0 (gloo)
    mine = {"rank": rank, "device": device, "kernel_ms_avg": avg_k, "elapsed_s": elapsed,
            "shard_match": parity.get("match"), "rows": [start, start + n]}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    result = None
    if rank == 0:
        par = f"row-range shards x{world}" + ((" + RCCL all-reduce/all-gather" if args.dist_backend == "nccl"
                                              else " + gloo collectives (rehearsal)") if world > 1 else "")
        if vote:
            par += " [one process per GPU: " + vote["reason"] + "]"
        result = headline(args, w, world, elapsed, avg_k, n * world, n, par, parity,
                          sel_rows=int(out[0]) if args.config == "sel" else None)
        if vote:
            result["config"]["form"] = vote
        if world > 1:
            result["multi_device"] = {"path": "one process per GPU (torch.distributed)", "ranks": world,
                                      "combine": ("RCCL (nccl group)" if args.dist_backend == "nccl" else "gloo"),
                                      "per_rank": per_rank}
        calibrate_into(conn, result, args.config)
        if not args.no_cpu and world == 1 and args.config in ("c2", "c2d", "c3", "c5", "sel"):
            result["cpu_baseline"] = cpu_baseline(args.cpu_seconds, "c2" if args.config == "c2d" else args.config)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    conn.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
        if not result["parity"].get("match", True) or not all(p["shard_match"] for p in per_rank):
            log("[bench] PARITY FAILURE: " + json.dumps(per_rank))
            raise SystemExit(3)


def dry_run(args, world, rank, form=None, vote=None):
    """Plumbing only (no GPU): every rank joins a gloo all-reduce of its rank id
    (after the device vote, when there is one) and rank 0 prints the JSON
    skeleton of the layout it would run."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([rank + 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
        dist.destroy_process_group()
    form = form or ("ranks" if args.ranks else "in-library")
    if rank == 0:
        if form == "ranks":
            mode, ngpu, devices = "ranks", world, None
            par = f"row-range shards x{world}" + (" + RCCL all-reduce/all-gather" if world > 1 else "")
            if vote:
                par += " [one process per GPU: " + vote["reason"] + "]"
            md = None
        else:
            plan = inlib_plan(args, world)
            mode, ngpu, devices, par = "in-library", plan["ngpu"], plan["devices"], plan["parallelism"]
            md = None
            if ngpu > 1:
                # what the real N > 1 line adds under multi_device (filled by a GPU run)
                md = {"rccl_selftest": {"devices": dev_map(range(ngpu)), "before": "the connection and the timed loop"},
                      "combine": {"timed_loop": sorted(combine_delta(ZERO_RCCL_STATS, ZERO_RCCL_STATS)),
                                  "rccl": ["state", "prepared_at_connect", "init_s", "check_us", "first_wait_ms",
                                           "ranks[].count", "ranks[].user_rank", "ranks[].cu_device",
                                           "saw_nranks", "proves_n_ranks", "last_collective"]},
                      "curve": {"points": [{"gpus": p, "devices": d} for p, d in
                                           curve_points(ngpu, plan["shards_per_gpu"])]
                                + [{"gpus": ngpu, "devices": plan["devices"], "the_headline": True}]}}
        cfg = {"workload": args.config, "rows_per_gpu": args.rows, "parallelism": par}
        if vote:
            cfg["form"] = vote
        line = {"metric": METRIC, "value": None, "unit": "rows/s", "n_gpus": ngpu,
                "dry_run": True, "mode": mode, "processes": world, "rank_id_sum": int(t.item()),
                "gpu_devices": devices, "config": cfg}
        if md:
            line["multi_device_plan"] = md
        print(json.dumps(line), flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(nproc, argv, port):
    """The torch.distributed.run command line that starts `nproc` ranks of this
    script with the same arguments (one process per GPU, rendezvous on
    127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(nproc, argv):
    """Runs N ranks as a child launcher and forwards rank 0's JSON line to
    stdout; returns the launcher's exit status."""
    import subprocess
    cmd = launcher_cmd(nproc, argv, free_port())
    log("[launcher] " + " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in p.stdout:
        t = line.strip()
        if t.startswith("{") and t.endswith("}"):
            print(t, flush=True)
        else:
            log(line.rstrip("\n"))
    return p.wait()


def one_count(conn):
    rr = conn.query_raw("SELECT COUNT(*) FROM c4")
    v = int(rr.value(0, 0))
    rr.close()
    return v


def bench_c4(mbx, conn, n, args):
    """C4: Appender ingest -> device column -> Arrow read-back (host-link bound).
    Reports H2D ingest GB/s and Arrow int64 read-back GB/s (1e6-row slices,
    the MoonBit decoder cap); values verified bit-exact."""
    import numpy as np
    batch = 10_000_000
    i = np.arange(n, dtype=np.uint64)
    v = ((i * np.uint64(2654435761)) & np.uint64(2**63 - 1)).astype(np.int64)
    # untimed warm-up: the process's first large pageable H2D costs ~50 ms of
    # one-time runtime setup (tools/c4_probe.py, profiles/r02_c4_probe.log)
    conn.query("CREATE TABLE c4w (v BIGINT)")
    ap = conn.create_appender("main", "c4w").value
    ap.append_column(0, v[:min(batch, n)])
    assert isinstance(ap.commit(min(batch, n)), mbx.Ok)
    ap.close()
    conn.query("DROP TABLE c4w")
    conn.query("CREATE TABLE c4 (v BIGINT)")
    ap = conn.create_appender("main", "c4").value
    t0 = time.perf_counter()
    for s in range(0, n, batch):
        ap.append_column(0, v[s:s + batch])
        assert isinstance(ap.commit(min(batch, n - s)), mbx.Ok)
    ap.close()
    t_in = time.perf_counter() - t0
    # read-back in 1e6-row slices (the MoonBit decoders' cap, duckdb_arrow_native.mbt:435):
    # query_arrow + duckdb_mb_arrow_get_column_int64 timed, the check of each
    # returned Bytes ([i32 count][int64 LE values]) done outside the clock
    import ctypes

    def readback(ks, check=True):
        t_q = t_g = 0.0
        good = True
        for k in ks:
            a0 = time.perf_counter()
            a = conn.query_arrow(f"SELECT v FROM c4 LIMIT 1000000 OFFSET {k}").value
            a1 = time.perf_counter()
            bp = mbx.lib.duckdb_mb_arrow_get_column_int64(a._h, 0)
            a2 = time.perf_counter()
            t_q += a1 - a0
            t_g += a2 - a1
            if check:
                m = min(1_000_000, n - k)
                ln = mbx.lib.duckdb_mbx_bytes_len(bp)
                got = np.ctypeslib.as_array(ctypes.cast(bp, ctypes.POINTER(ctypes.c_uint8)), shape=(max(ln, 1),))
                good &= ln == 4 + 8 * m and np.array_equal(got[4:4 + 8 * m].view(np.int64), v[k:k + m])
            mbx.lib.duckdb_mbx_bytes_free(bp)
            a.close()
        return t_q, t_g, good

    slices = list(range(0, n, 1_000_000))
    # untimed getter warm-up: the library's first 15 calls per size class are
    # its trial blocks (5 per copy method, hostlink.cpp MidLink), then it keeps
    # the fastest method; the timed loop is the steady state after them
    readback(slices[:20], check=False)
    t_q, t_g, ok = readback(slices)
    t_out = t_q + t_g
    link = mbx.link_stats()
    # in-run A/B on this box: the runtime's own copy pinned vs the measured
    # choice, alternated in blocks of 25 slices (getter time only)
    ab = {"runtime_copy": [], "adaptive": []}
    blk = slices[:25]
    for _ in range(2):
        for name, mode in (("runtime_copy", 0), ("adaptive", -1)):
            mbx.set_link_mode(mode)
            readback(blk[:3], check=False)  # settle after the switch
            _, tg, good = readback(blk)
            ok &= good
            ab[name].append(len(blk) * 8e6 / tg / 1e9)
    mbx.set_link_mode(-1)
    ok &= one_count(conn) == n
    conn.close()
    # the same round trip through the reference's row-wise Appender API
    # (begin_row / append_bigint / end_row per row), driven natively from C
    row_api = native_harness(["c4", str(n)])
    # and through 2048-row data chunks (duckdb_mb_append_data_chunk, ref duckdb_native.c:2109-2132)
    chunk_api = native_harness(["c4chunk", str(n)])
    res = {"metric": "C4 appender ingest + arrow read-back", "value": n / (t_in + t_out), "unit": "rows/s",
           "n_gpus": 1, "ingest_gbs": n * 8 / t_in / 1e9, "readback_gbs": n * 8 / t_out / 1e9,
           "ingest_s": t_in, "readback_s": t_out, "readback_getter_gbs": n * 8 / t_g / 1e9, "readback_query_s": t_q,
           "rows": n, "bit_exact": ok,
           "readback_note": "steady state after an untimed warm-up of 20 getter calls (the library's 15 trial calls per size class included)",
           "link_mid_stats": link, "readback_ab_getter_gbs": ab,
           "bound": "host link (PCIe Gen5 x16, 63 GB/s spec) + host-side wire-buffer assembly",
           "ingest_api": "columnar duckdb_mbx_append_column (extension), from Python",
           "row_appender_native": row_api, "chunk_appender_native": chunk_api}
    print(json.dumps(res), flush=True)


def native_harness(argv):
    """Runs tests/c_harness/mb_harness.c (gcc-built against include/duckdb_mb.h,
    linked to the library) with `argv`; returns its JSON line or {"error": …}.
    It drives the C-ABI the way MoonBit's native target does, so per-call FFI
    costs are native rather than ctypes'."""
    import subprocess
    import tempfile
    try:
        lib = os.path.join(HERE, "duckdb.mbt_amd")
        exe = os.path.join(tempfile.mkdtemp(), "mb_harness")
        subprocess.run(["gcc", "-O2", "-std=c11", "-I", os.path.join(HERE, "include"),
                        os.path.join(HERE, "tests", "c_harness", "mb_harness.c"), "-o", exe, "-L", lib,
                        "-lduckdb_mb_amd", f"-Wl,-rpath,{lib}"], check=True, capture_output=True)
        p = subprocess.run([exe] + argv, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            return {"error": (p.stdout + p.stderr)[-400:]}
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as ex:  # noqa: BLE001
        return {"error": str(ex)}


def bench_c1():
    """C1 (BASELINE.json configs[0]): SELECT i FROM range(1000000) WHERE i%2=0,
    consumed natively as the MoonBit driver does (per-cell query loop, stream
    chunk loop); exact 500 000 rows, sum 249 999 500 000."""
    r = native_harness(["c1", "5"])
    res = {"metric": "C1 SELECT i FROM range(1e6) WHERE i%2=0, rows/s consumed through the C-ABI",
           "value": r.get("query_rows_per_s"), "unit": "rows/s", "n_gpus": 1, "higher_is_better": True,
           "config": {"workload": "C1 (plumbing): per-cell Connection::query loop and query_stream chunks, native C"},
           "native": r}
    print(json.dumps(res), flush=True)


def host_share(world):
    """Oracle threads for the parity check: this host's cores split between
    the ranks that run it at the same time."""
    return max(1, len(os.sched_getaffinity(0)) // max(1, world))


def l3_bytes():
    """Total L3 of this host (sum over instances), from sysfs; 0 if unknown."""
    seen, total = set(), 0
    base = "/sys/devices/system/cpu"
    try:
        for cpu in os.listdir(base):
            p = os.path.join(base, cpu, "cache", "index3")
            if not cpu.startswith("cpu") or not os.path.isdir(p):
                continue
            ids = open(os.path.join(p, "shared_cpu_list")).read().strip()
            if ids in seen:
                continue
            seen.add(ids)
            sz = open(os.path.join(p, "size")).read().strip()
            mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(sz[-1], 1)
            total += int(sz.rstrip("KMG")) * mult
    except OSError:
        pass
    return total


def cpu_model():
    import platform
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def cgroup_cpus():
    """The cgroup CPU quota in cores (None when unlimited or unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def cpu_baseline(seconds, config="c2", groups=100_000):
    """The oracle's multi-threaded C scan over a materialised sample of the same
    column(s): orc_filter_agg_i64 (C2/C5: COUNT/SUM/MIN/MAX WHERE x > 24),
    orc_groupby_sum_i32_i64 (C3: per-key COUNT and int128 SUM) or
    orc_select_i64 (sel).  The sample is >= 4x the host's total L3, so it
    streams from DRAM as the full column would; generation is outside the
    timed loop.  Two thread counts are timed: ceil(cgroup CPU quota) (what the
    container may actually use) and one pthread per CPU of the affinity mask;
    each is the median of 3 windows.  `value` is the better of the two."""
    import math
    import statistics
    sys.path.insert(0, HERE)
    from oracle import Oracle
    orc = Oracle()
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    qthreads = min(aff, max(1, math.ceil(quota))) if quota else aff
    l3 = l3_bytes()
    bpr = 12 if config in ("c3", "c3h") else 8
    sample = max(250_000_000, -(-4 * l3 // bpr))
    if config in ("c3", "c3h"):
        nk = 32 if config == "c3" else groups
        k = orc.synth_i32(sample, 7, 0, nk, 0)
        v = orc.synth_i64(sample, 9, 0, 1 << 40, -(1 << 39))
        mk = lambda th: (lambda: orc.groupby_sum(k, v, 0, nk, th))  # noqa: E731
        what = f"GROUP BY k: COUNT(*), SUM(v) (int128), {nk} keys" + \
            (" (direct-indexed per-thread tables of the oracle; INT32 keys)" if config == "c3h" else "")
    elif config == "sel":
        import numpy as np
        x = orc.synth_i64(sample, 42, 0, 50, 1)
        buf = np.empty(sample, dtype=np.int64)
        buf.fill(0)  # first touch outside the timed loop
        mk = lambda th: (lambda: orc.select_i64(x, 25, 2**63 - 1, th, out=buf))  # noqa: E731
        what = "SELECT x WHERE x > 24: count pass + order-preserving copy of the passing rows"
    else:
        x = orc.synth_i64(sample, 42, 0, 50, 1)
        mk = lambda th: (lambda: orc.filter_agg_i64(x, 25, 2**63 - 1, th))  # noqa: E731
        what = "COUNT/SUM/MIN/MAX with x > 24"
    counts = sorted({qthreads, aff})
    if config == "c3h":
        # per-thread tables of `groups` keys: one thread count (the quota), so
        # the baseline stays bounded (256 threads x 1e6-key tables take GBs)
        counts = [qthreads]
    window = seconds / (3 * len(counts))
    per = {}
    for th in counts:
        log(f"[bench] cpu baseline: {th} threads, {what}")
        run = mk(th)
        run()  # first touch / thread start-up outside the timed windows
        rates = []
        for _ in range(3):
            scanned = 0
            t0 = time.perf_counter()
            while True:
                run()
                scanned += sample
                if time.perf_counter() - t0 >= window:
                    break
            rates.append(scanned / (time.perf_counter() - t0))
        per[th] = {"median_rows_per_s": statistics.median(rates), "windows_rows_per_s": rates}
    best = max(per, key=lambda th: per[th]["median_rows_per_s"])
    val = per[best]["median_rows_per_s"]
    return {"value": val, "unit": "rows/s", "cores": best, "kind": "port",
            "nproc": os.cpu_count(), "cpu": cpu_model(), "l3_bytes": l3, "cgroup_cpu_quota": quota,
            "gbs": val * bpr / 1e9,
            "by_threads": {str(th): per[th] for th in counts},
            "sample": f"{sample} rows ({sample * bpr / 1e9:.2f} GB, >= 4x L3 = {4 * l3 / 1e9:.2f} GB) of the same "
                      f"columns, {what}; pthreads = ceil(cgroup quota) = {qthreads} and = affinity = {aff}, "
                      f"each the median of 3 windows of {window:.1f} s; value = the better median"}


if __name__ == "__main__":
    main()
