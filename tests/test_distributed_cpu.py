"""The N>1 combine path on the CPU: world_size 2 with the gloo backend.  Each
rank computes its shard's partial with the oracle (standing in for the GPU
shard query) and the exact int128 combine must equal the single-process
answer over the whole range."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import importlib.util
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location("mbx_dist", os.path.join(ROOT, "duckdb.mbt_amd", "distributed.py"))
    d = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(d)
    from oracle import Oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle()
    start = rank * n
    c, s = o.synth_filter_count(42, start, n, 50, 1, 25, 2**63 - 1, 2)
    gc, gs = d.global_count_sum(c, s)
    tc = d.allreduce_count(c)
    # the async forms the bench overlaps with the next step's query: several in flight
    pend = [(d.allreduce_count_async(c + k), d.global_count_sum_async(c, s + k)) for k in range(3)]
    asy = [(a.result(), b.result()) for a, b in pend]
    # huge partials: carries across the 64-bit boundary must survive
    big = d.allgather_i128([(2**100 + rank) * (1 if rank else -1), -(2**63) - rank])
    dist.destroy_process_group()
    q.put((rank, gc, gs, tc, big, asy))


@pytest.mark.parametrize("world", [2, 4])
def test_global_count_sum_gloo(world):
    n = 200_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from oracle import Oracle
    c, s = Oracle().synth_filter_count(42, 0, n * world, 50, 1, 25, 2**63 - 1, 4)
    for rank, gc, gs, tc, big, asy in out:
        assert (gc, gs, tc) == (c, s, c)
        assert asy == [(c + world * k, (c, s + world * k)) for k in range(3)]
        assert big == [[(2**100 + r) * (1 if r else -1), -(2**63) - r] for r in range(world)]


def test_i128_codec():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mbx_dist", os.path.join(ROOT, "duckdb.mbt_amd", "distributed.py"))
    d = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(d)
    for v in [0, 1, -1, 2**63, -(2**63) - 1, 2**127 - 1, -(2**127), 123456789 * 2**70]:
        assert d.decode_i128(*d.encode_i128(v)) == v


def _group_worker(rank, world, port, n, q):
    import importlib.util
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    spec = importlib.util.spec_from_file_location("mbx_dist", os.path.join(ROOT, "duckdb.mbt_amd", "distributed.py"))
    d = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(d)
    from oracle import Oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle()
    # this rank's row-range shard of the C3 table, partials from the oracle
    k = o.synth_i32(n * world, 7, 0, 32, 0)[rank * n:(rank + 1) * n]
    v = o.synth_i64(n * world, 9, 0, 2**40, -2**39)[rank * n:(rank + 1) * n]
    counts, sums = o.groupby_sum(k, v, 0, 32, 2)
    local = [(i, counts[i], sums[i]) for i in range(32) if counts[i]]
    if rank == 1:
        # ragged tables: rank 1 drops a key and adds a NULL group and a NULL-sum group
        local = [g for g in local if g[0] != 5] + [(None, 3, 2**70), (1000, 2, None)]
    res = d.global_group_count_sum(local)
    dist.destroy_process_group()
    q.put((rank, res))


def test_global_group_count_sum_gloo():
    world, n = 2, 100_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from oracle import Oracle
    o = Oracle()
    k = o.synth_i32(n * world, 7, 0, 32, 0)
    v = o.synth_i64(n * world, 9, 0, 2**40, -2**39)
    # expected: full-table groups, minus rank 1's key-5 rows, plus the extra groups
    k1, v1 = k[n:], v[n:]
    c_all, s_all = o.groupby_sum(k, v, 0, 32, 2)
    m5 = k1 == 5
    exp = []
    for i in range(32):
        c, s = c_all[i], s_all[i]
        if i == 5:
            c -= int(m5.sum())
            s -= int(v1[m5].astype(object).sum())
        if c:
            exp.append((i, c, s))
    exp += [(1000, 2, None), (None, 3, 2**70)]
    for _, res in out:
        assert res == exp
