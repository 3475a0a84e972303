"""Multi-GPU combine of per-shard aggregate partials.

One process per GPU, each owning a contiguous row-range shard of the table.
The only exchange is the final combine of the global aggregates: COUNT is an
int64 all-reduce; SUM is an exact int128 (DuckDB HUGEINT), which no RCCL
reduction op supports, so every rank all-gathers its partial as two int64
lanes (lo, hi) and combines them exactly (carry-correct) afterwards.  A
GROUP BY (config C3) exchanges its per-shard group table the same way: one
fixed-width row per group ("32 x 24 B per GPU").  On ROCm,
backend "nccl" is RCCL (over xGMI); tests use "gloo" on the CPU.
"""
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

MASK64 = (1 << 64) - 1


def encode_i128(v: int):
    lo = v & MASK64
    hi = (v >> 64) & MASK64
    as_signed = lambda x: x - (1 << 64) if x >= 1 << 63 else x
    return as_signed(lo), as_signed(hi)


def decode_i128(lo: int, hi: int) -> int:
    v = ((hi & MASK64) << 64) | (lo & MASK64)
    return v - (1 << 128) if v >= 1 << 127 else v


def allgather_i128(values: Sequence[int], device="cpu", group=None) -> List[List[int]]:
    """All-gathers a fixed-length list of (up to int128) integers per rank."""
    world = dist.get_world_size(group)
    flat = []
    for v in values:
        flat.extend(encode_i128(int(v)))
    t = torch.tensor(flat, dtype=torch.int64, device=device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    res = []
    for o in outs:
        o = o.cpu().tolist()
        res.append([decode_i128(o[2 * i], o[2 * i + 1]) for i in range(len(values))])
    return res


def combine_count_sum(parts: List[List[int]]):
    """parts[rank] = [count, sum]; sum may be None-encoded as 0 when count==0."""
    count = sum(p[0] for p in parts)
    total = sum(p[1] for p in parts)
    return count, (total if count else None)


def global_count_sum(local_count: int, local_sum, device="cpu", group=None):
    """Global COUNT(*) / SUM(x) (x > ..) over all shards, exact."""
    parts = allgather_i128([local_count, 0 if local_sum is None else local_sum], device, group)
    return combine_count_sum(parts)


_count_buf = {}


def allreduce_count(local_count: int, device="cpu", group=None) -> int:
    """Global COUNT(*): one int64 all-reduce (sum).  The one-element buffer is
    reused across calls, so a step pays only the fill, the collective and the
    read-back."""
    key = (str(device), id(group))
    t = _count_buf.get(key)
    if t is None:
        t = _count_buf[key] = torch.zeros(1, dtype=torch.int64, device=device)
    t.fill_(int(local_count))
    dist.all_reduce(t, group=group)
    return int(t.item())


# One exchanged row per group: [flags, key, count, sum_lo, sum_hi]
#   flags bit0 = row present (ranks pad to the largest group table),
#         bit1 = key is NULL, bit2 = the SUM is non-NULL.
_GROUP_W = 5


def global_group_count_sum(groups: Sequence[Tuple[Optional[int], int, Optional[int]]], device="cpu",
                           group=None) -> List[Tuple[Optional[int], int, Optional[int]]]:
    """Exact global ``SELECT k, COUNT(*), SUM(v) ... GROUP BY k`` from per-shard
    partials.  ``groups`` holds (key | None, count, sum | None) for this rank's
    shard; the result is ordered by key with the NULL group last (DuckDB's
    NULLS LAST).  Keys and counts are int64; sums are int128 (HUGEINT)."""
    world = dist.get_world_size(group)
    g = torch.tensor([len(groups)], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(g, op=dist.ReduceOp.MAX, group=group)
    width = max(int(g.item()), 1)
    rows = [[0] * _GROUP_W for _ in range(width)]
    for i, (k, c, sm) in enumerate(groups):
        lo, hi = encode_i128(0 if sm is None else int(sm))
        rows[i] = [1 | (2 if k is None else 0) | (0 if sm is None else 4), 0 if k is None else int(k), int(c), lo, hi]
    t = torch.tensor(rows, dtype=torch.int64, device=device)
    outs = [torch.empty_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(outs, t, group=group)
    else:
        outs = [t]
    acc = {}
    for o in outs:
        for flags, k, c, lo, hi in o.cpu().tolist():
            if not flags & 1:
                continue
            key = None if flags & 2 else k
            cc, ss = acc.get(key, (0, None))
            if flags & 4:
                ss = (ss or 0) + decode_i128(lo, hi)
            acc[key] = (cc + c, ss)
    keys = sorted(k for k in acc if k is not None) + ([None] if None in acc else [])
    return [(k, acc[k][0], acc[k][1]) for k in keys]


# ---- asynchronous combines: the collective of step i runs on RCCL's stream
# while the engine stream executes step i+1's query; .result() waits.
class PendingCombine:
    def __init__(self, work, finish):
        self._work, self._finish = work, finish

    def result(self):
        if self._work is not None:
            self._work.wait()
        return self._finish()


def allreduce_count_async(local_count: int, device="cpu", group=None) -> PendingCombine:
    """Global COUNT(*) as an asynchronous int64 all-reduce (sum)."""
    t = torch.full((1,), int(local_count), dtype=torch.int64, device=device)
    w = dist.all_reduce(t, group=group, async_op=True)
    return PendingCombine(w, lambda: int(t.item()))


def global_count_sum_async(local_count: int, local_sum, device="cpu", group=None) -> PendingCombine:
    """Global COUNT(*) / exact int128 SUM as an asynchronous all-gather."""
    world = dist.get_world_size(group)
    flat = []
    for v in (local_count, 0 if local_sum is None else local_sum):
        flat.extend(encode_i128(int(v)))
    t = torch.tensor(flat, dtype=torch.int64, device=device)
    outs = [torch.empty_like(t) for _ in range(world)]
    w = dist.all_gather(outs, t, group=group, async_op=True)

    def finish():
        parts = []
        for o in outs:
            o = o.cpu().tolist()
            parts.append([decode_i128(o[0], o[1]), decode_i128(o[2], o[3])])
        return combine_count_sum(parts)

    return PendingCombine(w, finish)
