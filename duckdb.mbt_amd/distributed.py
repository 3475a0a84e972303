"""Multi-GPU combine of per-shard aggregate partials.

One process per GPU, each owning a contiguous row-range shard of the table.
The only exchange is the final combine of the global aggregates: COUNT is an
int64 all-reduce; SUM is an exact int128 (DuckDB HUGEINT), which no RCCL
reduction op supports, so every rank all-gathers its partial as two int64
lanes (lo, hi) and combines them exactly (carry-correct) afterwards.  On
ROCm, backend "nccl" is RCCL (over xGMI); tests use "gloo" on the CPU.
"""
from typing import List, Sequence

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


def allreduce_count(local_count: int, device="cpu", group=None) -> int:
    t = torch.tensor([int(local_count)], dtype=torch.int64, device=device)
    dist.all_reduce(t, group=group)
    return int(t.item())
