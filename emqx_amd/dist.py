"""Multi-GPU layouts of the match path (one process per GPU, torch.distributed).

``shard="filters"`` (the north-star layout): the subscription set is partitioned by
``hash(filter) mod G``; every rank holds the trie + route keys of its shard.  Per batch, rank 0
broadcasts the packed topic batch (RCCL over xGMI), each rank matches it against its shard,
and the per-rank CSR results are gathered to rank 0 and merged (a topic's row is the union of
its rows on every shard; shards are disjoint, so there is nothing to dedupe).

``shard="topics"`` (replicas): every rank holds the whole index (it fits: SURVEY 8e capacity
note) and matches its own batch; no collective is on the data path.

The collective code is device-agnostic: with the gloo backend the same functions run on CPU
tensors, which is how tests/test_dist.py covers world_size 2 without a GPU (there the per-rank
matcher is injected by the test).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

NONE = 0xFFFFFFFF
_P = np.uint64(0x100000001B3)


def filter_shards(fbytes: np.ndarray, foff: np.ndarray, world: int) -> np.ndarray:
    """Shard of each packed filter: a 64-bit polynomial hash of its bytes, mod `world`.
    A function of the filter string only, so every node and rank agrees on placement."""
    n = len(foff) - 1
    if world == 1 or n == 0:
        return np.zeros(n, np.int64)
    foff = foff.astype(np.int64)
    lens = np.diff(foff)
    pos = np.arange(int(foff[-1]), dtype=np.int64) - np.repeat(foff[:-1], lens)
    with np.errstate(over="ignore"):
        mult = np.ones(int(lens.max()) + 1, np.uint64)
        for i in range(1, len(mult)):
            mult[i] = mult[i - 1] * _P
        terms = (fbytes[: int(foff[-1])].astype(np.uint64) + np.uint64(1)) * mult[pos]
        h = np.zeros(n, np.uint64)
        nz = lens > 0
        if terms.size:
            sums = np.add.reduceat(terms, foff[:-1][nz])
            h[nz] = sums
        h ^= h >> np.uint64(29)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(32)
    return (h % np.uint64(world)).astype(np.int64)


@dataclass
class Merged:
    row_ptr: torch.Tensor    # int64 [n+1]
    filter_id: torch.Tensor  # int64 [pairs] global filter ids
    exact_id: torch.Tensor   # int64 [n] global id or NONE


def broadcast_batch(tbytes: Optional[torch.Tensor], toff: Optional[torch.Tensor], device,
                    src: int = 0, group=None):
    """Rank `src` broadcasts the packed topic batch (u8 bytes, i32 offsets) to every rank."""
    meta = torch.zeros(2, dtype=torch.int64, device=device)
    if dist.get_rank(group) == src:
        meta[0] = tbytes.numel()
        meta[1] = toff.numel()
    dist.broadcast(meta, src, group=group)
    nb, no = int(meta[0]), int(meta[1])
    if dist.get_rank(group) != src:
        tbytes = torch.empty(nb, dtype=torch.uint8, device=device)
        toff = torch.empty(no, dtype=torch.int32, device=device)
    if nb:
        dist.broadcast(tbytes, src, group=group)
    dist.broadcast(toff, src, group=group)
    return tbytes, toff


def gather_merge(row: torch.Tensor, gid: torch.Tensor, exact: torch.Tensor, dst: int = 0,
                 group=None) -> Optional[Merged]:
    """Gather each rank's CSR (row int64[n+1], gid int64[pairs], exact int64[n]) to `dst` and
    merge rows topic by topic.  Returns the merged result on `dst`, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    device = row.device
    n = row.numel() - 1
    sizes = torch.tensor([gid.numel()], dtype=torch.int64, device=device)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    maxp = int(max(int(s) for s in all_sizes))
    pad = torch.full((maxp,), -1, dtype=torch.int64, device=device)
    pad[: gid.numel()] = gid
    rows = [torch.zeros_like(row) for _ in range(world)]
    gids = [torch.zeros_like(pad) for _ in range(world)]
    exs = [torch.zeros_like(exact) for _ in range(world)]
    # all_gather works on every backend (gloo and RCCL); only dst keeps the merge
    dist.all_gather(rows, row, group=group)
    dist.all_gather(gids, pad, group=group)
    dist.all_gather(exs, exact, group=group)
    if rank != dst:
        return None
    counts = torch.stack([r[1:] - r[:-1] for r in rows])          # [world, n]
    total = counts.sum(0)
    out_row = torch.zeros(n + 1, dtype=torch.int64, device=device)
    out_row[1:] = torch.cumsum(total, 0)
    before = torch.cumsum(counts, 0) - counts                    # pairs of lower ranks per topic
    out = torch.empty(int(out_row[-1]), dtype=torch.int64, device=device)
    ar = torch.arange(n, device=device)
    for r in range(world):
        c = counts[r]
        p = int(all_sizes[r])
        if p == 0:
            continue
        topic = torch.repeat_interleave(ar, c)
        j = torch.arange(p, device=device) - rows[r][:-1][topic]
        out[out_row[:-1][topic] + before[r][topic] + j] = gids[r][:p]
    ex = torch.stack(exs).min(0).values  # a route key lives on exactly one shard
    return Merged(out_row, out, ex)


def device_result_to_torch(engine, dres, device) -> tuple:
    """Copy an engine's device-resident result into torch tensors on `device` (D2D)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    n, p = dres.n, dres.n_pairs
    row = torch.empty(n + 1, dtype=torch.int32, device=device)
    fid = torch.empty(max(p, 1), dtype=torch.int32, device=device)
    ex = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    for dst, src, nb in ((row, dres.row_ptr, (n + 1) * 4), (fid, dres.filter_id, p * 4),
                         (ex, dres.exact_id, n * 4)):
        if nb and hip.hipMemcpy(dst.data_ptr(), src, nb, 3) != 0:
            raise RuntimeError("hipMemcpy D2D failed")
    u32 = lambda t: t.to(torch.int64) & 0xFFFFFFFF  # noqa: E731
    return u32(row), u32(fid[:p]), u32(ex[:n])
