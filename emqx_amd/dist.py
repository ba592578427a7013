"""Multi-GPU layouts of the match path (one process per GPU, torch.distributed).

``shard="filters"`` (the north-star layout): the subscription set is partitioned by
``hash(filter) mod G``; every rank holds the trie + route keys of its shard.  Per batch:

1. rank 0 broadcasts the packed topic batch (RCCL over xGMI);
2. every rank matches it against its shard on its GPU and exports the CSR with its local filter
   ids mapped to global ids (``emqxgm_export``, one kernel);
3. the ranks' pair counts are exchanged with one all_gather of G integers, and rank 0 receives
   each rank's CSR with sized point-to-point receives (``batch_isend_irecv``: grouped
   send/recv, each rank's list crosses xGMI once, only to rank 0);
4. rank 0 merges the G CSRs topic by topic in a HIP kernel (``emqxgm_merge``: shards are
   disjoint, nothing to dedupe; a topic's exact route key lives on exactly one shard).

Host synchronisations per step: the batch size on the receiving ranks (step 1), the match pass
itself, and the pair counts on rank 0 (step 3).

``shard="topics"`` (replicas): every rank holds the whole index (it fits: SURVEY 8e capacity
note) and matches its own batch; no collective is on the data path.

The collective code (broadcast_batch, gather_to_root) is device-agnostic: with the gloo backend
it runs on CPU tensors, which is how tests/test_dist.py covers world_size 2 without a GPU (the
per-rank matcher and the merge there are the test's own).  The merge (merge_parts) is HIP only.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

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


def _comm_on_cpu(group=None) -> bool:
    """gloo moves CPU tensors only (its CUDA support stops at a few collectives): a gloo
    rehearsal of the N>1 path stages its messages through host memory."""
    return dist.get_backend(group) == "gloo"


def broadcast_batch(tbytes: Optional[torch.Tensor], toff: Optional[torch.Tensor], device,
                    src: int = 0, group=None):
    """Rank `src` broadcasts the packed topic batch (u8 bytes, i32 offsets) to every rank."""
    cpu = _comm_on_cpu(group)
    cdev = "cpu" if cpu else device
    meta = torch.zeros(2, dtype=torch.int64, device=cdev)
    if dist.get_rank(group) == src:
        meta[0] = tbytes.numel()
        meta[1] = toff.numel()
    dist.broadcast(meta, src, group=group)
    nb, no = int(meta[0]), int(meta[1])
    if dist.get_rank(group) != src:
        tbytes = torch.empty(nb, dtype=torch.uint8, device=cdev)
        toff = torch.empty(no, dtype=torch.int32, device=cdev)
    else:
        tbytes, toff = tbytes.to(cdev), toff.to(cdev)
    if nb:
        dist.broadcast(tbytes, src, group=group)
    dist.broadcast(toff, src, group=group)
    return tbytes.to(device), toff.to(device)


Part = Tuple[torch.Tensor, torch.Tensor, torch.Tensor]  # (row [n+1], fid [pairs], exact [n])


def gather_to_root(row: torch.Tensor, fid: torch.Tensor, exact: torch.Tensor, n_pairs: int,
                   root: int = 0, group=None) -> Optional[List[Part]]:
    """Each rank's CSR (int32 row [n+1], fid [>= n_pairs], exact [n]) to `root`: the pair counts
    with one all_gather of G integers, then sized point-to-point receives on the root only.
    Returns on the root the G parts in rank order (its own included), None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = row.device
    cpu = _comm_on_cpu(group)
    cdev = "cpu" if cpu else dev
    cnt = torch.tensor([n_pairs], dtype=torch.int64, device=cdev)
    allc = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(world)]
    dist.all_gather(allc, cnt, group=group)
    fid = fid[:n_pairs]
    if rank != root:
        ops = [dist.P2POp(dist.isend, row.to(cdev), root, group),
               dist.P2POp(dist.isend, exact.to(cdev), root, group)]
        if n_pairs:
            ops.append(dist.P2POp(dist.isend, fid.to(cdev), root, group))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        return None
    counts = [int(c) for c in torch.cat(allc).tolist()]
    parts: List[Part] = []
    ops = []
    for r in range(world):
        if r == root:
            parts.append((row, fid, exact))
            continue
        rr = torch.empty(row.numel(), dtype=row.dtype, device=cdev)
        ee = torch.empty(exact.numel(), dtype=exact.dtype, device=cdev)
        ff = torch.empty(counts[r], dtype=fid.dtype, device=cdev)
        ops += [dist.P2POp(dist.irecv, rr, r, group), dist.P2POp(dist.irecv, ee, r, group)]
        if counts[r]:
            ops.append(dist.P2POp(dist.irecv, ff, r, group))
        parts.append((rr, ff, ee))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return [(a.to(dev), b.to(dev), c.to(dev)) for a, b, c in parts]


@dataclass
class Merged:
    row_ptr: torch.Tensor    # int32 [n+1]
    filter_id: torch.Tensor  # int32 [pairs] global filter ids (u32 bits)
    exact_id: torch.Tensor   # int32 [n] global id or NONE (u32 bits)


def merge_parts(eng, parts: Sequence[Part], n: int) -> Merged:
    """Merge the shards' CSRs topic by topic on the device (emqxgm_merge, a HIP kernel)."""
    dev = parts[0][0].device
    if dev.type != "cuda":
        raise RuntimeError("merge_parts runs on the GPU (emqxgm_merge); there is no CPU merge")
    total = sum(int(p[1].numel()) for p in parts)
    row = torch.empty(n + 1, dtype=torch.int32, device=dev)
    fid = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    ex = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    torch.cuda.current_stream(dev).synchronize()  # the parts came in on torch's streams
    got = eng.merge([p[0].data_ptr() for p in parts],
                    [p[1].data_ptr() if p[1].numel() else 0 for p in parts],
                    [p[2].data_ptr() for p in parts], n, row.data_ptr(),
                    fid.data_ptr() if total else 0, ex.data_ptr())
    assert got == total, (got, total)
    return Merged(row, fid[:total], ex[:n])


class ShardedMatcher:
    """The filter-sharded match step of one rank: `eng` holds this rank's filter
    shard, `gid_map` (int32 device tensor) maps its local filter ids to global ids."""

    def __init__(self, eng, gid_map: torch.Tensor, device, group=None, root: int = 0):
        self.eng = eng
        self.gid_map = gid_map
        self.device = device
        self.group = group
        self.root = root
        self._bufs = None

    def _out(self, n: int, pairs: int):
        cap_n, cap_p = (0, 0) if self._bufs is None else (self._bufs[2].numel(), self._bufs[1].numel())
        if n + 1 > cap_n or pairs > cap_p:
            self._bufs = (torch.empty(max(n + 1, cap_n), dtype=torch.int32, device=self.device),
                          torch.empty(max(pairs, cap_p, 1), dtype=torch.int32, device=self.device),
                          torch.empty(max(n + 1, cap_n), dtype=torch.int32, device=self.device))
        row, fid, ex = self._bufs
        return row[: n + 1], fid, ex[:n]

    def step(self, tbytes: Optional[torch.Tensor] = None,
             toff: Optional[torch.Tensor] = None) -> Optional[Merged]:
        """One batch (given on the root): broadcast, match this shard, gather, merge on root."""
        b, o = broadcast_batch(tbytes, toff, self.device, self.root, self.group)
        n = o.numel() - 1
        torch.cuda.current_stream(self.device).synchronize()  # the engine's stream reads them
        r = self.eng.match_device(b.data_ptr(), o.data_ptr(), n, b.numel())
        row, fid, ex = self._out(n, r.n_pairs)
        self.eng.export(r, self.gid_map.data_ptr(), row.data_ptr(),
                        fid.data_ptr() if r.n_pairs else 0, ex.data_ptr() if n else 0)
        parts = gather_to_root(row, fid, ex, r.n_pairs, self.root, self.group)
        if parts is None:
            return None
        return merge_parts(self.eng, parts, n)
