"""Multi-GPU layouts of the match path (one process per GPU, torch.distributed).

``shard="filters"`` (the north-star layout): the subscription set is partitioned by
``hash(filter) mod G``; every rank holds the trie + route keys of its shard.  Per batch:

1. rank 0 broadcasts the packed topic batch (RCCL over xGMI);
2. every rank matches it against its shard on its GPU and exports the CSR with its local filter
   ids mapped to global ids (``emqxgm_export``, one kernel);
3. every rank puts its result in the compact wire form (``emqxgm_export_wire``: u8 pair counts,
   global ids, sparse exact hits); the lengths go round in one all_gather of 3 x G integers and
   rank 0 receives each rank's part with sized point-to-point receives (``batch_isend_irecv``);
4. rank 0 merges the G parts topic by topic in HIP kernels (``emqxgm_merge_wire``: shards are
   disjoint, nothing to dedupe; a topic's exact route key lives on exactly one shard).

Steps are pipelined (``ShardedMatcher.run``): batch k+1 is broadcast while the engine walks batch
k.  Host synchronisations per step: the match pass (its pair count sizes the export), the
export's entry counts, and the lengths on rank 0; the batch shape is known to every rank.

``shard="topics"`` (replicas): every rank holds the whole index (it fits: SURVEY 8e capacity
note) and matches its own batch; no collective is on the data path.

``shard="keys"`` (r06, SURVEY 8e's alternative for a route-key-heavy index, cfg4): the plain route
keys are partitioned by key hash (``emqxgm_key_owners``), every rank also holds every wildcard
filter.  Per batch, broadcast to every rank: rank r matches its block of topics [r n / G,
(r + 1) n / G) (tokenizer, trie walk, wildcard-key probe, and the plain keys it owns) and probes
the route key of every name it owns (``emqxgm_exact_owned_device``: a hash per name, one probe per
owned name on a table of 1/G of the keys -- below the TLB's reach at cfg4); the dense per-rank
parts go to rank 0 and are merged by ``emqxgm_merge`` (a topic's trie row comes from its block's
rank, its exact id from its key's owner).  ``KeyShardedMatcher``; DESIGN.md 5 models when it pays.

The collective code (broadcast_batch, gather_wire_to_root) is device-agnostic: with the gloo
backend it runs on CPU tensors, which is how tests/test_dist.py covers world_size 2 without a GPU
(the per-rank matcher, the wire export and the merge there are the test's torch restatements).
The export and the merge (merge_wire) are HIP only.
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


WIRE_CNT2, WIRE_ID24 = 1, 2  # include/emqx_gpumatch.h EMQXGM_WIRE_*


def wire_flags(n: int, pairs: int, n_global: int) -> int:
    """The wire form for a result: 2-bit counts when pairs are sparse (at most one per two
    topics: few counts reach 3), 24-bit ids when every global id fits."""
    return (WIRE_CNT2 if 2 * pairs <= n else 0) | (WIRE_ID24 if n_global <= (1 << 24) else 0)


def wire_sizes(flags: int, n: int, pairs: int) -> Tuple[int, int]:
    """Bytes of the count and id sections."""
    cnt = 16 * ((n + 63) // 64) if flags & WIRE_CNT2 else n
    return cnt, (3 if flags & WIRE_ID24 else 4) * pairs


@dataclass
class WirePart:
    """One shard's result in the compact wire form (emqxgm_export_wire): pair counts (u8 or two
    bit planes), the pairs' global ids (u32 or u16 + u8 planes), and (topic, exact id) /
    (topic, count) pairs of the topics that equal a route key / outgrow the count width."""
    flags: int
    pairs: int
    cnt: torch.Tensor   # uint8 [wire_sizes[0]]
    fid: torch.Tensor   # uint8 [wire_sizes[1]]
    xs: torch.Tensor    # int32 [2 * nx]
    ovf: torch.Tensor   # int32 [2 * novf]

    def nbytes(self) -> int:
        return sum(int(t.numel()) * t.element_size() for t in (self.cnt, self.fid, self.xs, self.ovf))


def gather_wire_to_root(part: WirePart, root: int = 0, group=None) -> Optional[List[WirePart]]:
    """Each rank's wire part to `root`: (flags, pairs, exact, overflow) with one all_gather of
    4 x G integers (the root's one host synchronisation: it sizes the receives), then sized
    point-to-point receives on the root only.  Per non-root rank a 2-bit-count, 24-bit-id part
    is n / 4 + 3 pairs + 8 (exact hits + overflows) bytes, against 8 n + 4 pairs for dense u32
    row pointers and exact ids.  Returns on the root the G parts in rank order (its own
    included), None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = part.cnt.device
    cpu = _comm_on_cpu(group)
    cdev = "cpu" if cpu else dev
    lens = torch.tensor([part.flags, part.pairs, part.xs.numel() // 2, part.ovf.numel() // 2,
                         part.cnt.numel()], dtype=torch.int64, device=cdev)
    alll = [torch.zeros(5, dtype=torch.int64, device=cdev) for _ in range(world)]
    dist.all_gather(alll, lens, group=group)
    if rank != root:
        ops = []
        for t in (part.cnt, part.fid, part.xs, part.ovf):
            if t.numel():
                ops.append(dist.P2POp(dist.isend, t.to(cdev), root, group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return None
    ls = torch.stack(alll).tolist()
    parts: List[WirePart] = []
    ops = []
    for r in range(world):
        if r == root:
            parts.append(part)
            continue
        fl, p, nx, no, nc = (int(x) for x in ls[r])
        q = WirePart(fl, p, torch.empty(nc, dtype=torch.uint8, device=cdev),
                     torch.empty((3 if fl & WIRE_ID24 else 4) * p, dtype=torch.uint8, device=cdev),
                     torch.empty(2 * nx, dtype=torch.int32, device=cdev),
                     torch.empty(2 * no, dtype=torch.int32, device=cdev))
        for t in (q.cnt, q.fid, q.xs, q.ovf):
            if t.numel():
                ops.append(dist.P2POp(dist.irecv, t, r, group))
        parts.append(q)
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return [WirePart(q.flags, q.pairs, *(t.to(dev) for t in (q.cnt, q.fid, q.xs, q.ovf)))
            for q in parts]


@dataclass
class Merged:
    row_ptr: torch.Tensor    # int32 [n+1]
    filter_id: torch.Tensor  # int32 [pairs] global filter ids (u32 bits)
    exact_id: torch.Tensor   # int32 [n] global id or NONE (u32 bits)


Part = Tuple[torch.Tensor, torch.Tensor, torch.Tensor]  # (row [n+1], fid [pairs], exact [n])


def merge_parts(eng, parts: Sequence[Part], n: int) -> Merged:
    """Merge dense per-shard CSRs (emqxgm_export's form) topic by topic (emqxgm_merge)."""
    dev = parts[0][0].device
    if dev.type != "cuda":
        raise RuntimeError("merge_parts runs on the GPU (emqxgm_merge); there is no CPU merge")
    total = sum(int(p[1].numel()) for p in parts)
    row = torch.empty(n + 1, dtype=torch.int32, device=dev)
    fid = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    ex = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    torch.cuda.current_stream(dev).synchronize()
    got = eng.merge([p[0].data_ptr() for p in parts],
                    [p[1].data_ptr() if p[1].numel() else 0 for p in parts],
                    [p[2].data_ptr() for p in parts], n, row.data_ptr(),
                    fid.data_ptr() if total else 0, ex.data_ptr())
    assert got == total, (got, total)
    return Merged(row, fid[:total], ex[:n])


def merge_wire(eng, parts: Sequence[WirePart], n: int) -> Merged:
    """Merge the shards' wire parts topic by topic on the device (emqxgm_merge_wire)."""
    dev = parts[0].cnt.device
    if dev.type != "cuda":
        raise RuntimeError("merge_wire runs on the GPU (emqxgm_merge_wire); there is no CPU merge")
    total = sum(p.pairs for p in parts)
    row = torch.empty(n + 1, dtype=torch.int32, device=dev)
    fid = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    ex = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    torch.cuda.current_stream(dev).synchronize()  # the parts came in on torch's streams
    ptr = lambda t: t.data_ptr() if t.numel() else 0  # noqa: E731
    got = eng.merge_wire([p.flags for p in parts], [ptr(p.cnt) for p in parts],
                         [ptr(p.fid) for p in parts], [p.pairs for p in parts],
                         [ptr(p.xs) for p in parts], [p.xs.numel() // 2 for p in parts],
                         [ptr(p.ovf) for p in parts], [p.ovf.numel() // 2 for p in parts], n,
                         row.data_ptr(), fid.data_ptr() if total else 0, ex.data_ptr())
    assert got == total, (got, total)
    return Merged(row, fid[:total], ex[:n])


class ShardedMatcher:
    """The filter-sharded match step of one rank: `eng` holds this rank's filter
    shard, `gid_map` (int32 device tensor) maps its local filter ids to global ids.

    ``run(batches)`` pipelines steps: while the engine walks batch k (emqxgm_match_device_submit
    on its own stream), rank 0 already broadcasts batch k+1 into the other of two receive buffers;
    then batch k's result goes to rank 0 in the wire form and is merged there.  The batch shape
    (bytes, topics) is given to every rank, so no size message precedes a broadcast."""

    def __init__(self, eng, gid_map: torch.Tensor, device, group=None, root: int = 0,
                 n_global: int = 1 << 32):
        self.eng = eng
        self.gid_map = gid_map
        self.device = device
        self.group = group
        self.root = root
        self.n_global = n_global  # global filter ids < n_global (24-bit ids when <= 2^24)
        self._wire = None
        self.bytes_to_root = 0   # per step, summed over the ranks that send (set on the root)
        self.bytes_broadcast = 0

    def _wire_bufs(self, n: int, pairs: int):
        cap_n, cap_p = (0, 0) if self._wire is None else (self._wire[2].numel() // 2, self._wire[1].numel() // 4)
        if n > cap_n or pairs > cap_p:
            n2, p2 = max(n, cap_n, 64), max(pairs, cap_p, 1)
            self._wire = (torch.empty(n2 + 64, dtype=torch.uint8, device=self.device),
                          torch.empty(4 * p2, dtype=torch.uint8, device=self.device),
                          torch.empty(2 * n2, dtype=torch.int32, device=self.device),
                          torch.empty(2 * n2, dtype=torch.int32, device=self.device))
        return self._wire

    def _bcast(self, tb, to, shape):
        nb, nt = shape
        cpu = _comm_on_cpu(self.group)
        cdev = "cpu" if cpu else self.device
        if dist.get_rank(self.group) == self.root:
            b, o = tb.to(cdev), to.to(cdev)
        else:
            b = torch.empty(nb, dtype=torch.uint8, device=cdev)
            o = torch.empty(nt + 1, dtype=torch.int32, device=cdev)
        if nb:
            dist.broadcast(b, self.root, group=self.group)
        dist.broadcast(o, self.root, group=self.group)
        self.bytes_broadcast = (nb + 4 * (nt + 1)) * (dist.get_world_size(self.group) - 1)
        return b.to(self.device), o.to(self.device)

    def _finish(self, ticket, n: int) -> Optional[Merged]:
        r = self.eng.match_device_wait(ticket)
        cnt, fid, xs, ovf = self._wire_bufs(n, r.n_pairs)
        fl = wire_flags(n, r.n_pairs, self.n_global)
        nc, nf = wire_sizes(fl, n, r.n_pairs)
        nx, no = self.eng.export_wire(r, self.gid_map.data_ptr(), fl, cnt.data_ptr() if n else 0,
                                      fid.data_ptr() if r.n_pairs else 0, xs.data_ptr(),
                                      ovf.data_ptr())
        part = WirePart(fl, r.n_pairs, cnt[:nc], fid[:nf], xs[:2 * nx], ovf[:2 * no])
        parts = gather_wire_to_root(part, self.root, self.group)
        if parts is None:
            return None
        self.bytes_to_root = sum(p.nbytes() for i, p in enumerate(parts) if i != self.root)
        return merge_wire(self.eng, parts, n)

    def run(self, batches, shapes):
        """Yields the merged result of every batch on the root (None elsewhere).  `batches`:
        (bytes, offsets) tensors per step on the root (ignored elsewhere); `shapes`: (bytes,
        topics) per step on every rank."""
        it = iter(batches)
        shapes = list(shapes)
        b, o = self._bcast(*next(it), shapes[0])
        for k, (nb, nt) in enumerate(shapes):
            torch.cuda.current_stream(self.device).synchronize()  # batch k is in HBM
            ticket = self.eng.match_device_submit(b.data_ptr(), o.data_ptr(), nt, nb)
            nxt = None
            if k + 1 < len(shapes):  # batch k+1 crosses xGMI while the engine walks batch k
                nxt = self._bcast(*next(it), shapes[k + 1])
            yield self._finish(ticket, nt)
            if nxt is not None:
                b, o = nxt

    def step(self, tbytes: Optional[torch.Tensor], toff: Optional[torch.Tensor], shape) -> Optional[Merged]:
        """One batch: broadcast, match this shard, wire to root, merge there."""
        return next(self.run([(tbytes, toff)], [shape]))


# ---- shard="keys": plain route keys partitioned by key hash, wildcard filters on every rank ----

def key_shard_filters(eng, fbytes: np.ndarray, foff: np.ndarray, fwild: np.ndarray,
                      world: int, rank: int) -> np.ndarray:
    """Global indices of the filters rank `rank` holds in the key-partitioned layout: every
    wildcard filter, and the plain route keys whose owner (emqxgm_key_owners, over the packed
    filters as they are) is `rank`."""
    wild = np.asarray(fwild).astype(bool)
    if world == 1:
        return np.arange(len(wild))
    own = eng.key_owners(fbytes, np.asarray(foff, np.uint64), world)
    return np.nonzero(wild | (own == rank))[0]


def gather_dense_to_root(part: Part, root: int = 0, group=None) -> Optional[List[Part]]:
    """Each rank's dense part (row [n+1], fid [pairs], exact [n]; int32 device tensors) to
    `root`: the pair counts by one all_gather, then sized point-to-point receives."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    row, fid, ex = part
    dev = row.device
    cdev = "cpu" if _comm_on_cpu(group) else dev
    mine = torch.tensor([fid.numel()], dtype=torch.int64, device=cdev)
    allp = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(world)]
    dist.all_gather(allp, mine, group=group)
    if rank != root:
        ops = [dist.P2POp(dist.isend, t.to(cdev), root, group) for t in (row, fid, ex) if t.numel()]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        return None
    out, ops = [], []
    for r in range(world):
        if r == root:
            out.append(part)
            continue
        q = (torch.empty_like(row, device=cdev), torch.empty(int(allp[r]), dtype=torch.int32, device=cdev),
             torch.empty_like(ex, device=cdev))
        ops += [dist.P2POp(dist.irecv, t, r, group) for t in q if t.numel()]
        out.append(q)
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return [tuple(t.to(dev) for t in q) for q in out]


class KeyShardedMatcher:
    """One rank of the key-partitioned layout (shard="keys"): `eng` holds every wildcard filter
    and this rank's plain route keys (``key_shard_filters``), `gid_map` (int32 device tensor)
    maps its local ids to global ones.  ``step`` broadcasts a batch from the root, matches this
    rank's topic block and probes the names it owns, and merges every rank's part on the root."""

    def __init__(self, eng, gid_map: torch.Tensor, device, group=None, root: int = 0):
        self.eng = eng
        self.gid_map = gid_map.to(torch.int64)
        self.device = device
        self.group = group
        self.root = root
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def _global(self, ids: torch.Tensor) -> torch.Tensor:
        """local ids (int32, NONE = -1) -> global ids (int32 bits)"""
        hit = ids != -1
        g = torch.full_like(ids, -1)
        g[hit] = self.gid_map[ids[hit].to(torch.int64)].to(torch.int32)
        return g

    def part(self, b: torch.Tensor, o: torch.Tensor, n: int) -> Part:
        """This rank's dense part of a batch already in HBM (bytes u8, offsets i32 [n+1])."""
        G, r = self.world, self.rank
        b0, b1 = n * r // G, n * (r + 1) // G
        lo, hi = (int(x) for x in o[[b0, b1]].tolist())
        bo = (o[b0:b1 + 1] - lo).contiguous()
        bb = b[lo:hi].contiguous() if hi > lo else torch.zeros(1, dtype=torch.uint8, device=self.device)
        own = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        torch.cuda.current_stream(self.device).synchronize()
        self.eng.exact_owned_device(b.data_ptr(), o.data_ptr(), n, G, r, own.data_ptr())
        res = self.eng.match_device(bb.data_ptr(), bo.data_ptr(), b1 - b0, hi - lo)
        m = b1 - b0
        brow = torch.empty(m + 1, dtype=torch.int32, device=self.device)
        bfid = torch.empty(max(res.n_pairs, 1), dtype=torch.int32, device=self.device)
        bex = torch.empty(max(m, 1), dtype=torch.int32, device=self.device)
        self.eng.export(res, 0, brow.data_ptr(), bfid.data_ptr(), bex.data_ptr())
        row = torch.empty(n + 1, dtype=torch.int32, device=self.device)
        row[:b0 + 1] = 0
        row[b0:b1 + 1] = brow
        row[b1 + 1:] = brow[m]
        fid = self._global(bfid[:res.n_pairs])
        ex = self._global(own[:n])
        if m:
            blk = self._global(bex[:m])
            ex[b0:b1] = torch.where(ex[b0:b1] != -1, ex[b0:b1], blk)
        return row, fid, ex

    def step(self, tbytes: Optional[torch.Tensor], toff: Optional[torch.Tensor], shape) -> Optional[Merged]:
        nb, nt = shape
        cdev = "cpu" if _comm_on_cpu(self.group) else self.device
        if self.rank == self.root:
            b, o = tbytes.to(cdev), toff.to(cdev)
        else:
            b = torch.empty(nb, dtype=torch.uint8, device=cdev)
            o = torch.empty(nt + 1, dtype=torch.int32, device=cdev)
        if nb:
            dist.broadcast(b, self.root, group=self.group)
        dist.broadcast(o, self.root, group=self.group)
        p = self.part(b.to(self.device), o.to(self.device), nt)
        parts = gather_dense_to_root(p, self.root, self.group)
        if parts is None:
            return None
        return merge_parts(self.eng, parts, nt)
