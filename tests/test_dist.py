"""world_size-2 gloo test of the filter-sharded layout's collective protocol (emqx_amd/dist.py)
on CPU.

Each rank holds one filter shard; rank 0 broadcasts the topic batch, every rank matches it
against its shard and puts the result in the compact wire form (u8 counts, global ids, sparse
exact hits and overflow counts), the lengths are all-gathered and every rank's part reaches
rank 0 through sized point-to-point receives; merged there, it must equal the unsharded answer.
The per-rank matcher is the oracle, the wire export and the merge numpy restatements of
emqxgm_export_wire / emqxgm_merge_wire (no GPU in this container); on the GPU box bench.py runs
the same collective code with the HIP engine and RCCL, and tests/test_gpu_dist.py checks the
HIP export / merge against these restatements."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _subset(w, idx):
    lens = (w.foff[idx + 1] - w.foff[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    starts = w.foff[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
    return w.fbytes[pos], off


def _ref_merge(parts, n):
    """Torch restatement of emqxgm_merge (gm_kernels.hip k_merge_*): topic t's row is shard 0's
    row, then shard 1's, ...; the exact id the one shard's that has it.  Returns int64 numpy
    (row [n+1], fid, exact)."""
    u = [(p[0].numpy().view(np.uint32).astype(np.int64), p[1].numpy().view(np.uint32).astype(np.int64),
          p[2].numpy().view(np.uint32).astype(np.int64)) for p in parts]
    cnt = sum(np.diff(r) for r, _, _ in u)
    row = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=row[1:])
    fid = np.empty(int(row[-1]), np.int64)
    for t in range(n):
        d = int(row[t])
        for r, f, _ in u:
            seg = f[int(r[t]):int(r[t + 1])]
            fid[d:d + len(seg)] = seg
            d += len(seg)
    ex = np.min(np.stack([e for _, _, e in u]), axis=0)
    return row, fid, ex


def parts_len(p):
    return int(p[0][-1])


def _ref_export_wire(row, gid, exg, flags=0):
    """numpy restatement of emqxgm_export_wire (gm_kernels.hip k_wire_export): counts as u8
    (255: see ovf) or, flags & 1, as two bit planes of 64 topics (3: see ovf); ids as u32 or,
    flags & 2, as u16 low halves then u8 high bytes; (topic, exact id) and (topic, count) pairs
    (any order).  Returns (cnt bytes, fid bytes, xs, ovf)."""
    cnt = np.diff(row.astype(np.int64))
    n = len(cnt)
    t = np.arange(n, dtype=np.int64)
    cap = 3 if flags & 1 else 255
    hit, big = exg != 0xFFFFFFFF, cnt >= cap
    xs = np.stack([t[hit], exg[hit].astype(np.int64)], 1).reshape(-1)
    ovf = np.stack([t[big], cnt[big]], 1).reshape(-1)
    if flags & 1:
        code = np.zeros(((n + 63) // 64) * 64, np.uint64)
        code[:n] = np.minimum(cnt, 3)
        g = code.reshape(-1, 64)
        w = (np.uint64(1) << np.arange(64, dtype=np.uint64))
        p0 = ((g & np.uint64(1)) * w).sum(1, dtype=np.uint64)
        p1 = (((g >> np.uint64(1)) & np.uint64(1)) * w).sum(1, dtype=np.uint64)
        cb = np.stack([p0, p1], 1).reshape(-1).view(np.uint8)
    else:
        cb = np.minimum(cnt, 255).astype(np.uint8)
    gid = gid.astype(np.uint32)
    fb = (np.concatenate([(gid & 0xFFFF).astype(np.uint16).view(np.uint8), (gid >> 16).astype(np.uint8)])
          if flags & 2 else gid.view(np.uint8))
    return cb, fb, xs.astype(np.uint32), ovf.astype(np.uint32)


def _ref_merge_wire(parts, n):
    """numpy restatement of emqxgm_merge_wire over (flags, pairs, cnt bytes, fid bytes, xs, ovf)
    parts: each part's rows from its counts and overflow list, its ids widened, the exact ids
    from the sparse pairs, then _ref_merge."""
    dense = []
    ex = np.full(n, 0xFFFFFFFF, np.uint32)
    for flags, pairs, cb, fb, xs, ovf in parts:
        if flags & 1:
            pl = cb.view(np.uint64).reshape(-1, 2)
            b = np.arange(n, dtype=np.uint64)
            g = (b >> np.uint64(6)).astype(np.int64)
            sh = b & np.uint64(63)
            cnt = (((pl[g, 0] >> sh) & np.uint64(1)) | (((pl[g, 1] >> sh) & np.uint64(1)) << np.uint64(1))).astype(np.int64)
        else:
            cnt = cb.astype(np.int64)
        o = ovf.reshape(-1, 2).astype(np.int64)
        cnt[o[:, 0]] = o[:, 1]
        row = np.zeros(n + 1, np.int64)
        np.cumsum(cnt, out=row[1:])
        fid = (fb[:2 * pairs].view(np.uint16).astype(np.uint32) | (fb[2 * pairs:].astype(np.uint32) << 16)
               if flags & 2 else fb.view(np.uint32))
        x = xs.reshape(-1, 2).astype(np.int64)
        ex[x[:, 0]] = x[:, 1]
        dense.append((row, fid))
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))  # noqa: E731
    return _ref_merge([(i32(r), i32(f), i32(ex)) for r, f in dense], n)


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_wire_restatement_round_trip(flags):
    """Counts the width cannot hold go through the overflow list; exact ids through the sparse
    pairs; 24-bit ids through the two planes."""
    rng = np.random.default_rng(5 + flags)
    n = 3000
    parts_dense, parts_wire = [], []
    owner = rng.integers(-1, 3, n)
    for r in range(3):
        cnt = rng.integers(0, 4, n)
        cnt[rng.integers(0, n, 20)] = rng.integers(250, 700, 20)
        row = np.zeros(n + 1, np.uint32)
        np.cumsum(cnt, out=row[1:])
        gid = rng.integers(0, 1 << 24 if flags & 2 else 1 << 32, int(row[-1])).astype(np.uint32)
        exg = np.where(owner == r, rng.integers(0, 10 ** 6, n), 0xFFFFFFFF).astype(np.uint32)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))  # noqa: E731
        parts_dense.append((i32(row), i32(gid), i32(exg)))
        parts_wire.append((flags, len(gid)) + _ref_export_wire(row, gid, exg, flags))
    a, b = _ref_merge(parts_dense, n), _ref_merge_wire(parts_wire, n)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert sum(len(w[5]) for w in parts_wire) > 0  # overflow entries were exercised


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import workloads
        from emqx_amd import dist as D
        from oracle.cref import RefIndex
        w = workloads.generate(2, 20000, 3000)
        shard = D.filter_shards(w.fbytes, w.foff, world)
        mine = np.nonzero(shard == rank)[0]
        fb, fo = _subset(w, mine)
        kinds = 2 + w.fwild[mine]
        ref = RefIndex(True)
        ref.add_many(fb, fo, kinds)
        tb = torch.from_numpy(w.tbytes) if rank == 0 else None
        to = torch.from_numpy(w.toff.view(np.int32)) if rank == 0 else None
        tb, to = D.broadcast_batch(tb, to, "cpu")
        row, ids, ex = ref.match(tb.numpy(), to.numpy().view(np.uint32))
        gid = mine[ids.astype(np.int64)].astype(np.uint32)
        exg = np.where(ex == D.NONE, D.NONE, mine[np.minimum(ex, len(mine) - 1).astype(np.int64)])
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))  # noqa: E731
        fl = D.wire_flags(w.nt, len(gid), w.nf) if rank == 0 else 3  # rank 1: the sparse form
        cb, fb, xs, ovf = _ref_export_wire(row, gid, exg.astype(np.uint32), fl)
        part = D.WirePart(fl, len(gid), torch.from_numpy(cb), torch.from_numpy(fb), i32(xs), i32(ovf))
        parts = D.gather_wire_to_root(part)
        if rank != 0:
            assert parts is None
        else:
            u = lambda t: t.numpy().view(np.uint32) if t.dtype == torch.int32 else t.numpy()  # noqa: E731
            merged = _ref_merge_wire([(p.flags, p.pairs) + tuple(u(t) for t in (p.cnt, p.fid, p.xs, p.ovf))
                                      for p in parts], w.nt)
            p1 = parts[1]
            assert p1.flags == 3 and p1.nbytes() == (16 * ((w.nt + 63) // 64) + 3 * p1.pairs
                                                     + 4 * (p1.xs.numel() + p1.ovf.numel()))
            full = RefIndex(True)
            full.add_many(w.fbytes, w.foff, 2 + w.fwild)
            frow, fids, fex = full.match(w.tbytes, w.toff)
            ok = np.array_equal(merged[0], frow.astype(np.int64))
            got = merged[1]
            for t in range(w.nt):
                a, b = int(frow[t]), int(frow[t + 1])
                ok = ok and np.array_equal(np.sort(got[a:b]), fids[a:b].astype(np.int64))
            ok = ok and np.array_equal(merged[2], fex.astype(np.int64))
            assert int(frow[-1]) > 0 and (fex != D.NONE).any()
            q.put(("ok" if ok else "mismatch", int(shard.sum()), len(shard)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_filter_sharded_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, on_rank1, total = q.get(timeout=5)
    assert status == "ok", status
    assert 0 < on_rank1 < total  # both shards hold filters


def test_filter_shards_stable_and_balanced():
    from emqx_amd import dist as D
    from emqx_amd.engine import pack
    fs = [f"site/{i}/device/{j}/#".encode() for i in range(100) for j in range(100)] + [b""]
    fb, fo = pack(fs)
    for world in (2, 4, 8):
        s = D.filter_shards(fb, fo, world)
        assert s.min() >= 0 and s.max() < world
        counts = np.bincount(s, minlength=world)
        assert counts.min() > 0.8 * len(fs) / world
        assert np.array_equal(s, D.filter_shards(fb, fo, world))


def _worker_keys(rank, world, port, q, libpath):
    """The key-partitioned layout (dist.KeyShardedMatcher, shard="keys") with the oracle as each
    rank's matcher: rank r holds every wildcard filter and the plain keys emqxgm_key_owners gives
    it (the engine's host code, on the fake HIP runtime); its part is its topic block's rows and
    the exact ids of the names it owns; gather_dense_to_root brings the parts to rank 0, whose
    merge (the restatement of emqxgm_merge) must equal the unsharded answer."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import workloads
        from emqx_amd import dist as D
        from emqx_amd.engine import Engine, load_library
        from oracle.cref import RefIndex
        eng = Engine(library=load_library(libpath, allow_missing=True))
        w = workloads.generate(4, 40_400, 6000)
        mine = D.key_shard_filters(eng, w.fbytes, w.foff, w.fwild, world, rank)
        assert w.fwild[mine].sum() == w.fwild.sum()  # every wildcard filter on every rank
        fb, fo = _subset(w, mine)
        ref = RefIndex(True)
        ref.add_many(fb, fo, 2 + w.fwild[mine])
        tb = torch.from_numpy(w.tbytes) if rank == 0 else None
        to = torch.from_numpy(w.toff.view(np.int32)) if rank == 0 else None
        tb, to = D.broadcast_batch(tb, to, "cpu")
        tbn, ton = tb.numpy(), to.numpy().view(np.uint32)
        n = len(ton) - 1
        b0, b1 = n * rank // world, n * (rank + 1) // world
        # the block's rows (local ids -> global)
        bo = (ton[b0:b1 + 1] - ton[b0]).astype(np.uint32)
        brow, bids, bex = ref.match(tbn[ton[b0]:ton[b1]], bo)
        # the owned names' exact ids: every name's, kept where this rank owns the name
        _, _, ex_all = ref.match(tbn, ton)
        names = [tbn[ton[t]:ton[t + 1]].tobytes() for t in range(n)]
        from emqx_amd.engine import pack
        nb, no = pack(names)
        own = eng.key_owners(nb, no, world)
        g = lambda a: np.where(a == D.NONE, D.NONE, mine[np.minimum(a, len(mine) - 1).astype(np.int64)]).astype(np.uint32)  # noqa: E731
        ex = np.where(own == rank, g(ex_all), D.NONE).astype(np.uint32)
        blk = g(bex)
        ex[b0:b1] = np.where(ex[b0:b1] != D.NONE, ex[b0:b1], blk)
        row = np.zeros(n + 1, np.uint32)
        row[b0:b1 + 1] = brow
        row[b1 + 1:] = brow[-1]
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))  # noqa: E731
        parts = D.gather_dense_to_root((i32(row), i32(g(bids)), i32(ex)))
        if rank != 0:
            assert parts is None
        else:
            merged = _ref_merge(parts, n)
            full = RefIndex(True)
            full.add_many(w.fbytes, w.foff, 2 + w.fwild)
            frow, fids, fex = full.match(w.tbytes, w.toff)
            ok = np.array_equal(merged[0], frow.astype(np.int64))
            for t in range(n):
                a, b = int(frow[t]), int(frow[t + 1])
                ok = ok and np.array_equal(np.sort(merged[1][a:b]), fids[a:b].astype(np.int64))
            ok = ok and np.array_equal(merged[2], fex.astype(np.int64))
            assert (fex != D.NONE).sum() > 4000 and int(frow[-1]) > 0
            q.put(("ok" if ok else "mismatch", len(mine), w.nf))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_key_sharded_world2_gloo():
    """the routing and the merge of the key-partitioned cfg4 layout."""
    from tests.test_route_mirror import build_fake_lib
    lib = build_fake_lib()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_keys, args=(r, 2, port, q, lib)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, on_rank0, total = q.get(timeout=5)
    assert status == "ok", status
    assert 0 < on_rank0 < total
