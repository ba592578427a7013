"""world_size-2 gloo test of the filter-sharded layout's collective protocol (emqx_amd/dist.py)
on CPU.

Each rank holds one filter shard; rank 0 broadcasts the topic batch, every rank matches it
against its shard, the pair counts are all-gathered and every rank's CSR reaches rank 0 through
sized point-to-point receives; merged there, it must equal the unsharded answer.  The per-rank
matcher is the oracle and the merge a torch restatement of emqxgm_merge (no GPU in this
container); on the GPU box bench.py runs the same collective code with the HIP engine (match,
export, merge) and RCCL, and tests/test_gpu_dist.py checks emqxgm_merge against _ref_merge."""
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
        # rank 1 sends a padded fid buffer: only its first n_pairs entries may travel
        pad = np.concatenate([gid, np.full(7, 12345, np.uint32)])
        parts = D.gather_to_root(i32(row), i32(pad if rank else gid), i32(exg), len(gid))
        if rank != 0:
            assert parts is None
        else:
            merged = _ref_merge(parts, w.nt)
        if rank == 0:
            assert [p[1].numel() for p in parts][1] == parts_len(parts[1])
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
