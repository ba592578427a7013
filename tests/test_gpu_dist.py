"""The filter-sharded layout's device side (emqx_amd/dist.py): emqxgm_export /
emqxgm_export_wire (a shard's result with global ids, dense or in the compact wire form) and
emqxgm_merge / emqxgm_merge_wire (G shards merged topic by topic on the device), checked against
tests/test_dist.py's restatements, and the pipelined ShardedMatcher rehearsed with two ranks
sharing this box's GPU (gloo: RCCL refuses two ranks on one device) against the unsharded
oracle."""
import os
import socket

import numpy as np
import pytest
import torch

from tests.test_dist import _ref_export_wire, _ref_merge, _ref_merge_wire, _subset

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def emqx():
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def _rand_part(rng, n, nf, has_exact):
    cnt = rng.integers(0, 5, n)
    row = np.zeros(n + 1, np.uint32)
    np.cumsum(cnt, out=row[1:])
    fid = rng.integers(0, nf, int(row[-1])).astype(np.uint32)
    ex = np.where(has_exact, rng.integers(0, nf, n), 0xFFFFFFFF).astype(np.uint32)
    t = lambda a: torch.from_numpy(a.view(np.int32)).cuda()  # noqa: E731
    return t(row), t(fid), t(ex)


def test_merge_matches_reference(emqx):
    from emqx_amd import dist as D
    eng = emqx.Engine()
    rng = np.random.default_rng(1)
    for n, g in ((0, 2), (1, 1), (1000, 3), (70000, 8)):
        owner = rng.integers(-1, g, n)  # which shard (if any) holds the topic's exact key
        parts = [_rand_part(rng, n, 10 ** 6, owner == r) for r in range(g)]
        m = D.merge_parts(eng, parts, n)
        cpu = [tuple(x.cpu() for x in p) for p in parts]
        row, fid, ex = _ref_merge(cpu, n)
        assert np.array_equal(m.row_ptr.cpu().numpy().view(np.uint32).astype(np.int64), row)
        assert np.array_equal(m.filter_id.cpu().numpy().view(np.uint32).astype(np.int64), fid)
        assert np.array_equal(m.exact_id.cpu().numpy().view(np.uint32).astype(np.int64), ex)
    eng.close()


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_merge_wire_matches_reference(emqx, flags):
    """Wire parts (counts beyond the width through the overflow list, 24-bit id planes) merged on
    the device equal the restatement, and equal emqxgm_merge over the same parts in dense form."""
    from emqx_amd import dist as D
    eng = emqx.Engine()
    rng = np.random.default_rng(2 + flags)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for n, g in ((0, 2), (1, 1), (1000, 3), (70000, 8)):
        owner = rng.integers(-1, g, n)
        wires, dense, parts = [], [], []
        for r in range(g):
            cnt = rng.integers(0, 4, n)
            if n:
                cnt[rng.integers(0, n, 5)] = rng.integers(255, 600, 5)
            row = np.zeros(n + 1, np.uint32)
            np.cumsum(cnt, out=row[1:])
            gid = rng.integers(0, 1 << 24 if flags & 2 else 10 ** 9, int(row[-1])).astype(np.uint32)
            exg = np.where(owner == r, rng.integers(0, 10 ** 6, n), 0xFFFFFFFF).astype(np.uint32)
            cb, fb, x, o = _ref_export_wire(row, gid, exg, flags)
            wires.append((flags, len(gid), cb, fb, x, o))
            dense.append(tuple(cu(a.view(np.int32)) for a in (row, gid, exg)))
            parts.append(D.WirePart(flags, len(gid), cu(cb), cu(fb), cu(x.view(np.int32)),
                                    cu(o.view(np.int32))))
        m = D.merge_wire(eng, parts, n)
        row, fid, ex = _ref_merge_wire(wires, n)
        assert np.array_equal(m.row_ptr.cpu().numpy().view(np.uint32).astype(np.int64), row)
        assert np.array_equal(m.filter_id.cpu().numpy().view(np.uint32).astype(np.int64), fid)
        assert np.array_equal(m.exact_id.cpu().numpy().view(np.uint32).astype(np.int64), ex)
        md = D.merge_parts(eng, dense, n)
        assert torch.equal(md.row_ptr, m.row_ptr) and torch.equal(md.filter_id, m.filter_id)
        assert torch.equal(md.exact_id, m.exact_id)
    eng.close()


@pytest.mark.parametrize("flags", [0, 3])
def test_export_wire_matches_restatement(emqx, flags):
    import workloads
    w = workloads.generate(2, 30000, 4000)
    eng = emqx.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.nonzero(w.fwild)[0]
    wb, wo = _subset(w, wi)
    eng.trie_insert_many(wb, wo)
    eng.commit()
    db = torch.from_numpy(w.tbytes).cuda()
    do = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    r = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, int(w.toff[-1]))
    row = torch.empty(w.nt + 1, dtype=torch.int32, device="cuda")
    fid = torch.empty(r.n_pairs, dtype=torch.int32, device="cuda")
    ex = torch.empty(w.nt, dtype=torch.int32, device="cuda")
    eng.export(r, 0, row.data_ptr(), fid.data_ptr(), ex.data_ptr())
    c8 = torch.empty(w.nt + 64, dtype=torch.uint8, device="cuda")
    f2 = torch.empty(4 * r.n_pairs, dtype=torch.uint8, device="cuda")
    xs = torch.empty(2 * w.nt, dtype=torch.int32, device="cuda")
    ov = torch.empty(2 * w.nt, dtype=torch.int32, device="cuda")
    nx, no = eng.export_wire(r, 0, flags, c8.data_ptr(), f2.data_ptr(), xs.data_ptr(), ov.data_ptr())
    u = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
    c, f, x, o = _ref_export_wire(u(row), u(fid), u(ex), flags)
    assert np.array_equal(c8.cpu().numpy()[:len(c)], c) and np.array_equal(f2.cpu().numpy()[:len(f)], f)
    assert nx == len(x) // 2 and no == len(o) // 2 and nx > 0
    key = lambda a: sorted(map(tuple, a.reshape(-1, 2).tolist()))  # noqa: E731
    assert key(u(xs)[:2 * nx]) == key(x) and key(u(ov)[:2 * no]) == key(o)
    eng.close()


def test_export_maps_ids(emqx):
    eng = emqx.Engine()
    fs = [b"a/+", b"a/#", b"+/b", b"a/b"]
    ids = [eng.trie_insert(f) for f in fs[:3]] + [eng.route_ref(fs[3])]
    eng.commit()
    topics = [b"a/b", b"a/c", b"x/b", b"q"]
    buf, off = emqx.engine.pack(topics, np.uint32)
    db = torch.from_numpy(buf).cuda()
    do = torch.from_numpy(off.view(np.int32)).cuda()
    torch.cuda.synchronize()
    r = eng.match_device(db.data_ptr(), do.data_ptr(), len(topics), int(off[-1]))
    gmap = np.full(max(ids) + 1, 0xFFFFFFFF, np.uint32)
    gmap[ids] = [100, 200, 300, 400]
    gm = torch.from_numpy(gmap.view(np.int32)).cuda()
    row = torch.empty(len(topics) + 1, dtype=torch.int32, device="cuda")
    fid = torch.empty(r.n_pairs, dtype=torch.int32, device="cuda")
    ex = torch.empty(len(topics), dtype=torch.int32, device="cuda")
    eng.export(r, gm.data_ptr(), row.data_ptr(), fid.data_ptr(), ex.data_ptr())
    row, fid = row.cpu().numpy(), fid.cpu().numpy().view(np.uint32)
    rows = [sorted(fid[row[i]:row[i + 1]].tolist()) for i in range(len(topics))]
    assert rows == [[100, 200, 300], [100, 200], [300], []]
    assert ex.cpu().numpy().view(np.uint32).tolist() == [400, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF]
    eng.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, backend="gloo", shape=(2, 30000, 5000)):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # nccl (= RCCL): one GPU per rank; gloo: both ranks on GPU 0 (RCCL refuses that)
    gpu = rank if backend == "nccl" else 0
    torch.cuda.set_device(gpu)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import workloads
        from emqx_amd import Engine
        from emqx_amd import dist as D
        from oracle.cref import RefIndex
        dev = torch.device("cuda", gpu)
        w = workloads.generate(*shape)
        mine = np.nonzero(D.filter_shards(w.fbytes, w.foff, world) == rank)[0]
        fb, fo = _subset(w, mine)
        eng = Engine(device=gpu)
        rid = eng.route_ref_many(fb, fo)
        wsel = np.nonzero(w.fwild[mine])[0]
        wb, wo = _subset(type("W", (), {"fbytes": fb, "foff": fo})(), wsel)
        tid = eng.trie_insert_many(wb, wo)
        eng.commit()
        gid = np.full(int(max(rid.max(), tid.max(initial=0))) + 1, 0xFFFFFFFF, np.uint32)
        gid[rid] = mine
        gid[tid] = mine[wsel]
        sm = D.ShardedMatcher(eng, torch.from_numpy(gid.view(np.int32)).to(dev), dev, n_global=w.nf)
        tb = torch.from_numpy(w.tbytes).to(dev) if rank == 0 else None
        to = torch.from_numpy(w.toff.view(np.int32)).to(dev) if rank == 0 else None
        shape = (int(w.toff[-1]), w.nt)
        # three pipelined steps (batch k+1 broadcast while batch k is walked; buffers reused)
        ms = list(sm.run([(tb, to)] * 3, [shape] * 3))
        m = ms[-1]
        if rank == 0:
            assert all(x is not None for x in ms) and sm.bytes_to_root > 0
            full = RefIndex(True)
            full.add_many(w.fbytes, w.foff, 2 + w.fwild)
            frow, fids, fex = full.match(w.tbytes, w.toff)
            row = m.row_ptr.cpu().numpy().astype(np.int64)
            got = m.filter_id.cpu().numpy().view(np.uint32)
            ok = np.array_equal(row, frow.astype(np.int64))
            for t in range(w.nt):
                a, b = int(frow[t]), int(frow[t + 1])
                ok = ok and np.array_equal(np.sort(got[a:b]), fids[a:b])
            ok = ok and np.array_equal(m.exact_id.cpu().numpy().view(np.uint32), fex)
            q.put(("ok" if ok else "mismatch", int(frow[-1]), len(mine)))
        else:
            assert m is None
        eng.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_sharded_matcher_two_ranks(emqx, backend):
    """gloo: two ranks sharing this box's GPU; nccl: the RCCL branch, one rank per GPU -- run
    where two GPUs are visible (the driver's multi-GPU node), skipped on a one-GPU box."""
    if backend == "nccl" and torch.cuda.device_count() < 2:
        pytest.skip("the RCCL branch needs two GPUs (this box has one)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, backend)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(360)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, pairs, on_rank0 = q.get(timeout=5)
    assert status == "ok", status
    assert pairs > 0 and on_rank0 > 0


@pytest.mark.timeout(900)
@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_sharded_matcher_cfg3_slice_every_gpu(emqx, backend):
    """The north-star layout at a BASELINE shape: a 1M-filter slice of cfg3
    (site/+/device/+/#) sharded by filter hash, 200k topics broadcast, the wire results merged on
    rank 0 -- every row and exact id equal to the unsharded oracle's (oracle/ref_trie.cpp).  nccl:
    one rank per GPU over RCCL on every GPU of the node (up to 8), skipped on a one-GPU box (the
    first multi-GPU GPUTEST pins it); gloo: the same control flow with two ranks sharing this
    box's GPU."""
    world = 2 if backend == "gloo" else min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("the RCCL branch needs two or more GPUs (this box has one)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, backend, (3, 1_000_000, 200_000)))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(840)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, pairs, on_rank0 = q.get(timeout=5)
    assert status == "ok", status
    assert pairs > 50_000 and on_rank0 > 0


def _rank_keys(rank, world, port, q, backend="gloo", shape=(4, 404_000, 50_000)):
    """One rank of the key-partitioned layout (dist.KeyShardedMatcher): every wildcard filter and
    this rank's plain route keys; the merged result on rank 0 against the unsharded oracle."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpu = rank if backend == "nccl" else 0
    torch.cuda.set_device(gpu)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import workloads
        from emqx_amd import Engine
        from emqx_amd import dist as D
        from oracle.cref import RefIndex
        dev = torch.device("cuda", gpu)
        w = workloads.generate(*shape)
        eng = Engine(device=gpu)
        mine = D.key_shard_filters(eng, w.fbytes, w.foff, w.fwild, world, rank)
        fb, fo = _subset(w, mine)
        rid = eng.route_ref_many(fb, fo)
        wsel = np.nonzero(w.fwild[mine])[0]
        wb, wo = _subset(type("W", (), {"fbytes": fb, "foff": fo})(), wsel)
        tid = eng.trie_insert_many(wb, wo)
        eng.commit()
        gid = np.full(int(max(rid.max(), tid.max(initial=0))) + 1, 0xFFFFFFFF, np.uint32)
        gid[rid] = mine
        gid[tid] = mine[wsel]
        km = D.KeyShardedMatcher(eng, torch.from_numpy(gid.view(np.int32)).to(dev), dev)
        tb = torch.from_numpy(w.tbytes).to(dev) if rank == 0 else None
        to = torch.from_numpy(w.toff.view(np.int32)).to(dev) if rank == 0 else None
        m = km.step(tb, to, (int(w.toff[-1]), w.nt))
        if rank == 0:
            full = RefIndex(True)
            full.add_many(w.fbytes, w.foff, 2 + w.fwild)
            frow, fids, fex = full.match(w.tbytes, w.toff)
            row = m.row_ptr.cpu().numpy().astype(np.int64)
            got = m.filter_id.cpu().numpy().view(np.uint32)
            ok = np.array_equal(row, frow.astype(np.int64))
            for t in range(w.nt):
                a, b = int(frow[t]), int(frow[t + 1])
                ok = ok and np.array_equal(np.sort(got[a:b]), fids[a:b])
            gx = m.exact_id.cpu().numpy().view(np.uint32)
            ok = ok and np.array_equal(gx, fex)
            q.put(("ok" if ok else "mismatch", int((fex != 0xFFFFFFFF).sum()), len(mine)))
        else:
            assert m is None
        eng.close()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("error", repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_key_sharded_matcher_cfg4_shape(emqx, backend):
    """SURVEY 8e's alternative for cfg4: plain route keys partitioned by key
    hash, wildcard filters on every rank; each name's route key probed by its owner only, each
    topic's trie walk by its block's rank; the merged rows and exact ids equal the unsharded
    oracle's (cfg4 shape: 400k exact keys + 4k wildcards, 50k topics, 90% exact hits).  gloo:
    two ranks sharing this box's GPU; nccl: every GPU of the node (skipped on one)."""
    world = 2 if backend == "gloo" else min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("the RCCL branch needs two or more GPUs (this box has one)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_keys, args=(r, world, port, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(560)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    status, hits, on_rank0 = q.get(timeout=5)
    assert status == "ok", status
    assert hits > 40_000 and 0 < on_rank0 < 404_000


def test_key_owners_partition(emqx):
    """emqxgm_key_owners splits keys evenly and every key has one owner; the owned-name probe
    finds exactly the owned keys' ids."""
    eng = emqx.Engine()
    keys = [b"dev/%09d/state" % i for i in range(20000)]
    buf, off = emqx.engine.pack(keys)
    own = eng.key_owners(buf, off, 4)
    assert set(own.tolist()) == {0, 1, 2, 3} and np.bincount(own).min() > 4500
    assert (eng.key_owners(buf, off, 1) == 0).all()
    mine = [k for k, o in zip(keys, own) if o == 1]
    ids = {eng.route_ref(k): k for k in mine}
    eng.commit()
    names = keys[:3000] + [b"x/y", b""]
    nb, no = emqx.engine.pack(names, np.uint32)
    db = torch.from_numpy(nb).cuda()
    do = torch.from_numpy(no.view(np.int32)).cuda()
    out = torch.empty(len(names), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    eng.exact_owned_device(db.data_ptr(), do.data_ptr(), len(names), 4, 1, out.data_ptr())
    got = out.cpu().numpy().view(np.uint32)
    want = [next((i for i, k in ids.items() if k == nm), 0xFFFFFFFF) for nm in names]
    assert got.tolist() == want
    eng.close()
