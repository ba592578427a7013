"""The NIF batcher core (emqxgm_batcher_*, include/emqx_gpumatch.h) on the device, driven the way
the emqx_trie_gpu NIF drives it (c_src/emqx_trie_gpu_nif.c): topics added one by one with the
caller's tag, a window flushed when full or due, the oldest window collected once
EMQXGM_HOST_PIPES are in flight.  Each topic's answer -- its exact route key plus its trie
filters' bytes -- expanded to routes equals emqx_router:match_routes/1 (emqx_router.erl:141-146)
of the oracle (oracle/emqx_ref.py Router; the C++ restatement for the cfg3 slice)."""
import random
import time

import numpy as np
import pytest

from oracle import emqx_ref as R
from oracle.cref import RefIndex

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def _drive(emqx, b, topics, pipes):
    """Adds every topic (tag = its index), flushing full windows and collecting the oldest
    window whenever `pipes` are in flight; returns {tag: (filters, exact_id)}."""
    out, inflight = {}, []

    def collect_oldest():
        w = b.collect(inflight.pop(0))
        for i in range(len(w.tag)):
            out[int(w.tag[i])] = (w.filters(i), int(w.exact_id[i]))

    def flush():
        if len(inflight) == pipes:
            collect_oldest()
        wid = b.flush()
        if wid:
            inflight.append(wid)

    for i, t in enumerate(topics):
        if b.add(t, i):
            flush()
        elif b.due(time.monotonic_ns()):
            flush()
    flush()
    while inflight:
        collect_oldest()
    return out


def test_batcher_cfg1_windows_match_routes(emqx):
    import workloads
    w = workloads.generate(1, None, 30_000)
    rng = random.Random(3)
    router, ref = emqx.Router(), R.Router()
    filters = [w.filter(i) for i in range(w.nf)]
    topics = [w.topic(i) for i in range(w.nt)]
    for f in filters:
        for d in rng.sample(["n1", "n2", ("g", "n1")], rng.randint(1, 2)):
            router.add_route(f, d)
            ref.add_route(f, d)
    for t in topics[::7]:  # exact routes: some published names have a route key of their own
        router.add_route(t, "n3")
        ref.add_route(t, "n3")
    router.commit()
    eng = router.engine
    b = emqx.Batcher(eng, window_topics=4096, window_us=200)
    res = _drive(emqx, b, topics, eng.HOST_PIPES)
    assert len(res) == len(topics)
    for i, t in enumerate(topics):
        fs, ex = res[i]
        # match_routes = lookup_routes(Topic) ++ lookup_routes(F) per trie match (:141-146);
        # the exact id says whether the topic itself is a route key
        routes = list(router.lookup_routes(t)) if ex != emqx.NONE else []
        assert (ex != emqx.NONE) == router.has_routes(t)
        for f in fs:
            routes += router.lookup_routes(f)
        assert sorted(map(repr, routes)) == sorted(map(repr, ref.match_routes(t))), t
    b.close()


def test_batcher_cfg3_slice_windows(emqx):
    import workloads
    w = workloads.generate(3, 1_000_000, 200_000)
    eng = emqx.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    eng.trie_insert_many(w.fbytes, w.foff)
    eng.commit()
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, (2 + w.fwild.astype(np.uint8)))
    row, ids, ex = ref.match(w.tbytes, w.toff, threads=16)
    topics = [w.topic(i) for i in range(w.nt)]
    b = emqx.Batcher(eng)  # the NIF's defaults: 65,536-topic windows, 50 us
    res = _drive(emqx, b, topics, eng.HOST_PIPES)
    for i in range(w.nt):
        fs, e = res[i]
        want = sorted(w.filter(int(x)) for x in ids[row[i]:row[i + 1]])
        assert sorted(fs) == want, topics[i]
        assert e == ex[i]  # ids coincide: both registered the filters in the same order
    b.close()


def test_batcher_protocol_edges(emqx):
    eng = emqx.Engine()
    for f in (b"a/+", b"a/#", b"#"):
        eng.route_ref(f)
        eng.trie_insert(f)
    eng.route_ref(b"a/b")
    eng.commit()
    b = emqx.Batcher(eng, window_topics=4, window_bytes=64, window_us=1000)
    assert b.flush() == 0  # empty window: nothing submitted
    assert not b.due(time.monotonic_ns() + 10**12)
    assert b.add(b"a/b", 7) is False and not b.due(time.monotonic_ns())
    assert b.due(time.monotonic_ns() + 2_000_000)
    for t in (b"a", b"", b"x/y"):
        full = b.add(t, 8)
    assert full is True
    with pytest.raises(emqx.EngineError, match="ENOSPC"):
        b.add(b"z", 9)
    with pytest.raises(emqx.EngineError, match="E2BIG"):
        b.add(b"q" * 65, 9)
    ws = [b.flush()]
    for k in range(eng.HOST_PIPES - 1):
        b.add(b"a/b/c", 10 + k)
        ws.append(b.flush())
    b.add(b"a/b", 20)
    with pytest.raises(emqx.EngineError, match="EBUSY"):
        b.flush()  # HOST_PIPES windows in flight: collect first
    w0 = b.collect(ws[0])
    assert list(w0.tag) == [7, 8, 8, 8]
    assert sorted(w0.filters(0)) == [b"#", b"a/#", b"a/+"] and w0.exact_id[0] != emqx.NONE
    assert sorted(w0.filters(1)) == [b"#", b"a/#"]  # "a" matches "a/#" (emqx_topic.erl:82-83)
    assert sorted(w0.filters(2)) == [b"#"] and w0.exact_id[2] == emqx.NONE
    assert w0.latency_ns > 0
    assert b.collect(ws[0]).tag.tolist() == [7, 8, 8, 8]  # collected results stay readable
    ws.append(b.flush())  # reopens ws[0]'s slot as the open window
    with pytest.raises(emqx.EngineError, match="ENOENT"):
        b.collect(ws[0])  # its id no longer names a result (it used to read in place)
    for wid in ws[1:]:
        assert len(b.collect(wid).tag) == 1
    with pytest.raises(emqx.EngineError, match="ENOENT"):
        b.collect(12345)
    b.close()


def test_batcher_add_many_packs_like_add(emqx):
    """add_many (the bulk form: one copy of the run of topics that fits) packs a window exactly
    like add one by one: the same answers per tag, partial adds when the window fills by topics
    or by bytes, a base offset != 0, and the errors of a bad first topic."""
    eng = emqx.Engine()
    for f in (b"a/+", b"a/#", b"#", b"b/+/c"):
        eng.route_ref(f)
        eng.trie_insert(f)
    eng.route_ref(b"a/b")
    eng.commit()
    rng = random.Random(5)
    topics = [rng.choice([b"a/b", b"a", b"", b"b/x/c", b"a/b/c/d", b"zz"]) for _ in range(300)]
    lens = np.array([len(t) for t in topics], np.uint32)
    pad = b"PAD"  # offsets start past 0: the run is copied from bytes[off[0]:]
    buf = np.frombuffer(pad + b"".join(topics), np.uint8)
    off = np.zeros(len(topics) + 1, np.uint32)
    np.cumsum(lens, out=off[1:])
    off += len(pad)
    # the reference packing: one add per topic, a flush whenever the window is full or has no
    # room for the next topic (-ENOSPC), never on time (window_us far away)
    one = {}
    b1 = emqx.Batcher(eng, window_topics=64, window_bytes=160, window_us=10**9)

    def flush1():
        wid = b1.flush()
        if not wid:
            return
        w1 = b1.collect(wid)
        for j in range(len(w1.tag)):
            one[int(w1.tag[j])] = (w1.filters(j), int(w1.exact_id[j]))

    for i, t in enumerate(topics):
        try:
            full = b1.add(t, i)
        except emqx.EngineError as e:
            assert "ENOSPC" in str(e)
            flush1()
            full = b1.add(t, i)
        if full:
            flush1()
    flush1()
    b1.close()
    b = emqx.Batcher(eng, window_topics=64, window_bytes=160)
    got, i = {}, 0
    while i < len(topics):
        k = b.add_many(buf, off[i:], i)
        assert 0 < k <= 64 and int(off[i + k] - off[i]) <= 160
        i += k
        w = b.collect(b.flush())
        for j in range(len(w.tag)):
            got[int(w.tag[j])] = (w.filters(j), int(w.exact_id[j]))
    assert got == one
    with pytest.raises(emqx.EngineError, match="EINVAL"):
        b.add_many(buf, np.array([5, 3], np.uint32))
    with pytest.raises(emqx.EngineError, match="E2BIG"):
        b.add_many(np.zeros(200, np.uint8), np.array([0, 200], np.uint32))
    assert b.add_many(buf, np.array([3, 6, 2], np.uint32)) == 1  # stops before the bad offset
    b.close()


def test_submit_filters_one_sync_equals_sync_gather(emqx):
    """emqxgm_match_batch_submit_filters enqueues the filter-byte gather and one packed copy of
    every result array behind the pass, sized from the pipe's recent windows; a window beyond
    those sizes (the first ones, a sudden denser window) is finished synchronously in the wait.
    Windows of changing size and density: identical to submit + the synchronous gather, and each
    pair's bytes are its filter's."""
    import workloads
    w = workloads.generate(1, None, 120_000)
    eng = emqx.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    eng.trie_insert_many(w.fbytes, w.foff)
    for i in range(0, w.nt, 9):  # some names are route keys: exact ids in the block
        eng.route_ref(w.topic(i))
    eng.commit()
    off = w.toff.astype(np.int64)
    dense = np.frombuffer(b"l0w0/l1w0/l2w0/l3w0" * 1, np.uint8)
    plan = [(0, 4096), (4096, 4096), (8192, 30000), (38192, 0), (38192, 100), (38292, 4096),
            (42388, 60000), (102388, 4096)]
    for k, (i, m) in enumerate(plan):
        buf = w.tbytes[off[i]:off[i + m]].copy()
        o = (off[i:i + m + 1] - off[i]).astype(np.uint32)
        if k == 5:  # a window of one dense topic repeated: far more pairs per topic than before
            buf = np.tile(dense, m)
            o = (np.arange(m + 1) * dense.size).astype(np.uint32)
        res = []
        for filters in (True, False):
            t = eng.match_batch_submit(buf, o, filters=filters)
            res.append(eng.match_batch_wait_filters(t))
        (a, fa, ba), (b, fb, bb) = res
        assert np.array_equal(a.row_ptr, b.row_ptr) and np.array_equal(a.filter_id, b.filter_id)
        assert np.array_equal(a.exact_id, b.exact_id), k
        assert np.array_equal(fa, fb) and np.array_equal(ba, bb), k
        for j in range(0, a.filter_id.size, 97):
            assert ba[fa[j]:fa[j + 1]].tobytes() == eng.filter_bytes(int(a.filter_id[j]))
