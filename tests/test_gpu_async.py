"""The NIF's publish path on the device.

* The level-triggered mirror (src/emqx_trie_gpu_sync.erl, emqx_amd/mirror.py) after the
  adversarial event orders -- two dests before either event, paired deletes, events queued while
  init scans, a restart on the same engines -- and random churn: every topic's
  match_routes over the device's answer (exact route key + trie row, emqx_router.erl:141-146)
  equals oracle.emqx_ref.Router.match_routes.
* The concurrent entry (emqxgm_async_*, the NIF's match_async/3): calls from Python one at a
  time (cancel, max_levels, wildcard names, empty topics), and the C load harness
  (tests/host_harness/async_load.cpp) with 16 and 64 publisher threads calling one topic at a
  time: EVERY call's answer (trie filter set, as count + order-independent hash of the filter
  bytes, and the exact-hit flag) equals the oracle's (oracle/ref_trie.cpp) for its topic -- on
  cfg1, on a 1M-filter cfg3 slice, and with two engines (replicas) taking windows round robin.
"""
import random
import time

import numpy as np
import pytest

from emqx_amd.mirror import RouteTableMirror
from oracle import emqx_ref as R
from oracle.cref import RefIndex

pytestmark = pytest.mark.gpu
NONE = 0xFFFFFFFF


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def _routes_device(eng, rt, topics):
    """match_routes(T) from the device's answer: routes of the exact key, then of every trie
    filter (emqx_router.erl:141-146), with the route bag's dests."""
    res = eng.match(topics)
    out = []
    for i, t in enumerate(topics):
        keys = []
        if res.exact_id[i] != NONE:
            keys.append(eng.filter_bytes(int(res.exact_id[i])))
        keys += [eng.filter_bytes(int(f)) for f in res.row(i)]
        if not res.row(i).size:  # match_trie [] -> lookup_routes(Topic) only
            keys = [t] if t in rt.bag else []
        out.append(sorted((k, str(d)) for k in keys for _, d in rt.lookup_routes(k)))
    return out


def _check_routes(eng, rt, topics):
    got = _routes_device(eng, rt, topics)
    for t, g in zip(topics, got):
        want = sorted((k, str(d)) for k, d in rt.match_routes(t))
        assert g == want, (t, g, want)


def test_mirror_adversarial_orders_match_routes(emqx):
    eng, rt = emqx.Engine(), R.Router()
    m = RouteTableMirror([eng], rt)
    m.init()
    probe = [b"a/b/c", b"a/x/c", b"x/y", b"x", b"s/1", b"k1", b"k2", b"z/q/z", b"a/+/c"]
    # two dests before either event
    for d in ("n1", "n2"):
        rt.add_route(b"a/+/c", d)
        m.event("write", b"a/+/c")
    m.handle_events()
    m.commit()
    _check_routes(eng, rt, probe)
    # paired deletes
    for d in ("n1", "n2"):
        rt.add_route(b"x/#", d)
    m.event("write", b"x/#")
    m.handle_events()
    m.commit()
    for d in ("n1", "n2"):
        rt.delete_route(b"x/#", d)
        m.event("delete_object", b"x/#")
    m.handle_events()
    m.commit()
    _check_routes(eng, rt, probe)
    # events queued while init scans (a second mirror on the same engines = a restart), with
    # changes nobody handled while "down"
    for t in (b"s/+", b"k1", b"k2"):
        rt.add_route(t, "n1")
    rt.delete_route(b"a/+/c", "n1")
    m2 = RouteTableMirror([eng], rt)
    for t in (b"s/+", b"k1"):
        m2.event("write", t)
    m2.init()
    _check_routes(eng, rt, probe)
    m2.handle_events()
    m2.commit()
    rt.add_route(b"z/+/z", "n3")
    rt.delete_route(b"k1", "n1")
    m2.event("write", b"z/+/z")
    m2.event("delete_object", b"k1")
    m2.handle_events()
    m2.commit()
    _check_routes(eng, rt, probe)


def test_mirror_random_churn_match_routes(emqx):
    rng = random.Random(7)
    engs = [emqx.Engine(), emqx.Engine()]  # the NIF's resource: one engine per GPU
    rt = R.Router()
    words = [b"a", b"b", b"c", b"+", b"#", b"", b"longword_x"]

    def topic(filt):
        n = rng.randint(1, 4)
        ws = [rng.choice(words if filt else [w for w in words if w not in (b"+", b"#")])
              for _ in range(n)]
        if b"#" in ws:
            ws = ws[:ws.index(b"#") + 1]
        return b"/".join(ws)
    m = RouteTableMirror(engs, rt)
    m.init()
    probes = list({topic(False) for _ in range(300)}) + [b"$SYS/a", b""]
    for step in range(400):
        r = rng.random()
        if r < 0.55:
            t = topic(True)
            d = rng.choice(["n1", "n2", ("g", "n1")])
            if rng.random() < 0.6:
                rt.add_route(t, d)
                m.event("write", t)
            else:
                if rt.has_routes(t):
                    d = rng.choice([x for _, x in rt.lookup_routes(t)])
                rt.delete_route(t, d)
                m.event(rng.choice(["delete_object", "delete"]), t)
        elif r < 0.85:
            m.handle_events(limit=rng.randint(0, 5))
        elif r < 0.9:
            m.resync()
        else:
            m.handle_events()
            m.commit()
            for e in engs:
                _check_routes(e, rt, probes)
    m.handle_events()
    m.commit()
    for e in engs:
        _check_routes(e, rt, probes)


def _cfg1(emqx, nf=None, nt=30_000, engines=1):
    import workloads
    w = workloads.generate(1, nf, nt)
    engs = []
    for _ in range(engines):
        e = emqx.Engine()
        e.route_ref_many(w.fbytes, w.foff)
        wi = np.nonzero(w.fwild)[0]
        for i in wi:
            e.trie_insert(w.filter(int(i)))
        e.commit()
        engs.append(e)
    return w, engs


def test_async_matcher_calls_one_at_a_time(emqx):
    w, (eng,) = _cfg1(emqx, nt=20_000)
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, 2 + w.fwild.astype(np.uint8))
    row, ids, ex = ref.match(w.tbytes, w.toff)
    flt = [w.filter(i) for i in range(w.nf)]
    am = emqx.AsyncMatcher([eng], window_topics=4096, window_us=100, max_levels=8)
    keys = []

    def call(topic, tag, owner):
        # -EBUSY (every window full or in flight: a publisher would take the reference's path)
        # is retried here, after the completers had a moment
        while True:
            rc = am.match(topic, tag, owner=owner)
            if rc != -16:
                return rc
            time.sleep(0.0002)
    for i in range(w.nt):
        assert call(w.topic(i), i, 1) == 0
        keys.append((i, 1))
    # edge calls: a wildcard name (trie [] but its exact key), an empty topic, too deep
    eng2_topics = [b"l0w1/+", b"", b"a/b/c/d/e/f/g/h/i"]
    assert call(eng2_topics[0], 10**9, 2) == 0
    assert call(eng2_topics[1], 10**9 + 1, 2) == 0
    assert call(eng2_topics[2], 10**9 + 2, 2) == -7  # -E2BIG: 9 levels > 8
    assert am.wait(keys + [(10**9, 2), (10**9 + 1, 2)], timeout=60)
    for i in range(w.nt):
        r = am.results[(i, 1)]
        assert r.status == 0
        assert sorted(r.filters) == sorted(flt[j] for j in ids[row[i]:row[i + 1]]), i
        assert (r.exact_id != NONE) == (ex[i] != NONE), i
    assert am.results[(10**9, 2)].filters == []
    pyr = R.Trie()
    for f in flt:
        if R.wildcard(f):
            pyr.insert(f)
    assert sorted(am.results[(10**9 + 1, 2)].filters) == sorted(pyr.match(b""))
    # cancel: either never reported (True) or already reported (False), never both
    outcomes = []
    for k in range(200):
        tag = 2 * 10**9 + k
        assert call(w.topic(k), tag, 3) == 0
        outcomes.append((tag, am.cancel(tag, owner=3)))
    st = am.stats()
    assert st["too_deep"] == 1
    am.close()  # reports every accepted call
    for tag, cancelled in outcomes:
        assert ((tag, 3) in am.results) != cancelled, tag
    assert all(r.status == 0 for r in am.results.values())


def _oracle_rows(w):
    from workloads import publishers
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, 2 + w.fwild.astype(np.uint8))
    row, ids, ex = ref.match(w.tbytes, w.toff, threads=8)
    fh = publishers.string_hashes(w.fbytes, w.foff)
    return np.diff(row).astype(np.uint32), publishers.row_hashes(row, ids, fh), ex != NONE


def _check_load(r, want):
    cnt, hsh, exact = want
    t = r["topic"]
    assert r["calls"] == len(t) and r["failed"] == 0
    bad = np.nonzero((r["count"] != cnt[t]) | (r["hash"] != hsh[t]) |
                     (r["exact"].astype(bool) != exact[t]))[0]
    assert bad.size == 0, (bad[:10], t[bad[:10]])


@pytest.mark.parametrize("threads,window,deliver,eager", [(16, 4096, 0, False), (64, 16384, 0, False),
                                                          (16, 16384, 8, False), (16, 4096, 0, True),
                                                          (64, 16384, 8, True)])
def test_async_load_cfg1_every_call(emqx, threads, window, deliver, eager):
    """deliver: the layer's report pool (emqxgm_async_cfg.deliver_threads): a window's calls
    reported in parts by several threads, each part's view offset into the window's result.
    eager: EMQXGM_ASYNC_EAGER, windows sealed as soon as a pipe is free."""
    from workloads import publishers
    w, (eng,) = _cfg1(emqx, nt=100_000)
    want = _oracle_rows(w)
    procs = max(1, window * 4 // threads)
    r = publishers.run([eng], w.tbytes, w.toff.astype(np.uint64), threads, procs,
                       max(2 * procs, 300_000 // threads), window, record=True,
                       deliver_threads=deliver, report_ns=200 if deliver else 0, eager=eager)
    _check_load(r, want)
    assert r["windows"] > 0 and r["calls_per_window"] > 1


def test_async_eager_idle_call_takes_one_pass(emqx):
    """An idle layer with EMQXGM_ASYNC_EAGER submits a lone call's window at once: its answer
    comes back well inside the window_us timer the default layer waits for (here 20 ms), and
    equals the oracle's."""
    import time
    w, (eng,) = _cfg1(emqx, nt=2_000)
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, 2 + w.fwild.astype(np.uint8))
    row, ids, _ = ref.match(w.tbytes, w.toff, threads=8)
    am = emqx.AsyncMatcher([eng], window_topics=4096, window_us=20_000, eager=True)
    for i in range(50):
        t0 = time.perf_counter()
        assert am.match(w.topic(i), i) == 0
        assert am.wait([(i, 0)], timeout=10)
        dt = time.perf_counter() - t0
        r = am.results.pop((i, 0))
        assert r.status == 0, r.status
        assert sorted(r.filters) == sorted(w.filter(int(j)) for j in ids[row[i]:row[i + 1]]), i
        assert dt < 0.01, dt
    am.close()


def test_async_load_two_replicas(emqx):
    from workloads import publishers
    w, engs = _cfg1(emqx, nt=50_000, engines=2)
    want = _oracle_rows(w)
    r = publishers.run(engs, w.tbytes, w.toff.astype(np.uint64), 16, 512, 10_000, 2048,
                       record=True)
    _check_load(r, want)


def test_async_load_cfg3_slice_every_call(emqx):
    import workloads
    from workloads import publishers
    w = workloads.generate(3, 1_000_000, 200_000)
    eng = emqx.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    eng.trie_insert_many(w.fbytes, w.foff)  # every cfg3 filter is a wildcard
    eng.commit()
    want = _oracle_rows(w)
    r = publishers.run([eng], w.tbytes, w.toff.astype(np.uint64), 64, 4096, 6_000, 65536,
                       record=True)
    _check_load(r, want)


def test_async_copy_through_long_and_odd_topics(emqx):
    """Windows of the concurrent entry go without DMA copies (k_tok reads the pinned window and
    stores the device copies the later kernels read; k_fb_pack writes the result block into
    pinned memory): topics long enough that a tile does not fit k_tok's LDS (the per-lane path
    copies them), a 65,535-byte topic, empty levels, '$' names -- every call's answer equals the
    host API's (DMA path) and, with copy-through off (zc_topics 0), the same."""
    w, (eng,) = _cfg1(emqx, nt=2_000)
    rng = random.Random(5)
    words = [w.topic(i).split(b"/") for i in range(200)]
    topics = []
    for i in range(600):
        base = list(rng.choice(words))
        if i % 3 == 0:  # long levels: a tile of these outgrows the LDS buffer
            base = base + [b"x" * rng.randint(80, 400) for _ in range(rng.randint(1, 3))]
        elif i % 7 == 0:
            base = [b"$SYS"] + base
        elif i % 11 == 0:
            base = base[:1] + [b""] + base[1:]
        topics.append(b"/".join(base))
    topics.append(b"a/" + b"b" * 65533)
    topics.append(b"")
    want = eng.match(topics)
    flt = {}

    def answer(am, owner):
        for i, t in enumerate(topics):
            while True:
                rc = am.match(t, i, owner=owner)
                if rc != -16:
                    break
                time.sleep(0.0002)
            assert rc == 0, (i, rc)
        assert am.wait([(i, owner) for i in range(len(topics))], timeout=60)
        return {i: sorted(am.results[(i, owner)].filters) for i in range(len(topics))}

    # the oracle (emqx_trie:match, oracle.emqx_ref) over the same filters: the copy-through
    # path's answers are pinned to the reference restatement, not only to the host API's
    trie = R.Trie()
    for i in range(w.nf):
        f = w.filter(i)
        if R.wildcard(f):
            trie.insert(f)
    for zc in (65536, 0):
        eng.tune("zc_topics", zc)
        am = emqx.AsyncMatcher([eng], window_topics=256, window_bytes=1 << 20, window_us=200,
                               max_levels=4096)
        got = answer(am, 7)
        am.close()
        for i in range(len(topics)):
            ids = want.row(i)
            exp = sorted(flt.setdefault(int(f), eng.filter_bytes(int(f))) for f in ids)
            assert got[i] == exp, (zc, i, topics[i][:80])
            assert got[i] == sorted(trie.match(topics[i])), (zc, i, topics[i][:80])
    eng.tune("zc_topics", 65536)


def test_async_single_long_topic_on_an_idle_layer(emqx):
    """a topic longer than a staging chunk (4 KB) goes into the open window
    on its own; on an idle layer the flusher must arm its window_us timer for it, so the call is
    answered within about window_us plus one pass -- not after the caller's 5 s timeout."""
    w, (eng,) = _cfg1(emqx, nt=10)
    trie = R.Trie()
    for i in range(w.nf):
        f = w.filter(i)
        if R.wildcard(f):
            trie.insert(f)
    am = emqx.AsyncMatcher([eng], window_topics=256, window_bytes=1 << 20, window_us=200)
    time.sleep(0.05)  # idle: the flusher sleeps with nothing pending
    for k, t in enumerate([w.topic(0) + b"/" + b"q" * 9000, b"l0w1/" + b"z" * 5000]):
        t0 = time.perf_counter()
        assert am.match(t, k, owner=1) == 0
        assert am.wait([(k, 1)], timeout=2.0), "a lone long topic was never submitted"
        dt = time.perf_counter() - t0
        assert dt < 0.05, dt
        assert sorted(am.results[(k, 1)].filters) == sorted(trie.match(t))
        time.sleep(0.05)
    am.close()


@pytest.mark.parametrize("deliver", [0, 4])
def test_async_publish_layer_every_call(emqx, deliver):
    """The publish layer (EMQXGM_ASYNC_PUBLISH: the NIF's publish_async/3, emqx_trie_gpu:route/2)
    from 16 threads, one topic a call: every call's aggre/1 entries and local dispatches equal
    oracle.emqx_ref.publish (emqx_broker.erl:218-300, 326-355) for its topic.  The broker state
    reaches the engine through the level-triggered mirror (route dests and subscriber lists)."""
    import threading
    import workloads
    from emqx_amd.mirror import RouteTableMirror
    w = workloads.generate(1, 4000, 12_000)
    rng = random.Random(3)
    rt, subs = R.Router(), {}
    dests = ["n1", "n2", "n3", ("g1", "n1"), ("g2", "n2"), ("g1", "n3")]
    names = [w.filter(i) for i in range(w.nf)]
    for f in names:
        for d in rng.sample(dests, rng.randint(1, 3)):
            rt.add_route(f, d)
        if rng.random() < 0.6:
            subs[f] = sorted({f"s{rng.randint(0, 40)}" for _ in range(rng.randint(1, 3))})
    for i in range(0, 12_000, 5):  # exact route keys: some topics are routed by their own name
        t = w.topic(i)
        rt.add_route(t, rng.choice(dests))
        subs.setdefault(t, ["x%d" % (i % 7)])
    eng = emqx.Engine()
    m = RouteTableMirror([eng], rt, subscribers=subs, local_node="n1")
    m.init()
    # deliver: the report pool (emqxgm_async_cfg.deliver_threads) -- full windows reported in
    # parts of >= 1,024 calls, each part's view offset into the window's publish result
    am = emqx.AsyncMatcher([eng], window_topics=4096, window_us=100, publish=True,
                           deliver_threads=deliver)
    topics = [w.topic(i) for i in range(w.nt)] + names[:200] + [b"", b"l0w1/+"]
    errors = []

    def publisher(k):
        try:
            for i in range(k, len(topics), 16):
                while True:
                    rc = am.match(topics[i], i, owner=k + 1)
                    if rc != -16:
                        break
                    time.sleep(0.0002)
                assert rc == 0, rc
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)
    ths = [threading.Thread(target=publisher, args=(k,)) for k in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    keys = [(i, i % 16 + 1) for i in range(len(topics))]
    assert am.wait(keys, timeout=120)
    H = m.handles.names

    def check(r, t):
        assert r.status == 0
        got_e = sorted(((to, H["group"][d & ~emqx.engine.DEST_GROUP] if d & emqx.engine.DEST_GROUP
                         else H["node"][d]) for to, d in r.routes), key=repr)
        got_d = sorted(((to, H["sub"][s]) for to, s in r.deliveries), key=repr)
        want_e, want_d = R.publish(rt, t, "n1", subs)
        assert got_e == sorted(want_e, key=repr), t
        assert got_d == sorted(want_d, key=repr), t
        return got_e, got_d
    for i, t in enumerate(topics):
        check(am.results[keys[i]], t)
    am.close()
    # the writing node's hooks: a new route + subscriber, visible on the very next publish
    am = emqx.AsyncMatcher([eng], window_topics=256, window_us=50, publish=True)
    rt.add_route(b"hook/+/x", "n1")
    subs[b"hook/+/x"] = ["sub-new"]
    m.route_changed(b"hook/+/x")
    m.subscribers_changed(b"hook/+/x")
    assert am.match(b"hook/7/x", 1, owner=99) == 0
    assert am.wait([(1, 99)], timeout=10)
    got_e, got_d = check(am.results[(1, 99)], b"hook/7/x")
    assert (b"hook/+/x", "n1") in got_e and (b"hook/+/x", "sub-new") in got_d
    am.close()


def test_mirror_restart_from_snapshot(emqx, tmp_path):
    """broker.perf.gpu_match.snapshot_dir on the GPU: the mirror saves its index, fresh engines
    start from it, the first resync commits what changed meanwhile as a delta, and match_routes
    equals the oracle's router afterwards."""
    rng = random.Random(5)
    rt = R.Router()
    topics = [b"site/%d/+/t" % i for i in range(2000)] + [b"k/%d" % i for i in range(2000)]
    for t in topics:
        rt.add_route(t, rng.choice(["n1", "n2", ("g", "n1")]))
    eng = emqx.Engine()
    m = RouteTableMirror([eng], rt)
    m.init()
    snap = str(tmp_path / "emqx_trie_gpu.route.snap")
    m.save(snap)
    eng.close()
    for t in rng.sample(topics, 300):
        rt.delete_route(t, rt.lookup_routes(t)[0][1])
    for i in range(100):
        rt.add_route(b"site/%d/#" % i, "n3")
    eng2 = emqx.Engine()
    f0 = eng2.stats()["full_commits"]
    m2 = RouteTableMirror([eng2], rt)
    m2.init(snapshot=snap)
    st = eng2.stats()
    assert st["full_commits"] == f0 + 1 and st["delta_commits"] >= 1, st
    probe = [b"site/%d/x/t" % i for i in range(0, 2000, 7)] + [b"k/%d" % i for i in range(0, 2000, 7)]
    _check_routes(eng2, rt, probe)
