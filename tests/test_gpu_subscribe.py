"""Subscribe-then-publish visibility on the device (r05).

The reference adds a subscriber's route inside the broker-pool call, before SUBACK
(emqx_broker.erl:163-168, 484-486 -> emqx_router.erl:124-138), so the node's next publish
matches it.  The writing node's hook here is emqxgm_route_set_batch(.., EMQXGM_SET_COMMIT)
(Engine.route_set_batch): no tick, and never a wait for a full build -- while one runs in the
background the change is a delta patch of the index readers have, replayed onto the new index at
its install.

* a subscribe / unsubscribe, then at once a device match of a topic it matches: the row equals
  the oracle's (emqx_trie:match, oracle.emqx_ref) with the change in, on a committed cfg1 index;
* the same while the full build of a 1M-filter (cfg2) index runs in the background: every single
  subscribe is visible on the next match, its commit takes far less than the build, the bulk
  shows from its install on, and afterwards 20k cfg2 topics equal the C++ oracle
  (oracle/ref_trie.cpp) over everything.
"""
import threading
import time

import numpy as np
import pytest

from oracle import emqx_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def _row(eng, res, i):
    return sorted(eng.filter_bytes(int(f)) for f in res.row(i))


def _instantiate(f: bytes, rng) -> bytes:
    out = []
    for w in f.split(b"/"):
        if w == b"#":
            out += [b"t%d" % rng.integers(0, 9) for _ in range(rng.integers(0, 3))]
            break
        out.append(b"w%d" % rng.integers(0, 50) if w == b"+" else w)
    return b"/".join(out)


def test_subscribe_visible_on_the_next_match(emqx):
    import workloads
    w = workloads.generate(1, 10_000, 0)
    eng = emqx.Engine()
    trie = R.Trie()
    items = []
    for i in range(w.nf):
        f = w.filter(i)
        items.append((f, True))
        if R.wildcard(f):
            trie.insert(f)
    eng.route_set_batch(items)
    rng = np.random.default_rng(5)
    mine = []
    lat = []
    for k in range(300):
        if mine and rng.integers(0, 4) == 0:
            f = mine.pop(int(rng.integers(0, len(mine))))
            present = False
            trie.delete(f)
        else:
            lv = [b"+" if rng.integers(0, 3) == 0 else b"l%dw%d" % (j, rng.integers(0, 8))
                  for j in range(int(rng.integers(1, 5)))]
            if rng.integers(0, 3) == 0:
                lv.append(b"#")
            f = b"/".join(lv)
            if not R.wildcard(f) or f in mine:
                continue
            mine.append(f)
            present = True
            trie.insert(f)
        t0 = time.perf_counter()
        eng.route_set_batch([(f, present)])
        lat.append(time.perf_counter() - t0)
        topics = [_instantiate(f, rng) for _ in range(3)] + [f]
        res = eng.match(topics)
        for i, t in enumerate(topics):
            assert _row(eng, res, i) == sorted(trie.match(t)), (k, f, t, present)
        # the route key itself: an exact hit exactly while present (match_routes of the name)
        assert (int(res.exact_id[3]) != 0xFFFFFFFF) == present, (f, present)
    st = eng.stats()
    # (a subscribe of a filter the cfg1 index already routes changes nothing: no commit)
    assert st["delta_commits"] >= 100 and len(lat) >= 150 and st["bg_waits"] == 0
    print(f"subscribe + commit: p50 {np.median(lat) * 1e6:.0f} us, p99 "
          f"{np.percentile(lat, 99) * 1e6:.0f} us over {len(lat)}")
    eng.close()


def test_subscribe_visible_while_a_1m_filter_build_runs(emqx):
    """cfg2 (1M filters, depth 6): the bulk commit's full build runs in the background, held
    back 1.5 s before its install.  Private 3-level filters subscribed meanwhile (no cfg2 filter
    can match a 3-level topic: every cfg2 filter has 6 levels) must be on the very next match."""
    import workloads
    from oracle import cref
    w = workloads.generate(2, 1_000_000, 20_000)
    eng = emqx.Engine()
    eng.tune("bg_build", 1)
    # (the index readers have until the install takes the subscribes as delta patches: sized for
    # 20k filters, its tables hold the ~4k nodes of 2000 more)
    base = [b"zz/b%d/+" % i for i in range(20000)]
    eng.route_set_batch([(f, True) for f in base])
    eng.route_set_many(w.fbytes, w.foff, True)  # the bulk: pending, committed on another thread
    eng.tune("bg_delay_ms", 1500)
    done = threading.Event()
    t_bulk = {}

    def bulk_commit():
        t0 = time.perf_counter()
        eng.commit()
        t_bulk["s"] = time.perf_counter() - t0
        done.set()

    th = threading.Thread(target=bulk_commit)
    th.start()
    t_wait = time.time() + 60
    while eng.stats()["bg_builds"] < 1:
        assert time.time() < t_wait and not done.is_set(), "the bulk commit did not build in the background"
        time.sleep(0.001)
    rng = np.random.default_rng(7)
    trie = R.Trie()
    for f in base:
        trie.insert(f)
    mine, lat, during = [], [], 0
    k = 0
    while not done.is_set() and k < 2000:
        f = b"zz/m%d/+" % k
        k += 1
        t0 = time.perf_counter()
        eng.route_set_batch([(f, True)])
        lat.append(time.perf_counter() - t0)
        mine.append(f)
        trie.insert(f)
        topics = [_instantiate(f, rng), b"zz/b%d/q" % rng.integers(0, 20000)]
        res = eng.match(topics)
        for i, t in enumerate(topics):
            assert _row(eng, res, i) == sorted(trie.match(t)), (f, t)
        during += 1 if not done.is_set() else 0
    th.join()
    st = eng.stats()
    assert during >= 20, during
    assert st["bg_builds"] >= 1 and st["bg_waits"] == 0, st
    p50, p99 = np.median(lat) * 1e3, np.percentile(lat, 99) * 1e3
    print(f"1M-filter build {st['last_build_ms']:.0f} ms (+1500 ms held), bulk commit "
          f"{t_bulk['s']:.2f} s; {during} subscribes during it: p50 {p50:.2f} ms, p99 {p99:.2f} ms; "
          f"catch-up {st['catchup_changes']}")
    assert p99 < 0.25 * t_bulk["s"] * 1e3, (p99, t_bulk)  # none waited for the build
    # everything is visible now: cfg2 topics against the C++ oracle over bulk + private filters
    ref = cref.RefIndex()
    ref.add_many(w.fbytes, w.foff, np.where(w.fwild.astype(bool), 3, 2).astype(np.uint8))
    priv = base + mine
    pb, po = emqx.engine.pack(priv, np.uint64)
    ref.add_many(pb, po, np.full(len(priv), 3, np.uint8))
    res = eng.match_packed(w.tbytes, w.toff)
    row, ids, _ = ref.match(w.tbytes, w.toff)
    names = [w.filter(i) for i in range(w.nf)] + priv
    for i in range(w.nt):
        want = sorted(names[j] for j in ids[row[i]:row[i + 1]])
        assert _row(eng, res, i) == want, i
    for f in mine[::7]:
        t = _instantiate(f, rng)
        assert _row(eng, eng.match([t]), 0) == sorted(trie.match(t))
    eng.close()
