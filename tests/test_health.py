"""Failing closed at the boundary (SURVEY 5 "Failure detection"), on the CPU.

The engine is the real host code (gm_engine.cpp: registry, commits, the health state) on the fake
HIP runtime of tests/host_harness; the route table is the oracle's route bag (oracle.emqx_ref.
Router: emqx_router.erl:124-188 with emqx_router_utils.erl:34-71); the mirror and the hooks are
emqx_amd/mirror.py (the restatement of src/emqx_trie_gpu{,_sync}.erl).  Failures are injected
with emqxgm_tune("fail_commits" / "fail_errno") into the commits of emqxgm_route_dests_batch /
emqxgm_subscribers_batch (EMQXGM_SET_COMMIT) and emqxgm_commit.

The invariant checked after every step: whenever the device would be offered to a publisher
(the index is published and the engine is not stale), its committed state is the table's as of
the last hook that returned -- route key <=> has_routes(T), trie member <=> the reference's trie
holds {T, 1}.  While the engine is stale every match entry refuses with -ESTALE before touching
the device (the publishers' reference path), and the hooks return "ok" whatever happened."""
import errno
import random

import pytest

from emqx_amd.engine import STALE_COMMIT, STALE_RESYNC, Engine, EngineError, load_library
from emqx_amd.mirror import RouteTableMirror
from oracle import emqx_ref as R
from tests.test_route_mirror import build_fake_lib


@pytest.fixture(scope="module")
def fakelib():
    return load_library(build_fake_lib(), allow_missing=True)


def _committed_is_table(eng, router, topics):
    for t in topics:
        assert eng.route_member(t) == router.has_routes(t), t
        assert eng.trie_member(t) == ((t, 1) in router.trie.tab), t


def _invariant(m, eng, router, topics):
    """No answer from an index that lacks a committed change: offered => committed == table."""
    if m.device_offered():
        _committed_is_table(eng, router, topics)
    else:
        with pytest.raises(EngineError, match="ESTALE"):
            eng.match([b"probe/topic"])


@pytest.mark.parametrize("err", [errno.ENOMEM, errno.EIO])
def test_refused_hook_commit_fails_closed_and_repairs(fakelib, err):
    eng, rt = Engine(library=fakelib), R.Router()
    topics = [b"a/+", b"a/b", b"c/#"]
    for t in topics:
        rt.add_route(t, "n1")
    m = RouteTableMirror([eng], rt)
    m.init()
    assert m.published and m.healthy()
    _committed_is_table(eng, rt, topics)
    # the subscriber's route is written (the reference's do_add_route/2 succeeded), then the
    # engine refuses the hook's commit
    eng.tune("fail_errno", err)
    eng.tune("fail_commits", 1)
    rt.add_route(b"new/+/x", "n1")
    topics.append(b"new/+/x")
    assert m.route_changed(b"new/+/x") == "ok"  # the hook returns ok (no badmatch crash)
    h = eng.health()
    assert h["stale"] & STALE_COMMIT and h["last_error"] == -err and m.repair_pending
    assert not eng.route_member(b"new/+/x")  # the index lacks it ...
    assert not m.device_offered()             # ... so the device is not offered
    _invariant(m, eng, rt, topics)
    with pytest.raises(EngineError, match="ESTALE"):
        eng.match([b"new/a/x"])
    assert eng.health()["refused"] >= 2
    # later hooks still succeed, but the engine stays stale until a repair
    rt.add_route(b"k9", "n2")
    topics.append(b"k9")
    assert m.route_changed(b"k9") == "ok"
    assert eng.health()["stale"] and not m.device_offered()
    _invariant(m, eng, rt, topics)
    # the repair: a full resync + commit, then the device is offered again with the change
    assert m.repair()
    assert m.healthy() and m.device_offered() and eng.health()["repairs"] == 1
    _committed_is_table(eng, rt, topics)


def test_refused_subscribers_commit_and_mirror_batch(fakelib):
    eng, rt = Engine(library=fakelib), R.Router()
    subs = {b"s/1": ["p1", "p2"]}
    m = RouteTableMirror([eng], rt, subscribers=subs)
    m.init()
    eng.tune("fail_commits", 1)
    subs[b"s/1"] = ["p1"]
    assert m.subscribers_changed(b"s/1") == "ok"
    assert eng.health()["stale"] and not m.device_offered()
    # a table-event batch of the mirror refused too: no crash, a repair queued
    eng.tune("fail_commits", 1)
    rt.add_route(b"e/+", "n1")
    m.event("write", b"e/+")
    m.handle_events()
    assert m.repair_pending and m.errors == 2
    assert m.repair() and m.healthy()
    _committed_is_table(eng, rt, [b"e/+"])


def test_host_mark_needs_a_resync_begun_after_it(fakelib):
    """emqxgm_mark_stale (a timeout the host saw): a commit alone does not clear it; a resync
    that began before the mark does not either; one begun after it does."""
    eng = Engine(library=fakelib)
    eng.route_set(b"x/+", True)
    eng.commit()
    g = eng.sync_begin()
    eng.mark_stale(errno.ETIMEDOUT)
    h = eng.health()
    assert h["stale"] == STALE_RESYNC and h["last_error"] == -errno.ETIMEDOUT
    with pytest.raises(EngineError, match="ESTALE"):
        eng.commit()  # committed, still stale: no resync since the mark
    eng.route_set(b"x/+", True)
    eng.sync_end(g)
    with pytest.raises(EngineError, match="ESTALE"):
        eng.commit()  # the resync began before the mark
    g = eng.sync_begin()
    eng.route_set(b"x/+", True)
    eng.sync_end(g)
    eng.commit()
    assert eng.health()["stale"] == 0
    assert eng.route_member(b"x/+") and eng.trie_member(b"x/+")


def test_mark_during_the_repair_keeps_it_stale(fakelib):
    eng = Engine(library=fakelib)
    eng.mark_stale(errno.EIO)
    g = eng.sync_begin()
    eng.mark_stale(errno.EIO)  # another failure while the resync runs
    eng.sync_end(g)
    with pytest.raises(EngineError, match="ESTALE"):
        eng.commit()
    g = eng.sync_begin()
    eng.sync_end(g)
    eng.commit()
    assert eng.health()["stale"] == 0


def test_repair_retries_with_backoff(fakelib):
    """The mirror's repair fails while the engine keeps refusing (a persistent -ENOMEM), with a
    doubling backoff, never a crash; the first success publishes and clears it."""
    eng, rt = Engine(library=fakelib), R.Router()
    rt.add_route(b"a/#", "n1")
    eng.tune("fail_errno", errno.ENOMEM)
    eng.tune("fail_commits", 3)
    m = RouteTableMirror([eng], rt)
    m.init()  # the first commit fails: not published, publishers take the reference path
    assert not m.published and m.repair_pending and not m.device_offered()
    assert m.match_routes(b"a/x") == rt.match_routes(b"a/x")  # the reference's answer
    delays = []
    while not m.repair():
        delays.append(m.backoff_ms)
    assert delays == [200, 400]  # (100 after init's failure, then doubled)
    assert m.published and m.healthy()
    _committed_is_table(eng, rt, [b"a/#"])


def test_resync_pending_filter_set_synchronously_is_committed(fakelib):
    """a resync chunk sets topic X (pending, uncommitted); the writing node's
    hook for X then finds nothing to change.  Its commit must still include X: the node's next
    publish sees X before the resync's own commit."""
    eng, rt = Engine(library=fakelib), R.Router()
    m = RouteTableMirror([eng], rt)
    m.init()
    rt.add_route(b"bulk/+/x", "n1")
    rt.add_route(b"other/#", "n1")
    gens = [e.sync_begin() for e in m.engines]
    m._dests([b"bulk/+/x", b"other/#"], commit=False)  # the resync's chunk: pending
    assert not eng.route_member(b"bulk/+/x")
    assert m.route_changed(b"bulk/+/x") == "ok"  # the hook: the same state, synchronously
    assert eng.route_member(b"bulk/+/x") and eng.trie_member(b"bulk/+/x")
    assert not eng.route_member(b"other/#")  # the rest of the chunk stays the resync's
    for e, g in zip(m.engines, gens):
        e.sync_end(g)
    m.commit()
    _committed_is_table(eng, rt, [b"bulk/+/x", b"other/#"])


@pytest.mark.parametrize("seed", [1, 2])
def test_random_failures_never_offer_a_diverged_index(fakelib, seed):
    """Random churn through the hooks and the mirror with random injected commit failures and
    host marks; after every step the invariant holds, and after the final repair the committed
    state is the table's."""
    rng = random.Random(seed)
    engs = [Engine(library=fakelib) for _ in range(1 + seed % 2)]
    rt = R.Router()
    words = [b"a", b"b", b"+", b"#", b"c"]
    topics = set()
    m = RouteTableMirror(engs, rt)
    m.init()
    for step in range(300):
        n = rng.randint(1, 3)
        ws = [rng.choice(words) for _ in range(n)]
        if b"#" in ws:
            ws = ws[:ws.index(b"#") + 1]
        t = b"/".join(ws)
        topics.add(t)
        r = rng.random()
        if r < 0.1:
            rng.choice(engs).tune("fail_commits", 1)
        elif r < 0.13:
            rng.choice(engs).mark_stale(errno.ETIMEDOUT)
        if rng.random() < 0.6:
            rt.add_route(t, rng.choice(["n1", "n2"]))
        else:
            for _, d in rt.lookup_routes(t)[:1]:
                rt.delete_route(t, d)
        if rng.random() < 0.7:
            assert m.route_changed(t) == "ok"
        else:
            m.event("write", t)
            m.handle_events()
        if m.repair_pending and rng.random() < 0.3:
            m.repair()
        for e in engs:
            if m.published and e.health()["stale"] == 0:
                _committed_is_table(e, rt, topics)
            else:
                with pytest.raises(EngineError, match="ESTALE"):
                    e.match([b"a/b"])
    for e in engs:
        e.tune("fail_commits", 0)
    assert m.repair()
    for e in engs:
        _committed_is_table(e, rt, topics)
