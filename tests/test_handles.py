"""Bounded handle tables: the handle registry
(emqxgm_handles_*, gm_async.cpp) and the mirror's handle table (emqx_amd/mirror.py Handles, the
restatement of src/emqx_trie_gpu.erl term_handle/2 and subscriber_down/1) under client churn, on
the CPU.  The reference removes every trace of a subscriber pid when it goes down
(emqx_broker.erl:361-380, emqx_broker_helper.erl:133-165); here a pid's handle is released after
the commits that removed it from every list, and reused -- so the registry, the mirror's table and
the NIF's term table (one slot per number) stay as large as the live subscribers, not as every
pid ever seen.  The publish answers under churn with reuse are checked against
oracle.emqx_ref.publish on the GPU (tests/test_gpu_handles.py)."""
import random

import pytest

from emqx_amd.engine import Engine, EngineError, HandleRegistry, load_library
from emqx_amd.mirror import RouteTableMirror
from oracle import emqx_ref as R
from tests.test_route_mirror import build_fake_lib


@pytest.fixture(scope="module")
def fakelib():
    return load_library(build_fake_lib(), allow_missing=True)


def test_registry_rules(fakelib):
    r = HandleRegistry(library=fakelib)
    assert [r.alloc("sub") for _ in range(3)] == [0, 1, 2]
    assert r.alloc("node") == 0  # kinds number independently
    r.release("sub", 1)
    with pytest.raises(EngineError, match="ENOENT"):
        r.release("sub", 1)
    with pytest.raises(EngineError, match="ENOENT"):
        r.release("sub", 7)
    assert r.alloc("sub") == 1  # no layer: nothing in flight, reused at once
    assert r.stats("sub") == {"made": 3, "live": 3, "waiting": 0, "free": 0}
    r.reset()
    assert r.stats("sub")["live"] == 0 and r.stats("node")["live"] == 0
    assert sorted(r.alloc("sub") for _ in range(4)) == [0, 1, 2, 3]


def test_registry_churn_one_million(fakelib):
    """1M short-lived subscribers through the mirror's handle table and the registry: at most
    LIVE alive at once, so no more than LIVE numbers are ever made and the table holds LIVE."""
    r = HandleRegistry(library=fakelib)
    m = RouteTableMirror([], R.Router(), registry=r)
    rng = random.Random(1)
    LIVE = 2000
    alive = []
    for k in range(1_000_000):
        alive.append(("pid", k))
        m.handles("sub", alive[-1])
        if len(alive) > LIVE:
            m.subscriber_down(alive.pop(rng.randrange(len(alive))))
    st = r.stats("sub")
    assert st["made"] <= LIVE + 1 and st["live"] == LIVE, st
    assert len(m.handles.ids) == LIVE + 1 and len(m.handles.names["sub"]) == LIVE  # (+ node n1)


def test_churn_through_the_engine_stays_bounded(fakelib):
    """200k short-lived subscribers over 64 topics through the hooks of the real engine host code:
    each join / leave a committed subscribers_changed/1, each leave then subscriber_down/1.  The
    numbers stay bounded; the committed lists always name live handles only (checked through a
    full resync: sync_end clears a list the resync did not give -- a topic whose subscribers all
    left -- so no released number survives in a list)."""
    eng = Engine(library=fakelib)
    rt = R.Router()
    topics = [b"t/%d/+" % i for i in range(64)]
    for t in topics:
        rt.add_route(t, "n1")
    subs = {t: [] for t in topics}
    r = HandleRegistry(library=fakelib)
    m = RouteTableMirror([eng], rt, subscribers=subs, registry=r)
    m.init()
    rng = random.Random(2)
    where = {}
    LIVE = 500
    for k in range(200_000):
        t = topics[rng.randrange(64)]
        pid = ("pid", k)
        subs[t].append(pid)
        where[pid] = t
        m.subscribers_changed(t)
        if len(where) > LIVE:
            old = rng.choice(list(where)) if k % 97 == 0 else next(iter(where))
            ot = where.pop(old)
            subs[ot].remove(old)
            m.subscribers_changed(ot)  # the lists without it, committed ...
            m.subscriber_down(old)     # ... then its handle goes back
        if k % 50_000 == 0:
            m.repair()  # a periodic resync in the middle of the churn
    st = r.stats("sub")
    assert st["made"] <= LIVE + 2 and st["live"] == LIVE, st
    assert eng.health()["stale"] == 0
    # every topic's subscribers gone: the lists empty out; a resync keeps them empty
    for t in topics:
        for pid in list(subs[t]):
            subs[t].remove(pid)
            where.pop(pid)
            m.subscribers_changed(t)
            m.subscriber_down(pid)
    assert r.stats("sub")["live"] == 0
    assert m.repair()
