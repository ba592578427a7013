"""Failing closed at the boundary on the MI355X (SURVEY 5 "Failure
detection"): the real engine and the concurrent entry (emqxgm_async_*, the NIF's match_async/3 and
publish_async/3), the mirror and hooks of emqx_amd/mirror.py over the oracle's route bag
(oracle.emqx_ref.Router: emqx_router.erl:124-188, emqx_router_utils.erl:34-71).

Failures come through emqxgm_tune: "fail_commits" (the hook's EMQXGM_SET_COMMIT commit fails with
-ENOMEM / -EIO) and "hang_ms" (every window's wait stalls past the publishers' timeout: a window
that does not complete).  Every answer a publisher gets -- from the device when it is offered,
from the reference's path (the oracle's match_routes, standing in for ETS) when the call is
refused (-ESTALE) or times out -- must equal oracle.emqx_ref.Router.match_routes of the table as
of the last hook that returned; the device must be offered again after the mirror's repair."""
import errno
import random
import time

import pytest

from emqx_amd.mirror import RouteTableMirror
from oracle import emqx_ref as R

pytestmark = pytest.mark.gpu
NONE = 0xFFFFFFFF
ESTALE = -errno.ESTALE


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def _key(routes):
    return sorted((t, str(d)) for t, d in routes)


def _table(seed=5, n=400):
    rng = random.Random(seed)
    rt = R.Router()
    words = [b"a", b"b", b"c", b"dev", b"+", b"#"]
    for _ in range(n):
        k = rng.randint(1, 4)
        ws = [rng.choice(words) for _ in range(k)]
        if b"#" in ws:
            ws = ws[:ws.index(b"#") + 1]
        rt.add_route(b"/".join(ws), rng.choice(["n1", "n2", ("g", "n1")]))
    topics = [b"/".join(rng.choice([b"a", b"b", b"c", b"dev", b"x"]) for _ in range(rng.randint(1, 4)))
              for _ in range(300)]
    return rt, topics


def _check_sync(m, rt, topics):
    """mirror.match_routes (device when offered, else the reference) == the oracle's."""
    for t in topics:
        assert _key(m.match_routes(t)) == _key(rt.match_routes(t)), t


def _async_routes(am, eng, rt, topics, timeout_s, tag0):
    """Each topic through the concurrent entry as a publisher does (src/emqx_trie_gpu.erl
    device_match/3): accepted calls waited for up to timeout_s, then cancelled; refused, failed or
    timed-out calls answered by the reference's path.  Returns (answers, outcome counts)."""
    out, n = [], {"device": 0, "refused": 0, "timeout": 0, "failed": 0}
    for i, t in enumerate(topics):
        tag = tag0 + i
        rc = am.match(t, tag)
        if rc != 0:
            assert rc in (ESTALE, -errno.EBUSY), rc
            n["refused"] += 1
            out.append(rt.match_routes(t))
            continue
        if not am.wait([(tag, 0)], timeout=timeout_s):
            if am.cancel(tag):
                n["timeout"] += 1
                out.append(rt.match_routes(t))
                continue
            assert am.wait([(tag, 0)], timeout=5.0)
        r = am.results.pop((tag, 0))
        if r.status != 0:
            n["failed"] += 1
            out.append(rt.match_routes(t))
            continue
        n["device"] += 1
        heads = ([t] if r.exact_id != NONE else []) + list(r.filters)
        out.append([x for f in heads for x in rt.lookup_routes(f)])
    return out, n


@pytest.mark.parametrize("err", [errno.ENOMEM, errno.EIO])
def test_refused_hook_commit_never_answers_from_the_diverged_index(emqx, err):
    rt, topics = _table()
    eng = emqx.Engine()
    m = RouteTableMirror([eng], rt)
    m.init()
    am = emqx.AsyncMatcher([eng], window_us=20, fail_threshold=3)
    try:
        _check_sync(m, rt, topics)
        got, n = _async_routes(am, eng, rt, topics[:50], 5.0, 1)
        assert n["device"] == 50
        # the writing node's subscribe: the route is in the table, the device refuses the commit
        eng.tune("fail_errno", err)
        eng.tune("fail_commits", 1)
        rt.add_route(b"dev/+/x", "n1")
        rt.add_route(b"a/#", "n3")
        assert m.route_changed(b"dev/+/x") == "ok"
        assert eng.health()["stale"] and m.repair_pending
        probe = topics + [b"dev/a/x", b"dev/q/x", b"a/b/c"]
        _check_sync(m, rt, probe)  # every answer is the reference's now
        got, n = _async_routes(am, eng, rt, probe, 5.0, 1000)
        assert n["device"] == 0 and n["refused"] == len(probe)
        for t, g in zip(probe, got):
            assert _key(g) == _key(rt.match_routes(t))
        # the second hook commits fine but the engine stays stale until the repair
        assert m.route_changed(b"a/#") == "ok"
        assert am.match(b"a/b", 5000) == ESTALE
        assert m.repair()
        assert eng.health() ["stale"] == 0 and eng.health()["repairs"] == 1
        got, n = _async_routes(am, eng, rt, probe, 5.0, 2000)
        assert n["device"] == len(probe)
        for t, g in zip(probe, got):
            assert _key(g) == _key(rt.match_routes(t)), t
        _check_sync(m, rt, probe)
    finally:
        am.close()
        eng.close()


def test_publish_layer_refuses_while_stale(emqx):
    """A publish layer (EMQXGM_ASYNC_PUBLISH): its windows' emqxgm_publish_batch refuses a stale
    index; calls are refused up front once every handle is stale."""
    rt, topics = _table(seed=9, n=100)
    eng = emqx.Engine()
    m = RouteTableMirror([eng], rt)
    m.init()
    am = emqx.AsyncMatcher([eng], window_us=20, publish=True, fail_threshold=3)
    try:
        assert am.match(topics[0], 1) == 0 and am.wait([(1, 0)], 5.0)
        assert am.results[(1, 0)].status == 0
        eng.tune("fail_commits", 1)
        rt.add_route(b"new/#", "n1")
        m.route_changed(b"new/#")
        assert am.match(topics[0], 2) == ESTALE
        assert am.health()["refused"] >= 1
        assert m.repair()
        assert am.match(b"new/1", 3) == 0 and am.wait([(3, 0)], 5.0)
        r = am.results[(3, 0)]
        assert r.status == 0 and (b"new/#", 0) in [(to, d) for to, d in r.routes]
    finally:
        am.close()
        eng.close()


def test_hung_window_costs_one_timeout_then_refuses_until_repair(emqx):
    """hang_ms: every window's wait stalls 1.5 s; publishers time out after 0.1 s and cancel.
    After fail_threshold (3) timeouts every later call is refused at once (-ESTALE), and only a
    few calls ever pay the timeout; answers stay the reference's; after the stall ends the
    mirror's repair (resync, commit, stream probe) offers the device again."""
    rt, topics = _table(seed=11)
    eng = emqx.Engine()
    m = RouteTableMirror([eng], rt)
    m.init()
    am = emqx.AsyncMatcher([eng], window_us=20, fail_threshold=3)
    try:
        eng.tune("hang_ms", 1500)
        t0 = time.time()
        got, n = _async_routes(am, eng, rt, topics[:40], 0.1, 1)
        dt = time.time() - t0
        for t, g in zip(topics[:40], got):
            assert _key(g) == _key(rt.match_routes(t))
        assert n["timeout"] == 3 and n["refused"] == 37, n  # one publisher: three timeouts, then refused
        assert dt < 3.0, dt
        assert am.health()["stale_handles"] == 1 and am.health()["timeouts"] == 3
        eng.tune("hang_ms", 0)
        time.sleep(2.0)  # the stalled windows finish (their cancelled calls are not reported)
        assert m.repair() and eng.health()["stale"] == 0
        got, n = _async_routes(am, eng, rt, topics, 5.0, 1000)
        assert n["device"] == len(topics), n
        for t, g in zip(topics, got):
            assert _key(g) == _key(rt.match_routes(t)), t
    finally:
        eng.tune("hang_ms", 0)
        am.close()
        eng.close()


def test_two_engines_one_refuses(emqx):
    """Two engines (two GPUs' replicas, here both on device 0): one refuses the hook's commit.
    It is stale and takes no windows; the other got the change and answers every call."""
    rt, topics = _table(seed=13, n=200)
    e0, e1 = emqx.Engine(), emqx.Engine()
    m = RouteTableMirror([e0, e1], rt)
    m.init()
    am = emqx.AsyncMatcher([e0, e1], window_us=20, fail_threshold=3)
    try:
        e0.tune("fail_commits", 1)
        rt.add_route(b"c/+/z", "n2")
        assert m.route_changed(b"c/+/z") == "ok"
        assert e0.health()["stale"] and not e1.health()["stale"]
        probe = topics[:100] + [b"c/a/z", b"c/dev/z"]
        got, n = _async_routes(am, e1, rt, probe, 5.0, 1)
        assert n["device"] == len(probe), n
        for t, g in zip(probe, got):
            assert _key(g) == _key(rt.match_routes(t)), t
        assert m.repair() and m.healthy()
    finally:
        am.close()
        e0.close()
        e1.close()
