"""Handle reuse on the MI355X: a publish layer (EMQXGM_ASYNC_PUBLISH, the
NIF's publish_async/3), the handle registry over it (emqxgm_handles_*) and the mirror's hooks
(emqx_amd/mirror.py: subscribers_changed/1 after each join / leave, subscriber_down/1 after each
leave) under client churn: 20k short-lived subscribers, at most 300 alive, so handle numbers are
reused thousands of times.  After every burst each published topic's answer -- aggre/1 entries and
local dispatches, the handles mapped back to their terms -- equals oracle.emqx_ref.publish
(emqx_broker.erl:218-355) for the table and subscribers of that moment, and the registry made no
more numbers than were ever alive at once."""
import random

import pytest

from emqx_amd.mirror import RouteTableMirror
from oracle import emqx_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


def test_publish_answers_under_churn_with_reused_handles(emqx):
    rng = random.Random(3)
    rt = R.Router()
    filters = [b"s/%d/+" % i for i in range(40)] + [b"s/%d/#" % i for i in range(0, 40, 3)] + \
        [b"s/%d/x" % i for i in range(40)]
    for f in filters:
        rt.add_route(f, rng.choice(["n1", "n1", "n2", ("g", "n1")]))
    subs = {f: [] for f in filters if any(d == "n1" for _, d in rt.lookup_routes(f))}
    eng = emqx.Engine()
    am = emqx.AsyncMatcher([eng], window_us=20, publish=True)
    reg = emqx.engine.HandleRegistry([am])
    m = RouteTableMirror([eng], rt, subscribers=subs, registry=reg)
    m.init()
    names = m.handles.names
    where, LIVE, k, tag = {}, 300, 0, 0
    topics = [b"s/%d/x" % i for i in range(40)] + [b"s/%d/y/z" % i for i in range(40)]
    for burst in range(40):
        for _ in range(500):
            f = rng.choice(list(subs))
            pid = ("pid", k)
            k += 1
            subs[f].append(pid)
            where[pid] = f
            m.subscribers_changed(f)
            if len(where) > LIVE:
                old = rng.choice(list(where))
                of = where.pop(old)
                subs[of].remove(old)
                m.subscribers_changed(of)
                m.subscriber_down(old)
        keys = []
        for t in rng.sample(topics, 20):
            tag += 1
            assert am.match(t, tag) == 0
            keys.append((tag, t))
        assert am.wait([(x, 0) for x, _ in keys], timeout=30)
        for x, t in keys:
            r = am.results.pop((x, 0))
            assert r.status == 0
            got_e = sorted(((to, names["group"][d & ~emqx.engine.DEST_GROUP]
                             if d & emqx.engine.DEST_GROUP else names["node"][d])
                            for to, d in r.routes), key=repr)
            got_d = sorted(((to, names["sub"][s]) for to, s in r.deliveries), key=repr)
            want_e, want_d = R.publish(rt, t, "n1", subs)
            assert got_e == sorted(want_e, key=repr), t
            assert got_d == sorted(want_d, key=repr), (burst, t)
    st = reg.stats("sub")
    assert st["made"] <= LIVE + 8 and st["live"] == LIVE, st
    assert k == 20_000
    am.close()
    eng.close()
