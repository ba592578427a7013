"""GPU parity of the publish fan-out (emqx_broker:publish/1 -> route(aggre(match_routes(T)))):
the engine's emqxgm_publish_batch through emqx_amd.Broker against oracle/emqx_ref.publish,
which restates emqx_broker.erl:218-300 and dispatch/2 (:326-355).  Entries and dispatches are
compared as sets per topic (route/2 folds over them; the engine's order is deterministic but
not the reference's fold order)."""
import random

import pytest

from oracle import emqx_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def emqx():
    import torch
    assert torch.cuda.is_available(), "gpu tests need the MI355X"
    import emqx_amd
    return emqx_amd


class _Both:
    """The same subscribe / route operations applied to the engine Broker and the oracle."""

    def __init__(self, emqx, node="n1"):
        self.b = emqx.Broker(node=node)
        self.r = R.Router()
        self.node = node
        self.subs = {}

    def subscribe(self, t, s):
        self.b.subscribe(t, s)
        lst = self.subs.setdefault(t, [])
        if s not in lst:
            lst.append(s)
            if len(lst) == 1:
                self.r.add_route(t, self.node)

    def unsubscribe(self, t, s):
        self.b.unsubscribe(t, s)
        lst = self.subs.get(t, [])
        if s in lst:
            lst.remove(s)
            if not lst:
                del self.subs[t]
                self.r.delete_route(t, self.node)

    def add_route(self, t, d):
        self.b.add_route(t, d)
        self.r.add_route(t, d)

    def delete_route(self, t, d):
        self.b.delete_route(t, d)
        self.r.delete_route(t, d)

    def check(self, topics):
        got = self.b.publish_batch(topics)
        for t, (entries, deliveries) in zip(topics, got):
            we, wd = R.publish(self.r, t, self.node, self.subs)
            assert sorted(entries, key=repr) == sorted(we, key=repr), t
            assert sorted(deliveries, key=repr) == sorted(wd, key=repr), t
        return got


def test_publish_hand_cases(emqx):
    x = _Both(emqx)
    x.subscribe(b"a/+", "s1")
    x.subscribe(b"a/+", "s2")
    x.subscribe(b"a/b", "s3")
    x.add_route(b"a/+", "n2")
    x.add_route(b"a/#", (b"g", "n2"))
    x.add_route(b"a/#", (b"g", "n3"))  # same group on two nodes: one {To, Group} entry
    x.add_route(b"a/#", (b"h", "n3"))
    x.add_route(b"#", "n3")
    x.add_route(b"$SYS/#", "n2")
    got = x.check([b"a/b", b"a", b"a/c", b"b", b"$SYS/x", b"a/+", b""])
    entries, deliveries = got[0]
    assert (b"a/#", b"g") in entries and entries.count((b"a/#", b"g")) == 1
    assert sorted(deliveries) == [(b"a/+", "s1"), (b"a/+", "s2"), (b"a/b", "s3")]
    # wildcard topic name: only its own exact routes (emqx_router.erl:143, trie [] )
    assert sorted(got[5][0], key=repr) == sorted([(b"a/+", "n1"), (b"a/+", "n2")], key=repr)
    # unsubscribing the last local subscriber drops {To, node()} (and the trie key if last)
    x.unsubscribe(b"a/b", "s3")
    x.unsubscribe(b"a/+", "s1")
    x.delete_route(b"#", "n3")
    x.check([b"a/b", b"a/c", b"b"])
    x.unsubscribe(b"a/+", "s2")
    x.delete_route(b"a/+", "n2")
    got = x.check([b"a/b", b"a/c"])
    assert all(f != b"a/+" for f, _ in got[0][0])


def test_publish_random(emqx):
    import workloads
    w = workloads.generate(1, 3000, 6000)
    rng = random.Random(5)
    x = _Both(emqx)
    filters = [w.filter(i) for i in range(w.nf)]
    for f in filters:
        k = rng.random()
        if k < 0.5:
            for s in rng.sample(range(40), rng.randint(1, 3)):
                x.subscribe(f, f"s{s}")
        if k > 0.3:
            x.add_route(f, rng.choice(["n2", "n3", "n4"]))
        if rng.random() < 0.2:
            x.add_route(f, (rng.choice([b"g1", b"g2"]), rng.choice(["n1", "n2", "n3"])))
    # exact (non-wildcard) route keys too
    topics = [w.topic(i) for i in range(w.nt)]
    for t in topics[:300]:
        x.subscribe(t, "exact-sub")
    x.check(topics)
    # churn, then again
    for f in rng.sample(filters, 400):
        x.unsubscribe(f, f"s{rng.randrange(40)}")
        x.delete_route(f, "n2")
    x.check(topics[:3000])


def test_publish_churn_delta_commits(emqx):
    """Rounds of subscribe / unsubscribe / route churn, each committed as a delta: the fan-out
    entries of changed filters are re-pointed at appended lists (gm_engine.cpp fan_commit),
    and every round's publish fan-out equals the oracle's."""
    rng = random.Random(17)
    x = _Both(emqx)
    vocab = ["a", "b", "c", "+", "dd"]
    filters = sorted({"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 4))).encode()
                      for _ in range(400)} | {b"#", b"a/#", b"+/#"})
    topics = ["/".join(rng.choice(["a", "b", "c", "dd", "e"]) for _ in range(rng.randint(1, 5)))
              .encode() for _ in range(1500)]
    for f in filters[:200]:
        x.subscribe(f, f"s{rng.randrange(20)}")
    x.check(topics)
    for _ in range(12):
        for _ in range(rng.randint(5, 60)):
            f = rng.choice(filters)
            r = rng.random()
            if r < 0.35:
                x.subscribe(f, f"s{rng.randrange(20)}")
            elif r < 0.6:
                x.unsubscribe(f, rng.choice(x.subs.get(f, ["none"])))
            elif r < 0.75:
                x.add_route(f, rng.choice(["n2", "n3"]))
            elif r < 0.85:
                x.add_route(f, (rng.choice([b"g1", b"g2"]), rng.choice(["n1", "n2"])))
            else:
                x.delete_route(f, rng.choice(["n2", "n3", (b"g1", "n1"), (b"g2", "n2")]))
        x.check(topics)
    st = x.b.engine.stats()
    assert st["delta_commits"] >= 10, st
