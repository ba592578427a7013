"""Delta commits: a commit with a small delta patches the committed device
tables in place (gm_engine.cpp commit_delta) instead of rebuilding them.  Every step of a random
subscribe / unsubscribe churn is checked against the Python oracle (oracle/emqx_ref.py Trie,
restating emqx_trie insert/delete/match) and against an engine that rebuilds on every commit.
"""
import random

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


VOCAB = ["a", "b", "", "$x", "c", "dd", "long-level-name-%d", "sensor"]


def _word(rng):
    w = rng.choice(VOCAB)
    return w % rng.randint(0, 3) if "%" in w else w


def _filter(rng):
    d = rng.randint(1, 6)
    ws = []
    for i in range(d):
        r = rng.random()
        ws.append("#" if (i == d - 1 and r < 0.15) else ("+" if r < 0.35 else _word(rng)))
    return "/".join(ws).encode()


def _topics(rng, n):
    return ["/".join(_word(rng) for _ in range(rng.randint(1, 7))).encode() for _ in range(n)]


def _check(eng, py, keys, topics):
    res = eng.match(topics)
    for i, t in enumerate(topics):
        got = sorted(eng.filter_bytes(int(f)) for f in res.row(i))
        assert got == sorted(py.match(t)), t
        ex = int(res.exact_id[i])
        if t in keys:
            assert ex != 0xFFFFFFFF and eng.filter_bytes(ex) == t
        else:
            assert ex == 0xFFFFFFFF, t
    return res


@pytest.mark.parametrize("bits", [0, 3])
def test_delta_churn_vs_oracle_and_full_build(emqx, bits):
    rng = random.Random(11 + bits)
    delta = emqx.Engine(word_hash_bits=bits)
    delta.tune("delta_commit", 2)
    full = emqx.Engine(word_hash_bits=bits)
    full.tune("delta_commit", 0)
    py = R.Trie()
    live, keys = set(), set()
    for step in range(40):
        for _ in range(rng.randint(1, 60)):
            r = rng.random()
            if r < 0.45 or not live:
                f = _filter(rng)
                for e in (delta, full):
                    e.trie_insert(f)
                py.insert(f)
                live.add(f)
            elif r < 0.8:
                f = rng.choice(sorted(live))
                for e in (delta, full):
                    e.trie_delete(f)
                py.delete(f)
                live.discard(f)
            elif r < 0.92:
                # route keys of both kinds: plain names and wildcard filter strings (the two
                # regions of the exact table)
                k = rng.choice(_topics(rng, 1)) if rng.random() < 0.5 else _filter(rng)
                if k not in keys:
                    for e in (delta, full):
                        e.route_ref(k)
                    keys.add(k)
            elif keys:
                k = rng.choice(sorted(keys))
                for e in (delta, full):
                    e.route_unref(k)
                keys.discard(k)
        delta.commit()
        full.commit()
        topics = _topics(rng, 400) + sorted(keys)[:50] + [f.replace(b"+", b"q").replace(b"#", b"z")
                                                          for f in sorted(live)[:50]]
        topics += sorted(live)[:30]  # wildcard names: exact key lookup only (emqx_router.erl:143)
        a = _check(delta, py, keys, topics)
        b = full.match(topics)
        assert np.array_equal(a.row_ptr, b.row_ptr)
        for i in range(len(topics)):
            assert sorted(a.row(i)) == sorted(b.row(i))
        assert delta.trie_empty() == (not live)
    st = delta.stats()
    assert full.stats()["delta_commits"] == 0
    if bits == 0:  # (3-bit test tokens collide into multi[] lists: those deltas rebuild)
        assert st["delta_commits"] >= 30, st  # most commits patched in place
        assert st["n_trie_filters"] == len(live) and st["n_route_keys"] == len(keys)
    delta.close()
    full.close()


def test_delta_delete_everything_then_reinsert(emqx):
    """Tombstoned slots and exact entries are reused; an index emptied by deltas answers
    empty, and refilled answers as before."""
    rng = random.Random(3)
    eng = emqx.Engine()
    eng.tune("delta_commit", 2)
    filters = sorted({_filter(rng) for _ in range(300)})
    keys = sorted(set(_topics(rng, 200)))
    topics = _topics(rng, 500) + keys
    for f in filters:
        eng.trie_insert(f)
    for k in keys:
        eng.route_ref(k)
    eng.commit()
    py = R.Trie()
    for f in filters:
        py.insert(f)
    _check(eng, py, set(keys), topics)
    for f in filters:
        eng.trie_delete(f)
    for k in keys:
        eng.route_unref(k)
    eng.commit()
    assert eng.trie_empty()
    _check(eng, R.Trie(), set(), topics)
    for f in filters:  # same filters again: same ids, slots reused
        eng.trie_insert(f)
    for k in keys:
        eng.route_ref(k)
    eng.commit()
    _check(eng, py, set(keys), topics)
    st = eng.stats()
    assert st["full_commits"] == 2 and st["delta_commits"] == 2, st  # create + first load


def test_delta_growth_falls_back_to_full_build(emqx):
    """Deltas that would push a table past its load bound rebuild instead (auto mode)."""
    eng = emqx.Engine()
    py = R.Trie()
    for r in range(8):
        batch = [f"g{r}/{i}/+/x{i % 7}".encode() for i in range(200 * (r + 1))]
        for f in batch:
            eng.trie_insert(f)
            py.insert(f)
        eng.commit()
        topics = [f"g{r}/{i}/k/x{i % 7}".encode() for i in range(0, 200 * (r + 1), 3)]
        _check(eng, py, set(), topics)
    st = eng.stats()
    assert st["full_commits"] >= 2 and st["delta_commits"] >= 1, st


def test_delta_publish_fanout_tables_follow(emqx):
    """Fan-out tables are rebuilt on a delta commit when routes or subscribers changed."""
    b = emqx.Broker()
    b.subscribe(b"t/+", "s1")
    b.commit()
    assert b.publish(b"t/1") == ([(b"t/+", b.node)], [(b"t/+", "s1")])
    b.subscribe(b"t/1", "s2")
    b.add_route(b"t/#", "other@node")
    assert sorted(b.publish(b"t/1")[0]) == sorted([(b"t/+", b.node), (b"t/1", b.node),
                                                   (b"t/#", "other@node")])
    b.unsubscribe(b"t/+", "s1")
    ent, dl = b.publish(b"t/1")
    assert sorted(ent) == sorted([(b"t/1", b.node), (b"t/#", "other@node")])
    assert dl == [(b"t/1", "s2")]
    assert b.engine.stats()["delta_commits"] >= 2


def test_snapshot_roundtrip(emqx, tmp_path):
    """emqxgm_snapshot_save / _load: a fresh engine restored from a snapshot answers exactly as
    the saved one (trie rows, exact ids, publish fan-out) and keeps taking delta commits."""
    import workloads
    w = workloads.generate(2, 30000, 20000)
    eng = emqx.Engine()
    eng.set_local_node(1)
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.nonzero(w.fwild)[0]
    eng.trie_insert_many(*_subset(w, wi))
    for i in range(0, w.nf, 97):
        eng.route_add(w.filter(i), 1 + i % 2)
        eng.subscriber_add(w.filter(i), i % 5)
    eng.commit()
    eng.trie_insert(b"#")  # a pending change: save commits it first
    p = str(tmp_path / "idx.snap")
    eng.snapshot_save(p)
    want = eng.match_packed(w.tbytes, w.toff)
    wpub = eng.publish([w.topic(i) for i in range(2000)])
    got_eng = emqx.Engine()
    got_eng.snapshot_load(p)
    got = got_eng.match_packed(w.tbytes, w.toff)
    assert np.array_equal(got.row_ptr, want.row_ptr)
    assert np.array_equal(got.filter_id, want.filter_id)
    assert np.array_equal(got.exact_id, want.exact_id)
    gpub = got_eng.publish([w.topic(i) for i in range(2000)])
    for a, b in ((gpub.route_ptr, wpub.route_ptr), (gpub.route_filter, wpub.route_filter),
                 (gpub.route_dest, wpub.route_dest), (gpub.deliver_sub, wpub.deliver_sub)):
        assert np.array_equal(a, b)
    assert got_eng.stats()["n_trie_filters"] == eng.stats()["n_trie_filters"]
    # delta commits continue on the restored model
    for e in (eng, got_eng):
        e.trie_delete(b"#")
        e.trie_insert(b"l0w1/+/#")
        e.commit()
    assert got_eng.stats()["delta_commits"] >= 1
    a, b = eng.match_packed(w.tbytes, w.toff), got_eng.match_packed(w.tbytes, w.toff)
    assert np.array_equal(a.row_ptr, b.row_ptr) and np.array_equal(a.filter_id, b.filter_id)
    with pytest.raises(emqx.EngineError):
        got_eng.snapshot_load(p)  # not a fresh handle
    eng.close()
    got_eng.close()


def _subset(w, idx):
    lens = (w.foff[idx + 1] - w.foff[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    starts = w.foff[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
    return w.fbytes[pos], off
