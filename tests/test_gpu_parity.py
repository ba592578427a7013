"""GPU parity: the HIP engine (through the C-ABI) against the oracle, bit-exact.

Every test here runs on a real MI355X (``-m gpu``).  Expected results come from the oracle
(oracle/emqx_ref.py for golden/edge cases, oracle/ref_trie.cpp for the synthetic configs),
which is itself pinned to the reference's own suites (tests/test_oracle_*.py).
"""
import random

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


def B(s):
    return s.encode()


def _rows_as_sets(engine, res, n):
    return [sorted(engine.filter_bytes(int(f)) for f in res.row(i)) for i in range(n)]


def _rows_sorted(row_ptr, ids):
    """The CSR's ids with every row sorted ascending (one lexsort over (row, id))."""
    n = len(row_ptr) - 1
    if ids.size == 0:
        return ids
    seg = np.repeat(np.arange(n, dtype=np.int64), np.diff(row_ptr.astype(np.int64)))
    return ids[np.lexsort((ids, seg))]


def _assert_engine_equals_ref(eng, ref, names, tbytes, toff):
    """Compare engine CSR rows (ids) with the C++ oracle (same registration order)."""
    res = eng.match_packed(tbytes, toff)
    row, ids, ex = ref.match(tbytes, toff, threads=16)
    assert len(res.row_ptr) == len(row)
    n = len(row) - 1
    # rows as sorted id lists; ids are equal because both registered filters in the same order
    assert np.array_equal(res.row_ptr, row)
    g_sorted = _rows_sorted(res.row_ptr, res.filter_id)
    assert np.array_equal(g_sorted, ids)
    assert np.array_equal(res.exact_id, ex)
    return res


# ---------------------------------------------------------------- reference suites on device

@pytest.mark.parametrize("compact", [True, False])
def test_trie_suite_on_device(emqx, golden, compact):
    for case, steps in golden["trie_cases"].items():
        trie = emqx.Trie()
        trie.set_compact(compact)
        for step in steps:
            op = step[0]
            if op == "insert":
                with trie.transaction():
                    for f in step[1]:
                        trie.insert(B(f))
            elif op == "delete":
                with trie.transaction():
                    for f in step[1]:
                        trie.delete(B(f))
            elif op == "match":
                assert sorted(trie.match(B(step[1]))) == [B(x) for x in step[2]], (case, step)
            elif op == "match_len":
                assert len(trie.match(B(step[1]))) == step[2], (case, step)
            elif op == "empty":
                assert trie.empty() is step[1], (case, step)
            elif op == "lookup_topic":
                assert trie.lookup_topic(B(step[1])) == [B(x) for x in step[2]], (case, step)
        trie.engine.close()


def test_session_router_churn_vs_oracle(emqx):
    """emqx_session_router (emqx_session_router.erl:126-176) over the session trie
    (emqx_trie.erl:117-176): random do_add_route / do_delete_route / delete_routes churn with
    session ids as dests, beside a main Router taking its own churn.  After every commit the
    session router's match_routes and Trie.match_session / empty_session equal the oracle's
    Router on a second table (oracle/emqx_ref.py Router = emqx_router's route assembly over its
    own bag and trie), and the main router's answers equal its own oracle: the two tables never
    see each other's routes."""
    rng = random.Random(17)
    vocab = ["a", "b", "", "$s", "c", "long-word-%d"]

    def word():
        w = rng.choice(vocab)
        return w % rng.randint(0, 2) if "%" in w else w

    def filt():
        d = rng.randint(1, 5)
        return "/".join("#" if i == d - 1 and rng.random() < 0.2 else
                        "+" if rng.random() < 0.35 else word() for i in range(d)).encode()

    trie = emqx.Trie()
    srt = emqx.SessionRouter(trie)
    main = emqx.Router()
    ref_s, ref_m = R.Router(), R.Router()
    filters = sorted({filt() for _ in range(300)})
    sessions = [f"session-{i}" for i in range(12)]
    topics = ["/".join(word() for _ in range(rng.randint(1, 6))).encode() for _ in range(400)]
    topics += filters[:20]  # wildcard names: exact lookups only
    live = []
    for step in range(14):
        for _ in range(rng.randint(20, 80)):
            op = rng.random()
            if op < 0.6 or not live:
                f, sid = rng.choice(filters), rng.choice(sessions)
                srt.do_add_route(f, sid)
                ref_s.add_route(f, sid)
                live.append((f, sid))
            elif op < 0.9:
                f, sid = live.pop(rng.randrange(len(live)))
                srt.do_delete_route(f, sid)
                ref_s.delete_route(f, sid)
            else:  # a session goes away: delete_routes(SessionID, Subscriptions)
                sid = rng.choice(sessions)
                subs = [f for f, s in live if s == sid]
                srt.delete_routes(sid, subs)
                for f in subs:
                    ref_s.delete_route(f, sid)
                live = [(f, s) for f, s in live if s != sid]
            if rng.random() < 0.3:
                f = rng.choice(filters)
                main.add_route(f, "node1")
                ref_m.add_route(f, "node1")
        got_s = srt.match_routes_batch(topics)
        got_m = main.match_routes_batch(topics)
        for i, t in enumerate(topics):
            assert sorted(got_s[i]) == sorted(ref_s.match_routes(t)), (step, t)
            assert sorted(got_m[i]) == sorted(ref_m.match_routes(t)), (step, t)
            assert sorted(trie.match_session(t)) == sorted(ref_s.match_trie(t)), (step, t)
        assert trie.empty_session() == ref_s.trie.empty()
    for f, sid in list(live):
        srt.do_delete_route(f, sid)
    assert trie.empty_session() and srt.match_routes(b"a/b") == []
    assert not main.engine.trie_empty() or ref_m.trie.empty()


def test_router_suite_on_device(emqx, golden):
    for case, steps in golden["router_cases"].items():
        r = emqx.Router()
        for step in steps:
            if step[0] == "add_route":
                for f, d in step[1]:
                    r.add_route(B(f), d)
            elif step[0] == "delete_route":
                for f, d in step[1]:
                    r.delete_route(B(f), d)
            elif step[0] == "match_routes":
                assert sorted(r.match_routes(B(step[1]))) == sorted(
                    (B(f), d) for f, d in step[2]), (case, step)


def test_match_vectors_as_single_filter_tries(emqx, golden):
    """Every emqx_topic:match/2 vector, asked as: does a trie holding only F return F for N."""
    cases = golden["match"] + golden["client_dollar"]
    eng = emqx.Engine()
    for name, filt, exp in cases:
        if not R.wildcard(B(filt)):
            continue  # exact filters are route keys, not trie members (emqx_router.erl:131-137)
        eng.trie_insert(B(filt))
    eng.commit()
    topics = [B(n) for n, _, _ in cases]
    res = eng.match(topics)
    for i, (name, filt, exp) in enumerate(cases):
        if not R.wildcard(B(filt)):
            continue
        got = eng.filter_bytes(eng.lookup_id(B(filt))) in {eng.filter_bytes(int(f)) for f in res.row(i)}
        assert got is exp, (name, filt)


def test_client_matrix(emqx, golden):
    topics = [B(t) for t in golden["client_topics"]] + [B(golden["client_dollar"][0][0])]
    wild = [B(w) for w in golden["client_wild"]]
    t = emqx.Trie()
    with t.transaction():
        for w in wild:
            t.insert(w)
    got = t.match_batch(topics)
    for i, topic in enumerate(topics):
        assert sorted(got[i]) == sorted(w for w in wild if R.match(topic, w)), topic


# ---------------------------------------------------------------- cfg5 edge semantics

EDGE_FILTERS = ["$SYS/#", "$SYS/+", "+/#", "#", "+", "/+", "/#", "+/+", "$share/g/#", "$share/g/x",
                "a/+", "a/#", "a//+", "+//b", "+/", "/", "a/+/#", "$x", "sport/+", "#/x",
                "a/#/b", "++", "a/b+", "$SYS", "+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#",
                "a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]
EDGE_TOPICS = ["$share/g/x", "$SYS", "$SYS/a", "", "/", "//", "a//b", "/a", "a/", "a", "a/b",
               "$x", "sport/", "sport", "a/+", "#", "+", "$SYS/+",
               "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z",
               "/".join(str(i) for i in range(32)), "/".join("w" for _ in range(128)),
               "/".join("w" for _ in range(129)), "x" * 65535]


def _edge_engine(emqx, **kw):
    eng = emqx.Engine(**kw)
    filters = [B(f) for f in EDGE_FILTERS]
    for f in filters:
        eng.trie_insert(f)
        eng.route_ref(f)
    for f in (b"a/b", b"a//b", b"", b"x" * 65535, b"$share/g/x"):
        eng.route_ref(f)
    eng.trie_insert(b"a/b")  # non-wildcard key inserted straight into the trie (t_insert style)
    eng.commit()
    return eng, filters


def _expected_edge(filters, topics):
    py = R.Trie()
    for f in filters + [b"a/b"]:
        py.insert(f)
    return [sorted(py.match(t)) for t in topics]


@pytest.mark.parametrize("bits", [(0, 64), (40, 64), (2, 3), (1, 1)])
def test_edge_semantics(emqx, bits):
    eng, filters = _edge_engine(emqx, word_hash_bits=bits[0], full_hash_bits=bits[1])
    topics = [B(t) for t in EDGE_TOPICS]
    res = eng.match(topics)
    exp = _expected_edge(filters, topics)
    keys = set(filters) | {b"a/b", b"a//b", b"", b"x" * 65535, b"$share/g/x"}
    for i, t in enumerate(topics):
        got = sorted(eng.filter_bytes(int(f)) for f in res.row(i))
        assert got == exp[i], (t[:40], got, exp[i])
        ex = int(res.exact_id[i])
        if t in keys:
            assert ex != emqx.NONE and eng.filter_bytes(ex) == t  # match_routes exact lookup
        else:
            assert ex == emqx.NONE


def test_wildcard_topic_routes_exact_only(emqx):
    r = emqx.Router()
    r.add_route(b"a/+")
    r.add_route(b"a/#")
    r.add_route(b"a/b")
    assert r.match_routes(b"a/+") == [(b"a/+", "node")]  # emqx_router.erl:143 exact key only
    assert sorted(r.match_routes(b"a/b")) == [(b"a/#", "node"), (b"a/+", "node"),
                                               (b"a/b", "node")]


@pytest.mark.parametrize("range_kb", [0, 1])
@pytest.mark.parametrize("full_bits", [64, 2])
@pytest.mark.parametrize("kinds", ["wild", "plain", "both"])
def test_route_key_regions(emqx, kinds, full_bits, range_kb):
    """Route keys live in two regions of the exact table (plain names, wildcard strings): a
    publish name only probes the region of its own kind.  Only-wildcard keys (the IoT-tree
    case: no probe for plain names at all), only-plain keys, both; 2-bit key hashes force every
    key of a region onto one probe chain; a 40 kB wildcard name takes the global-memory path.
    range_kb=1: the probe is partitioned over 16-bucket ranges (k_xhash + k_exact_part, the
    option for tables beyond the TLB's reach), chains running across range ends and the region
    boundary."""
    rng = random.Random(17)
    wild = [f"s/{i}/+/#".encode() for i in range(300)] + [b"+", b"#", b"a/+/b", b"+/+"]
    plain = [f"s/{i}/x/y".encode() for i in range(300)] + [b"", b"a", b"a//b", b"$SYS/x"]
    longw = b"/".join([b"w" * 50] * 800) + b"/+"
    keys = (wild + [longw] if kinds != "plain" else []) + (plain if kinds != "wild" else [])
    eng = emqx.Engine(full_hash_bits=full_bits)
    eng.tune("exact_range_kb", range_kb)
    for k in keys:
        eng.route_ref(k)
    eng.commit()
    names = wild + plain + [longw, longw[:-1] + b"#", b"s/1/+", b"s/1/x", b"s/1/x/y/z"]
    names += [f"s/{rng.randrange(400)}/x/y".encode() for _ in range(200)]
    rng.shuffle(names)
    res = eng.match(names)
    ks = set(keys)
    for i, t in enumerate(names):
        ex = int(res.exact_id[i])
        if t in ks:
            assert ex != emqx.NONE and eng.filter_bytes(ex) == t, t[:40]
        else:
            assert ex == emqx.NONE, t[:40]
    # delta commits move keys in and out of both regions
    eng.tune("delta_commit", 2)
    gone = set(rng.sample(sorted(ks), len(ks) // 3))
    for k in gone:
        eng.route_unref(k)
    new = [f"n/{i}/+".encode() for i in range(50)] + [f"n/{i}".encode() for i in range(50)]
    for k in new:
        eng.route_ref(k)
    eng.commit()
    ks = (ks - gone) | set(new)
    res = eng.match(names + new)
    for i, t in enumerate(names + new):
        ex = int(res.exact_id[i])
        assert (ex != emqx.NONE and eng.filter_bytes(ex) == t) if t in ks else ex == emqx.NONE
    eng.close()


def test_empty_batch_and_empty_index(emqx):
    eng = emqx.Engine()
    res = eng.match([])
    assert list(res.row_ptr) == [0] and res.filter_id.size == 0
    res = eng.match([b"a/b", b""])
    assert list(res.row_ptr) == [0, 0, 0] and list(res.exact_id) == [emqx.NONE] * 2
    eng.route_ref(b"a/b")
    eng.commit()
    res = eng.match([b"a/b", b""])
    assert list(res.row_ptr) == [0, 0, 0] and res.exact_id[0] != emqx.NONE


def test_commit_epochs_and_delete(emqx):
    t = emqx.Trie()
    with t.transaction():
        for f in (b"sensor/+", b"sensor/+/metric/2", b"sensor/#"):
            t.insert(f)
    assert sorted(t.match(b"sensor/1")) == [b"sensor/#", b"sensor/+"]
    e0 = t.engine.commit()
    t.delete(b"sensor/+")  # pending until commit: the committed epoch still answers
    assert sorted(t.engine.filter_bytes(int(f)) for f in t.engine.match([b"sensor/1"]).row(0)) == \
        [b"sensor/#", b"sensor/+"]
    assert t.engine.commit() == e0 + 1
    assert t.match(b"sensor/1") == [b"sensor/#"]
    t.delete(b"never/inserted")
    assert t.match(b"sensor/1") == [b"sensor/#"]


def test_many_matches_vs_oracle(emqx):
    eng = emqx.Engine()
    filters = [f"+/{i}/#".encode() for i in range(600)] + [f"+/{i}/+".encode() for i in range(600)]
    filters += [b"#", b"+/#", b"+/+/#"]
    for f in filters:
        eng.trie_insert(f)
    eng.commit()
    topics = [f"t{j}/{j % 600}/z".encode() for j in range(4000)]
    topics += [f"t{j}/{j % 7}".encode() for j in range(3000)]
    res = eng.match(topics)
    ref = RefIndex(True)
    from emqx_amd.engine import pack
    fb, fo = pack(filters)
    ref.add_many(fb, fo, np.ones(len(filters), np.uint8))
    tb, to = pack(topics, np.uint32)
    row, ids, _ = ref.match(tb, to, threads=8)
    assert np.array_equal(res.row_ptr, row)
    for i in range(len(topics)):
        assert sorted(res.row(i)) == list(ids[row[i]:row[i + 1]])


def test_packed_staging_rank_overflow_redo(emqx):
    """Pairs are staged packed (8-B words, StgFmt in gm_kernels.h) when the batch's topic ids,
    the index's filter ids and a rank field fit; a topic with more pairs than the rank field
    holds makes the walk flag the pass, which is redone wide, and the epoch stays wide.  The
    rank field is capped at 3 bits here (tune "stage_rank_bits"): every topic with more than 8
    matches overflows it."""
    from emqx_amd.engine import pack
    eng = emqx.Engine()
    filters = [f"+/{i}/{w}".encode() for w in "#+z" for i in range(40)]
    filters += [b"#", b"+/#", b"+/+/#", b"+/+/+", b"+/+/z", b"+/+"]
    filters += [f"t{j}/+/#".encode() for j in range(0, 300, 2)] + [f"t{j}/+/+".encode() for j in range(0, 300, 3)]
    filters += [f"t{j}/#".encode() for j in range(0, 300, 5)]
    filters += [f"t{j}/{j % 40}/z".encode() for j in range(0, 300, 3)]  # (up to 11 per topic)
    for f in filters:
        eng.trie_insert(f)
    eng.commit()
    ref = RefIndex(True)
    fb, fo = pack(filters)
    ref.add_many(fb, fo, np.ones(len(filters), np.uint8))
    topics = [f"t{j}/{j % 40}/z".encode() for j in range(300)] + [f"t{j}/{j % 9}".encode() for j in range(200)]
    tb, to = pack(topics, np.uint32)
    row, ids, _ = ref.match(tb, to, threads=8)
    assert np.diff(row).max() > 8

    def check(res):
        assert np.array_equal(res.row_ptr, row)
        for i in range(len(topics)):
            assert sorted(res.row(i)) == list(ids[row[i]:row[i + 1]])

    r0 = eng.stats()["reruns"]
    check(eng.match(topics))  # packed, fits
    assert eng.stats()["reruns"] == r0
    eng.tune("stage_rank_bits", 3)
    check(eng.match(topics))  # packed, overflows: redone wide
    r1 = eng.stats()["reruns"]
    assert r1 == r0 + 1
    check(eng.match(topics))  # the epoch stays wide: no redo
    assert eng.stats()["reruns"] == r1
    eng.trie_insert(b"x/y")
    eng.commit()  # a new epoch starts packed again
    check(eng.match(topics))
    assert eng.stats()["reruns"] == r1 + 1
    eng.tune("stage_rank_bits", 0)
    eng.close()


def test_staging_overflow_rerun_and_deep_stack(emqx):
    """Filters {a,+}^k/# for k <= 10: a 12-level topic a/a/.../a matches all 2047 of them, the
    walk frontier doubles per level (stack deeper than the 8 LDS entries -> HBM spill) and
    600 topics stage 1.2M pairs > the initial capacity max(1Mi, 4n) -> overflow re-run."""
    import itertools
    eng = emqx.Engine()
    filters = []
    for k in range(11):
        for combo in itertools.product(["a", "+"], repeat=k):
            filters.append(("/".join(list(combo) + ["#"])).encode())
    for f in filters:
        eng.trie_insert(f)
    eng.commit()
    topics = [b"/".join([b"a"] * 12)] * 600 + [b"/".join([b"a"] * 5 + [b"b"])] * 10
    res = eng.match(topics)
    assert eng.stats()["reruns"] >= 1
    py = R.Trie()
    for f in filters:
        py.insert(f)
    exp0 = sorted(py.match(topics[0]))
    exp1 = sorted(py.match(topics[-1]))
    assert len(exp0) == 2047
    for i, t in enumerate(topics):
        got = sorted(eng.filter_bytes(int(f)) for f in res.row(i))
        assert got == (exp0 if i < 600 else exp1)


def test_compact_items_deep_levels(emqx):
    """The walk's LDS items are 32-bit (node | kind | level < 16).  An item past the 12-item
    shallow stack, or of level >= 16 (filters of 16+ levels), flags the pass, which is redone one
    variant up (24 compact items, then {node, level} pairs with the global spill).  A batch
    mixing such topics with shallow ones: rows equal the oracle's."""
    import itertools
    filters = []
    for k in range(9):
        for combo in itertools.product(["a", "+"], repeat=k):
            filters.append(("/".join(list(combo) + ["#"])).encode())
    filters += [b"/".join([b"a"] * k) for k in (1, 5, 15, 16, 17, 20)]
    filters += [b"/".join([b"+"] * 17 + [b"b"]), b"/".join([b"a"] * 16 + [b"+", b"#"])]
    rng = random.Random(7)
    topics = []
    for i in range(3000):
        n = rng.choice([1, 2, 3, 6, 9, 12, 15, 16, 17, 18, 20, 24])
        topics.append(b"/".join(rng.choice([b"a", b"a", b"b"]) for _ in range(n)))
    eng = emqx.Engine()
    for f in filters:
        eng.trie_insert(f)
    eng.commit()
    res = eng.match(topics)
    assert eng.stats()["reruns"] >= 1
    py = R.Trie()
    for f in filters:
        py.insert(f)
    for i, t in enumerate(topics):
        got = sorted(eng.filter_bytes(int(f)) for f in res.row(i))
        assert got == sorted(py.match(t)), t
    # the shallow-only batch of the same index runs on the learnt variant: same answer
    res2 = eng.match(topics[:100])
    for i in range(100):
        assert list(res2.row(i)) == list(res.row(i))


# ---------------------------------------------------------------- synthetic configs vs oracle

def _load_both(emqx, w, **kw):
    eng = emqx.Engine(**kw)
    wild = w.fwild.astype(bool)
    idx = np.arange(w.nf)
    # register in input order so that ids coincide with the oracle's first-registration ids
    eng.route_ref_many(w.fbytes, w.foff)
    wi = idx[wild]
    if wi.size:
        sub_off = np.zeros(wi.size + 1, np.uint64)
        lens = (w.foff[wi + 1] - w.foff[wi]).astype(np.uint64)
        np.cumsum(lens, out=sub_off[1:])
        sub = np.concatenate([w.fbytes[w.foff[i]:w.foff[i + 1]] for i in wi]) if wi.size < 200000 \
            else _gather(w, wi)
        eng.trie_insert_many(sub, sub_off)
    eng.commit()
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, (2 + wild.astype(np.uint8)))
    return eng, ref


def _gather(w, wi):
    lens = (w.foff[wi + 1] - w.foff[wi]).astype(np.int64)
    starts = w.foff[wi].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
    return w.fbytes[pos]


def test_cfg1_full(emqx):
    import workloads
    w = workloads.generate(1)
    eng, ref = _load_both(emqx, w)
    _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)


def test_cfg2_full(emqx):
    import workloads
    w = workloads.generate(2)
    eng, ref = _load_both(emqx, w)
    res = _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    assert int(res.row_ptr[-1]) > 0 and (res.exact_id != emqx.NONE).any()


@pytest.mark.parametrize("cfg", [1, 2])
def test_pair_walk_with_claims(emqx, cfg):
    """walk_pair = 2: every batch walked by two lanes per topic, claims past the grid's lanes
    (cfg1's 100k topics and cfg2's 1M) -- bit-exact against the oracle like the default walk."""
    import workloads
    w = workloads.generate(cfg)
    eng, ref = _load_both(emqx, w)
    eng.tune("walk_pair", 2)
    _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    eng.tune("walk_pair", 0)  # and one lane per topic for the same batch
    _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)


def test_cfg3_sample_at_1m_filters(emqx):
    import workloads
    w = workloads.generate(3, 1_000_000, 200_000)
    eng, ref = _load_both(emqx, w)
    _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)


def _sample_packed(w, idx):
    """Topics idx of workload w, packed (bytes, u32 offsets)."""
    lens = (w.toff[idx + 1] - w.toff[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint32)
    np.cumsum(lens, out=off[1:])
    starts = w.toff[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
    return w.tbytes[pos], off


def _rows_unique(res):
    """No (topic, filter) pair twice in the CSR result (the trie returns sets)."""
    n = len(res.row_ptr) - 1
    if res.filter_id.size == 0:
        return True
    t = np.repeat(np.arange(n, dtype=np.int64), np.diff(res.row_ptr.astype(np.int64)))
    key = t * (1 << 32) + res.filter_id.astype(np.int64)
    key.sort()
    return bool((np.diff(key) != 0).all())


def test_cfg3_full_size(emqx):
    """BASELINE config 3 at the bench's size: 10M filters, the 4M-topic batch of the bench's first
    seed.  The whole batch runs on the device and EVERY topic is checked bit-exact against the
    oracle (C++ restatement of emqx_trie match_compact, 16 threads); plus no duplicate pair in
    any row, and on a 50k sample S(t) equal to the oracle's trie-state count."""
    import workloads
    w = workloads.generate(3, n_topics=4_000_000)
    eng, ref = _load_both(emqx, w)
    res = eng.match_packed(w.tbytes, w.toff)
    assert int(res.row_ptr[-1]) == res.filter_id.size > w.nt
    assert _rows_unique(res)
    row, ids, ex = ref.match(w.tbytes, w.toff, threads=16)
    assert np.array_equal(res.row_ptr, row)
    assert np.array_equal(_rows_sorted(res.row_ptr, res.filter_id), ids)
    assert np.array_equal(res.exact_id, ex)
    del row, ids, ex
    idx = np.arange(0, w.nt, 80)
    sb, so = _sample_packed(w, idx)
    import torch
    tb = torch.from_numpy(sb).cuda()
    to = torch.from_numpy(so.view(np.int32)).cuda()
    pruned = eng.walk_census(tb.data_ptr(), to.data_ptr(), len(idx), int(so[-1]))
    eng.tune("leaf_prune", 0)  # S(t) counts every matched prefix state
    census = eng.walk_census(tb.data_ptr(), to.data_ptr(), len(idx), int(so[-1]))
    sample_pairs = int((res.row_ptr[idx + 1].astype(np.int64) - res.row_ptr[idx]).sum())
    assert census["pairs"] == pruned["pairs"] == sample_pairs
    assert census["states"] == int(ref.states(sb, so, threads=16).sum())
    assert pruned["states"] < census["states"]


def test_cfg4_exact_heavy_10m(emqx):
    """BASELINE config 4's shape at 10M exact per-device keys + 100k wildcards (the full 100M
    needs ~30 GB of host memory for the ordered-set oracle): the exact route-key table at scale
    and the long-word (hashed token) verification path, bit-exact on a 100k-topic batch."""
    import workloads
    w = workloads.generate(4, 10_100_000, 100_000)
    eng, ref = _load_both(emqx, w)
    res = _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    assert (res.exact_id != emqx.NONE).mean() > 0.85
    # the same batch probed partitioned over 64-MiB bucket ranges (k_exact_part, the option)
    eng.tune("exact_range_kb", 64 << 10)
    res2 = eng.match_packed(w.tbytes, w.toff)
    assert np.array_equal(res2.exact_id, res.exact_id)
    assert np.array_equal(res2.row_ptr, res.row_ptr) and np.array_equal(res2.filter_id, res.filter_id)


def test_cfg4_full_size(emqx):
    """BASELINE config 4 at its stated size: 100M exact dev/{id:09}/state route keys + 1M
    wildcards, one 1M-topic batch.  Checked by properties over the whole batch and bit-exactly on
    a 50k sample:
    * the generator defines the exact key set (key i is dev/{i:09}/state, registered in order, so
      its id is i): every topic's exact id is its own key's id, or NONE for an id past the keys;
    * the hit rate is the generator's 90%;
    * every exact hit's filter bytes are the topic's bytes;
    * rows have no duplicate pair;
    * a 50k-topic sample: trie rows and exact hits equal the C++ oracle's (built on the 1M
      wildcards and the sample's keys; compared by filter bytes)."""
    import workloads
    w = workloads.generate(4)
    n_wild = w.nf // 101
    n_exact = w.nf - n_wild
    eng = emqx.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.arange(n_exact, w.nf)
    wb, wo = _sample_filters(w, wi)
    eng.trie_insert_many(wb, wo)
    eng.commit()
    res = eng.match_packed(w.tbytes, w.toff)
    assert _rows_unique(res)
    # topic t = b"dev/" + 9 digits + b"/state": its id from the digits
    tb = w.tbytes.reshape(w.nt, 19)
    assert np.all(np.diff(w.toff.astype(np.int64)) == 19)
    digits = (tb[:, 4:13].astype(np.int64) - ord("0"))
    ids = (digits * (10 ** np.arange(8, -1, -1, dtype=np.int64))).sum(1)
    want = np.where(ids < n_exact, ids, emqx.NONE).astype(np.uint32)
    assert np.array_equal(res.exact_id, want)
    rate = float((res.exact_id != emqx.NONE).mean())
    assert 0.89 < rate < 0.91, rate
    hits = np.nonzero(res.exact_id != emqx.NONE)[0][::97]
    assert eng.filters_bytes(res.exact_id[hits]) == [w.topic(int(i)) for i in hits]
    # 50k-topic sample against the oracle
    idx = np.arange(0, w.nt, 20)
    sb, so = _sample_packed(w, idx)
    ref = RefIndex(True)
    ref.add_many(wb, wo, np.full(len(wi), 3, np.uint8))
    keys = sorted({w.topic(int(i)) for i in idx if ids[i] < n_exact})
    kb, ko = emqx.engine.pack(keys)
    ref.add_many(kb, ko, np.full(len(keys), 2, np.uint8))
    row, rid, rex = ref.match(sb, so, threads=16)
    ref_names = [wb[int(wo[j]):int(wo[j + 1])].tobytes() for j in range(len(wi))] + keys
    for j, i in enumerate(idx):
        got = sorted(eng.filters_bytes(res.filter_id[res.row_ptr[i]:res.row_ptr[i + 1]]))
        assert got == sorted(ref_names[int(f)] for f in rid[row[j]:row[j + 1]]), w.topic(int(i))
        ex = int(res.exact_id[i])
        assert (ex == emqx.NONE) == (int(rex[j]) == emqx.NONE)
        if ex != emqx.NONE:
            assert eng.filter_bytes(ex) == ref_names[int(rex[j])]
    eng.close()


def _sample_filters(w, idx):
    lens = (w.foff[idx + 1] - w.foff[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    starts = w.foff[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
    return w.fbytes[pos], off


def test_cfg4_slice_long_words(emqx):
    """cfg4 shape (dev/{id:09}/state exact keys + wildcards): 9-byte levels get hashed tokens,
    so these pairs go through byte verification in production mode."""
    import workloads
    w = workloads.generate(4, 101_000, 50_000)
    eng, ref = _load_both(emqx, w)
    res = _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    assert (res.exact_id != emqx.NONE).mean() > 0.8


@pytest.mark.parametrize("bits", [(4, 6, 0), (8, 16, 0), (12, 16, 0), (4, 6, 16)])
def test_cfg2_slice_forced_collisions(emqx, bits):
    """Few level-token hash bits: massive edge merging and exact-table collisions; the
    verification must restore the exact reference result -- on the in-line path (k_scatter's
    rank adjustment) and, with a tiny reject capacity, on the legacy compaction path."""
    import workloads
    w = workloads.generate(2, 20_000, 20_000)
    eng, ref = _load_both(emqx, w, word_hash_bits=bits[0], full_hash_bits=bits[1],
                          reject_cap=bits[2])
    _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    st = eng.stats()
    assert st["rejected_pairs"] > 0 or st["legacy_batches"] > 0
    if bits[2]:
        assert st["legacy_batches"] >= 1


def test_random_fuzz_against_python_oracle(emqx):
    rng = random.Random(5)
    vocab = ["a", "b", "", "$x", "c", "dd"]
    filters = set()
    while len(filters) < 500:
        d = rng.randint(1, 6)
        ws = []
        for i in range(d):
            r = rng.random()
            ws.append("#" if (i == d - 1 and r < 0.15) else ("+" if r < 0.4 else rng.choice(vocab)))
        filters.add("/".join(ws).encode())
    filters = sorted(filters)
    topics = ["/".join(rng.choice(vocab) for _ in range(rng.randint(1, 7))).encode()
              for _ in range(3000)]
    for bits in (0, 3):
        eng = emqx.Engine(word_hash_bits=bits)
        py = R.Trie()
        for f in filters:
            eng.trie_insert(f)
            py.insert(f)
        eng.commit()
        res = eng.match(topics)
        for i, t in enumerate(topics):
            assert sorted(eng.filter_bytes(int(f)) for f in res.row(i)) == sorted(py.match(t)), t


def test_device_api_matches_host_api(emqx):
    import torch
    import workloads
    w = workloads.generate(1, 5000, 20000)
    eng, _ = _load_both(emqx, w)
    host = eng.match_packed(w.tbytes, w.toff)
    db = torch.from_numpy(w.tbytes).cuda()
    do = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    d = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, int(w.toff[-1]))
    assert d.n_pairs == int(host.row_ptr[-1])
    import ctypes
    row = np.empty(w.nt + 1, np.uint32)
    fid = np.empty(d.n_pairs, np.uint32)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(row.ctypes.data, d.row_ptr, row.nbytes, 2) == 0
    assert hip.hipMemcpy(fid.ctypes.data, d.filter_id, fid.nbytes, 2) == 0
    assert np.array_equal(row.astype(np.uint64), host.row_ptr)
    assert np.array_equal(fid, host.filter_id)


def _dev_to_host(d, n):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    row = np.empty(n + 1, np.uint32)
    fid = np.empty(d.n_pairs, np.uint32)
    ex = np.empty(n, np.uint32)
    for a, p in ((row, d.row_ptr), (fid, d.filter_id), (ex, d.exact_id)):
        if a.nbytes:
            assert hip.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0
    return row, fid, ex


def test_pipelined_passes(emqx):
    """emqxgm_match_device_submit/_wait: several batches in flight on the pipes give exactly the
    synchronous results; a staging overflow inside a pipe is redone; empty batches; -EBUSY for a
    third submission before the first wait; a commit completes the passes in flight against the
    index they were submitted on."""
    import torch
    import workloads
    w = workloads.generate(1, 5000, 30000)
    eng, _ = _load_both(emqx, w)
    # batches: three slices of the workload, an empty one, and one with > 1M pairs (overflows
    # the default staging capacity of max(1M, 4n) pairs inside its pipe)
    import itertools
    words = "abcdefghij"
    many = set()
    for k in range(11):  # every filter matching a/b/.../j: literal or '+' per level, '#' tails
        for pat in itertools.product((0, 1), repeat=k):
            lv = ["+" if x else words[i] for i, x in enumerate(pat)]
            many.add("/".join(lv + ["#"]) if k < 10 else "/".join(lv))
    for f in sorted(many):
        eng.trie_insert(f.encode())
    eng.commit()
    heavy = ["/".join(words).encode()] * 1000  # ~2M pairs: overflows a fresh pipe's staging
    hb, ho = emqx.engine.pack(heavy)
    batches = [(w.tbytes[:int(w.toff[k])], w.toff[:k + 1]) for k in (10000, 20000, 30000)]
    batches = [(b[int(o[0]):], o - o[0]) for b, o in batches]
    batches += [(np.zeros(1, np.uint8), np.zeros(1, np.uint32)), (hb, ho)] + batches
    dev = [(torch.from_numpy(b).cuda(), torch.from_numpy(o.astype(np.uint32).view(np.int32)).cuda())
           for b, o in batches]
    torch.cuda.synchronize()
    want = []
    for (b, o), (db, do) in zip(batches, dev):
        n = len(o) - 1
        want.append(_dev_to_host(eng.match_device(db.data_ptr(), do.data_ptr(), n, int(o[-1])), n))
    tickets = []
    got = []
    for i, ((b, o), (db, do)) in enumerate(zip(batches, dev)):
        tickets.append(eng.match_device_submit(db.data_ptr(), do.data_ptr(), len(o) - 1, int(o[-1])))
        if i >= 1:
            j = i - 1
            got.append(_dev_to_host(eng.match_device_wait(tickets[j]), len(batches[j][1]) - 1))
    with pytest.raises(emqx.EngineError):
        eng.match_device_wait(tickets[0])  # result already taken
    db, do = dev[0]
    n0 = len(batches[0][1]) - 1
    t_a = eng.match_device_submit(db.data_ptr(), do.data_ptr(), n0, int(batches[0][1][-1]))
    extra = [eng.match_device_submit(db.data_ptr(), do.data_ptr(), n0, int(batches[0][1][-1]))
             for _ in range(eng.PIPES - 2)]  # every pipe holds a pass now
    with pytest.raises(emqx.EngineError):  # pipe of the oldest ticket still holds its pass
        eng.match_device_submit(db.data_ptr(), do.data_ptr(), n0, int(batches[0][1][-1]))
    got.append(_dev_to_host(eng.match_device_wait(tickets[-1]), len(batches[-1][1]) - 1))
    for t in extra:
        assert all(np.array_equal(x, y) for x, y in zip(_dev_to_host(eng.match_device_wait(t), n0),
                                                        want[0]))
    for i, (a, b) in enumerate(zip(want, got)):
        for x, y in zip(a, b):
            assert np.array_equal(x, y), i
    # a commit completes the pass in flight; its result reflects the index it was submitted on
    eng.trie_insert(b"#")
    eng.commit()
    row, fid, ex = _dev_to_host(eng.match_device_wait(t_a), n0)
    assert all(np.array_equal(x, y) for x, y in zip((row, fid, ex), want[0]))
    assert eng.stats()["reruns"] >= 1
    eng.close()


@pytest.mark.parametrize("cfg", [2, 3])
def test_leaf_prune_is_exact(emqx, cfg):
    """CF_LEAFP pruning (skip children that are all leaves when the topic goes deeper) returns
    exactly the unpruned walk's rows and the oracle's, and makes fewer edge loads."""
    import workloads
    nf, nt = (30_000, 30_000) if cfg == 2 else (200_000, 50_000)
    w = workloads.generate(cfg, nf, nt)
    eng, ref = _load_both(emqx, w)
    res = _assert_engine_equals_ref(eng, ref, None, w.tbytes, w.toff)
    import torch
    db = torch.from_numpy(w.tbytes).cuda()
    do = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    pruned = eng.walk_census(db.data_ptr(), do.data_ptr(), w.nt, int(w.toff[-1]))
    eng.tune("leaf_prune", 0)
    full = eng.walk_census(db.data_ptr(), do.data_ptr(), w.nt, int(w.toff[-1]))
    res0 = eng.match_packed(w.tbytes, w.toff)
    assert np.array_equal(res0.row_ptr, res.row_ptr)
    rid = np.repeat(np.arange(w.nt), np.diff(res.row_ptr.astype(np.int64)))
    srt = lambda f: f[np.lexsort((f, rid))]  # noqa: E731  rows as sorted sets
    assert np.array_equal(srt(res0.filter_id), srt(res.filter_id))
    assert pruned["pairs"] == full["pairs"]
    assert pruned["slot_loads"] <= full["slot_loads"]
    if cfg == 3:
        assert pruned["slot_loads"] < 0.9 * full["slot_loads"], (pruned, full)
    eng.close()


def test_host_batch_chunks_and_pinned_io(emqx):
    """emqxgm_match_batch splits a batch larger than batch_max into device passes; row pointers
    (u64, built on the device) continue across chunks and the pinned result buffers grow; topic
    bytes staged in emqxgm_host_alloc memory give the same answer."""
    import workloads
    w = workloads.generate(1, 5000, 20000)
    ref_eng, _ = _load_both(emqx, w)
    want = ref_eng.match_packed(w.tbytes, w.toff)
    eng, _ = _load_both(emqx, w, batch_max=3000)  # 7 chunks
    got = eng.match_packed(w.tbytes, w.toff)
    assert np.array_equal(got.row_ptr, want.row_ptr)
    assert np.array_equal(got.filter_id, want.filter_id)
    assert np.array_equal(got.exact_id, want.exact_id)
    hb = eng.pinned(len(w.tbytes))
    hb[:] = w.tbytes
    ho = eng.pinned(w.nt + 1, np.uint32)
    ho[:] = w.toff
    view = eng.match_packed(hb, ho, copy=False)
    assert np.array_equal(view.row_ptr, want.row_ptr)
    assert np.array_equal(view.filter_id, want.filter_id)
    empty = eng.match([])
    assert list(empty.row_ptr) == [0] and empty.filter_id.size == 0
    eng.close()
    ref_eng.close()
