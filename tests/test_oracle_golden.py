"""Pins the CPU oracle (oracle/emqx_ref.py) to the reference's own asserted vectors.

CPU only.  Each table in tests/golden/reference_vectors.json cites the reference suite it was
transcribed from (tests/golden/make_golden.py)."""
import itertools
import random

import pytest

from oracle import emqx_ref as R


def B(s):
    return s.encode()


def W(x):
    if isinstance(x, dict) and "atom" in x:
        return x["atom"]
    if isinstance(x, dict) and "words_of" in x:
        return R.words(B(x["words_of"]))
    return B(x)


def test_match_vectors(golden):
    for name, filt, exp in golden["match"]:
        assert R.match(B(name), B(filt)) is exp, (name, filt)


def test_wildcard_words_tokens_levels(golden):
    for t, exp in golden["wildcard"]:
        assert R.wildcard(B(t)) is exp
    for t, exp in golden["words"]:
        assert R.words(B(t)) == [W(x) for x in exp]
    for t, exp in golden["tokens"]:
        assert R.tokens(B(t)) == [B(x) for x in exp]
    for t, exp in golden["levels"]:
        assert R.levels(B(t)) == exp


def test_join(golden):
    for ws, exp in golden["join"]:
        ws = W(ws) if isinstance(ws, dict) else [W(x) for x in ws]
        assert R.join(ws) == B(exp)


def test_validate(golden):
    long_topic = b"".join(str(i).encode() + b"/" for i in range(0, 66667))
    for kind, topic, exp in golden["validate"]:
        t = long_topic if isinstance(topic, dict) else B(topic)
        if exp is True:
            assert R.validate((kind, t)) is True
        else:
            with pytest.raises(R.TopicError) as ei:
                R.validate((kind, t))
            assert ei.value.args[0] == exp


def test_prepend_parse(golden):
    for parent, w, exp in golden["prepend"]:
        p = None if parent is None else W(parent)
        assert R.prepend(p, B(w)) == B(exp)
    for inp, opts, exp in golden["parse"]:
        o = {k: (B(v) if isinstance(v, str) else v) for k, v in opts.items()}
        if isinstance(exp, dict):
            with pytest.raises(R.TopicError):
                R.parse(B(inp), o)
        else:
            topic, eo = R.parse(B(inp), o)
            assert topic == B(exp[0])
            assert eo == {k: (B(v) if isinstance(v, str) else v) for k, v in exp[1].items()}


def test_trie_key_layout(golden):
    for compact, filt, tk, prefixes in golden["make_keys"]:
        t = R.Trie(compact)
        assert t.make_keys(B(filt)) == ((B(tk), 1), [(B(p), 0) for p in prefixes])
    for compact, filt, prefixes in golden["make_prefixes"]:
        assert R.Trie(compact).make_prefixes(R.words(B(filt))) == [B(p) for p in prefixes]
    for filt, segs in golden["do_compact"]:
        assert R.do_compact(R.words(B(filt))) == [B(s) for s in segs]


@pytest.mark.parametrize("compact", [True, False])
def test_trie_suite(golden, compact):
    for case, steps in golden["trie_cases"].items():
        t = R.Trie(compact)
        for step in steps:
            op = step[0]
            if op == "insert":
                for f in step[1]:
                    t.insert(B(f))
            elif op == "delete":
                for f in step[1]:
                    t.delete(B(f))
            elif op == "match":
                assert sorted(t.match(B(step[1]))) == [B(x) for x in step[2]], (case, step)
            elif op == "match_len":
                assert len(t.match(B(step[1]))) == step[2], (case, step)
            elif op == "empty":
                assert t.empty() is step[1], (case, step)
            elif op == "lookup_topic":
                assert t.lookup_topic(B(step[1])) == [B(x) for x in step[2]], (case, step)


def test_router_suite(golden):
    for case, steps in golden["router_cases"].items():
        r = R.Router()
        for step in steps:
            op = step[0]
            if op == "add_route":
                for f, d in step[1]:
                    r.add_route(B(f), d)
            elif op == "delete_route":
                for f, d in step[1]:
                    r.delete_route(B(f), d)
            elif op == "match_routes":
                got = sorted(r.match_routes(B(step[1])))
                assert got == sorted((B(f), d) for f, d in step[2]), (case, step)


def test_client_matrix(golden):
    topics = [B(t) for t in golden["client_topics"]]
    wild = [B(w) for w in golden["client_wild"]]
    tr = R.Trie()
    for w in wild:
        tr.insert(w)
    for t in topics:
        assert sorted(tr.match(t)) == sorted(w for w in wild if R.match(t, w))
    for name, filt, exp in golden["client_dollar"]:
        assert R.match(B(name), B(filt)) is exp
        t2 = R.Trie()
        t2.insert(B(filt))
        assert (B(filt) in t2.match(B(name))) is exp


def test_bench_pattern_one_route(golden):
    """emqx_broker_bench: sub_ptn rendered per id/num, each publisher topic has 1 route."""
    bp = golden["bench_patterns"]
    r = R.Router()
    subs, sub_ops = 8, 50
    for i in range(1, subs + 1):
        for n in range(1, sub_ops + 1):
            r.add_route(B(bp["sub_ptn"].replace("{{id}}", str(i)).replace("{{num}}", str(n))))
    for i in range(1, subs + 1):
        topic = B(bp["pub_ptn"].replace("{{id}}", str(i)).replace("{{num}}", "1"))
        assert len(r.match_routes(topic)) == bp["expect_routes_per_lookup"]


# --- the two independent restatements agree (SURVEY 8c "Golden vectors") ----------------

def _rand_filters(rng, vocab, n, depth):
    out = set()
    while len(out) < n:
        d = rng.randint(1, depth)
        ws = []
        for i in range(d):
            r = rng.random()
            if i == d - 1 and r < 0.15:
                ws.append("#")
            elif r < 0.35:
                ws.append("+")
            else:
                ws.append(rng.choice(vocab))
        out.add(B("/".join(ws)))
    return sorted(out)


def _rand_topics(rng, vocab, n, depth):
    out = []
    for _ in range(n):
        d = rng.randint(1, depth)
        ws = [rng.choice(vocab) for _ in range(d)]
        if rng.random() < 0.1:
            ws[0] = "$SYS"
        out.append(B("/".join(ws)))
    return out


@pytest.mark.parametrize("compact", [True, False])
def test_trie_walk_equals_bruteforce(compact):
    rng = random.Random(7)
    vocab = ["a", "b", "c", "", "$x", "dd"]
    filters = _rand_filters(rng, vocab, 400, 5)
    topics = _rand_topics(rng, vocab, 600, 6) + [b"", b"/", b"//", b"a//b", b"/a", b"a/",
                                                 b"$SYS", b"$x", b"a/+", b"#"]
    t = R.Trie(compact)
    for f in filters:
        t.insert(f)
    for topic in topics:
        got = t.match(topic)
        assert len(got) == len(set(got)), topic  # no duplicates
        assert sorted(got) == sorted(R.trie_match_bruteforce(topic, filters, [
            f for f in filters if not R.wildcard(f)])), topic


def test_trie_delete_restores_state():
    rng = random.Random(3)
    vocab = ["a", "b", "", "c"]
    filters = _rand_filters(rng, vocab, 120, 4)
    for compact in (True, False):
        t = R.Trie(compact)
        for f in filters:
            t.insert(f)
            t.insert(f)  # idempotent
        keep = filters[::2]
        for f in filters[1::2]:
            t.delete(f)
            t.delete(f)  # no-op
        ref = R.Trie(compact)
        for f in keep:
            ref.insert(f)
        assert t.tab == ref.tab


def test_aggre():
    routes = [(b"a", "n1"), (b"b", ("g", "n1")), (b"b", ("g", "n2"))]
    assert R.aggre([]) == []
    assert R.aggre([(b"a", "n1")]) == [(b"a", "n1")]
    assert R.aggre([(b"a", ("g", "n1"))]) == [(b"a", "g")]
    assert R.aggre(routes) == [(b"a", "n1"), (b"b", "g")]


def test_publish_oracle_fanout():
    """oracle publish = route(aggre(match_routes(T))) with local dispatch
    (emqx_broker.erl:218-300, 326-355): group dests collapse per filter, only {To, node()}
    entries dispatch, a wildcard topic name keeps only its own exact routes."""
    r = R.Router()
    r.add_route(b"a/+", "n1")
    r.add_route(b"a/+", "n2")
    r.add_route(b"a/b", "n1")
    r.add_route(b"a/#", (b"g", "n2"))
    r.add_route(b"a/#", (b"g", "n3"))
    subs = {b"a/+": ["s1", "s2"], b"a/b": ["s3"], b"a/#": ["x"]}
    entries, deliv = R.publish(r, b"a/b", "n1", subs)
    assert sorted(entries, key=repr) == sorted([(b"a/#", b"g"), (b"a/+", "n1"), (b"a/+", "n2"),
                                               (b"a/b", "n1")], key=repr)
    assert deliv == [(b"a/+", "s1"), (b"a/+", "s2"), (b"a/b", "s3")]
    entries, deliv = R.publish(r, b"a/+", "n1", subs)
    assert sorted(entries, key=repr) == sorted([(b"a/+", "n1"), (b"a/+", "n2")], key=repr)
    assert R.publish(r, b"zz", "n1", subs) == ([], [])


# ---------------------------------------------------------------- retainer

def _pat(x):
    """Decode a golden pattern: lists, {"atom": a}, {"improper": [...]}, binaries."""
    if isinstance(x, dict) and "improper" in x:
        return R.Improper([_pat(y) for y in x["improper"]])
    if isinstance(x, dict) and "atom" in x:
        return x["atom"]
    if isinstance(x, list):
        return [_pat(y) for y in x]
    return B(x)


def _key(x):
    """Golden index key / condition/2 pattern [[Index], [IndexPart, OtherPart]] -> tuples."""
    ix, (a, b) = x
    conv = (lambda p: tuple(p) if isinstance(p, list) else p)
    return (tuple(ix), (conv(_pat(a)), conv(_pat(b))))


def test_retainer_index_vectors(golden):
    g = golden["retainer_index"]
    for ix, ws, key in g["to_index_key"]:
        assert R.retainer_to_index_key(ix, [W(w) for w in ws]) == _key(key)
    for ix, ws, score in g["index_score"]:
        assert R.retainer_index_score(ix, [W(w) for w in ws]) == score, (ix, ws)
    for ws, indices, sel in g["select_index"]:
        assert R.retainer_select_index([W(w) for w in ws], indices) == sel
    for ws, pat in g["condition"]:
        assert R.retainer_condition([W(w) for w in ws]) == _pat(pat), ws
    for ix, ws, pat in g["condition_index"]:
        got = R.retainer_condition_index(ix, [W(w) for w in ws])
        exp_ix, (a, b) = pat
        assert got == (tuple(exp_ix), (_pat(a), _pat(b))), (ix, ws, got)
    for key, ws in g["restore_topic"]:
        assert R.retainer_restore_topic(_key(key)) == [W(w) for w in ws]


@pytest.mark.parametrize("indices", [[], [[1, 2], [2, 3]], [[1], [3, 4], [1, 2, 3]]])
def test_retainer_suite_cases(golden, indices):
    for case, steps in golden["retainer_cases"].items():
        r = R.Retainer(indices)
        for st in steps:
            if st[0] == "store":
                r.store_retained(B(st[1]), st[2])
            elif st[0] == "delete":
                r.delete_message(B(st[1]))
            elif st[0] == "clean":
                r.clean()
            else:
                _, filters, now, n = st
                got = sum(len(r.match_messages(B(f), now)) for f in filters)
                assert got == n, (case, st, indices)


def test_retainer_index_path_quirk():
    """With index specs configured, 5.0.14's index path over-selects when a filter ends before
    the index's last position (condition/2's `[_|_], []` clause leaves the index part open,
    emqx_retainer_index.erl:180-181): with the default specs (emqx_retainer_schema.erl:24-29)
    'a/+' also selects 'a/x/y'.  The scan path (index_specs = []) selects exactly condition/1's
    set; the engine implements both, the index path by default."""
    default = [[1, 2, 3], [1, 3], [2, 3], [3]]
    q, plain = R.Retainer(default), R.Retainer()
    for t in (b"a/x", b"a/x/y", b"b/x"):
        q.store_retained(t)
        plain.store_retained(t)
    assert sorted(q.match_messages(b"a/+", 1)) == [b"a/x", b"a/x/y"]
    assert plain.match_messages(b"a/+", 1) == [b"a/x"]


def test_retainer_index_path_covers_scan():
    """search_table's index path never misses what the scan selects (it may over-select, see
    the quirk above), and the scan equals the predicate form."""
    rng = random.Random(4)
    vocab = [b"a", b"b", b"", b"$s", b"cc"]
    topics = {b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 5))) for _ in range(400)}
    plain, indexed = R.Retainer(), R.Retainer([[1, 2], [2, 3], [1, 3, 4]])
    for t in topics:
        e = rng.choice([0, 0, 50, 150])
        plain.store_retained(t, e)
        indexed.store_retained(t, e)
    for _ in range(300):
        d = rng.randint(1, 5)
        ws = [rng.choice([b"+", b"a", b"b", b"", b"$s"]) for _ in range(d)]
        if rng.random() < 0.3:
            ws[-1] = b"#"
        f = b"/".join(ws)
        a = sorted(plain.match_messages(f, 100))
        assert set(a) <= set(indexed.match_messages(f, 100)), f
        live = [t for t in topics if plain.msgs[tuple(R.words(t))] in (0, 150)]
        assert a == sorted(R.retained_match(f, live)), f


@pytest.mark.parametrize("specs", [[[1, 2, 3], [1, 3], [2, 3], [3]], [[1, 2], [2, 3], [1, 3, 4]],
                                   [[2]], [[1, 2, 3, 4, 5]]])
def test_retainer_indexed_predicate_equals_search_table(specs):
    """The predicate form of the index path (R.retained_match_indexed, the set the engine's
    filter plan reproduces: a cut after the first '#', an open index tail) equals the index
    search of the restated emqx_retainer_mnesia (Retainer.search_table) -- including filters
    with '#' not last and filters shorter than the index."""
    rng = random.Random(len(specs))
    vocab = [b"a", b"b", b"", b"$s", b"cc"]
    topics = {b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 6))) for _ in range(500)}
    r = R.Retainer(specs)
    for t in topics:
        r.store_retained(t, 0)
    for _ in range(400):
        d = rng.randint(1, 6)
        ws = [rng.choice([b"+", b"+", b"a", b"b", b"", b"#"]) for _ in range(d)]
        f = b"/".join(ws)
        assert sorted(r.match_messages(f, 1)) == sorted(R.retained_match_indexed(f, topics, specs)), f
