"""GPU parity of the retained-topic store (emqxgm_retain_*) against the
oracle's emqx_retainer_mnesia restatement (oracle/emqx_ref.py Retainer: search_table/3 with the
reference's default index specs -- the index path -- and with index_specs = [], the full scan),
itself pinned to the retainer suites (tests/test_oracle_golden.py)."""
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


def B(s):
    return s.encode()


def _wkey(t):
    return tuple(t.split(b"/"))


DEFAULT = [[1, 2, 3], [1, 3], [2, 3], [3]]  # emqx_retainer_schema.erl:24-29


@pytest.mark.parametrize("specs", [DEFAULT, []])
def test_retainer_suite_cases_on_device(emqx, golden, specs):
    for case, steps in golden["retainer_cases"].items():
        r = emqx.Retainer(index_specs=specs)
        for st in steps:
            if st[0] == "store":
                r.store_retained(B(st[1]), st[2])
            elif st[0] == "delete":
                r.delete_message(B(st[1]))
            elif st[0] == "clean":
                r.clean()
            else:
                _, filters, now, n = st
                got = sum(len(x) for x in r.match_messages_batch([B(f) for f in filters], now))
                assert got == n, (case, st)
        r.close()


def test_retainer_index_path_quirk_on_device(emqx):
    """The default index specs' open index tail (emqx_retainer_index.erl:180-181): 'a/+' also
    selects 'a/x/y', 'a' selects 'a/x' and 'a/x/y'; a '#' not last cuts the filter there."""
    r, q = emqx.Retainer(), R.Retainer(DEFAULT)
    topics = [b"a", b"a/x", b"a/x/y", b"a/x/y/z", b"b/x", b"b/x/y", b"x/b/c"]
    for t in topics:
        r.store_retained(t)
        q.store_retained(t)
    cases = {b"a/+": [b"a/x", b"a/x/y"], b"a": [b"a", b"a/x", b"a/x/y"],
             b"a/#/c": [b"a", b"a/x", b"a/x/y", b"a/x/y/z"],
             b"+/x": [b"a/x", b"a/x/y", b"b/x", b"b/x/y"],  # [2,3]: a tail of one
             b"+/b": [b"x/b/c"], b"#": sorted(topics, key=_wkey)}
    got = r.match_messages_batch(list(cases), 1)
    for (f, exp), g in zip(cases.items(), got):
        assert sorted(q.match_messages(f, 1), key=_wkey) == exp, f  # hand list == oracle
        assert sorted(g, key=_wkey) == exp, (f, g)
    r.set_index_specs([])  # the full scan: exactly condition/1's set
    assert r.match_messages(b"a/+", 1) == [b"a/x"] and r.match_messages(b"a/#/c", 1) == []


def test_retainer_edges(emqx):
    r = emqx.Retainer(index_specs=[])
    assert r.match_messages(b"#", 1) == []  # empty store
    topics = [b"a", b"a/b", b"a/b/c", b"a//c", b"/", b"", b"$SYS/x", b"$SYS", b"b/a",
              b"long-level-word/x", b"long-level-wordy/x", b"a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q"]
    for t in topics:
        r.store_retained(t)
    cases = {
        b"#": sorted(topics, key=_wkey),  # no '$' rule in the retainer's match spec
        b"+": [b"", b"$SYS", b"a"],
        b"a/#": [b"a", b"a//c", b"a/b", b"a/b/c", b"a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q"],
        b"a/+": [b"a/b"],
        b"a/+/c": [b"a//c", b"a/b/c"],
        b"+/+": [b"/", b"$SYS/x", b"a/b", b"b/a", b"long-level-word/x", b"long-level-wordy/x"],
        b"": [b""],
        b"/": [b"/"],
        b"/#": [b"", b"/"],  # the pattern ['' | '_'] also matches the one-word topic "" 
        b"a/#/c": [],  # '#' not last selects nothing (topics never hold a '#' word)
        b"long-level-word/+": [b"long-level-word/x"],
        b"+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+": [b"a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q"],
        b"$SYS/#": [b"$SYS", b"$SYS/x"],
    }
    got = r.match_messages_batch(list(cases), 1)
    for (f, exp), g in zip(cases.items(), got):
        assert exp == sorted(R.retained_match(f, topics), key=_wkey), f  # hand list == oracle
        assert g == exp, (f, g)
    # the same edges on the index path of the default specs
    r.set_index_specs(DEFAULT)
    q = R.Retainer(DEFAULT)
    for t in topics:
        q.store_retained(t)
    got = r.match_messages_batch(list(cases), 1)
    for f, g in zip(cases, got):
        assert sorted(g, key=_wkey) == sorted(q.match_messages(f, 1), key=_wkey), (f, g)
    assert r.size() == len(topics)
    assert r.read_message(b"a/b", 1) == [b"a/b"] and r.read_message(b"a/x", 1) == []


@pytest.mark.parametrize("seed,dmax,specs", [(1, -1, DEFAULT), (2, -1, []), (3, 0, DEFAULT),
                                             (4, 10**9, DEFAULT), (5, -1, [[2], [1, 3, 4]]),
                                             (6, 10**9, [])])
def test_retainer_random_vs_oracle(emqx, seed, dmax, specs):
    """dmax: delta topics before a base rebuild (0: rebuild at every commit; 10**9: the base
    is only ever patched -- deletions and re-stores -- and new topics live in the delta);
    specs: the index specs (the wildcard delete selects by them too, :166-180)."""
    rng = random.Random(seed)
    vocab = [b"a", b"b", b"", b"$s", b"cc", b"long-word-%d" % seed, b"long-word-x"]
    ref, dev = R.Retainer(specs), emqx.Retainer(index_specs=specs)
    dev.tune("delta_max", dmax)
    big = dmax == 10**9
    for step in range(6):
        for _ in range(rng.randint(50, 400)):
            t = b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 6)))
            if rng.random() < 0.75:
                e = rng.choice([0, 0, 0, 50, 150])
                ref.store_retained(t, e)
                dev.store_retained(t, e)
            else:
                ref.delete_message(t)
                dev.delete_message(t)
        if big and step == 2:  # fill the base once; every later change patches or goes to delta
            dev.tune("delta_max", 0)
            dev.commit()
            dev.tune("delta_max", dmax)
        if step == 3:  # a wildcard delete (Now = 0: every selected message)
            ref.delete_message(b"a/+/#")
            dev.delete_message(b"a/+/#")
        filters = []
        for _ in range(300):
            ws = [rng.choice([b"+", b"a", b"b", b"", b"$s", b"cc", b"long-word-x"])
                  for _ in range(rng.randint(1, 6))]
            if rng.random() < 0.3:
                ws[-1] = b"#"
            filters.append(b"/".join(ws))
        got = dev.match_messages_batch(filters, 100)
        for f, g in zip(filters, got):
            exp = ref.match_messages(f, 100)
            # base topics first, then the delta's, each in topic word order
            assert sorted(g, key=_wkey) == sorted(exp, key=_wkey) and len(set(g)) == len(g), (step, f)
        assert dev.size() == ref.size()
    st = dev.stats()
    if dmax == 0:
        assert st["delta_commits"] == 0, st
    elif big:
        assert st["full_builds"] == 2 and st["delta_commits"] >= 3 and st["base_topics"] > 0, st
    dev.close()


@pytest.mark.parametrize("specs", [DEFAULT, []])
def test_retainer_cfg3_scale(emqx, specs):
    """200k cfg3 topics; a sample of subscription-shaped filters against the predicate forms
    (R.retained_match_indexed is checked against the restated search_table on the CPU)."""
    import workloads
    w = workloads.generate(3, 2000, 200_000)
    topics = [w.topic(i) for i in range(w.nt)]
    r = emqx.Retainer(index_specs=specs)
    for t in topics:
        r.store_retained(t)
    uniq = sorted(set(topics), key=_wkey)
    filters = [w.filter(i) for i in range(0, w.nf, 100)] + [b"site/+/device/+/m1/#", b"#"]
    got = r.match_messages_batch(filters, 1)
    for f, g in zip(filters, got):
        assert sorted(g, key=_wkey) == sorted(R.retained_match_indexed(f, uniq, specs), key=_wkey), f
    assert r.size() == len(uniq)
