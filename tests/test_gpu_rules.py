"""GPU parity of batched rule matching (emqxgm_match_rules) against the
oracle's emqx_topic:match/2 (oracle/emqx_ref.py, emqx_topic.erl:67-89): on binaries for
emqx_rewrite:match_and_rewrite/3, on word lists for emqx_authz_rule:match_topics/3, and word
equality for authz {eq, Filter} rules."""
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


def _first(names, rules, words):
    out = []
    for n in names:
        hit = None
        for i, r in enumerate(rules):
            if isinstance(r, tuple):
                ok = R.words(n) == R.words(r[1])
            elif words:
                ok = R.match(R.words(n), R.words(r))
            else:
                ok = R.match(n, r)
            if ok:
                hit = i
                break
        out.append(hit)
    return out


def _rand(rng, vocab, wild):
    ws = []
    d = rng.randint(1, 5)
    for i in range(d):
        r = rng.random()
        if wild and i == d - 1 and r < 0.15:
            ws.append("#")
        elif wild and r < 0.3:
            ws.append("+")
        else:
            ws.append(rng.choice(vocab))
    return "/".join(ws).encode()


def test_rules_hand_cases(emqx):
    from emqx_amd.rules import authz_match_topics, rewrite_rule
    eng = emqx.Engine()
    names = [b"$SYS/brokers", b"a/b", b"a", b"a/+", b"x/y/z", b"", b"/", b"$q"]
    # rewrite: binaries, '$' names never match a root wildcard (emqx_topic.erl:70-73)
    assert rewrite_rule(names, [b"#"], eng) == [None, 0, 0, 0, 0, 0, 0, None]
    # authz: word lists, no '$' clauses; subscribe filters match literally ('+' == '+')
    assert authz_match_topics(names, [b"#"], eng) == [True] * 8
    assert authz_match_topics([b"a/+", b"a/b"], [("eq", b"a/+")], eng) == [True, False]
    assert authz_match_topics([b"a/+"], [b"a/b"], eng) == [False]
    assert rewrite_rule([b"x/y/z", b"x/q"], [b"x/q", b"x/#", b"x/+/z"], eng) == [1, 0]


@pytest.mark.parametrize("words", [False, True])
@pytest.mark.parametrize("big", [False, True])
def test_rules_random_vs_oracle(emqx, words, big):
    rng = random.Random(7 + words + 2 * big)
    vocab = ["a", "b", "", "$s", "c", "long-word-%d" % 7, "+x"]
    n_rules = 3000 if big else 60  # big: beyond the LDS-staged rule set
    rules = []
    for _ in range(n_rules):
        f = _rand(rng, vocab, True)
        rules.append(("eq", f.replace(b"#", b"z")) if words and rng.random() < 0.1 else f)
    names = [_rand(rng, vocab, rng.random() < 0.1) for _ in range(4000)]
    names += [b"$SYS/x", b"$", b"", b"/", b"//"]
    eng = emqx.Engine()
    from emqx_amd.rules import TopicRules
    got = TopicRules(rules, words=words, engine=eng).first_match(names)
    assert got == _first(names, rules, words)
