"""Fat buckets (gm_common.h FAT_ID) on the device: a node at depth 2, 4 or 6 whose only literal
child is G keeps G's slot in the second half of its own bucket line, and the root's only literal
child rides in the walk's arguments.  Chain-heavy tries (most nodes with one literal child, some
with '+' and '#' filters, '$' topics) are matched with fat buckets on and off against the
Python restatement of emqx_trie (oracle/emqx_ref.py, emqx_trie.erl:282-348), and delta commits
that give fat nodes a second literal child (the half moves out) or delete halves are checked
after every commit."""
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


def _chain_tree(rng, n_paths, max_depth=9):
    """Filters over a trie where most nodes have a single literal child."""
    kids = {(): ["r"]}  # the root's only literal child: a fat root
    filters = set()
    for _ in range(n_paths):
        path = []
        for d in range(rng.randint(1, max_depth)):
            opts = kids.setdefault(tuple(path), [])
            r = rng.random()
            if not opts or (r < 0.12 and len(opts) < 4):
                opts.append(rng.choice(["a", "b", "c", "dd", "", "$x", "long-word-%d" % d]))
            w = "+" if rng.random() < 0.1 and d > 0 else rng.choice(opts)
            path.append(w)
        if rng.random() < 0.2:
            path.append("#")
        filters.add("/".join(path).encode())
        if rng.random() < 0.05:
            filters.add(("+/" + "/".join(path[1:])).encode())  # a root '+' branch
    return sorted(filters), kids


def _topics(rng, kids, n):
    out = []
    for _ in range(n):
        path = []
        for _ in range(rng.randint(1, 10)):
            opts = kids.get(tuple(path)) or ["zz"]
            path.append(rng.choice(opts) if rng.random() < 0.9 else rng.choice(["a", "q", ""]))
        t = "/".join(path)
        if rng.random() < 0.05:
            t = "$SYS/" + t
        out.append(t.encode())
    return out


def _check(eng, py, topics):
    res = eng.match(topics)
    for i, t in enumerate(topics):
        got = sorted(eng.filter_bytes(int(f)) for f in res.row(i))
        assert got == sorted(py.match(t)), t


@pytest.mark.parametrize("fat", [1, 0])
@pytest.mark.parametrize("bits", [0, 3])
def test_fat_buckets_full_build(emqx, fat, bits):
    rng = random.Random(17 + bits)
    filters, kids = _chain_tree(rng, 1500)
    topics = _topics(rng, kids, 4000)
    eng = emqx.Engine(word_hash_bits=bits)
    eng.tune("fat_buckets", fat)
    py = R.Trie()
    for f in filters:
        eng.trie_insert(f)
        py.insert(f)
    eng.commit()
    _check(eng, py, topics)


def test_fat_buckets_delta_churn(emqx):
    rng = random.Random(29)
    filters, kids = _chain_tree(rng, 800)
    topics = _topics(rng, kids, 3000)
    eng = emqx.Engine()
    eng.tune("delta_commit", 2)  # patch whenever possible
    py = R.Trie()
    for f in filters:
        eng.trie_insert(f)
        py.insert(f)
    eng.commit()
    _check(eng, py, topics)
    live = list(filters)
    for _ in range(12):
        for _ in range(40):
            if rng.random() < 0.5 and live:  # unsubscribe: may free a fat half
                f = live.pop(rng.randrange(len(live)))
                eng.trie_delete(f)
                py.delete(f)
            else:  # a sibling of an existing level: a fat node's second literal child
                base = rng.choice(live or filters).split(b"/")
                k = rng.randint(1, len(base))
                f = b"/".join(base[:k - 1] + [rng.choice([b"a", b"e", b"ff", b""])] + base[k:])
                if f not in live:
                    live.append(f)
                    eng.trie_insert(f)
                    py.insert(f)
        eng.commit()
        _check(eng, py, topics)
    assert eng.stats()["delta_commits"] > 0


def _wide_tree(rng, n):
    """Filters whose nodes have many literal children, some shared between a literal parent and
    its '+' twin (the cfg3 shape site/S/device/D vs site/+/device/D), plus '#', '$' and deep
    levels past the topic record's 7 tokens."""
    filters = set()
    for _ in range(n):
        s = rng.randrange(40)
        d = s * 100 + rng.randrange(100)
        r = rng.random()
        if r < 0.5:
            f = f"site/{s}/device/{d}/#"
        elif r < 0.7:
            f = f"site/+/device/{d}/#"
        elif r < 0.8:
            f = f"site/{s}/device/{d}/+/{rng.randrange(8)}"
        elif r < 0.9:
            f = f"site/{s}/device/{d}/a/b/c/d/e/{rng.randrange(4)}"
        else:
            f = f"{rng.choice(['$SYS', 'x', ''])}/{rng.randrange(60)}/{rng.choice(['+', 'q'])}"
        filters.add(f.encode())
    return sorted(filters)


@pytest.mark.parametrize("keyed", [0, 1, 2])
@pytest.mark.parametrize("bits", [0, 4])
def test_keyed_parents_full_build_and_delta(emqx, keyed, bits):
    """Token-keyed parents (gm_common.h edge_home; tune "keyed": 0 none, 1 auto, 2 every
    eligible node): full build, then delta churn that adds and removes children of keyed
    parents, checked against the Python restatement after every commit."""
    rng = random.Random(41 + keyed + bits)
    filters = _wide_tree(rng, 3000)
    topics = []
    for _ in range(4000):
        s = rng.randrange(45)
        d = s * 100 + rng.randrange(110)
        tail = "/".join(str(rng.randrange(9)) if rng.random() < 0.5 else rng.choice("abcdeq")
                        for _ in range(rng.randint(0, 7)))
        topics.append((f"site/{s}/device/{d}" + ("/" + tail if tail else "")).encode())
    topics += [f"{p}/{k}/q".encode() for p in ("$SYS", "x", "") for k in range(0, 70, 7)]
    eng = emqx.Engine(word_hash_bits=bits)
    eng.tune("keyed", keyed)
    eng.tune("delta_commit", 2)
    py = R.Trie()
    for f in filters:
        eng.trie_insert(f)
        py.insert(f)
    eng.commit()
    _check(eng, py, topics)
    live = list(filters)
    for _ in range(6):
        for _ in range(60):
            if rng.random() < 0.45 and live:
                f = live.pop(rng.randrange(len(live)))
                eng.trie_delete(f)
                py.delete(f)
            else:
                f = rng.choice(_wide_tree(rng, 1))
                if f not in live:
                    live.append(f)
                    eng.trie_insert(f)
                    py.insert(f)
        eng.commit()
        _check(eng, py, topics)
