"""Pins the C++ restatement (oracle/ref_trie.cpp) to the golden vectors and to the Python
restatement, and checks its trie walk against brute-force emqx_topic:match/2.  CPU only."""
import random

import numpy as np
import pytest

from oracle import emqx_ref as R
from oracle.cref import RefIndex
from emqx_amd.engine import pack


def _ids_to_sets(row, ids, names):
    return [sorted(names[i] for i in ids[row[t]:row[t + 1]]) for t in range(len(row) - 1)]


def _run_ref(filters, topics, compact, kinds=None):
    ref = RefIndex(compact)
    fb, fo = pack(filters)
    kinds = np.array(kinds if kinds is not None else [1] * len(filters), np.uint8)
    ref.add_many(fb, fo, kinds)
    tb, to = pack(topics, np.uint32)
    row, ids, ex = ref.match(tb, to, threads=2)
    return ref, row, ids, ex


@pytest.mark.parametrize("compact", [True, False])
def test_cpp_trie_suite(golden, compact):
    for case, steps in golden["trie_cases"].items():
        inserted = []
        deleted = []
        for step in steps:
            if step[0] == "insert":
                inserted += [s.encode() for s in step[1]]
            elif step[0] == "delete":
                deleted += [s.encode() for s in step[1]]
        ref = RefIndex(compact)
        fb, fo = pack(inserted)
        ref.add_many(fb, fo, np.ones(len(inserted), np.uint8))
        names = list(dict.fromkeys(inserted))
        for d in deleted:
            ref.trie_delete(d)
        for step in steps:
            if step[0] in ("match", "match_len"):
                tb, to = pack([step[1].encode()], np.uint32)
                row, ids, _ = ref.match(tb, to)
                got = _ids_to_sets(row, ids, names)[0]
                if step[0] == "match":
                    assert got == sorted(x.encode() for x in step[2]), (case, step)
                else:
                    assert len(got) == step[2]


@pytest.mark.parametrize("compact", [True, False])
def test_cpp_equals_python_and_bruteforce(compact):
    rng = random.Random(11)
    vocab = ["a", "b", "", "$x", "cc", "+x"]
    filters = set()
    while len(filters) < 300:
        d = rng.randint(1, 5)
        ws = []
        for i in range(d):
            r = rng.random()
            ws.append("#" if (i == d - 1 and r < 0.15) else ("+" if r < 0.4 else rng.choice(vocab)))
        filters.add("/".join(ws).encode())
    filters = sorted(filters)
    topics = ["/".join(rng.choice(vocab[:5]) for _ in range(rng.randint(1, 6))).encode()
              for _ in range(500)] + [b"", b"/", b"$SYS", b"$x", b"a/+", b"#", b"a//b"]
    ref, row, ids, _ = _run_ref(filters, topics, compact)
    got = _ids_to_sets(row, ids, filters)
    py = R.Trie(compact)
    for f in filters:
        py.insert(f)
    tb, to = pack(topics, np.uint32)
    brow, bids = ref.bruteforce(tb, to)
    brute = _ids_to_sets(brow, bids, filters)
    for i, t in enumerate(topics):
        assert got[i] == sorted(py.match(t)), t
        assert got[i] == brute[i], t


def test_cpp_exact_keys_and_states():
    filters = [b"a/b", b"a/+", b"a/#", b"x/y/z", b"+/+"]
    kinds = [2, 3, 3, 2, 3]  # exact keys are route-only, wildcards trie+route
    topics = [b"a/b", b"a/+", b"x/y/z", b"q"]
    ref, row, ids, ex = _run_ref(filters, topics, True, kinds)
    assert list(ex) == [0, 1, 3, 0xFFFFFFFF]
    got = _ids_to_sets(row, ids, filters)
    assert got[0] == sorted([b"a/+", b"a/#", b"+/+"])
    assert got[1] == []  # wildcard topic name: trie returns []
    tb, to = pack(topics, np.uint32)
    st = ref.states(tb, to)
    # a/b: root, a, +, a/+ ( '+/+' path: '+' then '+/+' ) -> root + {a,+} + {a/+, +/+}
    assert st[0] == 1 + 2 + 2
    assert st[1] == 0


def test_cfg1_slice_bruteforce():
    import workloads
    w = workloads.generate(1, 2000, 3000)
    ref = RefIndex(True)
    ref.add_many(w.fbytes, w.foff, np.ones(w.nf, np.uint8))
    row, ids, _ = ref.match(w.tbytes, w.toff, threads=4)
    brow, bids = ref.bruteforce(w.tbytes, w.toff)
    assert np.array_equal(row, brow) and np.array_equal(ids, bids)
    ref2 = RefIndex(False)
    ref2.add_many(w.fbytes, w.foff, np.ones(w.nf, np.uint8))
    row2, ids2, _ = ref2.match(w.tbytes, w.toff, threads=4)
    assert np.array_equal(row, row2) and np.array_equal(ids, ids2)
    assert ids.size > 0
