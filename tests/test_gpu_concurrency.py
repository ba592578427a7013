"""Epochs: match calls read the last committed index and never wait for a writer (SURVEY 8b:
the reference reads with read_concurrency while writers commit in mria transactions,
emqx_trie.erl:70-75, emqx_router_utils.erl:74-135), and the pipelined host-in/host-out path
(emqxgm_match_batch_submit/_wait, the NIF batcher's call, emqx_broker.erl:231).

* a delta commit followed at once by a pipelined pass: the pass sees the whole delta (its
  patches are ordered before it on the GPU), checked against the Python oracle;
* a writer thread committing deltas in a loop while the main thread matches: every result is
  exactly the old or the new epoch's, never a mix;
* a full rebuild of a 10M-filter index in a writer thread while the main thread matches: the
  matches keep returning (each within a pass time) with the old epoch's answer, and switch to the
  new one once the commit has returned;
* the host pipes give exactly emqxgm_match_batch's result (several in flight, an empty batch,
  -EBUSY, a staging overflow redone inside a pipe, both result-copy modes).
"""
import threading
import time

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


def _load(emqx, w, **kw):
    eng = emqx.Engine(**kw)
    wild = w.fwild.astype(bool)
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.nonzero(wild)[0]
    if wi.size:
        lens = (w.foff[wi + 1] - w.foff[wi]).astype(np.int64)
        starts = w.foff[wi].astype(np.int64)
        pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        off = np.zeros(wi.size + 1, np.uint64)
        np.cumsum(lens, out=off[1:])
        eng.trie_insert_many(w.fbytes[pos], off)
    eng.commit()
    return eng


def _dev_result(d, n):
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


def _sets(eng, row, fid, i):
    return sorted(eng.filter_bytes(int(f)) for f in fid[int(row[i]):int(row[i + 1])])


def test_delta_commit_then_pipelined_pass_sees_it(emqx):
    """after a small delta commit the next pipelined pass must read the fully
    patched tables, on the device pipes and on the host pipes alike."""
    import torch
    rng = np.random.default_rng(3)
    vocab = [b"a", b"b", b"", b"c", b"dd", b"sensor", b"long-level-name"]
    topics = [b"/".join(vocab[j] for j in rng.integers(0, len(vocab), rng.integers(1, 6)))
              for _ in range(400)]
    buf, off = emqx.engine.pack(topics, np.uint32)
    db = torch.from_numpy(buf.copy()).cuda()
    do = torch.from_numpy(off.view(np.int32).copy()).cuda()
    torch.cuda.synchronize()
    eng = emqx.Engine()
    py = R.Trie()
    base = [b"a/+", b"+/b/#", b"sensor/#"]
    for f in base:
        eng.trie_insert(f)
        py.insert(f)
    eng.commit()
    adds = [b"#", b"+/+", b"a/b/c", b"+/dd/#", b"long-level-name/+/#", b"c/+/+/#", b"/#"]
    hb = eng.pinned(len(buf))
    hb[:] = buf
    ho = eng.pinned(len(off), np.uint32)
    ho[:] = off
    for step, f in enumerate(adds * 2):
        if step < len(adds):
            eng.trie_insert(f)
            py.insert(f)
        else:
            eng.trie_delete(f)
            py.delete(f)
        eng.commit()
        assert eng.stats()["delta_commits"] >= 1
        t1 = eng.match_device_submit(db.data_ptr(), do.data_ptr(), len(topics), int(off[-1]))
        t2 = eng.match_batch_submit(hb, ho)
        row, fid, _ = _dev_result(eng.match_device_wait(t1), len(topics))
        hres = eng.match_batch_wait(t2)
        for i, t in enumerate(topics):
            want = sorted(py.match(t))
            assert _sets(eng, row, fid, i) == want, (step, t)
            assert sorted(eng.filter_bytes(int(x)) for x in hres.row(i)) == want, (step, t)
    eng.close()


def test_writer_thread_deltas_while_matching(emqx):
    """A writer thread adds and removes the filter '#' (matches every non-'$' topic) with a
    delta commit each time, while this thread keeps matching: every result has exactly the old
    or the new epoch's rows (total pairs base or base + n), on the sync and pipelined paths."""
    import torch
    import workloads
    w = workloads.generate(1, 5000, 20000)
    eng = _load(emqx, w)
    db = torch.from_numpy(w.tbytes).cuda()
    do = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    nb = int(w.toff[-1])
    base = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, nb).n_pairs
    not_dollar = sum(1 for i in range(w.nt) if not w.topic(i).startswith(b"$"))
    stop = threading.Event()
    errors = []
    commits = [0]

    def writer():
        try:
            while not stop.is_set():
                eng.trie_insert(b"#")
                eng.commit()
                eng.trie_delete(b"#")
                eng.commit()
                commits[0] += 2
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = threading.Thread(target=writer)
    th.start()
    seen = set()
    try:
        t_end = time.time() + 6.0
        pend = []
        while time.time() < t_end:
            seen.add(eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, nb).n_pairs)
            pend.append(eng.match_device_submit(db.data_ptr(), do.data_ptr(), w.nt, nb))
            if len(pend) == eng.PIPES:
                seen.add(eng.match_device_wait(pend.pop(0)).n_pairs)
        for t in pend:
            seen.add(eng.match_device_wait(t).n_pairs)
    finally:
        stop.set()
        th.join()
    assert not errors, errors
    assert commits[0] >= 10
    assert seen <= {base, base + not_dollar}, (seen, base, not_dollar)
    assert eng.stats()["delta_commits"] >= 10
    eng.close()


def test_matches_never_wait_for_a_full_rebuild(emqx):
    """cfg3 at 10M filters: a writer thread adds one filter and commits with delta commits off
    (a full rebuild, seconds of host work plus GBs of uploads).  Matches issued meanwhile return
    within a pass time against the old epoch; once commit() has returned they see the new one."""
    import torch
    import workloads
    w = workloads.generate(3, 10_000_000, 200_000)
    eng = _load(emqx, w)
    db = torch.from_numpy(w.tbytes).cuda()
    do = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    nb = int(w.toff[-1])
    old = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, nb)
    old_rows = _dev_result(old, w.nt)
    eng.tune("delta_commit", 0)
    eng.trie_insert(b"site/+/device/+/+/+")  # matches every cfg3 topic: one more pair per row
    done = threading.Event()
    t_commit = {}

    def writer():
        t0 = time.perf_counter()
        eng.commit()
        t_commit["s"] = time.perf_counter() - t0
        done.set()

    th = threading.Thread(target=writer)
    th.start()
    during, lat = [], []
    while not done.is_set():
        t0 = time.perf_counter()
        d = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, nb)
        lat.append(time.perf_counter() - t0)
        if not done.is_set():
            during.append(d.n_pairs)
    th.join()
    new = eng.match_device(db.data_ptr(), do.data_ptr(), w.nt, nb)
    assert new.n_pairs == old.n_pairs + w.nt
    print(f"full rebuild {t_commit['s']:.2f}s; {len(lat)} matches meanwhile, "
          f"max {max(lat) * 1e3:.1f} ms, median {np.median(lat) * 1e3:.2f} ms")
    assert t_commit["s"] > 1.0  # a real rebuild ran
    # every match had the old or the new answer, and once one saw the new epoch none saw the
    # old one again (the swap is atomic); most of the rebuild ran against the old epoch
    assert set(during) <= {old.n_pairs, new.n_pairs}
    k = during.index(new.n_pairs) if new.n_pairs in during else len(during)
    assert all(x == new.n_pairs for x in during[k:])
    assert k >= 20, k
    assert np.median(lat) < 0.05 and max(lat) < 0.5, (np.median(lat), max(lat))
    row, fid, ex = _dev_result(new, w.nt)
    assert np.array_equal(ex, old_rows[2])
    assert np.array_equal(np.diff(row.astype(np.int64)), np.diff(old_rows[0].astype(np.int64)) + 1)
    eng.close()


def test_host_pipes_equal_match_batch(emqx):
    import itertools
    import workloads
    w = workloads.generate(1, 5000, 30000)
    eng = _load(emqx, w)
    words = "abcdefghij"
    for k in range(11):
        for pat in itertools.product((0, 1), repeat=k):
            lv = ["+" if x else words[i] for i, x in enumerate(pat)]
            eng.trie_insert(("/".join(lv + ["#"]) if k < 10 else "/".join(lv)).encode())
    # plain route keys for some names of the first batch only: the other batches have no exact
    # hit, so their exact ids come from the pipe's all-NONE buffer (no download, CTL_XHIT)
    for i in range(0, 10000, 7):
        eng.route_ref(w.topic(i))
    eng.commit()
    heavy = ["/".join(words).encode()] * 1000  # ~2M pairs: overflows a fresh pipe's staging
    batches = []
    for a, b in ((0, 10000), (10000, 20000), (20000, 30000)):
        o = (w.toff[a:b + 1] - w.toff[a]).astype(np.uint32)
        batches.append((w.tbytes[int(w.toff[a]):int(w.toff[b])].copy(), o))
    hb, ho = emqx.engine.pack(heavy, np.uint32)
    batches = batches[:1] + [(np.zeros(0, np.uint8), np.zeros(1, np.uint32)), (hb, ho)] + batches[1:]
    want = [eng.match_packed(b, o) for b, o in batches]
    for mode in (1, 0):
        eng.tune("host_out", mode)
        got, pend = [], []
        for b, o in batches + batches:
            pend.append(eng.match_batch_submit(b, o))
            if len(pend) == eng.HOST_PIPES:
                got.append(eng.match_batch_wait(pend.pop(0)))
        got += [eng.match_batch_wait(t) for t in pend]
        for i, g in enumerate(got):
            wnt = want[i % len(batches)]
            assert np.array_equal(g.row_ptr, wnt.row_ptr), (mode, i)
            assert np.array_equal(g.filter_id, wnt.filter_id), (mode, i)
            assert np.array_equal(g.exact_id, wnt.exact_id), (mode, i)
    b, o = batches[0]
    ts = [eng.match_batch_submit(b, o) for _ in range(eng.HOST_PIPES)]
    with pytest.raises(emqx.EngineError):
        eng.match_batch_submit(b, o)  # every host pipe holds a pass
    for t in ts:
        eng.match_batch_wait(t)
    with pytest.raises(emqx.EngineError):
        eng.match_batch_wait(ts[0])  # already taken
    assert eng.stats()["reruns"] >= 1
    eng.close()


def test_filters_copy(emqx):
    eng = emqx.Engine()
    fs = [b"a/+", b"", b"x" * 300, b"$SYS/#", b"b/c"]
    ids = [eng.trie_insert(f) if b"+" in f or b"#" in f else eng.route_ref(f) for f in fs]
    eng.commit()
    assert eng.filters_bytes(ids[::-1]) == fs[::-1]
    assert [eng.filter_bytes(i) for i in ids] == fs
    eng.close()
