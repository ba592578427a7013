"""r04: what differs in the GM_SMALL_WS=4 build's failure of test_host_pipes_equal_match_batch
(gpurun_out/r03s3_ws/pytest.log: equal row pointers, different filter ids in batch 0's tail) --
the set of a row, or only the order of its ids?  Runs the test's exact sequence with whatever
engine library is in place and compares each pipe result with the synchronous one row by row,
as arrays and as sets, and both with the oracle's rows (as sets).  Prints one JSON line."""
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import emqx_amd  # noqa: E402
import workloads  # noqa: E402
from oracle.cref import RefIndex  # noqa: E402


def main():
    w = workloads.generate(1, 5000, 30000)
    eng = emqx_amd.Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.nonzero(w.fwild.astype(bool))[0]
    for i in wi:
        eng.trie_insert(w.filter(int(i)))
    words = "abcdefghij"
    extra = []
    for k in range(11):
        for pat in itertools.product((0, 1), repeat=k):
            lv = ["+" if x else words[i] for i, x in enumerate(pat)]
            f = ("/".join(lv + ["#"]) if k < 10 else "/".join(lv)).encode()
            eng.trie_insert(f)
            extra.append(f)
    for i in range(0, 10000, 7):
        eng.route_ref(w.topic(i))
    eng.commit()
    heavy = ["/".join(words).encode()] * 1000
    batches = []
    for a, b in ((0, 10000), (10000, 20000), (20000, 30000)):
        o = (w.toff[a:b + 1] - w.toff[a]).astype(np.uint32)
        batches.append((w.tbytes[int(w.toff[a]):int(w.toff[b])].copy(), o))
    hb, ho = emqx_amd.engine.pack(heavy, np.uint32)
    batches = batches[:1] + [(np.zeros(0, np.uint8), np.zeros(1, np.uint32)), (hb, ho)] + batches[1:]
    want = [eng.match_packed(b, o) for b, o in batches]
    res = {"batches": []}
    eng.tune("host_out", 1)
    got, pend = [], []
    for b, o in batches + batches:
        pend.append(eng.match_batch_submit(b, o))
        if len(pend) == eng.HOST_PIPES:
            got.append(eng.match_batch_wait(pend.pop(0)))
    got += [eng.match_batch_wait(t) for t in pend]
    for i, g in enumerate(got):
        wnt = want[i % len(batches)]
        rows_order = rows_set = 0
        n = len(wnt.row_ptr) - 1
        for t in range(n):
            a = g.filter_id[int(g.row_ptr[t]):int(g.row_ptr[t + 1])]
            bb = wnt.filter_id[int(wnt.row_ptr[t]):int(wnt.row_ptr[t + 1])]
            if not np.array_equal(a, bb):
                if np.array_equal(np.sort(a), np.sort(bb)):
                    rows_order += 1
                else:
                    rows_set += 1
        res["batches"].append({"i": i, "rows": n, "rows_equal_ptr": bool(np.array_equal(g.row_ptr, wnt.row_ptr)),
                               "rows_order_only": rows_order, "rows_set_differs": rows_set})
    # the synchronous result of batch 0 against the oracle (sets)
    ref = RefIndex(True)
    fb = np.concatenate([w.fbytes, np.frombuffer(b"".join(extra), np.uint8)])
    lens = np.array([len(f) for f in extra], np.uint64)
    fo = np.concatenate([w.foff, w.foff[-1] + np.cumsum(lens)])
    kinds = np.concatenate([2 + w.fwild.astype(np.uint8), np.full(len(extra), 1, np.uint8)])
    ref.add_many(fb, fo.astype(np.uint64), kinds)
    b0, o0 = batches[0]
    rrow, rfil, _ = ref.match(b0, o0)
    bad = 0
    for t in range(len(o0) - 1):
        mine = {eng.filter_bytes(int(x)) for x in want[0].filter_id[int(want[0].row_ptr[t]):int(want[0].row_ptr[t + 1])]}
        theirs = {bytes(fb[int(fo[x]):int(fo[x + 1])]) for x in rfil[int(rrow[t]):int(rrow[t + 1])]}
        bad += mine != theirs
    res["batch0_sync_rows_differing_from_oracle"] = bad
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
