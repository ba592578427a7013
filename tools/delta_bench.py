"""Subscribe-rate measurement for delta commits on the full cfg3 index.

Loads the BASELINE cfg3 index (10M filters: route keys + wildcard trie filters), then runs
rounds of K subscribes (route key + trie filter for wildcards, as emqx_router:do_add_route) and
a commit, and K unsubscribes of the same filters and a commit.  Reports the full-build commit
time, the delta-commit times, and checks a topic sample after every round against the answer
of the untouched index (the index is back to its initial content after each round, so the
answer must be bit-identical; rows compared as sorted id lists).

  python tools/delta_bench.py [--filters 10000000] [--k 1000] [--rounds 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rows(res):
    rp = res.row_ptr.astype(np.int64)
    return rp, np.concatenate([np.sort(res.filter_id[rp[i]:rp[i + 1]]) for i in range(len(rp) - 1)])


_last = {"delta": 0}


def _kind(eng):
    d = eng.stats()["delta_commits"]
    k = "delta" if d > _last["delta"] else "full"
    _last["delta"] = d
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=10_000_000)
    ap.add_argument("--topics", type=int, default=100_000)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()

    import workloads
    from emqx_amd import Engine

    t0 = time.time()
    w = workloads.generate(3, args.filters, args.topics)
    churn = workloads.generate(3, args.k * args.rounds * 8, 1, seed_f=9_999_991, seed_t=1)
    print(f"generated in {time.time() - t0:.1f}s", flush=True)

    eng = Engine()
    wild = np.nonzero(w.fwild)[0]
    eng.route_ref_many(w.fbytes, w.foff)
    fo = w.foff.astype(np.int64)
    lens = fo[wild + 1] - fo[wild]
    wo = np.zeros(len(wild) + 1, np.int64)
    wo[1:] = np.cumsum(lens)
    wb = w.fbytes[np.repeat(fo[wild] - wo[:-1], lens) + np.arange(wo[-1])]
    eng.trie_insert_many(wb, wo.astype(np.uint64))
    t0 = time.time()
    eng.commit()
    full_ms = (time.time() - t0) * 1e3
    st = eng.stats()
    print(f"full build: {full_ms:.0f} ms ({st['n_trie_filters']} trie filters, "
          f"{st['n_route_keys']} keys, {st['n_nodes']} nodes)", flush=True)

    base = eng.match_packed(w.tbytes, w.toff)
    brp, bids = _rows(base)
    cf = churn.foff.astype(np.int64)
    subs = [bytes(churn.fbytes[cf[i]:cf[i + 1]]) for i in range(churn.nf)]
    cwild = churn.fwild.astype(bool)
    fresh = [i for i in range(churn.nf) if eng.lookup_id(subs[i]) is None]  # new filters only
    args.k = min(args.k, len(fresh) // args.rounds)
    subs = [subs[i] for i in fresh]
    cwild = cwild[fresh]

    add_ms, del_ms, kinds = [], [], []
    for r in range(args.rounds):
        batch = range(r * args.k, (r + 1) * args.k)
        t0 = time.time()
        for i in batch:
            eng.route_ref(subs[i])
            if cwild[i]:
                eng.trie_insert(subs[i])
        t1 = time.time()
        eng.commit()
        add_ms.append((time.time() - t1) * 1e3)
        kinds.append(_kind(eng))
        reg_ms = (t1 - t0) * 1e3
        for i in batch:
            eng.route_unref(subs[i])
            if cwild[i]:
                eng.trie_delete(subs[i])
        t1 = time.time()
        eng.commit()
        del_ms.append((time.time() - t1) * 1e3)
        kinds.append(_kind(eng))
        rp, ids = _rows(eng.match_packed(w.tbytes, w.toff))
        assert np.array_equal(rp, brp) and np.array_equal(ids, bids), f"round {r}: answer changed"
        print(f"round {r}: +{args.k} commit {add_ms[-1]:.1f} ms, -{args.k} commit "
              f"{del_ms[-1]:.1f} ms (registry {reg_ms:.1f} ms) {kinds[-2:]}", flush=True)

    st = eng.stats()
    out = {"filters": args.filters, "k": args.k, "rounds": args.rounds,
           "full_commit_ms": round(full_ms, 1),
           "delta_add_commit_ms_median": round(float(np.median(add_ms)), 2),
           "delta_del_commit_ms_median": round(float(np.median(del_ms)), 2),
           "subscribes_per_s_via_delta": round(args.k / (np.median(add_ms) / 1e3)),
           "commit_kinds": kinds, "delta_commits": st["delta_commits"],
           "full_commits": st["full_commits"], "parity": "identical after every round"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
