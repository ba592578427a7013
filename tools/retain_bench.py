"""Reverse-match throughput of the retained-topic store: N cfg3 topics
retained, a batch of cfg3-shaped subscription filters matched against them (emqxgm_retain_match,
end to end: host filters in, host CSR of topic ids out).

  python tools/retain_bench.py [--topics 2000000] [--filters 100000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topics", type=int, default=2_000_000)
    ap.add_argument("--filters", type=int, default=100_000)
    args = ap.parse_args()
    import workloads
    from emqx_amd import Retainer
    w = workloads.generate(3, args.filters, args.topics)
    r = Retainer()
    t0 = time.perf_counter()
    to = w.toff.astype(np.int64)
    for i in range(w.nt):
        r.store_retained(bytes(w.tbytes[to[i]:to[i + 1]]))
    t1 = time.perf_counter()
    r.commit()
    t2 = time.perf_counter()
    filters = [w.filter(i) for i in range(w.nf)]
    r.match_ids(filters[:1000], 1)
    best, n_ids = 1e9, 0
    for _ in range(3):
        t3 = time.perf_counter()
        ptr, ids = r.match_ids(filters, 1)
        best = min(best, time.perf_counter() - t3)
        n_ids = len(ids)
    # delta commits: 10k new retained topics, then 10k deletions of base topics
    extra = [b"x/" + w.topic(i) for i in range(10_000)]
    t4 = time.perf_counter()
    for t in extra:
        r.store_retained(t)
    t5 = time.perf_counter()
    r.commit()
    t6 = time.perf_counter()
    for i in range(10_000):
        r.delete_message(w.topic(i))
    r.commit()
    t7 = time.perf_counter()
    ptr2, ids2 = r.match_ids(filters, 1)
    st = r.stats()
    print(json.dumps({
        "delta_store_10k_commit_s": round(t6 - t5, 4), "delta_store_10k_registry_s": round(t5 - t4, 4),
        "delete_10k_base_topics_incl_registry_s": round(t7 - t6, 4), "stats": st,
        "ids_after_churn": int(len(ids2))}), flush=True)
    print(json.dumps({
        "retained_topics": r.size(), "filters": len(filters), "ids_selected": n_ids,
        "store_registry_s": round(t1 - t0, 3), "commit_build_s": round(t2 - t1, 3),
        "match_s": round(best, 4), "filters_per_s": round(len(filters) / best),
        "ids_per_s": round(n_ids / best)}), flush=True)


if __name__ == "__main__":
    main()
