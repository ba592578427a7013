"""emqx_broker_bench:run1/0 on the MI355X engine (apps/emqx/src/emqx_broker_bench.erl:25-86).

The reference bench: 80 subscribers x 1,000 `emqx_broker:subscribe` of
``device/{{id}}/+/{{num}}/#`` (InsertRps), then 80 publishers x 10,000
`emqx_router:match_routes` of ``device/{{id}}/foo/{{num}}/bar/1/2/3/4/5`` with num = 1, each
expecting exactly one route (LookupRps, :163-170), then unsubscribe all until
`emqx_trie:empty()` (TimeToUnsubscribeAll).

Here a subscribe is the engine's subscriber_add + route_add (the route {Topic, node()} and,
for a wildcard, its trie filter: emqx_router_utils.erl:34-39), through the C-ABI.  Routes become
visible at a commit; two insert rates are reported:
  * insert_rps_group_commit: all 80,000 subscribes, then one commit;
  * insert_rps_commit_each: subscribe + commit, one at a time (every subscribe visible before
    the next, as the reference's synchronous transaction), over the first --strict subscribes.
The 800,000 lookups run as one batch: device-resident (kernel pipeline) and end-to-end (host
topic bytes in, host CSR out), with every row checked to hold exactly one route.

  python tools/broker_bench.py [--subs 80] [--sub-ops 1000] [--pubs 80] [--pub-ops 10000]
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
    ap.add_argument("--subs", type=int, default=80)
    ap.add_argument("--sub-ops", type=int, default=1000)
    ap.add_argument("--pubs", type=int, default=80)
    ap.add_argument("--pub-ops", type=int, default=10000)
    ap.add_argument("--strict", type=int, default=2000)
    args = ap.parse_args()

    import torch
    from emqx_amd import Engine
    from emqx_amd.engine import pack

    node = 0
    sub_topics = [f"device/{i}/+/{n}/#".encode() for i in range(1, args.subs + 1)
                  for n in range(1, args.sub_ops + 1)]
    pub_topics = [f"device/{(p % args.subs) + 1}/foo/1/bar/1/2/3/4/5".encode()
                  for p in range(1, args.pubs + 1) for _ in range(args.pub_ops)]
    out = {"bench": "emqx_broker_bench:run1", "subscribers": args.subs, "sub_ops": args.sub_ops,
           "publishers": args.pubs, "pub_ops": args.pub_ops}

    # ---- strict: every subscribe committed before the next (delta commits) ----
    eng = Engine()
    eng.set_local_node(node)
    k = min(args.strict, len(sub_topics))
    t0 = time.perf_counter()
    for s, f in enumerate(sub_topics[:k]):
        eng.subscriber_add(f, s)
        eng.route_add(f, node)
        eng.commit()
    dt = time.perf_counter() - t0
    out["insert_rps_commit_each"] = round(k / dt)
    out["strict_sample"] = k
    out["strict_delta_commits"] = eng.stats()["delta_commits"]
    eng.close()

    # ---- group commit: InsertRps over all subscribes ----
    eng = Engine()
    eng.set_local_node(node)
    t0 = time.perf_counter()
    for s, f in enumerate(sub_topics):
        eng.subscriber_add(f, s)
        eng.route_add(f, node)
    t1 = time.perf_counter()
    eng.commit()
    t2 = time.perf_counter()
    out["insert_rps_group_commit"] = round(len(sub_topics) / (t2 - t0))
    out["insert_registry_s"] = round(t1 - t0, 4)
    out["insert_commit_s"] = round(t2 - t1, 4)

    # ---- lookups: one batch of pubs x pub_ops topics ----
    tb, to = pack(pub_topics, np.uint32)
    t0 = time.perf_counter()
    res = eng.match_packed(tb, to)
    e2e = time.perf_counter() - t0
    t0 = time.perf_counter()
    res = eng.match_packed(tb, to)
    e2e = min(e2e, time.perf_counter() - t0)
    counts = np.diff(res.row_ptr.astype(np.int64))
    assert np.all(counts == 1), "every lookup must match exactly one route ([_] = match_routes)"
    exp = {f"device/{i}/+/1/#".encode() for i in range(1, args.subs + 1)}
    assert {eng.filter_bytes(int(f)) for f in np.unique(res.filter_id)} == exp
    dev = torch.device("cuda", 0)
    db = torch.from_numpy(tb).to(dev)
    do = torch.from_numpy(to.view(np.int32)).to(dev)
    for _ in range(3):
        eng.match_device(db.data_ptr(), do.data_ptr(), len(pub_topics), int(to[-1]))
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.match_device(db.data_ptr(), do.data_ptr(), len(pub_topics), int(to[-1]))
    torch.cuda.synchronize()
    kt = (time.perf_counter() - t0) / reps
    out["lookup_rps_device_resident"] = round(len(pub_topics) / kt)
    out["lookup_rps_end_to_end"] = round(len(pub_topics) / e2e)
    st = eng.stats()
    out["index"] = {"trie_filters": st["n_trie_filters"], "route_keys": st["n_route_keys"],
                    "nodes": st["n_nodes"], "device_bytes": st["device_bytes"]}

    # ---- unsubscribe all until the trie is empty ----
    t0 = time.perf_counter()
    for s, f in enumerate(sub_topics):
        eng.subscriber_delete(f, s)
        eng.route_delete(f, node)
    eng.commit()
    assert eng.trie_empty()
    out["time_to_unsubscribe_all_s"] = round(time.perf_counter() - t0, 4)
    out["commits"] = {"full": eng.stats()["full_commits"], "delta": eng.stats()["delta_commits"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
