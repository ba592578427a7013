"""The subscribe path's tail during a background rebuild of the bench's cfg3 index (diagnosis):
bench.py's _subscribe_latency, with EMQXGM_DEBUG_SLOW=<ms> naming the writer-side steps slower
than that on stderr.

    EMQXGM_DEBUG_SLOW=10 python tools/subscribe_probe.py [--filters 10000000]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import bench
    import workloads
    from emqx_amd import Engine
    w = workloads.generate(3, a.filters, 1000)
    eng = Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    eng.trie_insert_many(w.fbytes, w.foff)
    t0 = time.time()
    eng.commit()
    print(f"index in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    for r in range(a.rounds):
        print(json.dumps(bench._subscribe_latency(eng, w)), flush=True)


if __name__ == "__main__":
    main()
