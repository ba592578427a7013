"""Throughput of emqxgm_match_rules: 1M cfg3 topic names against an ordered
ACL-style rule list, end to end (host names in, host first-match indices out).

  python tools/rules_bench.py [--names 1000000] [--rules 64]
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
    ap.add_argument("--names", type=int, default=1_000_000)
    ap.add_argument("--rules", type=int, default=64)
    args = ap.parse_args()
    import workloads
    from emqx_amd import Engine, NONE
    from emqx_amd.engine import RULE_WORDS
    w = workloads.generate(3, 1000, args.names)
    names = [w.topic(i) for i in range(w.nt)]
    # rules never matching until the last few: every name scans most of the list
    rules = [f"site/{s}/device/+/m{s % 32}/#".encode() for s in range(10_000, 10_000 + args.rules - 2)]
    rules += [b"site/+/device/+/m7/#", b"site/#"]
    eng = Engine()
    out = {}
    for words in (False, True):
        fl = [RULE_WORDS if words else 0] * len(rules)
        r = eng.match_rules(names[:1000], rules, fl)
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            r = eng.match_rules(names, rules, fl)
            best = min(best, time.perf_counter() - t0)
        hits = int((r != NONE).sum())
        out["words" if words else "binary"] = {
            "names_per_s_end_to_end": round(len(names) / best),
            "rule_evals_per_s": round(float(np.where(r == NONE, len(rules), r + 1).sum()) / best),
            "matched": hits}
    print(json.dumps({"names": len(names), "rules": len(rules), **out}), flush=True)


if __name__ == "__main__":
    main()
