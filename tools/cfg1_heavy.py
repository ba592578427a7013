"""Which cfg1 topics set the walk's floor (MEASUREMENTS r06 "what bounds cfg1's walk").

Walks batches of 6,250 cfg1 topics chosen by their number of trie matches (the engine's own rows
for the whole 100k batch; parity is the tests' business):
the lightest, a random sample, and the heaviest.  If the ~29 us floor of a small batch comes
from its heaviest topics' chains, the light batch walks much faster; if it is a per-launch or
per-iteration cost, all three take about as long.  Prints one JSON line of walk times (HIP
events, mean over --reps passes) and each batch's match counts.

    python tools/cfg1_heavy.py [--n 6250] [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=6250)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import numpy as np
    import torch
    import workloads
    from emqx_amd import Engine

    w = workloads.generate(1, None, 100_000)
    eng = Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    for i in np.nonzero(w.fwild)[0]:
        eng.trie_insert(w.filter(int(i)))
    eng.commit()
    res = eng.match_packed(w.tbytes, w.toff.astype(np.uint32))
    cnt = np.diff(np.asarray(res.row_ptr, dtype=np.int64))
    order = np.argsort(cnt, kind="stable")
    rng = np.random.default_rng(1)
    picks = {"lightest": order[:a.n], "random": rng.choice(len(cnt), a.n, replace=False),
             "heaviest": order[-a.n:]}
    dev = torch.device("cuda", 0)
    out = {"topics": a.n}
    for name, idx in picks.items():
        idx = np.sort(idx)
        parts = [w.topic(int(i)) for i in idx]
        tb = np.frombuffer(b"".join(parts), np.uint8)
        to = np.zeros(len(parts) + 1, np.uint32)
        to[1:] = np.cumsum([len(p) for p in parts])
        db = torch.from_numpy(tb.copy()).to(dev)
        do = torch.from_numpy(to.view(np.int32).copy()).to(dev)
        for _ in range(5):
            eng.match_device(db.data_ptr(), do.data_ptr(), len(parts), len(tb))
        torch.cuda.synchronize()
        eng.set_profiling(True)
        s0 = eng.stats()
        for _ in range(a.reps):
            eng.match_device(db.data_ptr(), do.data_ptr(), len(parts), len(tb))
        torch.cuda.synchronize()
        s1 = eng.stats()
        eng.set_profiling(False)
        k = max(1, s1["walk_launches"] - s0["walk_launches"])
        c = cnt[idx]
        out[name] = {"walk_us": round((s1["walk_ms"] - s0["walk_ms"]) / k * 1e3, 2),
                     "matches_mean": round(float(c.mean()), 1), "matches_max": int(c.max())}
    out["all_100k_matches_max"] = int(cnt.max())
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
