"""cfg4's key-partitioned layout measured on one GPU (SURVEY 8e's
alternative).  Builds the index one rank of G would hold (every wildcard filter and
the plain route keys emqxgm_key_owners gives part 0: 12.5M of cfg4's 100M at G = 8, an exact table
of ~1.1 GB, under the TLB's reach) and times, on the full 1M-name batch:

  shard_pass     the normal pass over all names against the shard's index (its k_exact is the
                 per-name figure on the 1/G table; every name probed)
  owned_pass     emqxgm_exact_owned_device: every name hashed, only the owned ones probed
  block_pass     the pass over this rank's block of n / G topics (tokenizer, walk, wildcard keys)

and, with --baseline, the normal pass against the whole cfg4 index (the replica layout's).
Kernel averages come from rocprofv3 (run it under `rocprofv3 --kernel-trace --stats`); the JSON
line has wall-clock means of the synchronous calls.

    python tools/key_shard_bench.py [--parts 8] [--baseline] [--reps 50]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--baseline", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import torch
    import workloads
    from emqx_amd import Engine
    from emqx_amd import dist as D
    from tests.test_dist import _subset

    dev = torch.device("cuda", 0)
    t0 = time.time()
    w = workloads.generate(4, a.filters, a.topics)
    print(f"generated {w.nf} filters, {w.nt} topics in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    tb = torch.from_numpy(w.tbytes).to(dev)
    to = torch.from_numpy(w.toff.view(np.int32)).to(dev)
    n, nbytes = w.nt, int(w.toff[-1])
    G = a.parts
    out = {"workload": f"cfg4: {w.nf} filters, {n} names", "parts": G}

    def build(idx):
        eng = Engine()
        fb, fo = _subset(w, idx)
        eng.route_ref_many(fb, fo)
        wi = np.nonzero(w.fwild[idx])[0]
        wb, wo = _subset(type("W", (), {"fbytes": fb, "foff": fo})(), wi)
        eng.trie_insert_many(wb, wo)
        t1 = time.time()
        eng.commit()
        st = eng.stats()
        return eng, {"filters": int(len(idx)), "route_keys": int(st["n_route_keys"]),
                     "exact_table_bytes": int(st["exact_slots"]) * 32, "build_s": round(time.time() - t1, 1)}

    def timed(f):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(a.reps):
            f()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t1) / a.reps * 1e3, 4)

    def pass_kernels(eng, b, o, m, mb):
        eng.set_profiling(True)
        s0 = eng.stats()
        ms = timed(lambda: eng.match_device(b.data_ptr(), o.data_ptr(), m, mb))
        s1 = eng.stats()
        eng.set_profiling(False)
        k = max(1, s1["walk_launches"] - s0["walk_launches"])
        return {"wall_ms": ms, "k_tok_ms": round((s1["tok_ms"] - s0["tok_ms"]) / k, 4),
                "k_exact_ms": round((s1["exact_ms"] - s0["exact_ms"]) / k, 4),
                "k_walk_ms": round((s1["walk_ms"] - s0["walk_ms"]) / k, 4)}

    if a.baseline:
        eng, info = build(np.arange(w.nf))
        out["replica"] = dict(info, pass_=pass_kernels(eng, tb, to, n, nbytes))
        eng.close()
        del eng
    t0 = time.time()
    probe = Engine()
    mine = D.key_shard_filters(probe, w.fbytes, w.foff, w.fwild, G, 0)
    probe.close()
    out["owners_s"] = round(time.time() - t0, 1)
    eng, info = build(mine)
    shard = dict(info)
    shard["shard_pass"] = pass_kernels(eng, tb, to, n, nbytes)
    own = torch.empty(n, dtype=torch.int32, device=dev)
    shard["owned_pass_wall_ms"] = timed(
        lambda: eng.exact_owned_device(tb.data_ptr(), to.data_ptr(), n, G, 0, own.data_ptr()))
    shard["owned_names_found"] = int((own != -1).sum())
    b0, b1 = 0, n // G
    lo, hi = (int(x) for x in to[[b0, b1]].tolist())
    bo = (to[b0:b1 + 1] - lo).contiguous()
    bb = tb[lo:hi].contiguous()
    shard["block_pass"] = pass_kernels(eng, bb, bo, b1 - b0, hi - lo)
    out["shard"] = shard
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
