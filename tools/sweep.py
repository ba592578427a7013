"""Tuning sweep on one GPU: build the cfg index once, then time the match pipeline for several
walk geometries (and batch sizes).  Prints one line per setting.

    python tools/sweep.py [--cfg 3] [--wg 2,4,6,8] [--topics 2000000] [--steps 10]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--wg", default="2,4,6,8")
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import workloads
    from emqx_amd import Engine
    t0 = time.time()
    w = workloads.generate(args.cfg, args.filters, args.topics)
    eng = Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    wild = np.nonzero(w.fwild)[0]
    if len(wild) == w.nf:
        eng.trie_insert_many(w.fbytes, w.foff)
    else:
        for i in wild:  # small configs only
            eng.trie_insert(w.filter(int(i)))
    eng.commit()
    print(f"setup {time.time() - t0:.1f}s  {eng.stats()['n_nodes']} nodes", flush=True)
    tb = torch.from_numpy(w.tbytes).cuda()
    to = torch.from_numpy(w.toff.view(np.int32)).cuda()
    nb = int(w.toff[-1])
    for wg in [int(x) for x in args.wg.split(",")]:
        eng.tune("walk_wg_per_cu", wg)
        for _ in range(2):
            eng.match_device(tb.data_ptr(), to.data_ptr(), w.nt, nb)
        s0 = eng.stats()
        eng.set_profiling(True)
        t = time.perf_counter()
        for _ in range(args.steps):
            eng.match_device(tb.data_ptr(), to.data_ptr(), w.nt, nb)
        dt = (time.perf_counter() - t) / args.steps
        eng.set_profiling(False)
        s1 = eng.stats()
        walk = (s1["walk_ms"] - s0["walk_ms"]) / max(1, s1["walk_launches"] - s0["walk_launches"])
        pipe = (s1["total_ms"] - s0["total_ms"]) / args.steps
        print(f"wg_per_cu={wg}: step {dt * 1e3:.3f} ms  pipeline {pipe:.3f} ms  walk {walk:.3f} ms "
              f" -> {w.nt / dt / 1e9:.3f} G topics/s", flush=True)


if __name__ == "__main__":
    main()
