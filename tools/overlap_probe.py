"""Experiment: do two concurrent device passes (two engine handles = two HIP streams, driven
from two host threads) overlap one pass's walk tail with the other's work?

    python tools/overlap_probe.py [--topics 2000000] [--steps 20]
Prints topics/s for one handle stepping alone and for two handles stepping concurrently.
"""
import argparse
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads  # noqa: E402
from emqx_amd import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topics", type=int, default=2_000_000)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    nf, _, sf, st = workloads.DEFAULTS[3]
    w = workloads.generate(3, nf, a.topics, sf, st)
    dev = torch.device("cuda", 0)
    engs = []
    for _ in range(2):
        e = Engine(device=0)
        e.route_ref_many(w.fbytes, w.foff)
        wild = np.nonzero(w.fwild.astype(bool))[0]
        e.trie_insert_many(*_sub(w.fbytes, w.foff, wild))
        e.commit()
        engs.append(e)
    tb = torch.from_numpy(w.tbytes).to(dev)
    to = torch.from_numpy(w.toff.view(np.int32)).to(dev)
    nb = int(w.toff[-1])
    args = (tb.data_ptr(), to.data_ptr(), w.nt, nb)
    for e in engs:
        for _ in range(3):
            e.match_device(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        engs[0].match_device(*args)
    one = time.perf_counter() - t0

    def run(e):
        for _ in range(a.steps):
            e.match_device(*args)
    th = [threading.Thread(target=run, args=(e,)) for e in engs]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    two = time.perf_counter() - t0
    print(f"one handle : {a.steps * w.nt / one / 1e9:.3f} G topics/s ({one / a.steps * 1e3:.3f} ms/batch)")
    print(f"two handles: {2 * a.steps * w.nt / two / 1e9:.3f} G topics/s ({two / a.steps / 2 * 1e3:.3f} ms/batch)")


def _sub(fb, fo, idx):
    lens = (fo[idx + 1] - fo[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    parts = [fb[int(fo[i]):int(fo[i + 1])] for i in idx] if len(idx) < 1000 else None
    if parts is not None:
        return np.concatenate(parts), off
    starts = fo[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + \
        np.arange(int(lens.sum()), dtype=np.int64)
    return fb[pos], off


if __name__ == "__main__":
    main()
