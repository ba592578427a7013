"""Where a NIF window's time goes: per-call wall time of the batcher core's add_many / flush /
collect (emqxgm_batcher_*) on cfg3 windows, with 1 and EMQXGM_HOST_PIPES windows in flight.

    python tools/window_probe.py [--filters 10000000] [--windows 16384,65536]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--filters", type=int, default=10_000_000)
ap.add_argument("--windows", default="16384,65536")
ap.add_argument("--count", type=int, default=40)
a = ap.parse_args()

import emqx_amd  # noqa: E402
import workloads  # noqa: E402

w = workloads.generate(3, a.filters, 1_048_576)
eng = emqx_amd.Engine()
eng.route_ref_many(w.fbytes, w.foff)
eng.trie_insert_many(w.fbytes, w.foff)
eng.commit()
off = w.toff.astype(np.int64)
out = {}
for W in [int(x) for x in a.windows.split(",")]:
    cuts = [(w.tbytes[off[i]:off[i + W]], (off[i:i + W + 1] - off[i]).astype(np.uint32), i)
            for i in range(0, w.nt - W + 1, W)]
    for inflight_max in (1, eng.HOST_PIPES):
        b = emqx_amd.Batcher(eng, window_topics=W, window_bytes=64 * W)
        t_add, t_flush, t_coll, lat, inflight = [], [], [], [], []
        t0 = None
        for k in range(a.count + 5):
            if k == 5:
                t_add.clear(), t_flush.clear(), t_coll.clear(), lat.clear()
                t0 = time.perf_counter()
            buf, rel, i = cuts[k % len(cuts)]
            s = time.perf_counter_ns()
            b.add_many(buf, rel, i)
            t_add.append(time.perf_counter_ns() - s)
            if len(inflight) == inflight_max:
                s = time.perf_counter_ns()
                _, _, _, ns = b.collect(inflight.pop(0), materialize=False)
                t_coll.append(time.perf_counter_ns() - s)
                lat.append(ns)
            s = time.perf_counter_ns()
            inflight.append(b.flush())
            t_flush.append(time.perf_counter_ns() - s)
        while inflight:
            b.collect(inflight.pop(0), materialize=False)
        el = time.perf_counter() - t0
        b.close()
        med = lambda v: round(float(np.median(v)) / 1e3, 1)  # noqa: E731
        out[f"{W}/{inflight_max}"] = {"topics_per_s": round(a.count * W / el), "add_us": med(t_add),
                                      "flush_us": med(t_flush), "collect_us": med(t_coll),
                                      "flush_to_collected_us": med(lat)}
        print(W, inflight_max, out[f"{W}/{inflight_max}"], flush=True)
print(json.dumps(out))
