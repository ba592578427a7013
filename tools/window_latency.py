"""One window's latency with nothing else in flight (diagnostic for VERDICT r03 item 5): per
window size, the wall time of emqxgm_match_batch_submit_filters + _wait_filters (the concurrent
entry's per-window work: H2D, the pass, the filter-byte gather, one D2H) and of
emqxgm_match_device (the device pass alone, one stream synchronisation), p50 / p10 / p90 over
`--reps` windows of cfg3 topics.

    python tools/window_latency.py [--filters 10000000] [--sizes 1,16,256,4096,16384,65536]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--filters", type=int, default=10_000_000)
ap.add_argument("--sizes", default="1,16,256,4096,16384,65536")
ap.add_argument("--reps", type=int, default=60)
ap.add_argument("--tune", action="append", default=[])
a = ap.parse_args()

import torch  # noqa: E402

import emqx_amd  # noqa: E402
from emqx_amd import engine as E  # noqa: E402
import workloads  # noqa: E402

sizes = [int(x) for x in a.sizes.replace(":", ",").split(",")]  # (":" for tools/job.sh)
w = workloads.generate(3, a.filters, max(sizes) * 4)
eng = emqx_amd.Engine()
for kv in a.tune:
    k, v = kv.split("=")
    eng.tune(k, int(v))
eng.route_ref_many(w.fbytes, w.foff)
eng.trie_insert_many(w.fbytes, w.foff)
eng.commit()
lib, h = eng._lib, eng._h


def pct(x):
    x = np.asarray(x) / 1e3
    return {"p10": round(float(np.percentile(x, 10)), 1), "p50": round(float(np.percentile(x, 50)), 1),
            "p90": round(float(np.percentile(x, 90)), 1)}


out = {"env": {k: os.environ.get(k) for k in ("HSA_ENABLE_SDMA", "GPU_MAX_HW_QUEUES")},
       "filters": a.filters, "tune": a.tune, "us": {}}
for n in sizes:
    res = {}
    for rot in range(2):  # first pass over the sizes warms the pipes' buffers up
        toff = w.toff[rot * n: rot * n + n + 1].astype(np.int64)
        lo, hi = int(toff[0]), int(toff[-1])
        buf = eng.pinned(max(1, hi - lo))
        buf[:hi - lo] = w.tbytes[lo:hi]
        off = eng.pinned(n + 1, np.uint32)
        off[:] = (toff - lo).astype(np.uint32)
        host = []
        for _ in range(a.reps):
            t = C.c_uint64(0)
            o = E._BatchOut()
            fo, fb = E._U32P(), E._U8P()
            t0 = time.perf_counter_ns()
            rc = lib.emqxgm_match_batch_submit_filters(h, E._ptr(buf), E._ptr(off), n, C.byref(t))
            t1 = time.perf_counter_ns()
            rc = rc or lib.emqxgm_match_batch_wait_filters(h, t.value, C.byref(o), C.byref(fo), C.byref(fb))
            t2 = time.perf_counter_ns()
            assert rc == 0, rc
            host.append((t2 - t0, t1 - t0))
        db = torch.from_numpy(np.array(buf[:max(1, hi - lo)])).cuda()
        do = torch.from_numpy(np.array(off).view(np.int32)).cuda()
        torch.cuda.synchronize()
        dev = []
        for _ in range(a.reps):
            t0 = time.perf_counter_ns()
            eng.match_device(db.data_ptr(), do.data_ptr(), n, hi - lo)
            dev.append(time.perf_counter_ns() - t0)
        res = {"host_in_out": pct([x[0] for x in host]), "submit_call": pct([x[1] for x in host]),
               "device_pass": pct(dev)}
    out["us"][str(n)] = res
    print(n, res, flush=True)
print(json.dumps(out))
