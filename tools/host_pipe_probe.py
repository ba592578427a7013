"""Where the host-in/host-out pipes spend their time on a config: per-call submit / wait times
with 1..HOST_PIPES batches in flight, and the engine's rerun count (diagnostic)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import workloads  # noqa: E402
from emqx_amd import Engine  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.cuda.set_device(0)  # torch's HIP context before the engine's, as bench.py does
w = workloads.generate(cfg)
eng = Engine()
eng.route_ref_many(w.fbytes, w.foff)
wi = np.nonzero(w.fwild)[0]
lens = (w.foff[wi + 1] - w.foff[wi]).astype(np.int64)
off = np.zeros(len(wi) + 1, np.uint64)
np.cumsum(lens, out=off[1:])
starts = w.foff[wi].astype(np.int64)
pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
eng.trie_insert_many(w.fbytes[pos], off)
eng.commit()
hb = eng.pinned(len(w.tbytes))
hb[:] = w.tbytes
ho = eng.pinned(w.nt + 1, np.uint32)
ho[:] = w.toff
out = {"cfg": cfg, "topics": w.nt}
if len(sys.argv) > 2 and sys.argv[2] == "bench-like":
    # what bench.py does before its host-path timing: census passes, device pipes, profiling
    tb = torch.from_numpy(w.tbytes).cuda()
    to = torch.from_numpy(w.toff.view(np.int32)).cuda()
    torch.cuda.synchronize()
    eng.tune("leaf_prune", 0)
    eng.walk_census(tb.data_ptr(), to.data_ptr(), w.nt, int(w.toff[-1]))
    eng.tune("leaf_prune", 1)
    eng.walk_census(tb.data_ptr(), to.data_ptr(), w.nt, int(w.toff[-1]))
    pend = []
    for _ in range(8):
        pend.append(eng.match_device_submit(tb.data_ptr(), to.data_ptr(), w.nt, int(w.toff[-1])))
        if len(pend) == eng.PIPES:
            eng.match_device_wait(pend.pop(0))
    while pend:
        eng.match_device_wait(pend.pop(0))
    eng.set_profiling(True)
    for _ in range(3):
        eng.match_device(tb.data_ptr(), to.data_ptr(), w.nt, int(w.toff[-1]))
    eng.set_profiling(False)
    out["mode"] = "bench-like"
for inflight in range(1, eng.HOST_PIPES + 1):
    pend, ts, tw = [], [], []
    r0 = eng.stats()["reruns"]
    t0 = None
    for it in range(24):
        if it == 4:
            t0 = time.perf_counter()
        a = time.perf_counter()
        pend.append(eng.match_batch_submit(hb, ho))
        b = time.perf_counter()
        if it >= 4:
            ts.append(b - a)
        if len(pend) >= inflight:
            a = time.perf_counter()
            eng.match_batch_wait(pend.pop(0), copy=False)
            if it >= 4:
                tw.append(time.perf_counter() - a)
    while pend:
        eng.match_batch_wait(pend.pop(0), copy=False)
    dt = (time.perf_counter() - t0) / 20
    out[f"inflight{inflight}"] = {"ms_per_batch": round(dt * 1e3, 3), "Mtopics_s": round(w.nt / dt / 1e6, 1),
                                  "submit_ms_med": round(float(np.median(ts)) * 1e3, 3),
                                  "wait_ms_med": round(float(np.median(tw)) * 1e3, 3),
                                  "reruns": eng.stats()["reruns"] - r0}
a = time.perf_counter()
for _ in range(10):
    eng.match_packed(hb, ho, copy=False)
out["match_batch_ms"] = round((time.perf_counter() - a) / 10 * 1e3, 3)
print(json.dumps(out))
