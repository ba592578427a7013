"""PCIe rates of this box for the host-in/host-out path: H2D of a cfg3 batch's size from pinned
memory, D2H of its result size, both at once, and the engine's pipelined host path with each
result-copy mode (kernel PCIe writes vs hipMemcpyAsync)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


dev = torch.device("cuda", 0)
up = torch.empty(82 << 20, dtype=torch.uint8).pin_memory()
dn = torch.empty(28 << 20, dtype=torch.uint8).pin_memory()
d_up = torch.empty(82 << 20, dtype=torch.uint8, device=dev)
d_dn = torch.empty(28 << 20, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
out = {"h2d_GBs": rate(lambda: d_up.copy_(up, non_blocking=True), up.numel()),
       "d2h_GBs": rate(lambda: dn.copy_(d_dn, non_blocking=True), dn.numel())}


def both():
    with torch.cuda.stream(s1):
        d_up.copy_(up, non_blocking=True)
    with torch.cuda.stream(s2):
        dn.copy_(d_dn, non_blocking=True)


out["both_GBs"] = rate(both, up.numel() + dn.numel())
if len(sys.argv) > 1:
    import workloads
    from emqx_amd import Engine
    w = workloads.generate(3, 10_000_000, 2_000_000)
    eng = Engine()
    eng.route_ref_many(w.fbytes, w.foff)
    wi = np.nonzero(w.fwild)[0]
    eng.trie_insert_many(w.fbytes, w.foff)
    eng.commit()
    hb = eng.pinned(len(w.tbytes))
    hb[:] = w.tbytes
    ho = eng.pinned(w.nt + 1, np.uint32)
    ho[:] = w.toff
    for mode in (1, 0):
        eng.tune("host_out", mode)
        for inflight in (2, 3):
            pend = []
            k = 12
            for it in range(k + 3):
                if it == 3:
                    t0 = time.perf_counter()
                pend.append(eng.match_batch_submit(hb, ho))
                if len(pend) >= inflight:
                    eng.match_batch_wait(pend.pop(0), copy=False)
            while pend:
                eng.match_batch_wait(pend.pop(0), copy=False)
            dt = (time.perf_counter() - t0) / (k + 3 - 3)
            out[f"e2e_mode{mode}_inflight{inflight}_Gtopics"] = w.nt / dt / 1e9
print(json.dumps(out))
