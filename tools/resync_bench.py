"""The mirror's full resync at scale: emqx_trie_gpu_sync's resync/1 over the
C-ABI calls the NIF makes, on a cfg3 route table of 10M routes, with 1 and with 8 engines (the
NIF resource's one-engine-per-GPU replicas; here all on this box's GPU).

Per engine count:
  * first sync  -- sync_begin, every topic in chunks of 64k per call (emqxgm_route_set_many: the
    NIF's route_set_many/3), sync_end, commit (the first full build);
  * resync      -- the same over the unchanged table (the periodic / repair pass): no change,
    so the commit has nothing to do;
  * a hook during the resync -- a single subscribe committed with EMQXGM_SET_COMMIT from another
    thread (emqx_trie_gpu:route_changed/1 on the writing node) while the chunks run: its
    latency (it waits for at most one chunk's writer-lock hold), versus an event queued in the
    mirror process's mailbox, which is handled after the whole resync (its lag = the resync).

    python tools/resync_bench.py [--filters 10000000] [--engines 1,8] [--out file.json]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def chunks(w, size):
    for a in range(0, w.nf, size):
        b = min(w.nf, a + size)
        off = (w.foff[a:b + 1] - w.foff[a]).astype(np.uint64)
        yield w.fbytes[int(w.foff[a]):int(w.foff[b])], off


def resync(engs, w, size, pool=None):
    gens = [e.sync_begin() for e in engs]
    t0 = time.perf_counter()
    n = 0
    last = t0
    for buf, off in chunks(w, size):
        if pool is None:
            for e in engs:  # every engine in turn, per chunk
                e.route_set_many(buf, off, True)
        else:  # one thread per engine, as the NIF's on_engines (ctypes drops the GIL)
            list(pool.map(lambda e: e.route_set_many(buf, off, True), engs))
        n += 1
        if time.perf_counter() - last > 30:
            last = time.perf_counter()
            print(f"  ... {n} chunks", flush=True)
    t_chunks = time.perf_counter() - t0
    removed = [e.sync_end(g) for e, g in zip(engs, gens)]
    t1 = time.perf_counter()
    if pool is None:
        for e in engs:
            e.commit()
    else:
        list(pool.map(lambda e: e.commit(), engs))
    print("  ... committed", flush=True)
    return {"chunks": n, "set_s": round(t_chunks, 3), "sync_end_s": round(t1 - t0 - t_chunks, 3),
            "commit_s": round(time.perf_counter() - t1, 3), "removed": int(removed[0]),
            "total_s": round(time.perf_counter() - t0, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=10_000_000)
    ap.add_argument("--engines", default="1,8,8p",
                    help="engine counts; a 'p' suffix: one thread per engine per chunk")
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import workloads
    from emqx_amd import Engine
    w = workloads.generate(3, args.filters, 1)
    out = {"workload": f"cfg3 route table: {w.nf} routes (every filter a wildcard: trie + route key)",
           "chunk_topics": args.chunk, "runs": {}}
    from concurrent.futures import ThreadPoolExecutor
    for spec in args.engines.split(","):
        k = int(spec.rstrip("p"))
        pool = ThreadPoolExecutor(k) if spec.endswith("p") and k > 1 else None
        engs = [Engine() for _ in range(k)]
        r = {"first_sync": resync(engs, w, args.chunk, pool)}
        print(f"[{spec} engines] first sync {r['first_sync']}", flush=True)
        r["resync"] = resync(engs, w, args.chunk, pool)
        print(f"[{spec} engines] resync {r['resync']}", flush=True)
        # a hook on the writing node while the resync runs
        lat, stop = [], threading.Event()

        def hook():
            i = 0
            while not stop.is_set():
                f = b"site/hook/device/%d/+" % i
                t0 = time.perf_counter()
                for e in engs:
                    e.route_set_batch([(f, True)])
                lat.append(time.perf_counter() - t0)
                i += 1
                time.sleep(0.002)
        th = threading.Thread(target=hook)
        th.start()
        r["resync_with_hooks"] = resync(engs, w, args.chunk, pool)
        stop.set()
        th.join()
        v = np.asarray(lat) * 1e3
        r["hook_during_resync_ms"] = {"n": int(v.size), "p50": round(float(np.median(v)), 3),
                                      "p99": round(float(np.percentile(v, 99)), 3),
                                      "max": round(float(v.max()), 3)}
        r["queued_event_lag_s"] = r["resync_with_hooks"]["total_s"]
        print(f"[{spec} engines] hooks during resync {r['hook_during_resync_ms']}", flush=True)
        out["runs"][spec] = r
        if pool is not None:
            pool.shutdown()
        for e in engs:
            e.close()
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
