"""Benchmark: published topics matched per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): 10M wildcard filters of the IoT tree
``site/+/device/+/#`` family, every GPU matching batches of ``site/{s}/device/{d}/{m}/{k}``
topics.  One step = one full match pass over one batch already resident in HBM: tokenise +
hash, route-key probe (when the index has plain route keys), trie walk, byte re-check of the
pairs whose filters hold a hashed (> 7-byte) word (cfg3 has none: its words are all <= 7 bytes,
whose level tokens are injective, so no pair needs one and k_verify does not launch), CSR build.
Steps rotate over --batches distinct batches (different topic seeds, default 3), so no pass
re-matches the batch the previous pass just warmed the caches with.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cfg 3] [--shard topics|filters]

N>1 is launched by the driver with torch.distributed.run (one rank per GPU).  ``--shard topics``
(default) = every GPU holds the whole 10M-filter index and matches its own batch (weak scaling,
no collective on the data path); ``--shard filters`` = the north-star layout (filters split by
hash, batch broadcast + results gathered with RCCL every step).

Rank 0 prints one JSON line.  ``roofline`` is for the step's dominant kernel (HIP-event timed,
one pass at a time): for the trie walk / exact probe, random 64-B line accesses per second
against the measured random-gather ceiling, with SURVEY 8d algorithmic bytes and PMC counter
bytes beside it as fractions of the 8 TB/s HBM peak (DESIGN.md "Roofline").
``cpu_baseline`` is the C++ restatement of the reference's emqx_trie match (oracle/ref_trie.cpp)
timed on this host's cores on a bounded sample of the same topics (rank 0, N=1 only).
``subscribe`` (N=1): the writing node's subscribe path -- emqxgm_route_set_batch with
EMQXGM_SET_COMMIT, then a one-topic match that must see it -- idle and during a background
rebuild of the whole index (p50 / p99 / max).  ``nif_concurrent`` (N=1): the concurrent publish
entry under T publisher threads; points ``..._R<ns>_D<k>`` model the NIF's per-call report as
<ns> of work, reported by k threads.  N>1: ``config.filter_sharded`` holds the filter-sharded
layout's step, or the error / timeout its watchdog recorded.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-s", type=float, default=0.5,
                    help="untimed steps for this long before the warmup steps: the GPU's clocks "
                         "ramp over ~100 ms of load (r04: 20 timed steps after 5 warmup steps "
                         "ran 6%% slower than after 300), 0 = none")
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=None, help="topics per GPU batch")
    ap.add_argument("--batches", type=int, default=3,
                    help="distinct topic batches (topic seeds) rotated through warm-up and the "
                         "timed region")
    ap.add_argument("--shard", choices=["topics", "filters"], default="topics")
    ap.add_argument("--wg-per-cu", type=int, default=0)
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="emqxgm_tune before the index is built (A/B runs), e.g. fat_buckets=0")
    ap.add_argument("--filter-shard", action="store_true",
                    help="(default since r05) N>1: the filter-sharded layout is measured beside "
                         "the replicas, after their figure is final, under a watchdog")
    ap.add_argument("--no-filter-shard", action="store_true",
                    help="N>1: leave the filter-sharded layout out")
    ap.add_argument("--filter-shard-timeout", type=float, default=120.0,
                    help="N>1: seconds the filter-sharded run may take before the watchdog prints "
                         "the line with config.filter_sharded = {error: timeout} and ends the rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-in/host-out timing")
    ap.add_argument("--no-subscribe", action="store_true",
                    help="skip the subscribe-to-visible latency (idle and during a background rebuild)")
    ap.add_argument("--windows", default="16384,65536,262144,1048576",
                    help="NIF batcher window sizes (topics) for the operating-point sweep "
                         "('' = skip); rank 0, N=1, with the host-in/host-out timing")
    ap.add_argument("--nif", default="16:16384,16:65536,64:16384,64:65536,16:16384:1024,16:65536:4096,"
                                     "16:65536:0:500:1,16:65536:0:500:8",
                    help="concurrent publish entry load (threads:window[:processes per thread"
                         "[:ns of work per reported call:report threads]], '' = skip): publisher "
                         "threads each calling emqxgm_async_match one topic at a time; processes "
                         "default (0) to (host pipes + 1) windows outstanding; rank 0, N=1")
    ap.add_argument("--only-nif", action="store_true",
                    help="build the index and run only the concurrent-entry load (no timed steps)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=0,
                    help="device passes in flight (default: EMQXGM_PIPES)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one pass at a time (emqxgm_match_device) instead of two in flight")
    ap.add_argument("--no-route-keys", action="store_true",
                    help="experiment: trie only (no exact route-key table)")
    ap.add_argument("--topic-order", choices=["as-is", "xcd", "sorted"], default="as-is",
                    help="experiment: permute the batch (outside the timed region) so that topics "
                         "of one first-two-level prefix group share an XCD shard, or fully sorted")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EMQXGM_DIST_BACKEND=gloo rehearses the N>1 control flow with several ranks sharing the
    # GPUs of a smaller box (RCCL refuses two ranks on one device); production is RCCL ("nccl")
    if world > 1:
        dist.init_process_group(os.environ.get("EMQXGM_DIST_BACKEND", "nccl"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import workloads
    from emqx_amd import Engine
    from emqx_amd import dist as D

    nf_default, nt_default, sf, st = workloads.DEFAULTS[args.cfg]
    if args.cfg == 3:
        # batches of 1M-8M topics; the headline takes 4M (the middle of the range:
        # profiles/r02/batch_sweep.json has 1M / 2M / 4M / 8M on one box)
        nt_default = 4_000_000
    nf = args.filters or nf_default
    nt = args.topics or nt_default

    t0 = time.time()
    seed_t = st + (1000 * rank if args.shard == "topics" else 0)
    w = workloads.generate(args.cfg, nf, nt, sf, seed_t)
    # further batches: the same distribution under other topic seeds (no filters drawn again)
    nb = max(1, args.batches)
    extra = [workloads.generate(args.cfg, nf, nt, sf, seed_t + 7919 * b, topics_only=True)
             for b in range(1, nb)]
    log(f"[rank {rank}] generated {w.nf} filters, {nb} x {w.nt} topics in {time.time() - t0:.1f}s")

    # the CPU baseline's index (reference-style ordered set) builds in the background while the
    # GPU is measured; ctypes releases the GIL, so the two do not interleave on the host
    cpu_job = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_job = _CpuIndexJob(w, args.cfg)

    # ---- index ----
    t0 = time.time()
    eng, _ = _build_engine(Engine, w, np.arange(w.nf), args, local)
    est = eng.stats()
    log(f"[rank {rank}] index: {est['n_trie_filters']} trie filters, {est['n_route_keys']} route "
        f"keys, {est['n_nodes']} nodes ({est['keyed_nodes']} token-keyed), "
        f"{est['device_bytes'] / 2**20:.0f} MiB in {time.time() - t0:.1f}s")

    if args.only_nif:
        out = _nif_concurrent(eng, w, args.nif)
        print(json.dumps({"config": f"cfg{args.cfg}: {w.nf} filters, {w.nt} topics",
                          "nif_concurrent": out}), flush=True)
        return

    if args.topic_order != "as-is":
        w = _reorder_topics(w, args.topic_order)
        extra = [_reorder_topics(x, args.topic_order) for x in extra]
    hosts = [w] + extra
    dbat = [(torch.from_numpy(x.tbytes).to(dev), torch.from_numpy(x.toff.view(np.int32)).to(dev),
             int(x.toff[-1])) for x in hosts]
    tb, to, nbytes = dbat[0]
    nbytes_mean = sum(b[2] for b in dbat) / nb
    torch.cuda.synchronize()

    # ---- diagnostic census passes (outside the timed region): S(t), slot loads, pairs, as the
    # mean over the batches ----
    # S(t) as SURVEY 8d defines it (every matched prefix state) comes from a census of the
    # unpruned walk; the production walk skips leaf-only children a deeper topic cannot match
    # (CF_LEAFP), so its own loads and iterations come from a second census
    eng.tune("leaf_prune", 0)
    census_full = _census_mean(eng, dbat, w.nt)
    eng.tune("leaf_prune", 1)
    census = _census_mean(eng, dbat, w.nt)
    census["states_visited"] = census["states"]
    census["states"] = census_full["states"]

    # pipelined steps (default): each step submits its batch and completes the previous one, so
    # two passes are in flight on the engine's two pipes (emqxgm_match_device_submit/_wait) and
    # one batch's walk tail overlaps the next batch's tokenizer and walk; drain() completes the
    # last one inside the timed region.  Every batch is matched in full either way.
    pipelined = not args.no_pipeline
    dev_inflight = min(args.inflight or eng.PIPES, eng.PIPES)
    pending = []
    turn = [0]

    def next_batch():
        b = dbat[turn[0] % nb]
        turn[0] += 1
        return b

    def step_sync():
        b_, o_, n_ = next_batch()
        return eng.match_device(b_.data_ptr(), o_.data_ptr(), w.nt, n_)

    def step_pipe():
        b_, o_, n_ = next_batch()
        pending.append(eng.match_device_submit(b_.data_ptr(), o_.data_ptr(), w.nt, n_))
        if len(pending) == dev_inflight:
            eng.match_device_wait(pending.pop(0))

    def drain():
        while pending:
            eng.match_device_wait(pending.pop(0))

    def step():
        return step_pipe() if pipelined else step_sync()

    # settle: untimed steps until the GPU runs at its loaded clocks (then the W warmup steps)
    settle_steps = 0
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_s:
        step()
        settle_steps += 1
    drain()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the same batches one pass at a time, reported beside `value` (outside the timed region)
    sync_ms = None
    if pipelined:
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step_sync()
        torch.cuda.synchronize()
        sync_ms = (time.perf_counter() - t1) / args.steps * 1e3
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # N > 1: the north-star layout beside the replicas, on the same ranks (filters split by hash,
    # rank 0's batch broadcast, results gathered and merged on rank 0 every step)
    fsh = None
    if world > 1 and args.shard == "filters":  # the north-star layout as the headline
        fsh = _filter_sharded_run(Engine, D, args, w, dbat, rank, world, dev, local)
    # kernel timing with HIP events on the engine's stream, in extra passes after the timed
    # region (the events themselves add gaps between launches), one pass at a time so that a
    # launch's duration is its own (not stretched by the other pipe's overlapping work)
    s0 = eng.stats()
    eng.set_profiling(True)
    for _ in range(max(3, min(args.steps, 10))):
        step() if not pipelined else step_sync()
    torch.cuda.synchronize()
    eng.set_profiling(False)
    s1 = eng.stats()

    launches = s1["tok_launches"] - s0["tok_launches"]
    walks = s1["walk_launches"] - s0["walk_launches"]
    tok_ms = (s1["tok_ms"] - s0["tok_ms"]) / max(1, launches)
    exact_ms = (s1["exact_ms"] - s0["exact_ms"]) / max(1, launches)
    walk_ms = (s1["walk_ms"] - s0["walk_ms"]) / max(1, walks)
    pipe_ms = (s1["total_ms"] - s0["total_ms"]) / max(1, launches)
    topics_total = w.nt * world
    compulsory = nbytes_mean + 4 * w.nt + 8 * census["pairs"]
    value = topics_total / (elapsed / args.steps)
    if args.shard == "filters" and fsh is not None:
        # the north-star layout as the headline: one batch per step over all GPUs
        topics_total, elapsed = w.nt, fsh["ms_per_step"] * 1e-3 * args.steps
        value = fsh["value"]
    pmc = _pmc(args.cfg, w.nt, nb)
    roofline = _roofline(w.nt, nbytes_mean, census, pmc, tok_ms, exact_ms, walk_ms, pipe_ms,
                         exact_table_bytes=32 * int(est.get("exact_slots", 0)))
    roofline["compulsory_bytes_per_batch"] = int(compulsory)
    roofline["compulsory_frac"] = round(compulsory / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4)

    cpu = _cpu_baseline(w, args, cpu_job) if cpu_job is not None else None
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        # host-resident batch in, host CSR out (PCIe both ways): reported beside `value`.  The
        # topics sit in pinned host memory, as a NIF batcher packs its window
        # (emqxgm_host_alloc); results are read in the handle's pinned buffers (no copy).
        hbat = []
        for x in hosts:
            hb = eng.pinned(len(x.tbytes))
            hb[:] = x.tbytes
            ho = eng.pinned(x.nt + 1, np.uint32)
            ho[:] = x.toff
            hbat.append((hb, ho))
        hturn = [0]

        def next_host():
            b = hbat[hturn[0] % nb]
            hturn[0] += 1
            return b
        eng.match_packed(*next_host(), copy=False)
        best = 1e9
        for _ in range(5):
            hb, ho = next_host()
            t1 = time.perf_counter()
            eng.match_packed(hb, ho, copy=False)
            best = min(best, time.perf_counter() - t1)
        # the NIF batcher's call: emqxgm_match_batch_submit/_wait with 2 and with 3 (all host
        # pipes) batches in flight: one batch's upload and pass overlap another's download.  Which
        # is faster depends on the batch (tools/host_pipe_probe.py,
        # profiles/r02/session2/host_pipe_probe_*.json: 2 for small batches); both are reported
        k = max(20, args.steps)
        pend = []
        for _ in range(2 * eng.HOST_PIPES):  # every pipe's scratch and buffers at their size
            pend.append(eng.match_batch_submit(*next_host()))
            if len(pend) == eng.HOST_PIPES:
                eng.match_batch_wait(pend.pop(0), copy=False)
        while pend:
            eng.match_batch_wait(pend.pop(0), copy=False)
        by_inflight = {}
        for inflight in (2, eng.HOST_PIPES):
            r0 = eng.stats()["reruns"]
            t1 = time.perf_counter()
            for _ in range(k):
                pend.append(eng.match_batch_submit(*next_host()))
                if len(pend) == inflight:
                    eng.match_batch_wait(pend.pop(0), copy=False)
            while pend:
                eng.match_batch_wait(pend.pop(0), copy=False)
            s_ = (time.perf_counter() - t1) / k
            by_inflight[inflight] = (s_, eng.stats()["reruns"] - r0)
        inflight = min(by_inflight, key=lambda x: by_inflight[x][0])
        pipe_s, reruns = by_inflight[inflight]
        e2e = {"value": round(w.nt / pipe_s, 1), "unit": "topics/s",
               "ms_per_batch": round(pipe_s * 1e3, 3), "batches_in_flight": inflight,
               "ms_per_batch_by_inflight": {str(i): round(v[0] * 1e3, 3) for i, v in by_inflight.items()},
               "reruns": int(reruns),
               "includes": "H2D topic bytes + offsets from pinned host memory, the device pass, "
                           "row pointers (u32) + filter ids + exact ids written into pinned host "
                           "memory (emqxgm_match_batch_submit/_wait)",
               "one_call_at_a_time": {"value": round(w.nt / best, 1),
                                      "ms_per_batch": round(best * 1e3, 3),
                                      "api": "emqxgm_match_batch (u64 row pointers)"}}

    # (before the load blocks: measured in the wake of their publisher and layer threads, which
    # spend the job's CPU quota, the idle hook took p50 51 us / max 1.0 ms in r06, against p50
    # 25 us / max 0.27 ms in tools/subscribe_probe.py's quiet process; the cgroup's throttling
    # during the block is recorded beside it)
    subscribe = None
    if rank == 0 and world == 1 and not args.no_subscribe:
        th0 = _cgroup_throttled()
        subscribe = _subscribe_latency(eng, w)
        th1 = _cgroup_throttled()
        if th0 and th1:
            subscribe["cgroup_throttled"] = {"periods": th1[0] - th0[0], "us": th1[1] - th0[1]}

    nif = None
    if rank == 0 and world == 1 and args.nif:
        nif = _nif_concurrent(eng, w, args.nif)

    windows = None
    if rank == 0 and world == 1 and not args.no_e2e and args.windows:
        from emqx_amd.engine import Batcher
        windows = _window_sweep(Batcher, eng, w, [int(x) for x in args.windows.split(",")])

    # the low-load crossover: one publish answered by the device at idle (a
    # window's timer and one pass) against the reference's walk on one core (emqx_trie_gpu's
    # adaptive_below_rate chooses between them by the measured rate)
    crossover = None
    if cpu and nif and cpu.get("one_thread") and "idle_T16_P1" in nif:
        one_us = cpu["one_thread"]["us_per_topic"]
        # one publisher on an idle broker, eager windows (the broker's default)
        ipt = next(k for k in ("idle_T1_P1_eager", "idle_T16_P1_eager", "idle_T16_P1") if k in nif)
        idle = nif[ipt]
        crossover = {
            "device_idle_p50_us": idle["latency_us_p50"], "device_idle_p99_us": idle["latency_us_p99"],
            "device_idle_point": ipt,
            "device_idle_p50_us_window_timer": nif.get("idle_T1_P1", nif["idle_T16_P1"])["latency_us_p50"],
            "reference_us_per_topic_one_core": one_us,
            "reference_capacity_topics_per_s": cpu["value"], "reference_cores": cpu["cores"],
            "reference_faster_at_idle": one_us < idle["latency_us_p50"],
            # the rate at which the reference path needs half of the cores the baseline used:
            # below it, answering on the publishers' cores costs little and is faster at idle
            "reference_half_cores_rate": round(0.5 * cpu["value"], 1),
            "note": ("broker.perf.gpu_match.adaptive_below_rate: publishes/s under which "
                     "emqx_trie_gpu answers on the publisher's core (0 = never)")}

    line = None
    if rank == 0:
        line = {
            "metric": ("published topics matched/sec at 10M filters" if args.cfg == 3
                       else f"published topics matched/sec (cfg{args.cfg})"),
            "value": round(value, 1),
            "unit": "topics/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if (args.shard == "topics" or world == 1) else "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"cfg{args.cfg}: {w.nf} filters "
                            + ("(IoT site/+/device/+/# tree)" if args.cfg == 3 else ""),
                "filters": int(w.nf), "topics_per_gpu_batch": int(w.nt),
                "distinct_batches": nb,
                "topic_seeds": [int(seed_t + 7919 * b) for b in range(nb)],
                "global_batch": int(topics_total), "parallelism":
                    (f"topic-replica x{world}" if args.shard == "topics" or world == 1
                     else f"filter-shard x{world}"),
                "pairs_per_batch": int(census["pairs"]),
                "trie_nodes": int(est["n_nodes"]), "token_keyed_nodes": int(est["keyed_nodes"]),
                "trie_states_per_batch": int(census["states"]),
                "walk_states_visited_per_batch": int(census["states_visited"]),
                "edge_slot_loads_unpruned_per_batch": int(census_full["slot_loads"]),
                "edge_slot_loads_per_batch": int(census["slot_loads"]),
                "walk_lane_iterations_per_batch": int(census["lane_iters"]),
                "walk_wave_iterations_per_batch": int(census["wave_iters"]),
                # the pruned walk's edge-bucket loads by probed level (literal / '+' probes)
                "edge_loads_by_level": {k: [int(x) for x in v[:max(1, _last_nz(v) + 1)]]
                                        for k, v in census["loads_by_level"].items()},
                "pipeline_ms_per_batch": round(pipe_ms, 4),
                "tune": args.tune,
                "settle": {"seconds": args.settle_s, "untimed_steps": settle_steps},
                "passes_in_flight": dev_inflight if pipelined else 1,
                "one_pass_at_a_time": (None if sync_ms is None else {
                    "value": round(topics_total / (sync_ms * 1e-3), 1), "ms_per_step": round(sync_ms, 4)}),
                "pairs_per_s": round(census["pairs"] * (topics_total / w.nt) / (elapsed / args.steps), 1),
                "filter_sharded": fsh,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "crossover": crossover,
            "end_to_end": e2e,
            "nif_windows": windows,
            "nif_concurrent": nif,
            "subscribe": subscribe,
        }
    if world > 1 and args.shard == "topics" and not args.no_filter_shard:
        # the north-star layout beside the replicas (filters split by hash, rank 0's
        # batch broadcast over RCCL, results gathered and merged on rank 0), measured after the
        # replicas' figure is final and under a watchdog: a hang or an error of its collectives
        # is recorded in config.filter_sharded instead of losing the line
        fsh = _guarded(lambda: _filter_sharded_run(Engine, D, args, w, dbat, rank, world, dev, local),
                       args.filter_shard_timeout, rank, line)
        if rank == 0:
            line["config"]["filter_sharded"] = fsh
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


WATCHDOG_EXIT = 3  # the rank's exit status when the N>1 watchdog ends it


def _guarded(run, timeout_s, rank, line):
    """run() under a watchdog thread: past timeout_s the rank ends itself (rank 0 first prints
    the line with the timeout recorded), so a collective that never completes cannot take the
    measurement with it; an exception is recorded as the result."""
    import threading
    done = threading.Event()

    def watchdog():
        if done.wait(timeout_s):
            return
        if rank == 0:
            line["config"]["filter_sharded"] = {"error": f"timeout after {timeout_s:.0f} s"}
            print(json.dumps(line), flush=True)
        log(f"[rank {rank}] filter-sharded run timed out after {timeout_s:.0f} s: exiting")
        sys.stdout.flush()
        sys.stderr.flush()
        # non-zero: a hung collective is a failure the driver must see, even with the line printed
        os._exit(WATCHDOG_EXIT)
    threading.Thread(target=watchdog, daemon=True).start()
    try:
        r = run()
    except Exception as e:  # a collective's error: recorded, the replicas' line stands
        log(f"[rank {rank}] filter-sharded run failed: {e!r}")
        r = {"error": repr(e)[:500]}
    done.set()
    return r


def _build_engine(Engine, w, idx, args, local):
    """An engine holding filters idx of w: every filter a route key (the route bag), the
    wildcard ones in the trie (emqx_router_utils.erl:34-39).  Returns (engine, gid_map): the
    global filter index of each engine-local id, from the ids the engine returned."""
    eng = Engine(device=local, walk_wg_per_cu=args.wg_per_cu)
    for kv in args.tune:
        k, v = kv.split("=", 1)
        eng.tune(k, int(v))
    fb, fo = _subset(w, idx)
    wild = w.fwild[idx].astype(bool)
    gid = np.full(max(1, len(idx)), 0xFFFFFFFF, np.uint32)
    if not args.no_route_keys:
        rid = eng.route_ref_many(fb, fo)
        gid = np.full(max(1, int(rid.max(initial=0)) + 1), 0xFFFFFFFF, np.uint32)
        gid[rid] = idx
    wsel = np.nonzero(wild)[0]
    wb, wo = _subset_packed(fb, fo, wsel)
    tid = eng.trie_insert_many(wb, wo)
    if tid.size and int(tid.max()) >= len(gid):
        g2 = np.full(int(tid.max()) + 1, 0xFFFFFFFF, np.uint32)
        g2[:len(gid)] = gid
        gid = g2
    gid[tid] = idx[wsel]
    eng.commit()
    return eng, gid


def _window_sweep(Batcher, eng, w, sizes):
    """The NIF's operating point (a batcher in front of emqx_trie:match/1): batch 0's
    topics streamed through an emqxgm_batcher of each window size -- packed into pinned windows
    (emqxgm_batcher_add_many), flushed, the oldest window collected whenever EMQXGM_HOST_PIPES
    are in flight (H2D, the device pass, results to pinned host memory, every pair's filter
    bytes copied into the window's arena).  Host-in/host-out topics/s and the flush -> collected
    latency per window (p50 / p99).  The driver loop is Python (one add_many / flush / collect
    call per window, ~tens of us), as a NIF batcher process would make the same three calls."""
    off = w.toff.astype(np.int64)
    out = {}
    # every size with EMQXGM_HOST_PIPES windows in flight, and the two smallest also with one
    # (the latency of a window that waits for no other)
    runs = [(W, eng.HOST_PIPES) for W in sizes] + [(W, 1) for W in sorted(sizes)[:2]]
    for W, depth in runs:
        W = min(W, w.nt)
        b = Batcher(eng, window_topics=W, window_bytes=64 * W)
        inflight, lat = [], []
        state = {"pos": 0, "done": 0}
        # the batch cut into windows once, outside the timed loop (a NIF packs each topic as
        # its caller's message arrives; here every window is one add_many into pinned memory)
        cuts = [(w.tbytes[off[i]:off[min(i + W, w.nt)]],
                 (off[i:min(i + W, w.nt) + 1] - off[i]).astype(np.uint32), i)
                for i in range(0, w.nt, W)]

        def collect():
            n_, _, _, ns = b.collect(inflight.pop(0), materialize=False)
            lat.append(ns)
            state["done"] += n_

        def run(total):
            added = 0
            while added < total:
                buf, rel, i = cuts[state["pos"] % len(cuts)]
                k = b.add_many(buf, rel, i)
                state["pos"] += 1
                added += k
                if len(inflight) == depth:
                    collect()
                inflight.append(b.flush())
            while inflight:
                collect()
        run(min(4 * W, 1 << 21))  # warm-up: pinned buffers and the engine's scratch at size
        lat.clear()
        state["done"] = 0
        total = max(20 * W, 2_000_000)
        t0 = time.perf_counter()
        run(total)
        el = time.perf_counter() - t0
        b.close()
        la = np.array(lat, np.float64) / 1e3
        key = str(W) if depth == eng.HOST_PIPES else f"{W}_inflight{depth}"
        out[key] = {"topics_per_s": round(state["done"] / el, 1), "windows": len(lat),
                    "latency_us_p50": round(float(np.percentile(la, 50)), 1),
                    "latency_us_p99": round(float(np.percentile(la, 99)), 1)}
    out["includes"] = ("topics packed into pinned windows, H2D, the device pass, row pointers + "
                       "filter ids + exact ids and every pair's filter bytes (gathered on the "
                       "device) in pinned host memory (emqxgm_batcher_*), 3 windows in flight "
                       "(*_inflight1: one); latency = flush -> collected; the caller's reading of "
                       "the result (the NIF's term building) is not included")
    return out


POINT_S = 1.0              # a load point's measured duration at least
NIF_MAX_CALLS = 160_000_000  # (4 B of latency per call kept for the percentiles)


def _nif_concurrent(eng, w, spec):
    """The NIF's concurrent entry under load: T publisher threads (BEAM
    schedulers) each run P publisher processes calling emqxgm_async_match one topic at a time --
    no caller-side batching -- and a call ends when the engine's completer thread reports it
    (tests/host_harness/async_load.cpp over the engine: emqxgm_async_*).  P = enough calls for
    the pipes' windows to fill by size (window x (EMQXGM_HOST_PIPES + 1) / T); topics/s and the
    call -> result latency per call (p50 / p99).  Plus an idle-broker point: one call in flight
    per thread, windows flushed by the window_us timer."""
    from workloads import publishers
    tb = np.ascontiguousarray(w.tbytes)
    to = w.toff.astype(np.uint64)
    out = {}
    runs = [tuple(int(x) for x in item.split(":")) for item in spec.split(",") if item]
    for run in runs:
        T, W = run[0], run[1]
        # closed loop: calls outstanding = T x procs, so by Little's law the latency is that over
        # the rate -- (pipes + 1) windows' worth saturates the pipes, one window's worth shows
        # the latency at a lighter load
        procs = run[2] if len(run) > 2 and run[2] else max(1, -(-W * (eng.HOST_PIPES + 1) // T))
        # T:W[:P[:R:D]]: R ns of work per reported call standing for the NIF's terms + enif_send,
        # reported by D threads (emqxgm_async_cfg.deliver_threads)
        rns, dth = (run[3], run[4]) if len(run) > 4 else (0, 0)
        key = f"T{T}_W{W}" + (f"_P{procs}" if len(run) > 2 and run[2] else "") + \
            (f"_R{rns}_D{dth}" if len(run) > 4 else "")
        calls = max(2 * procs, min(8_000_000, 100 * W) // T)
        publishers.run([eng], tb, to, T, procs, min(calls, 4 * procs), W, deliver_threads=dth,
                       report_ns=rns)  # warm-up
        # the measured point lasts at least POINT_S (its p99.9 and max are then
        # a steady-state tail, not ~100 windows'): calls sized from a pilot run's rate
        pilot = publishers.run([eng], tb, to, T, procs, calls, W, deliver_threads=dth, report_ns=rns)
        rate = pilot["calls"] / max(pilot["seconds"], 1e-6)
        calls = max(calls, min(int(rate * POINT_S * 1.1) // T + 1, NIF_MAX_CALLS // T))
        th0, s0 = _cgroup_throttled(), eng.stats()
        r = publishers.run([eng], tb, to, T, procs, calls, W, deliver_threads=dth, report_ns=rns)
        th1, s1 = _cgroup_throttled(), eng.stats()
        out[key] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        out[key]["processes_per_thread"] = procs
        # stalls inside the engine during the point: buffer reallocations (a hipFree syncs the
        # device), windows whose filter block outgrew its estimate, passes redone
        out[key]["engine"] = {k: s1[k] - s0[k] for k in ("buffer_grows", "sync_gathers", "reruns")}
        if th0 and th1:  # the job's CPU quota stopping every thread (publishers + the layer's)
            out[key]["cgroup_throttled"] = {"periods": th1[0] - th0[0], "us": th1[1] - th0[1]}
    if runs:
        # the idle point: one call in flight per thread, so ~1 / latency calls per second each;
        # with EMQXGM_ASYNC_EAGER (the broker's default since r06: a window goes out as soon as a
        # pipe is free) and without it (window_us after a window's first call)
        r = publishers.run([eng], tb, to, 16, 1, 20000, 65536)
        out["idle_T16_P1"] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        r = publishers.run([eng], tb, to, 16, 1, 20000, 65536, eager=True)
        out["idle_T16_P1_eager"] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        # a truly idle broker: one publisher, one call at a time (16 such callers are a light load,
        # where eager windows trade the timer's batching for more, smaller passes)
        for eager in (False, True):
            r = publishers.run([eng], tb, to, 1, 1, 5000, 65536, eager=eager)
            out["idle_T1_P1" + ("_eager" if eager else "")] = {
                k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
        # a loaded point with it: windows still grow while every pipe is busy
        T, W = 16, 16384
        procs = max(1, -(-W * (eng.HOST_PIPES + 1) // T))
        calls = max(2 * procs, min(int(out.get(f"T{T}_W{W}", {}).get("calls", 0)) // T, NIF_MAX_CALLS // T))
        if calls > 2 * procs:
            publishers.run([eng], tb, to, T, procs, 4 * procs, W, eager=True)  # warm-up
            r = publishers.run([eng], tb, to, T, procs, calls, W, eager=True)
            out[f"T{T}_W{W}_eager"] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}
    out["includes"] = ("T threads x P processes, one emqxgm_async_match call per topic (the NIF's "
                       "match_async/3), windows filled lock-free and flushed when full or "
                       "window_us (50) after their first call, the window read from pinned memory "
                       "(copy-through up to 64k topics, else H2D), the device pass, every pair's "
                       "filter bytes to pinned memory, the callback reporting each call; "
                       "latency = call -> its report (the NIF's term building and enif_send "
                       "excluded)")
    return out


def _subscribe_latency(eng, w, n_idle=400, max_build_s=30.0):
    """The writing node's subscribe path (emqxgm_route_set_batch with EMQXGM_SET_COMMIT: the hook
    after emqx_router:do_add_route/2, emqx_router.erl:124-138): the time from the call to the
    new filter being visible to every later match, on the bench's index -- idle, and while a full
    rebuild of the whole index runs in the background (emqxgm_tune "rebuild").  Each subscribe is
    followed by a one-topic match that must contain it (the check is not timed); everything is
    unsubscribed again afterwards."""
    def pcts(v):
        v = np.asarray(v) * 1e6
        return {"n": int(v.size), "p50_us": round(float(np.percentile(v, 50)), 1),
                "p99_us": round(float(np.percentile(v, 99)), 1),
                "max_us": round(float(v.max()), 1), "max_at": int(v.argmax())} if v.size else {"n": 0}

    base = w.topic(0).split(b"/")

    def filt(k):  # a new wildcard filter under an existing prefix: site/S/device/D/bench{k}/+
        return b"/".join(base[:4] + [b"bench%d" % k, b"+"])

    def topic(k):
        return b"/".join(base[:4] + [b"bench%d" % k, b"7"])

    def sub(k, present, lat):
        t0 = time.perf_counter()
        eng.route_set_batch([(filt(k), present)])
        lat.append(time.perf_counter() - t0)
        row = eng.match([topic(k)]).row(0)
        got = {eng.filter_bytes(int(f)) for f in row}
        assert (filt(k) in got) == present, ("subscribe not visible", k, present)

    idle = []
    for k in range(n_idle):
        sub(k, True, idle)
    for k in range(n_idle):
        sub(k, False, [])
    s0 = eng.stats()
    during, build = [], None
    try:
        eng.tune("rebuild", 1)
    except Exception as e:  # (bg builds off for this index size)
        return {"idle": pcts(idle), "during_rebuild": None, "note": str(e)}
    t0 = time.perf_counter()
    k = n_idle
    while eng.stats()["full_commits"] == s0["full_commits"] and time.perf_counter() - t0 < max_build_s:
        if len(during) < 4000:
            sub(k, True, during)
            k += 1
        time.sleep(0.001)  # a subscribe every ~1 ms while the build runs
    build = time.perf_counter() - t0
    s1 = eng.stats()
    for j in range(n_idle, k):
        sub(j, False, [])
    return {"api": "emqxgm_route_set_batch(.., EMQXGM_SET_COMMIT) then a one-topic match sees it",
            "idle": pcts(idle),
            "during_rebuild": dict(pcts(during), rebuild_s=round(build, 2),
                                   build_ms=round(s1["last_build_ms"], 1),
                                   waited_for_build=int(s1["bg_waits"] - s0["bg_waits"]),
                                   catchup_changes=int(s1["catchup_changes"]))}


def _census_mean(eng, dbat, nt):
    """walk_census over every batch, as the mean per batch."""
    acc = None
    for b_, o_, n_ in dbat:
        c = eng.walk_census(b_.data_ptr(), o_.data_ptr(), nt, n_)
        if acc is None:
            acc = c
            continue
        for k, v in c.items():
            if isinstance(v, dict):
                for kk, vv in v.items():
                    acc[k][kk] = [a + b for a, b in zip(acc[k][kk], vv)]
            else:
                acc[k] += v
    k = len(dbat)
    return {key: ({kk: [x / k for x in vv] for kk, vv in v.items()} if isinstance(v, dict) else v / k)
            for key, v in acc.items()}


def _filter_sharded_run(Engine, D, args, w, dbat, rank, world, dev, local):
    """The north-star layout on these ranks: this rank's filter shard in an engine of its own,
    rank 0's batch broadcast, matched on every shard, gathered and merged on rank 0 (dist.py
    ShardedMatcher).  Same steps / warmup as the replica measurement; max over ranks."""
    t0 = time.time()
    mine = np.nonzero(D.filter_shards(w.fbytes, w.foff, world) == rank)[0]
    seng, gid = _build_engine(Engine, w, mine, args, local)
    log(f"[rank {rank}] filter shard: {len(mine)} filters in {time.time() - t0:.1f}s")
    sm = D.ShardedMatcher(seng, torch.from_numpy(gid.view(np.int32)).to(dev), dev, n_global=w.nf)
    # the root's batch shapes, once, outside the timed region (every rank drew its own batches
    # for the replica measurement)
    cdev = "cpu" if D._comm_on_cpu() else dev
    shp = torch.tensor([b[2] for b in dbat], dtype=torch.int64, device=cdev)
    dist.broadcast(shp, 0)
    root_nb = [int(x) for x in shp.tolist()]

    def batches(k0, k):
        return [((dbat[(k0 + i) % len(dbat)][0], dbat[(k0 + i) % len(dbat)][1]) if rank == 0
                 else (None, None)) for i in range(k)]

    def shapes(k0, k):
        return [(root_nb[(k0 + i) % len(dbat)], w.nt) for i in range(k)]
    for _ in sm.run(batches(0, args.warmup), shapes(0, args.warmup)):
        pass
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    pairs = 0
    for m in sm.run(batches(args.warmup, args.steps), shapes(args.warmup, args.steps)):
        if m is not None:
            pairs = int(m.filter_id.numel())
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    step_s = float(el.item()) / args.steps
    to_root = torch.tensor([sm.bytes_to_root], dtype=torch.float64, device=dev)
    dist.all_reduce(to_root, op=dist.ReduceOp.MAX)
    seng.close()
    nb = float(np.mean(root_nb))
    dense = (8 * w.nt + 4) * (world - 1) + 4 * pairs * (world - 1) / world
    return {"value": round(w.nt / step_s, 1), "unit": "topics/s", "ms_per_step": round(step_s * 1e3, 4),
            "scaling": "strong", "parallelism": f"filter-shard x{world}",
            "filters_per_rank": int(len(mine)), "topics_per_step": int(w.nt),
            "pairs_per_batch": pairs,
            "bytes_broadcast_per_step": int((nb + 4 * (w.nt + 1)) * (world - 1)),
            "bytes_to_root_per_step": int(to_root.item()),
            "bytes_to_root_dense_r02_estimate": int(dense),
            "step": "rank 0's batch broadcast (RCCL; batch k+1 while the engines walk batch k), "
                    "matched on each shard, results in the compact wire form (2-bit or u8 counts, "
                    "24- or 32-bit global ids, sparse exact hits) to rank 0 by grouped "
                    "send/recv, merged by emqxgm_merge_wire"}


def _last_nz(v):
    return max([i for i, x in enumerate(v) if x] or [0])


def _subset(w, idx):
    return _subset_packed(w.fbytes, w.foff, idx)


def _subset_packed(fbytes, foff, idx):
    idx = np.asarray(idx, dtype=np.int64)
    if len(idx) == len(foff) - 1 and (len(idx) == 0 or (idx[0] == 0 and idx[-1] == len(idx) - 1)):
        return fbytes, foff
    lens = (foff[idx + 1] - foff[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    starts = foff[idx].astype(np.int64)
    pos = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64), lens) \
        + np.arange(int(lens.sum()), dtype=np.int64)
    return fbytes[pos], off


def _reorder_topics(w, how):
    """Experiment only: a permutation of the batch (same topics, other order)."""
    import dataclasses
    topics = [w.topic(i) for i in range(w.nt)]
    if how == "sorted":
        order = sorted(range(w.nt), key=lambda i: topics[i])
    else:  # group by a hash of the first two levels into 8 shards, random order inside
        import zlib
        rng = np.random.default_rng(7)
        grp = np.array([zlib.crc32(b"/".join(t.split(b"/")[:2])) % 8 for t in topics])
        order = np.concatenate([rng.permutation(np.nonzero(grp == g)[0]) for g in range(8)])
    lens = np.array([len(topics[i]) for i in order], np.uint32)
    off = np.zeros(w.nt + 1, np.uint32)
    np.cumsum(lens, out=off[1:])
    tbytes = np.frombuffer(b"".join(topics[i] for i in order), np.uint8).copy()
    return dataclasses.replace(w, tbytes=tbytes, toff=off)


# Random 64-B line accesses per second the memory system sustains for a table beyond the L2
# (tools/gather_bench.hip, profiles/r01/gather_sizes.txt: 2 GiB table, 64-B lines, 52.1-53.0 G/s;
# 64-192 MiB tables 53-58 G/s) and for an L2-resident one (8 MiB: 99-109 G/s).
RANDOM_LINES_PEAK = 53.0e9
RANDOM_LINES_L2 = 104.0e9
# Beyond ~3 GiB the page translations bind, not the lines: dependent random 64-B loads over
# tables of 4 / 6 / 8 / 16 GiB (profiles/r02/gather_tlb.txt; contiguous and 1-GiB-granule
# allocations the same, profiles/r02/gather_alloc.txt).
RANDOM_LINES_BY_TABLE = [(3 << 30, 51.0e9), (4 << 30, 22.6e9), (6 << 30, 18.5e9),
                         (8 << 30, 17.1e9), (16 << 30, 16.3e9)]


def _random_lines_ceiling(table_bytes):
    """Measured random-line ceiling for a table of this size (linear between the points)."""
    pts = RANDOM_LINES_BY_TABLE
    if table_bytes <= pts[0][0]:
        return RANDOM_LINES_PEAK
    for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
        if table_bytes <= x1:
            return y0 + (y1 - y0) * (table_bytes - x0) / (x1 - x0)
    return pts[-1][1]


def _pmc(cfg, nt, nb):
    """Per-kernel PMC summary of this config from profiles/ (HBM bytes, L2 hits/misses and
    TCP->TCC read requests per launch, tools/pmc_traffic.py), if one was committed for this
    batch size and number of distinct batches."""
    for name in (f"pmc_cfg{cfg}.json",):
        p = os.path.join(ROOT, "profiles", name)
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if int(d.get("topics", -1)) != nt or int(d.get("batches", 1)) != nb:
            continue
        return {k: dict(v, source=f"profiles/{name}") for k, v in d.get("kernels", {}).items()}
    return {}


def _roofline(nt, nbytes, census, pmc, tok_ms, exact_ms, walk_ms, pipe_ms, exact_table_bytes=0):
    """Roofline of the step's dominant kernel (by HIP-event time, one pass at a time).

    k_walk and k_exact are dependent random gathers: the binding resource is the rate of random
    64-B line requests the memory system serves beyond the L1 (RANDOM_LINES_PEAK from beyond the
    L2, RANDOM_LINES_L2 from it: tools/gather_bench.hip, whose every load misses the L1), not HBM
    bandwidth.  `achieved` counts the requests that reach the L2: for k_walk the PMC
    TCP_TCC_READ_REQ per launch of the committed HEAD profile (profiles/pmc_cfg<N>.json, same
    batch size and batches), for k_exact one bucket line per name; the census edge-bucket loads
    (L1 hits included) are `edge_loads_per_s`.  Beside it the SURVEY 8d algorithmic bytes and the
    PMC counter bytes as fractions of the 8 TB/s HBM peak.  k_tok streams: bound HBM."""
    kernels = {"k_tok": tok_ms, "k_exact": exact_ms, "k_walk": walk_ms}
    dom = max(kernels, key=lambda k: kernels[k])
    post = max(0.0, pipe_ms - tok_ms - exact_ms - walk_ms)
    ms = kernels[dom]
    sec = ms * 1e-3 if ms > 0 else float("inf")
    p = pmc.get(dom, {})
    traffic = p.get("hbm_bytes_per_launch")
    out = {"kernel": dom}
    if dom == "k_tok":
        # topic bytes + offsets in; 64-B record, level count and exact id out per topic
        alg = nbytes + 4 * (nt + 1) + (64 + 4 + 4) * nt
        ach = alg / sec / 1e9
        out.update({"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "algorithmic_bytes_per_launch": int(alg)})
    else:
        edge_loads = None
        if dom == "k_walk":
            edge_loads = census["slot_loads"]
            req = p.get("tcp_tcc_read_req")
            lines = req if req else edge_loads
            src = ("PMC TCP_TCC_READ_REQ per launch (" + str(p.get("source")) + ")" if req else
                   "census edge-bucket loads (no PMC request count committed for this batch: "
                   "L1 hits included, an over-count)")
            # the bytes this design must move per launch: one 64-B bucket line per edge probe the
            # production walk makes (census), the 64-B topic record and 4-B count per topic, an
            # 8-B staged pair per match (packed staging, gm_kernels.h StgFmt: every bench config
            # fits it; a pass redone wide shows in "reruns").  SURVEY 8d's model (3 x 16-B probes per matched trie
            # state, 16-B pairs) is kept beside it, labelled: it counts states the upper levels
            # serve from the L2 and the fat buckets never probe, so it can pass the HBM peak
            alg = 64 * census["slot_loads"] + (64 + 4) * nt + 8 * census["pairs"]
            model = (64 + 4) * nt + 48 * census["states"] + 16 * census["pairs"]
            pruned = 48 * (census["states"] - census.get("states_visited", census["states"]))
        else:
            lines = nt
            src = "one route-key bucket line per name"
            alg = nbytes + 8 * nt + 64 * nt + 4 * nt
            model = alg
            pruned = 0
        ach = lines / sec
        # the ceiling of this access mix: a request that misses the L2 costs 1 / RANDOM_LINES_PEAK,
        # one that hits 1 / RANDOM_LINES_L2 (the measured gather rates); the miss share comes
        # from the committed PMC run of this config (per-launch hit / miss counters).  The
        # route-key probe's bucket lines are all misses; over a table beyond the TLB's reach
        # their ceiling is the measured rate for that table size.
        peak = RANDOM_LINES_PEAK
        mr = None
        if dom == "k_exact":
            peak = _random_lines_ceiling(exact_table_bytes)
        elif p.get("tcc_miss") is not None and (p.get("tcc_hit") or 0) + p["tcc_miss"] > 0:
            mr = float(p["tcc_miss"]) / (float(p["tcc_miss"]) + float(p.get("tcc_hit") or 0))
            peak = 1.0 / (mr / RANDOM_LINES_PEAK + (1.0 - mr) / RANDOM_LINES_L2)
        out.update({
            "bound": "random-access", "achieved": round(ach / 1e9, 2),
            "peak": round(peak / 1e9, 2), "unit": "G lines/s",
            "frac": round(ach / peak, 4), "traffic": traffic,
            "l2_requests_per_launch": int(lines), "achieved_source": src,
            "exact_table_bytes": int(exact_table_bytes) if dom == "k_exact" else None,
            "l2_miss_share": None if mr is None else round(mr, 4),
            "peak_source": ("measured dependent random 64-B gather rate over a table of the route-"
                            "key table's size (tools/gather_bench.hip, profiles/r02/gather_tlb.txt)"
                            if dom == "k_exact" else
                            "measured dependent random 64-B gather rates (tools/gather_bench.hip, "
                            "profiles/r01/gather_sizes.txt): 53 G/s from beyond the L2, 104 G/s "
                            "from it, weighted by this kernel's L2 miss share (PMC)"),
            "hbm_algorithmic": {"bytes_per_launch": int(alg),
                                "counts": ("64-B line per edge probe (census) + 68 B per topic "
                                           "(record, count) + 8 B per staged pair (packed)"
                                           if dom == "k_walk" else
                                           "topic bytes + offsets + one 64-B bucket line + 4-B "
                                           "exact id per name"),
                                "achieved_GBs": round(alg / sec / 1e9, 1),
                                "frac": round(alg / sec / 1e9 / HBM_PEAK_GBS, 4)},
            "survey_8d_model": {"bytes_per_launch": int(model), "pruned_state_bytes": int(pruned),
                                "frac": round(model / sec / 1e9 / HBM_PEAK_GBS, 4),
                                "note": "SURVEY 8d's per-state model (48 B per matched trie "
                                        "state), a model of the reference's probes, not of this "
                                        "design's traffic: may exceed 1"},
        })
        if edge_loads is not None:
            out["edge_loads_per_launch"] = int(edge_loads)
            out["edge_loads_per_s"] = round(edge_loads / sec / 1e9, 2)
        if traffic:
            out["hbm_counter"] = {"bytes_per_launch": traffic,
                                  "achieved_GBs": round(traffic / sec / 1e9, 1),
                                  "frac": round(traffic / sec / 1e9 / HBM_PEAK_GBS, 4),
                                  "source": p.get("source")}
        if p.get("tcc_miss") is not None:
            miss, hit = float(p["tcc_miss"]), float(p.get("tcc_hit") or 0.0)
            model = miss / RANDOM_LINES_PEAK + hit / RANDOM_LINES_L2
            out["l2_lines"] = {"miss_per_launch": miss, "hit_per_launch": hit,
                               "miss_rate_G": round(miss / sec / 1e9, 2),
                               "frac_miss_lines": round(miss / sec / RANDOM_LINES_PEAK, 4),
                               # time the misses and hits would take at the measured gather
                               # ceilings, over the kernel's time
                               "frac_mixed_ceiling": round(model / sec, 4),
                               "source": p.get("source")}
        if p.get("stalls"):
            # the memory-subsystem stall counters of the committed HEAD profile (tools/
            # pmc_stalls.py): which unit bounds the kernel ("What bounds the walk")
            out["stall_counters"] = {k: v for k, v in p["stalls"].items() if k != "raw"}
        if p.get("duration_us") is not None:
            # the PMC run's kernel average over the default (pipelined) command: walks beside the
            # other pass's kernels at three workgroups per CU, not the one-pass time used above
            out["rocprof_pipelined_avg_us"] = p.get("duration_us")
    out["kernels_ms"] = {"k_tok": round(tok_ms, 4), "k_exact": round(exact_ms, 4),
                         "k_walk": round(walk_ms, 4), "verify+scan+scatter": round(post, 4),
                         "pass": round(pipe_ms, 4)}
    out["walk_ms_per_launch"] = round(walk_ms, 4)
    return out


def _cfg4_cpu_index(w):
    """cfg4's CPU index without the 100M-key ordered set (tens of GB of host memory, minutes to
    build): the 1M wildcard filters (trie + route keys) and the route keys the batch's topics
    name.  The reference's route table is an ets bag (a hash, emqx_router.erl:143-145), so a
    lookup costs the same whatever the number of other keys; the trie holds only wildcards."""
    n_exact = w.nf - w.nf // 101  # workloads/gen.cpp gen_cfg4: keys dev/{i:09}/state, i < n_exact
    wi = np.nonzero(w.fwild)[0]
    wb, wo = _subset(w, wi)
    rows = w.tbytes.reshape(w.nt, -1)
    digits = rows[:, 4:13].astype(np.int64) - ord("0")
    ids = (digits * (10 ** np.arange(8, -1, -1, dtype=np.int64))).sum(1)
    keys = np.unique(rows[ids < n_exact], axis=0)
    fb = np.concatenate([wb, keys.reshape(-1)])
    fo = np.concatenate([wo, int(wo[-1]) + np.arange(1, len(keys) + 1, dtype=np.uint64) * rows.shape[1]])
    kinds = np.concatenate([np.full(len(wi), 3, np.uint8), np.full(len(keys), 2, np.uint8)])
    note = (f"; index: the {len(wi)} wildcard filters + the {len(keys)} route keys the batch's "
            f"topics name (of {n_exact}: the reference's route table is a hash bag, a lookup "
            f"costs the same at any size)")
    return fb, fo.astype(np.uint64), kinds, note


class _CpuIndexJob:
    def __init__(self, w, cfg=3):
        import threading
        from oracle.cref import RefIndex
        self.ref = RefIndex(True)
        self.t0 = time.time()
        self.build_s = None
        self.note = ""

        def run():
            if cfg == 4:
                fb, fo, kinds, self.note = _cfg4_cpu_index(w)
                self.ref.add_many(fb, fo, kinds)
            else:
                self.ref.add_many(w.fbytes, w.foff, 2 + w.fwild)
            self.build_s = time.time() - self.t0
        self.th = threading.Thread(target=run, daemon=True)
        self.th.start()

    def wait(self):
        self.th.join()
        return self.ref, self.build_s


def _cpu_leg(ref, w, threads, seconds):
    """Topics/s of the reference restatement on `threads` threads over a bounded sample."""
    n = min(w.nt, 20000)
    dt, _ = ref.time_match(w.tbytes, w.toff[: n + 1], threads)
    rate = n / max(dt, 1e-9)
    n2 = int(min(w.nt, max(n, rate * seconds)))
    if n2 > n:
        dt, _ = ref.time_match(w.tbytes, w.toff[: n2 + 1], threads)
        n = n2
    reps = 1
    if dt < seconds / 2:
        # the whole batch takes less than the bounded sample's time: match it again and again
        reps = max(1, int(seconds / max(dt, 1e-3)))
        t0 = time.perf_counter()
        for _ in range(reps):
            ref.time_match(w.tbytes, w.toff[: n + 1], threads)
        dt = (time.perf_counter() - t0) / reps
    return n / dt, n, reps, dt


def _cgroup_throttled():
    """(nr_throttled, throttled_usec) of this cgroup (v2 cpu.stat), or None: the quota's
    periods in which every thread of the job was stopped."""
    try:
        st = {}
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                st[k] = int(v)
        return st.get("nr_throttled", 0), st.get("throttled_usec", 0)
    except (OSError, ValueError):
        return None


def _cgroup_cpus():
    """CPUs the cgroup's quota lets this process use (cgroup v2 cpu.max "quota period", v1
    cpu.cfs_quota_us / cpu.cfs_period_us), or None when unlimited / unknown."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        return max(1, math.ceil(q / p)) if q > 0 else None
    except (OSError, ValueError):
        return None


def effective_cpus():
    """(effective CPUs, affinity CPUs, cgroup quota CPUs or None): SURVEY 8d's "nproc" = the CPUs
    this process can actually use -- its affinity set, capped by the cgroup's CPU quota (r03's
    line said 256 from the affinity alone on a lease quota-limited to ~16: 16 and 256 threads
    gave the same rate)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = _cgroup_cpus()
    return (min(aff, quota) if quota else aff), aff, quota


def _cpu_baseline(w, args, job):
    """The reference algorithm (C++ restatement of emqx_trie match_compact with an ordered-set
    index, oracle/ref_trie.cpp) on this host's cores, over a bounded sample of the topics.
    T = the CPUs this process can use (effective_cpus: affinity capped by the cgroup quota; one
    thread per BEAM scheduler), and beside it the same leg at the affinity count when that is
    larger (to show the quota binds)."""
    eff, aff, quota = effective_cpus()
    threads = args.cpu_threads or eff
    ref, build_s = job.wait()
    rate, n, reps, dt = _cpu_leg(ref, w, threads, args.cpu_seconds)
    log(f"cpu baseline: index build {build_s:.1f}s, {n} topics in {dt:.2f}s on {threads} threads "
        f"(affinity {aff}, quota {quota})")
    # one thread: the reference's per-topic latency on the publisher's own core (the crossover)
    r1, n1, reps1, dt1 = _cpu_leg(ref, w, 1, args.cpu_seconds / 4)
    one_thread = {"value": round(r1, 1), "us_per_topic": round(1e6 / max(r1, 1e-9), 2),
                  "sample": f"first {n1} topics" + (f" (x{reps1}, mean)" if reps1 > 1 else "")}
    share_leg = None
    if aff > threads:
        r2, n2, reps2, dt2 = _cpu_leg(ref, w, aff, args.cpu_seconds / 2)
        share_leg = {"value": round(r2, 1), "threads": aff,
                     "sample": f"first {n2} topics" + (f" (x{reps2}, mean)" if reps2 > 1 else "")}
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": round(rate, 1), "unit": "topics/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpus": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_quota_cpus": quota, "effective_cpus": eff,
            "at_affinity_threads": share_leg,
            "one_thread": one_thread,
            "index_build_s": round(build_s, 1),
            "sample": f"first {n} topics of batch 0" + (f" (x{reps}, mean)" if reps > 1 else "")
                  + f" against the same {w.nf} filters "
                      f"(emqx_trie match_compact restated in C++, std::map ordered set), "
                      f"{dt * reps:.1f}s wall" + job.note}


if __name__ == "__main__":
    main()
