"""Turns the rocprofv3 passes of tools/r03_prof.sh over the bench workload into
profiles/pmc_cfg<N>.json: per kernel the HBM traffic, L2 hits/misses, TCP->TCC read requests
per launch and the rocprof average duration that bench.py reports beside its roofline.

FETCH_SIZE / WRITE_SIZE are in KiB.  Calibrated on this MI355X with tools/calib_fetch.sh
(profiles/r01/calib_fetch.txt): a random 16-, 32- or 64-B gather costs exactly one 64-B
memory-side read request (TCC_EA0_RDREQ) and FETCH_SIZE = 64 B x TCC_EA0_RDREQ, so for the
random-access kernels (k_walk, k_exact) FETCH_SIZE is taken as is; for wide coalesced streaming
reads (k_tok, k_scatter, k_verify) gfx950 reports half the bytes (MI355X_MICROARCH.md "HBM"), so
those are doubled.

    python tools/pmc_traffic.py gpurun_out/TAG/pmc_cfg3 --cfg 3 --topics 4000000 --batches 3 \
        [--stats gpurun_out/TAG/stats_cfg3/run_kernel_stats.csv] [--out profiles/pmc_cfg3.json]
"""
import argparse
import csv
import json
import os
import re

STREAMING = ("k_tok", "k_scatter", "k_verify", "k_scan")

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--cfg", type=int, default=3)
ap.add_argument("--topics", type=int, default=4000000)
ap.add_argument("--batches", type=int, default=3)
ap.add_argument("--stats", default=None)
ap.add_argument("--out", default=None)
ap.add_argument("--sq", default=None, help="tools/job.sh sq=N output dir: issue counters of k_walk")
a = ap.parse_args()
s = json.load(open(os.path.join(a.root, "summary.json")))
dur = {}
if a.stats and os.path.exists(a.stats):
    for r in csv.DictReader(open(a.stats)):
        m = re.search(r"(k_[a-z_]+)(<[^>]*>)?\(", r["Name"])
        if m:
            dur[m.group(1) + (m.group(2) or "")] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
kern = {}
for name, k in s.items():
    if "FETCH_SIZE" not in k and "TCP_TCC_READ_REQ_sum" not in k:
        continue
    short = name.split("<")[0]
    corr = 2.0 if short.startswith(STREAMING) else 1.0
    fetch = k.get("FETCH_SIZE", 0.0) * 1024.0 * corr
    write = k.get("WRITE_SIZE", 0.0) * 1024.0
    ent = {"kernel": name, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write, "fetch_correction": corr,
           "tcc_hit": k.get("TCC_HIT_sum"), "tcc_miss": k.get("TCC_MISS_sum"),
           "tcp_tcc_read_req": k.get("TCP_TCC_READ_REQ_sum"),
           "tcp_accesses": k.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
           "tcp_tcc_read_latency_cycles": (k["TCP_TCC_READ_REQ_LATENCY_sum"] / k["TCP_TCC_READ_REQ_sum"]
                                           if k.get("TCP_TCC_READ_REQ_sum") and
                                           k.get("TCP_TCC_READ_REQ_LATENCY_sum") else None)}
    if name in dur:
        ent["duration_us"], ent["stats_calls"] = dur[name]
    # the production variant of a kernel (not a census walk; the one with the most launches)
    # wins over the others
    census = name.startswith("k_walk<true")
    ent["n"] = k.get("n", 0)
    prev = kern.get(short)
    if prev is None or (prev["census"] and not census) or (
            prev["census"] == census and ent["n"] > prev["n"]):
        ent["census"] = census
        kern[short] = ent
out = {"topics": a.topics, "batches": a.batches, "cfg": a.cfg, "source": a.root,
       "stats": a.stats, "kernels": kern}
if a.sq and os.path.exists(os.path.join(a.sq, "summary.json")):
    # per launch of the production walk (not the census one): instructions per wave, issue share
    for name, k in json.load(open(os.path.join(a.sq, "summary.json"))).items():
        if not name.startswith("k_walk<false") or "SQ_WAVES" not in k:
            continue
        waves = k["SQ_WAVES"]
        sq = {c: v for c, v in k.items() if c.startswith(("SQ_", "GRBM_"))}
        sq["insts_per_wave"] = (k.get("SQ_INSTS_VALU", 0) + k.get("SQ_INSTS_SALU", 0) +
                                k.get("SQ_INSTS_LDS", 0) + k.get("SQ_INSTS_VMEM_RD", 0) +
                                k.get("SQ_INSTS_VMEM_WR", 0)) / waves
        sq["source"] = a.sq
        if "k_walk" in kern and kern["k_walk"]["kernel"] == name:
            kern["k_walk"]["sq"] = sq
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = a.out or os.path.join(root, "profiles", f"pmc_cfg{a.cfg}.json")
json.dump(out, open(p, "w"), indent=1)
print(p, json.dumps(out, indent=1))
