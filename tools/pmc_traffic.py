"""Turns a tools/pmc.sh run over the bench workload into profiles/pmc_cfg<N>.json: per kernel,
the HBM traffic and L2 hits/misses per launch that bench.py reports beside its roofline.

FETCH_SIZE / WRITE_SIZE are in KiB.  Calibrated on this MI355X with tools/calib_fetch.sh
(profiles/r01/calib_fetch.txt): a random 16-, 32- or 64-B gather costs exactly one 64-B
memory-side read request (TCC_EA0_RDREQ) and FETCH_SIZE = 64 B x TCC_EA0_RDREQ, so for the
random-access kernels (k_walk, k_exact) FETCH_SIZE is taken as is; for wide coalesced streaming
reads (k_tok, k_scatter, k_verify) gfx950 reports half the bytes (MI355X_MICROARCH.md "HBM"), so
those are doubled.

    python tools/pmc_traffic.py gpurun_out/pmc_TAG --cfg 3 --topics 2000000
"""
import argparse
import json
import os

STREAMING = ("k_tok", "k_scatter", "k_verify", "k_scan")

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--cfg", type=int, default=3)
ap.add_argument("--topics", type=int, default=2000000)
a = ap.parse_args()
s = json.load(open(os.path.join(a.root, "summary.json")))
kern = {}
for name, k in s.items():
    if "FETCH_SIZE" not in k:
        continue
    if "n" not in k:  # summaries written before launch counts were recorded
        k["n"] = 1
    short = name.split("<")[0]
    corr = 2.0 if short.startswith(STREAMING) else 1.0
    fetch = k["FETCH_SIZE"] * 1024.0 * corr
    write = k.get("WRITE_SIZE", 0.0) * 1024.0
    ent = {"kernel": name, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "hbm_bytes_per_launch": fetch + write, "fetch_correction": corr,
           "tcc_hit": k.get("TCC_HIT_sum"), "tcc_miss": k.get("TCC_MISS_sum")}
    # the production variant of a kernel (not a census walk; the one with the most launches)
    # wins over the others
    census = name.startswith("k_walk<true")
    ent["n"] = k.get("n", 0)
    prev = kern.get(short)
    if prev is None or (prev["census"] and not census) or (
            prev["census"] == census and ent["n"] > prev["n"]):
        ent["census"] = census
        kern[short] = ent
out = {"topics": a.topics, "cfg": a.cfg, "source": a.root, "kernels": kern}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = os.path.join(root, "profiles", f"pmc_cfg{a.cfg}.json")
json.dump(out, open(p, "w"), indent=1)
print(p, json.dumps(out, indent=1))
