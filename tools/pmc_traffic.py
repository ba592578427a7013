"""Turns a tools/pmc.sh run over the bench workload into profiles/pmc_walk_cfg<N>.json, the HBM
traffic per k_walk launch that bench.py reports as roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB.  Calibrated on this MI355X with tools/calib_fetch.sh
(profiles/r01/calib_fetch.txt): a random 16-, 32- or 64-B gather costs exactly one 64-B
memory-side read request (TCC_EA0_RDREQ) and FETCH_SIZE = 64 B x TCC_EA0_RDREQ, so for the
walk's random slot loads FETCH_SIZE is taken as is (no x2: that correction applies to wide
coalesced streaming reads only, MI355X_MICROARCH.md "HBM").

    python tools/pmc_traffic.py gpurun_out/pmc_TAG --cfg 3 --topics 2000000
"""
import argparse
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--cfg", type=int, default=3)
ap.add_argument("--topics", type=int, default=2000000)
ap.add_argument("--kernel", default="k_walk<false, false>")
a = ap.parse_args()
s = json.load(open(os.path.join(a.root, "summary.json")))
k = s[a.kernel]
fetch = k["FETCH_SIZE"] * 1024.0
write = k.get("WRITE_SIZE", 0.0) * 1024.0
out = {"kernel": a.kernel, "topics": a.topics, "cfg": a.cfg,
       "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
       "hbm_bytes_per_launch": fetch + write,
       "tcc_hit": k.get("TCC_HIT_sum"), "tcc_miss": k.get("TCC_MISS_sum"),
       "source": a.root}
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
p = os.path.join(root, "profiles", f"pmc_walk_cfg{a.cfg}.json")
json.dump(out, open(p, "w"), indent=1)
print(p, out)
