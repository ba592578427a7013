"""Prints the bench lines of a tools/r03_ab.sh run side by side: value, step, walk, loads."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.json"))):
    try:
        d = json.load(open(f))
    except ValueError:
        print(os.path.basename(f), "unreadable")
        continue
    r, c = d["roofline"], d["config"]
    print(f"{os.path.basename(f):18s} {d['value'] / 1e9:7.3f} G/s  step {d['ms_per_step']:.4f} ms  "
          f"walk {r['kernels_ms']['k_walk']:.4f}  tok {r['kernels_ms']['k_tok']:.4f}  "
          f"pass {r['kernels_ms']['pass']:.4f}  loads {c['edge_slot_loads_per_batch']:.0f}  "
          f"wave_it {c['walk_wave_iterations_per_batch']:.0f}  tune {c.get('tune')}")
