"""Prints the bench lines of a tools/r03_ab_lib.sh run (<variant>_c<cfg>_<topics>.json) side by
side: value, pipelined step, one-pass walk and pass times."""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_c*_*.json"))):
    try:
        d = json.load(open(f))
    except ValueError:
        print(os.path.basename(f), "unreadable")
        continue
    k = d["roofline"]["kernels_ms"]
    print(f"{os.path.basename(f):28s} {d['value'] / 1e9:7.3f} G/s  step {d['ms_per_step']:.4f}  "
          f"walk {k['k_walk']:.4f}  tok {k['k_tok']:.4f}  pass {k['pass']:.4f}")
