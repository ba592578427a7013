"""Average rocprofv3 PMC counter values per kernel over the dispatches of tools/pmc.sh."""
import collections
import re
import csv
import glob
import json
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or "?"
        m = re.search(r"(k_[a-z_]+)(<[^>]*>)?\(", name)
        short = (m.group(1) + (m.group(2) or "")) if m else name[:40]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    out[k] = {c: sum(v) / len(v) for c, v in d.items()}
    out[k]["n"] = max(len(v) for v in d.values())
    print(k)
    for c in sorted(d):
        print(f"   {c:24s} {out[k][c]:16.1f}  (n={len(d[c])})")
json.dump(out, open(root + "/summary.json", "w"), indent=1)
