"""Print the headline fields of bench JSON lines (files given on the command line)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001 - a missing / partial file is reported, not fatal
        print(f, "unreadable:", e)
        continue
    r = d.get("roofline") or {}
    c = d.get("config") or {}
    print(f, round(d["value"] / 1e9, 3), d["ms_per_step"],
          (c.get("one_pass_at_a_time") or {}).get("ms_per_step"), r.get("kernels_ms"), r.get("frac"))
