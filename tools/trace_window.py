"""Timeline of one host window from a rocprofv3 trace of tools/window_latency.py (tools/job.sh
wintrace): the HIP API calls on the submitting thread and the kernels / copies they enqueue,
in microseconds from the window's first H2D copy call.

    python tools/trace_window.py gpurun_out/TAG/wintrace [--window K ...]

Windows are delimited by their first hipMemcpyAsync host-to-device call (the device-only passes
of the script copy nothing).
"""
import argparse
import csv
import glob
import os


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--window", type=int, action="append", default=[])
a = ap.parse_args()

api = rows(a.dir, "*hip_api_trace.csv")
ker = rows(a.dir, "*kernel_trace.csv")
cpy = rows(a.dir, "*memory_copy_trace.csv")
ev = []
for r in api:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"],
               r.get("Correlation_Id")))
for r in ker:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", r["Kernel_Name"][:40],
               r.get("Correlation_Id")))
for r in cpy:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy",
               r.get("Direction", "copy"), r.get("Correlation_Id")))
ev.sort()
# window starts: a hipMemcpyAsync API call whose copy goes host -> device
h2d_corr = {r.get("Correlation_Id") for r in cpy if "HOST_TO_DEVICE" in r.get("Direction", "").upper()}
starts = [e for e in ev if e[2] == "api" and e[3] == "hipMemcpyAsync" and e[4] in h2d_corr]
# every window issues two H2D copies (bytes, offsets): the first of each pair starts a window
starts = starts[::2]
print(f"{len(starts)} windows")
wins = a.window or [len(starts) // 4, len(starts) - 2]
for k in wins:
    t0 = starts[k][0]
    t1 = starts[k + 1][0] if k + 1 < len(starts) else ev[-1][1]
    print(f"\n== window {k}: {(t1 - t0) / 1e3:.1f} us to the next window's first copy")
    for s, e, kind, name, _ in ev:
        if t0 <= s < t1:
            print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  {kind:4s} {name}")
