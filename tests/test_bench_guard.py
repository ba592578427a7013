"""bench.py's watchdog around the filter-sharded N>1 run: a run that hangs
ends the rank after the timeout -- with exit status 3 -- with the replicas' line printed and the
timeout recorded in config.filter_sharded; a run that raises is recorded as the result.  CPU only (no collective:
the run is a stand-in that sleeps or raises)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, sys, time
sys.path.insert(0, {root!r})
import bench
line = {{"metric": "m", "value": 1.0, "config": {{"workload": "w"}}}}
mode = sys.argv[1]
if mode == "hang":
    bench._guarded(lambda: time.sleep(60), 0.5, 0, line)
    print("not reached", flush=True)
else:
    def boom():
        raise RuntimeError("collective failed")
    r = bench._guarded(boom, 30.0, 0, line)
    line["config"]["filter_sharded"] = r
    print(json.dumps(line), flush=True)
"""


def _run(mode):
    p = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT), mode], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120)
    return p.returncode, p.stdout.strip().splitlines()


def test_hanging_filter_sharded_run_still_prints_the_line():
    """...and exits non-zero (a hung RCCL run must not report success)."""
    rc, out = _run("hang")
    assert rc == 3  # bench.WATCHDOG_EXIT
    assert len(out) == 1, out  # one JSON line, and the code after the hang never ran
    line = json.loads(out[0])
    assert line["value"] == 1.0
    assert line["config"]["filter_sharded"]["error"].startswith("timeout after")


def test_failing_filter_sharded_run_is_recorded():
    rc, out = _run("raise")
    assert rc == 0
    line = json.loads(out[-1])
    assert "collective failed" in line["config"]["filter_sharded"]["error"]
