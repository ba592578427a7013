"""Per-wave timeline of one census walk (diagnostic).

GPU box:  EMQXGM_WAVE_TIMES=gpurun_out/wt.bin python bench.py --steps 1 ...
          python tools/wave_times.py gpurun_out/wt.bin
Each wave records {start, claims exhausted, end} with wall_clock64() (100 MHz).
"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], np.uint64).reshape(-1, 3).astype(np.int64)
t = t[t[:, 2] > 0]
t0 = t[:, 0].min()
us = (t - t0) / 100.0  # 100 MHz -> us
s, d, e = us[:, 0], us[:, 1], us[:, 2]
q = lambda x: " ".join(f"{v:7.1f}" for v in np.percentile(x, [0, 1, 10, 50, 90, 99, 100]))
print(f"waves {len(t)}  (percentiles 0 1 10 50 90 99 100, us from the first wave start)")
print("start          ", q(s))
print("claims gone    ", q(d))
print("end            ", q(e))
print("end - gone     ", q(e - d))
