#!/bin/bash
# r03: per-wave census timelines of small walks (cfg1 100k, cfg3 64k)
set -o pipefail
O=gpurun_out/${1:-r03_wt}; mkdir -p $O
EMQXGM_WAVE_TIMES=$O/wt_cfg1.bin timeout -k 10 240 python -u bench.py --cfg 1 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --windows "" > $O/b1.log 2>&1 &&
python tools/wave_times.py $O/wt_cfg1.bin > $O/wt_cfg1.txt &&
EMQXGM_WAVE_TIMES=$O/wt_cfg3.bin timeout -k 10 300 python -u bench.py --cfg 3 --topics 65536 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --windows "" > $O/b3.log 2>&1 &&
python tools/wave_times.py $O/wt_cfg3.bin > $O/wt_cfg3.txt
