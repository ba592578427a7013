#!/bin/bash
# r03: the small-batch regime -- per-wave walk timelines of census walks at cfg1 (100k topics)
# and cfg3 at 64k / 256k topics, then a kernel trace of one-pass-at-a-time cfg1 steps (gaps
# between a pass's launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_small}
mkdir -p $O
cd $R
for spec in "1 100000" "3 65536" "3 262144"; do
  set -- $spec
  EMQXGM_WAVE_TIMES=$O/wt_cfg$1_$2.bin timeout -k 10 300 python -u bench.py --cfg $1 --topics $2 --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > $O/b_cfg$1_$2.json 2> $O/b_cfg$1_$2.log || exit 1
  python3 tools/wave_times.py $O/wt_cfg$1_$2.bin > $O/wt_cfg$1_$2.txt || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_cfg1 -o run --output-format csv -- python3 $R/bench.py --cfg 1 --no-cpu-baseline --no-e2e --no-pipeline --steps 20 --warmup 3 > $O/trace_cfg1.log 2>&1 || exit 1
