#!/bin/bash
# r03: instruction-issue counters of the walk (cfg1 100k, cfg3 64k, cfg3 4M) -- one PMC pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_sqi}
mkdir -p $O
G="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
for c in "1 100000" "3 65536" "3 4000000"; do
  set -- $c
  timeout -s KILL 400 rocprofv3 --pmc $G --kernel-include-regex "k_walk" -d $O/sq_$1_$2 -o run --output-format csv -- python3 $R/bench.py --cfg $1 --topics $2 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/sq_$1_$2.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py $O/sq_$1_$2 > $O/sq_$1_$2_summary.txt 2>&1 || exit 1
done
