#!/bin/bash
# r03 final: rocprofv3 kernel stats of the cfg3 bench one pass at a time (the roofline's kernel
# time) and pipelined, PMC passes of cfg3 (tools/r03_prof.sh), then every config's default bench
# line at HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_final}
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/onepass -o run --output-format csv -- python3 $R/bench.py --no-pipeline --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > $O/onepass.json 2> $O/onepass.log || exit 1
CFGS="3" bash $R/tools/r03_prof.sh $T/prof || exit 1
cd $R
for c in 3 1 2 4; do
  timeout -k 10 400 python -u bench.py --cfg $c > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
