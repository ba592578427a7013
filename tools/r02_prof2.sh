#!/bin/bash
# rocprofv3 kernel stats + PMC traffic passes (tools/r02_prof.sh) for CFGS, then cfg3's kernel
# stats with one pass at a time (every walk launch alone, as the roofline's HIP-event timing)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_prof2}
mkdir -p $O
CFGS=${CFGS:-3 2} bash $R/tools/r02_prof.sh ${1:-r02_prof2} || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_cfg3_onepass -o run --output-format csv -- python3 $R/bench.py --no-pipeline --no-cpu-baseline --no-e2e --steps 10 --warmup 2 > $O/stats_cfg3_onepass.log 2>&1
