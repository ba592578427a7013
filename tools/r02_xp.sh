#!/bin/bash
# experiment: cfg3 pipelined step vs walk workgroups per CU (k_tok of the next pass co-resident
# with the walk only where LDS / VGPRs leave room)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_xp}
mkdir -p $O
cd $R
for wg in 3 2; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-e2e --wg-per-cu $wg > $O/wg$wg.json 2> $O/wg$wg.err || exit 1
done
