#!/bin/bash
# per-config bench lines (cfg1, cfg2, cfg4 with their CPU baselines; cfg3 is the default bench),
# then the N=2 rehearsal of the multi-GPU path on this box; each step bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_results}
mkdir -p $O
cd $R
for c in ${CFGS:-1 2 4}; do
  timeout -k 10 400 python -u bench.py --cfg $c --steps 10 > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
timeout -k 10 300 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
bash tools/run_dist_rehearsal.sh ${1:-r02_results}/dist > $O/dist.txt 2>&1
