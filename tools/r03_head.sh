#!/bin/bash
# r03: the default bench line at HEAD (3 distinct batches), then kernel stats + PMC of every
# config (tools/r03_prof.sh); each step bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_head}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
bash $R/tools/r03_prof.sh ${1:-r03_head}/prof || exit 1
