#!/bin/bash
# r03: GPU tests with three device pipes (EMQXGM_PIPES 3), then 3 vs 2 passes in flight
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_pipes3}
cd $R
TESTS=1 SPECS="3:0 3:65536 3:16384 1:0 2:0" STEPS=50 VARIANT="--inflight 2" bash tools/r03_tune_ab.sh $T || exit 1
