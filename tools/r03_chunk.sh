#!/bin/bash
# r03: GPU tests with the static first staged-pair chunk per walk wave, the A/B of walk builds,
# then the SQ issue/wait mix of the cfg1 walk
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_chunk}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
SPECS="1:0 3:65536 3:262144 3:0 2:0" STEPS=30 bash tools/r03_ab_lib.sh $T/ab nostatchunk nostatic neither2 || exit 1
CFGS="1" bash tools/r03_sq.sh $T/sq || exit 1
