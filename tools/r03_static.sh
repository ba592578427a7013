#!/bin/bash
# r03: the GPU tests with the static small-batch walk, then the A/B of walk builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_static}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
SPECS="3:65536 3:262144 1:0 3:0" STEPS=30 bash tools/r03_ab_lib.sh ${1:-r03_static}/ab nostatic nosmall2 || exit 1
