#!/bin/bash
# r03: A/B of the 4-slot one-topic-per-lane walk (build/lib_ws2: 2 slots) on small batches
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_ws_ab}
cd $R
SPECS="1:0 3:16384 3:65536 3:196608" STEPS=50 bash tools/r03_ab_lib.sh $T/ab ws2 || exit 1
