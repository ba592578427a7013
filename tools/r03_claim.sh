#!/bin/bash
# r03: GPU tests + smoke with static first claims and the control words mirrored by the row
# scan, then the A/B against build/lib_noclaim and build/lib_ctlk (control words by k_ctl_out)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_claim}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
SPECS="3:0 3:65536 1:0 2:0" STEPS=50 bash tools/r03_ab_lib.sh $T/ab noclaim ctlk || exit 1
