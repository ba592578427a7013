#!/bin/bash
# r03: GPU tests + smoke, the window probe (one-sync windows), then the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_win2}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/window_probe.py > $O/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
