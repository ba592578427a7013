#!/bin/bash
# GPU tests + smoke + the default (cfg3) bench line, each step under its own time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_run}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${TESTS} > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err
