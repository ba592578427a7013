#!/bin/bash
# r03: GPU tests (all, or $TESTSEL), smoke, then the default bench line and $CFGS bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_check}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest ${TESTSEL:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py $BENCHARGS > $O/cfg3.json 2> $O/cfg3.log || exit 1
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --cfg $c --no-cpu-baseline $BENCHARGS > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
