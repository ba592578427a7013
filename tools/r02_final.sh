#!/bin/bash
# round-end rehearsal on one box: GPU tests, smoke, the default bench line, the other configs'
# bench lines, and cfg2's PMC traffic passes; each step bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
for c in ${CFGS:-1 2 4}; do
  timeout -k 10 400 python -u bench.py --cfg $c > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
