#!/bin/bash
# r03: optional GPU tests, then bench lines per spec ("cfg:topics", topics 0 = the config's
# default) with and without a runtime tune (new, old = $VARIANT, new again); each step bounded.
#   TESTS=1 SPECS="1:0 3:0" VARIANT="--tune walk_defer=0" tools/r03_tune_ab.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_tune_ab}
mkdir -p $O
cd $R
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest ${TESTSEL:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
  timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
fi
for spec in ${SPECS:-3:0}; do
  c=${spec%%:*}; t=${spec##*:}
  T=""; [ "$t" != 0 ] && T="--topics $t"
  X="--cfg $c $T --no-cpu-baseline --no-e2e --steps ${STEPS:-30} --warmup 5"
  for v in new1 old new2; do
    V=""; [ $v = old ] && V="$VARIANT"
    timeout -k 10 300 python -u bench.py $X $V > $O/${v}_c${c}_${t}.json 2> $O/${v}_c${c}_${t}.log || exit 1
  done
done
