#!/bin/bash
# r03 A/B on one box: optional GPU tests, then bench.py per config with and without the
# variant's tune flags (B first, then A, then B again to bracket drift); each step bounded.
#   TESTS=1 CFGS="3 2 1" VARIANT="--tune fat_buckets=0" tools/r03_ab.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_ab}
mkdir -p $O
cd $R
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
  timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
fi
for c in ${CFGS:-3}; do
  X="--cfg $c --no-cpu-baseline --no-e2e --steps ${STEPS:-50} --warmup 5"
  timeout -k 10 300 python -u bench.py $X > $O/cfg${c}_new1.json 2> $O/cfg${c}_new1.log || exit 1
  timeout -k 10 300 python -u bench.py $X $VARIANT > $O/cfg${c}_old.json 2> $O/cfg${c}_old.log || exit 1
  timeout -k 10 300 python -u bench.py $X > $O/cfg${c}_new2.json 2> $O/cfg${c}_new2.log || exit 1
done
