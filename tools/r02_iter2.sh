#!/bin/bash
# one iteration on the box: GPU parity tests (TESTS, default the parity file), then cfg3 and
# cfg2 bench lines (no CPU baseline / host-pipe leg)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_it}
mkdir -p $O
cd $R
TESTS=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-e2e > $O/cfg3.json 2> $O/cfg3.err || exit 1
timeout -k 10 240 python -u bench.py --cfg 2 --no-cpu-baseline --no-e2e > $O/cfg2.json 2> $O/cfg2.err || exit 1
for wg in ${WGS:-}; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-e2e --wg-per-cu $wg > $O/cfg3_wg$wg.json 2> $O/cfg3_wg$wg.err || exit 1
done
