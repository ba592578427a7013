#!/bin/bash
# quick iteration: a parity subset, the cfg3 / cfg4 / cfg2 bench lines (no CPU baseline), and
# random-gather rates of large tables (TLB reach)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_iter}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py} > $O/pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
timeout -k 10 300 python -u bench.py --cfg 4 --steps 10 --no-cpu-baseline --no-e2e > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 200 python -u bench.py --cfg 2 --steps 10 --no-cpu-baseline --no-e2e > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
if [ -n "$GATHER" ]; then for mb in $GATHER; do timeout -k 10 60 tools/gather_bench $mb 8 4 1 >> $O/gather.txt 2>&1 || exit 1; done; fi
if [ -n "$PCIE" ]; then timeout -k 10 300 python -u tools/pcie_probe.py e2e > $O/pcie.json 2> $O/pcie.err || exit 1; fi
