#!/bin/bash
# exact-probe work: the route-key parity tests (incl. cfg4 at full size), then the cfg4 bench
# under rocprofv3 kernel stats; each step bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_exact}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTK:-route_key_regions or cfg4}" > $O/pytest.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_cfg4 -o run --output-format csv -- python3 $R/bench.py --cfg 4 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
