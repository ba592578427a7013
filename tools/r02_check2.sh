#!/bin/bash
# host pipes + route-key tests, then the cfg3 and cfg4 bench lines; each step bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_check2}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "${TESTK:-host_pipes or route_key_regions or pipelined or host_batch}" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
timeout -k 10 400 python -u bench.py --cfg 4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
