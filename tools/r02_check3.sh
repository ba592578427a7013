#!/bin/bash
# pipe tests (device + host pipes, concurrency), then the cfg1 and cfg3 bench lines; each bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_check3}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -v --timeout 400 --timeout-method thread -k "concurrency or pipelined or host_batch or dist or merge" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --cfg 1 --steps 10 > $O/cfg1.json 2> $O/cfg1.log || exit 1
timeout -k 10 300 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log
