#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r02_abq
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > $O/default.json 2> $O/default.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > $O/q8.json 2> $O/q8.err
