#!/bin/bash
# cfg3 bench line at batch sizes across BASELINE's 1M-8M topic range (no CPU baseline / e2e)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_sweep}
mkdir -p $O
cd $R
for nt in ${SIZES:-1000000 2000000 4000000 8000000}; do
  timeout -k 10 240 python -u bench.py --topics $nt --no-cpu-baseline --no-e2e > $O/bench_$nt.json 2> $O/bench_$nt.err || exit 1
done
