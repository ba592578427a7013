#!/bin/bash
# the bench line of the other BASELINE configs (cfg4, cfg2, cfg1), with CPU baselines and the
# host-in/host-out leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_benches}
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --cfg 4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 300 python -u bench.py --cfg 2 --steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 300 python -u bench.py --cfg 1 --steps 20 > $O/bench_cfg1.json 2> $O/bench_cfg1.err
