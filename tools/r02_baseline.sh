#!/bin/bash
# round-2 baseline on a fresh box: default bench (timed), cfg4 and cfg2 bench lines, and
# rocprofv3 kernel stats for cfg2 and cfg4
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02_base
mkdir -p $O
cd $R
( time timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err ) 2> $O/bench_default.time && \
( time timeout -k 10 400 python -u bench.py --cfg 4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err ) 2> $O/bench_cfg4.time && \
( time timeout -k 10 300 python -u bench.py --cfg 2 --steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err ) 2> $O/bench_cfg2.time
