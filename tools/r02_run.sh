#!/bin/bash
# GPU tests + smoke + the bench line of every BASELINE config (cfg3 default, cfg4, cfg2)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_run}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${TESTS} > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err && \
timeout -k 10 400 python -u bench.py --cfg 4 --steps 10 > $O/bench_cfg4.json 2> $O/bench_cfg4.err && \
timeout -k 10 300 python -u bench.py --cfg 2 --steps 10 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
