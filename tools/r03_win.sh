#!/bin/bash
# r03: the batcher GPU tests, then where a NIF window's time goes (tools/window_probe.py), plain
# and under a kernel + memory-copy trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_win}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_batcher.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/window_probe.py > $O/probe.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/window_probe.py --windows 65536 --count 20 > $O/probe_trace.log 2>&1 || exit 1
