#!/bin/bash
# parity tests (GPU), A/B against build/lib_nt8.so on cfg2 / cfg4, rocprof kernel stats of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_it3}
mkdir -p $O $R/gpurun_out/ab
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || exit 1
CFGS="2 4" bash tools/run_ab_lib.sh nt8 > $O/ab.txt 2>&1 || exit 1
cp build/lib_base.so emqx_amd/libemqx_gpumatch.so
for c in 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_c$c -o run --output-format csv -- python3 bench.py --cfg $c --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $O/stats_c$c.log 2>&1 || exit 1
done
