#!/bin/bash
# A/B on one box: this tree's build (2 device pipes) on cfg2 and cfg3, then abtmp/lib_pipes3.so
# (the same sources with EMQXGM_PIPES 3) on cfg3 at 4 and 5 walk workgroups per CU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_abp}
mkdir -p $O
cd $R
timeout -k 10 240 python -u bench.py --cfg 2 --no-cpu-baseline --no-e2e > $O/p2_cfg2.json 2> $O/p2_cfg2.err || exit 1
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-e2e > $O/p2_cfg3.json 2> $O/p2_cfg3.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
cp abtmp/lib_pipes3.so emqx_amd/libemqx_gpumatch.so && sed -i 's/    PIPES = 2  # EMQXGM_PIPES/    PIPES = 3  # EMQXGM_PIPES/' emqx_amd/engine.py || exit 1
for wg in 4 5; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-e2e --wg-per-cu $wg > $O/p3_wg$wg.json 2> $O/p3_wg$wg.err || exit 1
done
