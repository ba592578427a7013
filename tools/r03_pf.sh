#!/bin/bash
# r03: deep-level token prefetch (build/lib_pf.so, -DGM_DEEP_PF=1) -- A/B against the product
# build, then the GPU tests with lib_pf in place of the product library
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r03_pf}
cd $R
mkdir -p gpurun_out/$T
SPECS="1:0 3:0 3:65536" STEPS=50 bash tools/r03_ab_lib.sh $T/ab pf || exit 1
python tools/ab_lib_summary.py gpurun_out/$T/ab
cp emqx_amd/libemqx_gpumatch.so build/lib_prod.so && cp build/lib_pf.so emqx_amd/libemqx_gpumatch.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests_pf.log 2>&1; rc=$?
cp build/lib_prod.so emqx_amd/libemqx_gpumatch.so
tail -3 gpurun_out/$T/gpu_tests_pf.log
exit $rc
