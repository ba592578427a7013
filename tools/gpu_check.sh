#!/bin/bash
# GPU-box check: smoke() then the -m gpu parity suite; logs land in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo smoke_exit=$?; tail -1 gpurun_out/smoke.log
[ $(grep -c "smoke ok" gpurun_out/smoke.log) -ge 1 ] || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo tests_exit=$rc
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -40
exit $rc
