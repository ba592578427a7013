# GPU box: pipelined-pass test, then bench (2M default) + kernel-stats profile.
cd "${GRAFT_REPO_ROOT}"; R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pipelined or route_key or device_api" -x -q --timeout 200 --timeout-method thread > gpurun_out/tp.log 2>&1
rc=$?; echo tests_exit=$rc; tail -15 gpurun_out/tp.log; [ $rc -eq 0 ] || exit $rc
bash tools/bench_prof.sh v27
