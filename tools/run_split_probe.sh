cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_delta.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?; echo tests_exit=$rc; tail -3 gpurun_out/t1.log; [ $rc -eq 0 ] || exit $rc
for n in 2000000 4000000 8000000; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --topics $n --steps 20 > gpurun_out/b_$n.json 2> gpurun_out/b_$n.log || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['walk_ms_per_launch'])" gpurun_out/b_$n.json
done
