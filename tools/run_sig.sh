# GPU box: full check, then cfg3 and cfg2 bench lines (no CPU baseline / e2e).
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_check.sh > gpurun_out/check.txt 2>&1; rc=$?
tail -2 gpurun_out/check.txt; grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head
[ $rc -eq 0 ] || exit $rc
for c in 3 2; do
timeout -k 10 300 python -u bench.py --cfg $c --no-cpu-baseline --no-e2e > gpurun_out/sig_$c.json 2> gpurun_out/sig_$c.log || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['walk_ms_per_launch'], c['edge_slot_loads_per_batch'], c['one_pass_at_a_time'])" gpurun_out/sig_$c.json
done
