# GPU box: A/B of the walk grid (workgroups per CU) under pipelined steps.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for wg in 4 3 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --wg-per-cu $wg > gpurun_out/wg_$wg.json 2> gpurun_out/wg_$wg.log || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['walk_ms_per_launch'], d['config']['one_pass_at_a_time'])" gpurun_out/wg_$wg.json
done
