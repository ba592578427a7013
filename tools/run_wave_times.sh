# GPU box: per-wave walk timelines at 2M and 8M topics, then a kernel-stats profile at 2M.
cd "${GRAFT_REPO_ROOT}"; R=$(pwd)
mkdir -p gpurun_out
for n in 2000000 8000000; do
EMQXGM_WAVE_TIMES=gpurun_out/wt_$n.bin timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --topics $n --steps 5 > gpurun_out/wb_$n.json 2> gpurun_out/wb_$n.log || exit 1
python3 tools/wave_times.py gpurun_out/wt_$n.bin
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_v26 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 1 > $R/gpurun_out/prof_v26.log 2>&1 || exit 1
python3 - "$R/gpurun_out/prof_v26" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:48]:48s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):6.2f}")
PY
