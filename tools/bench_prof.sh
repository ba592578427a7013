#!/bin/bash
# GPU-box: bench.py (1 GPU) then a rocprofv3 kernel-trace/stats pass of the same workload.
# usage: tools/bench_prof.sh TAG [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log
rc=$?; echo bench_exit=$rc; cat gpurun_out/bench_$TAG.json; tail -4 gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo prof_exit=$rc
python3 - "$R/gpurun_out/prof_$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:48]:48s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):6.2f}")
PY
exit $rc
