#!/bin/bash
# GPU-box: bench.py (1 GPU) for every BASELINE config -> gpurun_out/results/cfgN.json
# (kernel topics/s, end-to-end topics/s, roofline of k_walk, CPU restatement beside it).
# cfg4 (100M exact keys + 1M wildcards) skips the CPU baseline: its ordered-set index alone
# takes minutes on the host.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/results
for c in ${CFGS:-1 2 4}; do
  extra=""
  [ "$c" = 4 ] && extra="--no-cpu-baseline"
  timeout -k 10 900 python -u bench.py --cfg $c --steps 10 --cpu-seconds 5 $extra \
    > gpurun_out/results/cfg$c.json 2> gpurun_out/results/cfg$c.log
  rc=$?; echo "cfg$c exit=$rc"; cat gpurun_out/results/cfg$c.json
  [ $rc -eq 0 ] || exit $rc
done
