#!/bin/bash
# rocprofv3 kernel-trace/stats and PMC passes (FETCH_SIZE; WRITE_SIZE + L2 hit/miss) of the
# bench workload of each config in $CFGS, each pass in its own bounded run
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_prof}
mkdir -p $O
KRE="k_walk|k_tok|k_exact|k_scatter|k_verify|k_scan"
for c in ${CFGS:-3 2 4}; do
  steps=5; [ $c = 3 ] && steps=10
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_cfg$c -o run --output-format csv -- python3 $R/bench.py --cfg $c --no-cpu-baseline --no-e2e --steps $steps --warmup 2 > $O/stats_cfg$c.log 2>&1 || exit 1
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $O/pmc_cfg$c/p$i -o run --output-format csv -- python3 $R/bench.py --cfg $c --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc_cfg${c}_p$i.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py $O/pmc_cfg$c > $O/pmc_cfg${c}_summary.txt 2>&1 || exit 1
done
