#!/bin/bash
# rocprofv3 kernel stats and PMC passes of the bench workload of each config in $CFGS at HEAD:
# kernel-trace/stats; FETCH_SIZE; WRITE_SIZE + L2 hit/miss; TCP->TCC requests + latency.
# Every pass in its own bounded run; the bench rotates its default 3 distinct batches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_prof}
mkdir -p $O
KRE="k_walk|k_tok|k_exact|k_scatter|k_verify|k_scan"
for c in ${CFGS:-3 1 2 4}; do
  steps=5; [ $c = 3 ] && steps=10
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats_cfg$c -o run --output-format csv -- python3 $R/bench.py --cfg $c --no-cpu-baseline --no-e2e --steps $steps --warmup 2 > $O/stats_cfg$c.json 2> $O/stats_cfg$c.log || exit 1
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d $O/pmc_cfg$c/p$i -o run --output-format csv -- python3 $R/bench.py --cfg $c --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc_cfg${c}_p$i.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py $O/pmc_cfg$c > $O/pmc_cfg${c}_summary.txt 2>&1 || exit 1
done
