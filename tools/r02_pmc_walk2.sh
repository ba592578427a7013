#!/bin/bash
# cfg3 walk PMC at the bench batch: issue / wait mix and the vector-memory pipeline (TA/TD/TCP),
# each pass in its own bounded run (the traffic passes are tools/r02_prof.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_pmcw2}
mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp --kernel-include-regex "k_walk" -d $O/pmc_walk/p$i -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc_walk_p$i.log 2>&1 || exit 1
done
python3 $R/tools/pmc_summary.py $O/pmc_walk > $O/pmc_walk_summary.txt 2>&1 || exit 1
