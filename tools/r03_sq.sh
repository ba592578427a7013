#!/bin/bash
# r03: issue / wait mix of the production walk per config (SQ counters, two passes of 8 SQ
# counters each), every pass its own bounded run.  usage: CFGS="1 2" tools/r03_sq.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_sq}
mkdir -p $O
for c in ${CFGS:-1 2 3}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "k_walk|k_scatter" -d $O/sq_cfg$c/p$i -o run --output-format csv -- python3 $R/bench.py --cfg $c --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/sq_cfg${c}_p$i.log 2>&1 || exit 1
  done
  python3 $R/tools/pmc_summary.py $O/sq_cfg$c > $O/sq_cfg${c}_summary.txt 2>&1 || exit 1
done
