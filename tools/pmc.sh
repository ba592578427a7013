#!/bin/bash
# GPU-box: rocprofv3 PMC passes (one counter group per run, as the guide requires) over the
# bench workload, restricted to the kernels matching $KREGEX.
# usage: [KREGEX=..] [PASSES="grp1;grp2;..."] tools/pmc.sh TAG [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); TAG=${1:-pmc}; shift
KREGEX=${KREGEX:-k_walk|k_tok}
PASSES=${PASSES:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"}
mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra GROUPS_ <<< "$PASSES"
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -d $R/gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $R/gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?
  echo "pass $i exit=$rc"
  [ $rc -eq 0 ] || break
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_$TAG
