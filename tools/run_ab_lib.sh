#!/bin/bash
# GPU box: A/B of an alternative engine build (build/lib_$1.so) against the in-tree one on
# cfg2 and cfg3 (kernel rate only).  usage: tools/run_ab_lib.sh VARIANT
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
V=$1
run() {  # tag cfg
  timeout -k 10 300 python -u bench.py --cfg $2 --no-cpu-baseline --no-e2e \
    > gpurun_out/ab/$1_c$2.json 2> gpurun_out/ab/$1_c$2.log || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['walk_ms_per_launch'], c['edge_slot_loads_per_batch'])" gpurun_out/ab/$1_c$2.json
}
run base 2 && run base 3
cp build/lib_$V.so emqx_amd/libemqx_gpumatch.so
run $V 2 && run $V 3
