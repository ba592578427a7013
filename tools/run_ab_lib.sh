#!/bin/bash
# GPU box: A/B of alternative engine builds (build/lib_<V>.so) against the in-tree one
# (kernel rate only).  usage: [CFGS="2 3"] [ARGS_<V>="--wg-per-cu 5"] tools/run_ab_lib.sh VARIANT...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
run() {  # tag cfg
  local extra; eval "extra=\${ARGS_$1:-}"
  timeout -k 10 300 python -u bench.py --cfg $2 --no-cpu-baseline --no-e2e $extra \
    > gpurun_out/ab/$1_c$2.json 2> gpurun_out/ab/$1_c$2.log || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[1], round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['walk_ms_per_launch'], c['edge_slot_loads_per_batch'])" gpurun_out/ab/$1_c$2.json
}
cp emqx_amd/libemqx_gpumatch.so build/lib_base.so
for V in base "$@"; do
  cp build/lib_$V.so emqx_amd/libemqx_gpumatch.so
  for c in ${CFGS:-2 3}; do run $V $c; done
done
