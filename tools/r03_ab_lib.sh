#!/bin/bash
# r03 A/B of engine builds (build/lib_<V>.so, tools/ab_build.sh) on one box: each variant's
# bench lines for the specs in $SPECS ("cfg:topics" ..., topics 0 = the config's default),
# base first and last to bracket drift.  usage: SPECS="3:0 3:65536 1:0" tools/r03_ab_lib.sh TAG V...
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_ablib}
shift
mkdir -p $O
cd $R
cp emqx_amd/libemqx_gpumatch.so build/lib_base.so
for V in base "$@" base; do
  cp build/lib_$V.so emqx_amd/libemqx_gpumatch.so || exit 1
  for spec in ${SPECS:-3:0}; do
    c=${spec%%:*}; t=${spec##*:}
    T=""; [ "$t" != 0 ] && T="--topics $t"
    timeout -k 10 300 python -u bench.py --cfg $c $T --no-cpu-baseline --no-e2e --steps ${STEPS:-50} --warmup 5 > $O/${V}_c${c}_${t}.json 2> $O/${V}_c${c}_${t}.log || exit 1
  done
done
cp build/lib_base.so emqx_amd/libemqx_gpumatch.so
