#!/bin/bash
# Alternating A/B repeats on the GPU box: the in-tree engine (base) and ablib/lib_VARIANT.so
# (tools/ab_build.sh), 3 runs each, cfg3 default batch, 100 timed steps.
#   tools/ab_repeat.sh TAG VARIANT
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; V=$2; mkdir -p $O
cp $R/emqx_amd/libemqx_gpumatch.so $R/ablib/lib_base.so || exit 1
for i in 1 2 3; do
  for v in base $V; do
    cp $R/ablib/lib_$v.so $R/emqx_amd/libemqx_gpumatch.so || exit 1
    (cd $R && timeout -k 10 300 python -u bench.py --cfg 3 --no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 100 --warmup 10) > $O/${v}_c3_r$i.json 2> $O/${v}_r$i.log || { cp $R/ablib/lib_base.so $R/emqx_amd/libemqx_gpumatch.so; exit 1; }
    echo "[ab] $v $i done"
  done
done
cp $R/ablib/lib_base.so $R/emqx_amd/libemqx_gpumatch.so
python3 $R/tools/ab_lib_summary.py $O > $O/ab_summary.txt 2>&1
