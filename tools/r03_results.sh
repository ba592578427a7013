#!/bin/bash
# r03: the 18-item deep compact stack A/B on cfg2 (4 blocks per CU instead of 3; alternating
# builds), then every config's default bench line (CPU baseline, host path) at HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_results}
O=$R/gpurun_out/$T
mkdir -p $O/ab
cd $R
cp emqx_amd/libemqx_gpumatch.so build/lib_base.so
X="--cfg 2 --no-cpu-baseline --no-e2e --steps 30 --warmup 5"
for i in 1 2; do
  for V in base deep18; do
    cp build/lib_$V.so emqx_amd/libemqx_gpumatch.so || exit 1
    timeout -k 10 300 python -u bench.py $X > $O/ab/${V}_c2_$i.json 2> $O/ab/${V}_c2_$i.log || exit 1
  done
done
cp build/lib_base.so emqx_amd/libemqx_gpumatch.so
for c in 1 2 4 3; do
  timeout -k 10 400 python -u bench.py --cfg $c > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
