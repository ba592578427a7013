#!/bin/bash
# r03: cfg3 4M alternating A/B of HEAD vs build/lib_memset (three pairs), then the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03_alt}
O=$R/gpurun_out/$T
mkdir -p $O/ab
cd $R
cp emqx_amd/libemqx_gpumatch.so build/lib_base.so
X="--cfg 3 --no-cpu-baseline --no-e2e --steps 100 --warmup 10"
for i in 1 2 3; do
  for V in base memset; do
    cp build/lib_$V.so emqx_amd/libemqx_gpumatch.so || exit 1
    timeout -k 10 300 python -u bench.py $X > $O/ab/${V}_c3_$i.json 2> $O/ab/${V}_c3_$i.log || exit 1
  done
done
cp build/lib_base.so emqx_amd/libemqx_gpumatch.so
timeout -k 10 400 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
