#!/bin/bash
# Random-line ceilings: vector gathers by allocation kind over tables beyond the TLB reach, and
# scalar + vector mixes (tools/sgather_bench.hip); each run bounded
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_gather}
mkdir -p $O
for a in 0 1 2; do
  for mb in 2048 8192; do
    timeout -k 10 60 $R/tools/gather_bench $mb 8 4 1 $a >> $O/gather_alloc.txt 2>&1
    rc=$?; [ $rc -le 1 ] || exit $rc   # 1 = an allocation kind refused (printed), go on
  done
done
for mb in 2048 64; do
  timeout -k 10 90 $R/tools/sgather_bench $mb 8 64 >> $O/sgather.txt 2>&1 || exit 1
done
timeout -k 10 90 $R/tools/sgather_bench 2048 4 64 >> $O/sgather.txt 2>&1 || exit 1
