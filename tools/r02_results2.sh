#!/bin/bash
# every config's default bench line at HEAD (the GPU tests ran on this HEAD separately)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02_results2}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py > $O/cfg3.json 2> $O/cfg3.log || exit 1
for c in 1 2 4; do
  timeout -k 10 400 python -u bench.py --cfg $c > $O/cfg$c.json 2> $O/cfg$c.log || exit 1
done
