#!/bin/bash
# GPU-box: calibrate FETCH_SIZE / TCC_EA0_RDREQ for random gathers of known size (gather_bench,
# 2 GiB table, 1024 x 256 lanes x 64 dependent rounds = 16,777,216 accesses per dispatch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/calib; cd /tmp && export TMPDIR=/tmp
for W in 1 2 4; do
  for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $grp | cut -c1-10)
    timeout -s KILL 60 rocprofv3 --pmc $grp -d $R/gpurun_out/calib/w${W}_$tag -o run --output-format csv -- $R/tools/gather_bench 2048 4 $W 1 > $R/gpurun_out/calib/w${W}_$tag.log 2>&1 || exit 1
  done
done
python3 - "$R/gpurun_out/calib" <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/calib/")[1].split("/")[0], {k: v for k, v in acc.items()})
PY
