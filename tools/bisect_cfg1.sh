set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bisect; mkdir -p $O
A="--cfg 1 --no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 200 --warmup 20"
(cd $R && timeout -k 10 240 python -u bench.py $A > $O/HEAD.json 2> $O/HEAD.log) &&
for c in 30e2b53 2d2e06a 1754034 5b7e875 5f07789 07c3b37; do
  (cd $R/abtree/$c && timeout -k 10 240 python -u bench.py $A > $O/$c.json 2> $O/$c.log) || exit 1
done
(cd $R && timeout -k 10 240 python -u bench.py $A > $O/HEAD2.json 2> $O/HEAD2.log)
