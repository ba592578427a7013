# cfg2 / cfg1 pipelined step against the pipelined walk's workgroups per CU.
# GPU box: bash tools/pipe_sweep2.sh
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pipe_sweep2; mkdir -p $O
A="--no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 50 --warmup 10"
for c in 2 1; do
  for w in 3 4 2 3; do
    (cd $R && timeout -k 10 300 python -u bench.py --cfg $c $A --tune walk_wg_per_cu_pipe=$w > $O/c${c}_wg$w.$RANDOM.json 2> $O/c${c}_wg$w.log) || exit 1
  done
done
