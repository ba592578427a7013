# cfg3 pipelined step against the pipelined walk's workgroups per CU (emqxgm_tune
# "walk_wg_per_cu_pipe"), then one kernel trace of the default for the passes' overlap.
# GPU box: bash tools/pipe_sweep.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pipe_sweep; mkdir -p $O
A="--no-cpu-baseline --no-e2e --nif= --no-subscribe --steps 100 --warmup 10"
for w in 3 2 4 3; do
  (cd $R && timeout -k 10 300 python -u bench.py $A --tune walk_wg_per_cu_pipe=$w > $O/wg$w.$RANDOM.json 2> $O/wg$w.log) || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv \
  -- python3 $R/bench.py $A --steps 20 --settle-s 0 > $O/trace.json 2> $O/trace.log
